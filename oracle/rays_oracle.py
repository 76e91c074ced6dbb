"""CPU oracle for ray generation.

TEST INFRASTRUCTURE ONLY -- imported by ``tests/`` alone.

Restates ``datasets/ray_utils.py`` in PyTorch-CPU fp32 with the reference's
op order: ``get_ray_directions`` (:5-24; kornia's ``create_meshgrid`` with
``normalized_coordinates=False`` gives i = column, j = row, no +0.5),
``get_rays`` (:27-50) and ``get_ndc_rays`` (:53-93).  The reference module
imports kornia, which is absent here, so it cannot be imported whole; its
kornia-free ``get_rays`` and ``get_ndc_rays`` are run as they stand by
tests/golden/make_golden_rays.py, and tests/test_rays_golden.py pins this
restatement to their outputs (bit-exact on the fixture host).
``get_ray_directions`` (kornia's meshgrid) stays pinned only by that
restatement of kornia 0.2.0's documented semantics.
"""
from __future__ import annotations

import torch


def get_ray_directions(H: int, W: int, focal: float) -> torch.Tensor:
    j, i = torch.meshgrid(torch.arange(H, dtype=torch.float32),
                          torch.arange(W, dtype=torch.float32), indexing="ij")
    return torch.stack([(i - W / 2) / focal, -(j - H / 2) / focal, -torch.ones_like(i)], -1)


def get_rays(directions: torch.Tensor, c2w: torch.Tensor):
    rays_d = directions @ c2w[:, :3].T
    rays_d = rays_d / torch.norm(rays_d, dim=-1, keepdim=True)
    rays_o = c2w[:, 3].expand(rays_d.shape)
    return rays_o.reshape(-1, 3), rays_d.reshape(-1, 3)


def get_ndc_rays(H, W, focal, near, rays_o, rays_d):
    t = -(near + rays_o[..., 2]) / rays_d[..., 2]
    rays_o = rays_o + t[..., None] * rays_d
    ox_oz = rays_o[..., 0] / rays_o[..., 2]
    oy_oz = rays_o[..., 1] / rays_o[..., 2]
    o0 = -1. / (W / (2. * focal)) * ox_oz
    o1 = -1. / (H / (2. * focal)) * oy_oz
    o2 = 1. + 2. * near / rays_o[..., 2]
    d0 = -1. / (W / (2. * focal)) * (rays_d[..., 0] / rays_d[..., 2] - ox_oz)
    d1 = -1. / (H / (2. * focal)) * (rays_d[..., 1] / rays_d[..., 2] - oy_oz)
    d2 = 1 - o2
    return torch.stack([o0, o1, o2], -1), torch.stack([d0, d1, d2], -1)


def ray_buffer(poses: torch.Tensor, H: int, W: int, focal: float, near: float, far: float,
               ndc: bool = False) -> torch.Tensor:
    """(n_poses*H*W, 8) like datasets/blender.py:79-83 / llff.py:231-249."""
    dirs = get_ray_directions(H, W, focal)
    out = []
    for c2w in poses:
        o, d = get_rays(dirs, c2w)
        if ndc:
            o, d = get_ndc_rays(H, W, focal, 1.0, o, d)
            near, far = 0.0, 1.0
        out.append(torch.cat([o, d, near * torch.ones_like(o[:, :1]),
                              far * torch.ones_like(o[:, :1])], 1))
    return torch.cat(out, 0)
