"""Synthetic ray generation (restates ``datasets/ray_utils.py`` and the Blender /
LLFF camera conventions of ``datasets/blender.py`` / ``datasets/llff.py``).

These build the ``(N, 8) = [o, d, near, far]`` ray buffers the hot path
consumes.  They are plain tensor algebra on whatever device the inputs live on;
there is no dataset I/O (no data exists in this environment), so poses are
generated on a sphere like the reference's spheric render path
(``datasets/llff.py:128-149``).
"""
from __future__ import annotations

import math

import torch

LEGO_CAMERA_ANGLE_X = 0.6911112070083618   # nerf_synthetic/lego transforms_train.json


def blender_focal(img_w: int, camera_angle_x: float = LEGO_CAMERA_ANGLE_X) -> float:
    """datasets/blender.py:34-37: focal at 800 px, rescaled to ``img_w``."""
    return 0.5 * 800 / math.tan(0.5 * camera_angle_x) * img_w / 800


def get_ray_directions(H: int, W: int, focal: float, device=None) -> torch.Tensor:
    """ray_utils.py:5-24 -- camera-frame directions, no +0.5 pixel centering.
    ``i`` is the column (x) index and ``j`` the row (y) index, as kornia's
    ``create_meshgrid(H, W, normalized_coordinates=False)`` yields them."""
    j, i = torch.meshgrid(torch.arange(H, dtype=torch.float32, device=device),
                          torch.arange(W, dtype=torch.float32, device=device), indexing="ij")
    return torch.stack([(i - W / 2) / focal, -(j - H / 2) / focal, -torch.ones_like(i)], -1)


def get_rays(directions: torch.Tensor, c2w: torch.Tensor):
    """ray_utils.py:27-50 -- world-frame origins and unit directions."""
    rays_d = directions @ c2w[:, :3].T
    rays_d = rays_d / torch.norm(rays_d, dim=-1, keepdim=True)
    rays_o = c2w[:, 3].expand(rays_d.shape)
    return rays_o.reshape(-1, 3), rays_d.reshape(-1, 3)


def get_ndc_rays(H: int, W: int, focal: float, near: float, rays_o: torch.Tensor,
                 rays_d: torch.Tensor):
    """ray_utils.py:53-93 -- forward-facing (LLFF) NDC transform."""
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


def pose_spherical(theta_deg: float, phi_deg: float, radius: float) -> torch.Tensor:
    """(3,4) camera-to-world matrix looking at the origin from a sphere."""
    th, ph = math.radians(theta_deg), math.radians(phi_deg)
    trans = torch.tensor([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, radius], [0, 0, 0, 1]],
                         dtype=torch.float64)
    rot_phi = torch.tensor([[1, 0, 0, 0],
                            [0, math.cos(ph), -math.sin(ph), 0],
                            [0, math.sin(ph), math.cos(ph), 0],
                            [0, 0, 0, 1]], dtype=torch.float64)
    rot_theta = torch.tensor([[math.cos(th), 0, -math.sin(th), 0],
                              [0, 1, 0, 0],
                              [math.sin(th), 0, math.cos(th), 0],
                              [0, 0, 0, 1]], dtype=torch.float64)
    flip = torch.tensor([[-1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]],
                        dtype=torch.float64)
    c2w = flip @ rot_theta @ rot_phi @ trans
    return c2w[:3, :4].float()


def blender_rays(img_wh: int, n_poses: int, near: float = 1.0, far: float = 200.0,
                 radius: float = 4.0, phi_deg: float = -30.0, device=None) -> torch.Tensor:
    """Ray buffer (n_poses*H*W, 8) of a synthetic Blender-lego camera orbit.

    near/far default to this fork's Blender bounds (datasets/blender.py:40-41)."""
    H = W = img_wh
    focal = blender_focal(W)
    dirs = get_ray_directions(H, W, focal, device=device)
    out = []
    for k in range(n_poses):
        theta = -180.0 + 360.0 * k / n_poses
        c2w = pose_spherical(theta, phi_deg, radius).to(device)
        o, d = get_rays(dirs, c2w)
        nf = torch.tensor([near, far], dtype=torch.float32, device=device).expand(o.shape[0], 2)
        out.append(torch.cat([o, d, nf], 1))
    return torch.cat(out, 0)


def llff_ndc_rays(img_w: int = 504, img_h: int = 378, n_poses: int = 4,
                  focal: float = 407.0, device=None) -> torch.Tensor:
    """Forward-facing NDC rays (near/far 0/1) like datasets/llff.py:236-242."""
    dirs = get_ray_directions(img_h, img_w, focal, device=device)
    out = []
    for k in range(n_poses):
        ang = 2 * math.pi * k / max(n_poses, 1)
        c2w = torch.eye(4, dtype=torch.float32)[:3]
        c2w[:, 3] = torch.tensor([0.1 * math.cos(ang), 0.1 * math.sin(ang), 0.0])
        c2w = c2w.to(device)
        o, d = get_rays(dirs, c2w)                       # llff.py:234
        o_ndc, d_ndc = get_ndc_rays(img_h, img_w, focal, 1.0, o, d)   # llff.py:237-238
        nf = torch.tensor([0.0, 1.0], dtype=torch.float32, device=device).expand(o.shape[0], 2)
        out.append(torch.cat([o_ndc, d_ndc, nf], 1))
    return torch.cat(out, 0)


def generate_rays(c2w: torch.Tensor, H: int, W: int, focal: float, near: float, far: float,
                  sel: torch.Tensor = None, ndc: bool = False, ndc_near: float = 1.0,
                  rgb_pool: torch.Tensor = None):
    """Rays (n, 8) for global pixel indices ``sel`` (pose*H*W + row*W + col) of
    the poses ``c2w`` (n_poses, 3, 4), generated on the device by
    ``nr_gen_rays`` -- the batch the reference assembles from its precomputed
    ray buffer (datasets/blender.py:54-86, llff.py:213-249).  ``sel=None``
    means every pixel of every pose.  With ``rgb_pool`` (n_poses*H*W, 3) the
    target colours of the same pixels are returned too.  With ``ndc`` the
    forward-facing transform (get_ndc_rays, near plane ``ndc_near``) is applied
    and near/far become 0/1 (llff.py:236-242)."""
    from . import ops
    from ._lib import call, ptr, stream_of
    c2w = ops._dev(c2w.to(torch.float32), "c2w")
    if c2w.shape[-2:] != (3, 4):
        raise ValueError(f"c2w must be (n_poses, 3, 4), got {tuple(c2w.shape)}")
    dev = c2w.device
    n_poses = c2w.reshape(-1, 12).shape[0]
    if sel is not None:
        sel = sel.to(device=dev, dtype=torch.int64).contiguous()
        n = sel.shape[0]
    else:
        n = n_poses * H * W
    rays = torch.empty(n, 8, device=dev)
    rgb_out = None
    if rgb_pool is not None:
        rgb_pool = ops._dev(rgb_pool, "rgb_pool", 3)
        rgb_out = torch.empty(n, 3, device=dev)
    if ndc:
        near, far = 0.0, 1.0
    call("nr_gen_rays", ptr(c2w), n_poses, H, W, float(W / 2), float(H / 2), float(focal),
         float(near), float(far), int(ndc), float(ndc_near), -1. / (W / (2. * focal)),
         -1. / (H / (2. * focal)), 2. * ndc_near, ptr(sel), n, ptr(rgb_pool), ptr(rgb_out),
         ptr(rays), stream_of(dev))
    return (rays, rgb_out) if rgb_pool is not None else rays


class RaySampler:
    """Shuffled training batches generated on the device -- replaces the
    reference's ray buffer + ``DataLoader(shuffle=True, batch_size=B)``
    (train.py:89-94): each epoch is a random permutation of all pixels of all
    poses, each batch is produced by one ``nr_gen_rays`` launch that also
    gathers the target colours.

    Data-parallel runs partition every epoch like the ``DistributedSampler``
    that Lightning's DDP backend installs (train.py:175), and with
    its very permutation: ``torch.randperm`` of the epoch on a CPU generator
    seeded ``seed + epoch`` (identical on every rank), padded with its head to a
    multiple of ``world``, rank r taking ``perm[r::world]`` -- the ranks'
    batches are disjoint and together cover the epoch.  An epoch ends when the
    rank's shard cannot fill another batch (the remainder is dropped).  The
    permutation is drawn on the host by a worker thread one epoch ahead and
    only the rank's shard is copied to the device: a device-side randperm of a
    64M-pixel pool (cfg4) costs every rank a 64M-key radix sort per epoch, and
    with several ranks sharing one GPU (the one-GPU rehearsal of the 8-GPU
    run) four concurrent sorts did not finish in 100 s."""

    def __init__(self, c2w, H, W, focal, near, far, rgb_pool=None, ndc=False, seed=0, rank=0,
                 world=1):
        if not 0 <= rank < world:
            raise ValueError(f"RaySampler: rank {rank} outside world {world}")
        self.c2w = c2w
        self.H, self.W, self.focal, self.near, self.far = H, W, focal, near, far
        self.rgb_pool, self.ndc = rgb_pool, ndc
        self.total = c2w.reshape(-1, 12).shape[0] * H * W
        self.seed, self.rank, self.world = seed, rank, world
        self.device = c2w.device
        self.epoch, self.shard, self.pos = -1, None, 0
        self._pool = None
        self._ahead = None      # (epoch, future of its host shard)

    def _host_shard(self, epoch):
        gen = torch.Generator().manual_seed(self.seed + epoch)
        perm = torch.randperm(self.total, generator=gen)
        pad = (-self.total) % self.world          # DistributedSampler(drop_last=False)
        if pad:
            perm = torch.cat([perm, perm[:pad]])
        shard = perm[self.rank::self.world].contiguous()
        return shard.pin_memory() if self.device.type == "cuda" else shard

    def _new_epoch(self):
        import concurrent.futures
        self.epoch += 1
        if self._pool is None:
            self._pool = concurrent.futures.ThreadPoolExecutor(max_workers=1)
        if self._ahead is not None and self._ahead[0] == self.epoch:
            host = self._ahead[1].result()
        else:
            host = self._host_shard(self.epoch)
        self._ahead = (self.epoch + 1, self._pool.submit(self._host_shard, self.epoch + 1))
        self.shard = host.to(self.device, non_blocking=True)
        self.pos = 0

    def next_indices(self, batch: int):
        """Global pixel indices of the next batch (pose*H*W + row*W + col)."""
        if self.shard is None or self.pos + batch > self.shard.shape[0]:
            self._new_epoch()
            if batch > self.shard.shape[0]:
                raise ValueError(f"RaySampler: batch {batch} exceeds the rank's "
                                 f"{self.shard.shape[0]} rays per epoch")
        sel = self.shard[self.pos:self.pos + batch]
        self.pos += batch
        return sel

    def next(self, batch: int):
        sel = self.next_indices(batch)
        return generate_rays(self.c2w, self.H, self.W, self.focal, self.near, self.far, sel,
                             self.ndc, rgb_pool=self.rgb_pool)
