"""``render_rays`` for rays that live on the host: BASELINE configs[0]
("Blender lego 64x64, N_samples=32, N_importance=0, batch 256 on PyTorch CPU,
plumbing, no GPU").

The reference runs wherever its ``rays`` tensor lives (models/rendering.py:178,
216, 231 take ``device=rays.device``), so a CPU batch is a legitimate call of
its API.  This module is that call's path: plain PyTorch CPU ops in the
reference's order, autograd through them, the models' own ``nn.Linear``
layers (``NeRF.forward_layers``) and embeddings.  It is chosen by the device
of ``rays`` alone (nerf_pl_amd.rendering.render_rays); a HIP-device batch never
comes here -- it runs on the HIP kernels or raises, and nothing here is a
stand-in for a missing library.  Default randomness is the global torch
generator in the reference's draw order (rng.TorchRNG), so with the same
``torch.manual_seed`` a CPU call draws exactly the reference's numbers.

Pinned by tests/test_host_path.py against the golden fixtures produced by
running the reference (cfg1_s32, cfg1_grad and the other cases) at 1e-4
absolute.  It imports nothing from the repository's test infrastructure
(tests/test_host_path.py checks every module of the package for that).
"""
from __future__ import annotations

import torch

__all__ = ["render_rays_host"]


def _stratified(rays, n, use_disp, perturb, u):
    """coarse depths, rendering.py:216-232"""
    near, far = rays[:, 6:7], rays[:, 7:8]
    t = torch.linspace(0, 1, n, device=rays.device)
    if use_disp:
        z = 1 / (1 / near * (1 - t) + 1 / far * t)
    else:
        z = near * (1 - t) + far * t
    z = z.expand(rays.shape[0], n)
    if perturb > 0:
        mid = 0.5 * (z[:, :-1] + z[:, 1:])
        hi = torch.cat([mid, z[:, -1:]], -1)
        lo = torch.cat([z[:, :1], mid], -1)
        z = lo + (hi - lo) * (perturb * u)
    return z


def _composite(sigma, rgb, z, dirs, noise, white_back, weights_only):
    """alpha compositing, rendering.py:169-198 (exclusive transmittance)"""
    gaps = z[:, 1:] - z[:, :-1]
    gaps = torch.cat([gaps, 1e10 * torch.ones_like(gaps[:, :1])], -1)
    gaps = gaps * torch.norm(dirs.unsqueeze(1), dim=-1)
    alpha = 1 - torch.exp(-gaps * torch.relu(sigma + noise))
    trans = torch.cumprod(torch.cat([torch.ones_like(alpha[:, :1]), 1 - alpha + 1e-10], -1), -1)
    w = alpha * trans[:, :-1]
    if weights_only:
        return None, None, w
    color = torch.sum(w.unsqueeze(-1) * rgb, -2)
    depth = torch.sum(w * z, -1)
    if white_back:
        color = color + 1 - w.sum(1).unsqueeze(-1)
    return color, depth, w


def _importance(rays, w, n_imp, u, jit, eps=1e-5):
    """uniform-bin inverse CDF, rendering.py:14-48 (searchsorted side='right')"""
    nb = w.shape[1]
    w = w + eps
    cdf = torch.cumsum(w / torch.sum(w, -1, keepdim=True), -1)
    cdf = torch.cat([torch.zeros_like(cdf[:, :1]), cdf], -1)
    idx = torch.clamp_min(torch.searchsorted(cdf.contiguous(), u.contiguous(), right=True).float() - 1, 0)
    t = (idx + jit) / nb
    return rays[:, -2:-1] * (1 - t) + rays[:, -1:] * t


def _mlp(model, embeddings, xyz, dir_emb, chunk, sigma_only):
    """inference()'s chunk loop, rendering.py:141-161: embed xyz per chunk, the
    direction embedding repeated per sample, the model on the concatenation"""
    n_rays, spr = xyz.shape[:2]
    pts = xyz.reshape(-1, 3)
    if not sigma_only:
        dir_rep = torch.repeat_interleave(dir_emb, repeats=spr, dim=0)
    outs = []
    for i in range(0, pts.shape[0], chunk):
        e = embeddings[0](pts[i:i + chunk])
        if not sigma_only:
            e = torch.cat([e, dir_rep[i:i + chunk]], 1)
        outs.append(model.forward_layers(e, sigma_only=sigma_only))
    return torch.cat(outs, 0)


def render_rays_host(models, embeddings, rays, N_samples, use_disp, perturb, noise_std,
                     N_importance, chunk, white_back, test_time, rng, capture=None):
    """rendering.py:84-272 on host tensors (see the module docstring)"""
    if embeddings is None:
        raise ValueError("nerf_pl_amd.render_rays: a host batch needs its embeddings")
    for m in models:
        if m is not None and any(p.device != rays.device for p in m.parameters()):
            raise RuntimeError("nerf_pl_amd.render_rays: rays are on the host but a model's "
                               "parameters are not (move both to one device)")
    cap = capture if capture is not None else {}
    dev = rays.device
    n = rays.shape[0]
    if n == 0:
        raise ValueError("nerf_pl_amd.render_rays: empty ray batch (the reference's "
                         "inference() concatenates an empty chunk list, rendering.py:161)")
    origins, dirs = rays[:, 0:3], rays[:, 3:6]
    dir_emb = embeddings[1](dirs)
    u1 = rng.rand((n, N_samples), dev) if perturb > 0 else None
    z = _stratified(rays, N_samples, use_disp, perturb, u1)
    cap["z_coarse"] = z
    xyz = origins.unsqueeze(1) + dirs.unsqueeze(1) * z.unsqueeze(2)
    result = {}
    noise_c = rng.randn((n, N_samples), dev) * noise_std
    if test_time:
        with torch.no_grad():
            raw = _mlp(models[0], embeddings, xyz, None, chunk, True)
            _, _, w_c = _composite(raw.view(n, N_samples), None, z, dirs, noise_c, white_back, True)
        result["opacity_coarse"] = w_c.sum(1)
    else:
        raw = _mlp(models[0], embeddings, xyz, dir_emb, chunk, False).view(n, N_samples, 4)
        rgb_c, depth_c, w_c = _composite(raw[..., 3], raw[..., :3], z, dirs, noise_c, white_back,
                                         False)
        result["rgb_coarse"] = rgb_c
        result["depth_coarse"] = depth_c
        result["opacity_coarse"] = w_c.sum(1)
    cap["weights_coarse"] = w_c
    if N_importance > 0:
        u = rng.rand((n, N_importance), dev)
        jit = rng.rand((n, N_importance), dev)
        z_imp = _importance(rays, w_c[:, 1:-1].detach(), N_importance, u, jit).detach()
        z_f, _ = torch.sort(torch.cat([z, z_imp], -1), -1)
        cap["z_fine"] = z_f
        s_f = z_f.shape[1]
        xyz_f = origins.unsqueeze(1) + dirs.unsqueeze(1) * z_f.unsqueeze(2)
        raw_f = _mlp(models[1], embeddings, xyz_f, dir_emb, chunk, False).view(n, s_f, 4)
        noise_f = rng.randn((n, s_f), dev) * noise_std
        rgb_f, depth_f, w_f = _composite(raw_f[..., 3], raw_f[..., :3], z_f, dirs, noise_f,
                                         white_back, False)
        cap["weights_fine"] = w_f
        result["rgb_fine"] = rgb_f
        result["depth_fine"] = depth_f
        result["opacity_fine"] = w_f.sum(1)
    return result
