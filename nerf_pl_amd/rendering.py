"""``render_rays`` and ``sample_pdf`` with the reference signatures
(models/rendering.py:14-48, 84-272), executed by the HIP kernels.

Drop-in notes
* ``render_rays(models, embeddings, rays, N_samples, use_disp, perturb,
  noise_std, N_importance, chunk, white_back, test_time)`` -- same positional
  order as the callers in train.py:55-64 / eval.py:69-79; returns the same
  dict keys.  One keyword is added: ``rng`` (see :mod:`nerf_pl_amd.rng`).
* ``chunk`` is accepted and ignored: the reference chunks the MLP only to bound
  memory (rendering.py:151-159); the fused kernel streams samples through
  registers and results do not depend on it.
* ``embeddings`` must be the reference defaults (Embedding(3,10), Embedding(3,4));
  the positional encoding is computed inside the fused MLP kernel.
* Everything runs on the HIP device that holds ``rays``; there is no CPU path.
"""
from __future__ import annotations

import torch

from . import ops
from .functions import composite_apply, mlp_apply
from .rng import (STREAM_JITTER, STREAM_NOISE_COARSE, STREAM_NOISE_FINE, STREAM_PERTURB,
                  STREAM_U, PhiloxRNG)

__all__ = ["render_rays", "sample_pdf"]


def _check_embeddings(embeddings):
    if embeddings is None:
        return
    e_xyz, e_dir = embeddings[0], embeddings[1]
    for e, nf in ((e_xyz, 10), (e_dir, 4)):
        if getattr(e, "N_freqs", nf) != nf or getattr(e, "in_channels", 3) != 3:
            raise NotImplementedError("nerf_pl_amd.render_rays: embeddings must be "
                                      "[Embedding(3, 10), Embedding(3, 4)] (train.py:34-35)")


def sample_pdf(rays, weights, N_importance, det=False, eps=1e-5, *, rng=None):
    """rendering.py:14-48 -- importance depths (N_rays, N_importance).

    ``weights`` are the (N_rays, N_samples-2) interior coarse weights, exactly
    as the reference receives them (``weights_coarse[:, 1:-1]``).  ``det`` is
    ignored, as in the reference."""
    del det
    if eps != 1e-5:
        raise NotImplementedError("nerf_pl_amd.sample_pdf: eps is fixed at 1e-5")
    rng = PhiloxRNG() if rng is None else rng
    n_rays, nb = weights.shape
    # the kernel reads bins 1..S-2 of a full (N_rays, S) weight row: pad both ends
    w_full = torch.nn.functional.pad(weights.detach(), (1, 1))
    u = rng.rand((n_rays, N_importance), rays.device)
    jit = rng.rand((n_rays, N_importance), rays.device)
    z, _ = ops.sample_pdf(w_full, rays, N_importance, u=u, jitter=jit, seed=rng.seed)
    return z


def render_rays(models, embeddings, rays, N_samples=64, use_disp=False, perturb=0, noise_std=1,
                N_importance=0, chunk=1024 * 32, white_back=False, test_time=False, *, rng=None,
                _capture=None):
    del chunk
    _check_embeddings(embeddings)
    rays = ops._dev(rays, "rays", 8)
    dev = rays.device
    n_rays = rays.shape[0]
    if n_rays == 0:
        # the reference fails here too: its chunk loop yields no chunk and
        # torch.cat([]) raises (rendering.py:150-161)
        raise ValueError("nerf_pl_amd.render_rays: empty ray batch (the reference's "
                         "inference() concatenates an empty chunk list, rendering.py:161)")
    rng = PhiloxRNG() if rng is None else rng
    seed = rng.seed

    # stratified coarse depths (rendering.py:216-232)
    u1 = rng.rand((n_rays, N_samples), dev) if perturb > 0 else None
    z_c = ops.coarse_z(rays, N_samples, use_disp, perturb, u=u1, seed=seed)
    noise_c = rng.randn((n_rays, N_samples), dev)

    cap = _capture if _capture is not None else {}
    cap["z_coarse"] = z_c
    result = {}
    if test_time:
        # sigma-only coarse pass, weights only (rendering.py:237-241)
        with torch.no_grad():
            sig = mlp_apply(models[0], rays=rays, z=z_c, spr=N_samples, sigma_only=True)
            _, _, opac_c, w_c = ops.composite_forward(sig, z_c, rays, noise_c, noise_std, seed,
                                                      STREAM_NOISE_COARSE, white_back,
                                                      weights_only=True)
        result["opacity_coarse"] = opac_c
    else:
        raw_c = mlp_apply(models[0], rays=rays, z=z_c, spr=N_samples)
        rgb_c, depth_c, opac_c, w_c = composite_apply(raw_c, z_c, rays, noise_c, noise_std, seed,
                                                      STREAM_NOISE_COARSE, white_back)
        result["rgb_coarse"] = rgb_c
        result["depth_coarse"] = depth_c
        result["opacity_coarse"] = opac_c

    if N_importance > 0:
        # sample_pdf + sort(cat[z, z_pdf]) (rendering.py:253-257), weights detached
        u = rng.rand((n_rays, N_importance), dev)
        jit = rng.rand((n_rays, N_importance), dev)
        _, z_f = ops.sample_pdf(w_c.detach(), rays, N_importance, u=u, jitter=jit, seed=seed,
                                z_coarse=z_c, merge=True)
        cap["weights_coarse"] = w_c
        cap["z_fine"] = z_f
        s_f = N_samples + N_importance
        noise_f = rng.randn((n_rays, s_f), dev)
        raw_f = mlp_apply(models[1], rays=rays, z=z_f, spr=s_f)
        rgb_f, depth_f, opac_f, _ = composite_apply(raw_f, z_f, rays, noise_f, noise_std, seed,
                                                    STREAM_NOISE_FINE, white_back)
        result["rgb_fine"] = rgb_f
        result["depth_fine"] = depth_f
        result["opacity_fine"] = opac_f
    return result


# stream ids documented in rng.py; referenced here so the kernel contract is visible
_STREAMS = (STREAM_PERTURB, STREAM_NOISE_COARSE, STREAM_U, STREAM_JITTER, STREAM_NOISE_FINE)
