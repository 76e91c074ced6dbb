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
* with the reference defaults (Embedding(3,10), Embedding(3,4), NeRF()) the
  positional encoding and the MLP run in the fused kernels; any other
  embeddings or NeRF configuration takes the composable path (the reference's
  ``inference`` sequence -- xyz, embeddings, model -- on device GEMMs), with
  sampling and compositing on the same HIP kernels either way.
* Everything runs on the HIP device that holds ``rays``.  A batch on the host
  (BASELINE configs[0], "PyTorch CPU, plumbing") runs nerf_pl_amd.host: the
  reference's sequence in PyTorch CPU ops, as the reference itself runs on
  whichever device ``rays`` lives (rendering.py:178, 216, 231).  The choice is
  the batch's device alone: a HIP-device batch runs the kernels or raises.
"""
from __future__ import annotations

import functools
import os

import torch

from . import ops
from .functions import composite_apply, mlp_apply
from .rng import (STREAM_JITTER, STREAM_NOISE_COARSE, STREAM_NOISE_FINE, STREAM_PERTURB,
                  STREAM_U, PhiloxRNG, TorchRNG)

__all__ = ["render_rays", "sample_pdf"]

# A training call runs the fine pass (MLP forward + compositing) on a side
# stream, so that autograd -- which runs every backward node on the stream its
# forward ran on -- executes the fine model's backward there too, beside the
# coarse model's on the caller's stream: the two chains are independent after
# sample_pdf's detach (rendering.py:253-255) and fill each other's kernel
# tails.  NERF_PL_AMD_FINE_STREAM=0 keeps everything on the caller's stream.
FINE_STREAM = os.environ.get("NERF_PL_AMD_FINE_STREAM", "1") != "0"
# HIP priority of that stream (-1 high, 0 normal).  Same-box A/B
# (profiles/r06/ab_stream): side stream 510.4k vs one stream 497.0k rays/s;
# priority -1 511.0k (no difference); the coarse pass on the side stream
# instead (its backward then queues behind the fine one's) 507.1k vs 507.9k
FINE_STREAM_PRIORITY = int(os.environ.get("NERF_PL_AMD_FINE_STREAM_PRIORITY", "0"))


# one-shot callables run right before the next fine pass is enqueued (after the
# coarse pass): pipeline.PipelinedStep on the distributed path defers the fine
# model's all-reduce and Adam there, so that issuing the collective -- which
# waits on the host for the fine backward -- comes after the next step's
# coarse pass has been enqueued
BEFORE_FINE = []


@functools.lru_cache(maxsize=None)
def _side_stream(device_index: int):
    return torch.cuda.Stream(device=torch.device("cuda", device_index),
                             priority=FINE_STREAM_PRIORITY)


def _fused_ok(models, embeddings):
    """True when the fused kernels implement this call: default NeRF models
    and the reference's embeddings (train.py:34-35)."""
    if any(m is not None and not getattr(m, "_fused", False) for m in models):
        return False
    if embeddings is None:
        return True
    for e, nf in ((embeddings[0], 10), (embeddings[1], 4)):
        if (getattr(e, "N_freqs", None) != nf or getattr(e, "in_channels", None) != 3
                or not getattr(e, "logscale", True)):
            return False
    return True


def _check_embeddings(embeddings, models=()):
    """The shadow-mapping path (rendering_shadows) runs the fused kernels only."""
    if not _fused_ok(models, embeddings):
        raise NotImplementedError("nerf_pl_amd.rendering_shadows: the default NeRF() and "
                                  "[Embedding(3, 10), Embedding(3, 4)] only (train_efficient_sm.py:45-56)")


def _composable_mlp(model, embeddings, rays, z, spr, sigma_only=False):
    """rendering.py:141-161 for a configuration the fused kernels do not
    implement: xyz = o + d z (:234, multiply then add), the embeddings, and the
    model on the embedded input (dir embedding repeated per sample, :145)."""
    if embeddings is None:
        raise ValueError("nerf_pl_amd.render_rays: a non-default NeRF needs its embeddings")
    n = rays.shape[0]
    dz = rays[:, None, 3:6] * z.reshape(n, spr)[:, :, None]
    xyz = (rays[:, None, 0:3] + dz).reshape(-1, 3)
    e = embeddings[0](xyz)
    if sigma_only:
        return model(e, sigma_only=True)
    d = torch.repeat_interleave(embeddings[1](rays[:, 3:6]), repeats=spr, dim=0)
    return model(torch.cat([e, d], 1))


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
    if isinstance(rays, torch.Tensor) and rays.device.type == "cpu":
        if rays.dtype != torch.float32:
            raise TypeError(f"rays: expected float32, got {rays.dtype}")
        if rays.dim() != 2 or rays.shape[-1] != 8:
            raise ValueError(f"rays: expected (N, 8), got {tuple(rays.shape)}")
        from .host import render_rays_host
        return render_rays_host(models, embeddings, rays, N_samples, use_disp, perturb, noise_std,
                                N_importance, chunk, white_back, test_time,
                                TorchRNG() if rng is None else rng, _capture)
    del chunk
    fused = _fused_ok(models, embeddings)

    def mlp(model, z, spr, sigma_only=False):
        if fused:
            return mlp_apply(model, rays=rays, z=z, spr=spr, sigma_only=sigma_only)
        return _composable_mlp(model, embeddings, rays, z, spr, sigma_only)

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
            sig = mlp(models[0], z_c, N_samples, sigma_only=True)
            _, _, opac_c, w_c = ops.composite_forward(sig, z_c, rays, noise_c, noise_std, seed,
                                                      STREAM_NOISE_COARSE, white_back,
                                                      weights_only=True)
        result["opacity_coarse"] = opac_c
    else:
        raw_c = mlp(models[0], z_c, N_samples)
        rgb_c, depth_c, opac_c, w_c = composite_apply(raw_c, z_c, rays, noise_c, noise_std, seed,
                                                      STREAM_NOISE_COARSE, white_back)
        result["rgb_coarse"] = rgb_c
        result["depth_coarse"] = depth_c
        result["opacity_coarse"] = opac_c

    cap["weights_coarse"] = w_c
    if N_importance > 0:
        # sample_pdf + sort(cat[z, z_pdf]) (rendering.py:253-257), weights detached
        u = rng.rand((n_rays, N_importance), dev)
        jit = rng.rand((n_rays, N_importance), dev)
        _, z_f = ops.sample_pdf(w_c.detach(), rays, N_importance, u=u, jitter=jit, seed=seed,
                                z_coarse=z_c, merge=True)
        cap["z_fine"] = z_f
        s_f = N_samples + N_importance

        def fine_pass():
            noise_f = rng.randn((n_rays, s_f), dev)
            raw_f = mlp(models[1], z_f, s_f)
            return composite_apply(raw_f, z_f, rays, noise_f, noise_std, seed, STREAM_NOISE_FINE,
                                   white_back)

        while BEFORE_FINE:
            BEFORE_FINE.pop(0)()
        if FINE_STREAM and torch.is_grad_enabled() and any(
                p.requires_grad for p in models[1].parameters()):
            main = torch.cuda.current_stream(dev)
            side = _side_stream(dev.index)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                outs = fine_pass()
            main.wait_stream(side)
            # the caching allocator must not hand out blocks one stream still uses
            for t in (rays, z_f):
                t.record_stream(side)
            for t in outs:
                t.record_stream(main)
            rgb_f, depth_f, opac_f, w_f = outs
        else:
            rgb_f, depth_f, opac_f, w_f = fine_pass()
        cap["weights_fine"] = w_f
        result["rgb_fine"] = rgb_f
        result["depth_fine"] = depth_f
        result["opacity_fine"] = opac_f
    return result


# stream ids documented in rng.py; referenced here so the kernel contract is visible
_STREAMS = (STREAM_PERTURB, STREAM_NOISE_COARSE, STREAM_U, STREAM_JITTER, STREAM_NOISE_FINE)
