"""Shadow-mapping render path -- models/rendering_shadows.py (config 5,
train_efficient_sm.py), executed by the HIP kernels.

* ``render_rays(models, embeddings, rays, N_samples, use_disp, perturb,
  noise_std, N_importance, chunk, white_back, test_time,
  were_gradients_computed)`` -- :84-272: the sigma-only render.  Every MLP call
  is the fused sigma-only kernel (the reference calls
  ``model(x, sigma_only=True)`` for coarse and fine, :151-159); compositing
  produces depth / opacity / weights without an rgb head; returns
  ``depth_*``, ``opacity_*``, ``disp_map_*`` (``opacity_coarse`` only when
  ``test_time``).  Same RNG draw order as ``rendering.render_rays``.
* ``efficient_sm(...)`` -- :359-482: shadow maps of the camera depths against
  the light's depth map (``nr_sm_forward`` / ``nr_sm_backward``); the
  reference's per-ray ``torch.equal`` run-splitting loop (:377-396) becomes a
  device scan.  Differentiable in the camera depths and, when the light render
  was run with gradients (``--grad_on_light``, train_efficient_sm.py:158-162),
  in the light depths too.

``chunk`` and ``white_back`` are accepted and unused (the reference ignores
``white_back`` here too); ``rng`` is the added keyword of ``rendering.py``.
"""
from __future__ import annotations

import torch

from . import ops
from .efficient_shadow_mapping import EPSILON, _cam, normed_depth, shadow_map
from .functions import composite_apply, mlp_apply
from .rendering import _check_embeddings
from .rng import STREAM_NOISE_COARSE, STREAM_NOISE_FINE, PhiloxRNG

__all__ = ["render_rays", "render_rays_sharded", "efficient_sm"]


def _disp(depth, opac):
    # rendering_shadows.py:193, 1 / max(1e-10 * ones, depth / opac): the same
    # values (and NaN propagation) in three launches instead of five
    return torch.reciprocal(torch.clamp_min(depth / opac, 1e-10))


def render_rays(models, embeddings, rays, N_samples=64, use_disp=False, perturb=0, noise_std=1,
                N_importance=0, chunk=1024 * 32, white_back=False, test_time=False,
                were_gradients_computed=True, *, rng=None, _capture=None):
    del chunk, white_back, were_gradients_computed
    _check_embeddings(embeddings, models)
    rays = ops._dev(rays, "rays", 8)
    dev = rays.device
    n_rays = rays.shape[0]
    rng = PhiloxRNG() if rng is None else rng
    seed = rng.seed

    u1 = rng.rand((n_rays, N_samples), dev) if perturb > 0 else None
    z_c = ops.coarse_z(rays, N_samples, use_disp, perturb, u=u1, seed=seed)
    noise_c = rng.randn((n_rays, N_samples), dev)
    cap = _capture if _capture is not None else {}
    cap["z_coarse"] = z_c
    result = {}
    if test_time:
        with torch.no_grad():
            sig = mlp_apply(models[0], rays=rays, z=z_c, spr=N_samples, sigma_only=True)
            _, _, opac_c, w_c = ops.composite_forward(sig, z_c, rays, noise_c, noise_std, seed,
                                                      STREAM_NOISE_COARSE, False,
                                                      weights_only=True)
        result["opacity_coarse"] = opac_c
    else:
        sig = mlp_apply(models[0], rays=rays, z=z_c, spr=N_samples, sigma_only=True)
        _, depth_c, opac_c, w_c = composite_apply(sig, z_c, rays, noise_c, noise_std, seed,
                                                  STREAM_NOISE_COARSE, False)
        result["depth_coarse"] = depth_c
        result["opacity_coarse"] = opac_c
        result["disp_map_coarse"] = _disp(depth_c, opac_c)

    if N_importance > 0:
        u = rng.rand((n_rays, N_importance), dev)
        jit = rng.rand((n_rays, N_importance), dev)
        _, z_f = ops.sample_pdf(w_c.detach(), rays, N_importance, u=u, jitter=jit, seed=seed,
                                z_coarse=z_c, merge=True)
        cap["weights_coarse"] = w_c
        cap["z_fine"] = z_f
        s_f = N_samples + N_importance
        noise_f = rng.randn((n_rays, s_f), dev)
        sig_f = mlp_apply(models[1], rays=rays, z=z_f, spr=s_f, sigma_only=True)
        _, depth_f, opac_f, _ = composite_apply(sig_f, z_f, rays, noise_f, noise_std, seed,
                                                STREAM_NOISE_FINE, False)
        result["depth_fine"] = depth_f
        result["opacity_fine"] = opac_f
        result["disp_map_fine"] = _disp(depth_f, opac_f)
    return result


def render_rays_sharded(models, embeddings, rays, N_samples=64, use_disp=False, perturb=0,
                        noise_std=1, N_importance=0, chunk=1024 * 32, white_back=False,
                        test_time=False, *, group=None, rng=None, rng_for_rows=None):
    """The light-image render of train_efficient_sm.py:158-168 split over the
    ranks of ``group`` (SURVEY 8e, config 5 "phase 2"): each rank renders its
    contiguous slice of ``rays`` and all-gathers every output map
    (``distributed.sharded_map``), instead of every rank rendering the whole
    image as the reference does.  Per-ray results do not depend on the other
    rays of a call, so with the same random draws the gathered maps equal the
    replicated render bit for bit; ``rng_for_rows(lo, hi)`` supplies the draws
    of rows lo..hi (e.g. a ReplayRNG of the sliced tensors), else each rank
    draws from ``rng`` (default: its own Philox stream -- distribution-equivalent,
    like the reference's per-process generators).

    Follows the caller's grad mode like the reference: under ``torch.no_grad()``
    (the default light render, :164-168) nothing is recorded; with gradients
    enabled (``--grad_on_light``, :158-162) the gathered maps stay
    differentiable and their gradients are reduce-scattered back to the rank
    that rendered each row.  ``N_importance`` must be the same on every rank
    (checked: ``sharded_map`` raises on mismatched outputs)."""
    from .distributed import sharded_map

    def fn(r, rng=rng):
        return render_rays(models, embeddings, r.contiguous(), N_samples, use_disp, perturb,
                           noise_std, N_importance, chunk, white_back, test_time, False,
                           rng=rng)
    extra = (lambda lo, hi: {"rng": rng_for_rows(lo, hi)}) if rng_for_rows else None
    return sharded_map(fn, rays, group, extra)


def _ppc_arrays(ppc, n):
    if isinstance(ppc, (list, tuple)):        # train_efficient_sm.py:172-173 (batch_size 1)
        ppc = ppc[0]
    eye, cam = ppc["eye_pos"], ppc["camera"]
    if not isinstance(eye, torch.Tensor):
        eye, cam = torch.stack(list(eye)), torch.stack(list(cam))
    return eye.reshape(-1, 3), cam.reshape(-1, 3, 3)


def efficient_sm(cam_pixels, light_pixels, cam_results, light_results, ppc, light_ppc,
                 image_shape, fine_sampling, Light_N_importance, shadow_method):
    """rendering_shadows.py:359-482.  ``ppc`` = {'eye_pos': (B,3), 'camera':
    (B,3,3)} (collated per ray); ``light_ppc`` a ``Camera`` or the same dict for
    one camera.  Writes ``rgb_coarse`` (and ``rgb_fine``) = shadow + 1e-5 into
    ``cam_results`` and returns it."""
    d_c = cam_results["depth_coarse"]
    dev = d_c.device
    n = d_c.shape[0]
    eye, cams = _ppc_arrays(ppc, n)
    leye, lcam = _cam(light_ppc)
    leye = ops.to_device_f32(leye.reshape(3), dev)
    lcam = ops.to_device_f32(lcam.reshape(3, 3), dev)
    cam_pixels = ops.to_device_f32(cam_pixels, dev)
    light_pixels = ops.to_device_f32(light_pixels, dev).reshape(-1, 3)

    light_c = normed_depth(lcam, light_pixels, light_results["depth_coarse"])
    sm_c = shadow_map(d_c, cam_pixels, eye, cams, leye, lcam, light_c, image_shape,
                      shadow_method, out_eps=EPSILON)
    cam_results["rgb_coarse"] = sm_c
    if fine_sampling:
        light_f = (normed_depth(lcam, light_pixels, light_results["depth_fine"])
                   if Light_N_importance else light_c)
        cam_results["rgb_fine"] = shadow_map(cam_results["depth_fine"], cam_pixels, eye, cams,
                                             leye, lcam, light_f, image_shape, shadow_method,
                                             out_eps=EPSILON)
    return cam_results
