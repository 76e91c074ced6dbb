"""CPU oracle for the shadow-mapping path.

TEST INFRASTRUCTURE ONLY -- imported by ``tests/`` alone, never by the
product package (which has no CPU path).

Restates, in PyTorch-CPU fp32 with the reference's op order:

* ``models/rendering_shadows.py:84-272``  ``render_rays``: the sigma-only
  render of depth / opacity / disparity (no rgb head), same RNG draw order as
  ``models/rendering.py`` (rand(B,S) if perturb, randn(B,S), rand(B,I),
  rand_like(B,I), randn(B,S+I));
* ``models/rendering_shadows.py:359-482``  ``efficient_sm``: per-run shadow
  mapping of camera depths against the light's depth map, where a run is a
  maximal stretch of consecutive rays whose eye position equals the run's first
  (the ``torch.equal`` split loop at :377-396);
* ``models/efficient_shadow_mapping.py:10-130`` (``normalize_min_max``,
  ``get_normed_w``, ``get_diff_projections``, ``get_projected_depths``,
  ``generate_shadow_map``) and ``models/camera.py:121-132``
  (``get_transformation_to``).

Pinned by ``tests/test_shadow_golden.py`` against fixtures produced by running
the reference (``tests/golden/make_golden_shadow.py``).
"""
from __future__ import annotations

from typing import List, Optional

import torch

from .nerf_oracle import (DIR_FREQS, Params, TorchRNG, coarse_z, embed, run_mlp,
                          sample_pdf)

EPSILON = 1e-5          # efficient_shadow_mapping.py:8 and rendering_shadows.py:356


# --------------------------------------------------------------------------
# models/rendering_shadows.py:84-272 -- sigma-only render
# --------------------------------------------------------------------------
def _sigma_inference(p: Params, xyz, rays_d, z_vals, chunk, noise_std, rng, weights_only):
    """rendering_shadows.py:117-198."""
    n_rays, n_s = xyz.shape[:2]
    sig = run_mlp(p, xyz, None, chunk, sigma_only=True).view(n_rays, n_s)
    deltas = z_vals[:, 1:] - z_vals[:, :-1]
    deltas = torch.cat([deltas, 1e10 * torch.ones_like(deltas[:, :1])], -1)
    deltas = deltas * torch.norm(rays_d.unsqueeze(1), dim=-1)
    noise = rng.randn(tuple(sig.shape)) * noise_std
    alphas = 1 - torch.exp(-deltas * torch.relu(sig + noise))
    shifted = torch.cat([torch.ones_like(alphas[:, :1]), 1 - alphas + 1e-10], -1)
    weights = alphas * torch.cumprod(shifted, -1)[:, :-1]
    if weights_only:
        return weights
    depth = torch.sum(weights * z_vals, -1)
    disp = 1. / torch.max(1e-10 * torch.ones_like(depth), depth / torch.sum(weights, -1))
    return depth, weights, disp


def render_rays(models: List[Params], rays, N_samples=64, use_disp=False, perturb=0,
                noise_std=1, N_importance=0, chunk=1024 * 32, white_back=False,
                test_time=False, rng=None, capture: Optional[dict] = None):
    """rendering_shadows.py:84-272 (``white_back`` is unused there too)."""
    del white_back
    rng = rng if rng is not None else TorchRNG()
    cap = capture if capture is not None else {}
    rays_o, rays_d = rays[:, 0:3], rays[:, 3:6]
    embed(rays_d, DIR_FREQS)                 # computed and unused by the reference (:213)
    z = coarse_z(rays, N_samples, use_disp, perturb, rng)
    cap["z_coarse"] = z
    xyz = rays_o.unsqueeze(1) + rays_d.unsqueeze(1) * z.unsqueeze(2)
    if test_time:
        w_c = _sigma_inference(models[0], xyz, rays_d, z, chunk, noise_std, rng, True)
        result = {"opacity_coarse": w_c.sum(1)}
    else:
        d_c, w_c, disp_c = _sigma_inference(models[0], xyz, rays_d, z, chunk, noise_std, rng,
                                            False)
        result = {"depth_coarse": d_c, "opacity_coarse": w_c.sum(1), "disp_map_coarse": disp_c}
    cap["weights_coarse"] = w_c
    if N_importance > 0:
        z_pdf = sample_pdf(rays, w_c[:, 1:-1], N_importance, rng).detach()
        cap["z_pdf"] = z_pdf
        z_f, _ = torch.sort(torch.cat([z, z_pdf], -1), -1)
        cap["z_fine"] = z_f
        xyz_f = rays_o.unsqueeze(1) + rays_d.unsqueeze(1) * z_f.unsqueeze(2)
        d_f, w_f, disp_f = _sigma_inference(models[1], xyz_f, rays_d, z_f, chunk, noise_std,
                                            rng, False)
        result["depth_fine"] = d_f
        result["opacity_fine"] = w_f.sum(1)
        result["disp_map_fine"] = disp_f
    return result


# --------------------------------------------------------------------------
# models/efficient_shadow_mapping.py + camera.py
# --------------------------------------------------------------------------
def normalize_min_max(t, new_max=1.0, new_min=0.0):
    """efficient_shadow_mapping.py:10-11."""
    return (t - t.min()) / (t.max() - t.min() + EPSILON) * (new_max - new_min) + new_min


def get_normed_w(camera: torch.Tensor, pixel_depth: torch.Tensor) -> torch.Tensor:
    """efficient_shadow_mapping.py:41-58: [i, j, 1, depth / (|M p| + 1e-5)]."""
    px = pixel_depth[:, :3]
    coords = torch.sum(px[..., None, :] * camera, -1)
    norm = torch.linalg.norm(coords, dim=1)
    norm = norm + EPSILON * torch.ones_like(norm)
    return torch.cat([px, (pixel_depth[:, 3] / norm).view(-1, 1)], dim=1)


def transformation_to(eye, camera, light_eye, light_camera):
    """camera.py:121-132: R = M_L^-1 M, Q = M_L^-1 (O - L)."""
    ml_inv = torch.inverse(light_camera)
    return ml_inv @ camera, ml_inv @ (eye - light_eye)


def get_diff_projections(pixels, w_cam, R, Q):
    """efficient_shadow_mapping.py:61-82 -> K = [u_l, v_l, w_l]."""
    proj = torch.sum(pixels[..., None, :] * R, -1)
    coords = torch.stack([w_cam, w_cam, w_cam], axis=1) * proj + Q
    ul, vl, wl = torch.unbind(coords, dim=1)
    return torch.stack([torch.div(ul, wl), torch.div(vl, wl), wl], axis=1)


def get_projected_depths(res, K, w_light):
    """efficient_shadow_mapping.py:84-101 (clamped nearest-texel gather)."""
    w, h = res
    ul_, vl_, wl = torch.unbind(K, dim=1)
    ul = torch.minimum(torch.tensor(w - 1.), torch.maximum(torch.tensor(0.), ul_))
    vl = torch.minimum(torch.tensor(h - 1.), torch.maximum(torch.tensor(0.), vl_))
    return wl, w_light.view(w, h)[vl.to(torch.long), ul.to(torch.long)]


def generate_shadow_map(wl, wlb, delta=1e-2, epsilon=0.0, new_min=0.0, new_max=1.0,
                        sigmoid=False, mode="shadow_method_1"):
    """efficient_shadow_mapping.py:104-130."""
    diff = wl - wlb
    if mode == "shadow_method_1":
        diff = torch.max(diff / delta, torch.tensor(epsilon))
    elif mode == "shadow_method_2":
        # the reference ignores new_min/new_max here (:120 calls the defaults)
        diff = normalize_min_max(diff)
        if sigmoid:
            diff = torch.sigmoid(diff)
    else:
        raise ValueError(f"{mode} not found")
    return torch.stack([diff, diff, diff], dim=1).clip(0.0, 1.0)


def run_shadow_mapping(res, eye, camera, light_eye, light_camera, mesh_range_cam,
                       normed_light_w, mode="shadow_method_1", delta=1e-2, epsilon=0.0,
                       new_min=0.0, new_max=1.0, sigmoid=False):
    """efficient_shadow_mapping.py:19-38 for one camera."""
    w_cam = get_normed_w(camera, mesh_range_cam)
    R, Q = transformation_to(eye, camera, light_eye, light_camera)
    K = get_diff_projections(w_cam[:, :3], w_cam[:, 3], R, Q)
    wl, wlb = get_projected_depths(res, K, normed_light_w)
    return generate_shadow_map(wl, wlb, delta, epsilon, new_min, new_max, sigmoid, mode)


def shadow_runs(eye_pos: torch.Tensor):
    """Run boundaries of rendering_shadows.py:377-396: [(start, end), ...]."""
    runs, start = [], 0
    for i in range(eye_pos.shape[0]):
        if not torch.equal(eye_pos[start], eye_pos[i]):
            runs.append((start, i))
            start = i
    runs.append((start, eye_pos.shape[0]))
    return runs


def _sm_batched(res, ppc, light_eye, light_cam, mesh_range_cam, normed_light_w, mode):
    parts = []
    for s, e in shadow_runs(ppc["eye_pos"]):
        parts.append(run_shadow_mapping(res, ppc["eye_pos"][s], ppc["camera"][s], light_eye,
                                        light_cam, mesh_range_cam[s:e], normed_light_w, mode))
    return torch.cat(parts, 0)


def efficient_sm(cam_pixels, light_pixels, cam_results, light_results, ppc, light_eye,
                 light_cam, image_shape, fine_sampling, Light_N_importance, shadow_method):
    """rendering_shadows.py:359-482.  ``ppc`` = {'eye_pos': (B,3), 'camera': (B,3,3)};
    the light camera is given as (eye (3,), matrix (3,3))."""
    out = dict(cam_results)
    d_c = cam_results["depth_coarse"]
    mesh_c = torch.cat([cam_pixels, d_c.view(-1, 1)], dim=1)
    light_c = get_normed_w(light_cam, torch.cat([light_pixels,
                                                 light_results["depth_coarse"].view(-1, 1)], 1))
    sm_c = _sm_batched(image_shape, ppc, light_eye, light_cam, mesh_c, light_c[:, 3],
                       shadow_method).view(-1, 3)
    out["rgb_coarse"] = sm_c + EPSILON * torch.ones_like(sm_c)
    if fine_sampling:
        mesh_f = torch.cat([cam_pixels, cam_results["depth_fine"].view(-1, 1)], dim=1)
        if Light_N_importance:
            light_f = get_normed_w(light_cam, torch.cat(
                [light_pixels, light_results["depth_fine"].view(-1, 1)], 1))
        else:
            light_f = light_c
        sm_f = _sm_batched(image_shape, ppc, light_eye, light_cam, mesh_f, light_f[:, 3],
                           shadow_method).view(-1, 3)
        out["rgb_fine"] = sm_f + EPSILON * torch.ones_like(sm_c)
    return out
