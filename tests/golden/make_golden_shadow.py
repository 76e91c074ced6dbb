"""Golden fixtures for the shadow-mapping path (config 5), made by running the
REFERENCE (``models/rendering_shadows.py``, ``models/efficient_shadow_mapping.py``,
``models/camera.py``) here, in the build container:

    python tests/golden/make_golden_shadow.py

One case = one step of ``train_efficient_sm.py:training_step`` (:143-199) on a
synthetic scene: the sigma-only render of a camera batch (with gradients), the
sigma-only render of the whole light image (no_grad, :166-170), ``efficient_sm``
(:175-182), the MSE loss (losses.py:4-14) and its backward.  Camera batches are
built as consecutive per-pose runs (pose A, pose B, pose A again) so the
reference's run-splitting loop (rendering_shadows.py:377-396) is exercised.

Recorded: every random draw (rand / randn / rand_like, in call order across the
camera and light renders), the inputs (rays, pixels, per-ray eye/camera, light
camera), render outputs, light normed depth map, the shadow outputs, the loss,
d(loss)/d(depth_coarse|fine) and parameter-gradient probes.  Same torchsearchsorted
shim as make_golden.py.  Output: ``tests/golden/shadow/<case>.npz`` (no pickle).

``--grad_on_light`` cases (``gol_*``; train_efficient_sm.py:158-162, the mode
60 of the reference's 63 launchers use) render the light image under autograd,
so the loss reaches both NeRFs through the light depths too; they also record
d(loss)/d(light depth_coarse|fine) and, per parameter tensor, the normwise
distance of the reference's fp32 gradient from the same step evaluated in
float64 by the oracle (``*_bound64``: the fp32 noise floor the GPU test bounds
its own deviation by, as tests/test_gpu_random.py does).

The cfg5-shaped cases (``cfg5_*``: a 64x64 light image -- 128x128 for
``cfg5_128_sm2``, BASELINE configs[4] exactly -- 512 camera rays, 64 + 64
samples, light 64 + 64, noise_std 0 as every reference launcher) hold too
many random draws to commit; they store each draw's kind, shape and checksum
and the test re-draws them from the recorded seed with the CPU generator
(``draws_seed``), checking the checksums first.

    python tests/golden/make_golden_shadow.py [case ...]   # default: all
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from make_golden import PROBE_PER_TENSOR, RecordingTorch, import_reference  # noqa: E402
from oracle import nerf_oracle as O  # noqa: E402
from oracle import shadow_oracle as SO  # noqa: E402
from oracle.nerf_oracle import make_params  # noqa: E402
from nerf_pl_amd.rays import (LEGO_CAMERA_ANGLE_X, blender_focal, get_ray_directions,  # noqa: E402
                              get_rays, pose_spherical)

OUT = os.path.join(HERE, "shadow")


def pixels_of(w, h):
    """datasets/blender_efficient_sm.py:193-198: [i + 0.5, j + 0.5, 1] per ray."""
    i, j = np.meshgrid(np.arange(h), np.arange(w), indexing="xy")
    i = torch.tensor(i) + 0.5
    j = torch.tensor(j) + 0.5
    return torch.stack([i, j, torch.ones_like(i)], axis=-1).view(-1, 3)


def scene(wh, Camera):
    """Light and camera poses, rays and pixels (datasets/blender_efficient_sm.py)."""
    w = h = wh
    focal = blender_focal(w)
    hfov = LEGO_CAMERA_ANGLE_X * 180. / np.pi
    dirs = get_ray_directions(h, w, focal)
    l2w = pose_spherical(35.0, -55.0, 4.0).float()
    light = Camera(hfov, (h, w))
    light.set_pose_using_blender_matrix(l2w, False)
    lo, ld = get_rays(dirs, l2w)
    light_rays = torch.cat([lo, ld, torch.ones_like(lo[:, :1]), 200. * torch.ones_like(lo[:, :1])], 1)
    cams = []
    for theta in (-20.0, 60.0):
        c2w = pose_spherical(theta, -30.0, 4.0).float()
        cam = Camera(hfov, (h, w))
        cam.set_pose_using_blender_matrix(c2w, False)
        o, d = get_rays(dirs, c2w)
        rays = torch.cat([o, d, torch.ones_like(o[:, :1]), 200. * torch.ones_like(o[:, :1])], 1)
        cams.append((cam, rays))
    return light, light_rays, pixels_of(w, h), cams


def draw_checksums(kind, t):
    """(float64 sum, first 8 values) of a recorded draw, for re-drawn replays."""
    flat = t.reshape(-1).double()
    return np.array([float(flat.sum()), float((flat * flat).sum())] + flat[:8].tolist())


def oracle_bound64(fx_out, rays, light_rays, pix, light_pixels, ppc, light, draws, cfg,
                   ref_grads, probes, grad_on_light):
    """Per parameter tensor: |g_ref32 - g_oracle64| / |g_ref32|, full tensor and
    on the recorded probes -- the same step (same draws) in float64."""
    wh, S, I, LI, method, sigma_bias, perturb, noise_std = cfg
    dt = torch.float64
    n_models = 2 if I > 0 or LI > 0 else 1
    params = [{k: v.to(dt).requires_grad_(True) for k, v in make_params(s, sigma_bias).items()}
              for s in (31, 32)[:n_models]]
    rng = O.ReplayRNG([d for _, d in draws])
    rng._queue = [q.to(dt) for q in rng._queue]
    cam = SO.render_rays(params, rays.to(dt), S, False, perturb, noise_std, I, rng=rng)
    with torch.set_grad_enabled(grad_on_light):     # the reference's light render mode
        lres = SO.render_rays(params, light_rays.to(dt), S, False, perturb, noise_std, LI, rng=rng)
    assert rng.exhausted()
    ppc64 = {"eye_pos": ppc["eye_pos"].to(dt), "camera": ppc["camera"].to(dt)}
    out = SO.efficient_sm(pix.to(dt), light_pixels.to(dt), cam, lres, ppc64,
                          light.eye_pos.to(dt), light.camera.to(dt), (wh, wh), I > 0, LI > 0,
                          method)
    tgt = torch.from_numpy(fx_out["target"]).to(dt)
    loss = torch.mean((out["rgb_coarse"] - tgt) ** 2)
    if "rgb_fine" in out:
        loss = loss + torch.mean((out["rgb_fine"] - tgt) ** 2)
    loss.backward()
    for m, p in enumerate(params):
        for name, w in p.items():
            key = f"grad{m}_{name}"
            if key not in ref_grads:
                continue
            g32 = ref_grads[key].astype(np.float64).reshape(-1)
            g64 = (w.grad.reshape(-1).numpy() if w.grad is not None else np.zeros_like(g32))
            fx_out[key + "_bound64"] = np.array(np.linalg.norm(g32 - g64) /
                                                (np.linalg.norm(g32) + 1e-300))
            if key in probes:
                idx = probes[key]
                fx_out[key + "_pbound64"] = np.array(np.linalg.norm(g32[idx] - g64[idx]) /
                                                     (np.linalg.norm(g32[idx]) + 1e-300))


def run_case(ref, name, wh, runs, N_samples, N_importance, light_importance, method,
             sigma_bias, perturb=1.0, noise_std=1.0, seed=77, grad_on_light=False,
             store_draws=True, n_probe=PROBE_PER_TENSOR):
    ref_nerf, rs, camera_mod = ref
    torch.manual_seed(seed)
    light, light_rays, pixels, cams = scene(wh, camera_mod.Camera)
    g = torch.Generator().manual_seed(seed)
    rays, pix, eyes, mats = [], [], [], []
    for pose, count in runs:
        cam, crays = cams[pose]
        idx = torch.randperm(crays.shape[0], generator=g)[:count]
        rays.append(crays[idx]); pix.append(pixels[idx])
        eyes.append(cam.eye_pos.expand(count, 3)); mats.append(cam.camera.expand(count, 3, 3))
    rays, pix = torch.cat(rays).contiguous(), torch.cat(pix).contiguous()
    ppc = {"eye_pos": torch.cat(eyes).contiguous(), "camera": torch.cat(mats).contiguous()}

    models = []
    n_models = 2 if N_importance > 0 or light_importance > 0 else 1
    for m, s in enumerate((31, 32)[:n_models]):
        net = ref_nerf.NeRF()
        net.load_state_dict(make_params(s, sigma_bias=sigma_bias))
        models.append(net)
    emb = [ref_nerf.Embedding(3, 10), ref_nerf.Embedding(3, 4)]

    torch.manual_seed(seed)                  # the render draws (re-drawable from this seed)
    rec = RecordingTorch()
    saved = rs.torch
    rs.torch = rec
    try:
        cam_res = rs.render_rays(models, emb, rays, N_samples, False, perturb, noise_std,
                                 N_importance, 32768, False)
        if grad_on_light:       # train_efficient_sm.py:158-162
            light_res = rs.render_rays(models, emb, light_rays, N_samples, False, perturb,
                                       noise_std, light_importance, 32768, False,
                                       were_gradients_computed=False)
        else:                   # :164-168
            with torch.no_grad():
                light_res = rs.render_rays(models, emb, light_rays, N_samples, False, perturb,
                                           noise_std, light_importance, 32768, False)
    finally:
        rs.torch = saved
    for k in ("depth_coarse", "depth_fine"):
        if k in cam_res:
            cam_res[k].retain_grad()
        if grad_on_light and k in light_res:
            light_res[k].retain_grad()
    depths = {k: cam_res[k] for k in ("depth_coarse", "depth_fine") if k in cam_res}
    light_depths = ({k: light_res[k] for k in ("depth_coarse", "depth_fine") if k in light_res}
                    if grad_on_light else {})
    cam_out = rs.efficient_sm(pix, pixels, cam_res, light_res, ppc, light, image_shape=(wh, wh),
                              fine_sampling=N_importance > 0,
                              Light_N_importance=light_importance > 0, shadow_method=method)
    target = torch.rand(rays.shape[0], 3, generator=g)
    loss = torch.mean((cam_out["rgb_coarse"] - target) ** 2)
    if "rgb_fine" in cam_out:
        loss = loss + torch.mean((cam_out["rgb_fine"] - target) ** 2)
    loss.backward()

    out = {
        "cfg": np.array([wh, N_samples, N_importance, light_importance,
                         1 if method == "shadow_method_1" else 2, sigma_bias, perturb,
                         noise_std, 31, 32, 1 if grad_on_light else 0], dtype=np.float64),
        "rays": rays.numpy(), "pixels": pix.numpy(), "light_rays": light_rays.numpy(),
        "light_pixels": pixels.numpy(), "eye_pos": ppc["eye_pos"].numpy(),
        "camera": ppc["camera"].numpy(), "light_eye": light.eye_pos.numpy(),
        "light_camera": light.camera.numpy(), "target": target.numpy(),
        "loss": np.array(loss.item(), dtype=np.float64), "n_draws": np.array(len(rec.draws)),
    }
    if not store_draws:
        out["draws_seed"] = np.array(seed)
        # the re-draw must reproduce the recorded stream
        torch.manual_seed(seed)
        for kind, t in rec.draws:
            again = torch.randn(t.shape) if kind == "randn" else torch.rand(t.shape)
            assert torch.equal(again, t), f"{name}: re-drawn {kind} {tuple(t.shape)} differs"
    for i, (kind, t) in enumerate(rec.draws):
        if store_draws:
            out[f"draw{i}"] = t.numpy()
        else:
            out[f"draw{i}_shape"] = np.array(t.shape, dtype=np.int64)
            out[f"draw{i}_sum"] = draw_checksums(kind, t)
        out[f"draw{i}_kind"] = np.array(kind)
    for k, v in cam_out.items():
        out[f"out_{k}"] = v.detach().numpy()
    for k, v in light_res.items():
        out[f"light_{k}"] = v.detach().numpy()
    for k, v in depths.items():
        out[f"grad_{k}"] = v.grad.numpy()
    for k, v in light_depths.items():
        out[f"grad_light_{k}"] = v.grad.numpy()
    pg = np.random.Generator(np.random.PCG64(5))
    ref_grads, probes = {}, {}
    for m, net in enumerate(models):
        for pname, p in net.named_parameters():
            if p.grad is None:
                continue
            gr = p.grad.detach().numpy().astype(np.float32)
            key = f"grad{m}_{pname}"
            ref_grads[key] = gr
            out[key + "_sum"] = np.array(gr.astype(np.float64).sum())
            out[key + "_l2"] = np.array(np.sqrt((gr.astype(np.float64) ** 2).sum()))
            flat = gr.reshape(-1)
            if flat.size <= 1024:
                out[key + "_full"] = gr
            else:
                idx = np.sort(pg.choice(flat.size, n_probe, replace=False))
                out[key + "_idx"] = idx.astype(np.int64)
                out[key + "_val"] = flat[idx]
                probes[key] = idx
    if True:        # every case: the fp32 noise floor of its gradients
        del models, cam_res, light_res, cam_out, loss
        oracle_bound64(out, rays, light_rays, pix, pixels, ppc, light, rec.draws,
                       (wh, N_samples, N_importance, light_importance, method, sigma_bias,
                        perturb, noise_std), ref_grads, probes, grad_on_light)
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: {len(rec.draws)} draws, loss {float(out['loss']):.6f}, "
          f"{os.path.getsize(path) / 1024:.1f} KiB")


CASES = {
    # config 5 defaults: shadow_method_2, Light_N_importance 0 (opt.py:95,104)
    "sm2_light_coarse": (16, [(0, 40), (1, 30), (0, 26)], 32, 32, 0, "shadow_method_2",
                         dict(sigma_bias=0.5)),
    "sm1_light_fine": (16, [(1, 50), (0, 46)], 32, 16, 16, "shadow_method_1",
                       dict(sigma_bias=1.0)),
    "sm2_coarse_only": (12, [(0, 64)], 24, 0, 0, "shadow_method_2", dict(sigma_bias=0.8)),
    # --grad_on_light (train_efficient_sm.py:158-162)
    "gol_sm2_light_fine": (16, [(0, 40), (1, 30), (0, 26)], 32, 32, 32, "shadow_method_2",
                           dict(sigma_bias=0.5, noise_std=0.0, grad_on_light=True,
                                n_probe=2048)),
    "gol_sm2_light_coarse": (16, [(1, 64), (0, 32)], 32, 16, 0, "shadow_method_2",
                             dict(sigma_bias=0.7, grad_on_light=True, n_probe=2048)),
    "gol_sm1_light_fine": (16, [(0, 50), (1, 46)], 32, 16, 16, "shadow_method_1",
                           dict(sigma_bias=1.0, noise_std=0.0, grad_on_light=True,
                                n_probe=2048)),
    # cfg5-shaped: 64^2 light image, 512 camera rays in three runs, 64 + 64
    "cfg5_sm2": (64, [(0, 200), (1, 180), (0, 132)], 64, 64, 64, "shadow_method_2",
                 dict(sigma_bias=0.5, noise_std=0.0, store_draws=False, seed=78)),
    # BASELINE configs[4] exactly: the 128x128 light image (16,384 light rays)
    "cfg5_128_sm2": (128, [(0, 300), (1, 212)], 64, 64, 64, "shadow_method_2",
                     dict(sigma_bias=0.5, noise_std=0.0, store_draws=False, seed=80)),
    "cfg5_gol_sm2": (64, [(1, 256), (0, 256)], 64, 64, 64, "shadow_method_2",
                     dict(sigma_bias=0.5, noise_std=0.0, store_draws=False, seed=79,
                          grad_on_light=True, n_probe=2048)),
}


def augment_bound64(name):
    """Add the *_bound64 / *_pbound64 noise floors to a committed fixture
    without rewriting its arrays (for fixtures written on another host, whose
    reference outputs this host would reproduce only to an ulp): the float64
    oracle's gradient against the fixture's recorded fp32 probes."""
    import test_shadow_golden as TSG
    path = os.path.join(OUT, f"{name}.npz")
    fx = TSG.load_shadow(name)
    cfg, params, _, _, out, _, _ = TSG.run_oracle(fx, requires_grad=True, dtype=torch.float64)
    TSG._loss(out, fx, torch.float64).backward()
    for m, p in enumerate(params):
        for pname, w in p.items():
            key = f"grad{m}_{pname}"
            if key + "_sum" not in fx:
                continue
            g64 = w.grad.reshape(-1).numpy()
            if key + "_full" in fx:
                g32, idx = fx[key + "_full"].reshape(-1).astype(np.float64), None
            else:
                g32, idx = fx[key + "_val"].astype(np.float64), fx[key + "_idx"]
            d = np.linalg.norm(g32 - (g64 if idx is None else g64[idx])) / (np.linalg.norm(g32) + 1e-300)
            fx[key + ("_bound64" if idx is None else "_pbound64")] = np.array(d)
    np.savez_compressed(path, **fx)
    print(f"{name}: noise floors added")


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    if sys.argv[1:2] == ["--augment"]:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        for name in sys.argv[2:]:
            augment_bound64(name)
        return
    ref_nerf, _ = import_reference()
    import models.camera as camera_mod             # noqa: E402
    import models.rendering_shadows as rs          # noqa: E402
    ref = (ref_nerf, rs, camera_mod)
    for name in sys.argv[1:] or list(CASES):
        wh, runs, S, I, LI, method, kw = CASES[name]
        run_case(ref, name, wh, runs, S, I, LI, method, **kw)


if __name__ == "__main__":
    main()
