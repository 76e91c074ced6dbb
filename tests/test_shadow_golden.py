"""Pins the shadow-mapping oracle (oracle/shadow_oracle.py) to fixtures produced
by running the reference (tests/golden/make_golden_shadow.py).  On the host
that wrote the fixtures the forward outputs were bit-identical; across hosts the
MLP GEMMs and row sums follow the CPU's SIMD width/BLAS (an ulp), which the
shadow reprojection amplifies (d/δ), so forward outputs are compared at 1e-5
relative and gradients at fp32 sum-order tolerance.  Same-host bit-exactness is
checked live by tests/test_oracle_live.py."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import nerf_oracle as O
from oracle import shadow_oracle as SO

SHADOW = os.path.join(GOLDEN, "shadow")
CASES = sorted(f[:-4] for f in os.listdir(SHADOW) if f.endswith(".npz"))


def load_shadow(name):
    with np.load(os.path.join(SHADOW, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def shadow_cfg(fx):
    c = fx["cfg"]
    return dict(wh=int(c[0]), N_samples=int(c[1]), N_importance=int(c[2]),
                light_importance=int(c[3]),
                method="shadow_method_1" if int(c[4]) == 1 else "shadow_method_2",
                sigma_bias=float(c[5]), perturb=float(c[6]), noise_std=float(c[7]),
                seeds=(int(c[8]), int(c[9])))


def run_oracle(fx, requires_grad=False):
    cfg = shadow_cfg(fx)
    n_models = 2 if cfg["N_importance"] > 0 else 1
    params = [O.make_params(s, sigma_bias=cfg["sigma_bias"]) for s in cfg["seeds"][:n_models]]
    if requires_grad:
        params = [{k: v.requires_grad_(True) for k, v in p.items()} for p in params]
    rng = O.ReplayRNG([fx[f"draw{i}"] for i in range(int(fx["n_draws"]))])
    t = torch.from_numpy
    cam = SO.render_rays(params, t(fx["rays"]), cfg["N_samples"], False, cfg["perturb"],
                         cfg["noise_std"], cfg["N_importance"], rng=rng)
    with torch.no_grad():
        light = SO.render_rays(params, t(fx["light_rays"]), cfg["N_samples"], False,
                               cfg["perturb"], cfg["noise_std"], cfg["light_importance"],
                               rng=rng)
    assert rng.exhausted()
    for k in ("depth_coarse", "depth_fine"):
        if k in cam and requires_grad:
            cam[k].retain_grad()
    depths = {k: cam[k] for k in ("depth_coarse", "depth_fine") if k in cam}
    ppc = {"eye_pos": t(fx["eye_pos"]), "camera": t(fx["camera"])}
    out = SO.efficient_sm(t(fx["pixels"]), t(fx["light_pixels"]), cam, light, ppc,
                          t(fx["light_eye"]), t(fx["light_camera"]), (cfg["wh"], cfg["wh"]),
                          cfg["N_importance"] > 0, cfg["light_importance"] > 0, cfg["method"])
    return cfg, params, cam, light, out, depths


@pytest.mark.parametrize("case", CASES)
def test_shadow_oracle_forward_matches(case):
    fx = load_shadow(case)
    _, _, _, light, out, _ = run_oracle(fx)
    for k, v in list(out.items()) + [("light_" + k, v) for k, v in light.items()]:
        ref = fx[k if k.startswith("light_") else f"out_{k}"]
        np.testing.assert_allclose(v.detach().numpy(), ref, rtol=1e-5,
                                   atol=1e-6 * max(1.0, float(np.abs(ref).max())), err_msg=k)


@pytest.mark.parametrize("case", CASES)
def test_shadow_oracle_gradients(case):
    fx = load_shadow(case)
    _, params, _, _, out, depths = run_oracle(fx, requires_grad=True)
    tgt = torch.from_numpy(fx["target"])
    loss = torch.mean((out["rgb_coarse"] - tgt) ** 2)
    if "rgb_fine" in out:
        loss = loss + torch.mean((out["rgb_fine"] - tgt) ** 2)
    assert loss.item() == pytest.approx(float(fx["loss"]), rel=1e-6)
    loss.backward()
    for k, d in depths.items():
        ref = fx[f"grad_{k}"]
        np.testing.assert_allclose(d.grad.numpy(), ref, rtol=1e-4,
                                   atol=1e-5 * max(1e-12, np.abs(ref).max()))
    for m, p in enumerate(params):
        for name, v in p.items():
            key = f"grad{m}_{name}"
            if key + "_sum" not in fx:
                assert v.grad is None, key
                continue
            g = v.grad.numpy().reshape(-1)
            scale = float(np.abs(fx.get(key + "_full", fx.get(key + "_val"))).max()) + 1e-30
            if key + "_full" in fx:
                np.testing.assert_allclose(g, fx[key + "_full"].reshape(-1), rtol=1e-3,
                                           atol=1e-4 * scale, err_msg=key)
            else:
                np.testing.assert_allclose(g[fx[key + "_idx"]], fx[key + "_val"], rtol=1e-3,
                                           atol=1e-4 * scale, err_msg=key)


def test_shadow_runs_split_like_reference():
    eye = torch.tensor([[0., 0, 1], [0, 0, 1], [1, 0, 0], [0, 0, 1], [0, 0, 1], [-0., 0, 1]])
    assert SO.shadow_runs(eye) == [(0, 2), (2, 3), (3, 6)]
