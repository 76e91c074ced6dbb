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
                seeds=(int(c[8]), int(c[9])),
                grad_on_light=len(c) > 10 and bool(c[10]))


def fixture_draws(fx):
    """The reference's random draws of a case, in call order: stored, or (the
    cfg5-shaped cases) re-drawn from the recorded seed with the CPU generator
    and checked against the recorded checksums."""
    n = int(fx["n_draws"])
    if "draws_seed" not in fx:
        return [fx[f"draw{i}"] for i in range(n)]
    torch.manual_seed(int(fx["draws_seed"]))
    out = []
    for i in range(n):
        shape = tuple(int(v) for v in fx[f"draw{i}_shape"])
        t = torch.randn(shape) if str(fx[f"draw{i}_kind"]) == "randn" else torch.rand(shape)
        flat = t.reshape(-1).double()
        got = np.array([float(flat.sum()), float((flat * flat).sum())] + flat[:8].tolist())
        np.testing.assert_allclose(got, fx[f"draw{i}_sum"], rtol=1e-12, atol=0,
                                   err_msg=f"re-drawn draw {i} differs from the reference's")
        out.append(t.numpy())
    return out


def n_models(cfg):
    return 2 if cfg["N_importance"] > 0 or cfg["light_importance"] > 0 else 1


def n_camera_draws(cfg):
    """draws of the camera render (rendering.py order): rand(B,S) if perturb,
    randn(B,S), and rand(B,I), rand_like(B,I), randn(B,S+I) if I > 0"""
    return (1 if cfg["perturb"] > 0 else 0) + 1 + (3 if cfg["N_importance"] > 0 else 0)


def run_oracle(fx, requires_grad=False, dtype=torch.float32, light_rows=None):
    """The oracle's training step on a fixture.  ``light_rows=k``: the light
    render is checked on its first k rows only (rendered with those rows of
    the draws -- rays are independent) and efficient_sm reads the fixture's
    (the reference's) light maps; the light outputs returned are the k rows."""
    cfg = shadow_cfg(fx)
    params = [{k: v.to(dtype) for k, v in O.make_params(s, sigma_bias=cfg["sigma_bias"]).items()}
              for s in cfg["seeds"][:n_models(cfg)]]
    if requires_grad:
        params = [{k: v.requires_grad_(True) for k, v in p.items()} for p in params]
    draws = fixture_draws(fx)
    nc = n_camera_draws(cfg)
    if light_rows is not None:
        draws = draws[:nc] + [d[:light_rows] for d in draws[nc:]]
    rng = O.ReplayRNG(draws)
    rng._queue = [q.to(dtype) for q in rng._queue]

    def t(k):
        return torch.from_numpy(fx[k]).to(dtype)
    cam = SO.render_rays(params, t("rays"), cfg["N_samples"], False, cfg["perturb"],
                         cfg["noise_std"], cfg["N_importance"], rng=rng)
    lrays = t("light_rays") if light_rows is None else t("light_rays")[:light_rows]
    with torch.set_grad_enabled(requires_grad and cfg["grad_on_light"]):
        light = SO.render_rays(params, lrays, cfg["N_samples"], False,
                               cfg["perturb"], cfg["noise_std"], cfg["light_importance"],
                               rng=rng)
    assert rng.exhausted()
    light_in = light if light_rows is None else \
        {k[6:]: t(k) for k in fx if k.startswith("light_depth")}
    depths, light_depths = {}, {}
    for k in ("depth_coarse", "depth_fine"):
        if k in cam and requires_grad:
            cam[k].retain_grad()
            depths[k] = cam[k]
        if k in light and light[k].requires_grad:
            light[k].retain_grad()
            light_depths[k] = light[k]
    ppc = {"eye_pos": t("eye_pos"), "camera": t("camera")}
    out = SO.efficient_sm(t("pixels"), t("light_pixels"), cam, light_in, ppc,
                          t("light_eye"), t("light_camera"), (cfg["wh"], cfg["wh"]),
                          cfg["N_importance"] > 0, cfg["light_importance"] > 0, cfg["method"])
    return cfg, params, cam, light, out, depths, light_depths


@pytest.mark.parametrize("case", CASES)
def test_shadow_oracle_forward_matches(case):
    fx = load_shadow(case)
    # cfg5-shaped fixtures: the light image (4,096 / 16,384 rays) checked on its
    # first 1,024 rows, the shadow stage on the reference's whole light maps --
    # the full light render would take minutes of CPU in this suite
    rows = 1024 if case.startswith("cfg5") else None
    with torch.no_grad():
        _, _, _, light, out, _, _ = run_oracle(fx, light_rows=rows)
    for k, v in list(out.items()) + [("light_" + k, v) for k, v in light.items()]:
        ref = fx[k if k.startswith("light_") else f"out_{k}"]
        if k.startswith("light_") and rows is not None:
            ref = ref[:rows]
        np.testing.assert_allclose(v.detach().numpy(), ref, rtol=1e-5,
                                   atol=1e-6 * max(1.0, float(np.abs(ref).max())), err_msg=k)


def _loss(out, fx, dtype=torch.float32):
    tgt = torch.from_numpy(fx["target"]).to(dtype)
    loss = torch.mean((out["rgb_coarse"] - tgt) ** 2)
    if "rgb_fine" in out:
        loss = loss + torch.mean((out["rgb_fine"] - tgt) ** 2)
    return loss


@pytest.mark.parametrize("case", [c for c in CASES if not c.startswith("cfg5")])
def test_shadow_oracle_gradients(case):
    """Gradients of the oracle's training step against the reference's: the
    camera depths, (--grad_on_light) the light depths, and every parameter."""
    fx = load_shadow(case)
    cfg, params, _, _, out, depths, light_depths = run_oracle(fx, requires_grad=True)
    assert bool(light_depths) == cfg["grad_on_light"]
    loss = _loss(out, fx)
    assert loss.item() == pytest.approx(float(fx["loss"]), rel=1e-6)
    loss.backward()
    for pre, dd in (("grad_", depths), ("grad_light_", light_depths)):
        for k, d in dd.items():
            ref = fx[pre + k]
            np.testing.assert_allclose(d.grad.numpy(), ref, rtol=1e-4,
                                       atol=1e-5 * max(1e-12, np.abs(ref).max()), err_msg=pre + k)
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


def test_cfg5_draws_redraw_from_seed():
    """The cfg5-shaped fixtures do not store their 1.3M random draws: the CPU
    generator re-draws them from the recorded seed (checksums must match)."""
    for case in [c for c in CASES if c.startswith("cfg5")]:
        fx = load_shadow(case)
        assert "draws_seed" in fx
        draws = fixture_draws(fx)
        assert len(draws) == int(fx["n_draws"])


def test_shadow_runs_split_like_reference():
    eye = torch.tensor([[0., 0, 1], [0, 0, 1], [1, 0, 0], [0, 0, 1], [0, 0, 1], [-0., 0, 1]])
    assert SO.shadow_runs(eye) == [(0, 2), (2, 3), (3, 6)]
