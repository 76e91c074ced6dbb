"""Pin the CPU oracle against fixtures produced by the reference itself
(tests/golden/make_golden.py).  The oracle uses the same PyTorch-CPU kernels as
the reference, so every forward output and intermediate must match exactly;
gradients must match to fp32 reduction-order tolerance."""
import numpy as np
import pytest
import torch

from conftest import golden_cases, golden_cfg, golden_draws, load_golden
from oracle import nerf_oracle as O


def _run_oracle(fx, grads=False):
    cfg = golden_cfg(fx)
    params = [O.make_params(cfg["seeds"][0], sigma_bias=cfg["sigma_bias"]),
              O.make_params(cfg["seeds"][1], sigma_bias=cfg["sigma_bias"])]
    if grads:
        params = [{k: v.clone().requires_grad_(True) for k, v in p.items()} for p in params]
    rays = torch.from_numpy(fx["rays"])
    rng = O.ReplayRNG(golden_draws(fx))
    cap = {}
    with torch.set_grad_enabled(grads):
        res = O.render_rays(params, rays, cfg["N_samples"], cfg["use_disp"], cfg["perturb"],
                            cfg["noise_std"], cfg["N_importance"], cfg["chunk"],
                            cfg["white_back"], cfg["test_time"], rng=rng, capture=cap)
    assert rng.exhausted(), "oracle consumed a different number of random draws"
    return params, res, cap


@pytest.mark.parametrize("case", golden_cases())
def test_oracle_forward_matches_reference(case):
    fx = load_golden(case)
    _, res, cap = _run_oracle(fx)
    keys = [k for k in fx if k.startswith("out_")]
    assert keys
    for k in keys:
        np.testing.assert_array_equal(res[k[4:]].detach().numpy(), fx[k], err_msg=k)
    np.testing.assert_array_equal(cap["raw_coarse"].numpy(), fx["raw_coarse"])
    if "raw_fine" in fx:
        np.testing.assert_array_equal(cap["raw_fine"].numpy(), fx["raw_fine"])
        np.testing.assert_array_equal(cap["z_pdf"].numpy(), fx["z_pdf"])


@pytest.mark.parametrize("case", [c for c in golden_cases() if c.endswith("_grad")])
def test_oracle_gradients_match_reference(case):
    fx = load_golden(case)
    params, res, _ = _run_oracle(fx, grads=True)
    loss = O.mse_loss(res, torch.from_numpy(fx["target"]))
    np.testing.assert_allclose(loss.item(), float(fx["loss"]), rtol=1e-6)
    loss.backward()
    n_checked = 0
    for m, p in enumerate(params):
        for name, t in p.items():
            key = f"grad{m}_{name}"
            if key + "_sum" not in fx:
                continue
            g = t.grad.numpy()
            scale = float(fx[key + "_l2"]) + 1e-12
            np.testing.assert_allclose(np.sqrt((g.astype(np.float64) ** 2).sum()), scale,
                                       rtol=1e-4)
            if key + "_full" in fx:
                np.testing.assert_allclose(g, fx[key + "_full"], rtol=1e-4,
                                           atol=1e-5 * scale, err_msg=key)
            else:
                np.testing.assert_allclose(g.reshape(-1)[fx[key + "_idx"]], fx[key + "_val"],
                                           rtol=1e-4, atol=1e-5 * scale, err_msg=key)
            n_checked += 1
    assert n_checked >= 18


def test_replay_rng_shape_mismatch_raises():
    rng = O.ReplayRNG([np.zeros((2, 3), np.float32)])
    with pytest.raises(ValueError):
        rng.rand((3, 2))


def test_make_params_matches_nerf_shapes():
    p = O.make_params(0)
    shapes = O.param_shapes()
    assert set(p) == set(shapes)
    assert sum(v.numel() for v in p.values()) == 595844
    for k, v in p.items():
        assert tuple(v.shape) == shapes[k]
        assert v.dtype == torch.float32
