"""Sigma-only training kernels: the shadow path trains the
sigma-only graph (models/rendering_shadows.py:167, NeRF.forward(x,
sigma_only=True) on every call), which every arithmetic (fp32 from round 4) runs on dedicated
kernels -- layers 1-8 and the sigma head only -- instead of the full kernels
with a zero rgb gradient.  Both must give the same step: the forward bit for
bit (the same sums), every gradient within 1e-6 normwise (only the sigma
head's split-K partition changes, so its slab sums round differently), and the
parameters outside the graph no gradient at all."""
import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
S, I = 32, 32


def _step(math, so_kernels, monkeypatch, n=700, seed=3, defer="none"):
    from nerf_pl_amd import Embedding, NeRF, ReplayRNG, functions, ops
    from nerf_pl_amd import rendering_shadows as RS
    from nerf_pl_amd.rays import blender_rays
    monkeypatch.setattr(ops, "MATH", math)
    monkeypatch.setattr(functions, "SIGMA_TRAIN_KERNELS", so_kernels)
    monkeypatch.setattr(functions, "DEFER_SAVE", defer)
    models = []
    for s in (41, 42):
        m = NeRF()
        m.load_state_dict(O.make_params(s, sigma_bias=0.5))
        models.append(m.to(DEV))
    rays = blender_rays(32, 1, near=2.0, far=6.0)[:n].contiguous().to(DEV)
    g = torch.Generator().manual_seed(seed)
    draws = [torch.rand(n, S, generator=g), torch.randn(n, S, generator=g),
             torch.rand(n, I, generator=g), torch.rand(n, I, generator=g),
             torch.randn(n, S + I, generator=g)]
    out = RS.render_rays(models, [Embedding(3, 10), Embedding(3, 4)], rays, S, False, 1.0, 1.0,
                         I, 32768, False, rng=ReplayRNG(draws))
    gg = torch.Generator().manual_seed(seed + 1)
    loss = 0
    for k in sorted(out):
        loss = loss + (out[k] * torch.randn(out[k].shape, generator=gg).to(DEV)).sum()
    loss.backward()
    torch.cuda.synchronize()
    return ({k: v.detach().cpu() for k, v in out.items()},
            [[(name, None if p.grad is None else p.grad.detach().cpu())
              for name, p in m.named_parameters()] for m in models])


@pytest.mark.parametrize("math,defer", [("f16x3", "none"), ("bf16x6", "none"), ("bf16", "none"),
                                        ("fp32", "none"), ("f16x3", "sigma"), ("bf16x6", "sigma"),
                                        ("fp32", "sigma")])
def test_sigma_only_training_kernels_match_full_kernels(math, defer, monkeypatch):
    """defer = "sigma": the deferred save -- the forward as
    inference, the listed samples re-evaluated in the backward"""
    out_a, grads_a = _step(math, True, monkeypatch, defer=defer)
    out_b, grads_b = _step(math, False, monkeypatch)
    for k in out_b:
        assert torch.equal(out_a[k], out_b[k]), k
    unused = {"xyz_encoding_final.weight", "xyz_encoding_final.bias", "dir_encoding.0.weight",
              "dir_encoding.0.bias", "rgb.0.weight", "rgb.0.bias"}
    exact = 0
    for ga, gb in zip(grads_a, grads_b):
        for (name, a), (_, b) in zip(ga, gb):
            if name in unused:
                assert a is None and b is None, name
                continue
            exact += int(torch.equal(a, b))
            dev = ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()
            assert dev <= 1e-6, f"{math} {name}: {dev:.3g}"
    print(f"{math} defer={defer}: {exact} of 36 gradient tensors bit-identical")


@pytest.mark.parametrize("math", ["f16x3", "bf16x6", "fp32"])
def test_deferred_save_equals_forward_time_save(math, monkeypatch):
    """The deferred save re-runs the same layers over the listed samples and
    feeds the backward the same positions in the same order as the sample-list
    backward over a forward-time save: every output and every gradient
    bit-identical."""
    out_a, grads_a = _step(math, True, monkeypatch, defer="sigma")
    out_b, grads_b = _step(math, True, monkeypatch, defer="none")
    for k in out_b:
        assert torch.equal(out_a[k], out_b[k]), k
    for ga, gb in zip(grads_a, grads_b):
        for (name, a), (_, b) in zip(ga, gb):
            assert (a is None) == (b is None), name
            if a is not None:
                assert torch.equal(a, b), f"{math} {name}"
