"""Zero-gradient samples: the backward (f16x3, bf16x6 and, from
round 4, exact fp32) works
on the samples with a nonzero output gradient only, packed densely
(``nr_active_samples`` + the ``*_active`` data- and weight-gradient entry
points, which gather the saved activations of the listed samples).  A sample
with a zero output gradient -- sigma clamped by the ReLU of
rendering.py:169-176, or a transmittance underflowed behind an opaque
surface -- adds exactly zero to every dz and weight-gradient sum, so the step
must equal the every-sample backward up to the order of the split-K partial
sums.  Checked: the sample list against numpy (partial last block, NaN,
negative zeros, empty), and the parameter gradients with the list against
those without it, through the render path and through hand-made upstream
gradients: scattered zero samples (the bench's random init), zero blocks,
one active sample, none."""
import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _samples(g_out):
    from nerf_pl_amd._lib import call, stream_of
    n = g_out.shape[0]
    sl = torch.full((n + 1 + 2 * ((n + 31) // 32),), -7, dtype=torch.int32, device=DEV)
    call("nr_active_samples", g_out.data_ptr() if n else 0, n, sl.data_ptr(), sl.data_ptr() + 4 * n,
         sl.data_ptr() + 4 * (n + 1), stream_of(DEV))
    torch.cuda.synchronize()
    c = int(sl[n].item())
    return sl[:c].cpu().numpy(), c


@pytest.mark.parametrize("n", [1, 31, 32, 33, 1000, 4096, 70001, 800017])
def test_active_sample_list_matches_numpy(n):
    g = torch.Generator().manual_seed(n)
    x = torch.randn(n, 4, generator=g)
    nb = (n + 31) // 32
    zb = torch.rand(nb, generator=g) < 0.4          # whole zero blocks
    for b in torch.nonzero(zb).flatten().tolist():
        x[32 * b:32 * b + 32] = 0
    x[torch.rand(n, generator=g) < 0.5] = 0          # and scattered zero rows
    x[torch.rand(n, generator=g) < 0.1, 1] = 0       # rows with a zero entry stay active
    if n > 100:
        x[40:64] = 0
        x[33] = 0
        x[33, 2] = float("nan")       # NaN counts as nonzero (it propagates)
        x[70:96] = -0.0               # negative zeros are zeros
    lst, c = _samples(x.to(DEV))
    xa = x.numpy()
    want = [i for i in range(n) if np.any(xa[i] != 0) or np.any(np.isnan(xa[i]))]
    assert c == len(want)
    assert lst.tolist() == want


def test_active_sample_list_empty_and_all_zero():
    assert _samples(torch.zeros(0, 4, device=DEV))[1] == 0
    assert _samples(torch.zeros(300, 4, device=DEV))[1] == 0


def _mlp_grads(math, active, g_out_fn, monkeypatch, n=4096, spr=64, sigma_only=False, seed=5,
               defer="none"):
    from nerf_pl_amd import NeRF, functions, ops
    from nerf_pl_amd.rays import blender_rays
    monkeypatch.setattr(ops, "MATH", math)
    monkeypatch.setattr(functions, "ACTIVE_SAMPLES", active)
    monkeypatch.setattr(functions, "DEFER_SAVE", defer)
    m = NeRF()
    m.load_state_dict(O.make_params(seed, sigma_bias=0.3))
    m = m.to(DEV)
    nr = n // spr
    rays = blender_rays(32, 1, near=2.0, far=6.0)[:nr].contiguous().to(DEV)
    g = torch.Generator().manual_seed(seed)
    z = (2.0 + 4.0 * torch.rand(nr, spr, generator=g)).sort(1).values.to(DEV)
    out = functions.mlp_apply(m, rays=rays, z=z, spr=spr, sigma_only=sigma_only)
    go = g_out_fn(out.shape, g).to(DEV)
    out.backward(go)
    torch.cuda.synchronize()
    return {k: (None if p.grad is None else p.grad.detach().cpu().double())
            for k, p in m.named_parameters()}


def _zeroed(kind):
    """upstream gradient with zero rows: scattered samples (the bench's random
    init), whole 32-sample blocks, runs, a single active sample, none"""
    def make(shape, g):
        n = shape[0]
        x = torch.randn(*shape, generator=g)
        if kind == "scattered":
            x[torch.rand(n, generator=g) < 0.5] = 0
        elif kind == "blocks":
            for b in range((n + 31) // 32):
                if b % 7 != 3:
                    x[32 * b:32 * b + 32] = 0
        elif kind == "runs":      # like rays: empty space, a surface, nothing behind it
            r = torch.rand(n, generator=g)
            x[(torch.arange(n) % 64 < 20) | (torch.arange(n) % 64 > 40) | (r < 0.3)] = 0
        elif kind == "one":
            keep = x[n // 2 + 5].clone()
            x.zero_()
            x[n // 2 + 5] = keep
        elif kind == "none":
            x.zero_()
        return x
    return make


CASES = ("dense", "scattered", "blocks", "runs", "one", "none")


@pytest.mark.parametrize("math", ["f16x3", "bf16x6", "fp32"])
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("sigma_only", [False, True])
def test_active_backward_matches_every_sample(math, case, sigma_only, monkeypatch):
    fn = _zeroed(case)
    a = _mlp_grads(math, True, fn, monkeypatch, sigma_only=sigma_only)
    b = _mlp_grads(math, False, fn, monkeypatch, sigma_only=sigma_only)
    for k in b:
        if b[k] is None:
            assert a[k] is None, k
            continue
        if case == "none":
            assert torch.count_nonzero(a[k]) == 0, k
            continue
        dev = ((a[k] - b[k]).norm() / (b[k].norm() + 1e-30)).item()
        assert dev <= 2e-6, f"{math} {case} {k}: {dev:.3g}"


@pytest.mark.parametrize("math", ["f16x3", "bf16x6", "fp32"])
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("sigma_only", [False, True])
def test_deferred_backward_matches_every_sample(math, case, sigma_only, monkeypatch):
    """the deferred save over every list shape, on a ragged
    sample count (61 rays x 48 samples = 91.5 blocks of 32): the listed
    re-run, data and weight gradients against the every-sample backward over a
    forward-time save; an empty list (case "none") gives exact zeros"""
    fn = _zeroed(case)
    a = _mlp_grads(math, True, fn, monkeypatch, n=61 * 48, spr=48, sigma_only=sigma_only,
                   defer="all")
    b = _mlp_grads(math, False, fn, monkeypatch, n=61 * 48, spr=48, sigma_only=sigma_only)
    for k in b:
        if b[k] is None:
            assert a[k] is None, k
            continue
        if case == "none":
            assert torch.count_nonzero(a[k]) == 0, k
            continue
        dev = ((a[k] - b[k]).norm() / (b[k].norm() + 1e-30)).item()
        assert dev <= 2e-6, f"{math} {case} {k}: {dev:.3g}"


@pytest.mark.parametrize("math", ["f16x3", "bf16x6", "fp32"])
def test_auto_defer_follows_the_listed_fraction(math, monkeypatch):
    """NERF_PL_AMD_DEFER_SAVE=auto (the default): a model's full-graph forward
    defers its save once the model's last backward listed fewer than
    DEFER_AUTO of the samples, and goes back to the forward-time save when a
    backward lists many; every step's gradients equal the forward-time save's
    bit for bit"""
    from nerf_pl_amd import NeRF, functions, ops
    from nerf_pl_amd.rays import blender_rays
    monkeypatch.setattr(ops, "MATH", math)
    monkeypatch.setattr(functions, "ACTIVE_SAMPLES", True)
    spr, nr = 64, 48
    rays = blender_rays(32, 1, near=2.0, far=6.0)[:nr].contiguous().to(DEV)
    g = torch.Generator().manual_seed(3)
    z = (2.0 + 4.0 * torch.rand(nr, spr, generator=g)).sort(1).values.to(DEV)
    models = {}
    for k in ("auto", "none"):
        m = NeRF()
        m.load_state_dict(O.make_params(8, sigma_bias=0.3))
        models[k] = m.to(DEV)

    def step(kind, case, seed):
        monkeypatch.setattr(functions, "DEFER_SAVE", kind)
        m = models[kind]
        for p in m.parameters():
            p.grad = None
        out = functions.mlp_apply(m, rays=rays, z=z, spr=spr)
        out.backward(_zeroed(case)(out.shape, torch.Generator().manual_seed(seed)).to(DEV))
        torch.cuda.synchronize()
        return [p.grad.detach().clone() for p in m.parameters()], m.__dict__["_nr_defer_last"]

    seen = []
    for i, case in enumerate(("one", "one", "dense", "dense", "scattered")):
        ga, deferred = step("auto", case, 40 + i)
        gb, _ = step("none", case, 40 + i)
        seen.append(deferred)
        for a, b in zip(ga, gb):
            assert torch.equal(a, b), (math, i, case)
    # no statistics yet; 1 of 3072 listed; still following step 1; all listed; ~half
    assert seen == [False, True, True, False, False], seen


@pytest.mark.parametrize("math", ["f16x3", "fp32"])
def test_deferred_save_full_graph(math, monkeypatch):
    """NERF_PL_AMD_DEFER_SAVE=all on the full graph (render_rays' training
    step): the forward as inference, the listed samples' activations
    re-evaluated in the backward and saved by position -- the same loss and
    the same gradients bit for bit as the sample-list backward over a
    forward-time save"""
    from nerf_pl_amd import Embedding, NeRF, ReplayRNG, functions, ops, render_rays
    from nerf_pl_amd.rays import blender_rays
    monkeypatch.setattr(ops, "MATH", math)
    n, S, I = 512, 64, 64
    rays = blender_rays(32, 1, near=2.0, far=6.0)[:n].contiguous().to(DEV)
    g = torch.Generator().manual_seed(19)
    draws = [torch.rand(n, S, generator=g), torch.randn(n, S, generator=g),
             torch.rand(n, I, generator=g), torch.rand(n, I, generator=g),
             torch.randn(n, S + I, generator=g)]
    tgt = torch.rand(n, 3, generator=g).to(DEV)
    res = []
    for defer in ("all", "none"):
        monkeypatch.setattr(functions, "DEFER_SAVE", defer)
        models = []
        for s in (13, 14):
            m = NeRF()
            m.load_state_dict(O.make_params(s, sigma_bias=0.2))
            models.append(m.to(DEV))
        out = render_rays(models, [Embedding(3, 10), Embedding(3, 4)], rays, S, False, 1.0, 1.0, I,
                          32768, False, rng=ReplayRNG([d.clone() for d in draws]))
        loss = ((out["rgb_coarse"] - tgt) ** 2).mean() + ((out["rgb_fine"] - tgt) ** 2).mean()
        loss.backward()
        torch.cuda.synchronize()
        res.append((loss.item(), [[p.grad.detach().cpu() for p in m.parameters()] for m in models]))
    assert res[0][0] == res[1][0]
    for ga, gb in zip(res[0][1], res[1][1]):
        for a, b in zip(ga, gb):
            assert torch.equal(a, b)


def test_active_backward_in_render_rays(monkeypatch):
    """the training step of render_rays (both models, coarse + fine) with and
    without the sample list: same loss, same gradients (1e-6 normwise)"""
    from nerf_pl_amd import Embedding, NeRF, ReplayRNG, functions, ops
    from nerf_pl_amd.rays import blender_rays
    monkeypatch.setattr(ops, "MATH", "f16x3")
    n, S, I = 1024, 64, 64
    rays = blender_rays(32, 1, near=2.0, far=6.0)[:n].contiguous().to(DEV)
    g = torch.Generator().manual_seed(9)
    draws = [torch.rand(n, S, generator=g), torch.randn(n, S, generator=g),
             torch.rand(n, I, generator=g), torch.rand(n, I, generator=g),
             torch.randn(n, S + I, generator=g)]
    tgt = torch.rand(n, 3, generator=g).to(DEV)
    res = []
    for active in (True, False):
        monkeypatch.setattr(functions, "ACTIVE_SAMPLES", active)
        models = []
        for s in (11, 12):
            m = NeRF()
            m.load_state_dict(O.make_params(s, sigma_bias=0.2))
            models.append(m.to(DEV))
        from nerf_pl_amd import render_rays
        out = render_rays(models, [Embedding(3, 10), Embedding(3, 4)], rays, S, False, 1.0, 1.0, I,
                          32768, False, rng=ReplayRNG([d.clone() for d in draws]))
        loss = ((out["rgb_coarse"] - tgt) ** 2).mean() + ((out["rgb_fine"] - tgt) ** 2).mean()
        loss.backward()
        torch.cuda.synchronize()
        res.append((loss.item(), [[p.grad.detach().cpu().double() for p in m.parameters()]
                                  for m in models]))
    assert res[0][0] == res[1][0]
    for ga, gb in zip(res[0][1], res[1][1]):
        for a, b in zip(ga, gb):
            dev = ((a - b).norm() / (b.norm() + 1e-30)).item()
            assert dev <= 1e-6, dev


def test_nerf_copies_after_auto_defer_backward(monkeypatch):
    """the auto deferral's per-model statistics (CUDA events) live
    outside the module, so after training steps a NeRF still deep-copies,
    pickles (torch.save) and wraps in AveragedModel, and the copy keeps no
    statistics of its own"""
    import copy
    import io
    from nerf_pl_amd import NeRF, functions, ops
    from nerf_pl_amd.rays import blender_rays
    monkeypatch.setattr(ops, "MATH", "f16x3")
    monkeypatch.setattr(functions, "ACTIVE_SAMPLES", True)
    monkeypatch.setattr(functions, "DEFER_SAVE", "auto")
    spr, nr = 64, 16
    rays = blender_rays(32, 1, near=2.0, far=6.0)[:nr].contiguous().to(DEV)
    z = (2.0 + 4.0 * torch.rand(nr, spr, generator=torch.Generator().manual_seed(1))).sort(1).values.to(DEV)
    m = NeRF()
    m.load_state_dict(O.make_params(3, sigma_bias=0.3))
    m = m.to(DEV)
    for i in range(3):
        out = functions.mlp_apply(m, rays=rays, z=z, spr=spr)
        out.backward(_zeroed("one")(out.shape, torch.Generator().manual_seed(i)).to(DEV))
    torch.cuda.synchronize()
    assert functions._listed_fraction(m, False) is not None
    c = copy.deepcopy(m)
    buf = io.BytesIO()
    torch.save(m, buf)
    torch.optim.swa_utils.AveragedModel(m)
    assert functions._listed_fraction(c, False) is None
    for a, b in zip(m.parameters(), c.parameters()):
        assert torch.equal(a, b)


@pytest.mark.parametrize("math", ["f16x3", "fp32"])
def test_deferred_save_strided_inputs(math, monkeypatch):
    """a direct mlp_apply caller passing strided rays / depth views;
    the deferred backward re-runs the forward on the very (contiguous) tensors
    the forward read, so its gradients equal the forward-time save's bit for bit"""
    from nerf_pl_amd import NeRF, functions, ops
    from nerf_pl_amd.rays import blender_rays
    monkeypatch.setattr(ops, "MATH", math)
    monkeypatch.setattr(functions, "ACTIVE_SAMPLES", True)
    spr, nr = 64, 48
    rays = blender_rays(32, 1, near=2.0, far=6.0)[:nr].contiguous()
    z = (2.0 + 4.0 * torch.rand(nr, spr, generator=torch.Generator().manual_seed(2))).sort(1).values
    rbig = torch.full((nr, 16), float("nan"))
    rbig[:, ::2] = rays
    zbig = torch.full((nr, 2 * spr), float("nan"))
    zbig[:, 1::2] = z
    rv, zv = rbig.to(DEV)[:, ::2], zbig.to(DEV)[:, 1::2]
    assert not rv.is_contiguous() and not zv.is_contiguous()
    go = _zeroed("scattered")((nr * spr, 4), torch.Generator().manual_seed(4)).to(DEV)
    grads = []
    for defer, (r, zz) in (("all", (rv, zv)), ("none", (rays.to(DEV), z.to(DEV)))):
        monkeypatch.setattr(functions, "DEFER_SAVE", defer)
        m = NeRF()
        m.load_state_dict(O.make_params(6, sigma_bias=0.3))
        m = m.to(DEV)
        out = functions.mlp_apply(m, rays=r, z=zz, spr=spr)
        out.backward(go)
        torch.cuda.synchronize()
        grads.append([p.grad.detach().clone() for p in m.parameters()])
    for a, b in zip(*grads):
        assert torch.equal(a, b)
