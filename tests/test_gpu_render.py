"""End-to-end parity of the drop-in ``render_rays`` (and its gradients) with the
reference, on the golden fixtures, replaying the reference's random draws.

Tolerance: 1e-4 ABSOLUTE on rgb, depth, opacity and the coarse and fine
compositing weights (the north-star bound, tests/parity.py).  Two reference discontinuities are screened per ray, not
hidden: (1) a sample_pdf bin flip -- u within ~1e-6 of a CDF knot, so an ulp of
difference in the coarse weights moves one fine depth by a whole bin (detected
as a z_fine mismatch); (2) the 1e10 last delta makes the last alpha a step
function of sign(sigma+noise).  Screened rays must stay rare.
"""
import numpy as np
import pytest
import torch

from conftest import golden_cases, golden_cfg, golden_draws, load_golden
from oracle import nerf_oracle as O
from parity import assert_forward
from screening import pdf_flips

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def build_models(cfg):
    from nerf_pl_amd import NeRF
    ms = []
    for m in range(2 if cfg["N_importance"] > 0 else 1):
        net = NeRF()
        net.load_state_dict(O.make_params(cfg["seeds"][m], sigma_bias=cfg["sigma_bias"]))
        ms.append(net.to(DEV))
    return ms


def run_ours(fx, cfg, models, grad=False):
    from nerf_pl_amd import Embedding, ReplayRNG, render_rays
    cap = {}
    rays = torch.from_numpy(fx["rays"]).to(DEV)
    with torch.set_grad_enabled(grad):
        res = render_rays(models, [Embedding(3, 10), Embedding(3, 4)], rays, cfg["N_samples"],
                          cfg["use_disp"], cfg["perturb"], cfg["noise_std"], cfg["N_importance"],
                          cfg["chunk"], cfg["white_back"], cfg["test_time"],
                          rng=ReplayRNG(golden_draws(fx)), _capture=cap)
    return res, cap


def screened_rays(fx, cfg, cap):
    """Rays excluded from the tight comparison, each explained: a z_fine move
    must come from reference importance samples whose u lies within 1e-5 of
    one of the reference's CDF knots (screening.pdf_flips)."""
    bad = np.zeros(fx["rays"].shape[0], bool)
    ocap = {}
    params = [O.make_params(cfg["seeds"][0], sigma_bias=cfg["sigma_bias"]),
              O.make_params(cfg["seeds"][1], sigma_bias=cfg["sigma_bias"])]
    O.render_rays(params, torch.from_numpy(fx["rays"]), cfg["N_samples"], cfg["use_disp"],
                  cfg["perturb"], cfg["noise_std"], cfg["N_importance"], cfg["chunk"],
                  cfg["white_back"], cfg["test_time"], rng=O.ReplayRNG(golden_draws(fx)),
                  capture=ocap)
    if "z_fine" in cap:
        zf = cap["z_fine"].cpu().numpy()
        flip = np.abs(zf - ocap["z_fine"].numpy()).max(1) > 1e-4 * np.maximum(1, np.abs(zf).max(1))
        moved, explained = pdf_flips(cap["z_fine"], ocap, golden_draws(fx)[-3])
        assert not (flip & ~moved).any(), "z_fine differs although every importance depth matches"
        assert not (moved & ~explained).any(), \
            f"z_fine moved away from any CDF knot: rays {np.nonzero(moved & ~explained)[0][:8]}"
        bad |= flip
    return bad, ocap


@pytest.mark.parametrize("case", [c for c in golden_cases() if not c.endswith("_grad")])
def test_render_rays_matches_reference(case):
    fx = load_golden(case)
    cfg = golden_cfg(fx)
    res, cap = run_ours(fx, cfg, build_models(cfg))
    bad, ocap = screened_rays(fx, cfg, cap)
    assert bad.mean() <= 0.05, f"{bad.sum()} screened rays"
    # outputs against the reference's own (the fixture), weights against the
    # oracle's capture (the fixtures hold no weights; the oracle is pinned to
    # the fixtures by tests/test_oracle_golden.py)
    ref = {k[4:]: fx[k] for k in fx if k.startswith("out_")}
    assert_forward(res, ref, cap, ocap, bad, label=case)


def test_render_rays_deterministic():
    fx = load_golden("cfg2_n26")
    cfg = golden_cfg(fx)
    models = build_models(cfg)
    a, _ = run_ours(fx, cfg, models)
    b, _ = run_ours(fx, cfg, models)
    for k in a:
        assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("case", ["cfg2_grad", "cfg1_grad"])
def test_gradients_match_reference(case):
    fx = load_golden(case)
    cfg = golden_cfg(fx)
    models = build_models(cfg)
    res, cap = run_ours(fx, cfg, models, grad=True)
    bad, _ = screened_rays(fx, cfg, cap)
    assert not bad.any(), "gradient fixture hit a sample_pdf flip; pick another seed"
    target = torch.from_numpy(fx["target"]).to(DEV)
    loss = torch.mean((res["rgb_coarse"] - target) ** 2)
    if "rgb_fine" in res:
        loss = loss + torch.mean((res["rgb_fine"] - target) ** 2)
    np.testing.assert_allclose(loss.item(), float(fx["loss"]), rtol=1e-5)
    loss.backward()
    n = 0
    for m, net in enumerate(models):
        for name, p in net.named_parameters():
            key = f"grad{m}_{name}"
            g = p.grad.detach().cpu().numpy()
            l2 = float(fx[key + "_l2"])
            gmax = np.abs(fx.get(key + "_full", fx.get(key + "_val"))).max()
            np.testing.assert_allclose(np.sqrt((g.astype(np.float64) ** 2).sum()), l2, rtol=1e-3,
                                       err_msg=key)
            if key + "_full" in fx:
                got, ref = g, fx[key + "_full"]
            else:
                got, ref = g.reshape(-1)[fx[key + "_idx"]], fx[key + "_val"]
            np.testing.assert_allclose(got, ref, rtol=1e-3, atol=1e-4 * gmax + 1e-12,
                                       err_msg=key)
            n += 1
    assert n == 24 * len(models)


@pytest.mark.parametrize("math,gscale,sboost,size", [
    ("fp32", 1.0, 1.0, (23, 37)), ("bf16x6", 1.0, 1.0, (23, 37)), ("f16x3", 1.0, 1.0, (23, 37)),
    ("f16x3", 1e-12, 1.0, (23, 37)), ("f16x3", 1e6, 1.0, (23, 37)), ("f16x3", 1.0, 1e8, (23, 37)),
    ("f16x3", 1.0, 1e-8, (23, 37)), ("f16x3", 1.0, 1e12, (23, 37)), ("f16x3", 1e-18, 1.0, (23, 37)),
    ("f16x3", 1.0, 1.0, (509, 61)), ("fp32", 1.0, 1.0, (509, 61))])
def test_mlp_backward_matches_autograd(math, gscale, sboost, size, monkeypatch):
    """Full-gradient check (every parameter entry) of the fused MLP backward on
    random per-sample output gradients, against torch CPU autograd of the
    oracle MLP.  Samples with a pre-activation within 2e-6 of the ReLU kink
    (where an ulp decides the mask) get no output gradient: they must stay
    rare.  gscale multiplies the output gradient: f16x3 must keep the same
    relative accuracy for gradients far outside fp16's range (its power-of-two
    range scaling).  sboost multiplies the sigma gradient alone (the 1e10
    last-sample delta of rendering.py:171 makes d sigma dwarf d rgb).  The
    (509, 61) size (31,049 samples, 971 blocks, ragged) runs the weight
    gradient with many workgroups per task, so the f16x3 fused task pairs
    (wgrad.hip kFused) split their block ranges the way a training step does."""
    from nerf_pl_amd import NeRF, ops
    from nerf_pl_amd.functions import mlp_apply
    monkeypatch.setattr(ops, "MATH", math)
    p = O.make_params(7, sigma_bias=0.4)
    g = torch.Generator().manual_seed(3)
    n_rays, spr = size
    rays = torch.cat([torch.randn(n_rays, 3, generator=g) * 0.3,
                      torch.nn.functional.normalize(torch.randn(n_rays, 3, generator=g), dim=-1),
                      torch.full((n_rays, 1), 2.0), torch.full((n_rays, 1), 6.0)], 1)
    z = 2 + 4 * torch.rand(n_rays, spr, generator=g)
    gout = torch.randn(n_rays * spr, 4, generator=g) * gscale
    # per-ray spread of magnitudes (2^-20 .. 1), as transmittance weights give
    gout *= torch.exp2(-20 * torch.rand(n_rays, 1, generator=g)).repeat_interleave(spr, 0)
    gout[:, 3] *= sboost
    if sboost > 1e10:      # opaque samples: no rgb gradient at all beside a huge d sigma
        gout[::3, :3] = 0
    # oracle
    pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    xyz = rays[:, None, :3] + rays[:, None, 3:6] * z[..., None]
    x = torch.cat([O.embed(xyz.reshape(-1, 3), 10),
                   O.embed(rays[:, 3:6], 4).repeat_interleave(spr, 0)], 1)
    # screen ReLU-kink samples (pre-activations of every layer, oracle arithmetic)
    with torch.no_grad():
        xe, de = x[:, :63], x[:, 63:]
        h, kink = xe, torch.zeros(x.shape[0], dtype=torch.bool)
        for i in range(8):
            if i == 4:
                h = torch.cat([xe, h], -1)
            pre = torch.nn.functional.linear(h, p[f"xyz_encoding_{i+1}.0.weight"],
                                             p[f"xyz_encoding_{i+1}.0.bias"])
            kink |= (pre.abs() < 2e-6).any(1)
            h = torch.relu(pre)
        feat = torch.nn.functional.linear(h, p["xyz_encoding_final.weight"],
                                          p["xyz_encoding_final.bias"])
        pre = torch.nn.functional.linear(torch.cat([feat, de], -1), p["dir_encoding.0.weight"],
                                         p["dir_encoding.0.bias"])
        kink |= (pre.abs() < 2e-6).any(1)
    assert kink.float().mean() < 0.1, kink.sum()
    gout[kink] = 0
    out_ref = O.nerf_forward(pr, x)
    (out_ref * gout).sum().backward()
    # ours
    net = NeRF()
    net.load_state_dict(p)
    net = net.to(DEV)
    out = mlp_apply(net, rays=rays.to(DEV), z=z.to(DEV), spr=spr)
    assert (out.detach().cpu() - out_ref.detach()).abs().max() < 2e-5
    (out * gout.to(DEV)).sum().backward()
    for name, q in net.named_parameters():
        ref = pr[name].grad
        got = q.grad.cpu()
        scale = ref.abs().max().item() + 1e-30
        err = (got - ref).abs().max().item()
        assert err <= 2e-4 * scale + 1e-6 * gscale * max(sboost, 1.0), \
            f"{name}: err {err:.3g} scale {scale:.3g}"


@pytest.mark.parametrize("optim", ["torch_adam", "fused_adam"])
def test_training_steps_reduce_loss(optim):
    """30 steps on a learnable target with either optimiser.  FusedAdam writes
    the parameters through raw pointers, so this also checks that the packed
    weights the kernels read follow every optimiser step (a stale pack cache
    would leave the output frozen at its step-0 value)."""
    from nerf_pl_amd import Embedding, NeRF, render_rays
    from nerf_pl_amd.optim import FusedAdam
    from nerf_pl_amd.rays import blender_rays
    torch.manual_seed(0)
    rays = blender_rays(32, 1, near=2.0, far=6.0, device=DEV)[:512].contiguous()
    # a learnable target: a smooth colour field over ray directions
    target = (0.5 + 0.4 * torch.sin(3 * rays[:, 3:6])).contiguous()
    models = [NeRF().to(DEV), NeRF().to(DEV)]
    params = [p for m in models for p in m.parameters()]
    opt = (torch.optim.Adam if optim == "torch_adam" else FusedAdam)(params, lr=5e-4)
    emb = [Embedding(3, 10), Embedding(3, 4)]
    probe = rays[:64].contiguous()

    def probe_out():
        with torch.no_grad():
            return render_rays(models, emb, probe, 32, False, 0.0, 0.0, 32, 1024,
                               False)["rgb_fine"].clone()

    out0 = probe_out()
    losses = []
    for _ in range(30):
        res = render_rays(models, emb, rays, 32, False, 1.0, 1.0, 32, 1024, False)
        loss = ((res["rgb_coarse"] - target) ** 2).mean() + ((res["rgb_fine"] - target) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert np.isfinite(losses).all()
    assert losses[-1] < 0.7 * losses[0], losses
    assert (probe_out() - out0).abs().max() > 1e-3
    # the cached pack equals a fresh pack of the current parameters
    from nerf_pl_amd import ops
    for m in models:
        pf, pb = m.packed(backward=True)
        assert torch.equal(pf, ops.pack_fwd(m.flat_params()))
        assert torch.equal(pb, ops.pack_bwd(m.flat_params()))


def test_fused_adam_invalidates_pack_cache():
    """One FusedAdam step must change the forward output of the next call."""
    from nerf_pl_amd import NeRF
    from nerf_pl_amd.functions import mlp_apply
    from nerf_pl_amd.optim import FusedAdam
    torch.manual_seed(0)
    net = NeRF().to(DEV)
    rays = torch.zeros(4, 8, device=DEV)
    rays[:, 3] = 1.0
    rays[:, 6], rays[:, 7] = 2.0, 6.0
    z = torch.linspace(2.0, 6.0, 32, device=DEV).repeat(4)
    out0 = mlp_apply(net, rays=rays, z=z, spr=32)
    out0.sum().backward()
    opt = FusedAdam(net.parameters(), lr=1e-2)
    opt.step()
    with torch.no_grad():
        out1 = mlp_apply(net, rays=rays, z=z, spr=32)
    assert (out1 - out0.detach()).abs().max() > 1e-4


@pytest.mark.parametrize("defer", [False, True])
def test_inplace_parameter_change_before_backward_raises(defer, monkeypatch):
    """The backward's nr_wgrad_dir_feat reads W_final, b_final and W_dir from
    the flat parameters the forward ran with; they are saved for backward, so
    an in-place edit between forward and backward raises autograd's version
    error (as the reference's nn.Linear graph does) instead of mixing old and
    new weights into one gradient."""
    from nerf_pl_amd import NeRF, functions
    from nerf_pl_amd.functions import mlp_apply
    monkeypatch.setattr(functions, "DEFER_SAVE", "all" if defer else "none")
    net = NeRF()
    net.load_state_dict(O.make_params(5, sigma_bias=0.5))
    net = net.to(DEV)
    rays = torch.zeros(4, 8, device=DEV)
    rays[:, 3] = 1.0
    rays[:, 6], rays[:, 7] = 2.0, 6.0
    z = torch.linspace(2.0, 6.0, 32, device=DEV).repeat(4)
    out = mlp_apply(net, rays=rays, z=z, spr=32)
    with torch.no_grad():
        net.xyz_encoding_final.weight.mul_(2.0)
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        out.sum().backward()
    # unchanged parameters: the same call back-propagates
    out = mlp_apply(net, rays=rays, z=z, spr=32)
    out.sum().backward()
    assert torch.isfinite(net.xyz_encoding_final.weight.grad).all()


def test_fine_stream_step_is_bitwise_the_single_stream_step(monkeypatch):
    """A training call runs the fine pass (and so, by autograd's stream rule,
    its backward) on a side stream beside the coarse pass's backward
    (rendering.FINE_STREAM).  Same inputs, same draws: outputs and every
    parameter gradient equal the single-stream step bit for bit, over three
    steps with FusedAdam in between (the caching allocator's cross-stream
    reuse is exercised by the repeated steps)."""
    from nerf_pl_amd import Embedding, NeRF, ReplayRNG, rendering, render_rays
    from nerf_pl_amd.optim import FusedAdam
    from nerf_pl_amd.rays import blender_rays
    rays = blender_rays(64, 1, near=1.0, far=200.0)[:1024].contiguous().to(DEV)
    target = torch.rand(1024, 3, generator=torch.Generator().manual_seed(1)).to(DEV)
    g = torch.Generator().manual_seed(2)
    draws = [[torch.rand(1024, 64, generator=g), torch.randn(1024, 64, generator=g),
              torch.rand(1024, 128, generator=g), torch.rand(1024, 128, generator=g),
              torch.randn(1024, 192, generator=g)] for _ in range(3)]
    runs = []
    for fs in (False, True):
        monkeypatch.setattr(rendering, "FINE_STREAM", fs)
        models = []
        for s in (41, 42):
            m = NeRF()
            m.load_state_dict(O.make_params(s, sigma_bias=0.5))
            models.append(m.to(DEV))
        opt = FusedAdam([p for m in models for p in m.parameters()], lr=5e-4)
        outs = []
        for d in draws:
            res = render_rays(models, [Embedding(3, 10), Embedding(3, 4)], rays, 64, False, 1.0, 1.0,
                              128, 32768, False, rng=ReplayRNG(d))
            loss = ((res["rgb_coarse"] - target) ** 2).mean() + ((res["rgb_fine"] - target) ** 2).mean()
            opt.zero_grad()
            loss.backward()
            outs.append({k: v.detach().clone() for k, v in res.items()})
            outs.append({f"{i}.{k}": p.grad.clone() for i, m in enumerate(models)
                         for k, p in m.named_parameters()})
            opt.step()
        torch.cuda.synchronize()
        runs.append(outs)
    for a, b in zip(*runs):
        for k in a:
            assert torch.equal(a[k], b[k]), k
