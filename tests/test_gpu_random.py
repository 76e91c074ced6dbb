"""Randomised parity sweep of the drop-in ``render_rays`` against the CPU oracle.

Each case draws its own configuration -- ray count, N_samples, N_importance
(0 or not), perturb, noise_std, use_disp, white_back, test_time, near/far and
un-normalised ray directions -- the flag combinations the reference accepts
(rendering.py:84-95), so shapes that are not multiples of the kernels' 32-sample
blocks and the less travelled branches get the same 1e-4 bound as the golden
cases (tests/test_gpu_render.py).  The reference's five draws are replayed in
its order.  ``sample_pdf`` bin flips (u within ~1e-6 of a CDF knot,
tests/test_gpu_render.py) are screened per ray and must stay rare.

Gradient cases (f16x3 and exact fp32): the parameter gradient of a random
linear functional of every output against the float64 oracle.  This gradient
is ill-conditioned in fp32 by construction -- xyz = o + d*z carries an fp32
rounding that the 2^9 positional-encoding frequency turns into ~1e-3 rad of
phase at |xyz| ~ 30, and ReLU kinks within an ulp of zero pick branches by
summation order -- so the oracle's own fp32 result sits up to 5e-3 of a
tensor's norm from float64 (median ~7e-4).  The bound (tests/grad64.py):
every tensor within max(1e-4, 2 x that fp32 distance) of float64, normwise,
the fp32 distance the largest at the weights and at two points one fp32 ulp
away, every evaluation's fine pass at our importance depths (which the
reference detaches, rendering.py:253-255), and the rays whose compositing ReLU
switched between ours and float64 out of the functional.
"""
import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O
import grad64
from parity import assert_forward
from screening import pdf_flips

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _config(seed):
    r = np.random.default_rng(seed)
    I = 0 if r.random() < 0.3 else int(r.integers(1, 140))
    S = int(r.integers(3 if I else 2, 100))
    n = int(r.integers(1, 400))
    near = float(r.uniform(0.05, 3.0))
    far = near + float(r.uniform(0.3, 60.0))
    return dict(n=n, S=S, I=I, perturb=float(r.choice([0.0, 1.0, 0.5])),
                noise=float(r.choice([0.0, 1.0])), use_disp=bool(r.random() < 0.25),
                white_back=bool(r.random() < 0.3), test_time=bool(r.random() < 0.2),
                near=near, far=far, seed=seed)


def _rays(c):
    g = torch.Generator().manual_seed(c["seed"])
    n = c["n"]
    o = torch.randn(n, 3, generator=g) * 0.5
    d = torch.randn(n, 3, generator=g)
    d = d / d.norm(dim=1, keepdim=True) * (0.5 + torch.rand(n, 1, generator=g))  # not unit
    nf = torch.tensor([c["near"], c["far"]]).expand(n, 2)
    return torch.cat([o, d, nf], 1).contiguous()


def _draws(c):
    g = torch.Generator().manual_seed(1000 + c["seed"])
    n, S, I = c["n"], c["S"], c["I"]
    d = []
    if c["perturb"] > 0:
        d.append(torch.rand(n, S, generator=g))
    d.append(torch.randn(n, S, generator=g))
    if I > 0:
        d += [torch.rand(n, I, generator=g), torch.rand(n, I, generator=g),
              torch.randn(n, S + I, generator=g)]
    return d


def _run(c, grad=False, want_cap=False):
    from nerf_pl_amd import Embedding, NeRF, ReplayRNG, render_rays
    params = [O.make_params(21 + c["seed"] % 5, sigma_bias=0.5),
              O.make_params(22 + c["seed"] % 5, sigma_bias=0.5)]
    models = []
    for p in params:
        m = NeRF()
        m.load_state_dict(p)
        models.append(m.to(DEV))
    rays, draws = _rays(c), _draws(c)
    args = (c["S"], c["use_disp"], c["perturb"], c["noise"], c["I"], 32768, c["white_back"],
            c["test_time"])
    cap, ocap = {}, {}
    with torch.set_grad_enabled(grad):
        res = render_rays(models, [Embedding(3, 10), Embedding(3, 4)], rays.to(DEV), *args,
                          rng=ReplayRNG(draws), _capture=cap)
    if grad:
        for p in params:
            for v in p.values():
                v.requires_grad_(True)
    with torch.set_grad_enabled(grad):
        ref = O.render_rays(params, rays, *args, rng=O.ReplayRNG(draws), capture=ocap)
    bad = np.zeros(c["n"], bool)
    if c["I"] > 0:
        zf, ozf = cap["z_fine"].detach().cpu().numpy(), ocap["z_fine"].detach().numpy()
        bad = np.abs(zf - ozf).max(1) > 1e-4 * np.maximum(1, np.abs(zf).max(1))
        # every screened ray explained by a u within 1e-5 of a reference CDF knot
        ocap = {k: v.detach() for k, v in ocap.items()}
        moved, explained = pdf_flips(cap["z_fine"], ocap, draws[-3])
        assert not (bad & ~moved).any(), f"z_fine differs without a moved importance depth, {c}"
        assert not (moved & ~explained).any(), f"z_fine moved away from any CDF knot, {c}"
    cap["_oracle"] = {k: v.detach() for k, v in ocap.items()}
    return (models, params, res, ref, bad, cap) if want_cap else (models, params, res, ref, bad)


CASES = list(range(24))


@pytest.mark.parametrize("seed,math", [(s, "f16x3") for s in CASES] +
                         [(s, m) for s in CASES[:6] for m in ("bf16x6", "fp32")])
def test_random_config_matches_oracle(seed, math, monkeypatch):
    """every fp32-accurate MLP arithmetic meets the same bound"""
    from nerf_pl_amd import ops
    monkeypatch.setattr(ops, "MATH", math)
    c = _config(seed)
    _, _, res, ref, bad, cap = _run(c, want_cap=True)
    assert bad.sum() <= max(1, 0.02 * c["n"]), f"{bad.sum()} sample_pdf bin flips in {c}"
    # rgb / depth / opacity and both passes' weights, 1e-4 absolute (tests/parity.py)
    assert_forward(res, ref, cap, cap["_oracle"], bad, label=f"{math} {c}")


def _oracle_grads(c, rays, draws, dt, ulp=None, z_fine=None):
    """the case's NeRF pair (optionally one fp32 ulp away, tests/grad64.py)
    through the oracle in dtype dt, the fine pass at depths z_fine when given"""
    params = []
    for s in (21 + c["seed"] % 5, 22 + c["seed"] % 5):
        p = O.make_params(s, sigma_bias=0.5)
        p = {k: v.to(dt) for k, v in p.items()} if ulp is None else grad64.ulp_perturbed(p, ulp + s, dt)
        params.append({k: v.requires_grad_(True) for k, v in p.items()})
    cap = {}
    args = (c["S"], c["use_disp"], c["perturb"], c["noise"], c["I"], 32768, c["white_back"], False)
    ref = O.render_rays(params, rays.to(dt), *args, rng=O.ReplayRNG([d.to(dt) for d in draws]),
                        capture=cap, z_fine_override=z_fine,
                        fp32_positions=dt == torch.float64)
    return params, ref, cap


def _functional(out, keep, seed):
    g = torch.Generator().manual_seed(seed)
    tot = 0
    for k in sorted(out):
        coef = torch.randn(out[k].shape, generator=g) * keep.view(-1, *[1] * (out[k].dim() - 1))
        tot = tot + (out[k] * coef.to(out[k].device, out[k].dtype)).sum()
    return tot


def _kinks(c, models, rays, draws, cap, cap64):
    """rays with a ReLU kink of the compositing between our sigma and the
    float64 oracle's (tests/grad64.py relu_kinks), coarse and fine"""
    from nerf_pl_amd import functions
    S, I, r = c["S"], c["I"], rays.to(DEV)
    passes = [(0, cap["z_coarse"], "raw_coarse", S, draws[1 if c["perturb"] > 0 else 0])]
    if I > 0:
        passes.append((1, cap["z_fine"], "raw_fine", S + I, draws[-1]))
    out = np.zeros(c["n"], bool)
    for mi, z, key, spr, noise in passes:
        with torch.no_grad():
            sig = functions.mlp_apply(models[mi], rays=r, z=z, spr=spr)[:, 3].view(-1, spr)
        k, e = grad64.relu_kinks(sig, cap64[key][..., 3].reshape(-1, spr), noise * c["noise"])
        assert e.all(), f"a compositing ReLU switched away from its kink, {c}"
        out |= k
    return out


def _mlp_kinks(c, saves, rays, cap, params, gmags):
    """rays with an MLP ReLU our training forward switched against float64
    (tests/grad64.py mlp_flips), every one explained by a float64
    pre-activation within 1e-5 of its kink"""
    passes = [cap["z_coarse"]] + ([cap["z_fine"]] if c["I"] > 0 else [])
    assert len(saves) == len(passes)
    out = np.zeros(c["n"], bool)
    for (save, n, _), z, p, gm in zip(saves, passes, params, gmags):
        z = z.detach().cpu()
        spr = z.shape[1]
        xyz = (rays[:, None, :3] + rays[:, None, 3:6] * z[:, :, None]).reshape(-1, 3)
        x64 = torch.cat([O.embed(xyz.double(), 10),
                         O.embed(rays[:, 3:6].double(), 4).repeat_interleave(spr, 0)], 1)
        flip, expl, _ = grad64.mlp_flips(save, n, x64, {k: v.detach().double() for k, v in p.items()},
                                         gmag=gm)
        assert expl.all(), f"an MLP ReLU switched away from its kink, {c}"
        out |= flip.reshape(-1, spr).any(1)
    return out


def _named(models_or_params, zeros_like=None):
    out = {}
    for i, m in enumerate(models_or_params):
        items = m.named_parameters() if hasattr(m, "named_parameters") else m.items()
        for k, v in items:
            g = v.grad
            out[f"m{i}.{k}"] = (torch.zeros(v.shape, dtype=torch.float64) if g is None
                                else g.detach().cpu().double())
    return out


@pytest.mark.parametrize("seed,math", [(s, m) for m in ("f16x3", "fp32")
                                       for s in (101, 102, 103, 104, 105)])
def test_random_config_gradients_match_oracle(seed, math, monkeypatch):
    """every parameter gradient within max(1e-4, 2 x the fp32 oracle's own
    distance from float64) of the float64 oracle (tests/grad64.py)"""
    from nerf_pl_amd import functions, ops
    monkeypatch.setattr(ops, "MATH", math)
    monkeypatch.setattr(functions, "_DEBUG", {})
    c = _config(seed)
    c["test_time"] = False
    c["n"] = max(c["n"], 64)
    models, params, res, _, _, cap_ours = _run(c, grad=True, want_cap=True)   # asserts the forward
    saves = functions._DEBUG["fwd_saves"]
    rays, draws = _rays(c), _draws(c)
    # every evaluation's fine pass at our depths (the reference detaches them,
    # rendering.py:253-255; see test_gpu_cfg4.py)
    zf = cap_ours["z_fine"].detach().cpu() if c["I"] > 0 else None
    pts = {u: (_oracle_grads(c, rays, draws, torch.float32, u, zf),
               _oracle_grads(c, rays, draws, torch.float64, u, zf)) for u in grad64.FLOOR_POINTS}
    (_, _, cap64) = pts[None][1]
    # rays whose compositing ReLU switched between ours and float64 are screened
    bad = _kinks(c, models, rays, draws, cap_ours, cap64)
    # ... and rays with an MLP ReLU our forward switched against float64 on a
    # sample whose output gradient matters (float64 d raw of the functional)
    raws = [cap64["raw_coarse"]] + ([cap64["raw_fine"]] if c["I"] > 0 else [])
    gm = torch.autograd.grad(_functional(pts[None][1][1], torch.ones(c["n"], dtype=torch.bool), seed),
                             raws, retain_graph=True)
    mk = _mlp_kinks(c, saves, rays, cap_ours, params, [g.abs().amax(1) for g in gm])
    print(f"{seed} {math}: {int(bad.sum())} rays with a compositing ReLU kink, {int(mk.sum())} with "
          f"an MLP ReLU flip, {int((bad | mk).sum())} of {c['n']} screened")
    bad |= mk
    keep = torch.from_numpy(~bad)
    # at most 10% of the rays: with up to 237 samples per ray x 2,304 ReLUs per
    # sample, an fp32 forward (ours or any) switches a few kinks on samples
    # that carry gradient (case 105: 10-17 of 281 rays, in both arithmetics)
    assert bad.sum() <= max(1, 0.1 * c["n"]), f"{bad.sum()} rays screened, {c}"
    _functional(res, keep, seed).backward()
    g32s, g64s = [], []
    for u, ((p32, r32, k32), (p64, r64, k64)) in pts.items():
        _functional(r32, keep, seed).backward()
        _functional(r64, keep, seed).backward()
        g32s.append(_named(p32))
        g64s.append(_named(p64))
    floor = grad64.fp32_floor(g32s, g64s)
    worst, where = grad64.check(_named(models), _named(pts[None][1][0]), floor, label=f"{seed} {math} {c}")
    print(f"{seed} {math}: worst {worst:.2f} of its bound ({where}, fp32 floor {floor[where]:.3g})")
