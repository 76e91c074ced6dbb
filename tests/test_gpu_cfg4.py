"""BASELINE.json configs[3] at its own size and shape: Blender lego 800x800,
64 coarse + 128 fine, rays sharded over 8 ranks (the Lightning DDP path,
train.py:167-178, whose DistributedSampler gives rank r perm[r::world] of the
shuffled pixel pool -- nerf_pl_amd.rays.RaySampler).  One rank's 4,096-ray
batch of the 100-pose orbit (64M rays in the pool) is drawn exactly as
bench.py --config cfg4 draws it on rank 5 of 8, generated on the device, and
checked against the CPU oracle (the reference's algorithm, pinned to the
reference by tests/golden) with the reference's random draws replayed:

* the rays themselves against the host restatement of get_ray_directions /
  get_rays (datasets/ray_utils.py) at 2e-6;
* render_rays' every output and both passes' weights at 1e-4 ABSOLUTE
  (tests/parity.py; depths reach ~200 at near/far 1/200), every ray whose
  fine depths moved explained by a sample_pdf knot flip (tests/screening.py);
* the training step's parameter gradients (MSE coarse + fine against the
  batch's target colours, train.py:107) on a 1,024-ray share of the batch,
  against the float64 oracle: within max(1e-4, 2 x the fp32 oracle's own
  distance from float64) per tensor (tests/grad64.py).  This step is
  ill-conditioned in fp32 (near/far 1/200: positions up to ~200 units out meet
  the 2^9 positional-encoding frequency), so the fp32 oracle's distance is
  taken at the unperturbed weights and at two points one fp32 ulp away (each
  against its own float64 evaluation), the largest of the three.
"""
import math

import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O
import grad64
from parity import assert_forward
from screening import pdf_flips

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
IMG, POSES, S, I, B = 800, 100, 64, 128, 4096
RANK, WORLD = 5, 8


def _batch():
    """rank RANK's first batch of bench.py --config cfg4 (same poses, pool,
    sampler seed and partition)"""
    from nerf_pl_amd.rays import RaySampler, blender_focal, generate_rays, pose_spherical
    poses = torch.stack([pose_spherical(-180.0 + 360.0 * k / POSES, -30.0, 4.0)
                         for k in range(POSES)])
    focal = blender_focal(IMG)
    torch.manual_seed(1234)
    pool_rgb = torch.rand(POSES * IMG * IMG, 3, device=DEV)
    sampler = RaySampler(poses.to(DEV), IMG, IMG, focal, 1.0, 200.0, rgb_pool=pool_rgb, seed=99,
                         rank=RANK, world=WORLD)
    sel = sampler.next_indices(B)
    rays, rgbs = generate_rays(poses.to(DEV), IMG, IMG, focal, 1.0, 200.0, sel, rgb_pool=pool_rgb)
    return poses, focal, sel.cpu(), rays.cpu(), rgbs.cpu()


def _draws(n, seed=17):
    g = torch.Generator().manual_seed(seed)
    return [torch.rand(n, S, generator=g), torch.randn(n, S, generator=g),
            torch.rand(n, I, generator=g), torch.rand(n, I, generator=g),
            torch.randn(n, S + I, generator=g)]


def _params(dt=torch.float32, grad=False):
    """the seeded NeRF pair"""
    return [{k: v.to(dt).requires_grad_(grad) for k, v in O.make_params(s, sigma_bias=0.5).items()}
            for s in (31, 32)]


def _models():
    from nerf_pl_amd import NeRF
    out = []
    for p in _params():
        m = NeRF()
        m.load_state_dict(p)
        out.append(m.to(DEV))
    return out


def _ours(models, rays, draws, cap=None):
    from nerf_pl_amd import Embedding, ReplayRNG, render_rays
    return render_rays(models, [Embedding(3, 10), Embedding(3, 4)], rays.to(DEV), S, False, 1.0,
                       1.0, I, 32768, False, rng=ReplayRNG(draws), _capture=cap)


def _screen(cap, ocap, draws):
    zf = cap["z_fine"].detach().cpu().numpy()
    ozf = ocap["z_fine"].detach().numpy()
    bad = np.abs(zf - ozf).max(1) > 1e-4 * np.maximum(1, np.abs(zf).max(1))
    moved, explained = pdf_flips(cap["z_fine"], {k: v.detach() for k, v in ocap.items()},
                                 draws[-3])
    assert not (bad & ~moved).any(), "z_fine differs although every importance depth matches"
    assert not (moved & ~explained).any(), \
        f"z_fine moved away from any CDF knot: rays {np.nonzero(moved & ~explained)[0][:8]}"
    return bad


def test_cfg4_rank_batch_rays():
    from nerf_pl_amd.rays import get_ray_directions, get_rays
    poses, focal, sel, rays, _ = _batch()
    assert rays.shape == (B, 8) and len(set(sel.tolist())) == B
    # rank r's share of the epoch: perm[r::world] of one permutation of all pixels
    assert int(sel.max()) < POSES * IMG * IMG
    dirs = get_ray_directions(IMG, IMG, focal).reshape(-1, 3)
    pose, pix = sel // (IMG * IMG), sel % (IMG * IMG)
    for k in torch.unique(pose).tolist():
        idx = torch.nonzero(pose == k).flatten()
        o, d = get_rays(dirs[pix[idx]], poses[k])
        torch.testing.assert_close(rays[idx, :3], o, rtol=0, atol=2e-6)
        torch.testing.assert_close(rays[idx, 3:6], d, rtol=0, atol=2e-6)
    assert (rays[:, 6] == 1.0).all() and (rays[:, 7] == 200.0).all()


def test_cfg4_rank_batch_matches_oracle():
    torch.set_num_threads(16)
    _, _, _, rays, _ = _batch()
    draws = _draws(B)
    cap, ocap = {}, {}
    with torch.no_grad():
        res = _ours(_models(), rays, draws, cap)
        ref = O.render_rays(_params(), rays, S, False, 1.0, 1.0, I, 32768, False,
                            rng=O.ReplayRNG(draws), capture=ocap)
    bad = _screen(cap, ocap, draws)
    assert bad.mean() <= 0.01, f"{bad.sum()} rays with a sample_pdf bin flip"
    assert_forward(res, ref, cap, ocap, bad, label="cfg4 rank batch")
    print(f"cfg4 rank batch: {int(bad.sum())} of {B} rays screened (sample_pdf knot flips)")


def _loss(out, tgt, keep):
    """losses.py MSELoss (coarse + fine) over the kept rays"""
    k = keep.to(out["rgb_coarse"].device, out["rgb_coarse"].dtype).view(-1, 1)
    t = tgt.to(out["rgb_coarse"].device, out["rgb_coarse"].dtype)
    n = k.sum() * 3
    return (((out["rgb_coarse"] - t) ** 2) * k).sum() / n + (((out["rgb_fine"] - t) ** 2) * k).sum() / n


def _oracle_point(dt, ulp, rays, draws, z_fine=None):
    """the seeded NeRF pair (optionally one fp32 ulp away) through the oracle in
    dtype dt, the fine pass at depths z_fine when given (the oracle's
    z_fine_override): (parameter dicts, outputs, captures)"""
    ps = []
    for s in (31, 32):
        p = O.make_params(s, sigma_bias=0.5)
        p = {k: v.to(dt) for k, v in p.items()} if ulp is None else grad64.ulp_perturbed(p, ulp + s, dt)
        ps.append({k: v.requires_grad_(True) for k, v in p.items()})
    cap = {}
    out = O.render_rays(ps, rays.to(dt), S, False, 1.0, 1.0, I, 32768, False,
                        rng=O.ReplayRNG([d.to(dt) for d in draws]), capture=cap,
                        z_fine_override=z_fine, fp32_positions=dt == torch.float64)
    return ps, out, cap


def _kinks(models, rays, cap, c64, draws):
    """rays with a ReLU kink of the compositing between our sigma and the
    float64 oracle's (grad64.relu_kinks; noise_std 1), coarse and fine"""
    from nerf_pl_amd import functions
    r = rays.to(DEV)
    with torch.no_grad():
        sc = functions.mlp_apply(models[0], rays=r, z=cap["z_coarse"], spr=S)[:, 3].view(-1, S)
        sf = functions.mlp_apply(models[1], rays=r, z=cap["z_fine"], spr=S + I)[:, 3].view(-1, S + I)
    kc, ec = grad64.relu_kinks(sc, c64["raw_coarse"][..., 3].view(-1, S), draws[1])
    kf, ef = grad64.relu_kinks(sf, c64["raw_fine"][..., 3].view(-1, S + I), draws[4])
    assert ec.all() and ef.all(), "a compositing ReLU switched away from its kink"
    print(f"cfg4: {int(kc.sum())} coarse / {int(kf.sum())} fine rays with a compositing ReLU kink")
    return kc | kf


def _mlp_kinks(saves, rays, cap, gmags):
    """rays with an MLP ReLU our forward switched against float64, coarse or
    fine (grad64.mlp_flips on the activations the training forward saved),
    every one explained by a float64 pre-activation within 1e-5 of its kink"""
    from oracle.nerf_oracle import embed
    p64 = [{k: v.double() for k, v in p.items()} for p in _params()]
    out = np.zeros(rays.shape[0], bool)
    counts = []
    for (save, n, _), z, p, gm in zip(saves, (cap["z_coarse"], cap["z_fine"]), p64, gmags):
        z = z.detach().cpu()
        spr = z.shape[1]
        xyz = (rays[:, None, :3] + rays[:, None, 3:6] * z[:, :, None]).reshape(-1, 3)
        x64 = torch.cat([embed(xyz.double(), 10),
                         embed(rays[:, 3:6].double(), 4).repeat_interleave(spr, 0)], 1)
        flip, expl, n_all = grad64.mlp_flips(save, n, x64, p, gmag=gm)
        assert expl.all(), f"an MLP ReLU switched away from its kink: samples {np.nonzero(~expl)[0][:8]}"
        counts.append((n_all, int(flip.sum())))
        out |= flip.reshape(-1, spr).any(1)
    print(f"cfg4: MLP ReLU flips against float64 (coarse, fine: all samples, samples with a "
          f"gradient >= 1e-5 of the largest): {counts}")
    return out


@pytest.mark.parametrize("math_", ["f16x3", "fp32"])
def test_cfg4_training_step_gradients_match_oracle(math_, monkeypatch):
    """every parameter gradient within max(1e-4, 2 x the fp32 oracle's own
    distance from float64) of the float64 oracle (tests/grad64.py), the float64
    evaluations on the fp32 sample positions our kernels see (the oracle's
    fp32_positions), so the floor measures the MLP's and the compositing's
    accumulation, not the input rounding"""
    from nerf_pl_amd import functions, ops
    monkeypatch.setattr(ops, "MATH", math_)
    monkeypatch.setattr(functions, "_DEBUG", {})
    torch.set_num_threads(16)
    n = 1024
    _, _, _, rays, rgbs = _batch()
    rays, rgbs = rays[:n].contiguous(), rgbs[:n]
    draws = _draws(B)
    draws = [d[:n] for d in draws]
    models = _models()
    cap = {}
    res = _ours(models, rays, draws, cap)
    saves = functions._DEBUG["fwd_saves"]
    assert len(saves) == 2 and saves[0][1] == n * S and saves[1][1] == n * (S + I)
    # the forward at the reference's own depths: every depth that moved is a
    # sample_pdf knot flip (asserted in _screen)
    (_, _, c32) = _oracle_point(torch.float32, None, rays, draws)
    _screen(cap, c32, draws)
    # the gradients with every evaluation's fine pass at our depths (the
    # reference detaches them, rendering.py:253-255): at near/far 1/200 the 2^9
    # encoding frequency turns the 1e-6 relative depth shift of a coarse pass's
    # rounding into 0.1 rad of phase -- a forward-precision matter the 1e-4
    # depth bound above covers, not a gradient one
    zf = cap["z_fine"].detach().cpu()
    pts = {u: (_oracle_point(torch.float32, u, rays, draws, zf), _oracle_point(torch.float64, u, rays, draws, zf))
           for u in grad64.FLOOR_POINTS}
    (_, _, c64) = pts[None][1]
    # rays whose compositing ReLU switched between ours and float64 leave the
    # loss (tests/grad64.py)
    bad = _kinks(models, rays, cap, c64, draws)
    # ... and so are rays with an MLP ReLU our forward switched against float64
    # on a sample whose output gradient matters (float64 d raw of the loss)
    gm = torch.autograd.grad(_loss(pts[None][1][1], rgbs, torch.ones(n, dtype=torch.bool)),
                             [c64["raw_coarse"], c64["raw_fine"]], retain_graph=True)
    bad |= _mlp_kinks(saves, rays, cap, [g.abs().amax(1) for g in gm])
    assert bad.mean() <= 0.02, f"{bad.sum()} rays screened"
    keep = torch.from_numpy(~bad)
    _loss(res, rgbs, keep).backward()
    ours = {f"m{i}.{k}": w.grad.detach().cpu() for i, m in enumerate(models)
            for k, w in m.named_parameters()}
    g32s, g64s = [], []
    for u, ((p32, o32, k32), (p64, o64, k64)) in pts.items():
        _loss(o32, rgbs, keep).backward()
        _loss(o64, rgbs, keep).backward()
        g32s.append({f"m{i}.{k}": v.grad for i, p in enumerate(p32) for k, v in p.items()})
        g64s.append({f"m{i}.{k}": v.grad for i, p in enumerate(p64) for k, v in p.items()})
    spread = {}
    floor = grad64.fp32_floor(g32s, g64s, spread)
    g64 = {f"m{i}.{k}": v.grad for i, p in enumerate(pts[None][1][0]) for k, v in p.items()}
    fl = sorted(floor.values())
    print(f"cfg4 {math_}: fp32 floors over {len(fl)} tensors: median {fl[len(fl) // 2]:.2g}, "
          f"{sum(f <= 1e-4 for f in fl)} at or below 1e-4, largest {fl[-1]:.2g} "
          f"({max(floor, key=floor.get)})")
    worst, where = grad64.check(ours, g64, floor, label=f"cfg4 {math_}")
    assert math.isfinite(worst)
    print(f"cfg4 {math_} gradients: worst {worst:.2f} of its bound ({where}, fp32 floor "
          f"{floor[where]:.3g}, {len(g32s)} floor points: "
          + " ".join(f"{v:.2g}" for v in spread[where]) + ")")
