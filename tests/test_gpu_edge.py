"""Edge cases and full-size parity of the drop-in ``render_rays``.

* full BASELINE batches (cfg2: 4096 rays, 64+128, near/far 1/200; cfg3: 4096
  NDC rays, 64+64) against the CPU oracle (the reference's algorithm,
  tests/test_oracle_golden.py pins it to the reference) with the reference's
  draws replayed: 1e-4 ABSOLUTE on rgb, depth, opacity and the coarse and
  fine weights (north star, tests/parity.py), sample_pdf bin flips screened
  per ray as in test_gpu_render.py;
* size-independent properties past what the oracle finishes in seconds:
  a ray's outputs do not depend on the rest of its batch (bit-exact, 65,536
  rays), and the parameter gradient of a summed loss is additive over a
  batch split (16,384 rays = 3.1M fine samples per MLP call, past the 2^31
  bytes of a saved segment);
* the reference's failure and corner cases: an empty batch raises (its
  inference() concatenates an empty chunk list, rendering.py:161), one ray,
  one sample per ray, non-device / wrongly shaped / wrongly typed inputs.
"""
import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O
from parity import assert_forward
from screening import pdf_flips

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _emb():
    from nerf_pl_amd import Embedding
    return [Embedding(3, 10), Embedding(3, 4)]


def _models(seeds=(11, 12), sigma_bias=0.5):
    from nerf_pl_amd import NeRF
    out = []
    for s in seeds:
        m = NeRF()
        m.load_state_dict(O.make_params(s, sigma_bias=sigma_bias))
        out.append(m.to(DEV))
    return out


def _draws(n, S, I, perturb, seed):
    """the reference's five draws in its order"""
    g = torch.Generator().manual_seed(seed)
    d = []
    if perturb > 0:
        d.append(torch.rand(n, S, generator=g))
    d.append(torch.randn(n, S, generator=g))
    if I > 0:
        d += [torch.rand(n, I, generator=g), torch.rand(n, I, generator=g),
              torch.randn(n, S + I, generator=g)]
    return d


def _slice_draws(draws, idx):
    return [t[idx] for t in draws]


def _ours(models, rays, S, I, draws, perturb=1.0, noise=1.0, grad=False, cap=None):
    from nerf_pl_amd import ReplayRNG, render_rays
    with torch.set_grad_enabled(grad):
        return render_rays(models, _emb(), rays.to(DEV), S, False, perturb, noise, I, 32768, False,
                           rng=ReplayRNG(draws), _capture=cap)


def _screen(cap, ocap, draws, limit=0.01):
    """rays whose fine depths moved (a sample_pdf bin flip), every one
    explained by a reference u within 1e-5 of a CDF knot (screening.pdf_flips)"""
    if "z_fine" not in cap:
        return np.zeros(cap["z_coarse"].shape[0], bool)
    bad = (cap["z_fine"].cpu().numpy() != ocap["z_fine"].numpy()).any(1)
    moved, explained = pdf_flips(cap["z_fine"], ocap, draws[-3])
    assert not (bad & ~moved).any(), "z_fine differs although every importance depth matches"
    assert not (moved & ~explained).any(), \
        f"z_fine moved away from any CDF knot: rays {np.nonzero(moved & ~explained)[0][:8]}"
    assert bad.mean() <= limit, f"{bad.sum()} rays with a sample_pdf bin flip"
    return bad


@pytest.mark.parametrize("kind", ["cfg2", "cfg3"])
def test_full_batch_matches_oracle(kind):
    """BASELINE configs[1] / [2] at their full batch of 4096 rays."""
    from nerf_pl_amd.rays import blender_rays, llff_ndc_rays
    torch.set_num_threads(16)
    g = torch.Generator().manual_seed(5)
    if kind == "cfg2":
        pool, S, I = blender_rays(400, 4, near=1.0, far=200.0), 64, 128
    else:
        pool, S, I = llff_ndc_rays(504, 378, n_poses=2), 64, 64
    rays = pool[torch.randperm(pool.shape[0], generator=g)[:4096]].contiguous()
    draws = _draws(4096, S, I, 1.0, 9)
    models = _models()
    cap = {}
    res = _ours(models, rays, S, I, draws, cap=cap)
    params = [O.make_params(11, sigma_bias=0.5), O.make_params(12, sigma_bias=0.5)]
    ocap = {}
    ref = O.render_rays(params, rays, S, False, 1.0, 1.0, I, 32768, False,
                        rng=O.ReplayRNG(draws), capture=ocap)
    bad = _screen(cap, ocap, draws)
    # rgb / depth / opacity and the coarse and fine weights, 1e-4 absolute
    assert_forward(res, ref, cap, ocap, bad, label=kind)


def test_rays_do_not_depend_on_their_batch():
    """65,536 rays (12.6M fine samples) vs 512 of them rendered alone: equal
    bit for bit, and the 512 match the oracle."""
    from nerf_pl_amd.rays import blender_rays
    n, S, I = 65536, 64, 128
    pool = blender_rays(256, 1, near=2.0, far=6.0)
    rays = pool[:n].contiguous()
    draws = _draws(n, S, I, 1.0, 3)
    models = _models()
    full = _ours(models, rays, S, I, draws)
    idx = torch.arange(7, n, n // 512)[:512]
    cap, ocap = {}, {}
    part = _ours(models, rays[idx].contiguous(), S, I, _slice_draws(draws, idx), cap=cap)
    for k in part:
        assert torch.equal(full[k][idx.to(DEV)], part[k]), k
    params = [O.make_params(11, sigma_bias=0.5), O.make_params(12, sigma_bias=0.5)]
    ref = O.render_rays(params, rays[idx].contiguous(), S, False, 1.0, 1.0, I, 32768, False,
                        rng=O.ReplayRNG(_slice_draws(draws, idx)), capture=ocap)
    bad = _screen(cap, ocap, _slice_draws(draws, idx))
    assert_forward(part, ref, cap, ocap, bad, label="512 of 65536")


@pytest.mark.parametrize("math", ["f16x3", "bf16"])
def test_gradient_is_additive_over_a_batch_split(math, monkeypatch):
    """sum-of-squares loss over 16,384 rays (64+128: 3.1M fine samples, every
    saved 256-wide segment > 2^31 bytes) = the same loss over its two halves:
    the parameter gradients add up (fp32 summation order only)."""
    from nerf_pl_amd import ops
    from nerf_pl_amd.rays import blender_rays
    monkeypatch.setattr(ops, "MATH", math)
    n, S, I = 16384, 64, 128
    rays = blender_rays(128, 1, near=2.0, far=6.0).contiguous()
    assert rays.shape[0] == n
    draws = _draws(n, S, I, 1.0, 4)
    target = (0.5 + 0.4 * torch.sin(3 * rays[:, 3:6])).to(DEV)
    models = _models()

    def grads(sel):
        for m in models:
            m.zero_grad(set_to_none=True)
        res = _ours(models, rays[sel].contiguous(), S, I, _slice_draws(draws, sel), grad=True)
        t = target[sel.to(DEV)]
        loss = ((res["rgb_coarse"] - t) ** 2).sum() + ((res["rgb_fine"] - t) ** 2).sum()
        loss.backward()
        return [p.grad.detach().clone() for m in models for p in m.parameters()], loss.item()

    allidx = torch.arange(n)
    g_all, l_all = grads(allidx)
    g_a, l_a = grads(allidx[: n // 2])
    g_b, l_b = grads(allidx[n // 2:])
    np.testing.assert_allclose(l_all, l_a + l_b, rtol=1e-5)
    names = [f"{i}.{k}" for i, m in enumerate(models) for k, _ in m.named_parameters()]
    for name, ga, a, b in zip(names, g_all, g_a, g_b):
        assert torch.isfinite(ga).all(), name
        s = a + b
        scale = s.abs().max().item() + 1e-30
        err = (ga - s).abs().max().item() / scale
        assert err < 1e-4, f"{math} {name}: |g(all) - g(half1) - g(half2)| = {err:.3g} of max|g|"


def test_single_ray_and_single_sample():
    from nerf_pl_amd.rays import blender_rays
    params = [O.make_params(11, sigma_bias=0.5), O.make_params(12, sigma_bias=0.5)]
    rays = blender_rays(16, 1, near=2.0, far=6.0)[100:101].contiguous()
    for S, I in ((64, 128), (3, 1), (1, 0)):
        draws = _draws(1, S, I, 1.0, 2)
        cap, ocap = {}, {}
        res = _ours(_models(), rays, S, I, draws, cap=cap)
        ref = O.render_rays(params, rays, S, False, 1.0, 1.0, I, 32768, False,
                            rng=O.ReplayRNG(draws), capture=ocap)
        assert_forward(res, ref, cap, ocap, np.zeros(1, bool), label=f"1 ray S={S} I={I}")


def test_empty_batch_raises_like_reference():
    with pytest.raises(ValueError):
        _ours(_models(), torch.zeros(0, 8), 64, 128, _draws(0, 64, 128, 1.0, 0))
    # the oracle (the reference's algorithm) fails the same way
    with pytest.raises((ValueError, RuntimeError)):
        O.render_rays([O.make_params(1), O.make_params(2)], torch.zeros(0, 8), 64, False, 1.0,
                      1.0, 128, 32768, False, rng=O.ReplayRNG(_draws(0, 64, 128, 1.0, 0)))
    # NeRF.forward on no samples returns an empty (0, 4) like nn.Linear
    out = _models()[0](torch.zeros(0, 90, device=DEV))
    assert tuple(out.shape) == (0, 4)


def test_bad_inputs_raise():
    from nerf_pl_amd import Embedding, ReplayRNG, render_rays
    models = _models()
    rays = torch.rand(8, 8, device=DEV)
    with pytest.raises(RuntimeError):            # no CPU path
        render_rays(models, _emb(), rays.cpu(), 8, False, 0, 1, 0)
    with pytest.raises(ValueError):              # rays must be (N, 8)
        render_rays(models, _emb(), rays[:, :7], 8, False, 0, 1, 0)
    with pytest.raises(TypeError):               # float32 only
        render_rays(models, _emb(), rays.double(), 8, False, 0, 1, 0)
    with pytest.raises((RuntimeError, ValueError)):   # embedding width != the model's input
        render_rays(models, [Embedding(3, 8), Embedding(3, 4)], rays, 8, False, 0, 1, 0)
    with pytest.raises(ValueError):              # replayed draw of the wrong shape
        render_rays(models, _emb(), rays, 8, False, 1.0, 1, 0,
                    rng=ReplayRNG([torch.rand(8, 9)]))
