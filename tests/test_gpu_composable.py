"""The composable path of the drop-in: configurations the fused
kernels do not implement -- other NeRF depths / widths / skips, other
embedding frequencies, linear frequency bands -- run the reference's
``inference`` sequence on device GEMMs, with the HIP sampling and compositing
kernels, and match the oracle (the same sequence on the CPU,
``oracle.nerf_oracle.render_rays(arch=...)``) at the north star's bound:
rgb / opacity 1e-4 abs, depth 1e-4 relative; parameter gradients within
max(1e-4, the oracle's own fp32-vs-float64 distance) of each tensor's norm
(the bound of tests/test_gpu_random.py: the 2^9 positional-encoding band
makes this gradient ill-conditioned in fp32).
Every reference caller uses the defaults; this is the boundary's fallback,
not the hot path."""
import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O
from parity import assert_forward

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)

ARCHS = [
    dict(D=4, W=64, skips=[2], xyz_freqs=6, dir_freqs=2, xyz_logscale=True, dir_logscale=True),
    dict(D=3, W=32, skips=[], xyz_freqs=4, dir_freqs=3, xyz_logscale=False, dir_logscale=True),
    dict(D=8, W=256, skips=[4], xyz_freqs=10, dir_freqs=4, xyz_logscale=True,
         dir_logscale=False),                      # default NeRF, linear dir bands
]


def _setup(arch, seed):
    from nerf_pl_amd import Embedding, NeRF
    in_xyz = 3 * (2 * arch["xyz_freqs"] + 1)
    in_dir = 3 * (2 * arch["dir_freqs"] + 1)
    torch.manual_seed(seed)
    models, params = [], []
    for _ in range(2):
        m = NeRF(arch["D"], arch["W"], in_xyz, in_dir, arch["skips"])
        with torch.no_grad():
            m.sigma.bias.fill_(0.5)
        params.append({k: v.detach().clone() for k, v in m.state_dict().items()})
        models.append(m.to(DEV))
    emb = [Embedding(3, arch["xyz_freqs"], arch["xyz_logscale"]),
           Embedding(3, arch["dir_freqs"], arch["dir_logscale"])]
    return models, params, emb


def _rays(n, seed):
    g = torch.Generator().manual_seed(seed)
    o = torch.randn(n, 3, generator=g) * 0.3
    d = torch.nn.functional.normalize(torch.randn(n, 3, generator=g), dim=1)
    return torch.cat([o, d, torch.full((n, 1), 2.0), torch.full((n, 1), 6.0)], 1)


def _draws(n, S, I, seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.rand(n, S, generator=g), torch.randn(n, S, generator=g),
            torch.rand(n, I, generator=g), torch.rand(n, I, generator=g),
            torch.randn(n, S + I, generator=g)]


@pytest.mark.parametrize("k", range(len(ARCHS)))
def test_composable_render_matches_oracle(k):
    from nerf_pl_amd import ReplayRNG, render_rays
    from nerf_pl_amd.rendering import _fused_ok
    arch = ARCHS[k]
    n, S, I = 300, 24, 20
    models, params, emb = _setup(arch, 30 + k)
    assert not _fused_ok(models, emb)
    rays, draws = _rays(n, k), _draws(n, S, I, 40 + k)
    for p in params:
        for v in p.values():
            v.requires_grad_(True)
    cap, ocap = {}, {}
    res = render_rays(models, emb, rays.to(DEV), S, False, 1.0, 1.0, I, 32768, False,
                      rng=ReplayRNG(draws), _capture=cap)
    ref = O.render_rays(params, rays, S, False, 1.0, 1.0, I, 32768, False,
                        rng=O.ReplayRNG(draws), capture=ocap, arch=arch)
    p64 = [{k_: v.detach().double().requires_grad_(True) for k_, v in p.items()} for p in params]
    cap64 = {}
    ref64 = O.render_rays(p64, rays.double(), S, False, 1.0, 1.0, I, 32768, False,
                          rng=O.ReplayRNG([d.double() for d in draws]), capture=cap64, arch=arch)
    zf, ozf = cap["z_fine"].detach().cpu().numpy(), ocap["z_fine"].detach().numpy()
    z64 = cap64["z_fine"].detach().numpy()
    bad = np.abs(zf - ozf).max(1) > 1e-4 * np.maximum(1, np.abs(zf).max(1))
    bad |= np.abs(z64 - ozf).max(1) > 1e-4 * np.maximum(1, np.abs(z64).max(1))
    assert bad.sum() <= 6
    # 1e-4 absolute on every output and both passes' weights (tests/parity.py);
    # rays screened above differ in their fine depths only
    assert_forward(res, ref, cap, {k_: v.detach() for k_, v in ocap.items()}, bad,
                   label=f"composable arch {k}")
    keep = torch.from_numpy(~bad)
    g = torch.Generator().manual_seed(k)
    coef = {key: torch.randn(ref[key].shape, generator=g) * keep.view(-1, *[1] * (ref[key].dim() - 1))
            for key in sorted(ref)}
    sum((res[key] * coef[key].to(DEV)).sum() for key in coef).backward()
    sum((ref[key] * coef[key]).sum() for key in coef).backward()
    sum((ref64[key] * coef[key].double()).sum() for key in coef).backward()
    for m, p, q in zip(models, params, p64):
        for name, w in m.named_parameters():
            exp = p[name].grad.double()
            scale = exp.norm() + 1e-30
            bound = max(1e-4, float((exp - q[name].grad).norm() / scale))
            dev = float((w.grad.detach().cpu().double() - exp).norm() / scale)
            assert dev <= bound, (name, dev, bound)


def test_composable_test_time_and_sigma_only():
    """test_time (sigma-only coarse pass, rendering.py:237-241) on the
    composable path, and NeRF.forward(x, sigma_only=True) on embedded input."""
    from nerf_pl_amd import ReplayRNG, render_rays
    arch = ARCHS[0]
    n, S, I = 64, 16, 8
    models, params, emb = _setup(arch, 50)
    rays, draws = _rays(n, 5), _draws(n, S, I, 6)
    with torch.no_grad():
        res = render_rays(models, emb, rays.to(DEV), S, False, 1.0, 1.0, I, 32768, False, True,
                          rng=ReplayRNG(draws))
    ref = O.render_rays(params, rays, S, False, 1.0, 1.0, I, 32768, False, True,
                        rng=O.ReplayRNG(draws), arch=arch)
    assert sorted(res) == sorted(ref)
    for key in ref:
        assert np.abs(res[key].cpu().numpy() - ref[key].numpy()).max() <= 1e-4, key
    x = torch.rand(50, 3 * (2 * arch["xyz_freqs"] + 1))
    got = models[0](x.to(DEV), sigma_only=True).detach().cpu()
    exp = O.nerf_forward(params[0], x, sigma_only=True, D=arch["D"], skips=arch["skips"],
                         in_xyz=x.shape[1])
    assert got.shape == exp.shape == (50, 1)
    assert (got - exp).abs().max().item() <= 1e-5
