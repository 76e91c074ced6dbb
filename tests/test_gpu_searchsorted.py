"""The standalone torchsearchsorted entry point (the reference's only native
API, models/rendering.py:2,37): bit-exact against torch.searchsorted -- the
replacement the reference itself uses (rendering_shadows.py:41) -- on the
golden fixtures' CDFs with their recorded u draws, both sides, plus broadcast
rows, ties, out-of-range values, NaN and empty shapes.  parity unpinned at the
upstream extension (absent from the container: empty submodule, no pinned
commit); pinned to the reference's call site by the golden fixtures."""
import numpy as np
import pytest
import torch

from conftest import golden_draws
from test_gpu_kernels import oracle_case

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _cdf(w):
    # rendering.py:29-33
    w = w[:, 1:-1] + 1e-5
    pdf = w / torch.sum(w, -1, keepdim=True)
    return torch.cat([torch.zeros_like(pdf[:, :1]), torch.cumsum(pdf, -1)], -1)


@pytest.mark.parametrize("case", ["cfg2_n1200", "cfg3_ndc", "ragged"])
@pytest.mark.parametrize("side", ["left", "right"])
def test_searchsorted_on_golden_cdfs(case, side):
    from nerf_pl_amd import searchsorted
    fx, cfg, _, cap = oracle_case(case)
    cdf = _cdf(cap["weights_coarse"]).contiguous()
    u = torch.from_numpy(golden_draws(fx)[-3]).contiguous()     # rand(B, I), rendering.py:36
    ref = torch.searchsorted(cdf, u, right=(side == "right"))
    got = searchsorted(cdf.to(DEV), u.to(DEV), side=side)
    assert got.dtype == torch.int64 and got.shape == ref.shape
    assert torch.equal(got.cpu(), ref)


def test_searchsorted_edges():
    from nerf_pl_amd import searchsorted
    a = torch.tensor([[0., 0.25, 0.25, 0.5, 1.0]])
    v = torch.tensor([[-1., 0., 0.25, 0.3, 1.0, 2.0, float("nan")]])
    for side in ("left", "right"):
        ref = torch.searchsorted(a, v, right=(side == "right"))
        assert torch.equal(searchsorted(a.to(DEV), v.to(DEV), side=side).cpu(), ref), side
    # broadcast: one row of a against many rows of v, and the reverse; float64; out=
    g = torch.Generator().manual_seed(3)
    a1 = torch.sort(torch.rand(1, 33, generator=g, dtype=torch.float64), -1).values
    vm = torch.rand(17, 9, generator=g, dtype=torch.float64)
    out = torch.empty(17, 9, dtype=torch.int64, device=DEV)
    r = searchsorted(a1.to(DEV), vm.to(DEV), out=out, side="right")
    assert r is out
    assert torch.equal(out.cpu(), torch.searchsorted(a1.expand(17, 33).contiguous(), vm, right=True))
    am = torch.sort(torch.rand(5, 8, generator=g), -1).values
    v1 = torch.rand(1, 6, generator=g)
    assert torch.equal(searchsorted(am.to(DEV), v1.to(DEV)).cpu(),
                       torch.searchsorted(am, v1.expand(5, 6).contiguous()))
    assert searchsorted(torch.zeros(0, 4, device=DEV), torch.zeros(0, 3, device=DEV)).shape == (0, 3)
    assert torch.equal(searchsorted(torch.zeros(2, 0, device=DEV), torch.rand(2, 3, device=DEV)).cpu(),
                       torch.zeros(2, 3, dtype=torch.int64))
    with pytest.raises(ValueError):
        searchsorted(torch.rand(3, 4, device=DEV), torch.rand(2, 4, device=DEV))
    with pytest.raises(RuntimeError):
        searchsorted(torch.rand(3, 4), torch.rand(3, 4))
