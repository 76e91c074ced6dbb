"""Same-host bit-exactness of the oracle against the REFERENCE run live.

Runs only in the build container, where /root/reference exists (it never exists
on the GPU box; the test skips there).  The reference is driven through the
fixture generator (tests/golden/make_golden.py: torchsearchsorted shim, recorded
random draws) into a temporary fixture, and the oracle replays the same draws:
on one host both use the same PyTorch-CPU kernels, so every output,
intermediate and the MLP's raw outputs must be bit-identical."""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN

REF = os.environ.get("NERF_REFERENCE", "/root/reference")
pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "models")),
                                reason="reference checkout not present (GPU box)")


@pytest.fixture(scope="module")
def mg():
    sys.path.insert(0, GOLDEN)
    import make_golden
    make_golden.import_reference()
    return make_golden


CASES = [
    dict(name="live_cfg2", n=24, seed=21, near=2.0, far=6.0, N_samples=64, N_importance=128,
         perturb=1.0, noise_std=1.0, sigma_bias=0.5),
    dict(name="live_cfg1", n=32, seed=22, near=1.0, far=200.0, N_samples=32, N_importance=0,
         perturb=1.0, noise_std=1.0),
    dict(name="live_testtime", n=16, seed=23, near=2.0, far=6.0, N_samples=64,
         N_importance=64, perturb=0.0, noise_std=0.0, test_time=True),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_oracle_bit_exact_vs_live_reference(case, mg, tmp_path, monkeypatch):
    import test_oracle_golden as T
    from conftest import load_golden_path
    c = dict(case)
    n, seed, near, far = c.pop("n"), c.pop("seed"), c.pop("near"), c.pop("far")
    rays = mg.pick(mg.blender_rays(64, 2, near=near, far=far), n, seed)
    monkeypatch.setattr(mg, "HERE", str(tmp_path))
    torch.manual_seed(0)
    mg.run_case(*mg.import_reference(), rays=rays, **c)
    fx = load_golden_path(os.path.join(str(tmp_path), c["name"] + ".npz"))
    _, res, cap = T._run_oracle(fx)
    for k in [k for k in fx if k.startswith("out_")]:
        np.testing.assert_array_equal(res[k[4:]].detach().numpy(), fx[k], err_msg=k)
    np.testing.assert_array_equal(cap["raw_coarse"].numpy(), fx["raw_coarse"])
    if "raw_fine" in fx:
        np.testing.assert_array_equal(cap["raw_fine"].numpy(), fx["raw_fine"])
        np.testing.assert_array_equal(cap["z_pdf"].numpy(), fx["z_pdf"])
