"""The ray-generation oracle (oracle/rays_oracle.py) against fixtures made by
the reference's own get_rays / get_ndc_rays (datasets/ray_utils.py:27-93;
tests/golden/make_golden_rays.py runs them on the same directions and poses).
Bit-exact on the host that made them; elsewhere the 3x3 product's BLAS order
may move an ulp, so the bound is 2 fp32 ulps of the value (relative 2.4e-7)
plus 1e-7 absolute for NDC's near-zero components."""
import os

import numpy as np
import torch

from oracle import rays_oracle as RO

FX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rays", "rays.npz")


def _cases():
    z = np.load(FX)
    for k in range(int(z["n_cases"])):
        H, W, f, ndc = z[f"c{k}_cfg"]
        yield (int(H), int(W), float(f), bool(ndc), torch.from_numpy(z[f"c{k}_poses"]),
               z[f"c{k}_rays_o"], z[f"c{k}_rays_d"], z[f"c{k}_dirs"])


def test_directions_restatement_shape_and_values():
    for H, W, f, _, _, _, _, dirs in _cases():
        got = RO.get_ray_directions(H, W, f).numpy()
        assert got.shape == (H, W, 3)
        assert np.array_equal(got, dirs)


def test_oracle_rays_match_reference_functions():
    for H, W, f, ndc, poses, ro, rd, _ in _cases():
        dirs = RO.get_ray_directions(H, W, f)
        os_, ds_ = [], []
        for c2w in poses:
            o, d = RO.get_rays(dirs, c2w)
            if ndc:
                o, d = RO.get_ndc_rays(H, W, f, 1.0, o, d)
            os_.append(o)
            ds_.append(d)
        for got, exp in ((torch.cat(os_).numpy(), ro), (torch.cat(ds_).numpy(), rd)):
            assert got.shape == exp.shape
            assert np.all(np.abs(got - exp) <= 2.4e-7 * np.abs(exp) + 1e-7), (H, W, ndc)
