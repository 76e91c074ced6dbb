import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


def golden_cases():
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz"))


def load_golden_path(path):
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def load_golden(name):
    return load_golden_path(os.path.join(GOLDEN, name + ".npz"))


def golden_cfg(fx):
    c = fx["cfg"]
    return dict(N_samples=int(c[0]), N_importance=int(c[1]), perturb=float(c[2]),
                noise_std=float(c[3]), use_disp=bool(c[4]), white_back=bool(c[5]),
                test_time=bool(c[6]), chunk=int(c[7]), sigma_bias=float(c[8]),
                seeds=(int(c[9]), int(c[10])))


def golden_draws(fx):
    return [fx[f"draw{i}"] for i in range(int(fx["n_draws"]))]


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    return torch.cuda.is_available()
