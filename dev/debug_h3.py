"""Debug the f16x3 backward on a golden gradient case: stats, non-finite
segments, segment maxima (GPU box; sets NERF_PL_AMD_DEBUG=1 itself).

    python dev/debug_h3.py cfg1_grad
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
os.environ["NERF_PL_AMD_DEBUG"] = "1"

from conftest import golden_cfg, load_golden  # noqa: E402
from nerf_pl_amd import functions, ops  # noqa: E402
import test_gpu_render as T  # noqa: E402


def main(case):
    fx = load_golden(case)
    cfg = golden_cfg(fx)
    models = T.build_models(cfg)
    res, _ = T.run_ours(fx, cfg, models, grad=True)
    target = torch.from_numpy(fx["target"]).to(T.DEV)
    loss = torch.mean((res["rgb_coarse"] - target) ** 2)
    if "rgb_fine" in res:
        loss = loss + torch.mean((res["rgb_fine"] - target) ** 2)
    loss.backward()
    torch.cuda.synchronize()
    d = functions._DEBUG
    n = d["n"]
    nb = ops.n_blocks(n)
    sv, gw = d["save"].cpu(), d["grad_ws"].cpu()
    print("n", n, "stats", sv[nb * ops.SAVE_PER_BLOCK:].tolist())
    print("g_out max", d["g_out"].abs().max(0).values.tolist())
    W = 32 * 256
    for l in range(9):
        seg = gw[l * W * nb:(l + 1) * W * nb]
        print(f"dz{l + 1}: max {seg.abs().max().item():.4g} finite {bool(torch.isfinite(seg).all())}")
    seg = gw[9 * W * nb: 9 * W * nb + 32 * 128 * nb]
    print(f"dzdir: max {seg.abs().max().item():.4g} finite {bool(torch.isfinite(seg).all())}")
    g = d["gflat"].cpu()
    bad = torch.nonzero(~torch.isfinite(g)).flatten()
    print("gflat non-finite:", bad.numel(), bad[:10].tolist())


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "cfg1_grad")
