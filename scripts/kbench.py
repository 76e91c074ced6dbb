"""Isolated timing of the fused MLP kernels at the cfg2 fine-pass size
(786,432 samples), for profiling (dev tool).
Usage: kbench.py [fwd|fwdsave|fwd3|fwd3save|bwd|bwd3|wgrad|wgrad3|fwdh3|fwdh3save|bwdh3|wgradh3
                  |fwdb1|fwdb1save|bwdb1|wgradb1|all|h3|b1] [reps]
                  (x3 = bf16x6, h3 = f16x3, b1 = plain bf16)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from nerf_pl_amd import ops, packing
from nerf_pl_amd._lib import call, stream_of
from nerf_pl_amd.functions import _wgrad_workspace

FLOP = {"fwd": 1186816, "fwdsave": 1186816, "fwd3": 1186816, "fwd3save": 1186816,
        "bwd": 1115392, "bwd3": 1115392, "wgrad": 1186816, "wgrad3": 1186816,
        "fwdh3": 1186816, "fwdh3save": 1186816, "bwdh3": 1115392, "wgradh3": 1186816,
        "fwdb1": 1186816, "fwdb1save": 1186816, "bwdb1": 1115392, "wgradb1": 1186816}
PEAK3 = 2516.6 / 6     # bf16 dense MFMA peak / 6 products: fp32-equivalent ceiling of bf16x6
PEAKH3 = 2516.6 / 3    # fp16 dense MFMA peak / 3 products: ceiling of f16x3


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    flat = (torch.rand(packing.N_PARAMS, device=dev) - 0.5) * 0.15
    if os.environ.get("NR_KB_ZERO") == "1":     # all-zero weights: the power (DVFS) control
        flat.zero_()
    pf, pb = ops.pack_fwd_fp32(flat), ops.pack_bwd_fp32(flat)
    p3, pb3 = ops.pack_fwd3(flat), ops.pack_bwd(flat, math="bf16x6")
    ph3, pbh3 = ops.pack_fwd3(flat, math="f16x3"), ops.pack_bwd(flat, math="f16x3")
    pb1, pbb1 = ops.pack_fwd3(flat, math="bf16"), ops.pack_bwd(flat, math="bf16")
    n_rays, spr = int(os.environ.get("NR_KB_RAYS", "4096")), 192   # NR_KB_RAYS: launch-size sweeps
    n = n_rays * spr
    rays = torch.randn(n_rays, 8, device=dev)
    rays[:, 3:6] = torch.nn.functional.normalize(rays[:, 3:6], dim=-1)
    rays[:, 6], rays[:, 7] = 2.0, 6.0
    z = (torch.rand(n, device=dev) * 4 + 2).contiguous()
    out, sv = ops.mlp_forward(pf, rays=rays, z=z, samples_per_ray=spr, save=True)
    gout = torch.randn(n, 4, device=dev)
    gw = torch.empty(ops.n_blocks(n) * ops.GRAD_PER_BLOCK, device=dev)
    ws = _wgrad_workspace(0)
    gflat = torch.empty(packing.N_PARAMS, device=dev)
    st = stream_of(dev)

    def run(k):
        if k == "fwd":
            call("nr_mlp_fwd", pf.data_ptr(), rays.data_ptr(), z.data_ptr(), n, spr, None, 0, 0,
                 out.data_ptr(), None, st)
        elif k == "fwdsave":
            call("nr_mlp_fwd", pf.data_ptr(), rays.data_ptr(), z.data_ptr(), n, spr, None, 0, 0,
                 out.data_ptr(), sv.data_ptr(), st)
        elif k == "fwd3":
            call("nr_mlp_fwd_x3", p3.data_ptr(), rays.data_ptr(), z.data_ptr(), n, spr, None, 0, 0,
                 out.data_ptr(), None, st)
        elif k == "fwd3save":
            call("nr_mlp_fwd_x3", p3.data_ptr(), rays.data_ptr(), z.data_ptr(), n, spr, None, 0, 0,
                 out.data_ptr(), sv.data_ptr(), st)
        elif k == "bwd":
            call("nr_mlp_bwd", pb.data_ptr(), ops.head_ptr(pf), out.data_ptr(), gout.data_ptr(),
                 sv.data_ptr(), n, gw.data_ptr(), st)
        elif k == "bwd3":
            call("nr_mlp_bwd_x3", pb3.data_ptr(), ops.head_ptr(p3), out.data_ptr(), gout.data_ptr(),
                 sv.data_ptr(), n, gw.data_ptr(), st)
        elif k == "wgrad3":
            call("nr_wgrad_x3", sv.data_ptr(), gw.data_ptr(), n, ws.data_ptr(), gflat.data_ptr(), st)
        elif k in ("fwdh3", "fwdh3save"):
            call("nr_mlp_fwd_h3", ph3.data_ptr(), rays.data_ptr(), z.data_ptr(), n, spr, None, 0,
                 0, out.data_ptr(), sv.data_ptr() if k == "fwdh3save" else None, st)
        elif k == "bwdh3":
            call("nr_mlp_bwd_h3", pbh3.data_ptr(), ops.head_ptr(ph3), out.data_ptr(),
                 gout.data_ptr(), sv.data_ptr(), n, gw.data_ptr(), st)
        elif k == "wgradh3":
            call("nr_wgrad_h3", sv.data_ptr(), gw.data_ptr(), n, ws.data_ptr(), gflat.data_ptr(), st)
        elif k in ("fwdb1", "fwdb1save"):
            call("nr_mlp_fwd_b1", pb1.data_ptr(), rays.data_ptr(), z.data_ptr(), n, spr, None, 0,
                 0, out.data_ptr(), sv.data_ptr() if k == "fwdb1save" else None, st)
        elif k == "bwdb1":
            call("nr_mlp_bwd_b1", pbb1.data_ptr(), ops.head_ptr(pb1), out.data_ptr(),
                 gout.data_ptr(), sv.data_ptr(), n, gw.data_ptr(), st)
        elif k == "wgradb1":
            call("nr_wgrad_b1", sv.data_ptr(), gw.data_ptr(), n, ws.data_ptr(), gflat.data_ptr(), st)
        elif k == "wgrad":
            call("nr_wgrad", sv.data_ptr(), gw.data_ptr(), n, ws.data_ptr(), gflat.data_ptr(), st)

    if which == "all":
        ks = ["fwd", "fwdsave", "fwd3", "fwd3save", "bwd", "bwd3", "wgrad", "wgrad3"]
    elif which == "h3":
        ks = ["fwdh3", "fwdh3save", "bwdh3", "wgradh3"]
    elif which == "b1":
        ks = ["fwdb1", "fwdb1save", "bwdb1", "wgradb1"]
    else:
        ks = which.split(",")
    if any("h3" in k for k in ks):   # f16x3: save buffer (and its statistics) by the h3 forward
        run("fwdh3save")
        run("bwdh3")
    elif any("b1" in k for k in ks):   # bf16: bf16 segments written by its own kernels
        run("fwdb1save")
        run("bwdb1")
    else:
        run("bwd")
    for k in ks:
        for _ in range(2):
            run(k)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run(k)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        tf = n * FLOP[k] / (ms * 1e-3) / 1e12
        extra = (f"  {tf / PEAKH3 * 100:5.1f}% of the f16x3 ceiling" if "h3" in k else
                 f"  {tf / PEAK3 * 100:5.1f}% of the bf16x6 ceiling" if "3" in k else "")
        print(f"{k:8s} n={n:8d} {ms:8.3f} ms  {tf:6.1f} TFLOP/s  {tf / 157.3 * 100:5.1f}% of fp32 MFMA peak"
              + extra, flush=True)


if __name__ == "__main__":
    main()
