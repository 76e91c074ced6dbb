"""dev: what a listed launch costs beyond its listed samples.

The listed re-run (nr_mlp_fwd_listed*), the listed data gradient and the
weight gradient size their grids for every sample and let the workgroups past
the device-side count exit at once.  This runs the training forward + backward
of one cfg2-size fine pass (4096 rays x 192 samples, f16x3, deferred save)
with a given fraction of samples carrying an output gradient -- 0 makes every
listed launch all-empty, so its kernel time IS the empty-workgroup overhead a
persistent grid could remove.  Run under rocprofv3 --kernel-trace --stats.

    python dev/empty_list_probe.py --frac 0 [--reps 10]
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frac", type=float, default=0.0)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    from oracle import nerf_oracle as O
    from nerf_pl_amd import NeRF, functions, ops
    from nerf_pl_amd.functions import mlp_apply
    ops.MATH = "f16x3"
    functions.DEFER_SAVE = "all"
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    n_rays, spr = 4096, 192
    rays = torch.cat([torch.randn(n_rays, 3, generator=g) * 0.3,
                      torch.nn.functional.normalize(torch.randn(n_rays, 3, generator=g), dim=-1),
                      torch.full((n_rays, 1), 2.0), torch.full((n_rays, 1), 6.0)], 1).to(dev)
    z = (2 + 4 * torch.rand(n_rays, spr, generator=g)).to(dev)
    gout = torch.randn(n_rays * spr, 4, generator=g)
    gout[torch.rand(n_rays * spr, generator=g) >= args.frac] = 0
    gout = gout.to(dev)
    net = NeRF()
    net.load_state_dict(O.make_params(7, sigma_bias=0.4))
    net = net.to(dev)
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(args.reps + 2):
        if r == 2:
            t0.record()
        out = mlp_apply(net, rays=rays, z=z, spr=spr)
        (out * gout).sum().backward()
        net.zero_grad(set_to_none=True)
    t1.record()
    torch.cuda.synchronize()
    listed = int((gout != 0).any(1).sum())
    print(f"frac {args.frac}: {listed} listed of {n_rays * spr}, "
          f"{t0.elapsed_time(t1) / args.reps:.3f} ms per forward + backward", flush=True)


if __name__ == "__main__":
    main()
