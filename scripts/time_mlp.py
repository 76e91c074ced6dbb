"""Quick timing of the fused MLP forward at bench sizes (dev tool)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from nerf_pl_amd import ops, packing

dev = torch.device("cuda", 0)
flat = (torch.rand(packing.N_PARAMS, device=dev) - 0.5) * 0.1
packed = ops.pack_fwd(flat)
n_rays = 4096
for spr in (64, 192):
    rays = torch.randn(n_rays, 8, device=dev)
    rays[:, 6] = 2.0; rays[:, 7] = 6.0
    z = torch.rand(n_rays * spr, device=dev) * 4 + 2
    for save in (False, True):
        for _ in range(3):
            ops.mlp_forward(packed, rays=rays, z=z, samples_per_ray=spr, save=save)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        K = 10
        e0.record()
        for _ in range(K):
            ops.mlp_forward(packed, rays=rays, z=z, samples_per_ray=spr, save=save)
        e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / K
        n = n_rays * spr
        tf = n * 1186816 / (ms * 1e-3) / 1e12
        print(f"spr={spr} save={save}: {ms:.3f} ms  {tf:.1f} TFLOP/s  ({tf/157.3*100:.1f}% of fp32 peak)")
