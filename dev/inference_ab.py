"""dev: the f16x3 inference forward alone (cfg2 fine size, full and sigma-only), for
same-box library A/B runs (NERF_PL_AMD_LIB=...; profiles/r05/inference_ab/)."""
import os, sys
sys.path.insert(0, os.getcwd())
import torch
from nerf_pl_amd import ops, packing
from nerf_pl_amd._lib import call, stream_of
dev = torch.device("cuda", 0)
torch.manual_seed(0)
flat = (torch.rand(packing.N_PARAMS, device=dev) - 0.5) * 0.15
ph3 = ops.pack_fwd3(flat, math="f16x3")
n_rays, spr = 4096, 192
n = n_rays * spr
rays = torch.randn(n_rays, 8, device=dev)
rays[:, 3:6] = torch.nn.functional.normalize(rays[:, 3:6], dim=-1)
rays[:, 6], rays[:, 7] = 2.0, 6.0
z = (torch.rand(n, device=dev) * 4 + 2).contiguous()
out = torch.empty(n, 4, device=dev)
st = stream_of(dev)
for so in (0, 1):
    for _ in range(5):
        call("nr_mlp_fwd_h3", ph3.data_ptr(), rays.data_ptr(), z.data_ptr(), n, spr, None, 0, so, out.data_ptr(), None, st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        call("nr_mlp_fwd_h3", ph3.data_ptr(), rays.data_ptr(), z.data_ptr(), n, spr, None, 0, so, out.data_ptr(), None, st)
    e1.record(); torch.cuda.synchronize()
    print(f"{'sigma' if so else 'full'} inference fwd: {e0.elapsed_time(e1) / 20:.3f} ms")
