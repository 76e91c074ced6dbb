"""Time the weight-gradient launch of one arithmetic at the cfg2 fine-pass size
(dev only).  NR_WGRAD_TASKMASK (read once by the library) restricts the launch
to a subset of tasks:  NR_WGRAD_TASKMASK=0x2 python dev/time_wgrad.py bf16"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nerf_pl_amd import ops, packing  # noqa: E402
from nerf_pl_amd._lib import call, stream_of  # noqa: E402
from nerf_pl_amd.functions import _wgrad_workspace  # noqa: E402

math = sys.argv[1] if len(sys.argv) > 1 else "f16x3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = torch.device("cuda", 0)
torch.manual_seed(0)
flat = (torch.rand(packing.N_PARAMS, device=dev) - 0.5) * 0.15
pf, pb = ops.pack_fwd(flat, math=math), ops.pack_bwd(flat, math=math)
n_rays, spr = 4096, 192
n = n_rays * spr
rays = torch.randn(n_rays, 8, device=dev)
rays[:, 3:6] = torch.nn.functional.normalize(rays[:, 3:6], dim=-1)
rays[:, 6], rays[:, 7] = 2.0, 6.0
z = (torch.rand(n, device=dev) * 4 + 2).contiguous()
out, sv = ops.mlp_forward(pf, rays=rays, z=z, samples_per_ray=spr, save=True)
gout = torch.randn(n, 4, device=dev) * 1e-4
gw = torch.empty(ops.n_blocks(n) * ops.GRAD_PER_BLOCK, device=dev)
call(ops.entry("nr_mlp_bwd", pb), pb.data_ptr(), ops.head_ptr(pf), out.data_ptr(), gout.data_ptr(),
     sv.data_ptr(), n, gw.data_ptr(), stream_of(dev))
ws = _wgrad_workspace(0)
gflat = torch.empty(packing.N_PARAMS, device=dev)
name = ops.entry("nr_wgrad", pb)


def run():
    call(name, sv.data_ptr(), gw.data_ptr(), n, ws.data_ptr(), gflat.data_ptr(), stream_of(dev))


for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    run()
e1.record()
torch.cuda.synchronize()
print(f"{math} mask {os.environ.get('NR_WGRAD_TASKMASK', 'all')}: {e0.elapsed_time(e1) / reps:.3f} ms",
      flush=True)
