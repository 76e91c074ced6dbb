"""f16x3 forward clock stamps (dev only; dev/libh3_dbg8.so = mlp_fwd3.hip with
-DNR_F16=1 -DNR_X3_DBG=8, built by dev/h3var.sh dbg8 -DNR_X3_DBG=8): per wave
the in-kernel clock, total cycles and each layer's cycles, the stamps written
to the out buffer.  `--save`: the training forward (activations saved)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nerf_pl_amd import ops, packing  # noqa: E402
from nerf_pl_amd._lib import stream_of  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
flat = (torch.rand(packing.N_PARAMS, device=dev) - 0.5) * 0.15
ph = ops.pack_fwd3(flat, math="f16x3")
n_rays, spr = 4096, 192
n = n_rays * spr
rays = torch.randn(n_rays, 8, device=dev)
rays[:, 3:6] = torch.nn.functional.normalize(rays[:, 3:6], dim=-1)
rays[:, 6], rays[:, 7] = 2.0, 6.0
z = (torch.rand(n, device=dev) * 4 + 2).contiguous()
save = "--save" in sys.argv
sv = torch.empty(ops.save_floats(n), device=dev) if save else None
L = ctypes.CDLL(os.path.abspath("dev/libh3_dbg8.so"))
f = L.nr_mlp_fwd_h3
P, I, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
f.argtypes = [P, P, P, I64, I, P, I, I, P, P, P]
nb = (n + 31) // 32
stp = torch.zeros(max(nb * 16, 2 * n), dtype=torch.int64, device=dev)   # the out buffer: (n, 4) fp32
svp = sv.data_ptr() if save else None
st = stream_of(dev)
for _ in range(30):
    f(ph.data_ptr(), rays.data_ptr(), z.data_ptr(), n, spr, None, 0, 0, stp.data_ptr(), svp, st)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    f(ph.data_ptr(), rays.data_ptr(), z.data_ptr(), n, spr, None, 0, 0, stp.data_ptr(), svp, st)
e1.record()
torch.cuda.synchronize()
w = stp[:nb * 16].view(nb, 16).cpu().double()
dt_real = (w[:, 1] - w[:, 0]).clamp(min=1)
clock = w[:, 2] / dt_real * 100
names = ["inputs+PE", "first group", "L1 (2 ks)", "L2", "L3", "L4", "L5 PE (2 ks)", "L5 h4", "L6", "L7",
         "L8", "final", "dir (9 groups)"]
groups = [0, 0, 4, 16, 16, 16, 4, 16, 16, 16, 16, 16, 9]
st_ = w[:, 3:16]
prev = torch.zeros(nb, dtype=torch.float64)
print(f"fwd ({'save' if save else 'no save'}) {e0.elapsed_time(e1) / 10:.3f} ms; clock median {clock.median().item():.0f} MHz; "
      f"wave cycles median {w[:, 2].median().item():.0f}", flush=True)
for i, (nm, gq) in enumerate(zip(names, groups)):
    d = (st_[:, i] - prev).median().item()
    prev = st_[:, i]
    ideal = gq * 768
    print(f"  {nm:16s} {d:8.0f} cycles" + (f"  ({gq} groups: {d / gq:6.0f}/group, MFMA-only 768)" if gq else ""),
          flush=True)
print(f"  {'heads + end':16s} {(w[:, 2] - st_[:, 12]).median().item():8.0f} cycles", flush=True)
