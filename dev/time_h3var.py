"""Time f16x3 kernel variants built by dev/h3var.sh at the cfg2 fine-pass size
(dev only): python dev/time_h3var.py base,nt,... [reps]
NR_VAR_MATH=bf16 times plain-bf16 variants (built with -DNR_F16=0 -DNR_BF1=1)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nerf_pl_amd import ops, packing  # noqa: E402
from nerf_pl_amd._lib import stream_of  # noqa: E402
from nerf_pl_amd.functions import _wgrad_workspace  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
flat = (torch.rand(packing.N_PARAMS, device=dev) - 0.5) * 0.15
MATH = os.environ.get("NR_VAR_MATH", "f16x3")
SFX, NP = {"f16x3": ("_h3", 2), "bf16": ("_b1", 1)}[MATH]
ph, pbh = ops.pack_fwd3(flat, math=MATH), ops.pack_bwd(flat, math=MATH)
n_rays, spr = int(os.environ.get("NR_VAR_RAYS", "4096")), 192
n = n_rays * spr
rays = torch.randn(n_rays, 8, device=dev)
rays[:, 3:6] = torch.nn.functional.normalize(rays[:, 3:6], dim=-1)
rays[:, 6], rays[:, 7] = 2.0, 6.0
z = (torch.rand(n, device=dev) * 4 + 2).contiguous()
out, sv = ops.mlp_forward(ph, rays=rays, z=z, samples_per_ray=spr, save=True)
gout = torch.randn(n, 4, device=dev) * 1e-4
gw = torch.empty(ops.n_blocks(n) * ops.GRAD_PER_BLOCK, device=dev)
ws = _wgrad_workspace(0)
gflat = torch.empty(packing.N_PARAMS, device=dev)
st = stream_of(dev)
P, I, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ref = None
for v in sys.argv[1].split(","):
    L = ctypes.CDLL(os.path.abspath(f"dev/libh3_{v}.so"))
    f, b, w = (getattr(L, "nr_mlp_fwd" + SFX), getattr(L, "nr_mlp_bwd" + SFX),
               getattr(L, "nr_wgrad" + SFX))
    pk, pkb = getattr(L, "nr_pack" + SFX), getattr(L, "nr_pack_bwd" + SFX)
    # weights packed by the variant itself (its weight scale may differ)
    pk.argtypes = [P, P, I64, P, P, P]
    pkb.argtypes = [P, P, I64, P, P]
    m, hm = ops._maps3(0, NP)
    mb = ops._map_bwd3(0, NP)
    assert pk(flat.data_ptr(), m.data_ptr(), m.numel(), hm.data_ptr(), ph.data_ptr(), st) == 0
    assert pkb(flat.data_ptr(), mb.data_ptr(), mb.numel(), pbh.data_ptr(), st) == 0
    f.argtypes = [P, P, P, I64, I, P, I, I, P, P, P]
    b.argtypes = [P, P, P, P, P, I64, P, P]
    w.argtypes = [P, P, I64, P, P, P]
    runs = {
        "fwd": lambda: f(ph.data_ptr(), rays.data_ptr(), z.data_ptr(), n, spr, None, 0, 0,
                         out.data_ptr(), None, st),
        "fwdsave": lambda: f(ph.data_ptr(), rays.data_ptr(), z.data_ptr(), n, spr, None, 0, 0,
                             out.data_ptr(), sv.data_ptr(), st),
        "bwd": lambda: b(pbh.data_ptr(), ops.head_ptr(ph), out.data_ptr(), gout.data_ptr(),
                         sv.data_ptr(), n, gw.data_ptr(), st),
        "wgrad": lambda: w(sv.data_ptr(), gw.data_ptr(), n, ws.data_ptr(), gflat.data_ptr(), st),
    }
    line = [f"{v:10s}"]
    for k in ("fwd", "fwdsave", "bwd", "wgrad"):
        for _ in range(2):
            runs[k]()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            runs[k]()
        e1.record()
        torch.cuda.synchronize()
        line.append(f"{k} {e0.elapsed_time(e1) / reps:6.3f}")
    g = gflat.clone()
    if ref is None:
        ref = g
    dev_ = (g - ref).abs().max().item() / (ref.abs().max().item() + 1e-30)
    line.append(f"grad dev vs first {dev_:.2e}")
    print("  ".join(line), flush=True)
