"""Time the NR_X3_DBG variants of the bf16x6 forward/backward (dev only)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from nerf_pl_amd import ops, packing
from nerf_pl_amd._lib import stream_of
dev = torch.device("cuda", 0)
torch.manual_seed(0)
flat = (torch.rand(packing.N_PARAMS, device=dev) - 0.5) * 0.15
p3, pb3 = ops.pack_fwd3(flat), ops.pack_bwd(flat, math="bf16x6")
n_rays, spr = 4096, 192
n = n_rays * spr
rays = torch.randn(n_rays, 8, device=dev)
rays[:, 3:6] = torch.nn.functional.normalize(rays[:, 3:6], dim=-1)
rays[:, 6], rays[:, 7] = 2.0, 6.0
z = (torch.rand(n, device=dev) * 4 + 2).contiguous()
out, sv = ops.mlp_forward(p3, rays=rays, z=z, samples_per_ray=spr, save=True)
gout = torch.randn(n, 4, device=dev)
gw = torch.empty(ops.n_blocks(n) * ops.GRAD_PER_BLOCK, device=dev)
st = stream_of(dev)
VARIANTS = sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "1", "2", "3", "4", "5", "s0", "s2", "8"]
for v in VARIANTS:
    L = ctypes.CDLL(os.path.abspath(f"dev/libx3dbg{v}.so"))
    f = L.nr_mlp_fwd_x3
    f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    b = L.nr_mlp_bwd_x3
    b.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
    runs = {
        "fwd3": lambda: f(p3.data_ptr(), rays.data_ptr(), z.data_ptr(), n, spr, None, 0, 0, out.data_ptr(), None, st),
        "fwd3save": lambda: f(p3.data_ptr(), rays.data_ptr(), z.data_ptr(), n, spr, None, 0, 0, out.data_ptr(), sv.data_ptr(), st),
        "bwd3": lambda: b(pb3.data_ptr(), ops.head_ptr(p3), out.data_ptr(), gout.data_ptr(), sv.data_ptr(), n, gw.data_ptr(), st),
    }
    if v == "8":   # clock stamps: full forward, no save; stamps written through the save pointer
        nb = (n + 31) // 32
        stp = torch.zeros(nb * 4, dtype=torch.int64, device=dev)
        for _ in range(20):
            f(p3.data_ptr(), rays.data_ptr(), z.data_ptr(), n, spr, None, 0, 0, out.data_ptr(), stp.data_ptr(), st)
        torch.cuda.synchronize()
        w = stp.view(nb, 4).cpu().double()
        dt_real = w[:, 1] - w[:, 0]
        clock = w[:, 2] / dt_real.clamp(min=1) * 100
        span = (w[:, 1].max() - w[:, 0].min()).item() / 100
        busy = dt_real.sum().item() / 100 / 1024
        print(f"dbg8 clock median {clock.median().item():.0f} MHz (p10 {clock.quantile(0.1).item():.0f}); "
              f"wave median {dt_real.median().item() / 100:.1f} us (p90 {dt_real.quantile(0.9).item() / 100:.1f}); "
              f"span {span:.1f} us, sum(wave)/1024 SIMDs {busy:.1f} us", flush=True)
        torch.save(w, "gpurun_out/stamps.pt")
        continue
    for k, fn in runs.items():
        fn(); fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"dbg{v} {k:9s} {e0.elapsed_time(e1) / 10:.3f} ms", flush=True)
