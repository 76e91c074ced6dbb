"""Time the NR_W3_DBG variants of wgrad3 (dev only)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from nerf_pl_amd import ops, packing
from nerf_pl_amd._lib import stream_of
from nerf_pl_amd.functions import _wgrad_workspace
dev = torch.device("cuda", 0)
n = 786432
sv = torch.randn(ops.n_blocks(n) * ops.SAVE_PER_BLOCK, device=dev)
gw = torch.randn(ops.n_blocks(n) * ops.GRAD_PER_BLOCK, device=dev)
ws = _wgrad_workspace(0)
gflat = torch.empty(packing.N_PARAMS, device=dev)
st = stream_of(dev)
for v in range(4):
    L = ctypes.CDLL(os.path.abspath(f"dev/libw3dbg{v}.so"))
    f = L.nr_wgrad_x3
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    run = lambda: f(sv.data_ptr(), gw.data_ptr(), n, ws.data_ptr(), gflat.data_ptr(), st)
    run(); run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        run()
    e1.record()
    torch.cuda.synchronize()
    print(f"w3dbg{v} {e0.elapsed_time(e1) / 10:.3f} ms", flush=True)
