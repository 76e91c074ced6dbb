"""Time nr_sample_pdf variants built by dev/pdfvar.sh at cfg2 (4096 rays, 64 + 128,
z_fine merged), dev only: python dev/time_pdf.py base,noscan,nosort [reps]"""
import ctypes
import os
import sys

import torch

dev = torch.device("cuda", 0)
n, S, I = 4096, 64, 128
g = torch.Generator().manual_seed(0)
w = torch.rand(n, S, generator=g).to(dev)
rays = torch.randn(n, 8, generator=g).to(dev)
rays[:, 6], rays[:, 7] = 2.0, 6.0
zc = torch.sort(torch.rand(n, S, generator=g) * 4 + 2, -1).values.to(dev)
u = torch.rand(n, I, generator=g).to(dev)
jt = torch.rand(n, I, generator=g).to(dev)
zp = torch.empty(n, I, device=dev)
zf = torch.empty(n, S + I, device=dev)
st = torch.cuda.current_stream(dev).cuda_stream
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
P, I_, I64, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64
ref = None
for v in sys.argv[1].split(","):
    L = ctypes.CDLL(os.path.abspath(f"dev/libpdf_{v}.so"))
    f = L.nr_sample_pdf
    f.argtypes = [P, I_, P, P, P, P, U64, I64, I_, P, P, P]
    for mode in ("replay", "philox"):
        uu, jj = (u.data_ptr(), jt.data_ptr()) if mode == "replay" else (None, None)
        run = lambda: f(w.data_ptr(), S, rays.data_ptr(), zc.data_ptr(), uu, jj, 7, n, I,
                        zp.data_ptr(), zf.data_ptr(), st)
        for _ in range(3):
            assert run() == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        out = zf.clone()
        if ref is None and mode == "replay":
            ref = out
        same = torch.equal(out, ref) if mode == "replay" else "-"
        print(f"{v:10s} {mode:6s} {e0.elapsed_time(e1) / reps * 1e3:8.1f} us  same as first: {same}",
              flush=True)
