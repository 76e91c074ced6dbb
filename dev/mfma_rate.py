import ctypes, os, torch
L = ctypes.CDLL(os.path.abspath("dev/libmfmarate.so"))
L.launch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
out = torch.empty(256 * 256 * 8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
for variant in (0, 1):
    iters = 2000
    L.launch(out.data_ptr(), 1024, iters, variant, st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); L.launch(out.data_ptr(), 1024, iters, variant, st); e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    flops = 1024 * 4 * iters * 48 * 32 * 32 * 16 * 2   # blocks x waves x MFMAs x MNK x 2
    print(f"variant {variant}: {ms:.3f} ms  {flops / ms / 1e9:.1f} TFLOP/s bf16  ({flops / ms / 1e9 / 2516.6 * 100:.1f}% of dense bf16 peak)")

L.launch16.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
iters = 2000
L.launch16(out.data_ptr(), 1024, iters, st)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); L.launch16(out.data_ptr(), 1024, iters, st); e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1)
flops = 1024 * 4 * iters * 96 * 16 * 16 * 32 * 2
print(f"16x16x32: {ms:.3f} ms  {flops / ms / 1e9:.1f} TFLOP/s bf16  ({flops / ms / 1e9 / 2516.6 * 100:.1f}% of dense bf16 peak)")
