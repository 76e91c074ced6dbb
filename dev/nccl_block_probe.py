"""Does issuing an RCCL collective (c10d, async_op=True) block the host until
the GPU has produced its input?  (the backward chains stop
overlapping on the distributed path.)  One rank; a ~100 ms matmul chain on a
side stream produces the tensor, then all_reduce / work.wait() are timed on
the host (dev tool):

    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 dev/nccl_block_probe.py
"""
import os
import time

import torch
import torch.distributed as dist


def main():
    dist.init_process_group("nccl")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    a = torch.randn(4096, 4096, device=dev)
    x = torch.zeros(1 << 20, device=dev)
    dist.all_reduce(x)                      # communicator set up
    torch.cuda.synchronize()
    s = torch.cuda.Stream(device=dev)
    for trial in range(3):
        with torch.cuda.stream(s):
            b = a
            for _ in range(40):
                b = b @ a * 1e-3
            x.copy_(b.reshape(-1)[: x.numel()])
            t0 = time.perf_counter()
            h = dist.all_reduce(x, async_op=True)
            t1 = time.perf_counter()
        t2 = time.perf_counter()
        h.wait()
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        print(f"trial {trial}: all_reduce issue {1e3 * (t1 - t0):.2f} ms, wait() {1e3 * (t3 - t2):.2f} ms, "
              f"rest of the GPU work {1e3 * (t4 - t3):.2f} ms", flush=True)
    print("env", {k: v for k, v in os.environ.items() if "NCCL" in k}, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
