"""bench.py under torch's synchronization debug mode (dev tool): every
synchronizing HIP call warns with its call site.
    python -W always scripts/sync_debug.py <bench.py arguments>
(also under torch.distributed.run)."""
import os
import runpy
import sys

import torch

torch.cuda.set_sync_debug_mode("warn")
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.argv = [os.path.join(root, "bench.py")] + sys.argv[1:]
sys.path.insert(0, root)
runpy.run_path(sys.argv[0], run_name="__main__")
