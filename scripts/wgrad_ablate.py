"""Time nr_wgrad on task subsets (NR_WGRAD_TASKMASK; launch plan only, same
kernel code) in child processes on the same device (dev tool)."""
import os
import subprocess
import sys

here = os.path.dirname(os.path.abspath(__file__))
BIG = sum(1 << t for t in (1, 2, 3, 5, 6, 7, 8, 9))
SUBSETS = {"all": -1, "big8 (256x256)": BIG, "t10 (128x256)": 1 << 10,
           "t0+t4 (256x64)": (1 << 0) | (1 << 4), "heads t11-13": (1 << 11) | (1 << 12) | (1 << 13),
           "one 256x256 (t1)": 1 << 1}
for name, m in SUBSETS.items():
    env = dict(os.environ, NR_WGRAD_TASKMASK=str(m))
    out = subprocess.run([sys.executable, os.path.join(here, "kbench.py"), "wgrad", "10"],
                         env=env, capture_output=True, text=True).stdout.strip().splitlines()
    print(f"{name:20s}: {out[-1] if out else '?'}", flush=True)
