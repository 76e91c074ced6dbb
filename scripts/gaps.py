"""Idle-GPU gaps per training step from a rocprofv3 kernel trace (dev tool):
python scripts/gaps.py <trace dir>.  A step ends at its Adam launch; per step:
wall time between Adam ends, summed kernel time, and the largest gaps with the
kernels either side (a gap = the host was behind the GPU)."""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
if len(ends) < 2:       # inference workloads: no optimizer; a step starts at its ray generation
    ends = [i - 1 for i, r in enumerate(rows) if "gen_rays_kernel" in r["Kernel_Name"] and i > 0]
for a, b in list(zip(ends[:-1], ends[1:]))[-3:]:
    seg = rows[a + 1:b + 1]
    wall = (int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e6
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e6
    prev, gaps = int(rows[a]["End_Timestamp"]), []
    for k, r in enumerate(seg):
        gaps.append(((int(r["Start_Timestamp"]) - prev) / 1e3,
                     seg[k - 1]["Kernel_Name"][:36] if k else "-", r["Kernel_Name"][:36]))
        prev = int(r["End_Timestamp"])
    print(f"wall {wall:.3f} ms  kernels {busy:.3f} ms  idle {wall - busy:.3f} ms  launches {len(seg)}")
    for g in sorted(gaps, reverse=True)[:4]:
        print(f"    {g[0]:8.1f} us  {g[1]} -> {g[2]}")
