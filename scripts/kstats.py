"""Summarise a rocprofv3 --kernel-trace --stats run (dev tool):
kstats.py <prof dir> <header line> > profiles/.../kernel_stats_vN.txt"""
import collections
import csv
import sys

d, header = sys.argv[1], sys.argv[2]
print(header)
print()
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
for r in rows[:14]:
    print(f"{r['Name'][:80]:80s} calls={int(r['Calls']):5d} avg_ms={float(r['AverageNs']) / 1e6:8.3f} "
          f"total%={float(r['Percentage']):6.2f}")
print()
print("per-launch durations by grid size (ms): kernel, grid threads, launches, mean")
by = collections.defaultdict(list)
for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")):
    name = r["Kernel_Name"]
    key = next((k for k in ("mlp_fwd3_kernel", "mlp_bwd3_kernel", "wgrad3_kernel", "mlp_fwd_kernel",
                            "mlp_bwd_kernel", "wgrad_kernel", "wgrad_reduce") if k in name), None)
    if key is None:
        continue
    by[(key, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
for (k, g), v in sorted(by.items()):
    print(f"{k:18s} grid={g:9d} n={len(v):3d} mean={sum(v) / len(v):8.3f}")
