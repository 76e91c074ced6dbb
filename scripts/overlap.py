"""Stream overlap of one training step from a rocprofv3 kernel trace (dev tool):
python scripts/overlap.py <trace dir> [--arith h3|fp32] [--out file].

Picks the last complete step (Adam to Adam) of the chosen arithmetic's region
(h3: the f16x3 kernels mlp_fwd3 / mlp_bwd3 / wgrad4; fp32: mlp_fwd / mlp_bwd /
wgrad), prints its launches per stream with start / end relative to the step,
and the time during which kernels of two streams ran at once -- the coarse
model's backward beside the fine model's (rendering.py puts the fine pass on a
side stream)."""
import argparse
import csv
import glob

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--arith", default="h3", choices=["h3", "fp32"])
ap.add_argument("--out")
a = ap.parse_args()
f = glob.glob(f"{a.trace}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
mark = "mlp_bwd3_kernel" if a.arith == "h3" else "mlp_bwd_kernel"
ends = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
steps = [(p, q) for p, q in zip(ends[:-1], ends[1:])
         if any(mark in r["Kernel_Name"] for r in rows[p + 1:q + 1])]
p, q = steps[-1]
seg = rows[p + 1:q + 1]
t0 = int(rows[p]["End_Timestamp"])
lines = []
for r in seg:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:48]
    lines.append(f"queue {r['Queue_Id']:>3}  {s:9.1f} {e:9.1f} us  {e - s:8.1f}  {name}")
# time with launches of >= 2 queues active
ev = []
for r in seg:
    ev += [(int(r["Start_Timestamp"]), 1, r["Queue_Id"]), (int(r["End_Timestamp"]), -1, r["Queue_Id"])]
ev.sort()
act, both, last = {}, 0, None
for t, d, qid in ev:
    if last is not None and sum(1 for v in act.values() if v > 0) >= 2:
        both += t - last
    act[qid] = act.get(qid, 0) + d
    last = t
wall = (int(rows[q]["End_Timestamp"]) - t0) / 1e3
lines.append(f"step wall {wall:.1f} us, launches {len(seg)}, queues {sorted({r['Queue_Id'] for r in seg})}, "
             f"two or more queues busy for {both / 1e3:.1f} us")
print("\n".join(lines))
if a.out:
    open(a.out, "w").write("\n".join(lines) + "\n")
