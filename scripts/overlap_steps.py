"""Launches of one pipelined training step (gen_rays to gen_rays) per HIP
queue from a rocprofv3 kernel trace, and the time two or more queues ran
kernels at once (dev tool):
    python scripts/overlap_steps.py <trace dir> [--out file]
With nerf_pl_amd.pipeline.PipelinedStep the next step's coarse pass (its
queue's gen_rays .. sample_pdf) runs beside the previous step's fine weight
gradient, so a step window starts while the previous fine chain is still
running: those launches are listed too (negative start)."""
import argparse
import csv
import glob

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--out")
a = ap.parse_args()
f = glob.glob(f"{a.trace}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "mlp_fwd_kernel" not in r["Kernel_Name"]]   # (no fp32-leg launches)
starts = [i for i, r in enumerate(rows) if "gen_rays_kernel" in r["Kernel_Name"]]
i0, i1 = starts[-3], starts[-2]
t0, t1 = int(rows[i0]["Start_Timestamp"]), int(rows[i1]["Start_Timestamp"])
seg = [r for r in rows if int(r["End_Timestamp"]) > t0 and int(r["Start_Timestamp"]) < t1]
lines, iv = [], []
for r in seg:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "")[:60]
    lines.append(f"queue {q:>3} {s:9.1f} {e:9.1f} us {e - s:8.1f}  {name}")
    iv.append((max(s, 0.0), min(e, (t1 - t0) / 1e3), q))
# time with kernels of >= 2 queues running
ev = sorted([(s, 1, q) for s, e, q in iv] + [(e, -1, q) for s, e, q in iv])
active, last, both = {}, 0.0, 0.0
for t, d, q in ev:
    if sum(1 for v in active.values() if v > 0) >= 2:
        both += t - last
    active[q] = active.get(q, 0) + d
    last = t
lines.append(f"step window {(t1 - t0) / 1e3:.1f} us (gen_rays to gen_rays), launches {len(seg)}, "
             f"two or more queues busy for {both:.1f} us")
out = "\n".join(lines)
print(out)
if a.out:
    open(a.out, "w").write(out + "\n")
