"""One line per A/B bench run of scripts/gpu.sh abalt (dev tool):
    python scripts/ab_summary.py gpurun_out/r06/<tag> [...]
value, serial per-kernel launch ms (fwd, dgrad, wgrad), the same from the timed
region (the two backward chains overlap there), and the MLP stage's union."""
import glob
import json
import os
import sys

for d in sys.argv[1:]:
    rows = []
    for f in sorted(glob.glob(os.path.join(d, "ab_*.log"))):
        line = next((l for l in open(f) if l.startswith("{")), None)
        if line is None:
            continue
        j = json.loads(line)
        r, c, m = j["rooflines"], j["rooflines_concurrent"], j["mlp_stage"]
        k = ("mlp_fwd", "mlp_bwd_dgrad", "mlp_wgrad")
        rows.append((os.path.basename(f)[3:-4], j["value"], [r[x]["avg_launch_ms"] for x in k],
                     [c[x]["avg_launch_ms"] for x in k], m["ms_per_step"]))
    for name, v, s, cc, u in sorted(rows):
        print(f"{name:16s} {v:9.1f}  serial {s[0]:.3f} {s[1]:.3f} {s[2]:.3f}  "
              f"concurrent {cc[0]:.3f} {cc[1]:.3f} {cc[2]:.3f}  union {u:.3f}")
