"""Per-launch HBM traffic of the fused MLP kernels inside bench.py's own
training step (dev tool, after scripts/pmc_bench.sh): the data-gradient and
weight-gradient launches work on the samples with a nonzero output gradient
(nr_active_samples), so their bytes depend on the step's data and are taken
from the bench workload itself rather than from isolated kernels.

    python scripts/pmc_bench.py <dir with fetch/ and write/ runs> <traffic.json> [arith]

Fine-pass launches are told from coarse ones by grid size (data gradient:
ceil(n / 128) workgroups) and, for the weight gradient (same grid either way),
by the data-gradient launch that precedes it.  FETCH_SIZE / WRITE_SIZE in KiB;
FETCH_SIZE x2 (MI355X_MICROARCH.md: gfx950 reports half the bytes of wide
streaming reads).  Entries are merged into <traffic.json> as
"<arith>/<tag>" with the samples of the fine pass (786,432 at cfg2)."""
import collections
import csv
import glob
import json
import os
import sys

TAGS = [("mlp_fwd3_kernel", "mlp_fwd"), ("mlp_bwd3_kernel", "mlp_bwd_dgrad"),
        ("wgrad3_kernel", "mlp_wgrad")]
FINE_SAMPLES = 786432
FINE_WG = FINE_SAMPLES // 128


def rows(path):
    out = []
    for f in sorted(glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            out.append(r)
    return out


def per_launch(path, counter):
    """[(dispatch id, tag, grid workgroups, value)] in dispatch order"""
    acc = collections.defaultdict(float)
    meta = {}
    for r in rows(path):
        if r.get("Counter_Name") != counter:
            continue
        tag = next((t for s, t in TAGS if s in r["Kernel_Name"]), None)
        if tag is None:
            continue
        did = int(r["Dispatch_Id"])
        acc[did] += float(r["Counter_Value"])
        grid = int(r.get("Grid_Size", 0) or 0)
        wg = int(r.get("Workgroup_Size", 0) or 0) or 1
        meta[did] = (tag, grid // wg)
    return [(d, meta[d][0], meta[d][1], acc[d]) for d in sorted(acc)]


def fine_means(launches):
    """mean per fine-pass launch of every tag"""
    vals = collections.defaultdict(list)
    last_dgrad_fine = False
    for _, tag, wgs, v in launches:
        if tag == "mlp_bwd_dgrad":
            last_dgrad_fine = wgs == FINE_WG
            fine = last_dgrad_fine
        elif tag == "mlp_wgrad":
            fine = last_dgrad_fine
        else:
            fine = wgs == FINE_WG
        if fine:
            vals[tag].append(v)
    return {t: sum(v) / len(v) for t, v in vals.items()}


def main():
    d, out = sys.argv[1], sys.argv[2]
    arith = sys.argv[3] if len(sys.argv) > 3 else "f16x3"
    fetch = fine_means(per_launch(os.path.join(d, "fetch"), "FETCH_SIZE"))
    write = fine_means(per_launch(os.path.join(d, "write"), "WRITE_SIZE"))
    tj = json.load(open(out)) if os.path.exists(out) else {}
    for tag in fetch:
        fb, wb = 2 * fetch[tag] * 1024, write.get(tag, 0.0) * 1024
        tj[f"{arith}/{tag}"] = dict(
            samples=FINE_SAMPLES, fetch_bytes=fb, write_bytes=wb, hbm_bytes=fb + wb,
            arithmetic=arith,
            method="rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes over bench.py's "
                   "cfg2 step (fine-pass launches; backward on the samples with a nonzero output "
                   "gradient); FETCH_SIZE x2 (gfx950 wide-stream correction)")
        print(f"{arith}/{tag}: fetch {fb / 1e9:.3f} GB, write {wb / 1e9:.3f} GB")
    with open(out, "w") as f:
        json.dump(tj, f, indent=1)


if __name__ == "__main__":
    main()
