"""Per-launch HBM traffic of the three fused MLP kernels at cfg2's fine pass, both
arithmetics, from scripts/gpu.sh's `traffic` step (rocprofv3 --pmc FETCH_SIZE
and --pmc WRITE_SIZE in separate runs of bench.py's short cfg2 run, which holds
the f16x3 main region and the exact-fp32 leg) (dev tool):

    python scripts/traffic.py <gpu.sh out dir> <out json>

(Rounds 1-4 wrote their traffic.json with an earlier form of this script.)

Fine-pass launches = the largest grid of each kernel, and of those the ones
taking >= 0.7 of the longest; median over them.
FETCH_SIZE / WRITE_SIZE are in KiB; FETCH_SIZE reports half the bytes of wide
coalesced streaming reads on gfx950 (MI355X_MICROARCH.md, HBM section), so it
is doubled.  The backward kernels run over the samples with a nonzero output
gradient: bench.py divides by its own listed count."""
import collections
import csv
import json
import sys

d, out = sys.argv[1], sys.argv[2]
# (kernel-name prefix, save/grad template filter, arithmetic, bench tag)
KERNELS = [("mlp_fwd3_kernel<0, false, true", "f16x3", "mlp_fwd"),
           ("mlp_bwd3_kernel<", "f16x3", "mlp_bwd_dgrad"),
           ("wgrad4_kernel<", "f16x3", "mlp_wgrad"),
           ("wgrad3_kernel<", "f16x3", "mlp_wgrad"),
           ("mlp_fwd_kernel<0, false, false>", "fp32", "mlp_fwd"),
           ("mlp_bwd_kernel<", "fp32", "mlp_bwd_dgrad"),
           ("wgrad_kernel<", "fp32", "mlp_wgrad")]


def load(counter):
    per = collections.defaultdict(list)     # key -> [(grid, value)]
    for r in csv.DictReader(open(f"{d}/{counter.split('_')[0].lower()}/run_counter_collection.csv")):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        for pre, ar, tag in KERNELS:
            if "::" + pre in name:
                per[f"{ar}/{tag}"].append((int(r["Grid_Size"]),
                                           int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                           float(r["Counter_Value"])))
                break
    res = {}
    for k, v in per.items():
        # the fine pass: the largest grid, and of those the long launches (the
        # weight gradient's grid does not depend on the sample count)
        g = max(x[0] for x in v)
        v = [x for x in v if x[0] == g]
        tmax = max(x[1] for x in v)
        vals = sorted(x[2] for x in v if x[1] >= 0.7 * tmax)
        res[k] = (vals[len(vals) // 2], len(vals))
    return res


fetch, write = load("FETCH_SIZE"), load("WRITE_SIZE")
res = {}
for k in sorted(fetch):
    if k not in write:
        continue
    fb, wb = fetch[k][0] * 1024 * 2, write[k][0] * 1024
    res[k] = {"samples": 786432, "fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb,
              "launches": fetch[k][1], "arithmetic": k.split("/")[0],
              "file": out,
              "method": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes over bench.py's "
                        "short cfg2 run (fine-pass launches: the largest grid; backward on the samples "
                        "with a nonzero output gradient); FETCH_SIZE x2 (gfx950 wide-stream correction)"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
