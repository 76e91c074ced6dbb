"""Per-launch HBM traffic of the fused kernels from rocprofv3 --pmc pass directories (scripts/gpu.sh traffic)
(dev tool): traffic.py <pmc dir> <out json> [--x3 | --arith f16x3 [--fwd-save-only]].

--arith NAME keeps the split-operand kernels only, stores the entries under
"NAME/<tag>" and merges them into an existing <out json>.

FETCH_SIZE / WRITE_SIZE are in KiB.  Per MI355X_MICROARCH.md (HBM section),
FETCH_SIZE on gfx950 reports half the bytes of wide coalesced streaming reads
(all our global loads are 16 B/lane streams), so it is doubled; WRITE_SIZE is
exact for 16 B/lane streaming stores."""
import collections
import csv
import glob
import json
import sys

d, out = sys.argv[1], sys.argv[2]
opts = sys.argv[3:]
ARITH = opts[opts.index("--arith") + 1] if "--arith" in opts else None
X3_ONLY = "--x3" in opts or ARITH is not None
FWD_SAVE_ONLY = "--fwd-save-only" in opts
# the bf16x6 kernels (the default arithmetic) and the fp32 ones map to the
# same bench tags; profile one arithmetic per run
TAGS = [("mlp_fwd3_kernel", "mlp_fwd"), ("mlp_bwd3_kernel", "mlp_bwd_dgrad"),
        ("wgrad3_kernel", "mlp_wgrad"),
        ("mlp_fwd_kernel", "mlp_fwd"), ("mlp_bwd_kernel", "mlp_bwd_dgrad"),
        ("wgrad_reduce", "wgrad_reduce"), ("wgrad_kernel", "mlp_wgrad")]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
    order, seen = {}, collections.Counter()
    for r in csv.DictReader(open(f)):
        hit = next(((s_, t) for s_, t in TAGS if s_ in r["Kernel_Name"]), None)
        if hit is None or (X3_ONLY and "3_kernel" not in hit[0] and "reduce" not in hit[0]):
            continue
        tag = hit[1]
        did = int(r["Dispatch_Id"])
        if did not in order:
            seen[tag] += 1
            order[did] = seen[tag]
        if tag == "mlp_fwd" and not FWD_SAVE_ONLY:
            tag = "mlp_fwd_nosave" if order[did] <= 5 else "mlp_fwd"
        vals[tag][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
if ARITH is not None:
    try:
        res = json.load(open(out))
    except FileNotFoundError:
        pass
for k, cs in vals.items():
    med = {c: sorted(x)[len(x) // 2] for c, x in cs.items()}
    if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
        fetch = med["FETCH_SIZE"] * 1024 * 2
        write = med["WRITE_SIZE"] * 1024
        key = f"{ARITH}/{k}" if ARITH else k
        res[key] = {"samples": 786432, "fetch_bytes": fetch, "write_bytes": write,
                  "hbm_bytes": fetch + write,
                  "arithmetic": ARITH or ("bf16x6" if X3_ONLY else "fp32"),
                  "method": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes; "
                            "FETCH_SIZE x2 (gfx950 wide-stream correction)"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
