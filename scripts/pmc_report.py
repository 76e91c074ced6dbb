"""Summarise rocprofv3 --pmc pass directories per kernel (dev tool): pmc_report.py <dir>"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
FWD_SPLIT = len(sys.argv) > 2 and sys.argv[2] == "split"
TAGS = [("mlp_fwd3_kernel", "mlp_fwd3"), ("mlp_bwd3_kernel", "mlp_bwd3"),
        ("wgrad3_kernel", "wgrad3"), ("mlp_fwd_kernel", "mlp_fwd"), ("mlp_bwd_kernel", "mlp_bwd"),
        ("wgrad_kernel", "wgrad"), ("wgrad_reduce", "wgrad_reduce")]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
    seen = collections.Counter()
    rows = list(csv.DictReader(open(f)))
    order = {}
    for r in rows:
        name = r["Kernel_Name"]
        tag = next((t for s, t in TAGS if s in name), None)
        if tag is None:
            continue
        did = int(r["Dispatch_Id"])
        if did not in order:
            seen[tag] += 1
            order[did] = seen[tag]
        k = tag
        if tag in ("mlp_fwd", "mlp_fwd3") and FWD_SPLIT:   # kbench: 5 fwd then 5 fwd+save
            k = tag if order[did] <= 5 else tag + "+save"
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
for k, cs in vals.items():
    med = {c: sorted(x)[len(x) // 2] for c, x in cs.items()}
    ms = sorted(dur[k])[len(dur[k]) // 2]
    print(f"== {k}  (profiled duration ~{ms:.2f} ms)")
    for c in sorted(med):
        print(f"   {c:28s} {med[c]:.4g}")
    if "SQ_WAVE_CYCLES" in med:
        wc = med["SQ_WAVE_CYCLES"]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in med:
                print(f"   {c}/WAVE_CYCLES = {med[c] / wc:.3f}")
    if "GRBM_GUI_ACTIVE" in med:
        print(f"   effective clock ~ {med['GRBM_GUI_ACTIVE'] / 8 / (ms * 1e-3) / 1e9:.2f} GHz")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in med and "GRBM_GUI_ACTIVE" in med:
        # per-SIMD busy fraction: MFMA busy cycles over (1024 SIMDs * gpu cycles)
        print(f"   MFMA busy ~ {med['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * med['GRBM_GUI_ACTIVE'] / 8):.3f}")
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        if c in med:
            print(f"   {c} = {med[c] / 1e6:.3f} GB (x1024 B; FETCH on gfx950 reads ~1/2 of streamed bytes)")
