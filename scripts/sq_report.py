"""Per-kernel limiter report from scripts/gpu.sh sq (round 4: prof_r04.sh) counter passes over
bench.py's own training step (dev tool).

    python scripts/sq_report.py gpurun_out/r04/<tag> [out.json]

Reads the rocprofv3 --pmc passes sq_a/ sq_b/ fetch/ write/ (each its own run of
the same bench command: the main region in the default arithmetic, then the
exact-fp32 leg) and, for the fused MLP kernels of each arithmetic, averages
every counter over the FINE-pass launches (the forward's and data gradient's
largest grids; a weight-gradient launch takes the class of the data-gradient
launch before it).  Derived per kernel:
  clock_ghz       GRBM_GUI_ACTIVE / 8 XCDs / kernel time (profiled run)
  mfma_busy       SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
  valu_per_mfma   SQ_INSTS_VALU / SQ_INSTS_MFMA
  wait_any, wait_inst, active_inst   SQ_WAIT_ANY / SQ_WAIT_INST_ANY /
                  SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES (the three partition it)
  lds_conflict    SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  fetch_gb, write_gb   FETCH_SIZE x 2 (gfx950 wide-stream correction) and WRITE_SIZE, GB
(MI355X_MICROARCH.md: PMC slots and units; SQ_WAVE_CYCLES / SQ_WAIT_* count
quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES cycles.)"""
import collections
import csv
import glob
import json
import os
import sys

# (substring of the kernel name, tag); fp32 names are prefixes of none of the split ones
KERNELS = [("mlp_fwd3_kernel", "mlp_fwd"), ("mlp_bwd3_kernel", "mlp_bwd_dgrad"),
           ("wgrad3_kernel", "mlp_wgrad"), ("wgrad4_kernel", "mlp_wgrad"), ("mlp_fwd_kernel", "fp32/mlp_fwd"),
           ("mlp_bwd_kernel", "fp32/mlp_bwd_dgrad"), ("wgrad_kernel", "fp32/mlp_wgrad")]


def tag_of(name):
    return next((t for s, t in KERNELS if s in name), None)


def launches(pass_dir):
    """{dispatch id: (tag, grid workgroups, {counter: value}, duration ns)} of one pass"""
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for f in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            tag = tag_of(r["Kernel_Name"])
            if tag is None:
                continue
            did = int(r["Dispatch_Id"])
            vals[did][r["Counter_Name"]] += float(r["Counter_Value"])
            grid = int(r.get("Grid_Size", 0) or 0)
            wg = int(r.get("Workgroup_Size", 0) or 0) or 1
            dur = int(r.get("End_Timestamp", 0) or 0) - int(r.get("Start_Timestamp", 0) or 0)
            meta[did] = (tag, grid // wg, dur)
    return {d: (meta[d][0], meta[d][1], dict(vals[d]), meta[d][2]) for d in sorted(vals)}


def fine_only(ls):
    """fine-pass launches: per tag the largest grid (forward / data gradient);
    a weight gradient follows its data gradient's class"""
    big = collections.defaultdict(int)
    for tag, grid, _, _ in ls.values():
        if "wgrad" not in tag:
            big[tag] = max(big[tag], grid)
    out = collections.defaultdict(list)
    last_fine = {}
    for d in sorted(ls):
        tag, grid, cv, dur = ls[d]
        arith = tag.split("/")[0] if "/" in tag else ""
        if "wgrad" in tag:
            fine = last_fine.get(arith, False)
        else:
            fine = grid == big[tag]
            if "dgrad" in tag:
                last_fine[arith] = fine
        if fine:
            out[tag].append((cv, dur))
    return out


def main():
    d = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in ("sq_a", "sq_b", "fetch", "write"):
        pd = os.path.join(d, p)
        if not os.path.isdir(pd):
            continue
        for tag, lst in fine_only(launches(pd)).items():
            for cv, dur in lst:
                for k, v in cv.items():
                    acc[tag][k].append(v)
                acc[tag][f"dur_ns_{p}"].append(dur)
    report = {}
    for tag in sorted(acc):
        m = {k: sum(v) / len(v) for k, v in acc[tag].items()}
        r = {"launches": len(acc[tag].get("dur_ns_sq_a", acc[tag].get("dur_ns_fetch", [])))}
        dur = m.get("dur_ns_sq_a") or m.get("dur_ns_sq_b")
        if dur:
            r["profiled_ms"] = round(dur * 1e-6, 4)
        g = m.get("GRBM_GUI_ACTIVE")
        if g and dur:
            r["clock_ghz"] = round(g / 8 / dur, 3)
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            r["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * g / 8), 3)
        if m.get("SQ_INSTS_MFMA"):
            r["valu_per_mfma"] = round(m.get("SQ_INSTS_VALU", 0) / m["SQ_INSTS_MFMA"], 2)
            r["lds_per_mfma"] = round(m.get("SQ_INSTS_LDS", 0) / m["SQ_INSTS_MFMA"], 3) \
                if "SQ_INSTS_LDS" in m else None
            r["vmem_wr_per_mfma"] = round(m.get("SQ_INSTS_VMEM_WR", 0) / m["SQ_INSTS_MFMA"], 3) \
                if "SQ_INSTS_VMEM_WR" in m else None
            r["vmem_rd_per_mfma"] = round(m.get("SQ_INSTS_VMEM_RD", 0) / m["SQ_INSTS_MFMA"], 3) \
                if "SQ_INSTS_VMEM_RD" in m else None
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for k, c in (("wait_any", "SQ_WAIT_ANY"), ("wait_inst", "SQ_WAIT_INST_ANY"),
                         ("active_inst", "SQ_ACTIVE_INST_ANY"), ("wait_inst_lds", "SQ_WAIT_INST_LDS")):
                if c in m:
                    r[k] = round(m[c] / wc, 3)
        if m.get("SQ_LDS_IDX_ACTIVE"):
            r["lds_conflict"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"], 3)
        if "FETCH_SIZE" in m:
            r["fetch_gb"] = round(2 * m["FETCH_SIZE"] * 1024 / 1e9, 3)
        if "WRITE_SIZE" in m:
            r["write_gb"] = round(m["WRITE_SIZE"] * 1024 / 1e9, 3)
        r["counters"] = {k: round(v, 1) for k, v in sorted(m.items()) if not k.startswith("dur_")}
        report[tag] = r
        print(tag, json.dumps({k: v for k, v in r.items() if k != "counters"}))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fh:
            json.dump(report, fh, indent=1)


if __name__ == "__main__":
    main()
