"""PSNR of this package vs the reference over draw seeds (BASELINE.json target:
"PSNR within 0.1 dB of the reference").

Reads the per-run JSON files of scripts/psnr_compare.py: this package's f16x3
runs (profiles/r02/psnr/ours_s*.json, unperturbed) and the reference's runs
(profiles/r01/psnr_reference_s*.json, profiles/r02/psnr/reference_s*.json,
unperturbed).  For every checkpoint it prints both means, standard
deviations, the difference of the means with its standard error, and the
same-seed differences; writes profiles/r02/psnr/summary.json.

    python scripts/psnr_summary.py
"""
import glob
import json
import math
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(pattern):
    runs = {}
    for f in sorted(glob.glob(os.path.join(REPO, pattern))):
        d = json.load(open(f))
        if d.get("perturb_ulp") or "eval_weights" in d:
            continue
        seed = int(re.search(r"_s(\d+)", os.path.basename(f)).group(1))
        runs[seed] = {p["step"]: p["psnr"] for p in d["psnr"]}
    return runs


def stats(xs):
    n = len(xs)
    m = sum(xs) / n
    sd = math.sqrt(sum((x - m) ** 2 for x in xs) / (n - 1)) if n > 1 else float("nan")
    return n, m, sd


def main():
    ours = load("profiles/r02/psnr/ours_s*.json")
    ref = load("profiles/r01/psnr_reference_s*.json")
    ref.update(load("profiles/r02/psnr/reference_s*.json"))
    out = {"ours_seeds": sorted(ours), "reference_seeds": sorted(ref), "checkpoints": []}
    for step in (500, 1000, 1500, 2000):
        o = [r[step] for r in ours.values() if step in r]
        f = [r[step] for r in ref.values() if step in r]
        if len(o) < 2 or not f:
            continue
        no, mo, so = stats(o)
        nf, mf, sf = stats(f)
        # standard error of the difference of the means (the reference's own
        # spread estimated from ours when it has a single run)
        sf_ = sf if nf > 1 else so
        se = math.sqrt(so ** 2 / no + sf_ ** 2 / nf)
        same = {s: round(ours[s][step] - ref[s][step], 3) for s in ref
                if s in ours and step in ours[s] and step in ref[s]}
        row = {"step": step, "ours_n": no, "ours_mean": round(mo, 3), "ours_std": round(so, 3),
               "ref_n": nf, "ref_mean": round(mf, 3), "ref_std": round(sf, 3) if nf > 1 else None,
               "mean_diff": round(mo - mf, 3), "mean_diff_se": round(se, 3),
               "same_seed_diff": same}
        out["checkpoints"].append(row)
        print(json.dumps(row))
    path = os.path.join(REPO, "profiles", "r02", "psnr", "summary.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
