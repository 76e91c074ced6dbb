"""PSNR against the reference over draw seeds (BASELINE.json target: "PSNR
within 0.1 dB of the reference"; runs from scripts/psnr.sh).

Groups of scripts/psnr_compare.py runs (2000 steps, PSNR at 500/1000/1500/2000,
fine rgb on 2 held-out views; unperturbed runs only):
  f16x3      this package, default arithmetic   profiles/r0[345]/psnr/f16x3_s*.json
  fp32       this package, exact fp32 MFMA      profiles/r0[345]/psnr/fp32_s*.json
  bf16       this package, the reduced-precision bf16 variant   profiles/r0[345]/psnr/bf16_s*.json
  ref_gpu    the reference's algorithm in PyTorch fp32 on the MI355X (the oracle,
             pinned bit-exact to the reference; hipBLAS GEMMs)   profiles/r0[345]/psnr/oracle_s*.json
  ref_cpu    the reference itself, CPU, here    profiles/r01/psnr_reference_s*.json,
             profiles/r02/psnr/reference_s*.json, profiles/r0[345]/psnr/reference_s*.json
Per checkpoint: each group's n / mean / std, and for every pair the difference
of the means, its standard error (Welch), the 95% interval and whether that
interval lies inside +-0.1 dB.  Paired too ("paired"): runs of the same draw
seed start from the same parameters and see the same ray batches and the same
render draws, so their PSNRs are correlated (r ~ 0.5-0.7) and the per-seed
difference has a smaller spread than two independent samples; mean and
Student-t interval of the per-seed differences over the seeds both groups ran.
Writes profiles/r05/psnr/summary.json (round 3's runs under profiles/r03/psnr,
round 4's under profiles/r04/psnr and round 5's under profiles/r05/psnr, one group per seed;
since round 6 each directory's run JSONs are packed into its runs.jsonl, read
through the same file patterns).

    python scripts/psnr_summary.py
"""
import fnmatch
import glob
import json
import math
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEPS = (500, 1000, 1500, 2000)


def _files(pat):
    """(basename, run) for every run matching pat: the JSON files themselves,
    or the entries of their directory's runs.jsonl (round 6 packed each psnr
    directory's runs into one file: {"file": basename, "run": the JSON})"""
    for f in sorted(glob.glob(os.path.join(REPO, pat))):
        yield os.path.basename(f), json.load(open(f))
    d, base = os.path.split(pat)
    for j in sorted(glob.glob(os.path.join(REPO, d, "runs.jsonl"))):
        for line in open(j):
            e = json.loads(line)
            if fnmatch.fnmatch(e["file"], base):
                yield e["file"], e["run"]


def load(*patterns):
    runs = {}
    for pat in patterns:
        for f, d in _files(pat):
            if d.get("perturb_ulp") or "eval_weights" in d or "psnr" not in d:
                continue
            seed = int(re.search(r"_s(\d+)", os.path.basename(f)).group(1))
            runs[seed] = {p["step"]: p["psnr"] for p in d["psnr"]}
    return runs


def stats(xs):
    n = len(xs)
    m = sum(xs) / n
    sd = math.sqrt(sum((x - m) ** 2 for x in xs) / (n - 1)) if n > 1 else float("nan")
    return n, m, sd


def t975(df):
    """two-sided 95% Student-t quantile (table + asymptote)."""
    table = {1: 12.71, 2: 4.30, 3: 3.18, 4: 2.78, 5: 2.57, 6: 2.45, 7: 2.36, 8: 2.31, 9: 2.26,
             10: 2.23, 12: 2.18, 15: 2.13, 20: 2.09, 25: 2.06, 30: 2.04, 40: 2.02, 60: 2.00}
    df = max(1, int(df))
    for k in sorted(table):
        if df <= k:
            return table[k]
    return 1.96


def main():
    groups = {
        "f16x3": load("profiles/r0[345]/psnr/f16x3_s*.json"),
        "fp32": load("profiles/r0[345]/psnr/fp32_s*.json"),
        "bf16": load("profiles/r0[345]/psnr/bf16_s*.json"),
        "ref_gpu": load("profiles/r0[345]/psnr/oracle_s*.json"),
        "ref_cpu": load("profiles/r01/psnr_reference_s*.json", "profiles/r02/psnr/reference_s*.json",
                        "profiles/r0[345]/psnr/reference_s*.json"),
    }
    groups["ref_all"] = {("g", s): v for s, v in groups["ref_gpu"].items()}
    groups["ref_all"].update({("c", s): v for s, v in groups["ref_cpu"].items()})
    pairs = [("f16x3", "ref_all"), ("fp32", "ref_all"), ("f16x3", "ref_gpu"), ("f16x3", "ref_cpu"),
             ("fp32", "ref_gpu"), ("f16x3", "fp32"), ("ref_gpu", "ref_cpu"), ("bf16", "ref_all"),
             ("bf16", "f16x3")]
    paired = [("f16x3", "ref_gpu"), ("fp32", "ref_gpu"), ("bf16", "ref_gpu"), ("f16x3", "fp32"),
              ("f16x3", "ref_cpu"), ("ref_gpu", "ref_cpu")]
    out = {"groups": {k: sorted(map(str, v)) for k, v in groups.items()}, "checkpoints": []}
    for step in STEPS:
        row = {"step": step, "groups": {}, "diffs": {}}
        vals = {k: [r[step] for r in v.values() if step in r] for k, v in groups.items()}
        for k, xs in vals.items():
            if xs:
                n, m, sd = stats(xs)
                row["groups"][k] = {"n": n, "mean": round(m, 3),
                                    "std": None if n < 2 else round(sd, 3)}
        for a, b in pairs:
            if len(vals[a]) < 2 or len(vals[b]) < 2:
                continue
            na, ma, sa = stats(vals[a])
            nb, mb, sb = stats(vals[b])
            va, vb = sa ** 2 / na, sb ** 2 / nb
            se = math.sqrt(va + vb)
            df = (va + vb) ** 2 / (va ** 2 / (na - 1) + vb ** 2 / (nb - 1))   # Welch
            half = t975(df) * se
            d = ma - mb
            row["diffs"][f"{a}-{b}"] = {
                "diff": round(d, 3), "se": round(se, 3), "ci95": [round(d - half, 3), round(d + half, 3)],
                "ci95_within_0.1dB": bool(abs(d) + half <= 0.1), "n": [na, nb]}
        row["paired"] = {}
        for a, b in paired:
            common = sorted(s for s in set(groups[a]) & set(groups[b])
                            if step in groups[a][s] and step in groups[b][s])
            if len(common) < 3:
                continue
            ds = [groups[a][s][step] - groups[b][s][step] for s in common]
            n, m, sd = stats(ds)
            se = sd / math.sqrt(n)
            half = t975(n - 1) * se
            xa = [groups[a][s][step] for s in common]
            xb = [groups[b][s][step] for s in common]
            _, ma, sa = stats(xa)
            _, mb, sb = stats(xb)
            r = sum((x - ma) * (y - mb) for x, y in zip(xa, xb)) / ((n - 1) * sa * sb)
            row["paired"][f"{a}-{b}"] = {
                "diff": round(m, 3), "se": round(se, 3), "ci95": [round(m - half, 3), round(m + half, 3)],
                "ci95_within_0.1dB": bool(abs(m) + half <= 0.1), "n": n, "corr": round(r, 2)}
        out["checkpoints"].append(row)
        print(json.dumps(row))
    path = os.path.join(REPO, "profiles", "r05", "psnr", "summary.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
