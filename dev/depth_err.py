"""the max ABSOLUTE errors of render_rays' depth and
weights (coarse and fine) against the oracle, split into where they come from.

Per case (golden fixtures, full cfg2 / cfg3 batches, the cfg4 rank batch):
  e2e   ours vs the fp32 oracle (the reference's algorithm), same draws
  comp  our compositing kernel on the oracle's own raw MLP outputs and depths
        vs the oracle's compositing (the composite's share of the error)
  f64   ours and the fp32 oracle vs the float64 oracle evaluated on the fp32
        sample positions (oracle fp32_positions), every fine pass at our depths
Prints one line per case and quantity; writes gpurun_out/depth_err.json.
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
from conftest import golden_cases, golden_cfg, golden_draws, load_golden  # noqa: E402
from oracle import nerf_oracle as O  # noqa: E402

DEV = torch.device("cuda", 0)
torch.set_num_threads(16)


def models_of(params):
    from nerf_pl_amd import NeRF
    out = []
    for p in params:
        m = NeRF()
        m.load_state_dict(p)
        out.append(m.to(DEV))
    return out


def run_case(name, rays, cfg, params, draws):
    from nerf_pl_amd import Embedding, ReplayRNG, ops, render_rays
    S, I = cfg["N_samples"], cfg["N_importance"]
    args = (S, cfg["use_disp"], cfg["perturb"], cfg["noise_std"], I, 32768, cfg["white_back"],
            cfg["test_time"])
    cap = {}
    with torch.no_grad():
        res = render_rays(models_of(params[:2 if I else 1]), [Embedding(3, 10), Embedding(3, 4)],
                          rays.to(DEV), *args, rng=ReplayRNG(draws), _capture=cap)
    ocap = {}
    ref = O.render_rays(params, rays, *args, rng=O.ReplayRNG(draws), capture=ocap)
    n = rays.shape[0]
    bad = np.zeros(n, bool)
    if "z_fine" in cap:
        zf = cap["z_fine"].cpu().numpy()
        bad = (zf != ocap["z_fine"].numpy()).any(1)
    row = {"rays": n, "screened": int(bad.sum())}

    def mx(a, b, rows=None):
        e = np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).reshape(n, -1).max(1)
        if rows is not None:
            e = e[rows]
        return float(e.max()) if e.size else 0.0

    good = ~bad
    for k in ref:
        if k.startswith("depth") or k.startswith("rgb") or k.startswith("opac"):
            row[f"e2e_{k}"] = mx(res[k].cpu(), ref[k], good)
            if k.startswith("depth"):
                row[f"max|{k}|"] = float(ref[k].abs().max())
    row["e2e_weights_coarse"] = mx(cap["weights_coarse"].cpu(), ocap["weights_coarse"]) \
        if "weights_coarse" in cap else None
    if "weights_fine" in cap:
        row["e2e_weights_fine"] = mx(cap["weights_fine"].cpu(), ocap["weights_fine"], good)

    # compositing alone, on the oracle's raw outputs and depths
    noise_c = draws[1 if cfg["perturb"] > 0 else 0]
    passes = [("coarse", ocap["raw_coarse"], ocap["z_coarse"], noise_c)]
    if I:
        passes.append(("fine", ocap["raw_fine"], ocap["z_fine"], draws[-1]))
    rd = rays.to(DEV)
    for which, raw, z, nz in passes:
        if raw.shape[-1] < 4:
            continue
        rgb, depth, opac, w = ops.composite_forward(raw.contiguous().to(DEV), z.contiguous().to(DEV), rd,
                                                    torch.as_tensor(nz).float().contiguous().to(DEV),
                                                    cfg["noise_std"], 0, 0, cfg["white_back"])
        ow = ocap[f"weights_{which}"]
        row[f"comp_depth_{which}"] = mx(depth.cpu(), (ow * z).sum(-1))
        row[f"comp_weights_{which}"] = mx(w.cpu(), ow)

    # float64 anchoring (fp32 positions, fine pass at our depths)
    zf_ours = cap["z_fine"].cpu() if "z_fine" in cap else None
    p64 = [{k: v.double() for k, v in p.items()} for p in params]
    c64, c32 = {}, {}
    o64 = O.render_rays(p64, rays, *args, rng=O.ReplayRNG(draws), capture=c64,
                        z_fine_override=zf_ours, fp32_positions=True)
    o32 = O.render_rays(params, rays, *args, rng=O.ReplayRNG(draws), capture=c32,
                        z_fine_override=zf_ours)
    for k in o64:
        if k.startswith("depth"):
            row[f"f64_ours_{k}"] = mx(res[k].cpu(), o64[k])
            row[f"f64_o32_{k}"] = mx(o32[k], o64[k])
    for which in ("coarse", "fine"):
        if f"weights_{which}" in cap:
            row[f"f64_ours_w_{which}"] = mx(cap[f"weights_{which}"].cpu(), c64[f"weights_{which}"])
            row[f"f64_o32_w_{which}"] = mx(c32[f"weights_{which}"], c64[f"weights_{which}"])
    print(name, json.dumps({k: (f"{v:.3g}" if isinstance(v, float) else v) for k, v in row.items()}),
          flush=True)
    return row


def draws_for(n, S, I, seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.rand(n, S, generator=g), torch.randn(n, S, generator=g),
            torch.rand(n, I, generator=g), torch.rand(n, I, generator=g),
            torch.randn(n, S + I, generator=g)]


def main():
    from nerf_pl_amd.rays import blender_rays, llff_ndc_rays
    out = {}
    for c in golden_cases():
        if c.endswith("_grad"):
            continue
        fx = load_golden(c)
        cfg = golden_cfg(fx)
        params = [O.make_params(cfg["seeds"][m], sigma_bias=cfg["sigma_bias"]) for m in range(2)]
        out[c] = run_case(c, torch.from_numpy(fx["rays"]), cfg, params,
                          [torch.from_numpy(d) for d in golden_draws(fx)])
    base = dict(use_disp=False, perturb=1.0, noise_std=1.0, white_back=False, test_time=False)
    params = [O.make_params(11, sigma_bias=0.5), O.make_params(12, sigma_bias=0.5)]
    for kind in ("cfg2", "cfg3"):
        g = torch.Generator().manual_seed(5)
        if kind == "cfg2":
            pool, S, I = blender_rays(400, 4, near=1.0, far=200.0), 64, 128
        else:
            pool, S, I = llff_ndc_rays(504, 378, n_poses=2), 64, 64
        rays = pool[torch.randperm(pool.shape[0], generator=g)[:4096]].contiguous()
        out[kind] = run_case(kind, rays, dict(base, N_samples=S, N_importance=I), params,
                             draws_for(4096, S, I, 9))
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/depth_err.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
