"""The training step on trained weights: the bench times the
reference's step at its random init, where ~half the samples carry a
gradient; a NeRF that has learnt its scene leaves most samples in empty
space or behind a surface, with an exactly zero gradient.  This times the
cfg2-shaped step (4,096 rays, 64 + 128 samples, perturb 1, noise 1, MSE,
Adam) on the PSNR scene's training views with weights trained by
scripts/psnr_compare.py --save-weights: the zero-gradient sample lists with
the adaptive deferred save (NERF_PL_AMD_DEFER_SAVE=auto, the default), with a
forward-time save (none), and the every-sample backward.

    python dev/trained_step.py <weights.safetensors> [--steps 20] [--out f.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("weights")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--out", default=None)
    ap.add_argument("--modes", default="auto,none,every_sample",
                    help="DEFER_SAVE settings to time (auto, all, none, sigma) and/or every_sample")
    args = ap.parse_args()
    import psnr_compare as pc
    from safetensors.torch import load_file
    from nerf_pl_amd import Embedding, NeRF, functions, render_rays
    from nerf_pl_amd.losses import MSELoss
    from nerf_pl_amd.optim import FusedAdam
    dev = torch.device("cuda", 0)
    train, train_rgb, _, _ = pc.scene()
    train, train_rgb = train.to(dev), train_rgb.to(dev)
    sd = load_file(args.weights)
    emb = [Embedding(3, 10), Embedding(3, 4)]
    res = {"weights": os.path.basename(args.weights), "rays": 4096, "samples": [64, 128]}
    for mode in args.modes.split(","):
        active = mode != "every_sample"
        functions.ACTIVE_SAMPLES = active
        functions.DEFER_SAVE = mode if active else "none"
        models = []
        for tag in ("coarse", "fine"):
            m = NeRF()
            m.load_state_dict({k[len(tag) + 1:]: v for k, v in sd.items() if k.startswith(tag + ".")})
            models.append(m.to(dev))
        opt = FusedAdam([p for m in models for p in m.parameters()], lr=5e-4, eps=1e-8)
        loss_fn = MSELoss()
        g = torch.Generator(device=dev).manual_seed(0)

        def step():
            idx = torch.randint(0, train.shape[0], (4096,), device=dev, generator=g)
            out = render_rays(models, emb, train[idx], 64, False, 1.0, 1.0, 128, 32768, False)
            loss = loss_fn(out, train_rgb[idx])
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            return loss

        for _ in range(args.warmup):
            step()
        functions.ACTIVE_LOG = [] if active else None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            loss = step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        row = {"ms_per_step": round(el / args.steps * 1e3, 3),
               "rays_per_s": round(4096 * args.steps / el, 1), "loss": round(loss.item(), 6)}
        if active:
            fr = [int(sl[i].item()) / i for sl, i in functions.ACTIVE_LOG]
            row["listed_fraction_fine"] = round(sum(fr[0::2]) / len(fr[0::2]), 4)
            row["listed_fraction_coarse"] = round(sum(fr[1::2]) / len(fr[1::2]), 4)
            functions.ACTIVE_LOG = None
            row["deferred_last_step"] = [bool(m.__dict__.get("_nr_defer_last")) for m in models]
        res[mode] = row
        print(mode, json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
