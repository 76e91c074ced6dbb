"""PSNR of a short training run: this package vs the reference (BASELINE.json
target: "PSNR within 0.1 dB of the reference").

    python scripts/psnr_compare.py --impl ours        # on the MI355X box
    python scripts/psnr_compare.py --impl reference   # here only (imports /root/reference)
    python scripts/psnr_compare.py --impl oracle      # on the MI355X box: the reference's
        # algorithm (oracle/nerf_oracle.py, pinned bit-exact to the reference) in PyTorch
        # fp32 on the GPU -- the reference as its authors ran it (PyTorch ops on a GPU,
        # here hipBLAS GEMMs); test infrastructure used as the checker, not the product

Both legs train the same NeRF pair (seeded parameters, oracle.make_params) with
the reference's training step (train.py:103-117: render_rays 64+64, perturb 1,
noise_std 1, MSE coarse+fine, Adam 5e-4 / eps 1e-8) on the same ray batches,
AND the same random draws: every rand/randn of render_rays is taken from the
CPU torch generator in the reference's draw order (the reference consumes the
global generator itself; our leg draws the same tensors and moves them to the
device).  Scene: an analytic density/colour field (three soft boxes), ground
truth rendered by 1024-sample quadrature in float64; 24 training views and 2
held-out views of 64x64 on a Blender-style orbit, near/far 2/6.  PSNR
(metrics.py:12-13) of the fine rgb on the held-out views is logged along the
way; results go to profiles/r01/psnr_<impl>.json.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from nerf_pl_amd.rays import blender_focal, get_ray_directions, get_rays, pose_spherical  # noqa: E402
from oracle.nerf_oracle import make_params  # noqa: E402

IMG = 64
NEAR, FAR = 2.0, 6.0
BOXES = [  # centre, half-size, colour
    ((0.0, 0.0, -0.3), (0.6, 0.6, 0.3), (0.85, 0.2, 0.15)),
    ((0.3, -0.2, 0.35), (0.25, 0.35, 0.35), (0.1, 0.6, 0.9)),
    ((-0.45, 0.35, 0.25), (0.2, 0.2, 0.5), (0.95, 0.85, 0.1)),
]


def field(x: torch.Tensor):
    """Analytic sigma (N,) and rgb (N,3) of three soft-edged boxes (float64)."""
    sig = torch.zeros(x.shape[0], dtype=x.dtype)
    col = torch.zeros(x.shape[0], 3, dtype=x.dtype)
    for c, h, rgb in BOXES:
        d = ((x - torch.tensor(c, dtype=x.dtype)).abs() - torch.tensor(h, dtype=x.dtype)).max(1).values
        s = 40.0 * torch.sigmoid(-d * 60.0)
        col += s[:, None] * torch.tensor(rgb, dtype=x.dtype)
        sig += s
    col = col / sig.clamp_min(1e-9)[:, None]
    return sig, col


def render_gt(rays: torch.Tensor, n=1024):
    o, d = rays[:, :3].double(), rays[:, 3:6].double()
    t = torch.linspace(NEAR, FAR, n, dtype=torch.float64)
    out = []
    for i in range(0, rays.shape[0], 2048):
        oo, dd = o[i:i + 2048], d[i:i + 2048]
        x = (oo[:, None] + dd[:, None] * t[None, :, None]).reshape(-1, 3)
        s, c = field(x)
        s, c = s.view(oo.shape[0], n), c.view(oo.shape[0], n, 3)
        delta = torch.full_like(s, (FAR - NEAR) / (n - 1))
        a = 1 - torch.exp(-s * delta)
        T = torch.cumprod(torch.cat([torch.ones_like(a[:, :1]), 1 - a + 1e-10], 1), 1)[:, :-1]
        out.append((a * T)[..., None].mul(c).sum(1))
    return torch.cat(out).float()


def scene():
    focal = blender_focal(IMG)
    dirs = get_ray_directions(IMG, IMG, focal)
    views = []
    for k in range(26):
        theta = -180.0 + 360.0 * k / 24 if k < 24 else 15.0 + 180.0 * (k - 24)
        phi = -30.0 if k < 24 else -45.0
        o, d = get_rays(dirs, pose_spherical(theta, phi, 4.0).float())
        rays = torch.cat([o, d, torch.full_like(o[:, :1], NEAR), torch.full_like(o[:, :1], FAR)], 1)
        views.append(rays)
    train = torch.cat(views[:24])
    test = torch.cat(views[24:])
    return train, render_gt(train), test, render_gt(test)


class CPUDraws:
    """rand/randn from the global CPU generator, moved to ``device``."""

    seed = 0

    def rand(self, shape, device):
        return torch.rand(*shape).to(device)

    def randn(self, shape, device):
        return torch.randn(*shape).to(device)


def import_reference():
    shim = types.ModuleType("torchsearchsorted")
    shim.searchsorted = lambda a, v, side="left", out=None: torch.searchsorted(
        a.contiguous(), v.contiguous(), right=(side == "right"))
    sys.modules["torchsearchsorted"] = shim
    sys.path.insert(0, os.environ.get("NERF_REFERENCE", "/root/reference"))
    import models.nerf as ref_nerf            # noqa: E402
    import models.rendering as ref_rendering  # noqa: E402
    return ref_nerf, ref_rendering


def initial_params(seed: int, perturb_ulp: bool):
    p = make_params(seed)
    if perturb_ulp:
        p = {k: torch.nextafter(v, torch.full_like(v, math.inf)) for k, v in p.items()}
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--impl", choices=["ours", "reference", "oracle"], required=True)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--eval-every", type=int, default=250)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--draw-seed", type=int, default=7,
                    help="seed of the render draws (run-to-run spread: vary it)")
    ap.add_argument("--perturb-ulp", action="store_true",
                    help="move every initial parameter up by one fp32 ulp (control run: the "
                         "PSNR spread that an ulp-level difference alone produces)")
    ap.add_argument("--save-weights", default=None,
                    help="write the trained parameters (safetensors) for --eval-weights")
    ap.add_argument("--eval-weights", default=None,
                    help="no training: render the held-out views with these trained "
                         "parameters and report the PSNR (same-weights renderer parity)")
    ap.add_argument("--draw-seeds", default=None,
                    help="draw seeds (comma-separated lo-hi ranges) run one after another in this process "
                         "(with --out-dir)")
    ap.add_argument("--out-dir", default="gpurun_out/psnr")
    ap.add_argument("--deadline-s", type=float, default=0,
                    help="with --draw-seeds: start no further seed once this many seconds "
                         "have passed since the first one started (the time-boxed GPU calls)")
    ap.add_argument("--out", default=None, help="JSON path (default profiles/r01/psnr_<impl>.json)")
    args = ap.parse_args()
    torch.set_num_threads(args.threads or min(16, os.cpu_count() or 1))
    S, I = 64, 64
    train, train_rgb, test, test_rgb = scene()
    if args.draw_seeds:
        # several runs in one process (the scene's ground truth is built once);
        # one JSON per seed under --out-dir, named like scripts/psnr.sh's
        seeds = []
        for part in args.draw_seeds.split(","):     # "lo-hi" ranges, comma-separated
            lo, _, hi = part.partition("-")
            seeds += range(int(lo), int(hi or lo) + 1)
        if args.impl == "ours":
            from nerf_pl_amd import ops
            tag = ops.MATH
        else:
            tag = args.impl
        os.makedirs(args.out_dir, exist_ok=True)
        t0 = time.time()
        for sd in seeds:
            if args.deadline_s and time.time() - t0 > args.deadline_s:
                print(json.dumps({"deadline": args.deadline_s, "next_seed": sd}), flush=True)
                break
            args.draw_seed = sd
            args.out = os.path.join(args.out_dir, f"{tag}_s{sd}.json")
            run_one(args, S, I, train, train_rgb, test, test_rgb)
        return
    run_one(args, S, I, train, train_rgb, test, test_rgb)



def run_one(args, S, I, train, train_rgb, test, test_rgb):
    """one training run (models, optimiser and draws from args.draw_seed)"""
    if args.impl == "ours":
        from nerf_pl_amd import Embedding, NeRF, render_rays
        dev = torch.device("cuda", 0)
        models = []
        for s in (101, 102):
            m = NeRF()
            m.load_state_dict(initial_params(s, args.perturb_ulp))
            models.append(m.to(dev))
        emb = [Embedding(3, 10), Embedding(3, 4)]
        draws = CPUDraws()

        def render(rays, test_time=False):
            return render_rays(models, emb, rays.to(dev), S, False, 1.0, 1.0, I, 32768, False,
                               test_time, rng=draws)
    elif args.impl == "oracle":
        from oracle import nerf_oracle as O
        dev = torch.device("cuda", 0)
        params = [{k: v.to(dev).requires_grad_(True)
                   for k, v in initial_params(s, args.perturb_ulp).items()} for s in (101, 102)]

        class _Holder(torch.nn.Module):      # parameters() / state_dict() for the harness
            def __init__(self, p):
                super().__init__()
                self._p = p

            def parameters(self, recurse=True):
                return iter(self._p.values())

            def state_dict(self, *a, **k):
                return dict(self._p)

            def load_state_dict(self, sd, *a, **k):
                with torch.no_grad():
                    for n, v in sd.items():
                        self._p[n].copy_(v)
        models = [_Holder(p) for p in params]

        class _DevDraws:
            def rand(self, shape):
                return torch.rand(*shape).to(dev)

            def randn(self, shape):
                return torch.randn(*shape).to(dev)
        odraws = _DevDraws()

        def render(rays, test_time=False):
            return O.render_rays(params, rays.to(dev), S, False, 1.0, 1.0, I, 32768, False,
                                 test_time, rng=odraws)
    else:
        ref_nerf, ref_rendering = import_reference()
        dev = torch.device("cpu")
        models = []
        for s in (101, 102):
            m = ref_nerf.NeRF()
            m.load_state_dict(initial_params(s, args.perturb_ulp))
            models.append(m)
        emb = [ref_nerf.Embedding(3, 10), ref_nerf.Embedding(3, 4)]

        def render(rays, test_time=False):
            return ref_rendering.render_rays(models, emb, rays, S, False, 1.0, 1.0, I, 32768,
                                             False, test_time)

    opt = torch.optim.Adam([p for m in models for p in m.parameters()], lr=5e-4, eps=1e-8)
    gen = torch.Generator().manual_seed(2024)
    torch.manual_seed(args.draw_seed)   # the render draws (both legs consume this stream)
    log, losses = [], []

    def evaluate(step):
        with torch.no_grad():
            pred = torch.cat([render(test[i:i + 4096])["rgb_fine"].cpu()
                              for i in range(0, test.shape[0], 4096)])
        p = float(-10.0 * torch.log10(torch.mean((pred - test_rgb) ** 2)))
        log.append({"step": step, "psnr": p, "elapsed_s": round(time.time() - t0, 1)})
        print(json.dumps(log[-1]), flush=True)

    t0 = time.time()
    if args.eval_weights:
        from safetensors.torch import load_file
        sd = load_file(args.eval_weights)
        for tag, m in zip(("coarse", "fine"), models):
            m.load_state_dict({k[len(tag) + 1:]: v.to(dev) for k, v in sd.items()
                               if k.startswith(tag + ".")})
        with torch.no_grad():
            pred = torch.cat([render(test[i:i + 4096])["rgb_fine"].cpu()
                              for i in range(0, test.shape[0], 4096)])
        p = float(-10.0 * torch.log10(torch.mean((pred - test_rgb) ** 2)))
        path = args.out or os.path.join(REPO, "profiles", "r02", f"psnr_eval_{args.impl}.json")
        np.save(path[:-5] + "_pred.npy", pred.numpy())
        out = {"impl": args.impl, "eval_weights": os.path.basename(args.eval_weights),
               "draw_seed": args.draw_seed, "psnr": p}
        if args.impl == "ours":
            from nerf_pl_amd import ops
            out["mlp_arithmetic"] = ops.MATH
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps(out))
        return
    for step in range(1, args.steps + 1):
        idx = torch.randint(0, train.shape[0], (args.batch,), generator=gen)
        rays, tgt = train[idx].to(dev), train_rgb[idx].to(dev)
        res = render(rays)
        loss = torch.mean((res["rgb_coarse"] - tgt) ** 2) + torch.mean((res["rgb_fine"] - tgt) ** 2)
        opt.zero_grad()
        loss.backward()
        opt.step()
        if step <= 20 or step % 50 == 0:
            losses.append({"step": step, "loss": loss.item()})
            print(json.dumps({"step": step, "loss": loss.item(),
                              "elapsed_s": round(time.time() - t0, 1)}), flush=True)
        if step % args.eval_every == 0:
            # eval consumes draws too; keep both legs in lockstep by saving the stream
            state = torch.get_rng_state()
            evaluate(step)
            torch.set_rng_state(state)
    if args.save_weights:
        from safetensors.torch import save_file
        save_file({f"{tag}.{k}": v.detach().cpu().contiguous()
                   for tag, m in zip(("coarse", "fine"), models)
                   for k, v in m.state_dict().items()}, args.save_weights)
    out = {"impl": args.impl, "steps": args.steps, "perturb_ulp": args.perturb_ulp, "batch": args.batch, "samples": [S, I],
           "img": IMG, "train_views": 24, "test_views": 2, "draw_seed": args.draw_seed, "psnr": log, "loss": losses,
           "final_psnr": log[-1]["psnr"] if log else None,
           "threads": torch.get_num_threads() if args.impl == "reference" else None}
    if args.impl == "ours":
        from nerf_pl_amd import ops
        out["mlp_arithmetic"] = ops.MATH
    elif args.impl == "oracle":
        out["mlp_arithmetic"] = "torch fp32 (hipBLAS) -- the reference algorithm on the GPU"
    path = args.out or os.path.join(REPO, "profiles", "r01", f"psnr_{args.impl}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
