"""How much of the forward's work lies behind an exactly-zero transmittance
(early ray termination): per ray of the bench's cfg2 batch, the
first sample at which T = prod (1 - alpha + 1e-10) (double, as the compositing
backward forms it) drops below a threshold, and the fraction of 32-sample
chunks that would then still be evaluated (dev tool).

    python dev/transmittance_probe.py [--rays N] [--device cpu|cuda] [--weights f.safetensors]
"""
import argparse
import json
import math
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=256)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--weights", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device(a.device)
    from nerf_pl_amd import Embedding, NeRF, render_rays
    from nerf_pl_amd.rays import RaySampler, blender_focal, pose_spherical
    W = H = 400
    focal, near, far = blender_focal(W), 1.0, 200.0
    poses = torch.stack([pose_spherical(-180.0 + 360.0 * k / 40, -30.0, 4.0) for k in range(40)]).to(dev)
    torch.manual_seed(1234)
    pool = torch.rand(poses.shape[0] * H * W, 3, device=dev)
    if dev.type == "cuda":
        sampler = RaySampler(poses, H, W, focal, near, far, rgb_pool=pool, seed=99)
    torch.manual_seed(0)
    models = [NeRF().to(dev), NeRF().to(dev)]
    if a.weights:
        from safetensors.torch import load_file
        sd = load_file(a.weights)
        for i, m in enumerate(models):
            m.load_state_dict({k[len(f"m{i}."):]: v for k, v in sd.items() if k.startswith(f"m{i}.")})
    emb = [Embedding(3, 10), Embedding(3, 4)]
    if dev.type == "cuda":
        rays, _ = sampler.next(a.rays)
    else:    # host: random pixels of random poses (rays.get_rays, the reference's formula)
        from nerf_pl_amd.rays import get_ray_directions, get_rays
        g = torch.Generator().manual_seed(99)
        d = get_ray_directions(H, W, focal).reshape(-1, 3)
        pi = torch.randint(0, poses.shape[0], (a.rays,), generator=g)
        px = torch.randint(0, H * W, (a.rays,), generator=g)
        o_l, d_l = [], []
        for k in range(a.rays):
            o, dd = get_rays(d[px[k]].view(1, 1, 3), poses[pi[k]])
            o_l.append(o.view(3)); d_l.append(dd.view(3))
        o, dd = torch.stack(o_l), torch.stack(d_l)
        rays = torch.cat([o, dd, torch.full((a.rays, 1), near), torch.full((a.rays, 1), far)], 1)
    cap = {}
    with torch.no_grad():
        render_rays(models, emb, rays, 64, False, 1.0, 1.0, 128, 32768, False, False, _capture=cap)
    out = {}
    for name, wkey, zkey in (("coarse", "weights_coarse", "z_coarse"), ("fine", "weights_fine", "z_fine")):
        w = cap[wkey].double().cpu()
        n, S = w.shape
        # T_i = w_i / alpha_i is not recoverable where alpha = 0; use the
        # suffix of exactly-zero weights instead: the first index from which
        # every weight is 0 (weights are alpha * T, T non-increasing)
        nz = (w != 0)
        last = torch.where(nz.any(1), S - 1 - nz.flip(1).int().argmax(1), torch.full((n,), -1))
        first_dead = last + 1          # samples >= first_dead have w == 0
        chunks = torch.clamp(torch.div(first_dead + 31, 32, rounding_mode="floor"), min=1)
        out[name] = {
            "samples_per_ray": S,
            "live_sample_fraction": float(first_dead.double().mean() / S),
            "zero_weight_fraction": float((w == 0).double().mean()),
            "chunk_fraction_evaluated": float(chunks.double().mean() / math.ceil(S / 32)),
            "first_dead_quantiles": [int(x) for x in torch.quantile(first_dead.double(),
                                      torch.tensor([0.1, 0.25, 0.5, 0.75, 0.9], dtype=torch.double))],
        }
    print(json.dumps(out, indent=1))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
