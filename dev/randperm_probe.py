"""what stalled the 4-rank cfg4 rehearsal
(profiles/r04/dist/cfg4_gloo4_hang_v1.log: every rank in ops.py:83's copy).

One process, no collective: the pre-fix sampler's first epoch at cfg4's pool
(100 poses x 800^2 = 64M pixels) exactly as round 3's RaySampler._new_epoch
drew it -- torch.randperm on the device with a device generator, padded, the
rank's shard sliced -- then the first cfg4 training step of bench.py's
workload (coarse_z's 4-byte table copy is the call the ranks were stuck in).
Every phase is timed with a host clock around a torch.cuda.synchronize();
run it under `rocprofv3 --kernel-trace --stats` to name the kernels.

    python dev/randperm_probe.py [--world 4] [--rank 0] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(name, fn, out):
    torch.cuda.synchronize()
    t = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    out.append((name, (time.perf_counter() - t) * 1e3))
    print(f"[probe] {name}: {out[-1][1]:.2f} ms", flush=True)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--poses", type=int, default=100)
    ap.add_argument("--img", type=int, default=800)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    total = a.poses * a.img * a.img
    log = []
    timed("torch init (empty + sync)", lambda: torch.empty(1, device=dev), log)
    pool = timed("pool_rgb torch.rand(64M x 3)",
                 lambda: torch.rand(total, 3, device=dev), log)

    def prefix_epoch(epoch):
        # round 3's RaySampler._new_epoch, line for line (git show db92dd6:nerf_pl_amd/rays.py)
        gen = torch.Generator(device=dev).manual_seed(99 + epoch)
        perm = torch.randperm(total, device=dev, generator=gen)
        pad = (-total) % a.world
        if pad:
            perm = torch.cat([perm, perm[:pad]])
        return perm[a.rank::a.world]

    shard = None
    for e in range(a.reps):
        shard = timed(f"pre-fix epoch {e}: device randperm({total}) + pad + shard", lambda: prefix_epoch(e), log)
    assert shard is not None and shard.numel() == -(-total // a.world)

    # the first cfg4 step on that shard, as bench.wl_nerf_train runs it
    from nerf_pl_amd import Embedding, NeRF, render_rays
    from nerf_pl_amd.losses import MSELoss
    from nerf_pl_amd.rays import blender_focal, generate_rays, pose_spherical
    poses = torch.stack([pose_spherical(-180.0 + 360.0 * k / a.poses, -30.0, 4.0)
                         for k in range(a.poses)]).to(dev)
    torch.manual_seed(0)
    models = [NeRF().to(dev), NeRF().to(dev)]
    emb = [Embedding(3, 10), Embedding(3, 4)]
    loss_fn = MSELoss()
    focal = blender_focal(a.img)
    for it in range(3):
        sel = shard[it * 4096:(it + 1) * 4096]
        rays, rgbs = timed(f"step {it}: generate_rays", lambda: generate_rays(
            poses, a.img, a.img, focal, 1.0, 200.0, sel, False, rgb_pool=pool), log)
        res = timed(f"step {it}: render_rays (64+128)", lambda: render_rays(
            models, emb, rays, 64, False, 1.0, 1.0, 128, 32768, False, False), log)
        timed(f"step {it}: loss + backward", lambda: loss_fn(res, rgbs).backward(), log)
    rec = {"total": total, "world": a.world, "rank": a.rank, "phases_ms": log,
           "torch": torch.__version__, "device": torch.cuda.get_device_name(0)}
    print(json.dumps(rec), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
