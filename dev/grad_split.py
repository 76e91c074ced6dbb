"""cfg4 gradient accuracy, MLP backward alone (VERDICT r5 item 5 follow-up).

The cfg4 rank batch's coarse pass: the per-sample output gradient d raw of the
training loss is taken from the float64 oracle (fp32 positions), then fed to
our fused MLP backward in each arithmetic and to float64 / fp32 autograd of
the oracle MLP on the same inputs.  Prints each parameter gradient's normwise
distance from float64, so an arithmetic's own error is seen without the
compositing or the forward in between."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import test_gpu_cfg4 as T  # noqa: E402
from oracle import nerf_oracle as O  # noqa: E402

DEV = torch.device("cuda", 0)
torch.set_num_threads(16)


def main(n=1024, which="coarse"):
    from nerf_pl_amd import NeRF, ops
    from nerf_pl_amd.functions import mlp_apply
    _, _, _, rays, rgbs = T._batch()
    rays, rgbs = rays[:n].contiguous(), rgbs[:n]
    draws = [d[:n] for d in T._draws(T.B)]
    mi = 0 if which == "coarse" else 1
    p32 = T._params()[mi]
    p64 = {k: v.double() for k, v in p32.items()}
    # depths and the loss's per-sample output gradient, float64 oracle
    cap = {}
    args = (T.S, False, 1.0, 1.0, T.I, 32768, False)
    pp64 = [{k: v.double() for k, v in p.items()} for p in T._params()]
    O.render_rays(pp64, rays, *args, rng=O.ReplayRNG(draws), capture=cap, fp32_positions=True)
    raw = cap[f"raw_{which}"].detach().clone().requires_grad_(True)
    cap2 = {}
    out = O.render_rays(pp64, rays, *args, rng=O.ReplayRNG(draws), capture=cap2,
                        raw_override={which: raw}, fp32_positions=True,
                        z_fine_override=cap["z_fine"] if which == "fine" else None)
    T._loss(out, rgbs, torch.ones(n, dtype=torch.bool)).backward()
    gout = raw.grad.detach()
    z = cap2[f"z_{which}"].float()
    spr = z.shape[1]
    a = gout.abs()
    print(f"{which}: {gout.shape[0]} samples; |d rgb| max {a[:, :3].max():.3g}, |d sigma| max "
          f"{a[:, 3].max():.3g}; nonzero {(a.sum(1) > 0).float().mean():.3f}; "
          f"quantiles of per-sample max: " +
          " ".join(f"{q}:{a.max(1).values.quantile(q).item():.3g}" for q in (0.5, 0.9, 0.99, 1.0)))
    # oracle MLP autograd, float64 and fp32, on the fp32 positions
    xyz = (rays[:, None, :3] + rays[:, None, 3:6] * z[:, :, None]).reshape(-1, 3)
    dirs = O.embed(rays[:, 3:6].double(), 4).repeat_interleave(spr, 0)
    ref = {}
    for dt in (torch.float64, torch.float32):
        p = {k: v.to(dt).requires_grad_(True) for k, v in p32.items()}
        x = torch.cat([O.embed(xyz.to(dt), 10), dirs.to(dt)], 1)
        (O.nerf_forward(p, x) * gout.to(dt)).sum().backward()
        ref[dt] = {k: v.grad.double() for k, v in p.items()}
    rows = {}
    for math in ("f16x3", "bf16x6", "fp32"):
        ops.MATH = math
        net = NeRF()
        net.load_state_dict(p32)
        net = net.to(DEV)
        o = mlp_apply(net, rays=rays.to(DEV), z=z.to(DEV), spr=spr)
        (o.double() * gout.to(DEV)).sum().backward()
        for k, q in net.named_parameters():
            e64 = ref[torch.float64][k]
            rows.setdefault(k, {})[math] = ((q.grad.cpu().double() - e64).norm() / e64.norm()).item()
    for k, r in rows.items():
        e64 = ref[torch.float64][k]
        f = ((ref[torch.float32][k] - e64).norm() / e64.norm()).item()
        print(f"{k:32s} fp32-oracle {f:.2e}  " + "  ".join(f"{m} {v:.2e}" for m, v in r.items()))


if __name__ == "__main__":
    main(which=sys.argv[1] if len(sys.argv) > 1 else "coarse")
