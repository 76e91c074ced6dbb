"""Where the f16x3 coarse sigma.bias gradient's distance from float64 comes
from at cfg4 (tests/test_gpu_cfg4.py): the forward's raw outputs (sigma, rgb)
of each arithmetic pushed through a float64 compositing + loss backward, so
d(sigma.bias) = sum d sigma is evaluated exactly on each forward's values."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import test_gpu_cfg4 as T  # noqa: E402
from oracle import nerf_oracle as O  # noqa: E402

DEV = torch.device("cuda", 0)
torch.set_num_threads(16)


def main(n=1024):
    from nerf_pl_amd import NeRF, ops
    from nerf_pl_amd.functions import mlp_apply
    _, _, _, rays, rgbs = T._batch()
    rays, rgbs = rays[:n].contiguous(), rgbs[:n]
    draws = [d[:n] for d in T._draws(T.B)]
    args = (T.S, False, 1.0, 1.0, T.I, 32768, False)
    pp64 = [{k: v.double() for k, v in p.items()} for p in T._params()]
    cap = {}
    O.render_rays(pp64, rays, *args, rng=O.ReplayRNG(draws), capture=cap, fp32_positions=True)
    z = cap["z_coarse"].float()
    raws = {"f64": cap["raw_coarse"].detach()}
    c32 = {}
    O.render_rays(T._params(), rays, *args, rng=O.ReplayRNG(draws), capture=c32,
                  z_fine_override=cap["z_fine"].float())
    raws["oracle fp32"] = c32["raw_coarse"].detach().double()
    for math in ("f16x3", "fp32", "bf16x6"):
        ops.MATH = math
        net = NeRF()
        net.load_state_dict(T._params()[0])
        net = net.to(DEV)
        with torch.no_grad():
            raws[math] = mlp_apply(net, rays=rays.to(DEV), z=z.to(DEV), spr=T.S).cpu().double()
    ref = None
    for name, raw in raws.items():
        r = raw.clone().requires_grad_(True)
        out = O.render_rays(pp64, rays, *args, rng=O.ReplayRNG(draws), raw_override={"coarse": r},
                            fp32_positions=True, z_fine_override=cap["z_fine"])
        T._loss(out, rgbs, torch.ones(n, dtype=torch.bool)).backward()
        gs = r.grad[:, 3]
        sb = gs.sum().item()
        if ref is None:
            ref = sb
            print(f"float64: d sigma.bias = {sb:.6e}, sum |d sigma| = {gs.abs().sum().item():.6e} "
                  f"(cancellation x{gs.abs().sum().item() / abs(sb):.0f})")
        e = (raw - raws["f64"]).abs()
        print(f"{name:12s} raw err: sigma max {e[:, 3].max():.2e}, rgb max {e[:, :3].max():.2e}; "
              f"d sigma.bias on its raw (float64 backward) {sb:.6e}, rel dev {abs(sb - ref) / abs(ref):.2e}")


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def per_ray(n=1024):
    """the rays that carry the coarse sigma.bias gradient's sensitivity to the
    fp32 rounding of the forward's outputs"""
    _, _, _, rays, rgbs = T._batch()
    rays, rgbs = rays[:n].contiguous(), rgbs[:n]
    draws = [d[:n] for d in T._draws(T.B)]
    args = (T.S, False, 1.0, 1.0, T.I, 32768, False)
    pp64 = [{k: v.double() for k, v in p.items()} for p in T._params()]
    cap = {}
    O.render_rays(pp64, rays, *args, rng=O.ReplayRNG(draws), capture=cap, fp32_positions=True)
    c32 = {}
    O.render_rays(T._params(), rays, *args, rng=O.ReplayRNG(draws), capture=c32,
                  z_fine_override=cap["z_fine"].float())
    gs = {}
    for name, raw in (("f64", cap["raw_coarse"].detach()), ("o32", c32["raw_coarse"].detach().double())):
        r = raw.clone().requires_grad_(True)
        out = O.render_rays(pp64, rays, *args, rng=O.ReplayRNG(draws), raw_override={"coarse": r},
                            fp32_positions=True, z_fine_override=cap["z_fine"])
        T._loss(out, rgbs, torch.ones(n, dtype=torch.bool)).backward()
        gs[name] = r.grad[:, 3].view(n, T.S)
    d = (gs["o32"] - gs["f64"]).sum(1)
    tot = gs["f64"].sum().item()
    order = d.abs().argsort(descending=True)
    noise = draws[1]
    sig = cap["raw_coarse"][:, 3].view(n, T.S).detach()
    rel = sig + noise.double()
    print(f"sum d sigma = {tot:.4e}; total deviation {d.sum().item():.3e}")
    for k in order[:12].tolist():
        rk = rel[k]
        pos = rk[rk > 0]
        print(f"ray {k}: dev {d[k].item():+.3e} ({d[k].item() / abs(tot):+.2e} of the sum), "
              f"sum d sigma {gs['f64'][k].sum().item():+.3e}, sum|d sigma| {gs['f64'][k].abs().sum().item():.3e}, "
              f"min |s+n| {rk.abs().min().item():.2e}, last s+n {rk[-1].item():+.3e}, "
              f"min positive {pos.min().item() if pos.numel() else float('nan'):.2e}")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "rays":
    per_ray()
