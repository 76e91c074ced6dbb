"""Follow-up of dev/grad_split.py: the f16x3 error of layers 1-3 on the cfg4
coarse pass, under output-gradient variants (range scaled, tiny samples
zeroed), against float64 autograd of the same variant."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import test_gpu_cfg4 as T  # noqa: E402
from oracle import nerf_oracle as O  # noqa: E402

DEV = torch.device("cuda", 0)
torch.set_num_threads(16)
KEYS = ["xyz_encoding_1.0.bias", "xyz_encoding_3.0.weight", "xyz_encoding_4.0.bias", "sigma.weight"]


def main(n=1024):
    from nerf_pl_amd import NeRF, ops
    from nerf_pl_amd.functions import mlp_apply
    _, _, _, rays, rgbs = T._batch()
    rays, rgbs = rays[:n].contiguous(), rgbs[:n]
    draws = [d[:n] for d in T._draws(T.B)]
    p32 = T._params()[0]
    cap = {}
    args = (T.S, False, 1.0, 1.0, T.I, 32768, False)
    pp64 = [{k: v.double() for k, v in p.items()} for p in T._params()]
    O.render_rays(pp64, rays, *args, rng=O.ReplayRNG(draws), capture=cap, fp32_positions=True)
    raw = cap["raw_coarse"].detach().clone().requires_grad_(True)
    cap2 = {}
    out = O.render_rays(pp64, rays, *args, rng=O.ReplayRNG(draws), capture=cap2,
                        raw_override={"coarse": raw}, fp32_positions=True)
    T._loss(out, rgbs, torch.ones(n, dtype=torch.bool)).backward()
    g0 = raw.grad.detach().float().double()      # what an fp32 backward hands the MLP
    z = cap2["z_coarse"].float()
    spr = z.shape[1]
    xyz = (rays[:, None, :3] + rays[:, None, 3:6] * z[:, :, None]).reshape(-1, 3)
    x64 = torch.cat([O.embed(xyz.double(), 10),
                     O.embed(rays[:, 3:6].double(), 4).repeat_interleave(spr, 0)], 1)
    pm = g0.abs().max(1).values
    variants = {"as is": g0, "x2^40": g0 * 2.0 ** 40, "x2^-40": g0 * 2.0 ** -40}
    for thr in (1e-30, 1e-20, 1e-12, 1e-8):
        variants[f"rows<{thr:g} zeroed"] = g0 * (pm >= thr).double()[:, None]
    variants["rows>=1e-12 only x1e-12"] = g0 * (pm < 1e-12).double()[:, None]
    # rows with a ReLU kink: a layer-1..8 pre-activation (float64) within thr of 0
    with torch.no_grad():
        pre_min = torch.full((x64.shape[0],), float("inf"), dtype=torch.float64)
        pre_min13 = pre_min.clone()
        h = x64[:, :63]
        for i in range(8):
            if i == 4:
                h = torch.cat([x64[:, :63], h], -1)
            pre = torch.nn.functional.linear(h, p32[f"xyz_encoding_{i+1}.0.weight"].double(),
                                             p32[f"xyz_encoding_{i+1}.0.bias"].double())
            pre_min = torch.minimum(pre_min, pre.abs().min(1).values)
            if i < 3:
                pre_min13 = torch.minimum(pre_min13, pre.abs().min(1).values)
            h = torch.relu(pre)
    big = pm >= 1e-8
    for thr in (1e-6, 1e-5, 1e-4, 1e-3):
        k = (pre_min13 < thr) & big
        print(f"kink rows |pre| < {thr:g} (layers 1-3) among {int(big.sum())} large-gradient rows: "
              f"{int(k.sum())}; any layer: {int(((pre_min < thr) & big).sum())}")
        variants[f"kink13<{thr:g} zeroed"] = g0 * (pre_min13 >= thr).double()[:, None]
    print(f"fp32-subnormal rows: {((pm > 0) & (pm < 1.18e-38)).sum().item()}, zero rows "
          f"{(pm == 0).sum().item()}, of {pm.numel()}")
    for name, g in variants.items():
        p = {k: v.double().requires_grad_(True) for k, v in p32.items()}
        (O.nerf_forward(p, x64) * g).sum().backward()
        line = []
        for math in ("f16x3", "fp32"):
            ops.MATH = math
            net = NeRF()
            net.load_state_dict(p32)
            net = net.to(DEV)
            o = mlp_apply(net, rays=rays.to(DEV), z=z.to(DEV), spr=spr)
            o.backward(g.float().to(DEV))
            gr = dict(net.named_parameters())
            for k in KEYS:
                e64 = p[k].grad
                e = ((gr[k].grad.cpu().double() - e64).norm() / (e64.norm() + 1e-300)).item()
                line.append(f"{math}:{k.split('.')[0][-1] if 'xyz' in k else k[:5]}{k[-4:]} {e:.1e}")
        print(f"{name:28s} " + "  ".join(line), flush=True)


if __name__ == "__main__":
    main()
