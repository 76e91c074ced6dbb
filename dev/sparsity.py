"""Zero fraction of the saved activations and gradient segments that the f16x3
weight gradient streams ("levers"): how many of the bytes it
reads are ReLU zeros, at the bench's default init and with trained weights.

    NERF_PL_AMD_DEBUG=1 python dev/sparsity.py [--weights trained.safetensors] [--out f.json]

One training render per model (128 stratified samples per ray, 4,096 rays of
the PSNR scene's training views, targets = the scene), backward, then the
buffers `functions._DEBUG` keeps: per segment, the fraction of exact zeros.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))

W32 = 32  # samples per block


def seg_zero(buf, off, width, nb):
    x = buf[off:off + width * W32 * nb]
    return float((x == 0).float().mean())


def block_stats(g_out):
    """fractions of samples / 32-sample blocks / 128-sample workgroups whose
    whole output gradient (d rgb, d sigma) is exactly zero"""
    n = g_out.shape[0]
    z = (g_out != 0).any(1)
    out = {"samples": n, "zero_grad_samples": round(1 - float(z.float().mean()), 4)}
    for k, name in ((32, "zero_grad_blocks32"), (128, "zero_grad_groups128")):
        m = n // k * k
        out[name] = round(1 - float(z[:m].view(-1, k).any(1).float().mean()), 4)
    return out


def bench_mode(out_path):
    """the bench's own cfg2 training step (seeded default init), a few steps"""
    import bench
    from nerf_pl_amd import functions
    from nerf_pl_amd.optim import FusedAdam
    args = bench.parse_args_for(["--config", "cfg2"]) if hasattr(bench, "parse_args_for") else None
    if args is None:
        sys.argv = ["bench.py"]
        args = bench.parse()
    dev = torch.device("cuda", 0)
    wl = bench.wl_nerf_train(args, dev, 0, ndc=False)
    params = [p for m in wl["models"] for p in m.parameters()]
    opt = FusedAdam(params, lr=5e-4, eps=1e-8)
    res = {"workload": wl["workload"], "steps": []}
    for it in range(6):
        functions._DEBUG.clear()
        loss = wl["step"]()
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        g = functions._DEBUG["g_outs"]      # fine backward first, then coarse
        row = {"step": it, "fine": block_stats(g[0]), "coarse": block_stats(g[1])}
        res["steps"].append(row)
        print(json.dumps(row), flush=True)
    if out_path:
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--weights", default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--bench", action="store_true", help="the bench's cfg2 step instead")
    args = ap.parse_args()
    assert os.environ.get("NERF_PL_AMD_DEBUG") == "1", "run with NERF_PL_AMD_DEBUG=1"
    if args.bench:
        return bench_mode(args.out)
    import psnr_compare as pc
    from nerf_pl_amd import Embedding, NeRF, functions, ops, render_rays
    dev = torch.device("cuda", 0)
    train, train_rgb, _, _ = pc.scene()
    g = torch.Generator().manual_seed(0)
    idx = torch.randint(0, train.shape[0], (4096,), generator=g)
    rays, tgt = train[idx].to(dev), train_rgb[idx].to(dev)
    emb = [Embedding(3, 10), Embedding(3, 4)]
    res = {"weights": os.path.basename(args.weights) if args.weights else "default init"}
    sd = None
    if args.weights:
        from safetensors.torch import load_file
        sd = load_file(args.weights)
    for tag, seed in (("coarse", 101), ("fine", 102)):
        m = NeRF()
        m.load_state_dict(pc.initial_params(seed, False))
        if sd is not None:
            m.load_state_dict({k[len(tag) + 1:]: v for k, v in sd.items() if k.startswith(tag + ".")})
        m = m.to(dev)
        out = render_rays([m], emb, rays, 128, False, 1, 0, 0, 32768, False, False)
        loss = torch.mean((out["rgb_coarse"] - tgt) ** 2)
        loss.backward()
        d = functions._DEBUG
        n = d["n"]
        nb = ops.n_blocks(n)
        save, gws = d["save"], d["grad_ws"]
        r = {"samples": n}
        r.update(block_stats(d["g_out"][:n]))
        r["pe"] = seg_zero(save, 0, 64, nb)
        for l in range(8):
            r[f"h{l + 1}"] = seg_zero(save, (64 + l * 256) * W32 * nb, 256, nb)
        r["hdir"] = seg_zero(save, (64 + 8 * 256) * W32 * nb, 128, nb)   # no feat segment (round 5)
        for l in range(8):
            r[f"dz{l + 1}"] = seg_zero(gws, l * 256 * W32 * nb, 256, nb)
        r["dzdir"] = seg_zero(gws, 8 * 256 * W32 * nb, 128, nb)   # no dfeat segment (round 5)
        # the wgrad operand bytes (17,808 B/sample): values that are zero
        widths = {"pe": 64, "hdir": 128, "dzdir": 128}
        widths.update({f"h{l + 1}": 256 for l in range(8)})
        widths.update({f"dz{l + 1}": 256 for l in range(8)})
        tot = sum(widths.values()) + 32 + 4 + 0   # + dir PE (32) + head (4): never zero
        r["zero_fraction_of_wgrad_values"] = round(
            sum(r[k] * w for k, w in widths.items()) / tot, 4)
        res[tag] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}
        print(tag, json.dumps(res[tag]), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
