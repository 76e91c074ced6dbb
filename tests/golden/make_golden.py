"""Generate the golden fixtures by running the REFERENCE implementation.

Run in the survey/build container only (it needs /root/reference, which never
exists on the GPU box):

    python tests/golden/make_golden.py

What it does
* imports ``models.nerf`` and ``models.rendering`` from /root/reference.  The
  reference's ``torchsearchsorted`` submodule is un-vendored (empty directory,
  ``.gitmodules:1-3``), so ``torchsearchsorted.searchsorted`` is provided as
  ``torch.searchsorted(..., right=(side == 'right'))`` -- the replacement the
  reference itself uses (``rendering.py:38`` commented, ``rendering_shadows.py:41``
  live).  Same numpy ``side='right'`` semantics.
* loads seeded parameters (``oracle.nerf_oracle.make_params``) into reference
  ``NeRF`` modules through ``load_state_dict``;
* swaps ``models.rendering.torch`` for a proxy that records every random draw
  (rand / randn / rand_like), so the oracle and the GPU path can replay them;
* wraps ``NeRF.forward`` and ``sample_pdf`` to record the raw MLP outputs and
  the importance depths;
* optionally back-propagates the reference MSE loss (``losses.py:4-14``) and
  stores gradient probes (full small tensors, 512 fixed entries of big ones,
  and per-tensor sums / L2 norms).

Fixtures are written as ``tests/golden/<case>.npz`` (plain arrays, no pickle).
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("NERF_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)

from oracle.nerf_oracle import make_params  # noqa: E402
from nerf_pl_amd.rays import blender_rays, llff_ndc_rays  # noqa: E402


def import_reference():
    shim = types.ModuleType("torchsearchsorted")
    shim.searchsorted = lambda a, v, side="left", out=None: torch.searchsorted(
        a.contiguous(), v.contiguous(), right=(side == "right"))
    sys.modules["torchsearchsorted"] = shim
    sys.path.insert(0, REF)
    import models.nerf as ref_nerf          # noqa: E402
    import models.rendering as ref_rendering  # noqa: E402
    return ref_nerf, ref_rendering


class RecordingTorch:
    """Delegates to torch, recording random draws in call order."""

    def __init__(self):
        self.draws = []

    def __getattr__(self, name):
        return getattr(torch, name)

    def rand(self, *a, **k):
        t = torch.rand(*a, **k)
        self.draws.append(("rand", t.detach().clone()))
        return t

    def randn(self, *a, **k):
        t = torch.randn(*a, **k)
        self.draws.append(("randn", t.detach().clone()))
        return t

    def rand_like(self, *a, **k):
        t = torch.rand_like(*a, **k)
        self.draws.append(("rand_like", t.detach().clone()))
        return t


PROBE_PER_TENSOR = 512


def run_case(ref_nerf, ref_rendering, name, rays, N_samples, N_importance, perturb, noise_std,
             use_disp=False, white_back=False, test_time=False, chunk=32768, sigma_bias=0.0,
             grads=False, seed=1234):
    torch.manual_seed(seed)
    models = []
    params_seeds = [11, 22]
    n_models = 2 if N_importance > 0 else 1
    for m in range(n_models):
        net = ref_nerf.NeRF()
        net.load_state_dict(make_params(params_seeds[m], sigma_bias=sigma_bias))
        models.append(net)
    emb = [ref_nerf.Embedding(3, 10), ref_nerf.Embedding(3, 4)]

    raw_log = {}

    def wrap_forward(net, tag):
        orig = net.forward

        def fwd(x, sigma_only=False):
            out = orig(x, sigma_only=sigma_only)
            raw_log.setdefault(tag, []).append(out.detach().clone())
            return out
        net.forward = fwd

    wrap_forward(models[0], "raw_coarse")
    if n_models > 1:
        wrap_forward(models[1], "raw_fine")

    pdf_log = {}
    orig_sample_pdf = ref_rendering.sample_pdf

    def sample_pdf_rec(*a, **k):
        z = orig_sample_pdf(*a, **k)
        pdf_log["z_pdf"] = z.detach().clone()
        return z

    rec = RecordingTorch()
    saved_torch = ref_rendering.torch
    ref_rendering.torch = rec
    ref_rendering.sample_pdf = sample_pdf_rec
    try:
        with torch.set_grad_enabled(grads):
            res = ref_rendering.render_rays(models, emb, rays, N_samples, use_disp, perturb,
                                            noise_std, N_importance, chunk, white_back,
                                            test_time)
    finally:
        ref_rendering.torch = saved_torch
        ref_rendering.sample_pdf = orig_sample_pdf

    out = {
        "rays": rays.numpy(),
        "cfg": np.array([N_samples, N_importance, perturb, noise_std, int(use_disp),
                         int(white_back), int(test_time), chunk, sigma_bias, params_seeds[0],
                         params_seeds[1]], dtype=np.float64),
        "n_draws": np.array(len(rec.draws)),
    }
    for i, (kind, t) in enumerate(rec.draws):
        out[f"draw{i}"] = t.numpy()
        out[f"draw{i}_kind"] = np.array(kind)
    for k, v in res.items():
        out[f"out_{k}"] = v.detach().numpy()
    for k, v in raw_log.items():
        out[k] = torch.cat(v, 0).numpy()
    if "z_pdf" in pdf_log:
        out["z_pdf"] = pdf_log["z_pdf"].numpy()

    if grads:
        g = torch.Generator().manual_seed(seed + 1)
        target = torch.rand(rays.shape[0], 3, generator=g)
        loss = torch.mean((res["rgb_coarse"] - target) ** 2)
        if "rgb_fine" in res:
            loss = loss + torch.mean((res["rgb_fine"] - target) ** 2)
        loss.backward()
        out["target"] = target.numpy()
        out["loss"] = np.array(loss.item(), dtype=np.float64)
        pg = np.random.Generator(np.random.PCG64(99))
        for m, net in enumerate(models):
            for pname, p in net.named_parameters():
                gr = p.grad.detach().numpy().astype(np.float32)
                key = f"grad{m}_{pname}"
                out[key + "_sum"] = np.array(gr.astype(np.float64).sum())
                out[key + "_l2"] = np.array(np.sqrt((gr.astype(np.float64) ** 2).sum()))
                flat = gr.reshape(-1)
                if flat.size <= 1024:
                    out[key + "_full"] = gr
                else:
                    idx = np.sort(pg.choice(flat.size, PROBE_PER_TENSOR, replace=False))
                    out[key + "_idx"] = idx.astype(np.int64)
                    out[key + "_val"] = flat[idx]
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: {len(rec.draws)} draws, keys={len(out)}, "
          f"{os.path.getsize(path) / 1024:.1f} KiB")


def pick(rays, n, seed):
    g = torch.Generator().manual_seed(seed)
    idx = torch.randperm(rays.shape[0], generator=g)[:n]
    return rays[idx].contiguous()


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    ref_nerf, ref_rendering = import_reference()
    lego64_n26 = blender_rays(64, 2, near=2.0, far=6.0)
    lego64_1200 = blender_rays(64, 2, near=1.0, far=200.0)
    fern = llff_ndc_rays(504, 378, n_poses=1)

    cases = [
        # config 1: 64x64, S=32, I=0, perturb on, noise on
        dict(name="cfg1_s32", rays=pick(lego64_1200, 64, 1), N_samples=32, N_importance=0,
             perturb=1.0, noise_std=1.0),
        # config 2 shapes at reduced ray counts
        dict(name="cfg2_n26", rays=pick(lego64_n26, 48, 2), N_samples=64, N_importance=128,
             perturb=1.0, noise_std=1.0),
        dict(name="cfg2_n1200", rays=pick(lego64_1200, 48, 3), N_samples=64, N_importance=128,
             perturb=1.0, noise_std=0.0),
        dict(name="cfg2_testtime", rays=pick(lego64_n26, 32, 4), N_samples=64,
             N_importance=128, perturb=0.0, noise_std=0.0, test_time=True),
        dict(name="cfg2_whiteback", rays=pick(lego64_n26, 32, 5), N_samples=64,
             N_importance=128, perturb=1.0, noise_std=1.0, white_back=True, sigma_bias=1.0),
        # config 3: NDC forward-facing rays, near/far 0/1, non-unit directions
        dict(name="cfg3_ndc", rays=pick(fern, 48, 6), N_samples=64, N_importance=64,
             perturb=1.0, noise_std=1.0, sigma_bias=2.0),
        # disparity sampling + small chunk (chunk loop exercised)
        dict(name="disp_chunk", rays=pick(lego64_n26, 24, 7), N_samples=64, N_importance=32,
             perturb=1.0, noise_std=1.0, use_disp=True, chunk=1000),
        # ragged sizes: sample counts that are not multiples of the wave tile
        dict(name="ragged", rays=pick(lego64_n26, 37, 8), N_samples=33, N_importance=17,
             perturb=1.0, noise_std=1.0, sigma_bias=0.5),
        # gradients through the full coarse+fine pass
        dict(name="cfg2_grad", rays=pick(lego64_n26, 32, 9), N_samples=64, N_importance=128,
             perturb=1.0, noise_std=1.0, sigma_bias=0.5, grads=True),
        dict(name="cfg1_grad", rays=pick(lego64_1200, 32, 10), N_samples=32, N_importance=0,
             perturb=1.0, noise_std=1.0, grads=True),
    ]
    for c in cases:
        run_case(ref_nerf, ref_rendering, **c)


if __name__ == "__main__":
    main()
