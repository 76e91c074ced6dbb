"""Fused Adam -- a drop-in for the ``torch.optim.Adam``
that the reference builds in ``utils/__init__.py:10-30`` (lr 5e-4, eps 1e-8,
weight_decay from opt.py).

``FusedAdam.step()`` updates every parameter tensor that has a gradient in
ONE ``nr_adam_step`` launch (up to ``nr_adam_max_tensors()`` tensors per
launch; the NeRF pair has 48), with torch's single-tensor Adam arithmetic.
Parameters without a gradient are skipped, like torch.  State keys
(``step``, ``exp_avg``, ``exp_avg_sq``) match torch's, so state dicts move
between the two optimizers.
"""
from __future__ import annotations

import ctypes

import torch

from ._lib import call, lib, stream_of

__all__ = ["FusedAdam"]


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 amsgrad=False):
        if amsgrad:
            raise NotImplementedError("nerf_pl_amd.FusedAdam: amsgrad is not supported")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        cap = int(lib().nr_adam_max_tensors())
        for group in self.param_groups:
            b1, b2 = group["betas"]
            batches = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse or p.dtype != torch.float32 or p.device.type != "cuda":
                    raise RuntimeError("nerf_pl_amd.FusedAdam: dense fp32 HIP-device "
                                       "parameters only")
                st = self.state[p]
                if not st:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                if not p.is_contiguous():
                    raise RuntimeError("nerf_pl_amd.FusedAdam: parameters must be contiguous")
                key = (int(st["step"].item()), p.device)
                batches.setdefault(key, []).append((p, g, st["exp_avg"], st["exp_avg_sq"]))
            for (step, dev), items in batches.items():
                for i in range(0, len(items), cap):
                    chunk = items[i:i + cap]
                    k = len(chunk)
                    arr = lambda xs: (ctypes.c_void_p * k)(*[x.data_ptr() for x in xs])  # noqa: E731
                    numel = (ctypes.c_int64 * k)(*[c[0].numel() for c in chunk])
                    call("nr_adam_step", arr([c[0] for c in chunk]), arr([c[1] for c in chunk]),
                         arr([c[2] for c in chunk]), arr([c[3] for c in chunk]), numel, k,
                         float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                         float(group["weight_decay"]), step, stream_of(dev))
                # the kernel wrote through raw pointers: bump the version
                # counters like torch's in-place Adam does, so autograd sees
                # the modification and NeRF.packed() re-packs the new weights
                torch.autograd.graph.increment_version([c[0] for c in items])
        return loss
