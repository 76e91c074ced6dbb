"""Data-parallel training glue (the exchange step of SURVEY.md 8e).

Rays are independent, so each rank renders its own ray batch and the only
collective is the gradient all-reduce that Lightning's DDP backend performs in
the reference (train.py:174-175): 2 x 595,844 fp32 parameters = 4.77 MB per
step.  Here it is ONE flat all-reduce (RCCL over xGMI with the ``nccl``
backend on ROCm; gloo on CPU for tests) instead of DDP's per-bucket hooks --
at 4.77 MB a single ring all-reduce is already latency-bound (tens of µs).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class GradAllReducer:
    """Averages the ``.grad`` of ``params`` over the default process group.

    Gradients are packed into one persistent flat buffer, all-reduced once and
    scattered back.  Parameters without a gradient on every rank are treated as
    zero (they contribute nothing to the sum), matching DDP's
    ``find_unused_parameters`` behaviour for a fixed graph."""

    def __init__(self, params, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)

    def __call__(self):
        world = dist.get_world_size(self.group)
        off = 0
        for p in self.params:
            k = p.numel()
            if p.grad is None:
                self.flat[off:off + k].zero_()
            else:
                self.flat[off:off + k].copy_(p.grad.reshape(-1))
            off += k
        dist.all_reduce(self.flat, group=self.group)
        self.flat.div_(world)
        off = 0
        for p in self.params:
            k = p.numel()
            g = self.flat[off:off + k].view_as(p)
            if p.grad is None:
                p.grad = g.clone()
            else:
                p.grad.copy_(g)
            off += k
