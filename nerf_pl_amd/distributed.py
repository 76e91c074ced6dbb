"""Data-parallel training glue (the exchange steps of SURVEY.md 8e).

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

    Gradients are gathered into one persistent flat buffer (one batched
    ``cat`` launch), all-reduced once (``AVG`` on RCCL; ``SUM`` and a scale on
    gloo, which has no average) and scattered back with one batched foreach
    copy -- a handful of launches per step instead of two per tensor.
    Parameters without a gradient on every rank are treated as zero (they
    contribute nothing to the sum), matching DDP's ``find_unused_parameters``
    behaviour for a fixed graph."""

    def __init__(self, params, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.views = []
        off = 0
        for p in self.params:
            self.views.append(self.flat[off:off + p.numel()].view_as(p))
            off += p.numel()

    def __call__(self):
        world = dist.get_world_size(self.group)
        for p in self.params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        grads = [p.grad for p in self.params]
        torch.cat([g.reshape(-1) for g in grads], out=self.flat)
        if dist.get_backend(self.group) == "nccl":
            dist.all_reduce(self.flat, op=dist.ReduceOp.AVG, group=self.group)
        else:
            dist.all_reduce(self.flat, group=self.group)
            self.flat.div_(world)
        torch._foreach_copy_(grads, self.views)


def sharded_map(fn, x: torch.Tensor, group=None, rank_args=None):
    """Row-sharded evaluation of ``fn`` over the ranks of ``group``: rank r
    applies ``fn`` to its contiguous slice of ``x`` (ceil(n / world) rows, the
    last slice shorter) and every rank receives the whole result, each output
    of ``fn`` (a dict of tensors with one leading row per input row) gathered
    with one all-gather per key (``all_gather_into_tensor`` on equal, padded
    slices).  ``rank_args(lo, hi)`` may supply extra keyword arguments for the
    rank's slice (e.g. a replay RNG holding the slice's random draws).

    Used for config 5's light image (SURVEY 8e "phase 2"): the reference
    renders the full light image on every rank (train_efficient_sm.py:158-168);
    sharding it divides that work by the world size at the cost of gathering
    ~B floats per output (64 KB per map at 128^2)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = x.shape[0]
    per = (n + world - 1) // world
    lo, hi = min(n, rank * per), min(n, (rank + 1) * per)
    if hi > lo:
        part = fn(x[lo:hi], **(rank_args(lo, hi) if rank_args else {}))
    else:       # an empty slice still takes part in every collective (same keys)
        part = fn(x[n - 1:n], **(rank_args(n - 1, n) if rank_args else {}))
    out = {}
    for k in sorted(part):
        v = part[k]
        if v is None:
            out[k] = None
            continue
        v = v.detach()[: hi - lo]
        buf = torch.zeros((per,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
        buf[: v.shape[0]] = v
        full = torch.empty((world * per,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
        dist.all_gather_into_tensor(full, buf, group=group)
        out[k] = full[:n]
    return out
