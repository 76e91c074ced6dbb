"""Data-parallel training glue (the exchange steps of SURVEY.md 8e).

Rays are independent, so each rank renders its own ray batch and the only
collective is the gradient all-reduce that Lightning's DDP backend performs in
the reference (train.py:174-175): 2 x 595,844 fp32 parameters = 4.77 MB per
step.  Here it is one flat all-reduce per model (RCCL over xGMI with the
``nccl`` backend on ROCm; gloo on CPU for tests) instead of DDP's 25 MB
buckets: at 4.77 MB a ring all-reduce is latency-bound (tens of µs), so the
buckets are coarse -- one per model, the fine model's overlapped with the
coarse model's backward.
"""
from __future__ import annotations

import contextlib
import functools

import hashlib

import torch
import torch.distributed as dist


class _Bucket:
    def __init__(self, params, dev):
        self.params = params
        self.flat = torch.zeros(sum(p.numel() for p in params), dtype=torch.float32, device=dev)
        self.views, off = [], 0
        for p in params:
            self.views.append(self.flat[off:off + p.numel()].view_as(p))
            off += p.numel()
        self.seen = set()
        self.handle = None
        self.stale = False
        self.ready = False
        self.stream = None      # the stream its last gradient was accumulated on


class GradAllReducer:
    """Averages the ``.grad`` of ``params`` over the default process group.

    ``buckets`` (optional) partitions the parameters, e.g. one bucket per
    model: a bucket's all-reduce is started from a post-accumulate-grad hook
    as soon as the last of its gradients has been accumulated, so it runs on
    RCCL's stream while the rest of the backward pass is still computing.  In
    ``render_rays`` the fine model's backward completes first (autograd runs
    the later-created graph first), so its 2.38 MB all-reduce hides behind the
    coarse model's backward; only the coarse model's remains exposed.  Without
    ``buckets`` all parameters form one bucket (the all-reduce starts when the
    whole backward is done).

    Per bucket: one batched ``cat`` into a persistent flat buffer, one
    all-reduce (``AVG`` on RCCL; ``SUM`` and a scale on gloo, which has no
    average), one batched foreach copy back.  Parameters without a gradient
    are treated as zero (they contribute nothing to the sum), like DDP's
    ``find_unused_parameters`` for a fixed graph.  A gradient accumulated
    again after its bucket was launched (a model used twice, or several
    backward passes before the call) marks the bucket stale: ``__call__`` then
    reduces it again from the final gradients.  Every rank must run the same
    graph (the same buckets complete in the same order), as with DDP."""

    def __init__(self, params, group=None, buckets=None, ordered=False, hook_launch=True):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        # ordered: the buckets' all-reduces are issued in bucket order (a ready
        # bucket waits for the ones before it).  They share one RCCL stream, so
        # issue order is execution order: pipeline.PipelinedStep finishes bucket
        # 0 (the coarse model) for the next step's coarse pass, and must not find
        # it queued behind bucket 1, whose gradients (the fine model's) the host
        # reaches first but the GPU produces last.
        self.ordered = ordered
        # hook_launch=False: the hooks only note which buckets are complete and
        # the collectives are issued by __call__ / finish, after the backward has
        # been enqueued (an RCCL collective issued from inside the
        # backward held the autograd thread until its input was computed, so the
        # coarse chain was enqueued only after the fine one had finished)
        self.hook_launch = hook_launch
        dev = self.params[0].device
        if buckets is None:
            groups = [self.params]
        else:
            ids = {id(p) for p in self.params}
            groups, seen = [], set()
            for b in buckets:
                g = [p for p in b if id(p) in ids and id(p) not in seen]
                seen.update(id(p) for p in g)
                if g:
                    groups.append(g)
            rest = [p for p in self.params if id(p) not in seen]
            if rest:
                groups.append(rest)
        self.buckets = [_Bucket(g, dev) for g in groups]
        self._hooks = [p.register_post_accumulate_grad_hook(functools.partial(self._ready, b))
                       for b in self.buckets for p in b.params]

    def _nccl(self):
        return dist.get_backend(self.group) == "nccl"

    def _ready(self, b, p):
        if b.handle is not None:
            b.stale = True
            return
        b.seen.add(id(p))
        if len(b.seen) == len(b.params):
            b.ready = True
            b.stream = torch.cuda.current_stream(p.device) if p.device.type == "cuda" else None
            if not self.hook_launch:
                return
            if not self.ordered:
                self._launch(b, b.stream)
                return
            for c in self.buckets:      # every ready bucket whose predecessors are issued
                if c.handle is None:
                    if not c.ready:
                        break
                    self._launch(c, c.stream)

    def _launch(self, b, stream=None):
        # from a hook: on the stream that accumulated the bucket's last gradient
        # (a bucket issued from another bucket's hook runs there too); from
        # __call__ / finish: on the caller's current stream
        with torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext():
            for p in b.params:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
            torch.cat([p.grad.reshape(-1) for p in b.params], out=b.flat)
            op = dist.ReduceOp.AVG if self._nccl() else dist.ReduceOp.SUM
            b.handle = dist.all_reduce(b.flat, op=op, group=self.group, async_op=True)

    def _start(self, b):
        if b.handle is not None and b.stale:
            b.handle.wait()
            b.handle = None
        if b.handle is None:
            self._launch(b)

    def _complete(self, b):
        b.handle.wait()
        if not self._nccl():
            b.flat.div_(dist.get_world_size(self.group))
        torch._foreach_copy_([p.grad for p in b.params], b.views)
        b.seen.clear()
        b.handle = None
        b.stale = False
        b.ready = False
        b.stream = None

    def __call__(self):
        for b in self.buckets:
            self._start(b)
        for b in self.buckets:
            self._complete(b)

    def finish(self, i):
        """Bucket i only: its averaged gradients into its parameters' ``.grad``,
        ordered on the current stream (``pipeline.PipelinedStep`` finishes each
        model's bucket on the stream of that model's optimizer step)."""
        b = self.buckets[i]
        self._start(b)
        self._complete(b)

    def remove(self):
        """Detach the gradient hooks."""
        for h in self._hooks:
            h.remove()
        self._hooks = []


class _GatherRows(torch.autograd.Function):
    """All-gather of equal padded row slices; its backward is the matching
    reduce-scatter (sum): rank r's slice receives the sum over ranks of the
    gradient of its rows, so after the usual parameter-gradient average every
    rank holds the gradient of the mean loss, as if each had rendered every
    row itself (the reference's replicated light render under DDP)."""

    @staticmethod
    def forward(ctx, buf, world, group):
        ctx.world, ctx.group = world, group
        full = torch.empty((world * buf.shape[0],) + tuple(buf.shape[1:]), dtype=buf.dtype,
                           device=buf.device)
        dist.all_gather_into_tensor(full, buf.contiguous(), group=group)
        return full

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        per = g.shape[0] // ctx.world
        if dist.get_backend(ctx.group) == "nccl":
            out = torch.empty((per,) + tuple(g.shape[1:]), dtype=g.dtype, device=g.device)
            dist.reduce_scatter_tensor(out, g, op=dist.ReduceOp.SUM, group=ctx.group)
        else:       # gloo has no reduce-scatter: sum everything, keep the own slice
            dist.all_reduce(g, op=dist.ReduceOp.SUM, group=ctx.group)
            rank = dist.get_rank(ctx.group)
            out = g[rank * per:(rank + 1) * per].clone()
        return out, None, None


def _check_signature(part, group):
    """Every rank must gather the same keys with the same trailing shapes and
    dtypes (e.g. the same N_importance); a mismatch would pair different
    tensors in the collectives or hang.  Raises on all ranks alike."""
    sig = sorted((k, None if v is None else (tuple(v.shape[1:]), str(v.dtype)))
                 for k, v in part.items())
    # the common case costs one 16-byte all-reduce (min and max of a stable
    # 63-bit digest of the signature) instead of pickling every rank's
    # signature through all_gather_object; that runs only to report a mismatch
    h = int.from_bytes(hashlib.blake2b(repr(sig).encode(), digest_size=8).digest(), "little") >> 1
    # the device follows the backend, not the outputs (a part whose
    # values are all None must still reduce on the device NCCL needs)
    if dist.get_backend(group) == "nccl":
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    t = torch.tensor([h, -h], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    lo, neg_hi = t.tolist()
    if lo == -neg_hi:
        return
    sigs = [None] * dist.get_world_size(group)
    dist.all_gather_object(sigs, sig, group=group)
    raise RuntimeError("sharded_map: ranks produced different outputs "
                       f"(keys / trailing shapes / dtypes): {sigs}")


def sharded_map(fn, x: torch.Tensor, group=None, rank_args=None, check=True):
    """Row-sharded evaluation of ``fn`` over the ranks of ``group``: rank r
    applies ``fn`` to its contiguous slice of ``x`` (ceil(n / world) rows, the
    last slice shorter) and every rank receives the whole result, each output
    of ``fn`` (a dict of tensors with one leading row per input row) gathered
    with one all-gather per key (``all_gather_into_tensor`` on equal, padded
    slices).  ``rank_args(lo, hi)`` may supply extra keyword arguments for the
    rank's slice (e.g. a replay RNG holding the slice's random draws).

    Outputs that require grad stay differentiable: the gather's backward is a
    reduce-scatter (``_GatherRows``).  ``check`` compares the ranks' output
    signatures (one 16-byte all-reduce of a digest) on every call, before any
    output is gathered, and raises on every rank if they differ: the key set
    can change from step to step (train_efficient_sm.py:153-154 draws
    Light_N_importance per step), so a check on some calls only would let a
    divergent step pair different tensors in the gathers or hang.

    Used for config 5's light image (SURVEY 8e "phase 2"): the reference
    renders the full light image on every rank (train_efficient_sm.py:158-168);
    sharding it divides that work by the world size at the cost of gathering
    ~B floats per output (64 KB per map at 128^2) and, with --grad_on_light,
    reduce-scattering their gradients."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = x.shape[0]
    per = (n + world - 1) // world
    lo, hi = min(n, rank * per), min(n, (rank + 1) * per)
    if hi > lo:
        part = fn(x[lo:hi], **(rank_args(lo, hi) if rank_args else {}))
    else:       # an empty slice still takes part in every collective (same keys)
        part = fn(x[n - 1:n], **(rank_args(n - 1, n) if rank_args else {}))
    if check:
        # one 16-byte all-reduce and a host read of it per call: measured
        # against the light render it guards, a few tens of microseconds
        _check_signature(part, group)
    out = {}
    for k in sorted(part):
        v = part[k]
        if v is None:
            out[k] = None
            continue
        v = v[: hi - lo]
        pad = per - v.shape[0]
        if v.requires_grad and torch.is_grad_enabled():
            buf = torch.cat([v, v.new_zeros((pad,) + tuple(v.shape[1:]))]) if pad else v
            out[k] = _GatherRows.apply(buf, world, group)[:n]
            continue
        v = v.detach()
        buf = torch.zeros((per,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
        buf[: v.shape[0]] = v
        full = torch.empty((world * per,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
        dist.all_gather_into_tensor(full, buf, group=group)
        out[k] = full[:n]
    return out
