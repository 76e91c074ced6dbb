"""Multi-process (world_size 2, gloo, CPU) check of the data-parallel exchange:
after GradAllReducer every rank holds the mean gradient, identical to what a
single process computes on the union of the ranks' batches (the property
SURVEY.md 4 asks for: k ranks reproduce the 1-rank averaged gradient)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp



def _to_np(x):
    """tensors -> numpy for the result queue: a tensor put on a multiprocessing
    queue is shared through a file descriptor that vanishes when the worker
    exits first (a race); numpy arrays are pickled by value"""
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    if isinstance(x, (list, tuple)):
        return type(x)(_to_np(v) for v in x)
    if isinstance(x, dict):
        return {k: _to_np(v) for k, v in x.items()}
    return x


def _to_t(x):
    import numpy as np
    if isinstance(x, np.ndarray):
        return torch.from_numpy(x)
    if isinstance(x, (list, tuple)):
        return type(x)(_to_t(v) for v in x)
    if isinstance(x, dict):
        return {k: _to_t(v) for k, v in x.items()}
    return x

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nerf_pl_amd.distributed import GradAllReducer
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.ReLU(), torch.nn.Linear(7, 3))
        unused = torch.nn.Parameter(torch.ones(2))           # never gets a gradient
        g = torch.Generator().manual_seed(100)
        x_all = torch.randn(8, 5, generator=g)
        y_all = torch.randn(8, 3, generator=g)
        x, y = x_all[rank::world], y_all[rank::world]
        loss = ((model(x) - y) ** 2).mean()
        loss.backward()
        red = GradAllReducer(list(model.parameters()) + [unused])
        red()
        q.put(_to_np(((rank, [p.grad.clone() for p in model.parameters()], unused.grad.clone()))))
    finally:
        dist.destroy_process_group()


import pytest


@pytest.mark.parametrize("world", [2, 8])
def test_grad_allreduce_matches_single_process(world):
    """world 8: the rank count of the driver's 8-GPU run (cfg4), one sample per
    rank, over gloo on the CPU"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [_to_t(q.get(timeout=120)) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference: mean of per-rank mean-losses == average of grads
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.ReLU(), torch.nn.Linear(7, 3))
    g = torch.Generator().manual_seed(100)
    x_all = torch.randn(8, 5, generator=g)
    y_all = torch.randn(8, 3, generator=g)
    loss = sum(((model(x_all[r::world]) - y_all[r::world]) ** 2).mean() for r in range(world)) / world
    loss.backward()
    ref = [p.grad for p in model.parameters()]
    for rank, grads, ug in res:
        for a, b in zip(grads, ref):
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)
        assert torch.all(ug == 0)


def _bucket_worker(rank, world, port, q, per_bucket=False):
    """two models in separate buckets, reducer built before backward (the
    buckets launch from the gradient hooks); model b is used twice in the loss
    and a second backward accumulates before the call (stale buckets).
    per_bucket: each bucket finished on its own (GradAllReducer.finish, as
    pipeline.PipelinedStep does), the coarse (first) bucket first, the
    all-reduces issued in bucket order (ordered=True)"""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nerf_pl_amd.distributed import GradAllReducer
        ma, mb, x_all, y_all = _two_models()
        red = GradAllReducer(list(ma.parameters()) + list(mb.parameters()),
                             buckets=[list(ma.parameters()), list(mb.parameters())],
                             ordered=per_bucket)
        x, y = x_all[rank::world], y_all[rank::world]
        out = []
        for it in range(2):
            for m in (ma, mb):
                m.zero_grad(set_to_none=True)
            for _ in range(1 + it):          # it 1: two backward passes accumulate
                _two_model_loss(ma, mb, x, y).backward()
            if per_bucket:
                red.finish(0)
                red.finish(1)
            else:
                red()
            # numpy: pickled by value (tensors would be shared through file
            # descriptors that die with this process)
            out.append([p.grad.numpy().copy() for p in list(ma.parameters()) + list(mb.parameters())])
        q.put(_to_np(((rank, out))))
    finally:
        dist.destroy_process_group()


def _two_models():
    torch.manual_seed(1)
    ma = torch.nn.Sequential(torch.nn.Linear(5, 6), torch.nn.ReLU(), torch.nn.Linear(6, 3))
    mb = torch.nn.Linear(5, 3)
    g = torch.Generator().manual_seed(7)
    return ma, mb, torch.randn(8, 5, generator=g), torch.randn(8, 3, generator=g)


def _two_model_loss(ma, mb, x, y):
    return ((ma(x) - y) ** 2).mean() + ((mb(x) + mb(2 * x) - y) ** 2).mean()


@pytest.mark.parametrize("per_bucket", [False, True])
def test_bucketed_allreduce_overlapped_from_hooks(per_bucket):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, q, per_bucket))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [_to_t(q.get(timeout=120)) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ma, mb, x_all, y_all = _two_models()
    for it in range(2):
        for m in (ma, mb):
            m.zero_grad(set_to_none=True)
        loss = sum(_two_model_loss(ma, mb, x_all[r::world], y_all[r::world])
                   for r in range(world)) / world * (1 + it)
        loss.backward()
        ref = [p.grad for p in list(ma.parameters()) + list(mb.parameters())]
        for rank, out in res:
            for a, b in zip(out[it], ref):
                torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)


def _shard_worker(rank, world, port, q, n):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nerf_pl_amd.distributed import sharded_map
        x = torch.arange(n * 3, dtype=torch.float32).view(n, 3)
        seen = []

        def fn(xs, tag=None):
            seen.append((xs.shape[0], tag))
            return {"sum": xs.sum(1), "twice": 2 * xs, "none": None}
        out = sharded_map(fn, x, rank_args=lambda lo, hi: {"tag": (lo, hi)})
        q.put(_to_np(((rank, out["sum"], out["twice"], out["none"], seen))))
    finally:
        dist.destroy_process_group()


def test_sharded_map_gathers_every_row():
    """distributed.sharded_map (config 5's sharded light render):
    every rank gets all n rows of every output, each row computed once by the
    rank owning it (uneven split, and a world larger than the remainder)."""
    for world, n in ((2, 7), (3, 2)):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q, n)) for r in range(world)]
        for p in procs:
            p.start()
        res = [_to_t(q.get(timeout=120)) for _ in range(world)]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        x = torch.arange(n * 3, dtype=torch.float32).view(n, 3)
        per = (n + world - 1) // world
        for rank, s, t, none, seen in res:
            torch.testing.assert_close(s, x.sum(1), rtol=0, atol=0)
            torch.testing.assert_close(t, 2 * x, rtol=0, atol=0)
            assert none is None
            lo, hi = min(n, rank * per), min(n, (rank + 1) * per)
            assert seen == [(hi - lo, (lo, hi))] if hi > lo else seen == [(1, (n - 1, n))]


def _shard_grad_worker(rank, world, port, q, n, mismatch):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nerf_pl_amd.distributed import sharded_map
        w = torch.nn.Parameter(torch.linspace(0.5, 1.5, 3))
        x = torch.arange(n * 3, dtype=torch.float32).view(n, 3)

        def fn(xs):
            out = {"y": (xs * w).sum(1)}
            if mismatch and rank == 1:
                out["extra"] = xs[:, 0]
            return out
        try:
            out = sharded_map(fn, x)
        except RuntimeError as e:
            q.put(_to_np(((rank, "raised", str(e)))))
            return
        # rank-dependent loss on the gathered rows (each rank's own camera batch)
        coef = torch.arange(n, dtype=torch.float32) * (rank + 1)
        (out["y"] * coef).sum().backward()
        q.put(_to_np(((rank, "ok", w.grad.clone()))))
    finally:
        dist.destroy_process_group()


def _run(world, target, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((_to_t(q.get(timeout=120)) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,n", [(2, 7), (8, 7), (8, 29)])
def test_sharded_map_backward_reduce_scatters(world, n):
    """--grad_on_light with the light image sharded: the gathered rows stay
    differentiable, and each rank's parameter gradient is what it gets from the
    rows it rendered under every rank's loss -- so the all-reduced average
    equals the reference's (every rank renders every row, DDP averages).
    (8, 7): a rank with no rows of its own."""
    res = _run(world, _shard_grad_worker, n, False)
    x = torch.arange(n * 3, dtype=torch.float32).view(n, 3)
    per = (n + world - 1) // world
    coef_sum = torch.arange(n, dtype=torch.float32) * sum(r + 1 for r in range(world))
    total = torch.zeros(3)
    for rank, status, g in res:
        assert status == "ok"
        lo, hi = min(n, rank * per), min(n, (rank + 1) * per)
        exp = (coef_sum[lo:hi, None] * x[lo:hi]).sum(0)
        torch.testing.assert_close(g, exp, rtol=1e-6, atol=1e-6)
        total += g
    # average over ranks == mean over ranks of the replicated per-rank gradients
    rep = [(torch.arange(n, dtype=torch.float32)[:, None] * (r + 1) * x).sum(0)
           for r in range(world)]
    torch.testing.assert_close(total / world, sum(rep) / world, rtol=1e-6, atol=1e-6)


def test_sharded_map_rejects_mismatched_outputs():
    """ranks drawing different N_importance (train_efficient_sm.py
    Light_N_importance == -1) produce different keys; sharded_map raises on
    every rank instead of pairing the wrong tensors or hanging."""
    res = _run(2, _shard_grad_worker, 5, True)
    for rank, status, msg in res:
        assert status == "raised" and "different outputs" in msg, (rank, status, msg)


def _check_schedule_worker(rank, world, port, q, calls, diverge_at):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nerf_pl_amd import distributed as D
        x = torch.arange(12, dtype=torch.float32).view(4, 3)
        out = None
        for c in range(1, calls + 1):
            def fn(xs, c=c):
                r = {"s": xs.sum(1)}
                if c == diverge_at and rank == 1:     # this rank drew a different N_importance
                    r["extra"] = xs
                return r
            try:
                out = D.sharded_map(fn, x)
            except RuntimeError as e:
                q.put(_to_np((rank, "raised", c, str(e))))
                return
        q.put(_to_np((rank, "ok", calls, out["s"])))
    finally:
        dist.destroy_process_group()


def test_sharded_map_checks_signatures_on_every_call():
    """the key set may change between steps (a per-step
    Light_N_importance draw), so the signature is compared on every call:
    ranks that diverge at call 3 -- not a power of two -- raise there, on
    every rank, before any gather pairs different tensors"""
    res = _run(2, _check_schedule_worker, 6, 3)
    for rank, status, c, msg in res:
        assert status == "raised" and c == 3 and "different outputs" in msg, (rank, status, c)
    res = _run(2, _check_schedule_worker, 5, -1)
    for rank, status, c, s in res:
        assert status == "ok" and c == 5
        torch.testing.assert_close(s, torch.arange(12, dtype=torch.float32).view(4, 3).sum(1))


def _sampler_worker(rank, world, port, q, total, batch, steps):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nerf_pl_amd.rays import RaySampler
        # CPU poses: only the index partitioning is exercised (no ray generation)
        s = RaySampler(torch.zeros(total, 3, 4), 1, 1, 1.0, 2.0, 6.0, seed=7, rank=rank,
                       world=world)
        q.put(_to_np(((rank, [s.next_indices(batch).clone() for _ in range(steps)], s.epoch))))
    finally:
        dist.destroy_process_group()


def test_ray_sampler_partitions_epochs_like_distributed_sampler():
    """SURVEY 8e / train.py:89-94 under DDP: one permutation per epoch shared by
    every rank, rank r taking perm[r::world] -- the ranks' batches are
    disjoint within an epoch and together cover it; the next epoch reshuffles."""
    world, total, batch = 2, 96, 12
    steps = total // world // batch          # one epoch
    res = _run(world, _sampler_worker, total, batch, steps + 1)
    ep = []
    for rank, batches, epoch in res:
        assert epoch == 1
        ep.append(torch.cat(batches[:steps]))
        assert all(b.shape == (batch,) for b in batches)
    a, b = ep
    assert not set(a.tolist()) & set(b.tolist())                 # disjoint
    assert sorted(a.tolist() + b.tolist()) == list(range(total))  # cover the epoch
    # identical to torch.utils.data.DistributedSampler's partition of the epoch
    g = torch.Generator().manual_seed(7)
    perm = torch.randperm(total, generator=g)
    for rank, e in enumerate(ep):
        torch.testing.assert_close(e, perm[rank::world], rtol=0, atol=0)
    # the second epoch is a different permutation
    assert not torch.equal(res[0][1][steps], res[0][1][0])


def test_ray_sampler_matches_distributed_sampler_at_eight_ranks():
    """the 8-rank partition of an epoch whose size the world does not divide
    (padded with the permutation's head, DistributedSampler(drop_last=False)),
    over two epochs, against torch.utils.data.DistributedSampler itself"""
    from torch.utils.data import DistributedSampler
    world, total, batch = 8, 100, 13            # 100 % 8 = 4 -> 4 padded indices
    steps = 1                                   # ceil(100 / 8) = 13 per rank per epoch
    res = _run(world, _sampler_worker, total, batch, 2 * steps)
    for rank, batches, epoch in res:
        assert epoch == 1
        for e in range(2):
            ds = DistributedSampler(range(total), num_replicas=world, rank=rank, shuffle=True,
                                    seed=7, drop_last=False)
            ds.set_epoch(e)
            assert batches[e].tolist() == list(ds), (rank, e)
