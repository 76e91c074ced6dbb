"""The data-parallel training step on the device: two gloo ranks
sharing the one GPU each render half of a ray batch through the HIP path,
back-propagate their own MSE (train.py:103-117) and average the gradient with
``GradAllReducer`` in per-model buckets launched from the gradient hooks (the
fine model's all-reduce overlapping the coarse model's backward).  Every rank
must end with the gradient one process computes for the mean of the two
ranks' losses (k ranks reproduce the 1-rank averaged gradient), up to fp32
summation order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import nerf_oracle as O

pytestmark = pytest.mark.gpu
S, I, N = 32, 32, 600


def _setup():
    from nerf_pl_amd import Embedding, NeRF
    from nerf_pl_amd.rays import blender_rays
    dev = torch.device("cuda", 0)
    models = []
    for seed in (21, 22):
        m = NeRF()
        m.load_state_dict(O.make_params(seed, sigma_bias=0.5))
        models.append(m.to(dev))
    rays = blender_rays(32, 1, near=2.0, far=6.0)[:N].contiguous()
    g = torch.Generator().manual_seed(8)
    draws = [torch.rand(N, S, generator=g), torch.randn(N, S, generator=g),
             torch.rand(N, I, generator=g), torch.rand(N, I, generator=g),
             torch.randn(N, S + I, generator=g)]
    target = 0.5 + 0.4 * torch.sin(3 * rays[:, 3:6])
    return models, [Embedding(3, 10), Embedding(3, 4)], rays.to(dev), draws, target.to(dev)


def _loss(models, emb, rays, draws, target, lo, hi):
    from nerf_pl_amd import ReplayRNG, render_rays
    res = render_rays(models, emb, rays[lo:hi].contiguous(), S, False, 1.0, 1.0, I, 32768, False,
                      rng=ReplayRNG([d[lo:hi] for d in draws]))
    t = target[lo:hi]
    return torch.mean((res["rgb_coarse"] - t) ** 2) + torch.mean((res["rgb_fine"] - t) ** 2)


def _worker(rank, world, port, q, backend="gloo"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nerf_pl_amd.distributed import GradAllReducer
        models, emb, rays, draws, target = _setup()
        params = [p for m in models for p in m.parameters()]
        red = GradAllReducer(params, buckets=[list(m.parameters()) for m in models])
        dist.barrier()          # communicator set up on the main thread (bench.py does the same)
        per = N // world
        _loss(models, emb, rays, draws, target, rank * per, (rank + 1) * per).backward()
        red()
        torch.cuda.synchronize()
        q.put((rank, [p.grad.cpu().numpy() for p in params]))
    finally:
        dist.destroy_process_group()


def test_two_rank_gradient_equals_single_process():
    models, emb, rays, draws, target = _setup()
    world = 2
    per = N // world
    loss = sum(_loss(models, emb, rays, draws, target, r * per, (r + 1) * per)
               for r in range(world)) / world
    loss.backward()
    ref = [p.grad.cpu().numpy() for m in models for p in m.parameters()]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, grads in res:
        assert len(grads) == len(ref)
        for a, b in zip(grads, ref):
            scale = np.abs(b).max() + 1e-30
            assert np.abs(a - b).max() <= 1e-5 * scale, (rank, np.abs(a - b).max() / scale)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_rccl_one_rank_step_is_the_local_step():
    """The RCCL (``nccl`` backend) path of the exchange on real hardware: one
    rank, its gradient all-reduces (``ReduceOp.AVG``) launched from the
    gradient hooks on autograd's thread, waited for before the optimizer
    step.  Averaging over one rank is the identity, and the kernels are
    deterministic, so the reduced gradient equals the local one bit for bit.
    (RCCL refuses two ranks on one GPU; the two-rank exchange is
    test_two_rank_gradient_equals_single_process, over gloo.)"""
    models, emb, rays, draws, target = _setup()
    _loss(models, emb, rays, draws, target, 0, N).backward()
    ref = [p.grad.cpu().numpy() for m in models for p in m.parameters()]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    proc = ctx.Process(target=_worker, args=(0, 1, _free_port(), q, "nccl"))
    proc.start()
    rank, grads = q.get(timeout=100)
    proc.join(timeout=60)
    assert proc.exitcode == 0
    assert len(grads) == len(ref)
    for a, b in zip(grads, ref):
        assert np.array_equal(a, b)
