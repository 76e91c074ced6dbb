"""Config 5's light-image render sharded over ranks (SURVEY 8e "phase 2",
rendering_shadows.render_rays_sharded): two gloo ranks on the one GPU each
render half of the light rays with the matching rows of the reference's random
draws, all-gather the maps, and must reproduce the replicated render
(train_efficient_sm.py:158-168, every rank rendering every light ray) bit for
bit -- per-ray results do not depend on the other rays of a call."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import nerf_oracle as O

pytestmark = pytest.mark.gpu
S, I, N = 32, 32, 777



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

def _setup():
    from nerf_pl_amd import Embedding, NeRF
    from nerf_pl_amd.rays import blender_rays
    dev = torch.device("cuda", 0)
    models = []
    for seed in (11, 12):
        m = NeRF()
        m.load_state_dict(O.make_params(seed, sigma_bias=0.5))
        models.append(m.to(dev))
    rays = blender_rays(32, 1, near=2.0, far=6.0)[:N].contiguous()
    g = torch.Generator().manual_seed(5)
    draws = [torch.rand(N, S, generator=g), torch.randn(N, S, generator=g),
             torch.rand(N, I, generator=g), torch.rand(N, I, generator=g),
             torch.randn(N, S + I, generator=g)]
    return models, [Embedding(3, 10), Embedding(3, 4)], rays.to(dev), draws


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nerf_pl_amd import ReplayRNG
        from nerf_pl_amd import rendering_shadows as RS
        models, emb, rays, draws = _setup()
        with torch.no_grad():      # the default light render (train_efficient_sm.py:164-168)
            out = RS.render_rays_sharded(
                models, emb, rays, S, False, 1.0, 0.0, I, 32768, False,
                rng_for_rows=lambda lo, hi: ReplayRNG([d[lo:hi] for d in draws]))
        torch.cuda.synchronize()
        q.put(_to_np(((rank, {k: v.cpu() for k, v in out.items()}))))
    finally:
        dist.destroy_process_group()


def test_sharded_light_render_matches_replicated():
    from nerf_pl_amd import ReplayRNG
    from nerf_pl_amd import rendering_shadows as RS
    models, emb, rays, draws = _setup()
    with torch.no_grad():
        ref = RS.render_rays(models, emb, rays, S, False, 1.0, 0.0, I, 32768, False,
                             rng=ReplayRNG(draws))
    ref = {k: v.cpu() for k, v in ref.items()}
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [_to_t(q.get(timeout=100)) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, out in res:
        assert sorted(out) == sorted(ref)
        for k in ref:
            assert torch.equal(out[k], ref[k]), (rank, k)


def _grad_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nerf_pl_amd import ReplayRNG
        from nerf_pl_amd import rendering_shadows as RS
        from nerf_pl_amd.distributed import GradAllReducer
        models, emb, rays, draws = _setup()
        # --grad_on_light: the sharded light render keeps its graph
        out = RS.render_rays_sharded(models, emb, rays, S, False, 1.0, 0.0, I, 32768, False,
                                     rng_for_rows=lambda lo, hi: ReplayRNG([d[lo:hi] for d in draws]))
        _rank_loss(out, rank).backward()
        params = [p for m in models for p in m.parameters()]
        GradAllReducer(params)()
        torch.cuda.synchronize()
        q.put(_to_np(((rank, [p.grad.cpu() if p.grad is not None else None for p in params]))))
    finally:
        dist.destroy_process_group()


def _rank_loss(out, rank):
    # each rank's own loss on the whole light map (its camera batch, under DDP)
    g = torch.Generator().manual_seed(100 + rank)
    loss = 0
    for k in ("depth_coarse", "depth_fine"):
        c = torch.randn(out[k].shape, generator=g).to(out[k].device)
        loss = loss + (out[k] * c).sum()
    return loss


def test_sharded_light_render_gradients_match_replicated():
    """--grad_on_light with the light image sharded over 2 ranks: after the
    gather's reduce-scatter backward and the parameter all-reduce, every rank
    holds the mean over ranks of the gradient each would get rendering the
    whole light image itself (the reference under DDP)."""
    from nerf_pl_amd import ReplayRNG
    from nerf_pl_amd import rendering_shadows as RS
    world = 2
    models, emb, rays, draws = _setup()
    params = [p for m in models for p in m.parameters()]
    ref = [torch.zeros_like(p) for p in params]
    for r in range(world):
        for p in params:
            p.grad = None
        out = RS.render_rays(models, emb, rays, S, False, 1.0, 0.0, I, 32768, False,
                             rng=ReplayRNG(draws))
        _rank_loss(out, r).backward()
        for acc, p in zip(ref, params):
            if p.grad is not None:
                acc += p.grad / world
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_grad_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [_to_t(q.get(timeout=100)) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, grads in res:
        for (name, _), g, e in zip([(n, p) for m in models for n, p in m.named_parameters()],
                                   grads, ref):
            e = e.cpu()
            g = torch.zeros_like(e) if g is None else g
            scale = e.abs().max().item() + 1e-30
            torch.testing.assert_close(g, e, rtol=1e-4, atol=1e-5 * scale,
                                       msg=lambda m: f"rank {rank} {name}: {m}")
