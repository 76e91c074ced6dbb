"""pipeline.PipelinedStep (the coarse model's Adam and the next step's coarse
pass beside the fine model's backward tail) against the sequential step
(one backward, one Adam over both models): the same parameters, bit for bit,
after several training steps -- every kernel must read exactly what it reads
in the sequential schedule (train.py:103-117)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _train(pipelined, steps, n_importance=64, flush=False):
    from nerf_pl_amd import Embedding, NeRF, render_rays
    from nerf_pl_amd.losses import MSELoss
    from nerf_pl_amd.optim import FusedAdam
    from nerf_pl_amd.pipeline import PipelinedStep
    from nerf_pl_amd.rays import RaySampler, blender_focal, pose_spherical
    dev = torch.device("cuda", 0)
    W = 64
    poses = torch.stack([pose_spherical(-180.0 + 45.0 * k, -30.0, 4.0) for k in range(8)]).to(dev)
    torch.manual_seed(1234)
    pool = torch.rand(8 * W * W, 3, device=dev)
    sampler = RaySampler(poses, W, W, blender_focal(W), 1.0, 200.0, rgb_pool=pool, seed=99)
    torch.manual_seed(0)
    models = [NeRF().to(dev), NeRF().to(dev)]
    emb = [Embedding(3, 10), Embedding(3, 4)]
    loss_fn = MSELoss()
    torch.manual_seed(4321)           # the per-step draws (perturb, noise) of render_rays

    def step_loss():
        rays, rgbs = sampler.next(1024)
        res = render_rays(models, emb, rays, 64, False, 1.0, 1.0, n_importance, 32768, False, False)
        return loss_fn(res, rgbs)

    losses = []
    if pipelined:
        ps = PipelinedStep(models, lr=5e-4, eps=1e-8)
        try:
            for _ in range(steps):
                losses.append(ps(step_loss).detach())
            if flush:
                ps.flush()
        finally:
            ps.remove()
        assert ps.mains[0] is not ps.mains[1]
    else:
        opt = FusedAdam([p for m in models for p in m.parameters()], lr=5e-4, eps=1e-8)
        for _ in range(steps):
            loss = step_loss()
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            losses.append(loss.detach())
    torch.cuda.synchronize()
    return [p.detach().clone() for m in models for p in m.parameters()], torch.stack(losses)


def test_pipelined_step_matches_sequential_bitwise():
    ref, ref_loss = _train(False, 5)
    got, got_loss = _train(True, 5)
    assert torch.equal(ref_loss, got_loss), (ref_loss, got_loss)
    assert len(ref) == len(got) == 48          # 24 tensors per NeRF
    for i, (a, b) in enumerate(zip(ref, got)):
        assert torch.equal(a, b), f"parameter {i}: max |diff| {float((a - b).abs().max()):.3g}"


def test_pipelined_step_changes_parameters():
    """the comparison above is not vacuous: the parameters move"""
    from nerf_pl_amd import NeRF
    torch.manual_seed(0)
    init = [p.detach().clone() for m in (NeRF(), NeRF()) for p in m.parameters()]
    got, _ = _train(True, 2)
    assert any(not torch.equal(a.cuda(), b) for a, b in zip(init, got))


def test_pipelined_step_with_rccl_reducer_matches_sequential_bitwise():
    """the distributed path at one rank (RCCL): the coarse bucket finished on
    the next step's stream, the fine bucket and Adam deferred to the next fine
    pass (rendering.BEFORE_FINE) -- the same parameters as the plain step"""
    import socket

    import torch.distributed as dist
    from nerf_pl_amd.distributed import GradAllReducer
    from nerf_pl_amd import pipeline
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    made = []
    orig = pipeline.PipelinedStep.__init__

    def init(self, models, *a, **kw):
        red = GradAllReducer([p for m in models for p in m.parameters()],
                             buckets=[list(m.parameters()) for m in models], hook_launch=False)
        made.append(red)
        orig(self, models, *a, reducer=red, **kw)
    try:
        pipeline.PipelinedStep.__init__ = init
        got, got_loss = _train(True, 5, flush=True)
    finally:
        pipeline.PipelinedStep.__init__ = orig
        for r in made:
            r.remove()
        dist.destroy_process_group()
    ref, ref_loss = _train(False, 5)
    assert made and made[0].hook_launch is False
    assert torch.equal(ref_loss, got_loss), (ref_loss, got_loss)
    for i, (a, b) in enumerate(zip(ref, got)):
        assert torch.equal(a, b), f"parameter {i}: max |diff| {float((a - b).abs().max()):.3g}"
