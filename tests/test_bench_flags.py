"""bench.py mirrors the hot-path flags of opt.py:18-37 (--perturb, --noise-std,
--lr, --chunk, --use-disp, --white-back) and hands them to render_rays the way
NeRFSystem.forward does (train.py:49-71: one render_rays call per chunk of
rays, results concatenated).  CPU only: the render function is a recorder."""
import ast
import os
import sys

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _parse(monkeypatch, *argv):
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py", *argv])
    return bench.parse()


@pytest.mark.parametrize("config,perturb,noise", [("cfg2", 1.0, 1.0), ("cfg3", 1.0, 1.0),
                                                  ("cfg4", 1.0, 1.0), ("cfg5", 1.0, 0.0),
                                                  ("eval", 0.0, 0.0)])
def test_workload_defaults(monkeypatch, config, perturb, noise):
    a = _parse(monkeypatch, "--config", config, "--steps", "9", "--warmup", "4")
    assert (a.perturb, a.noise_std) == (perturb, noise)
    assert a.lr == 5e-4 and a.chunk == 32 * 1024 and not a.use_disp and not a.white_back
    assert a.fp32_leg_steps == 9          # the exact-fp32 leg times as many steps as the main region


def test_flags_reach_render_rays(monkeypatch):
    import bench
    a = _parse(monkeypatch, "--config", "cfg2", "--perturb", "0", "--noise-std", "0",
               "--use-disp", "--white-back", "--chunk", "3", "--lr", "1e-3",
               "--fp32-leg-steps", "0")
    assert a.lr == 1e-3 and a.fp32_leg_steps == 0
    calls = []

    def render(models, emb, rays, S, use_disp, perturb, noise_std, I, chunk, white_back,
               test_time, **kw):
        calls.append(dict(n=rays.shape[0], S=S, use_disp=use_disp, perturb=perturb,
                          noise_std=noise_std, I=I, chunk=chunk, white_back=white_back,
                          test_time=test_time, kw=kw))
        return {"rgb_fine": rays[:, :3] * 2, "depth_fine": rays[:, 0]}

    rays = torch.arange(8 * 8, dtype=torch.float32).reshape(8, 8)
    out = bench.render_chunked(render, ["m"], ["e"], rays, a, 64, 128, extra=1)
    assert [c["n"] for c in calls] == [3, 3, 2]           # chunks of --chunk rays, in order
    for c in calls:
        assert c == dict(n=c["n"], S=64, use_disp=True, perturb=0.0, noise_std=0.0, I=128,
                         chunk=3, white_back=True, test_time=False, kw={"extra": 1})
    torch.testing.assert_close(out["rgb_fine"], rays[:, :3] * 2, rtol=0, atol=0)
    torch.testing.assert_close(out["depth_fine"], rays[:, 0], rtol=0, atol=0)
    assert "perturb=0, noise_std=0, use_disp, white_back, chunk=3" == bench.hyper(a)


def test_one_call_when_the_batch_fits_a_chunk(monkeypatch):
    import bench
    a = _parse(monkeypatch)
    calls = []
    out = bench.render_chunked(lambda *r, **k: calls.append(r) or {"x": r[2]}, [], [],
                               torch.zeros(4096, 8), a, 64, 128)
    assert len(calls) == 1 and out["x"].shape == (4096, 8)
    assert calls[0][3:11] == (64, False, 1.0, 1.0, 128, 32768, False, False)


def test_bench_workloads_call_render_through_the_flags():
    """No render_rays call in bench.py hard-codes the hyperparameters: each
    goes through render_chunked (or passes args.*)."""
    src = open(os.path.join(REPO, "bench.py")).read()
    for node in ast.walk(ast.parse(src)):
        if isinstance(node, ast.Call):
            f = node.func
            name = f.attr if isinstance(f, ast.Attribute) else getattr(f, "id", "")
            if name in ("render_rays", "render_rays_sharded") and len(node.args) >= 6:
                lits = [a for a in node.args[3:7] if isinstance(a, ast.Constant)]
                assert not lits, f"bench.py:{node.lineno} passes literal hyperparameters"


def test_vet_refuses_torch_io():
    """tests/golden/make_golden_rays.py vets the reference's get_rays source
    before executing it: only the torch functions those bodies use pass."""
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import make_golden_rays as M
    for body in ("torch.load(x)", "torch.save(x, x)", "torch.compile(x)", "x.__class__"):
        fn = ast.parse(f"def f(x):\n    return {body}\n").body[0]
        with pytest.raises(AssertionError):
            M._vet([fn])
    ok = ast.parse("def f(x):\n    return torch.stack([x, torch.ones_like(x)], -1)\n").body[0]
    M._vet([ok])
