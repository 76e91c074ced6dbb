"""FusedAdam (nr_adam_step) against torch.optim.Adam (single-tensor, CPU) on
the NeRF parameter shapes: 6 steps, weight decay on and off, a parameter
without gradient skipped.  The arithmetic is torch's single-tensor Adam op
for op, but torch's vectorised CPU kernels fuse some multiply-adds (lerp,
add with alpha), so the two drift by ulps -- and where g + wd*p cancels, Adam's
normalisation m / sqrt(v) turns that ulp into a visible fraction of one step.
Tolerance: parameters within 4 ulps of max(1,|p|) plus 2% of one step (lr);
moments within 1e-5 of the tensor's max."""
import pytest
import torch

from oracle import nerf_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("wd", [0.0, 1e-2])
def test_fused_adam_matches_torch(wd):
    from nerf_pl_amd.optim import FusedAdam
    shapes = list(O.param_shapes().values()) * 2            # the NeRF pair: 44 tensors
    g = torch.Generator().manual_seed(0)
    ref = [torch.randn(s, generator=g).requires_grad_(True) for s in shapes]
    ours = [torch.nn.Parameter(r.detach().clone().to(DEV)) for r in ref]
    o_ref = torch.optim.Adam(ref, lr=5e-4, eps=1e-8, weight_decay=wd, foreach=False)
    o_our = FusedAdam(ours, lr=5e-4, eps=1e-8, weight_decay=wd)
    for step in range(6):
        for k, (r, q) in enumerate(zip(ref, ours)):
            if k == 5 and step < 3:           # no gradient: skipped by both
                r.grad, q.grad = None, None
                continue
            gr = torch.randn(r.shape, generator=g) * (10 ** (k % 4 - 2))
            r.grad, q.grad = gr, gr.to(DEV)
        o_ref.step()
        o_our.step()
    worst = 0.0
    for r, q in zip(ref, ours):
        excess = (q.detach().cpu() - r.detach()).abs() - 4 * 2 ** -23 * r.detach().abs().clamp_min(1.0)
        worst = max(worst, excess.max().item())
    print("max param diff beyond 4 ulps, in units of lr:", worst / 5e-4)
    assert worst <= 0.02 * 5e-4
    for r, q in zip(ref, ours):
        for key in ("exp_avg", "exp_avg_sq"):
            a, b = o_our.state[q][key].cpu(), o_ref.state[r][key]
            assert (a - b).abs().max() <= 1e-5 * b.abs().max()
    st_r, st_o = o_ref.state[ref[0]], o_our.state[ours[0]]
    assert float(st_r["step"]) == float(st_o["step"]) == 6.0
    assert float(o_our.state[ours[5]]["step"]) == 3.0
    torch.testing.assert_close(st_o["exp_avg_sq"].cpu(), st_r["exp_avg_sq"], rtol=1e-6, atol=0)
