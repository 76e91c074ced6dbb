"""The fused training loss (nerf_pl_amd.losses, nr_mse_loss / nr_mse_loss_bwd)
against the reference's losses.py:4-27 / metrics.py:4-13 run by torch on the
same device tensors.

* forward: each term is the correctly rounded mean of the fp32 squares (the
  kernel sums in double); torch's fp32 reduction differs from it by
  reduction-order ulps, so torch is held to 1e-6 relative and the exact value
  to equality;
* backward: bit-identical to torch's mse_loss_backward ((2/n) * (x - t) * g)
  for both inputs, including a non-unit upstream gradient."""
import numpy as np
import pytest
import torch
from torch import nn

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _ref_loss(inputs, targets, key="rgb"):
    """losses.py:4-14 verbatim in behaviour"""
    loss_f = nn.MSELoss(reduction="mean")
    loss = loss_f(inputs[f"{key}_coarse"], targets)
    if f"{key}_fine" in inputs:
        loss += loss_f(inputs[f"{key}_fine"], targets)
    return loss


def _exact_mean(x, t):
    d = x.detach().cpu().numpy() - t.detach().cpu().numpy()      # fp32 ops, as the kernel
    return np.float32(np.mean((d * d).astype(np.float64)))


@pytest.mark.parametrize("n,fine", [(4096, True), (1, True), (777, False), (65536, True)])
def test_mse_loss_matches_reference(n, fine):
    from nerf_pl_amd.losses import MSELoss
    g = torch.Generator().manual_seed(n)
    t = torch.rand(n, 3, generator=g).to(DEV)
    inp = {"rgb_coarse": torch.rand(n, 3, generator=g).to(DEV).requires_grad_()}
    if fine:
        inp["rgb_fine"] = torch.rand(n, 3, generator=g).to(DEV).requires_grad_()
    ref_in = {k: v.detach().clone().requires_grad_() for k, v in inp.items()}
    crit = MSELoss()
    ours = crit(inp, t)
    ref = _ref_loss(ref_in, t)
    assert ours.shape == ref.shape == ()
    mc = _exact_mean(inp["rgb_coarse"], t)
    mf = _exact_mean(inp["rgb_fine"], t) if fine else np.float32(0)
    assert crit.last[0].item() == mc and crit.last[1].item() == mf
    assert ours.item() == (np.float32(mc + mf) if fine else mc)
    assert abs(ours.item() - ref.item()) <= 1e-6 * abs(ref.item())
    for scale in (1.0, 0.37):
        for v in list(inp.values()) + list(ref_in.values()):
            v.grad = None
        (ours * scale).backward(retain_graph=True)
        (ref * scale).backward(retain_graph=True)
        for k in inp:
            assert torch.equal(inp[k].grad, ref_in[k].grad), (k, scale)


def test_sm_loss_and_psnr():
    from nerf_pl_amd.losses import loss_dict, psnr
    g = torch.Generator().manual_seed(3)
    t = torch.rand(500, 3, generator=g).to(DEV)
    inp = {"sm_coarse": torch.rand(500, 3, generator=g).to(DEV),
           "sm_fine": torch.rand(500, 3, generator=g).to(DEV)}
    assert abs(loss_dict["sm"]()(inp, t).item() - _ref_loss(inp, t, "sm").item()) <= 1e-6
    p = psnr(inp["sm_fine"], t)
    ref = -10 * torch.log10(torch.mean((inp["sm_fine"] - t) ** 2))
    assert abs(p.item() - ref.item()) <= 1e-5
    mask = inp["sm_fine"][:, 0] > 0.5        # the masked form follows metrics.py as written
    assert abs(psnr(inp["sm_fine"], t, mask).item() -
               (-10 * torch.log10(torch.mean(((inp["sm_fine"] - t) ** 2)[mask]))).item()) <= 1e-6


def test_loss_rejects_bad_inputs():
    from nerf_pl_amd.losses import MSELoss
    t = torch.rand(8, 3, device=DEV)
    with pytest.raises(ValueError):
        MSELoss()({"rgb_coarse": torch.rand(8, 2, device=DEV)}, t)
    with pytest.raises(ValueError):
        MSELoss()({"rgb_coarse": torch.rand(8, 3)}, t)
    with pytest.raises(ValueError):
        MSELoss()({"rgb_coarse": torch.rand(0, 3, device=DEV)}, torch.rand(0, 3, device=DEV))
