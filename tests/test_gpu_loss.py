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


def test_loss_checks_the_target():
    """a CPU or non-float32 target raises like torch's device /
    dtype errors instead of handing the kernel a host pointer or misread bits;
    a target that requires grad receives nn.MSELoss's gradient."""
    from nerf_pl_amd.losses import MSELoss
    x = {"rgb_coarse": torch.rand(8, 3, device=DEV), "rgb_fine": torch.rand(8, 3, device=DEV)}
    with pytest.raises(ValueError, match="device"):
        MSELoss()(x, torch.rand(8, 3))
    with pytest.raises(ValueError, match="float32"):
        MSELoss()(x, torch.rand(8, 3, device=DEV, dtype=torch.float64))
    with pytest.raises(ValueError, match="float32"):
        MSELoss()(x, torch.rand(8, 3, device=DEV).half())
    t = torch.rand(8, 3, device=DEV, requires_grad=True)
    a = x["rgb_coarse"].clone().requires_grad_(True)
    b = x["rgb_fine"].clone().requires_grad_(True)
    MSELoss()({"rgb_coarse": a, "rgb_fine": b}, t).backward()
    t2 = t.detach().clone().requires_grad_(True)
    a2, b2 = a.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    (torch.nn.functional.mse_loss(a2, t2) + torch.nn.functional.mse_loss(b2, t2)).backward()
    for u, w in ((a, a2), (b, b2), (t, t2)):
        torch.testing.assert_close(u.grad, w.grad, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("n_t,n_o,fine,seed,nan", [(512, 4096, True, 0, False),
                                                   (300, 300, False, 1, False),
                                                   (7, 64, True, 2, False),
                                                   (512, 1024, True, 3, True)])
def test_opacity_loss_matches_reference(n_t, n_o, fine, seed, nan):
    """losses.py:28-73 OpactiyLoss, as train_efficient_sm.py:191 calls it: the
    light render's opacities indexed by the camera batch's shadow pixels.  A
    target row whose grey value is NaN is in neither torch.where set (:39-40):
    it changes neither count nor mean, and its opacity gets no gradient."""
    from oracle import nerf_oracle as O
    from nerf_pl_amd.losses import loss_dict
    g = torch.Generator().manual_seed(seed)
    tgt = torch.rand(n_t, 3, generator=g)
    if nan:
        tgt[::7, torch.arange(n_t)[::7] % 3] = float("nan")
    res = {"opacity_coarse": torch.rand(n_o, generator=g)}
    if fine:
        res["opacity_fine"] = torch.rand(n_o, generator=g)
    ref_in = {k: v.clone().requires_grad_(True) for k, v in res.items()}
    ref = O.opacity_loss(ref_in, tgt)
    ref.backward()
    dev_in = {k: v.to(DEV).requires_grad_(True) for k, v in res.items()}
    got = loss_dict["opacity"]()(dev_in, tgt.to(DEV))
    got.backward()
    assert abs(got.item() - ref.item()) <= 1e-3 * 1e-4 * abs(ref.item()) + 1e-4
    for k in res:
        torch.testing.assert_close(dev_in[k].grad.cpu(), ref_in[k].grad, rtol=1e-5, atol=1e-9)


def test_opacity_loss_empty_set_is_zero():
    from nerf_pl_amd.losses import OpactiyLoss
    tgt = torch.zeros(16, 3, device=DEV)          # no shadow pixel
    o = {"opacity_coarse": torch.rand(32, device=DEV, requires_grad=True)}
    loss = OpactiyLoss()(o, tgt)
    assert loss.item() == 0.0
    loss.backward()
    assert (o["opacity_coarse"].grad == 0).all()
    with pytest.raises(IndexError):
        OpactiyLoss()({"opacity_coarse": torch.rand(8, device=DEV)}, torch.rand(9, 3, device=DEV))
