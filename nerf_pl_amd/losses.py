"""The training loss of the reference's step on one fused
HIP launch each way: ``losses.py:4-27`` (``MSELoss``, ``SMMSELoss``,
``loss_dict``) and ``metrics.py:4-13`` (``mse``, ``psnr``).

``MSELoss()(results, targets)`` is ``nn.MSELoss(reduction='mean')`` on
``rgb_coarse`` plus the same on ``rgb_fine`` when present (the fine term added
in fp32, ``loss += ...``), computed by ``nr_mse_loss`` (squares in fp32,
fixed-order double sums: deterministic) with the backward of both terms in one
``nr_mse_loss_bwd`` launch, ``(2/n) * (x - t) * g`` as torch's
``mse_loss_backward``.  Inputs live on the device; there is no CPU path.
"""
from __future__ import annotations

import torch
from torch import nn

from ._lib import call, ptr, stream_of


def _check(x: torch.Tensor, t: torch.Tensor, what: str) -> torch.Tensor:
    if not x.is_cuda or x.dtype != torch.float32:
        raise ValueError(f"nerf_pl_amd.losses: {what} must be a float32 device tensor")
    if x.shape != t.shape:
        raise ValueError(f"nerf_pl_amd.losses: {what} shape {tuple(x.shape)} != target "
                         f"shape {tuple(t.shape)}")
    if x.numel() == 0:
        raise ValueError("nerf_pl_amd.losses: the mean of an empty batch is undefined")
    return x.contiguous()


class _MSEPair(torch.autograd.Function):
    """loss = mean((a - t)^2) [+ mean((b - t)^2)] -> (loss, per-term means)"""

    @staticmethod
    def forward(ctx, a, b, t):
        loss = torch.empty((), device=a.device, dtype=torch.float32)
        means = torch.empty(2, device=a.device, dtype=torch.float32)
        call("nr_mse_loss", a.data_ptr(), ptr(b), t.data_ptr(), a.numel(), loss.data_ptr(),
             means.data_ptr(), stream_of(a.device))
        ctx.save_for_backward(a, b, t)
        ctx.mark_non_differentiable(means)
        ctx.set_materialize_grads(False)
        return loss, means

    @staticmethod
    def backward(ctx, g, _g_means):   # noqa: ARG004 -- the means are not differentiable
        a, b, t = ctx.saved_tensors
        ga = torch.empty_like(a) if ctx.needs_input_grad[0] else None
        gb = torch.empty_like(b) if b is not None and ctx.needs_input_grad[1] else None
        if g is None or (ga is None and gb is None):
            return None, None, None
        g = g.to(torch.float32).contiguous()
        call("nr_mse_loss_bwd", a.data_ptr(), ptr(b), t.data_ptr(), a.numel(), g.data_ptr(),
             ptr(ga), ptr(gb), stream_of(a.device))
        return ga, gb, None


def mse_pair(a: torch.Tensor, b: torch.Tensor | None, target: torch.Tensor):
    """(loss, means): loss = mse(a, t) + mse(b, t) (b optional), means = the
    device vector [mse(a, t), mse(b, t)] (no host sync)."""
    t = target.contiguous()
    a = _check(a, t, "input")
    b = None if b is None else _check(b, t, "fine input")
    return _MSEPair.apply(a, b, t)


class MSELoss(nn.Module):
    """losses.py:4-14.  ``self.last`` holds the device vector [coarse mse, fine
    mse] of the last call (for ``psnr`` logging without another pass)."""

    key = "rgb"

    def __init__(self):
        super().__init__()
        self.last = None

    def forward(self, inputs, targets):
        fine = inputs.get(f"{self.key}_fine")
        loss, self.last = mse_pair(inputs[f"{self.key}_coarse"], fine, targets)
        return loss


class SMMSELoss(MSELoss):
    """losses.py:16-27: the same on the shadow-map outputs ``sm_coarse`` /
    ``sm_fine``."""

    key = "sm"


loss_dict = {"mse": MSELoss, "sm": SMMSELoss}


def mse(image_pred, image_gt, valid_mask=None, reduction="mean"):
    """metrics.py:4-10."""
    if valid_mask is not None or reduction != "mean":
        value = (image_pred - image_gt) ** 2
        if valid_mask is not None:
            value = value[valid_mask]
        return torch.mean(value) if reduction == "mean" else value
    return mse_pair(image_pred, None, image_gt)[0]


def psnr(image_pred, image_gt, valid_mask=None, reduction="mean"):
    """metrics.py:12-13."""
    return -10 * torch.log10(mse(image_pred, image_gt, valid_mask, reduction))
