"""The training loss of the reference's step on one fused
HIP launch each way: ``losses.py:4-76`` (``MSELoss``, ``SMMSELoss``,
``OpactiyLoss``, ``loss_dict``) and ``metrics.py:4-13`` (``mse``, ``psnr``).

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
    if x.device != t.device:
        raise ValueError(f"nerf_pl_amd.losses: target on {t.device}, {what} on {x.device} "
                         "(expected the same device)")
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
        need_t = ctx.needs_input_grad[2]
        ga = torch.empty_like(a) if ctx.needs_input_grad[0] or need_t else None
        gb = (torch.empty_like(b) if b is not None and (ctx.needs_input_grad[1] or need_t)
              else None)
        if g is None or (ga is None and gb is None):
            return None, None, None
        g = g.to(torch.float32).contiguous()
        call("nr_mse_loss_bwd", a.data_ptr(), ptr(b), t.data_ptr(), a.numel(), g.data_ptr(),
             ptr(ga), ptr(gb), stream_of(a.device))
        # nn.MSELoss propagates into a target that requires grad: d/dt = -(d/da + d/db)
        gt = (-(ga + gb) if gb is not None else -ga) if need_t else None
        return (ga if ctx.needs_input_grad[0] else None,
                gb if ctx.needs_input_grad[1] else None, gt)


def mse_pair(a: torch.Tensor, b: torch.Tensor | None, target: torch.Tensor):
    """(loss, means): loss = mse(a, t) + mse(b, t) (b optional), means = the
    device vector [mse(a, t), mse(b, t)] (no host sync)."""
    if not isinstance(target, torch.Tensor) or target.dtype != torch.float32:
        raise ValueError("nerf_pl_amd.losses: the target must be a float32 tensor, got "
                         f"{getattr(target, 'dtype', type(target))}")
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


class _Opacity(torch.autograd.Function):
    @staticmethod
    def forward(ctx, oc, of, t, thres, coeff):
        loss = torch.empty((), device=oc.device, dtype=torch.float32)
        stats = torch.empty(8, device=oc.device, dtype=torch.float32)
        call("nr_opacity_loss", oc.data_ptr(), ptr(of), t.data_ptr(), t.shape[0], oc.shape[0],
             float(thres), float(coeff), loss.data_ptr(), stats.data_ptr(), stream_of(oc.device))
        ctx.save_for_backward(t, stats)
        ctx.cfg = (oc.shape[0], float(thres), of is not None)
        return loss

    @staticmethod
    def backward(ctx, g):
        t, stats = ctx.saved_tensors
        n_o, thres, has_f = ctx.cfg
        gc = torch.empty(n_o, device=g.device) if ctx.needs_input_grad[0] else None
        gf = torch.empty(n_o, device=g.device) if has_f and ctx.needs_input_grad[1] else None
        g = g.to(torch.float32).contiguous()
        call("nr_opacity_loss_bwd", t.data_ptr(), t.shape[0], n_o, thres, stats.data_ptr(),
             g.data_ptr(), ptr(gc), ptr(gf), stream_of(g.device))
        return gc, gf, None, None, None


class OpactiyLoss(nn.Module):
    """losses.py:28-73 (the reference's spelling; ``OpacityLoss`` is an alias):
    ``coeff - L1(mean(opacity[non-shadow]), mean(opacity[shadow]))`` on
    ``opacity_coarse`` [+ the same on ``opacity_fine``], the shadow pixels being
    the target rows whose grey value (mean of the three channels) exceeds
    ``sm_thres``.  train_efficient_sm.py:43 constructs it and :191 evaluates it
    on the light render with the camera batch's targets (the targets index the
    first rows of the opacities).  One ``nr_opacity_loss`` launch each way.
    Differences: when either pixel set is empty the reference returns the
    Python float 0., here a 0-d device tensor (no host sync to decide); the
    reference's debug print of the target shape is not reproduced."""

    def __init__(self, coeff=2000.0, sm_thres=0.4):
        super().__init__()
        self.coeff = coeff
        self.sm_thres = sm_thres

    def forward(self, inputs, targets):
        oc = inputs["opacity_coarse"]
        of = inputs.get("opacity_fine")
        if not oc.is_cuda or oc.dtype != torch.float32:
            raise ValueError("nerf_pl_amd.losses: opacity must be a float32 device tensor")
        if not isinstance(targets, torch.Tensor) or targets.dtype != torch.float32 \
                or targets.device != oc.device or targets.dim() != 2 or targets.shape[1] != 3:
            raise ValueError("nerf_pl_amd.losses: targets must be a (n, 3) float32 tensor on "
                             f"{oc.device}")
        oc = oc.reshape(-1).contiguous()
        if of is not None:
            of = of.reshape(-1).contiguous()
            if of.shape != oc.shape:
                raise ValueError("nerf_pl_amd.losses: opacity_fine / opacity_coarse shapes differ")
        if targets.shape[0] > oc.shape[0]:
            raise IndexError(f"OpactiyLoss: {targets.shape[0]} targets index only "
                             f"{oc.shape[0]} opacities (losses.py:54)")
        return _Opacity.apply(oc, of, targets.contiguous(), self.sm_thres, self.coeff)


OpacityLoss = OpactiyLoss

loss_dict = {"mse": MSELoss, "sm": SMMSELoss, "opacity": OpactiyLoss}


def mse(image_pred, image_gt, valid_mask=None, reduction="mean"):
    """metrics.py:4-10.  float32 device tensors go through the HIP kernel; any
    other operands -- eval.py:143 passes a CPU tensor and a numpy image -- take
    the reference's own expression (evaluation glue, not the training path)."""
    dev = (isinstance(image_pred, torch.Tensor) and isinstance(image_gt, torch.Tensor)
           and image_pred.is_cuda and image_gt.is_cuda
           and image_pred.dtype == torch.float32 and image_gt.dtype == torch.float32)
    if valid_mask is not None or reduction != "mean" or not dev:
        value = (image_pred - image_gt) ** 2
        if valid_mask is not None:
            value = value[valid_mask]
        return torch.mean(value) if reduction == "mean" else value
    return mse_pair(image_pred, None, image_gt)[0]


def psnr(image_pred, image_gt, valid_mask=None, reduction="mean"):
    """metrics.py:12-13."""
    return -10 * torch.log10(mse(image_pred, image_gt, valid_mask, reduction))
