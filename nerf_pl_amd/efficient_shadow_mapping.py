"""Differentiable shadow mapping -- models/efficient_shadow_mapping.py, run by
the ``nr_sm_*`` HIP kernels (csrc/shadow.hip).

``run_shadow_mapping`` and ``get_normed_w`` keep the reference signatures
(:19-62).  ``_ShadowMap`` is the autograd op behind them and behind
``rendering_shadows.efficient_sm``: one launch sequence per batch, with the
reference's per-pose run splitting done on the device.  Both ops are
differentiable in every tensor the reference differentiates: the camera
depths and -- ``train_efficient_sm.py --grad_on_light`` (:158-162), the mode 60
of the reference's 63 ``train_efficient_sm`` launchers use -- the light's
normed depth map (texel-gather backward, ``nr_sm_backward``) and through it
the light render's depths (``_NormedDepth``, ``nr_sm_normed_depth_bwd``).
"""
from __future__ import annotations

import torch

from . import ops
from ._lib import call, stream_of

__all__ = ["run_shadow_mapping", "get_normed_w", "normalize_min_max", "shadow_map",
           "normed_depth", "EPSILON"]

EPSILON = 1e-5
_METHODS = {"shadow_method_1": 1, "shadow_method_2": 2}


def normalize_min_max(tensor, new_max=1.0, new_min=0.0):
    """:10-11 (a visualisation helper in the reference's eval loop)."""
    return (tensor - tensor.min()) / (tensor.max() - tensor.min() + EPSILON) * (new_max - new_min) \
        + new_min


def _cam(obj):
    """(eye (3,), matrix (3,3)) of a Camera-like object or {'eye_pos', 'camera'} dict."""
    if isinstance(obj, dict):
        return obj["eye_pos"], obj["camera"]
    return obj.eye_pos, obj.camera


class _NormedDepth(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cam, pixels, depth):
        out = torch.empty_like(depth)
        call("nr_sm_normed_depth", ops.ptr(cam), ops.ptr(pixels), ops.ptr(depth), depth.shape[0],
             ops.ptr(out), stream_of(depth.device))
        ctx.save_for_backward(cam, pixels)
        return out

    @staticmethod
    def backward(ctx, g):
        cam, pixels = ctx.saved_tensors
        g = g.contiguous()
        g_depth = torch.empty_like(g)
        call("nr_sm_normed_depth_bwd", ops.ptr(cam), ops.ptr(pixels), ops.ptr(g), g.shape[0],
             ops.ptr(g_depth), stream_of(g.device))
        return None, None, g_depth


def normed_depth(camera: torch.Tensor, pixels: torch.Tensor, depth: torch.Tensor):
    """depth / (|camera @ pixel| + 1e-5) (:47-62, column 3); differentiable in
    ``depth`` (the light render's depths under --grad_on_light)."""
    dev = depth.device
    pixels = ops._dev(ops.to_device_f32(pixels, dev), "pixels", 3)
    depth = ops._dev(depth.reshape(-1), "depth")
    cam = ops._dev(ops.to_device_f32(camera, dev).reshape(9), "camera")
    if pixels.shape[0] != depth.shape[0]:
        raise ValueError(f"normed_depth: {pixels.shape[0]} pixels for {depth.shape[0]} depths")
    return _NormedDepth.apply(cam, pixels, depth)


def get_normed_w(camera, pixel_depth, device="cpu"):
    """:41-58 -- [i, j, 1, depth / (|M p| + 1e-5)] for a (n,4) [pixel, depth] array."""
    del device
    _, m = _cam(camera)
    w = normed_depth(m, pixel_depth[:, :3].contiguous(), pixel_depth[:, 3].contiguous())
    return torch.cat([pixel_depth[:, :3], w.view(-1, 1)], dim=1)


class _ShadowMap(torch.autograd.Function):
    @staticmethod
    def forward(ctx, depth, pixels, eye, cams, per_ray, light_cam, light_eye, light_w, res,
                method, delta, epsilon, sigmoid, out_eps):
        n = depth.shape[0]
        dev = depth.device
        n_light = int(res[0]) * int(res[1])
        ws = torch.empty((int(call_ws_bytes(n, n_light)) + 7) // 8, dtype=torch.float64,
                         device=dev)
        out = torch.empty(n, 3, device=dev)
        call("nr_sm_forward", ops.ptr(pixels), ops.ptr(depth), ops.ptr(eye), ops.ptr(cams),
             int(per_ray), ops.ptr(light_cam), ops.ptr(light_eye), ops.ptr(light_w),
             int(res[0]), int(res[1]), method, float(delta), float(epsilon), int(sigmoid),
             float(out_eps), n, ops.ptr(ws), ops.ptr(out), stream_of(dev))
        ctx.save_for_backward(ws)
        ctx.cfg = (method, delta, epsilon, sigmoid, n, n_light)
        return out

    @staticmethod
    def backward(ctx, g_out):
        (ws,) = ctx.saved_tensors
        method, delta, epsilon, sigmoid, n, n_light = ctx.cfg
        need_depth, need_light = ctx.needs_input_grad[0], ctx.needs_input_grad[7]
        if not (need_depth or need_light):
            return (None,) * 14
        g_out = g_out.contiguous()
        dev = g_out.device
        g_depth = torch.empty(n, device=dev) if need_depth else None
        g_light = torch.empty(n_light, device=dev) if need_light else None
        call("nr_sm_backward", ops.ptr(g_out), ops.ptr(ws), method, float(delta), float(epsilon),
             int(sigmoid), n, n_light, ops.ptr(g_depth), ops.ptr(g_light), stream_of(dev))
        return (g_depth,) + (None,) * 6 + (g_light,) + (None,) * 6


def call_ws_bytes(n: int, n_light: int) -> int:
    from ._lib import lib
    return int(lib().nr_sm_workspace_bytes(n, n_light))


def shadow_map(depth, pixels, eye, cams, light_eye, light_cam, normed_light_w, res,
               mode="shadow_method_2", delta=1e-2, epsilon=0.0, sigmoid=False, out_eps=0.0):
    """Shadow values (n,3) of camera rays against the light's normed depth map.

    eye (n,3) / cams (n,3,3) per ray (split into runs of equal eye position
    like rendering_shadows.py:377-396), or eye (3,) / cams (3,3) for all rays.
    Differentiable w.r.t. ``depth`` and ``normed_light_w``."""
    if mode not in _METHODS:
        raise ValueError("{} not found".format(mode))
    dev = depth.device
    depth = ops._dev(depth.reshape(-1), "depth")
    n = depth.shape[0]
    pixels = ops._dev(ops.to_device_f32(pixels, dev), "pixels", 3)
    eye, cams = ops.to_device_f32(eye, dev), ops.to_device_f32(cams, dev)
    per_ray = eye.dim() == 2 and eye.shape[0] == n and n > 1
    if per_ray:
        eye = eye.reshape(n, 3).contiguous()
        cams = cams.reshape(n, 9).contiguous()
    else:
        eye = eye.reshape(-1, 3)[0].contiguous()
        cams = cams.reshape(-1, 9)[0].contiguous()
    w, h = int(res[0]), int(res[1])
    lw = ops._dev(normed_light_w.reshape(-1), "light depth map")
    if lw.shape[0] != w * h:
        raise ValueError(f"light depth map has {lw.shape[0]} entries, expected {w}x{h}")
    return _ShadowMap.apply(depth, pixels, eye, cams, per_ray,
                            ops.to_device_f32(light_cam, dev).reshape(9).contiguous(),
                            ops.to_device_f32(light_eye, dev).reshape(3).contiguous(), lw, (w, h),
                            _METHODS[mode], delta, epsilon, bool(sigmoid), out_eps)


def run_shadow_mapping(res, camera, light_cam, batched_mesh_range_cam, meshed_normed_light_cam,
                       device=None, mode="shadow_method_1", delta=1e-2, epsilon=0.0, new_min=0.0,
                       new_max=1.0, sigmoid=False, use_numpy_meshgrid=True):
    """:19-38 for one camera: (n,4) [pixel, depth] camera rays against the light's
    (H*W,4) normed [pixel, depth] map -> (n,3).  ``new_min``/``new_max`` are
    ignored, as in the reference (:120)."""
    del device, new_min, new_max, use_numpy_meshgrid
    eye, m = _cam(camera)
    leye, lm = _cam(light_cam)
    return shadow_map(batched_mesh_range_cam[:, 3], batched_mesh_range_cam[:, :3], eye, m, leye,
                      lm, meshed_normed_light_cam[:, 3], res, mode, delta, epsilon, sigmoid)
