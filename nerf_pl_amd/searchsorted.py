"""``torchsearchsorted.searchsorted`` on HIP -- the reference's only native
dependency (the un-vendored git submodule of .gitmodules:1-3, imported at
models/rendering.py:2 and models/rendering_rgb_sm.py:2, called at
rendering.py:37 / rendering_rgb_sm.py:40).

``searchsorted(a, v, out=None, side='left')`` keeps the extension's contract:
``a`` (nrows_a, ncols_a) sorted along each row, ``v`` (nrows_v, ncols_v), with
nrows_a == nrows_v or one of them 1; returns the int64 (nrows, ncols_v)
insertion indices, numpy ``searchsorted`` semantics per row (``side='right'``:
entries <= v; ``'left'``: entries < v), written into ``out`` when given.  One
``nr_searchsorted`` launch.  Device tensors only (this package has no CPU
path); float32 or float64.  Code that imports ``torchsearchsorted`` binds it
with ``sys.modules['torchsearchsorted'] = nerf_pl_amd.searchsorted``
(INTEGRATION.md).
"""
from __future__ import annotations

import torch

from ._lib import call, ptr, stream_of

__all__ = ["searchsorted"]


def searchsorted(a: torch.Tensor, v: torch.Tensor, out: torch.Tensor = None,
                 side: str = "left") -> torch.Tensor:
    if side not in ("left", "right"):
        raise ValueError(f"side must be 'left' or 'right', got {side!r}")
    for name, t in (("a", a), ("v", v)):
        if not isinstance(t, torch.Tensor) or t.dim() != 2:
            raise ValueError(f"searchsorted: {name} must be a 2-D tensor")
        if t.device.type != "cuda":
            raise RuntimeError(f"nerf_pl_amd.searchsorted: {name} must live on a HIP device "
                               f"(got {t.device}); this package has no CPU path")
    if a.dtype != v.dtype or a.dtype not in (torch.float32, torch.float64):
        raise TypeError(f"searchsorted: a and v must both be float32 or float64, got "
                        f"{a.dtype} / {v.dtype}")
    if a.device != v.device:
        raise ValueError("searchsorted: a and v on different devices")
    if a.shape[0] != v.shape[0] and 1 not in (a.shape[0], v.shape[0]):
        raise ValueError(f"searchsorted: a has {a.shape[0]} rows and v {v.shape[0]} "
                         "(need equal, or one of them 1)")
    nrows = max(a.shape[0], v.shape[0])
    shape = (nrows, v.shape[1])
    if out is None:
        out = torch.empty(shape, dtype=torch.int64, device=v.device)
    elif out.shape != shape or out.dtype != torch.int64 or out.device != v.device:
        raise ValueError(f"searchsorted: out must be an int64 {shape} tensor on {v.device}")
    a, v = a.contiguous(), v.contiguous()
    res = out if out.is_contiguous() else torch.empty(shape, dtype=torch.int64, device=v.device)
    entry = "nr_searchsorted" if a.dtype == torch.float32 else "nr_searchsorted_f64"
    call(entry, ptr(a), ptr(v), a.shape[0], a.shape[1], v.shape[0], v.shape[1],
         int(side == "right"), ptr(res), stream_of(v.device))
    if res is not out:
        out.copy_(res)
    return out
