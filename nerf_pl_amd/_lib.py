"""ctypes binding of the C-ABI library ``libnerf_pl_amd.so`` (include/nerf_pl_amd.h).

The library is built in-tree by ``make`` (or ``__graft_entry__.build()``).  There
is deliberately no fallback: if the library is missing or a call fails, a
``RuntimeError`` carrying ``nr_last_error()`` is raised.
"""
from __future__ import annotations

import ctypes
import os

# NERF_PL_AMD_LIB: another build of the same ABI (tests/test_abi_asan.py loads the
# host AddressSanitizer build through it)
LIB_PATH = os.environ.get("NERF_PL_AMD_LIB") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "libnerf_pl_amd.so")

_p = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64
_u64 = ctypes.c_uint64
_f = ctypes.c_float

# name -> argtypes; every entry returns int (0 = ok) unless listed in _RESTYPES
SIGNATURES = {
    "nr_mlp_fwd": [_p, _p, _p, _i64, _i, _p, _i, _i, _p, _p, _p],
    "nr_mlp_sigma_points": [_p, _p, _i64, _p, _p],
    "nr_fwd3_packed_bytes": [],
    "nr_pack_x3": [_p, _p, _i64, _p, _p, _p],
    "nr_mlp_fwd_x3": [_p, _p, _p, _i64, _i, _p, _i, _i, _p, _p, _p],
    "nr_mlp_sigma_points_x3": [_p, _p, _i64, _p, _p],
    "nr_pack_bwd_x3": [_p, _p, _i64, _p, _p],
    "nr_mlp_bwd_x3": [_p, _p, _p, _p, _p, _i64, _p, _p],
    "nr_mlp_bwd_sigma_x3": [_p, _p, _p, _p, _p, _i64, _p, _p],
    "nr_wgrad_x3": [_p, _p, _i64, _p, _p, _p],
    "nr_wgrad_sigma_x3": [_p, _p, _i64, _p, _p, _p],
    "nr_fwd3_packed_bytes_h3": [],
    "nr_pack_h3": [_p, _p, _i64, _p, _p, _p],
    "nr_mlp_fwd_h3": [_p, _p, _p, _i64, _i, _p, _i, _i, _p, _p, _p],
    "nr_mlp_sigma_points_h3": [_p, _p, _i64, _p, _p],
    "nr_pack_bwd_h3": [_p, _p, _i64, _p, _p],
    "nr_mlp_bwd_h3": [_p, _p, _p, _p, _p, _i64, _p, _p],
    "nr_mlp_bwd_sigma_h3": [_p, _p, _p, _p, _p, _i64, _p, _p],
    "nr_wgrad_h3": [_p, _p, _i64, _p, _p, _p],
    "nr_wgrad_sigma_h3": [_p, _p, _i64, _p, _p, _p],
    "nr_fwd3_packed_bytes_b1": [],
    "nr_pack_b1": [_p, _p, _i64, _p, _p, _p],
    "nr_mlp_fwd_b1": [_p, _p, _p, _i64, _i, _p, _i, _i, _p, _p, _p],
    "nr_mlp_sigma_points_b1": [_p, _p, _i64, _p, _p],
    "nr_pack_bwd_b1": [_p, _p, _i64, _p, _p],
    "nr_mlp_bwd_b1": [_p, _p, _p, _p, _p, _i64, _p, _p],
    "nr_mlp_bwd_sigma_b1": [_p, _p, _p, _p, _p, _i64, _p, _p],
    "nr_wgrad_b1": [_p, _p, _i64, _p, _p, _p],
    "nr_wgrad_sigma_b1": [_p, _p, _i64, _p, _p, _p],
    "nr_active_samples": [_p, _i64, _p, _p, _p, _p],
    "nr_active_scratch_ints": [_i64],
    "nr_mlp_bwd_active_x3": [_p, _p, _p, _p, _p, _i64, _p, _p, _p, _p],
    "nr_mlp_bwd_active_h3": [_p, _p, _p, _p, _p, _i64, _p, _p, _p, _p],
    "nr_mlp_bwd_sigma_active_x3": [_p, _p, _p, _p, _p, _i64, _p, _p, _p, _p],
    "nr_mlp_bwd_sigma_active_h3": [_p, _p, _p, _p, _p, _i64, _p, _p, _p, _p],
    "nr_wgrad_active_x3": [_p, _p, _i64, _p, _p, _p, _p, _p],
    "nr_wgrad_active_h3": [_p, _p, _i64, _p, _p, _p, _p, _p],
    "nr_wgrad_sigma_active_x3": [_p, _p, _i64, _p, _p, _p, _p, _p],
    "nr_wgrad_sigma_active_h3": [_p, _p, _i64, _p, _p, _p, _p, _p],
    "nr_mlp_bwd": [_p, _p, _p, _p, _p, _i64, _p, _p],
    "nr_mlp_bwd_sigma": [_p, _p, _p, _p, _p, _i64, _p, _p],
    "nr_mlp_bwd_active": [_p, _p, _p, _p, _p, _i64, _p, _p, _p, _p],
    "nr_mlp_bwd_sigma_active": [_p, _p, _p, _p, _p, _i64, _p, _p, _p, _p],
    "nr_wgrad_sigma": [_p, _p, _i64, _p, _p, _p],
    "nr_wgrad_active": [_p, _p, _i64, _p, _p, _p, _p, _p],
    "nr_wgrad_sigma_active": [_p, _p, _i64, _p, _p, _p, _p, _p],
    "nr_mlp_fwd_listed": [_p, _p, _p, _i64, _i, _i, _p, _p, _p, _p],
    "nr_mlp_bwd_listed": [_p, _p, _p, _p, _p, _i64, _p, _p, _p, _p],
    "nr_mlp_bwd_sigma_listed": [_p, _p, _p, _p, _p, _i64, _p, _p, _p, _p],
    "nr_wgrad_listed": [_p, _p, _i64, _p, _p, _p, _p, _p],
    "nr_wgrad_sigma_listed": [_p, _p, _i64, _p, _p, _p, _p, _p],
    "nr_mlp_fwd_listed_x3": [_p, _p, _p, _i64, _i, _i, _p, _p, _p, _p],
    "nr_mlp_bwd_listed_x3": [_p, _p, _p, _p, _p, _i64, _p, _p, _p, _p],
    "nr_mlp_bwd_sigma_listed_x3": [_p, _p, _p, _p, _p, _i64, _p, _p, _p, _p],
    "nr_wgrad_listed_x3": [_p, _p, _i64, _p, _p, _p, _p, _p],
    "nr_wgrad_sigma_listed_x3": [_p, _p, _i64, _p, _p, _p, _p, _p],
    "nr_mlp_fwd_listed_h3": [_p, _p, _p, _i64, _i, _i, _p, _p, _p, _p],
    "nr_mlp_bwd_listed_h3": [_p, _p, _p, _p, _p, _i64, _p, _p, _p, _p],
    "nr_mlp_bwd_sigma_listed_h3": [_p, _p, _p, _p, _p, _i64, _p, _p, _p, _p],
    "nr_wgrad_listed_h3": [_p, _p, _i64, _p, _p, _p, _p, _p],
    "nr_wgrad_sigma_listed_h3": [_p, _p, _i64, _p, _p, _p, _p, _p],
    "nr_wgrad_workspace_bytes": [_i64],
    "nr_wgrad_dir_feat": [_p, _p, _p],
    "nr_sm_workspace_bytes": [_i64, _i64],
    "nr_wgrad": [_p, _p, _i64, _p, _p, _p],
    "nr_coarse_z": [_p, _p, _i64, _i, _i, _f, _p, _u64, _p, _p],
    "nr_composite_fwd": [_p, _i, _i, _p, _p, _p, _f, _u64, _i, _i64, _i, _i, _i, _p, _p, _p,
                         _p, _p],
    "nr_composite_bwd": [_p, _i, _i, _p, _p, _p, _f, _u64, _i, _i64, _i, _i, _p, _p, _p, _p,
                         _p],
    "nr_gen_rays": [_p, _i64, _i, _i, _f, _f, _f, _f, _f, _i, _f, _f, _f, _f, _p, _i64, _p, _p,
                    _p, _p],
    "nr_adam_max_tensors": [],
    "nr_adam_step": [_p, _p, _p, _p, _p, _i, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                     ctypes.c_double, ctypes.c_double, _i64, _p],
    "nr_mse_loss": [_p, _p, _p, _i64, _p, _p, _p],
    "nr_opacity_loss": [_p, _p, _p, _i64, _i64, _f, _f, _p, _p, _p],
    "nr_opacity_loss_bwd": [_p, _i64, _i64, _f, _p, _p, _p, _p, _p],
    "nr_searchsorted": [_p, _p, _i64, _i64, _i64, _i64, _i, _p, _p],
    "nr_searchsorted_f64": [_p, _p, _i64, _i64, _i64, _i64, _i, _p, _p],
    "nr_mse_loss_bwd": [_p, _p, _p, _i64, _p, _p, _p, _p],
    "nr_sm_normed_depth": [_p, _p, _p, _i64, _p, _p],
    "nr_sm_normed_depth_bwd": [_p, _p, _p, _i64, _p, _p],
    "nr_sm_forward": [_p, _p, _p, _p, _i, _p, _p, _p, _i, _i, _i, _f, _f, _i, _f, _i64, _p, _p,
                      _p],
    "nr_sm_backward": [_p, _p, _i, _f, _f, _i, _i64, _i64, _p, _p, _p],
    "nr_sample_pdf": [_p, _i, _p, _p, _p, _p, _u64, _i64, _i, _p, _p, _p],
    "nr_embed": [_p, _i64, _i, _p, _p],
    "nr_pack": [_p, _p, _i64, _p, _p],
    "nr_probe_mfma32": [_p, _p, _p, _p],
    "nr_layout_query": [_i],
    "nr_last_error": [],
}
_RESTYPES = {"nr_layout_query": _i64, "nr_adam_max_tensors": _i, "nr_fwd3_packed_bytes": _i64,
             "nr_fwd3_packed_bytes_h3": _i64, "nr_fwd3_packed_bytes_b1": _i64,
             "nr_wgrad_workspace_bytes": _i64, "nr_active_scratch_ints": _i64,
             "nr_sm_workspace_bytes": _i64, "nr_last_error": ctypes.c_char_p}

_lib = None


def lib():
    """Load the library once; raise loudly if it is absent or incomplete."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"nerf_pl_amd: HIP library not built ({LIB_PATH}); "
                               "run `make` or __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            fn = getattr(L, name, None)
            if fn is None:          # reported by missing_symbols(); calling it raises
                continue
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, _i)
        _lib = L
    return _lib


def missing_symbols() -> list:
    L = lib()
    return [n for n in SIGNATURES if getattr(L, n, None) is None]


def last_error() -> str:
    return lib().nr_last_error().decode(errors="replace")


def call(name: str, *args) -> None:
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed (code {rc}): {last_error()}")


def ptr(t) -> int | None:
    """Device pointer of a tensor (or None)."""
    return None if t is None else t.data_ptr()


def stream_of(device) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream
