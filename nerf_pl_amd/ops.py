"""Tensor-level wrappers over the C ABI (one function per entry point).

All tensors must be float32, contiguous and on the same HIP device; kernels are
enqueued on the current torch stream.  No CPU path exists: non-device tensors
raise.
"""
from __future__ import annotations

import functools
import os

import numpy as np
import torch

from . import packing
from ._lib import call, lib, ptr, stream_of

BLK = 32                                                # samples per block (one wave)
# MLP arithmetic (fp32 operands and results in every case):
#   "f16x3"  each operand split into two fp16 pieces (hi + lo, 22 bits), the
#            three products hi*hi + hi*lo + lo*hi accumulated in fp32 on
#            v_mfma_f32_16x16x32_f16 with power-of-two range scaling (the
#            3xTF32 scheme on CDNA4); 5.3x the fp32 MFMA issue rate
#   "bf16x6" three bf16 pieces, six products on v_mfma_f32_16x16x32_bf16
#            (error <= 2^-25 relative per product); 2.67x
#   "fp32"   v_mfma_f32_32x32x2_f32
#   "bf16"   the reduced-precision variant of BASELINE configs[1]: operands
#            rounded once to bf16, one product, fp32 accumulation (16x the fp32
#            MFMA issue rate); fp32 inputs, outputs, activations and gradients.
#            Not fp32-accurate: judged on PSNR, never the default
MATHS = ("f16x3", "bf16x6", "fp32", "bf16")
MATH = os.environ.get("NERF_PL_AMD_MATH", "f16x3")
if MATH not in MATHS:
    raise ValueError(f"NERF_PL_AMD_MATH must be one of {MATHS}, got {MATH!r}")
# csrc/layout.h NR_SAVE_PER_BLOCK / NR_GRAD_PER_BLOCK (block-native layout);
# a save buffer ends with the f16x3 gradient statistics (nr_stats_floats:
# NR_STATS reduced maxima, then NR_STAT_SEGS per-wave maxima per block)
SAVE_PER_BLOCK = BLK * (64 + 8 * 256 + 128 + 32) + 9 * 256     # no feat segment (wgrad.hip task 10)
SAVE_STATS, STAT_SEGS = 16, 11


_LAYOUT_OK = False
# nr_layout_query(9): 2 = full-graph nr_wgrad* leave G for nr_wgrad_dir_feat
ABI_REVISION = 2


def _check_layout():
    """The library's save / gradient block sizes and ABI revision must be this
    module's: a library built from other sources would write past buffers
    sized here (the round-5 abort, tests/test_layout_guard.py) or leave
    gradients this module does not finish"""
    global _LAYOUT_OK
    if not _LAYOUT_OK:
        q = lib().nr_layout_query
        got = (int(q(3)), int(q(4)), int(q(9)))
        want = (SAVE_PER_BLOCK, GRAD_PER_BLOCK, ABI_REVISION)
        if got != want:
            raise RuntimeError(f"nerf_pl_amd: libnerf_pl_amd.so has (save block, grad block, ABI "
                               f"revision) {got}, the package {want}: rebuild the library (make)")
        _LAYOUT_OK = True


def save_floats(n: int) -> int:
    """Floats of a training save buffer for n samples."""
    _check_layout()
    nb = n_blocks(n)
    return nb * SAVE_PER_BLOCK + SAVE_STATS + STAT_SEGS * nb
GRAD_PER_BLOCK = BLK * (8 * 256 + 128 + 4)   # no dfeat segment (wgrad.hip task 10)


def n_blocks(n: int) -> int:
    """Blocks of a save / gradient buffer: padded to whole 4-wave workgroups
    (csrc/layout.h nr_blocks_pad)."""
    return (n + 4 * BLK - 1) // (4 * BLK) * 4
FWD_PACKED = packing.layer_offsets(packing.FWD_LAYERS)[1] + packing.HEAD_SIZE
BWD_PACKED = packing.layer_offsets(packing.BWD_LAYERS)[1]


def _dev(t: torch.Tensor, name: str, shape_last=None):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a tensor")
    if t.device.type != "cuda":
        raise RuntimeError(f"nerf_pl_amd: {name} must live on a HIP device (got {t.device}); "
                           "this package has no CPU path")
    if t.dtype != torch.float32:
        raise TypeError(f"{name}: expected float32, got {t.dtype}")
    if not t.is_contiguous():
        t = t.contiguous()
    if shape_last is not None and t.shape[-1] != shape_last:
        raise ValueError(f"{name}: last dim must be {shape_last}, got {tuple(t.shape)}")
    return t


def to_device_f32(t: torch.Tensor, dev: torch.device) -> torch.Tensor:
    """``t.to(dev, float32)`` without draining the stream: a host tensor (e.g.
    the light camera the reference keeps on the CPU, train_efficient_sm.py)
    is staged through pinned memory and copied asynchronously -- a pageable
    ``.to(dev)`` returns only once the stream has run dry, which left the GPU
    idle while the host queued the rest of the step.  The caching host
    allocator keeps the pinned block alive until the copy has run."""
    t = t.to(torch.float32)
    if t.device == dev:
        return t
    if t.device.type == "cpu":
        return t.contiguous().pin_memory().to(dev, non_blocking=True)
    return t.to(dev)


@functools.lru_cache(maxsize=None)
def _maps(device_index: int):
    dev = torch.device("cuda", device_index)
    fwd = torch.from_numpy(packing.build_fwd_map()).to(dev)
    bwd = torch.from_numpy(packing.build_bwd_map()).to(dev)
    return fwd, bwd


@functools.lru_cache(maxsize=None)
def linspace_table(n: int, device_index: int) -> torch.Tensor:
    # torch.linspace on the CPU -- the exact values the reference uses (rendering.py:216)
    return torch.linspace(0, 1, n).to(torch.device("cuda", device_index))


@functools.lru_cache(maxsize=None)
def _maps3(device_index: int, np_: int = 3):
    dev = torch.device("cuda", device_index)
    m, h = packing.build_fwd3_map(np_)
    return torch.from_numpy(m).to(dev), torch.from_numpy(h).to(dev)


FWD3_BYTES = packing.fwd3_offsets(3)[1]
FWDH3_BYTES = packing.fwd3_offsets(2)[1]
BWDH3_BYTES = packing.bwd3_bytes(2)
FWDB1_BYTES = packing.fwd3_offsets(1)[1]
BWDB1_BYTES = packing.bwd3_bytes(1)
# C-ABI suffix of the split-operand arithmetics
_SUFFIX = {"bf16x6": "_x3", "f16x3": "_h3", "bf16": "_b1"}


def arith_of(packed: torch.Tensor) -> str:
    """MLP arithmetic a packed (forward or backward) weight buffer was built for."""
    if packed.dtype != torch.uint8:
        return "fp32"
    if packed.numel() in (FWD3_BYTES, packing.BWD3_BYTES):
        return "bf16x6"
    if packed.numel() in (FWDH3_BYTES, BWDH3_BYTES):
        return "f16x3"
    if packed.numel() in (FWDB1_BYTES, BWDB1_BYTES):
        return "bf16"
    raise ValueError(f"nerf_pl_amd: unknown packed weight buffer of {packed.numel()} bytes")


def entry(base: str, packed: torch.Tensor) -> str:
    """C-ABI entry point of ``base`` for the arithmetic of ``packed``."""
    return base + _SUFFIX.get(arith_of(packed), "")


def pack_fwd(flat: torch.Tensor, out: torch.Tensor | None = None, math: str | None = None):
    """Forward weights in the layout of the MLP arithmetic (default ``MATH``):
    float32 fragment order, or the split-operand byte buffer (uint8 tensor)."""
    math = math or MATH
    if math in _SUFFIX:
        return pack_fwd3(flat, out, math)
    return pack_fwd_fp32(flat, out)


def pack_fwd3(flat: torch.Tensor, out: torch.Tensor | None = None,
              math: str = "bf16x6") -> torch.Tensor:
    np_ = packing.NPIECES[math]
    m, hm = _maps3(flat.device.index, np_)
    out = torch.empty(packing.fwd3_offsets(np_)[1], dtype=torch.uint8, device=flat.device) \
        if out is None else out
    call("nr_pack" + _SUFFIX[math], ptr(flat), ptr(m), m.numel(), ptr(hm), ptr(out),
         stream_of(flat.device))
    return out


def head_ptr(packed: torch.Tensor) -> int:
    """Address of the fp32 head block (biases, sigma/rgb heads) of a forward
    packed buffer of either layout."""
    if packed.dtype == torch.uint8:
        return packed.data_ptr()
    return packed.data_ptr() + 4 * packing.layer_offsets(packing.FWD_LAYERS)[1]


def pack_fwd_fp32(flat: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    m, _ = _maps(flat.device.index)
    out = torch.empty(FWD_PACKED, device=flat.device) if out is None else out
    call("nr_pack", ptr(flat), ptr(m), m.numel(), ptr(out), stream_of(flat.device))
    return out


@functools.lru_cache(maxsize=None)
def _map_bwd3(device_index: int, np_: int = 3):
    return torch.from_numpy(packing.build_bwd3_map(np_)).to(torch.device("cuda", device_index))


def pack_bwd(flat: torch.Tensor, out: torch.Tensor | None = None, math: str | None = None):
    """Transposed weights of the data-gradient chain in the arithmetic (default ``MATH``)."""
    math = math or MATH
    if math in _SUFFIX:
        np_ = packing.NPIECES[math]
        m = _map_bwd3(flat.device.index, np_)
        out = torch.empty(packing.bwd3_bytes(np_), dtype=torch.uint8, device=flat.device) \
            if out is None else out
        call("nr_pack_bwd" + _SUFFIX[math], ptr(flat), ptr(m), m.numel(), ptr(out),
             stream_of(flat.device))
        return out
    return pack_bwd_fp32(flat, out)


def pack_bwd_fp32(flat: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    _, m = _maps(flat.device.index)
    out = torch.empty(BWD_PACKED, device=flat.device) if out is None else out
    call("nr_pack", ptr(flat), ptr(m), m.numel(), ptr(out), stream_of(flat.device))
    return out


def mlp_forward(packed: torch.Tensor, *, rays=None, z=None, samples_per_ray=0, x=None,
                sigma_only=False, save=False):
    """Fused PE + MLP.  Either (rays (R,8), z (R*spr)) or pre-embedded x (n, 90|63).
    Returns (out (n,4)|(n,1), saved activations or None)."""
    if x is not None:
        x = _dev(x, "x")
        n, xstride = x.shape[0], x.shape[1]
    else:
        rays = _dev(rays, "rays", 8)
        z = _dev(z, "z")
        n, xstride = z.numel(), 0
    dev = packed.device
    # a sigma-only training run (save) writes (n, 4) rows [0, 0, 0, sigma]
    out = torch.empty(n, 1 if sigma_only and not save else 4, device=dev)
    sv = torch.empty(save_floats(n), device=dev) if save else None
    call(entry("nr_mlp_fwd", packed), ptr(packed), ptr(rays), ptr(z), n, int(samples_per_ray),
         ptr(x), xstride, int(sigma_only), ptr(out), ptr(sv), stream_of(dev))
    return out, sv


def sigma_points(packed, pts):
    """sigma (n,) of the fused sigma-only MLP at points (n,3)."""
    pts = _dev(pts, "pts", 3)
    out = torch.empty(pts.shape[0], device=pts.device)
    call(entry("nr_mlp_sigma_points", packed), ptr(packed), ptr(pts), pts.shape[0], ptr(out),
         stream_of(pts.device))
    return out


def coarse_z(rays, n_samples, use_disp, perturb, u=None, seed=0):
    rays = _dev(rays, "rays", 8)
    n_rays = rays.shape[0]
    z = torch.empty(n_rays, n_samples, device=rays.device)
    tl = linspace_table(n_samples, rays.device.index)
    call("nr_coarse_z", ptr(rays), ptr(tl), n_rays, n_samples, int(use_disp), float(perturb),
         ptr(u), seed, ptr(z), stream_of(rays.device))
    return z


def composite_forward(raw, z, rays, noise, noise_std, seed, rng_stream, white_back,
                      weights_only=False):
    """raw (R*S, 4) [rgb, sigma] or (R*S, 1) sigma (then rgb is None: the
    sigma-only render of rendering_shadows.py:164-198)."""
    z = _dev(z, "z")
    n_rays, S = z.shape
    stride = raw.shape[-1]
    dev = z.device
    opac = torch.empty(n_rays, device=dev)
    w = torch.empty(n_rays, S, device=dev)
    rgb = None if weights_only or stride < 4 else torch.empty(n_rays, 3, device=dev)
    depth = None if weights_only else torch.empty(n_rays, device=dev)
    call("nr_composite_fwd", ptr(raw), stride, stride - 1, ptr(z), ptr(rays), ptr(noise),
         float(noise_std), seed, rng_stream, n_rays, S, int(white_back), int(weights_only),
         ptr(rgb), ptr(depth), ptr(opac), ptr(w), stream_of(dev))
    return rgb, depth, opac, w


def composite_backward(raw, z, rays, noise, noise_std, seed, rng_stream, white_back,
                       g_rgb, g_depth, g_opacity):
    n_rays, S = z.shape
    stride = raw.shape[-1]
    g_raw = torch.empty(n_rays * S, stride, device=z.device)
    call("nr_composite_bwd", ptr(raw), stride, stride - 1, ptr(z), ptr(rays), ptr(noise), float(noise_std), seed,
         rng_stream, n_rays, S, int(white_back),
         ptr(None if g_rgb is None else g_rgb.contiguous()),
         ptr(None if g_depth is None else g_depth.contiguous()),
         ptr(None if g_opacity is None else g_opacity.contiguous()), ptr(g_raw),
         stream_of(z.device))
    return g_raw


def sample_pdf(weights, rays, n_importance, u=None, jitter=None, seed=0, z_coarse=None,
               merge=False):
    """Importance depths (R, I); with merge=True also the sorted (R, S+I) fine depths."""
    weights = _dev(weights, "weights")
    rays = _dev(rays, "rays", 8)
    n_rays, S = weights.shape
    dev = weights.device
    z_pdf = torch.empty(n_rays, n_importance, device=dev)
    z_fine = torch.empty(n_rays, S + n_importance, device=dev) if merge else None
    call("nr_sample_pdf", ptr(weights), S, ptr(rays), ptr(z_coarse), ptr(u), ptr(jitter), seed,
         n_rays, n_importance, ptr(z_pdf), ptr(z_fine), stream_of(dev))
    return z_pdf, z_fine


def embed(x, n_freqs):
    x = _dev(x, "x", 3)
    n = x.shape[0]
    out = torch.empty(n, 3 * (2 * n_freqs + 1), device=x.device)
    call("nr_embed", ptr(x), n, int(n_freqs), ptr(out), stream_of(x.device))
    return out


def probe_mfma32(a, b):
    d = torch.empty(32 * 32, device=a.device)
    call("nr_probe_mfma32", ptr(a), ptr(b), ptr(d), stream_of(a.device))
    return d.view(32, 32)


def layout_query(what: int) -> int:
    return int(lib().nr_layout_query(what))


def native_to_rows(seg: torch.Tensor, n: int, width: int) -> torch.Tensor:
    """Decode a block-native activation segment (layout.h) to (n, width) rows:
    element [block][t][q][lane=32h+j][e] is feature 32t+8q+4h+e of sample j."""
    nb = n_blocks(n)
    x = seg[: nb * BLK * width].view(nb, width // 32, 4, 2, BLK, 4)
    return x.permute(0, 4, 1, 2, 3, 5).reshape(nb * BLK, width)[:n]


def n16_to_rows(seg: torch.Tensor, n: int, width: int) -> torch.Tensor:
    """Decode an N16 segment of the bf16x6 pipeline (csrc/x3.h) to (n, width)
    rows: element [block][F][S][lane=16g+j][r] is column 16F+4g+r of sample
    16S+j (PE segments: columns are PE slots, packing.PE16_MAP / DIR16_MAP)."""
    nb = n_blocks(n)
    x = seg[: nb * BLK * width].view(nb, width // 16, 2, 4, 16, 4)
    return x.permute(0, 2, 4, 1, 3, 5).reshape(nb * BLK, width)[:n]


def saved_rows(seg: torch.Tensor, n: int, width: int) -> torch.Tensor:
    """An activation segment of a full-graph training forward (csrc/x3.h
    store_row; exact fp32: layout.h store_row_piece): sample-major rows of
    ``width`` values (PE segments: columns are PE slots, packing.PE16_MAP /
    DIR16_MAP, or for fp32 the packed k order 32h + g / 16h + g) -> (n, width)."""
    nb = n_blocks(n)
    return seg[: nb * BLK * width].view(nb * BLK, width)[:n]


def save_segments(sv: torch.Tensor, n: int) -> dict:
    """Named views of a training save buffer (csrc/layout.h NrSave order)."""
    nb = n_blocks(n)
    o, out = 0, {}
    for name, w in [("pe", 64)] + [(f"h{i}", 256) for i in range(1, 9)] + \
                   [("hdir", 128), ("dirpe", 32)]:
        out[name] = sv[o:o + nb * BLK * w]
        o += nb * BLK * w
    out["mask"] = sv[o:o + nb * 9 * 256]
    return out


def np_maps():
    return packing.build_fwd_map(), packing.build_bwd_map()


__all__ = [n for n in dir() if not n.startswith("_") and n not in ("np", "functools")]
