"""Fragment-order weight packing for the fused MLP kernels.

The fused kernels evaluate every layer in the *transposed* form
``D[out_feature][sample] = sum_k W[out_feature][k] * X[k][sample]`` on
``v_mfma_f32_32x32x2_f32`` tiles, so a layer's accumulator (features in
registers, sample on the lane) is directly the B operand of the next layer.
MFMA k-step ``g`` of a 256-wide activation therefore pairs the features

    kmap_acc(g, h) = 32*(g>>4) + (g&3) + 8*((g>>2)&3) + 4*h      (h = lane>>5)

and the A operand (weights) must be packed in that k order.  This module builds
int32 gather maps ``packed[i] = flat_params[map[i]]`` (``-1`` -> 0) once per
model geometry; ``nr_pack`` (HIP) applies them every step, because the weights
change every optimizer step.

Packed layout of one layer: ``[g//4][tile][lane][g%4]`` -- one ``float4`` per
lane per (4 k-steps, 32-row tile), i.e. one fully coalesced 1 KiB wave load.

Positional-encoding k-steps pair features of the same function so that both
lane halves evaluate the same transcendental (see ``pe_feature``):
  g=0: (x, y)   g=1: (z, pad)   g=2..: sin pairs   then cos pairs.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

W = 256
WD = 128
XYZ_CH = 63
DIR_CH = 27
PE_KSTEPS = 32
DIR_KSTEPS = 16

PARAM_ORDER = (
    [(f"xyz_encoding_{i}.0.weight", f"xyz_encoding_{i}.0.bias") for i in range(1, 9)]
    + [("xyz_encoding_final.weight", "xyz_encoding_final.bias"),
       ("dir_encoding.0.weight", "dir_encoding.0.bias"),
       ("sigma.weight", "sigma.bias"),
       ("rgb.0.weight", "rgb.0.bias")])


def param_shapes():
    s = OrderedDict()
    for i in range(1, 9):
        fan = XYZ_CH if i == 1 else (W + XYZ_CH if i == 5 else W)
        s[f"xyz_encoding_{i}.0.weight"] = (W, fan)
        s[f"xyz_encoding_{i}.0.bias"] = (W,)
    s["xyz_encoding_final.weight"] = (W, W)
    s["xyz_encoding_final.bias"] = (W,)
    s["dir_encoding.0.weight"] = (WD, W + DIR_CH)
    s["dir_encoding.0.bias"] = (WD,)
    s["sigma.weight"] = (1, W)
    s["sigma.bias"] = (1,)
    s["rgb.0.weight"] = (3, WD)
    s["rgb.0.bias"] = (3,)
    return s


def param_offsets():
    """Offsets of each parameter inside the flat fp32 parameter buffer."""
    offs, o = OrderedDict(), 0
    for name, shp in param_shapes().items():
        offs[name] = (o, shp)
        o += int(np.prod(shp))
    return offs, o


N_PARAMS = param_offsets()[1]   # 595,844


# -- k-step feature maps ------------------------------------------------------
def kmap_acc(g, h):
    g = np.asarray(g)
    return 32 * (g >> 4) + (g & 3) + 8 * ((g >> 2) & 3) + 4 * np.asarray(h)


def _pe_feature(g, h, n_pairs):
    """Original Embedding channel (or -1 for padding) of PE k-step g, half h.
    n_pairs: 15 for xyz (30 sin / 30 cos), 6 for dir (12 / 12)."""
    if g == 0:
        return h                      # x | y
    if g == 1:
        return 2 if h == 0 else -1    # z | pad
    if g < 2 + n_pairs:
        m = (g - 2) + n_pairs * h
        return 3 + 6 * (m // 3) + (m % 3)   # sin(2^(m//3) * x_(m%3))
    if g < 2 + 2 * n_pairs:
        m = (g - 2 - n_pairs) + n_pairs * h
        return 6 + 6 * (m // 3) + (m % 3)   # cos(...)
    return -1


def pe_feature(g, h):
    return _pe_feature(g, h, 15)


def dir_feature(g, h):
    return _pe_feature(g, h, 6)


PE_MAP = np.array([[pe_feature(g, h) for h in (0, 1)] for g in range(PE_KSTEPS)])
DIR_MAP = np.array([[dir_feature(g, h) for h in (0, 1)] for g in range(DIR_KSTEPS)])


def _frag_coords(ksteps, ntiles):
    """(g, T, lane) for every element of a packed layer, in packed order."""
    e = np.arange(ksteps * ntiles * 64)
    grp, rem = e // (ntiles * 256), e % (ntiles * 256)
    T = rem // 256
    lane = (rem % 256) // 4
    kk = rem % 4
    return grp * 4 + kk, T, lane


def _fwd_layer_map(w_name, segs, ntiles, offs):
    """segs: list of (ksteps, kind, col_offset); kind in {'acc','pe','dir'}."""
    w_off, (rows, fan) = offs[w_name]
    parts = []
    for ksteps, kind, col0 in segs:
        g, T, lane = _frag_coords(ksteps, ntiles)
        h = lane >> 5
        row = 32 * T + (lane & 31)
        if kind == "acc":
            col = kmap_acc(g, h)
        elif kind == "pe":
            col = PE_MAP[g, h]
        else:
            col = DIR_MAP[g, h]
        ok = (col >= 0) & (row < rows)
        idx = np.where(ok, w_off + row * fan + col0 + np.maximum(col, 0), -1)
        parts.append(idx)
    # interleave segments in k order: each segment is a whole number of 4-k groups
    return np.concatenate(parts)


def _bwd_layer_map(w_name, k_out, ntiles, col0, offs):
    """Transposed layer: k runs over the layer's OUTPUT features (acc layout),
    tiles over its input features starting at column col0."""
    w_off, (rows, fan) = offs[w_name]
    g, T, lane = _frag_coords(k_out // 2, ntiles)
    h = lane >> 5
    r = kmap_acc(g, h)          # W row (output feature of the layer)
    c = col0 + 32 * T + (lane & 31)
    return w_off + r * fan + c


def _head_map(offs):
    m = []
    for i in range(1, 9):
        o, _ = offs[f"xyz_encoding_{i}.0.bias"]
        m.append(o + np.arange(W))
    m.append(offs["xyz_encoding_final.bias"][0] + np.arange(W))
    m.append(offs["dir_encoding.0.bias"][0] + np.arange(WD))
    m.append(offs["sigma.weight"][0] + np.arange(W))
    m.append(np.array([offs["sigma.bias"][0], -1, -1, -1]))
    m.append(offs["rgb.0.weight"][0] + np.arange(3 * WD))
    m.append(np.array([offs["rgb.0.bias"][0] + i for i in range(3)] + [-1]))
    return np.concatenate(m)


# offsets (floats) inside the packed buffers -- mirrored in csrc/layout.h
FWD_LAYERS = OrderedDict([
    ("L1", (PE_KSTEPS, 8)),
    ("L2", (128, 8)), ("L3", (128, 8)), ("L4", (128, 8)),
    ("L5", (PE_KSTEPS + 128, 8)),
    ("L6", (128, 8)), ("L7", (128, 8)), ("L8", (128, 8)),
    ("final", (128, 8)),
    ("dir", (128 + DIR_KSTEPS, 4)),
])
BWD_LAYERS = OrderedDict([
    ("dirT", (64, 8)), ("finalT", (128, 8)),
    ("L8T", (128, 8)), ("L7T", (128, 8)), ("L6T", (128, 8)), ("L5T", (128, 8)),
    ("L4T", (128, 8)), ("L3T", (128, 8)), ("L2T", (128, 8)),
])
HEAD_SIZE = 8 * W + W + WD + W + 4 + 3 * WD + 4   # 3080


def layer_offsets(layers):
    offs, o = OrderedDict(), 0
    for k, (ks, nt) in layers.items():
        offs[k] = o
        o += ks * nt * 64
    return offs, o


def build_fwd_map():
    offs, _ = param_offsets()
    L = lambda i: f"xyz_encoding_{i}.0.weight"  # noqa: E731
    parts = [_fwd_layer_map(L(1), [(PE_KSTEPS, "pe", 0)], 8, offs)]
    for i in (2, 3, 4):
        parts.append(_fwd_layer_map(L(i), [(128, "acc", 0)], 8, offs))
    parts.append(_fwd_layer_map(L(5), [(PE_KSTEPS, "pe", 0), (128, "acc", XYZ_CH)], 8, offs))
    for i in (6, 7, 8):
        parts.append(_fwd_layer_map(L(i), [(128, "acc", 0)], 8, offs))
    parts.append(_fwd_layer_map("xyz_encoding_final.weight", [(128, "acc", 0)], 8, offs))
    parts.append(_fwd_layer_map("dir_encoding.0.weight",
                                [(128, "acc", 0), (DIR_KSTEPS, "dir", W)], 4, offs))
    parts.append(_head_map(offs))
    m = np.concatenate(parts).astype(np.int32)
    assert m.size == layer_offsets(FWD_LAYERS)[1] + HEAD_SIZE
    return m


def build_bwd_map():
    offs, _ = param_offsets()
    L = lambda i: f"xyz_encoding_{i}.0.weight"  # noqa: E731
    parts = [_bwd_layer_map("dir_encoding.0.weight", WD, 8, 0, offs),
             _bwd_layer_map("xyz_encoding_final.weight", W, 8, 0, offs)]
    for i in (8, 7, 6):
        parts.append(_bwd_layer_map(L(i), W, 8, 0, offs))
    parts.append(_bwd_layer_map(L(5), W, 8, XYZ_CH, offs))
    for i in (4, 3, 2):
        parts.append(_bwd_layer_map(L(i), W, 8, 0, offs))
    m = np.concatenate(parts).astype(np.int32)
    assert m.size == layer_offsets(BWD_LAYERS)[1]
    return m


# -- bf16x6 split-operand layout (v_mfma_f32_16x16x32_bf16) --------------------
# Each fp32 operand is split exactly into three bf16 pieces x = hi + mid + lo
# (round-to-nearest at each step) and a product is formed from the six piece
# products whose order is at most 2^-16 (hi*hi, hi*mid, mid*hi, hi*lo, lo*hi,
# mid*mid), accumulated in fp32: fp32-level accuracy (the dropped terms are
# <= 2^-25 relative) on the bf16 matrix cores.
#
# Register layout of a wave (32 samples = two 16-sample tiles S): an
# activation of width W is W/16 feature tiles F of 16x16 accumulators; lane l
# (g = l >> 4) holds rows 4g..4g+3 of every tile for sample 16 S + (l & 15).
# k-step s of a 256-wide input (32 features) takes, for lane group g, element
# j of its B fragment from tile 2s + (j >> 2), register j & 3:
#     kmap16(s, g, j) = 32 s + 16 (j >> 2) + 4 g + (j & 3).
# Positional encodings: lane group g of k-step s holds the 8 PE "slots"
# 32 s + 8 g + j, mapped to Embedding channels by PE16_MAP / DIR16_MAP (each
# lane evaluates sin and cos of the same 4 arguments).
#
# Packed group = (k-step, half of the outputs): [piece 3][tile 8][lane 64][j 8]
# bf16 = 24 KiB; tile t covers output rows 128 half + 16 t .. +15 (lane & 15),
# k = 8 (lane >> 4) + j.  One ds_read_b128 / global_load_lds_dwordx4 moves
# one (piece, tile) fragment.  Buffer: [head fp32, HEAD_SIZE floats][groups].
def kmap16(s, g, j):
    s, g, j = np.asarray(s), np.asarray(g), np.asarray(j)
    return 32 * s + 16 * (j >> 2) + 4 * g + (j & 3)


def _pe16_channel(slot, n_args, raw):
    """Embedding channel of PE slot (32 s + 8 g + j) or -1 (pad).  Cell
    c = slot // 8 holds arguments 4c..4c+3: sin at j = 0..3, cos at j = 4..7;
    the raw coordinates fill the slots left over after the last argument.
    raw: slot -> coordinate for the raw x/y/z channels."""
    if slot in raw:
        return raw[slot]
    c, j = divmod(slot, 8)
    a = 4 * c + (j & 3)
    if a >= n_args:
        return -1
    k, coord = divmod(a, 3)
    return (3 if j < 4 else 6) + 6 * k + coord


# xyz: 30 arguments (10 freqs x 3), slots 58, 59, 62 = raw x, y, z (cell 7:
# args 28, 29 at j = 0, 1 / 4, 5); dir: 12 arguments, cells 0..3 hold args
# 3g..3g+2 (j = 0..2 sin, 4..6 cos), raw coordinate g at j = 3.
PE16_MAP = np.array([_pe16_channel(q, 30, {58: 0, 59: 1, 62: 2}) for q in range(64)])


def _dir16_channel(slot):
    g, j = divmod(slot, 8)
    if j == 3:
        return g if g < 3 else -1
    if j == 7:
        return -1
    a = 3 * g + (j & 3)
    k, coord = divmod(a, 3)
    return (3 if j < 4 else 6) + 6 * k + coord


DIR16_MAP = np.array([_dir16_channel(q) for q in range(32)])

FWD3_LAYERS = OrderedDict([          # name -> (k-steps, output halves)
    ("L1", (2, 2)),
    ("L2", (8, 2)), ("L3", (8, 2)), ("L4", (8, 2)),
    ("L5", (10, 2)),
    ("L6", (8, 2)), ("L7", (8, 2)), ("L8", (8, 2)),
    ("final", (8, 2)),
    ("dir", (9, 1)),
])
# pieces per operand: 3 for bf16x6 (hi, mid, lo), 2 for f16x3 (hi, lo; the
# same layout with one piece fewer, csrc/x3.h NR_F16), 1 for plain bf16 (the
# reduced-precision variant, csrc/x3.h NR_BF1)
NPIECES = {"bf16x6": 3, "f16x3": 2, "bf16": 1}
GROUP_BYTES = 3 * 8 * 1024
HEAD_BYTES = HEAD_SIZE * 4


def group_bytes(np_=3):
    return np_ * 8 * 1024


def fwd3_offsets(np_=3):
    """Byte offset of every layer's first group, and the total buffer size."""
    offs, o = OrderedDict(), HEAD_BYTES
    for k, (ns, nh) in FWD3_LAYERS.items():
        offs[k] = o
        o += ns * nh * group_bytes(np_)
    return offs, o


def _group_coords(n, np_=3):
    """(piece, tile, lane, j) of every piece slot of n groups, and the group."""
    e = np.arange(n * np_ * 8 * 512)
    grp = e // (np_ * 8 * 512)
    rem = e % (np_ * 8 * 512)
    piece = rem // (8 * 512)
    t = (rem % (8 * 512)) // 512
    lane = (rem % 512) // 8
    j = rem % 8
    return grp, piece, t, lane, j


def _fwd3_layer_map(w_name, segs, nhalf, offs, np_=3):
    """int32 per bf16 slot: flat_index * 4 + piece, or -1 (zero).  segs:
    (k-steps, kind, column offset); groups run k-step major, output half minor."""
    w_off, (rows, fan) = offs[w_name]
    parts = []
    for nks, kind, col0 in segs:
        grp, piece, t, lane, j = _group_coords(nks * nhalf, np_)
        s, half = grp // nhalf, grp % nhalf
        g = lane >> 4
        row = 128 * half + 16 * t + (lane & 15)
        if kind == "acc":
            col = kmap16(s, g, j)
        elif kind == "pe":
            col = PE16_MAP[32 * s + 8 * g + j]
        else:
            col = DIR16_MAP[32 * s + 8 * g + j]
        ok = (col >= 0) & (row < rows)
        parts.append(np.where(ok, (w_off + row * fan + col0 + np.maximum(col, 0)) * 4 + piece, -1))
    return np.concatenate(parts)


def build_fwd3_map(np_=3):
    """(group map over every piece slot, head map over HEAD_SIZE floats)."""
    offs, _ = param_offsets()
    L = lambda i: f"xyz_encoding_{i}.0.weight"  # noqa: E731
    lm = lambda *a: _fwd3_layer_map(*a, offs, np_)  # noqa: E731
    parts = [lm(L(1), [(2, "pe", 0)], 2)]
    for i in (2, 3, 4):
        parts.append(lm(L(i), [(8, "acc", 0)], 2))
    parts.append(lm(L(5), [(2, "pe", 0), (8, "acc", XYZ_CH)], 2))
    for i in (6, 7, 8):
        parts.append(lm(L(i), [(8, "acc", 0)], 2))
    parts.append(lm("xyz_encoding_final.weight", [(8, "acc", 0)], 2))
    parts.append(lm("dir_encoding.0.weight", [(8, "acc", 0), (1, "dir", W)], 1))
    m = np.concatenate(parts).astype(np.int32)
    assert m.size * 2 + HEAD_BYTES == fwd3_offsets(np_)[1]
    return m, _head_map(offs).astype(np.int32)


BWD3_LAYERS = OrderedDict([          # transposed layers: (k-steps over outputs, input halves)
    ("dirT", (4, 2)), ("finalT", (8, 2)),
    ("L8T", (8, 2)), ("L7T", (8, 2)), ("L6T", (8, 2)), ("L5T", (8, 2)),
    ("L4T", (8, 2)), ("L3T", (8, 2)), ("L2T", (8, 2)),
])
def bwd3_bytes(np_=3):
    return sum(ns * nh * group_bytes(np_) for ns, nh in BWD3_LAYERS.values())


BWD3_BYTES = bwd3_bytes(3)


def _bwd3_layer_map(w_name, nks, col0, offs, np_=3):
    """Transposed layer: k runs over the forward layer's OUTPUT features
    (kmap16 order), the 16 tiles (two halves of 8) over its input columns
    col0 .. col0+255."""
    w_off, (rows, fan) = offs[w_name]
    grp, piece, t, lane, j = _group_coords(nks * 2, np_)
    s, half = grp // 2, grp % 2
    k_out = kmap16(s, lane >> 4, j)
    c_in = col0 + 128 * half + 16 * t + (lane & 15)
    return (w_off + k_out * fan + c_in) * 4 + piece


def build_bwd3_map(np_=3):
    offs, _ = param_offsets()
    L = lambda i: f"xyz_encoding_{i}.0.weight"  # noqa: E731
    lm = lambda *a: _bwd3_layer_map(*a, offs, np_)  # noqa: E731
    parts = [lm("dir_encoding.0.weight", 4, 0), lm("xyz_encoding_final.weight", 8, 0)]
    for i in (8, 7, 6):
        parts.append(lm(L(i), 8, 0))
    parts.append(lm(L(5), 8, XYZ_CH))
    for i in (4, 3, 2):
        parts.append(lm(L(i), 8, 0))
    m = np.concatenate(parts).astype(np.int32)
    assert m.size * 2 == bwd3_bytes(np_)
    return m
