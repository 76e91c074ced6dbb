// Packed-weight and saved-activation layouts.  Mirrors nerf_pl_amd/packing.py
// (checked by tests/test_packing.py through nr_layout_query()).
#pragma once
#include "common.h"

// packed layer size in floats: ksteps * tiles * 64 lanes
#define NR_PL(ks, nt) ((ks) * (nt) * 64)

// ---- forward packed buffer -------------------------------------------------
#define NR_F_L1 0
#define NR_F_L2 (NR_F_L1 + NR_PL(32, 8))
#define NR_F_L3 (NR_F_L2 + NR_PL(128, 8))
#define NR_F_L4 (NR_F_L3 + NR_PL(128, 8))
#define NR_F_L5 (NR_F_L4 + NR_PL(128, 8))
#define NR_F_L6 (NR_F_L5 + NR_PL(160, 8))
#define NR_F_L7 (NR_F_L6 + NR_PL(128, 8))
#define NR_F_L8 (NR_F_L7 + NR_PL(128, 8))
#define NR_F_FINAL (NR_F_L8 + NR_PL(128, 8))
#define NR_F_DIR (NR_F_FINAL + NR_PL(128, 8))
#define NR_F_HEAD (NR_F_DIR + NR_PL(144, 4))
// head block (floats, relative to NR_F_HEAD)
#define NR_H_BIAS(l) (((l) - 1) * 256)   // l = 1..8
#define NR_H_BFINAL (8 * 256)
#define NR_H_BDIR (NR_H_BFINAL + 256)
#define NR_H_WSIG (NR_H_BDIR + 128)
#define NR_H_BSIG (NR_H_WSIG + 256)
#define NR_H_WRGB (NR_H_BSIG + 4)
#define NR_H_BRGB (NR_H_WRGB + 384)
#define NR_H_SIZE (NR_H_BRGB + 4)
#define NR_F_TOTAL (NR_F_HEAD + NR_H_SIZE)

// ---- backward (transposed) packed buffer ----------------------------------
#define NR_B_DIRT 0
#define NR_B_FINALT (NR_B_DIRT + NR_PL(64, 8))
#define NR_B_L8T (NR_B_FINALT + NR_PL(128, 8))
#define NR_B_L7T (NR_B_L8T + NR_PL(128, 8))
#define NR_B_L6T (NR_B_L7T + NR_PL(128, 8))
#define NR_B_L5T (NR_B_L6T + NR_PL(128, 8))
#define NR_B_L4T (NR_B_L5T + NR_PL(128, 8))
#define NR_B_L3T (NR_B_L4T + NR_PL(128, 8))
#define NR_B_L2T (NR_B_L3T + NR_PL(128, 8))
#define NR_B_TOTAL (NR_B_L2T + NR_PL(128, 8))

// ---- saved activations / gradients: BLOCK-NATIVE layout ------------------
// Samples are grouped in blocks of 32 (one wave).  A width-W activation of a
// block is stored exactly as the wave's accumulators hold it: feature
// f = 32t + 8q + 4h + e of sample j (lane l = 32h + j) lives at
//     [block][t][q][lane][e]        (W*32 floats per block)
// so every wave store/load instruction moves one contiguous 1 KiB.
// PE segments hold the packed k-step values pe[g] as [block][g/4][lane][g%4].
// ReLU masks are bits: word d of a lane covers tiles 2d, 2d+1 (bit 16*(t&1)+r).
#define NR_BLK 32
#define NR_NATIVE(w) ((w) * NR_BLK)
// blocks held by a save / gradient buffer of n samples: padded to whole
// 4-wave workgroups, so a workgroup's dead waves store into padding instead
// of branching around their stores (ops.n_blocks)
__host__ __device__ __forceinline__ int64_t nr_blocks_pad(int64_t n) { return ((n + 127) / 128) * 4; }
#define NR_MASK_LAYERS 9          // h1..h8, hdir
// PE, h1..h8, hdir, dir PE, masks.  xyz_encoding_final's output (feat) is
// not saved: the weight gradient forms the dir layer's feat columns from h8
// (wgrad.hip task 10, nr_wgrad_dir_feat)
#define NR_SAVE_PER_BLOCK (NR_NATIVE(64) + 8 * NR_NATIVE(256) + NR_NATIVE(128) + NR_NATIVE(32) + \
                           NR_MASK_LAYERS * 256)

//   dz1..dz8, dzdir (128), dhead [block][j][4] = (dz_rgb, dsigma).  dfeat (the
//   gradient of xyz_encoding_final's output) is not stored: that layer's weight
//   gradient is W_dir[:, :256]^T G, G = sum dz_dir h8^T (wgrad.hip task 10)
#define NR_GRAD_PER_BLOCK (8 * NR_NATIVE(256) + NR_NATIVE(128) + NR_BLK * 4)

// keep x where mask bit b of word w is set, else +0 (ReLU backward)
__device__ __forceinline__ float nr_mask_bit(float x, uint32_t w, int b) {
    // signed one-bit field extract: 0 or all ones (v_bfe_i32 + v_and)
    const uint32_t keep = (uint32_t)__builtin_amdgcn_sbfe((int)w, b, 1);
    return __uint_as_float(__float_as_uint(x) & keep);
}

// On-demand segment addresses (keeps scalar register pressure low in the
// fully unrolled kernels): offsets in floats from the buffer base, nb blocks.
__host__ __device__ __forceinline__ int64_t nr_sv_pe(int64_t) { return 0; }
__host__ __device__ __forceinline__ int64_t nr_sv_h(int l, int64_t nb) {
    return (NR_NATIVE(64) + (int64_t)l * NR_NATIVE(256)) * nb;
}
__host__ __device__ __forceinline__ int64_t nr_sv_hdir(int64_t nb) { return nr_sv_h(8, nb); }
__host__ __device__ __forceinline__ int64_t nr_sv_dirpe(int64_t nb) {
    return nr_sv_hdir(nb) + NR_NATIVE(128) * nb;
}
__host__ __device__ __forceinline__ int64_t nr_sv_mask(int64_t nb) {
    return nr_sv_dirpe(nb) + NR_NATIVE(32) * nb;
}
// f16x3 statistics after the saved activations of a training forward:
// NR_STATS floats [l] = max |true gradient| of gradient segment l (0..7
// dz1..dz8, 8 dfeat, 9 dzdir, 10 dhead), then the per-wave maxima
// [l][nb] they reduce (mlp_bwd3.hip writes those with plain stores -- no
// contended atomics -- and wgrad.hip reduces them)
#define NR_STATS 16
#define NR_STAT_SEGS 11
__host__ __device__ __forceinline__ int64_t nr_sv_stats(int64_t nb) { return NR_SAVE_PER_BLOCK * nb; }
__host__ __device__ __forceinline__ int64_t nr_stats_floats(int64_t nb) {
    return NR_STATS + NR_STAT_SEGS * nb;
}
__host__ __device__ __forceinline__ int64_t nr_gd_dz(int l, int64_t nb) {   // l = 0..7
    return (int64_t)l * NR_NATIVE(256) * nb;
}
__host__ __device__ __forceinline__ int64_t nr_gd_dzdir(int64_t nb) { return nr_gd_dz(8, nb); }
__host__ __device__ __forceinline__ int64_t nr_gd_dhead(int64_t nb) {
    return nr_gd_dzdir(nb) + NR_NATIVE(128) * nb;
}

// wave-level helpers shared by the fused kernels ---------------------------
// Fused-MLP layer: acc[t] += sum_g Wpacked[g][t] * B(g), g in [0, KS).
// Weights stream as one float4 wave load per (4 k-steps x tile), double
// buffered one group ahead.  side(grp) runs right after the prefetch of each
// group is issued: the kernels use it to spread the previous layer's output
// stores over this layer, so that no weight-load wait (vmcnt counts stores and
// loads together, in issue order) sits behind a burst of stores.
template <int NT>
__device__ __forceinline__ void nr_ld_wgrp(const float* __restrict__ w, int grp, int lane,
                                           f32x4 (&dst)[NT]) {
    const f32x4* p = reinterpret_cast<const f32x4*>(w) + (size_t)grp * NT * 64 + lane;
#pragma unroll
    for (int t = 0; t < NT; ++t) dst[t] = p[t * 64];
}

// load group grp of a packed layer (N tiles) into the first N slots of dst
template <int N>
__device__ __forceinline__ void nr_ld_into(const float* __restrict__ w, int grp, int lane,
                                           f32x4 (&dst)[8]) {
    const f32x4* p = reinterpret_cast<const f32x4*>(w) + (size_t)grp * N * 64 + lane;
#pragma unroll
    for (int t = 0; t < N; ++t) dst[t] = p[t * 64];
}

struct NrNoSide {
    __device__ __forceinline__ void operator()(int) const {}
};

// Chained form: on entry wa[0..NT) already holds (or is loading) group 0 of
// w; when w_next != nullptr the first group of the next layer (NTN tiles) is
// prefetched into wa as soon as wa is free, so no layer starts with a cold
// L2/MALL round trip.
template <int KS, int NT, int NTN, typename GetB, typename Side = NrNoSide>
__device__ __forceinline__ void nr_mm_chain(const float* __restrict__ w,
                                            const float* __restrict__ w_next, int lane,
                                            f32x16 (&acc)[NT], f32x4 (&wa)[8], GetB getb,
                                            Side side = Side()) {
    static_assert(KS % 8 == 0, "k-steps must be a multiple of 8");
    f32x4 wb[NT];
#pragma unroll
    for (int grp = 0; grp < KS / 4; grp += 2) {
        nr_ld_wgrp<NT>(w, grp + 1, lane, wb);
        side(grp);
        __builtin_amdgcn_sched_barrier(0);   // keep the prefetch a full group ahead
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const float b = getb(grp * 4 + kk);
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = nr_mfma32(wa[t][kk], b, acc[t]);
        }
        if (grp + 2 < KS / 4) nr_ld_into<NT>(w, grp + 2, lane, wa);
        else if (w_next != nullptr) nr_ld_into<NTN>(w_next, 0, lane, wa);
        side(grp + 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const float b = getb(grp * 4 + 4 + kk);
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = nr_mfma32(wb[t][kk], b, acc[t]);
        }
    }
}

template <int NT>
__device__ __forceinline__ void nr_ld_first(const float* __restrict__ w, int lane, f32x4 (&wa)[8]) {
    nr_ld_into<NT>(w, 0, lane, wa);
}

// piece p (= 4t + q) of a block-native store: one float4 per lane
template <int NT>
__device__ __forceinline__ void store_native_piece(const f32x16 (&acc)[NT], int p,
                                                   float* __restrict__ blk, int lane) {
    const int t = p >> 2, q = p & 3;
    f32x4 v = {acc[t][4 * q + 0], acc[t][4 * q + 1], acc[t][4 * q + 2], acc[t][4 * q + 3]};
    *reinterpret_cast<f32x4*>(blk + (p * 64 + lane) * 4) = v;
}
// NR_F32_ROWS (A/B knob): the exact-fp32 full-graph forward saves rows
#ifndef NR_F32_ROWS
#define NR_F32_ROWS 1
#endif
// piece p (= 4t + q) of a width-W activation as sample-major rows (the fp32
// full-graph training save, like x3.h store_row): lane (h, j) holds features
// 32t + 8q + 4h .. +3 of sample j (nr_acc_row), stored at row j of the block's
// 32 rows of W floats, so the weight gradient can gather a sample's row whole
template <int NT>
__device__ __forceinline__ void store_row_piece(const f32x16 (&acc)[NT], int p, int W,
                                                float* __restrict__ rows, int lane) {
    const int t = p >> 2, q = p & 3;
    f32x4 v = {acc[t][4 * q + 0], acc[t][4 * q + 1], acc[t][4 * q + 2], acc[t][4 * q + 3]};
    *reinterpret_cast<f32x4*>(rows + (lane & 31) * W + 32 * t + 8 * q + 4 * (lane >> 5)) = v;
}
template <int NT>
__device__ __forceinline__ void store_rows(const f32x16 (&acc)[NT], float* __restrict__ rows, int lane) {
#pragma unroll
    for (int p = 0; p < 4 * NT; ++p) store_row_piece<NT>(acc, p, 32 * NT, rows, lane);
}

template <int NT>
__device__ __forceinline__ void store_native(const f32x16 (&acc)[NT], float* __restrict__ blk,
                                             int lane) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            f32x4 v = {acc[t][4 * q + 0], acc[t][4 * q + 1], acc[t][4 * q + 2], acc[t][4 * q + 3]};
            *reinterpret_cast<f32x4*>(blk + ((t * 4 + q) * 64 + lane) * 4) = v;
        }
}

template <int NT>
__device__ __forceinline__ void store_mask(const f32x16 (&acc)[NT], uint32_t* __restrict__ m,
                                           int lane) {
    // acc is post-ReLU (exactly +0 or positive): bit = (bits(x) != 0), VALU only
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
            w[t >> 1] |= min(__float_as_uint(acc[t][r]), 1u) << (16 * (t & 1) + r);
    *reinterpret_cast<uint4*>(m + lane * 4) = make_uint4(w[0], w[1], w[2], w[3]);
}
