// Fused MLP backward, data-gradient chain (autograd of models/nerf.py:83-124).
//
// Same geometry as the forward: one wave carries 32 samples backwards through
// every layer in transposed form D[in_feature][sample] = W^T[in][out] dz[out][sample]
// on v_mfma_f32_32x32x2_f32, with the transposed weights pre-packed in fragment
// order (packing.py BWD_LAYERS).  ReLU masks come from the saved activations.
// Every layer's pre-activation gradient dz is written out row-major [n][width]
// for the weight-gradient GEMMs (wgrad.hip).
#include "layout.h"

namespace {

constexpr int kWaves = 4;

template <int NT>
__device__ __forceinline__ void ld_wgrp(const float* __restrict__ w, int grp, int lane,
                                        f32x4 (&dst)[NT]) {
    const f32x4* p = reinterpret_cast<const f32x4*>(w) + (size_t)grp * NT * 64 + lane;
#pragma unroll
    for (int t = 0; t < NT; ++t) dst[t] = p[t * 64];
}

template <int KS, int NT, typename GetB>
__device__ __forceinline__ void mm_acc(const float* __restrict__ w, int lane, f32x16 (&acc)[NT],
                                       GetB getb) {
    static_assert(KS % 8 == 0, "k-steps must be a multiple of 8");
    f32x4 wa[NT], wb[NT];
    ld_wgrp<NT>(w, 0, lane, wa);
#pragma unroll
    for (int grp = 0; grp < KS / 4; grp += 2) {
        ld_wgrp<NT>(w, grp + 1, lane, wb);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const float b = getb(grp * 4 + kk);
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = nr_mfma32(wa[t][kk], b, acc[t]);
        }
        if (grp + 2 < KS / 4) ld_wgrp<NT>(w, grp + 2, lane, wa);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const float b = getb(grp * 4 + 4 + kk);
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = nr_mfma32(wb[t][kk], b, acc[t]);
        }
    }
}

template <int NT>
__device__ __forceinline__ void zero(f32x16 (&acc)[NT]) {
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
}

// acc *= [h > 0] with h the saved post-ReLU activation row (threshold_backward)
template <int NT>
__device__ __forceinline__ void relu_mask(f32x16 (&acc)[NT], const float* __restrict__ row, int h) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(row + 32 * t + 8 * q + 4 * h);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[t][4 * q + e] = v[e] > 0.f ? acc[t][4 * q + e] : 0.f;
        }
}

template <int NT>
__device__ __forceinline__ void store_rows(const f32x16 (&acc)[NT], float* __restrict__ row, int h) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            f32x4 v = {acc[t][4 * q + 0], acc[t][4 * q + 1], acc[t][4 * q + 2], acc[t][4 * q + 3]};
            *reinterpret_cast<f32x4*>(row + 32 * t + 8 * q + 4 * h) = v;
        }
}

struct BwdArgs {
    const float* packed_bwd;
    const float* packed_fwd;   // head block: sigma / rgb weights
    const float* out;          // (n,4) forward output [rgb, sigma]
    const float* g_out;        // (n,4) d[rgb, sigma]
    const float* save;
    int n;
    float* grad;
};

__global__ void __launch_bounds__(64 * kWaves, 1) mlp_bwd_kernel(BwdArgs a) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int h = lane >> 5;
    const int s_raw = (blockIdx.x * kWaves + wave) * 32 + (lane & 31);
    const bool valid = s_raw < a.n;
    const int s = valid ? s_raw : a.n - 1;
    const float* PB = a.packed_bwd;
    const float* H = a.packed_fwd + NR_F_HEAD;
    NrSave sv(const_cast<float*>(a.save), a.n);
    NrGrad gd(a.grad, a.n);

    const f32x4 go = *reinterpret_cast<const f32x4*>(a.g_out + (size_t)s * 4);
    const f32x4 yo = *reinterpret_cast<const f32x4*>(a.out + (size_t)s * 4);
    // sigmoid backward: grad * (1 - y) * y  (ATen sigmoid_backward)
    float dzr[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) dzr[c] = go[c] * (1.f - yo[c]) * yo[c];
    const float dsig = go[3];
    if (valid && h == 0) {
        f32x4 v = {dzr[0], dzr[1], dzr[2], dsig};
        *reinterpret_cast<f32x4*>(gd.dhead + (size_t)s * 4) = v;
    }

    // d hdir = W_rgb^T dz_rgb, masked by the dir-layer ReLU -> dz_dir (128)
    f32x16 C[4];
    {
        const float* hrow = sv.hdir + (size_t)s * 128;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int f = 32 * t + 8 * q + 4 * h;
                const f32x4 hv = *reinterpret_cast<const f32x4*>(hrow + f);
                const f32x4 w0 = *reinterpret_cast<const f32x4*>(H + NR_H_WRGB + f);
                const f32x4 w1 = *reinterpret_cast<const f32x4*>(H + NR_H_WRGB + 128 + f);
                const f32x4 w2 = *reinterpret_cast<const f32x4*>(H + NR_H_WRGB + 256 + f);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float d = fmaf(w2[e], dzr[2], fmaf(w1[e], dzr[1], w0[e] * dzr[0]));
                    C[t][4 * q + e] = hv[e] > 0.f ? d : 0.f;
                }
            }
        if (valid) store_rows<4>(C, gd.dzdir + (size_t)s * 128, h);
    }

    f32x16 A[8], B[8];
    // d feat = W_dir[:, :256]^T dz_dir   (xyz_encoding_final has no activation)
    zero<8>(A);
    mm_acc<64, 8>(PB + NR_B_DIRT, lane, A, [&](int g) { return C[g >> 4][g & 15]; });
    if (valid) store_rows<8>(A, gd.dfeat + (size_t)s * 256, h);

    // d h8 = W_final^T dfeat + W_sigma^T dsigma, masked by h8
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x4 w = *reinterpret_cast<const f32x4*>(H + NR_H_WSIG + 32 * t + 8 * q + 4 * h);
#pragma unroll
            for (int e = 0; e < 4; ++e) B[t][4 * q + e] = w[e] * dsig;
        }
    mm_acc<128, 8>(PB + NR_B_FINALT, lane, B, [&](int g) { return A[g >> 4][g & 15]; });
    relu_mask<8>(B, sv.h[7] + (size_t)s * 256, h);
    if (valid) store_rows<8>(B, gd.dz[7] + (size_t)s * 256, h);

#define NR_BACK(DST, SRC, LOFF, L)                                                    \
    zero<8>(DST);                                                                      \
    mm_acc<128, 8>(PB + LOFF, lane, DST, [&](int g) { return SRC[g >> 4][g & 15]; });  \
    relu_mask<8>(DST, sv.h[L - 1] + (size_t)s * 256, h);                               \
    if (valid) store_rows<8>(DST, gd.dz[L - 1] + (size_t)s * 256, h);

    NR_BACK(A, B, NR_B_L8T, 7)   // dz7 = (W8^T dz8) * [h7 > 0]
    NR_BACK(B, A, NR_B_L7T, 6)
    NR_BACK(A, B, NR_B_L6T, 5)
    NR_BACK(B, A, NR_B_L5T, 4)   // through the h4 columns of the skip layer
    NR_BACK(A, B, NR_B_L4T, 3)
    NR_BACK(B, A, NR_B_L3T, 2)
    NR_BACK(A, B, NR_B_L2T, 1)
#undef NR_BACK
}

}  // namespace

NR_API int nr_mlp_bwd(const float* packed_bwd, const float* packed_fwd, const float* out,
                      const float* g_out, const float* save, int64_t n, float* grad_ws,
                      void* stream) {
    NR_REQUIRE(n >= 0 && n < (int64_t)1 << 31, "nr_mlp_bwd: n out of range");
    if (n == 0) return 0;
    NR_REQUIRE(packed_bwd && packed_fwd && out && g_out && save && grad_ws,
               "nr_mlp_bwd: null pointer");
    NR_REQUIRE((((uintptr_t)out | (uintptr_t)g_out | (uintptr_t)save | (uintptr_t)grad_ws |
                 (uintptr_t)packed_bwd | (uintptr_t)packed_fwd) & 15) == 0,
               "nr_mlp_bwd: pointers must be 16-byte aligned");
    BwdArgs a{packed_bwd, packed_fwd, out, g_out, save, (int)n, grad_ws};
    const int blocks = (int)((n + 32 * kWaves - 1) / (32 * kWaves));
    mlp_bwd_kernel<<<blocks, 64 * kWaves, 0, (hipStream_t)stream>>>(a);
    NR_LAUNCH_CHECK("nr_mlp_bwd");
    return 0;
}
