// Fused MLP backward, data-gradient chain (autograd of models/nerf.py:83-124).
//
// Same geometry as the forward: one wave carries 32 samples backwards through
// every layer in transposed form D[in_feature][sample] = W^T[in][out] dz[out][sample]
// on v_mfma_f32_32x32x2_f32, with the transposed weights pre-packed in fragment
// order (packing.py BWD_LAYERS).  ReLU masks are the forward's bit masks.
// Every layer's pre-activation gradient dz is written out in the block-native
// layout (layout.h) for the weight-gradient GEMMs (wgrad.hip).
#include "layout.h"

namespace {

constexpr int kWaves = 4;

template <int NT>
__device__ __forceinline__ void zero(f32x16 (&acc)[NT]) {
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
}

// ReLU backward with the forward's mask bits (one uint4 per lane per layer)
template <int NT>
__device__ __forceinline__ void relu_mask(f32x16 (&acc)[NT], uint4 m) {
    const uint32_t w[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = nr_mask_bit(acc[t][r], w[t >> 1], 16 * (t & 1) + r);
}

struct BwdArgs {
    const float* packed_bwd;
    const float* head;         // fp32 head block: sigma / rgb weights
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
    const int blk = blockIdx.x * kWaves + wave;
    const int nb = (int)nr_blocks_pad(a.n);    // segment stride (padded)
    if (blk >= (a.n + 31) / 32) return;         // no barriers in this kernel
    const int s_raw = blk * 32 + (lane & 31);
    const bool valid = s_raw < a.n;
    const int s = valid ? s_raw : a.n - 1;
    const float* PB = a.packed_bwd;
    const float* H = a.head;
    const float* SV = a.save;
    float* const GD = a.grad;
    // The wave's 9 ReLU-mask words per lane arrive by LDS-DMA up front (one
    // HBM round trip per wave); per-layer HBM loads would otherwise sit in
    // front of every weight-load wait (vmcnt retires in issue order).
    __shared__ __attribute__((aligned(16))) uint4 smask[kWaves][NR_MASK_LAYERS][64];
    {
        const uint4* gm = reinterpret_cast<const uint4*>(SV + nr_sv_mask(nb)) +
                          (size_t)blk * NR_MASK_LAYERS * 64 + lane;
#pragma unroll
        for (int l = 0; l < NR_MASK_LAYERS; ++l)
            __builtin_amdgcn_global_load_lds(
                (const void*)(gm + l * 64),
                (__attribute__((address_space(3))) void*)&smask[wave][l][0], 16, 0, 0);
    }
    const uint4* mask = &smask[wave][0][lane];   // [layer * 64]

    f32x4 wq[8];                 // weight group in flight across layer boundaries
    nr_ld_first<8>(PB + NR_B_DIRT, lane, wq);
    const f32x4 go = *reinterpret_cast<const f32x4*>(a.g_out + (size_t)s * 4);
    const f32x4 yo = *reinterpret_cast<const f32x4*>(a.out + (size_t)s * 4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // masks landed in LDS (own wave only)
    // sigmoid backward: grad * (1 - y) * y  (ATen sigmoid_backward); tail lanes -> 0
    float dzr[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) dzr[c] = valid ? go[c] * (1.f - yo[c]) * yo[c] : 0.f;
    const float dsig = valid ? go[3] : 0.f;
    if (h == 0) {
        f32x4 v = {dzr[0], dzr[1], dzr[2], dsig};
        *reinterpret_cast<f32x4*>(GD + nr_gd_dhead(nb) + ((size_t)blk * 32 + (lane & 31)) * 4) = v;
    }

    // d hdir = W_rgb^T dz_rgb, masked by the dir-layer ReLU -> dz_dir (128)
    f32x16 C[4];
    {
        const uint4 mk = mask[8 * 64];
        const uint32_t mw[2] = {mk.x, mk.y};
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int f = 32 * t + 8 * q + 4 * h;
                const f32x4 w0 = *reinterpret_cast<const f32x4*>(H + NR_H_WRGB + f);
                const f32x4 w1 = *reinterpret_cast<const f32x4*>(H + NR_H_WRGB + 128 + f);
                const f32x4 w2 = *reinterpret_cast<const f32x4*>(H + NR_H_WRGB + 256 + f);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float d = fmaf(w2[e], dzr[2], fmaf(w1[e], dzr[1], w0[e] * dzr[0]));
                    C[t][4 * q + e] = nr_mask_bit(d, mw[t >> 1], 16 * (t & 1) + 4 * q + e);
                }
            }
    }

    f32x16 A[8], B[8];
    // each layer's dz is written while the next backward layer runs (side hook)
    auto dzseg = [&](int l) { return GD + nr_gd_dz(l, nb) + (size_t)blk * NR_NATIVE(256); };
    auto side8 = [&](const f32x16 (&X)[8], float* dst) {
        return [&X, dst, lane](int grp) { if (grp < 32) store_native_piece<8>(X, grp, dst, lane); };
    };
    // d feat = W_dir[:, :256]^T dz_dir   (xyz_encoding_final has no activation); stores dz_dir
    zero<8>(A);
    {
        float* cdst = GD + nr_gd_dzdir(nb) + (size_t)blk * NR_NATIVE(128);
        nr_mm_chain<64, 8, 8>(PB + NR_B_DIRT, PB + NR_B_FINALT, lane, A, wq,
                              [&](int g) { return C[g >> 4][g & 15]; },
                              [&](int grp) { store_native_piece<4>(C, grp, cdst, lane); });
    }

    // d h8 = W_final^T dfeat + W_sigma^T dsigma, masked by h8; stores dfeat
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x4 w = *reinterpret_cast<const f32x4*>(H + NR_H_WSIG + 32 * t + 8 * q + 4 * h);
#pragma unroll
            for (int e = 0; e < 4; ++e) B[t][4 * q + e] = w[e] * dsig;
        }
    {
        const uint4 mk = mask[7 * 64];
        nr_mm_chain<128, 8, 8>(PB + NR_B_FINALT, PB + NR_B_L8T, lane, B, wq,
                               [&](int g) { return A[g >> 4][g & 15]; }, side8(A, dzseg(8)));
        relu_mask<8>(B, mk);
    }

#define NR_BACK(DST, SRC, LOFF, NEXT, L)                                                     \
    {                                                                                         \
        const uint4 mk = mask[(L - 1) * 64];                                                  \
        zero<8>(DST);                                                                         \
        nr_mm_chain<128, 8, 8>(PB + LOFF, NEXT, lane, DST, wq,                                \
                               [&](int g) { return SRC[g >> 4][g & 15]; },                    \
                               side8(SRC, dzseg(L)));                                         \
        relu_mask<8>(DST, mk);                                                                \
    }

    NR_BACK(A, B, NR_B_L8T, PB + NR_B_L7T, 7)   // dz7 = (W8^T dz8) * [h7 > 0], stores dz8
    NR_BACK(B, A, NR_B_L7T, PB + NR_B_L6T, 6)
    NR_BACK(A, B, NR_B_L6T, PB + NR_B_L5T, 5)
    NR_BACK(B, A, NR_B_L5T, PB + NR_B_L4T, 4)   // through the h4 columns of the skip layer
    NR_BACK(A, B, NR_B_L4T, PB + NR_B_L3T, 3)
    NR_BACK(B, A, NR_B_L3T, PB + NR_B_L2T, 2)
    NR_BACK(A, B, NR_B_L2T, nullptr, 1)         // stores dz2, leaves dz1 in A
#undef NR_BACK
    store_native<8>(A, dzseg(0), lane);
}

}  // namespace

NR_API int nr_mlp_bwd(const float* packed_bwd, const float* head, const float* out,
                      const float* g_out, const float* save, int64_t n, float* grad_ws,
                      void* stream) {
    NR_REQUIRE(n >= 0 && n < (int64_t)1 << 31, "nr_mlp_bwd: n out of range");
    if (n == 0) return 0;
    NR_REQUIRE(packed_bwd && head && out && g_out && save && grad_ws,
               "nr_mlp_bwd: null pointer");
    NR_REQUIRE((((uintptr_t)out | (uintptr_t)g_out | (uintptr_t)save | (uintptr_t)grad_ws |
                 (uintptr_t)packed_bwd | (uintptr_t)head) & 15) == 0,
               "nr_mlp_bwd: pointers must be 16-byte aligned");
    BwdArgs a{packed_bwd, head, out, g_out, save, (int)n, grad_ws};
    const int blocks = (int)((n + 32 * kWaves - 1) / (32 * kWaves));
    mlp_bwd_kernel<<<blocks, 64 * kWaves, 0, (hipStream_t)stream>>>(a);
    NR_LAUNCH_CHECK("nr_mlp_bwd");
    return 0;
}
