// Fused MLP backward, data-gradient chain, on bf16x6 split-operand MFMA
// (autograd of models/nerf.py:83-124; same contract and outputs as
// mlp_bwd.hip).  Four waves x 32 samples per workgroup carry the gradient
// backwards through the transposed layers D[in][sample] = W^T[in][out]
// dz[out][sample]; the transposed weights (packing.BWD3_LAYERS, 136 k-groups
// of 24 KiB) stream through the LDS ring of x3.h.  ReLU masks are the
// forward's bit masks, staged in LDS by LDS-DMA; every layer's dz is written
// block-native for the weight-gradient GEMMs (wgrad.hip).
#include "x3.h"

namespace {

using namespace x3;

constexpr int kDirT = 0, kFinalT = 8, kL8T = 24, kL7T = 40, kL6T = 56, kL5T = 72, kL4T = 88,
              kL3T = 104, kL2T = 120, kQ = 136;
constexpr int kMaskBytes = kWaves * NR_MASK_LAYERS * 64 * 16;
constexpr int kLdsBytes = kRingBytes + kMaskBytes;

struct BwdTab {
    __host__ __device__ static constexpr int tiles(int) { return 8; }
    __host__ __device__ static constexpr int64_t off(int q) { return (int64_t)q * 8 * 3072; }
};
static_assert(BwdTab::off(kQ) == 3342336, "packed size must match packing.BWD3_BYTES");

template <int NT>
__device__ __forceinline__ void zero(f32x16 (&acc)[8]) {
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
}

template <int NT>
__device__ __forceinline__ void relu_mask(f32x16 (&acc)[8], uint4 m) {
    const uint32_t w[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = nr_mask_bit(acc[t][r], w[t >> 1], 16 * (t & 1) + r);
}

struct Bwd3Args {
    const char* packed;        // packing.build_bwd3_map layout
    const float* head;         // fp32 head block (sigma / rgb weights)
    const float* out; const float* g_out; const float* save;
    int n;
    float* grad;
};

__global__ void __launch_bounds__(64 * kWaves, 1) mlp_bwd3_kernel(Bwd3Args a) {
    __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int h = lane >> 5;
    const int blk = blockIdx.x * kWaves + wave;
    const int nb = (a.n + 31) / 32;
    const bool live = blk < nb;                  // dead waves still feed the ring and barriers
    const int bk = live ? blk : nb - 1;
    const int s_raw = bk * 32 + (lane & 31);
    const bool valid = live && s_raw < a.n;
    const int s = s_raw < a.n ? s_raw : a.n - 1;
    const char* PB = a.packed;
    const float* H = a.head;
    const float* SV = a.save;
    float* const GD = a.grad;

    // ReLU mask words (9 layers) by LDS-DMA, issued before the ring so the
    // ring's counted waits cover them
    uint4* smask = reinterpret_cast<uint4*>(smem + kRingBytes) + wave * NR_MASK_LAYERS * 64;
    {
        const uint4* gm = reinterpret_cast<const uint4*>(SV + nr_sv_mask(nb)) +
                          (size_t)bk * NR_MASK_LAYERS * 64 + lane;
#pragma unroll
        for (int l = 0; l < NR_MASK_LAYERS; ++l)
            __builtin_amdgcn_global_load_lds(
                (const void*)(gm + l * 64),
                (__attribute__((address_space(3))) void*)(smask + l * 64), 16, 0, 0);
    }
    prologue<BwdTab, kQ>(PB, smem, wave, lane);
    const f32x4 go = *reinterpret_cast<const f32x4*>(a.g_out + (size_t)s * 4);
    const f32x4 yo = *reinterpret_cast<const f32x4*>(a.out + (size_t)s * 4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // masks (and the prologue) landed
    const uint4* mask = smask + lane;                   // [layer * 64]
    Frag f0;                                            // tile-0 fragments of the next k-group
    enter<BwdTab, 0, kQ>(smem, lane, f0);

    float dzr[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) dzr[c] = valid ? go[c] * (1.f - yo[c]) * yo[c] : 0.f;
    const float dsig = valid ? go[3] : 0.f;
    if (live && h == 0) {
        f32x4 v = {dzr[0], dzr[1], dzr[2], dsig};
        *reinterpret_cast<f32x4*>(GD + nr_gd_dhead(nb) + ((size_t)bk * 32 + (lane & 31)) * 4) = v;
    }

    // d hdir = W_rgb^T dz_rgb, masked by the dir-layer ReLU -> dz_dir (128)
    f32x16 C[8];
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
    auto dzseg = [&](int l) { return GD + nr_gd_dz(l, nb) + (size_t)bk * NR_NATIVE(256); };
    auto side8 = [&](const f32x16 (&X)[8], float* dst) {
        return [&X, dst, lane, live](auto gc) {
            constexpr int g = decltype(gc)::value;
            if (!live) return;
            store_native_piece<8>(X, 2 * g, dst, lane);
            store_native_piece<8>(X, 2 * g + 1, dst, lane);
        };
    };
    auto from_acc = [](const f32x16 (&X)[8]) {
        return [&X](auto gc, float (&x)[8]) { acc_group<decltype(gc)::value>(X, x); };
    };

    // d feat = W_dir[:, :256]^T dz_dir (xyz_encoding_final has no activation); stores dz_dir
    zero<8>(A);
    {
        float* cdst = GD + nr_gd_dzdir(nb) + (size_t)bk * NR_NATIVE(128);
        auto gb = from_acc(C);
        auto sd = [&](auto gc) {
            constexpr int g = decltype(gc)::value;
            if (!live) return;
            store_native_piece<4>(reinterpret_cast<const f32x16(&)[4]>(C), 2 * g, cdst, lane);
            store_native_piece<4>(reinterpret_cast<const f32x16(&)[4]>(C), 2 * g + 1, cdst, lane);
        };
        segment<BwdTab, kDirT, 0, 8, 8, kQ>(PB, smem, wave, lane, A, gb, sd, f0);
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
        auto gb = from_acc(A);
        auto sd = side8(A, dzseg(8));
        segment<BwdTab, kFinalT, 0, 16, 8, kQ>(PB, smem, wave, lane, B, gb, sd, f0);
        relu_mask<8>(B, mk);
    }
#define NR_BACK3(DST, SRC, Q0, L)                                              \
    {                                                                          \
        const uint4 mk = mask[(L - 1) * 64];                                   \
        zero<8>(DST);                                                          \
        auto gb = from_acc(SRC);                                               \
        auto sd = side8(SRC, dzseg(L));                                        \
        segment<BwdTab, Q0, 0, 16, 8, kQ>(PB, smem, wave, lane, DST, gb, sd, f0); \
        relu_mask<8>(DST, mk);                                                 \
    }
    NR_BACK3(A, B, kL8T, 7)   // dz7 = (W8^T dz8) * [h7 > 0], stores dz8
    NR_BACK3(B, A, kL7T, 6)
    NR_BACK3(A, B, kL6T, 5)
    NR_BACK3(B, A, kL5T, 4)   // through the h4 columns of the skip layer
    NR_BACK3(A, B, kL4T, 3)
    NR_BACK3(B, A, kL3T, 2)
    NR_BACK3(A, B, kL2T, 1)   // stores dz2, leaves dz1 in A
#undef NR_BACK3
    if (live) store_native<8>(A, dzseg(0), lane);
}

__global__ void pack_x3_kernel(const float* __restrict__ flat, const int32_t* __restrict__ map,
                               int64_t n, __bf16* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t m = map[i];
    float v = 0.f;
    if (m >= 0) {
        const float w = flat[m >> 2];
        const float hi = (float)(__bf16)w;
        const float r1 = w - hi;
        const float mid = (float)(__bf16)r1;
        const int piece = m & 3;
        v = piece == 0 ? hi : (piece == 1 ? mid : r1 - mid);
    }
    out[i] = (__bf16)v;
}

}  // namespace

NR_API int nr_pack_bwd_x3(const float* flat, const int32_t* map, int64_t n, void* out,
                          void* stream) {
    NR_REQUIRE(n == BwdTab::off(kQ) / 2, "nr_pack_bwd_x3: map has %lld entries, expected %lld",
               (long long)n, (long long)(BwdTab::off(kQ) / 2));
    NR_REQUIRE(flat && map && out, "nr_pack_bwd_x3: null pointer");
    pack_x3_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        flat, map, n, reinterpret_cast<__bf16*>(out));
    NR_LAUNCH_CHECK("nr_pack_bwd_x3");
    return 0;
}

NR_API int nr_mlp_bwd_x3(const void* packed_bwd, const float* head, const float* out,
                         const float* g_out, const float* save, int64_t n, float* grad_ws,
                         void* stream) {
    NR_REQUIRE(n >= 0 && n < (int64_t)1 << 31, "nr_mlp_bwd_x3: n out of range");
    if (n == 0) return 0;
    NR_REQUIRE(packed_bwd && head && out && g_out && save && grad_ws,
               "nr_mlp_bwd_x3: null pointer");
    NR_REQUIRE((((uintptr_t)save | (uintptr_t)grad_ws | (uintptr_t)g_out | (uintptr_t)out |
                 (uintptr_t)packed_bwd | (uintptr_t)head) & 15) == 0,
               "nr_mlp_bwd_x3: buffers must be 16-byte aligned");
    Bwd3Args a{reinterpret_cast<const char*>(packed_bwd), head, out, g_out, save, (int)n, grad_ws};
    const int blocks = (int)((n + 32 * kWaves - 1) / (32 * kWaves));
    mlp_bwd3_kernel<<<blocks, 64 * kWaves, 0, (hipStream_t)stream>>>(a);
    NR_LAUNCH_CHECK("nr_mlp_bwd_x3");
    return 0;
}
