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
    // optional (the *_active entry points, active.hip): the ascending list of
    // the samples with a nonzero output gradient and its length m (device)
    const int32_t* slist; const int32_t* scount;
};

// SO: the sigma-only graph (rendering_shadows.py:167, sigma_only=True): no rgb
// head, dir layer or xyz_encoding_final, so the chain starts at d h8 =
// W_sigma^T dsigma masked by h8 and streams the transposed weights from layer 8.
// GA: over the packed sample list -- wave w takes positions 32w .. 32w+31, lane
// (h, j) sample slist[32w + j], gathering its output rows and its ReLU mask
// words (sample s keeps its bits in lanes s & 31 and 32 + (s & 31) of its
// block, one uint4 per lane and layer: exactly the word this lane needs), and
// writes every dz by position.  Positions past m carry zero gradients.
// GM = 2: the same list over a save buffer written by position
// (nr_mlp_fwd_listed, the deferred save): masks by position, only the output
// rows gathered
template <bool SO, int GM>
__global__ void __launch_bounds__(64 * kWaves, 1) mlp_bwd_kernel(BwdArgs a) {
    constexpr bool GA = GM != 0;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int h = lane >> 5;
    const int blk = blockIdx.x * kWaves + wave;   // block of (packed) positions
    const int nb = (int)nr_blocks_pad(a.n);    // segment stride (padded)
    const int m = GA ? __builtin_amdgcn_readfirstlane(*a.scount) : a.n;
    if (blk >= (m + 31) / 32) return;           // no barriers in this kernel
    const int s_raw = blk * 32 + (lane & 31);
    const bool valid = s_raw < m;
    const int s = GA ? a.slist[valid ? s_raw : m - 1] : (valid ? s_raw : a.n - 1);
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
                          (GM == 1 ? (size_t)(s >> 5) * NR_MASK_LAYERS * 64 + 32 * h + (s & 31)
                                   : (size_t)blk * NR_MASK_LAYERS * 64 + lane);
#pragma unroll
        for (int l = 0; l < (SO ? 8 : NR_MASK_LAYERS); ++l)   // SO: h1..h8, no hdir
            __builtin_amdgcn_global_load_lds(
                (const void*)(gm + l * 64),
                (__attribute__((address_space(3))) void*)&smask[wave][l][0], 16, 0, 0);
    }
    const uint4* mask = &smask[wave][0][lane];   // [layer * 64]

    f32x4 wq[8];                 // weight group in flight across layer boundaries
    nr_ld_first<8>(PB + (SO ? NR_B_L8T : NR_B_DIRT), lane, wq);
    const f32x4 go = *reinterpret_cast<const f32x4*>(a.g_out + (size_t)s * 4);
    const f32x4 yo = *reinterpret_cast<const f32x4*>(a.out + (size_t)s * 4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // masks landed in LDS (own wave only)
    // sigmoid backward: grad * (1 - y) * y  (ATen sigmoid_backward); tail lanes -> 0
    // (the sigma-only graph has no rgb output)
    float dzr[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) dzr[c] = valid && !SO ? go[c] * (1.f - yo[c]) * yo[c] : 0.f;
    const float dsig = valid ? go[3] : 0.f;
    if (h == 0) {
        f32x4 v = {dzr[0], dzr[1], dzr[2], dsig};
        *reinterpret_cast<f32x4*>(GD + nr_gd_dhead(nb) + ((size_t)blk * 32 + (lane & 31)) * 4) = v;
    }

    f32x16 A[8], B[8];
    // each layer's dz is written while the next backward layer runs (side hook)
    auto dzseg = [&](int l) { return GD + nr_gd_dz(l, nb) + (size_t)blk * NR_NATIVE(256); };
    auto side8 = [&](const f32x16 (&X)[8], float* dst) {
        return [&X, dst, lane](int grp) { if (grp < 32) store_native_piece<8>(X, grp, dst, lane); };
    };
    if constexpr (SO) {
        // d h8 = W_sigma^T dsigma, masked by h8
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const f32x4 w = *reinterpret_cast<const f32x4*>(H + NR_H_WSIG + 32 * t + 8 * q + 4 * h);
#pragma unroll
                for (int e = 0; e < 4; ++e) B[t][4 * q + e] = w[e] * dsig;
            }
        relu_mask<8>(B, mask[7 * 64]);
    } else {
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

    // d feat = W_dir[:, :256]^T dz_dir   (xyz_encoding_final has no activation); stores dz_dir
    zero<8>(A);
    {
        float* cdst = GD + nr_gd_dzdir(nb) + (size_t)blk * NR_NATIVE(128);
        nr_mm_chain<64, 8, 8>(PB + NR_B_DIRT, PB + NR_B_FINALT, lane, A, wq,
                              [&](int g) { return C[g >> 4][g & 15]; },
                              [&](int grp) { store_native_piece<4>(C, grp, cdst, lane); });
    }

    // d h8 = W_final^T dfeat + W_sigma^T dsigma, masked by h8.  dfeat is not
    // stored: xyz_encoding_final's weight gradient is W_dir[:, :256]^T G with
    // G = sum dz_dir h8^T (wgrad.hip task 10, nr_wgrad_dir_feat)
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
                               [&](int g) { return A[g >> 4][g & 15]; });
        relu_mask<8>(B, mk);
    }
    }   // !SO

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

namespace {
int bwd_launch(const char* name, bool so, const float* packed_bwd, const float* head,
               const float* out, const float* g_out, const float* save, int64_t n,
               float* grad_ws, const int32_t* slist, const int32_t* scount, void* stream,
               bool listed_save = false) {
    NR_REQUIRE(n >= 0 && n < (int64_t)1 << 31, "%s: n out of range", name);
    if (n == 0) return 0;
    NR_REQUIRE(packed_bwd && head && out && g_out && save && grad_ws, "%s: null pointer", name);
    NR_REQUIRE((((uintptr_t)out | (uintptr_t)g_out | (uintptr_t)save | (uintptr_t)grad_ws |
                 (uintptr_t)packed_bwd | (uintptr_t)head) & 15) == 0,
               "%s: pointers must be 16-byte aligned", name);
    BwdArgs a{packed_bwd, head, out, g_out, save, (int)n, grad_ws, slist, scount};
    const int blocks = (int)((n + 32 * kWaves - 1) / (32 * kWaves));
    hipStream_t st = (hipStream_t)stream;
    if (so && slist && listed_save) mlp_bwd_kernel<true, 2><<<blocks, 64 * kWaves, 0, st>>>(a);
    else if (slist && listed_save) mlp_bwd_kernel<false, 2><<<blocks, 64 * kWaves, 0, st>>>(a);
    else if (so && slist) mlp_bwd_kernel<true, 1><<<blocks, 64 * kWaves, 0, st>>>(a);
    else if (so) mlp_bwd_kernel<true, 0><<<blocks, 64 * kWaves, 0, st>>>(a);
    else if (slist) mlp_bwd_kernel<false, 1><<<blocks, 64 * kWaves, 0, st>>>(a);
    else mlp_bwd_kernel<false, 0><<<blocks, 64 * kWaves, 0, st>>>(a);
    NR_LAUNCH_CHECK(name);
    return 0;
}
}  // namespace

NR_API int nr_mlp_bwd(const float* packed_bwd, const float* head, const float* out,
                      const float* g_out, const float* save, int64_t n, float* grad_ws,
                      void* stream) {
    return bwd_launch("nr_mlp_bwd", false, packed_bwd, head, out, g_out, save, n, grad_ws,
                      nullptr, nullptr, stream);
}

// the sigma-only graph (g_out column 3 = d sigma, the rgb columns ignored):
// writes dz1..dz8 and the head gradient [0, 0, 0, dsigma] for nr_wgrad_sigma
NR_API int nr_mlp_bwd_sigma(const float* packed_bwd, const float* head, const float* out,
                            const float* g_out, const float* save, int64_t n, float* grad_ws,
                            void* stream) {
    return bwd_launch("nr_mlp_bwd_sigma", true, packed_bwd, head, out, g_out, save, n, grad_ws,
                      nullptr, nullptr, stream);
}

// over the samples nr_active_samples listed: position q of every gradient
// segment holds sample samples[q]'s rows; positions past *count are not read
NR_API int nr_mlp_bwd_active(const float* packed_bwd, const float* head, const float* out,
                             const float* g_out, const float* save, int64_t n, float* grad_ws,
                             const int32_t* samples, const int32_t* count, void* stream) {
    NR_REQUIRE(n == 0 || (samples && count), "nr_mlp_bwd_active: null sample list");
    return bwd_launch("nr_mlp_bwd_active", false, packed_bwd, head, out, g_out, save, n, grad_ws,
                      samples, count, stream);
}

NR_API int nr_mlp_bwd_sigma_active(const float* packed_bwd, const float* head, const float* out,
                                   const float* g_out, const float* save, int64_t n,
                                   float* grad_ws, const int32_t* samples, const int32_t* count,
                                   void* stream) {
    NR_REQUIRE(n == 0 || (samples && count), "nr_mlp_bwd_sigma_active: null sample list");
    return bwd_launch("nr_mlp_bwd_sigma_active", true, packed_bwd, head, out, g_out, save, n,
                      grad_ws, samples, count, stream);
}

// the deferred save (nr_mlp_fwd_listed): the listed samples' activations saved by position
NR_API int nr_mlp_bwd_listed(const float* packed_bwd, const float* head, const float* out,
                             const float* g_out, const float* save, int64_t n, float* grad_ws,
                             const int32_t* samples, const int32_t* count, void* stream) {
    NR_REQUIRE(n == 0 || (samples && count), "nr_mlp_bwd_listed: null sample list");
    return bwd_launch("nr_mlp_bwd_listed", false, packed_bwd, head, out, g_out, save, n, grad_ws,
                      samples, count, stream, true);
}

NR_API int nr_mlp_bwd_sigma_listed(const float* packed_bwd, const float* head, const float* out,
                                   const float* g_out, const float* save, int64_t n,
                                   float* grad_ws, const int32_t* samples, const int32_t* count,
                                   void* stream) {
    NR_REQUIRE(n == 0 || (samples && count), "nr_mlp_bwd_sigma_listed: null sample list");
    return bwd_launch("nr_mlp_bwd_sigma_listed", true, packed_bwd, head, out, g_out, save, n,
                      grad_ws, samples, count, stream, true);
}
