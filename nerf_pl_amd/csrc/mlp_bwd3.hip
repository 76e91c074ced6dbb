// Fused MLP backward, data-gradient chain, on bf16x6 split-operand MFMA
// (autograd of models/nerf.py:83-124; same contract and outputs as
// mlp_bwd.hip, activations in x3.h's N16 layout).  Four waves x 32 samples
// per workgroup carry the gradient backwards through the transposed layers
// D[in][sample] = W^T[in][out] dz[out][sample] on v_mfma_f32_16x16x32_bf16;
// the transposed weights (packing.BWD3_LAYERS, 136 k-groups of 24 KiB) stream
// through the LDS ring of x3.h.  ReLU masks are the forward's bit masks,
// staged in LDS by LDS-DMA; every layer's dz is written block-native (N16)
// for the weight-gradient GEMMs (wgrad.hip).
//
// NR_BWD_W2 = 1 (f16x3): two waves per SIMD -- eight waves per workgroup, each
// carrying ONE 16-sample tile of a 32-sample block (the pair of waves 2b, 2b+1
// holds block b's tiles S = 0, 1), so a wave's accumulators take 128 registers
// instead of 256 and the whole wave fits the 256 registers a second resident
// wave leaves it.  Memory layouts, outputs and the arithmetic are unchanged;
// the per-block maxima of the two waves are combined through LDS at the end.
// (measured, same box, alternating: fine data gradient 1.44-1.45 -> 1.32-1.34
// ms).  Default for f16x3; -DNR_BWD_W2=0 builds the
// one-wave-per-SIMD form of rounds 2-5.
#ifndef NR_BWD_W2
#if defined(NR_F16) && NR_F16
#define NR_BWD_W2 1
#else
#define NR_BWD_W2 0
#endif
#endif
#if NR_BWD_W2 && !NR_F16
#error "NR_BWD_W2 is an f16x3 variant"
#endif
#if NR_BWD_W2
#define NR_X3_WAVES 8
#endif
#include "x3.h"

namespace {

using namespace x3;

constexpr int kDirT = 0, kFinalT = 8, kL8T = 24, kL7T = 40, kL6T = 56, kL5T = 72, kL4T = 88,
              kL3T = 104, kL2T = 120, kQ = 136;
constexpr int kNS = NR_BWD_W2 ? 1 : 2;          // 16-sample tiles per wave
constexpr int kBlocks = kWaves * kNS / 2;        // 32-sample blocks per workgroup
constexpr int kMaskBytes = kBlocks * NR_MASK_LAYERS * 64 * 16;
constexpr int kHeadDma = (NR_H_SIZE * 4 + 1023) / 1024;   // fp32 head block, by LDS-DMA
constexpr int kMaxBytes = kNS == 1 ? kWaves * 16 * 4 : 0;  // per-wave segment maxima (kNS = 1)
constexpr int kLdsBytes = kRingBytes + kMaskBytes + kHeadDma * 1024 + kMaxBytes;
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");
static_assert(NR_STAT_SEGS <= 16, "maxima slots");

struct BwdTab {
    __host__ __device__ static constexpr int64_t off(int q) { return (int64_t)q * kSlotBytes; }
    // merged ring (x3.h): every transposed layer has two input halves per k-step
    __host__ __device__ static constexpr int sg(int q) { return q / 2; }
    __host__ __device__ static constexpr int first(int G) { return 2 * G; }
    __host__ __device__ static constexpr int size(int) { return 2; }
};
static_assert(BwdTab::off(kQ) == (NR_F16 ? 2228224 : (NR_BF1 ? 1114112 : 3342336)),
              "packed size must match packing.BWD3_BYTES");

// f16x3 gradient scaling.  Column (= sample) scaling commutes with the
// transposed layer, D = W^T (sigma dz) = sigma (W^T dz), so every sample
// carries its own power-of-two scale sigma: B values = sigma * true gradient.
// A layer's accumulator is 2^kWScale * sigma_in * (true output); the getter
// that splits it renormalises with the max |B| of its producer (the previous
// layer, complete by then): sigma_out = sigma_in * 2^(kGT - e(max)), so B values
// stay near 2^kGT whatever the gradient's magnitude, with 2^(15 - kGT) of
// headroom for one layer's growth (a layer's growth in max-norm is at most
// max_row sum|W|, 16 at the default init).  Gradient injected into a layer's
// accumulator (the sigma head's w_sigma dsigma into d h8) enters the
// renormalisation as a bound (GradU::inj).  Stored gradients are true values.
constexpr int kGT = 6;
constexpr int kGLim = 64;      // largest renormalisation step (binades)
constexpr int kSigLim = 120;   // |log2 sigma| bound
struct GScale {
    float ks[2] = {1.f, 1.f};    // accumulator -> B value
    float kst[2] = {1.f, 1.f};   // accumulator -> true value (stored)
    float sig[2] = {1.f, 1.f};   // scale of the B values
    float mx[2] = {0.f, 0.f};    // max |B value| seen by this lane, per sample tile
};

// (max_over_groups, x3.h: max over the 4 lane groups = the features of a sample)

// 1 / sig for a power of two sig in [2^-126, 2^126] (every sigma here: |log2| <=
// kSigLim), exact, so x * inv_pow2(sig) == x / sig bit for bit
__device__ __forceinline__ float inv_pow2(float sig) {
    return __uint_as_float(0x7f000000u - __float_as_uint(sig));
}

// renormalise after a producer: see GScale; inj = bound of the values injected
// into the accumulator, in the producer's B units
__device__ __forceinline__ void gscale_from(GScale& sc, const GScale& prod, const float (&inj)[2]) {
#pragma unroll
    for (int S = 0; S < kNS; ++S) {
        float f = pow2_norm(fmaxf(max_over_groups(prod.mx[S]), inj[S]), kGT, kGLim);
        // keep sigma in [2^-kSigLim, 2^kSigLim]: gradients so small that they
        // flush to zero in fp16 must not drive it to infinity (0 * inf = NaN)
        const int es = (int)((__float_as_uint(prod.sig[S]) >> 23) & 0xff) - 127;
        const int ef = (int)((__float_as_uint(f) >> 23) & 0xff) - 127;
        const int en = min(max(es + ef, -kSigLim), kSigLim);
        f = __uint_as_float((uint32_t)(127 + en - es) << 23);
        sc.sig[S] = prod.sig[S] * f;
        sc.ks[S] = f * kWUnscale;
        sc.kst[S] = kWUnscale * inv_pow2(prod.sig[S]);
    }
}

// max |true gradient| of a segment over the wave -> its per-wave slot
// (layout.h NR_STAT_SEGS; reduced by wgrad.hip)
__device__ __forceinline__ void report_max(float m, float* slot, int lane) {
    m = wave_max(m);
    if (lane == 0) *slot = m;
}
// segment l's maximum of this wave: to the block's slot (stw + l nb) when the
// wave holds the whole block, else to the wave's LDS row (combined with the
// partner's at the end of the kernel)
struct Rep {
    float* stw; int nb; int lane; float* lrow;
    __device__ __forceinline__ void operator()(float m, int l) const {
        if constexpr (kNS == 2) {
            report_max(m, stw + l * nb, lane);
        } else {
            m = wave_max(m);
            if (lane == 0) lrow[l] = m;
        }
    }
};

// B units of a gradient input dz (NF feature tiles): with MASK the ReLU mask
// of the forward activation applied (ReLU backward), and the values stored
// N16 as they are split (units p = 0, 1 of (k-step s, tile S) complete tile
// 2s, p = 2, 3 tile 2s+1) for the weight-gradient GEMMs
// f16x3: B values and stored values are scaled per sample (GScale); begin()
// renormalises from the getter whose B values produced X.  sb is the wave's
// tile index; s0 + sb the block's (masks, stored layout)
template <int NF, bool MASK, bool STORE = true>
struct GradU {
    static constexpr bool kStores = STORE;
    static constexpr bool kPaired = false;
    const f32x4 (&X)[NF][kNS];
    float* dst;
    uint32_t mw[4];
    int lane;
    int s0;
    float pend[2] = {0.f, 0.f};
    __device__ __forceinline__ int tile(int sb) const { return (kNS == 2 ? 0 : s0) + sb; }
    GScale sc;
    float inj[2] = {0.f, 0.f};
    template <typename P>
    __device__ __forceinline__ void begin(const P& prod) {
        if constexpr (NR_F16) gscale_from(sc, prod.sc, inj);
    }
    template <typename SC>
    __device__ __forceinline__ void operator()(SC, int sb, int p, float& x0, float& x1) {
        constexpr int s = SC::value;
        const int F = 2 * s + (p >> 1), r = 2 * (p & 1);
        x0 = acc_b(X, s, sb, 2 * p);
        x1 = acc_b(X, s, sb, 2 * p + 1);
        if constexpr (MASK) {
            x0 = mask_keep(x0, mw, F, tile(sb), r);
            x1 = mask_keep(x1, mw, F, tile(sb), r + 1);
        }
        float t0 = x0, t1 = x1;
        if constexpr (NR_F16) {
            t0 = x0 * sc.kst[sb];
            t1 = x1 * sc.kst[sb];
            x0 *= sc.ks[sb];
            x1 *= sc.ks[sb];
            sc.mx[sb] = fmaxf(sc.mx[sb], fmaxf(fabsf(x0), fabsf(x1)));
        }
        if constexpr (STORE) {
            if ((p & 1) == 0) {
                pend[0] = t0;
                pend[1] = t1;
            } else {
                store_n16(f32x4{pend[0], pend[1], t0, t1}, F, tile(sb), dst, lane);
            }
        }
    }
    // after the last split: the segment's max |true value| -> its stats slot
    __device__ __forceinline__ void report(const Rep& rep, int l) const {
        if constexpr (NR_F16) {
            float m = sc.mx[0] * inv_pow2(sc.sig[0]);
            if constexpr (kNS == 2) m = fmaxf(m, sc.mx[1] * inv_pow2(sc.sig[1]));
            rep(m, l);
        }
    }
};

// initial accumulator of d h8: W_sigma^T dsigma (nerf.py:115 sigma head)
struct SigInit {
    const float* w; int g; float d0, d1;
    __device__ __forceinline__ f32x4 operator()(int F, int S) const {
        const f32x4 v = *reinterpret_cast<const f32x4*>(w + 16 * F + 4 * g);
        const float d = S ? d1 : d0;
        return f32x4{v[0] * d, v[1] * d, v[2] * d, v[3] * d};
    }
};

struct Bwd3Args {
    const char* packed;        // packing.build_bwd3_map layout
    const float* head;         // fp32 head block (sigma / rgb weights)
    const float* out; const float* g_out; const float* save;
    int n;
    float* grad;
    float* stats;    // f16x3: per-wave maxima [NR_STAT_SEGS][nb] (layout.h, in the save buffer)
    // optional (active.hip): the ascending list of the samples with a nonzero
    // output gradient and its length m; the chain then runs over them packed
    // densely -- position q < m holds sample slist[q] -- and every output
    // (dz, dhead, stats) is indexed by position
    const int32_t* slist; const int32_t* scount;
};

// SO: the sigma-only graph (rendering_shadows.py:167, sigma_only=True): no rgb
// head, dir layer or xyz_encoding_final, so the chain starts at d h8 =
// W_sigma^T dsigma and the ring streams the transposed weights from layer 8
// on (the packed buffer from group kL8T, the group indices shifted by kB)
// GM (sample-list mode): 0 = every sample; 1 = over the packed sample list
// a.slist (the *_active entry points): position q < m runs sample slist[q],
// whose saved activations and masks are gathered; 2 = the same list over a
// save buffer written by position (nr_mlp_fwd_listed*, the deferred save):
// masks by position, only g_out / out gathered
template <bool SO, int GM>
__global__ void __launch_bounds__(64 * kWaves, 1) mlp_bwd3_kernel(Bwd3Args a) {
    constexpr int kB = SO ? kL8T : 0;      // first k-group streamed
    constexpr int QE = kQ - kB;            // groups streamed
    __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4;
    const int nreal = (a.n + 31) / 32;
    const int nb = (int)nr_blocks_pad(a.n);     // segment stride; dead waves write padding
    const int wb = kNS == 2 ? wave : wave >> 1;   // the wave's block within the workgroup
    const int s0 = kNS == 2 ? 0 : wave & 1;       // the block's first tile this wave holds
    const int blk = blockIdx.x * kBlocks + wb;    // block of (packed) positions
    // m: samples (positions) the chain runs over.  With a sample list,
    // workgroups past its end only zero their stats slots: the weight
    // gradient reads positions < m only
    int m = a.n;
    constexpr bool GA = GM != 0;
    if constexpr (GA) {
        m = __builtin_amdgcn_readfirstlane(*a.scount);
        if ((int)blockIdx.x * kBlocks * 32 >= m) {
            if constexpr (NR_F16) {
                if (s0 == 0) {
#pragma unroll 1
                    for (int l = 0; l < NR_STAT_SEGS; ++l) report_max(0.f, a.stats + l * nb + blk, lane);
                }
            }
            return;
        }
    }
    const bool live = blk < nreal;
    const char* PB = a.packed;
    const float* SV = a.save;
    float* const GD = a.grad;

    // ReLU mask words (9 layers) and the head block by LDS-DMA, issued before
    // the ring so the ring's counted waits cover them (kNS = 1: the two waves
    // of a block fill its words, alternate layers each)
    uint4* smask = reinterpret_cast<uint4*>(smem + kRingBytes) + wb * NR_MASK_LAYERS * 64;
    constexpr int kLStep = kNS == 2 ? 1 : 2;
    const int l0 = kNS == 2 ? 0 : s0;
    // the samples of the block's columns (tiles S = 0, 1): position
    // 32 blk + 16 S + (lane & 15), sample slist[position] with a list; the
    // wave's own tiles are s0 .. s0 + kNS - 1
    int sidx2[2];
    bool valid2[2];
#pragma unroll
    for (int S = 0; S < 2; ++S) {
        const int q = blk * 32 + 16 * S + (lane & 15);
        valid2[S] = q < m;
        sidx2[S] = !valid2[S] ? (GA ? 0 : a.n - 1) : (GA ? a.slist[q] : q);
    }
    int sidx[2];
    bool valid[2];
#pragma unroll
    for (int j = 0; j < kNS; ++j) {
        sidx[j] = sidx2[s0 + j];
        valid[j] = valid2[s0 + j];
    }
    if constexpr (GM != 1) {
        const uint4* gm = reinterpret_cast<const uint4*>(SV + nr_sv_mask(nb)) +
                          (size_t)blk * NR_MASK_LAYERS * 64 + lane;
#pragma unroll
        for (int l = l0; l < NR_MASK_LAYERS; l += kLStep)
            __builtin_amdgcn_global_load_lds(
                (const void*)(gm + l * 64),
                (__attribute__((address_space(3))) void*)(smask + l * 64), 16, 0, 0);
    } else {
        // gather: sample s = 32 b + 16 S' + c' keeps its ReLU bits in lane
        // 16 g + c' of block b, word k bits 8 i + 4 S' + r (x3.h mask_bits);
        // repack them at this lane's tile S (the block's waves read only its slots)
        const uint4* gm = reinterpret_cast<const uint4*>(SV + nr_sv_mask(nb));
        const uint4* src[2];
        int sh[2];
#pragma unroll
        for (int S = 0; S < 2; ++S) {
            const int s = sidx2[S];
            src[S] = gm + (size_t)(s >> 5) * NR_MASK_LAYERS * 64 + 16 * g + (s & 15);
            sh[S] = 4 * ((s >> 4) & 1);
        }
#pragma unroll
        for (int l = l0; l < NR_MASK_LAYERS; l += kLStep) {
            const uint4 w0 = src[0][l * 64], w1 = src[1][l * 64];
            auto mix = [&](uint32_t x0, uint32_t x1, int S0ok, int S1ok) {
                return (S0ok ? ((x0 >> sh[0]) & 0x0F0F0F0Fu) : 0u) |
                       (S1ok ? (((x1 >> sh[1]) & 0x0F0F0F0Fu) << 4) : 0u);
            };
            smask[l * 64 + lane] = make_uint4(mix(w0.x, w1.x, valid2[0], valid2[1]),
                                              mix(w0.y, w1.y, valid2[0], valid2[1]),
                                              mix(w0.z, w1.z, valid2[0], valid2[1]),
                                              mix(w0.w, w1.w, valid2[0], valid2[1]));
        }
    }
    float* Hs = reinterpret_cast<float*>(smem + kRingBytes + kMaskBytes);
    {
        const __amdgpu_buffer_rsrc_t hr =
            __builtin_amdgcn_make_buffer_rsrc((void*)a.head, 0, NR_H_SIZE * 4, 0x00020000);
        for (int i = wave; i < kHeadDma; i += kWaves)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                hr, (__attribute__((address_space(3))) void*)(Hs + i * 256), 16, lane * 16, i * 1024, 0, 0);
    }
    float* const lmax = reinterpret_cast<float*>(smem + kRingBytes + kMaskBytes + kHeadDma * 1024);
    const Dma dma = make_dma(PB + BwdTab::off(kB), BwdTab::off(QE), smem, wave, lane);
    prologue<BwdTab, QE>(dma);
    f32x4 go[2], yo[2];
#pragma unroll
    for (int S = 0; S < kNS; ++S) {
        go[S] = *reinterpret_cast<const f32x4*>(a.g_out + (size_t)sidx[S] * 4);
        yo[S] = *reinterpret_cast<const f32x4*>(a.out + (size_t)sidx[S] * 4);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // masks, head (and the prologue) landed
    __builtin_amdgcn_s_barrier();                       // head (and the partner's masks) visible
    const uint4* mask = smask + lane;                   // [layer * 64]
    const float* H = Hs;
    Ahead f0;                                           // the first tiles' fragments of the next k-group
    enter<BwdTab, 0, QE>(smem, lane, f0);
    float* const STW = a.stats + blk;     // + l * nb: the block's slot of segment l
    const Rep rep{STW, nb, lane, lmax + wave * 16};

    float dzr[2][3], dsig[2];
#pragma unroll
    for (int S = 0; S < kNS; ++S) {
#pragma unroll
        for (int c = 0; c < 3; ++c)   // (the sigma-only graph has no rgb output)
            dzr[S][c] = valid[S] && !SO ? go[S][c] * (1.f - yo[S][c]) * yo[S][c] : 0.f;
        dsig[S] = valid[S] ? go[S][3] : 0.f;
    }
    if (live && g < kNS) {     // lane group g < kNS writes the wave's tile g (block tile s0 + g)
        const int S = s0 + g;
        const int j = kNS == 2 ? g : 0;
        f32x4 v = {j ? dzr[1][0] : dzr[0][0], j ? dzr[1][1] : dzr[0][1],
                   j ? dzr[1][2] : dzr[0][2], j ? dsig[1] : dsig[0]};
#if NR_BF1     // bf16 [block][32 samples][4], 256 B per block (wgrad.hip's head DMA)
        *reinterpret_cast<u32x2*>(reinterpret_cast<char*>(GD + nr_gd_dhead(nb) + (size_t)blk * 64) +
                                  (16 * S + (lane & 15)) * 8) = pack_bf16x4(v);
#else
        *reinterpret_cast<f32x4*>(GD + nr_gd_dhead(nb) + ((size_t)blk * 32 + 16 * S + (lane & 15)) * 4) = v;
#endif
    }
    if constexpr (NR_F16) {
        float m = 0.f;
#pragma unroll
        for (int S = 0; S < kNS; ++S)
            m = fmaxf(m, fmaxf(fmaxf(fabsf(dzr[S][0]), fabsf(dzr[S][1])),
                               fmaxf(fabsf(dzr[S][2]), fabsf(dsig[S]))));
        rep(m, 10);
    }

    ActN<kNS> A, B;
    Pieces b[kNS];
    NoSide none;
    NoNext nonext;
    ZeroInit zero;
    auto dzseg = [&](int l) { return GD + nr_gd_dz(l, nb) + (size_t)blk * NR_SEGF(256); };
    auto mwords = [&](int l, uint32_t (&w)[4]) {
        const uint4 m = mask[l * 64];
        w[0] = m.x; w[1] = m.y; w[2] = m.z; w[3] = m.w;
    };
#define NR_GRADU(NAME, X, DZ, ML)                                       \
    GradU<16, true> NAME{X, dzseg(DZ), {0u, 0u, 0u, 0u}, lane, s0};     \
    mwords(ML, NAME.mw);

    NR_GRADU(u8, B, 7, 7)
    if constexpr (!SO) {
        // d hdir = W_rgb^T dz_rgb, masked by the dir-layer ReLU -> dz_dir (128)
        f32x4 C[8][kNS];
        {
            const uint4 mk = mask[8 * 64];
            const uint32_t mw[4] = {mk.x, mk.y, mk.z, mk.w};
#pragma unroll
            for (int F = 0; F < 8; ++F) {
                const int f = 16 * F + 4 * g;
                const f32x4 w0 = *reinterpret_cast<const f32x4*>(H + NR_H_WRGB + f);
                const f32x4 w1 = *reinterpret_cast<const f32x4*>(H + NR_H_WRGB + 128 + f);
                const f32x4 w2 = *reinterpret_cast<const f32x4*>(H + NR_H_WRGB + 256 + f);
#pragma unroll
                for (int S = 0; S < kNS; ++S)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float d = fmaf(w2[r], dzr[S][2], fmaf(w1[r], dzr[S][1], w0[r] * dzr[S][0]));
                        C[F][S][r] = mask_keep(d, mw, F, s0 + S, r);
                    }
            }
        }

        // d feat = W_dir[:, :256]^T dz_dir (xyz_encoding_final has no activation); stores dz_dir
        GradU<8, false> uc{C, GD + nr_gd_dzdir(nb) + (size_t)blk * NR_SEGF(128), {0u, 0u, 0u, 0u},
                           lane, s0};
        // dfeat, not stored: xyz_encoding_final's weight gradient is
        // W_dir[:, :256]^T G with G = sum dz_dir h8^T (wgrad.hip task 10)
        GradU<16, false, false> ua{A, nullptr, {0u, 0u, 0u, 0u}, lane, s0};
        // f16x3: the sigma head injects w_sigma dsigma (|.| <= max|w_sigma| |dsigma|)
        // into d h8.  The scales of dz_dir's and dfeat's B values are bounded by it
        // too, so the d h8 accumulator (which inherits dfeat's scale) stays finite
        // when dsigma dwarfs the rgb gradient (the 1e10 last-sample delta).
        float inj[2] = {0.f, 0.f};   // max|w_sigma| |dsigma|, true units
        if constexpr (NR_F16) {
            float wm = 0.f;
#pragma unroll
            for (int F = 0; F < 16; ++F) {
                const f32x4 v = *reinterpret_cast<const f32x4*>(H + NR_H_WSIG + 16 * F + 4 * g);
                wm = fmaxf(wm, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
            }
            wm = max_over_groups(wm);
#pragma unroll
            for (int S = 0; S < kNS; ++S) {
                inj[S] = wm * fabsf(dsig[S]);
                // dz_dir holds true values: its B scale from its own max (and the injection)
                float m = 0.f;
#pragma unroll
                for (int F = 0; F < 8; ++F)
#pragma unroll
                    for (int r = 0; r < 4; ++r) m = fmaxf(m, fabsf(C[F][S][r]));
                const float f = pow2_norm(fmaxf(max_over_groups(m), inj[S]), kGT, kGLim);
                uc.sc.ks[S] = f;
                uc.sc.sig[S] = f;
                ua.inj[S] = inj[S] * f;
            }
        }
        split_all(uc, b);
        segment<BwdTab, kDirT - kB, 4, 2, QE, true>(dma, lane, A, uc, ua, zero, none, b, f0);
        uc.report(rep, 9);
        // d h8 = W_final^T dfeat + W_sigma^T dsigma; dz8 = d h8 * [h8 > 0]
        if constexpr (NR_F16) {
#pragma unroll
            for (int S = 0; S < kNS; ++S) u8.inj[S] = inj[S] * ua.sc.sig[S];   // in dfeat's B units
        }
        {
            // the accumulator carries 2^kWScale sigma(dfeat) (f16x3), so does its C operand
            // (dsigma * sigma first: 2^kWScale * sigma alone may overflow when dsigma is 0)
            constexpr float kW = (float)(1 << kWScale);
            const float d0 = NR_F16 ? dsig[0] * ua.sc.sig[0] * kW : dsig[0];
            float d1 = 0.f;
            if constexpr (kNS == 2) d1 = NR_F16 ? dsig[1] * ua.sc.sig[1] * kW : dsig[1];
            SigInit si{H + NR_H_WSIG, g, d0, d1};
            segment<BwdTab, kFinalT - kB, 8, 2, QE, true>(dma, lane, B, ua, u8, si, none, b, f0);
        }
        ua.report(rep, 8);
    } else {
        // d h8 = W_sigma^T dsigma (nerf.py:112), the accumulator filled directly
        // in the units the full graph's xyz_encoding_final segment leaves it in
        // (2^kWScale x the producer's scale, here a unit-scale virtual producer)
        float inj[2] = {0.f, 0.f};
        if constexpr (NR_F16) {
            float wm = 0.f;
#pragma unroll
            for (int F = 0; F < 16; ++F) {
                const f32x4 v = *reinterpret_cast<const f32x4*>(H + NR_H_WSIG + 16 * F + 4 * g);
                wm = fmaxf(wm, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
            }
            wm = max_over_groups(wm);
#pragma unroll
            for (int S = 0; S < kNS; ++S) u8.inj[S] = inj[S] = wm * fabsf(dsig[S]);
        }
        constexpr float kW = NR_F16 ? (float)(1 << kWScale) : 1.f;
        const SigInit si{H + NR_H_WSIG, g, dsig[0] * kW, kNS == 2 ? dsig[1] * kW : 0.f};
#pragma unroll
        for (int F = 0; F < 16; ++F)
#pragma unroll
            for (int S = 0; S < kNS; ++S) B[F][S] = si(F, S);
        struct { GScale sc; } unit;
        u8.begin(unit);
        split_all(u8, b);
        if constexpr (NR_F16) {     // dfeat and dz_dir are not part of this graph
            rep(0.f, 8);
            rep(0.f, 9);
        }
    }
    NR_GRADU(u7, A, 6, 6)
    segment<BwdTab, kL8T - kB, 8, 2, QE, true>(dma, lane, A, u8, u7, zero, none, b, f0);
    u8.report(rep, 7);
    NR_GRADU(u6, B, 5, 5)
    segment<BwdTab, kL7T - kB, 8, 2, QE, true>(dma, lane, B, u7, u6, zero, none, b, f0);
    u7.report(rep, 6);
    NR_GRADU(u5, A, 4, 4)
    segment<BwdTab, kL6T - kB, 8, 2, QE, true>(dma, lane, A, u6, u5, zero, none, b, f0);
    u6.report(rep, 5);
    NR_GRADU(u4, B, 3, 3)   // through the h4 columns of the skip layer
    segment<BwdTab, kL5T - kB, 8, 2, QE, true>(dma, lane, B, u5, u4, zero, none, b, f0);
    u5.report(rep, 4);
    NR_GRADU(u3, A, 2, 2)
    segment<BwdTab, kL4T - kB, 8, 2, QE, true>(dma, lane, A, u4, u3, zero, none, b, f0);
    u4.report(rep, 3);
    NR_GRADU(u2, B, 1, 1)
    segment<BwdTab, kL3T - kB, 8, 2, QE, true>(dma, lane, B, u3, u2, zero, none, b, f0);
    u3.report(rep, 2);
    segment<BwdTab, kL2T - kB, 8, 2, QE, true>(dma, lane, A, u2, nonext, zero, none, b, f0);
    u2.report(rep, 1);
#undef NR_GRADU
    {   // dz1 = (W2^T dz2) * [h1 > 0]
        uint32_t mw[4];
        mwords(0, mw);
        float* d1 = dzseg(0);
        float m1 = 0.f;
        float k1[2];
#pragma unroll
        for (int S = 0; S < kNS; ++S) k1[S] = kWUnscale * inv_pow2(u2.sc.sig[S]);
#pragma unroll
        for (int F = 0; F < 16; ++F)
#pragma unroll
            for (int S = 0; S < kNS; ++S) {
                f32x4 v = A[F][S];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = mask_keep(v[r], mw, F, s0 + S, r);
                    if constexpr (NR_F16) {
                        v[r] *= k1[S];
                        m1 = fmaxf(m1, fabsf(v[r]));
                    }
                }
                store_n16(v, F, s0 + S, d1, lane);
            }
        if constexpr (NR_F16) rep(m1, 0);
    }
    if constexpr (NR_F16 && kNS == 1) {
        // the block's maxima: the larger of its two waves' (LDS rows 2 wb, 2 wb + 1)
        __syncthreads();
        if (s0 == 0 && lane < NR_STAT_SEGS)
            STW[lane * nb] = fmaxf(lmax[wave * 16 + lane], lmax[(wave + 1) * 16 + lane]);
    }
}

__global__ void pack_x3_kernel(const float* __restrict__ flat, const int32_t* __restrict__ map,
                               int64_t n, p1* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t m = map[i];
    float v = 0.f;
    if (m >= 0) {
        float w = flat[m >> 2];
        const int piece = m & 3;
#if NR_F16
        w *= (float)(1 << kWScale);
        const float hi = (float)(_Float16)w;
        v = piece == 0 ? hi : w - hi;
#elif NR_BF1
        (void)piece;
        v = (float)(__bf16)w;
#else
        const float hi = (float)(__bf16)w;
        const float r1 = w - hi;
        const float mid = (float)(__bf16)r1;
        v = piece == 0 ? hi : (piece == 1 ? mid : r1 - mid);
#endif
    }
    out[i] = (p1)v;
}

}  // namespace

NR_API int NR_X3_NAME(nr_pack_bwd)(const float* flat, const int32_t* map, int64_t n, void* out,
                          void* stream) {
    NR_REQUIRE(n == BwdTab::off(kQ) / 2, "nr_pack_bwd_x3: map has %lld entries, expected %lld",
               (long long)n, (long long)(BwdTab::off(kQ) / 2));
    NR_REQUIRE(flat && map && out, "nr_pack_bwd_x3: null pointer");
    pack_x3_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        flat, map, n, reinterpret_cast<p1*>(out));
    NR_LAUNCH_CHECK("nr_pack_bwd_x3");
    return 0;
}

namespace {
int bwd3_launch(const char* name, bool sigma_only, const void* packed_bwd, const float* head,
                const float* out, const float* g_out, const float* save, int64_t n,
                float* grad_ws, void* stream, const int32_t* slist = nullptr,
                const int32_t* scount = nullptr, bool listed_save = false) {
    NR_REQUIRE(n >= 0 && n < (int64_t)1 << 31, "%s: n out of range", name);
    if (n == 0) return 0;
    NR_REQUIRE(packed_bwd && head && out && g_out && save && grad_ws, "%s: null pointer", name);
    NR_REQUIRE((((uintptr_t)save | (uintptr_t)grad_ws | (uintptr_t)g_out | (uintptr_t)out |
                 (uintptr_t)packed_bwd | (uintptr_t)head) & 15) == 0,
               "%s: buffers must be 16-byte aligned", name);
    float* stats = const_cast<float*>(save) + nr_sv_stats(nr_blocks_pad(n)) + NR_STATS;
    Bwd3Args a{reinterpret_cast<const char*>(packed_bwd), head, out, g_out, save, (int)n, grad_ws,
               stats, slist, scount};
    const int blocks = (int)((n + 32 * kBlocks - 1) / (32 * kBlocks));
    hipStream_t st = (hipStream_t)stream;
#if NR_BF1     // no sample lists for the bf16 variant
    if (sigma_only) mlp_bwd3_kernel<true, 0><<<blocks, 64 * kWaves, 0, st>>>(a);
    else mlp_bwd3_kernel<false, 0><<<blocks, 64 * kWaves, 0, st>>>(a);
#else
    if (slist && listed_save) {
        if (sigma_only) mlp_bwd3_kernel<true, 2><<<blocks, 64 * kWaves, 0, st>>>(a);
        else mlp_bwd3_kernel<false, 2><<<blocks, 64 * kWaves, 0, st>>>(a);
    } else if (slist) {
        if (sigma_only) mlp_bwd3_kernel<true, 1><<<blocks, 64 * kWaves, 0, st>>>(a);
        else mlp_bwd3_kernel<false, 1><<<blocks, 64 * kWaves, 0, st>>>(a);
    } else {
        if (sigma_only) mlp_bwd3_kernel<true, 0><<<blocks, 64 * kWaves, 0, st>>>(a);
        else mlp_bwd3_kernel<false, 0><<<blocks, 64 * kWaves, 0, st>>>(a);
    }
#endif
    NR_LAUNCH_CHECK(name);
    return 0;
}
}  // namespace

NR_API int NR_X3_NAME(nr_mlp_bwd)(const void* packed_bwd, const float* head, const float* out,
                         const float* g_out, const float* save, int64_t n, float* grad_ws,
                         void* stream) {
    return bwd3_launch("nr_mlp_bwd_x3", false, packed_bwd, head, out, g_out, save, n, grad_ws,
                       stream);
}

// the sigma-only graph's data gradient (g_out column 3 = d sigma; the rgb
// columns are ignored): save from the sigma-only training forward
NR_API int NR_X3_NAME(nr_mlp_bwd_sigma)(const void* packed_bwd, const float* head,
                               const float* out, const float* g_out, const float* save,
                               int64_t n, float* grad_ws, void* stream) {
    return bwd3_launch("nr_mlp_bwd_sigma_x3", true, packed_bwd, head, out, g_out, save, n,
                       grad_ws, stream);
}

#if !NR_BF1
// the same over the samples nr_active_samples listed (samples / count on the
// device), packed: grad_ws holds position q's rows at q -- only the matching
// nr_wgrad*_active entry point (same list) may consume it
NR_API int NR_X3_NAME(nr_mlp_bwd_active)(const void* packed_bwd, const float* head,
                                         const float* out, const float* g_out, const float* save,
                                         int64_t n, float* grad_ws, const int32_t* samples,
                                         const int32_t* count, void* stream) {
    NR_REQUIRE(samples && count, "nr_mlp_bwd_active: null sample list");
    return bwd3_launch("nr_mlp_bwd_active", false, packed_bwd, head, out, g_out, save, n, grad_ws,
                       stream, samples, count);
}
NR_API int NR_X3_NAME(nr_mlp_bwd_sigma_active)(const void* packed_bwd, const float* head,
                                               const float* out, const float* g_out,
                                               const float* save, int64_t n, float* grad_ws,
                                               const int32_t* samples, const int32_t* count,
                                               void* stream) {
    NR_REQUIRE(samples && count, "nr_mlp_bwd_sigma_active: null sample list");
    return bwd3_launch("nr_mlp_bwd_sigma_active", true, packed_bwd, head, out, g_out, save, n,
                       grad_ws, stream, samples, count);
}
// the deferred save: the same list over a save buffer nr_mlp_fwd_listed* wrote
// by position (masks read by position, g_out / out gathered by the list)
NR_API int NR_X3_NAME(nr_mlp_bwd_listed)(const void* packed_bwd, const float* head,
                                         const float* out, const float* g_out, const float* save,
                                         int64_t n, float* grad_ws, const int32_t* samples,
                                         const int32_t* count, void* stream) {
    NR_REQUIRE(samples && count, "nr_mlp_bwd_listed: null sample list");
    return bwd3_launch("nr_mlp_bwd_listed", false, packed_bwd, head, out, g_out, save, n, grad_ws,
                       stream, samples, count, true);
}
NR_API int NR_X3_NAME(nr_mlp_bwd_sigma_listed)(const void* packed_bwd, const float* head,
                                               const float* out, const float* g_out,
                                               const float* save, int64_t n, float* grad_ws,
                                               const int32_t* samples, const int32_t* count,
                                               void* stream) {
    NR_REQUIRE(samples && count, "nr_mlp_bwd_sigma_listed: null sample list");
    return bwd3_launch("nr_mlp_bwd_sigma_listed", true, packed_bwd, head, out, g_out, save, n,
                       grad_ws, stream, samples, count, true);
}
#endif
