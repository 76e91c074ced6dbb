// bf16x6 split-operand MFMA machinery.
//
// Fused MLP kernels (mlp_fwd3.hip, mlp_bwd3.hip): v_mfma_f32_16x16x32_bf16 on
// the exact three-piece bf16 split of both operands, fed by an LDS ring of
// weight k-groups that LDS-DMA fills kSlots-1 groups ahead, one barrier per
// group.  16x16x32 sustains ~1.8x the clock of 32x32x16 on random operands
// (dev/mfma_rate.hip: 88% vs 48-55% of the dense bf16 peak), so the layers
// are tiled for it.
//
// Register layout of a wave (32 samples = two 16-sample tiles S): a width-W
// activation is Act = f32x4 [W/16 feature tiles F][2]; lane l (g = l >> 4)
// holds features 16F + 4g + r (r = 0..3) of sample 16S + (l & 15).  k-step s
// (32 inputs) of the next layer takes B element j of lane group g from
// acc[2s + (j >> 2)][S][j & 3]: the weights are packed in that k order
// (packing.kmap16), so no value crosses lanes between layers.
//
// A packed k-group is (k-step, half of the outputs): [piece 3][tile 8]
// [lane 64][8] bf16 = 24 KiB; tile t = output rows 16t .. 16t+15 of the half.
// A weight table TAB gives TAB::off(q), the byte offset of group q.
//
// wgrad.hip's weight-gradient GEMMs use the 32x32x16 helpers at the end.
//
// NR_F16 = 1 builds the same kernels as "f16x3" (the 3xTF32 scheme on CDNA4's
// fp16 matrix cores): each operand is split into two fp16 pieces x = hi + lo
// (22 significant bits) and the three products of order <= 2^-11
// (hi*hi, hi*lo, lo*hi) are accumulated in fp32 on
// v_mfma_f32_16x16x32_f16 / 32x32x16_f16: half the MFMAs of bf16x6 and 2/3 of
// its weight bytes.  fp16's 5-bit exponent is handled by exact power-of-two
// scaling: packed weights carry 2^kWScale (so their lo pieces stay normal),
// forward activations are split unscaled (|x| < 65504), gradients carry a
// per-sample scale renormalised layer by layer (mlp_bwd3.hip) and the weight
// gradient a per-layer scale from the observed maxima (wgrad.hip).  Error per
// product <= 3 * 2^-22 relative, plus an absolute floor of 2^-25 (fp16
// subnormal spacing / 2) per operand element.
#pragma once
#include <utility>
#include "layout.h"

// NR_X3_DBG (timing experiments only, never in the shipped build):
// 1 = no barrier, 2 = no DMA wait and no barrier, 3 = no DMA at all,
// 4 = no MFMA (fragments still read), 5 = no B split between k-steps,
// 8 = clock stamps (mlp_fwd3.hip writes s_memtime / s_memrealtime deltas),
// 9 = no saved-activation / gradient stores (store_n16)
#ifndef NR_X3_DBG
#define NR_X3_DBG 0
#endif
// NR_X3_SGB: interleave one MFMA with this many VALU instructions inside a
// tile (sched_group_barrier); 0 leaves the order to the scheduler
#ifndef NR_X3_SGB
#define NR_X3_SGB 1
#endif
#ifndef NR_F16
#define NR_F16 0
#endif
// NR_BF1 = 1 builds the same kernels as plain "bf16": one bf16 piece per
// operand, one product (hi*hi) per fp32 product, fp32 accumulation -- the
// reduced-precision MLP of BASELINE configs[1] ("bf16/fp32"), judged on PSNR
#ifndef NR_BF1
#define NR_BF1 0
#endif
#if NR_F16 && NR_BF1
#error "NR_F16 and NR_BF1 select different arithmetics"
#endif
// the bf16x6 object also carries the fp32-MFMA kernels and the shared entry points
#define NR_X3_BASE_OBJECT (!NR_F16 && !NR_BF1)
// exported C-ABI names of the split-operand entry points: _x3 (bf16x6), _h3 (f16x3), _b1 (bf16)
#if NR_F16
#define NR_X3_NAME(base) base##_h3
#elif NR_BF1
#define NR_X3_NAME(base) base##_b1
#else
#define NR_X3_NAME(base) base##_x3
#endif

namespace x3 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#if NR_F16
typedef f16x8 p8;                              // one MFMA operand fragment of a piece
typedef f16x2 p2;
typedef _Float16 p1;
constexpr int kNP = 2;                         // pieces per operand
constexpr int kNProd = 3;                      // piece products per fp32 product
#ifndef NR_H3_WSCALE
#define NR_H3_WSCALE 8
#endif
constexpr int kWScale = NR_H3_WSCALE;          // packed weights carry 2^kWScale
#elif NR_BF1
typedef bf16x8 p8;
typedef bf16x2 p2;
typedef __bf16 p1;
constexpr int kNP = 1;
constexpr int kNProd = 1;
constexpr int kWScale = 0;
#else
typedef bf16x8 p8;
typedef bf16x2 p2;
typedef __bf16 p1;
constexpr int kNP = 3;
constexpr int kNProd = 6;
constexpr int kWScale = 0;
#endif
// 2^-kWScale: takes a layer's accumulator (weights scaled) back to true values
constexpr float kWUnscale = 1.0f / (float)(1 << kWScale);

// waves per workgroup sharing one weight ring.  A kernel may set it before
// including this header (mlp_bwd3.hip's two-waves-per-SIMD form: 8 waves of
// one 16-sample tile each); the DMA of a group is split over the waves.
#ifndef NR_X3_WAVES
#define NR_X3_WAVES 4
#endif
constexpr int kWaves = NR_X3_WAVES;
constexpr int kTiles = 8;                          // output tiles (16 rows) per k-group
// ring depth in k-groups: the DMA of group q is issued kSlots-1 groups before
// q is consumed, and the wait for it also waits for every older store (vmcnt
// retires in issue order), so a deeper ring gives the saved-activation stores
// more time to be acknowledged.  f16x3 groups are 16 KiB: 6 slots fit.
#ifndef NR_X3_SLOTS
#define NR_X3_SLOTS (NR_F16 ? 6 : (NR_BF1 ? 8 : 4))
#endif
constexpr int kSlots = NR_X3_SLOTS;
constexpr int kSlotBytes = kNP * kTiles * 1024;    // pieces x 8 tiles x 1 KiB
constexpr int kDma = kNP * kTiles / kWaves;        // DMA instructions per wave per group
static_assert(kDma * kWaves == kNP * kTiles, "a group's DMA must split evenly over the waves");
// Merged ring (NR_X3_MERGE): the groups of one k-step (both output halves of a
// 256-wide layer) share one ring slot of 2 groups and ONE hand-over (wait +
// barrier) instead of one per group; the packed layout is unchanged (the two
// halves are adjacent).  TAB::sg(q) maps group q to its k-step ("super-group"),
// TAB::first(G) / TAB::size(G) give a super-group's first group and group
// count.  The DMA of super-group G + kSS - 1 is issued during G.  Halves the
// barriers of the 256-wide layers (dev/mb_w8.hip "32 KiB groups").
#ifndef NR_X3_MERGE
#define NR_X3_MERGE (NR_F16 || NR_BF1)
#endif
constexpr bool kMerge = NR_X3_MERGE;
#ifndef NR_X3_SSLOTS
#define NR_X3_SSLOTS (NR_F16 ? 3 : (NR_BF1 ? 6 : 2))
#endif
constexpr int kSS = NR_X3_SSLOTS;                  // super-slots of the merged ring
// the DMA issued during super-group G must be for G + 2 or later: for G + 1
// (kSS = 2) the hand-over's vmcnt, which leaves the current half's stores in
// flight, can leave that DMA's last instructions in flight too (measured: a
// run-to-run gradient difference)
static_assert(!kMerge || kSS >= 3, "merged ring needs >= 3 super-slots");
constexpr int kSuperBytes = 2 * kSlotBytes;
constexpr int kRingBytes = kMerge ? kSS * kSuperBytes : kSlots * kSlotBytes;

template <int V> using IC = std::integral_constant<int, V>;

typedef f32x4 Act[16][2];                      // 256-wide activation of one wave (two sample tiles)
template <int NS> using ActN = f32x4[16][NS];  // ... of NS sample tiles

// vm operations this wave issued after its DMA for group q by the time group
// q is consumed: the DMA of the kSlots-2 groups after it (merged ring: of the
// kSS-2 super-groups after q's) -- stores only add, so the count is a safe
// lower bound
template <class TAB, int Q, int QEND>
__host__ __device__ constexpr int wait_count() {
    int n = 0;
    if constexpr (kMerge) {
        const int G = TAB::sg(Q);
        for (int H = G + 1; H <= G + kSS - 2; ++H)
            for (int q = TAB::first(H); q < TAB::first(H) + TAB::size(H); ++q)
                if (q < QEND) n += kDma;
    } else {
        for (int k = Q + 1; k <= Q + kSlots - 2; ++k)
            if (k < QEND) n += kDma;
    }
    return n;
}

// LDS byte offset of group Q's ring slot
template <class TAB, int Q>
__host__ __device__ constexpr int slot_off() {
    if constexpr (kMerge)
        return (TAB::sg(Q) % kSS) * kSuperBytes + (Q - TAB::first(TAB::sg(Q))) * kSlotBytes;
    else
        return (Q % kSlots) * kSlotBytes;
}

// the group whose DMA instructions run during group Q (>= QEND: none).  Merged:
// position p of super-group G feeds position p of G + kSS - 1 (super-group
// sizes never grow along a kernel's sequence, checked here)
template <class TAB, int Q, int QEND>
__host__ __device__ constexpr int dma_target() {
    if constexpr (kMerge) {
        constexpr int G = TAB::sg(Q), p = Q - TAB::first(G), G2 = G + kSS - 1;
        static_assert(TAB::first(G2) >= QEND || TAB::size(G2) <= TAB::size(G),
                      "merged ring: a super-group larger than the one issuing its DMA");
        return p < TAB::size(G2) ? TAB::first(G2) + p : (1 << 30);
    } else {
        return Q + kSlots - 1;
    }
}

// LDS-DMA of the packed weights: buffer_load_dwordx4 ... lds with a scalar
// byte offset (group offset + fragment) and the lane's 16 B in voffset, the
// LDS destination (M0) scalar: no VALU per DMA instruction
struct Dma {
    __amdgpu_buffer_rsrc_t rsrc;
    char* ring;
    int wave;   // wave index, provably uniform (readfirstlane)
    int voff;   // lane * 16
};

__device__ __forceinline__ Dma make_dma(const char* packed, int64_t bytes, char* ring, int wave,
                                        int lane) {
    Dma d;
    d.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)packed, 0, (int)bytes, 0x00020000);
    d.ring = ring;
    d.wave = wave;
    d.voff = lane * 16;
    return d;
}

// DMA instruction k (of kDma) of this wave for group Q: fragment i = wave + 4k
template <class TAB, int Q, int QEND>
__device__ __forceinline__ void dma_one(const Dma& d, int k) {
    if constexpr (Q < QEND && NR_X3_DBG != 3) {
        const int i = d.wave + kWaves * k;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            d.rsrc, (__attribute__((address_space(3))) void*)(d.ring + slot_off<TAB, Q>() + i * 1024), 16,
            d.voff, (int)TAB::off(Q) + i * 1024, 0, 0);
    }
}

template <class TAB, int Q, int QEND>
__device__ __forceinline__ void stage(const Dma& d) {
#pragma unroll
    for (int k = 0; k < kDma; ++k) dma_one<TAB, Q, QEND>(d, k);
}

// stages groups 0 .. kSlots-2 (merged: super-groups 0 .. kSS-2)
template <class TAB, int QEND, int Q = 0>
__device__ __forceinline__ void prologue(const Dma& d) {
    constexpr int LIM = kMerge ? TAB::first(kSS - 1) : kSlots - 1;
    if constexpr (Q < LIM) {
        stage<TAB, Q, QEND>(d);
        prologue<TAB, QEND, Q + 1>(d);
    }
}

// group Q may be read once this wave's DMA landed and every wave passed here.
// vmcnt retires in issue order (loads, stores and LDS-DMA together), so the
// EXTRA stores issued after group Q's DMA in the current group are left in
// flight too; older stores are waited for (they have had a group to land).
template <class TAB, int Q, int QEND, int EXTRA = 0>
__device__ __forceinline__ void ring_enter() {
    if constexpr (NR_X3_DBG < 2)
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(wait_count<TAB, Q, QEND>() + EXTRA) : "memory");
    if constexpr (NR_X3_DBG == 0) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// exact 3-way split of fp32 values into bf16 pieces (round-to-nearest).  The
// conversions are packed (v_cvt_pk_bf16_f32) but the residual subtractions
// stay scalar: packed f32 VALU (v_pk_add_f32) costs ~13 cycles per
// instruction beside MFMAs (MI355X_MICROARCH.md), so the library is built
// with -fno-slp-vectorize.
__device__ __forceinline__ float bf16_as_f32(bf16x2 v, int i) {
    const uint32_t u = __builtin_bit_cast(uint32_t, v);
    return __uint_as_float(i == 0 ? u << 16 : u & 0xffff0000u);
}
__device__ __forceinline__ void split2(float x0, float x1, bf16x2& hi, bf16x2& mid, bf16x2& lo) {
    hi = __builtin_convertvector((f32x2){x0, x1}, bf16x2);
    const float r0 = x0 - bf16_as_f32(hi, 0), r1 = x1 - bf16_as_f32(hi, 1);
    mid = __builtin_convertvector((f32x2){r0, r1}, bf16x2);
    const float s0 = r0 - bf16_as_f32(mid, 0), s1 = r1 - bf16_as_f32(mid, 1);
    lo = __builtin_convertvector((f32x2){s0, s1}, bf16x2);
}
// f16x3: hi = RN(x) (v_cvt_pk_f16_f32), lo = RN(x - hi); x - hi is exact in
// fp32.  The residual is one v_fma_mix_f32 per value (-hi as an fp16 operand
// times 1.0 plus x, a single exact rounding) instead of a conversion and a
// subtraction: the split is VALU-issue-bound between MFMAs.
#ifndef NR_H3_MIX
#define NR_H3_MIX 1
#endif
__device__ __forceinline__ void split2h(float x0, float x1, f16x2& hi, f16x2& lo) {
    hi = __builtin_convertvector((f32x2){x0, x1}, f16x2);
#if NR_H3_MIX
    float r0, r1;
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r0) : "v"(hi), "v"(x0));
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r1) : "v"(hi), "v"(x1));
#else
    const float r0 = x0 - (float)hi[0], r1 = x1 - (float)hi[1];
#endif
    lo = __builtin_convertvector((f32x2){r0, r1}, f16x2);
}

#if NR_F16
struct Pieces { p8 hi, lo; };
#elif NR_BF1
struct Pieces { p8 hi; };
#else
struct Pieces { p8 hi, mid, lo; };
#endif

// pieces of two values as one p2 per piece (k = 0 hi, then mid (bf16x6), lo)
__device__ __forceinline__ void split_p2(float x0, float x1, p2 (&o)[kNP]) {
#if NR_F16
    split2h(x0, x1, o[0], o[1]);
#elif NR_BF1
    o[0] = __builtin_convertvector((f32x2){x0, x1}, bf16x2);
#else
    split2(x0, x1, o[0], o[1], o[2]);
#endif
}

// elements j = 2p, 2p+1 of a B fragment
__device__ __forceinline__ void split_pair(float x0, float x1, int p, Pieces& b) {
    p2 q[kNP];
    split_p2(x0, x1, q);
    b.hi[2 * p] = q[0][0]; b.hi[2 * p + 1] = q[0][1];
#if NR_F16
    b.lo[2 * p] = q[1][0]; b.lo[2 * p + 1] = q[1][1];
#elif NR_BF1
#else
    b.mid[2 * p] = q[1][0]; b.mid[2 * p + 1] = q[1][1];
    b.lo[2 * p] = q[2][0]; b.lo[2 * p + 1] = q[2][1];
#endif
}

// pin a value to this point of the instruction stream (the compiler would
// otherwise sink the next k-step's split down to its first use, after the
// barrier, where nothing hides it)
__device__ __forceinline__ void pin(Pieces& p) {
#if NR_F16
    asm volatile("" : "+v"(p.hi), "+v"(p.lo));
#elif NR_BF1
    asm volatile("" : "+v"(p.hi));
#else
    asm volatile("" : "+v"(p.hi), "+v"(p.mid), "+v"(p.lo));
#endif
}

// Lane-pair exchanges without an LDS round trip (__shfl_xor goes through
// ds_bpermute: ~100 cycles of latency each, exposed at one wave per SIMD).
// v_permlane16_swap (v_permlane32_swap) of x with itself leaves lanes l and
// l ^ 16 (l ^ 32) holding the pair {x[l], x[l ^ 16]} split across the two
// results, so for a commutative op, op(r0, r1) == op(x[l], x[l ^ 16]) in
// every lane -- bit for bit the __shfl_xor form (IEEE + and max commute).
__device__ __forceinline__ void pair16(float x, float& r0, float& r1) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    r0 = __uint_as_float(r[0]);
    r1 = __uint_as_float(r[1]);
}
__device__ __forceinline__ void pair32(float x, float& r0, float& r1) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    r0 = __uint_as_float(r[0]);
    r1 = __uint_as_float(r[1]);
}
// x[l] + x[l ^ 16] + x[l ^ 32] + x[l ^ 48] in the __shfl_xor order (16, then 32)
__device__ __forceinline__ float sum_over_groups(float x) {
    float a, b;
    pair16(x, a, b);
    x = a + b;
    pair32(x, a, b);
    return a + b;
}
// max over the 4 lane groups of 16 (l, l ^ 16, l ^ 32, l ^ 48)
__device__ __forceinline__ float max_over_groups(float x) {
    float a, b;
    pair16(x, a, b);
    x = fmaxf(a, b);
    pair32(x, a, b);
    return fmaxf(a, b);
}
// max over the wave, in every lane: DPP within rows of 16 (quad xor 1, xor 2,
// half-row mirror, row mirror), then the two swaps (max is order-free)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_max(float x) {
    x = fmaxf(x, dpp_f<0xB1>(x));     // quad_perm [1,0,3,2]
    x = fmaxf(x, dpp_f<0x4E>(x));     // quad_perm [2,3,0,1]
    x = fmaxf(x, dpp_f<0x141>(x));    // row_half_mirror
    x = fmaxf(x, dpp_f<0x140>(x));    // row_mirror
    return max_over_groups(x);
}

// ReLU as an integer max: negative floats (and -0) have the sign bit set
__device__ __forceinline__ float relu_i(float x) {
    return __int_as_float(max(__float_as_int(x), 0));
}

// the weight pieces of one output tile of a k-group
struct Frag { p8 p[kNP]; };

template <class TAB, int Q>
__device__ __forceinline__ void rd_frag(char* ring, int lane, int t, Frag& f) {
    const char* s = ring + slot_off<TAB, Q>() + lane * 16 + t * 1024;
#pragma unroll
    for (int k = 0; k < kNP; ++k) f.p[k] = *reinterpret_cast<const p8*>(s + k * kTiles * 1024);
}

// LDS fragment lookahead in tiles: the weight fragments of tile t + kPF are
// read while tile t multiplies (NR_X3_PF = 2 hands the next group over one
// tile earlier and keeps a third fragment set, 8 more VGPRs)
#ifndef NR_X3_PF
#define NR_X3_PF 1
#endif
constexpr int kPF = NR_X3_PF;
static_assert(kPF >= 1 && kPF <= 2, "fragment lookahead of 1 or 2 tiles");
// the fragments of the next group's first kPF tiles, carried between groups
struct Ahead { Frag f[kPF]; };

// hand group Q over (wait + barrier) and read its tile-0 fragments; in the
// merged ring a group that shares its predecessor's super-group arrived with
// it, and only its tile-0 fragments are read
template <class TAB, int Q, int QEND, int EXTRA = 0>
__device__ __forceinline__ void enter(char* ring, int lane, Frag& f0) {
    if constexpr (Q < QEND) {
        if constexpr (!(kMerge && Q > 0 && TAB::sg(Q) == TAB::sg(Q - 1)))
            ring_enter<TAB, Q, QEND, EXTRA>();
        rd_frag<TAB, Q>(ring, lane, 0, f0);
    }
}
template <class TAB, int Q, int QEND, int EXTRA = 0>
__device__ __forceinline__ void enter(char* ring, int lane, Ahead& a) {
    enter<TAB, Q, QEND, EXTRA>(ring, lane, a.f[0]);
    if constexpr (Q < QEND && kPF > 1) rd_frag<TAB, Q>(ring, lane, 1, a.f[1]);
}

__device__ __forceinline__ f32x4 mfma16(const p8& a, const p8& b, f32x4 c) {
#if NR_F16
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
#else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
#endif
}

// c[S] += W * B[S] for the wave's NS sample tiles: the piece products
// (bf16x6: six of order <= 2^-16; f16x3: three of order <= 2^-11), small
// terms first, the accumulators alternating
template <int NS>
__device__ __forceinline__ void x6_multi(const Frag& w, const Pieces (&b)[NS], f32x4 (&c)[NS]) {
    if constexpr (NR_X3_DBG == 4) {
#pragma unroll
        for (int j = 0; j < NS; ++j) asm volatile("" ::"v"(w.p[0]), "v"(w.p[kNP - 1]), "v"(b[j].hi));
        return;
    }
    auto prod = [&](const p8& a, auto piece) {
#pragma unroll
        for (int j = 0; j < NS; ++j) c[j] = mfma16(a, piece(b[j]), c[j]);
    };
#if NR_F16
    prod(w.p[1], [](const Pieces& x) { return x.hi; });
    prod(w.p[0], [](const Pieces& x) { return x.lo; });
    prod(w.p[0], [](const Pieces& x) { return x.hi; });
#elif NR_BF1
    prod(w.p[0], [](const Pieces& x) { return x.hi; });
#else
    prod(w.p[2], [](const Pieces& x) { return x.hi; });
    prod(w.p[0], [](const Pieces& x) { return x.lo; });
    prod(w.p[1], [](const Pieces& x) { return x.mid; });
    prod(w.p[1], [](const Pieces& x) { return x.hi; });
    prod(w.p[0], [](const Pieces& x) { return x.mid; });
    prod(w.p[0], [](const Pieces& x) { return x.hi; });
#endif
}

// initial accumulator of the first k-step of a layer
struct ZeroInit {
    __device__ __forceinline__ f32x4 operator()(int, int) const { return f32x4{0.f, 0.f, 0.f, 0.f}; }
};
struct BiasInit {     // bias[16F + 4g .. +3] (LDS), the same for both sample tiles
    const float* b; int g;
    __device__ __forceinline__ f32x4 operator()(int F, int) const {
        return *reinterpret_cast<const f32x4*>(b + 16 * F + 4 * g);
    }
};

// one k-group: acc[F0 + t][S] (+)= W_q[t] * B[S] for the 8 output tiles; with
// INIT the k-group starts from cinit(F, S) instead of acc.  On entry a holds
// tiles 0 .. kPF-1 of group Q; the fragments of tile t+kPF are read while tile
// t multiplies, and the hand-over of group Q+1 (wait, barrier, its tile-0
// read) is done before the MFMAs of tile 8 - kPF, so both the barrier and the
// first LDS latency of the next group hide under MFMAs in flight.  On exit a
// holds tiles 0 .. kPF-1 of group Q+1.  hook(t) runs inside tile t; its VALU
// work is interleaved with the tile's 2 kNProd MFMAs.  EXTRA: the stores the
// hooks issue before the hand-over tile (left in flight by its vmcnt wait).
// Accumulators of a tile in AGPRs ("a") or VGPRs ("v"); at two waves per SIMD
// a wave has 256 registers in all, so the split is the compiler's
#ifndef NR_X3_ACC_AGPR
#define NR_X3_ACC_AGPR 1
#endif
template <int NS>
__device__ __forceinline__ void pin_acc(f32x4 (&d)[NS]) {
#if NR_X3_ACC_AGPR
    if constexpr (NS == 2) {     // one statement for the pair (the round-5 register assignment)
        asm volatile("" : "+a"(d[0]), "+a"(d[1]));
        return;
    }
#endif
#pragma unroll
    for (int j = 0; j < NS; ++j) {
#if NR_X3_ACC_AGPR
        asm volatile("" : "+a"(d[j]));
#else
        asm volatile("" : "+v"(d[j]));
#endif
    }
}

template <class TAB, int Q, int QEND, int F0, bool INIT, int EXTRA, typename CInit, typename Hook, int NF,
          int NS>
__device__ __forceinline__ void group_mm(char* ring, int lane, f32x4 (&acc)[NF][NS],
                                         const Pieces (&b)[NS], CInit& cinit, Hook& hook, Ahead& a) {
    constexpr int NR = kPF + 1;       // fragment sets in registers
    Frag f[NR];
#pragma unroll
    for (int i = 0; i < kPF; ++i) f[i] = a.f[i];
    f32x4 ci[2][NS];
    if constexpr (INIT) {
#pragma unroll
        for (int j = 0; j < NS; ++j) ci[0][j] = cinit(F0, j);
    }
#pragma unroll
    for (int t = 0; t < kTiles; ++t) {
        const int tn = t + kPF;
        if (tn < kTiles) rd_frag<TAB, Q>(ring, lane, tn, f[tn % NR]);
        else if (tn == kTiles) enter<TAB, Q + 1, QEND, EXTRA>(ring, lane, a.f[0]);
        else if constexpr (Q + 1 < QEND) rd_frag<TAB, Q + 1>(ring, lane, tn - kTiles, a.f[tn - kTiles]);
        if constexpr (INIT) {
            if (t + 1 < kTiles) {
#pragma unroll
                for (int j = 0; j < NS; ++j) ci[(t + 1) & 1][j] = cinit(F0 + t + 1, j);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        f32x4 (&d)[NS] = acc[F0 + t];
        if constexpr (INIT) {
#pragma unroll
            for (int j = 0; j < NS; ++j) d[j] = ci[t & 1][j];
        }
        x6_multi<NS>(f[t % NR], b, d);
        // keep the tile's MFMAs in this tile: MFMA intrinsics have no side
        // effects, so without an ordered use the instruction selector may
        // float them anywhere in the (huge) basic block
        pin_acc<NS>(d);
        hook(t);
#if NR_X3_SGB
#pragma unroll
        for (int i = 0; i < NS * kNProd; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);          // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, NR_X3_SGB, 0);  // VALU
        }
#endif
        __builtin_amdgcn_sched_barrier(0);
    }
}

// ---- layer segments ---------------------------------------------------------
// A segment is KS k-steps of one layer's inputs with NH output halves: group
// Q0 + NH s + hf multiplies k-step s into output tiles 8hf .. 8hf+7.
//   getu(IC<s>, S, p, x0, x1): B elements 2p, 2p+1 of k-step s, sample tile S
//     (the producer's activation applied: bias is already in the values)
//   nextu: getu of the segment that follows; its k-step 0 is split during
//     this segment's last k-step, so no layer boundary waits on a split
//   cinit(F, S): initial accumulator (INIT: the layer's first segment)
//   side(IC<G>, t): side work at tile t of group G (output stores)
// The 8 split units (S, p) of the next k-step run one per tile of the last
// half's group; one DMA instruction of group Q+3 runs per tile 0..5.
//   Getters declare kStores (a global store per odd unit), sides before(T),
//   the stores they issue in a group before its tile T (the hand-over tile,
//   where the next group's DMA is waited for).
// Getters also have begin(producer): called before their first unit once the
// getter that fed this layer (the producer) has split all of its units.
struct NoNext {
    static constexpr bool kStores = false;
    static constexpr bool kPaired = false;
    template <typename P> __device__ __forceinline__ void begin(const P&) {}
    template <typename T> __device__ __forceinline__ void operator()(T, int, int, float& x0, float& x1) const {
        x0 = x1 = 0.f;
    }
};
template <typename T> struct IsNoNext { static constexpr bool value = false; };
template <> struct IsNoNext<NoNext> { static constexpr bool value = true; };

struct NoSide {
    static constexpr int before(int) { return 0; }
    template <typename T> __device__ __forceinline__ void operator()(T, int) const {}
};

template <typename GetU, int s, int NS>
__device__ __forceinline__ void split_unit(GetU& getu, IC<s>, int u, Pieces (&bn)[NS]) {
    if constexpr (NR_X3_DBG == 5) return;
    const int sb = u >> 2, p = u & 3;
    float x0, x1;
    getu(IC<s>(), sb, p, x0, x1);
    split_pair(x0, x1, p, bn[sb]);
    pin(bn[sb]);
}

template <typename GetU, int NS>
__device__ __forceinline__ void split_all(GetU& getu, Pieces (&b)[NS]) {
#pragma unroll
    for (int u = 0; u < 4 * NS; ++u) {
        const int sb = u >> 2, p = u & 3;
        float x0, x1;
        getu(IC<0>(), sb, p, x0, x1);
        split_pair(x0, x1, p, b[sb]);
    }
}

// split unit u (= 4 S + p) run at tile t of half HF: NH = 2 spreads the 4 NS
// units over tiles 3 .. 2 + 2 NS of both halves (the last k-step's units read
// output tiles 0, 1 of the layer, final after tiles 0, 1 of half 0); NH = 1
// runs one per tile
template <int NH, int HF, int NS = 2>
__host__ __device__ constexpr int unit_at(int t) {
    if constexpr (NH == 1) return t < 4 * NS ? t : -1;
    else return t >= 3 && t < 3 + 2 * NS ? 2 * NS * HF + t - 3 : -1;
}
// the tile whose start hands the next group over (x3.h group_mm)
constexpr int kHandTile = kTiles - kPF;
// stores a storing getter issues before the hand-over tile of its group: one
// per odd unit, or (PAIRED: the two halves of a 128-B row line together, x3.h
// store_row_pair) two per unit p = 3
template <int NH, int HF, bool PAIRED = false, int NS = 2>
__host__ __device__ constexpr int stores_before_hand() {
    int n = 0;
    for (int t = 0; t < kHandTile; ++t) {
        const int u = unit_at<NH, HF, NS>(t);
        if (u < 0) continue;
        if (PAIRED) n += (u & 3) == 3 ? 2 : 0;
        else n += u & 1;
    }
    return n;
}

template <class TAB, int Q0, int S, int KS, int NH, int QEND, bool INIT, int HF, typename GetU,
          typename NextU, typename CInit, typename Side, int NF, int NS>
__device__ __forceinline__ void seg_group(const Dma& dma, int lane, f32x4 (&acc)[NF][NS], GetU& getu,
                                          NextU& nextu, CInit& cinit, Side& side,
                                          const Pieces (&b)[NS], Pieces (&bn)[NS], Ahead& f0) {
    if constexpr (HF < NH) {
        constexpr int Q = Q0 + NH * S + HF;
        auto hook = [&](int t) {
            if (t < kDma) dma_one<TAB, dma_target<TAB, Q, QEND>(), QEND>(dma, t);
            const int u = unit_at<NH, HF, NS>(t);
            if (u >= 0) {
                if constexpr (S + 1 < KS) split_unit(getu, IC<S + 1>(), u, bn);
                else if constexpr (!IsNoNext<NextU>::value) {
                    if (u == 0) nextu.begin(getu);   // getu's splits are complete
                    split_unit(nextu, IC<0>(), u, bn);
                }
            }
            side(IC<NH * S + HF>(), t);
        };
        constexpr bool ust = S + 1 < KS ? GetU::kStores : NextU::kStores;
        constexpr bool upr = S + 1 < KS ? GetU::kPaired : NextU::kPaired;
        constexpr int extra = (ust ? stores_before_hand<NH, HF, upr, NS>() : 0) + Side::before(kHandTile);
        group_mm<TAB, Q, QEND, 8 * HF, INIT && S == 0, extra>(dma.ring, lane, acc, b, cinit, hook, f0);
        seg_group<TAB, Q0, S, KS, NH, QEND, INIT, HF + 1>(dma, lane, acc, getu, nextu, cinit, side,
                                                          b, bn, f0);
    }
}

template <class TAB, int Q0, int S, int KS, int NH, int QEND, bool INIT, typename GetU,
          typename NextU, typename CInit, typename Side, int NF, int NS>
__device__ __forceinline__ void seg_from(const Dma& dma, int lane, f32x4 (&acc)[NF][NS], GetU& getu,
                                         NextU& nextu, CInit& cinit, Side& side,
                                         Pieces (&b)[NS], Ahead& f0) {
    if constexpr (S < KS) {
        Pieces bn[NS];
        seg_group<TAB, Q0, S, KS, NH, QEND, INIT, 0>(dma, lane, acc, getu, nextu, cinit, side, b, bn, f0);
#pragma unroll
        for (int j = 0; j < NS; ++j) b[j] = bn[j];
        seg_from<TAB, Q0, S + 1, KS, NH, QEND, INIT>(dma, lane, acc, getu, nextu, cinit, side, b, f0);
    }
}

// b: on entry the pieces of this segment's k-step 0, on exit those of the
// next segment's k-step 0 (split by nextu)
template <class TAB, int Q0, int KS, int NH, int QEND, bool INIT, typename GetU, typename NextU,
          typename CInit, typename Side, int NF, int NS>
__device__ __forceinline__ void segment(const Dma& dma, int lane, f32x4 (&acc)[NF][NS], GetU& getu,
                                        NextU& nextu, CInit& cinit, Side& side, Pieces (&b)[NS],
                                        Ahead& f0) {
    seg_from<TAB, Q0, 0, KS, NH, QEND, INIT>(dma, lane, acc, getu, nextu, cinit, side, b, f0);
}

// B fragment element of k-step s from an accumulator input (packing.kmap16)
template <int NF, int NS>
__device__ __forceinline__ float acc_b(const f32x4 (&X)[NF][NS], int s, int sb, int j) {
    return X[2 * s + (j >> 2)][sb][j & 3];
}

// ---- block-native saved layout of the bf16x6 pipeline ("N16") -------------
// Width-W segment of a 32-sample block: [F = W/16][S 2][lane 64][4] floats,
// element (F, S, l, r) = feature 16F + 4(l >> 4) + r of sample 16S + (l & 15):
// one wave store of acc[F][S] moves a contiguous 1 KiB.
// saved activations / gradients are written with non-temporal stores: they
// are re-read only by a later kernel, and streaming them past L2 keeps the
// weight ring's L2 lines resident (f16x3 fine pass: fwd+save 2.86 -> 2.63 ms,
// dgrad 3.07 -> 2.56 ms)
#ifndef NR_NT_STORE
#define NR_NT_STORE 1
#endif
// NR_BF1 (plain bf16): a saved segment holds the values rounded to bf16 --
// exactly what the weight gradient's bf16 MFMA operands are, so nothing is
// lost.  Chunk (F, S) of a block (16 features x 16 samples, 512 B) is stored
// sample-major: sample 16S + j, features 16F + 4g .. +3 (the lane 16g + j
// float4 of the fp32 layout) at 8-B slot 4j + g, i.e. [sample][16 features]
// rows of 32 B.  One wave store still covers the chunk's contiguous 512 B,
// and wgrad.hip's LDS-DMA copies chunks as they are and reads its MFMA
// fragments with ds_read_b64_tr_b16 (one 4-sample x 16-feature block per
// 16 lanes).  Blocks are packed at half the fp32 block stride (NR_SEGF):
// segments keep their fp32 offsets and sizes inside the buffers, and a
// segment's blocks fill the first half of it contiguously -- at the fp32
// stride every read skipped every other 16 KiB, which left the weight
// gradient's stream at 58% of HBM bandwidth.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
// floats from one block of a width-w saved segment to the next
#if NR_BF1
#define NR_SEGF(w) (NR_NATIVE(w) / 2)
#else
#define NR_SEGF(w) NR_NATIVE(w)
#endif
__device__ __forceinline__ u32x2 pack_bf16x4(const f32x4& v) {
    const bf16x2 a = __builtin_convertvector((f32x2){v[0], v[1]}, bf16x2);
    const bf16x2 b = __builtin_convertvector((f32x2){v[2], v[3]}, bf16x2);
    return u32x2{__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b)};
}
__device__ __forceinline__ f32x4 unpack_bf16x4(u32x2 u) {
    return f32x4{__uint_as_float(u[0] << 16), __uint_as_float(u[0] & 0xffff0000u),
                 __uint_as_float(u[1] << 16), __uint_as_float(u[1] & 0xffff0000u)};
}
// four values (one lane's float4) to float4 slot `idx` of a saved segment
// slot of the float4 idx = 64 chunk + 16 g + j of the fp32 layout in the bf16 layout
__host__ __device__ __forceinline__ int64_t bf16_slot(int64_t idx) {
    return (idx & ~(int64_t)63) | (4 * (idx & 15) + ((idx >> 4) & 3));
}
__device__ __forceinline__ void store_slot(const f32x4& v, float* __restrict__ seg, int64_t idx) {
#if NR_BF1
    u32x2* p = reinterpret_cast<u32x2*>(seg) + bf16_slot(idx);
#if NR_X3_DBG == 9
    asm volatile("" ::"v"(v), "v"(p));
#elif NR_NT_STORE
    __builtin_nontemporal_store(pack_bf16x4(v), p);
#else
    *p = pack_bf16x4(v);
#endif
#else
    f32x4* p = reinterpret_cast<f32x4*>(seg) + idx;
#if NR_X3_DBG == 9
    asm volatile("" ::"v"(v), "v"(p));
#elif NR_NT_STORE && NR_ROW_NT
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
#endif
}
__device__ __forceinline__ void store_n16(const f32x4& v, int F, int S, float* __restrict__ blk,
                                          int lane) {
#if NR_BF1
    store_slot(v, blk, (F * 2 + S) * 64 + lane);
    return;
#endif
    f32x4* p = reinterpret_cast<f32x4*>(blk + ((F * 2 + S) * 64 + lane) * 4);
#if NR_X3_DBG == 9
    asm volatile("" ::"v"(v), "v"(p));     // timing experiment: no stores
#elif NR_NT_STORE
    __builtin_nontemporal_store(v, p);     // streamed: keep L2 for the weight ring
#else
    *p = v;
#endif
}

// A forward activation saved for the weight gradient (f16x3 / bf16x6):
// sample-major rows of W floats, block of 32 samples after block -- the
// lane's four values (features 16 F + 4 g .. +3 of sample 16 S + j, lane =
// 16 g + j) go to row 16 S + j.  A store instruction writes 16 rows x 64 B;
// the weight gradient then reads any sample's row contiguously, so gathering
// the samples with a nonzero output gradient (active.hip) moves only their
// bytes.  The bf16 variant keeps its N16 slots (store_slot, read by LDS-DMA).
#ifndef NR_ROW_NT
#define NR_ROW_NT 1      // row stores non-temporal like the N16 ones (A/B knob)
#endif
template <int W>
__device__ __forceinline__ void store_row(const f32x4& v, int F, int S, float* __restrict__ blk,
                                          int lane) {
#if NR_BF1
    store_n16(v, F, S, blk, lane);
#else
    f32x4* p = reinterpret_cast<f32x4*>(blk + (16 * S + (lane & 15)) * W + 16 * F + 4 * (lane >> 4));
#if NR_X3_DBG == 9
    asm volatile("" ::"v"(v), "v"(p));
#elif NR_NT_STORE && NR_ROW_NT
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
#endif
}

// NR_ROW_PAIR (the row stores of the full graph's forward): 0 = each 64-B
// half of a sample's 128-B row line stored as soon as its tile is split (two
// units apart; round 3); 1 = both halves stored back to back; 2 (shipped) =
// whole lines: the odd tile's values rotated by 8 lanes within each 16-lane
// row (DPP row_ror:8 with bank masks), so that one store writes 8 samples x
// 128 B.  Measured (profiles/r04/ab_rowpair, abalt_pair2): the fine forward's
// WRITE_SIZE 10.63 -> 8.33 GB (1.30x -> 1.02x its 8.18 GB of activations),
// its time unchanged, the data gradient that follows it 1.54 -> 1.45 ms and
// the cfg2 step +1.5% (three alternating rounds on one box)
#ifndef NR_ROW_PAIR
#define NR_ROW_PAIR 2
#endif
constexpr bool kRowPair = NR_ROW_PAIR != 0 && !NR_BF1;

// tiles F0 (even) and F0 + 1 of sample tile S: the 128-B row line [16 F0, 16 F0 + 32)
template <int W>
__device__ __forceinline__ void store_row_pair(const f32x4& t0, const f32x4& t1, int F0, int S,
                                               float* __restrict__ blk, int lane) {
#if NR_ROW_PAIR == 2
    // lane (g, j): A = samples 16S + (j & 7), B = samples 16S + 8 + (j & 7);
    // in A lanes j < 8 write their own tile F0, lanes j >= 8 tile F0 + 1 of
    // lane j - 8; in B the other way round
    const int j = lane & 15, g = lane >> 4;
    f32x4 a, b;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int o = __float_as_int(t0[r]), s1 = __float_as_int(t1[r]);
        a[r] = __int_as_float(__builtin_amdgcn_update_dpp(o, s1, 0x128, 0xF, 0xC, false));
        b[r] = __int_as_float(__builtin_amdgcn_update_dpp(o, s1, 0x128, 0xF, 0x3, false));
    }
    const int hi = j >> 3;
    f32x4* pa = reinterpret_cast<f32x4*>(blk + (16 * S + (j & 7)) * W + 16 * F0 + 16 * hi + 4 * g);
    f32x4* pb = reinterpret_cast<f32x4*>(blk + (16 * S + 8 + (j & 7)) * W + 16 * F0 + 16 * (1 - hi) + 4 * g);
#if NR_X3_DBG == 9
    asm volatile("" ::"v"(a), "v"(b), "v"(pa), "v"(pb));
#elif NR_NT_STORE && NR_ROW_NT
    __builtin_nontemporal_store(a, pa);
    __builtin_nontemporal_store(b, pb);
#else
    *pa = a;
    *pb = b;
#endif
#else
    store_row<W>(t0, F0, S, blk, lane);
    store_row<W>(t1, F0 + 1, S, blk, lane);
#endif
}

// ReLU mask bits of a post-ReLU activation: word F >> 2 of the lane, bit
// 8 (F & 3) + 4 S + r (VALU only: bits(x) != 0)
__device__ __forceinline__ void mask_bits(const f32x4& v, int F, int S, uint32_t (&w)[4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
        w[F >> 2] |= min(__float_as_uint(v[r]), 1u) << (8 * (F & 3) + 4 * S + r);
}
__device__ __forceinline__ float mask_keep(float x, const uint32_t (&w)[4], int F, int S, int r) {
    return nr_mask_bit(x, w[F >> 2], 8 * (F & 3) + 4 * S + r);
}

// ---- 32x32x16 helpers (wgrad.hip) ------------------------------------------
__device__ __forceinline__ f32x16 mfma32(const p8& a, const p8& b, f32x16 c) {
#if NR_F16
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
#else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
#endif
}

// acc += A * B, small products first; a = the A pieces (hi[, mid], lo)
__device__ __forceinline__ f32x16 mfma_xp(const p8 (&a)[kNP], const Pieces& b, f32x16 acc) {
#if NR_F16
    acc = mfma32(a[1], b.hi, acc);
    acc = mfma32(a[0], b.lo, acc);
    acc = mfma32(a[0], b.hi, acc);
#elif NR_BF1
    acc = mfma32(a[0], b.hi, acc);
#else
    acc = mfma32(a[2], b.hi, acc);
    acc = mfma32(a[0], b.lo, acc);
    acc = mfma32(a[1], b.mid, acc);
    acc = mfma32(a[1], b.hi, acc);
    acc = mfma32(a[0], b.mid, acc);
    acc = mfma32(a[0], b.hi, acc);
#endif
    return acc;
}

// acc[j] += A * B[j] for NJ accumulators sharing the A pieces, product-major
template <int NJ>
__device__ __forceinline__ void mfma_xp_multi(const p8 (&a)[kNP], const Pieces (&b)[NJ], f32x16* acc) {
#if NR_F16
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = mfma32(a[1], b[j].hi, acc[j]);
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = mfma32(a[0], b[j].lo, acc[j]);
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = mfma32(a[0], b[j].hi, acc[j]);
#elif NR_BF1
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = mfma32(a[0], b[j].hi, acc[j]);
#else
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = mfma32(a[2], b[j].hi, acc[j]);
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = mfma32(a[0], b[j].lo, acc[j]);
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = mfma32(a[1], b[j].mid, acc[j]);
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = mfma32(a[1], b[j].hi, acc[j]);
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = mfma32(a[0], b[j].mid, acc[j]);
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = mfma32(a[0], b[j].hi, acc[j]);
#endif
}

// power of two 2^(target - e), e = the binary exponent of m (m in [2^e, 2^(e+1))),
// shift clamped to [-lim, lim]; 1 for m == 0 (or a non-finite m)
__device__ __forceinline__ float pow2_norm(float m, int target, int lim) {
    const int e = (int)((__float_as_uint(m) >> 23) & 0xff) - 127;
    if (!(m > 0.f) || e == 128) return 1.f;
    const int sh = min(max(target - e, -lim), lim);
    return __uint_as_float((uint32_t)(127 + sh) << 23);
}

}  // namespace x3
