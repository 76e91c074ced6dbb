// bf16x6 split-operand MFMA machinery shared by the fused MLP kernels
// (mlp_fwd3.hip, mlp_bwd3.hip): the exact three-piece bf16 split, the
// six-product v_mfma_f32_32x32x16_bf16 step, and the LDS ring of weight
// k-groups filled by LDS-DMA and handed over with one barrier per group.
//
// A weight table TAB describes the k-group sequence of one packed buffer:
//   TAB::tiles(q)  output tiles (32 rows) of group q (8 or 4)
//   TAB::off(q)    byte offset of group q; a group is [piece 3][tile][lane 64][8] bf16
#pragma once
#include <utility>
#include "layout.h"

// NR_X3_DBG (timing experiments only, never in the shipped build):
// 1 = no barrier, 2 = no DMA wait and no barrier, 3 = no DMA at all
#ifndef NR_X3_DBG
#define NR_X3_DBG 0
#endif

namespace x3 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kWaves = 4;
constexpr int kSlots = 4;                      // ring depth in k-groups
constexpr int kSlotBytes = 3 * 8 * 1024;       // 3 pieces x 8 tiles x 1 KiB
constexpr int kRingBytes = kSlots * kSlotBytes;

template <int V> using IC = std::integral_constant<int, V>;

// DMA instructions one wave issues for group q (each moves one 1 KiB fragment)
template <class TAB>
__host__ __device__ constexpr int grp_dma(int q) { return TAB::tiles(q) * 3 / kWaves; }

// vm operations this wave issued after its DMA for group q by the time group
// q is consumed: the DMA of the kSlots-2 groups after it (stores only add,
// so the count is a safe lower bound)
template <class TAB, int Q, int QEND>
__host__ __device__ constexpr int wait_count() {
    int n = 0;
    for (int k = Q + 1; k <= Q + kSlots - 2; ++k)
        if (k < QEND) n += grp_dma<TAB>(k);
    return n;
}

__device__ __forceinline__ char* slot_ptr(char* ring, int q) { return ring + (q % kSlots) * kSlotBytes; }

template <class TAB, int Q, int QEND>
__device__ __forceinline__ void stage(const char* __restrict__ packed, char* ring, int wave,
                                      int lane) {
    if constexpr (Q < QEND && NR_X3_DBG != 3) {
        constexpr int NT = TAB::tiles(Q);
        const char* src = packed + TAB::off(Q);
        char* dst = slot_ptr(ring, Q);
#pragma unroll
        for (int k = 0; k < NT * 3 / kWaves; ++k) {
            const int i = wave + kWaves * k;
            __builtin_amdgcn_global_load_lds(
                (const void*)(src + i * 1024 + lane * 16),
                (__attribute__((address_space(3))) void*)(dst + i * 1024), 16, 0, 0);
        }
    }
}

template <class TAB, int QEND>
__device__ __forceinline__ void prologue(const char* __restrict__ packed, char* ring, int wave,
                                         int lane) {
    static_assert(kSlots == 4, "prologue stages kSlots-1 groups");
    stage<TAB, 0, QEND>(packed, ring, wave, lane);
    stage<TAB, 1, QEND>(packed, ring, wave, lane);
    stage<TAB, 2, QEND>(packed, ring, wave, lane);
}
// forward declaration order: enter<> is defined below; kernels call
// enter<TAB, 0, QEND>(ring, lane, f0) once after the prologue.

// group Q may be read once this wave's DMA landed and every wave passed here
template <class TAB, int Q, int QEND>
__device__ __forceinline__ void ring_enter() {
    if constexpr (NR_X3_DBG < 2)
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(wait_count<TAB, Q, QEND>()) : "memory");
    if constexpr (NR_X3_DBG == 0) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// exact 3-way split of fp32 values into bf16 pieces (round-to-nearest).  The
// conversions are packed (v_cvt_pk_bf16_f32 is nearly free beside MFMAs) but
// the residual subtractions stay scalar: packed f32 VALU (v_pk_add_f32) costs
// ~13 cycles per instruction beside MFMAs (MI355X_MICROARCH.md), so the
// library is built with -fno-slp-vectorize.
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

struct Pieces { bf16x8 hi, mid, lo; };
__device__ __forceinline__ Pieces split8(const float (&x)[8]) {
    Pieces p;
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
        bf16x2 h, m, l;
        split2(x[i], x[i + 1], h, m, l);
        p.hi[i] = h[0]; p.hi[i + 1] = h[1];
        p.mid[i] = m[0]; p.mid[i + 1] = m[1];
        p.lo[i] = l[0]; p.lo[i + 1] = l[1];
    }
    return p;
}

// acc += A * B with both operands given as pieces: the six products of order
// <= 2^-16, small terms first
__device__ __forceinline__ f32x16 mfma_x6(const bf16x8& ah, const bf16x8& am, const bf16x8& al,
                                          const Pieces& b, f32x16 acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, b.hi, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, b.lo, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, b.mid, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, b.hi, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, b.mid, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, b.hi, acc, 0, 0, 0);
    return acc;
}

// pin a value to this point of the instruction stream (the compiler would
// otherwise sink the next group's split down to its first use, after the
// barrier, where nothing hides it)
__device__ __forceinline__ void pin(Pieces& p) {
    asm volatile("" : "+v"(p.hi), "+v"(p.mid), "+v"(p.lo));
}

// the three weight pieces of one output tile of a k-group
struct Frag { bf16x8 p[3]; };

template <int Q, int NT>
__device__ __forceinline__ void rd_frag(char* ring, int lane, int t, Frag& f) {
    const char* s = slot_ptr(ring, Q) + lane * 16 + t * 1024;
    f.p[0] = *reinterpret_cast<const bf16x8*>(s);
    f.p[1] = *reinterpret_cast<const bf16x8*>(s + NT * 1024);
    f.p[2] = *reinterpret_cast<const bf16x8*>(s + 2 * NT * 1024);
}

// hand group Q over (wait + barrier) and read its tile-0 fragments
template <class TAB, int Q, int QEND>
__device__ __forceinline__ void enter(char* ring, int lane, Frag& f0) {
    if constexpr (Q < QEND) {
        ring_enter<TAB, Q, QEND>();
        rd_frag<Q, TAB::tiles(Q)>(ring, lane, 0, f0);
    }
}

// acc[j] += A * B[j] for NJ accumulators sharing the A pieces, product-major
// (independent accumulators alternate, so no MFMA waits on its predecessor)
template <int NJ>
__device__ __forceinline__ void mfma_x6_multi(const bf16x8& ah, const bf16x8& am, const bf16x8& al,
                                              const Pieces (&b)[NJ], f32x16* acc) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, b[j].hi, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, b[j].lo, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, b[j].mid, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, b[j].hi, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, b[j].mid, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, b[j].hi, acc[j], 0, 0, 0);
}

// one k-group: acc[t] += W_q[t] * B for the NT output tiles.  On entry f0
// holds tile 0 of group Q; the fragments of tile t+1 are read while tile t
// multiplies, and the hand-over of group Q+1 (wait, barrier, its tile-0 read)
// is done before the last tile's MFMAs, so both the barrier and the first LDS
// latency of the next group hide under MFMAs in flight.  On exit f0 holds
// tile 0 of group Q+1.  hook(t) runs after tile t's MFMAs are issued.
template <class TAB, int Q, int NT, int QEND, typename Hook>
__device__ __forceinline__ void group_mm(char* ring, int lane, f32x16 (&acc)[8], const Pieces& b,
                                         Hook& hook, Frag& f0) {
    Frag f[2];
    f[0] = f0;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        if (t + 1 < NT) rd_frag<Q, NT>(ring, lane, t + 1, f[(t + 1) & 1]);
        if (t == NT - 1) enter<TAB, Q + 1, QEND>(ring, lane, f0);
        __builtin_amdgcn_sched_barrier(0);
        acc[t] = mfma_x6(f[t & 1].p[0], f[t & 1].p[1], f[t & 1].p[2], b, acc[t]);
        hook(t);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// A layer segment of NG k-groups starting at global group Q0 (compile-time
// recursion: ring slots, DMA sources and wait counts are constants).
//   getb(IC<g>, float (&x)[8]): the 8 fp32 B values of local group g
//   side(IC<g>): output stores of the previous layer, spread over the groups
// b holds the pieces of group G (split one group ahead, inside group G-1);
// f0 carries the next group's tile-0 fragments across groups and segments.
template <class TAB, int Q0, int G, int NG, int NT, int QEND, typename GetB, typename Side>
__device__ __forceinline__ void segment_from(const char* __restrict__ packed, char* ring, int wave,
                                             int lane, f32x16 (&acc)[8], GetB& getb, Side& side,
                                             const Pieces& b, Frag& f0) {
    if constexpr (G < NG) {
        constexpr int Q = Q0 + G;
        Pieces bn = b;
        auto hook = [&](int t) {
            if (t == 0) stage<TAB, Q + kSlots - 1, QEND>(packed, ring, wave, lane);
            if (t == 1) {
                if constexpr (G + 1 < NG) {
                    float x[8];
                    getb(IC<G + 1>(), x);
                    bn = split8(x);
                    pin(bn);
                }
            }
            if (t == 2) side(IC<G>());
        };
        group_mm<TAB, Q, NT, QEND>(ring, lane, acc, b, hook, f0);
        segment_from<TAB, Q0, G + 1, NG, NT, QEND>(packed, ring, wave, lane, acc, getb, side, bn,
                                                   f0);
    }
}

template <class TAB, int Q0, int G, int NG, int NT, int QEND, typename GetB, typename Side>
__device__ __forceinline__ void segment(const char* __restrict__ packed, char* ring, int wave,
                                        int lane, f32x16 (&acc)[8], GetB& getb, Side& side,
                                        Frag& f0) {
    float x[8];
    getb(IC<0>(), x);
    const Pieces b = split8(x);
    segment_from<TAB, Q0, 0, NG, NT, QEND>(packed, ring, wave, lane, acc, getb, side, b, f0);
}

// B values of k-group g of a 256-wide accumulator input (packing.kmap3)
template <int g>
__device__ __forceinline__ void acc_group(const f32x16 (&X)[8], float (&x)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = X[g >> 1][8 * (g & 1) + j];
}

struct NoSide {
    template <typename T> __device__ __forceinline__ void operator()(T) const {}
};

}  // namespace x3
