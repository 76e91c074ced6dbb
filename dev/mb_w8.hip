// Microbenchmark (dev only): the f16x3 layer loop of mlp_fwd3 (16x16x32 f16
// tiles, LDS ring of 16 KiB weight k-groups filled by LDS-DMA, one barrier per
// group) at two occupancies:
//   W4: 4 waves per workgroup, one per SIMD, 32 samples (2 sample tiles) per wave
//       -- the shipped layout;
//   W8: 8 waves per workgroup, two per SIMD, 16 samples (1 sample tile) per wave
//       -- same 128 samples per workgroup, same weight reuse, half the registers
//       per wave, so a partner wave can issue while the other waits on a store,
//       the barrier or an LDS read.
// STORE 0: no saving stores; 1: every activation saved (1 KiB per dwordx4
// wave store, unique addresses) + ReLU mask bits, as in training.
// 8 layers of 256 -> 256 per sample; prints ms per launch and fp32-equivalent TF.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -fno-slp-vectorize dev/mb_w8.hip -o dev/mb_w8
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#ifndef MB_SLOTS
#define MB_SLOTS 4
#endif
constexpr int kSlots = MB_SLOTS, kSlotBytes = 16384, kGroups = 16;   // k-groups per layer

__device__ __forceinline__ float relu_i(float x) { return __int_as_float(max(__float_as_int(x), 0)); }

__device__ __forceinline__ void split_pair(float x0, float x1, f16x2& hi, f16x2& lo, float& u0, float& u1) {
    x0 = relu_i(x0) * (1.0f / 256.0f);
    x1 = relu_i(x1) * (1.0f / 256.0f);
    hi = __builtin_convertvector((f32x2){x0, x1}, f16x2);
    float r0, r1;
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r0) : "v"(hi), "v"(x0));
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r1) : "v"(hi), "v"(x1));
    lo = __builtin_convertvector((f32x2){r0, r1}, f16x2);
    u0 = x0; u1 = x1;
}

struct Pieces { f16x8 hi, lo; };
struct Frag { f16x8 hi, lo; };

__device__ __forceinline__ void put(Pieces& b, int p, f16x2 h, f16x2 l) {
    b.hi[2 * p] = h[0]; b.hi[2 * p + 1] = h[1];
    b.lo[2 * p] = l[0]; b.lo[2 * p + 1] = l[1];
}
__device__ __forceinline__ void pin(Pieces& p) { asm volatile("" : "+v"(p.hi), "+v"(p.lo)); }

struct Ring {
    __amdgpu_buffer_rsrc_t rsrc;
    char* lds;
    int wave, voff;
};

// DMA instruction k (0 .. 16/NW - 1) of this wave for layer-local group g
template <int NW>
__device__ __forceinline__ void dma(const Ring& r, int g, int k) {
    const int i = r.wave + NW * k;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        r.rsrc, (__attribute__((address_space(3))) void*)(r.lds + (g % kSlots) * kSlotBytes + i * 1024),
        16, r.voff, (g % kGroups) * kSlotBytes + i * 1024, 0, 0);
}

__device__ __forceinline__ void rd(const Ring& r, int lane, int slot, int t, Frag& f) {
    const char* s = r.lds + slot * kSlotBytes + lane * 16 + t * 1024;
    f.hi = *reinterpret_cast<const f16x8*>(s);
    f.lo = *reinterpret_cast<const f16x8*>(s + 8192);
}

template <int N>
__device__ __forceinline__ void enter() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ void store4(const f32x4& v, float* p) {
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
}

__device__ __forceinline__ void mask4(const f32x4& v, int sh, uint32_t& w) {
#pragma unroll
    for (int r = 0; r < 4; ++r) w |= min(__float_as_uint(v[r]), 1u) << (sh + r);
}

__device__ __forceinline__ f32x4 mf16(const f16x8& a, const f16x8& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

#ifndef MB_SGB
#define MB_SGB 1
#endif
#ifndef MB_DMA
#define MB_DMA 1
#endif

// ============ W4: 2 sample tiles per wave (mlp_fwd3 today) ===================
typedef f32x4 Act2[16][2];
__host__ __device__ constexpr int unit_at2(int t, int hf) { return t >= 3 && t <= 6 ? 4 * hf + t - 3 : -1; }

template <int STORE>
__device__ __forceinline__ void layer_w4(const Ring& rg, int lane, Act2& X, Act2& Y, Pieces (&b)[2],
                                         Frag& f0, float* __restrict__ sv, uint32_t* __restrict__ msk) {
    float pend[2] = {0.f, 0.f};
    uint32_t mw[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        Pieces bn[2];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            const int g = 2 * s + hf;
            Frag f[2];
            f[0] = f0;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                if (t + 1 < 8) rd(rg, lane, g % kSlots, t + 1, f[(t + 1) & 1]);
                if (t == 7) {
                    if constexpr (MB_DMA == 0) { if constexpr (STORE) enter<6>(); else enter<0>(); }
                    else if constexpr (STORE) enter<14>(); else enter<8>();
                    rd(rg, lane, (g + 1) % kSlots, 0, f0);
                }
                __builtin_amdgcn_sched_barrier(0);
                const Frag& w = f[t & 1];
#pragma unroll
                for (int S = 0; S < 2; ++S) {
                    f32x4 c = s == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : Y[8 * hf + t][S];
                    c = mf16(w.lo, b[S].hi, c);
                    c = mf16(w.hi, b[S].lo, c);
                    Y[8 * hf + t][S] = mf16(w.hi, b[S].hi, c);
                }
                asm volatile("" : "+a"(Y[8 * hf + t][0]), "+a"(Y[8 * hf + t][1]));
#if MB_DMA == 0        // no weight DMA after the prologue (the ring keeps stale weights): its price
#elif MB_DMA == 2      // spread over the odd tiles
                if (t & 1) dma<4>(rg, g + kSlots - 1, t >> 1);
#else
                if (t < 4) dma<4>(rg, g + kSlots - 1, t);
#endif
                const int u = unit_at2(t, hf);
                if (u >= 0) {
                    const int S = u >> 2, p = u & 3;
                    const int F = s < 7 ? 2 * (s + 1) + (p >> 1) : (p >> 1);
                    const f32x4& src = s < 7 ? X[F][S] : Y[F][S];
                    f16x2 h, l;
                    float u0, u1;
                    split_pair(src[2 * (p & 1)], src[2 * (p & 1) + 1], h, l, u0, u1);
                    put(bn[S], p, h, l);
                    pin(bn[S]);
                    if constexpr (STORE) {
                        if ((p & 1) == 0) { pend[0] = u0; pend[1] = u1; }
                        else {
                            const f32x4 v = {pend[0], pend[1], u0, u1};
                            store4(v, sv + ((F * 2 + S) * 64 + lane) * 4);
                            mask4(v, 8 * (F & 3) + 4 * S, mw[F >> 2]);
                        }
                    }
                }
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, MB_SGB, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        b[0] = bn[0];
        b[1] = bn[1];
    }
    if constexpr (STORE)
        *reinterpret_cast<uint4*>(msk + lane * 4) = make_uint4(mw[0], mw[1], mw[2], mw[3]);
}

// ============ W8: 1 sample tile per wave, two waves per SIMD ==================
typedef f32x4 Act1[16];
// the 4 split units of the next k-step at tiles 3 and 5 of both halves
__host__ __device__ constexpr int unit_at1(int t, int hf) { return t == 3 ? 2 * hf : (t == 5 ? 2 * hf + 1 : -1); }

template <int STORE>
__device__ __forceinline__ void layer_w8(const Ring& rg, int lane, Act1& X, Act1& Y, Pieces& b,
                                         Frag& f0, float* __restrict__ sv, uint32_t* __restrict__ msk) {
    float pend[2] = {0.f, 0.f};
    uint32_t mw[2] = {0u, 0u};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        Pieces bn;
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            const int g = 2 * s + hf;
            Frag f[2];
            f[0] = f0;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                if (t + 1 < 8) rd(rg, lane, g % kSlots, t + 1, f[(t + 1) & 1]);
                if (t == 7) {
                    // after DMA(g+1): 2 DMA for each of the kSlots-2 groups between + 1 store per group
                    if constexpr (STORE) enter<2 * (kSlots - 2) + (kSlots - 1)>(); else enter<2 * (kSlots - 2)>();
                    rd(rg, lane, (g + 1) % kSlots, 0, f0);
                }
                __builtin_amdgcn_sched_barrier(0);
                const Frag& w = f[t & 1];
                f32x4 c = s == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : Y[8 * hf + t];
                c = mf16(w.lo, b.hi, c);
                c = mf16(w.hi, b.lo, c);
                Y[8 * hf + t] = mf16(w.hi, b.hi, c);
                asm volatile("" : "+a"(Y[8 * hf + t]));
                if (t < 2) dma<8>(rg, g + kSlots - 1, t);
                const int p = unit_at1(t, hf);
                if (p >= 0) {
                    const int F = s < 7 ? 2 * (s + 1) + (p >> 1) : (p >> 1);
                    const f32x4& src = s < 7 ? X[F] : Y[F];
                    f16x2 h, l;
                    float u0, u1;
                    split_pair(src[2 * (p & 1)], src[2 * (p & 1) + 1], h, l, u0, u1);
                    put(bn, p, h, l);
                    pin(bn);
                    if constexpr (STORE) {
                        if ((p & 1) == 0) { pend[0] = u0; pend[1] = u1; }
                        else {
                            const f32x4 v = {pend[0], pend[1], u0, u1};
                            store4(v, sv + (F * 64 + lane) * 4);
                            mask4(v, 4 * (F & 7), mw[F >> 3]);
                        }
                    }
                }
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, MB_SGB, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        b = bn;
    }
    if constexpr (STORE)
        *reinterpret_cast<uint2*>(msk + lane * 2) = make_uint2(mw[0], mw[1]);
}

// ============ W4, 32 KiB groups: one k-step (16 tiles) per group, 3-slot ring ======
// the ring's slots are 2 x the 16 KiB slots above: slot index q % 3 of a 3 x 32 KiB ring
constexpr int kBigSlots = 3, kBigBytes = 32768;
__device__ __forceinline__ void dma_big(const Ring& r, int g, int k) {   // k = 0..7
    const int i = r.wave + 4 * k;                 // 1 KiB fragment i of 32
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        r.rsrc, (__attribute__((address_space(3))) void*)(r.lds + (g % kBigSlots) * kBigBytes + i * 1024),
        16, r.voff, (g % 8) * kBigBytes + i * 1024, 0, 0);
}
__device__ __forceinline__ void rd_big(const Ring& r, int lane, int slot, int t, Frag& f) {
    // tile t of 16: half t >> 3 is a 16 KiB [piece 2][tile 8] block
    const char* s = r.lds + slot * kBigBytes + (t >> 3) * 16384 + lane * 16 + (t & 7) * 1024;
    f.hi = *reinterpret_cast<const f16x8*>(s);
    f.lo = *reinterpret_cast<const f16x8*>(s + 8192);
}
__host__ __device__ constexpr int unit_big(int t) { return t >= 6 && t <= 13 ? t - 6 : -1; }

template <int STORE>
__device__ __forceinline__ void layer_w4b(const Ring& rg, int lane, Act2& X, Act2& Y, Pieces (&b)[2],
                                          Frag& f0, float* __restrict__ sv, uint32_t* __restrict__ msk) {
    float pend[2] = {0.f, 0.f};
    uint32_t mw[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        Pieces bn[2];
        const int g = s;
        Frag f[2];
        f[0] = f0;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            if (t + 1 < 16) rd_big(rg, lane, g % kBigSlots, t + 1, f[(t + 1) & 1]);
            if (t == 15) {
                // after DMA(g+1) (issued in group g-1): group g's 8 DMA + its stores before t 15
                if constexpr (STORE) enter<8 + 3>(); else enter<8>();
                rd_big(rg, lane, (g + 1) % kBigSlots, 0, f0);
            }
            __builtin_amdgcn_sched_barrier(0);
            const Frag& w = f[t & 1];
#pragma unroll
            for (int S = 0; S < 2; ++S) {
                f32x4 c = s == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : Y[t][S];
                c = mf16(w.lo, b[S].hi, c);
                c = mf16(w.hi, b[S].lo, c);
                Y[t][S] = mf16(w.hi, b[S].hi, c);
            }
            asm volatile("" : "+a"(Y[t][0]), "+a"(Y[t][1]));
            if (t < 8) dma_big(rg, g + kBigSlots - 1, t);
            const int u = unit_big(t);
            if (u >= 0) {
                const int S = u >> 2, p = u & 3;
                const int F = s < 7 ? 2 * (s + 1) + (p >> 1) : (p >> 1);
                const f32x4& src = s < 7 ? X[F][S] : Y[F][S];
                f16x2 h, l;
                float u0, u1;
                split_pair(src[2 * (p & 1)], src[2 * (p & 1) + 1], h, l, u0, u1);
                put(bn[S], p, h, l);
                pin(bn[S]);
                if constexpr (STORE) {
                    if ((p & 1) == 0) { pend[0] = u0; pend[1] = u1; }
                    else {
                        const f32x4 v = {pend[0], pend[1], u0, u1};
                        store4(v, sv + ((F * 2 + S) * 64 + lane) * 4);
                        mask4(v, 8 * (F & 3) + 4 * S, mw[F >> 2]);
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, MB_SGB, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        b[0] = bn[0];
        b[1] = bn[1];
    }
    if constexpr (STORE)
        *reinterpret_cast<uint4*>(msk + lane * 4) = make_uint4(mw[0], mw[1], mw[2], mw[3]);
}

// samples per workgroup: 128 in both layouts
template <int NW_, int STORE>
__global__ void __launch_bounds__(64 * (NW_ == 5 ? 4 : NW_), 1) mb_kernel(const char* __restrict__ w, int pairs,
                                                        float* __restrict__ save, float* __restrict__ out,
                                                        uint64_t* __restrict__ stamps) {
    constexpr int NW = NW_ == 5 ? 4 : NW_;
    constexpr bool BIG = NW_ == 5;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    __shared__ __attribute__((aligned(16))) char lds[BIG ? kBigSlots * kBigBytes : kSlots * kSlotBytes];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wv = blockIdx.x * NW + wave;          // wave index in the grid
    Ring rg;
    rg.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)w, 0, kGroups * kSlotBytes, 0x00020000);
    rg.lds = lds;
    rg.wave = wave;
    rg.voff = lane * 16;
    if constexpr (BIG) {
#pragma unroll
        for (int g = 0; g < kBigSlots - 1; ++g)
#pragma unroll
            for (int k = 0; k < 8; ++k) dma_big(rg, g, k);
    } else {
#pragma unroll
        for (int g = 0; g < kSlots - 1; ++g)
#pragma unroll
            for (int k = 0; k < 16 / NW; ++k) dma<NW>(rg, g, k);
    }
    const float seed = (float)(wv * 64 + lane) * 1e-4f;
    Frag f0;
    float acc_sum = 0.f;
    // saved floats per wave per layer: 32 samples x 256 (W4), 16 x 256 (W8)
    constexpr int kLayerFloats = NW == 4 ? 8192 : 4096;
    constexpr int kMaskWords = NW == 4 ? 256 : 128;
    const size_t nwaves = (size_t)gridDim.x * NW;
    if constexpr (NW == 4) {
        Act2 X, Y;
        Pieces b[2];
#pragma unroll
        for (int F = 0; F < 16; ++F)
#pragma unroll
            for (int S = 0; S < 2; ++S)
#pragma unroll
                for (int r = 0; r < 4; ++r) X[F][S][r] = 256.f * __sinf(seed + F * 0.37f + S * 0.11f + r * 0.05f);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            f16x2 h, l;
            float u0, u1;
            const int S = u >> 2, p = u & 3;
            split_pair(X[p >> 1][S][2 * (p & 1)], X[p >> 1][S][2 * (p & 1) + 1], h, l, u0, u1);
            put(b[S], p, h, l);
        }
        enter<0>();
        if constexpr (BIG) rd_big(rg, lane, 0, 0, f0);
        else rd(rg, lane, 0, 0, f0);
        for (int it = 0; it < pairs; ++it) {
            float* sv = save + ((size_t)(wv * pairs + it) * 2) * kLayerFloats;
            uint32_t* mk = reinterpret_cast<uint32_t*>(save) + nwaves * pairs * 2 * kLayerFloats +
                           ((size_t)(wv * pairs + it) * 2) * kMaskWords;
            if constexpr (BIG) {
                layer_w4b<STORE>(rg, lane, X, Y, b, f0, sv, mk);
                layer_w4b<STORE>(rg, lane, Y, X, b, f0, sv + kLayerFloats, mk + kMaskWords);
            } else {
                layer_w4<STORE>(rg, lane, X, Y, b, f0, sv, mk);
                layer_w4<STORE>(rg, lane, Y, X, b, f0, sv + kLayerFloats, mk + kMaskWords);
            }
        }
#pragma unroll
        for (int F = 0; F < 16; ++F) acc_sum += X[F][0][0] + X[F][1][3];
    } else {
        Act1 X, Y;
        Pieces b;
#pragma unroll
        for (int F = 0; F < 16; ++F)
#pragma unroll
            for (int r = 0; r < 4; ++r) X[F][r] = 256.f * __sinf(seed + F * 0.37f + r * 0.05f);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            f16x2 h, l;
            float u0, u1;
            split_pair(X[p >> 1][2 * (p & 1)], X[p >> 1][2 * (p & 1) + 1], h, l, u0, u1);
            put(b, p, h, l);
        }
        enter<0>();
        rd(rg, lane, 0, 0, f0);
        for (int it = 0; it < pairs; ++it) {
            float* sv = save + ((size_t)(wv * pairs + it) * 2) * kLayerFloats;
            uint32_t* mk = reinterpret_cast<uint32_t*>(save) + nwaves * pairs * 2 * kLayerFloats +
                           ((size_t)(wv * pairs + it) * 2) * kMaskWords;
            layer_w8<STORE>(rg, lane, X, Y, b, f0, sv, mk);
            layer_w8<STORE>(rg, lane, Y, X, b, f0, sv + kLayerFloats, mk + kMaskWords);
        }
#pragma unroll
        for (int F = 0; F < 16; ++F) acc_sum += X[F][0] + X[F][3];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    out[wv * 64 + lane] = acc_sum;
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int NW_, int STORE>
void bench(const char* w, int blocks, int pairs, float* save, float* out, uint64_t* stamps, int reps) {
    constexpr int NW = NW_ == 5 ? 4 : NW_;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) mb_kernel<NW_, STORE><<<blocks, 64 * NW>>>(w, pairs, save, out, stamps);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) mb_kernel<NW_, STORE><<<blocks, 64 * NW>>>(w, pairs, save, out, stamps);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    const double samples = (double)blocks * 128, flop = samples * pairs * 2 * 2.0 * 256 * 256;
    uint64_t* hs = (uint64_t*)malloc(blocks * 16);
    CK(hipMemcpy(hs, stamps, blocks * 16, hipMemcpyDeviceToHost));
    double cyc = 0, rt = 0;
    for (int i = 0; i < blocks; ++i) { cyc += hs[2 * i]; rt += hs[2 * i + 1]; }
    free(hs);
    printf("waves %d%s store %d slots %d sgb %d: %.3f ms  %.1f TF fp32-equiv (%.1f%% of 839)  clock %.2f GHz  WG %.0f cyc\n",
           NW, NW_ == 5 ? " (32 KiB groups)" : "", STORE, NW_ == 5 ? kBigSlots : kSlots, MB_SGB, ms, flop / ms / 1e9, flop / ms / 1e9 / 8.389, cyc / rt * 0.1, cyc / blocks);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
    const int blocks = 6144, pairs = 4, reps = argc > 1 ? atoi(argv[1]) : 20;
    char* w;
    float *save, *out;
    uint64_t* stamps;
    CK(hipMalloc(&w, kGroups * kSlotBytes));   // 16 x 16 KiB = 8 x 32 KiB
    uint16_t* hw = (uint16_t*)malloc(kGroups * kSlotBytes);
    srand(1);
    for (int i = 0; i < kGroups * kSlotBytes / 2; ++i) {
        _Float16 v = (_Float16)(((rand() & 0xffff) / 65536.0f - 0.5f) * 0.1f);
        hw[i] = __builtin_bit_cast(uint16_t, v);
    }
    CK(hipMemcpy(w, hw, kGroups * kSlotBytes, hipMemcpyHostToDevice));
    const size_t sv_floats = (size_t)blocks * 128 * pairs * 2 * (256 + 8);
    CK(hipMalloc(&save, sv_floats * 4));
    CK(hipMalloc(&out, (size_t)blocks * 512 * 4));
    CK(hipMalloc(&stamps, (size_t)blocks * 16));
    for (int r = 0; r < 2; ++r) {
        bench<4, 0>(w, blocks, pairs, save, out, stamps, reps);
        bench<5, 0>(w, blocks, pairs, save, out, stamps, reps);
        bench<8, 0>(w, blocks, pairs, save, out, stamps, reps);
        bench<4, 1>(w, blocks, pairs, save, out, stamps, reps);
        bench<5, 1>(w, blocks, pairs, save, out, stamps, reps);
        bench<8, 1>(w, blocks, pairs, save, out, stamps, reps);
    }
    return 0;
}
