// Microbenchmark (dev only): the f16x3 layer loop of mlp_fwd3 (16x16x32 f16
// tiles, LDS ring of 16 KiB weight k-groups filled by LDS-DMA, one barrier per
// group, 4 waves per workgroup, one per SIMD) with NS 16-sample tiles per wave:
// NS = 2 is the shipped layout (32 samples per wave, 128 per workgroup); NS =
// 3 holds 48 samples per wave, so every weight fragment a wave reads from LDS
// feeds 9 instead of 6 MFMAs -- a CU's LDS read traffic per FLOP drops by a
// third ("What the layers' remaining ~25% is").
// STORE 0: no saving stores; 1: every activation saved (1 KiB per dwordx4
// wave store) + ReLU mask bits, as in training.  8 layers of 256 -> 256.
// MB_NP=1: the plain-bf16 loop instead (one bf16 piece, one MFMA per product,
// 8 KiB groups: LDS demand 2x f16x3's per MFMA cycle).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -fno-slp-vectorize dev/mb_s3.hip -o dev/mb_s3
//   hipcc ... -DMB_NP=1 dev/mb_s3.hip -o dev/mb_s3_b1
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#ifndef MB_NP
#define MB_NP 2
#endif
constexpr int kNP = MB_NP;
constexpr int kSlots = 4, kSlotBytes = kNP * 8192, kGroups = 16;   // k-groups per layer
constexpr int kDmaPerWave = kNP * 2;                               // 1 KiB DMAs per wave per group

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

__device__ __forceinline__ void dma(const Ring& r, int g, int k) {
    const int i = r.wave + 4 * k;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        r.rsrc, (__attribute__((address_space(3))) void*)(r.lds + (g % kSlots) * kSlotBytes + i * 1024),
        16, r.voff, (g % kGroups) * kSlotBytes + i * 1024, 0, 0);
}

__device__ __forceinline__ void rd(const Ring& r, int lane, int slot, int t, Frag& f) {
    const char* s = r.lds + slot * kSlotBytes + lane * 16 + t * 1024;
    f.hi = *reinterpret_cast<const f16x8*>(s);
    if constexpr (kNP == 2) f.lo = *reinterpret_cast<const f16x8*>(s + 8192);
}

template <int N>
__device__ __forceinline__ void enter() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ f32x4 mf16(const f16x8& a, const f16x8& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x4 mbf16(const f16x8& a, const f16x8& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                   c, 0, 0, 0);
}

// split unit u (= 4 S + p) of the next k-step at tile t of half hf: NS = 2 the
// shipped slots (tiles 3..6 of both halves), NS = 3 tiles 2..7 of both (the
// last k-step's units read output tiles 0, 1, final after tile 1 of half 0)
template <int NS>
__host__ __device__ constexpr int unit_at(int t, int hf) {
    if constexpr (NS == 2) return t >= 3 && t <= 6 ? 4 * hf + t - 3 : -1;
    else return t >= 2 ? 6 * hf + t - 2 : -1;
}
// stores this wave issued after DMA(g + 1) by the hand-over into g + 1 (one per
// odd unit): the kSlots - 2 groups before g in full, g's before tile 7
template <int NS>
__host__ __device__ constexpr int extra_stores() {
    int before7 = 0, all = 0;
    for (int t = 0; t < 8; ++t) {
        const int u = unit_at<NS>(t, 0);
        if (u >= 0 && (u & 1)) { ++all; if (t < 7) ++before7; }
    }
    return before7 + (kSlots - 2) * all;   // (kDmaPerWave DMAs per group counted by the caller)
}

template <int NS>
using Act = f32x4[16][NS];

template <int NS, int STORE>
__device__ __forceinline__ void layer(const Ring& rg, int lane, Act<NS>& X, Act<NS>& Y, Pieces (&b)[NS],
                                      Frag& f0, float* __restrict__ sv, uint32_t* __restrict__ msk) {
    float pend[2] = {0.f, 0.f};
    uint32_t mw[2 * NS] = {};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        Pieces bn[NS];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            const int g = 2 * s + hf;
            Frag f[2];
            f[0] = f0;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                if (t + 1 < 8) rd(rg, lane, g % kSlots, t + 1, f[(t + 1) & 1]);
                if (t == 7) {
                    if constexpr (STORE) enter<kDmaPerWave * (kSlots - 2) + extra_stores<NS>()>();
                    else enter<kDmaPerWave * (kSlots - 2)>();
                    rd(rg, lane, (g + 1) % kSlots, 0, f0);
                }
                __builtin_amdgcn_sched_barrier(0);
                const Frag& w = f[t & 1];
#pragma unroll
                for (int S = 0; S < NS; ++S) {
                    f32x4 c = s == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : Y[8 * hf + t][S];
                    if constexpr (kNP == 2) {
                        c = mf16(w.lo, b[S].hi, c);
                        c = mf16(w.hi, b[S].lo, c);
                        Y[8 * hf + t][S] = mf16(w.hi, b[S].hi, c);
                    } else {
                        Y[8 * hf + t][S] = mbf16(w.hi, b[S].hi, c);
                    }
                }
                if (t < kDmaPerWave) dma(rg, g + kSlots - 1, t);
                const int u = unit_at<NS>(t, hf);
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
                            __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(sv + ((F * NS + S) * 64 + lane) * 4));
                            const int bit = (F * NS + S) * 4;
#pragma unroll
                            for (int r = 0; r < 4; ++r) mw[(bit + r) >> 5] |= min(__float_as_uint(v[r]), 1u) << ((bit + r) & 31);
                        }
                    }
                }
#pragma unroll
                for (int i = 0; i < (kNP == 2 ? 3 : 1) * NS; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int S = 0; S < NS; ++S) b[S] = bn[S];
    }
    if constexpr (STORE) {
#pragma unroll
        for (int i = 0; i < 2 * NS; ++i) msk[i * 64 + lane] = mw[i];
    }
}

template <int NS, int STORE>
__global__ void __launch_bounds__(256, 1) mb_kernel(const char* __restrict__ w, int pairs,
                                                    float* __restrict__ save, float* __restrict__ out,
                                                    uint64_t* __restrict__ stamps) {
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    __shared__ __attribute__((aligned(16))) char lds[kSlots * kSlotBytes];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wv = blockIdx.x * 4 + wave;
    Ring rg;
    rg.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)w, 0, kGroups * kSlotBytes, 0x00020000);
    rg.lds = lds;
    rg.wave = wave;
    rg.voff = lane * 16;
#pragma unroll
    for (int g = 0; g < kSlots - 1; ++g)
#pragma unroll
        for (int k = 0; k < kDmaPerWave; ++k) dma(rg, g, k);
    const float seed = (float)(wv * 64 + lane) * 1e-4f;
    Frag f0;
    constexpr int kLayerFloats = NS * 4096;
    constexpr int kMaskWords = 2 * NS * 64;
    const size_t nwaves = (size_t)gridDim.x * 4;
    Act<NS> X, Y;
    Pieces b[NS];
#pragma unroll
    for (int F = 0; F < 16; ++F)
#pragma unroll
        for (int S = 0; S < NS; ++S)
#pragma unroll
            for (int r = 0; r < 4; ++r) X[F][S][r] = 256.f * __sinf(seed + F * 0.37f + S * 0.11f + r * 0.05f);
#pragma unroll
    for (int u = 0; u < 4 * NS; ++u) {
        f16x2 h, l;
        float u0, u1;
        const int S = u >> 2, p = u & 3;
        split_pair(X[p >> 1][S][2 * (p & 1)], X[p >> 1][S][2 * (p & 1) + 1], h, l, u0, u1);
        put(b[S], p, h, l);
    }
    enter<0>();
    rd(rg, lane, 0, 0, f0);
    for (int it = 0; it < pairs; ++it) {
        float* sv = save + ((size_t)(wv * pairs + it) * 2) * kLayerFloats;
        uint32_t* mk = reinterpret_cast<uint32_t*>(save) + nwaves * pairs * 2 * kLayerFloats +
                       ((size_t)(wv * pairs + it) * 2) * kMaskWords;
        layer<NS, STORE>(rg, lane, X, Y, b, f0, sv, mk);
        layer<NS, STORE>(rg, lane, Y, X, b, f0, sv + kLayerFloats, mk + kMaskWords);
    }
    float acc_sum = 0.f;
#pragma unroll
    for (int F = 0; F < 16; ++F) acc_sum += X[F][0][0] + X[F][NS - 1][3];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    out[wv * 64 + lane] = acc_sum;
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int NS, int STORE>
void bench(const char* w, int pairs, float* save, float* out, uint64_t* stamps, int reps) {
    const int blocks = 786432 / (64 * NS);    // the cfg2 fine pass: 786,432 samples
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) mb_kernel<NS, STORE><<<blocks, 256>>>(w, pairs, save, out, stamps);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) mb_kernel<NS, STORE><<<blocks, 256>>>(w, pairs, save, out, stamps);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    const double samples = (double)blocks * 64 * NS, flop = samples * pairs * 2 * 2.0 * 256 * 256;
    const double peak = kNP == 2 ? 8.389 : 25.166;   // fp32-equivalent ceiling (f16x3: 2517/3) / bf16 peak, x100 GF
    uint64_t* hs = (uint64_t*)malloc(blocks * 16);
    CK(hipMemcpy(hs, stamps, blocks * 16, hipMemcpyDeviceToHost));
    double cyc = 0, rt = 0;
    for (int i = 0; i < blocks; ++i) { cyc += hs[2 * i]; rt += hs[2 * i + 1]; }
    free(hs);
    printf("np %d samples/wave %d store %d: %.3f ms  %.1f TF (%.1f%% of ceiling)  clock %.2f GHz  "
           "WG %.0f cyc (%.0f per 128 samples)\n",
           kNP, 16 * NS, STORE, ms, flop / ms / 1e9, flop / ms / 1e9 / peak, cyc / rt * 0.1, cyc / blocks,
           cyc / blocks * 128.0 / (64 * NS));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
    const int pairs = 4, reps = argc > 1 ? atoi(argv[1]) : 20;
    char* w;
    float *save, *out;
    uint64_t* stamps;
    CK(hipMalloc(&w, kGroups * kSlotBytes));
    uint16_t* hw = (uint16_t*)malloc(kGroups * kSlotBytes);
    srand(1);
    for (int i = 0; i < kGroups * kSlotBytes / 2; ++i) {
        _Float16 v = (_Float16)(((rand() & 0xffff) / 65536.0f - 0.5f) * 0.1f);
        hw[i] = __builtin_bit_cast(uint16_t, v);
    }
    CK(hipMemcpy(w, hw, kGroups * kSlotBytes, hipMemcpyHostToDevice));
    const size_t sv_floats = (size_t)786432 * pairs * 2 * (256 + 8);
    CK(hipMalloc(&save, sv_floats * 4));
    CK(hipMalloc(&out, (size_t)786432 / 16 * 64 * 4));   // one float per lane of every wave (NS >= 1)
    CK(hipMalloc(&stamps, (size_t)786432 / 128 * 16));
    for (int r = 0; r < 2; ++r) {
        bench<2, 0>(w, pairs, save, out, stamps, reps);
        bench<3, 0>(w, pairs, save, out, stamps, reps);
        bench<2, 1>(w, pairs, save, out, stamps, reps);
        bench<3, 1>(w, pairs, save, out, stamps, reps);
    }
    return 0;
}
