// Microbenchmark (dev only): the f16x3 layer loop of mlp_fwd3 on
// v_mfma_f32_16x16x32_f16 tiles (2 sample tiles of 16 per wave) against the
// same loop on v_mfma_f32_32x32x16_f16 tiles (one 32-sample tile per wave).
// Same LDS ring (4 x 16 KiB k-groups filled by LDS-DMA, one barrier per group),
// same MFMA work per FLOP, same split of the next k-step's B operand (ReLU,
// 2^-8 unscale, hi/lo fp16 split) and optionally the saving stores + ReLU mask
// bits.  8 layers of 256 -> 256 per sample.  Prints ms per launch and the
// fp32-equivalent TFLOP/s.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -fno-slp-vectorize [-DMB_MIX=1] [-DMB_SGB=n]
//         dev/mb_shape.hip -o dev/mb_shape
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kSlots = 4, kSlotBytes = 16384, kGroups = 16;   // k-groups per layer

__device__ __forceinline__ float relu_i(float x) { return __int_as_float(max(__float_as_int(x), 0)); }

#ifndef MB_MIX
#define MB_MIX 0
#endif
#ifndef MB_SGB16
#define MB_SGB16 1
#endif
#ifndef MB_SGB32
#define MB_SGB32 3
#endif

// relu'd, unscaled pair -> hi = RN16(x), lo = RN16(x - hi).  MB_MIX 1 fuses the
// 2^-8 unscale into v_fma_mix{lo,hi}_f16 (hi straight from the scaled value,
// lo = RN16(x 2^-8 - hi)); the unscaled f32 values are then not formed.
__device__ __forceinline__ void split_pair(float x0, float x1, f16x2& hi, f16x2& lo, float& u0, float& u1) {
    x0 = relu_i(x0);
    x1 = relu_i(x1);
#if MB_MIX
    const float s = 1.0f / 256.0f;
    uint32_t h = 0, l = 0;
    asm("v_fma_mixlo_f16 %0, %1, %2, 0" : "+v"(h) : "v"(x0), "s"(s));
    asm("v_fma_mixhi_f16 %0, %1, %2, 0" : "+v"(h) : "v"(x1), "s"(s));
    asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel_hi:[0,0,1]" : "+v"(l) : "v"(x0), "s"(s), "v"(h));
    asm("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(l) : "v"(x1), "s"(s), "v"(h));
    hi = __builtin_bit_cast(f16x2, h);
    lo = __builtin_bit_cast(f16x2, l);
    u0 = x0; u1 = x1;        // stored scaled
#else
    x0 *= 1.0f / 256.0f;
    x1 *= 1.0f / 256.0f;
    hi = __builtin_convertvector((f32x2){x0, x1}, f16x2);
    float r0, r1;
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r0) : "v"(hi), "v"(x0));
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r1) : "v"(hi), "v"(x1));
    lo = __builtin_convertvector((f32x2){r0, r1}, f16x2);
    u0 = x0; u1 = x1;
#endif
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

// DMA instruction k (0..3) of this wave for layer-local group g
__device__ __forceinline__ void dma(const Ring& r, int g, int k) {
    const int i = r.wave + 4 * k;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        r.rsrc, (__attribute__((address_space(3))) void*)(r.lds + (g % kSlots) * kSlotBytes + i * 1024),
        16, r.voff, (g % kGroups) * kSlotBytes + i * 1024, 0, 0);
}

__device__ __forceinline__ void rd(const Ring& r, int lane, int slot, int t, Frag& f) {
    const char* s = r.lds + slot * kSlotBytes + lane * 16 + t * 1024;
    f.hi = *reinterpret_cast<const f16x8*>(s);
    f.lo = *reinterpret_cast<const f16x8*>(s + 8192);
}

template <int STORE>
__device__ __forceinline__ void enter() {
    // group g's DMA was issued kSlots-1 groups ago; the 2 groups after it (8 DMA)
    // and the 2 stores of each of the 3 groups since may be in flight
    if constexpr (STORE == 4) asm volatile("s_waitcnt vmcnt(11) lgkmcnt(0)" ::: "memory");
    else if constexpr (STORE) asm volatile("s_waitcnt vmcnt(14) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

#ifndef MB_NT
#define MB_NT 1
#endif
__device__ __forceinline__ void store4(const f32x4& v, float* p) {
#if MB_NT
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
#else
    *reinterpret_cast<f32x4*>(p) = v;
#endif
}

__device__ __forceinline__ void mask4(const f32x4& v, int sh, uint32_t& w) {
#pragma unroll
    for (int r = 0; r < 4; ++r) w |= min(__float_as_uint(v[r]), 1u) << (sh + r);
}

// unit u of a k-step (of 8): sample tile / sub-step u >> 2, pair p = u & 3; run at
// tile t of half hf (tiles 3..6 of both halves)
__host__ __device__ constexpr int unit_at(int t, int hf) { return t >= 3 && t <= 6 ? 4 * hf + t - 3 : -1; }

// ============================ 16x16x32 ======================================
__device__ __forceinline__ f32x4 mf16(const f16x8& a, const f16x8& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
typedef f32x4 Act16[16][2];

template <int STORE>
__device__ __forceinline__ void layer16(const Ring& rg, int lane, Act16& X, Act16& Y, Pieces (&b)[2],
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
                if (t == 7) { enter<STORE>(); rd(rg, lane, (g + 1) % kSlots, 0, f0); }
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
                if (t < 4) dma(rg, g + 3, t);
                const int u = unit_at(t, hf);
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
                            if (STORE == 3) store4(v, sv + lane * 4);
                            else if (STORE != 4 || (u & 2)) store4(v, sv + ((F * 2 + S) * 64 + lane) * 4);
                            mask4(v, 8 * (F & 3) + 4 * S, mw[F >> 2]);
                        }
                    }
                }
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, MB_SGB16, 0);
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

// ============================ 32x32x16 ======================================
__device__ __forceinline__ f32x16 mf32(const f16x8& a, const f16x8& b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
typedef f32x16 Act32[8];

// group (s, hf): k-step s = 32 inputs = sub-steps u = 0, 1 of 16 (X tile s, regs
// 8u .. 8u+7); output tiles 4hf .. 4hf+3; iteration i = 2 t + u reads fragment i
template <int STORE>
__device__ __forceinline__ void layer32(const Ring& rg, int lane, Act32& X, Act32& Y, Pieces (&b)[2],
                                        Frag& f0, float* __restrict__ sv, uint32_t* __restrict__ msk) {
    float pend[2] = {0.f, 0.f};
    uint32_t mw[2] = {0u, 0u};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        Pieces bn[2];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            const int g = 2 * s + hf;
            Frag f[2];
            f[0] = f0;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int t = i >> 1, u = i & 1;
                if (i + 1 < 8) rd(rg, lane, g % kSlots, i + 1, f[(i + 1) & 1]);
                if (i == 7) { enter<STORE>(); rd(rg, lane, (g + 1) % kSlots, 0, f0); }
                __builtin_amdgcn_sched_barrier(0);
                const Frag& w = f[i & 1];
                f32x16 c = (s == 0 && u == 0) ? f32x16{} : Y[4 * hf + t];
                c = mf32(w.lo, b[u].hi, c);
                c = mf32(w.hi, b[u].lo, c);
                Y[4 * hf + t] = mf32(w.hi, b[u].hi, c);
                asm volatile("" : "+a"(Y[4 * hf + t]));
                if (i < 4) dma(rg, g + 3, i);
                const int un = unit_at(i, hf);
                if (un >= 0) {
                    const int uu = un >> 2, p = un & 3;
                    const f32x16& src = s < 7 ? X[s + 1] : Y[0];
                    f16x2 h, l;
                    float u0, u1;
                    split_pair(src[8 * uu + 2 * p], src[8 * uu + 2 * p + 1], h, l, u0, u1);
                    put(bn[uu], p, h, l);
                    pin(bn[uu]);
                    if constexpr (STORE) {
                        if ((p & 1) == 0) { pend[0] = u0; pend[1] = u1; }
                        else {
                            const int T = s < 7 ? s + 1 : 0, q = 2 * uu + (p >> 1);
                            const f32x4 v = {pend[0], pend[1], u0, u1};
                            if (STORE == 3) store4(v, sv + lane * 4);
                            else if (STORE != 4 || (un & 2)) store4(v, sv + ((T * 4 + q) * 64 + lane) * 4);
                            mask4(v, 16 * (T & 1) + 4 * q, mw[T >> 1 & 1]);
                        }
                    }
                }
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, MB_SGB32, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        b[0] = bn[0];
        b[1] = bn[1];
    }
    if constexpr (STORE)
        *reinterpret_cast<uint2*>(msk + lane * 2) = make_uint2(mw[0], mw[1]);
}

template <int SHAPE, int STORE>
__global__ void __launch_bounds__(256, 1) mb_kernel(const char* __restrict__ w, int pairs,
                                                    float* __restrict__ save, float* __restrict__ out,
                                                    uint64_t* __restrict__ stamps) {
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    __shared__ __attribute__((aligned(16))) char lds[kSlots * kSlotBytes];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int blk = blockIdx.x * 4 + wave;
    Ring rg;
    rg.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)w, 0, kGroups * kSlotBytes, 0x00020000);
    rg.lds = lds;
    rg.wave = wave;
    rg.voff = lane * 16;
#pragma unroll
    for (int g = 0; g < kSlots - 1; ++g)
#pragma unroll
        for (int k = 0; k < 4; ++k) dma(rg, g, k);
    const float seed = (float)(blk * 64 + lane) * 1e-4f;
    Frag f0;
    Pieces b[2];
    float acc_sum = 0.f;
    if constexpr (SHAPE == 16) {
        Act16 X, Y;
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
        enter<false>();
        rd(rg, lane, 0, 0, f0);
        for (int it = 0; it < pairs; ++it) {
            float* sv = save + (STORE == 3 ? (size_t)blk * 256 : ((size_t)(blk * pairs + it) * 2) * 8192);
            uint32_t* mk = reinterpret_cast<uint32_t*>(save) + (size_t)gridDim.x * 4 * pairs * 2 * 8192 +
                           ((size_t)(blk * pairs + it) * 2) * 256;
            layer16<STORE>(rg, lane, X, Y, b, f0, sv, mk);
            layer16<STORE>(rg, lane, Y, X, b, f0, sv + 8192, mk + 256);
        }
#pragma unroll
        for (int F = 0; F < 16; ++F) acc_sum += X[F][0][0] + X[F][1][3];
    } else {
        Act32 X, Y;
#pragma unroll
        for (int T = 0; T < 8; ++T)
#pragma unroll
            for (int r = 0; r < 16; ++r) X[T][r] = 256.f * __sinf(seed + T * 0.37f + r * 0.05f);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            f16x2 h, l;
            float u0, u1;
            const int uu = u >> 2, p = u & 3;
            split_pair(X[0][8 * uu + 2 * p], X[0][8 * uu + 2 * p + 1], h, l, u0, u1);
            put(b[uu], p, h, l);
        }
        enter<false>();
        rd(rg, lane, 0, 0, f0);
        for (int it = 0; it < pairs; ++it) {
            float* sv = save + (STORE == 3 ? (size_t)blk * 256 : ((size_t)(blk * pairs + it) * 2) * 8192);
            uint32_t* mk = reinterpret_cast<uint32_t*>(save) + (size_t)gridDim.x * 4 * pairs * 2 * 8192 +
                           ((size_t)(blk * pairs + it) * 2) * 256;
            layer32<STORE>(rg, lane, X, Y, b, f0, sv, mk);
            layer32<STORE>(rg, lane, Y, X, b, f0, sv + 8192, mk + 256);
        }
#pragma unroll
        for (int T = 0; T < 8; ++T) acc_sum += X[T][0] + X[T][15];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    out[blk * 64 + lane] = acc_sum;
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int SHAPE, int STORE>
void bench(const char* w, int blocks, int pairs, float* save, float* out, int reps) {
    static uint64_t* stamps = nullptr;
    if (!stamps) CK(hipMalloc(&stamps, blocks * 16));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) mb_kernel<SHAPE, STORE><<<blocks, 256>>>(w, pairs, save, out, stamps);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) mb_kernel<SHAPE, STORE><<<blocks, 256>>>(w, pairs, save, out, stamps);
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
    printf("shape %dx%d store %d mix %d sgb %d/%d: %.3f ms  %.1f TF fp32-equiv (%.1f%% of 839)  clock %.2f GHz  WG %.0f cyc\n",
           SHAPE, SHAPE, (int)STORE, MB_MIX, MB_SGB16, MB_SGB32, ms, flop / ms / 1e9, flop / ms / 1e9 / 8.389,
           cyc / rt * 0.1, cyc / blocks);
}

int main(int argc, char** argv) {
    const int blocks = 6144, pairs = 4, reps = argc > 1 ? atoi(argv[1]) : 20;
    char* w;
    float *save, *out;
    CK(hipMalloc(&w, kGroups * kSlotBytes));
    uint16_t* hw = (uint16_t*)malloc(kGroups * kSlotBytes);
    srand(1);
    for (int i = 0; i < kGroups * kSlotBytes / 2; ++i) {
        _Float16 v = (_Float16)(((rand() & 0xffff) / 65536.0f - 0.5f) * 0.1f);
        hw[i] = __builtin_bit_cast(uint16_t, v);
    }
    CK(hipMemcpy(w, hw, kGroups * kSlotBytes, hipMemcpyHostToDevice));
    const size_t sv_floats = (size_t)blocks * 4 * pairs * 2 * (8192 + 256);
    CK(hipMalloc(&save, sv_floats * 4));
    CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
    for (int r = 0; r < 2; ++r) {
        bench<16, 0>(w, blocks, pairs, save, out, reps);
        bench<32, 0>(w, blocks, pairs, save, out, reps);
        bench<16, 1>(w, blocks, pairs, save, out, reps);
        bench<32, 1>(w, blocks, pairs, save, out, reps);
        bench<16, 3>(w, blocks, pairs, save, out, reps);
        bench<32, 3>(w, blocks, pairs, save, out, reps);
        bench<16, 4>(w, blocks, pairs, save, out, reps);
        bench<32, 4>(w, blocks, pairs, save, out, reps);
    }
    return 0;
}
