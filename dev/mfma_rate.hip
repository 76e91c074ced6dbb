// dev microbenchmark: sustained rate of the bf16x6 MFMA pattern
// (8 accumulators x 6 dependent v_mfma_f32_32x32x16_bf16, operands in registers)
#include "../nerf_pl_amd/csrc/x3.h"
using namespace x3;
extern "C" __global__ void __launch_bounds__(256, 1) rate_kernel(float* out, int iters, int variant) {
    const int lane = threadIdx.x & 63;
    f32x16 acc[8];
    for (int t = 0; t < 8; ++t) acc[t] = f32x16{};
    bf16x8 a[3];
    Pieces b;
    for (int j = 0; j < 8; ++j) {
        auto rnd = [&](int k) {   // hashed pseudo-random operand in [-1, 1)
            uint32_t x = (uint32_t)(lane * 8 + j) * 2654435761u + (uint32_t)k * 40503u + blockIdx.x;
            x ^= x >> 15; x *= 2246822519u; x ^= x >> 13;
            return (float)(x & 0xffffff) / 8388608.f - 1.f;
        };
        a[0][j] = (__bf16)rnd(0); a[1][j] = (__bf16)(rnd(1) * 0.004f); a[2][j] = (__bf16)(rnd(2) * 1.5e-5f);
        b.hi[j] = (__bf16)rnd(3); b.mid[j] = (__bf16)(rnd(4) * 0.004f); b.lo[j] = (__bf16)(rnd(5) * 1.5e-5f);
    }
    for (int it = 0; it < iters; ++it) {
        if (variant == 0) {
#pragma unroll
            for (int t = 0; t < 8; ++t) acc[t] = mfma_x6(a[0], a[1], a[2], b, acc[t]);
        } else {
            // interleaved: product k over all tiles, then k+1
#pragma unroll
            for (int t = 0; t < 8; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b.hi, acc[t], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < 8; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b.lo, acc[t], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < 8; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b.mid, acc[t], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < 8; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b.hi, acc[t], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < 8; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b.mid, acc[t], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < 8; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b.hi, acc[t], 0, 0, 0);
        }
    }
    float s = 0.f;
    for (int t = 0; t < 8; ++t) for (int r = 0; r < 16; ++r) s += acc[t][r];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
typedef float f32x4v __attribute__((ext_vector_type(4)));
extern "C" __global__ void __launch_bounds__(256, 1) rate16_kernel(float* out, int iters) {
    const int lane = threadIdx.x & 63;
    f32x4v acc[32];
    for (int t = 0; t < 32; ++t) acc[t] = f32x4v{};
    bf16x8 a[3];
    Pieces b;
    for (int j = 0; j < 8; ++j) {
        auto rnd = [&](int k) {   // hashed pseudo-random operand in [-1, 1)
            uint32_t x = (uint32_t)(lane * 8 + j) * 2654435761u + (uint32_t)k * 40503u + blockIdx.x;
            x ^= x >> 15; x *= 2246822519u; x ^= x >> 13;
            return (float)(x & 0xffffff) / 8388608.f - 1.f;
        };
        a[0][j] = (__bf16)rnd(0); a[1][j] = (__bf16)(rnd(1) * 0.004f); a[2][j] = (__bf16)(rnd(2) * 1.5e-5f);
        b.hi[j] = (__bf16)rnd(3); b.mid[j] = (__bf16)(rnd(4) * 0.004f); b.lo[j] = (__bf16)(rnd(5) * 1.5e-5f);
    }
    for (int it = 0; it < iters; ++it) {
        // same MACs as 8 tiles of 32x32x16 x6: 32 tiles of 16x16x32 x6 per 2 iterations
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            f32x4v c = acc[t];
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b.hi, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b.lo, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b.mid, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b.hi, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b.mid, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b.hi, c, 0, 0, 0);
            acc[t] = c;
        }
    }
    float s = 0.f;
    for (int t = 0; t < 32; ++t) for (int r = 0; r < 4; ++r) s += acc[t][r];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
extern "C" void launch16(float* out, int blocks, int iters, void* stream) {
    rate16_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(out, iters);
}
extern "C" void launch(float* out, int blocks, int iters, int variant, void* stream) {
    rate_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(out, iters, variant);
}
