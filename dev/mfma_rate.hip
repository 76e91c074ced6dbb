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
        a[0][j] = (__bf16)(float)(lane + j); a[1][j] = (__bf16)(0.01f * j); a[2][j] = (__bf16)(0.0001f);
        b.hi[j] = (__bf16)(float)j; b.mid[j] = (__bf16)0.001f; b.lo[j] = (__bf16)0.00001f;
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
extern "C" void launch(float* out, int blocks, int iters, int variant, void* stream) {
    rate_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(out, iters, variant);
}
