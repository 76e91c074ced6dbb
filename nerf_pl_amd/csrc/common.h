// Shared device/host helpers for the nerf_pl_amd HIP kernels (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define NR_API extern "C" __attribute__((visibility("default")))

// ---------------------------------------------------------------------------
// error reporting across the C ABI: 0 = ok, else a hipError_t or NR_E* code;
// message retrievable with nr_last_error() (thread-local).
// ---------------------------------------------------------------------------
enum {
    NR_OK = 0,
    NR_EINVAL = 10001,   // bad shape / argument
    NR_EALIGN = 10002,   // misaligned pointer
};

void nr_set_error(const char* fmt, ...);

#define NR_REQUIRE(cond, ...)                 \
    do {                                       \
        if (!(cond)) {                         \
            nr_set_error(__VA_ARGS__);         \
            return NR_EINVAL;                  \
        }                                      \
    } while (0)

#define NR_LAUNCH_CHECK(what)                                                    \
    do {                                                                          \
        hipError_t e_ = hipGetLastError();                                        \
        if (e_ != hipSuccess) {                                                   \
            nr_set_error("%s: launch failed: %s", what, hipGetErrorString(e_));   \
            return (int)e_;                                                       \
        }                                                                         \
    } while (0)

// ---------------------------------------------------------------------------
// Model geometry (models/nerf.py:41-81 defaults: D=8, W=256, 63/27 inputs)
// ---------------------------------------------------------------------------
#define NR_W 256
#define NR_WD 128        // W // 2 (dir branch)
#define NR_XYZ_CH 63
#define NR_DIR_CH 27
#define NR_PE_KSTEPS 32  // 63 xyz-PE channels + 1 pad, 2 per MFMA k-step
#define NR_DIR_KSTEPS 16 // 27 dir-PE channels + 5 pad, 2 per MFMA k-step

// Saved-activation record, per sample, in floats (each segment is a separate
// [n_samples][width] row-major array inside one buffer).
#define NR_SAVE_PE 64
#define NR_SAVE_DIR 32

// ---------------------------------------------------------------------------
// Philox4x32-10 counter RNG (production randomness; replay tensors are used
// for parity).  uniform in [0,1) with 24 random mantissa bits, like
// torch.rand's float path.
// ---------------------------------------------------------------------------
struct nr_u4 { uint32_t x, y, z, w; };

__device__ __forceinline__ nr_u4 nr_philox(uint32_t c0, uint32_t c1, uint32_t c2,
                                           uint32_t c3, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
        uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
        uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += W0; k1 += W1;
    }
    nr_u4 o = {c0, c1, c2, c3};
    return o;
}

__device__ __forceinline__ float nr_u01(uint32_t x) {
    return (float)(x >> 8) * (1.0f / 16777216.0f);
}

// stream = which of the 5 draws of a render_rays call
__device__ __forceinline__ float nr_rand_uniform(uint64_t seed, uint32_t stream, uint64_t idx) {
    nr_u4 r = nr_philox((uint32_t)idx, (uint32_t)(idx >> 32), stream, 0u,
                        (uint32_t)seed, (uint32_t)(seed >> 32));
    return nr_u01(r.x);
}

__device__ __forceinline__ float nr_rand_normal(uint64_t seed, uint32_t stream, uint64_t idx) {
    nr_u4 r = nr_philox((uint32_t)idx, (uint32_t)(idx >> 32), stream, 1u,
                        (uint32_t)seed, (uint32_t)(seed >> 32));
    float u1 = ((float)(r.x >> 8) + 1.0f) * (1.0f / 16777216.0f);   // (0,1]
    float u2 = nr_u01(r.y);
    return sqrtf(-2.0f * logf(u1)) * cosf(6.28318530717958647692f * u2);
}

// ---------------------------------------------------------------------------
// fp32 MFMA 32x32x2 (v_mfma_f32_32x32x2_f32), exact f32 fma-chain numerics.
// A[i][k]: lane l holds A[l&31][l>>5];  B[k][j]: lane l holds B[l>>5][l&31];
// D[i][j]: lane l, reg r holds D[(r&3) + 8*(r>>2) + 4*(l>>5)][l&31].
// ---------------------------------------------------------------------------
__device__ __forceinline__ f32x16 nr_mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// Row of accumulator register r for lane-half h (transposed-activation layout:
// rows are features, the lane's column is its sample).
__host__ __device__ __forceinline__ int nr_acc_row(int r, int h) {
    return (r & 3) + 8 * (r >> 2) + 4 * h;
}

// no-contraction helpers: the reference computes these with separate fp32
// multiply and add (PyTorch CPU elementwise kernels), so keep them unfused.
__device__ __forceinline__ float nr_mul(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float nr_add(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float nr_sub(float a, float b) { return __fsub_rn(a, b); }
