// The training loss of the reference: losses.py:4-14
// MSELoss = nn.MSELoss(reduction='mean')(rgb_coarse, target)
//           [+ the same for rgb_fine], and metrics.py:4-13 mse / psnr.
//
// One launch for the forward of both terms and one for the backward of both,
// instead of torch's sub / pow / mean / add chain and its autograd (about 20
// kernels of a few µs each per step at cfg2).
//
// Forward: one workgroup; the squared differences are formed in fp32 as torch
// does ((x - t) * (x - t)) and summed in double in a fixed order (lane-strided
// partial sums, then a fixed tree), so the result is deterministic and at
// least as accurate as the fp32 sum; each mean is rounded to fp32 and the two
// are added in fp32, as `loss = mse_c; loss += mse_f` does.
// loss[0] = loss; means (optional) = [mean over a, mean over b (0 without b)].
//
// Backward: d loss / d x = (2 / n) * (x - t) * g, the form of torch's
// mse_loss_backward, for both inputs in one elementwise launch; g is read from
// device memory (the upstream gradient of the scalar), so no host sync.
#include "common.h"

namespace {

constexpr int kT = 1024;

__global__ void __launch_bounds__(kT) mse_fwd_kernel(const float* __restrict__ a,
                                                     const float* __restrict__ b,
                                                     const float* __restrict__ t, int64_t n,
                                                     float* __restrict__ loss,
                                                     float* __restrict__ means) {
    double sa = 0.0, sb = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += kT) {
        const float ti = t[i];
        const float da = nr_sub(a[i], ti);
        sa += (double)nr_mul(da, da);
        if (b) {
            const float db = nr_sub(b[i], ti);
            sb += (double)nr_mul(db, db);
        }
    }
    __shared__ double ra[kT / 64], rb[kT / 64];
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
        sa += __shfl_xor(sa, d);
        sb += __shfl_xor(sb, d);
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) { ra[wave] = sa; rb[wave] = sb; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double ta = 0.0, tb = 0.0;
        for (int w = 0; w < kT / 64; ++w) { ta += ra[w]; tb += rb[w]; }
        const float ma = (float)(ta / (double)n);
        const float mb = b ? (float)(tb / (double)n) : 0.f;
        loss[0] = b ? nr_add(ma, mb) : ma;
        if (means) { means[0] = ma; means[1] = mb; }
    }
}

__global__ void __launch_bounds__(256) mse_bwd_kernel(const float* __restrict__ a,
                                                      const float* __restrict__ b,
                                                      const float* __restrict__ t, int64_t n,
                                                      float norm, const float* __restrict__ g,
                                                      float* __restrict__ ga,
                                                      float* __restrict__ gb) {
    const float gs = g[0];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float ti = t[i];
        if (ga) ga[i] = nr_mul(nr_mul(norm, nr_sub(a[i], ti)), gs);
        if (gb) gb[i] = nr_mul(nr_mul(norm, nr_sub(b[i], ti)), gs);
    }
}

}  // namespace

NR_API int nr_mse_loss(const float* a, const float* b, const float* target, int64_t n, float* loss,
                       float* means, void* stream) {
    NR_REQUIRE(n > 0, "nr_mse_loss: n = %lld (the mean of no elements is undefined)",
               (long long)n);
    NR_REQUIRE(a && target && loss, "nr_mse_loss: null pointer");
    mse_fwd_kernel<<<1, kT, 0, (hipStream_t)stream>>>(a, b, target, n, loss, means);
    NR_LAUNCH_CHECK("nr_mse_loss");
    return 0;
}

NR_API int nr_mse_loss_bwd(const float* a, const float* b, const float* target, int64_t n,
                           const float* g, float* ga, float* gb, void* stream) {
    NR_REQUIRE(n > 0, "nr_mse_loss_bwd: n = %lld", (long long)n);
    NR_REQUIRE(a && target && g, "nr_mse_loss_bwd: null pointer");
    NR_REQUIRE(!gb || b, "nr_mse_loss_bwd: gradient of b requested without b");
    if (!ga && !gb) return 0;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    mse_bwd_kernel<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(
        a, b, target, n, (float)(2.0 / (double)n), g, ga, gb);
    NR_LAUNCH_CHECK("nr_mse_loss_bwd");
    return 0;
}
