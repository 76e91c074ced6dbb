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

// ---------------------------------------------------------------------------
// losses.py:28-73 OpactiyLoss (loss_dict['opacity'], constructed by
// train_efficient_sm.py:43 and evaluated on the light render at :191):
//   gray = (t[:,0] + t[:,1] + t[:,2]) / 3;  sm = gray > thres, non = gray <= thres
//   (torch.where on each comparison: a NaN grey value is in neither set)
//   loss = coeff - |mean(o_c[non]) - mean(o_c[sm])|  [+ the same on o_f]
// (L1Loss of two scalars), 0 when either set is empty.  The targets index the
// opacity rows (the reference indexes the light render's opacities with the
// camera batch's pixel indices), so n_t <= n_o.  One workgroup, fp32 gray
// values and comparisons as torch, double sums in a fixed order.
// stats (8 floats): [n_sm, n_non, mean_sm_c, mean_non_c, mean_sm_f, mean_non_f,
// valid, 0] for the backward.
// ---------------------------------------------------------------------------
namespace {

// 0: shadow pixel (gray > thres), 1: non-shadow (gray <= thres), -1: neither (NaN)
__device__ __forceinline__ int op_set(const float* t, int64_t i, float thres) {
    const float gray = nr_add(nr_add(t[3 * i], t[3 * i + 1]), t[3 * i + 2]) / 3.0f;
    return gray > thres ? 0 : (gray <= thres ? 1 : -1);
}

__global__ void __launch_bounds__(kT) opacity_fwd_kernel(const float* __restrict__ oc,
                                                         const float* __restrict__ of,
                                                         const float* __restrict__ t, int64_t n,
                                                         float thres, float coeff,
                                                         float* __restrict__ loss,
                                                         float* __restrict__ stats) {
    double v[6] = {0, 0, 0, 0, 0, 0};   // n_sm, n_non, sum_sm_c, sum_non_c, sum_sm_f, sum_non_f
    for (int64_t i = threadIdx.x; i < n; i += kT) {
        const int s = op_set(t, i, thres);
        if (s < 0) continue;
        v[s] += 1.0;
        v[2 + s] += (double)oc[i];
        if (of) v[4 + s] += (double)of[i];
    }
    __shared__ double part[kT / 64][6];
#pragma unroll
    for (int k = 0; k < 6; ++k)
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) v[k] += __shfl_xor(v[k], d);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0)
        for (int k = 0; k < 6; ++k) part[wave][k] = v[k];
    __syncthreads();
    if (threadIdx.x == 0) {
        double s[6] = {0, 0, 0, 0, 0, 0};
        for (int w = 0; w < kT / 64; ++w)
            for (int k = 0; k < 6; ++k) s[k] += part[w][k];
        const bool valid = s[0] > 0 && s[1] > 0;
        float out = 0.f, m[4] = {0, 0, 0, 0};
        if (valid) {
            m[0] = (float)(s[2] / s[0]); m[1] = (float)(s[3] / s[1]);
            out = nr_sub(coeff, fabsf(nr_sub(m[1], m[0])));
            if (of) {
                m[2] = (float)(s[4] / s[0]); m[3] = (float)(s[5] / s[1]);
                out = nr_add(out, nr_sub(coeff, fabsf(nr_sub(m[3], m[2]))));
            }
        }
        loss[0] = out;
        stats[0] = (float)s[0]; stats[1] = (float)s[1];
        stats[2] = m[0]; stats[3] = m[1]; stats[4] = m[2]; stats[5] = m[3];
        stats[6] = valid ? 1.f : 0.f; stats[7] = 0.f;
    }
}

__device__ __forceinline__ float op_sign(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

// d loss / d o_i = g * (-sign(a - b) / n_non for i in non, +sign(a - b) / n_sm for i in sm),
// a = mean(o[non]), b = mean(o[sm]); rows i >= n_t (not indexed) get 0
__global__ void __launch_bounds__(256) opacity_bwd_kernel(const float* __restrict__ t, int64_t n_t,
                                                          int64_t n_o, float thres,
                                                          const float* __restrict__ stats,
                                                          const float* __restrict__ g,
                                                          float* __restrict__ gc,
                                                          float* __restrict__ gf) {
    const float gs = g[0];
    const bool valid = stats[6] != 0.f;
    const float sc = op_sign(nr_sub(stats[3], stats[2]));
    const float sf = op_sign(nr_sub(stats[5], stats[4]));
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_o;
         i += (int64_t)gridDim.x * blockDim.x) {
        float vc = 0.f, vf = 0.f;
        const int set = (valid && i < n_t) ? op_set(t, i, thres) : -1;
        if (set >= 0) {
            const bool sm = set == 0;
            const float cnt = sm ? stats[0] : stats[1];
            vc = nr_mul(gs, sm ? sc : -sc) / cnt;
            vf = nr_mul(gs, sm ? sf : -sf) / cnt;
        }
        if (gc) gc[i] = vc;
        if (gf) gf[i] = vf;
    }
}

}  // namespace

NR_API int nr_opacity_loss(const float* opacity_c, const float* opacity_f, const float* target,
                           int64_t n_t, int64_t n_o, float thres, float coeff, float* loss,
                           float* stats, void* stream) {
    NR_REQUIRE(n_t >= 0 && n_o >= 0, "nr_opacity_loss: bad sizes");
    NR_REQUIRE(n_t <= n_o, "nr_opacity_loss: %lld targets index only %lld opacities",
               (long long)n_t, (long long)n_o);
    NR_REQUIRE(opacity_c && loss && stats && (target || n_t == 0), "nr_opacity_loss: null pointer");
    opacity_fwd_kernel<<<1, kT, 0, (hipStream_t)stream>>>(opacity_c, opacity_f, target, n_t, thres,
                                                         coeff, loss, stats);
    NR_LAUNCH_CHECK("nr_opacity_loss");
    return 0;
}

NR_API int nr_opacity_loss_bwd(const float* target, int64_t n_t, int64_t n_o, float thres,
                               const float* stats, const float* g, float* g_opacity_c,
                               float* g_opacity_f, void* stream) {
    NR_REQUIRE(n_t >= 0 && n_o >= 0 && n_t <= n_o, "nr_opacity_loss_bwd: bad sizes");
    NR_REQUIRE(stats && g && (target || n_t == 0), "nr_opacity_loss_bwd: null pointer");
    if ((!g_opacity_c && !g_opacity_f) || n_o == 0) return 0;
    int64_t blocks = (n_o + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    opacity_bwd_kernel<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(
        target, n_t, n_o, thres, stats, g, g_opacity_c, g_opacity_f);
    NR_LAUNCH_CHECK("nr_opacity_loss_bwd");
    return 0;
}
