// Fused Adam step over every parameter tensor of the NeRF pair (SURVEY.md 8f
// row 3; the reference's optimizer is torch.optim.Adam built by
// utils/__init__.py:10-30, lr 5e-4, eps 1e-8).
//
// One launch updates all tensors: the tensor table travels in the kernel
// arguments (no pointer array in memory), each thread finds its tensor by a
// binary search over the table's prefix offsets, and reads g, m, v, p once /
// writes m, v, p once -- instead of the five full passes of torch's foreach
// implementation (lerp, mul, addcmul, sqrt/div/add, addcdiv).  Arithmetic is
// torch's single-tensor Adam (torch/optim/adam.py), op for op:
//   g += wd * p;  m = lerp(m, g, 1 - b1);  v = b2 * v + (1 - b2) * g * g
//   p -= step_size * m / (sqrt(v) / sqrt(bc2) + eps),  step_size = lr / bc1
#include "common.h"

namespace {

constexpr int kAdamMax = 48;

struct AdamArgs {
    float* p[kAdamMax];
    const float* g[kAdamMax];
    float* m[kAdamMax];
    float* v[kAdamMax];
    int64_t start[kAdamMax + 1];
    int count;
    float w1, beta2, w2, eps, wd, step_size, bc2_sqrt;
};

__global__ void __launch_bounds__(256) adam_kernel(const AdamArgs a) {
    const int64_t total = a.start[a.count];
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        int lo = 0, hi = a.count - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (a.start[mid] <= e) lo = mid; else hi = mid - 1;
        }
        const int64_t i = e - a.start[lo];
        float p = a.p[lo][i];
        float g = a.g[lo] ? a.g[lo][i] : 0.f;
        if (a.wd != 0.f) g = nr_add(g, nr_mul(p, a.wd));
        float m = a.m[lo][i], v = a.v[lo][i];
        m = nr_add(m, nr_mul(a.w1, nr_sub(g, m)));           // lerp, weight 1-b1 < 0.5
        v = nr_add(nr_mul(v, a.beta2), nr_mul(nr_mul(a.w2, g), g));   // mul_ then addcmul_
        const float denom = nr_add(sqrtf(v) / a.bc2_sqrt, a.eps);
        p = nr_sub(p, nr_mul(a.step_size, m / denom));
        a.m[lo][i] = m; a.v[lo][i] = v; a.p[lo][i] = p;
    }
}

}  // namespace

NR_API int nr_adam_max_tensors(void) { return kAdamMax; }

NR_API int nr_adam_step(float* const* params, const float* const* grads, float* const* exp_avg,
                        float* const* exp_avg_sq, const int64_t* numel, int count, double lr,
                        double beta1, double beta2, double eps, double weight_decay,
                        int64_t step, void* stream) {
    NR_REQUIRE(count >= 0 && count <= kAdamMax, "nr_adam_step: count %d outside [0, %d]", count,
               kAdamMax);
    NR_REQUIRE(step >= 1, "nr_adam_step: step counts from 1");
    if (count == 0) return 0;
    NR_REQUIRE(params && exp_avg && exp_avg_sq && numel && grads, "nr_adam_step: null table");
    AdamArgs a{};
    a.start[0] = 0;
    for (int k = 0; k < count; ++k) {
        NR_REQUIRE(numel[k] >= 0, "nr_adam_step: bad numel");
        a.p[k] = params[k]; a.g[k] = grads[k]; a.m[k] = exp_avg[k]; a.v[k] = exp_avg_sq[k];
        a.start[k + 1] = a.start[k] + numel[k];
    }
    a.count = count;
    // scalars as torch forms them: python doubles, rounded to fp32 when applied
    a.w1 = (float)(1.0 - beta1); a.beta2 = (float)beta2; a.w2 = (float)(1.0 - beta2);
    a.eps = (float)eps; a.wd = (float)weight_decay;
    const double bc1 = 1.0 - __builtin_pow(beta1, (double)step);
    const double bc2 = 1.0 - __builtin_pow(beta2, (double)step);
    a.step_size = (float)(lr / bc1);
    a.bc2_sqrt = (float)__builtin_sqrt(bc2);
    const int64_t total = a.start[count];
    if (total == 0) return 0;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    adam_kernel<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(a);
    NR_LAUNCH_CHECK("nr_adam_step");
    return 0;
}
