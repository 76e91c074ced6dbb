// Differentiable shadow mapping (config 5): efficient_sm / run_shadow_mapping.
//
// Reference: models/rendering_shadows.py:359-482 (efficient_sm and its run
// splitting loop :377-396), models/efficient_shadow_mapping.py:10-130,
// models/camera.py:121-132.  The reference walks the ray batch in Python,
// splitting it into runs of equal eye position with one torch.equal per ray
// and launching ~15 small torch ops per run.  Here one pass over the batch:
//
//   sm_runs_kernel      run start of every ray (segmented max-scan, 1 block)
//   sm_project_kernel   per ray: normed depth, 3x3 reprojection into the light
//                       camera, clamped nearest-texel gather of the light's
//                       normed depth map, shadow_method_1 output or the raw
//                       difference for shadow_method_2
//   sm_minmax_kernel    shadow_method_2: per-run min / max (one wave per run)
//   sm_norm_kernel      shadow_method_2: min-max normalisation, clip
//   backward: sm_bwd_reduce_kernel (per-run sums of the normalisation
//   gradient) + sm_bwd_kernel (d loss / d camera depth, and each ray's
//   contribution -d loss / d shadow difference to its gathered texel), then
//   for gradients into the light map (train_efficient_sm.py --grad_on_light,
//   :158-162) sm_scatter_kernel + sm_light_finish_kernel: the backward of the
//   texel gather w_light.view(w, h)[v, u] (efficient_shadow_mapping.py:98) as
//   a deterministic scatter-add -- every contribution converted to a 64-bit
//   fixed-point integer at one power-of-two scale per call (chosen from the
//   largest |contribution| so that no sum can overflow) and added with integer
//   atomics, which are associative: the texel sums do not depend on the order
//   the atomics land in, and they are exact to ~2^-60 of the largest term
//   (the reference's index_put_ accumulates in fp32, ray by ray).
//
// Arithmetic follows the reference's fp32 op order; the 3x3 products that set
// up the run's transform (M_L^-1 M, M_L^-1 (O - L)) are formed in double and
// rounded once (the reference uses LAPACK/BLAS in fp32 there).
#include "common.h"

#include <mutex>

namespace {

constexpr float kEps = 1e-5f;   // efficient_shadow_mapping.py:8

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ float wmin(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wmax(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

// sum(p[None, :] * M, -1) for one row of M (efficient_shadow_mapping.py:49-50)
__device__ __forceinline__ float rowdot(const float* p, const float* row) {
    return nr_add(nr_add(nr_mul(p[0], row[0]), nr_mul(p[1], row[1])), nr_mul(p[2], row[2]));
}

// workspace layout: per ray the run start, shadow difference, projection
// z-row, normed-depth denominator, per-run [min, max] and backward sums, the
// gathered texel and the texel-gradient contribution; then (8-byte aligned)
// the largest |contribution| and, per light texel, a 64-bit fixed-point
// accumulator and a non-finite flag
struct SmWs {
    int32_t* run; float* t; float* proj2; float* normp; float* mm; float* sums;
    int32_t* key; float* c; uint32_t* cmax; unsigned long long* acc; int32_t* flag;
};
__host__ __device__ inline int64_t sm_ray_words(int64_t n) { return (12 * n + 1) & ~(int64_t)1; }
__host__ __device__ inline SmWs sm_ws(void* base, int64_t n, int64_t n_light) {
    SmWs w;
    w.run = reinterpret_cast<int32_t*>(base);
    float* f = reinterpret_cast<float*>(base) + n;
    w.t = f; w.proj2 = f + n; w.normp = f + 2 * n; w.mm = f + 3 * n; w.sums = f + 5 * n;
    w.key = reinterpret_cast<int32_t*>(f + 9 * n);
    w.c = f + 10 * n;
    w.cmax = reinterpret_cast<uint32_t*>(base) + sm_ray_words(n);
    w.acc = reinterpret_cast<unsigned long long*>(w.cmax + 2);
    w.flag = reinterpret_cast<int32_t*>(w.acc + n_light);
    return w;
}
// bytes of the zero-initialised tail (cmax, acc, flag)
__host__ inline int64_t sm_tail_bytes(int64_t n_light) { return 8 + 12 * n_light; }

struct SmArgs {
    const float* pixels; const float* depth; const float* eye; const float* cams; int per_ray;
    const float* light_cam; const float* light_eye; const float* light_w; int res_w, res_h;
    int method; float delta, epsilon; int sigmoid; float out_eps; int n;
    SmWs ws; float* out;
};

// rendering_shadows.py:377-396: a run continues while eye_pos equals the run's
// first eye_pos (exact equality is transitive, so comparing neighbours is the
// same test).  One block; each thread owns a contiguous chunk, chunk results
// are combined with a max-scan of the last start seen.
__global__ void __launch_bounds__(1024) sm_runs_kernel(const float* __restrict__ eye,
                                                       int per_ray, int n,
                                                       int32_t* __restrict__ run) {
    __shared__ int32_t agg[1024];
    const int t = threadIdx.x;
    const int chunk = (n + 1023) / 1024;
    const int b = t * chunk, e = min(n, b + chunk);
    int32_t last = -1;
    for (int i = b; i < e; ++i) {
        bool start = i == 0;
        if (per_ray && i > 0) {
            const float* a = eye + (size_t)i * 3;
            start = !(a[0] == a[-3] && a[1] == a[-2] && a[2] == a[-1]);
        }
        if (start) last = i;
        run[i] = last;
    }
    agg[t] = last;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int32_t v = t >= o ? agg[t - o] : -1;
        __syncthreads();
        agg[t] = max(agg[t], v);
        __syncthreads();
    }
    const int32_t carry = t > 0 ? agg[t - 1] : -1;
    for (int i = b; i < e; ++i)
        if (run[i] < 0) run[i] = carry;
}

__device__ void inv3_double(const float* a, double* r) {
    const double a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3], a4 = a[4], a5 = a[5];
    const double a6 = a[6], a7 = a[7], a8 = a[8];
    const double c0 = a4 * a8 - a5 * a7, c1 = a5 * a6 - a3 * a8, c2 = a3 * a7 - a4 * a6;
    const double det = a0 * c0 + a1 * c1 + a2 * c2;
    const double id = 1.0 / det;
    r[0] = c0 * id; r[1] = (a2 * a7 - a1 * a8) * id; r[2] = (a1 * a5 - a2 * a4) * id;
    r[3] = c1 * id; r[4] = (a0 * a8 - a2 * a6) * id; r[5] = (a2 * a3 - a0 * a5) * id;
    r[6] = c2 * id; r[7] = (a1 * a6 - a0 * a7) * id; r[8] = (a0 * a4 - a1 * a3) * id;
}

// clip(x, 0, 1) with NaN passing through, like torch.clamp
__device__ __forceinline__ float clip01(float x) { return x < 0.f ? 0.f : (x > 1.f ? 1.f : x); }

__global__ void __launch_bounds__(256) sm_project_kernel(SmArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const int s = a.ws.run[i];
    const float* M = a.cams + (a.per_ray ? (size_t)s * 9 : 0);
    const float* E = a.eye + (a.per_ray ? (size_t)s * 3 : 0);
    const float p[3] = {a.pixels[(size_t)i * 3], a.pixels[(size_t)i * 3 + 1],
                        a.pixels[(size_t)i * 3 + 2]};
    // get_normed_w (efficient_shadow_mapping.py:41-58)
    const float c0 = rowdot(p, M), c1 = rowdot(p, M + 3), c2 = rowdot(p, M + 6);
    const float norm = sqrtf(nr_add(nr_add(nr_mul(c0, c0), nr_mul(c1, c1)), nr_mul(c2, c2)));
    const float normp = nr_add(norm, kEps);
    const float w = a.depth[i] / normp;
    // camera.py:121-132: R = M_L^-1 M, Q = M_L^-1 (O - L)
    double li[9];
    inv3_double(a.light_cam, li);
    float R[9], Q[3];
    const float om[3] = {nr_sub(E[0], a.light_eye[0]), nr_sub(E[1], a.light_eye[1]),
                         nr_sub(E[2], a.light_eye[2])};
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c)
            R[r * 3 + c] = (float)(li[r * 3] * M[c] + li[r * 3 + 1] * M[3 + c] +
                                   li[r * 3 + 2] * M[6 + c]);
        Q[r] = (float)(li[r * 3] * om[0] + li[r * 3 + 1] * om[1] + li[r * 3 + 2] * om[2]);
    }
    // get_diff_projections (:61-82)
    const float k0 = nr_add(nr_mul(w, rowdot(p, R)), Q[0]);
    const float k1 = nr_add(nr_mul(w, rowdot(p, R + 3)), Q[1]);
    const float proj2 = rowdot(p, R + 6);
    const float wl = nr_add(nr_mul(w, proj2), Q[2]);
    const float ul = k0 / wl, vl = k1 / wl;
    // get_projected_depths (:84-101): clamp, truncate, gather w_light.view(w, h)[v, u]
    const float uc = fminf((float)(a.res_w - 1), fmaxf(0.f, ul));
    const float vc = fminf((float)(a.res_h - 1), fmaxf(0.f, vl));
    const int key = (int)vc * a.res_h + (int)uc;
    const float wlb = a.light_w[key];
    const float d = nr_sub(wl, wlb);
    a.ws.key[i] = key;
    a.ws.t[i] = d;
    a.ws.proj2[i] = proj2;
    a.ws.normp[i] = normp;
    if (a.method == 1) {
        // generate_shadow_map shadow_method_1 (:117-119)
        float m = d / a.delta;
        m = (m < a.epsilon) ? a.epsilon : m;
        const float o = nr_add(clip01(m), a.out_eps);
        a.out[(size_t)i * 3 + 0] = o; a.out[(size_t)i * 3 + 1] = o; a.out[(size_t)i * 3 + 2] = o;
    }
}

// shadow_method_2: per-run min and max of the difference (one wave per run
// start found in the wave's 64 rays; runs are contiguous, so the scan of a
// run stops at the first chunk it does not fill).
__global__ void __launch_bounds__(256) sm_minmax_kernel(int n, SmWs ws) {
    const int lane = threadIdx.x & 63;
    const int base = ((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 64;
    if (base >= n) return;
    uint64_t starts = __ballot(base + lane < n && ws.run[base + lane] == base + lane);
    while (starts) {
        const int s = base + __ffsll((unsigned long long)starts) - 1;
        starts &= starts - 1;
        float mn = INFINITY, mx = -INFINITY;
        for (int j0 = s;; j0 += 64) {
            const int j = j0 + lane;
            const bool in = j < n && ws.run[j] == s;
            if (in) { const float v = ws.t[j]; mn = fminf(mn, v); mx = fmaxf(mx, v); }
            if (!__all(in)) break;
        }
        mn = wmin(mn); mx = wmax(mx);
        if (lane == 0) { ws.mm[2 * s] = mn; ws.mm[2 * s + 1] = mx; }
    }
}

__device__ __forceinline__ float sigmoidf_ref(float x) { return 1.f / (1.f + expf(-x)); }

// normalize_min_max (:10-11) then optional sigmoid and clip (:120-129)
__global__ void __launch_bounds__(256) sm_norm_kernel(SmArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const int s = a.ws.run[i];
    const float mn = a.ws.mm[2 * s], mx = a.ws.mm[2 * s + 1];
    float v = nr_sub(a.ws.t[i], mn) / nr_add(nr_sub(mx, mn), kEps);
    if (a.sigmoid) v = sigmoidf_ref(v);
    const float o = nr_add(clip01(v), a.out_eps);
    a.out[(size_t)i * 3 + 0] = o; a.out[(size_t)i * 3 + 1] = o; a.out[(size_t)i * 3 + 2] = o;
}

struct SmBwdArgs {
    const float* g_out; int method; float delta, epsilon; int sigmoid; int n; int n_light;
    SmWs ws; float* g_depth; float* g_light;
};

__device__ __forceinline__ float gsum3(const float* g, int i) {
    return nr_add(nr_add(g[(size_t)i * 3], g[(size_t)i * 3 + 1]), g[(size_t)i * 3 + 2]);
}

// d(output) / d(normalised value) for shadow_method_2 at ray i; also returns
// a = t - min and the denominator b
__device__ __forceinline__ float m2_gc(const SmBwdArgs& a, int i, float mn, float mx, float* pa,
                                       float* pb) {
    const float av = nr_sub(a.ws.t[i], mn);
    const float b = nr_add(nr_sub(mx, mn), kEps);
    float v = av / b;
    float g = gsum3(a.g_out, i);
    if (a.sigmoid) {
        const float y = sigmoidf_ref(v);
        g = (y >= 0.f && y <= 1.f) ? nr_mul(nr_mul(g, 1.f - y), y) : 0.f;
    } else {
        g = (v >= 0.f && v <= 1.f) ? g : 0.f;
    }
    *pa = av; *pb = b;
    return g;   // * (new_max - new_min) = 1
}

// per run: S_a = sum g_c / b, G_b = sum -g_c * ((a / b) / b), tie counts of min and max
__global__ void __launch_bounds__(256) sm_bwd_reduce_kernel(SmBwdArgs a) {
    const int lane = threadIdx.x & 63;
    const int base = ((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 64;
    if (base >= a.n) return;
    uint64_t starts = __ballot(base + lane < a.n && a.ws.run[base + lane] == base + lane);
    while (starts) {
        const int s = base + __ffsll((unsigned long long)starts) - 1;
        starts &= starts - 1;
        const float mn = a.ws.mm[2 * s], mx = a.ws.mm[2 * s + 1];
        float sa = 0.f, gb = 0.f, cmn = 0.f, cmx = 0.f;
        for (int j0 = s;; j0 += 64) {
            const int j = j0 + lane;
            const bool in = j < a.n && a.ws.run[j] == s;
            if (in) {
                float av, b;
                const float gc = m2_gc(a, j, mn, mx, &av, &b);
                sa += gc / b;
                gb += -gc * ((av / b) / b);
                const float t = a.ws.t[j];
                cmn += t == mn ? 1.f : 0.f;
                cmx += t == mx ? 1.f : 0.f;
            }
            if (!__all(in)) break;
        }
        sa = wsum(sa); gb = wsum(gb); cmn = wsum(cmn); cmx = wsum(cmx);
        if (lane == 0) {
            float* o = a.ws.sums + 4 * (size_t)s;
            o[0] = sa; o[1] = gb; o[2] = cmn; o[3] = cmx;
        }
    }
}

__device__ float sm_bwd_ray(const SmBwdArgs& a, int i) {
    float gt;
    if (a.method == 1) {
        // clip -> max(x/delta, eps) -> /delta   (torch.maximum splits ties)
        const float m = a.ws.t[i] / a.delta;
        const float mx = m < a.epsilon ? a.epsilon : m;
        const float g = (mx >= 0.f && mx <= 1.f) ? gsum3(a.g_out, i) : 0.f;
        const float gm = m > a.epsilon ? g : (m == a.epsilon ? 0.5f * g : 0.f);
        gt = gm / a.delta;
    } else {
        const int s = a.ws.run[i];
        const float mn = a.ws.mm[2 * s], mx = a.ws.mm[2 * s + 1];
        const float* su = a.ws.sums + 4 * (size_t)s;
        float av, b;
        const float gc = m2_gc(a, i, mn, mx, &av, &b);
        gt = gc / b;
        const float t = a.ws.t[i];
        // the two tensor.min() calls get -S_a and -G_b; tensor.max() gets G_b,
        // each spread evenly over its ties (torch's min/max backward)
        if (t == mn) gt += (-su[0]) / su[2] + (-su[1]) / su[2];
        if (t == mx) gt += su[1] / su[3];
    }
    return gt;   // d loss / d (wl - w_light_bounded)
}

__global__ void __launch_bounds__(256) sm_bwd_kernel(SmBwdArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = i < a.n;
    const float gt = in ? sm_bwd_ray(a, i) : 0.f;
    // wl = w * proj2 + Q2, w = depth / normp   (the texel index carries no gradient)
    if (in && a.g_depth) a.g_depth[i] = nr_mul(gt, a.ws.proj2[i]) / a.ws.normp[i];
    if (a.g_light) {
        // diff = wl - w_light_bounded: the gathered texel receives -gt
        const float c = -gt;
        if (in) a.ws.c[i] = c;
        float m = (in && __builtin_isfinite(c)) ? fabsf(c) : 0.f;
        m = wmax(m);      // every lane of the wave takes part
        if ((threadIdx.x & 63) == 0 && m > 0.f) atomicMax(a.ws.cmax, __float_as_uint(m));
    }
}

// fixed-point scale of the scatter: 2^(62 - E - L) with max|c| < 2^E and
// n < 2^L, so that |sum| < n max|c| stays below 2^62
__device__ __forceinline__ int sm_fix_exp(uint32_t cmax_bits, int n) {
    int e;
    (void)frexpf(__uint_as_float(cmax_bits), &e);
    const int l = 64 - __clzll((unsigned long long)n);
    return 62 - e - l;
}

__global__ void __launch_bounds__(256) sm_scatter_kernel(SmBwdArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t mb = *a.ws.cmax;
    const float c = a.ws.c[i];
    const int k = a.ws.key[i];
    if (!__builtin_isfinite(c)) { a.ws.flag[k] = 1; return; }
    if (mb == 0u || c == 0.f) return;
    const long long q = __double2ll_rn(ldexp((double)c, sm_fix_exp(mb, a.n)));
    atomicAdd(a.ws.acc + k, (unsigned long long)q);
}

__global__ void __launch_bounds__(256) sm_light_finish_kernel(SmBwdArgs a) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.n_light) return;
    const uint32_t mb = *a.ws.cmax;
    float g = 0.f;
    if (a.ws.flag[k]) g = __builtin_nanf("");
    else if (mb != 0u)
        g = (float)ldexp((double)(long long)a.ws.acc[k], -sm_fix_exp(mb, a.n));
    a.g_light[k] = g;
}

__global__ void __launch_bounds__(256) sm_normed_kernel(const float* __restrict__ M,
                                                        const float* __restrict__ pixels,
                                                        const float* __restrict__ depth, int n,
                                                        float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float p[3] = {pixels[(size_t)i * 3], pixels[(size_t)i * 3 + 1], pixels[(size_t)i * 3 + 2]};
    const float c0 = rowdot(p, M), c1 = rowdot(p, M + 3), c2 = rowdot(p, M + 6);
    const float norm = sqrtf(nr_add(nr_add(nr_mul(c0, c0), nr_mul(c1, c1)), nr_mul(c2, c2)));
    out[i] = depth[i] / nr_add(norm, kEps);
}

// its backward: d/d depth of depth / (|M p| + 1e-5) (torch's DivBackward: g / b)
__global__ void __launch_bounds__(256) sm_normed_bwd_kernel(const float* __restrict__ M,
                                                            const float* __restrict__ pixels,
                                                            const float* __restrict__ g, int n,
                                                            float* __restrict__ g_depth) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float p[3] = {pixels[(size_t)i * 3], pixels[(size_t)i * 3 + 1], pixels[(size_t)i * 3 + 2]};
    const float c0 = rowdot(p, M), c1 = rowdot(p, M + 3), c2 = rowdot(p, M + 6);
    const float norm = sqrtf(nr_add(nr_add(nr_mul(c0, c0), nr_mul(c1, c1)), nr_mul(c2, c2)));
    g_depth[i] = g[i] / nr_add(norm, kEps);
}

// The backward re-derives the workspace layout from (n, n_light) and clears
// and atomically adds into its tail, so it must see the layout the forward
// used.  The forward records, per workspace base address, the (n, n_light) it
// laid out; the backward refuses any other pair (a wrong n_light would write
// past the buffer).  Host-side and bounded: the most recent kWsSlots
// workspaces (a training step uses one or two).
constexpr int kWsSlots = 1024;
struct WsRecord { const void* base; int64_t n, n_light; };
std::mutex g_ws_mu;
WsRecord g_ws[kWsSlots];
int g_ws_next = 0;

void ws_record(const void* base, int64_t n, int64_t n_light) {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    for (auto& r : g_ws)
        if (r.base == base) { r.n = n; r.n_light = n_light; return; }
    g_ws[g_ws_next] = WsRecord{base, n, n_light};
    g_ws_next = (g_ws_next + 1) % kWsSlots;
}

// 0: laid out by the forward for (n, n_light); 1: for another pair; 2: unknown
int ws_check(const void* base, int64_t n, int64_t n_light, int64_t* fn, int64_t* fl) {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    for (const auto& r : g_ws)
        if (r.base == base) {
            *fn = r.n; *fl = r.n_light;
            return (r.n == n && r.n_light == n_light) ? 0 : 1;
        }
    return 2;
}

}  // namespace

NR_API int64_t nr_sm_workspace_bytes(int64_t n, int64_t n_light) {
    if (n < 0 || n_light < 0) return -1;
    return sm_ray_words(n) * 4 + sm_tail_bytes(n_light);
}

NR_API int nr_sm_normed_depth(const float* camera, const float* pixels, const float* depth,
                              int64_t n, float* out, void* stream) {
    NR_REQUIRE(n >= 0 && n < ((int64_t)1 << 31), "nr_sm_normed_depth: bad size");
    if (n == 0) return 0;
    NR_REQUIRE(camera && pixels && depth && out, "nr_sm_normed_depth: null pointer");
    sm_normed_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        camera, pixels, depth, (int)n, out);
    NR_LAUNCH_CHECK("nr_sm_normed_depth");
    return 0;
}

NR_API int nr_sm_normed_depth_bwd(const float* camera, const float* pixels, const float* g_out,
                                  int64_t n, float* g_depth, void* stream) {
    NR_REQUIRE(n >= 0 && n < ((int64_t)1 << 31), "nr_sm_normed_depth_bwd: bad size");
    if (n == 0) return 0;
    NR_REQUIRE(camera && pixels && g_out && g_depth, "nr_sm_normed_depth_bwd: null pointer");
    sm_normed_bwd_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        camera, pixels, g_out, (int)n, g_depth);
    NR_LAUNCH_CHECK("nr_sm_normed_depth_bwd");
    return 0;
}

NR_API int nr_sm_forward(const float* pixels, const float* depth, const float* eye,
                         const float* cameras, int per_ray, const float* light_camera,
                         const float* light_eye, const float* light_w, int res_w, int res_h,
                         int method, float delta, float epsilon, int sigmoid, float out_eps,
                         int64_t n, void* workspace, float* out, void* stream) {
    NR_REQUIRE(n >= 0 && n < ((int64_t)1 << 31), "nr_sm_forward: bad size");
    NR_REQUIRE(method == 1 || method == 2, "nr_sm_forward: method must be 1 or 2");
    NR_REQUIRE(res_w > 0 && res_h > 0 && res_h <= res_w,
               "nr_sm_forward: need res_h <= res_w (w_light.view(w, h)[v, u] with v < h), "
               "got %dx%d", res_w, res_h);
    if (n == 0) return 0;
    NR_REQUIRE(pixels && depth && eye && cameras && light_camera && light_eye && light_w &&
               workspace && out, "nr_sm_forward: null pointer");
    // 64-bit fixed-point accumulators live in the tail (8-byte aligned relative to the base)
    NR_REQUIRE(((uintptr_t)workspace & 7) == 0, "nr_sm_forward: workspace must be 8-byte aligned");
    hipStream_t st = (hipStream_t)stream;
    SmArgs a{pixels, depth, eye, cameras, per_ray, light_camera, light_eye, light_w, res_w,
             res_h, method, delta, epsilon, sigmoid, out_eps, (int)n,
             sm_ws(workspace, n, (int64_t)res_w * res_h), out};
    sm_runs_kernel<<<1, 1024, 0, st>>>(eye, per_ray, (int)n, a.ws.run);
    const unsigned blocks = (unsigned)((n + 255) / 256);
    sm_project_kernel<<<blocks, 256, 0, st>>>(a);
    if (method == 2) {
        sm_minmax_kernel<<<blocks, 256, 0, st>>>((int)n, a.ws);
        sm_norm_kernel<<<blocks, 256, 0, st>>>(a);
    }
    NR_LAUNCH_CHECK("nr_sm_forward");
    ws_record(workspace, n, (int64_t)res_w * res_h);
    return 0;
}

NR_API int nr_sm_backward(const float* g_out, void* workspace, int method, float delta,
                          float epsilon, int sigmoid, int64_t n, int64_t n_light, float* g_depth,
                          float* g_light_w, void* stream) {
    NR_REQUIRE(n >= 0 && n < ((int64_t)1 << 31), "nr_sm_backward: bad size");
    NR_REQUIRE(n_light > 0 && n_light < ((int64_t)1 << 31), "nr_sm_backward: bad light map size");
    NR_REQUIRE(method == 1 || method == 2, "nr_sm_backward: method must be 1 or 2");
    hipStream_t st = (hipStream_t)stream;
    if (n == 0) {
        // no camera rays: the light map receives no gradient
        if (g_light_w && hipMemsetAsync(g_light_w, 0, (size_t)n_light * 4, st) != hipSuccess) {
            nr_set_error("nr_sm_backward: memset failed");
            return NR_EINVAL;
        }
        return 0;
    }
    NR_REQUIRE(g_out && workspace && (g_depth || g_light_w), "nr_sm_backward: null pointer");
    NR_REQUIRE(((uintptr_t)workspace & 7) == 0, "nr_sm_backward: workspace must be 8-byte aligned");
    {
        int64_t fn = 0, fl = 0;
        const int w = ws_check(workspace, n, n_light, &fn, &fl);
        NR_REQUIRE(w != 2, "nr_sm_backward: workspace %p was not laid out by nr_sm_forward",
                   workspace);
        NR_REQUIRE(w == 0, "nr_sm_backward: workspace laid out by nr_sm_forward for n=%lld rays "
                   "and a %lld-texel light map, called with n=%lld, n_light=%lld",
                   (long long)fn, (long long)fl, (long long)n, (long long)n_light);
    }
    SmBwdArgs a{g_out, method, delta, epsilon, sigmoid, (int)n, (int)n_light,
                sm_ws(workspace, n, n_light), g_depth, g_light_w};
    const unsigned blocks = (unsigned)((n + 255) / 256);
    if (g_light_w) {
        const hipError_t e = hipMemsetAsync(a.ws.cmax, 0, (size_t)sm_tail_bytes(n_light), st);
        if (e != hipSuccess) {
            nr_set_error("nr_sm_backward: memset failed: %s", hipGetErrorString(e));
            return (int)e;
        }
    }
    if (method == 2) sm_bwd_reduce_kernel<<<blocks, 256, 0, st>>>(a);
    sm_bwd_kernel<<<blocks, 256, 0, st>>>(a);
    if (g_light_w) {
        sm_scatter_kernel<<<blocks, 256, 0, st>>>(a);
        sm_light_finish_kernel<<<(unsigned)((n_light + 255) / 256), 256, 0, st>>>(a);
    }
    NR_LAUNCH_CHECK("nr_sm_backward");
    return 0;
}
