// Per-ray kernels of models/rendering.py: stratified depths (:216-232), volume
// compositing (:169-198) and its backward, the uniform-bin inverse-CDF
// sample_pdf (:14-48) fused with the sort/merge of coarse+fine depths
// (:257), plus the weight-pack gather used by the fused MLP kernels.
//
// One wave per ray for the scans (64 lanes over the samples, chunked by 64);
// element-parallel for the depth generation and the pack.
#include "layout.h"

namespace {

__device__ __forceinline__ double wave_incl_prod(double v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const double o = __shfl_up(v, d);
        if (lane >= d) v *= o;
    }
    return v;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    return v;
}

// Reverse (suffix) scan of affine maps R -> a*R + b, composed right-to-left:
// returns for lane i the composition f_i o f_{i+1} o ... o f_63 as (A, B).
template <typename T>
__device__ __forceinline__ void wave_suffix_affine(T& a, T& b, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const T na = __shfl_down(a, d);
        const T nb = __shfl_down(b, d);
        if (lane + d < 64) {   // f_i o g: R -> a*(na*R + nb) + b
            b = fma(a, nb, b);
            a = a * na;
        }
    }
}

// ---------------------------------------------------------------------------
// stratified coarse depths, rendering.py:216-232
// ---------------------------------------------------------------------------
__global__ void coarse_z_kernel(const float* __restrict__ rays, const float* __restrict__ tlin,
                                int n_rays, int S, int use_disp, float perturb,
                                const float* __restrict__ u, uint64_t seed,
                                float* __restrict__ z_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)n_rays * S) return;
    const int ray = (int)(i / S), k = (int)(i % S);
    const float near = rays[(size_t)ray * 8 + 6], far = rays[(size_t)ray * 8 + 7];
    auto zat = [&](int kk) -> float {
        const float t = tlin[kk];
        if (!use_disp) return nr_add(nr_mul(near, 1.f - t), nr_mul(far, t));
        const float inv = nr_add(nr_mul(1.f / near, 1.f - t), nr_mul(1.f / far, t));
        return 1.f / inv;
    };
    float z = zat(k);
    if (perturb > 0.f) {
        const float zl = k > 0 ? zat(k - 1) : z;
        const float zr = k < S - 1 ? zat(k + 1) : z;
        const float lower = k > 0 ? nr_mul(0.5f, nr_add(zl, z)) : z;
        const float upper = k < S - 1 ? nr_mul(0.5f, nr_add(z, zr)) : z;
        const float r = u ? u[i] : nr_rand_uniform(seed, 0, (uint64_t)i);
        z = nr_add(lower, nr_mul(nr_sub(upper, lower), nr_mul(perturb, r)));
    }
    z_out[i] = z;
}

// ---------------------------------------------------------------------------
// volume compositing, rendering.py:169-198 (one wave per ray)
// raw: per-sample rows of raw_stride floats, sigma at column sig_col, rgb at 0..2
// ---------------------------------------------------------------------------
struct CompArgs {
    const float* raw; int raw_stride; int sig_col;
    const float* z; const float* rays; const float* noise;
    float noise_std; uint64_t seed; uint32_t stream;
    int n_rays, S, white_back, weights_only;
    float* rgb; float* depth; float* opacity; float* weights;
};

__device__ __forceinline__ float ray_dnorm(const float* r) {
    // torch.norm(rays_d, dim=-1) (rendering.py:176)
    return sqrtf(nr_add(nr_add(nr_mul(r[3], r[3]), nr_mul(r[4], r[4])), nr_mul(r[5], r[5])));
}

__device__ __forceinline__ float sample_noise(const float* noise, float noise_std, uint64_t seed,
                                              uint32_t stream, int64_t idx) {
    if (noise) return nr_mul(noise[idx], noise_std);
    if (noise_std == 0.f) return 0.f;
    return nr_mul(nr_rand_normal(seed, stream, (uint64_t)idx), noise_std);
}

// the last sample's delta, 1e10 * |d| (rendering.py:171).  With one sample per
// ray the reference's delta_inf = ones_like(deltas[:, :1]) is an empty column,
// so nothing is composited (weights (N, 0), every output 0): delta 0 gives
// alpha 0 and the same outputs and (zero) gradients
__device__ __forceinline__ float last_delta(int S, float dn) { return S > 1 ? nr_mul(1e10f, dn) : 0.f; }

// alpha = 1 - exp(-delta * relu(sigma + noise))   (rendering.py:181)
__device__ __forceinline__ float alpha_of(float sigma, float noise, float delta) {
    const float s = nr_add(sigma, noise);
    const float r = s > 0.f ? s : 0.f;
    return 1.f - expf(nr_mul(-delta, r));
}

__global__ void composite_fwd_kernel(CompArgs a) {
    const int lane = threadIdx.x & 63;
    const int ray = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (ray >= a.n_rays) return;
    const float* r = a.rays + (size_t)ray * 8;
    const float dn = ray_dnorm(r);
    const int S = a.S;
    const int64_t base = (int64_t)ray * S;
    double carry = 1.0;
    float acc_w = 0.f, acc_r = 0.f, acc_g = 0.f, acc_b = 0.f;
    // depth = sum w_i z_i (rendering.py:185) in double: at near/far 1/200 the
    // terms reach ~200, where an fp32 sum over 192 samples drifts by ~3e-5 --
    // a third of the north star's 1e-4 abs.  In double our depth is the exact
    // sum of the fp32 products rounded once, so its distance from the
    // reference is the reference's own (fp32) summation error
    double acc_d = 0.0;
    for (int c0 = 0; c0 < S; c0 += 64) {
        const int i = c0 + lane;
        const bool v = i < S;
        float alpha = 0.f, zi = 0.f;
        if (v) {
            zi = a.z[base + i];
            const float delta = i + 1 < S ? nr_mul(nr_sub(a.z[base + i + 1], zi), dn)
                                          : last_delta(S, dn);
            const float sigma = a.raw[(base + i) * a.raw_stride + a.sig_col];
            alpha = alpha_of(sigma, sample_noise(a.noise, a.noise_std, a.seed, a.stream, base + i),
                             delta);
        }
        // T_i = prod_{j<i} (1 - alpha_j + 1e-10), accumulated in double like
        // the reference's CPU cumprod (acc_type<float> = double)
        const float fac = v ? nr_add(1.f - alpha, 1e-10f) : 1.f;
        const double incl = wave_incl_prod((double)fac, lane);
        double excl = __shfl_up(incl, 1);
        if (lane == 0) excl = 1.0;
        const float T = (float)(carry * excl);
        carry *= __shfl(incl, 63);
        const float w = nr_mul(alpha, T);
        if (v) {
            a.weights[base + i] = w;
            acc_w += w;
            if (!a.weights_only) {
                if (a.rgb) {
                    const float* rr = a.raw + (base + i) * a.raw_stride;
                    acc_r = fmaf(w, rr[0], acc_r);
                    acc_g = fmaf(w, rr[1], acc_g);
                    acc_b = fmaf(w, rr[2], acc_b);
                }
                acc_d = fma((double)w, (double)zi, acc_d);
            }
        }
    }
    acc_w = wave_sum(acc_w);
    if (a.weights_only) {
        if (lane == 0) a.opacity[ray] = acc_w;
        return;
    }
    acc_r = wave_sum(acc_r); acc_g = wave_sum(acc_g); acc_b = wave_sum(acc_b);
    acc_d = wave_sum(acc_d);
    if (lane == 0) {
        const float bg = a.white_back ? 1.f - acc_w : 0.f;   // rendering.py:195-196
        if (a.rgb) {
            a.rgb[(size_t)ray * 3 + 0] = acc_r + bg;
            a.rgb[(size_t)ray * 3 + 1] = acc_g + bg;
            a.rgb[(size_t)ray * 3 + 2] = acc_b + bg;
        }
        a.depth[ray] = (float)acc_d;
        a.opacity[ray] = acc_w;
    }
}

// ---------------------------------------------------------------------------
// compositing backward: d(rgb, depth, opacity) -> d(raw rgb, raw sigma)
//   dw_i  = <drgb, c_i> + ddepth z_i + dopac (- sum drgb if white_back)
//   R_i   = sum_{k>i} dw_k a_k prod_{i<j<k} f_j,   f_j = 1 - a_j + 1e-10
//   da_i  = T_i (dw_i - R_i)
//   dsig  = da_i * exp(-delta r) * delta * [sigma + n > 0]
//   dc_i  = w_i * drgb
// Evaluated in double from the fp32 inputs (sigma + noise as the forward
// rounds it, depths, directions), each gradient rounded to fp32 once:
// dw_i - R_i cancels (a sample's own colour against the transmittance-weighted
// colours behind it), and in fp32 that cancellation made d sigma -- and the
// sigma bias's gradient, a sum of d sigma over every sample -- the one
// gradient measurably farther from float64 than the reference's fp32
// autograd (tests/test_gpu_cfg4.py at near/far 1/200)
// ---------------------------------------------------------------------------
struct CompBwdArgs {
    const float* raw; int raw_stride; int sig_col; const float* z; const float* rays; const float* noise;
    float noise_std; uint64_t seed; uint32_t stream;
    int n_rays, S, white_back;
    const float* g_rgb; const float* g_depth; const float* g_opacity;
    float* g_raw;   // (n_rays*S, raw_stride)
};

// delta_i in double from the fp32 depths (the last: 1e10 |d|, rendering.py:171)
__device__ __forceinline__ double delta_d(const float* z, int64_t base, int i, int S, double dn) {
    if (i + 1 < S) return ((double)z[base + i + 1] - (double)z[base + i]) * dn;
    return S > 1 ? 1e10 * dn : 0.0;
}

__global__ void composite_bwd_kernel(CompBwdArgs a) {
    const int lane = threadIdx.x & 63;
    const int ray = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (ray >= a.n_rays) return;
    const float* r = a.rays + (size_t)ray * 8;
    const double dn = sqrt((double)r[3] * r[3] + (double)r[4] * r[4] + (double)r[5] * r[5]);
    const int S = a.S;
    const int64_t base = (int64_t)ray * S;
    const float gr = a.g_rgb ? a.g_rgb[(size_t)ray * 3 + 0] : 0.f;
    const float gg = a.g_rgb ? a.g_rgb[(size_t)ray * 3 + 1] : 0.f;
    const float gb = a.g_rgb ? a.g_rgb[(size_t)ray * 3 + 2] : 0.f;
    const float gd = a.g_depth ? a.g_depth[ray] : 0.f;
    double go = a.g_opacity ? a.g_opacity[ray] : 0.f;
    if (a.white_back) go -= (double)gr + (double)gg + (double)gb;
    const int nchunks = (S + 63) >> 6;
    // relu(sigma + noise) as the forward forms it (fp32 add), widened
    auto rel = [&](int i) {
        const float s = nr_add(a.raw[(base + i) * a.raw_stride + a.sig_col],
                               sample_noise(a.noise, a.noise_std, a.seed, a.stream, base + i));
        return s;
    };

    // pass 1: forward transmittance carry per chunk start, kept implicitly by
    // recomputation; pass 2 walks chunks from the back carrying R.
    double Rcarry = 0.0;  // R at the first sample of the following chunk, seen from before it
    for (int ci = nchunks - 1; ci >= 0; --ci) {
        const int c0 = ci * 64;
        // transmittance entering this chunk
        double carry = 1.0;
        for (int cj = 0; cj < ci; ++cj) {
            const int j = cj * 64 + lane;
            double fac = 1.0;
            if (j < S) {
                const float s = rel(j);
                fac = exp(-delta_d(a.z, base, j, S, dn) * (s > 0.f ? (double)s : 0.0)) + 1e-10;
            }
            carry *= __shfl(wave_incl_prod(fac, lane), 63);
        }
        const int i = c0 + lane;
        const bool v = i < S;
        double alpha = 0.0, e = 1.0, delta = 0.0;
        float srel = 0.f, cr = 0.f, cg = 0.f, cb = 0.f, zi = 0.f;
        if (v) {
            zi = a.z[base + i];
            delta = delta_d(a.z, base, i, S, dn);
            const float* rr = a.raw + (base + i) * a.raw_stride;
            if (a.raw_stride == 4) { cr = rr[0]; cg = rr[1]; cb = rr[2]; }
            srel = rel(i);
            e = exp(-delta * (srel > 0.f ? (double)srel : 0.0));
            alpha = 1.0 - e;
        }
        const double fac = v ? e + 1e-10 : 1.0;       // 1 - alpha + 1e-10
        const double incl = wave_incl_prod(fac, lane);
        double excl = __shfl_up(incl, 1);
        if (lane == 0) excl = 1.0;
        const double T = carry * excl;
        double dw = 0.0;
        if (v) dw = (double)gr * cr + (double)gg * cg + (double)gb * cb + (double)gd * zi + go;
        // suffix affine scan inside the chunk: element i contributes the map
        // R -> f_i R + dw_i a_i to the samples before it.
        double A = fac, Bv = v ? dw * alpha : 0.0;
        wave_suffix_affine(A, Bv, lane);   // lane i: composition f_i..f_63
        // R_i = composition of lanes i+1..63 applied to Rcarry
        double An = __shfl_down(A, 1), Bn = __shfl_down(Bv, 1);
        if (lane == 63) { An = 1.0; Bn = 0.0; }
        const double Ri = fma(An, Rcarry, Bn);
        const double Rnext = fma(__shfl(A, 0), Rcarry, __shfl(Bv, 0));
        if (v) {
            const float dsig = srel > 0.f ? (float)(T * (dw - Ri) * e * delta) : 0.f;
            const float w = (float)(alpha * T);
            if (a.raw_stride == 4) {
                f32x4 o = {w * gr, w * gg, w * gb, dsig};
                *reinterpret_cast<f32x4*>(a.g_raw + (base + i) * 4) = o;
            } else {
                a.g_raw[(base + i) * a.raw_stride + a.sig_col] = dsig;
            }
        }
        Rcarry = Rnext;
    }
}

// ---------------------------------------------------------------------------
// sample_pdf (rendering.py:14-48) + sort(cat[z_coarse, z_pdf]) (:257)
// one wave per ray; cdf and merge staged in (dynamic) LDS:
//   cdf [nb + 1] | coarse depths [S] | importance depths [P = pow2 >= I]
// ---------------------------------------------------------------------------
constexpr int kPdfMaxBins = 1024;
constexpr int kMergeMax = 2048;

struct PdfArgs {
    const float* weights; int S;      // coarse weights (n_rays, S); bins = w[:, 1:S-1]
    const float* rays; const float* z_coarse;
    const float* u; const float* jitter; uint64_t seed;
    int n_rays, I, P;  // P: the importance region padded to a power of two
    float* z_pdf;      // (n_rays, I) or null
    float* z_fine;     // (n_rays, S + I) sorted, or null
};

// number of the n sorted values v[] that are < x (UPPER: <= x)
template <bool UPPER>
__device__ __forceinline__ int count_below(const float* v, int n, float x) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (UPPER ? v[mid] <= x : v[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(64) sample_pdf_kernel(PdfArgs a) {
    extern __shared__ float pdf_lds[];
    const int lane = threadIdx.x;
    const int ray = blockIdx.x;
    if (ray >= a.n_rays) return;
    const int nb = a.S - 2;                     // N_samples_ - 2 bins
    float* cdf = pdf_lds;
    float* vals = pdf_lds + nb + 1;             // [coarse S | importance P]
    const float* w = a.weights + (size_t)ray * a.S + 1;
    for (int k = lane; k < nb; k += 64) cdf[k + 1] = w[k] + 1e-5f;   // :30
    __syncthreads();
    // torch.sum (:31) then torch.cumsum (:32); CPU cumsum accumulates in
    // double.  The two accumulations stay sequential (lane 0, the reference's
    // order); the divisions by the sum run on every lane.
    __shared__ float psum;
    if (lane == 0) {
        double tot = 0.0;
        for (int k = 0; k < nb; ++k) tot += (double)cdf[k + 1];
        psum = (float)tot;
    }
    __syncthreads();
    const float sum = psum;
    for (int k = lane; k < nb; k += 64) cdf[k + 1] = cdf[k + 1] / sum;
    __syncthreads();
    if (lane == 0) {
        double run = 0.0;
        cdf[0] = 0.f;
        for (int k = 0; k < nb; ++k) {
            run += (double)cdf[k + 1];
            cdf[k + 1] = (float)run;
        }
    }
    __syncthreads();
    const float near = a.rays[(size_t)ray * 8 + 6], far = a.rays[(size_t)ray * 8 + 7];
    const int I = a.I, S = a.S, SF = S + I, P = a.P;
    float* imp = vals + S;
    for (int j = lane; j < I; j += 64) {
        const int64_t idx = (int64_t)ray * I + j;
        const float u = a.u ? a.u[idx] : nr_rand_uniform(a.seed, 2, (uint64_t)idx);
        // searchsorted(cdf, u, side='right'): number of cdf entries <= u
        float ind = (float)count_below<true>(cdf, nb + 1, u) - 1.f;
        ind = ind < 0.f ? 0.f : ind;                                    // :39
        const float jt = a.jitter ? a.jitter[idx] : nr_rand_uniform(a.seed, 3, (uint64_t)idx);
        const float t = nr_add(ind, jt) / (float)nb;                    // :41
        const float zs = nr_add(nr_mul(near, 1.f - t), nr_mul(far, t)); // :45
        if (a.z_pdf) a.z_pdf[idx] = zs;
        imp[j] = zs;
    }
    if (!a.z_fine) return;
    for (int j = I + lane; j < P; j += 64) imp[j] = __builtin_inff();
    bool ok = true;
    for (int k = lane; k < S; k += 64) vals[k] = a.z_coarse[(size_t)ray * S + k];
    __syncthreads();
    for (int k = lane; k + 1 < S; k += 64) ok &= vals[k] <= vals[k + 1];
    float* out = a.z_fine + (size_t)ray * SF;
    // torch.sort of the values only: any sorting network gives the same
    // output.  Coarse depths ascending (they are by construction, :216-232):
    // bitonic sort of the importance depths, then a merge by binary searches
    // (coarse first on ties).
    if (__ballot(!ok) == 0) {
        for (int k = 2; k <= P; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int i = lane; i < P; i += 64) {
                    const int ixj = i ^ j;
                    if (ixj > i) {
                        const float x = imp[i], y = imp[ixj];
                        if ((x > y) == ((i & k) == 0)) { imp[i] = y; imp[ixj] = x; }
                    }
                }
                __syncthreads();
            }
        for (int i = lane; i < S; i += 64) {
            const float c = vals[i];
            out[i + count_below<false>(imp, I, c)] = c;
        }
        for (int j = lane; j < I; j += 64) {
            const float p = imp[j];
            out[j + count_below<true>(vals, S, p)] = p;
        }
        return;
    }
    // otherwise a rank sort (stable on ties): position = #smaller + #equal-before
    for (int i = lane; i < SF; i += 64) {
        const float v = vals[i];
        int rank = 0;
        for (int k = 0; k < SF; ++k) {
            const float o = vals[k];
            rank += (o < v) | ((o == v) & (k < i));
        }
        out[rank] = v;
    }
}

__global__ void pack_kernel(const float* __restrict__ flat, const int32_t* __restrict__ map,
                            int64_t n, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const int32_t m = map[i];
        out[i] = m >= 0 ? flat[m] : 0.f;
    }
}

}  // namespace

NR_API int nr_coarse_z(const float* rays, const float* tlin, int64_t n_rays, int n_samples,
                       int use_disp, float perturb, const float* u, uint64_t seed, float* z_out,
                       void* stream) {
    NR_REQUIRE(n_rays >= 0 && n_samples > 0, "nr_coarse_z: bad sizes");
    const int64_t n = n_rays * n_samples;
    if (n == 0) return 0;
    NR_REQUIRE(rays && tlin && z_out, "nr_coarse_z: null pointer");
    coarse_z_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        rays, tlin, (int)n_rays, n_samples, use_disp, perturb, u, seed, z_out);
    NR_LAUNCH_CHECK("nr_coarse_z");
    return 0;
}

NR_API int nr_composite_fwd(const float* raw, int raw_stride, int sig_col, const float* z,
                            const float* rays, const float* noise, float noise_std, uint64_t seed,
                            int rng_stream, int64_t n_rays, int n_samples, int white_back,
                            int weights_only, float* rgb, float* depth, float* opacity,
                            float* weights, void* stream) {
    NR_REQUIRE(n_rays >= 0 && n_samples > 0, "nr_composite_fwd: bad sizes");
    if (n_rays == 0) return 0;
    NR_REQUIRE(raw && z && rays && opacity && weights, "nr_composite_fwd: null pointer");
    NR_REQUIRE(weights_only || depth, "nr_composite_fwd: null depth");
    NR_REQUIRE(sig_col >= 0 && sig_col < raw_stride && (!rgb || raw_stride >= 4),
               "nr_composite_fwd: bad raw layout (stride %d, sigma column %d)", raw_stride,
               sig_col);
    CompArgs a{raw, raw_stride, sig_col, z, rays, noise, noise_std, seed, (uint32_t)rng_stream,
               (int)n_rays, n_samples, white_back, weights_only, rgb, depth, opacity, weights};
    const int wpb = 4;
    composite_fwd_kernel<<<(unsigned)((n_rays + wpb - 1) / wpb), 64 * wpb, 0,
                           (hipStream_t)stream>>>(a);
    NR_LAUNCH_CHECK("nr_composite_fwd");
    return 0;
}

NR_API int nr_composite_bwd(const float* raw, int raw_stride, int sig_col, const float* z,
                            const float* rays,
                            const float* noise, float noise_std, uint64_t seed, int rng_stream,
                            int64_t n_rays, int n_samples, int white_back, const float* g_rgb,
                            const float* g_depth, const float* g_opacity, float* g_raw,
                            void* stream) {
    NR_REQUIRE(n_rays >= 0 && n_samples > 0, "nr_composite_bwd: bad sizes");
    if (n_rays == 0) return 0;
    NR_REQUIRE(raw && z && rays && g_raw, "nr_composite_bwd: null pointer");
    NR_REQUIRE(raw_stride == 4 ? sig_col == 3 : (raw_stride == 1 && sig_col == 0),
               "nr_composite_bwd: raw rows must be [rgb, sigma] or [sigma]");
    NR_REQUIRE(raw_stride != 4 || ((uintptr_t)g_raw & 15) == 0,
               "nr_composite_bwd: g_raw must be 16-byte aligned");
    CompBwdArgs a{raw, raw_stride, sig_col, z, rays, noise, noise_std, seed, (uint32_t)rng_stream, (int)n_rays,
                  n_samples, white_back, g_rgb, g_depth, g_opacity, g_raw};
    const int wpb = 4;
    composite_bwd_kernel<<<(unsigned)((n_rays + wpb - 1) / wpb), 64 * wpb, 0,
                           (hipStream_t)stream>>>(a);
    NR_LAUNCH_CHECK("nr_composite_bwd");
    return 0;
}

NR_API int nr_sample_pdf(const float* weights, int n_samples, const float* rays,
                         const float* z_coarse, const float* u, const float* jitter, uint64_t seed,
                         int64_t n_rays, int n_importance, float* z_pdf, float* z_fine,
                         void* stream) {
    NR_REQUIRE(n_rays >= 0 && n_importance >= 0, "nr_sample_pdf: bad sizes");
    NR_REQUIRE(n_samples >= 3 && n_samples - 2 <= kPdfMaxBins,
               "nr_sample_pdf: n_samples=%d must be in [3, %d]", n_samples, kPdfMaxBins + 2);
    NR_REQUIRE(!z_fine || n_samples + n_importance <= kMergeMax,
               "nr_sample_pdf: n_samples+n_importance=%d exceeds %d", n_samples + n_importance,
               kMergeMax);
    NR_REQUIRE(n_importance <= kMergeMax - n_samples, "nr_sample_pdf: n_importance too large");
    if (n_rays == 0 || n_importance == 0) return 0;
    NR_REQUIRE(weights && rays && (z_pdf || z_fine), "nr_sample_pdf: null pointer");
    NR_REQUIRE(!z_fine || z_coarse, "nr_sample_pdf: z_fine needs z_coarse");
    int P = 1;
    while (P < n_importance) P <<= 1;
    PdfArgs a{weights, n_samples, rays, z_coarse, u, jitter, seed, (int)n_rays, n_importance, P,
              z_pdf, z_fine};
    const size_t lds = sizeof(float) * (size_t)(n_samples - 1 + n_samples + P);
    sample_pdf_kernel<<<(unsigned)n_rays, 64, lds, (hipStream_t)stream>>>(a);
    NR_LAUNCH_CHECK("nr_sample_pdf");
    return 0;
}

NR_API int nr_pack(const float* flat, const int32_t* map, int64_t n, float* out, void* stream) {
    NR_REQUIRE(n >= 0, "nr_pack: bad size");
    if (n == 0) return 0;
    NR_REQUIRE(flat && map && out, "nr_pack: null pointer");
    pack_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(flat, map, n, out);
    NR_LAUNCH_CHECK("nr_pack");
    return 0;
}

// ---------------------------------------------------------------------------
// Embedding.forward (models/nerf.py:21-38): out = [x, sin(2^0 x), cos(2^0 x), ...]
// ---------------------------------------------------------------------------
namespace {
__global__ void embed_kernel(const float* __restrict__ x, int64_t n, int nf,
                             float* __restrict__ out) {
    const int ch = 3 * (2 * nf + 1);
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * ch) return;
    const int64_t row = i / ch;
    const int c = (int)(i % ch);
    if (c < 3) { out[i] = x[row * 3 + c]; return; }
    const int q = c - 3, k = q / 6, rem = q % 6, comp = rem % 3;
    const float arg = x[row * 3 + comp] * (float)(1 << k);
    out[i] = rem < 3 ? sinf(arg) : cosf(arg);
}
}  // namespace

NR_API int nr_embed(const float* x, int64_t n, int n_freqs, float* out, void* stream) {
    NR_REQUIRE(n >= 0 && n_freqs >= 0 && n_freqs < 31, "nr_embed: bad sizes");
    const int64_t tot = n * 3 * (2 * n_freqs + 1);
    if (tot == 0) return 0;
    NR_REQUIRE(x && out, "nr_embed: null pointer");
    embed_kernel<<<(unsigned)((tot + 255) / 256), 256, 0, (hipStream_t)stream>>>(x, n, n_freqs, out);
    NR_LAUNCH_CHECK("nr_embed");
    return 0;
}
