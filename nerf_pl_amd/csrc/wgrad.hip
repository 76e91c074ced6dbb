// MLP backward, weight gradients: dW = sum_s dz[s]^T x[s] and db = sum_s dz[s]
// for every layer of NeRF (autograd of the nn.Linear layers, nerf.py:60-81).
//
// Grouped split-K GEMM on v_mfma_f32_32x32x2_f32.  Each of the 14 tasks
// (dz segment x input segment, both row-major [n][width] as written by
// mlp_fwd/mlp_bwd) is a <=256x256 output tile reduced over all n samples.  The
// sample axis is split over the workgroups of a single, fully resident round
// (grid <= 256 = one workgroup per CU), each task getting workgroups in
// proportion to its cost.  A workgroup stages 16-sample slices of dz and x in
// LDS (double buffered, coalesced float4 loads), its 4 waves each own a
// 128x128 quadrant of the output, and it writes a partial slab; a second
// kernel sums the slabs of each task in a fixed order (bitwise reproducible)
// and scatters the result into the flat gradient buffer in
// NeRF.named_parameters() order.
#include "layout.h"

namespace {

constexpr int kTasks = 14;
constexpr int kMaxWG = 256;
constexpr int kSlab = 256 * 256 + 256;   // partial dW tile + partial bias
constexpr int kTS = 16;                  // samples per LDS stage

// flat parameter offsets, NeRF.named_parameters() order (packing.py param_offsets)
struct POff {
    int w[12], b[12], fan[12];
};
constexpr POff make_poff() {
    POff p{};
    const int rows[12] = {256, 256, 256, 256, 256, 256, 256, 256, 256, 128, 1, 3};
    const int fans[12] = {63, 256, 256, 256, 319, 256, 256, 256, 256, 283, 256, 128};
    int o = 0;
    for (int i = 0; i < 12; ++i) {
        p.w[i] = o;
        p.fan[i] = fans[i];
        o += rows[i] * fans[i];
        p.b[i] = o;
        o += rows[i];
    }
    return p;
}
constexpr POff kP = make_poff();
static_assert(kP.b[11] + 3 == 595844, "parameter count");
// layer ids: 0..7 = xyz_encoding_1..8, 8 = final, 9 = dir, 10 = sigma, 11 = rgb

__device__ __forceinline__ int pe_feature(int g, int h, int np) {
    if (g == 0) return h;
    if (g == 1) return h == 0 ? 2 : -1;
    if (g < 2 + np) { const int m = g - 2 + np * h; return 3 + 6 * (m / 3) + m % 3; }
    if (g < 2 + 2 * np) { const int m = g - 2 - np + np * h; return 6 + 6 * (m / 3) + m % 3; }
    return -1;
}

struct WgTask {
    const float* dz; const float* x;
    int dz_stride, x_stride, M, N;
};

struct WgArgs {
    WgTask task[kTasks];
    int wg_start[kTasks + 1];
    int n;
    float* slab;
};

__device__ __forceinline__ int log2i(int v) { return 31 - __clz(v); }

// Main loop of one workgroup; MT x NT = this wave's 32x32 tiles (compile
// time, so accumulators stay in registers without per-MFMA branches).  Every
// wave runs the same number of stages and barriers whatever its MT/NT.
template <int MT, int NT>
__device__ __forceinline__ void wgrad_body(const WgTask& T, int s0, int s1, int m0, int n0,
                                           bool do_bias, float (*lds)[2][kTS][256],
                                           float* __restrict__ slab) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int M4 = T.M >> 2, N4 = T.N >> 2;        // float4s per row (powers of 2)
    const int lm = log2i(M4), ln = log2i(N4);
    f32x16 acc[MT > 0 ? MT : 1][NT > 0 ? NT : 1];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x16{};
    float bsum[MT > 0 ? MT : 1];
#pragma unroll
    for (int i = 0; i < MT; ++i) bsum[i] = 0.f;

    f32x4 ra[4], rb[4];
    auto load = [&](int s) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = tid + 256 * i;
            ra[i] = f32x4{};
            rb[i] = f32x4{};
            if (e < (kTS << lm)) {
                const int r = e >> lm, q = e & (M4 - 1);
                if (s + r < s1)
                    ra[i] = *reinterpret_cast<const f32x4*>(T.dz + (size_t)(s + r) * T.dz_stride + 4 * q);
            }
            if (e < (kTS << ln)) {
                const int r = e >> ln, q = e & (N4 - 1);
                if (s + r < s1)
                    rb[i] = *reinterpret_cast<const f32x4*>(T.x + (size_t)(s + r) * T.x_stride + 4 * q);
            }
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = tid + 256 * i;
            if (e < (kTS << lm))
                *reinterpret_cast<f32x4*>(&lds[buf][0][e >> lm][4 * (e & (M4 - 1))]) = ra[i];
            if (e < (kTS << ln))
                *reinterpret_cast<f32x4*>(&lds[buf][1][e >> ln][4 * (e & (N4 - 1))]) = rb[i];
        }
    };

    const int nst = (s1 - s0 + kTS - 1) / kTS;
    if (nst > 0) {
        load(s0);
        store(0);
    }
    __syncthreads();
    const int h = lane >> 5, col = lane & 31;
#pragma unroll 1
    for (int st = 0; st < nst; ++st) {
        const int buf = st & 1;
        if (st + 1 < nst) load(s0 + (st + 1) * kTS);
        if constexpr (MT > 0 && NT > 0) {
#pragma unroll
            for (int kk = 0; kk < kTS / 2; ++kk) {
                const float* ar = &lds[buf][0][2 * kk + h][0];
                const float* br = &lds[buf][1][2 * kk + h][0];
                float av[MT], bv[NT];
#pragma unroll
                for (int i = 0; i < MT; ++i) av[i] = ar[m0 + 32 * i + col];
#pragma unroll
                for (int j = 0; j < NT; ++j) bv[j] = br[n0 + 32 * j + col];
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j) acc[i][j] = nr_mfma32(av[i], bv[j], acc[i][j]);
                if (do_bias)
#pragma unroll
                    for (int i = 0; i < MT; ++i) bsum[i] += av[i];
            }
        }
        if (st + 1 < nst) store(buf ^ 1);
        __syncthreads();
    }
    if constexpr (MT > 0 && NT > 0) {
#pragma unroll
        for (int i = 0; i < MT; ++i) {
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int o = m0 + 32 * i + nr_acc_row(r, h);
                    slab[o * 256 + n0 + 32 * j + col] = acc[i][j][r];
                }
            if (do_bias) {
                const float b = bsum[i] + __shfl_xor(bsum[i], 32);
                if (h == 0) slab[256 * 256 + m0 + 32 * i + col] = b;
            }
        }
    }
}

__global__ void __launch_bounds__(256, 1) wgrad_kernel(WgArgs a) {
    __shared__ float lds[2][2][kTS][256];   // [buf][A|B][sample][col]  64 KiB
    int t = 0;
#pragma unroll 1
    while (t + 1 < kTasks && (int)blockIdx.x >= a.wg_start[t + 1]) ++t;
    const WgTask T = a.task[t];
    const int G = a.wg_start[t + 1] - a.wg_start[t];
    const int c = blockIdx.x - a.wg_start[t];
    const int nblk = (a.n + kTS - 1) / kTS;
    const int s0 = (int)((int64_t)c * nblk / G) * kTS;
    const int s1 = min((int)((int64_t)(c + 1) * nblk / G) * kTS, a.n);
    const int wave = threadIdx.x >> 6;
    const int m0 = 128 * (wave >> 1), n0 = 128 * (wave & 1);
    const int mtc = max(0, min(4, (T.M - m0 + 31) / 32));
    const int ntc = max(0, min(4, (T.N - n0 + 31) / 32));
    const bool do_bias = (wave & 1) == 0;
    float* slab = a.slab + (size_t)blockIdx.x * kSlab;
    // wave-uniform dispatch on this wave's tile counts (the shapes of the 14 tasks)
    const int key = __builtin_amdgcn_readfirstlane(mtc * 8 + ntc);
    switch (key) {
        case 4 * 8 + 4: wgrad_body<4, 4>(T, s0, s1, m0, n0, do_bias, lds, slab); break;
        case 4 * 8 + 2: wgrad_body<4, 2>(T, s0, s1, m0, n0, do_bias, lds, slab); break;
        case 4 * 8 + 1: wgrad_body<4, 1>(T, s0, s1, m0, n0, do_bias, lds, slab); break;
        case 1 * 8 + 4: wgrad_body<1, 4>(T, s0, s1, m0, n0, do_bias, lds, slab); break;
        default: wgrad_body<0, 0>(T, s0, s1, m0, n0, do_bias, lds, slab); break;
    }
}

// destination of output element (o, c) of task t in the flat gradient (-1 = none)
__device__ int wgrad_dest(int t, int o, int c) {
    switch (t) {
        case 0: { const int f = pe_feature(c >> 1, c & 1, 15);
                  return f < 0 ? -1 : kP.w[0] + o * kP.fan[0] + f; }
        case 1: case 2: case 3: return kP.w[t] + o * kP.fan[t] + c;
        case 4: { const int f = pe_feature(c >> 1, c & 1, 15);
                  return f < 0 ? -1 : kP.w[4] + o * kP.fan[4] + f; }
        case 5: return kP.w[4] + o * kP.fan[4] + NR_XYZ_CH + c;
        case 6: case 7: case 8: case 9: return kP.w[t - 1] + o * kP.fan[t - 1] + c;
        case 10: return kP.w[9] + o * kP.fan[9] + c;
        case 11: { const int f = pe_feature(c >> 1, c & 1, 6);
                   return f < 0 ? -1 : kP.w[9] + o * kP.fan[9] + 256 + f; }
        case 12: return o == 3 ? kP.w[10] + c : -1;
        case 13: return o < 3 ? kP.w[11] + o * kP.fan[11] + c : -1;
    }
    return -1;
}

__device__ int wgrad_bias_dest(int t, int o) {
    switch (t) {
        case 0: return kP.b[0] + o;
        case 1: case 2: case 3: return kP.b[t] + o;
        case 4: return kP.b[4] + o;
        case 6: case 7: case 8: case 9: return kP.b[t - 1] + o;
        case 10: return kP.b[9] + o;
        case 12: return o == 3 ? kP.b[10] : kP.b[11] + o;
    }
    return -1;
}

__global__ void wgrad_reduce_kernel(WgArgs a, float* __restrict__ grad) {
    const int t = blockIdx.y;
    const WgTask T = a.task[t];
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    const int nw = T.M * T.N;
    if (e >= nw + T.M) return;
    int off, dst;
    if (e < nw) {
        const int o = e / T.N, c = e % T.N;
        off = o * 256 + c;
        dst = wgrad_dest(t, o, c);
    } else {
        const int o = e - nw;
        off = 256 * 256 + o;
        dst = wgrad_bias_dest(t, o);
    }
    if (dst < 0) return;
    const float* p = a.slab + (size_t)a.wg_start[t] * kSlab + off;
    float s = 0.f;
    for (int w = a.wg_start[t]; w < a.wg_start[t + 1]; ++w, p += kSlab) s += *p;
    grad[dst] = s;
}

// per-sample cost of a task for its busiest wave (MFMA tile pairs)
int task_cost(int M, int N) {
    int best = 0;
    for (int w = 0; w < 4; ++w) {
        const int m0 = 128 * (w >> 1), n0 = 128 * (w & 1);
        const int mt = std::max(0, std::min(4, (M - m0 + 31) / 32));
        const int nt = std::max(0, std::min(4, (N - n0 + 31) / 32));
        best = std::max(best, mt * nt);
    }
    return best;
}

}  // namespace

NR_API int64_t nr_wgrad_workspace_bytes(int64_t n) {
    (void)n;
    return (int64_t)kMaxWG * kSlab * sizeof(float);
}

NR_API int nr_wgrad(const float* save, const float* grad_ws, int64_t n, float* workspace,
                    float* grad_flat, void* stream) {
    NR_REQUIRE(n >= 0 && n < (int64_t)1 << 31, "nr_wgrad: n out of range");
    NR_REQUIRE(save && grad_ws && workspace && grad_flat, "nr_wgrad: null pointer");
    NR_REQUIRE((((uintptr_t)save | (uintptr_t)grad_ws) & 15) == 0,
               "nr_wgrad: save/grad_ws must be 16-byte aligned");
    hipStream_t st = (hipStream_t)stream;
    if (n == 0) {
        hipError_t e = hipMemsetAsync(grad_flat, 0, 595844 * sizeof(float), st);
        if (e != hipSuccess) { nr_set_error("nr_wgrad: memset failed"); return (int)e; }
        return 0;
    }
    NrSave sv(const_cast<float*>(save), n);
    NrGrad gd(const_cast<float*>(grad_ws), n);
    WgArgs a{};
    const WgTask tasks[kTasks] = {
        {gd.dz[0], sv.pe, 256, 64, 256, 64},
        {gd.dz[1], sv.h[0], 256, 256, 256, 256},
        {gd.dz[2], sv.h[1], 256, 256, 256, 256},
        {gd.dz[3], sv.h[2], 256, 256, 256, 256},
        {gd.dz[4], sv.pe, 256, 64, 256, 64},
        {gd.dz[4], sv.h[3], 256, 256, 256, 256},
        {gd.dz[5], sv.h[4], 256, 256, 256, 256},
        {gd.dz[6], sv.h[5], 256, 256, 256, 256},
        {gd.dz[7], sv.h[6], 256, 256, 256, 256},
        {gd.dfeat, sv.h[7], 256, 256, 256, 256},
        {gd.dzdir, sv.feat, 128, 256, 128, 256},
        {gd.dzdir, sv.dirpe, 128, 32, 128, 32},
        {gd.dhead, sv.h[7], 4, 256, 4, 256},
        {gd.dhead, sv.hdir, 4, 128, 4, 128},
    };
    int cost[kTasks], tot = 0;
    for (int t = 0; t < kTasks; ++t) {
        a.task[t] = tasks[t];
        cost[t] = task_cost(tasks[t].M, tasks[t].N);
        tot += cost[t];
    }
    // one resident round: floor share of 256 workgroups, at least one each,
    // and no more workgroups than 16-sample stages
    const int nblk = (int)((n + kTS - 1) / kTS);
    a.wg_start[0] = 0;
    for (int t = 0; t < kTasks; ++t) {
        int g = std::max(1, (kMaxWG - kTasks) * cost[t] / tot);
        g = std::min(g, nblk);
        a.wg_start[t + 1] = a.wg_start[t] + g;
    }
    a.n = (int)n;
    a.slab = workspace;
    const int nwg = a.wg_start[kTasks];
    wgrad_kernel<<<nwg, 256, 0, st>>>(a);
    NR_LAUNCH_CHECK("nr_wgrad");
    dim3 rg((256 * 256 + 256 + 255) / 256, kTasks);
    wgrad_reduce_kernel<<<rg, 256, 0, st>>>(a, grad_flat);
    NR_LAUNCH_CHECK("nr_wgrad_reduce");
    return 0;
}
