// MLP backward, weight gradients: dW = sum_s dz[s]^T x[s] and db = sum_s dz[s]
// for every layer of NeRF (autograd of the nn.Linear layers, nerf.py:60-81).
//
// Grouped split-K GEMM on v_mfma_f32_32x32x2_f32.  Each of the 14 tasks
// (a gradient segment dz x an input segment x, both in the block-native layout
// of layout.h) is a <=256x256 output reduced over all samples.  Every task's
// sample blocks are split over G_t workgroups (G_t proportional to its cost,
// ~2 resident rounds in total).  A workgroup streams its blocks one 32-sample
// block per stage into LDS, transposing the block-native chunks to
// [sample][column] with ds_write_b128 (row stride 260: conflict-free), double
// buffered; its 4 waves split the task's output with a per-task wave grid so
// every SIMD holds MFMA work; k-step kk of a stage pairs samples 2kk and 2kk+1.
// Each workgroup writes one partial slab; a second kernel sums a task's slabs
// in a fixed order (bitwise reproducible) and scatters the result into the flat
// gradient buffer in NeRF.named_parameters() order.
#include <stdlib.h>

#include "layout.h"

namespace {

constexpr int kTasks = 14;
constexpr int kTargetWG = 760;   // ~3 rounds of one workgroup per CU (short tail)
constexpr int kThreads = 512;    // 8 waves: two per SIMD, so one wave's staging and
                                 // barrier time overlaps its partner's MFMAs
constexpr int kCol = 36;         // LDS column stride (floats): [column][32 samples + 4 pad]
constexpr int kBufA = 256 * kCol;  // one operand region
constexpr int kBuf = 2 * kBufA;    // one buffer = A + B regions

enum SegKind { SEG_ACC = 0, SEG_PE = 1, SEG_DPE = 2, SEG_HEAD = 3 };

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

struct WgSeg {
    const float* base;   // segment start (block-native)
    int kind, width;     // SegKind, columns
};

struct WgTask {
    WgSeg a, b;          // a = gradient (M = a.width), b = input (N = b.width)
    int wm, wn;          // wave grid (wm * wn == 4)
    int G;               // workgroups
    int64_t slab;        // slab offset (floats) of workgroup 0
    int id;              // task id: selects the gradient destination and the kernel shape
};

struct WgArgs {
    WgTask task[kTasks];
    int wg_start[kTasks + 1];
    int nb, n;
    float* slab;
};

// Staging geometry of one 32-sample block of a segment, all compile time:
// float4 e = tid + 512*i lands at LDS [sample j][column c].  In the
// block-native order float4 e is (t = e>>8, q = (e>>6)&3, lane = e&63).
template <int KIND, int W>
struct SegGeo {
    static constexpr int F4 = KIND == SEG_HEAD ? 32 : W * 8;     // float4 per block
    static constexpr int ITERS = (F4 + kThreads - 1) / kThreads;
    __device__ static __forceinline__ int j(int tid) { return KIND == SEG_HEAD ? tid : (tid & 31); }
    // column of float4 #i of thread tid
    __device__ static __forceinline__ int c(int tid, int i) {
        const int h = (tid >> 5) & 1, w = (tid >> 6) & 3, hi = tid >> 8;
        if constexpr (KIND == SEG_ACC) return 32 * (2 * i + hi) + 8 * w + 4 * h;   // t = 2i+hi, q = w
        else if constexpr (KIND == SEG_PE) return 32 * h + 4 * (8 * i + 4 * hi + w);  // gq = 8i+4hi+w
        else if constexpr (KIND == SEG_DPE) return 16 * h + 4 * w;               // gq = w (hi = 0)
        else return 0;
    }
};

template <int KA, int WA, int KB, int WB, int WM, int WN>
__device__ __forceinline__ void wgrad_body(const WgArgs& a, const WgTask& T, int b0, int b1,
                                           float* lds, float* __restrict__ slab) {
    using GA = SegGeo<KA, WA>;
    using GB = SegGeo<KB, WB>;
    constexpr int MT = (WA / WM + 31) / 32, NT = (WB / WN + 31) / 32;
    constexpr int M = WA, N = WB;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool active = wave < WM * WN;          // waves beyond the grid only stage
    const int mi = wave / WN, ni = wave % WN;
    const int m0 = 32 * MT * mi, n0 = 32 * NT * ni;
    const bool do_bias = active && ni == 0;

    f32x16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x16{};
    float bsum[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) bsum[i] = 0.f;

    // per-thread staging addresses: global float4 index tid + 256 i, LDS [j][c]
    const bool ta = tid < GA::F4, tb = tid < GB::F4;
    const int ja = GA::j(tid), jb = GB::j(tid);
    f32x4 ra[GA::ITERS], rb[GB::ITERS];
    auto load = [&](int blk) {
        const f32x4* pa = reinterpret_cast<const f32x4*>(T.a.base) + (size_t)blk * GA::F4 + tid;
        const f32x4* pb = reinterpret_cast<const f32x4*>(T.b.base) + (size_t)blk * GB::F4 + tid;
#pragma unroll
        for (int i = 0; i < GA::ITERS; ++i) if (ta) ra[i] = pa[kThreads * i];
#pragma unroll
        for (int i = 0; i < GB::ITERS; ++i) if (tb) rb[i] = pb[kThreads * i];
    };
    // write the staged block to LDS as [column][sample] (4 ds_write_b32 per
    // float4; lanes are consecutive samples -> conflict-free); samples >= n of
    // the tail block become 0
    auto store = [&](int buf, int blk) {
        const int nval = a.n - blk * 32;
        const bool ka = ja < nval, kb = jb < nval;
        float* la = lds + buf * kBuf + ja;
        float* lb = lds + buf * kBuf + kBufA + jb;
        if (ta)
#pragma unroll
            for (int i = 0; i < GA::ITERS; ++i) {
                const f32x4 v = ka ? ra[i] : f32x4{};
                const int c = GA::c(tid, i);
#pragma unroll
                for (int e = 0; e < 4; ++e) la[(c + e) * kCol] = v[e];
            }
        if (tb)
#pragma unroll
            for (int i = 0; i < GB::ITERS; ++i) {
                const f32x4 v = kb ? rb[i] : f32x4{};
                const int c = GB::c(tid, i);
#pragma unroll
                for (int e = 0; e < 4; ++e) lb[(c + e) * kCol] = v[e];
            }
    };

    const int nst = b1 - b0;
    if (nst > 0) {
        load(b0);
        store(0, b0);
    }
    __syncthreads();
    const int h = lane >> 5, col = lane & 31;
#pragma unroll 1
    for (int st = 0; st < nst; ++st) {
        const int buf = st & 1;
        if (st + 1 < nst) load(b0 + st + 1);
        // k-step kk pairs samples kk (lane half 0) and 16 + kk (half 1): a lane's
        // 16 samples of one column are contiguous -> 4 ds_read_b128 per column
        const float* la = lds + buf * kBuf + (m0 + col) * kCol + 16 * h;
        const float* lb = lds + buf * kBuf + kBufA + (n0 + col) * kCol + 16 * h;
        if (active) {
            f32x4 av[2][MT], bv[2][NT];
            auto rd = [&](int q, int p) {   // samples 4q..4q+3 of this lane half
#pragma unroll
                for (int i = 0; i < MT; ++i) av[p][i] = *reinterpret_cast<const f32x4*>(la + 32 * i * kCol + 4 * q);
#pragma unroll
                for (int j = 0; j < NT; ++j) bv[p][j] = *reinterpret_cast<const f32x4*>(lb + 32 * j * kCol + 4 * q);
            };
            auto mm = [&](int p) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
#pragma unroll
                    for (int i = 0; i < MT; ++i)
#pragma unroll
                        for (int j = 0; j < NT; ++j)
                            acc[i][j] = nr_mfma32(av[p][i][e], bv[p][j][e], acc[i][j]);
#pragma unroll
                    for (int i = 0; i < MT; ++i) bsum[i] += av[p][i][e];
                }
            };
            rd(0, 0);
            rd(1, 1);
            __builtin_amdgcn_sched_barrier(0);
            mm(0);
            rd(2, 0);
            __builtin_amdgcn_sched_barrier(0);
            mm(1);
            rd(3, 1);
            __builtin_amdgcn_sched_barrier(0);
            mm(0);
            __builtin_amdgcn_sched_barrier(0);
            mm(1);
        }
        if (st + 1 < nst) store(buf ^ 1, b0 + st + 1);
        __syncthreads();
    }
    if (!active) return;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int o = m0 + 32 * i + nr_acc_row(r, h);
                const int c = n0 + 32 * j + col;
                if (o < M && c < N) slab[o * N + c] = acc[i][j][r];
            }
        if (do_bias) {
            const float b = bsum[i] + __shfl_xor(bsum[i], 32);
            const int o = m0 + 32 * i + col;
            if (h == 0 && o < M) slab[M * N + o] = b;
        }
    }
}

__global__ void __launch_bounds__(kThreads, 2) wgrad_kernel(WgArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[2 * kBuf];   // 144 KiB
    int t = 0;
#pragma unroll 1
    while (t + 1 < kTasks && (int)blockIdx.x >= a.wg_start[t + 1]) ++t;
    const WgTask& T = a.task[t];
    const int c = blockIdx.x - a.wg_start[t];
    const int b0 = (int)((int64_t)c * a.nb / T.G);
    const int b1 = (int)((int64_t)(c + 1) * a.nb / T.G);
    float* slab = a.slab + T.slab + (int64_t)c * (T.a.width * T.b.width + T.a.width);
    // task shapes (see nr_wgrad's task list); wave-uniform
    // (WM, WN) = wave grid over the task's output (<= 8 waves; 128 accumulators max)
    switch (__builtin_amdgcn_readfirstlane(T.id)) {
        case 0: case 4:
            wgrad_body<SEG_ACC, 256, SEG_PE, 64, 8, 1>(a, T, b0, b1, lds, slab); break;
        case 10:
            wgrad_body<SEG_ACC, 128, SEG_ACC, 256, 2, 4>(a, T, b0, b1, lds, slab); break;
        case 11:
            wgrad_body<SEG_ACC, 128, SEG_DPE, 32, 4, 1>(a, T, b0, b1, lds, slab); break;
        case 12:
            wgrad_body<SEG_HEAD, 4, SEG_ACC, 256, 1, 8>(a, T, b0, b1, lds, slab); break;
        case 13:
            wgrad_body<SEG_HEAD, 4, SEG_ACC, 128, 1, 4>(a, T, b0, b1, lds, slab); break;
        default:
            wgrad_body<SEG_ACC, 256, SEG_ACC, 256, 2, 4>(a, T, b0, b1, lds, slab); break;
    }
}

// destination of output element (o, c) of task t in the flat gradient (-1 = none)
__device__ int wgrad_dest(int t, int o, int c) {
    switch (t) {
        case 0: { const int f = pe_feature(c & 31, c >> 5, 15);
                  return f < 0 ? -1 : kP.w[0] + o * kP.fan[0] + f; }
        case 1: case 2: case 3: return kP.w[t] + o * kP.fan[t] + c;
        case 4: { const int f = pe_feature(c & 31, c >> 5, 15);
                  return f < 0 ? -1 : kP.w[4] + o * kP.fan[4] + f; }
        case 5: return kP.w[4] + o * kP.fan[4] + NR_XYZ_CH + c;
        case 6: case 7: case 8: case 9: return kP.w[t - 1] + o * kP.fan[t - 1] + c;
        case 10: return kP.w[9] + o * kP.fan[9] + c;
        case 11: { const int f = pe_feature(c & 15, c >> 4, 6);
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
    const WgTask& T = a.task[t];
    const int M = T.a.width, N = T.b.width;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    const int nw = M * N, sz = nw + M;
    if (e >= sz) return;
    const int dst = e < nw ? wgrad_dest(T.id, e / N, e % N) : wgrad_bias_dest(T.id, e - nw);
    if (dst < 0) return;
    const float* p = a.slab + T.slab + e;
    float s = 0.f;
    for (int w = 0; w < T.G; ++w, p += sz) s += *p;
    grad[dst] = s;
}

}  // namespace

NR_API int64_t nr_wgrad_workspace_bytes(int64_t n) {
    (void)n;
    // upper bound of sum_t G_t * (M_t N_t + M_t) for the task list below
    return (int64_t)(3 * kTargetWG + kTasks) * (256 * 256 + 256) * sizeof(float);
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
    const int64_t nb = (n + 31) / 32;
    float* SV = const_cast<float*>(save);
    float* GD = const_cast<float*>(grad_ws);
    auto acc = [](float* p, int w) { return WgSeg{p, SEG_ACC, w}; };
    const WgSeg pe{SV, SEG_PE, 64}, dpe{SV + nr_sv_dirpe(nb), SEG_DPE, 32};
    const WgSeg head{GD + nr_gd_dhead(nb), SEG_HEAD, 4};
    auto H = [&](int l) { return acc(SV + nr_sv_h(l, nb), 256); };
    auto DZ = [&](int l) { return acc(GD + nr_gd_dz(l, nb), 256); };
    const WgSeg feat = acc(SV + nr_sv_feat(nb), 256), hdir = acc(SV + nr_sv_hdir(nb), 128);
    const WgSeg dzdir = acc(GD + nr_gd_dzdir(nb), 128);
    // (a, b, wm, wn); task order fixes wgrad_dest / wgrad_bias_dest
    const WgTask tasks[kTasks] = {
        {DZ(0), pe, 8, 1}, {DZ(1), H(0), 2, 4}, {DZ(2), H(1), 2, 4}, {DZ(3), H(2), 2, 4},
        {DZ(4), pe, 8, 1}, {DZ(4), H(3), 2, 4}, {DZ(5), H(4), 2, 4}, {DZ(6), H(5), 2, 4},
        {DZ(7), H(6), 2, 4}, {DZ(8), H(7), 2, 4}, {dzdir, feat, 2, 4}, {dzdir, dpe, 4, 1},
        {head, H(7), 1, 8}, {head, hdir, 1, 4},
    };
    WgArgs a{};
    // per-block cost of a task's workgroup, in cycles: the MFMA time of its
    // busiest SIMD, or the staging of (M + N) x 32 floats at ~8 B/cycle per CU,
    // plus a fixed barrier/LDS-store overhead
    int64_t cost[kTasks], tot = 0;
    for (int t = 0; t < kTasks; ++t) {
        const int mt = (tasks[t].a.width / tasks[t].wm + 31) / 32;
        const int nt = (tasks[t].b.width / tasks[t].wn + 31) / 32;
        const int64_t mfma = 16 * mt * nt * 64 * (tasks[t].wm * tasks[t].wn > 4 ? 2 : 1);
        const int64_t bytes = (int64_t)(tasks[t].a.width + tasks[t].b.width) * 32 * 4;
        cost[t] = std::max<int64_t>(mfma, bytes / 8) + 512;
        tot += cost[t];
    }
    // dispatch order: the heavy 256x256 tasks first; the small, memory-bound
    // tasks last and split ~3x finer, so their short workgroups fill the tail
    // of the final round
    int order[kTasks], no = 0;
    for (int pass = 0; pass < 2; ++pass)
        for (int t = 0; t < kTasks; ++t)
            if ((cost[t] >= 16384) == (pass == 0)) order[no++] = t;
    a.wg_start[0] = 0;
    int64_t slab = 0;
    // diagnostic: NR_WGRAD_TASKMASK limits the launch to a subset of task ids
    // (the kernel code is unchanged; gradients of the other tasks are then stale)
    static const long long tmask =
        getenv("NR_WGRAD_TASKMASK") ? strtoll(getenv("NR_WGRAD_TASKMASK"), nullptr, 0) : -1;
    for (int k = 0; k < kTasks; ++k) {
        const int t = order[k];
        const int split = cost[t] >= 16384 ? 1 : 3;
        int64_t g = split * ((kTargetWG * cost[t] + tot - 1) / tot);
        g = std::max<int64_t>(1, std::min<int64_t>(g, nb));
        if (!((tmask >> t) & 1)) g = 0;
        a.task[k] = tasks[t];
        a.task[k].id = t;
        a.task[k].G = (int)g;
        a.task[k].slab = slab;
        slab += g * (tasks[t].a.width * tasks[t].b.width + tasks[t].a.width);
        a.wg_start[k + 1] = a.wg_start[k] + (int)g;
    }
    a.nb = (int)nb;
    a.n = (int)n;
    a.slab = workspace;
    wgrad_kernel<<<a.wg_start[kTasks], kThreads, 0, st>>>(a);
    NR_LAUNCH_CHECK("nr_wgrad");
    dim3 rg((256 * 256 + 256 + 255) / 256, kTasks);
    wgrad_reduce_kernel<<<rg, 256, 0, st>>>(a, grad_flat);
    NR_LAUNCH_CHECK("nr_wgrad_reduce");
    return 0;
}
