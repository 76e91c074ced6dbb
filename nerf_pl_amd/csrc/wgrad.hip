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

#include <type_traits>

#include "x3.h"

namespace {

constexpr int kTasks = 14;
#ifndef NR_WGRAD_TARGET_WG
#define NR_WGRAD_TARGET_WG 760
#endif
constexpr int kTargetWG = NR_WGRAD_TARGET_WG;   // ~3 rounds of one workgroup per CU (short tail)
// the gathering kernels (a sample list, gathered inputs): 1024 measured 1.5%
// faster than 760 at cfg2's fine pass (three alternating rounds, profiles/r04/abalt_tw)
#ifndef NR_WGRAD_TARGET_WG_GA
#define NR_WGRAD_TARGET_WG_GA 1024
#endif
// the LDS-DMA kernel (wgrad4_kernel, one workgroup per CU) over a sample list:
// 1536 measured 3% faster than 1024 (768: +0.5%, 2048: -1.5%) at cfg2's fine
// pass (two alternating rounds, profiles/r05/ab/u_*)
#ifndef NR_WGRAD_TARGET_WG_W4
#define NR_WGRAD_TARGET_WG_W4 1536
#endif
constexpr int kMax2(int x, int y) { return x > y ? x : y; }
[[maybe_unused]] constexpr int kTargetWGMax =
    kMax2(kMax2(NR_WGRAD_TARGET_WG, NR_WGRAD_TARGET_WG_GA), NR_WGRAD_TARGET_WG_W4);
constexpr int kThreads = 512;    // 8 waves: two per SIMD, so one wave's staging and
                                 // barrier time overlaps its partner's MFMAs
constexpr int kCol = 36;         // LDS column stride (floats): [column][32 samples + 4 pad]
constexpr int kBufA = 256 * kCol;  // one operand region
[[maybe_unused]] constexpr int kBuf = 2 * kBufA;    // one buffer = A + B regions

enum SegKind { SEG_ACC = 0, SEG_PE = 1, SEG_DPE = 2, SEG_HEAD = 3 };

// f16x3: the task pairs that read the same saved segment (wgrad_launch:
// DZ(4), H(7), dz_dir) run fused -- one workgroup stages the shared segment
// once and computes both outputs.  Runtime switch NR_WGRAD_FUSE=0 (host).
constexpr bool kFuse = NR_F16 || NR_BF1;
#ifndef NR_WG_PE_WM
#define NR_WG_PE_WM 4            // wave grid rows of the fused PE output (256 x 64)
#endif
#ifndef NR_WGRAD_FUSE_MASK
// bit i: pair i of wgrad_launch's kFused (f16x3 6: no spills, measured slower)
#define NR_WGRAD_FUSE_MASK 7
#endif
// the same for the gathering kernels (the *_active entry points): the fused
// PE pair (bit 0) leaves wgrad3_kernel<true, ROWS> 33 spilled VGPRs (8
// without it), and unfused its fine-pass launch runs 1.97 -> 1.83 ms
// (three alternating same-box rounds, profiles/r04/abalt_fuse6)
#ifndef NR_WGRAD_FUSE_MASK_GA
#define NR_WGRAD_FUSE_MASK_GA 6
#endif

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
    int stat;            // f16x3: stats slot of the gradient operand (layout.h NR_STATS)
    int fuse;            // f16x3: index (in WgArgs::task) of the task whose output this task's
                         // workgroups also compute (same block ranges, its own slab), or -1
    int pa, pb;          // slab row / column order (wgrad4_kernel): 1 natural; V: each
                         // 32V-wide chunk holds its V interleaved MFMA tiles one after
                         // another (w4_unperm)
};

struct WgArgs {
    WgTask task[kTasks];
    int wg_start[kTasks + 1];
    int nb, n;
    float* slab;
    bool x3;             // segments in the bf16x6 pipeline's N16 layout (x3.h)
    const float* stats;  // f16x3: max |gradient| per segment (mlp_bwd3.hip), else null
    // optional (active.hip, split arithmetics' wgrad3_body only): the ascending
    // list of the samples with a nonzero output gradient and its length m on
    // the device.  The gradient segments (mlp_bwd3.hip *_active) then hold
    // position q's rows at q; the split-K ranges cover the ceil(m / 32) blocks
    // of positions, and the input operands are gathered from sample slist[q]
    const int32_t* slist; const int32_t* scount;
};

// samples (positions) a launch works on
__device__ __forceinline__ int wg_m(const WgArgs& a) {
    return a.slist ? __builtin_amdgcn_readfirstlane(*a.scount) : a.n;
}
// blocks of positions a launch's split-K ranges cover
__device__ __forceinline__ int wg_nact(const WgArgs& a) {
    return a.slist ? (wg_m(a) + 31) / 32 : a.nb;
}

// f16x3: the gradient operand of a task is scaled by 2^(kWT - e(max |dz|)) so
// its largest element sits in [2^kWT, 2^(kWT+1)) < 65504; the input operand
// (activations, |x| < 65504) is split unscaled.  The reduction divides the
// weight part of the slab sums by the same power of two (bias sums come from
// the unscaled values).
__device__ __forceinline__ float task_scale(const WgArgs& a, const WgTask& T) {
#if NR_F16
    constexpr int kWT = 14;
    return x3::pow2_norm(a.stats[T.stat], kWT, 126);
#else
    (void)a; (void)T;
    return 1.f;
#endif
}

#if NR_X3_BASE_OBJECT   // the fp32-MFMA kernel lives in the bf16x6 object only
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

// ROWS staging geometry of an input segment (sample-major rows of W): float4
// e = tid + 512 i is chunk (e & 3) + 4 (e >> 7) of sample (e >> 2) & 31, so a
// wave instruction reads 16 rows x 64 contiguous bytes (not 32 rows x 32 B)
// while the [column][sample] image writes stay at most 2-way bank conflicted
// (free for ds_write_b32); a thread's sample is the same in every iteration
template <int KIND, int W>
struct RowGeo {
    static constexpr int F4 = W * 8;
    static constexpr int ITERS = (F4 + kThreads - 1) / kThreads;
    __device__ static __forceinline__ int j(int tid) { return (tid >> 2) & 31; }
    __device__ static __forceinline__ int c(int tid, int i) {
        return 4 * ((tid & 3) + 4 * ((tid + kThreads * i) >> 7));
    }
};

// GAT: over the packed sample list (the fp32 *_active entry points): the
// gradient operand is read by position, the input operand gathered, each
// thread resolving one sample per stage; positions past m stage zeros.
// ROWS: the input operand saved as sample-major rows (mlp_fwd.hip, the full
// graph): the float4 of column c of sample s is row s at c -- a gathered
// sample's 128-B lines are read whole, and the same thread -> (sample,
// column) mapping keeps the LDS image writes conflict-free.  Else
// block-native: the float4 sits at (s >> 5) * F4 + (e & ~31) + (s & 31).
template <int KA, int WA, int KB, int WB, int WM, int WN, bool GAT = false, bool ROWS = false>
__device__ __forceinline__ void wgrad_body(const WgArgs& a, const WgTask& T, int b0, int b1,
                                           float* lds, float* __restrict__ slab) {
    using GA = SegGeo<KA, WA>;
    using GB = std::conditional_t<ROWS && KB != SEG_HEAD, RowGeo<KB, WB>, SegGeo<KB, WB>>;
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
    const int m = wg_m(a);
    auto load = [&](int blk) {
        const f32x4* pa = reinterpret_cast<const f32x4*>(T.a.base) + (size_t)blk * GA::F4 + tid;
        const f32x4* pb;
        if constexpr (ROWS) {
            const int sj = GAT ? a.slist[min(blk * 32 + jb, m - 1)] : blk * 32 + jb;
            const float* row = T.b.base + (size_t)sj * WB;
#pragma unroll
            for (int i = 0; i < GA::ITERS; ++i) if (ta) ra[i] = pa[kThreads * i];
#pragma unroll
            for (int i = 0; i < GB::ITERS; ++i)
                if (tb) rb[i] = *reinterpret_cast<const f32x4*>(row + GB::c(tid, i));
            return;
        } else if constexpr (GAT) {
            const int sj = a.slist[min(blk * 32 + jb, m - 1)];
            pb = reinterpret_cast<const f32x4*>(T.b.base) + (size_t)(sj >> 5) * GB::F4 +
                 (tid - jb) + (sj & 31);
        } else {
            pb = reinterpret_cast<const f32x4*>(T.b.base) + (size_t)blk * GB::F4 + tid;
        }
#pragma unroll
        for (int i = 0; i < GA::ITERS; ++i) if (ta) ra[i] = pa[kThreads * i];
#pragma unroll
        for (int i = 0; i < GB::ITERS; ++i) if (tb) rb[i] = pb[kThreads * i];
    };
    // write the staged block to LDS as [column][sample] (4 ds_write_b32 per
    // float4; lanes are consecutive samples -> conflict-free); samples >= n of
    // the tail block become 0
    auto store = [&](int buf, int blk) {
        const int nval = m - blk * 32;
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

template <bool GA, bool ROWS>
__global__ void __launch_bounds__(kThreads, 2) wgrad_kernel(WgArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[2 * kBuf];   // 144 KiB
    int t = 0;
#pragma unroll 1
    while (t + 1 < kTasks && (int)blockIdx.x >= a.wg_start[t + 1]) ++t;
    const int c = blockIdx.x - a.wg_start[t];
    const WgTask& T = a.task[t];
    const int nact = wg_nact(a);
    const int b0 = (int)((int64_t)c * nact / T.G);
    const int b1 = (int)((int64_t)(c + 1) * nact / T.G);
    float* slab = a.slab + T.slab + (int64_t)c * (T.a.width * T.b.width + T.a.width);
    // task shapes (see nr_wgrad's task list); wave-uniform
    // (WM, WN) = wave grid over the task's output (<= 8 waves; 128 accumulators max)
    switch (__builtin_amdgcn_readfirstlane(T.id)) {
        case 0: case 4:
            wgrad_body<SEG_ACC, 256, SEG_PE, 64, 8, 1, GA, ROWS>(a, T, b0, b1, lds, slab); break;
        case 10:
            wgrad_body<SEG_ACC, 128, SEG_ACC, 256, 2, 4, GA, ROWS>(a, T, b0, b1, lds, slab); break;
        case 11:
            wgrad_body<SEG_ACC, 128, SEG_DPE, 32, 4, 1, GA, ROWS>(a, T, b0, b1, lds, slab); break;
        case 12:
            wgrad_body<SEG_HEAD, 4, SEG_ACC, 256, 1, 8, GA, ROWS>(a, T, b0, b1, lds, slab); break;
        case 13:
            wgrad_body<SEG_HEAD, 4, SEG_ACC, 128, 1, 4, GA, ROWS>(a, T, b0, b1, lds, slab); break;
        default:
            wgrad_body<SEG_ACC, 256, SEG_ACC, 256, 2, 4, GA, ROWS>(a, T, b0, b1, lds, slab); break;
    }
}

#endif  // NR_X3_BASE_OBJECT

// ---------------------------------------------------------------------------
// bf16x6 variant: the same task list and slabs on v_mfma_f32_32x32x16_bf16.
// A stage is 16 samples (half a block): each thread loads the float4s of two
// adjacent samples of one 4-column chunk, splits them exactly into three bf16
// pieces (x3.h) and writes them as [piece][column][16 samples] images
// (column stride 48 B: conflict-free ds_read_b128 fragments), double
// buffered; the bias sums come from the fp32 values during staging.
// ---------------------------------------------------------------------------
// NR_W3_DBG (timing experiments only): 1 = no MFMAs, 2 = no global loads after
// the first stage, 3 = no LDS staging stores, 4 = input operand loaded but not
// staged (the price of its split and LDS stores)
#ifndef NR_W3_DBG
#define NR_W3_DBG 0
#endif
#ifndef NR_W3_SGB
#define NR_W3_SGB 1
#endif
#ifndef NR_W3_MULTI
#define NR_W3_MULTI 1
#endif
#ifndef NR_W3_EARLY
#define NR_W3_EARLY 0
#endif
// Cache policy of the saved-segment reads (each byte is read once).  The
// bf16 LDS-DMA reads are non-temporal: fine-pass wgrad 1.447 -> 1.388 ms
// (NR_W3_DMA_NT).  Non-temporal register loads in the f16x3 / bf16x6 staging
// (NR_W3_NT=1) measured slower, 3.02 -> 3.13 ms (profiles/r02/nt_ab.txt).
#ifndef NR_W3_NT
#define NR_W3_NT 0
#endif
#ifndef NR_W3_DMA_NT
#define NR_W3_DMA_NT 1
#endif
namespace w3 {
template <class T>
__device__ __forceinline__ T ld_seg(const T* p) {
#if NR_W3_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
// cache policy bits of the bf16 segment DMA (2 = nt)
[[maybe_unused]] constexpr int kDmaAux = NR_W3_DMA_NT ? 2 : 0;
constexpr int kColB = 48;                        // bytes per column (16 pieces + pad)
constexpr int kPlane = 256 * kColB;              // one piece of one operand
constexpr int kOpnd = x3::kNP * kPlane;          // one operand (all pieces)
constexpr int kXPlane = 64 * kColB;              // one piece of a fused task's extra operand
constexpr int kXOpnd = kFuse ? x3::kNP * kXPlane : 0;
constexpr int kBufB = 2 * kOpnd + kXOpnd;        // one stage buffer (A + B [+ X])
constexpr int kLds = 2 * kBufB;                  // double buffered: 147,456 B (bf16x6), 110,592 B (f16x3)

// The bf16x6 pipeline saves every segment in x3.h's N16 layout: float4 (F,
// S, lane 16g + j) = columns 16F + 4g .. +3 of sample 16S + j (PE segments:
// columns = PE slots, packing.PE16_MAP / DIR16_MAP).  A staging chunk k is
// columns 8k .. 8k+7; half h of it is float4 group g = 2(k & 1) + h of tile
// F = k >> 1.
template <int KIND, int W>
struct Geo3 {
    static constexpr int CHUNKS = KIND == SEG_ACC ? W / 8 : (KIND == SEG_PE ? 8 : (KIND == SEG_DPE ? 4 : 0));
    __device__ static __forceinline__ int col(int k, int h) { return 8 * k + 4 * h; }
    // float4 index inside a block of sample j of half-block hb
    __device__ static __forceinline__ int f4(int k, int h, int hb, int j) {
        return ((k >> 1) * 2 + hb) * 64 + 16 * (2 * (k & 1) + h) + j;
    }
};

// one operand's half-block: loads (2 float4 per thread) and the split/store.
// ROWS: an input segment saved sample-major (x3.h store_row: row width
// RW = the segment's columns); else N16 slots (gradient segments)
template <int KIND, int W, bool ROWS = false>
struct Stager {
    static constexpr int RW = Geo3<KIND, W>::CHUNKS * 8;
    bool act;      // this thread owns a pair (loads run for every thread, clamped)
    int k, h, jp;  // chunk, lane half, sample pair
    f32x4 v0, v1;
    static constexpr bool ALL = KIND != SEG_HEAD && Geo3<KIND, W>::CHUNKS * 16 >= kThreads;
    __device__ __forceinline__ void init(int tid) {
        if constexpr (KIND == SEG_HEAD) {
            act = tid < 8; k = 0; h = 0; jp = tid & 7;
        } else {
            k = tid >> 4; h = (tid >> 3) & 1; jp = tid & 7;
            act = ALL || k < Geo3<KIND, W>::CHUNKS;
            k = act ? k : 0;
        }
    }
    // samples 16 hb + 2 jp and +1 of block blk (unconditional: keeps the
    // compiler's vmcnt bookkeeping exact across the prefetch)
    __device__ __forceinline__ void load(const float* base, int blk, int hb) {
        if constexpr (KIND == SEG_HEAD) {
            const f32x4* p = reinterpret_cast<const f32x4*>(base) + (size_t)blk * 32 + 16 * hb + 2 * jp;
            v0 = ld_seg(p); v1 = ld_seg(p + 1);
        } else {
            constexpr int F4 = Geo3<KIND, W>::CHUNKS * 64;
#if NR_BF1      // bf16 segments (x3.h store_slot): 8-B slots, sample-major chunks, NR_SEGF block stride
            const x3::u32x2* p = reinterpret_cast<const x3::u32x2*>(base) + (size_t)blk * F4 +
                                 x3::bf16_slot(Geo3<KIND, W>::f4(k, h, hb, 2 * jp));
            v0 = x3::unpack_bf16x4(p[0]); v1 = x3::unpack_bf16x4(p[4]);
#else
            if constexpr (ROWS) {
                const float* r = base + ((size_t)blk * 32 + 16 * hb + 2 * jp) * RW + Geo3<KIND, W>::col(k, h);
                v0 = ld_seg(reinterpret_cast<const f32x4*>(r));
                v1 = ld_seg(reinterpret_cast<const f32x4*>(r + RW));
            } else {
                const f32x4* p = reinterpret_cast<const f32x4*>(base) + (size_t)blk * F4 +
                                 Geo3<KIND, W>::f4(k, h, hb, 2 * jp);
                v0 = ld_seg(p); v1 = ld_seg(p + 1);
            }
#endif
        }
    }
    // the same two samples gathered: sample s of the list (s0, s1) sits at
    // block s / 32, half-block (s / 16) & 1, lane column s & 15
    __device__ __forceinline__ void load_g(const float* base, int s0, int s1) {
        static_assert(KIND != SEG_HEAD, "head segments are gradients (packed by position)");
#if NR_BF1
        (void)base; (void)s0; (void)s1;
#else
        if constexpr (ROWS) {
            v0 = ld_seg(reinterpret_cast<const f32x4*>(base + (size_t)s0 * RW + Geo3<KIND, W>::col(k, h)));
            v1 = ld_seg(reinterpret_cast<const f32x4*>(base + (size_t)s1 * RW + Geo3<KIND, W>::col(k, h)));
        } else {    // N16: block s / 32, half-block (s / 16) & 1, lane column s & 15
            constexpr int F4 = Geo3<KIND, W>::CHUNKS * 64;
            const f32x4* b = reinterpret_cast<const f32x4*>(base);
            v0 = ld_seg(b + (size_t)(s0 >> 5) * F4 + Geo3<KIND, W>::f4(k, h, (s0 >> 4) & 1, s0 & 15));
            v1 = ld_seg(b + (size_t)(s1 >> 5) * F4 + Geo3<KIND, W>::f4(k, h, (s1 >> 4) & 1, s1 & 15));
        }
#endif
    }
    // split + store column e of this thread's chunk into an operand image
    // (values times sc, a power of two); samples >= nval become 0; adds the two
    // samples' unscaled sum (bias) to s
    __device__ __forceinline__ void store_e(char* img, int nval, int e, float& s, float sc,
                                            int plane = kPlane) {
        if (!ALL && !act) return;
        const int j = 2 * jp;
        const float x0 = j < nval ? v0[e] : 0.f, x1 = j + 1 < nval ? v1[e] : 0.f;
        const int c0 = KIND == SEG_HEAD ? 0 : Geo3<KIND, W>::col(k, h);
        s += x0 + x1;
        x3::p2 pc[x3::kNP];
        x3::split_p2(x0 * sc, x1 * sc, pc);
        char* q = img + (c0 + e) * kColB + 4 * jp;
#pragma unroll
        for (int i = 0; i < x3::kNP; ++i) *reinterpret_cast<x3::p2*>(q + i * plane) = pc[i];
    }
};

// A fused task's extra operand, staged thin: thread q < W * 8 loads one float2
// (columns 2cp, 2cp + 1 of sample j of the half-block, q = 16 cp + j) -- 2
// registers per set instead of Stager's 8 -- and writes single pieces.
// ROWS: an input segment (sample-major rows of W), else the head gradient.
template <int KIND, int W, bool ROWS = false>
struct ThinStager {
    static constexpr int Q = W * 8;            // float2 per half-block
    bool act;
    int j, c;                                  // sample, first column
    x3::f32x2 v;
    __device__ __forceinline__ void init(int tid) {
        act = tid < Q;
        const int q = act ? tid : 0;
        j = q & 15; c = 2 * (q >> 4);
    }
    __device__ __forceinline__ void load(const float* base, int blk, int hb) {
        size_t f;   // float offset of the pair
        if constexpr (KIND == SEG_HEAD) f = 4 * ((size_t)blk * 32 + 16 * hb + j) + c;
        else if constexpr (ROWS) f = ((size_t)blk * 32 + 16 * hb + j) * W + c;
        else f = 4 * ((size_t)blk * (W / 8) * 64 + ((c >> 4) * 2 + hb) * 64 + 16 * ((c & 15) >> 2) + j) + (c & 3);
#if NR_BF1
        static_assert(KIND == SEG_HEAD, "bf16 runs no fused task pairs (kFuse)");
#endif
        v = ld_seg(reinterpret_cast<const x3::f32x2*>(base + f));
    }
    // the same pair of sample s (gathered, see Stager::load_g)
    __device__ __forceinline__ void load_g(const float* base, int s) {
        static_assert(KIND != SEG_HEAD, "head segments are gradients (packed by position)");
        const size_t f = ROWS ? (size_t)s * W + c
                              : 4 * ((size_t)(s >> 5) * (W / 8) * 64 + ((c >> 4) * 2 + ((s >> 4) & 1)) * 64 +
                                     16 * ((c & 15) >> 2) + (s & 15)) + (c & 3);
        v = ld_seg(reinterpret_cast<const x3::f32x2*>(base + f));
    }
    // split + store this thread's pair (times sc); s0/s1 += the unscaled values
    __device__ __forceinline__ void store(char* img, int nval, float& s0, float& s1, float sc) {
        if (!act) return;
        const float x0 = j < nval ? v[0] : 0.f, x1 = j < nval ? v[1] : 0.f;
        s0 += x0; s1 += x1;
        x3::p2 pc[x3::kNP];
        x3::split_p2(x0 * sc, x1 * sc, pc);
        char* q = img + c * kColB + 2 * j;
#pragma unroll
        for (int i = 0; i < x3::kNP; ++i) {
            *reinterpret_cast<x3::p1*>(q + i * kXPlane) = pc[i][0];
            *reinterpret_cast<x3::p1*>(q + kColB + i * kXPlane) = pc[i][1];
        }
    }
};

// the pieces of one 32-column fragment at q (plane stride `plane`)
__device__ __forceinline__ x3::Pieces frag(const char* q, int plane) {
    x3::Pieces f;
    f.hi = *reinterpret_cast<const x3::p8*>(q);
#if NR_F16
    f.lo = *reinterpret_cast<const x3::p8*>(q + plane);
#elif NR_BF1
    (void)plane;
#else
    f.mid = *reinterpret_cast<const x3::p8*>(q + plane);
    f.lo = *reinterpret_cast<const x3::p8*>(q + 2 * plane);
#endif
    return f;
}
}  // namespace w3

// One task's workgroup.  Optional fused extra operand X (kFuse, f16x3): XS = 0
// X is a second input segment sharing the gradient operand A (extra output
// M x XW), XS = 1 a second gradient segment sharing the input operand B (the
// 4-row head: extra output XW x N); its XWM x XWN wave grid covers the extra
// output (grids smaller than 8 waves are computed twice, written once) and the
// result goes to the partner task's slab `xslab`.
template <bool GA, bool ROWS, int KA, int WA, int KB, int WB, int WM, int WN, int XK = -1,
          int XW = 0, int XS = 0, int XWM = 1, int XWN = 1>
__device__ __forceinline__ void wgrad3_body(const WgArgs& a, const WgTask& T, int b0, int b1,
                                            char* lds, float* __restrict__ slab,
                                            float* __restrict__ xslab = nullptr) {
    using namespace w3;
    constexpr int MT = (WA / WM + 31) / 32, NT = (WB / WN + 31) / 32;
    constexpr int M = WA, N = WB;
    constexpr bool HX = XK >= 0;
    constexpr int XKK = HX ? XK : SEG_HEAD, XWW = HX ? XW : 4;
    constexpr int XM = XS ? XW : M, XN = XS ? N : XW;              // extra output
    constexpr int XMT = XS ? 1 : (M / XWM + 31) / 32;
    constexpr int XNT = XS ? (N / XWN + 31) / 32 : (XWW / XWN + 31) / 32;
    static_assert(!HX || (kFuse && XWM * XWN <= 8 && 8 % (XWM * XWN) == 0), "extra operand grid");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool active = wave < WM * WN;
    const int mi = wave / WN, ni = wave % WN;
    const int m0 = 32 * MT * mi, n0 = 32 * NT * ni;
    const int xw = wave % (XWM * XWN);
    const int xm0 = 32 * XMT * (xw / XWN), xn0 = 32 * XNT * (xw % XWN);
    const int h = lane >> 5, col = lane & 31;

    f32x16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x16{};
    f32x16 xacc[HX ? XMT : 1][HX ? XNT : 1];
    if constexpr (HX) {
#pragma unroll
        for (int i = 0; i < XMT; ++i)
#pragma unroll
            for (int j = 0; j < XNT; ++j) xacc[i][j] = f32x16{};
    }
    float bacc[4] = {0.f, 0.f, 0.f, 0.f};
    float xbacc[2] = {0.f, 0.f};

    // two register sets per operand: the loads run two stages ahead
    Stager<KA, WA> sa[2];          // gradient operand (N16 slots, by position)
    Stager<KB, WB, ROWS> sb[2];    // input operand (sample-major rows, or N16)
    ThinStager<XKK, XWW, ROWS && HX && XS == 0> sx[2];
    sa[0].init(tid); sa[1].init(tid);
    sb[0].init(tid); sb[1].init(tid);
    if constexpr (HX) { sx[0].init(tid); sx[1].init(tid); }
    if constexpr (KA == SEG_HEAD) {     // rows 4..31 of the 4-row gradient image stay 0
        for (int i = tid; i < 2 * x3::kNP * 32 * kColB / 4; i += kThreads) {
            const int b = i / (x3::kNP * 32 * kColB / 4), r = i % (x3::kNP * 32 * kColB / 4);
            const int p = r / (32 * kColB / 4), o = r % (32 * kColB / 4);
            reinterpret_cast<uint32_t*>(lds + b * kBufB + p * kPlane)[o] = 0u;
        }
    }
    if constexpr (HX && XS == 1) {      // same for a head extra operand (whole X image)
        for (int i = tid; i < 2 * kXOpnd / 4; i += kThreads) {
            constexpr int kW = kXOpnd > 0 ? kXOpnd / 4 : 1;
            const int b = i / kW, o = i % kW;
            reinterpret_cast<uint32_t*>(lds + b * kBufB + 2 * kOpnd)[o] = 0u;
        }
    }
    if constexpr (KA == SEG_HEAD || (HX && XS == 1)) __syncthreads();
    const int nst = 2 * (b1 - b0);      // half-block stages
    // stages past the end load a valid block and store zeros into a buffer
    // nobody reads again
    const int blast = b1 > b0 ? b1 - 1 : b0;
    const float* xbase = HX ? (XS ? a.task[T.fuse].a.base : a.task[T.fuse].b.base) : nullptr;
    // [b0, b1) are blocks of positions.  With a sample list (a.slist) the
    // gradient operands are packed by position and the input operands are
    // gathered: position q holds sample slist[q] (positions past m load
    // sample 0 and stage zeros).  Each register set holds the list entries of
    // the stage it loads next, fetched when its previous stage was loaded
    const int m = wg_m(a);
    constexpr bool gat = GA;
    auto sample_at = [&](int st, int j) {   // positions past m: sample 0 (staged as zeros)
        const int q = min(b0 + (st >> 1), blast) * 32 + 16 * (st & 1) + j;
        return q < m ? a.slist[q] : 0;
    };
    constexpr bool XIN = HX && XS == 0;    // the extra operand is an input segment
    int ns[2][2] = {{0, 0}, {0, 0}}, nx[2] = {0, 0};
    // B operand (input segment): this thread's samples 2 jp, 2 jp + 1; the
    // extra input operand: sample j of its ThinStager
    auto fetch = [&](int set, int st) {
        if constexpr (!gat) return;
        ns[set][0] = sample_at(st, 2 * sb[set].jp);
        ns[set][1] = sample_at(st, 2 * sb[set].jp + 1);
        if constexpr (XIN) nx[set] = sample_at(st, sx[set].j);
    };
    fetch(0, 0);
    fetch(1, 1);
    auto load = [&](int set, int st) {
        if (NR_W3_DBG == 2 && st > 1) return;
        const int blk = min(b0 + (st >> 1), blast), hb = st & 1;
        sa[set].load(T.a.base, blk, hb);
        if constexpr (gat) {
            sb[set].load_g(T.b.base, ns[set][0], ns[set][1]);
            if constexpr (XIN) sx[set].load_g(xbase, nx[set]);
            else if constexpr (HX) sx[set].load(xbase, blk, hb);
            fetch(set, st + 2);
        } else {
            sb[set].load(T.b.base, blk, hb);
            if constexpr (HX) sx[set].load(xbase, blk, hb);
        }
    };
    const float sca = task_scale(a, T);
    const float scx = HX && XS ? task_scale(a, a.task[T.fuse]) : 1.f;
    auto store = [&](int set, int buf, int st) {
        const int nval = st < nst ? m - (b0 + (st >> 1)) * 32 - 16 * (st & 1) : 0;
        float sdummy = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            sa[set].store_e(lds + buf * kBufB, nval, e, bacc[e], sca);
            sb[set].store_e(lds + buf * kBufB + kOpnd, nval, e, sdummy, 1.f);
        }
        if constexpr (HX) sx[set].store(lds + buf * kBufB + 2 * kOpnd, nval, xbacc[0], xbacc[1], scx);
    };
    // LDS-only barrier: keeps the prefetched global loads in flight
    auto barrier = [] {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    // compute stage (buffer buf) from LDS while staging the next stage from
    // register set `set` into buffer buf ^ 1: the 8 store units (2 operands x
    // 4 columns) are spread between the row tiles' MFMAs so their VALU and
    // LDS-store work overlaps the MFMAs in flight instead of idling both waves
    // of a SIMD at the same time; the extra operand's 4 units follow its MFMAs
    // NR_W3_EARLY: all store units first, then the reload of the freed set
    // (after(): two compute phases of latency for the loads instead of one),
    // then the MFMAs -- the partner wave of the SIMD covers the staging VALU
    auto compute_store = [&](int buf, int set, int st_next, auto after) {
        const int nval = st_next < nst ? m - (b0 + (st_next >> 1)) * 32 - 16 * (st_next & 1) : 0;
        char* ia = lds + (buf ^ 1) * kBufB;
        char* ib = ia + kOpnd;
        char* ix = ia + 2 * kOpnd;
        float sdummy = 0.f;
        auto unit = [&](int u) {
            if (NR_W3_DBG == 3) return;
            if (u < 4) sa[set].store_e(ia, nval, u, bacc[u], sca);
            else if (NR_W3_DBG == 4) asm volatile("" ::"v"(sb[set].v0), "v"(sb[set].v1));   // loads kept, no B staging
            else sb[set].store_e(ib, nval, u - 4, sdummy, 1.f);
        };
        const char* cur = lds + buf * kBufB;
        const char* la = cur + (m0 + col) * kColB + 16 * h;
        const char* lb = cur + kOpnd + (n0 + col) * kColB + 16 * h;
        const bool go = (WM * WN == 8 || active) && NR_W3_DBG != 1;
        if constexpr (NR_W3_EARLY) {
#pragma unroll
            for (int u = 0; u < 8; ++u) unit(u);
            if constexpr (HX) if (NR_W3_DBG != 3) sx[set].store(ix, nval, xbacc[0], xbacc[1], scx);
            after();
        }
        x3::Pieces bp[NT];
        if (go) {
#pragma unroll
            for (int j = 0; j < NT; ++j) bp[j] = frag(lb + 32 * j * kColB, kPlane);
        }
        constexpr int UPT = (8 + MT - 1) / MT;   // store units per row tile
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            if (go) {
                x3::p8 ap[x3::kNP];
#pragma unroll
                for (int k = 0; k < x3::kNP; ++k)
                    ap[k] = *reinterpret_cast<const x3::p8*>(la + 32 * i * kColB + k * kPlane);
#if NR_W3_MULTI
                x3::mfma_xp_multi<NT>(ap, bp, acc[i]);
#else
#pragma unroll
                for (int j = 0; j < NT; ++j) acc[i][j] = x3::mfma_xp(ap, bp[j], acc[i][j]);
#endif
            }
            if constexpr (!NR_W3_EARLY) {
#pragma unroll
                for (int v = 0; v < UPT; ++v)
                    if (i * UPT + v < 8) unit(i * UPT + v);
            }
        }
        if constexpr (HX) {
            // extra output: A rows from the A image (XS = 0) or the X image,
            // B columns from the X image (XS = 0) or the B image
            const char* xa = (XS ? cur + 2 * kOpnd : cur) + (xm0 + col) * kColB + 16 * h;
            const char* xb = (XS ? cur + kOpnd : cur + 2 * kOpnd) + (xn0 + col) * kColB + 16 * h;
            constexpr int PA = XS ? kXPlane : kPlane, PB = XS ? kPlane : kXPlane;
            x3::Pieces xp[XNT];
#pragma unroll
            for (int j = 0; j < XNT; ++j) xp[j] = frag(xb + 32 * j * kColB, PB);
#pragma unroll
            for (int i = 0; i < XMT; ++i) {
                x3::p8 ap[x3::kNP];
#pragma unroll
                for (int k = 0; k < x3::kNP; ++k)
                    ap[k] = *reinterpret_cast<const x3::p8*>(xa + 32 * i * kColB + k * PA);
                x3::mfma_xp_multi<XNT>(ap, xp, xacc[i]);
            }
            if constexpr (!NR_W3_EARLY) if (NR_W3_DBG != 3) sx[set].store(ix, nval, xbacc[0], xbacc[1], scx);
        }
#if NR_W3_SGB
        // interleave: per row tile, its fragment reads, then each MFMA followed
        // by two VALU ops of the store units, then the units' LDS stores
        if constexpr (WM * WN == 8 && !NR_W3_EARLY) {
            __builtin_amdgcn_sched_group_barrier(0x100, x3::kNP * NT, 0);
#pragma unroll
            for (int i = 0; i < MT; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x100, x3::kNP, 0);
#pragma unroll
                for (int r = 0; r < x3::kNProd * NT; ++r) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, NR_W3_SGB, 0);
                }
                __builtin_amdgcn_sched_group_barrier(0x200, x3::kNP * UPT, 0);
            }
            if constexpr (HX) {
                __builtin_amdgcn_sched_group_barrier(0x100, x3::kNP * (XNT + XMT), 0);
#pragma unroll
                for (int r = 0; r < x3::kNProd * XNT * XMT; ++r) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, NR_W3_SGB, 0);
                }
                __builtin_amdgcn_sched_group_barrier(0x200, x3::kNP * 2, 0);
            }
        }
#endif
        if constexpr (!NR_W3_EARLY) after();
    };
    // stage st lives in LDS buffer st & 1 and register set st & 1; a set is
    // reloaded (two stages ahead) as soon as its stage has been stored
    load(0, 0);
    load(1, 1);
    store(0, 0, 0);
    load(0, 2);
    barrier();
#pragma unroll 1
    for (int st = 0; st < nst; st += 2) {
        // stage st from buffer 0; set 1 (stage st+1) -> buffer 1, then set 1 reloaded
        compute_store(0, 1, st + 1, [&] { load(1, st + 3); });
        barrier();
        // stage st+1 from buffer 1; set 0 (stage st+2) -> buffer 0, then set 0 reloaded
        compute_store(1, 0, st + 2, [&] { load(0, st + 4); });
        barrier();
    }
    // bias sums: reduce the 8 sample pairs of each (chunk, half) group of the
    // gradient operand; lane jp == 0 writes
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        bacc[e] += __shfl_xor(bacc[e], 1);
        bacc[e] += __shfl_xor(bacc[e], 2);
        bacc[e] += __shfl_xor(bacc[e], 4);
    }
    if constexpr (HX && XS == 1) {      // over the 16 samples of each column pair
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int d = 1; d < 16; d <<= 1) xbacc[e] += __shfl_xor(xbacc[e], d);
    }
    if (sa[0].act && sa[0].jp == 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int o = KA == SEG_HEAD ? e : Geo3<KA, WA>::col(sa[0].k, sa[0].h) + e;
            if (o < M) {
                slab[M * N + o] = bacc[e];
                if constexpr (HX && XS == 0) xslab[XM * XN + o] = bacc[e];   // shared gradient operand
            }
        }
    }
    if constexpr (HX && XS == 1) {      // the head extra operand is a gradient: its bias sums
        if (sx[0].act && sx[0].j == 0) {
#pragma unroll
            for (int e = 0; e < 2; ++e)
                if (sx[0].c + e < XM) xslab[XM * XN + sx[0].c + e] = xbacc[e];
        }
    }
    if constexpr (HX) {
        if (wave < XWM * XWN) {
#pragma unroll
            for (int i = 0; i < XMT; ++i)
#pragma unroll
                for (int j = 0; j < XNT; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int o = xm0 + 32 * i + nr_acc_row(r, h);
                        const int c = xn0 + 32 * j + col;
                        if (o < XM && c < XN) xslab[o * XN + c] = xacc[i][j][r];
                    }
        }
    }
    if (!active) return;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int o = m0 + 32 * i + nr_acc_row(r, h);
                const int c = n0 + 32 * j + col;
                if (o < M && c < N) slab[o * N + c] = acc[i][j][r];
            }
}

#if NR_BF1
// ---------------------------------------------------------------------------
// bf16 variant: no register staging at all.  The saved segments already hold
// the bf16 operands in sample-major 16x16 chunks (x3.h store_slot), so a
// workgroup copies whole blocks of both operands into an LDS ring by LDS-DMA
// (buffer_load_dwordx4 ... lds: one 1-KiB instruction per 16-feature tile,
// kB1Depth blocks in flight) and reads its v_mfma_f32_32x32x16_bf16 fragments
// with ds_read_b64_tr_b16 (16 lanes gather a 4-sample x 16-feature block
// column-major: two reads = one lane's 8 consecutive samples of one
// feature).  A tile's two 512-B chunks sit in 1152 B of LDS: the 128-B pad
// puts the next tile's chunk in the other half of the banks, so both 16-lane
// groups of a 32-lane half read conflict-free.  Samples past n are harmless:
// their gradient rows are exact zeros (mlp_bwd3.hip), their inputs finite
// copies of the last sample.  Bias sums come from the gradient fragments.
// ---------------------------------------------------------------------------
namespace b1 {
constexpr int kTile = 1152;      // LDS bytes per 16-feature tile of a block
constexpr int kDepth = 4;        // blocks in the ring
// the whole LDS: 256 + 256 features per block (+ a fused task's extra operand)
constexpr int kLds = 160 * 1024;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

// fragment rows r0 .. r0+31 (features), k-step S (samples 16S .. 16S+15) of a block image
// (TS: the image's tile stride -- kTile, or 1024 for an unpadded extra operand)
template <int TS = kTile>
__device__ __forceinline__ x3::p8 frag_tr(const char* img, int r0, int S, int lane) {
    const int g4 = lane >> 4, i = lane & 15;
    const char* p = img + ((r0 >> 4) + (g4 & 1)) * TS + S * 512 + 32 * (8 * (g4 >> 1) + (i >> 2)) +
                    8 * (i & 3);
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 128));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(x3::p8, v);
}

// the head operand's fragment (HEADA): lane 4q + p of each 16-lane group
// addresses sample 8h + q (+4) of k-step S -- all four p the same 8 B, so
// columns 0..3 (the 4 gradient columns) are right and the rest repeat them
__device__ __forceinline__ x3::p8 frag_head(const char* img, int S, int lane) {
    const char* p = img + 8 * (16 * S + 8 * (lane >> 5) + ((lane & 15) >> 2));
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 32));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(x3::p8, v);
}

__device__ __forceinline__ float frag_sum(const x3::p8& f) {
    typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
    const u32x4_t u = __builtin_bit_cast(u32x4_t, f);
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) s += __uint_as_float(u[e] << 16) + __uint_as_float(u[e] & 0xffff0000u);
    return s;
}
}  // namespace b1

// HEADA: the gradient operand is the 4-column head segment [dz_rgb, dsigma],
// bf16 [block][32 samples][4] (mlp_bwd3.hip): one 256-B dword LDS-DMA per
// block, and every lane of a transposed read points at its sample's 4 values
// (rows 4 .. 31 of the fragment repeat them and are never written out)
//
// Fused task pairs (XMODE, as wgrad3_body's extra operand): XMODE 1 -- a
// second input segment X (XW columns, XW / 16 tiles) shares the gradient
// operand A; the waves of grid column 0 also compute A x X into the partner's
// slab `xslab` (dz_dir x [feat | dir PE]).  XMODE 2 -- a second gradient
// segment, the 4-column head (dword DMA, frag_head), shares the input operand
// B; the waves of grid row 0 also compute head x B ([dfeat | head] x h8).
// Either way the shared segment is read once.
template <int WA, int WB, int WM, int WN, bool HEADA = false, int XMODE = 0, int XW = 0>
__device__ __forceinline__ void wgrad_b1_body(const WgArgs& a, const WgTask& T, int b0, int b1_,
                                              char* lds, float* __restrict__ slab,
                                              float* __restrict__ xslab = nullptr) {
    using namespace b1;
    static_assert(!HEADA || WA == 4, "head operand");
    static_assert(XMODE == 0 || (!HEADA && (XMODE == 2 || XW % 32 == 0)), "extra operand");
    constexpr int TA = HEADA ? 1 : WA / 16, TB = WB / 16;
    constexpr int TX = XMODE == 1 ? XW / 16 : (XMODE == 2 ? 1 : 0);
    constexpr int NDMA = TA + TB + TX;
    constexpr int ABYTES = HEADA ? 256 : TA * kTile;
    constexpr int XOFF = ABYTES + TB * kTile;                       // extra image
    // the extra operand's tiles go unpadded (2-way bank conflicts on its
    // fragment reads) when padded ones would not fit the 4-block ring
    constexpr int XTS = kDepth * (XOFF + TX * kTile) <= b1::kLds ? kTile : 1024;
    constexpr int IMG = XOFF + (XMODE == 1 ? TX * XTS : (XMODE == 2 ? 256 : 0));
    static_assert(kDepth * IMG <= b1::kLds, "ring");
    constexpr int MT = (WA / WM + 31) / 32, NT = (WB / WN + 31) / 32;
    constexpr int XNT = XMODE == 1 ? XW / 32 : 1;
    // this wave's DMAs issued after a block's (waves issuing more wait a little longer)
    constexpr int kWait = (kDepth - 2) * (NDMA / 8);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool active = wave < WM * WN;
    const int mi = wave / WN, ni = wave % WN;
    const int m0 = 32 * MT * mi, n0 = 32 * NT * ni;
    // the resources start at this workgroup's first block: buffer offsets and
    // sizes are 32-bit, and a whole segment passes 2^31 bytes at 2^16 blocks
    // (2.1M samples per call) while one workgroup's slice stays far below
    constexpr int64_t ABLK = HEADA ? 256 : WA * 64, BBLK = WB * 64;   // bytes per block (NR_SEGF)
    constexpr int64_t XBLK = XMODE == 1 ? XW * 64 : 256;
    const int nblk = b1_ - b0;
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(reinterpret_cast<const char*>(T.a.base) + (int64_t)b0 * ABLK), 0, (int)(nblk * ABLK), 0x00020000);
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(reinterpret_cast<const char*>(T.b.base) + (int64_t)b0 * BBLK), 0, (int)(nblk * BBLK), 0x00020000);
    const float* xbase = XMODE == 1 ? a.task[T.fuse].b.base : (XMODE == 2 ? a.task[T.fuse].a.base : T.a.base);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(reinterpret_cast<const char*>(xbase) + (int64_t)b0 * XBLK), 0,
        XMODE ? (int)(nblk * XBLK) : 0, 0x00020000);
    // block b -> ring slot: tile i < TA of A, then the TB tiles of B, then the
    // extra operand's tiles (or its 256-B head block), 1 KiB each
    auto dma = [&](int b, int slot) {
        b = min(b, b1_ - 1) - b0; // past the end: re-read the last block (keeps vmcnt exact)
        char* img = lds + slot * IMG;
        typedef __attribute__((address_space(3))) void* lds_ptr;
        // one branch per operand (i is wave-uniform): each names its own
        // buffer resource -- a run-time choice among three put them in scratch
#pragma unroll
        for (int i = wave; i < NDMA; i += 8) {
            if (i < TA) {
                if (HEADA)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr)img, 4, lane * 4, b * 256, 0, w3::kDmaAux);
                else
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr)(img + i * kTile), 16, lane * 16,
                                                             b * WA * 64 + i * 1024, 0, w3::kDmaAux);
            } else if (i < TA + TB) {
                const int t = i - TA;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr)(img + ABYTES + t * kTile), 16,
                                                         lane * 16, b * WB * 64 + t * 1024, 0, w3::kDmaAux);
            } else if constexpr (XMODE == 2) {
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr)(img + XOFF), 4, lane * 4, b * 256, 0, w3::kDmaAux);
            } else if constexpr (XMODE == 1) {
                const int t = i - TA - TB;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr)(img + XOFF + t * XTS), 16,
                                                         lane * 16, b * XW * 64 + t * 1024, 0, w3::kDmaAux);
            }
        }
    };
    f32x16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x16{};
    // extra output: XMODE 1 the (WA/32) x XNT 32x32 tiles dealt to the waves
    // (tile e = wave + 8k, XTPW per wave); XMODE 2 [1][NT] the head row tile x
    // B column tiles (grid row 0)
    constexpr int XRT = WA / 32, XT = XRT * XNT, XTPW = (XT + 7) / 8;
    static_assert(XMODE != 1 || WA % 32 == 0, "extra tiles");
    constexpr int XA = XMODE == 1 ? XTPW : 1, XB = XMODE == 2 ? NT : 1;
    f32x16 xacc[XMODE ? XA : 1][XMODE ? XB : 1];
    if constexpr (XMODE) {
#pragma unroll
        for (int i = 0; i < XA; ++i)
#pragma unroll
            for (int j = 0; j < XB; ++j) xacc[i][j] = f32x16{};
    }
    float bsum[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) bsum[i] = 0.f;
    float xsum = 0.f;
    const bool xw = XMODE == 1 ? wave < XT : mi == 0;   // this wave computes extra output
#pragma unroll
    for (int d = 0; d < kDepth - 1; ++d) dma(b0 + d, d);
#pragma unroll 1
    for (int b = b0, it = 0; b < b1_; ++b, ++it) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kWait) : "memory");
        __builtin_amdgcn_s_barrier();          // every wave's DMA of block b landed; slot it-1 free
        asm volatile("" ::: "memory");
        dma(b + kDepth - 1, (it + kDepth - 1) % kDepth);
        if (!active) continue;
        const char* img = lds + (it % kDepth) * IMG;
#pragma unroll
        for (int S = 0; S < 2; ++S) {
            x3::p8 bf[NT];
#pragma unroll
            for (int j = 0; j < NT; ++j) bf[j] = frag_tr(img + ABYTES, n0 + 32 * j, S, lane);
#pragma unroll
            for (int i = 0; i < MT; ++i) {
                const x3::p8 af = HEADA ? frag_head(img, S, lane) : frag_tr(img, m0 + 32 * i, S, lane);
#pragma unroll
                for (int j = 0; j < NT; ++j) acc[i][j] = x3::mfma32(af, bf[j], acc[i][j]);
                if (ni == 0) bsum[i] += frag_sum(af);
            }
            if constexpr (XMODE == 1) {
#pragma unroll
                for (int k = 0; k < XTPW; ++k) {
                    const int e = wave + 8 * k;
                    if (e < XT)
                        xacc[k][0] = x3::mfma32(frag_tr(img, 32 * (e % XRT), S, lane),
                                                frag_tr<XTS>(img + XOFF, 32 * (e / XRT), S, lane), xacc[k][0]);
                }
            }
            if constexpr (XMODE == 2) {
                if (xw) {
                    const x3::p8 hf = frag_head(img + XOFF, S, lane);
#pragma unroll
                    for (int j = 0; j < NT; ++j) xacc[0][j] = x3::mfma32(hf, bf[j], xacc[0][j]);
                    if (ni == 0) xsum += frag_sum(hf);
                }
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the tail's clamped DMAs
    if (!active) return;
    const int h = lane >> 5, col = lane & 31;
    if (ni == 0) {
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            const float s = bsum[i] + __shfl_xor(bsum[i], 32);
            const int o = m0 + 32 * i + col;
            if (h == 0 && o < WA) {
                slab[WA * WB + o] = s;
                if constexpr (XMODE == 1) xslab[WA * XW + o] = s;   // shared gradient operand
            }
        }
    }
    if constexpr (XMODE == 1) {
#pragma unroll
        for (int k = 0; k < XTPW; ++k) {
            const int e = wave + 8 * k;
            if (e < XT) {
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    xslab[(32 * (e % XRT) + nr_acc_row(r, h)) * XW + 32 * (e / XRT) + col] = xacc[k][0][r];
            }
        }
    }
    if constexpr (XMODE == 2) {
        if (xw) {
            if (ni == 0) {
                const float s = xsum + __shfl_xor(xsum, 32);
                if (h == 0 && col < 4) xslab[4 * WB + col] = s;
            }
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int o = nr_acc_row(r, h);
                    const int c = n0 + 32 * j + col;
                    if (o < 4 && c < WB) xslab[o * WB + c] = xacc[0][j][r];
                }
        }
    }
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int o = m0 + 32 * i + nr_acc_row(r, h);
                const int c = n0 + 32 * j + col;
                if (o < WA && c < WB) slab[o * WB + c] = acc[i][j][r];
            }
}
#endif  // NR_BF1

// GA: the packed sample list a.slist (the *_active entry points); ROWS: the
// input segments are sample-major rows (the full graph's forward), else N16
// (the sigma-only training forward, mlp_fwd3.hip kRows)
template <bool GA, bool ROWS>
__global__ void __launch_bounds__(kThreads, 1) wgrad3_kernel(WgArgs a) {
#if NR_BF1
    __shared__ __attribute__((aligned(16))) char lds[b1::kLds > w3::kLds ? b1::kLds : w3::kLds];
#else
    __shared__ __attribute__((aligned(16))) char lds[w3::kLds];
#endif
    int t = 0;
#pragma unroll 1
    while (t + 1 < kTasks && (int)blockIdx.x >= a.wg_start[t + 1]) ++t;
    const int c = blockIdx.x - a.wg_start[t];
    const WgTask& T = a.task[t];
    const int nact = wg_nact(a);
    const int b0 = (int)((int64_t)c * nact / T.G);
    const int b1 = (int)((int64_t)(c + 1) * nact / T.G);
    float* slab = a.slab + T.slab + (int64_t)c * (T.a.width * T.b.width + T.a.width);
    const int fu = __builtin_amdgcn_readfirstlane(T.fuse);
    if constexpr (kFuse) if (fu >= 0) {
        const WgTask& P = a.task[fu];
        float* xslab = a.slab + P.slab + (int64_t)c * (P.a.width * P.b.width + P.a.width);
#if NR_BF1
        switch (__builtin_amdgcn_readfirstlane(T.id)) {
#if NR_WGRAD_FUSE_MASK & 1
            case 5:    // DZ(4) x [H(3) | PE]: xyz_encoding_5 (skip layer)
                wgrad_b1_body<256, 256, 2, 4, false, 1, 64>(a, T, b0, b1, lds, slab, xslab); break;
#endif
            case 10:   // [dz_dir | head] x H(7): dir_encoding's feat columns (as G) and sigma
                wgrad_b1_body<128, 256, 2, 4, false, 2, 4>(a, T, b0, b1, lds, slab, xslab); break;
        }
#else
        switch (__builtin_amdgcn_readfirstlane(T.id)) {
#if NR_WGRAD_FUSE_MASK & 1
            case 5:    // DZ(4) x [H(3) | PE]: xyz_encoding_5 (skip layer)
                if constexpr (!GA || (NR_WGRAD_FUSE_MASK_GA & 1))
                    wgrad3_body<GA, ROWS, SEG_ACC, 256, SEG_ACC, 256, 2, 4, SEG_PE, 64, 0, NR_WG_PE_WM,
                                8 / NR_WG_PE_WM>(a, T, b0, b1, lds, slab, xslab);
                break;
#endif
#if NR_WGRAD_FUSE_MASK & 2
            case 10:   // [dz_dir | head] x H(7): dir_encoding's feat columns (as G) and sigma
                wgrad3_body<GA, ROWS, SEG_ACC, 128, SEG_ACC, 256, 2, 4, SEG_HEAD, 4, 1, 1, 8>(
                    a, T, b0, b1, lds, slab, xslab); break;
#endif
        }
#endif
        return;
    }
#if NR_BF1
    switch (__builtin_amdgcn_readfirstlane(T.id)) {
        case 0: case 4:
            wgrad_b1_body<256, 64, 8, 1>(a, T, b0, b1, lds, slab); return;
        case 10:
            wgrad_b1_body<128, 256, 2, 4>(a, T, b0, b1, lds, slab); return;
        case 11:
            wgrad_b1_body<128, 32, 4, 1>(a, T, b0, b1, lds, slab); return;
        case 12:
            wgrad_b1_body<4, 256, 1, 8, true>(a, T, b0, b1, lds, slab); return;
        case 13:
            wgrad_b1_body<4, 128, 1, 4, true>(a, T, b0, b1, lds, slab); return;
        default:
            wgrad_b1_body<256, 256, 2, 4>(a, T, b0, b1, lds, slab); return;
    }
#endif
    switch (__builtin_amdgcn_readfirstlane(T.id)) {
        case 0: case 4:
            wgrad3_body<GA, ROWS, SEG_ACC, 256, SEG_PE, 64, 8, 1>(a, T, b0, b1, lds, slab); break;
        case 10:
            wgrad3_body<GA, ROWS, SEG_ACC, 128, SEG_ACC, 256, 2, 4>(a, T, b0, b1, lds, slab); break;
        case 11:
            wgrad3_body<GA, ROWS, SEG_ACC, 128, SEG_DPE, 32, 4, 1>(a, T, b0, b1, lds, slab); break;
        case 12:
            wgrad3_body<GA, ROWS, SEG_HEAD, 4, SEG_ACC, 256, 1, 8>(a, T, b0, b1, lds, slab); break;
        case 13:
            wgrad3_body<GA, ROWS, SEG_HEAD, 4, SEG_ACC, 128, 1, 4>(a, T, b0, b1, lds, slab); break;
        default:
            wgrad3_body<GA, ROWS, SEG_ACC, 256, SEG_ACC, 256, 2, 4>(a, T, b0, b1, lds, slab); break;
    }
}

#ifndef NR_W4
#define NR_W4 1
#endif
// slab index p (row or column) of a WgTask::pa / pb order -> the natural index
__device__ __forceinline__ int w4_unperm(int p, int v) {
    if (v <= 1) return p;
    const int w = 32 * v, r = p % w;
    return p - r + v * (r & 31) + (r >> 5);
}
#ifndef NR_W4_SGB
#define NR_W4_SGB 0      // (unused)
#endif
// NR_W4_DBG (timing experiments only): 1 = no MFMAs (pieces kept alive),
// 4 = splits reduced to the hi conversion (no scale, no residual),
// 2 = no DMA after the prologue, 3 = no LDS reads / splits after the prologue
#ifndef NR_W4_DBG
#define NR_W4_DBG 0
#endif

#if NR_F16
// ---------------------------------------------------------------------------
// f16x3 weight gradient of the full graph, LDS-DMA form (round 5).  The
// register-staged wgrad3_body holds two stages of both operands in VGPRs
// next to its accumulators (two waves per SIMD: 8 spilled VGPRs), which caps
// the bytes in flight per CU; its gathered rows waited ~half of the wave
// cycles.  Here nothing is staged through registers: a workgroup of 4 waves
// (one per SIMD, 512 VGPRs each) copies every 16-sample stage of both operands
// into an LDS ring of kD stages with global_load_lds (3 stages = ~100 KiB in
// flight per CU), and each wave reads its MFMA fragments from LDS as fp32 and
// splits them into the f16 pieces itself, between the MFMAs of the previous
// stage.  One wave's float4 read feeds four 32x32x16 tiles at once: lane c of a
// 128-row chunk holds rows 4c .. 4c + 3, i.e. tile i of the chunk holds rows
// 4 rho + i (the slab stores tiles in that order, the reduction undoes it,
// WgTask::pa / pb).
//   gradient operand (N16 slots by position): one 1-KiB instruction per
//     16-feature piece, its lanes permuted so that the LDS piece is sample-major
//     [sample 16][4 features x 4]; pieces 1088 B apart, so the float4 reads of
//     one instruction's lane groups (x3.h / MICROARCH.md ds_read_b128 groups)
//     fall in distinct banks;
//   input operand (sample-major rows, gathered): one instruction per 1 KiB of
//     rows (1 row of h, 4 PE rows, 8 dir-PE rows), LDS image [sample][W];
//   sample list (GA): each wave DMAs the 16 list entries of stage t + 2kD - 1
//     into its own slot of an index ring, so the row addresses of a stage come
//     from LDS (ordinary loads would make the compiler drain vmcnt, and
//     scalar loads would hold every LDS wait behind their latency).
// A barrier per stage hands it over; positions >= m of the last stage are
// zeroed in LDS.
// ---------------------------------------------------------------------------
namespace w4 {
constexpr int kWaves = 4, kT = 256;
constexpr int kD = 4;                          // ring stages of 16 samples
constexpr int kPS = 1088;                      // LDS stride of a gradient piece (1 KiB + 64 B)
constexpr int kAImg = 16 * kPS;                // gradient image (<= 16 pieces)
constexpr int kBImg = 16 * 1024;               // input image (16 rows x <= 256 floats)
constexpr int kHImg = 256;                     // head gradient [16][4]
constexpr int kSlot = kAImg + kBImg + kHImg;   // 34,048 B
constexpr int kIdxStages = 2 * kD;             // index ring
constexpr int kIdxWave = 256;                  // one wave's copy of a stage's list entries (64 x 4 B)
constexpr int kIdxOff = kD * kSlot;
constexpr int kDummyOff = kIdxOff + kIdxStages * kWaves * kIdxWave;
constexpr int kLds = kDummyOff + 256;          // 144,640 B
typedef __attribute__((address_space(3))) void* lds_ptr;
// buffer_load ... lds (the global_load_lds form makes the compiler wait
// vmcnt(0) before every later DMA and LDS read: it cannot tell the ring slots
// apart); voffset per lane, soffset uniform, byte offsets within the resource
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, int voff, int soff, char* l) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr)l, 16, voff, soff, 0, 0);
}
__device__ __forceinline__ void dma4(__amdgpu_buffer_rsrc_t r, int voff, int soff, char* l) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr)l, 4, voff, soff, 0, 0);
}
// (the record count is an unsigned 32-bit byte count: at n just under 2^21 a
// 256-wide gradient segment is exactly 2^31 bytes, past int's range)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0,
                                             (int)(uint32_t)min(bytes, (int64_t)0xffffffff), 0x00020000);
}
template <int V> struct Vec { typedef float T __attribute__((ext_vector_type(V))); };
template <> struct Vec<1> { typedef float T; };
template <int V>
__device__ __forceinline__ float vget(const typename Vec<V>::T& v, int j) {
    if constexpr (V == 1) return v;
    else return v[j];
}
// the pieces of 8 values as two fragments (x0..x7 times sc): built from packed
// pairs, so each fragment stays 4 VGPRs (element-wise inserts into an f16x8
// keep one half per register)
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void split8(const float (&x)[8], float sc, x3::Pieces& f) {
    uint32_t hi[4], lo[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
#if NR_W4_DBG == 4      // timing experiment: hi pieces only, unscaled (wrong results)
        (void)sc;
        hi[p] = lo[p] = __builtin_bit_cast(uint32_t, __builtin_convertvector((x3::f32x2){x[2 * p], x[2 * p + 1]}, x3::f16x2));
        continue;
#endif
        x3::p2 q[x3::kNP];
        x3::split_p2(x[2 * p] * sc, x[2 * p + 1] * sc, q);
        hi[p] = __builtin_bit_cast(uint32_t, q[0]);
        lo[p] = __builtin_bit_cast(uint32_t, q[1]);
    }
    f.hi = __builtin_bit_cast(x3::p8, (u32x4_t){hi[0], hi[1], hi[2], hi[3]});
    f.lo = __builtin_bit_cast(x3::p8, (u32x4_t){lo[0], lo[1], lo[2], lo[3]});
}
// A x B over one 32x32x16 tile, f16x3 (small products first, as x3::mfma_xp)
__device__ __forceinline__ f32x16 mfma3(const x3::Pieces& a, const x3::Pieces& b, f32x16 acc) {
    acc = x3::mfma32(a.lo, b.hi, acc);
    acc = x3::mfma32(a.hi, b.lo, acc);
    return x3::mfma32(a.hi, b.hi, acc);
}
}  // namespace w4

// One task's workgroup.  MA: rows of the gradient segment (256, 128; 0: the
// task's gradient is the 4-row head); HD: the head gradient rides along as one
// more row tile (MA > 0: the fused partner's, written to xslab); WB: columns
// of the input segment, VB: columns per lane (float, float2, float4 reads);
// NWA x NWB: the wave grid (128-row chunks x 32 VB-column chunks).
template <bool GA, int MA, bool HD, int WB, int VB, int NWA, int NWB>
__device__ __forceinline__ void wgrad4_body(const WgArgs& a, const WgTask& T, int b0, int b1, char* lds,
                                            float* __restrict__ slab, float* __restrict__ xslab) {
    using namespace w4;
    constexpr int NA = MA / 16;                   // gradient pieces per stage
    constexpr int RPI = 256 / WB;                 // input rows per DMA instruction
    constexpr int NBI = 16 / RPI;                 // input instructions per stage
    constexpr int KA = NA / 4, KB = NBI / 4;      // per wave: gradient pieces, full input rounds
    constexpr int RB = NBI % 4;                   // input instructions left over
    constexpr int NX = (HD ? 1 : 0) + RB;         // leftover instructions (one slot per wave)
    constexpr int K = KA + KB + (NX > 0 ? 1 : 0); // DMA instructions per wave and stage
    constexpr int KV = K + (GA ? 1 : 0);          // vm instructions per wave and issue step
    static_assert(NA % 4 == 0 && NX <= kWaves, "DMA assignment");
    constexpr int TA = (MA ? 4 : 0) + (HD ? 1 : 0);
    constexpr int HT = MA ? 4 : 0;                // the head's tile index
    constexpr int RSB = WB * 4;                   // input row stride in LDS (bytes)
    static_assert(NWA * NWB <= kWaves && NWB * 32 * VB == WB && (MA == 0 ? NWA == 1 : NWA * 128 == MA),
                  "wave grid");
    static_assert(RPI * NBI == 16 && WB * 4 * 16 <= kBImg && MA <= 256, "stage geometry");
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 31, h = lane >> 5;
    const int wa = wave / NWB, wb = wave % NWB;
    const bool active = wave < NWA * NWB;
    const int m = wg_m(a);
    const int nst = 2 * (b1 - b0);
    const int blast = b1 > b0 ? b1 - 1 : b0;
    const int mlast = max(m - 1, 0);
    const float* Abase = T.a.base;
    const float* Hbase = MA ? (HD ? a.task[T.fuse].a.base : T.a.base) : T.a.base;
    const float* Bbase = T.b.base;
    const float sca = task_scale(a, T);
    const float sch = HD && MA ? task_scale(a, a.task[T.fuse]) : sca;
    float* hslab = MA ? xslab : slab;             // the head tile's output

    auto q0_of = [&](int t) { return min(b0 + (t >> 1), blast) * 32 + 16 * (t & 1); };
    auto idx_slot = [&](int u) {
        return lds + kIdxOff + (u % kIdxStages) * (kWaves * kIdxWave) + wave * kIdxWave;
    };
    // buffer resources (the host keeps every segment under 2 GiB: wgrad_launch)
    const __amdgpu_buffer_rsrc_t ra = rsrc(Abase, (int64_t)a.nb * (MA ? MA : 4) * 128);
    const __amdgpu_buffer_rsrc_t rh = rsrc(Hbase, (int64_t)a.nb * 512);
    const __amdgpu_buffer_rsrc_t rb = rsrc(Bbase, (int64_t)a.n * WB * 4);
    const __amdgpu_buffer_rsrc_t rl = rsrc(a.slist, GA ? (int64_t)a.n * 4 : 0);
    auto idx_dma = [&](int u) {     // list entries q0(u) .. +63 (clamped) -> this wave's index slot
        dma4(rl, 4 * min(q0_of(u) + lane, mlast), 0, idx_slot(u));
    };
    // one issue step: stage t's DMA into ring slot t % kD (+ the list entries of
    // stage t + 2kD - 1).  Wave w issues gradient pieces w + 4k and input
    // instructions w + 4k (types fixed per k), then one leftover slot: the head,
    // the input instructions past a multiple of 4, or a dummy
    const int voff_a = 16 * (16 * (lane & 3) + (lane >> 2));
    auto b_dma = [&](char* slot, const int* idx, int q0, int r, int s1) {
        if constexpr (RPI == 1) {           // one row per instruction: uniform sample s1
            dma16(rb, 16 * lane, s1 * (WB * 4), slot + kAImg + r * 1024);
        } else {
            const int row = r * RPI + lane / (WB / 4);
            const int s = GA ? idx[row] : min(q0 + row, mlast);
            dma16(rb, s * (WB * 4) + 16 * (lane % (WB / 4)), 0, slot + kAImg + r * 1024);
        }
    };
    // the uniform samples of this wave's one-row instructions of stage t (rows
    // wave * KB + k), from the index ring (one LDS read) or by position
    struct Rows { int s[KB > 0 ? KB : 1]; };
    // (the LDS read and the scalar take of them apart: rows_raw / rows_take)
    auto rows_raw = [&](int t) {
        int4 v{};
        if constexpr (RPI == 1 && GA) v = *reinterpret_cast<const int4*>(idx_slot(t) + 16 * wave);
        return v;
    };
    auto rows_take = [&](int t, const int4 v) {
        Rows r{};
        if constexpr (RPI == 1) {
            if constexpr (GA) {
                static_assert(KB == 4, "one float4 of list entries per wave");
                r.s[0] = __builtin_amdgcn_readfirstlane(v.x);
                r.s[1] = __builtin_amdgcn_readfirstlane(v.y);
                r.s[2] = __builtin_amdgcn_readfirstlane(v.z);
                r.s[3] = __builtin_amdgcn_readfirstlane(v.w);
            } else {
#pragma unroll
                for (int k = 0; k < KB; ++k) r.s[k] = min(q0_of(t) + wave * KB + k, mlast);
            }
        }
        return r;
    };
    auto rows_of = [&](int t) { return rows_take(t, rows_raw(t)); };
    // instruction k (< KV) of this wave's issue step for stage t
    auto issue_k = [&](int t, int k, const Rows& rw) {
        char* slot = lds + (t % kD) * kSlot;
        const int q0 = q0_of(t);
        const int blk = q0 >> 5, hb = (q0 >> 4) & 1;
        const int* idx = reinterpret_cast<const int*>(idx_slot(t));
        if (k < KA) {
            const int i = wave + 4 * k;     // piece i: lane 4j + g <- float4 (g, sample j)
            dma16(ra, voff_a, blk * (MA * 128) + (i * 2 + hb) * 1024, slot + i * kPS);
        } else if (k < KA + KB) {
            const int r = wave * KB + k - KA;
            b_dma(slot, idx, q0, r, rw.s[(k - KA) % (KB > 0 ? KB : 1)]);
        } else if (NX > 0 && k == KA + KB) {
            const int r = 4 * KB + wave - (HD ? 1 : 0);   // an input instruction left over
            if (HD && wave == 0) dma4(rh, 4 * lane, (blk * 32 + 16 * hb) * 16, slot + kAImg + kBImg);
            else if (wave - (HD ? 1 : 0) < RB)
                b_dma(slot, idx, q0, r, RPI == 1 ? (GA ? idx[r] : min(q0 + r, mlast)) : 0);
            else dma4(ra, 4 * lane, 0, lds + kDummyOff);   // keeps every wave's vm count per step equal
        } else if (GA) {
            idx_dma(t + 2 * kD - 1);
        }
    };
    auto issue = [&](int t) {
        const Rows rw = rows_of(t);
#pragma unroll
        for (int k = 0; k < KV; ++k) issue_k(t, k, rw);
    };
    // positions >= m of stage t (the launch's last block): zero both operands in LDS
    auto mask_tail = [&](int t) {
        const int nval = m - q0_of(t);
        if (t >= nst || nval >= 16) return;
        char* slot = lds + (t % kD) * kSlot;
        const int j0 = max(nval, 0);
        if constexpr (NA > 0)
            for (int e = tid; e < (16 - j0) * 16 * NA; e += kT) {   // 16 dwords per piece and sample
                const int j = j0 + e / (16 * NA), r = e % (16 * NA);
                reinterpret_cast<float*>(slot + (r >> 4) * kPS + 64 * j)[r & 15] = 0.f;
            }
        for (int e = tid; e < (16 - j0) * WB; e += kT)
            reinterpret_cast<float*>(slot + kAImg + j0 * RSB)[e] = 0.f;
        if (HD)
            for (int e = tid; e < (16 - j0) * 4; e += kT)
                reinterpret_cast<float*>(slot + kAImg + kBImg + j0 * 16)[e] = 0.f;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };

    f32x16 acc[TA][VB];
#pragma unroll
    for (int i = 0; i < TA; ++i)
#pragma unroll
        for (int j = 0; j < VB; ++j) acc[i][j] = f32x16{};
    f32x4 bsv = {0.f, 0.f, 0.f, 0.f};
    float hs = 0.f;

    // fragments of stage t: ds_read_b32 of one row / column and 8 samples per
    // lane (lanes c of a 32-lane half: 32 consecutive features, conflict-free
    // in both images), split into the f16 pieces right away
    auto split_a = [&](int t, int i, x3::Pieces& f) {
        const char* slot = lds + (t % kD) * kSlot;
        float x[8];
        if (HD && i == HT) {
            const float* ph = reinterpret_cast<const float*>(slot + kAImg + kBImg + 128 * h) + (c & 3);
            float sum = 0.f;
#pragma unroll
            for (int k = 0; k < 8; ++k) { x[k] = c < 4 ? ph[4 * k] : 0.f; sum += x[k]; }
            hs += t < nst ? sum : 0.f;      // (stage nst: the clamped read past the end)
            split8(x, sch, f);
        } else if constexpr (MA > 0) {
            const int fe = 128 * wa + 32 * i + c;
            const float* pa = reinterpret_cast<const float*>(slot + (fe >> 4) * kPS + 512 * h) + (fe & 15);
            float sum = 0.f;
#pragma unroll
            for (int k = 0; k < 8; ++k) { x[k] = pa[16 * k]; sum += x[k]; }
            bsv[i & 3] += t < nst ? sum : 0.f;
            split8(x, sca, f);
        }
    };
    // wide form (VB > 1 / the gradient chunk): lane c holds rows 4c .. 4c + 3 of
    // its 128-row chunk (columns VB c .. VB c + VB - 1 of its column chunk), so
    // one ds_read_b128 (b64) per sample feeds 4 (VB) tiles: tile i holds rows
    // 4 rho + i.  8 + 8 wide reads per stage instead of 32 + 32 ds_read_b32
    // (one wave per SIMD issues those at a fraction of the LDS rate).  The
    // slab is written in that order (WgTask::pa / pb, undone by the reduction).
    using BV = typename Vec<VB>::T;
    struct RawA { f32x4 v[MA > 0 ? 8 : 1]; };
    struct RawB { BV v[8]; };
    auto read_a = [&](int t, RawA& r) {
        if constexpr (MA > 0) {
            const char* pa = lds + (t % kD) * kSlot + (8 * wa + (c >> 2)) * kPS + 512 * h + 16 * (c & 3);
#pragma unroll
            for (int k = 0; k < 8; ++k) r.v[k] = *reinterpret_cast<const f32x4*>(pa + 64 * k);
        }
    };
    auto read_b = [&](int t, RawB& r) {
        const char* pb = lds + (t % kD) * kSlot + kAImg + 8 * h * RSB + (32 * VB * wb + VB * c) * 4;
#pragma unroll
        for (int k = 0; k < 8; ++k) r.v[k] = *reinterpret_cast<const BV*>(pb + k * RSB);
    };
    // stage t's gradient rows, once per stage: their bias sums (the four row
    // tiles at once, in packed fp32 pairs; wb == 0 writes them), then the rows
    // times sca in place (packed too), so the splits below take them as they are
    // (a stage's sums enter bsv one stage later, so those of stage nst -- the
    // clamped read past the end -- never do, without a branch)
    f32x4 bpend = {0.f, 0.f, 0.f, 0.f};
    auto prep_sum = [&](const RawA& r) {
        if constexpr (MA > 0) {
            f32x4 sum = r.v[0];
#pragma unroll
            for (int k = 1; k < 8; ++k) sum += r.v[k];
            bsv += bpend;
            bpend = sum;
        }
    };
    auto prep_scale = [&](RawA& r) {
        if constexpr (MA > 0)
#pragma unroll
            for (int k = 0; k < 8; ++k) r.v[k] *= sca;
    };
    auto prep_a = [&](int t, RawA& r) {
        (void)t;
        prep_sum(r);
        prep_scale(r);
    };
    // the head tile (HD) of stage t: its 8 values (read) and its pieces (split)
    auto read_h = [&](int t, float (&x)[8]) {
        const float* ph = reinterpret_cast<const float*>(lds + (t % kD) * kSlot + kAImg + kBImg + 128 * h) +
                          (c & 3);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float v = ph[4 * k];
            x[k] = c < 4 ? v : 0.f;
        }
    };
    auto split_h = [&](const float (&x)[8], x3::Pieces& f) {
        float sum = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) sum += x[k];
        hs += sum;
        split8(x, sch, f);
    };
    auto split_a_raw = [&](int t, const RawA& r, int i, x3::Pieces& f) {
        if (HD && i == HT) { split_a(t, i, f); return; }
        if constexpr (MA > 0) {
            float x[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = r.v[k][i & 3];
            split8(x, 1.f, f);
        }
    };
    auto split_b_raw = [&](const RawB& r, int j, x3::Pieces& f) {
        float x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = vget<VB>(r.v[k], j);
        split8(x, 1.f, f);
    };

    // (nst == 0: the clamped, bounds-checked DMAs of block b0 run, nothing is
    // multiplied and the slab is written as zeros)
    {
        if constexpr (GA) {
#pragma unroll 1
            for (int u = 0; u < 2 * kD - 1; ++u) idx_dma(u);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
#pragma unroll
        for (int t = 0; t < kD; ++t) issue(t);
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((kD - 1) * KV) : "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        mask_tail(0);
        // pieces of the stage being multiplied: row tiles fa (each rewritten with
        // the next stage's right after its MFMAs issued), column tiles fb / fn
        // (the next stage's go to the other set: every row tile still reads them)
        // every wave multiplies (a wave outside the grid reads in-bounds LDS
        // and writes nothing): no branch around the accumulators
        x3::Pieces fa[TA], fb[VB], fn[VB];
        // PH: the phased stage below (row tiles > 1, uniform input rows);
        // else every split of stage s + 1 follows the row tile that frees it
        constexpr bool PH = TA > 1 && RPI == 1;
        RawA rA, rB;
        int4 iv = rows_raw(kD);
        {
            RawB q0;
            read_a(0, rA);
            read_b(0, q0);
            prep_a(0, rA);
#pragma unroll
            for (int i = 0; i < (PH ? TA - 1 : TA); ++i) split_a_raw(0, rA, i, fa[i]);
#pragma unroll
            for (int j = 0; j < VB; ++j) split_b_raw(q0, j, fb[j]);
        }
        // stage s: fa x cur, then stage s + 1 split into fa and nxt (the two
        // column-piece sets trade roles from stage to stage: no copies)
        auto stage = [&](int s, x3::Pieces (&cur)[VB], x3::Pieces (&nxt)[VB]) {
            // stage s + 1 landed (every wave's DMA) and stage s's slot is no longer read
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((kD - 2) * KV) : "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            mask_tail(s + 1);
            // stage s + kD's DMA goes out between this stage's MFMAs (its list
            // entries read first: one LDS read, used a row tile later)
            const Rows rw = rows_of(s + kD);
            RawA ra1;
            RawB rb1;
            if (NR_W4_DBG != 3) { read_a(s + 1, ra1); read_b(s + 1, rb1); }
            // row tile i: its MFMAs (products outermost: VB independent
            // accumulators between dependent ones), a share of the DMA, then
            // the split of the next stage's column tiles (i = 0) or of row tile
            // i - 1 (whose MFMAs have issued)
#pragma unroll
            for (int i = 0; i < TA; ++i) {
#pragma unroll
                for (int p = 0; p < 3; ++p)
#pragma unroll
                    for (int j = 0; j < VB; ++j) {
                        if (NR_W4_DBG == 1) { asm volatile("" ::"v"(fa[i].lo), "v"(fa[i].hi), "v"(cur[j].lo), "v"(cur[j].hi)); continue; }
                        acc[i][j] = p == 0 ? x3::mfma32(fa[i].lo, cur[j].hi, acc[i][j])
                                  : p == 1 ? x3::mfma32(fa[i].hi, cur[j].lo, acc[i][j])
                                           : x3::mfma32(fa[i].hi, cur[j].hi, acc[i][j]);
                        asm volatile("" : "+a"(acc[i][j]));   // accumulators stay in AGPRs
                    }
#pragma unroll
                for (int k = i * KV / TA; k < (i + 1) * KV / TA; ++k)
                    if (NR_W4_DBG != 2) issue_k(s + kD, k, rw);
                if (NR_W4_DBG == 3) continue;
                if (i == 0) {
#pragma unroll
                    for (int j = 0; j < VB; ++j) split_b_raw(rb1, j, nxt[j]);
                    prep_a(s + 1, ra1);
                } else {
                    split_a_raw(s + 1, ra1, i - 1, fa[i - 1]);
                }
            }
            if (NR_W4_DBG == 3) return;
            split_a_raw(s + 1, ra1, TA - 1, fa[TA - 1]);
        };
        // PH: stage s's reads (the head's values, then stage s + 1's input and
        // gradient rows) all go out before the first MFMA, and the VALU work
        // rides between the MFMAs, each piece after the MFMA that frees its
        // registers and late enough that its reads have landed -- tile 0: the
        // split of stage s's last row tile (deferred from stage s - 1: its raw
        // values stay in registers; HD: the head tile); tile 1: stage s + 1's
        // column tiles; tile 2: its bias sums, scaling and row tiles 0, 1; tile
        // i > 2: row tile i - 1.  A sched_barrier before every MFMA fixes the
        // interleave.  The next stage's list entries are read last (the
        // top-of-stage wait covers that read).
        auto stage_ph = [&](int s, x3::Pieces (&cur)[VB], x3::Pieces (&nxt)[VB], RawA& rc, RawA& rn) {
            if constexpr (PH) {
                asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((kD - 2) * KV) : "memory");
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
                mask_tail(s + 1);
                const Rows rw = rows_take(s + kD, iv);
                float xh[8];
                if constexpr (HD) read_h(s, xh);
                RawB rb1;
                read_b(s + 1, rb1);
                read_a(s + 1, rn);
                // the VALU work after MFMA m of row tile i (NM per tile), each
                // result pinned where it is made: later passes would otherwise
                // sink it past the next stage's mask_tail branch
                constexpr int NM = 3 * VB;
                // (and its inputs pinned there too: the selector would hoist
                // it above the MFMAs otherwise)
                auto work = [&](int i, int m) {
                    if (i == 0 && m == 0) {
                        if constexpr (HD) {
#pragma unroll
                            for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(xh[k]));
                            split_h(xh, fa[TA - 1]);
                        } else {
#pragma unroll
                            for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(rc.v[k]));
                            split_a_raw(s, rc, TA - 1, fa[TA - 1]);
                        }
                        x3::pin(fa[TA - 1]);
                    } else if (i == 1 && m % 3 == 0) {
                        if (m == 0)
#pragma unroll
                            for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(rb1.v[k]));
                        split_b_raw(rb1, m / 3, nxt[m / 3]);
                        x3::pin(nxt[m / 3]);
                    } else if (i == 2 && m == 0) {
#pragma unroll
                        for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(rn.v[k]));
                        prep_sum(rn);
                        asm volatile("" : "+v"(bsv), "+v"(bpend));
                    } else if (i == 2 && m == 1) {
                        prep_scale(rn);
#pragma unroll
                        for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(rn.v[k]));
                    } else if (i == 2 && (m == NM / 3 || m == 2 * NM / 3)) {
                        const int t = m == NM / 3 ? 0 : 1;
                        split_a_raw(s + 1, rn, t, fa[t]);
                        x3::pin(fa[t]);
                    } else if (i > 2 && m == 0) {
                        split_a_raw(s + 1, rn, i - 1, fa[i - 1]);
                        x3::pin(fa[i - 1]);
                    }
                    if (m == 1)
#pragma unroll
                        for (int k = i * KV / TA; k < (i + 1) * KV / TA; ++k) issue_k(s + kD, k, rw);
                    if (i == TA - 1 && m == NM - 1) iv = rows_raw(s + 1 + kD);
                };
#pragma unroll
                for (int i = 0; i < TA; ++i)
#pragma unroll
                    for (int p = 0; p < 3; ++p)
#pragma unroll
                        for (int j = 0; j < VB; ++j) {
                            __builtin_amdgcn_sched_barrier(0);
                            acc[i][j] = p == 0 ? x3::mfma32(fa[i].lo, cur[j].hi, acc[i][j])
                                      : p == 1 ? x3::mfma32(fa[i].hi, cur[j].lo, acc[i][j])
                                               : x3::mfma32(fa[i].hi, cur[j].hi, acc[i][j]);
                            asm volatile("" : "+a"(acc[i][j]));
                            work(i, p * VB + j);
                        }
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        // (nst is even: two stages per 32-sample block)
#pragma unroll 1
        for (int s = 0; s < nst; s += 2) {
            if constexpr (PH) {
                stage_ph(s, fb, fn, rA, rB);
                stage_ph(s + 1, fn, fb, rB, rA);
            } else {
                stage(s, fb, fn);
                stage(s + 1, fn, fb);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the clamped DMAs past the end
    }
    if (!active) return;
    // bias sums: lanes c (h = 0, 1: samples 0..7, 8..15 of each stage)
#pragma unroll
    for (int i = 0; i < 4; ++i) bsv[i] += __shfl_xor(bsv[i], 32);
    hs += __shfl_xor(hs, 32);
    if (wb == 0 && h == 0) {
        if constexpr (MA > 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) slab[MA * WB + 128 * wa + 4 * c + i] = bsv[i];
        }
        if constexpr (HD) if (c < 4) hslab[4 * WB + c] = hs;
    }
    // tile (i, j) to slab rows 128 wa + 32 i + rho, columns 32 VB wb + 32 j + c
    // (the natural row 128 wa + 4 rho + i, column 32 VB wb + VB c + j: w4_unperm)
#pragma unroll
    for (int i = 0; i < TA; ++i)
#pragma unroll
        for (int j = 0; j < VB; ++j) {
            const f32x16 v = acc[i][j];
            const int cc = 32 * VB * wb + 32 * j + c;
            float* dst = HD && i == HT ? hslab + cc : slab + (128 * wa + 32 * i) * WB + cc;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int rho = nr_acc_row(r, h);
                if (!(HD && i == HT) || rho < 4) dst[rho * WB] = v[r];
            }
        }
}

// GA: gathered input rows (the *_active entry points), else by position
template <bool GA>
__global__ void __launch_bounds__(w4::kT, 1) wgrad4_kernel(WgArgs a) {
    __shared__ __attribute__((aligned(16))) char lds[w4::kLds];
    int t = 0;
#pragma unroll 1
    while (t + 1 < kTasks && (int)blockIdx.x >= a.wg_start[t + 1]) ++t;
    const int c = blockIdx.x - a.wg_start[t];
    const WgTask& T = a.task[t];
    const int nact = wg_nact(a);
    const int b0 = (int)((int64_t)c * nact / T.G);
    const int b1 = (int)((int64_t)(c + 1) * nact / T.G);
    float* slab = a.slab + T.slab + (int64_t)c * (T.a.width * T.b.width + T.a.width);
    const int fu = __builtin_amdgcn_readfirstlane(T.fuse);
    float* xslab = nullptr;
    if (fu >= 0) {
        const WgTask& P = a.task[fu];
        xslab = a.slab + P.slab + (int64_t)c * (P.a.width * P.b.width + P.a.width);
    }
    switch (__builtin_amdgcn_readfirstlane(T.id)) {
        case 0: case 4:     // DZ x PE
            wgrad4_body<GA, 256, false, 64, 1, 2, 2>(a, T, b0, b1, lds, slab, xslab); break;
        case 10:            // dz_dir x h8 (the dir layer's feat columns as G) [+ the sigma head, task 12]
            if (fu >= 0) wgrad4_body<GA, 128, true, 256, 2, 1, 4>(a, T, b0, b1, lds, slab, xslab);
            else wgrad4_body<GA, 128, false, 256, 2, 1, 4>(a, T, b0, b1, lds, slab, xslab);
            break;
        case 11:            // dz_dir x dir PE
            wgrad4_body<GA, 128, false, 32, 1, 1, 1>(a, T, b0, b1, lds, slab, xslab); break;
        case 12:            // head x h8
            wgrad4_body<GA, 0, true, 256, 2, 1, 4>(a, T, b0, b1, lds, slab, xslab); break;
        case 13:            // head x hdir
            wgrad4_body<GA, 0, true, 128, 1, 1, 4>(a, T, b0, b1, lds, slab, xslab); break;
        default:            // DZ x h
            wgrad4_body<GA, 256, false, 256, 4, 2, 2>(a, T, b0, b1, lds, slab, xslab); break;
    }
}
#endif  // NR_F16

// Embedding channel of bf16x6 PE slot q (packing._pe16_channel / _dir16_channel)
__device__ __forceinline__ int pe16_channel(int q) {
    if (q == 58 || q == 59) return q - 58;
    if (q == 62) return 2;
    const int c = q >> 3, j = q & 7, m = 4 * c + (j & 3);
    if (m >= 30) return -1;
    return (j < 4 ? 3 : 6) + 6 * (m / 3) + m % 3;
}
__device__ __forceinline__ int dir16_channel(int q) {
    const int g = q >> 3, j = q & 7;
    if (j == 3) return g < 3 ? g : -1;
    if (j == 7) return -1;
    return (j < 4 ? 3 : 6) + 6 * g + (j & 3);
}

// destination of output element (o, c) of task t in the flat gradient (-1 = none)
__device__ int wgrad_dest(int t, int o, int c, bool x3) {
    switch (t) {
        case 0: { const int f = x3 ? pe16_channel(c) : pe_feature(c & 31, c >> 5, 15);
                  return f < 0 ? -1 : kP.w[0] + o * kP.fan[0] + f; }
        case 1: case 2: case 3: return kP.w[t] + o * kP.fan[t] + c;
        case 4: { const int f = x3 ? pe16_channel(c) : pe_feature(c & 31, c >> 5, 15);
                  return f < 0 ? -1 : kP.w[4] + o * kP.fan[4] + f; }
        case 5: return kP.w[4] + o * kP.fan[4] + NR_XYZ_CH + c;
        case 6: case 7: case 8: case 9: return kP.w[t - 1] + o * kP.fan[t - 1] + c;
        case 10: return kP.w[9] + o * kP.fan[9] + c;
        case 11: { const int f = x3 ? dir16_channel(c) : pe_feature(c & 15, c >> 4, 6);
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

#if NR_F16
// stats[l] = max over the per-wave maxima [l][nb] written by mlp_bwd3.hip;
// 1024 threads per segment, four independent loads in flight per thread (the
// max is order-independent: the result does not depend on the schedule)
constexpr int kStatT = 1024;
__global__ void __launch_bounds__(kStatT) stats_reduce_kernel(float* __restrict__ stats, int nb) {
    const int l = blockIdx.x;
    const float* w = stats + NR_STATS + (int64_t)l * nb;
    float m0 = 0.f, m1 = 0.f, m2 = 0.f, m3 = 0.f;
    int i = threadIdx.x;
    for (; i + 3 * kStatT < nb; i += 4 * kStatT) {
        m0 = fmaxf(m0, w[i]);
        m1 = fmaxf(m1, w[i + kStatT]);
        m2 = fmaxf(m2, w[i + 2 * kStatT]);
        m3 = fmaxf(m3, w[i + 3 * kStatT]);
    }
    for (; i < nb; i += kStatT) m0 = fmaxf(m0, w[i]);
    float m = fmaxf(fmaxf(m0, m1), fmaxf(m2, m3));
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) m = fmaxf(m, __shfl_xor(m, d));
    __shared__ float red[kStatT / 64];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < kStatT / 64; ++k) m = fmaxf(m, red[k]);
        stats[l] = m;
    }
}
#endif

__global__ void wgrad_reduce_kernel(WgArgs a, float* __restrict__ grad) {
    const int t = blockIdx.y;
    const WgTask& T = a.task[t];
    const int M = T.a.width, N = T.b.width;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    const int nw = M * N, sz = nw + M;
    if (e >= sz) return;
    const int dst = e < nw ? wgrad_dest(T.id, w4_unperm(e / N, T.pa), w4_unperm(e % N, T.pb), a.x3)
                           : wgrad_bias_dest(T.id, e - nw);
    if (dst < 0) return;
    // 8 independent partial sums (fixed order: bitwise reproducible) keep 8
    // slab loads in flight per thread instead of one dependent chain
    const float* p = a.slab + T.slab + e;
    float q[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int w = 0;
    for (; w + 8 <= T.G; w += 8, p += 8 * (int64_t)sz)
#pragma unroll
        for (int i = 0; i < 8; ++i) q[i] += p[(int64_t)i * sz];
    for (int i = 0; w < T.G; ++w, ++i, p += sz) q[i] += *p;
    float s = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
    if (e < nw) s /= task_scale(a, T);    // exact: a power of two
    grad[dst] = s;
}

}  // namespace

#if NR_X3_BASE_OBJECT
// dir_encoding.0.weight's first 256 columns (the xyz_encoding_final input,
// nerf.py:118): the weight-gradient launch leaves G = sum_s dz_dir h8^T there
// (task 10); the gradient of the reference's dW = sum_s dz_dir feat^T with
// feat = W_final h8 + b_final is G W_final^T + db_dir b_final^T.  One
// workgroup per output row (in place: a row reads only itself), fp32 fma
// chains over k in order.
__global__ void __launch_bounds__(256) dir_feat_kernel(const float* __restrict__ params,
                                                       float* __restrict__ grad) {
    __shared__ float g[256];
    const int o = blockIdx.x, c = threadIdx.x;
    constexpr int kFan = 283;                       // dir_encoding.0 fan-in
    float* row = grad + kP.w[9] + o * kFan;
    g[c] = row[c];
    __syncthreads();
    const float* w = params + kP.w[8] + c * 256;    // xyz_encoding_final.weight row c
    float acc = 0.f;
#pragma unroll 8
    for (int k = 0; k < 256; ++k) acc = fmaf(g[k], w[k], acc);
    row[c] = fmaf(grad[kP.b[9] + o], params[kP.b[8] + c], acc);
}

// xyz_encoding_final (nerf.py:116): dW = W_dir[:, :256]^T G, db = W_dir[:, :256]^T db_dir
// (dfeat = W_dir[:, :256]^T dz_dir is not stored).  Runs before dir_feat_kernel
// rewrites G.  Workgroup c = output row, thread k = column; fp32 fma chains over
// the 128 dir outputs in order.
__global__ void __launch_bounds__(256) final_from_g_kernel(const float* __restrict__ params,
                                                          float* __restrict__ grad) {
    const int c = blockIdx.x, k = threadIdx.x;
    constexpr int kFan = 283;
    const float* G = grad + kP.w[9];                 // G[o][k] at o * 283 + k
    const float* W = params + kP.w[9];               // W_dir[o][c] at o * 283 + c
    float acc = 0.f, b = 0.f;
#pragma unroll 8
    for (int o = 0; o < 128; ++o) {
        const float w = W[o * kFan + c];
        acc = fmaf(w, G[o * kFan + k], acc);
        if (k == 0) b = fmaf(w, grad[kP.b[9] + o], b);
    }
    grad[kP.w[8] + c * 256 + k] = acc;
    if (k == 0) grad[kP.b[8] + c] = b;
}

NR_API int nr_wgrad_dir_feat(const float* params, float* grad_flat, void* stream) {
    NR_REQUIRE(params && grad_flat, "nr_wgrad_dir_feat: null pointer");
    final_from_g_kernel<<<256, 256, 0, (hipStream_t)stream>>>(params, grad_flat);
    NR_LAUNCH_CHECK("nr_wgrad_dir_feat");
    dir_feat_kernel<<<128, 256, 0, (hipStream_t)stream>>>(params, grad_flat);
    NR_LAUNCH_CHECK("nr_wgrad_dir_feat");
    return 0;
}

NR_API int64_t nr_wgrad_workspace_bytes(int64_t n) {
    (void)n;
    // upper bound of sum_t G_t * (M_t N_t + M_t) for the task list below
    return (int64_t)(3 * kTargetWGMax + kTasks) * (256 * 256 + 256) * sizeof(float);
}
#endif

namespace {
// slist / scount: the launch covers positions 0 .. *scount of the buffers; with
// gather the input operands are gathered from sample slist[q] (the *_active
// entry points), else they were saved by position (the *_listed ones)
int wgrad_launch(bool x3, bool sigma_only, const float* save, const float* grad_ws, int64_t n,
                 float* workspace, float* grad_flat, void* stream,
                 const int32_t* slist = nullptr, const int32_t* scount = nullptr,
                 bool gather = true) {
    const char* name = sigma_only ? "nr_wgrad_sigma" : "nr_wgrad";
    NR_REQUIRE(n >= 0 && n < (int64_t)1 << 31, "%s: n out of range", name);
    NR_REQUIRE(save && grad_ws && workspace && grad_flat, "%s: null pointer", name);
    NR_REQUIRE((((uintptr_t)save | (uintptr_t)grad_ws) & 15) == 0,
               "nr_wgrad: save/grad_ws must be 16-byte aligned");
    hipStream_t st = (hipStream_t)stream;
    if (n == 0) {
        hipError_t e = hipMemsetAsync(grad_flat, 0, 595844 * sizeof(float), st);
        if (e != hipSuccess) { nr_set_error("nr_wgrad: memset failed"); return (int)e; }
        return 0;
    }
    const int64_t nb = (n + 31) / 32;          // blocks holding samples (the work)
    const int64_t nbp = nr_blocks_pad(n);      // segment stride of the buffers
    float* SV = const_cast<float*>(save);
    float* GD = const_cast<float*>(grad_ws);
    auto acc = [](float* p, int w) { return WgSeg{p, SEG_ACC, w}; };
    const WgSeg pe{SV, SEG_PE, 64}, dpe{SV + nr_sv_dirpe(nbp), SEG_DPE, 32};
    const WgSeg head{GD + nr_gd_dhead(nbp), SEG_HEAD, 4};
    auto H = [&](int l) { return acc(SV + nr_sv_h(l, nbp), 256); };
    auto DZ = [&](int l) { return acc(GD + nr_gd_dz(l, nbp), 256); };
    // task 10 (dir_encoding's feat columns) reads h8, not xyz_encoding_final's
    // output: dW = sum dz_dir feat^T = G W_final^T + db_dir b_final^T with
    // G = sum dz_dir h8^T (nerf.py:116, feat = W_final h8 + b_final), so the
    // forward saves no feat.  And task 9 (xyz_encoding_final) launches nothing:
    // its dW = sum dfeat h8^T with dfeat = W_dir[:, :256]^T dz_dir is
    // W_dir[:, :256]^T G (db = W_dir[:, :256]^T db_dir), so the data gradient
    // stores no dfeat either.  nr_wgrad_dir_feat forms both from G
    // (DESIGN.md 13); task 9's entry keeps the id order (its slot: a dummy)
    const WgSeg hdir = acc(SV + nr_sv_hdir(nbp), 128);
    const WgSeg dzdir = acc(GD + nr_gd_dzdir(nbp), 128);
    // (a, b, wm, wn); task order fixes wgrad_dest / wgrad_bias_dest
    const WgTask tasks[kTasks] = {
        {DZ(0), pe, 8, 1}, {DZ(1), H(0), 2, 4}, {DZ(2), H(1), 2, 4}, {DZ(3), H(2), 2, 4},
        {DZ(4), pe, 8, 1}, {DZ(4), H(3), 2, 4}, {DZ(5), H(4), 2, 4}, {DZ(6), H(5), 2, 4},
        {DZ(7), H(6), 2, 4}, {DZ(0), H(7), 2, 4} /* 9: dummy, no workgroups */,
        {dzdir, H(7), 2, 4}, {dzdir, dpe, 4, 1},
        {head, H(7), 1, 8}, {head, hdir, 1, 4},
    };
    WgArgs a{};
    // per-block cost of a task's workgroup, in cycles: the MFMA time of its
    // busiest SIMD (fp32: 16 k-steps x 64 cycles per tile; bf16x6: 2 x 6 x 32),
    // or the staging of (M + N) x 32 floats at ~8 B/cycle per CU, plus a fixed
    // barrier/LDS-store overhead
    int64_t cost[kTasks], tot = 0;
    for (int t = 0; t < kTasks; ++t) {
        const int mt = (tasks[t].a.width / tasks[t].wm + 31) / 32;
        const int nt = (tasks[t].b.width / tasks[t].wn + 31) / 32;
        const int64_t per_tile = x3 ? 64 * x3::kNProd : 1024;
        const int64_t mfma = per_tile * mt * nt * (tasks[t].wm * tasks[t].wn > 4 ? 2 : 1);
        const int64_t bytes = (int64_t)(tasks[t].a.width + tasks[t].b.width) * 32 * 4;
        cost[t] = std::max<int64_t>(mfma, bytes / 8) + 512;
        tot += cost[t];
    }
    // dispatch order: the heavy tasks first; the small ones last and split ~3x
    // finer, so their short workgroups fill the tail of the final round
    const int64_t heavy = x3 ? 1024 * x3::kNProd : 16384;
    int order[kTasks], no = 0;
    for (int pass = 0; pass < 2; ++pass)
        for (int t = 0; t < kTasks; ++t)
            if ((cost[t] >= heavy) == (pass == 0)) order[no++] = t;
    a.wg_start[0] = 0;
    int64_t slab = 0;
    // diagnostic: NR_WGRAD_TASKMASK limits the launch to a subset of task ids
    // (the kernel code is unchanged; gradients of the other tasks are then stale)
    // gradient operand's stats slot (layout.h NR_STATS) of every task id
    static const int kStat[kTasks] = {0, 1, 2, 3, 4, 4, 5, 6, 7, 8, 9, 9, 10, 10};
    static const long long tmask_env =
        getenv("NR_WGRAD_TASKMASK") ? strtoll(getenv("NR_WGRAD_TASKMASK"), nullptr, 0) : -1;
    // the sigma-only graph (rendering_shadows.py:167) has no xyz_encoding_final
    // (task 9), dir_encoding (10, 11) or rgb head (13): their gradients are not
    // computed (written as 0; the autograd leaves them None)
    const long long tmask = sigma_only ? (tmask_env & ~((1LL << 9) | (1LL << 10) | (1LL << 11) | (1LL << 13)))
                                       : tmask_env;
    // every launch over a sample list -- gathering (*_active) or over buffers
    // saved by position (*_listed, the deferred save) -- uses the same split-K
    // partition, so the two give bit-identical sums
    // f16x3, full graph: the LDS-DMA weight gradient (wgrad4_kernel; NR_W4=0 at
    // build time: the register-staged wgrad3_kernel).  32-bit buffer offsets:
    // every segment it reads stays under 2 GiB below 2M samples.
    // NR_WGRAD_W4=0 in the environment: the register-staged kernel, for A/B
    // runs and the cross-check test (read per launch)
    const char* w4_env = getenv("NR_WGRAD_W4");
    const bool use_w4 = NR_F16 && NR_W4 && !sigma_only && n < ((int64_t)1 << 21) &&
                        !(w4_env && atoi(w4_env) == 0);
    const int64_t target_wg = !slist ? kTargetWG : (use_w4 ? NR_WGRAD_TARGET_WG_W4 : NR_WGRAD_TARGET_WG_GA);
    int64_t gt[kTasks];
    int pos[kTasks];
    for (int k = 0; k < kTasks; ++k) {
        const int t = order[k];
        // the 4-row head tasks' per-block time is mostly fixed cost, not
        // bytes: always split finer, so they fill the tail of the last round
        const int split = cost[t] >= heavy && tasks[t].a.kind != SEG_HEAD ? 1 : 3;
        int64_t g = split * ((target_wg * cost[t] + tot - 1) / tot);
        gt[t] = std::max<int64_t>(1, std::min<int64_t>(g, nb));
        if (!((tmask >> t) & 1) || t == 9) gt[t] = 0;   // task 9: nr_wgrad_dir_feat
        pos[t] = k;
    }
    // f16x3: the tasks that read the same saved segment run fused (kFuse,
    // wgrad3_body's extra operand): the primary's workgroups also compute the
    // partner's output over the same block ranges into the partner's slabs, so
    // DZ(4), H(7) and dz_dir (2.5 KB/sample) are read once.  The partner keeps
    // its slabs and its reduction but launches no workgroups of its own.
    // (round 5: task 9, xyz_encoding_final = DZ(8) x H(7), launches nothing --
    // its gradient is W_dir[:, :256]^T G, nr_wgrad_dir_feat -- so the sigma
    // head pairs with task 10, which reads H(7) too)
    static const int kFused[2][2] = {{5, 4}, {10, 12}};   // {primary, partner}
    static const bool fuse_on = !getenv("NR_WGRAD_FUSE") || atoi(getenv("NR_WGRAD_FUSE")) != 0;
    int partner[kTasks];
    bool absorbed[kTasks];
    for (int t = 0; t < kTasks; ++t) { partner[t] = -1; absorbed[t] = false; }
    if (kFuse && x3 && fuse_on && (tmask_env == -1)) {
        // launches over a sample list have their own pair set (see target_wg)
        // (wgrad4_kernel fuses the sigma head into task 10 only)
        const int fmask = use_w4 ? 2
                        : (slist && !NR_BF1) ? (NR_WGRAD_FUSE_MASK & NR_WGRAD_FUSE_MASK_GA)
                                             : NR_WGRAD_FUSE_MASK;
        for (int i = 0; i < 2; ++i) {
            if (!((fmask >> i) & 1)) continue;
            const auto& pr = kFused[i];
            if (!((tmask >> pr[0]) & 1) || !((tmask >> pr[1]) & 1)) continue;   // both must run
            gt[pr[1]] = gt[pr[0]] = std::max<int64_t>(1, std::min<int64_t>(
                (target_wg * (cost[pr[0]] + cost[pr[1]]) + tot - 1) / tot, nb));
            partner[pr[0]] = pr[1];
            absorbed[pr[1]] = true;
        }
    }
    for (int k = 0; k < kTasks; ++k) {
        const int t = order[k];
        const int64_t g = gt[t];
        a.task[k] = tasks[t];
        a.task[k].id = t;
        a.task[k].stat = kStat[t];
        a.task[k].G = (int)g;
        a.task[k].slab = slab;
        a.task[k].fuse = partner[t] >= 0 ? pos[partner[t]] : -1;
        // wgrad4_kernel's slab orders: gradient rows 4-interleaved (not the head's), input
        // columns VB-interleaved (its dispatch below)
        static const int kW4Pa[kTasks] = {4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 1, 1};
        static const int kW4Pb[kTasks] = {1, 4, 4, 4, 1, 4, 4, 4, 4, 4, 2, 1, 2, 1};
        a.task[k].pa = use_w4 ? kW4Pa[t] : 1;
        a.task[k].pb = use_w4 ? kW4Pb[t] : 1;
        slab += g * (tasks[t].a.width * tasks[t].b.width + tasks[t].a.width);
        a.wg_start[k + 1] = a.wg_start[k] + (absorbed[t] ? 0 : (int)g);
    }
    a.nb = (int)nb;
    a.n = (int)n;
    a.slab = workspace;
    a.x3 = x3;
    a.stats = NR_F16 ? SV + nr_sv_stats(nbp) : nullptr;
    a.slist = slist;
    a.scount = scount;
#if NR_F16
    stats_reduce_kernel<<<NR_STAT_SEGS, kStatT, 0, st>>>(SV + nr_sv_stats(nbp), (int)nbp);
    NR_LAUNCH_CHECK("nr_wgrad_stats");
    if (use_w4 && slist && gather) wgrad4_kernel<true><<<a.wg_start[kTasks], w4::kT, 0, st>>>(a);
    else if (use_w4) wgrad4_kernel<false><<<a.wg_start[kTasks], w4::kT, 0, st>>>(a);
    else if (slist && gather && !sigma_only) wgrad3_kernel<true, true><<<a.wg_start[kTasks], kThreads, 0, st>>>(a);
    else if (slist && gather) wgrad3_kernel<true, false><<<a.wg_start[kTasks], kThreads, 0, st>>>(a);
    else if (!sigma_only) wgrad3_kernel<false, true><<<a.wg_start[kTasks], kThreads, 0, st>>>(a);
    else wgrad3_kernel<false, false><<<a.wg_start[kTasks], kThreads, 0, st>>>(a);
#elif NR_BF1
    wgrad3_kernel<false, false><<<a.wg_start[kTasks], kThreads, 0, st>>>(a);
#else
    if (x3 && slist && gather && !sigma_only) wgrad3_kernel<true, true><<<a.wg_start[kTasks], kThreads, 0, st>>>(a);
    else if (x3 && slist && gather) wgrad3_kernel<true, false><<<a.wg_start[kTasks], kThreads, 0, st>>>(a);
    else if (x3 && !sigma_only) wgrad3_kernel<false, true><<<a.wg_start[kTasks], kThreads, 0, st>>>(a);
    else if (x3) wgrad3_kernel<false, false><<<a.wg_start[kTasks], kThreads, 0, st>>>(a);
    // the full graph's inputs are sample-major rows (mlp_fwd.hip ROWS), the
    // sigma-only graph's block-native
    else if (slist && gather && !sigma_only && NR_F32_ROWS) wgrad_kernel<true, true><<<a.wg_start[kTasks], kThreads, 0, st>>>(a);
    else if (slist && gather) wgrad_kernel<true, false><<<a.wg_start[kTasks], kThreads, 0, st>>>(a);
    else if (!sigma_only && NR_F32_ROWS) wgrad_kernel<false, true><<<a.wg_start[kTasks], kThreads, 0, st>>>(a);
    else wgrad_kernel<false, false><<<a.wg_start[kTasks], kThreads, 0, st>>>(a);
#endif
    NR_LAUNCH_CHECK("nr_wgrad");
    dim3 rg((256 * 256 + 256 + 255) / 256, kTasks);
    wgrad_reduce_kernel<<<rg, 256, 0, st>>>(a, grad_flat);
    NR_LAUNCH_CHECK("nr_wgrad_reduce");
    return 0;
}
}  // namespace

#if NR_X3_BASE_OBJECT
NR_API int nr_wgrad(const float* save, const float* grad_ws, int64_t n, float* workspace,
                    float* grad_flat, void* stream) {
    return wgrad_launch(false, false, save, grad_ws, n, workspace, grad_flat, stream);
}
// the exact-fp32 arithmetic's sigma-only and sample-list twins (as the split
// arithmetics' below)
NR_API int nr_wgrad_sigma(const float* save, const float* grad_ws, int64_t n, float* workspace,
                          float* grad_flat, void* stream) {
    return wgrad_launch(false, true, save, grad_ws, n, workspace, grad_flat, stream);
}
NR_API int nr_wgrad_active(const float* save, const float* grad_ws, int64_t n, float* workspace,
                           float* grad_flat, const int32_t* samples, const int32_t* count,
                           void* stream) {
    NR_REQUIRE(samples && count, "nr_wgrad_active: null sample list");
    return wgrad_launch(false, false, save, grad_ws, n, workspace, grad_flat, stream, samples, count);
}
NR_API int nr_wgrad_sigma_active(const float* save, const float* grad_ws, int64_t n,
                                 float* workspace, float* grad_flat, const int32_t* samples,
                                 const int32_t* count, void* stream) {
    NR_REQUIRE(samples && count, "nr_wgrad_sigma_active: null sample list");
    return wgrad_launch(false, true, save, grad_ws, n, workspace, grad_flat, stream, samples, count);
}
NR_API int nr_wgrad_listed(const float* save, const float* grad_ws, int64_t n, float* workspace,
                           float* grad_flat, const int32_t* samples, const int32_t* count,
                           void* stream) {
    NR_REQUIRE(samples && count, "nr_wgrad_listed: null sample list");
    return wgrad_launch(false, false, save, grad_ws, n, workspace, grad_flat, stream, samples, count,
                        false);
}
NR_API int nr_wgrad_sigma_listed(const float* save, const float* grad_ws, int64_t n,
                                 float* workspace, float* grad_flat, const int32_t* samples,
                                 const int32_t* count, void* stream) {
    NR_REQUIRE(samples && count, "nr_wgrad_sigma_listed: null sample list");
    return wgrad_launch(false, true, save, grad_ws, n, workspace, grad_flat, stream, samples, count,
                        false);
}
#endif

NR_API int NR_X3_NAME(nr_wgrad)(const float* save, const float* grad_ws, int64_t n, float* workspace,
                       float* grad_flat, void* stream) {
    return wgrad_launch(true, false, save, grad_ws, n, workspace, grad_flat, stream);
}

// the sigma-only graph's weight gradients (after nr_mlp_bwd_sigma*): every
// layer up to xyz_encoding_8 and the sigma head; the other parameters get 0
NR_API int NR_X3_NAME(nr_wgrad_sigma)(const float* save, const float* grad_ws, int64_t n,
                             float* workspace, float* grad_flat, void* stream) {
    return wgrad_launch(true, true, save, grad_ws, n, workspace, grad_flat, stream);
}

#if !NR_BF1
// over the samples nr_active_samples listed (after nr_mlp_bwd*_active with the
// same list); the other samples' output gradients are exactly zero, so the
// sums are those of nr_wgrad* up to the order of the split-K partial sums
NR_API int NR_X3_NAME(nr_wgrad_active)(const float* save, const float* grad_ws, int64_t n,
                                       float* workspace, float* grad_flat, const int32_t* samples,
                                       const int32_t* count, void* stream) {
    NR_REQUIRE(samples && count, "nr_wgrad_active: null sample list");
    return wgrad_launch(true, false, save, grad_ws, n, workspace, grad_flat, stream, samples, count);
}
NR_API int NR_X3_NAME(nr_wgrad_sigma_active)(const float* save, const float* grad_ws, int64_t n,
                                             float* workspace, float* grad_flat,
                                             const int32_t* samples, const int32_t* count,
                                             void* stream) {
    NR_REQUIRE(samples && count, "nr_wgrad_sigma_active: null sample list");
    return wgrad_launch(true, true, save, grad_ws, n, workspace, grad_flat, stream, samples, count);
}
// over the first *count positions of buffers written by position
// (nr_mlp_fwd_listed* + nr_mlp_bwd*_listed, the deferred save)
NR_API int NR_X3_NAME(nr_wgrad_listed)(const float* save, const float* grad_ws, int64_t n,
                                       float* workspace, float* grad_flat, const int32_t* samples,
                                       const int32_t* count, void* stream) {
    NR_REQUIRE(samples && count, "nr_wgrad_listed: null sample list");
    return wgrad_launch(true, false, save, grad_ws, n, workspace, grad_flat, stream, samples, count,
                        false);
}
NR_API int NR_X3_NAME(nr_wgrad_sigma_listed)(const float* save, const float* grad_ws, int64_t n,
                                             float* workspace, float* grad_flat,
                                             const int32_t* samples, const int32_t* count,
                                             void* stream) {
    NR_REQUIRE(samples && count, "nr_wgrad_sigma_listed: null sample list");
    return wgrad_launch(true, true, save, grad_ws, n, workspace, grad_flat, stream, samples, count,
                        false);
}
#endif
