// Fused positional-encoding + NeRF MLP forward on bf16x6 split-operand MFMA.
//
// Same contract and outputs as mlp_fwd.hip (models/nerf.py:21-38, 83-124; the
// chunked loop of models/rendering.py:141-161), but every layer runs on
// v_mfma_f32_16x16x32_bf16: each fp32 operand is split exactly into three
// bf16 pieces (hi + mid + lo, round-to-nearest at each step) and the six
// piece products of order <= 2^-16 are accumulated in fp32 -- fp32-level
// accuracy at 16/6 = 2.67x the fp32 MFMA rate (packing.py, "bf16x6").
//
// Structure: a workgroup of 4 waves (one per SIMD) evaluates 4 x 32 samples.
// A wave keeps its activations in registers as x3::Act (features x samples,
// 16x16 accumulator tiles); k-step s of the next layer reads its B fragment
// from tiles 2s, 2s+1 of the lane's own registers.  The weights are shared by
// the 4 waves through an LDS ring of k-groups (32 inputs x 128 outputs x 3
// pieces = 24 KiB), filled by LDS-DMA (global_load_lds dwordx4) kSlots-1
// groups ahead; one barrier per group hands a slot over.  The B split of the
// next k-step and the previous layer's saved-activation stores are spread
// between the MFMAs of the current k-step.
//
// NR_FWD_W2 = 1 (f16x3): two waves per SIMD -- eight waves per workgroup,
// each carrying one 16-sample tile of a 32-sample block (waves 2b, 2b+1 hold
// block b's tiles S = 0, 1), as mlp_bwd3.hip's NR_BWD_W2.  Saved layouts are
// unchanged; a block's ReLU mask words, which interleave both tiles' bits,
// are combined from its two waves through LDS (MaskX).
#ifndef NR_FWD_W2
#define NR_FWD_W2 0
#endif
#if NR_FWD_W2 && !NR_F16
#error "NR_FWD_W2 is an f16x3 variant"
#endif
#if NR_FWD_W2
#define NR_X3_WAVES 8
#endif
#include "x3.h"

namespace {

using namespace x3;

constexpr int kHeadBytes = NR_H_SIZE * 4;
constexpr int kHeadDma = (kHeadBytes + 1023) / 1024;   // 1 KiB LDS-DMA instructions for the head
constexpr int kHeadLds = kHeadDma * 1024;
// NR_PE_REGS: keep the encodings in registers for layer 5 and the dir layer
// (224 VGPRs, no spill) instead of parking them in LDS (48 KiB).  Measured
// (profiles/r04/abalt_peregs, three alternating rounds): fine forward 2.81 ->
// 2.73 ms; the 48 KiB freed for a 4-super-slot ring (NR_X3_SSLOTS=4 on this
// object) bought nothing -- ring depth is not what the hand-overs wait for
#ifndef NR_PE_REGS
#define NR_PE_REGS (NR_F16 || NR_BF1)   // bf16x6's three pieces leave no room (18-30 spills)
#endif
constexpr int kPeQ = 12;                          // float4 per lane: xyz PE slots (8), dir PE (4)
constexpr int kPeBytes = NR_PE_REGS ? 0 : kWaves * kPeQ * 64 * 16;  // each wave's encodings, parked for layer 5 / dir
constexpr int kNS = NR_FWD_W2 ? 1 : 2;            // 16-sample tiles per wave
constexpr int kBlocks = kWaves * kNS / 2;         // 32-sample blocks per workgroup
static_assert(NR_PE_REGS || kNS == 2, "encodings parked in LDS: two tiles per wave only");
constexpr int kXchBytes = kNS == 1 ? kWaves * 2 * 64 * 16 : 0;   // MaskX slots
constexpr int kLdsBytes = kRingBytes + kHeadLds + kPeBytes + kXchBytes;
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");

// ---- the k-group sequence (packing.py FWD3_LAYERS) --------------------------
constexpr int kL1 = 0, kL2 = 4, kL3 = 20, kL4 = 36, kL5 = 52, kL6 = 72, kL7 = 88, kL8 = 104;
constexpr int kFinal = 120, kDir = 136, kQAll = 145, kQSigma = 120;

struct FwdTab {
    // byte offset of group q inside the packed buffer (head first)
    __host__ __device__ static constexpr int64_t off(int q) {
        return (int64_t)kHeadBytes + (int64_t)q * kSlotBytes;
    }
    // merged ring (x3.h): the 256-wide layers' k-steps pair their two output
    // halves; the dir layer's groups (one half) stand alone
    __host__ __device__ static constexpr int sg(int q) { return q < kDir ? q / 2 : kDir / 2 + (q - kDir); }
    __host__ __device__ static constexpr int first(int G) { return G < kDir / 2 ? 2 * G : kDir + (G - kDir / 2); }
    __host__ __device__ static constexpr int size(int G) { return G < kDir / 2 ? 2 : 1; }
};
static_assert(FwdTab::off(kQAll) == (NR_F16 ? 2388000 : (NR_BF1 ? 1200160 : 3575840)),
              "packed size must match packing.fwd3_offsets()");

// w . relu(x) for the wave's sample tiles, reduced over the 4 lane groups
template <bool RELU, int NF, int NS>
__device__ __forceinline__ void head_dot(const f32x4 (&acc)[NF][NS], const float* __restrict__ w,
                                         int g, float (&p)[2]) {
    p[0] = p[1] = 0.f;
#pragma unroll
    for (int F = 0; F < NF; ++F) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(w + 16 * F + 4 * g);
#pragma unroll
        for (int S = 0; S < NS; ++S)
#pragma unroll
            for (int r = 0; r < 4; ++r) p[S] = fmaf(RELU ? relu_i(acc[F][S][r]) : acc[F][S][r], v[r], p[S]);
    }
#pragma unroll
    for (int S = 0; S < NS; ++S) p[S] = sum_over_groups(p[S]);
}

// xyz positional encoding in the slot order of packing.PE16_MAP: lane group g
// holds slots 32s + 8g + j (s = 0, 1), i.e. cells c = 4s + g of 4 arguments
// (sin at j = 0..3, cos at j = 4..7); argument m = 4c + i is coordinate m % 3
// at frequency 2^(m / 3); cell 7 ends with the raw x, y (j = 2, 3) and z (j = 6)
__device__ __forceinline__ void pe_encode(float (&pe)[16], float px, float py, float pz, int g) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = 4 * (4 * s + g) + i;
            const int k = (m * 11) >> 5;     // m / 3 for m < 32
            const int c = m - 3 * k;
            const float v = c == 0 ? px : (c == 1 ? py : pz);
            float sn, cs;
            sincosf(v * __uint_as_float((uint32_t)(127 + k) << 23), &sn, &cs);
            pe[8 * s + i] = sn;
            pe[8 * s + 4 + i] = cs;
        }
    if (g == 3) {
        pe[10] = px; pe[11] = py; pe[14] = pz; pe[15] = 0.f;
    }
}

__device__ __forceinline__ void pe_gather(float (&pe)[16], const float* __restrict__ row, int g) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = min(4 * (4 * s + g) + i, 29);
            const int k = (m * 11) >> 5;
            const int c = m - 3 * k;
            pe[8 * s + i] = row[3 + 6 * k + c];
            pe[8 * s + 4 + i] = row[6 + 6 * k + c];
        }
    if (g == 3) {
        pe[10] = row[0]; pe[11] = row[1]; pe[14] = row[2]; pe[15] = 0.f;
    }
}

// direction encoding (packing.DIR16_MAP): lane group g = frequency 2^g, sin of
// the 3 coordinates at j = 0..2, cos at j = 4..6, raw coordinate g at j = 3
__device__ __forceinline__ void dir_encode(float (&d)[8], float dx, float dy, float dz, int g) {
    const float sc = __uint_as_float((uint32_t)(127 + g) << 23);
    sincosf(dx * sc, &d[0], &d[4]);
    sincosf(dy * sc, &d[1], &d[5]);
    sincosf(dz * sc, &d[2], &d[6]);
    d[3] = g == 0 ? dx : (g == 1 ? dy : (g == 2 ? dz : 0.f));
    d[7] = 0.f;
}

__device__ __forceinline__ void dir_gather(float (&d)[8], const float* __restrict__ row, int g) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        d[c] = row[3 + 6 * g + c];
        d[4 + c] = row[6 + 6 * g + c];
    }
    d[3] = g < 3 ? row[min(g, 2)] : 0.f;
    d[7] = 0.f;
}

// slot values 4u .. 4u+3 (u = 2s + jh of the lane's 8-slot cells) -> the
// saved slots 32s + 8g + 4jh = tile 2s + (g >> 1), group 2(g & 1) + jh: N16
// (bf16, and the sigma-only training forward) or the sample-major rows of W
// slots (ROWS, x3.h store_row)
template <int W, bool ROWS>
__device__ __forceinline__ void store_pe4(const float* v, int s, int jh, int S, int g,
                                          float* __restrict__ blk, int lane) {
    const int T = 2 * s + (g >> 1), gp = 2 * (g & 1) + jh;
#if NR_BF1
    store_slot(f32x4{v[0], v[1], v[2], v[3]}, blk, (T * 2 + S) * 64 + 16 * gp + (lane & 15));
#else
    if constexpr (ROWS)
        *reinterpret_cast<f32x4*>(blk + (16 * S + (lane & 15)) * W + 16 * T + 4 * gp) =
            f32x4{v[0], v[1], v[2], v[3]};
    else
        *reinterpret_cast<f32x4*>(blk + ((T * 2 + S) * 64 + 16 * gp + (lane & 15)) * 4) =
            f32x4{v[0], v[1], v[2], v[3]};
#endif
}

struct MaskWords { uint32_t w[4] = {0u, 0u, 0u, 0u}; };

// A block's ReLU mask words (layout.h: lane word F >> 2, bit 8 (F & 3) + 4 S + r)
// hold both sample tiles' bits.  With one tile per wave (kNS = 1) each wave
// publishes its words of layer l in its LDS slot l & 1 when the layer is
// complete, and the block's even wave, one layer later (ring barriers in
// between), ORs the pair's words of layer l - 1 and stores them; the last
// layer is stored after a workgroup barrier (last()).  kNS = 2 stores directly.
struct MaskX {
    uint4* lds;        // this wave's two slots of 64 uint4 (the partner's follow it)
    uint32_t* base;    // the block's mask segment (layer l at + 256 l)
    int lane;
    bool even;
    __device__ __forceinline__ void flush(int l) const {
        const uint4 a = lds[(l & 1) * 64 + lane], b = lds[128 + (l & 1) * 64 + lane];
        *reinterpret_cast<uint4*>(base + l * 256 + lane * 4) =
            make_uint4(a.x | b.x, a.y | b.y, a.z | b.z, a.w | b.w);
    }
    __device__ __forceinline__ void put(int l, const uint32_t (&w)[4]) const {
        if constexpr (kNS == 2) {
            *reinterpret_cast<uint4*>(base + l * 256 + lane * 4) = make_uint4(w[0], w[1], w[2], w[3]);
        } else {
            lds[(l & 1) * 64 + lane] = make_uint4(w[0], w[1], w[2], w[3]);
            if (l > 0 && even) flush(l - 1);
        }
    }
    // after the last put(l): the block's words of layer l
    __device__ __forceinline__ void last(int l) const {
        if constexpr (kNS == 1) {
            __syncthreads();
            if (even) flush(l);
        }
    }
};

enum FwdMode { FWD_RAYS = 0, FWD_EMB = 1, FWD_PTS = 2 };

// layer 1's side: the xyz PE slots saved, 2 float4 per group (tiles 2, 6)
template <bool SAVE, bool ROWS>
struct PeSide {
    // stores at tiles 2 and 6 (one tile per wave: at tile 2)
    static constexpr int before(int T) { return SAVE ? (T > 2) + (kNS == 2 && T > 6) : 0; }
    const float (&pe)[kNS][16];
    float* dst;
    int g, lane, s0;
    template <typename GC>
    __device__ __forceinline__ void operator()(GC, int t) const {
        if constexpr (SAVE && kNS == 2) {
            if (t == 2 || t == 6) {
                const int u = 2 * GC::value + (t == 6), S = u >> 2, s = (u >> 1) & 1, jh = u & 1;
                store_pe4<64, ROWS>(&pe[S][8 * s + 4 * jh], s, jh, S, g, dst, lane);
            }
        } else if constexpr (SAVE) {
            if (t == 2) {
                const int u = GC::value, s = u >> 1, jh = u & 1;
                store_pe4<64, ROWS>(&pe[0][8 * s + 4 * jh], s, jh, s0, g, dst, lane);
            }
        }
    }
};

// the dir layer's PE part: the dir PE slots saved N16 at tiles 1, 3, 5, 7
template <bool SAVE>
struct DirPeSide {
    // stores at the odd tiles (one tile per wave: at tiles 1 and 5)
    static constexpr int before(int T) { return SAVE ? (kNS == 2 ? T / 2 : (T > 1) + (T > 5)) : 0; }
    const float (&dpe)[kNS][8];
    float* dst;
    int g, lane, s0;
    template <typename GC>
    __device__ __forceinline__ void operator()(GC, int t) const {
        if constexpr (SAVE && kNS == 2) {
            if (t & 1) {
                const int u = t >> 1;
                store_pe4<32, true>(&dpe[u >> 1][4 * (u & 1)], 0, u & 1, u >> 1, g, dst, lane);
            }
        } else if constexpr (SAVE) {
            if (t == 1 || t == 5) {
                const int h = t >> 2;
                store_pe4<32, true>(&dpe[0][4 * h], 0, h, s0, g, dst, lane);
            }
        }
    }
};

struct Fwd3Args {
    const char* packed;  // packing.build_fwd3_map layout: head fp32, then bf16 groups
    const float* pts; const float* rays; const float* z; const float* x;
    int n, spr, xstride;
    float* out; float* save;
    // LIST (nr_mlp_fwd_listed*): position q < *scount evaluates sample
    // slist[q]; activations are saved by position, no output is written
    const int32_t* slist; const int32_t* scount;
};

// B units of an accumulator input (x3.h Act): the producer's activation
// applied (RELU) and, with STORE, the values saved N16 as they are split --
// units p = 0, 1 of (k-step s, tile S) complete feature tile 2s, p = 2, 3 tile
// 2s+1 -- with their ReLU bits (MASK); SIG accumulates the sigma head
// w_sigma . x over the split values (x = h8), so no pass re-reads h8.
// ROWS: saved as sample-major rows (the full graph, x3.h store_row), else N16
// (the sigma-only training forward, whose backward gathers almost nothing)
template <bool RELU, bool STORE, bool MASK, bool SIG, bool ROWS = true>
struct AccU {
    static constexpr bool kStores = STORE;
    static constexpr bool kPaired = STORE && ROWS && kRowPair;
    template <typename P> __device__ __forceinline__ void begin(const P&) {}
    const f32x4 (&X)[16][kNS];
    float* dst;
    uint32_t* msk;     // MASK: the layer's mask words (kNS = 2)
    const MaskX* mx;   // ... or their exchange (kNS = 1), and the layer
    int ml;
    const float* wsig;
    int lane, g, s0;
    float pend[2] = {0.f, 0.f};
    f32x4 held = {0.f, 0.f, 0.f, 0.f};   // kPaired: the even tile, stored with the odd one
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    float sig[2] = {0.f, 0.f};
    // SIG: the sigma weights of k-step s (features kmap16(s, g, 2p) and +1)
    // are read one k-step ahead, into wsg[s & 1], so no LDS read is waited on
    // right where it is used; preload() reads k-step 0's a segment early
    f32x2 wsg[2][4];
    __device__ __forceinline__ f32x2 wsig_of(int s, int p) const {
        return *reinterpret_cast<const f32x2*>(wsig + 32 * s + 16 * (p >> 1) + 4 * g + 2 * (p & 1));
    }
    __device__ __forceinline__ void preload() {
        if constexpr (SIG)
#pragma unroll
            for (int p = 0; p < 4; ++p) wsg[0][p] = wsig_of(0, p);
    }
    template <typename SC>
    __device__ __forceinline__ void operator()(SC, int sb, int p, float& x0, float& x1) {
        constexpr int s = SC::value;
        x0 = acc_b(X, s, sb, 2 * p);
        x1 = acc_b(X, s, sb, 2 * p + 1);
        if constexpr (RELU) { x0 = relu_i(x0); x1 = relu_i(x1); }
        if constexpr (kWScale != 0) { x0 *= kWUnscale; x1 *= kWUnscale; }   // exact
        if constexpr (SIG) {
            // (units run s-major, sb = 0 before 1: wsg[(s + 1) & 1][p] was
            // last read by unit (s - 1, 1, p))
            if (sb == 0 && s + 1 < 8) wsg[(s + 1) & 1][p] = wsig_of(s + 1, p);
            const f32x2 wv = wsg[s & 1][p];
            sig[sb] = fmaf(x0, wv[0], sig[sb]);
            sig[sb] = fmaf(x1, wv[1], sig[sb]);
        }
        if constexpr (STORE) {
            if ((p & 1) == 0) {
                pend[0] = x0;
                pend[1] = x1;
            } else {
                const int F = 2 * s + (p >> 1);
                const f32x4 v = {pend[0], pend[1], x0, x1};
                const int S = (kNS == 2 ? 0 : s0) + sb;     // the block's tile
                if constexpr (kPaired) {
                    if (p == 1) held = v;
                    else store_row_pair<256>(held, v, 2 * s, S, dst, lane);
                } else if constexpr (ROWS) {
                    store_row<256>(v, F, S, dst, lane);
                } else {
                    store_n16(v, F, S, dst, lane);
                }
                if constexpr (MASK) {
                    mask_bits(v, F, S, w);
                    if (s == 7 && sb == kNS - 1 && p == 3) {
                        if constexpr (kNS == 2)
                            *reinterpret_cast<uint4*>(msk + lane * 4) = make_uint4(w[0], w[1], w[2], w[3]);
                        else
                            mx->put(ml, w);
                    }
                }
            }
        }
    }
};

// B units of a positional encoding held per sample tile as [S][8 k + j]
template <int N>
struct PeU {
    static constexpr bool kStores = false;
    static constexpr bool kPaired = false;
    template <typename P> __device__ __forceinline__ void begin(const P&) {}
    const float (&pe)[kNS][N];
    template <typename SC>
    __device__ __forceinline__ void operator()(SC, int sb, int p, float& x0, float& x1) const {
        constexpr int s = SC::value;
        x0 = pe[sb][8 * s + 2 * p];
        x1 = pe[sb][8 * s + 2 * p + 1];
    }
};

// NR_X3_DBG 8 (dev timing build): per-layer clock stamps, 16 uint64 per wave
// in the out buffer (no outputs written; saving as asked): [0] start
// realtime, [1] end realtime, [2] cycles,
// [3 + i] cycles at stamp i (0 inputs+PE, 1 first hand-over, 2.. segments)
#if NR_X3_DBG == 8
#define NR_STAMP(i) (stamps[i] = (uint32_t)(__builtin_amdgcn_s_memtime() - t0))
#else
#define NR_STAMP(i) ((void)0)
#endif

// run a getter over every B unit of the 8 k-steps of a 256-wide activation
// (its stores as side effect) when no layer consumes it
template <int S = 0, typename GetU>
__device__ __forceinline__ void drain_all(GetU& u) {
    if constexpr (S < 8) {
#pragma unroll
        for (int sb = 0; sb < kNS; ++sb)
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                float x0, x1;
                u(IC<S>(), sb, p, x0, x1);
            }
        drain_all<S + 1>(u);
    }
}

// LIST: the deferred save of a training forward (nr_mlp_fwd_listed*): the
// forward ran without saving (the inference kernel, whose layers are these
// layers bit for bit), and the backward re-evaluates only the samples its
// sample list names, saving their activations packed by position -- the
// sigma-only graph's backward lists ~0.1% of a light image's samples and
// ~20% of the camera rays' (DESIGN.md 11).  blk is then a block of positions.
template <int MODE, bool SIGMA_ONLY, bool SAVE, bool LIST = false>
__global__ void __launch_bounds__(64 * kWaves, 1) mlp_fwd3_kernel(Fwd3Args a) {
    constexpr bool EMB = MODE == FWD_EMB;
    constexpr int QEND = SIGMA_ONLY ? kQSigma : kQAll;
    static_assert(!LIST || (SAVE && MODE == FWD_RAYS), "a listed run saves, on the ray path");
    __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4;
    const int wb = kNS == 2 ? wave : wave >> 1;   // the wave's block within the workgroup
    const int s0 = kNS == 2 ? 0 : wave & 1;       // the block's first tile this wave holds
    const int blk = blockIdx.x * kBlocks + wb;
    const int m = LIST ? __builtin_amdgcn_readfirstlane(*a.scount) : a.n;
    if (LIST && (int)blockIdx.x * kBlocks * 32 >= m) return;   // whole workgroup: before any barrier
    int smp[2];
    bool valid[2];
#pragma unroll
    for (int S = 0; S < kNS; ++S) {
        const int s_raw = blk * 32 + 16 * (s0 + S) + (lane & 15);
        valid[S] = s_raw < m;
        if constexpr (LIST) smp[S] = a.slist[valid[S] ? s_raw : 0];
        else smp[S] = valid[S] ? s_raw : a.n - 1;
    }
    const char* P = a.packed;
#if NR_X3_DBG == 8
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t stamps[13] = {};
#endif

    // sample inputs first: they are waited for while the weight DMA below
    // stays in flight (vmcnt retires in issue order)
    float pe[kNS][16], dg[kNS][8];
    float in[kNS][7];
#pragma unroll
    for (int S = 0; S < kNS; ++S) {
        const int s = smp[S];
        if constexpr (EMB) {
            pe_gather(pe[S], a.x + (size_t)s * a.xstride, g);
            if constexpr (!SIGMA_ONLY) dir_gather(dg[S], a.x + (size_t)s * a.xstride + NR_XYZ_CH, g);
        } else if constexpr (MODE == FWD_PTS) {
#pragma unroll
            for (int c = 0; c < 3; ++c) in[S][c] = a.pts[(size_t)s * 3 + c];
        } else {
            const float* r = a.rays + (size_t)(s / a.spr) * 8;
#pragma unroll
            for (int c = 0; c < 6; ++c) in[S][c] = r[c];
            in[S][6] = a.z[s];
        }
    }

    // head block (biases, sigma/rgb heads) and the first weight groups by
    // LDS-DMA; the first ring hand-over waits for both
    float* Hs = reinterpret_cast<float*>(smem + kRingBytes);
    const Dma dma = make_dma(P, FwdTab::off(kQAll), smem, wave, lane);
#pragma unroll
    for (int i = wave; i < kHeadDma; i += kWaves)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            dma.rsrc, (__attribute__((address_space(3))) void*)(smem + kRingBytes + i * 1024), 16,
            dma.voff, i * 1024, 0, 0);
    prologue<FwdTab, QEND>(dma);
    const float* H = Hs;
    const int nb = (int)nr_blocks_pad(a.n);
    float* const SV = a.save;

    // PE slots of both sample tiles (and the direction PE): computed once,
    // parked in LDS for layer 5 and the dir layer
    [[maybe_unused]] f32x4* pe_lds =
        reinterpret_cast<f32x4*>(smem + kRingBytes + kHeadLds) + wave * kPeQ * 64 + lane;
#pragma unroll
    for (int S = 0; S < kNS; ++S) {
        if constexpr (MODE == FWD_PTS) {
            pe_encode(pe[S], in[S][0], in[S][1], in[S][2], g);
        } else if constexpr (MODE == FWD_RAYS) {
            const float zz = in[S][6];
            pe_encode(pe[S], nr_add(in[S][0], nr_mul(in[S][3], zz)),   // rendering.py:234, no FMA
                      nr_add(in[S][1], nr_mul(in[S][4], zz)), nr_add(in[S][2], nr_mul(in[S][5], zz)), g);
            if constexpr (!SIGMA_ONLY) dir_encode(dg[S], in[S][3], in[S][4], in[S][5], g);
        }
    }
#if !NR_PE_REGS
#pragma unroll
    for (int q = 0; q < 8; ++q)
        pe_lds[q * 64] = f32x4{pe[q >> 2][4 * (q & 3)], pe[q >> 2][4 * (q & 3) + 1],
                               pe[q >> 2][4 * (q & 3) + 2], pe[q >> 2][4 * (q & 3) + 3]};
    if constexpr (!SIGMA_ONLY) {
#pragma unroll
        for (int S = 0; S < 2; ++S) {
            pe_lds[(8 + 2 * S) * 64] = f32x4{dg[S][0], dg[S][1], dg[S][2], dg[S][3]};
            pe_lds[(9 + 2 * S) * 64] = f32x4{dg[S][4], dg[S][5], dg[S][6], dg[S][7]};
        }
    }
#endif
#if NR_X3_DBG == 8
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
    NR_STAMP(0);       // inputs + positional encoding

    Ahead f0;          // the first tiles' fragments of the next k-group
    enter<FwdTab, 0, QEND>(smem, lane, f0);
    NR_STAMP(1);       // prologue: + first weight group

    ActN<kNS> A, B;
    Pieces b[kNS];     // pieces of the next k-step
    auto hseg = [&](int l) { return SV + nr_sv_h(l, nb) + (size_t)blk * NR_SEGF(256); };
    auto mseg = [&](int l) {
        return reinterpret_cast<uint32_t*>(SV + nr_sv_mask(nb)) + ((size_t)blk * NR_MASK_LAYERS + l) * 256;
    };
    NoSide none;
    NoNext nonext;
    ZeroInit zero;
    auto bias = [&](int off) { return BiasInit{H + off, g}; };
    // the full graph saves sample-major rows, the sigma-only training forward N16
    // (wgrad.hip reads each as its task list expects)
    constexpr bool kRows = !SIGMA_ONLY;
    using U = AccU<true, SAVE, SAVE, false, kRows>;
    const MaskX mx{reinterpret_cast<uint4*>(smem + kRingBytes + kHeadLds + kPeBytes) + 128 * wave,
                   mseg(0), lane, s0 == 0};

    // layer 1: PE(63) -> 256; stores the PE slots
    PeU<16> peu{pe};
    split_all(peu, b);
    U u1{A, hseg(0), mseg(0), &mx, 0, nullptr, lane, g, s0};
    {
        PeSide<SAVE, kRows> side{pe, SV + (size_t)blk * NR_SEGF(64), g, lane, s0};
        auto bi = bias(NR_H_BIAS(1));
        segment<FwdTab, kL1, 2, 2, QEND, true>(dma, lane, A, peu, u1, bi, side, b, f0);
    }
    NR_STAMP(2);
    U u2{B, hseg(1), mseg(1), &mx, 1, nullptr, lane, g, s0};
    { auto bi = bias(NR_H_BIAS(2)); segment<FwdTab, kL2, 8, 2, QEND, true>(dma, lane, B, u1, u2, bi, none, b, f0); }
    NR_STAMP(3);
    U u3{A, hseg(2), mseg(2), &mx, 2, nullptr, lane, g, s0};
    { auto bi = bias(NR_H_BIAS(3)); segment<FwdTab, kL3, 8, 2, QEND, true>(dma, lane, A, u2, u3, bi, none, b, f0); }
    NR_STAMP(4);
    float pe5[kNS][16];
#if NR_PE_REGS
#pragma unroll
    for (int S = 0; S < kNS; ++S)
#pragma unroll
        for (int i = 0; i < 16; ++i) pe5[S][i] = pe[S][i];
#else
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const f32x4 v = pe_lds[q * 64];
#pragma unroll
        for (int e = 0; e < 4; ++e) pe5[q >> 2][4 * (q & 3) + e] = v[e];
    }
#endif
    PeU<16> pe5u{pe5};
    { auto bi = bias(NR_H_BIAS(4)); segment<FwdTab, kL4, 8, 2, QEND, true>(dma, lane, B, u3, pe5u, bi, none, b, f0); }
    NR_STAMP(5);
    // layer 5: cat[PE, h4] -> 256 (nerf.py:108-109)
    U u4{B, hseg(3), mseg(3), &mx, 3, nullptr, lane, g, s0};
    { auto bi = bias(NR_H_BIAS(5)); segment<FwdTab, kL5, 2, 2, QEND, true>(dma, lane, A, pe5u, u4, bi, none, b, f0); }
    NR_STAMP(6);
    U u5{A, hseg(4), mseg(4), &mx, 4, nullptr, lane, g, s0};
    segment<FwdTab, kL5 + 4, 8, 2, QEND, false>(dma, lane, A, u4, u5, zero, none, b, f0);
    NR_STAMP(7);
    U u6{B, hseg(5), mseg(5), &mx, 5, nullptr, lane, g, s0};
    { auto bi = bias(NR_H_BIAS(6)); segment<FwdTab, kL6, 8, 2, QEND, true>(dma, lane, B, u5, u6, bi, none, b, f0); }
    NR_STAMP(8);
    U u7{A, hseg(6), mseg(6), &mx, 6, nullptr, lane, g, s0};
    { auto bi = bias(NR_H_BIAS(7)); segment<FwdTab, kL7, 8, 2, QEND, true>(dma, lane, A, u6, u7, bi, none, b, f0); }
    NR_STAMP(9);

    // lane group g < kNS writes the wave's sample tile g
    const int Sw = kNS == 2 ? (g & 1) : 0;
    const bool wr = g < kNS && valid[Sw];
    const int sw = smp[Sw];
    if constexpr (SIGMA_ONLY && SAVE) {
        // training a sigma-only graph (rendering_shadows.py:167, the shadow
        // path's every MLP call): layers 1-8 and the sigma head only.  h8 and
        // its ReLU mask are saved exactly as the full graph saves them while
        // splitting h8 for xyz_encoding_final, and sigma comes from the same
        // sums; out rows are (n, 4) [0, 0, 0, sigma] for the backward's contract
        { auto bi = bias(NR_H_BIAS(8)); segment<FwdTab, kL8, 8, 2, QEND, true>(dma, lane, B, u7, nonext, bi, none, b, f0); }
        AccU<true, true, true, true, false> u8{B, hseg(7), mseg(7), &mx, 7, H + NR_H_WSIG, lane, g, s0};
        u8.preload();
        drain_all(u8);
        mx.last(7);
        float sigma[2];
#pragma unroll
        for (int S = 0; S < kNS; ++S) {
            sigma[S] = sum_over_groups(u8.sig[S]) + H[NR_H_BSIG];
        }
        if (wr && !LIST)
            *reinterpret_cast<f32x4*>(a.out + (size_t)sw * 4) = f32x4{0.f, 0.f, 0.f, Sw ? sigma[1] : sigma[0]};
        return;
    } else if constexpr (SIGMA_ONLY) {
        { auto bi = bias(NR_H_BIAS(8)); segment<FwdTab, kL8, 8, 2, QEND, true>(dma, lane, B, u7, nonext, bi, none, b, f0); }
        float sigma[2];
        head_dot<true>(B, H + NR_H_WSIG, g, sigma);
        if (wr) a.out[sw] = (Sw ? sigma[1] : sigma[0]) * kWUnscale + H[NR_H_BSIG];
        return;
    } else {
        // h8 feeds xyz_encoding_final and, while it is split, the sigma head
        AccU<true, SAVE, SAVE, true> u8{B, hseg(7), mseg(7), &mx, 7, H + NR_H_WSIG, lane, g, s0};
        u8.preload();
        { auto bi = bias(NR_H_BIAS(8)); segment<FwdTab, kL8, 8, 2, QEND, true>(dma, lane, B, u7, u8, bi, none, b, f0); }
        NR_STAMP(10);
        // dir_encoding: ReLU(Linear(283,128)(cat[feat, PE(dir)])) (nerf.py:118-119)
        float dpe[kNS][8];
#if NR_PE_REGS
#pragma unroll
        for (int S = 0; S < kNS; ++S)
#pragma unroll
            for (int i = 0; i < 8; ++i) dpe[S][i] = dg[S][i];
#else
#pragma unroll
        for (int S = 0; S < 2; ++S)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const f32x4 v = pe_lds[(8 + 2 * S + h) * 64];
#pragma unroll
                for (int e = 0; e < 4; ++e) dpe[S][4 * h + e] = v[e];
            }
#endif
        PeU<8> dpeu{dpe};
        // xyz_encoding_final: no activation (nerf.py:116)
        // not saved: the weight gradient of the dir layer's feat columns is
        // formed from h8 (wgrad.hip task 10, nr_wgrad_dir_feat) -- 1 KiB per
        // sample fewer stores, and the densest store phase of the kernel gone
        AccU<false, false, false, false> uf{A, nullptr, nullptr, nullptr, 0, nullptr, lane, g, s0};
        { auto bi = bias(NR_H_BFINAL); segment<FwdTab, kFinal, 8, 2, QEND, true>(dma, lane, A, u8, uf, bi, none, b, f0); }
        NR_STAMP(11);
        float sigma[2];
#pragma unroll
        for (int S = 0; S < kNS; ++S) {
            sigma[S] = sum_over_groups(u8.sig[S]) + H[NR_H_BSIG];
        }
        f32x4 C[8][kNS];
        { auto bi = bias(NR_H_BDIR); segment<FwdTab, kDir, 8, 1, QEND, true>(dma, lane, C, uf, dpeu, bi, none, b, f0); }
        {   // PE(dir) part (stores the dir PE slots)
            DirPeSide<SAVE> side{dpe, SV + nr_sv_dirpe(nb) + (size_t)blk * NR_SEGF(32), g, lane, s0};
            segment<FwdTab, kDir + 8, 1, 1, QEND, false>(dma, lane, C, dpeu, nonext, zero, side, b, f0);
        }
        NR_STAMP(12);
        float zc[3][2];
#pragma unroll
        for (int c = 0; c < 3; ++c) head_dot<true>(C, H + NR_H_WRGB + 128 * c, g, zc[c]);
        if (wr && !LIST && NR_X3_DBG != 8) {
            f32x4 o;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float z = (Sw ? zc[c][1] : zc[c][0]) * kWUnscale + H[NR_H_BRGB + c];
                o[c] = 1.f / (1.f + expf(-z));
            }
            o[3] = Sw ? sigma[1] : sigma[0];
            *reinterpret_cast<f32x4*>(a.out + (size_t)sw * 4) = o;
        }
#if NR_X3_DBG == 8
        if (lane == 0) {
            uint64_t* st = reinterpret_cast<uint64_t*>(a.out) + (size_t)(blockIdx.x * kWaves + wave) * 16;
            st[0] = r0;
            st[1] = __builtin_amdgcn_s_memrealtime();
            st[2] = __builtin_amdgcn_s_memtime() - t0;
            for (int i = 0; i < 13; ++i) st[3 + i] = stamps[i];
        }
#endif
        if constexpr (SAVE) {
            float* hd = SV + nr_sv_hdir(nb) + (size_t)blk * NR_SEGF(128);
            uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int F = 0; F < 8; ++F)
#pragma unroll
                for (int S = 0; S < kNS; ++S) {
                    f32x4 v = C[F][S];
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = relu_i(v[r]) * kWUnscale;
                    store_row<128>(v, F, s0 + S, hd, lane);
                    mask_bits(v, F, s0 + S, w);
                }
            if constexpr (kNS == 2) {
                *reinterpret_cast<uint4*>(mseg(8) + lane * 4) = make_uint4(w[0], w[1], w[2], w[3]);
            } else {
                mx.put(8, w);
                mx.last(8);
            }
        }
    }
}

// pack: the weight pieces (map: flat*4 + piece, -1 = 0) after the fp32 head
// block (head_map: flat index, -1 = 0).  f16x3: weights and the layer biases
// (the MFMA C operand, head entries before NR_H_WSIG) carry 2^kWScale.
__device__ __forceinline__ float weight_piece(float w, int piece) {
#if NR_F16
    w *= (float)(1 << kWScale);
    const float hi = (float)(_Float16)w;
    return piece == 0 ? hi : w - hi;
#elif NR_BF1
    (void)piece;
    return (float)(__bf16)w;
#else
    const float hi = (float)(__bf16)w;
    const float r1 = w - hi;
    const float mid = (float)(__bf16)r1;
    return piece == 0 ? hi : (piece == 1 ? mid : r1 - mid);
#endif
}

__global__ void pack3_kernel(const float* __restrict__ flat, const int32_t* __restrict__ map,
                             int64_t n, const int32_t* __restrict__ head_map,
                             char* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < NR_H_SIZE) {
        const int32_t m = head_map[i];
        const float sc = i < NR_H_WSIG ? (float)(1 << kWScale) : 1.f;
        reinterpret_cast<float*>(out)[i] = m >= 0 ? flat[m] * sc : 0.f;
    }
    if (i >= n) return;
    const int32_t m = map[i];
    const float v = m >= 0 ? weight_piece(flat[m >> 2], m & 3) : 0.f;
    reinterpret_cast<p1*>(out + kHeadBytes)[i] = (p1)v;
}

}  // namespace

#if NR_F16
#define NR_FWD3_BYTES_NAME nr_fwd3_packed_bytes_h3
#elif NR_BF1
#define NR_FWD3_BYTES_NAME nr_fwd3_packed_bytes_b1
#else
#define NR_FWD3_BYTES_NAME nr_fwd3_packed_bytes
#endif
NR_API int64_t NR_FWD3_BYTES_NAME(void) { return FwdTab::off(kQAll); }

NR_API int NR_X3_NAME(nr_pack)(const float* flat, const int32_t* map, int64_t n, const int32_t* head_map,
                      void* out, void* stream) {
    NR_REQUIRE(n == (FwdTab::off(kQAll) - kHeadBytes) / 2, "nr_pack_x3: map has %lld entries, "
               "expected %lld", (long long)n, (long long)((FwdTab::off(kQAll) - kHeadBytes) / 2));
    NR_REQUIRE(flat && map && head_map && out, "nr_pack_x3: null pointer");
    pack3_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        flat, map, n, head_map, reinterpret_cast<char*>(out));
    NR_LAUNCH_CHECK("nr_pack_x3");
    return 0;
}

NR_API int NR_X3_NAME(nr_mlp_fwd)(const void* packed, const float* rays, const float* z, int64_t n,
                         int samples_per_ray, const float* x, int xstride, int sigma_only,
                         float* out, float* save, void* stream) {
    NR_REQUIRE(n >= 0 && n < (int64_t)1 << 31, "nr_mlp_fwd_x3: n=%lld out of range", (long long)n);
    if (n == 0) return 0;
    NR_REQUIRE(packed && out, "nr_mlp_fwd_x3: null packed/out");
    NR_REQUIRE(((uintptr_t)packed & 15) == 0 && ((uintptr_t)out & 15) == 0 &&
                   ((uintptr_t)save & 15) == 0,
               "nr_mlp_fwd_x3: packed/out/save must be 16-byte aligned");
    const bool emb = x != nullptr;
    if (emb) {
        NR_REQUIRE(xstride >= (sigma_only ? NR_XYZ_CH : NR_XYZ_CH + NR_DIR_CH),
                   "nr_mlp_fwd_x3: xstride %d too small", xstride);
    } else {
        NR_REQUIRE(rays && z && samples_per_ray > 0, "nr_mlp_fwd_x3: rays/z/samples_per_ray");
    }
    NR_REQUIRE(!(sigma_only && save && emb),
               "nr_mlp_fwd_x3: a sigma_only run keeps activations only on the ray path");
    Fwd3Args a{reinterpret_cast<const char*>(packed), nullptr, rays, z, x, (int)n,
               samples_per_ray, xstride, out, save};
    const int blocks = (int)((n + 32 * kBlocks - 1) / (32 * kBlocks));
    hipStream_t st = (hipStream_t)stream;
    const bool sv = save != nullptr;
    if (emb) {
        if (sigma_only) mlp_fwd3_kernel<FWD_EMB, true, false><<<blocks, 64 * kWaves, 0, st>>>(a);
        else if (sv) mlp_fwd3_kernel<FWD_EMB, false, true><<<blocks, 64 * kWaves, 0, st>>>(a);
        else mlp_fwd3_kernel<FWD_EMB, false, false><<<blocks, 64 * kWaves, 0, st>>>(a);
    } else {
        // sigma_only with save: the sigma-only training forward (out (n, 4))
        if (sigma_only && sv) mlp_fwd3_kernel<FWD_RAYS, true, true><<<blocks, 64 * kWaves, 0, st>>>(a);
        else if (sigma_only) mlp_fwd3_kernel<FWD_RAYS, true, false><<<blocks, 64 * kWaves, 0, st>>>(a);
        else if (sv) mlp_fwd3_kernel<FWD_RAYS, false, true><<<blocks, 64 * kWaves, 0, st>>>(a);
        else mlp_fwd3_kernel<FWD_RAYS, false, false><<<blocks, 64 * kWaves, 0, st>>>(a);
    }
    NR_LAUNCH_CHECK("nr_mlp_fwd_x3");
    return 0;
}

#if !NR_BF1   // no sample lists for the bf16 variant
// the deferred save (LIST above): the training forward's activations of the
// samples listed in samples[0 .. *count) (nr_active_samples), saved by
// position into save (sized for n samples, as nr_mlp_fwd's); no output
NR_API int NR_X3_NAME(nr_mlp_fwd_listed)(const void* packed, const float* rays, const float* z,
                                         int64_t n, int samples_per_ray, int sigma_only,
                                         float* save, const int32_t* samples,
                                         const int32_t* count, void* stream) {
    NR_REQUIRE(n >= 0 && n < (int64_t)1 << 31, "nr_mlp_fwd_listed: n=%lld out of range", (long long)n);
    if (n == 0) return 0;
    NR_REQUIRE(packed && rays && z && save && samples && count && samples_per_ray > 0,
               "nr_mlp_fwd_listed: null pointer or samples_per_ray");
    NR_REQUIRE(((uintptr_t)packed & 15) == 0 && ((uintptr_t)save & 15) == 0,
               "nr_mlp_fwd_listed: packed/save must be 16-byte aligned");
    Fwd3Args a{reinterpret_cast<const char*>(packed), nullptr, rays, z, nullptr, (int)n,
               samples_per_ray, 0, nullptr, save, samples, count};
    const int blocks = (int)((n + 32 * kBlocks - 1) / (32 * kBlocks));
    hipStream_t st = (hipStream_t)stream;
    if (sigma_only) mlp_fwd3_kernel<FWD_RAYS, true, true, true><<<blocks, 64 * kWaves, 0, st>>>(a);
    else mlp_fwd3_kernel<FWD_RAYS, false, true, true><<<blocks, 64 * kWaves, 0, st>>>(a);
    NR_LAUNCH_CHECK("nr_mlp_fwd_listed");
    return 0;
}
#endif

NR_API int NR_X3_NAME(nr_mlp_sigma_points)(const void* packed, const float* pts, int64_t n,
                                  float* sigma_out, void* stream) {
    NR_REQUIRE(n >= 0 && n < (int64_t)1 << 31, "nr_mlp_sigma_points_x3: n out of range");
    if (n == 0) return 0;
    NR_REQUIRE(packed && pts && sigma_out, "nr_mlp_sigma_points_x3: null pointer");
    NR_REQUIRE(((uintptr_t)packed & 15) == 0, "nr_mlp_sigma_points_x3: packed alignment");
    Fwd3Args a{reinterpret_cast<const char*>(packed), pts, nullptr, nullptr, nullptr, (int)n, 1, 0,
               sigma_out, nullptr};
    const int blocks = (int)((n + 32 * kBlocks - 1) / (32 * kBlocks));
    mlp_fwd3_kernel<FWD_PTS, true, false><<<blocks, 64 * kWaves, 0, (hipStream_t)stream>>>(a);
    NR_LAUNCH_CHECK("nr_mlp_sigma_points_x3");
    return 0;
}
