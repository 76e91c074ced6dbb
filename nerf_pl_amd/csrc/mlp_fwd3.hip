// Fused positional-encoding + NeRF MLP forward on bf16x6 split-operand MFMA.
//
// Same contract and outputs as mlp_fwd.hip (models/nerf.py:21-38, 83-124; the
// chunked loop of models/rendering.py:141-161), but every layer runs on
// v_mfma_f32_32x32x16_bf16: each fp32 operand is split exactly into three
// bf16 pieces (hi + mid + lo, round-to-nearest at each step) and the six
// piece products of order <= 2^-16 are accumulated in fp32 -- fp32-level
// accuracy at 16/6 = 2.67x the fp32 MFMA rate (packing.py, "bf16x6").
//
// Structure: a workgroup of 4 waves (one per SIMD) evaluates 4 x 32 samples.
// A wave keeps its activations in registers in transposed form
// D[feature][sample] (a layer's accumulator registers 8s..8s+7 of tile t are
// the B fragment of k-group 2t+s of the next layer).  The weights are shared
// by the 4 waves through an LDS ring of k-groups (16 input features x all
// output tiles x 3 pieces = 24 KiB), filled by LDS-DMA (global_load_lds
// dwordx4) kSlots-1 groups ahead; one barrier per group hands a slot over.
// The B-fragment split costs ~45 VALU ops per k-group, hidden between MFMAs.
#include "x3.h"

namespace {

using namespace x3;

constexpr int kHeadBytes = NR_H_SIZE * 4;
constexpr int kLdsBytes = kRingBytes + kHeadBytes;

// ---- the k-group sequence (packing.py FWD3_LAYERS) --------------------------
constexpr int kL1 = 0, kL2 = 4, kL3 = 20, kL4 = 36, kL5 = 52, kL6 = 72, kL7 = 88, kL8 = 104;
constexpr int kFinal = 120, kDir = 136, kQAll = 154, kQSigma = 120;

struct FwdTab {
    __host__ __device__ static constexpr int tiles(int q) { return q >= kDir ? 4 : 8; }
    // byte offset of group q inside the packed buffer (head first)
    __host__ __device__ static constexpr int64_t off(int q) {
        return (int64_t)kHeadBytes + (q <= kDir ? (int64_t)q * 8 * 3072
                                                : (int64_t)kDir * 8 * 3072 + (int64_t)(q - kDir) * 4 * 3072);
    }
};
static_assert(FwdTab::off(kQAll) == 3575840, "packed size must match packing.fwd3_offsets()");

template <int NT>
__device__ __forceinline__ void init_bias(f32x16 (&acc)[8], const float* __restrict__ b, int h) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(b + 32 * t + 8 * q + 4 * h);
            acc[t][4 * q + 0] = v[0];
            acc[t][4 * q + 1] = v[1];
            acc[t][4 * q + 2] = v[2];
            acc[t][4 * q + 3] = v[3];
        }
}

template <int NT>
__device__ __forceinline__ void relu(f32x16 (&acc)[8]) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = acc[t][r] > 0.f ? acc[t][r] : 0.f;
}

template <int NT>
__device__ __forceinline__ float head_dot(const f32x16 (&acc)[8], const float* __restrict__ w, int h) {
    float p = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(w + 32 * t + 8 * q + 4 * h);
#pragma unroll
            for (int e = 0; e < 4; ++e) p = fmaf(acc[t][4 * q + e], v[e], p);
        }
    return p + __shfl_xor(p, 32);
}

// positional encoding in the per-lane k-step order of packing.pe_feature
template <int NP, int KS>
__device__ __forceinline__ void pe_encode(float (&pe)[KS], float px, float py, float pz, int h) {
    pe[0] = h ? py : px;
    pe[1] = h ? 0.f : pz;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int m = i + NP * h;
        const int k = (m * 11) >> 5;     // m / 3 for m < 32
        const int c = m - 3 * k;
        const float v = c == 0 ? px : (c == 1 ? py : pz);
        const float arg = v * (float)(1 << k);
        float sn, cs;
        sincosf(arg, &sn, &cs);
        pe[2 + i] = sn;
        pe[2 + NP + i] = cs;
    }
#pragma unroll
    for (int g = 2 + 2 * NP; g < KS; ++g) pe[g] = 0.f;
}

template <int NP, int KS>
__device__ __forceinline__ void pe_gather(float (&pe)[KS], const float* __restrict__ row, int h) {
    pe[0] = row[h];
    pe[1] = h ? 0.f : row[2];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int m = i + NP * h;
        const int k = (m * 11) >> 5;
        const int c = m - 3 * k;
        pe[2 + i] = row[3 + 6 * k + c];
        pe[2 + NP + i] = row[6 + 6 * k + c];
    }
#pragma unroll
    for (int g = 2 + 2 * NP; g < KS; ++g) pe[g] = 0.f;
}

enum FwdMode { FWD_RAYS = 0, FWD_EMB = 1, FWD_PTS = 2 };

struct Fwd3Args {
    const char* packed;  // packing.build_fwd3_map layout: head fp32, then bf16 groups
    const float* pts; const float* rays; const float* z; const float* x;
    int n, spr, xstride;
    float* out; float* save;
};

template <int MODE, bool SIGMA_ONLY>
__global__ void __launch_bounds__(64 * kWaves, 1) mlp_fwd3_kernel(Fwd3Args a) {
    constexpr bool EMB = MODE == FWD_EMB;
    constexpr int QEND = SIGMA_ONLY ? kQSigma : kQAll;
    __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int h = lane >> 5;
    const int blk = blockIdx.x * kWaves + wave;
    const int s_raw = blk * 32 + (lane & 31);
    const bool valid = s_raw < a.n;
    const int s = valid ? s_raw : a.n - 1;
    const char* P = a.packed;

    // head block (biases, sigma/rgb heads) -> LDS, then start the weight ring
    float* Hs = reinterpret_cast<float*>(smem + kRingBytes);
    {
        const f32x4* src = reinterpret_cast<const f32x4*>(P);
        for (int i = threadIdx.x; i < NR_H_SIZE / 4; i += 64 * kWaves)
            reinterpret_cast<f32x4*>(Hs)[i] = src[i];
    }
    prologue<FwdTab, QEND>(P, smem, wave, lane);
    __syncthreads();   // head visible (the DMA stays in flight: waited per group)
    Frag f0;           // tile-0 fragments of the next k-group
    enter<FwdTab, 0, QEND>(smem, lane, f0);
    const float* H = Hs;
    const int nb = (a.n + 31) / 32;
    const bool save = a.save != nullptr && blk < nb;
    float* const SV = a.save;

    float px, py, pz, dx = 0.f, dy = 0.f, dz = 0.f;
    const float* xrow = nullptr;
    if constexpr (EMB) {
        xrow = a.x + (size_t)s * a.xstride;
        px = py = pz = 0.f;
    } else if constexpr (MODE == FWD_PTS) {
        px = a.pts[(size_t)s * 3 + 0];
        py = a.pts[(size_t)s * 3 + 1];
        pz = a.pts[(size_t)s * 3 + 2];
    } else {
        const int ray = s / a.spr;
        const float* r = a.rays + (size_t)ray * 8;
        const float zz = a.z[s];
        px = nr_add(r[0], nr_mul(r[3], zz));   // rendering.py:234, no FMA
        py = nr_add(r[1], nr_mul(r[4], zz));
        pz = nr_add(r[2], nr_mul(r[5], zz));
        dx = r[3]; dy = r[4]; dz = r[5];
    }

    f32x16 A[8], B[8];
    auto hseg = [&](int l) { return SV + nr_sv_h(l, nb) + (size_t)blk * NR_NATIVE(256); };
    auto mseg = [&](int l) {
        return reinterpret_cast<uint32_t*>(SV + nr_sv_mask(nb)) + ((size_t)blk * NR_MASK_LAYERS + l) * 256;
    };
    // previous layer's 32 output pieces, 2 per k-group, + its ReLU mask
    auto side_acc = [&](const f32x16 (&X)[8], float* dst, uint32_t* msk) {
        return [&X, dst, msk, save, lane](auto gc) {
            constexpr int g = decltype(gc)::value;
            if (!save) return;
            store_native_piece<8>(reinterpret_cast<const f32x16(&)[8]>(X), 2 * g, dst, lane);
            store_native_piece<8>(reinterpret_cast<const f32x16(&)[8]>(X), 2 * g + 1, dst, lane);
            if (g == 0 && msk) store_mask<8>(reinterpret_cast<const f32x16(&)[8]>(X), msk, lane);
        };
    };
    auto from_acc = [](const f32x16 (&X)[8]) {
        return [&X](auto gc, float (&x)[8]) { acc_group<decltype(gc)::value>(X, x); };
    };
    NoSide none;

    {   // layer 1: PE(63) -> 256
        float pe[NR_PE_KSTEPS];
        if constexpr (EMB) pe_gather<15, NR_PE_KSTEPS>(pe, xrow, h);
        else pe_encode<15, NR_PE_KSTEPS>(pe, px, py, pz, h);
        float* pdst = SV + (size_t)blk * NR_NATIVE(64);
        init_bias<8>(A, H + NR_H_BIAS(1), h);
        auto getb = [&](auto gc, float (&x)[8]) {
            constexpr int g = decltype(gc)::value;
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = pe[8 * g + j];
        };
        auto side = [&](auto gc) {     // PE values, 2 float4 per group
            constexpr int g = decltype(gc)::value;
            if (!save) return;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int grp = 2 * g + u;
                f32x4 v = {pe[4 * grp], pe[4 * grp + 1], pe[4 * grp + 2], pe[4 * grp + 3]};
                *reinterpret_cast<f32x4*>(pdst + (grp * 64 + lane) * 4) = v;
            }
        };
        segment<FwdTab, kL1, 0, 4, 8, QEND>(P, smem, wave, lane, A, getb, side, f0);
        relu<8>(A);
    }
#define NR_DENSE3(DST, SRC, Q0, L)                                              \
    {                                                                           \
        init_bias<8>(DST, H + NR_H_BIAS(L), h);                                 \
        auto gb = from_acc(SRC);                                                \
        auto sd = side_acc(SRC, hseg(L - 2), mseg(L - 2));                      \
        segment<FwdTab, Q0, 0, 16, 8, QEND>(P, smem, wave, lane, DST, gb, sd, f0);      \
        relu<8>(DST);                                                           \
    }
    NR_DENSE3(B, A, kL2, 2)
    NR_DENSE3(A, B, kL3, 3)
    NR_DENSE3(B, A, kL4, 4)
    {   // layer 5: cat[PE, h4] -> 256 (nerf.py:108-109)
        float pe[NR_PE_KSTEPS];
        if constexpr (EMB) pe_gather<15, NR_PE_KSTEPS>(pe, xrow, h);
        else pe_encode<15, NR_PE_KSTEPS>(pe, px, py, pz, h);
        init_bias<8>(A, H + NR_H_BIAS(5), h);
        auto getb = [&](auto gc, float (&x)[8]) {
            constexpr int g = decltype(gc)::value;
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = pe[8 * g + j];
        };
        segment<FwdTab, kL5, 0, 4, 8, QEND>(P, smem, wave, lane, A, getb, none, f0);
        auto gb = from_acc(B);
        auto sd = side_acc(B, hseg(3), mseg(3));
        segment<FwdTab, kL5 + 4, 0, 16, 8, QEND>(P, smem, wave, lane, A, gb, sd, f0);
        relu<8>(A);
    }
    NR_DENSE3(B, A, kL6, 6)
    NR_DENSE3(A, B, kL7, 7)
    NR_DENSE3(B, A, kL8, 8)
#undef NR_DENSE3

    const float sigma = head_dot<8>(B, H + NR_H_WSIG, h) + H[NR_H_BSIG];
    if constexpr (SIGMA_ONLY) {
        if (valid && h == 0) a.out[s] = sigma;
        return;
    } else {
        {   // xyz_encoding_final: no activation (nerf.py:116); stores h8
            init_bias<8>(A, H + NR_H_BFINAL, h);
            auto gb = from_acc(B);
            auto sd = side_acc(B, hseg(7), mseg(7));
            segment<FwdTab, kFinal, 0, 16, 8, QEND>(P, smem, wave, lane, A, gb, sd, f0);
        }
        // dir_encoding: ReLU(Linear(283,128)(cat[feat, PE(dir)])) (nerf.py:118-119)
        float dpe[NR_DIR_KSTEPS];
        if constexpr (EMB) pe_gather<6, NR_DIR_KSTEPS>(dpe, xrow + NR_XYZ_CH, h);
        else pe_encode<6, NR_DIR_KSTEPS>(dpe, dx, dy, dz, h);
        f32x16 C[8];
        init_bias<4>(C, H + NR_H_BDIR, h);
        {
            float* fdst = SV + nr_sv_feat(nb) + (size_t)blk * NR_NATIVE(256);
            auto gb = from_acc(A);
            auto sd = side_acc(A, fdst, nullptr);
            segment<FwdTab, kDir, 0, 16, 4, QEND>(P, smem, wave, lane, C, gb, sd, f0);
        }
        {
            float* ddst = SV + nr_sv_dirpe(nb) + (size_t)blk * NR_NATIVE(32);
            auto getb = [&](auto gc, float (&x)[8]) {
                constexpr int g = decltype(gc)::value;
#pragma unroll
                for (int j = 0; j < 8; ++j) x[j] = dpe[8 * g + j];
            };
            auto side = [&](auto gc) {
                constexpr int g = decltype(gc)::value;
                if (!save) return;
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int grp = 2 * g + u;
                    f32x4 v = {dpe[4 * grp], dpe[4 * grp + 1], dpe[4 * grp + 2], dpe[4 * grp + 3]};
                    *reinterpret_cast<f32x4*>(ddst + (grp * 64 + lane) * 4) = v;
                }
            };
            segment<FwdTab, kDir + 16, 0, 2, 4, QEND>(P, smem, wave, lane, C, getb, side, f0);
        }
        relu<4>(C);
        float rgb[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float zc = head_dot<4>(C, H + NR_H_WRGB + 128 * c, h) + H[NR_H_BRGB + c];
            rgb[c] = 1.f / (1.f + expf(-zc));
        }
        if (valid && h == 0) {
            f32x4 o = {rgb[0], rgb[1], rgb[2], sigma};
            *reinterpret_cast<f32x4*>(a.out + (size_t)s * 4) = o;
        }
        if (save) {
            store_native<4>(reinterpret_cast<const f32x16(&)[4]>(C),
                            SV + nr_sv_hdir(nb) + (size_t)blk * NR_NATIVE(128), lane);
            store_mask<4>(reinterpret_cast<const f32x16(&)[4]>(C), mseg(8), lane);
        }
    }
}

// pack: bf16 pieces of the weights (map: flat*4 + piece, -1 = 0) after the
// fp32 head block (head_map: flat index, -1 = 0)
__global__ void pack3_kernel(const float* __restrict__ flat, const int32_t* __restrict__ map,
                             int64_t n, const int32_t* __restrict__ head_map,
                             char* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < NR_H_SIZE) {
        const int32_t m = head_map[i];
        reinterpret_cast<float*>(out)[i] = m >= 0 ? flat[m] : 0.f;
    }
    if (i >= n) return;
    const int32_t m = map[i];
    float v = 0.f;
    if (m >= 0) {
        const float w = flat[m >> 2];
        const int piece = m & 3;
        const float hi = (float)(__bf16)w;
        const float r1 = w - hi;
        const float mid = (float)(__bf16)r1;
        v = piece == 0 ? hi : (piece == 1 ? mid : r1 - mid);
    }
    reinterpret_cast<__bf16*>(out + kHeadBytes)[i] = (__bf16)v;
}

}  // namespace

NR_API int64_t nr_fwd3_packed_bytes(void) { return FwdTab::off(kQAll); }

NR_API int nr_pack_x3(const float* flat, const int32_t* map, int64_t n, const int32_t* head_map,
                      void* out, void* stream) {
    NR_REQUIRE(n == (FwdTab::off(kQAll) - kHeadBytes) / 2, "nr_pack_x3: map has %lld entries, "
               "expected %lld", (long long)n, (long long)((FwdTab::off(kQAll) - kHeadBytes) / 2));
    NR_REQUIRE(flat && map && head_map && out, "nr_pack_x3: null pointer");
    pack3_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        flat, map, n, head_map, reinterpret_cast<char*>(out));
    NR_LAUNCH_CHECK("nr_pack_x3");
    return 0;
}

NR_API int nr_mlp_fwd_x3(const void* packed, const float* rays, const float* z, int64_t n,
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
    Fwd3Args a{reinterpret_cast<const char*>(packed), nullptr, rays, z, x, (int)n,
               samples_per_ray, xstride, out, save};
    const int blocks = (int)((n + 32 * kWaves - 1) / (32 * kWaves));
    hipStream_t st = (hipStream_t)stream;
    if (emb) {
        if (sigma_only) mlp_fwd3_kernel<FWD_EMB, true><<<blocks, 64 * kWaves, 0, st>>>(a);
        else mlp_fwd3_kernel<FWD_EMB, false><<<blocks, 64 * kWaves, 0, st>>>(a);
    } else {
        if (sigma_only) mlp_fwd3_kernel<FWD_RAYS, true><<<blocks, 64 * kWaves, 0, st>>>(a);
        else mlp_fwd3_kernel<FWD_RAYS, false><<<blocks, 64 * kWaves, 0, st>>>(a);
    }
    NR_LAUNCH_CHECK("nr_mlp_fwd_x3");
    return 0;
}

NR_API int nr_mlp_sigma_points_x3(const void* packed, const float* pts, int64_t n,
                                  float* sigma_out, void* stream) {
    NR_REQUIRE(n >= 0 && n < (int64_t)1 << 31, "nr_mlp_sigma_points_x3: n out of range");
    if (n == 0) return 0;
    NR_REQUIRE(packed && pts && sigma_out, "nr_mlp_sigma_points_x3: null pointer");
    NR_REQUIRE(((uintptr_t)packed & 15) == 0, "nr_mlp_sigma_points_x3: packed alignment");
    Fwd3Args a{reinterpret_cast<const char*>(packed), pts, nullptr, nullptr, nullptr, (int)n, 1, 0,
               sigma_out, nullptr};
    const int blocks = (int)((n + 32 * kWaves - 1) / (32 * kWaves));
    mlp_fwd3_kernel<FWD_PTS, true><<<blocks, 64 * kWaves, 0, (hipStream_t)stream>>>(a);
    NR_LAUNCH_CHECK("nr_mlp_sigma_points_x3");
    return 0;
}
