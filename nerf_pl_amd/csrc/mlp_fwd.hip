// Fused positional-encoding + NeRF MLP forward (models/nerf.py:21-38, 83-124;
// the chunked MLP loop of models/rendering.py:141-161).
//
// One wave evaluates 32 samples through all layers.  Every layer is computed in
// transposed form D[feature][sample] on v_mfma_f32_32x32x2_f32 so the
// accumulators (feature in registers, sample on the lane) are directly the B
// operand of the next layer: activations never leave registers.  Weights are
// pre-packed in MFMA A-fragment order (packing.py) and streamed from L2/HBM as
// one coalesced 1 KiB float4 wave load per (4 k-steps x 32 rows), prefetched
// one group ahead.  sin/cos positional encodings are computed in registers
// and fed straight into the first layer and the skip layer.
#include "layout.h"

namespace {

constexpr int kWaves = 4;   // waves per workgroup (one per SIMD)

template <int NT>
__device__ __forceinline__ void init_bias(f32x16 (&acc)[NT], const float* __restrict__ b, int h) {
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
__device__ __forceinline__ void relu(f32x16 (&acc)[NT]) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = acc[t][r] > 0.f ? acc[t][r] : 0.f;
}

// <w, acc> over this lane's features, then summed over both lane halves.
template <int NT>
__device__ __forceinline__ float head_dot(const f32x16 (&acc)[NT], const float* __restrict__ w, int h) {
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

// Positional encoding of one point, in packed k order (packing.py pe_feature):
// g=0 (x|y), g=1 (z|pad), g=2..1+NP sin pairs, g=2+NP..1+2NP cos pairs.
// Lane half h evaluates pair member m = i + NP*h: sin/cos(2^(m/3) * p[m%3]).
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
        const float arg = v * (float)(1 << k);   // freq * x, freq = 2^k exactly (nerf.py:17,36)
        float s, co;
        sincosf(arg, &s, &co);
        pe[2 + i] = s;
        pe[2 + NP + i] = co;
    }
#pragma unroll
    for (int g = 2 + 2 * NP; g < KS; ++g) pe[g] = 0.f;
}

// Same channels gathered from a pre-embedded row (NeRF.forward(x) API path).
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

struct FwdArgs {
    const float* packed;
    const float* pts;    // (n, 3) points (FWD_PTS: dense sigma query)
    const float* rays;   // (n_rays, 8) [o, d, near, far]
    const float* z;      // (n) depths, sample-major (ray*spr + k)
    const float* x;      // (n, xstride) embedded input (EMB path)
    int n;               // samples
    int spr;             // samples per ray
    int xstride;
    float* out;          // (n, 4) [rgb, sigma] or (n, 1) sigma
    float* save;         // saved activations (training) or nullptr
    // LIST (nr_mlp_fwd_listed): position q < *scount evaluates sample slist[q],
    // activations saved by position, no output
    const int32_t* slist; const int32_t* scount;
};

// LIST: the deferred save of a training forward (mlp_fwd3.hip);
// blk is then a block of positions.  The full graph saves its activations as
// sample-major rows (layout.h store_row_piece; PE and dir PE rows hold the
// packed k order, column 32h + g / 16h + g), so the weight gradient of a
// sample list gathers whole 128-B lines (the block-native
// layout made it fetch 1.69x the listed samples' bytes); the sigma-only
// training forward keeps the block-native layout
template <int MODE, bool SIGMA_ONLY, bool LIST = false>
__global__ void __launch_bounds__(64 * kWaves, 1) mlp_fwd_kernel(FwdArgs a) {
    constexpr bool EMB = MODE == FWD_EMB;
    constexpr bool ROWS = NR_F32_ROWS && !SIGMA_ONLY;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int h = lane >> 5;
    const int blk = blockIdx.x * kWaves + wave;           // 32-sample block of this wave
    const int m = LIST ? __builtin_amdgcn_readfirstlane(*a.scount) : a.n;
    if (LIST && (int)blockIdx.x * kWaves * 32 >= m) return;   // whole workgroup, before the barrier
    const int s_raw = blk * 32 + (lane & 31);
    const bool valid = s_raw < m;
    const int s = LIST ? a.slist[valid ? s_raw : 0] : (valid ? s_raw : a.n - 1);
    const float* P = a.packed;
    // biases and the sigma/rgb heads come from LDS so their reads never queue
    // behind in-flight weight loads (vmcnt retires in issue order)
    __shared__ __attribute__((aligned(16))) float Hs[NR_H_SIZE];
    {
        const f32x4* src = reinterpret_cast<const f32x4*>(a.packed + NR_F_HEAD);
        for (int i = threadIdx.x; i < NR_H_SIZE / 4; i += 64 * kWaves)
            reinterpret_cast<f32x4*>(Hs)[i] = src[i];
        __syncthreads();
    }
    const float* H = Hs;
    const int nb = (int)nr_blocks_pad(a.n);             // segment stride (padded)
    const bool save = a.save != nullptr && blk < (m + 31) / 32;   // whole block, tail lanes included
    float* const SV = a.save;

    // ---- point and direction ------------------------------------------------
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
        // rendering.py:234 -- o + d*z as separate fp32 mul and add
        px = nr_add(r[0], nr_mul(r[3], zz));
        py = nr_add(r[1], nr_mul(r[4], zz));
        pz = nr_add(r[2], nr_mul(r[5], zz));
        dx = r[3]; dy = r[4]; dz = r[5];
    }

    f32x16 A[8], B[8];
    f32x4 wq[8];                 // weight group in flight across layer boundaries
    nr_ld_first<8>(P + NR_F_L1, lane, wq);
    // Saved-activation stores (training): each layer's output is written while
    // the next layer runs (side hook), one float4 per weight group.
    auto hseg = [&](int l) { return SV + nr_sv_h(l, nb) + (size_t)blk * NR_NATIVE(256); };
    auto mseg = [&](int l) {
        return reinterpret_cast<uint32_t*>(SV + nr_sv_mask(nb)) + ((size_t)blk * NR_MASK_LAYERS + l) * 256;
    };
    auto side_acc8 = [&](const f32x16 (&X)[8], float* dst, uint32_t* msk) {
        return [&X, dst, msk, save, lane](int grp) {
            if (!save) return;
            if (grp < 32) {
                if constexpr (ROWS) store_row_piece<8>(X, grp, 256, dst, lane);
                else store_native_piece<8>(X, grp, dst, lane);
            }
            if (grp == 0 && msk) store_mask<8>(X, msk, lane);
        };
    };
    {   // layer 1: PE(63) -> 256
        float pe[NR_PE_KSTEPS];
        if constexpr (EMB) pe_gather<15, NR_PE_KSTEPS>(pe, xrow, h);
        else pe_encode<15, NR_PE_KSTEPS>(pe, px, py, pz, h);
        float* pdst = SV + (size_t)blk * NR_NATIVE(64);
        init_bias<8>(A, H + NR_H_BIAS(1), h);
        nr_mm_chain<NR_PE_KSTEPS, 8, 8>(P + NR_F_L1, P + NR_F_L2, lane, A, wq,
                                        [&](int g) { return pe[g]; },
                                        [&](int grp) {
                                            if (!save) return;
                                            f32x4 v = {pe[4 * grp], pe[4 * grp + 1], pe[4 * grp + 2],
                                                       pe[4 * grp + 3]};
                                            float* d = ROWS ? pdst + (lane & 31) * 64 + 32 * h + 4 * grp
                                                            : pdst + (grp * 64 + lane) * 4;
                                            *reinterpret_cast<f32x4*>(d) = v;
                                        });
        relu<8>(A);
    }

#define NR_DENSE(DST, SRC, LOFF, NEXT, L)                                                    \
    init_bias<8>(DST, H + NR_H_BIAS(L), h);                                                   \
    nr_mm_chain<128, 8, 8>(P + LOFF, P + NEXT, lane, DST, wq,                                 \
                           [&](int g) { return SRC[g >> 4][g & 15]; },                        \
                           side_acc8(SRC, hseg(L - 2), mseg(L - 2)));                         \
    relu<8>(DST);

    NR_DENSE(B, A, NR_F_L2, NR_F_L3, 2)   // stores h1 while computing h2
    NR_DENSE(A, B, NR_F_L3, NR_F_L4, 3)
    NR_DENSE(B, A, NR_F_L4, NR_F_L5, 4)
    {   // layer 5: cat[PE, h4] -> 256 (skip, nerf.py:108-109); PE recomputed
        float pe[NR_PE_KSTEPS];
        if constexpr (EMB) pe_gather<15, NR_PE_KSTEPS>(pe, xrow, h);
        else pe_encode<15, NR_PE_KSTEPS>(pe, px, py, pz, h);
        init_bias<8>(A, H + NR_H_BIAS(5), h);
        const float* l5h = P + NR_F_L5 + NR_PL(NR_PE_KSTEPS, 8);
        nr_mm_chain<NR_PE_KSTEPS, 8, 8>(P + NR_F_L5, l5h, lane, A, wq, [&](int g) { return pe[g]; });
        nr_mm_chain<128, 8, 8>(l5h, P + NR_F_L6, lane, A, wq,
                               [&](int g) { return B[g >> 4][g & 15]; },
                               side_acc8(B, hseg(3), mseg(3)));
        relu<8>(A);
    }
    NR_DENSE(B, A, NR_F_L6, NR_F_L7, 6)
    NR_DENSE(A, B, NR_F_L7, NR_F_L8, 7)
    {   // layer 8 (chains into `final` unless sigma-only)
        init_bias<8>(B, H + NR_H_BIAS(8), h);
        nr_mm_chain<128, 8, 8>(P + NR_F_L8, SIGMA_ONLY ? nullptr : P + NR_F_FINAL, lane, B, wq,
                               [&](int g) { return A[g >> 4][g & 15]; },
                               side_acc8(A, hseg(6), mseg(6)));
        relu<8>(B);
    }
#undef NR_DENSE

    // sigma = Linear(256, 1)(h8), raw (nerf.py:112)
    const float sigma = head_dot<8>(B, H + NR_H_WSIG, h) + H[NR_H_BSIG];
    if constexpr (SIGMA_ONLY) {
        if (a.save != nullptr) {
            // training a sigma-only graph (rendering_shadows.py:167): layers 1-8
            // and the sigma head only; h8 and its ReLU mask saved where the full
            // graph saves them, out rows (n, 4) [0, 0, 0, sigma] for the
            // backward's contract (as mlp_fwd3.hip's sigma-only training forward)
            if (save) {
                store_native<8>(B, hseg(7), lane);
                store_mask<8>(B, mseg(7), lane);
            }
            if (valid && h == 0 && !LIST)
                *reinterpret_cast<f32x4*>(a.out + (size_t)s * 4) = f32x4{0.f, 0.f, 0.f, sigma};
        } else if (valid && h == 0) {
            a.out[s] = sigma;
        }
        return;
    } else {
        // xyz_encoding_final: Linear(256,256), no activation (nerf.py:116); stores h8
        init_bias<8>(A, H + NR_H_BFINAL, h);
        nr_mm_chain<128, 8, 4>(P + NR_F_FINAL, P + NR_F_DIR, lane, A, wq,
                               [&](int g) { return B[g >> 4][g & 15]; },
                               side_acc8(B, hseg(7), mseg(7)));

        // dir_encoding: ReLU(Linear(283,128)(cat[feat, PE(dir)])) (nerf.py:118-119)
        float dpe[NR_DIR_KSTEPS];
        if constexpr (EMB) pe_gather<6, NR_DIR_KSTEPS>(dpe, xrow + NR_XYZ_CH, h);
        else pe_encode<6, NR_DIR_KSTEPS>(dpe, dx, dy, dz, h);
        f32x16 C[4];
        init_bias<4>(C, H + NR_H_BDIR, h);
        // feat is not saved: the dir layer's feat-column weight gradient is
        // formed from h8 (wgrad.hip task 10, nr_wgrad_dir_feat)
        const float* dpw = P + NR_F_DIR + NR_PL(128, 4);
        nr_mm_chain<128, 4, 4>(P + NR_F_DIR, dpw, lane, C, wq,
                               [&](int g) { return A[g >> 4][g & 15]; });
        float* ddst = SV + nr_sv_dirpe(nb) + (size_t)blk * NR_NATIVE(32);
        nr_mm_chain<NR_DIR_KSTEPS, 4, 4>(dpw, nullptr, lane, C, wq,
                                         [&](int g) { return dpe[g]; },
                                         [&](int grp) {
                                             if (!save) return;
                                             f32x4 v = {dpe[4 * grp], dpe[4 * grp + 1],
                                                        dpe[4 * grp + 2], dpe[4 * grp + 3]};
                                             float* d = ROWS ? ddst + (lane & 31) * 32 + 16 * h + 4 * grp
                                                             : ddst + (grp * 64 + lane) * 4;
                                             *reinterpret_cast<f32x4*>(d) = v;
                                         });
        relu<4>(C);

        // rgb = Sigmoid(Linear(128,3)) (nerf.py:79-81,120)
        float rgb[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float zc = head_dot<4>(C, H + NR_H_WRGB + 128 * c, h) + H[NR_H_BRGB + c];
            rgb[c] = 1.f / (1.f + expf(-zc));
        }
        if (valid && h == 0 && !LIST) {
            f32x4 o = {rgb[0], rgb[1], rgb[2], sigma};
            *reinterpret_cast<f32x4*>(a.out + (size_t)s * 4) = o;
        }
        if (save) {   // hdir: last layer, stored at the end
            float* hd = SV + nr_sv_hdir(nb) + (size_t)blk * NR_NATIVE(128);
            if constexpr (ROWS) store_rows<4>(C, hd, lane);
            else store_native<4>(C, hd, lane);
            store_mask<4>(C, mseg(8), lane);
        }
    }
}

}  // namespace

NR_API int nr_mlp_fwd(const float* packed, const float* rays, const float* z, int64_t n,
                      int samples_per_ray, const float* x, int xstride, int sigma_only,
                      float* out, float* save, void* stream) {
    NR_REQUIRE(n >= 0 && n < (int64_t)1 << 31, "nr_mlp_fwd: n=%lld out of range", (long long)n);
    if (n == 0) return 0;
    NR_REQUIRE(packed && out, "nr_mlp_fwd: null packed/out");
    NR_REQUIRE(((uintptr_t)packed & 15) == 0 && ((uintptr_t)out & 15) == 0 &&
                   ((uintptr_t)save & 15) == 0,
               "nr_mlp_fwd: packed/out/save must be 16-byte aligned");
    const bool emb = x != nullptr;
    NR_REQUIRE(!(sigma_only && save && emb),
               "nr_mlp_fwd: a sigma_only run keeps activations only on the ray path");
    if (emb) {
        NR_REQUIRE(xstride >= (sigma_only ? NR_XYZ_CH : NR_XYZ_CH + NR_DIR_CH),
                   "nr_mlp_fwd: xstride %d too small", xstride);
    } else {
        NR_REQUIRE(rays && z && samples_per_ray > 0, "nr_mlp_fwd: rays/z/samples_per_ray");
    }
    FwdArgs a{packed, nullptr, rays, z, x, (int)n, samples_per_ray, xstride, out, save};
    const int blocks = (int)((n + 32 * kWaves - 1) / (32 * kWaves));
    hipStream_t st = (hipStream_t)stream;
    if (emb) {
        if (sigma_only) mlp_fwd_kernel<FWD_EMB, true><<<blocks, 64 * kWaves, 0, st>>>(a);
        else mlp_fwd_kernel<FWD_EMB, false><<<blocks, 64 * kWaves, 0, st>>>(a);
    } else {
        if (sigma_only) mlp_fwd_kernel<FWD_RAYS, true><<<blocks, 64 * kWaves, 0, st>>>(a);
        else mlp_fwd_kernel<FWD_RAYS, false><<<blocks, 64 * kWaves, 0, st>>>(a);
    }
    NR_LAUNCH_CHECK("nr_mlp_fwd");
    return 0;
}

// the deferred save: the training forward's activations of the samples listed
// in samples[0 .. *count), saved by position into save (sized for n samples)
NR_API int nr_mlp_fwd_listed(const float* packed, const float* rays, const float* z, int64_t n,
                             int samples_per_ray, int sigma_only, float* save,
                             const int32_t* samples, const int32_t* count, void* stream) {
    NR_REQUIRE(n >= 0 && n < (int64_t)1 << 31, "nr_mlp_fwd_listed: n=%lld out of range", (long long)n);
    if (n == 0) return 0;
    NR_REQUIRE(packed && rays && z && save && samples && count && samples_per_ray > 0,
               "nr_mlp_fwd_listed: null pointer or samples_per_ray");
    NR_REQUIRE(((uintptr_t)packed & 15) == 0 && ((uintptr_t)save & 15) == 0,
               "nr_mlp_fwd_listed: packed/save must be 16-byte aligned");
    FwdArgs a{packed, nullptr, rays, z, nullptr, (int)n, samples_per_ray, 0, nullptr, save, samples,
              count};
    const int blocks = (int)((n + 32 * kWaves - 1) / (32 * kWaves));
    hipStream_t st = (hipStream_t)stream;
    if (sigma_only) mlp_fwd_kernel<FWD_RAYS, true, true><<<blocks, 64 * kWaves, 0, st>>>(a);
    else mlp_fwd_kernel<FWD_RAYS, false, true><<<blocks, 64 * kWaves, 0, st>>>(a);
    NR_LAUNCH_CHECK("nr_mlp_fwd_listed");
    return 0;
}

// Dense sigma query at points (extract_color_mesh.py:114-137): sigma-only MLP on
// (n,3) points with the positional encoding computed in-kernel.
NR_API int nr_mlp_sigma_points(const float* packed_fwd, const float* pts, int64_t n,
                               float* sigma_out, void* stream) {
    NR_REQUIRE(n >= 0 && n < (int64_t)1 << 31, "nr_mlp_sigma_points: n out of range");
    if (n == 0) return 0;
    NR_REQUIRE(packed_fwd && pts && sigma_out, "nr_mlp_sigma_points: null pointer");
    NR_REQUIRE(((uintptr_t)packed_fwd & 15) == 0, "nr_mlp_sigma_points: packed must be 16-byte aligned");
    FwdArgs a{packed_fwd, pts, nullptr, nullptr, nullptr, (int)n, 1, 0, sigma_out, nullptr};
    const int blocks = (int)((n + 32 * kWaves - 1) / (32 * kWaves));
    mlp_fwd_kernel<FWD_PTS, true><<<blocks, 64 * kWaves, 0, (hipStream_t)stream>>>(a);
    NR_LAUNCH_CHECK("nr_mlp_sigma_points");
    return 0;
}
