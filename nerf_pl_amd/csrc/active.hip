// Active samples of a training backward ("zero-gradient
// samples").  A sample whose output gradient (d rgb, d sigma) is exactly zero
// -- sigma <= 0 after the ReLU of rendering.py:169-176 (alpha = 0, so its
// weight is 0 and the ReLU passes no sigma gradient), or a transmittance
// underflowed behind an opaque surface -- contributes exactly zero to every
// dz of the data-gradient chain and to every weight-gradient sum.  At the
// bench's random init about half the samples are such (sigma + noise <= 0),
// scattered; with trained weights ~93%, mostly in runs (empty space, and
// everything behind a surface).  nr_active_samples lists the others in
// ascending order (deterministic: the weight gradient's split-K partition
// depends only on the list); the *_active entry points then run the
// data-gradient chain over the listed samples, packed densely (positions
// 0..m-1), and the weight gradient gathers the saved activations of the
// listed samples.
#include "common.h"
#include "layout.h"

namespace {

constexpr int kWaves = 4;
constexpr int kScanT = 1024;

// per 32-sample block b: bits[b] = which of its samples have a nonzero output
// gradient row (NaN counts as nonzero: it propagates), cnt[b] = how many.
// One wave per block, 64 lanes x float2 (lane 2j + i holds columns 2i, 2i+1
// of sample j).
__global__ void __launch_bounds__(64 * kWaves) active_bits_kernel(
        const float* __restrict__ g_out, int64_t n, uint32_t* __restrict__ bits,
        int32_t* __restrict__ cnt) {
    const int lane = threadIdx.x & 63;
    const int64_t blk = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
    const int64_t nreal = (n + 31) / 32;
    if (blk >= nreal) return;
    const int64_t s = blk * 32 + (lane >> 1);
    bool nz = false;
    if (s < n) {
        const float2 v = *reinterpret_cast<const float2*>(g_out + s * 4 + 2 * (lane & 1));
        nz = !(v.x == 0.f) || !(v.y == 0.f);
    }
    const uint64_t b = __ballot(nz);
    // sample j active if lane 2j or 2j + 1 saw a nonzero: fold the bit pairs
    uint64_t x = (b | (b >> 1)) & 0x5555555555555555ull;
    x = (x | (x >> 1)) & 0x3333333333333333ull;
    x = (x | (x >> 2)) & 0x0f0f0f0f0f0f0f0full;
    x = (x | (x >> 4)) & 0x00ff00ff00ff00ffull;
    x = (x | (x >> 8)) & 0x0000ffff0000ffffull;
    x = (x | (x >> 16)) & 0x00000000ffffffffull;
    if (lane == 0) {
        bits[blk] = (uint32_t)x;
        cnt[blk] = __popc((uint32_t)x);
    }
}

// exclusive scan of cnt (in place, nreal entries) by one workgroup: thread t
// owns the contiguous run [t K, t K + K), K = ceil(nreal / kScanT).  Pass 1
// sums each run (its loads independent, several in flight), one block-wide
// scan of the run sums, pass 2 rewrites each run with its offsets (the
// values re-read from L2).  The walk in kScanT-entry chunks it replaces waited
// for one dependent load round trip per chunk (cfg2's fine pass: 24 chunks,
// 16.6 us); *count = the total
__global__ void __launch_bounds__(kScanT) active_scan_kernel(int32_t* __restrict__ cnt,
                                                             int64_t nreal,
                                                             int32_t* __restrict__ count) {
    __shared__ int wsum[kScanT / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t K = (nreal + kScanT - 1) / kScanT;
    const int64_t r0 = min((int64_t)tid * K, nreal), r1 = min(r0 + K, nreal);
    int run = 0;
    {
        int part[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int64_t b = r0;
        for (; b + 8 <= r1; b += 8)
#pragma unroll
            for (int i = 0; i < 8; ++i) part[i] += cnt[b + i];
        // the tail (< 8 entries) goes to part[0]: a runtime index into part
        // would put the array in scratch
        for (; b < r1; ++b) part[0] += cnt[b];
#pragma unroll
        for (int i = 0; i < 8; ++i) run += part[i];
    }
    int x = run;        // inclusive scan of the run sums within the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kScanT / 64; ++w) {
        const int t = wsum[w];
        before += w < wave ? t : 0;
        total += t;
    }
    int off = before + x - run;
    int64_t b = r0;
    for (; b + 8 <= r1; b += 8) {       // 8 loads in flight, then their 8 stores
        int v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = cnt[b + i];
#pragma unroll
        for (int i = 0; i < 8; ++i) { cnt[b + i] = off; off += v[i]; }
    }
    for (; b < r1; ++b) {
        const int v = cnt[b];
        cnt[b] = off;
        off += v;
    }
    if (tid == 0) *count = total;
}

// samples[offset[b] + rank of j among b's active samples] = 32 b + j
__global__ void __launch_bounds__(256) active_scatter_kernel(const uint32_t* __restrict__ bits,
                                                             const int32_t* __restrict__ off,
                                                             int64_t n,
                                                             int32_t* __restrict__ samples) {
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= n) return;
    const uint32_t m = bits[s >> 5];
    const int j = (int)(s & 31);
    if ((m >> j) & 1u) samples[off[s >> 5] + __popc(m & ((1u << j) - 1u))] = (int32_t)s;
}

}  // namespace

NR_API int64_t nr_active_scratch_ints(int64_t n) { return 2 * ((n + 31) / 32); }

// samples: n int32 (the first *count entries: the active samples, ascending);
// count: one int32; scratch: nr_active_scratch_ints(n) int32.
NR_API int nr_active_samples(const float* g_out, int64_t n, int32_t* samples, int32_t* count,
                             int32_t* scratch, void* stream) {
    NR_REQUIRE(n >= 0 && n < (int64_t)1 << 31, "nr_active_samples: n out of range");
    NR_REQUIRE(count && (n == 0 || (g_out && samples && scratch)), "nr_active_samples: null pointer");
    NR_REQUIRE(((uintptr_t)g_out & 7) == 0, "nr_active_samples: g_out must be 8-byte aligned");
    hipStream_t st = (hipStream_t)stream;
    const int64_t nreal = (n + 31) / 32;
    uint32_t* bits = reinterpret_cast<uint32_t*>(scratch);
    int32_t* cnt = scratch + nreal;
    if (nreal > 0) {
        active_bits_kernel<<<(unsigned)((nreal + kWaves - 1) / kWaves), 64 * kWaves, 0, st>>>(
            g_out, n, bits, cnt);
        NR_LAUNCH_CHECK("nr_active_samples");
    }
    active_scan_kernel<<<1, kScanT, 0, st>>>(cnt, nreal, count);
    NR_LAUNCH_CHECK("nr_active_samples");
    if (n > 0) {
        active_scatter_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(bits, cnt, n, samples);
        NR_LAUNCH_CHECK("nr_active_samples");
    }
    return 0;
}
