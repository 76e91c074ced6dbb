// torchsearchsorted.searchsorted(a, v, out=None, side='left') -- the
// reference's only native dependency (git submodule, .gitmodules:1-3; called
// at models/rendering.py:2,37 and models/rendering_rgb_sm.py:2,40), as a
// standalone entry point.  The render path does not use it: nr_sample_pdf
// fuses the search into the inverse-CDF kernel.
//
// Per row r and query j: the number of entries of the sorted row a[r] that are
// < v[r, j] (side left) or <= v[r, j] (side right), i.e. numpy's
// searchsorted, written as int64.  One thread per query, a branch-free binary
// search over the row (rows are short -- 63 CDF knots at cfg2 -- and stay in
// L1/L2 across the row's queries).  Either operand may have a single row,
// which is then shared by every row of the other (the package's broadcast).
#include "common.h"

namespace {

template <typename T, bool Right>
__global__ void __launch_bounds__(256) searchsorted_kernel(const T* __restrict__ a,
                                                           const T* __restrict__ v,
                                                           int64_t nrows, int64_t na, int64_t nv,
                                                           int a_shared, int v_shared,
                                                           int64_t* __restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nrows * nv) return;
    const int64_t r = q / nv, j = q - r * nv;
    const T* row = a + (a_shared ? 0 : r * na);
    const T x = v[(v_shared ? 0 : r * nv) + j];
    // lo = count of entries ordered before x; invariant: row[0..lo) precede x
    int64_t lo = 0, len = na;
    while (len > 0) {
        const int64_t half = len >> 1;
        const T m = row[lo + half];
        // torch.searchsorted's comparisons (NaN queries land after every entry)
        const bool before = Right ? !(m > x) : !(m >= x);
        lo = before ? lo + half + 1 : lo;
        len = before ? len - half - 1 : half;
    }
    out[q] = lo;
}

template <typename T>
int launch(const char* name, const T* a, const T* v, int64_t nrows_a, int64_t na,
           int64_t nrows_v, int64_t nv, int right, int64_t* out, void* stream) {
    NR_REQUIRE(nrows_a >= 0 && nrows_v >= 0 && na >= 0 && nv >= 0, "%s: negative size", name);
    NR_REQUIRE(nrows_a == nrows_v || nrows_a == 1 || nrows_v == 1,
               "%s: a has %lld rows, v %lld (need equal, or one of them 1)", name,
               (long long)nrows_a, (long long)nrows_v);
    const int64_t nrows = nrows_a > nrows_v ? nrows_a : nrows_v;
    if (nrows_a == 0 || nrows_v == 0 || nv == 0) return 0;
    NR_REQUIRE((a || na == 0) && v && out, "%s: null pointer", name);
    const int64_t total = nrows * nv;
    NR_REQUIRE(total / 256 < ((int64_t)1 << 31), "%s: too many queries", name);
    const unsigned blocks = (unsigned)((total + 255) / 256);
    const int as = nrows_a == 1 && nrows > 1, vs = nrows_v == 1 && nrows > 1;
    hipStream_t st = (hipStream_t)stream;
    if (right)
        searchsorted_kernel<T, true><<<blocks, 256, 0, st>>>(a, v, nrows, na, nv, as, vs, out);
    else
        searchsorted_kernel<T, false><<<blocks, 256, 0, st>>>(a, v, nrows, na, nv, as, vs, out);
    NR_LAUNCH_CHECK(name);
    return 0;
}

}  // namespace

NR_API int nr_searchsorted(const float* a, const float* v, int64_t nrows_a, int64_t ncols_a,
                           int64_t nrows_v, int64_t ncols_v, int side_right, int64_t* out,
                           void* stream) {
    return launch("nr_searchsorted", a, v, nrows_a, ncols_a, nrows_v, ncols_v, side_right, out,
                  stream);
}

NR_API int nr_searchsorted_f64(const double* a, const double* v, int64_t nrows_a,
                               int64_t ncols_a, int64_t nrows_v, int64_t ncols_v, int side_right,
                               int64_t* out, void* stream) {
    return launch("nr_searchsorted_f64", a, v, nrows_a, ncols_a, nrows_v, ncols_v, side_right,
                  out, stream);
}
