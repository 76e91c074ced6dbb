// Microbenchmark (dev only): HBM write / read / copy bandwidth on MI355X with
// float4 accesses (plain and non-temporal), to price the saved-activation and
// gradient streams of the MLP kernels.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 dev/mb_bw.hip -o dev/mb_bw
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MODE>   // 0 write, 1 write nt, 2 read, 3 copy nt
__global__ void __launch_bounds__(256) bw_kernel(f32x4* __restrict__ dst, const f32x4* __restrict__ src,
                                                 size_t n, float* __restrict__ sink) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const f32x4 v = {1.f, 2.f, 3.f, (float)threadIdx.x};
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if constexpr (MODE == 0) dst[i] = v;
        else if constexpr (MODE == 1) __builtin_nontemporal_store(v, dst + i);
        else if constexpr (MODE == 2) acc += src[i];
        else __builtin_nontemporal_store(src[i], dst + i);
    }
    if constexpr (MODE == 2)
        if (acc[0] == 123.f) sink[0] = acc[1];
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int MODE>
void run(f32x4* d, f32x4* s, size_t n, float* sink, int blocks, const char* name) {
    for (int i = 0; i < 2; ++i) bw_kernel<MODE><<<blocks, 256>>>(d, s, n, sink);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int reps = 10;
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) bw_kernel<MODE><<<blocks, 256>>>(d, s, n, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    const double bytes = (double)n * 16 * (MODE == 3 ? 2 : 1);
    printf("%-10s blocks %6d: %.3f ms  %.2f TB/s\n", name, blocks, ms, bytes / ms / 1e9);
}

int main() {
    const size_t bytes = (size_t)6 << 30, n = bytes / 16;
    f32x4 *d, *s;
    float* sink;
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&s, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(s, 0, bytes));
    for (int blocks : {2048, 8192, 32768}) {
        run<0>(d, s, n, sink, blocks, "write");
        run<1>(d, s, n, sink, blocks, "write-nt");
        run<2>(d, s, n, sink, blocks, "read");
        run<3>(d, s, n / 2, sink, blocks, "copy-nt");
    }
    return 0;
}
