// Self-checks exported through the C ABI: layout constants (callable without a
// GPU) and an MFMA lane-map probe (tests/test_gpu_kernels.py).
#include "layout.h"

NR_API int64_t nr_layout_query(int what) {
    switch (what) {
        case 0: return NR_F_TOTAL;
        case 1: return NR_F_HEAD;
        case 2: return NR_B_TOTAL;
        case 3: return NR_SAVE_PER_BLOCK;
        case 4: return NR_GRAD_PER_BLOCK;
        case 5: return NR_H_SIZE;
        case 6: return NR_F_L5;
        case 7: return NR_F_DIR;
        case 8: return NR_B_L5T;
        // ABI revision: 2 = a full-graph nr_wgrad* launch leaves G = sum dz_dir h8^T
        // in dir_encoding.0.weight[:, :256] and zeros in xyz_encoding_final, and
        // nr_wgrad_dir_feat must follow it (round 5; 1 = every gradient final)
        case 9: return 2;
        default: return -1;
    }
}

namespace {
// D = A(32x2) * B(2x32) with A[i][k] = a_in[i*2+k], B[k][j] = b_in[k*32+j];
// writes D[row][col] = d_out[row*32+col] using the documented C/D lane map.
__global__ void probe_mfma_kernel(const float* a_in, const float* b_in, float* d_out) {
    const int l = threadIdx.x;
    const float a = a_in[(l & 31) * 2 + (l >> 5)];
    const float b = b_in[(l >> 5) * 32 + (l & 31)];
    f32x16 c = {};
    c = nr_mfma32(a, b, c);
    for (int r = 0; r < 16; ++r) d_out[nr_acc_row(r, l >> 5) * 32 + (l & 31)] = c[r];
}
}  // namespace

NR_API int nr_probe_mfma32(const float* a, const float* b, float* d, void* stream) {
    probe_mfma_kernel<<<1, 64, 0, (hipStream_t)stream>>>(a, b, d);
    NR_LAUNCH_CHECK("nr_probe_mfma32");
    return 0;
}
