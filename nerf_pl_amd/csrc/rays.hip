// On-device ray generation for the training batch.
//
// Reference: datasets/ray_utils.py:5-93 (get_ray_directions, get_rays,
// get_ndc_rays), datasets/blender.py:54-86 and datasets/llff.py:213-249 (the
// (n_images*H*W, 8) ray buffer), train.py:89-94 (a shuffled DataLoader over
// it).  Here a batch is generated straight from the camera poses: ray k is
// global pixel g = sel[k] (or k) = pose * H*W + row * W + col, so the ray
// buffer and its host->device copy disappear; the target colours of the same
// pixels are gathered in the same pass.
#include "common.h"

namespace {

struct RayGenArgs {
    const float* c2w;  // (n_poses, 3, 4)
    int64_t n_poses; int H, W;
    float w_half, h_half, focal, near, far;
    int ndc; float ndc_near, ndc_cw, ndc_ch, ndc_2near;
    const int64_t* sel; int64_t n;
    const float* rgb_pool; float* rgb_out;
    float* rays;
};

__global__ void __launch_bounds__(256) gen_rays_kernel(RayGenArgs a) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.n) return;
    const int64_t g = a.sel ? a.sel[k] : k;
    const int64_t hw = (int64_t)a.H * a.W;
    if (g < 0 || g >= a.n_poses * hw) {          // out-of-range selection: NaN ray, no read
        const float q = __builtin_nanf("");
        f32x4* out = reinterpret_cast<f32x4*>(a.rays + k * 8);
        out[0] = f32x4{q, q, q, q};
        out[1] = f32x4{q, q, q, q};
        if (a.rgb_out) a.rgb_out[k * 3] = a.rgb_out[k * 3 + 1] = a.rgb_out[k * 3 + 2] = q;
        return;
    }
    const int64_t p = g / hw;
    const int64_t pix = g - p * hw;
    const float i = (float)(pix % a.W), j = (float)(pix / a.W);
    // get_ray_directions (ray_utils.py:19-22): no +0.5 centering
    const float dc[3] = {nr_sub(i, a.w_half) / a.focal, -(nr_sub(j, a.h_half) / a.focal), -1.f};
    const float* m = a.c2w + p * 12;
    // get_rays (:42-43): d = dirs @ c2w[:, :3].T, normalised
    float d[3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
        d[r] = nr_add(nr_add(nr_mul(dc[0], m[r * 4]), nr_mul(dc[1], m[r * 4 + 1])),
                      nr_mul(dc[2], m[r * 4 + 2]));
    const float nrm = sqrtf(nr_add(nr_add(nr_mul(d[0], d[0]), nr_mul(d[1], d[1])), nr_mul(d[2], d[2])));
    d[0] = d[0] / nrm; d[1] = d[1] / nrm; d[2] = d[2] / nrm;
    float o[3] = {m[3], m[7], m[11]};
    float near = a.near, far = a.far;
    if (a.ndc) {
        // get_ndc_rays (:75-93) with near plane ndc_near; near/far become 0/1
        const float t = -nr_add(a.ndc_near, o[2]) / d[2];
        o[0] = nr_add(o[0], nr_mul(t, d[0]));
        o[1] = nr_add(o[1], nr_mul(t, d[1]));
        o[2] = nr_add(o[2], nr_mul(t, d[2]));
        const float ox = o[0] / o[2], oy = o[1] / o[2];
        const float o2 = nr_add(1.f, a.ndc_2near / o[2]);
        const float n0 = nr_mul(a.ndc_cw, ox), n1 = nr_mul(a.ndc_ch, oy);
        const float e0 = nr_mul(a.ndc_cw, nr_sub(d[0] / d[2], ox));
        const float e1 = nr_mul(a.ndc_ch, nr_sub(d[1] / d[2], oy));
        o[0] = n0; o[1] = n1; o[2] = o2;
        d[0] = e0; d[1] = e1; d[2] = 1.f - o2;
    }
    f32x4* out = reinterpret_cast<f32x4*>(a.rays + k * 8);
    out[0] = f32x4{o[0], o[1], o[2], d[0]};
    out[1] = f32x4{d[1], d[2], near, far};
    if (a.rgb_out) {
        a.rgb_out[k * 3 + 0] = a.rgb_pool[g * 3 + 0];
        a.rgb_out[k * 3 + 1] = a.rgb_pool[g * 3 + 1];
        a.rgb_out[k * 3 + 2] = a.rgb_pool[g * 3 + 2];
    }
}

}  // namespace

NR_API int nr_gen_rays(const float* c2w, int64_t n_poses, int H, int W, float w_half,
                       float h_half, float focal, float near, float far, int ndc, float ndc_near,
                       float ndc_cw, float ndc_ch, float ndc_2near, const int64_t* sel, int64_t n,
                       const float* rgb_pool, float* rgb_out, float* rays, void* stream) {
    NR_REQUIRE(n >= 0 && n_poses > 0 && H > 0 && W > 0, "nr_gen_rays: bad sizes");
    if (n == 0) return 0;
    NR_REQUIRE(c2w && rays, "nr_gen_rays: null pointer");
    NR_REQUIRE(!rgb_out || rgb_pool, "nr_gen_rays: rgb_out needs rgb_pool");
    NR_REQUIRE(((uintptr_t)rays & 15) == 0, "nr_gen_rays: rays must be 16-byte aligned");
    NR_REQUIRE(sel || n <= n_poses * H * W, "nr_gen_rays: n exceeds the pixel count");
    RayGenArgs a{c2w, n_poses, H, W, w_half, h_half, focal, near, far, ndc, ndc_near, ndc_cw,
                 ndc_ch, ndc_2near, sel, n, rgb_pool, rgb_out, rays};
    gen_rays_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(a);
    NR_LAUNCH_CHECK("nr_gen_rays");
    return 0;
}
