/* nerf_pl_amd -- C ABI of the MI355X (gfx950) volumetric-rendering hot path.
 *
 * Drop-in boundary for ktiwary2/nerf_pl's render_rays / sample_pdf / NeRF
 * path (models/rendering.py, models/nerf.py).  The reference is pure Python on
 * PyTorch; its only native dependency is the torchsearchsorted extension
 * (.gitmodules:1-3), which nr_sample_pdf replaces.  Each entry point below
 * names the reference code it stands in for.
 *
 * Conventions
 *   - every pointer is device memory allocated by the caller (float32, rows
 *     contiguous); the library never allocates, frees or retains pointers;
 *   - `stream` is a hipStream_t (e.g. torch.cuda.current_stream().cuda_stream);
 *     work is enqueued asynchronously and no call synchronises the host;
 *   - return 0 on success, a hipError_t or NR_EINVAL (10001) / NR_EALIGN (10002)
 *     otherwise; nr_last_error() gives a thread-local message;
 *   - "rays" are (n_rays, 8) = [origin(3), direction(3), near, far]
 *     (rendering.py:209-210); per-sample arrays are ray-major (ray*S + k).
 *   - random draws: a non-NULL replay array is used verbatim (parity with the
 *     reference's torch.rand / torch.randn); NULL means draw in-kernel from
 *     Philox4x32-10 keyed by (seed, stream id, element index).
 */
#ifndef NERF_PL_AMD_H
#define NERF_PL_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Thread-local text of the last error. */
const char* nr_last_error(void);

/* Layout constants shared with the Python packer (0: forward packed floats,
 * 1: head offset, 2: backward packed floats, 3: saved floats/sample,
 * 4: gradient floats/sample, 5: head floats, 6..8: layer offsets) and
 * 9: the ABI revision -- 2 since full-graph nr_wgrad* launches leave G in
 * dir_encoding.0.weight[:, :256] for nr_wgrad_dir_feat to finish (see
 * nr_wgrad below); a caller built against revision 1 must refuse it. */
int64_t nr_layout_query(int what);

/* Gather the flat parameter buffer (595,844 floats, NeRF.named_parameters()
 * order) into MFMA fragment order: out[i] = map[i] >= 0 ? flat[map[i]] : 0.
 * Replaces nothing in the reference (its GEMMs read nn.Linear weights
 * directly, nerf.py:60-81); run once per weight update. */
int nr_pack(const float* flat, const int32_t* map, int64_t n, float* out, void* stream);

/* Embedding.forward (models/nerf.py:21-38): x (n,3) -> out (n, 3*(2*n_freqs+1)). */
int nr_embed(const float* x, int64_t n, int n_freqs, float* out, void* stream);

/* Fused positional encoding + NeRF MLP forward -- replaces the chunked
 * `embedding_xyz` + `NeRF.forward` loop of inference() (rendering.py:141-161,
 * nerf.py:83-124).
 *   Ray path (x == NULL): sample s uses point o + d*z[s] of ray s/samples_per_ray
 *     (rendering.py:234-235) and that ray's direction encoding.
 *   Embedded path (x != NULL): x is (n, xstride) pre-embedded [xyz_emb(63),
 *     dir_emb(27)] or xyz_emb only when sigma_only (NeRF.forward(x) API).
 *   out: (n,4) [rgb, sigma] or (n,1) sigma when sigma_only.
 *   save: NULL for inference, else nr_blocks_pad(n) * (nr_layout_query(3) + 11) + 16
 *     floats: activations kept for nr_mlp_bwd / nr_wgrad (training), then the
 *     f16x3 gradient statistics (layout.h nr_stats_floats). */
int nr_mlp_fwd(const float* packed_fwd, const float* rays, const float* z, int64_t n,
               int samples_per_ray, const float* x, int xstride, int sigma_only, float* out,
               float* save, void* stream);

/* bf16x6 arithmetic: every fp32 operand split exactly into three
 * bf16 pieces, the six piece products of order <= 2^-16 accumulated in fp32 on
 * v_mfma_f32_32x32x16_bf16 -- fp32-level accuracy at 2.67x the fp32 MFMA rate.
 * nr_pack_x3 builds its forward weight buffer (nr_fwd3_packed_bytes() bytes:
 * the fp32 head block, then bf16 k-groups) from the flat parameters with the
 * maps of packing.build_fwd3_map (map: flat*4 + piece, -1 = 0; n entries);
 * nr_mlp_fwd_x3 / nr_mlp_sigma_points_x3 have the contracts of nr_mlp_fwd /
 * nr_mlp_sigma_points and write the same saved activations. */
int64_t nr_fwd3_packed_bytes(void);
int nr_pack_x3(const float* flat, const int32_t* map, int64_t n, const int32_t* head_map,
               void* out, void* stream);
int nr_mlp_fwd_x3(const void* packed, const float* rays, const float* z, int64_t n,
                  int samples_per_ray, const float* x, int xstride, int sigma_only, float* out,
                  float* save, void* stream);
int nr_mlp_sigma_points_x3(const void* packed, const float* pts, int64_t n, float* sigma_out,
                           void* stream);
/* bf16x6 data-gradient chain: nr_pack_bwd_x3 packs the transposed weights
 * (packing.build_bwd3_map, n entries, 3,342,336 bytes); nr_mlp_bwd_x3 has the
 * contract of nr_mlp_bwd. */
int nr_pack_bwd_x3(const float* flat, const int32_t* map, int64_t n, void* out, void* stream);
int nr_mlp_bwd_x3(const void* packed_bwd, const float* head, const float* out, const float* g_out,
                  const float* save, int64_t n, float* grad_ws, void* stream);

/* f16x3 arithmetic (the default; the 3xTF32 scheme on CDNA4's fp16 matrix
 * cores): every fp32 operand split into two fp16 pieces (hi + lo, 22 bits),
 * the three products hi*hi + hi*lo + lo*hi accumulated in fp32 on
 * v_mfma_f32_16x16x32_f16 / 32x32x16_f16, with exact power-of-two range
 * scaling (weights x 2^8; gradients per-sample in the data-gradient chain and
 * per-layer in the weight gradient).  The *_h3 entry points have the contracts
 * of their *_x3 twins; buffers: forward nr_fwd3_packed_bytes_h3() = 2,388,000
 * bytes (fp32 head block with the layer biases x 2^8, then fp16 k-groups of
 * packing.build_fwd3_map(2)), backward 2,228,224 bytes (build_bwd3_map(2)).
 * A training save buffer carries, after the activations, the gradient
 * statistics (layout.h nr_stats_floats): nr_mlp_bwd_h3 writes per-wave maxima,
 * nr_wgrad_h3 reduces and uses them. */
int64_t nr_fwd3_packed_bytes_h3(void);
int nr_pack_h3(const float* flat, const int32_t* map, int64_t n, const int32_t* head_map,
               void* out, void* stream);
int nr_mlp_fwd_h3(const void* packed, const float* rays, const float* z, int64_t n,
                  int samples_per_ray, const float* x, int xstride, int sigma_only, float* out,
                  float* save, void* stream);
int nr_mlp_sigma_points_h3(const void* packed, const float* pts, int64_t n, float* sigma_out,
                           void* stream);
int nr_pack_bwd_h3(const float* flat, const int32_t* map, int64_t n, void* out, void* stream);
int nr_mlp_bwd_h3(const void* packed_bwd, const float* head, const float* out, const float* g_out,
                  const float* save, int64_t n, float* grad_ws, void* stream);
int nr_wgrad_h3(const float* save, const float* grad_ws, int64_t n, float* workspace,
                float* grad_flat, void* stream);

/* plain bf16 arithmetic (BASELINE configs[1] "bf16/fp32": the reduced-precision
 * MLP variant, judged on PSNR): every operand rounded once to bf16, one
 * product per fp32 product accumulated in fp32 on v_mfma_f32_16x16x32_bf16 /
 * 32x32x16_bf16; inputs, outputs, saved activations and gradients stay fp32.
 * The *_b1 entry points have the contracts of their *_x3 twins; buffers:
 * forward nr_fwd3_packed_bytes_b1() = 1,200,160 bytes (fp32 head block, then
 * bf16 k-groups of packing.build_fwd3_map(1)), backward 1,114,112 bytes
 * (build_bwd3_map(1)). */
int64_t nr_fwd3_packed_bytes_b1(void);
int nr_pack_b1(const float* flat, const int32_t* map, int64_t n, const int32_t* head_map,
               void* out, void* stream);
int nr_mlp_fwd_b1(const void* packed, const float* rays, const float* z, int64_t n,
                  int samples_per_ray, const float* x, int xstride, int sigma_only, float* out,
                  float* save, void* stream);
int nr_mlp_sigma_points_b1(const void* packed, const float* pts, int64_t n, float* sigma_out,
                           void* stream);
int nr_pack_bwd_b1(const float* flat, const int32_t* map, int64_t n, void* out, void* stream);
int nr_mlp_bwd_b1(const void* packed_bwd, const float* head, const float* out, const float* g_out,
                  const float* save, int64_t n, float* grad_ws, void* stream);
int nr_wgrad_b1(const float* save, const float* grad_ws, int64_t n, float* workspace,
                float* grad_flat, void* stream);

/* Training the sigma-only graph (models/rendering_shadows.py:167: every MLP
 * call of the shadow path is NeRF.forward(x, sigma_only=True)), in every
 * arithmetic: nr_mlp_fwd{,_x3,_h3,_b1} with sigma_only = 1 AND a save buffer
 * (ray path) runs layers 1-8 and the sigma head only, keeps the activations
 * those layers need and writes (n, 4) rows [0, 0, 0, sigma];
 * nr_mlp_bwd_sigma_* (g_out column 3 = d sigma, the rgb columns ignored)
 * starts the data-gradient chain at d h8 = W_sigma^T d sigma; nr_wgrad_sigma_*
 * computes the weight gradients of xyz_encoding_1..8 and the sigma head and
 * writes 0 for xyz_encoding_final, dir_encoding and rgb (not in the graph).
 * Contracts otherwise those of nr_mlp_bwd_* / nr_wgrad_*. */
int nr_mlp_bwd_sigma(const float* packed_bwd, const float* head, const float* out,
                     const float* g_out, const float* save, int64_t n, float* grad_ws,
                     void* stream);
int nr_mlp_bwd_sigma_x3(const void* packed_bwd, const float* head, const float* out,
                        const float* g_out, const float* save, int64_t n, float* grad_ws,
                        void* stream);
int nr_mlp_bwd_sigma_h3(const void* packed_bwd, const float* head, const float* out,
                        const float* g_out, const float* save, int64_t n, float* grad_ws,
                        void* stream);
int nr_mlp_bwd_sigma_b1(const void* packed_bwd, const float* head, const float* out,
                        const float* g_out, const float* save, int64_t n, float* grad_ws,
                        void* stream);
int nr_wgrad_sigma(const float* save, const float* grad_ws, int64_t n, float* workspace,
                   float* grad_flat, void* stream);
int nr_wgrad_sigma_x3(const float* save, const float* grad_ws, int64_t n, float* workspace,
                      float* grad_flat, void* stream);
int nr_wgrad_sigma_h3(const float* save, const float* grad_ws, int64_t n, float* workspace,
                      float* grad_flat, void* stream);
int nr_wgrad_sigma_b1(const float* save, const float* grad_ws, int64_t n, float* workspace,
                      float* grad_flat, void* stream);

/* Zero-gradient samples (the training backward of rendering.py:169-176 under
 * autograd, train.py:107-111).  A sample whose output gradient g_out row
 * (d rgb, d sigma) is exactly zero -- sigma clamped by the ReLU (alpha = 0:
 * weight 0 and no sigma gradient) or a transmittance underflowed behind an
 * opaque surface -- adds exactly zero to every layer's dz and weight-gradient
 * sum.  nr_active_samples writes the indices of the other samples (a nonzero
 * or NaN entry in their row), ascending, to samples[0 .. m) (n int32), m to
 * *count (device memory, no host sync); scratch: nr_active_scratch_ints(n)
 * int32.  The *_active data- and weight-gradient entry points (plain twins'
 * arguments plus samples / count) then run over the m listed samples packed
 * densely: grad_ws holds position q's rows (q < m, sample samples[q]), so it
 * feeds only nr_wgrad*_active with the same list, which gathers the saved
 * activations of samples[q]; the weight gradients equal the plain entry
 * points' up to the order of the split-K partial sums (a fixed order:
 * reproducible).  fp32 (no suffix), bf16x6 (x3) and f16x3 (h3); not the bf16
 * variant (b1). */
int64_t nr_active_scratch_ints(int64_t n);
int nr_active_samples(const float* g_out, int64_t n, int32_t* samples, int32_t* count,
                      int32_t* scratch, void* stream);
int nr_mlp_bwd_active(const float* packed_bwd, const float* head, const float* out,
                      const float* g_out, const float* save, int64_t n, float* grad_ws,
                      const int32_t* samples, const int32_t* count, void* stream);
int nr_mlp_bwd_sigma_active(const float* packed_bwd, const float* head, const float* out,
                            const float* g_out, const float* save, int64_t n, float* grad_ws,
                            const int32_t* samples, const int32_t* count, void* stream);
int nr_wgrad_active(const float* save, const float* grad_ws, int64_t n, float* workspace,
                    float* grad_flat, const int32_t* samples, const int32_t* count, void* stream);
int nr_wgrad_sigma_active(const float* save, const float* grad_ws, int64_t n, float* workspace,
                          float* grad_flat, const int32_t* samples, const int32_t* count,
                          void* stream);
int nr_mlp_bwd_active_x3(const void* packed_bwd, const float* head, const float* out,
                         const float* g_out, const float* save, int64_t n, float* grad_ws,
                         const int32_t* samples, const int32_t* count, void* stream);
int nr_mlp_bwd_active_h3(const void* packed_bwd, const float* head, const float* out,
                         const float* g_out, const float* save, int64_t n, float* grad_ws,
                         const int32_t* samples, const int32_t* count, void* stream);
int nr_mlp_bwd_sigma_active_x3(const void* packed_bwd, const float* head, const float* out,
                               const float* g_out, const float* save, int64_t n, float* grad_ws,
                               const int32_t* samples, const int32_t* count, void* stream);
int nr_mlp_bwd_sigma_active_h3(const void* packed_bwd, const float* head, const float* out,
                               const float* g_out, const float* save, int64_t n, float* grad_ws,
                               const int32_t* samples, const int32_t* count, void* stream);
int nr_wgrad_active_x3(const float* save, const float* grad_ws, int64_t n, float* workspace,
                       float* grad_flat, const int32_t* samples, const int32_t* count, void* stream);
int nr_wgrad_active_h3(const float* save, const float* grad_ws, int64_t n, float* workspace,
                       float* grad_flat, const int32_t* samples, const int32_t* count, void* stream);
int nr_wgrad_sigma_active_x3(const float* save, const float* grad_ws, int64_t n, float* workspace,
                             float* grad_flat, const int32_t* samples, const int32_t* count,
                             void* stream);
int nr_wgrad_sigma_active_h3(const float* save, const float* grad_ws, int64_t n, float* workspace,
                             float* grad_flat, const int32_t* samples, const int32_t* count,
                             void* stream);

/* Deferred save.  A training forward whose backward lists few
 * samples (the sigma-only graphs of the shadow path: ~0.1% of a light image's
 * samples, ~20% of the camera rays') runs as inference (nr_mlp_fwd* without a
 * save buffer); its backward lists the samples (nr_active_samples), then
 * nr_mlp_fwd_listed* re-evaluates the training forward for samples[q],
 * q < *count only -- the same layers bit for bit -- saving their activations
 * by POSITION q into save (sized for n samples, nr_layout_query(3) per block,
 * as nr_mlp_fwd's; sigma_only selects the sigma-only graph), and no output.
 * nr_mlp_bwd[_sigma]_listed* / nr_wgrad[_sigma]_listed* are the data and
 * weight gradients over those positions (g_out / out rows gathered by the
 * list): the same sums, in the same split-K order, as the *_active entry
 * points over a forward-time save.  fp32 (no suffix), bf16x6 (_x3), f16x3
 * (_h3). */
int nr_mlp_fwd_listed(const float* packed, const float* rays, const float* z, int64_t n,
                      int samples_per_ray, int sigma_only, float* save, const int32_t* samples,
                      const int32_t* count, void* stream);
int nr_mlp_fwd_listed_x3(const void* packed, const float* rays, const float* z, int64_t n,
                         int samples_per_ray, int sigma_only, float* save, const int32_t* samples,
                         const int32_t* count, void* stream);
int nr_mlp_fwd_listed_h3(const void* packed, const float* rays, const float* z, int64_t n,
                         int samples_per_ray, int sigma_only, float* save, const int32_t* samples,
                         const int32_t* count, void* stream);
int nr_mlp_bwd_listed(const float* packed_bwd, const float* head, const float* out,
                      const float* g_out, const float* save, int64_t n, float* grad_ws,
                      const int32_t* samples, const int32_t* count, void* stream);
int nr_mlp_bwd_listed_x3(const void* packed_bwd, const float* head, const float* out,
                         const float* g_out, const float* save, int64_t n, float* grad_ws,
                         const int32_t* samples, const int32_t* count, void* stream);
int nr_mlp_bwd_listed_h3(const void* packed_bwd, const float* head, const float* out,
                         const float* g_out, const float* save, int64_t n, float* grad_ws,
                         const int32_t* samples, const int32_t* count, void* stream);
int nr_mlp_bwd_sigma_listed(const float* packed_bwd, const float* head, const float* out,
                            const float* g_out, const float* save, int64_t n, float* grad_ws,
                            const int32_t* samples, const int32_t* count, void* stream);
int nr_mlp_bwd_sigma_listed_x3(const void* packed_bwd, const float* head, const float* out,
                               const float* g_out, const float* save, int64_t n, float* grad_ws,
                               const int32_t* samples, const int32_t* count, void* stream);
int nr_mlp_bwd_sigma_listed_h3(const void* packed_bwd, const float* head, const float* out,
                               const float* g_out, const float* save, int64_t n, float* grad_ws,
                               const int32_t* samples, const int32_t* count, void* stream);
int nr_wgrad_listed(const float* save, const float* grad_ws, int64_t n, float* workspace,
                    float* grad_flat, const int32_t* samples, const int32_t* count, void* stream);
int nr_wgrad_listed_x3(const float* save, const float* grad_ws, int64_t n, float* workspace,
                       float* grad_flat, const int32_t* samples, const int32_t* count, void* stream);
int nr_wgrad_listed_h3(const float* save, const float* grad_ws, int64_t n, float* workspace,
                       float* grad_flat, const int32_t* samples, const int32_t* count, void* stream);
int nr_wgrad_sigma_listed(const float* save, const float* grad_ws, int64_t n, float* workspace,
                          float* grad_flat, const int32_t* samples, const int32_t* count,
                          void* stream);
int nr_wgrad_sigma_listed_x3(const float* save, const float* grad_ws, int64_t n, float* workspace,
                             float* grad_flat, const int32_t* samples, const int32_t* count,
                             void* stream);
int nr_wgrad_sigma_listed_h3(const float* save, const float* grad_ws, int64_t n, float* workspace,
                             float* grad_flat, const int32_t* samples, const int32_t* count,
                             void* stream);

/* Dense sigma query (extract_color_mesh.py:114-137, the marching-cubes grid):
 * sigma_out (n) = NeRF sigma head at points pts (n,3) -- the sigma-only fused
 * kernel with the positional encoding computed in-kernel (sigma does not
 * depend on the view direction, nerf.py:112). */
int nr_mlp_sigma_points(const float* packed_fwd, const float* pts, int64_t n, float* sigma_out,
                        void* stream);

/* MLP backward, data-gradient chain (autograd of nerf.py:83-124): from
 * g_out (n,4) = d[rgb, sigma] writes every layer's pre-activation gradient to
 * grad_ws (n*nr_layout_query(4) floats).  head: the fp32 head block of the
 * forward weights (nr_layout_query(5) floats: packed_fwd + nr_layout_query(1)
 * floats for the fp32 layout, the start of the bf16x6 buffer). */
int nr_mlp_bwd(const float* packed_bwd, const float* head, const float* out,
               const float* g_out, const float* save, int64_t n, float* grad_ws, void* stream);

/* MLP backward, weight gradients: sum over all n samples of dz^T x for every
 * layer (split over workgroups, reduced in a fixed order), written as
 * d(loss)/d(params) into grad_flat (595,844 floats, named_parameters order).
 * The forward does not save xyz_encoding_final's output (feat): every
 * nr_wgrad* entry point of the full graph leaves G = sum dz_dir h8^T in
 * dir_encoding.0.weight's first 256 columns, and nr_wgrad_dir_feat, given the
 * flat fp32 parameters the forward ran with, turns them into the gradient
 * G W_final^T + d(bias_dir) b_final^T (feat = W_final h8 + b_final,
 * nerf.py:116-118; replaces autograd's sum dz_dir feat^T).  The data gradient
 * does not save d feat either: the same call writes xyz_encoding_final's
 * gradients W_dir[:, :256]^T G (weight) and W_dir[:, :256]^T d(bias_dir)
 * (bias) -- autograd's sum d feat h8^T and sum d feat with
 * d feat = W_dir[:, :256]^T dz_dir (nerf.py:116-119); the nr_wgrad* launch
 * itself leaves that layer's slots zero. */
int64_t nr_wgrad_workspace_bytes(int64_t n);
int nr_wgrad(const float* save, const float* grad_ws, int64_t n, float* workspace,
             float* grad_flat, void* stream);
int nr_wgrad_dir_feat(const float* params, float* grad_flat, void* stream);
/* The same weight gradients on bf16x6 split-operand MFMA (fp32-level accuracy). */
int nr_wgrad_x3(const float* save, const float* grad_ws, int64_t n, float* workspace,
                float* grad_flat, void* stream);

/* Stratified coarse depths (rendering.py:216-232).  tlin = torch.linspace(0,1,S)
 * values; u: (n_rays,S) replay of torch.rand or NULL. */
int nr_coarse_z(const float* rays, const float* tlin, int64_t n_rays, int n_samples,
                int use_disp, float perturb, const float* u, uint64_t seed, float* z_out,
                void* stream);

/* Volume compositing (rendering.py:169-198; sigma-only variant
 * rendering_shadows.py:164-198), one wave per ray.  raw rows of raw_stride
 * floats with sigma at sig_col and, when rgb != NULL, rgb at 0..2.  noise:
 * (n_rays,S) replay of torch.randn or NULL.  Writes weights (n_rays,S),
 * opacity, and unless weights_only depth and (if rgb != NULL) rgb (n_rays,3). */
int nr_composite_fwd(const float* raw, int raw_stride, int sig_col, const float* z,
                     const float* rays, const float* noise, float noise_std, uint64_t seed,
                     int rng_stream, int64_t n_rays, int n_samples, int white_back,
                     int weights_only, float* rgb, float* depth, float* opacity,
                     float* weights, void* stream);

/* Autograd of the compositing step: d(rgb, depth, opacity) -> g_raw, rows of
 * raw_stride floats like raw: d sigma_i at sig_col and, when raw_stride == 4,
 * d rgb_i at 0..2.  Any gradient pointer may be NULL (zero). */
int nr_composite_bwd(const float* raw, int raw_stride, int sig_col, const float* z, const float* rays, const float* noise,
                     float noise_std, uint64_t seed, int rng_stream, int64_t n_rays,
                     int n_samples, int white_back, const float* g_rgb, const float* g_depth,
                     const float* g_opacity, float* g_raw, void* stream);

/* sample_pdf (rendering.py:14-48) replacing torchsearchsorted.searchsorted
 * (side='right', rendering.py:37), fused with sort(cat[z_coarse, z_pdf])
 * (rendering.py:257).  weights: coarse weights (n_rays, n_samples), bins are
 * columns 1..n_samples-2.  u, jitter: (n_rays, n_importance) replays or NULL.
 * z_pdf (n_rays, n_importance) and/or z_fine (n_rays, n_samples+n_importance). */
int nr_sample_pdf(const float* weights, int n_samples, const float* rays,
                  const float* z_coarse, const float* u, const float* jitter, uint64_t seed,
                  int64_t n_rays, int n_importance, float* z_pdf, float* z_fine, void* stream);

/* Training-batch ray generation (datasets/ray_utils.py:5-93 get_ray_directions
 * + get_rays [+ get_ndc_rays], the ray buffers of datasets/blender.py:54-86 and
 * llff.py:213-249): ray k is global pixel g = sel[k] (or k when sel == NULL) =
 * pose*H*W + row*W + col of the poses c2w (n_poses,3,4).  Direction
 * ((col - w_half)/focal, -(row - h_half)/focal, -1) rotated by c2w and
 * normalised, origin c2w[:,3]; rays (n,8) = [o, d, near, far].  ndc != 0 applies
 * get_ndc_rays with near plane ndc_near and the host-evaluated constants
 * ndc_cw = -1/(W/(2 focal)), ndc_ch = -1/(H/(2 focal)), ndc_2near = 2 ndc_near.
 * rgb_pool (n_poses*H*W, 3) / rgb_out (n,3): optional target gather.  An
 * out-of-range sel entry yields a NaN ray. */
int nr_gen_rays(const float* c2w, int64_t n_poses, int H, int W, float w_half, float h_half,
                float focal, float near, float far, int ndc, float ndc_near, float ndc_cw,
                float ndc_ch, float ndc_2near, const int64_t* sel, int64_t n,
                const float* rgb_pool, float* rgb_out, float* rays, void* stream);

/* Fused Adam step (torch.optim.Adam as built by utils/__init__.py:10-30, the
 * single-tensor formulas op for op) over `count` <= nr_adam_max_tensors()
 * tensors in one launch: tables of device pointers (host arrays) to params,
 * grads (an entry may be NULL: zero gradient), exp_avg, exp_avg_sq and their
 * element counts.  step = the step number after increment (1 on the first). */
int nr_adam_max_tensors(void);
int nr_adam_step(float* const* params, const float* const* grads, float* const* exp_avg,
                 float* const* exp_avg_sq, const int64_t* numel, int count, double lr,
                 double beta1, double beta2, double eps, double weight_decay, int64_t step,
                 void* stream);

/* Training loss (losses.py:4-14 MSELoss: nn.MSELoss(reduction='mean') on
 * rgb_coarse [+ on rgb_fine], the fine term added in fp32; metrics.py:4-13
 * mse).  a, b (b may be NULL), target: n floats each.  loss (1 float, device);
 * means (2 floats, device, may be NULL) = [mean (a-t)^2, mean (b-t)^2 (0
 * without b)]; squares in fp32, sums in double in a fixed order
 * (deterministic).  One launch. */
int nr_mse_loss(const float* a, const float* b, const float* target, int64_t n, float* loss,
                float* means, void* stream);
/* Its backward: ga = (2/n) * (a - t) * g, gb likewise (torch's
 * mse_loss_backward), g = the upstream gradient of the loss scalar (device
 * pointer, 1 float); ga / gb may be NULL (not needed).  One launch. */
int nr_mse_loss_bwd(const float* a, const float* b, const float* target, int64_t n,
                    const float* g, float* ga, float* gb, void* stream);

/* losses.py:28-73 OpactiyLoss (loss_dict['opacity']; train_efficient_sm.py:43
 * constructs it, :191 evaluates it on the light render): with gray = (t0 + t1 +
 * t2) / 3 of target rows t (n_t,3), sm = gray > thres, non = !sm,
 *   loss = coeff - |mean(o_c[non]) - mean(o_c[sm])| [+ the same on o_f],
 * 0 when either set is empty.  The targets index rows 0..n_t-1 of the n_o
 * opacities (n_t <= n_o).  loss: 1 float; stats: 8 floats kept for the
 * backward.  One launch, fixed-order double sums (deterministic). */
int nr_opacity_loss(const float* opacity_c, const float* opacity_f, const float* target,
                    int64_t n_t, int64_t n_o, float thres, float coeff, float* loss, float* stats,
                    void* stream);
/* Its backward: g (device, 1 float) -> g_opacity_c / g_opacity_f (n_o each,
 * either may be NULL); rows >= n_t get 0.  One launch. */
int nr_opacity_loss_bwd(const float* target, int64_t n_t, int64_t n_o, float thres,
                        const float* stats, const float* g, float* g_opacity_c,
                        float* g_opacity_f, void* stream);

/* torchsearchsorted.searchsorted(a, v, out, side) -- the reference's only
 * native dependency (.gitmodules:1-3; rendering.py:2,37, rendering_rgb_sm.py:2,40)
 * as a standalone call (nr_sample_pdf fuses it on the render path): out
 * (nrows, ncols_v) int64 = per row the number of entries of the sorted row of a
 * that are < v (side_right = 0) or <= v (side_right = 1).  nrows_a == nrows_v,
 * or either is 1 (shared by every row).  torch.searchsorted's comparisons (a
 * NaN query lands after every entry).  float32 and float64 variants. */
int nr_searchsorted(const float* a, const float* v, int64_t nrows_a, int64_t ncols_a,
                    int64_t nrows_v, int64_t ncols_v, int side_right, int64_t* out, void* stream);
int nr_searchsorted_f64(const double* a, const double* v, int64_t nrows_a, int64_t ncols_a,
                        int64_t nrows_v, int64_t ncols_v, int side_right, int64_t* out,
                        void* stream);

/* ---- shadow mapping (config 5: train_efficient_sm.py) ---------------------
 * get_normed_w column 3 (efficient_shadow_mapping.py:47-62): out (n) =
 * depth / (|camera @ pixel| + 1e-5); camera (3,3) row-major, pixels (n,3). */
int nr_sm_normed_depth(const float* camera, const float* pixels, const float* depth, int64_t n,
                       float* out, void* stream);
/* Its autograd (:59, `pixel_depth[:,3] / norm`): g_depth (n) = g_out / (|camera @ pixel| +
 * 1e-5).  The light render's path to its depths when the light map is trained
 * (train_efficient_sm.py --grad_on_light, :158-162). */
int nr_sm_normed_depth_bwd(const float* camera, const float* pixels, const float* g_out,
                           int64_t n, float* g_depth, void* stream);

/* efficient_sm's shadow maps (rendering_shadows.py:359-482 with
 * efficient_shadow_mapping.py:19-130): for camera rays with pixels (n,3) and
 * depth (n), per-ray eye (n,3) and camera (n,3,3) (per_ray=1; runs of equal
 * eye position are split exactly like the reference's torch.equal loop and use
 * the run's first camera) or one eye/camera for all (per_ray=0), the light
 * camera (3,3) + eye (3) and the light's normed depth map light_w (res_w*res_h)
 * -> out (n,3) = shadow value + out_eps.  method 1: clip(max(d/delta, epsilon));
 * method 2: per-run min-max normalisation (+ sigmoid).  workspace:
 * nr_sm_workspace_bytes(n, res_w*res_h) bytes; keep it for nr_sm_backward. */
int64_t nr_sm_workspace_bytes(int64_t n, int64_t n_light);
int nr_sm_forward(const float* pixels, const float* depth, const float* eye, const float* cameras,
                  int per_ray, const float* light_camera, const float* light_eye,
                  const float* light_w, int res_w, int res_h, int method, float delta,
                  float epsilon, int sigmoid, float out_eps, int64_t n, void* workspace,
                  float* out, void* stream);
/* Autograd of nr_sm_forward: g_out (n,3) -> g_depth (n), the camera depths,
 * and g_light_w (n_light = res_w*res_h), the light's normed depth map (the
 * backward of the texel gather w_light.view(w,h)[v,u], :98, including the
 * min-max normalisation's dependence on each run's extremes, :10-11,122).
 * Either output may be NULL (not needed; train_efficient_sm.py renders the
 * light under no_grad unless --grad_on_light).  The light-map gradient is a
 * deterministic scatter-add (64-bit fixed point at one power-of-two scale per
 * call, integer atomics: bitwise reproducible, exact to ~2^-60 of the largest
 * contribution); untouched texels get 0. */
int nr_sm_backward(const float* g_out, void* workspace, int method, float delta, float epsilon,
                   int sigmoid, int64_t n, int64_t n_light, float* g_depth, float* g_light_w,
                   void* stream);

/* Test hook: one v_mfma_f32_32x32x2_f32 on A (32x2), B (2x32) -> D (32x32). */
int nr_probe_mfma32(const float* a, const float* b, float* d, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NERF_PL_AMD_H */
