/*
 * dro_amd.h -- C ABI of the MI355X (gfx950) hot-path library libdro_amd.so.
 *
 * The reference (xyang9527/dro-sfm) is pure Python/PyTorch; every hot-path op
 * there is a chain of stock ATen kernels.  Each entry point below replaces one
 * such chain with hand-written HIP for CDNA4 and is bound from Python by
 * dro-sfm_amd/hip/_lib.py (ctypes).  Conventions shared by every function:
 *
 *   * plain device pointers (fp32, dense NCHW / row-major, caller allocated);
 *     the library never allocates or frees; outputs are fully overwritten;
 *   * `stream` is a hipStream_t passed as void* (NULL = default stream); all
 *     work is enqueued asynchronously on it and is hipGraph-capturable (no
 *     host synchronisation, no allocation; buffers are zeroed by kernels, not
 *     hipMemsetAsync, which is not recorded when issued into a capture);
 *   * return value: 0 on success, a negative DRO_E_* code for an invalid
 *     argument (nothing is launched), or a positive hipError_t from the launch.
 *     dro_last_error() returns a static message for the last failure on the
 *     calling thread.
 *
 * Pose encodings (pose_mode):
 *   DRO_POSE_EULER  : 6 floats per pose  [tx,ty,tz, rx,ry,rz], R = Rx*Ry*Rz
 *                     (geometry/pose_utils.py:40-85, Pose.from_vec pose.py:38-45)
 *   DRO_POSE_MATRIX : 12 floats per pose, row-major [R | t] (the top 3 rows of
 *                     a Pose.mat [4,4], geometry/pose.py:7-98)
 * Depth encodings (depth_mode) for the target depth map:
 *   DRO_DEPTH_METRIC  : metric depth as given
 *   DRO_DEPTH_INV     : inverse depth; depth = inv2depth(x) (utils/depth.py:102-121)
 *   DRO_DEPTH_DISP    : sigmoid disparity; depth = inv2depth(disp_to_depth(x)[0])
 *                       (networks/layers/resnet/layers.py:11-20), using min_disp/max_disp
 */
#ifndef DRO_AMD_H
#define DRO_AMD_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DRO_POSE_EULER 0
#define DRO_POSE_MATRIX 1

#define DRO_DEPTH_METRIC 0
#define DRO_DEPTH_INV 1
#define DRO_DEPTH_DISP 2

#define DRO_OK 0
#define DRO_E_NULL (-1)     /* a required pointer is NULL            */
#define DRO_E_SHAPE (-2)    /* a size is out of the supported range  */
#define DRO_E_MODE (-3)     /* unknown pose/depth mode or option     */

const char* dro_last_error(void);
int dro_abi_version(void);   /* 10: BatchNorm fused into the 3x3 convs (dro_conv2d_bn_forward / dro_conv2d_bn_backward_data, dro_bn_state_bytes); 9: dro_png_decode (GPU PNG inflate + unfilter); 8: dro_convgru_candidate_backward / dro_convgru_gates_backward (the GRU's elementwise stages in the conv data-gradient epilogues); 7: warp-cost forward/backward take ref_layout (channels-last reference maps); 6: photometric calls take clip_loss (and the backward the l1_signs test hook); 5: warp-cost / photometric backward take the `cells` test hook, view synthesis entry points; 4: convex upsample takes the fused add/mul; 3: conv calls take split-bf16 weights (dro_weight_split); 2: dro_adam_step reads its hyper-parameters from device memory */

/* In-graph step timeline (diagnostics, tools/step_timeline.py): record the
 * device's constant-rate real-time counter into buf[slot] when `stream`
 * reaches this launch (capturable: replays overwrite the same slot). */
int dro_timestamp(unsigned long long* buf, int slot, void* stream);
int dro_wall_clock_hz(long long* hz);   /* that counter's rate */

/* ------------------------------------------------------------------------
 * Inverse warp + feature cost.
 * Replaces DepthPoseNet.get_cost_each (networks/depth_pose/DepthPoseNet.py:76-96)
 * and, with reduce_mean=1 over N refs, DepthPoseNet.depth_cost_calc (:98-105):
 *   Camera(K).scaled(scale).reconstruct(depth) -> Camera(ref_K, Tcw=pose)
 *   .scaled(scale).project(normalize=True) -> grid_sample(bilinear, zeros,
 *   align_corners=True) -> (fmap - warped)^2
 *   fmap [B,C,h,w]; fmap_ref [N,B,C,h,w]; depth [B,1,h,w]; K, ref_K [B,3,3];
 *   pose [N,B,6|12]; cost [B,C,h,w] (reduce_mean) or [N,B,C,h,w].
 * scale == 1.0f leaves K untouched (Camera.scaled returns self, camera.py:103-104).
 * ref_layout: 0 = fmap_ref (and grad_fmap_ref) NCHW [N,B,C,h,w]; 1 =
 * channels-last [N,B,h,w,C] -- the tap gathers and scatter atomics are then
 * coalesced over channels whatever the warp's geometry (the layout the
 * training step uses; the other maps stay NCHW either way).
 * ---------------------------------------------------------------------- */
int dro_warp_cost_forward(const float* fmap, const float* fmap_ref, const float* depth,
                          int depth_mode, float min_disp, float max_disp,
                          const float* K, const float* ref_K, float scale,
                          const float* pose, int pose_mode,
                          int B, int N, int C, int h, int w, int reduce_mean,
                          int ref_layout, float* cost, void* stream);

size_t dro_warp_cost_workspace_bytes(int B, int N, int h, int w);

/* Gradients of sum(cost * grad_cost).  Any grad_* may be NULL (not computed).
 * grad_depth is w.r.t. the depth input in its depth_mode encoding; grad_pose
 * is w.r.t. the pose input in its pose_mode encoding.  `workspace` must hold
 * dro_warp_cost_workspace_bytes() bytes when grad_depth or grad_pose is set.
 * accumulate: bit 0 adds into grad_fmap, bit 1 into grad_fmap_ref, bit 2 into
 * grad_depth (otherwise they are overwritten) -- the feature maps are shared by
 * every cost call of a step and the depth state by the cost, the depth encoder
 * and the update, so their gradients can be summed in place (hip.grad_sink).
 * cells (test hook, NULL in production): int32 [N,B,h,w] receives the bilinear
 * cell each pixel's sampling position fell in, packed ((y0 + 32768) << 16) |
 * (x0 + 32768) -- the branch of grid_sample's piecewise-linear derivative this
 * backward took (parity tests hand it to the fp64 oracle). */
int dro_warp_cost_backward(const float* fmap, const float* fmap_ref, const float* depth,
                           int depth_mode, float min_disp, float max_disp,
                           const float* K, const float* ref_K, float scale,
                           const float* pose, int pose_mode,
                           int B, int N, int C, int h, int w, int reduce_mean,
                           int ref_layout, const float* grad_cost, float* grad_fmap, float* grad_fmap_ref,
                           float* grad_depth, float* grad_pose, int accumulate, void* workspace,
                           int* cells, void* stream);

/* View synthesis (geometry/camera_utils.py:23-56): the reference maps warped
 * into the target view, warped[n,b] = grid_sample(ref_image[n,b],
 * Camera(ref_K, Tcw=pose[n,b]).scaled(scale).project(Camera(K).scaled(scale)
 * .reconstruct(depth[b]))), bilinear, zeros padding, align_corners=True.
 *   ref_image [N,B,C,H,W]; depth [B,1,H,W] (depth_mode); pose [N,B,6|12];
 *   warped [N,B,C,H,W].  The same kernels as the cost (one launch for all N).
 * Backward: grad_ref_image (bilinear scatter, fp32 atomics), grad_depth (summed
 * over the N views), grad_pose; any may be NULL.  workspace as
 * dro_warp_cost_workspace_bytes(B, N, H, W); cells as in dro_warp_cost_backward. */
int dro_view_synthesis_forward(const float* ref_image, const float* depth, int depth_mode,
                               float min_disp, float max_disp, const float* K, const float* ref_K,
                               float scale, const float* pose, int pose_mode, int B, int N, int C,
                               int H, int W, float* warped, void* stream);
int dro_view_synthesis_backward(const float* ref_image, const float* depth, int depth_mode,
                                float min_disp, float max_disp, const float* K, const float* ref_K,
                                float scale, const float* pose, int pose_mode, int B, int N, int C,
                                int H, int W, const float* grad_warped, float* grad_ref_image,
                                float* grad_depth, float* grad_pose, void* workspace, int* cells,
                                void* stream);

/* D fronto-parallel hypothesis planes (SURVEY.md §8(d) measurement extension):
 * for each plane d, depth = inv2depth(disp_to_depth(disp[d])) everywhere and
 * cost[b,d] = get_cost_each(pose, fmap, fmap_ref, depth).  disp [D] (device);
 * pose [B,6|12]; cost [B,D,C,h,w]. */
int dro_plane_sweep_forward(const float* fmap, const float* fmap_ref, const float* disp, int D,
                            float min_disp, float max_disp, const float* K, const float* ref_K,
                            float scale, const float* pose, int pose_mode,
                            int B, int C, int h, int w, float* cost, void* stream);

/* ------------------------------------------------------------------------
 * Multi-view photometric decay loss + edge-aware smoothness.
 * Replaces MultiViewPhotometricDecayLoss.forward
 * (losses/multiview_photometric_loss_mf.py:303-361) with padding_mode
 * 'zeros': view_synthesis (geometry/camera_utils.py:23-56), SSIM (:15-54), L1,
 * clip_loss (:223-227: each candidate map clamped at mean + clip_loss * std of
 * itself; 0 = off, as in every reference yaml; the constructor's default is
 * 0.5), automask (:346-351), min/mean reduce and 0.85^(n-i-1) decay
 * (:231-269), calc_smoothness (utils/depth.py:166-199) (:273-299).
 *   image [B,3,H,W]; context [N,B,3,H,W]; inv_depths [n,B,1,H,W];
 *   K, ref_K [B,3,3] (scaled by DW/W = 1 -> unscaled); pose [N,n,B,6|12].
 *   out [3] = {loss, photometric_loss metric, smoothness_loss metric}.
 * `workspace` (dro_photometric_workspace_bytes) carries the forward state the
 * backward needs; keep it alive and unmodified in between. */
size_t dro_photometric_workspace_bytes(int B, int N, int n, int H, int W, float clip_loss);

/* With clip_loss > 0: byte offsets in that workspace, after the forward, of
 * which = 0: the warped photometric maps, fp32 [N,n,B,H,W] (unclamped);
 * which = 1: the fp32 clamp thresholds -- N*n for the warped maps (index
 * j*n + i), then N for the unwarped (automask) maps.  The tests pin the fp64
 * oracle to the kernel's clamp decisions (a pixel within rounding of its
 * map's threshold is clamped or not by rounding). */
size_t dro_photometric_clip_offset(int B, int N, int n, int H, int W, int which);

int dro_photometric_forward(const float* image, const float* context, const float* inv_depths,
                            const float* K, const float* ref_K, const float* pose, int pose_mode,
                            int B, int N, int n, int H, int W,
                            float ssim_w, float C1, float C2, float smooth_w,
                            int automask, int reduce_min, float clip_loss,
                            float* out, void* workspace, void* stream);

/* grad_out: device pointer to d(total)/d(loss) (1 float).  Writes
 * grad_inv_depths [n,B,1,H,W] and (if non-NULL) grad_pose [N,n,B,6|12].
 * cells (test hook, NULL in production): int32 [N,n,B,H,W], the bilinear cell
 * of every pixel's warp whose derivative this backward used (packed as in
 * dro_warp_cost_backward; pixels of a (ref, tile) with no selected candidate
 * are skipped and left as they were).  l1_signs (test hook, NULL in
 * production): int8 [N,n,B,3,H,W], the sign of (warped - target) the L1
 * term's derivative used, 1 / -1 / 2 (zero), at every pixel whose candidate
 * passed a gradient (others left as they were). */
int dro_photometric_backward(const float* image, const float* context, const float* inv_depths,
                             const float* K, const float* ref_K, const float* pose, int pose_mode,
                             int B, int N, int n, int H, int W,
                             float ssim_w, float C1, float C2, float smooth_w,
                             int automask, int reduce_min, float clip_loss,
                             const float* grad_out, float* grad_inv_depths, float* grad_pose,
                             void* workspace, int* cells, signed char* l1_signs, void* stream);

/* ------------------------------------------------------------------------
 * Supervised depth + pose loss (sparse-l1).
 * Replaces SupervisedDepthPoseLoss.forward (losses/supervised_loss.py:343-371):
 * calculate_loss (:244-277) + calc_pose_loss (:293-325) with get_ref_coords
 * (:279-291), for predictions at the ground-truth resolution.
 *   gt_inv [B,1,H,W]; inv_depths [n,B,1,H,W]; K, ref_K [B,3,3];
 *   gt_pose [N,B,12] (row-major [R|t], the Tcw of each context frame);
 *   pose [N,n,B,6|12] predicted poses; min_depth/max_depth as in the loss.
 *   out [3] = {loss, depth_loss metric, pose_loss metric}.
 * `workspace` (dro_supervised_workspace_bytes) is scratch only; forward and
 * backward share no state. */
size_t dro_supervised_workspace_bytes(int B, int N, int n, int H, int W);

int dro_supervised_forward(const float* gt_inv, const float* inv_depths, const float* K,
                           const float* ref_K, const float* gt_pose, const float* pose,
                           int pose_mode, int B, int N, int n, int H, int W,
                           float min_depth, float max_depth, float* out,
                           void* workspace, void* stream);

/* grad_out: device pointer to d(total)/d(loss) (1 float).  Writes
 * grad_inv_depths [n,B,1,H,W] and grad_pose [N,n,B,6|12]. */
int dro_supervised_backward(const float* gt_inv, const float* inv_depths, const float* K,
                            const float* ref_K, const float* gt_pose, const float* pose,
                            int pose_mode, int B, int N, int n, int H, int W,
                            float min_depth, float max_depth, const float* grad_out,
                            float* grad_inv_depths, float* grad_pose, void* workspace,
                            void* stream);

/* ------------------------------------------------------------------------
 * Convex 8x upsampling: DepthPoseNet.upsample_depth (DepthPoseNet.py:63-74),
 * followed by out = add + mul * up (DepthPoseNet.scale_inv_depth, the
 * disp_to_depth scaling of every prediction, DepthPoseNet.py:128/181; add = 0,
 * mul = 1 for the plain upsample), computed as a multiply then an add.
 *   inv [B,1,h,w]; mask [B,9*r*r,h,w] -> out [B,1,h*r,w*r]
 * The backward takes the same `mul` (d out / d up).
 * ---------------------------------------------------------------------- */
int dro_convex_upsample_forward(const float* inv, const float* mask, int B, int h, int w,
                                int ratio, float add, float mul, float* out, void* stream);
int dro_convex_upsample_backward(const float* inv, const float* mask, const float* grad_out,
                                 int B, int h, int w, int ratio, float mul,
                                 float* grad_inv, float* grad_mask, void* stream);
/* n predictions (1..32) in one launch each way -- every kept prediction of a
 * training step, which the losses read stacked (DepthPoseNet.py:180-181 per
 * iteration, multiview_photometric_loss_mf.py / supervised_loss stacks):
 *   inv[i] [B,1,h,w], mask[i] [B,9*r*r,h,w] (host pointer tables)
 *   -> out [n,B,1,h*r,w*r] (add + mul * up, as the single call).
 * Backward: grad_out [n,B,1,h*r,w*r] -> grad_mask[i] (required) and
 * grad_inv[i] (table and entries nullable), both WRITTEN; deterministic (no
 * atomics): the tap sums go through a workspace of
 * dro_convex_upsample_many_workspace_bytes(n, B, h, w) bytes. */
int dro_convex_upsample_many_forward(const float* const* inv, const float* const* mask, int n, int B,
                                     int h, int w, int ratio, float add, float mul, float* out,
                                     void* stream);
size_t dro_convex_upsample_many_workspace_bytes(int n, int B, int h, int w);
int dro_convex_upsample_many_backward(const float* const* inv, const float* const* mask,
                                      const float* grad_out, int n, int B, int h, int w, int ratio,
                                      float mul, float* const* grad_inv, float* const* grad_mask,
                                      void* workspace, size_t workspace_bytes, void* stream);

/* Bilinear 2x upsampling, align_corners=False (F.interpolate(scale_factor=2,
 * mode="bilinear") in networks/optim/extractor.py:91-97 of the reference).
 *   x [planes, h, w] -> out [planes, 2h, 2w]; backward gathers (deterministic). */
int dro_bilinear_upsample2x_forward(const float* x, long long planes, int h, int w,
                                    float* out, void* stream);
int dro_bilinear_upsample2x_backward(const float* grad_out, long long planes, int h, int w,
                                     float* grad_x, void* stream);

/* 3x3 / stride 2 / pad 1 max pooling of the ResNet-18 stem
 * (F.max_pool2d(x, 3, 2, 1) in ResNetEncoder, networks/optim/extractor.py:60-66
 * of the reference).  x [planes, H, W] -> y [planes, Ho, Wo], Ho = (H-1)/2+1,
 * and one argmax byte per output (dy*3+dx within the window; ATen's tie order).
 * The backward gathers in ATen's window order: bit-identical to max_pool2d's
 * backward. */
int dro_maxpool3x3s2_forward(const float* x, long long planes, int H, int W, float* y,
                             unsigned char* argmax, void* stream);
int dro_maxpool3x3s2_backward(const float* grad_y, const unsigned char* argmax,
                              long long planes, int H, int W, float* grad_x, void* stream);

/* Depth evaluation metrics (compute_depth_metrics, dro_sfm/utils/depth.py:259-343
 * of the reference).  gt [B,1,H,W] metric depth, pred [B,1,h,w] predicted depth.
 * prepare: pred_up [B,H,W] = max(bilinear(pred, align_corners=True), 1e-6),
 *   ratio [B,H,W] = gt / pred_up where valid (min < gt < max, inside the crop
 *   rectangle [y1,y2) x [x1,x2) unless y1 < 0) and +inf elsewhere, and
 *   block_counts [B, dro_depth_metrics_blocks(H,W)] valid pixels per block.
 * reduce: with scale [B] (the per-image median of the valid ratios; NULL = no
 *   ground-truth scaling) writes metrics[9] = batch means of abs_rel, sq_rel,
 *   rmse, rmse_log, a1, a2, a3, SILog, iabs_diff.  Per-pixel terms in fp32 as
 *   the reference writes them, sums in fp64 in a fixed order (deterministic). */
int dro_depth_metrics_blocks(int H, int W);
size_t dro_depth_metrics_workspace_bytes(int B);
int dro_depth_metrics_prepare(const float* gt, const float* pred, int B, int H, int W, int h, int w,
                              float min_depth, float max_depth, int crop_y1, int crop_y2,
                              int crop_x1, int crop_x2, float* pred_up, float* ratio,
                              int* block_counts, void* stream);
/* median: scale[b] = the ((n_b - 1) / 2)-th smallest valid ratio of image b
 * (torch.median's lower middle element; 1 when n_b = 0), by a 4-pass radix
 * select on the device (no host round trip). */
size_t dro_depth_metrics_median_workspace_bytes(int B);
int dro_depth_metrics_median(const float* ratio, const int* block_counts, int B, int H, int W,
                             float* scale, void* workspace, void* stream);
int dro_depth_metrics_reduce(const float* gt, const float* pred_up, const float* scale, int B, int H,
                             int W, float min_depth, float max_depth, int crop_y1, int crop_y2,
                             int crop_x1, int crop_x2, float* metrics, void* workspace, void* stream);

/* compute_depth_metrics_demon (dro_sfm/utils/depth.py:343-398, ScanNet/DeMoN
 * evaluation): prepare -> dro_depth_metrics_median -> reduce as above, no crop,
 * no clamp of the (scaled) prediction to [min_depth, max_depth].  gt_pose:
 * per image the first reference's ground-truth transform (row-major 4x4 or
 * 3x4 floats at gt_pose + b * pose_stride); the ground truth is divided by the
 * norm of its translation.  gt_pose NULL = use_gt_scale False (then scale is
 * NULL too). */
int dro_depth_metrics_demon_prepare(const float* gt, const float* pred, const float* gt_pose,
                                    long long pose_stride, int B, int H, int W, int h, int w,
                                    float min_depth, float max_depth, float* pred_up, float* ratio,
                                    int* block_counts, void* stream);
int dro_depth_metrics_demon_reduce(const float* gt, const float* pred_up, const float* scale,
                                   const float* gt_pose, long long pose_stride, int B, int H, int W,
                                   float min_depth, float max_depth, float* metrics, void* workspace,
                                   void* stream);

/* Resize + ToTensor of decoded uint8 RGB frames, bit-identical to Pillow's
 * BILINEAR resampling (torchvision Resize on PIL images, datasets/
 * augmentations.py:69-111, then ToTensor :149-160 of the reference).
 * src [N, H0, W0, 3] uint8 -> dst [N, 3, H, W] float32 (value / 255).
 * xbounds [W][2] / ybounds [H][2] = (first input index, tap count) and
 * xcoef [W][KX] / ycoef [H][KY] = Pillow's 22-bit fixed-point weights per
 * output column / row; tmp [N, H0, W, 3] uint8 holds the horizontal pass. */
int dro_resize_rgb8_to_tensor(const unsigned char* src, int N, int H0, int W0, int H, int W,
                              const int* xbounds, const int* xcoef, int KX, const int* ybounds,
                              const int* ycoef, int KY, unsigned char* tmp, float* dst, void* stream);

/* torchvision ColorJitter over PIL frames (colorjitter_sample,
 * datasets/augmentations.py:213-258 of the reference), in place on uint8
 * [N, H, W, 3] frames, bit-identical to Pillow's ImageEnhance / HSV code.
 * params [N][8] 32-bit words per frame: order[4] (0 brightness, 1 contrast,
 * 2 saturation, 3 hue), brightness / contrast / saturation factors (float
 * bits), hue delta (uint8 added to H).  workspace: N x uint64. */
/* Resize alone (uint8 HWC out: the resized PIL image) and ToTensor alone, for
 * the jittered path: resize -> jitter in place -> to tensor. */
int dro_resize_rgb8(const unsigned char* src, int N, int H0, int W0, int H, int W,
                    const int* xbounds, const int* xcoef, int KX, const int* ybounds,
                    const int* ycoef, int KY, unsigned char* tmp, unsigned char* dst, void* stream);
int dro_rgb8_to_tensor(const unsigned char* src, int N, int H, int W, float* dst, void* stream);

/* PNG decode of N images of one geometry (the reference's load_image =
 * PIL.Image.open of KITTI frames, utils/image.py:13-27 via
 * datasets/kitti_dataset.py:354, :387, and read_png_depth,
 * kitti_dataset.py:38-44), bit-identical to Pillow.  zdata: the concatenated
 * IDAT payloads (zlib streams), image i at byte zoff[i] (4-byte aligned) to
 * zoff[i+1] (N+1 int64 offsets).  kind: 0 grey8, 2 RGB8, 6 RGBA8 -> out uint8
 * [N, H, W, 3] (PIL convert("RGB")); 16 grey16 -> out float32 [N, H, W] =
 * value / 256, -1 where 0.  filtered: workspace of N x
 * dro_png_filtered_bytes(H, W, bytes per pixel) bytes.  status[i] (int32,
 * device): 0 decoded, > 0 a malformed stream (the output is then undefined).
 * Non-interlaced images only; rows of at most 16384 bytes. */
size_t dro_png_filtered_bytes(int H, int W, int bpp);
int dro_png_decode(const unsigned char* zdata, const long long* zoff, int N, int H, int W, int kind,
                   unsigned char* filtered, void* out, int* status, void* stream);
int dro_color_jitter_rgb8(unsigned char* frames, int N, int H, int W, const int* params,
                          unsigned long long* workspace, void* stream);

/* Training-mode BatchNorm2d fused with the ReLU / residual add that follows it
 * in the ResNet-18 encoders (networks/optim/extractor.py:7-107 of the reference;
 * BasicBlock: relu(bn(conv(x)) [+ skip])).  Replaces torch.nn.functional.
 * batch_norm(training=True, momentum) + relu: y = act((x - mean) * invstd *
 * gamma + beta + skip) with biased batch variance; running_mean / running_var
 * (nullable together) move by `momentum` toward the batch mean / unbiased
 * variance; *num_batches_tracked (nullable) is incremented.  x, y, skip: NCHW
 * [N, C, HW]; save_mean / save_invstd [C] feed the backward.  Two launches each
 * way, fixed-order fp64 reductions (deterministic).  `workspace` holds
 * dro_batchnorm_workspace_bytes(N, C, HW) bytes; relu is 0 or 1.
 * Backward: grad_x = gamma * invstd * (g - mean(g) - xhat * mean(g * xhat)) with
 * g = grad_out * [y > 0] (relu) or grad_out; grad_gamma = sum(g * xhat),
 * grad_beta = sum(g), grad_skip = g (each nullable). */
size_t dro_batchnorm_workspace_bytes(int N, int C, int HW);
int dro_batchnorm_relu_forward(const float* x, const float* gamma, const float* beta,
                               const float* skip, int relu, int N, int C, int HW, float eps,
                               float momentum, float* running_mean, float* running_var,
                               long long* num_batches_tracked, float* y, float* save_mean,
                               float* save_invstd, void* workspace, size_t workspace_bytes,
                               void* stream);
int dro_batchnorm_relu_backward(const float* grad_out, const float* x, const float* y,
                                const float* gamma, const float* save_mean,
                                const float* save_invstd, int relu, int N, int C, int HW,
                                float* grad_x, float* grad_gamma, float* grad_beta,
                                float* grad_skip, void* workspace, size_t workspace_bytes,
                                void* stream);

/* ------------------------------------------------------------------------
 * Stride-1 'same' convolutions on f32 MFMA for the recurrent update blocks.
 * Replace the nn.Conv2d + activation + torch.cat chains of
 * networks/optim/update.py:5-199 (SepConvGRU :47-74, ProjectionInput* :77-124,
 * heads :5-28, mask :150-153).  The input is the VIRTUAL channel concatenation
 * of 1..4 slices (no copy).  weight [Cout][Cin][KH][KW] with Cin = sum of
 * slice channels; odd KH, KW; padding KH/2, KW/2.
 * act: 0 none, 1 relu, 2 sigmoid, 3 tanh, applied in the epilogue after bias,
 * then the result is multiplied by alpha (alpha != 1 only with act none: the
 * 0.25-scaled mask heads, update.py:153).  The output goes to channels
 * [out_coff, out_coff+Cout) of a [B,out_ctot,H,W] tensor.
 * Limits: C < 4096, C*KH*KW < 65535, every tensor < 2^30 elements.
 * Every call is bitwise run-to-run deterministic (no atomics).
 * ---------------------------------------------------------------------- */
typedef struct dro_slice {
  const float* data;      /* base of a dense [B, total_channels, H, W] tensor */
  int channels;           /* channels taken */
  int total_channels;     /* channel count of the underlying tensor */
  int channel_offset;     /* first channel taken */
  int broadcast;          /* 1: data is [B, total_channels, 1, 1], constant over H x W
                             (e.g. the pose map of ProjectionInputPose, update.py:119) */
} dro_slice;

#define DRO_ACT_NONE 0
#define DRO_ACT_RELU 1
#define DRO_ACT_SIGMOID 2
#define DRO_ACT_TANH 3

/* Split-bf16 operands (the xconv engine).  dro_weight_split writes a weight
 * [Cout][Cin][KH][KW] as three bf16 planes w = w0 + w1 + w2 (24 significant
 * bits): the forward layout `fwd` ([3][Cout][ceil(Cin/32)*KH*KW*32]) and/or the
 * transposed, tap-flipped data-gradient layout `bwd` ([3][Cin][ceil(Cout/32)*
 * KH*KW*32]); sizes from dro_weight_split_bytes(..., transposed 0 / 1).  A conv
 * call given `wsplit` (the layout of its GEMM: fwd for the forward calls, bwd
 * for the data gradient of dro_conv2d_backward) runs its 1x5 / 5x1 / 3x3 / 1x1
 * GEMM on bf16 MFMA as six split products per term (a0b0 + a0b1 + a1b0 + a0b2 +
 * a1b1 + a2b0, f32 accumulation): f32 accuracy (dropped terms < 2^-24 |ab|) at
 * 2.67x the f32 MFMA rate.  wsplit = NULL: the f32-MFMA engine.  The split
 * must be redone whenever the weight changes (the Python layer re-splits once
 * per forward pass).  Replaces the weight side of the same nn.Conv2d calls. */
size_t dro_weight_split_bytes(int Cout, int Cin, int KH, int KW, int transposed);
int dro_weight_split(const float* weight, int Cout, int Cin, int KH, int KW, void* fwd, void* bwd,
                     void* stream);

/* Scratch needed by any conv call below for this shape (split-K partials,
 * weight-gradient partials, the pre-activation gradient); pass a device buffer
 * of at least this size as `workspace`.  No call keeps state in it. */
size_t dro_conv2d_workspace_bytes(int B, int H, int W, int Cin, int Cout, int KH, int KW);

/* Diagnostics: the launch plan the forward (rows = Cout, kch = Cin) or data
 * gradient (rows = Cin, kch = Cout) would use, as 16 integers: halo, BM,
 * row tiles, pixel tiles, K splits, chunks per split, TH, TW, halo row width,
 * channel stride, tiles per row, tiles per image, channels per chunk, LDS bytes,
 * split-K partial bytes, 0. */
int dro_conv2d_plan(int rows, int kch, int KH, int KW, int B, int H, int W, long long* info);

/* Diagnostics only: with a device buffer of >= 16 * (grid blocks) u64, every
 * following halo-conv launch writes per-block s_memtime stamps (kernel start,
 * after the prologue, after each K iteration, after the reductions, after
 * the epilogue) into it; NULL turns it off.  Not thread safe; not for
 * production launches. */
int dro_debug_conv_stamps(void* buffer);

/* Diagnostics: with dro_conv_log(1) every following conv-engine launch records
 * (kernel instantiation name as rocprof prints it, e.g. "dconv_kernel<32, 1,
 * 5, 0, 2, 2, 4>", launch count, algorithmic FLOPs 2*Cout*Cin*KH*KW*B*H*W
 * [* uses]) in a host-side table (cleared on enable); dro_conv_log_read copies
 * it as "name\tlaunches\tflops\n" lines into buf (NUL-terminated, truncated
 * at cap) and returns the full length.  Feeds the per-kernel roofline table
 * (tools/conv_roofline.py). */
int dro_conv_log(int enable);
long long dro_conv_log_read(char* buf, long long cap);

int dro_conv2d_forward(const dro_slice* srcs, int nsrc, const float* weight, const float* bias,
                       int B, int H, int W, int Cout, int KH, int KW, int act, float alpha,
                       float* out, int out_ctot, int out_coff, const void* wsplit,
                       void* workspace, size_t workspace_bytes, void* stream);

/* SepConvGRU z|r gates (update.py:64-65 / :71-72) with r*h fused:
 * zr = sigmoid(conv([h; x]) + b) into a dense [B, 2hd, H, W] (z first) and
 * rh = r * h into a dense [B, hd, H, W].  srcs[0] must be the dense hidden
 * state h (hd channels); weight = cat(convz.weight, convr.weight). */
int dro_convgru_gates_forward(const dro_slice* srcs, int nsrc, const float* weight,
                              const float* bias, int B, int H, int W, int hd, int KH, int KW,
                              float* zr, float* rh, const void* wsplit, void* workspace,
                              size_t workspace_bytes, void* stream);

/* SepConvGRU candidate with the blend fused (update.py:66-67 / :73-74):
 * q = tanh(conv([r*h; x]) + b) saved to q_out (dense [B, Cout, H, W]) and
 * out = (1 - z) * h + z * q into channels [out_coff, +Cout) of [B,out_ctot,H,W]. */
int dro_convgru_blend_forward(const dro_slice* srcs, int nsrc, const float* weight,
                              const float* bias, int B, int H, int W, int Cout, int KH, int KW,
                              const dro_slice* z, const dro_slice* h, float* q_out, float* out,
                              int out_ctot, int out_coff, const void* wsplit, void* workspace,
                              size_t workspace_bytes, void* stream);

/* Gradients of dro_conv2d_forward given dout [B,Cout,H,W] (dense) and, for
 * act != 0, the saved activation output y (the pre-activation gradient
 * alpha*dout*act'(y) is formed in the workspace).  grad_srcs[i] (nullable)
 * receives d/d(source i) into channels [grad_coff[i], +C_i) of a
 * [B, grad_ctot[i], H, W] tensor, overwritten or added (grad_accumulate[i]);
 * a broadcast source receives its per-pixel gradient (the caller sums over
 * H x W).  grad_weight / grad_bias (nullable; grad_bias needs grad_weight)
 * are overwritten, or added to when grad_weight_accumulate is set (a weight
 * shared by several convs of one forward collects one summed gradient). */
int dro_conv2d_backward(const dro_slice* srcs, int nsrc, const float* weight, int B, int H, int W,
                        int Cout, int KH, int KW, int act, float alpha, const dro_slice* y,
                        const float* dout, float* const* grad_srcs, const int* grad_ctot,
                        const int* grad_coff, const int* grad_accumulate, float* grad_weight,
                        float* grad_bias, int grad_weight_accumulate, const void* wsplit,
                        void* workspace, size_t workspace_bytes, void* stream);

/* Weight (+ bias) gradient of ONE weight over several convolutions that use it
 * (the recurrent update blocks apply each weight once per iteration): one
 * launch (+ one split reduction) for all uses instead of one pair per use.
 * Every use has the same geometry and channel split (nsrc slices); act/alpha
 * as in dro_conv2d_forward (the activation derivative is taken from each use's
 * saved output y).  grad_weight [Cout][Cin][KH][KW] / grad_bias [Cout]
 * (nullable) are overwritten or, with accumulate, added to.  1 <= nuse <= 16;
 * kernel shapes 1x1, 1x5, 5x1, 3x3.  Deterministic (fixed reduction order). */
/* Strided convolutions of the ResNet encoders (extractor.py:7-107: the 7x7/s2
 * stems, 3x3/s2 stage entries, 1x1/s2 downsamples of torchvision's ResNet-18).
 * x dense [B, Cin, Hi, Wi]; weight [Cout, Cin, KH, KW]; stride 1 or 2;
 * symmetric zero padding `pad`; out [B, Cout, Ho, Wo] with
 * Ho = (Hi + 2 pad - KH) / stride + 1.  Forward: bias (nullable) and act
 * (0 none, 1 relu, 2 sigmoid, 3 tanh) in the epilogue.  Backward (act none):
 * grad_x (nullable; grad_x_accumulate adds into it), grad_weight / grad_bias
 * (nullable; grad_weight_accumulate adds).  Workspace from
 * dro_conv2d_strided_workspace_bytes.  Flattened implicit GEMM on f32 MFMA,
 * deterministic. */
size_t dro_conv2d_strided_workspace_bytes(int B, int Hi, int Wi, int Cin, int Cout, int KH, int KW,
                                          int stride, int pad);
int dro_conv2d_strided_forward(const float* x, const float* weight, const float* bias, int B, int Hi,
                               int Wi, int Cin, int Cout, int KH, int KW, int stride, int pad, int act,
                               float* out, void* workspace, size_t workspace_bytes, void* stream);
int dro_conv2d_strided_backward(const float* x, const float* weight, const float* dout, int B, int Hi,
                                int Wi, int Cin, int Cout, int KH, int KW, int stride, int pad,
                                float* grad_x, int grad_x_accumulate, float* grad_weight,
                                float* grad_bias, int grad_weight_accumulate, void* workspace,
                                size_t workspace_bytes, void* stream);

/* PoseHead spatial mean + rotation scale + pose update (update.py:16-28,
 * 189-197): out[b, c] = (pose ? pose[b, c] : 0) + mean_{HW} y[b, c] * s_c with
 * s_c = 1 for c < 3, rot_scale (0.01) otherwise.  y dense [B, C, HW].
 * Backward: gy[b, c, p] = gout[b, c] * s_c / HW (the pose gradient is gout). */
int dro_pose_mean_forward(const float* y, const float* pose, float* out, int B, int C, int HW,
                          float rot_scale, void* stream);
int dro_pose_mean_backward(const float* gout, float* gy, int B, int C, int HW, float rot_scale,
                           void* stream);

typedef struct dro_wgrad_use {
  const dro_slice* srcs;  /* the nsrc input slices of this use */
  const float* dout;      /* dense [B,Cout,H,W] gradient w.r.t. this use's output */
  const float* y;         /* dense [B,Cout,H,W] saved output (act != 0), else NULL */
} dro_wgrad_use;

size_t dro_conv2d_weight_grad_multi_workspace_bytes(int nuse, int B, int H, int W, int Cin, int Cout,
                                                    int KH, int KW);

int dro_conv2d_weight_grad_multi(const dro_wgrad_use* uses, int nuse, int nsrc, int B, int H, int W,
                                 int Cout, int KH, int KW, int act, float alpha, float* grad_weight,
                                 float* grad_bias, int accumulate, void* workspace,
                                 size_t workspace_bytes, void* stream);

/* SepConvGRU backward, elementwise parts (update.py:67-70): with zr the saved
 * sigmoid gates [B,2hd,H,W] (z first), q the saved candidate [B,hd,H,W].
 * Outputs are gradients w.r.t. the gates' PRE-activations (feed them to
 * dro_conv2d_backward with act = DRO_ACT_NONE):
 *   stage 1: dq = dh' z (1-q^2); dzr[:, :hd] = dh' (q-h) z (1-z); dh = dh' (1-z)
 *   stage 2: dzr[:, hd:] = drh h r (1-r); dh += drh r     (drh = dL/d(r*h)) */
int dro_gru_backward_elem(int stage, int B, int hd, int H, int W, const float* dhn,
                          const float* zr, const float* q, const float* h, const float* drh,
                          float* dq, float* dzr, float* dh, void* stream);

/* The candidate conv's data gradient with stage 2 in its epilogue (ABI 8):
 * dro_conv2d_backward of q~ = conv([r*h, x...]) for Cout = hd, act NONE, no
 * weight gradient, given dq (stage 1's output), except that source 0 (r*h,
 * hd channels) is not stored: each d(r*h) element becomes
 *   dzr[:, hd:] = d(r*h) h r (1-r);  dh += d(r*h) r
 * (stage 2 of dro_gru_backward_elem, one launch fewer per GRU half).
 * grad_srcs[0] / grad_ctot[0] / grad_coff[0] / grad_accumulate[0] are ignored;
 * sources 1.. behave as in dro_conv2d_backward.  Workspace: the
 * dro_conv2d_workspace_bytes of the conv.  Replaces the d(r*h) path of
 * SepConvGRU's backward (dro_sfm/networks/optim/update.py:67-70, autograd). */
int dro_convgru_candidate_backward(const dro_slice* srcs, int nsrc, const float* weight, int B, int H, int W,
                                   int hd, int KH, int KW, const float* dq, const float* zr, const float* h,
                                   float* dzr, float* dh, float* const* grad_srcs, const int* grad_ctot,
                                   const int* grad_coff, const int* grad_accumulate, void* workspace,
                                   size_t workspace_bytes, void* stream);

/* The gate conv's data gradient of a SepConvGRU's SECOND half with the FIRST
 * half's stage 1 in its epilogue (ABI 8): dro_conv2d_backward of
 * [z|r]~ = conv([h, x...]) (Cout = 2 hd, act NONE, no weight gradient) given
 * dzr_in, source 0 = this half's h (hd channels, gradient target
 * grad_srcs[0] dense [B,hd,H,W], always accumulated).  h is the first half's
 * output, so its finished gradient is the first half's dh'; each element gn
 * is stored and turned into the first half's stage 1 (dro_gru_backward_elem):
 *   prev_dq = gn z (1-q^2); prev_dzr[:, :hd] = gn (q-h) z (1-z);
 *   prev_dh = gn (1-z)  (added into when prev_dh_accumulate)
 * with z, q, h the first half's saved gate, candidate and input state. */
int dro_convgru_gates_backward(const dro_slice* srcs, int nsrc, const float* weight, int B, int H, int W,
                               int hd, int KH, int KW, const float* dzr_in, float* const* grad_srcs,
                               const int* grad_ctot, const int* grad_coff, const int* grad_accumulate,
                               const float* prev_zr, const float* prev_q, const float* prev_h, float* prev_dq,
                               float* prev_dzr, float* prev_dh, int prev_dh_accumulate, void* workspace,
                               size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------
 * BatchNorm fused into the encoders' 3x3 stride-1 convolutions (ABI 10).
 * Replaces the separate BN launches of the ResNet-18 BasicBlocks
 * (dro_sfm/networks/optim/extractor.py:67-107 via torchvision's BasicBlock:
 * conv1 -> bn1 -> relu -> conv2 -> bn2 (+ skip) -> relu) with work inside the
 * convolutions, batchnorm.hip's arithmetic (fixed-order fp64 statistics,
 * torch.nn.functional.batch_norm training semantics):
 *   - the PRODUCING conv's epilogue takes the batch statistics of its output
 *     (per pixel tile, folded by the last block to finish: no statistics
 *     launch), writes save_mean / save_invstd / the running statistics and
 *     the coefficients its consumer needs into `out_state`;
 *   - the CONSUMING conv stages relu(bn(x) [+ skip]) from those coefficients
 *     and stores it once per pixel into `in_y` (the BN output the weight
 *     gradient and the ReLU mask need): no apply launch;
 *   - backward, the consumer's data gradient takes g = dy [y > 0] and the BN
 *     backward's statistics in its epilogue (grad_x receives g), and the
 *     producer's data gradient stages dz = k (g - mean(g) - xhat mean(g xhat))
 *     and stores it to `gin_dz` for the producer's weight gradient.
 * A BN state is per site and direction: dro_bn_state_bytes of the BN's
 * activation geometry, ZERO-FILLED once before its first use (its counters
 * reset themselves; one call at a time per state). */
typedef struct dro_bn_params {   /* forward statistics of a training-mode BatchNorm2d */
  const float* gamma;            /* nullable (1) */
  const float* beta;             /* nullable (0) */
  float* running_mean;           /* nullable together with running_var */
  float* running_var;
  long long* num_batches_tracked;/* nullable */
  float eps, momentum;
  float* save_mean;              /* [C] out */
  float* save_invstd;            /* [C] out */
} dro_bn_params;

typedef struct dro_bn_grad_params {   /* backward statistics of BN + ReLU */
  const float* y;                /* the ReLU output (mask y > 0), dense [B, C, H, W] */
  const float* z;                /* the BN input, dense [B, C, H, W] */
  const float* gamma;            /* nullable (1) */
  const float* save_mean;
  const float* save_invstd;
  float* grad_gamma;             /* [C] out, nullable */
  float* grad_beta;              /* [C] out, nullable */
} dro_bn_grad_params;

size_t dro_bn_state_bytes(int B, int H, int W, int C);

/* y = relu(bn(x) [+ skip]) (relu 0/1) from a BN state a producing
 * dro_conv2d_bn_forward filled: the BN output of a site whose consumer is not
 * a 3x3 stride-1 conv (one launch instead of statistics + apply). */
int dro_bn_apply(const float* x, const float* skip, int relu, int B, int C, int H, int W, const void* state,
                 float* y, void* stream);

/* dz = k (g - mean(g) - xhat mean(g xhat)) from the backward BN state a
 * consumer's dro_conv2d_bn_backward_data (src_bn) filled, g its grad_x and z
 * the BN input: the BN backward's apply for a producer whose data gradient
 * does not stage it (gin_state). */
int dro_bn_backward_apply(const float* g, const float* z, int B, int C, int H, int W, const void* state,
                          float* dz, void* stream);

/* out [B, Cout, H, W] = conv3x3(s) (stride 1, pad 1, no bias), s = x or, with
 * in_state (the producer's out_state), s = relu(bn(x) [+ in_skip]) stored to
 * in_y; with bn / out_state the BN statistics of out.  Workspace:
 * dro_conv2d_workspace_bytes(B, H, W, Cin, Cout, 3, 3). */
int dro_conv2d_bn_forward(const float* x, int B, int H, int W, int Cin, const float* weight, int Cout,
                          const void* in_state, const float* in_skip, float* in_y,
                          const dro_bn_params* bn, void* out_state, float* out, void* workspace,
                          size_t workspace_bytes, void* stream);

/* Data gradient of out = conv3x3(s) into grad_x [B, Cin, H, W] (added when
 * grad_x_accumulate) from dout [B, Cout, H, W]; with gin_state (the output
 * BN's state after its consumer's backward) dout is that BN's g and the
 * conv's output gradient dz is formed in staging (z = gin_z) and stored to
 * gin_dz; with src_bn / src_state the source is relu(bn(z)) and grad_x
 * receives g = dy [y > 0] (dense, not accumulated) plus the BN backward's
 * statistics (src_state, grad_gamma / grad_beta). */
int dro_conv2d_bn_backward_data(const float* weight, int B, int H, int W, int Cin, int Cout, const float* dout,
                                const void* gin_state, const float* gin_z, float* gin_dz,
                                const dro_bn_grad_params* src_bn, void* src_state, float* grad_x,
                                int grad_x_accumulate, void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Fused Adam over flat fp32 buffers (the data-parallel trainer's parameters,
 * gradients and moments; torch.optim.Adam semantics, amsgrad off).  `step` is
 * the device-side step counter AFTER the increment for this update; `hyper`
 * points to 5 device floats {lr, beta1, beta2, eps, weight_decay}, read at
 * run time so a captured graph follows a learning-rate schedule.  All four
 * buffers 16-byte aligned.  Replaces the optimizer step of the reference's
 * training loop (trainers/horovod_trainer.py:113-116, torch.optim.Adam).
 * ---------------------------------------------------------------------- */
int dro_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long long n,
                  const float* step, const float* hyper, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DRO_AMD_H */
