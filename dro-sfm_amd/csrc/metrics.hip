// Depth evaluation metrics on the GPU.
//
// Replaces compute_depth_metrics (dro_sfm/utils/depth.py:259-343 of the
// reference): bilinear (align_corners=True) upsampling of the prediction to the
// ground-truth resolution, clamp 1e-6, validity (min < gt < max, optional
// garg / eigen_nyu crop), optional ground-truth median scaling, then
// abs_rel, sq_rel, rmse, rmse_log, a1..a3, SILog and iabs_diff per image,
// averaged over the batch.  The reference loops over images in Python with
// ~25 ATen launches each and boolean-index compaction; here:
//   prepare : one pass, writes the upsampled prediction and gt/pred ratios
//             (+inf where invalid, so a k-th-smallest selection over the row
//             is the median of the valid ratios) and per-block valid counts;
//   reduce  : one pass over (image, pixel block) with the per-image scale,
//             per-pixel terms in fp32 exactly as the reference writes them,
//             block partials in fp64 (fixed order: deterministic);
//   finalize: one block, fixed-order sums -> the 9 metrics.
// Roofline: HBM bound.  Algorithmic bytes per gt pixel: prepare 4 (gt) +
// 8 (pred_up, ratio written) + the low-res prediction once; reduce 8 (gt,
// pred_up).
#include <hip/hip_runtime.h>
#include <math.h>

#include "dro_common.hpp"

namespace dro {

constexpr int kMetThreads = 256;
// per-image sums: n, a1, a2, a3 counts, |d|/g, d^2/g, d^2, (log g - log p)^2,
// |1/p - 1/g|, sum (log g - log p)
constexpr int kMetSlots = 10;

struct MetArgs {
  int B, H, W, h, w;
  float min_d, max_d;
  int y1, y2, x1, x2;   // crop rectangle [y1, y2) x [x1, x2); y1 < 0: no crop
  float sy, sx;         // (h-1)/(H-1), (w-1)/(W-1) in fp32 (ATen's area_pixel_compute_scale)
  int same;             // prediction already at the gt resolution
  // compute_depth_metrics_demon (utils/depth.py:343-398): no clamp to the
  // depth range; with gt scaling the gt is divided by the norm of the first
  // reference's gt translation, gpose[b * pose_stride + {3, 7, 11}]
  int demon;
  const float* gpose;
  long long pose_stride;
};

// |t| of image b's first-reference gt translation (torch.sqrt(t.dot(t)) in fp32)
__device__ __forceinline__ float met_tnorm(const MetArgs& a, int b) {
  const float* p = a.gpose + (size_t)b * a.pose_stride;
  const float x = p[3], y = p[7], z = p[11];
  return sqrtf(__fadd_rn(__fadd_rn(__fmul_rn(x, x), __fmul_rn(y, y)), __fmul_rn(z, z)));
}

__device__ __forceinline__ bool met_valid(const MetArgs& a, float g, int y, int x) {
  bool v = g > a.min_d && g < a.max_d;
  if (a.y1 >= 0) v = v && y >= a.y1 && y < a.y2 && x >= a.x1 && x < a.x2;
  return v;
}

// upsample_bilinear2d, align_corners=True (ATen: src = scale * dst, i0 = (int)src,
// i1 = i0 + (i0 < in - 1), lambda = src - i0)
__device__ __forceinline__ float met_upsample(const MetArgs& a, const float* __restrict__ p, int y, int x) {
  if (a.same) return p[(size_t)y * a.w + x];
  const float ry = a.sy * (float)y, rx = a.sx * (float)x;
  const int y0 = (int)ry, x0 = (int)rx;
  const int yp = y0 < a.h - 1 ? 1 : 0, xp = x0 < a.w - 1 ? 1 : 0;
  const float ly1 = ry - (float)y0, lx1 = rx - (float)x0;
  const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
  const float* r0 = p + (size_t)y0 * a.w + x0;
  const float* r1 = r0 + (size_t)yp * a.w;
  return ly0 * (lx0 * r0[0] + lx1 * r0[xp]) + ly1 * (lx0 * r1[0] + lx1 * r1[xp]);
}

__global__ __launch_bounds__(kMetThreads) void metrics_prepare_kernel(MetArgs a, const float* __restrict__ gt,
                                                                     const float* __restrict__ pred,
                                                                     float* __restrict__ pred_up,
                                                                     float* __restrict__ ratio,
                                                                     int* __restrict__ counts) {
  __shared__ int wcount[kMetThreads / kWave];
  const int b = blockIdx.y;
  const size_t HW = (size_t)a.H * a.W;
  const size_t p = (size_t)blockIdx.x * kMetThreads + threadIdx.x;
  int v = 0;
  const float tn = a.gpose ? met_tnorm(a, b) : 1.f;
  if (p < HW) {
    const int y = (int)(p / a.W), x = (int)(p % a.W);
    const float g = gt[b * HW + p];
    const float pv = fmaxf(met_upsample(a, pred + (size_t)b * a.h * a.w, y, x), 1e-6f);
    pred_up[b * HW + p] = pv;
    v = met_valid(a, g, y, x) ? 1 : 0;
    ratio[b * HW + p] = v ? (a.gpose ? g / tn : g) / pv : INFINITY;
  }
  // block count of valid pixels (wave ballot, then the block's waves in order)
  const unsigned long long m = __ballot(v);
  if ((threadIdx.x & 63) == 0) wcount[threadIdx.x >> 6] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int i = 0; i < kMetThreads / kWave; ++i) s += wcount[i];
    counts[(size_t)b * gridDim.x + blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(kMetThreads) void metrics_reduce_kernel(MetArgs a, const float* __restrict__ gt,
                                                                    const float* __restrict__ pred_up,
                                                                    const float* __restrict__ scale,
                                                                    double* __restrict__ partial) {
  __shared__ double red[kMetSlots][kMetThreads / kWave];
  const int b = blockIdx.y;
  const size_t HW = (size_t)a.H * a.W;
  const float s = scale ? scale[b] : 1.f;
  const float tn = a.gpose ? met_tnorm(a, b) : 1.f;
  double acc[kMetSlots];
#pragma unroll
  for (int k = 0; k < kMetSlots; ++k) acc[k] = 0.0;
  // grid-stride over the image: a fixed pixel -> (block, thread) assignment
  for (size_t p = (size_t)blockIdx.x * kMetThreads + threadIdx.x; p < HW; p += (size_t)gridDim.x * kMetThreads) {
    const int y = (int)(p / a.W), x = (int)(p % a.W);
    float g = gt[b * HW + p];
    if (!met_valid(a, g, y, x)) continue;
    float pv = pred_up[b * HW + p];
    if (a.demon) {                                              // :364-373: no clamps
      if (a.gpose) g = g / tn;
      if (scale) pv = pv * s;
    } else {
      if (scale) pv = fminf(fmaxf(pv * s, a.min_d), a.max_d);   // median scaling + clamp
      pv = fminf(fmaxf(pv, a.min_d), a.max_d);
    }
    const float th = fmaxf(g / pv, pv / g);
    const float d = g - pv;
    const float ld = logf(g) - logf(pv);
    acc[0] += 1.0;
    acc[1] += th < 1.25f ? 1.0 : 0.0;
    acc[2] += th < 1.5625f ? 1.0 : 0.0;
    acc[3] += th < 1.953125f ? 1.0 : 0.0;
    acc[4] += (double)(fabsf(d) / g);
    acc[5] += (double)(d * d / g);
    acc[6] += (double)(d * d);
    acc[7] += (double)(ld * ld);
    acc[8] += (double)fabsf(1.f / pv - 1.f / g);
    acc[9] += (double)ld;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < kMetSlots; ++k) {
    double v = acc[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[k][wid] = v;
  }
  __syncthreads();
  if (threadIdx.x < kMetSlots) {
    double v = 0.0;
    for (int i = 0; i < kMetThreads / kWave; ++i) v += red[threadIdx.x][i];
    partial[((size_t)b * gridDim.x + blockIdx.x) * kMetSlots + threadIdx.x] = v;
  }
}

// metrics[9] = batch means of abs_rel, sq_rel, rmse, rmse_log, a1, a2, a3,
// SILog, iabs_diff (images without valid pixels contribute 0, as in the
// reference's `continue` with the division by the full batch size)
__global__ __launch_bounds__(256) void metrics_finalize_kernel(int B, int nblk, const double* __restrict__ partial,
                                                               float* __restrict__ metrics) {
  __shared__ double red[kMetSlots][4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  double out[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int b = 0; b < B; ++b) {
    // thread k holds block partial k (and k + 256, ...); fixed shuffle tree, then the 4 waves in order
#pragma unroll
    for (int t = 0; t < kMetSlots; ++t) {
      double v = 0.0;
      for (int k = threadIdx.x; k < nblk; k += 256) v += partial[((size_t)b * nblk + k) * kMetSlots + t];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (lane == 0) red[t][wid] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double S[kMetSlots];
      for (int t = 0; t < kMetSlots; ++t) S[t] = ((red[t][0] + red[t][1]) + red[t][2]) + red[t][3];
      const double n = S[0];
      if (n > 0.0) {
        out[0] += S[4] / n;
        out[1] += S[5] / n;
        out[2] += sqrt(S[6] / n);
        out[3] += sqrt(S[7] / n);
        out[4] += S[1] / n;
        out[5] += S[2] / n;
        out[6] += S[3] / n;
        out[7] += sqrt(fmax(S[7] / n - (S[9] * S[9]) / (n * n), 0.0));
        out[8] += S[8] / n;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0)
    for (int k = 0; k < 9; ++k) metrics[k] = (float)(out[k] / B);
}

// ------------------------------------------------------------------ per-image median (radix select)
// torch.median of the valid ratios = the ((n-1)/2)-th smallest (0-based).
// Ratios are positive floats or +inf (invalid), whose IEEE bit patterns order
// like the values, so the k-th smallest of the whole row is found digit by
// digit: 4 passes of an 8-bit histogram over the keys that match the prefix
// found so far (LDS counts, then integer atomics per bin: exact), each
// followed by a one-block select.  No host round trip.
// state[b] = {prefix, k remaining, n valid}
__global__ __launch_bounds__(256) void median_init_kernel(const int* __restrict__ counts, int nblk,
                                                          unsigned* __restrict__ state,
                                                          unsigned* __restrict__ hist) {
  __shared__ long long wsum[4];
  const int b = blockIdx.x;
  hist[b * 256 + threadIdx.x] = 0u;
  long long n = 0;   // integer sums: exact in any order
  for (int k = threadIdx.x; k < nblk; k += 256) n += counts[(size_t)b * nblk + k];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) {
    n = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    state[3 * b + 0] = 0u;
    state[3 * b + 1] = n > 0 ? (unsigned)((n - 1) / 2) : 0u;
    state[3 * b + 2] = (unsigned)n;
  }
}

__global__ __launch_bounds__(256) void median_hist_kernel(const float* __restrict__ ratio, unsigned HW,
                                                          const unsigned* __restrict__ state, int shift,
                                                          unsigned* __restrict__ hist) {
  __shared__ unsigned h[256];
  h[threadIdx.x] = 0u;
  __syncthreads();
  const int b = blockIdx.y;
  const unsigned hi = shift == 24 ? 0u : (0xFFFFFFFFu << (shift + 8));
  const unsigned prefix = state[3 * b] & hi;
  const float* __restrict__ r = ratio + (size_t)b * HW;
  for (unsigned p = blockIdx.x * 256u + threadIdx.x; p < HW; p += gridDim.x * 256u) {
    const unsigned key = __float_as_uint(r[p]);
    if ((key & hi) == prefix) atomicAdd(&h[(key >> shift) & 255u], 1u);
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&hist[b * 256 + threadIdx.x], h[threadIdx.x]);
}

__global__ __launch_bounds__(256) void median_select_kernel(unsigned* __restrict__ state,
                                                            unsigned* __restrict__ hist, int shift,
                                                            float* __restrict__ scale) {
  __shared__ unsigned hs[256];
  const int b = blockIdx.x;
  hs[threadIdx.x] = hist[b * 256 + threadIdx.x];
  hist[b * 256 + threadIdx.x] = 0u;   // ready for the next pass
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned krem = state[3 * b + 1], prefix = state[3 * b];
    for (int bin = 0; bin < 256; ++bin) {
      if (krem < hs[bin]) {
        prefix |= (unsigned)bin << shift;
        break;
      }
      krem -= hs[bin];
    }
    state[3 * b] = prefix;
    state[3 * b + 1] = krem;
    if (shift == 0) scale[b] = state[3 * b + 2] > 0u ? __uint_as_float(prefix) : 1.f;
  }
}

}  // namespace dro

using namespace dro;

namespace {
constexpr int kReduceBlocks = 256;  // pixel blocks per image in the reduce pass (>= 4 waves per SIMD at B = 4)

int met_setup(MetArgs& a, int B, int H, int W, int h, int w, float min_d, float max_d, int y1, int y2,
              int x1, int x2) {
  if (B < 1 || H < 1 || W < 1 || h < 1 || w < 1 || B > 65535 || (long long)H * W >= (1LL << 31)) {
    set_error("depth_metrics: sizes out of range");
    return DRO_E_SHAPE;
  }
  if (y1 >= 0 && (y2 < y1 || x2 < x1 || x1 < 0)) {
    set_error("depth_metrics: bad crop rectangle");
    return DRO_E_SHAPE;
  }
  a.B = B;
  a.H = H;
  a.W = W;
  a.h = h;
  a.w = w;
  a.min_d = min_d;
  a.max_d = max_d;
  a.y1 = y1;
  a.y2 = y2;
  a.x1 = x1;
  a.x2 = x2;
  a.same = (h == H && w == W) ? 1 : 0;
  a.sy = H > 1 ? (float)(h - 1) / (float)(H - 1) : 0.f;
  a.sx = W > 1 ? (float)(w - 1) / (float)(W - 1) : 0.f;
  a.demon = 0;
  a.gpose = nullptr;
  a.pose_stride = 0;
  return DRO_OK;
}
}  // namespace

extern "C" int dro_depth_metrics_blocks(int H, int W) {
  return (int)(((long long)H * W + kMetThreads - 1) / kMetThreads);
}

extern "C" size_t dro_depth_metrics_workspace_bytes(int B) {
  return sizeof(double) * (size_t)B * kReduceBlocks * kMetSlots;
}

extern "C" size_t dro_depth_metrics_median_workspace_bytes(int B) {
  return sizeof(unsigned) * (size_t)B * (256 + 3);
}

extern "C" int dro_depth_metrics_median(const float* ratio, const int* block_counts, int B, int H, int W,
                                        float* scale, void* workspace, void* stream) {
  if (!ratio || !block_counts || !scale || !workspace) {
    set_error("depth_metrics_median: NULL pointer");
    return DRO_E_NULL;
  }
  if (B < 1 || B > 65535 || H < 1 || W < 1 || (long long)H * W >= (1LL << 31)) {
    set_error("depth_metrics_median: sizes out of range");
    return DRO_E_SHAPE;
  }
  hipStream_t s = (hipStream_t)stream;
  unsigned* hist = (unsigned*)workspace;
  unsigned* state = hist + (size_t)B * 256;
  const unsigned HW = (unsigned)((long long)H * W);
  const int nblk = dro_depth_metrics_blocks(H, W);
  hipLaunchKernelGGL(median_init_kernel, dim3(B), dim3(256), 0, s, block_counts, nblk, state, hist);
  int st = launch_status("median_init_kernel launch failed");
  if (st) return st;
  const unsigned hblk = min(256u, (HW + 255u) / 256u);
  for (int shift = 24; shift >= 0; shift -= 8) {
    hipLaunchKernelGGL(median_hist_kernel, dim3(hblk, B), dim3(256), 0, s, ratio, HW, state, shift, hist);
    if ((st = launch_status("median_hist_kernel launch failed"))) return st;
    hipLaunchKernelGGL(median_select_kernel, dim3(B), dim3(256), 0, s, state, hist, shift, scale);
    if ((st = launch_status("median_select_kernel launch failed"))) return st;
  }
  return DRO_OK;
}

extern "C" int dro_depth_metrics_prepare(const float* gt, const float* pred, int B, int H, int W,
                                         int h, int w, float min_depth, float max_depth, int crop_y1,
                                         int crop_y2, int crop_x1, int crop_x2, float* pred_up,
                                         float* ratio, int* block_counts, void* stream) {
  if (!gt || !pred || !pred_up || !ratio || !block_counts) {
    set_error("depth_metrics_prepare: NULL pointer");
    return DRO_E_NULL;
  }
  MetArgs a;
  int st = met_setup(a, B, H, W, h, w, min_depth, max_depth, crop_y1, crop_y2, crop_x1, crop_x2);
  if (st) return st;
  hipLaunchKernelGGL(metrics_prepare_kernel, dim3(dro_depth_metrics_blocks(H, W), B), dim3(kMetThreads), 0,
                     (hipStream_t)stream, a, gt, pred, pred_up, ratio, block_counts);
  return launch_status("metrics_prepare_kernel launch failed");
}

extern "C" int dro_depth_metrics_reduce(const float* gt, const float* pred_up, const float* scale, int B,
                                        int H, int W, float min_depth, float max_depth, int crop_y1,
                                        int crop_y2, int crop_x1, int crop_x2, float* metrics,
                                        void* workspace, void* stream) {
  if (!gt || !pred_up || !metrics || !workspace) {
    set_error("depth_metrics_reduce: NULL pointer");
    return DRO_E_NULL;
  }
  MetArgs a;
  int st = met_setup(a, B, H, W, H, W, min_depth, max_depth, crop_y1, crop_y2, crop_x1, crop_x2);
  if (st) return st;
  double* partial = (double*)workspace;
  hipLaunchKernelGGL(metrics_reduce_kernel, dim3(kReduceBlocks, B), dim3(kMetThreads), 0, (hipStream_t)stream,
                     a, gt, pred_up, scale, partial);
  if ((st = launch_status("metrics_reduce_kernel launch failed"))) return st;
  hipLaunchKernelGGL(metrics_finalize_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, B, kReduceBlocks,
                     partial, metrics);
  return launch_status("metrics_finalize_kernel launch failed");
}

// compute_depth_metrics_demon (utils/depth.py:343-398): the same three passes
// (prepare, dro_depth_metrics_median, reduce) without crop or clamps; with
// gt_pose (gt scaling on) the ground truth is divided by |t| of each image's
// first-reference gt translation (gt_pose + b * pose_stride floats, a row-major
// 4x4 or 3x4 transform).  gt_pose NULL: no gt normalisation (use_gt_scale False).
extern "C" int dro_depth_metrics_demon_prepare(const float* gt, const float* pred, const float* gt_pose,
                                               long long pose_stride, int B, int H, int W, int h, int w,
                                               float min_depth, float max_depth, float* pred_up, float* ratio,
                                               int* block_counts, void* stream) {
  if (!gt || !pred || !pred_up || !ratio || !block_counts) {
    set_error("depth_metrics_demon_prepare: NULL pointer");
    return DRO_E_NULL;
  }
  MetArgs a;
  int st = met_setup(a, B, H, W, h, w, min_depth, max_depth, -1, -1, -1, -1);
  if (st) return st;
  a.demon = 1;
  a.gpose = gt_pose;
  a.pose_stride = pose_stride;
  hipLaunchKernelGGL(metrics_prepare_kernel, dim3(dro_depth_metrics_blocks(H, W), B), dim3(kMetThreads), 0,
                     (hipStream_t)stream, a, gt, pred, pred_up, ratio, block_counts);
  return launch_status("metrics_prepare_kernel launch failed");
}

extern "C" int dro_depth_metrics_demon_reduce(const float* gt, const float* pred_up, const float* scale,
                                              const float* gt_pose, long long pose_stride, int B, int H, int W,
                                              float min_depth, float max_depth, float* metrics, void* workspace,
                                              void* stream) {
  if (!gt || !pred_up || !metrics || !workspace) {
    set_error("depth_metrics_demon_reduce: NULL pointer");
    return DRO_E_NULL;
  }
  MetArgs a;
  int st = met_setup(a, B, H, W, H, W, min_depth, max_depth, -1, -1, -1, -1);
  if (st) return st;
  a.demon = 1;
  a.gpose = gt_pose;
  a.pose_stride = pose_stride;
  double* partial = (double*)workspace;
  hipLaunchKernelGGL(metrics_reduce_kernel, dim3(kReduceBlocks, B), dim3(kMetThreads), 0, (hipStream_t)stream,
                     a, gt, pred_up, scale, partial);
  if ((st = launch_status("metrics_reduce_kernel launch failed"))) return st;
  hipLaunchKernelGGL(metrics_finalize_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, B, kReduceBlocks,
                     partial, metrics);
  return launch_status("metrics_finalize_kernel launch failed");
}
