// Convex 8x upsampling of the 1/8-resolution inverse depth.
//
// Replaces DepthPoseNet.upsample_depth (dro_sfm/networks/depth_pose/
// DepthPoseNet.py:63-74): view -> softmax over the 9 taps -> unfold(3x3, zero
// pad) -> weighted sum -> permute -> reshape (6 ATen kernels forward, ~8
// backward) with one launch each way.
//   out[b, y*r+a, x*r+c] = sum_k softmax_k(mask[b, k*r*r + a*r + c, y, x])
//                          * inv_pad[b, y+ky-1, x+kx-1],   k = 3*ky + kx
// One thread per (b, a, y, x) handles the r sub-pixel columns c: every mask
// load of a wave is a coalesced row segment and the r outputs it writes are
// contiguous.  Roofline: HBM bound, bytes = 4*(9r^2 + 1)*hw read +
// 4*r^2*hw written per image.
#include <hip/hip_runtime.h>

#include "dro_common.hpp"

namespace dro {

constexpr int kMaxR = 8;

__global__ __launch_bounds__(256) void convex_up_fwd_kernel(const float* __restrict__ inv,
                                                            const float* __restrict__ mask, int B,
                                                            int h, int w, int r,
                                                            float* __restrict__ out) {
  const int hw = h * w;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * r * hw) return;
  const int pix = idx % hw, a = (idx / hw) % r, b = idx / (hw * r);
  const int y = pix / w, x = pix % w;
  float d[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
    d[k] = (yy >= 0 && yy < h && xx >= 0 && xx < w) ? inv[(size_t)b * hw + yy * w + xx] : 0.f;
  }
  const float* mb = mask + (size_t)b * 9 * r * r * hw + pix;
  float* ob = out + ((size_t)b * h * r + (size_t)y * r + a) * (w * r) + (size_t)x * r;
  for (int c = 0; c < r; ++c) {
    float m[9], mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      m[k] = mb[(size_t)(k * r * r + a * r + c) * hw];
      mx = fmaxf(mx, m[k]);
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      m[k] = expf(m[k] - mx);
      s += m[k];
    }
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) acc += (m[k] / s) * d[k];
    ob[c] = acc;
  }
}

__global__ __launch_bounds__(256) void convex_up_bwd_kernel(
    const float* __restrict__ inv, const float* __restrict__ mask, const float* __restrict__ gout,
    int B, int h, int w, int r, float* __restrict__ ginv, float* __restrict__ gmask) {
  const int hw = h * w;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * r * hw) return;
  const int pix = idx % hw, a = (idx / hw) % r, b = idx / (hw * r);
  const int y = pix / w, x = pix % w;
  float d[9], gd[9];
  bool ok[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
    ok[k] = yy >= 0 && yy < h && xx >= 0 && xx < w;
    d[k] = ok[k] ? inv[(size_t)b * hw + yy * w + xx] : 0.f;
    gd[k] = 0.f;
  }
  const float* mb = mask + (size_t)b * 9 * r * r * hw + pix;
  float* gmb = gmask + (size_t)b * 9 * r * r * hw + pix;
  const float* gb = gout + ((size_t)b * h * r + (size_t)y * r + a) * (w * r) + (size_t)x * r;
  for (int c = 0; c < r; ++c) {
    const float G = gb[c];
    float m[9], mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      m[k] = mb[(size_t)(k * r * r + a * r + c) * hw];
      mx = fmaxf(mx, m[k]);
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      m[k] = expf(m[k] - mx);
      s += m[k];
    }
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      m[k] = m[k] / s;          // softmax
      gd[k] += m[k] * G;        // d/d inv tap
      dot += m[k] * (G * d[k]);
    }
#pragma unroll
    for (int k = 0; k < 9; ++k)
      gmb[(size_t)(k * r * r + a * r + c) * hw] = m[k] * (G * d[k] - dot);
  }
  if (ginv) {
#pragma unroll
    for (int k = 0; k < 9; ++k)
      if (ok[k]) atomicAdd(ginv + (size_t)b * hw + (y + k / 3 - 1) * w + (x + k % 3 - 1), gd[k]);
  }
}

}  // namespace dro

using namespace dro;

static int up_check(const float* inv, const float* mask, int B, int h, int w, int ratio) {
  if (!inv || !mask) {
    set_error("convex_upsample: NULL input");
    return DRO_E_NULL;
  }
  if (B < 1 || h < 1 || w < 1 || ratio < 1 || ratio > kMaxR) {
    set_error("convex_upsample: sizes out of range (ratio 1..8)");
    return DRO_E_SHAPE;
  }
  return DRO_OK;
}

extern "C" int dro_convex_upsample_forward(const float* inv, const float* mask, int B, int h, int w,
                                           int ratio, float* out, void* stream) {
  int st = up_check(inv, mask, B, h, w, ratio);
  if (st) return st;
  if (!out) {
    set_error("convex_upsample_forward: NULL out");
    return DRO_E_NULL;
  }
  const int total = B * ratio * h * w;
  hipLaunchKernelGGL(convex_up_fwd_kernel, dim3((total + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, inv, mask, B, h, w, ratio, out);
  return launch_status("convex_up_fwd_kernel launch failed");
}

extern "C" int dro_convex_upsample_backward(const float* inv, const float* mask,
                                            const float* grad_out, int B, int h, int w, int ratio,
                                            float* grad_inv, float* grad_mask, void* stream) {
  int st = up_check(inv, mask, B, h, w, ratio);
  if (st) return st;
  if (!grad_out || !grad_mask) {
    set_error("convex_upsample_backward: NULL grad_out/grad_mask");
    return DRO_E_NULL;
  }
  hipStream_t s = (hipStream_t)stream;
  if (grad_inv && (st = launch_zero(grad_inv, (size_t)B * h * w, s))) return st;
  const int total = B * ratio * h * w;
  hipLaunchKernelGGL(convex_up_bwd_kernel, dim3((total + 255) / 256), dim3(256), 0, s, inv, mask,
                     grad_out, B, h, w, ratio, grad_inv, grad_mask);
  return launch_status("convex_up_bwd_kernel launch failed");
}
