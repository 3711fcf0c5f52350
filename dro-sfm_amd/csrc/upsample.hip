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

#include <cstddef>

#include "dro_common.hpp"

namespace dro {

constexpr int kMaxR = 8;

// out = add + mul * upsample (the disp_to_depth scaling of DepthPoseNet.scale_inv_depth,
// DepthPoseNet.py:128/181, fused: a multiply then an add, as the reference)
__global__ __launch_bounds__(256) void convex_up_fwd_kernel(const float* __restrict__ inv,
                                                            const float* __restrict__ mask, int B,
                                                            int h, int w, int r, float add, float mul,
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
    ob[c] = __fadd_rn(add, __fmul_rn(mul, acc));
  }
}

__global__ __launch_bounds__(256) void convex_up_bwd_kernel(
    const float* __restrict__ inv, const float* __restrict__ mask, const float* __restrict__ gout,
    int B, int h, int w, int r, float mul, float* __restrict__ ginv, float* __restrict__ gmask) {
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
    const float G = __fmul_rn(gb[c], mul);
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

// One thread per OUTPUT pixel (b, y*r+a, x*r+c), lanes running along the
// output row (c fastest): r x more threads than the per-(a, y, x) kernels
// above (30 720 -> 245 760 at KITTI B=2, which left 3/4 of the chip idle) and
// every output store a contiguous row segment.  Per output the arithmetic is
// the per-(a, y, x) kernels' inner iteration, so results are bit-identical;
// the backward sums the inverse-depth tap gradients of the r sub-pixel lanes
// of one (a, y, x) in lane order c = 0..r-1 (the old loop order) before the
// atomics.  Requires 64 % r == 0 (r-lane groups inside one wave).
__device__ __forceinline__ void cu_decode(int idx, int h, int w, int r, int& b, int& a, int& y, int& x, int& c) {
  const int wr = w * r;
  const int q = idx % wr;
  int t = idx / wr;
  x = q / r;
  c = q - x * r;
  y = t % h;
  t /= h;
  a = t % r;
  b = t / r;
}

__global__ __launch_bounds__(256) void convex_up_fwd_px_kernel(const float* __restrict__ inv,
                                                               const float* __restrict__ mask, int B,
                                                               int h, int w, int r, float add, float mul,
                                                               float* __restrict__ out) {
  const int hw = h * w;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * r * hw * r) return;
  int b, a, y, x, c;
  cu_decode(idx, h, w, r, b, a, y, x, c);
  const int pix = y * w + x;
  float d[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
    d[k] = (yy >= 0 && yy < h && xx >= 0 && xx < w) ? inv[(size_t)b * hw + yy * w + xx] : 0.f;
  }
  const float* mb = mask + (size_t)b * 9 * r * r * hw + pix;
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
  out[((size_t)b * h * r + (size_t)y * r + a) * (w * r) + (size_t)x * r + c] = __fadd_rn(add, __fmul_rn(mul, acc));
}

__global__ __launch_bounds__(256) void convex_up_bwd_px_kernel(
    const float* __restrict__ inv, const float* __restrict__ mask, const float* __restrict__ gout,
    int B, int h, int w, int r, float mul, float* __restrict__ ginv, float* __restrict__ gmask) {
  const int hw = h * w;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = idx < B * r * hw * r;     // whole r-lane groups are live or not
  int b, a, y, x, c;
  cu_decode(live ? idx : 0, h, w, r, b, a, y, x, c);
  const int pix = y * w + x;
  float d[9], gd[9];
  bool ok[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
    ok[k] = yy >= 0 && yy < h && xx >= 0 && xx < w;
    d[k] = ok[k] ? inv[(size_t)b * hw + yy * w + xx] : 0.f;
  }
  const float* mb = mask + (size_t)b * 9 * r * r * hw + pix;
  const float G = __fmul_rn(gout[((size_t)b * h * r + (size_t)y * r + a) * (w * r) + (size_t)x * r + c], mul);
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
    m[k] = m[k] / s;
    gd[k] = m[k] * G;
    dot += m[k] * (G * d[k]);
  }
  if (live) {
    float* gmb = gmask + (size_t)b * 9 * r * r * hw + pix;
#pragma unroll
    for (int k = 0; k < 9; ++k) gmb[(size_t)(k * r * r + a * r + c) * hw] = m[k] * (G * d[k] - dot);
  }
  if (ginv) {
    const int lane = threadIdx.x & 63, base = lane - c;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      float t = 0.f;
      for (int cc = 0; cc < r; ++cc) t += __shfl(gd[k], base + cc, 64);   // c = 0..r-1 in order
      gd[k] = t;
    }
    if (live && c == 0) {
#pragma unroll
      for (int k = 0; k < 9; ++k)
        if (ok[k]) atomicAdd(ginv + (size_t)b * hw + (y + k / 3 - 1) * w + (x + k % 3 - 1), gd[k]);
    }
  }
}

// Backward with one wave per sub-pixel column c and lanes along 64 consecutive
// low-res pixels: every mask load and mask-gradient store of a wave is one
// contiguous 256-B row segment (the row-along-x mapping above stores 8 x 32 B).
// The r waves of a block are the r columns c of one (b, a, 64-pixel run); the
// inverse-depth tap gradients are summed over c through LDS in the order
// c = 0..r-1 (as the per-(a, y, x) kernel's loop) before the atomics.
// Block = 64 * r threads (r <= 8).
__global__ __launch_bounds__(512) void convex_up_bwd_cw_kernel(
    const float* __restrict__ inv, const float* __restrict__ mask, const float* __restrict__ gout,
    int B, int h, int w, int r, float mul, float* __restrict__ ginv, float* __restrict__ gmask) {
  __shared__ float red[kMaxR][9][64];
  const int hw = h * w;
  const int lane = threadIdx.x & 63, c = threadIdx.x >> 6;
  const int a = blockIdx.y, b = blockIdx.z;
  const int pix = blockIdx.x * 64 + lane;
  const bool live = pix < hw;
  const int pp = live ? pix : 0;
  const int y = pp / w, x = pp - y * w;
  float d[9];
  bool ok[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
    ok[k] = yy >= 0 && yy < h && xx >= 0 && xx < w;
    d[k] = ok[k] ? inv[(size_t)b * hw + yy * w + xx] : 0.f;
  }
  const float* mb = mask + (size_t)b * 9 * r * r * hw + pp;
  const float G = __fmul_rn(gout[((size_t)b * h * r + (size_t)y * r + a) * (w * r) + (size_t)x * r + c], mul);
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
    m[k] = m[k] / s;
    red[c][k][lane] = m[k] * G;
    dot += m[k] * (G * d[k]);
  }
  if (live) {
    float* gmb = gmask + (size_t)b * 9 * r * r * hw + pix;
#pragma unroll
    for (int k = 0; k < 9; ++k) gmb[(size_t)(k * r * r + a * r + c) * hw] = m[k] * (G * d[k] - dot);
  }
  if (ginv) {
    __syncthreads();
    if (c == 0 && live) {
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        float t = 0.f;
        for (int cc = 0; cc < r; ++cc) t += red[cc][k][lane];
        if (ok[k]) atomicAdd(ginv + (size_t)b * hw + (y + k / 3 - 1) * w + (x + k % 3 - 1), t);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// n predictions in one launch each way (every kept prediction of a training
// step: DepthPoseNet.py:180-181 per iteration, stacked by the losses).  The
// forward writes [n, B, 1, hr, wr] directly (the losses' stack is a view).
// The backward is deterministic: one block per (pred, image, 64-pixel run),
// wave c = sub-pixel column, each thread loops over the r sub-pixel rows and
// keeps its 9 tap sums; the waves' sums are added in the order c = 0..r-1
// through LDS and written per (tap, low-res pixel) to a workspace; a second
// launch gathers each low-res pixel's 9 neighbour-tap sums in tap order
// (no atomics, no zero-fill of the inverse-depth gradient).
constexpr int kMaxPred = 32;
struct UpMany {
  const float* inv[kMaxPred];
  const float* mask[kMaxPred];
  float* ginv[kMaxPred];
  float* gmask[kMaxPred];
};
typedef __attribute__((address_space(4))) const char* KArg;
template <typename Tp>
__device__ __forceinline__ Tp up_ptr(size_t field, int i) {   // table entry read from the kernarg segment
  return *(__attribute__((address_space(4))) Tp const*)((KArg)__builtin_amdgcn_kernarg_segment_ptr() + field +
                                                       (size_t)i * sizeof(Tp));
}

__global__ __launch_bounds__(256) void convex_up_many_fwd_kernel(UpMany t, int B, int h, int w, int r, float add,
                                                                float mul, float* __restrict__ out) {
  const int hw = h * w, pred = blockIdx.y;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * r * hw * r) return;
  const float* __restrict__ inv = up_ptr<const float*>(offsetof(UpMany, inv), pred);
  const float* __restrict__ mask = up_ptr<const float*>(offsetof(UpMany, mask), pred);
  int b, a, y, x, c;
  cu_decode(idx, h, w, r, b, a, y, x, c);
  const int pix = y * w + x;
  float d[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
    d[k] = (yy >= 0 && yy < h && xx >= 0 && xx < w) ? inv[(size_t)b * hw + yy * w + xx] : 0.f;
  }
  const float* mb = mask + (size_t)b * 9 * r * r * hw + pix;
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
  out[(size_t)pred * B * hw * r * r + ((size_t)b * h * r + (size_t)y * r + a) * (w * r) + (size_t)x * r + c] =
      __fadd_rn(add, __fmul_rn(mul, acc));
}

// block = 64 * r threads; grid (ceil(hw / 64), B, n); tsum [n][B][9][hw].
// R > 0: the ratio as a compile-time constant (the sub-pixel row loop fully
// unrolled, so every row's mask loads are in flight together); R = 0: runtime r.
template <int R>
__global__ __launch_bounds__(512) void convex_up_many_bwd_kernel(UpMany t, const float* __restrict__ gout, int B,
                                                                int h, int w, int r_, float mul,
                                                                float* __restrict__ tsum) {
  const int r = R > 0 ? R : r_;
  __shared__ float red[kMaxR][9][64];
  const int hw = h * w, pred = blockIdx.z, b = blockIdx.y;
  const int lane = threadIdx.x & 63, c = threadIdx.x >> 6;
  const int pix = blockIdx.x * 64 + lane;
  const bool live = pix < hw;
  const int pp = live ? pix : 0;
  const int y = pp / w, x = pp - y * w;
  const float* __restrict__ inv = up_ptr<const float*>(offsetof(UpMany, inv), pred);
  const float* __restrict__ mask = up_ptr<const float*>(offsetof(UpMany, mask), pred);
  float* __restrict__ gmask = up_ptr<float*>(offsetof(UpMany, gmask), pred);
  const bool want_inv = up_ptr<float*>(offsetof(UpMany, ginv), pred) != nullptr;
  float d[9], tk[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
    d[k] = (yy >= 0 && yy < h && xx >= 0 && xx < w) ? inv[(size_t)b * hw + yy * w + xx] : 0.f;
    tk[k] = 0.f;
  }
  const float* mb = mask + (size_t)b * 9 * r * r * hw + pp;
  float* gmb = gmask + (size_t)b * 9 * r * r * hw + pix;
  const float* gb = gout + (size_t)pred * B * hw * r * r + ((size_t)b * h * r + (size_t)y * r) * (w * r) +
                    (size_t)x * r + c;
#pragma unroll
  for (int a = 0; a < (R > 0 ? R : kMaxR); ++a) {
    if (R == 0 && a >= r) break;
    const float G = __fmul_rn(gb[(size_t)a * (w * r)], mul);
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
      m[k] = m[k] / s;
      tk[k] += m[k] * G;
      dot += m[k] * (G * d[k]);
    }
    if (live) {
#pragma unroll
      for (int k = 0; k < 9; ++k) gmb[(size_t)(k * r * r + a * r + c) * hw] = m[k] * (G * d[k] - dot);
    }
  }
  if (!want_inv) return;   // block-uniform
#pragma unroll
  for (int k = 0; k < 9; ++k) red[c][k][lane] = tk[k];
  __syncthreads();
  if (c == 0 && live) {
    float* ts = tsum + ((size_t)pred * B + b) * 9 * hw + pix;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      float v = 0.f;
      for (int cc = 0; cc < r; ++cc) v += red[cc][k][lane];
      ts[(size_t)k * hw] = v;
    }
  }
}

// ginv[pred][b][q] = sum_k tsum[pred][b][k][q - off(k)], off(k) = (k/3 - 1, k%3 - 1)
__global__ __launch_bounds__(256) void convex_up_many_gather_kernel(UpMany t, const float* __restrict__ tsum, int B,
                                                                   int h, int w) {
  const int hw = h * w, pred = blockIdx.z, b = blockIdx.y;
  const int q = blockIdx.x * 256 + threadIdx.x;
  float* __restrict__ ginv = up_ptr<float*>(offsetof(UpMany, ginv), pred);
  if (q >= hw || ginv == nullptr) return;
  const int qy = q / w, qx = q - qy * w;
  const float* ts = tsum + ((size_t)pred * B + b) * 9 * hw;
  float v = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int py = qy - (k / 3 - 1), px = qx - (k % 3 - 1);
    if (py >= 0 && py < h && px >= 0 && px < w) v += ts[(size_t)k * hw + py * w + px];
  }
  ginv[(size_t)b * hw + q] = v;
}

// ---------------------------------------------------------------------------
// Bilinear 2x upsampling (align_corners=False) of the feature/context trunks:
// F.interpolate(x, scale_factor=2, mode="bilinear") in networks/optim/
// extractor.py:91-97 of the reference.  ATen's kernel runs one thread per
// output pixel looping over all N*C planes (~325 us at [6,256,12,40]); here
// one thread per output element (forward) and, for the backward, one thread
// per input element gathering its <= 4x4 output taps in a fixed order (no
// atomics, deterministic).  Source index as ATen: max(0.5*(dst+0.5)-0.5, 0).
// HBM bound: 4 bytes read + 16 written per input element (forward).
__device__ __forceinline__ void bl2_src(int dst, int n, int& i0, int& i1, float& l1) {
  float s = 0.5f * ((float)dst + 0.5f) - 0.5f;
  s = s < 0.f ? 0.f : s;
  i0 = (int)s;
  i1 = i0 + (i0 < n - 1 ? 1 : 0);
  l1 = s - (float)i0;
}

// grid (pixel blocks, planes): 32-bit in-plane arithmetic (64-bit division by
// runtime sizes dominated these launches)
__global__ __launch_bounds__(256) void bilinear2x_fwd_kernel(const float* __restrict__ x, int h, int w,
                                                            float* __restrict__ out) {
  const int H = 2 * h, W = 2 * w;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= H * W) return;
  const int Y = i / W, X = i - Y * W;
  const size_t pl = blockIdx.y;
  int y0, y1, x0, x1;
  float ly, lx;
  bl2_src(Y, h, y0, y1, ly);
  bl2_src(X, w, x0, x1, lx);
  const float* p = x + pl * h * w;
  const float a = p[y0 * w + x0], b = p[y0 * w + x1], c = p[y1 * w + x0], d = p[y1 * w + x1];
  out[pl * H * W + i] = (1.f - ly) * ((1.f - lx) * a + lx * b) + ly * ((1.f - lx) * c + lx * d);
}

// weight of input index i in the taps of output index dst
__device__ __forceinline__ float bl2_weight(int dst, int n, int i) {
  int i0, i1;
  float l1;
  bl2_src(dst, n, i0, i1, l1);
  return (i0 == i ? 1.f - l1 : 0.f) + (i1 == i ? l1 : 0.f);
}

__global__ __launch_bounds__(256) void bilinear2x_bwd_kernel(const float* __restrict__ gout, int h, int w,
                                                            float* __restrict__ gx) {
  const int H = 2 * h, W = 2 * w;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= h * w) return;
  const int yi = i / w, xi = i - yi * w;
  const size_t pl = blockIdx.y;
  const float* g = gout + pl * H * W;
  float wx[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int X = 2 * xi - 1 + j;
    wx[j] = (X >= 0 && X < W) ? bl2_weight(X, w, xi) : 0.f;
  }
  float acc = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int Y = 2 * yi - 1 + r;
    if (Y < 0 || Y >= H) continue;
    const float wy = bl2_weight(Y, h, yi);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int X = 2 * xi - 1 + j;
      if (wx[j] != 0.f) q += wx[j] * g[Y * W + X];
    }
    acc += wy * q;
  }
  gx[pl * h * w + i] = acc;
}

}  // namespace dro

using namespace dro;

static int up_check(const float* inv, const float* mask, int B, int h, int w, int ratio) {
  if (!inv || !mask) {
    set_error("convex_upsample: NULL input");
    return DRO_E_NULL;
  }
  if (B < 1 || h < 1 || w < 1 || ratio < 1 || ratio > kMaxR || (long long)B * ratio * ratio * h * w >= (1LL << 31)) {
    set_error("convex_upsample: sizes out of range (ratio 1..8)");
    return DRO_E_SHAPE;
  }
  return DRO_OK;
}

extern "C" int dro_convex_upsample_forward(const float* inv, const float* mask, int B, int h, int w,
                                           int ratio, float add, float mul, float* out, void* stream) {
  int st = up_check(inv, mask, B, h, w, ratio);
  if (st) return st;
  if (!out) {
    set_error("convex_upsample_forward: NULL out");
    return DRO_E_NULL;
  }
  const int total = B * ratio * h * w;
  if (64 % ratio == 0) {
    hipLaunchKernelGGL(convex_up_fwd_px_kernel, dim3((total * ratio + 255) / 256), dim3(256), 0,
                       (hipStream_t)stream, inv, mask, B, h, w, ratio, add, mul, out);
    return launch_status("convex_up_fwd_px_kernel launch failed");
  }
  hipLaunchKernelGGL(convex_up_fwd_kernel, dim3((total + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, inv, mask, B, h, w, ratio, add, mul, out);
  return launch_status("convex_up_fwd_kernel launch failed");
}

extern "C" int dro_convex_upsample_backward(const float* inv, const float* mask,
                                            const float* grad_out, int B, int h, int w, int ratio,
                                            float mul, float* grad_inv, float* grad_mask, void* stream) {
  int st = up_check(inv, mask, B, h, w, ratio);
  if (st) return st;
  if (!grad_out || !grad_mask) {
    set_error("convex_upsample_backward: NULL grad_out/grad_mask");
    return DRO_E_NULL;
  }
  hipStream_t s = (hipStream_t)stream;
  if (grad_inv && (st = launch_zero(grad_inv, (size_t)B * h * w, s))) return st;
  const int total = B * ratio * h * w;
  if (B <= 65535) {
    hipLaunchKernelGGL(convex_up_bwd_cw_kernel, dim3((h * w + 63) / 64, ratio, B), dim3(64 * ratio), 0, s, inv,
                       mask, grad_out, B, h, w, ratio, mul, grad_inv, grad_mask);
    return launch_status("convex_up_bwd_cw_kernel launch failed");
  }
  if (64 % ratio == 0) {
    hipLaunchKernelGGL(convex_up_bwd_px_kernel, dim3((total * ratio + 255) / 256), dim3(256), 0, s, inv, mask,
                       grad_out, B, h, w, ratio, mul, grad_inv, grad_mask);
    return launch_status("convex_up_bwd_px_kernel launch failed");
  }
  hipLaunchKernelGGL(convex_up_bwd_kernel, dim3((total + 255) / 256), dim3(256), 0, s, inv, mask,
                     grad_out, B, h, w, ratio, mul, grad_inv, grad_mask);
  return launch_status("convex_up_bwd_kernel launch failed");
}

static int up_many_check(const float* const* inv, const float* const* mask, int n, int B, int h, int w,
                         int ratio, UpMany& t) {
  if (!inv || !mask) {
    set_error("convex_upsample_many: NULL pointer table");
    return DRO_E_NULL;
  }
  if (n < 1 || n > kMaxPred) {
    set_error("convex_upsample_many: 1..32 predictions per call");
    return DRO_E_SHAPE;
  }
  for (int i = 0; i < n; ++i) {
    int st = up_check(inv[i], mask[i], B, h, w, ratio);
    if (st) return st;
    if ((long long)n * B * ratio * ratio * h * w >= (1LL << 31)) {
      set_error("convex_upsample_many: output of >= 2^31 elements");
      return DRO_E_SHAPE;
    }
    t.inv[i] = inv[i];
    t.mask[i] = mask[i];
  }
  return DRO_OK;
}

extern "C" int dro_convex_upsample_many_forward(const float* const* inv, const float* const* mask, int n, int B,
                                                int h, int w, int ratio, float add, float mul, float* out,
                                                void* stream) {
  UpMany t = {};
  int st = up_many_check(inv, mask, n, B, h, w, ratio, t);
  if (st) return st;
  if (!out) {
    set_error("convex_upsample_many_forward: NULL out");
    return DRO_E_NULL;
  }
  const int total = B * ratio * h * w * ratio;
  hipLaunchKernelGGL(convex_up_many_fwd_kernel, dim3((total + 255) / 256, n), dim3(256), 0, (hipStream_t)stream, t,
                     B, h, w, ratio, add, mul, out);
  return launch_status("convex_up_many_fwd_kernel launch failed");
}

extern "C" size_t dro_convex_upsample_many_workspace_bytes(int n, int B, int h, int w) {
  if (n < 1 || B < 1 || h < 1 || w < 1) return 0;
  return (size_t)n * B * 9 * h * w * sizeof(float);
}

extern "C" int dro_convex_upsample_many_backward(const float* const* inv, const float* const* mask,
                                                 const float* grad_out, int n, int B, int h, int w, int ratio,
                                                 float mul, float* const* grad_inv, float* const* grad_mask,
                                                 void* workspace, size_t workspace_bytes, void* stream) {
  UpMany t = {};
  int st = up_many_check(inv, mask, n, B, h, w, ratio, t);
  if (st) return st;
  if (!grad_out || !grad_mask || B > 65535) {
    set_error("convex_upsample_many_backward: NULL grad_out/grad_mask table, or B > 65535");
    return DRO_E_NULL;
  }
  bool any_inv = false;
  for (int i = 0; i < n; ++i) {
    if (!grad_mask[i]) {
      set_error("convex_upsample_many_backward: NULL grad_mask entry");
      return DRO_E_NULL;
    }
    t.gmask[i] = grad_mask[i];
    t.ginv[i] = grad_inv ? grad_inv[i] : nullptr;
    any_inv |= t.ginv[i] != nullptr;
  }
  if (any_inv && (!workspace || workspace_bytes < dro_convex_upsample_many_workspace_bytes(n, B, h, w))) {
    set_error("convex_upsample_many_backward: workspace too small (dro_convex_upsample_many_workspace_bytes)");
    return DRO_E_SHAPE;
  }
  hipStream_t s = (hipStream_t)stream;
  float* tsum = static_cast<float*>(workspace);
  if (ratio == 8)
    hipLaunchKernelGGL(convex_up_many_bwd_kernel<8>, dim3((h * w + 63) / 64, B, n), dim3(64 * ratio), 0, s, t,
                       grad_out, B, h, w, ratio, mul, tsum);
  else
    hipLaunchKernelGGL(convex_up_many_bwd_kernel<0>, dim3((h * w + 63) / 64, B, n), dim3(64 * ratio), 0, s, t,
                       grad_out, B, h, w, ratio, mul, tsum);
  if ((st = launch_status("convex_up_many_bwd_kernel launch failed"))) return st;
  if (!any_inv) return DRO_OK;
  hipLaunchKernelGGL(convex_up_many_gather_kernel, dim3((h * w + 255) / 256, B, n), dim3(256), 0, s, t, tsum, B, h,
                     w);
  return launch_status("convex_up_many_gather_kernel launch failed");
}

static int bl2_check(const float* a, const float* b, long long planes, int h, int w) {
  if (!a || !b) {
    set_error("bilinear_upsample2x: NULL pointer");
    return DRO_E_NULL;
  }
  if (planes < 1 || planes >= (1LL << 40) || h < 1 || w < 1 || 4LL * h * w >= (1LL << 30)) {
    set_error("bilinear_upsample2x: sizes out of range");
    return DRO_E_SHAPE;
  }
  return DRO_OK;
}

extern "C" int dro_bilinear_upsample2x_forward(const float* x, long long planes, int h, int w,
                                               float* out, void* stream) {
  int st = bl2_check(x, out, planes, h, w);
  if (st) return st;
  // planes ride grid.y (<= 65535 per launch): larger batches go in chunks
  for (long long p0 = 0; p0 < planes; p0 += 65535) {
    const long long np = planes - p0 < 65535 ? planes - p0 : 65535;
    hipLaunchKernelGGL(bilinear2x_fwd_kernel, dim3((4 * h * w + 255) / 256, (unsigned)np), dim3(256), 0,
                       (hipStream_t)stream, x + p0 * h * w, h, w, out + p0 * 4 * h * w);
    if ((st = launch_status("bilinear2x_fwd_kernel launch failed"))) return st;
  }
  return DRO_OK;
}

extern "C" int dro_bilinear_upsample2x_backward(const float* grad_out, long long planes, int h,
                                                int w, float* grad_x, void* stream) {
  int st = bl2_check(grad_out, grad_x, planes, h, w);
  if (st) return st;
  for (long long p0 = 0; p0 < planes; p0 += 65535) {
    const long long np = planes - p0 < 65535 ? planes - p0 : 65535;
    hipLaunchKernelGGL(bilinear2x_bwd_kernel, dim3((h * w + 255) / 256, (unsigned)np), dim3(256), 0,
                       (hipStream_t)stream, grad_out + p0 * 4 * h * w, h, w, grad_x + p0 * h * w);
    if ((st = launch_status("bilinear2x_bwd_kernel launch failed"))) return st;
  }
  return DRO_OK;
}
