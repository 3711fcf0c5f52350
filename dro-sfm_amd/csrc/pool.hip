// 3x3 / stride 2 / pad 1 max pooling of the ResNet-18 stem (fwd + bwd).
//
// Replaces F.max_pool2d(x, 3, 2, 1) after conv1/bn1/relu in ResNetEncoder
// (dro_sfm/networks/optim/extractor.py:60-66 of the reference, torchvision's
// ResNet stem).  ATen's NCHW kernels took 20 us forward and 55 us backward per
// call at the fnet shape (6 x 64 x 96 x 320): the backward recomputes window
// bounds per input pixel and reads int64 indices.  Here:
//   forward  : one thread per output pixel, max over the clipped window in
//              ATen's scan order (rows, then columns; `v > max || isnan(v)`),
//              argmax kept as one byte per output (dy * 3 + dx);
//   backward : one thread per 2 x 2 input block reads the (at most 2 x 2)
//              windows that cover it once for its 4 pixels (round 4; was one
//              thread per input pixel, 60 us per fnet call) and sums each
//              pixel's matches in ATen's (ph, pw) ascending order, so the
//              float sums are bit-identical to max_pool2d's backward.
// Roofline: HBM bound.  Algorithmic bytes per plane: forward 4*H*W read +
// 5*Ho*Wo written; backward 5*Ho*Wo read + 4*H*W written.
#include <hip/hip_runtime.h>
#include <math.h>

#include "dro_common.hpp"

namespace dro {

constexpr int kPoolThreads = 256;

// grid (pixel blocks, planes): 32-bit pixel arithmetic inside a plane (64-bit
// division/modulo by runtime sizes costs more than the memory traffic here)
__global__ __launch_bounds__(kPoolThreads) void maxpool3s2_fwd_kernel(const float* __restrict__ x, int H, int W,
                                                                     int Ho, int Wo,
                                                                     float* __restrict__ y,
                                                                     unsigned char* __restrict__ idx) {
  const int o = blockIdx.x * kPoolThreads + threadIdx.x;
  if (o >= Ho * Wo) return;
  const int oy = o / Wo, ox = o - oy * Wo;
  const size_t pl = blockIdx.y;
  const float* __restrict__ p = x + pl * H * W;
  const int y0 = 2 * oy - 1, x0 = 2 * ox - 1;
  float m = -INFINITY;
  int arg = -1;
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const int yy = y0 + dy;
    if (yy < 0 || yy >= H) continue;
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int xx = x0 + dx;
      if (xx < 0 || xx >= W) continue;
      const float v = p[yy * W + xx];
      if (arg < 0) arg = dy * 3 + dx;   // ATen's initial index: the first in-range tap
      if (v > m || isnan(v)) {
        m = v;
        arg = dy * 3 + dx;
      }
    }
  }
  y[pl * Ho * Wo + o] = m;
  idx[pl * Ho * Wo + o] = (unsigned char)arg;
}

// One thread per 2x2 input block {2k, 2k+1} x {2m, 2m+1}: the (at most) four
// windows (k|k+1, m|m+1) that cover it are read once (4 gradients + 4 argmax
// bytes) for its 4 pixels, instead of once per covering pixel; each pixel
// sums its matching windows in ATen's order (row of windows ascending, then
// column) -- bit-identical to F.max_pool2d's backward.  Window codes: the
// pixel's offset from the window start (2 oy - 1, 2 ox - 1) as dy * 3 + dx.
__global__ __launch_bounds__(kPoolThreads) void maxpool3s2_bwd_quad_kernel(const float* __restrict__ gy,
                                                                          const unsigned char* __restrict__ idx,
                                                                          int H, int W, int Ho, int Wo, int Wq,
                                                                          int nq, float* __restrict__ gx) {
  const int t = blockIdx.x * kPoolThreads + threadIdx.x;
  if (t >= nq) return;
  const int k = t / Wq, m = t - k * Wq;
  const size_t pl = blockIdx.y;
  const float* __restrict__ g = gy + pl * Ho * Wo;
  const unsigned char* __restrict__ id = idx + pl * Ho * Wo;
  const bool r1 = k + 1 < Ho, c1 = m + 1 < Wo;          // windows (k+1, .) and (., m+1) exist
  const int w00 = k * Wo + m;
  const float g00 = g[w00];
  const float g01 = c1 ? g[w00 + 1] : 0.f;
  const float g10 = r1 ? g[w00 + Wo] : 0.f;
  const float g11 = (r1 && c1) ? g[w00 + Wo + 1] : 0.f;
  const int i00 = id[w00];
  const int i01 = c1 ? id[w00 + 1] : -1;
  const int i10 = r1 ? id[w00 + Wo] : -1;
  const int i11 = (r1 && c1) ? id[w00 + Wo + 1] : -1;
  float* __restrict__ out = gx + pl * H * W;
  const int y = 2 * k, x = 2 * m;
  {   // (2k, 2m): window (k, m), code 4
    float a = 0.f;
    if (i00 == 4) a += g00;
    out[y * W + x] = a;
  }
  if (x + 1 < W) {   // (2k, 2m+1): (k, m) code 5, (k, m+1) code 3
    float a = 0.f;
    if (i00 == 5) a += g00;
    if (i01 == 3) a += g01;
    out[y * W + x + 1] = a;
  }
  if (y + 1 < H) {
    {   // (2k+1, 2m): (k, m) code 7, (k+1, m) code 1
      float a = 0.f;
      if (i00 == 7) a += g00;
      if (i10 == 1) a += g10;
      out[(y + 1) * W + x] = a;
    }
    if (x + 1 < W) {   // (2k+1, 2m+1): (k, m) 8, (k, m+1) 6, (k+1, m) 2, (k+1, m+1) 0
      float a = 0.f;
      if (i00 == 8) a += g00;
      if (i01 == 6) a += g01;
      if (i10 == 2) a += g10;
      if (i11 == 0) a += g11;
      out[(y + 1) * W + x + 1] = a;
    }
  }
}

}  // namespace dro

using namespace dro;

static int pool_check(const void* a, const void* b, const void* c, long long planes, int H, int W) {
  if (!a || !b || !c) {
    set_error("maxpool3x3s2: NULL pointer");
    return DRO_E_NULL;
  }
  if (planes < 1 || planes >= (1LL << 40) || H < 1 || W < 1 || (long long)H * W >= (1LL << 30)) {
    set_error("maxpool3x3s2: sizes out of range");
    return DRO_E_SHAPE;
  }
  return DRO_OK;
}

extern "C" int dro_maxpool3x3s2_forward(const float* x, long long planes, int H, int W, float* y,
                                        unsigned char* argmax, void* stream) {
  int st = pool_check(x, y, argmax, planes, H, W);
  if (st) return st;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  // planes ride grid.y (<= 65535 per launch): larger batches go in chunks
  for (long long p0 = 0; p0 < planes; p0 += 65535) {
    const long long np = planes - p0 < 65535 ? planes - p0 : 65535;
    hipLaunchKernelGGL(maxpool3s2_fwd_kernel, dim3((Ho * Wo + kPoolThreads - 1) / kPoolThreads, (unsigned)np),
                       dim3(kPoolThreads), 0, (hipStream_t)stream, x + p0 * H * W, H, W, Ho, Wo,
                       y + p0 * Ho * Wo, argmax + p0 * Ho * Wo);
    if ((st = launch_status("maxpool3s2_fwd_kernel launch failed"))) return st;
  }
  return DRO_OK;
}

extern "C" int dro_maxpool3x3s2_backward(const float* grad_y, const unsigned char* argmax,
                                         long long planes, int H, int W, float* grad_x,
                                         void* stream) {
  int st = pool_check(grad_y, argmax, grad_x, planes, H, W);
  if (st) return st;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  for (long long p0 = 0; p0 < planes; p0 += 65535) {
    const long long np = planes - p0 < 65535 ? planes - p0 : 65535;
    // 2x2 input blocks: (H+1)/2 x (W+1)/2 of them, each inside the window grid
    const int Hq = (H + 1) / 2, Wq = (W + 1) / 2, nq = Hq * Wq;
    hipLaunchKernelGGL(maxpool3s2_bwd_quad_kernel, dim3((nq + kPoolThreads - 1) / kPoolThreads, (unsigned)np),
                       dim3(kPoolThreads), 0, (hipStream_t)stream, grad_y + p0 * Ho * Wo, argmax + p0 * Ho * Wo,
                       H, W, Ho, Wo, Wq, nq, grad_x + p0 * H * W);
    if ((st = launch_status("maxpool3s2_bwd_quad_kernel launch failed"))) return st;
  }
  return DRO_OK;
}
