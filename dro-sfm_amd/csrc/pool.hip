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
//   backward : one thread per input pixel gathers the (at most 2 x 2) windows
//              that contain it, in ATen's (ph, pw) ascending order, so the
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

__global__ __launch_bounds__(kPoolThreads) void maxpool3s2_bwd_kernel(const float* __restrict__ gy,
                                                                     const unsigned char* __restrict__ idx,
                                                                     int H, int W, int Ho, int Wo,
                                                                     float* __restrict__ gx) {
  const int i = blockIdx.x * kPoolThreads + threadIdx.x;
  if (i >= H * W) return;
  const int yy = i / W, xx = i - yy * W;
  const size_t pl = blockIdx.y;
  // windows oy with 2*oy-1 <= yy <= 2*oy+1 (ATen p_start / p_end for k3 s2 p1)
  const int ph0 = (yy + 1 < 3) ? 0 : (yy + 1 - 3) / 2 + 1, ph1 = min((yy + 1) / 2 + 1, Ho);
  const int pw0 = (xx + 1 < 3) ? 0 : (xx + 1 - 3) / 2 + 1, pw1 = min((xx + 1) / 2 + 1, Wo);
  const float* __restrict__ g = gy + pl * Ho * Wo;
  const unsigned char* __restrict__ id = idx + pl * Ho * Wo;
  float acc = 0.f;
  for (int ph = ph0; ph < ph1; ++ph)
    for (int pw = pw0; pw < pw1; ++pw) {
      const int code = (yy - 2 * ph + 1) * 3 + (xx - 2 * pw + 1);
      const int k = ph * Wo + pw;
      if (id[k] == code) acc += g[k];
    }
  gx[pl * H * W + i] = acc;
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
    hipLaunchKernelGGL(maxpool3s2_bwd_kernel, dim3((H * W + kPoolThreads - 1) / kPoolThreads, (unsigned)np),
                       dim3(kPoolThreads), 0, (hipStream_t)stream, grad_y + p0 * Ho * Wo, argmax + p0 * Ho * Wo,
                       H, W, Ho, Wo, grad_x + p0 * H * W);
    if ((st = launch_status("maxpool3s2_bwd_kernel launch failed"))) return st;
  }
  return DRO_OK;
}
