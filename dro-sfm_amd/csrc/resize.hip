// GPU-side image resize + to-tensor of the training data pipeline.
//
// Replaces, for decoded uint8 RGB frames, torchvision Resize((H, W),
// BILINEAR) on PIL images followed by ToTensor
// (dro_sfm/datasets/augmentations.py:69-111 resize_sample_image_and_intrinsics,
// :149-160 to_tensor): PIL's separable resampling (Pillow Resample.c,
// "bilinear" = triangle filter widened by the downscale factor) with its
// 8-bit fixed-point coefficients (22 fractional bits, round-half-up, clip),
// horizontal pass first with a uint8 intermediate exactly as Pillow does, then
// the vertical pass fused with ToTensor (value / 255 as float32, HWC -> CHW).
// Bit-identical to Pillow (tests/test_resize.py checks against PIL itself).
// The per-output-column / -row coefficient tables are built on the host
// (dro_sfm_amd/datasets/gpu_transforms.py) once per (input, output) size.
// Roofline: HBM bound.  Algorithmic bytes per frame: 3*H0*W0 read + 3*H0*W
// (intermediate, written and read) + 12*H*W written.
#include <hip/hip_runtime.h>

#include "dro_common.hpp"

namespace dro {

constexpr int kRsThreads = 256;
constexpr int kPrec = 22;

__device__ __forceinline__ unsigned char clip8(long long ss) {
  const long long v = ss >> kPrec;
  return (unsigned char)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// tmp[n, y, x, c] = sum_k xk[x][k] * src[n, y, xmin(x) + k, c]   (uint8 HWC)
__global__ __launch_bounds__(kRsThreads) void resize_h_kernel(const unsigned char* __restrict__ src, int N,
                                                             int H0, int W0, int W,
                                                             const int* __restrict__ xb,
                                                             const int* __restrict__ xk, int KX,
                                                             unsigned char* __restrict__ tmp) {
  const long long i = (long long)blockIdx.x * kRsThreads + threadIdx.x;
  if (i >= (long long)N * H0 * W) return;
  const int x = (int)(i % W);
  const long long ny = i / W;   // n * H0 + y
  const int xmin = xb[2 * x], cnt = xb[2 * x + 1];
  const unsigned char* row = src + (ny * W0 + xmin) * 3;
  long long s0 = 1LL << (kPrec - 1), s1 = s0, s2 = s0;
  for (int k = 0; k < cnt; ++k) {
    const long long w = xk[x * KX + k];
    s0 += w * row[3 * k + 0];
    s1 += w * row[3 * k + 1];
    s2 += w * row[3 * k + 2];
  }
  unsigned char* o = tmp + i * 3;
  o[0] = clip8(s0);
  o[1] = clip8(s1);
  o[2] = clip8(s2);
}

// dst[n, c, y, x] = clip8(sum_k yk[y][k] * tmp[n, ymin(y) + k, x, c]) / 255
__global__ __launch_bounds__(kRsThreads) void resize_v_kernel(const unsigned char* __restrict__ tmp, int N,
                                                             int H0, int H, int W,
                                                             const int* __restrict__ yb,
                                                             const int* __restrict__ yk, int KY,
                                                             float* __restrict__ dst) {
  const long long i = (long long)blockIdx.x * kRsThreads + threadIdx.x;
  if (i >= (long long)N * H * W) return;
  const int x = (int)(i % W);
  const long long t = i / W;
  const int y = (int)(t % H);
  const long long n = t / H;
  const int ymin = yb[2 * y], cnt = yb[2 * y + 1];
  const unsigned char* col = tmp + ((n * H0 + ymin) * (long long)W + x) * 3;
  const long long stride = (long long)W * 3;
  long long s0 = 1LL << (kPrec - 1), s1 = s0, s2 = s0;
  for (int k = 0; k < cnt; ++k) {
    const long long w = yk[y * KY + k];
    const unsigned char* p = col + k * stride;
    s0 += w * p[0];
    s1 += w * p[1];
    s2 += w * p[2];
  }
  const size_t HWo = (size_t)H * W, pix = (size_t)y * W + x;
  float* o = dst + (size_t)n * 3 * HWo + pix;
  o[0] = (float)clip8(s0) / 255.f;
  o[HWo] = (float)clip8(s1) / 255.f;
  o[2 * HWo] = (float)clip8(s2) / 255.f;
}

}  // namespace dro

using namespace dro;

extern "C" int dro_resize_rgb8_to_tensor(const unsigned char* src, int N, int H0, int W0, int H, int W,
                                         const int* xbounds, const int* xcoef, int KX, const int* ybounds,
                                         const int* ycoef, int KY, unsigned char* tmp, float* dst,
                                         void* stream) {
  if (!src || !xbounds || !xcoef || !ybounds || !ycoef || !tmp || !dst) {
    set_error("resize_rgb8_to_tensor: NULL pointer");
    return DRO_E_NULL;
  }
  if (N < 1 || H0 < 1 || W0 < 1 || H < 1 || W < 1 || KX < 1 || KY < 1 ||
      (long long)N * H0 * (W > W0 ? W : W0) * 3 >= (1LL << 40) || (long long)N * H * W * 3 >= (1LL << 40)) {
    set_error("resize_rgb8_to_tensor: sizes out of range");
    return DRO_E_SHAPE;
  }
  hipStream_t s = (hipStream_t)stream;
  const long long nh = (long long)N * H0 * W;
  hipLaunchKernelGGL(resize_h_kernel, dim3((unsigned)((nh + kRsThreads - 1) / kRsThreads)), dim3(kRsThreads), 0,
                     s, src, N, H0, W0, W, xbounds, xcoef, KX, tmp);
  int st = launch_status("resize_h_kernel launch failed");
  if (st) return st;
  const long long nv = (long long)N * H * W;
  hipLaunchKernelGGL(resize_v_kernel, dim3((unsigned)((nv + kRsThreads - 1) / kRsThreads)), dim3(kRsThreads), 0,
                     s, tmp, N, H0, H, W, ybounds, ycoef, KY, dst);
  return launch_status("resize_v_kernel launch failed");
}
