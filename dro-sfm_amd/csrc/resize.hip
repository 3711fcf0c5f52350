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
#include <math.h>

#include "dro_common.hpp"

// Pillow's 8-bit colour arithmetic is separate IEEE multiplies and adds (an
// x86-64 baseline build: no FMA); contraction would change truncated results.
#pragma clang fp contract(off)

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

// vertical pass into uint8 HWC (the resized PIL image, before jitter)
__global__ __launch_bounds__(kRsThreads) void resize_v_u8_kernel(const unsigned char* __restrict__ tmp, int N,
                                                                int H0, int H, int W,
                                                                const int* __restrict__ yb,
                                                                const int* __restrict__ yk, int KY,
                                                                unsigned char* __restrict__ dst) {
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
  unsigned char* o = dst + i * 3;
  o[0] = clip8(s0);
  o[1] = clip8(s1);
  o[2] = clip8(s2);
}

// ToTensor: uint8 HWC -> float CHW / 255
__global__ __launch_bounds__(kRsThreads) void rgb8_to_tensor_kernel(const unsigned char* __restrict__ src, int HW,
                                                                   float* __restrict__ dst) {
  const int p = blockIdx.x * kRsThreads + threadIdx.x;
  if (p >= HW) return;
  const size_t n = blockIdx.y;
  const unsigned char* s = src + (n * HW + p) * 3;
  float* o = dst + n * 3 * HW + p;
  o[0] = (float)s[0] / 255.f;
  o[HW] = (float)s[1] / 255.f;
  o[2 * (size_t)HW] = (float)s[2] / 255.f;
}

// ------------------------------------------------------------------ colour jitter
// torchvision ColorJitter over PIL images (datasets/augmentations.py:213-258 of
// the reference): per frame a random order of brightness / contrast /
// saturation / hue with random factors (sampled on the host exactly as
// torchvision's get_params).  Pillow semantics, verified exhaustively on the
// CPU (oracle/dro_oracle.py):
//   blend(d, x, f) = (uint8) trunc(float(d) + f * float(x - d)), clipped to
//     [0, 255] when f is outside [0, 1] (Image.blend);
//   brightness: d = 0;  contrast: d = int(mean(L) + 0.5) of the current frame;
//   saturation: d = L = (19595 R + 38470 G + 7471 B + 2^15) >> 16 per pixel;
//   hue: Pillow RGB -> HSV (float, with double intermediates), h += delta
//     (uint8 wrap), HSV -> RGB.
// A frame's ops before its contrast step run in the first pass, which also
// sums L of the result (64-bit integer atomics: exact); the second pass
// applies the contrast blend and the ops after it.
struct JitterFrame {
  int order[4];     // op ids (0 brightness, 1 contrast, 2 saturation, 3 hue) in application order
  float factor[3];  // brightness, contrast, saturation
  int hue_delta;    // uint8 added to H (mod 256)
};

__device__ __forceinline__ unsigned char pil_blend(int d, int x, float f) {
  const float v = __fadd_rn((float)d, __fmul_rn(f, (float)(x - d)));
  if (f >= 0.f && f <= 1.f) return (unsigned char)(int)v;
  if (v <= 0.f) return 0;
  if (v >= 255.f) return 255;
  return (unsigned char)(int)v;
}

__device__ __forceinline__ int pil_luma(int r, int g, int b) {
  return (r * 19595 + g * 38470 + b * 7471 + 0x8000) >> 16;
}

__device__ __forceinline__ void pil_rgb2hsv(int r, int g, int b, int& H, int& S, int& V) {
  const int maxc = max(r, max(g, b)), minc = min(r, min(g, b));
  V = maxc;
  if (minc == maxc) {
    H = 0;
    S = 0;
    return;
  }
  const float cr = (float)(maxc - minc);
  const float s = cr / (float)maxc;
  const float rc = (float)(maxc - r) / cr, gc = (float)(maxc - g) / cr, bc = (float)(maxc - b) / cr;
  float h;
  if (r == maxc) h = bc - gc;
  else if (g == maxc) h = (float)(2.0 + (double)rc - (double)bc);
  else h = (float)(4.0 + (double)gc - (double)rc);
  h = (float)fmod((double)h / 6.0 + 1.0, 1.0);
  H = min(max((int)((double)h * 255.0), 0), 255);
  S = min(max((int)((double)s * 255.0), 0), 255);
}

__device__ __forceinline__ void pil_hsv2rgb(int h, int s, int v, int& r, int& g, int& b) {
  if (s == 0) {
    r = g = b = v;
    return;
  }
  const double hd = (double)(float)h * 6.0 / 255.0;
  const int i = (int)floor(hd);
  const float f = (float)(hd - (double)(float)i);
  const float fs = (float)((double)(float)s / 255.0);
  const double vf = (double)(float)v;
  const int p = (int)rint(vf * (1.0 - (double)fs));
  const int q = (int)rint(vf * (1.0 - (double)__fmul_rn(fs, f)));
  const int t = (int)rint(vf * (1.0 - (double)__fmul_rn(fs, __fsub_rn(1.f, f))));
  const int up = min(max(p, 0), 255), uq = min(max(q, 0), 255), ut = min(max(t, 0), 255);
  switch (i % 6) {
    case 0: r = v; g = ut; b = up; break;
    case 1: r = uq; g = v; b = up; break;
    case 2: r = up; g = v; b = ut; break;
    case 3: r = up; g = uq; b = v; break;
    case 4: r = ut; g = up; b = v; break;
    default: r = v; g = up; b = uq; break;
  }
}

__device__ __forceinline__ void jitter_op(const JitterFrame& fr, int op, int mean, int& r, int& g, int& b) {
  if (op == 0) {
    const float f = fr.factor[0];
    r = pil_blend(0, r, f);
    g = pil_blend(0, g, f);
    b = pil_blend(0, b, f);
  } else if (op == 1) {
    const float f = fr.factor[1];
    r = pil_blend(mean, r, f);
    g = pil_blend(mean, g, f);
    b = pil_blend(mean, b, f);
  } else if (op == 2) {
    const float f = fr.factor[2];
    const int L = pil_luma(r, g, b);
    r = pil_blend(L, r, f);
    g = pil_blend(L, g, f);
    b = pil_blend(L, b, f);
  } else {
    int H, S, V;
    pil_rgb2hsv(r, g, b, H, S, V);
    pil_hsv2rgb((H + fr.hue_delta) & 255, S, V, r, g, b);
  }
}

// pass 1: ops before contrast; lsum[n] += sum of L over the frame
__global__ __launch_bounds__(kRsThreads) void jitter_pre_kernel(unsigned char* __restrict__ img, int HW,
                                                               const JitterFrame* __restrict__ frames,
                                                               unsigned long long* __restrict__ lsum) {
  __shared__ unsigned long long wsum[kRsThreads / 64];
  const int p = blockIdx.x * kRsThreads + threadIdx.x;
  const int n = blockIdx.y;
  const JitterFrame fr = frames[n];
  unsigned long long l = 0;
  if (p < HW) {
    unsigned char* px = img + ((size_t)n * HW + p) * 3;
    int r = px[0], g = px[1], b = px[2];
    for (int k = 0; k < 4 && fr.order[k] != 1; ++k) jitter_op(fr, fr.order[k], 0, r, g, b);
    px[0] = (unsigned char)r;
    px[1] = (unsigned char)g;
    px[2] = (unsigned char)b;
    l = (unsigned long long)pil_luma(r, g, b);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) l += __shfl_xor(l, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = l;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int i = 0; i < kRsThreads / 64; ++i) t += wsum[i];
    atomicAdd(lsum + n, t);   // integer: exact in any order
  }
}

// pass 2: contrast (Pillow: int(mean + 0.5) of the L image) and the ops after it
__global__ __launch_bounds__(kRsThreads) void jitter_post_kernel(unsigned char* __restrict__ img, int HW,
                                                                const JitterFrame* __restrict__ frames,
                                                                const unsigned long long* __restrict__ lsum) {
  const int p = blockIdx.x * kRsThreads + threadIdx.x;
  if (p >= HW) return;
  const int n = blockIdx.y;
  const JitterFrame fr = frames[n];
  const int mean = (int)((double)lsum[n] / (double)HW + 0.5);
  unsigned char* px = img + ((size_t)n * HW + p) * 3;
  int r = px[0], g = px[1], b = px[2];
  int k = 0;
  while (k < 4 && fr.order[k] != 1) ++k;
  for (; k < 4; ++k) jitter_op(fr, fr.order[k], mean, r, g, b);
  px[0] = (unsigned char)r;
  px[1] = (unsigned char)g;
  px[2] = (unsigned char)b;
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

extern "C" int dro_color_jitter_rgb8(unsigned char* frames, int N, int H, int W, const int* params,
                                     unsigned long long* workspace, void* stream) {
  if (!frames || !params || !workspace) {
    set_error("color_jitter_rgb8: NULL pointer");
    return DRO_E_NULL;
  }
  if (N < 1 || N > 65535 || H < 1 || W < 1 || (long long)H * W * 3 >= (1LL << 31)) {
    set_error("color_jitter_rgb8: sizes out of range");
    return DRO_E_SHAPE;
  }
  static_assert(sizeof(JitterFrame) == 8 * sizeof(int), "JitterFrame layout = 8 x 32-bit per frame");
  hipStream_t s = (hipStream_t)stream;
  const int HW = H * W;
  int st = launch_zero(reinterpret_cast<float*>(workspace), 2 * (size_t)N, s);   // N x u64 luma sums
  if (st) return st;
  const JitterFrame* fr = reinterpret_cast<const JitterFrame*>(params);
  const dim3 grid((HW + kRsThreads - 1) / kRsThreads, N);
  hipLaunchKernelGGL(jitter_pre_kernel, grid, dim3(kRsThreads), 0, s, frames, HW, fr, workspace);
  st = launch_status("jitter_pre_kernel launch failed");
  if (st) return st;
  hipLaunchKernelGGL(jitter_post_kernel, grid, dim3(kRsThreads), 0, s, frames, HW, fr, workspace);
  return launch_status("jitter_post_kernel launch failed");
}

extern "C" int dro_resize_rgb8(const unsigned char* src, int N, int H0, int W0, int H, int W,
                               const int* xbounds, const int* xcoef, int KX, const int* ybounds,
                               const int* ycoef, int KY, unsigned char* tmp, unsigned char* dst,
                               void* stream) {
  if (!src || !xbounds || !xcoef || !ybounds || !ycoef || !tmp || !dst) {
    set_error("resize_rgb8: NULL pointer");
    return DRO_E_NULL;
  }
  if (N < 1 || H0 < 1 || W0 < 1 || H < 1 || W < 1 || KX < 1 || KY < 1 ||
      (long long)N * H0 * (W > W0 ? W : W0) * 3 >= (1LL << 40) || (long long)N * H * W * 3 >= (1LL << 40)) {
    set_error("resize_rgb8: sizes out of range");
    return DRO_E_SHAPE;
  }
  hipStream_t s = (hipStream_t)stream;
  const long long nh = (long long)N * H0 * W;
  hipLaunchKernelGGL(resize_h_kernel, dim3((unsigned)((nh + kRsThreads - 1) / kRsThreads)), dim3(kRsThreads), 0,
                     s, src, N, H0, W0, W, xbounds, xcoef, KX, tmp);
  int st = launch_status("resize_h_kernel launch failed");
  if (st) return st;
  const long long nv = (long long)N * H * W;
  hipLaunchKernelGGL(resize_v_u8_kernel, dim3((unsigned)((nv + kRsThreads - 1) / kRsThreads)), dim3(kRsThreads),
                     0, s, tmp, N, H0, H, W, ybounds, ycoef, KY, dst);
  return launch_status("resize_v_u8_kernel launch failed");
}

extern "C" int dro_rgb8_to_tensor(const unsigned char* src, int N, int H, int W, float* dst, void* stream) {
  if (!src || !dst) {
    set_error("rgb8_to_tensor: NULL pointer");
    return DRO_E_NULL;
  }
  if (N < 1 || N > 65535 || H < 1 || W < 1 || (long long)H * W * 3 >= (1LL << 31)) {
    set_error("rgb8_to_tensor: sizes out of range");
    return DRO_E_SHAPE;
  }
  const int HW = H * W;
  hipLaunchKernelGGL(rgb8_to_tensor_kernel, dim3((HW + kRsThreads - 1) / kRsThreads, N), dim3(kRsThreads), 0,
                     (hipStream_t)stream, src, HW, dst);
  return launch_status("rgb8_to_tensor_kernel launch failed");
}
