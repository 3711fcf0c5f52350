// Training-mode BatchNorm2d fused with the ReLU (and the residual add) that
// follows it in the ResNet-18 encoders of DepthPoseNet
// (networks/optim/extractor.py:7-107 of the reference: conv -> BN -> ReLU, and
// BasicBlock's relu(bn2(conv2(.)) + skip)).  PyTorch runs each such site as
// 6-9 launches (statistics, transform, relu, running-stat update, counter
// increment; threshold backward, BN backward reduce + elementwise); here it is
// two launches forward and two backward, all deterministic (fixed-order
// reductions, no atomics):
//   bn_stats_kernel     per (channel, image, chunk) partial sum / sum of squares (fp64)
//   bn_apply_kernel     every block folds its channel's partials (fixed order) into
//                       mean / invstd, normalises, adds skip, applies ReLU; the first
//                       block of a channel writes save_mean / save_invstd and the
//                       running statistics (and bumps num_batches_tracked)
//   bn_bwd_reduce_kernel  partial sums of g and g * xhat, g = dy * [y > 0]
//   bn_bwd_apply_kernel   dx = gamma * invstd * (g - mean(g) - xhat * mean(g xhat)),
//                       dskip = g; first block of a channel writes dgamma, dbeta
// Sites whose channels hold <= 16 K elements take ONE launch each way
// (bn_fused_fwd_kernel / bn_fused_bwd_kernel, a block per channel, below).
// Statistics follow torch.nn.functional.batch_norm (biased variance for the
// normalisation, unbiased for running_var, running = (1 - m) * running + m * batch).
// Layout: NCHW fp32, planes of HW contiguous floats.
#include "dro_common.hpp"

namespace dro {
namespace {

constexpr int kBnThreads = 256;

struct BnGeom {
  int N, C, HW;
  int Q;            // chunks per plane in the reduction kernels
  int chunk;        // floats per reduction chunk (multiple of 4)
};

template <bool VEC>
__device__ __forceinline__ float4 ld4(const float* __restrict__ p, long long i) {
  if (VEC) return *reinterpret_cast<const float4*>(p + i);
  return make_float4(p[i], p[i + 1], p[i + 2], p[i + 3]);
}

template <bool VEC>
__device__ __forceinline__ void st4(float* __restrict__ p, long long i, float4 v) {
  if (VEC) {
    *reinterpret_cast<float4*>(p + i) = v;
  } else {
    p[i] = v.x;
    p[i + 1] = v.y;
    p[i + 2] = v.z;
    p[i + 3] = v.w;
  }
}

__device__ __forceinline__ double block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < kBnThreads / 64; ++i) s += red[i];
  return s;
}

// partial[(c * N + n) * Q + q] = {sum, sum of squares} over chunk q of plane (n, c)
template <bool VEC>
__global__ __launch_bounds__(kBnThreads) void bn_stats_kernel(const float* __restrict__ x, BnGeom g,
                                                              double2* __restrict__ partial) {
  __shared__ double red[kBnThreads / 64];
  const int q = blockIdx.x, n = blockIdx.y, c = blockIdx.z;
  const long long base = ((long long)n * g.C + c) * g.HW;
  const int lo = q * g.chunk, hi = min(g.HW, lo + g.chunk);
  double s1 = 0.0, s2 = 0.0;
  const int hi4 = lo + ((hi - lo) & ~3);
  for (int i = lo + 4 * threadIdx.x; i < hi4; i += 4 * kBnThreads) {
    const float4 v = ld4<VEC>(x, base + i);
    s1 += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
    s2 += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
  }
  for (int i = hi4 + threadIdx.x; i < hi; i += kBnThreads) {
    const double v = x[base + i];
    s1 += v;
    s2 += v * v;
  }
  s1 = block_sum(s1, red);
  s2 = block_sum(s2, red);
  if (threadIdx.x == 0) partial[((long long)c * g.N + n) * g.Q + q] = make_double2(s1, s2);
}

// sum of a channel's N * Q partials in a fixed order
__device__ __forceinline__ double2 fold(const double2* __restrict__ p, int cnt) {
  double a = 0.0, b = 0.0;
  for (int i = 0; i < cnt; ++i) {
    const double2 v = p[i];
    a += v.x;
    b += v.y;
  }
  return make_double2(a, b);
}

struct BnFwdArgs {
  const float* x;
  const float* gamma;
  const float* beta;
  const float* skip;       // nullable: added before the ReLU
  int relu;
  float eps, momentum;
  float* running_mean;     // nullable (track_running_stats=False)
  float* running_var;
  long long* num_batches;  // nullable
  float* y;
  float* save_mean;
  float* save_invstd;
  const double2* partial;
};

// grid (blocks per plane, N * C)
template <bool VEC>
__global__ __launch_bounds__(kBnThreads) void bn_apply_kernel(BnFwdArgs a, BnGeom g) {
  __shared__ float coef[3];
  const int plane = blockIdx.y, c = plane % g.C;
  if (threadIdx.x == 0) {
    const long long L = (long long)g.N * g.HW;
    const double2 s = fold(a.partial + (long long)c * g.N * g.Q, g.N * g.Q);
    const double mean = s.x / (double)L;
    double var = s.y / (double)L - mean * mean;
    var = var > 0.0 ? var : 0.0;
    const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
    const float gm = a.gamma ? a.gamma[c] : 1.f;
    // y = (x - mean) * (gamma * invstd) + beta: centre first (x * k + (beta - mean * k)
    // cancels catastrophically when |mean| >> std)
    coef[0] = gm * invstd;
    coef[1] = a.beta ? a.beta[c] : 0.f;
    coef[2] = (float)mean;
    if (plane < g.C && blockIdx.x == 0) {                    // first block of the channel (n == 0)
      a.save_mean[c] = (float)mean;
      a.save_invstd[c] = invstd;
      if (a.running_mean) {
        const double unb = L > 1 ? var * (double)L / (double)(L - 1) : var;
        a.running_mean[c] = (1.f - a.momentum) * a.running_mean[c] + a.momentum * (float)mean;
        a.running_var[c] = (1.f - a.momentum) * a.running_var[c] + a.momentum * (float)unb;
      }
      if (c == 0 && a.num_batches) *a.num_batches += 1;
    }
  }
  __syncthreads();
  const float k = coef[0], o = coef[1], mu = coef[2];
  const long long base = (long long)plane * g.HW;
  auto f = [&](float v, float s) {
    float r = fmaf(v - mu, k, o) + s;
    return a.relu ? fmaxf(r, 0.f) : r;
  };
  const int hw4 = g.HW & ~3;
  for (int i = 4 * (blockIdx.x * kBnThreads + threadIdx.x); i < hw4; i += 4 * kBnThreads * gridDim.x) {
    const float4 v = ld4<VEC>(a.x, base + i);
    const float4 s = a.skip ? ld4<VEC>(a.skip, base + i) : make_float4(0.f, 0.f, 0.f, 0.f);
    st4<VEC>(a.y, base + i, make_float4(f(v.x, s.x), f(v.y, s.y), f(v.z, s.z), f(v.w, s.w)));
  }
  for (int i = hw4 + blockIdx.x * kBnThreads + threadIdx.x; i < g.HW; i += kBnThreads * gridDim.x)
    a.y[base + i] = f(a.x[base + i], a.skip ? a.skip[base + i] : 0.f);
}

struct BnBwdArgs {
  const float* dy;
  const float* x;
  const float* y;          // output (ReLU mask y > 0); nullable when relu == 0
  const float* gamma;
  const float* save_mean;
  const float* save_invstd;
  int relu;
  float* dx;
  float* dgamma;           // nullable
  float* dbeta;            // nullable
  float* dskip;            // nullable: receives g
  double2* partial;
};

__device__ __forceinline__ float grad_in(float dy, float y, int relu) {
  return relu ? (y > 0.f ? dy : 0.f) : dy;
}

template <bool VEC>
__global__ __launch_bounds__(kBnThreads) void bn_bwd_reduce_kernel(BnBwdArgs a, BnGeom g) {
  __shared__ double red[kBnThreads / 64];
  const int q = blockIdx.x, n = blockIdx.y, c = blockIdx.z;
  const long long base = ((long long)n * g.C + c) * g.HW;
  const float mean = a.save_mean[c], invstd = a.save_invstd[c];
  const int lo = q * g.chunk, hi = min(g.HW, lo + g.chunk);
  double s1 = 0.0, s2 = 0.0;
  const int hi4 = lo + ((hi - lo) & ~3);
  const float* ysrc = a.relu ? a.y : a.dy;
  for (int i = lo + 4 * threadIdx.x; i < hi4; i += 4 * kBnThreads) {
    const float4 d = ld4<VEC>(a.dy, base + i), v = ld4<VEC>(a.x, base + i), yy = ld4<VEC>(ysrc, base + i);
    const float g0 = grad_in(d.x, yy.x, a.relu), g1 = grad_in(d.y, yy.y, a.relu);
    const float g2 = grad_in(d.z, yy.z, a.relu), g3 = grad_in(d.w, yy.w, a.relu);
    s1 += (double)g0 + (double)g1 + (double)g2 + (double)g3;
    s2 += (double)(g0 * ((v.x - mean) * invstd)) + (double)(g1 * ((v.y - mean) * invstd)) +
          (double)(g2 * ((v.z - mean) * invstd)) + (double)(g3 * ((v.w - mean) * invstd));
  }
  for (int i = hi4 + threadIdx.x; i < hi; i += kBnThreads) {
    const float gi = grad_in(a.dy[base + i], ysrc[base + i], a.relu);
    s1 += gi;
    s2 += (double)(gi * ((a.x[base + i] - mean) * invstd));
  }
  s1 = block_sum(s1, red);
  s2 = block_sum(s2, red);
  if (threadIdx.x == 0) a.partial[((long long)c * g.N + n) * g.Q + q] = make_double2(s1, s2);
}

template <bool VEC>
__global__ __launch_bounds__(kBnThreads) void bn_bwd_apply_kernel(BnBwdArgs a, BnGeom g) {
  __shared__ float coef[3];
  const int plane = blockIdx.y, c = plane % g.C;
  const float mean = a.save_mean[c], invstd = a.save_invstd[c];
  if (threadIdx.x == 0) {
    const long long L = (long long)g.N * g.HW;
    const double2 s = fold(a.partial + (long long)c * g.N * g.Q, g.N * g.Q);
    const float gm = a.gamma ? a.gamma[c] : 1.f;
    coef[0] = gm * invstd;
    coef[1] = (float)(s.x / (double)L);
    coef[2] = (float)(s.y / (double)L);
    if (plane < g.C && blockIdx.x == 0) {
      if (a.dgamma) a.dgamma[c] = (float)s.y;
      if (a.dbeta) a.dbeta[c] = (float)s.x;
    }
  }
  __syncthreads();
  const float k = coef[0], mg = coef[1], mgx = coef[2];
  const long long base = (long long)plane * g.HW;
  const float* ysrc = a.relu ? a.y : a.dy;
  auto f = [&](float gi, float v) { return k * (gi - mg - ((v - mean) * invstd) * mgx); };
  const int hw4 = g.HW & ~3;
  for (int i = 4 * (blockIdx.x * kBnThreads + threadIdx.x); i < hw4; i += 4 * kBnThreads * gridDim.x) {
    const float4 d = ld4<VEC>(a.dy, base + i), v = ld4<VEC>(a.x, base + i), yy = ld4<VEC>(ysrc, base + i);
    const float4 gi = make_float4(grad_in(d.x, yy.x, a.relu), grad_in(d.y, yy.y, a.relu),
                                  grad_in(d.z, yy.z, a.relu), grad_in(d.w, yy.w, a.relu));
    st4<VEC>(a.dx, base + i, make_float4(f(gi.x, v.x), f(gi.y, v.y), f(gi.z, v.z), f(gi.w, v.w)));
    if (a.dskip) st4<VEC>(a.dskip, base + i, gi);
  }
  for (int i = hw4 + blockIdx.x * kBnThreads + threadIdx.x; i < g.HW; i += kBnThreads * gridDim.x) {
    const float gi = grad_in(a.dy[base + i], ysrc[base + i], a.relu);
    a.dx[base + i] = f(gi, a.x[base + i]);
    if (a.dskip) a.dskip[base + i] = gi;
  }
}

// ---------------------------------------------------------------- one launch per direction
// Small sites (a channel's N * HW <= 16 K elements: the encoders' layer2 /
// layer3 at KITTI size, 480-1920 pixels per plane): ONE block of 1024 threads
// per channel keeps its elements in registers (thread t holds elements
// t + 1024 k, k < EPT), reduces them in a fixed order (per thread in k order,
// then the block tree), and applies the transform from the registers -- one
// launch forward and one backward instead of two each, no partials.
constexpr int kFusedThreads = 1024;
constexpr int kFusedMaxEPT = 16;

__device__ __forceinline__ double block_sum_fused(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < kFusedThreads / 64; ++i) s += red[i];
  return s;
}

// element e of channel c (e < N * HW) -> its offset in the NCHW tensor
__device__ __forceinline__ long long chan_off(int e, int c, const BnGeom& g) {
  const int n = e / g.HW, i = e - n * g.HW;
  return ((long long)n * g.C + c) * g.HW + i;
}

template <int EPT>
__global__ __launch_bounds__(kFusedThreads) void bn_fused_fwd_kernel(BnFwdArgs a, BnGeom g) {
  __shared__ double red[kFusedThreads / 64];
  const int c = blockIdx.x;
  const int L = g.N * g.HW;
  float xv[EPT];
  double s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = threadIdx.x + kFusedThreads * k;
    xv[k] = e < L ? a.x[chan_off(e, c, g)] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const double v = xv[k];
    s1 += v;
    s2 += v * v;
  }
  s1 = block_sum_fused(s1, red);
  s2 = block_sum_fused(s2, red);
  const double mean = s1 / (double)L;
  double var = s2 / (double)L - mean * mean;
  var = var > 0.0 ? var : 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
  const float k0 = (a.gamma ? a.gamma[c] : 1.f) * invstd, o = a.beta ? a.beta[c] : 0.f, mu = (float)mean;
  if (threadIdx.x == 0) {
    a.save_mean[c] = mu;
    a.save_invstd[c] = invstd;
    if (a.running_mean) {
      const double unb = L > 1 ? var * (double)L / (double)(L - 1) : var;
      a.running_mean[c] = (1.f - a.momentum) * a.running_mean[c] + a.momentum * mu;
      a.running_var[c] = (1.f - a.momentum) * a.running_var[c] + a.momentum * (float)unb;
    }
    if (c == 0 && a.num_batches) *a.num_batches += 1;
  }
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = threadIdx.x + kFusedThreads * k;
    if (e >= L) continue;
    const long long q = chan_off(e, c, g);      // recomputed: keeping EPT 64-bit offsets costs registers
    float r = fmaf(xv[k] - mu, k0, o) + (a.skip ? a.skip[q] : 0.f);
    a.y[q] = a.relu ? fmaxf(r, 0.f) : r;
  }
}

template <int EPT>
__global__ __launch_bounds__(kFusedThreads) void bn_fused_bwd_kernel(BnBwdArgs a, BnGeom g) {
  __shared__ double red[kFusedThreads / 64];
  const int c = blockIdx.x;
  const int L = g.N * g.HW;
  const float mean = a.save_mean[c], invstd = a.save_invstd[c];
  const float* ysrc = a.relu ? a.y : a.dy;
  float gv[EPT], xh[EPT];
  double s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = threadIdx.x + kFusedThreads * k;
    const long long q = e < L ? chan_off(e, c, g) : 0;
    const float d = a.dy[q], v = a.x[q], yy = ysrc[q];
    gv[k] = e < L ? grad_in(d, yy, a.relu) : 0.f;
    // lanes past the channel read element 0 (in bounds) but must add nothing:
    // 0 * xh would be NaN for an Inf/NaN x[0]
    xh[k] = e < L ? (v - mean) * invstd : 0.f;
  }
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    s1 += gv[k];
    s2 += (double)(gv[k] * xh[k]);
  }
  s1 = block_sum_fused(s1, red);
  s2 = block_sum_fused(s2, red);
  const float kk = (a.gamma ? a.gamma[c] : 1.f) * invstd;
  const float mg = (float)(s1 / (double)L), mgx = (float)(s2 / (double)L);
  if (threadIdx.x == 0) {
    if (a.dgamma) a.dgamma[c] = (float)s2;
    if (a.dbeta) a.dbeta[c] = (float)s1;
  }
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = threadIdx.x + kFusedThreads * k;
    if (e >= L) continue;
    const long long q = chan_off(e, c, g);
    a.dx[q] = kk * (gv[k] - mg - xh[k] * mgx);
    if (a.dskip) a.dskip[q] = gv[k];
  }
}

// EPT for the one-launch path, 0 = the two-launch path
int fused_ept(int N, int HW) {
  const long long L = (long long)N * HW;
  for (int e = 1; e <= kFusedMaxEPT; e *= 2)
    if (L <= (long long)kFusedThreads * e) return e;
  return 0;
}

// reduction chunking: ~1-2 K blocks over the whole tensor, chunks of >= 1 K floats
BnGeom bn_geom(int N, int C, int HW) {
  BnGeom g;
  g.N = N;
  g.C = C;
  g.HW = HW;
  const long long planes = (long long)N * C;
  long long q = (1536 + planes - 1) / planes;
  const long long qmax = (HW + 1023) / 1024;
  if (q > qmax) q = qmax;
  if (q < 1) q = 1;
  int chunk = (int)((HW + q - 1) / q);
  chunk = (chunk + 3) & ~3;
  g.chunk = chunk;
  g.Q = (HW + chunk - 1) / chunk;
  return g;
}

// elementwise kernels: blocks per plane so that the grid has >= ~2 K blocks
int apply_blocks(const BnGeom& g) {
  const long long planes = (long long)g.N * g.C;
  long long per = (2048 + planes - 1) / planes;
  const long long need = (g.HW + 4 * kBnThreads - 1) / (4 * kBnThreads);
  if (per > need) per = need;
  if (per < 1) per = 1;
  return (int)per;
}

int bn_check(int N, int C, int HW) {
  if (N < 1 || C < 1 || HW < 1 || (long long)N * C > 65535LL * 65535LL || C > 65535 || N > 65535 ||
      (long long)N * C * HW >= (1LL << 40)) {
    set_error("batchnorm: sizes out of range");
    return DRO_E_SHAPE;
  }
  return DRO_OK;
}

bool aligned16(const void* p) { return p == nullptr || (reinterpret_cast<size_t>(p) & 15) == 0; }

}  // namespace
}  // namespace dro

using namespace dro;

extern "C" size_t dro_batchnorm_workspace_bytes(int N, int C, int HW) {
  if (bn_check(N, C, HW)) return 0;
  const BnGeom g = bn_geom(N, C, HW);
  return (size_t)C * N * g.Q * sizeof(double2);
}

extern "C" int dro_batchnorm_relu_forward(const float* x, const float* gamma, const float* beta,
                                          const float* skip, int relu, int N, int C, int HW,
                                          float eps, float momentum, float* running_mean,
                                          float* running_var, long long* num_batches_tracked,
                                          float* y, float* save_mean, float* save_invstd,
                                          void* workspace, size_t workspace_bytes, void* stream) {
  int st = bn_check(N, C, HW);
  if (st) return st;
  if (!x || !y || !save_mean || !save_invstd || !workspace || (!running_mean) != (!running_var)) {
    set_error("batchnorm_relu_forward: NULL pointer");
    return DRO_E_NULL;
  }
  if (relu != 0 && relu != 1) {
    set_error("batchnorm_relu_forward: relu must be 0 or 1");
    return DRO_E_MODE;
  }
  const BnGeom g = bn_geom(N, C, HW);
  if (workspace_bytes < (size_t)C * N * g.Q * sizeof(double2)) {
    set_error("batchnorm_relu_forward: workspace too small");
    return DRO_E_SHAPE;
  }
  hipStream_t s = (hipStream_t)stream;
  double2* part = static_cast<double2*>(workspace);
  if (const int ept = fused_ept(N, HW)) {
    BnFwdArgs a{x, gamma, beta, skip, relu, eps, momentum, running_mean, running_var,
                num_batches_tracked, y, save_mean, save_invstd, nullptr};
    switch (ept) {
      case 1: hipLaunchKernelGGL(bn_fused_fwd_kernel<1>, dim3(C), dim3(kFusedThreads), 0, s, a, g); break;
      case 2: hipLaunchKernelGGL(bn_fused_fwd_kernel<2>, dim3(C), dim3(kFusedThreads), 0, s, a, g); break;
      case 4: hipLaunchKernelGGL(bn_fused_fwd_kernel<4>, dim3(C), dim3(kFusedThreads), 0, s, a, g); break;
      case 8: hipLaunchKernelGGL(bn_fused_fwd_kernel<8>, dim3(C), dim3(kFusedThreads), 0, s, a, g); break;
      default: hipLaunchKernelGGL(bn_fused_fwd_kernel<16>, dim3(C), dim3(kFusedThreads), 0, s, a, g);
    }
    return launch_status("bn_fused_fwd_kernel launch failed");
  }
  const bool vec = (HW & 3) == 0 && aligned16(x) && aligned16(y) && aligned16(skip);
  const dim3 rg(g.Q, N, C);
  if (vec)
    hipLaunchKernelGGL(bn_stats_kernel<true>, rg, dim3(kBnThreads), 0, s, x, g, part);
  else
    hipLaunchKernelGGL(bn_stats_kernel<false>, rg, dim3(kBnThreads), 0, s, x, g, part);
  st = launch_status("bn_stats_kernel launch failed");
  if (st) return st;
  BnFwdArgs a{x, gamma, beta, skip, relu, eps, momentum, running_mean, running_var,
              num_batches_tracked, y, save_mean, save_invstd, part};
  const dim3 ag(apply_blocks(g), (unsigned)N * C);
  if (vec)
    hipLaunchKernelGGL(bn_apply_kernel<true>, ag, dim3(kBnThreads), 0, s, a, g);
  else
    hipLaunchKernelGGL(bn_apply_kernel<false>, ag, dim3(kBnThreads), 0, s, a, g);
  return launch_status("bn_apply_kernel launch failed");
}

extern "C" int dro_batchnorm_relu_backward(const float* grad_out, const float* x, const float* y,
                                           const float* gamma, const float* save_mean,
                                           const float* save_invstd, int relu, int N, int C,
                                           int HW, float* grad_x, float* grad_gamma,
                                           float* grad_beta, float* grad_skip, void* workspace,
                                           size_t workspace_bytes, void* stream) {
  int st = bn_check(N, C, HW);
  if (st) return st;
  if (!grad_out || !x || !save_mean || !save_invstd || !grad_x || !workspace || (relu && !y)) {
    set_error("batchnorm_relu_backward: NULL pointer");
    return DRO_E_NULL;
  }
  if (relu != 0 && relu != 1) {
    set_error("batchnorm_relu_backward: relu must be 0 or 1");
    return DRO_E_MODE;
  }
  const BnGeom g = bn_geom(N, C, HW);
  if (workspace_bytes < (size_t)C * N * g.Q * sizeof(double2)) {
    set_error("batchnorm_relu_backward: workspace too small");
    return DRO_E_SHAPE;
  }
  hipStream_t s = (hipStream_t)stream;
  BnBwdArgs a{grad_out, x, y, gamma, save_mean, save_invstd, relu, grad_x, grad_gamma, grad_beta,
              grad_skip, static_cast<double2*>(workspace)};
  if (const int ept = fused_ept(N, HW)) {
    switch (ept) {
      case 1: hipLaunchKernelGGL(bn_fused_bwd_kernel<1>, dim3(C), dim3(kFusedThreads), 0, s, a, g); break;
      case 2: hipLaunchKernelGGL(bn_fused_bwd_kernel<2>, dim3(C), dim3(kFusedThreads), 0, s, a, g); break;
      case 4: hipLaunchKernelGGL(bn_fused_bwd_kernel<4>, dim3(C), dim3(kFusedThreads), 0, s, a, g); break;
      case 8: hipLaunchKernelGGL(bn_fused_bwd_kernel<8>, dim3(C), dim3(kFusedThreads), 0, s, a, g); break;
      default: hipLaunchKernelGGL(bn_fused_bwd_kernel<16>, dim3(C), dim3(kFusedThreads), 0, s, a, g);
    }
    return launch_status("bn_fused_bwd_kernel launch failed");
  }
  const bool vec = (HW & 3) == 0 && aligned16(grad_out) && aligned16(x) && aligned16(y) &&
                   aligned16(grad_x) && aligned16(grad_skip);
  const dim3 rg(g.Q, N, C);
  if (vec)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<true>, rg, dim3(kBnThreads), 0, s, a, g);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<false>, rg, dim3(kBnThreads), 0, s, a, g);
  st = launch_status("bn_bwd_reduce_kernel launch failed");
  if (st) return st;
  const dim3 ag(apply_blocks(g), (unsigned)N * C);
  if (vec)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<true>, ag, dim3(kBnThreads), 0, s, a, g);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<false>, ag, dim3(kBnThreads), 0, s, a, g);
  return launch_status("bn_bwd_apply_kernel launch failed");
}
