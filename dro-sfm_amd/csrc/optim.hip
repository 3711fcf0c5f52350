// Fused Adam over the flat parameter / gradient buffers of the data-parallel
// trainer (trainers/dp_trainer.py): one launch for all 221 tensors instead of
// the per-tensor kernels of torch.optim.Adam(capturable=True).  Same update as
// torch.optim.Adam (amsgrad off; the step counter lives on the device so the
// step can be captured in a hipGraph):
//   t += 1 (done by the caller before the launch)
//   g += wd * p;  m += (1-b1) (g - m);  v = b2 v + (1-b2) g^2
//   p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// HBM-bound: 16 B read + 12 B written per parameter (p, g, m, v / p, m, v).
// Every hyper-parameter is read from DEVICE memory (hyper = {lr, beta1, beta2,
// eps, weight_decay}), like the step counter: a replayed hipGraph picks up a
// learning-rate schedule (torch.optim.lr_scheduler.StepLR in the reference,
// model_wrapper.py:192-193) written between replays.
#include <hip/hip_runtime.h>

#include "dro_common.hpp"

namespace dro {

__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, float b1, float b2,
                                      float eps, float wd, float step_size, float bc2_sqrt) {
  if (wd != 0.f) g = fmaf(wd, p, g);
  m = fmaf(1.f - b1, g - m, m);
  v = fmaf(1.f - b2, g * g, v * b2);
  const float denom = sqrtf(v) / bc2_sqrt + eps;
  p = p - step_size * (m / denom);
}

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   long long n, const float* __restrict__ step,
                                                   const float* __restrict__ hyper) {
  const float t = *step;
  const float lr = hyper[0], b1 = hyper[1], b2 = hyper[2], eps = hyper[3], wd = hyper[4];
  const float bc1 = 1.f - powf(b1, t), bc2 = 1.f - powf(b2, t);
  const float step_size = lr / bc1, bc2_sqrt = sqrtf(bc2);
  const long long n4 = n / 4;
  const long long stride = (long long)gridDim.x * blockDim.x;
  float4* p4 = reinterpret_cast<float4*>(p);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  float4* m4 = reinterpret_cast<float4*>(m);
  float4* v4 = reinterpret_cast<float4*>(v);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pp = p4[i], mm = m4[i], vv = v4[i];
    const float4 gg = g4[i];
    adam1(pp.x, gg.x, mm.x, vv.x, b1, b2, eps, wd, step_size, bc2_sqrt);
    adam1(pp.y, gg.y, mm.y, vv.y, b1, b2, eps, wd, step_size, bc2_sqrt);
    adam1(pp.z, gg.z, mm.z, vv.z, b1, b2, eps, wd, step_size, bc2_sqrt);
    adam1(pp.w, gg.w, mm.w, vv.w, b1, b2, eps, wd, step_size, bc2_sqrt);
    p4[i] = pp;
    m4[i] = mm;
    v4[i] = vv;
  }
  for (long long i = n4 * 4 + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    adam1(p[i], g[i], m[i], v[i], b1, b2, eps, wd, step_size, bc2_sqrt);
}

}  // namespace dro

extern "C" int dro_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                             long long n, const float* step, const float* hyper, void* stream) {
  if (!param || !grad || !exp_avg || !exp_avg_sq || !step || !hyper) {
    dro::set_error("adam_step: NULL pointer");
    return DRO_E_NULL;
  }
  if (n < 1 || (reinterpret_cast<uintptr_t>(param) | reinterpret_cast<uintptr_t>(grad) |
                reinterpret_cast<uintptr_t>(exp_avg) | reinterpret_cast<uintptr_t>(exp_avg_sq)) % 16) {
    dro::set_error("adam_step: n < 1 or buffers not 16-byte aligned");
    return DRO_E_SHAPE;
  }
  long long blocks = (n / 4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(dro::adam_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, param, grad,
                     exp_avg, exp_avg_sq, n, step, hyper);
  return dro::launch_status("adam_kernel launch failed");
}
