// PoseHead's spatial mean and rotation scale, fused with the pose update
// (dro_sfm/networks/optim/update.py:16-28 PoseHead.forward -- mean over
// (H, W) of the 6-channel map, rotation entries x 0.01 -- and :189-197
// `pose = pose + self.pose_head(net)`).  Through ATen: mean, mul, add forward
// and expand/div/mul/sum launches backward per call (16 calls per KITTI it8
// step); here one launch each way.
// Forward: one block per (sample, channel) plane sums its H*W values in a
// fixed order (per-thread strided partials, then a fixed shuffle / LDS tree:
// deterministic).  Backward: d(out)/d(y) = scale_c / (H*W) broadcast;
// d(out)/d(pose) is the identity (no launch).
// Roofline: HBM, 4 bytes per map element each way; launch-latency bound at
// these sizes (6 x 1920 values per sample).
#include <hip/hip_runtime.h>

#include "dro_common.hpp"

namespace dro {

__global__ __launch_bounds__(256) void pose_mean_fwd_kernel(const float* __restrict__ y,
                                                            const float* __restrict__ pose,
                                                            float* __restrict__ out, int C, int HW,
                                                            float rot_scale) {
  __shared__ float red[256 / kWave];
  const int plane = blockIdx.x, c = plane % C;
  const float* p = y + (size_t)plane * HW;
  float s = 0.f;
  for (int i = threadIdx.x; i < HW; i += 256) s += p[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float tot = (red[0] + red[1]) + (red[2] + red[3]);
    const float v = (tot / (float)HW) * (c >= 3 ? rot_scale : 1.f);
    out[plane] = pose ? pose[plane] + v : v;
  }
}

__global__ __launch_bounds__(256) void pose_mean_bwd_kernel(const float* __restrict__ gout,
                                                            float* __restrict__ gy, int C, int HW,
                                                            long long total, float rot_scale) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    const int plane = (int)(e / HW), c = plane % C;
    gy[e] = gout[plane] * (c >= 3 ? rot_scale : 1.f) / (float)HW;
  }
}

}  // namespace dro

using namespace dro;

extern "C" int dro_pose_mean_forward(const float* y, const float* pose, float* out, int B, int C, int HW,
                                     float rot_scale, void* stream) {
  if (!y || !out) {
    set_error("pose_mean_forward: NULL pointer");
    return DRO_E_NULL;
  }
  if (B < 1 || C < 1 || HW < 1 || (long long)B * C > 65535 * 64) {
    set_error("pose_mean_forward: sizes out of range");
    return DRO_E_SHAPE;
  }
  hipLaunchKernelGGL(pose_mean_fwd_kernel, dim3((unsigned)(B * C)), dim3(256), 0, (hipStream_t)stream, y, pose,
                     out, C, HW, rot_scale);
  return launch_status("pose_mean_fwd_kernel launch failed");
}

extern "C" int dro_pose_mean_backward(const float* gout, float* gy, int B, int C, int HW, float rot_scale,
                                      void* stream) {
  if (!gout || !gy) {
    set_error("pose_mean_backward: NULL pointer");
    return DRO_E_NULL;
  }
  if (B < 1 || C < 1 || HW < 1) {
    set_error("pose_mean_backward: sizes out of range");
    return DRO_E_SHAPE;
  }
  const long long total = (long long)B * C * HW;
  long long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(pose_mean_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, gout, gy,
                     C, HW, total, rot_scale);
  return launch_status("pose_mean_bwd_kernel launch failed");
}
