// Fused supervised depth + pose loss (forward + backward).
//
// Replaces SupervisedDepthPoseLoss.forward (dro_sfm/losses/supervised_loss.py:
// 343-371) with supervised_method 'sparse-l1' (every reference yaml):
//   * calculate_loss (:244-277): masked inverse-depth L1 per prediction,
//     valid = 1/max_depth < gt_inv < 1/min_depth, mean over B*H*W, 0.85^(n-i-1)
//     decay normalised by its sum;
//   * calc_pose_loss (:293-325): every gt-depth pixel (min_depth < d <
//     max_depth/4) reconstructed in the target camera and projected into ref j
//     under the ground-truth pose and under prediction i's pose
//     (get_ref_coords :279-291 -> camera.py:111-194, normalize=True); the
//     per-coordinate |difference| clamped to 1 where both projections land in
//     [-1, 1], mean over [B,H,W,2], averaged over the N refs, same decay.
// The reference loops n x N in Python with two reconstruct+project chains per
// pair (~60 ATen launches per pair, ~500 per step at n=4, N=2); here the
// forward is 2 launches and the backward 2.
//
// Grid: (pixel blocks, B, prediction i).  A block owns kPxBlock consecutive
// pixels of one image for one prediction; the depth term and the N pose terms
// of that prediction are accumulated per thread and block-reduced into fixed
// partial slots (no atomics: every output is bitwise deterministic).
//
// Roofline: HBM bound.  Algorithmic bytes per pixel and prediction: forward
// 8 (gt_inv + inv_i), backward 12 (gt_inv + inv_i read, grad_i written).
#include <hip/hip_runtime.h>

#include "dro_common.hpp"

namespace dro {

constexpr int kSupThreads = 256;
constexpr int kSupPPT = 4;
constexpr int kPxBlock = kSupThreads * kSupPPT;

struct SupArgs {
  const float* gt_inv;   // [B, HW]
  const float* inv;      // [n, B, HW]
  const float* K;        // [B, 9]
  const float* ref_K;    // [B, 9]
  const float* gt_pose;  // [N, B, 12] row-major [R | t]
  const float* pose;     // [N, n, B, 6|12]
  int pose_mode;
  int B, N, n, H, W;
  float lo_disp, hi_disp;   // 1/max_depth, 1/min_depth (depth term validity)
  float min_d, max_d4;      // min_depth, max_depth/4   (pose term validity)
  int nblk;                 // pixel blocks per image
  float* part;              // forward: float [n][B][nblk][2]; backward: double [N][n][B][nblk][12]
};

// normalised projection of one reconstructed pixel (camera.py:178-184)
__device__ __forceinline__ void norm_coords(const Proj& q, float wm1, float hm1, float& un,
                                            float& vn) {
  un = 2.f * (q.x[0] / q.Z) / wm1 - 1.f;
  vn = 2.f * (q.x[1] / q.Z) / hm1 - 1.f;
}

__device__ __forceinline__ bool in_unit(float c) { return (c >= -1.f) && (c <= 1.f); }

__device__ __forceinline__ float sgn(float x) { return (float)((x > 0.f) - (x < 0.f)); }

// Normalised decay weight of prediction i (supervised_loss.py:263-277).
__device__ __forceinline__ float decay_weight(int i, int n) {
  float wi = 1.f, tot = 0.f, w = 1.f;
  for (int k = n - 1; k >= 0; --k) {  // w = 0.85^(n-k-1)
    if (k == i) wi = w;
    tot += w;
    w *= 0.85f;
  }
  return wi / tot;
}

template <bool BACKWARD>
__global__ __launch_bounds__(kSupThreads) void sup_loss_kernel(SupArgs a, const float* __restrict__ gout,
                                                               float* __restrict__ ginv) {
  __shared__ float scratch[12 * (kSupThreads / kWave)];
  __shared__ double dscratch[12 * (kSupThreads / kWave)];
  const int b = blockIdx.y, i = blockIdx.z;
  const int HW = a.H * a.W;
  const float wm1 = (float)(a.W - 1), hm1 = (float)(a.H - 1);
  float k[9], ki[9], kr[9];
#pragma unroll
  for (int e = 0; e < 9; ++e) {
    k[e] = a.K[b * 9 + e];
    kr[e] = a.ref_K[b * 9 + e];
  }
  K_inverse(k, ki);
  const float* gt_inv = a.gt_inv + (size_t)b * HW;
  const float* inv = a.inv + ((size_t)i * a.B + b) * HW;
  const int ps = pose_stride(a.pose_mode);

  // backward coefficients: d(total)/d(term) * decay / mean divisor
  float cd = 0.f, cp = 0.f;
  if (BACKWARD) {
    const float g = gout[0] * decay_weight(i, a.n);
    cd = g / (float)((double)a.B * HW);
    cp = g / (float)a.N / (float)(2.0 * a.B * HW);
  }

  const int p0 = blockIdx.x * kPxBlock + threadIdx.x;
  // depth term (all pixels of the block)
  float dsum = 0.f;
  float dep[kSupPPT];
  bool dmask[kSupPPT];
#pragma unroll
  for (int r = 0; r < kSupPPT; ++r) {
    const int p = p0 + r * kSupThreads;
    const bool live = p < HW;
    const float gv = live ? gt_inv[p] : 0.f;
    const float pv = live ? inv[p] : 0.f;
    const bool valid = live && (gv > a.lo_disp) && (gv < a.hi_disp);
    const float diff = gv - pv;
    if (BACKWARD) {
      if (live) ginv[((size_t)i * a.B + b) * HW + p] = valid ? -cd * sgn(diff) : 0.f;
    } else {
      dsum += valid ? fabsf(diff) : 0.f;
    }
    float dd;
    const float d = decode_depth(gv, DRO_DEPTH_INV, 0.f, 0.f, &dd);  // inv2depth
    dep[r] = d;
    dmask[r] = live && (d > a.min_d) && (d < a.max_d4);
  }

  // pose term: N refs of this prediction
  float psum = 0.f;
  for (int j = 0; j < a.N; ++j) {
    float Rg[9], tg[3], R[9], t[3];
    load_pose(a.gt_pose + ((size_t)j * a.B + b) * 12, DRO_POSE_MATRIX, Rg, tg);
    load_pose(a.pose + (((size_t)j * a.n + i) * a.B + b) * ps, a.pose_mode, R, t);
    float acc[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) acc[e] = 0.f;
#pragma unroll
    for (int r = 0; r < kSupPPT; ++r) {
      if (!dmask[r]) continue;
      const int p = p0 + r * kSupThreads;
      const float u = (float)(p % a.W), v = (float)(p / a.W);
      Proj qg, q;
      project(ki, kr, Rg, tg, u, v, dep[r], a.H, a.W, qg);
      project(ki, kr, R, t, u, v, dep[r], a.H, a.W, q);
      float ug, vg, up, vp;
      norm_coords(qg, wm1, hm1, ug, vg);
      norm_coords(q, wm1, hm1, up, vp);
      const float du = up - ug, dv = vp - vg;
      const bool mu = in_unit(ug) && in_unit(up), mv = in_unit(vg) && in_unit(vp);
      if (BACKWARD) {
        // d|d|/dd = sign(d); clamp(-1,1) passes the gradient where |d| <= 1
        const float gu = (mu && fabsf(du) <= 1.f) ? cp * sgn(du) : 0.f;
        const float gv = (mv && fabsf(dv) <= 1.f) ? cp * sgn(dv) : 0.f;
        if (gu != 0.f || gv != 0.f)
          project_backward(q, kr, R, gu * (2.f / wm1), gv * (2.f / hm1), acc, acc + 9);
      } else {
        psum += (mu ? fminf(fabsf(du), 1.f) : 0.f) + (mv ? fminf(fabsf(dv), 1.f) : 0.f);
      }
    }
    if (BACKWARD) {
      double sum[12];
      block_sum_d<12>(acc, sum, dscratch);
      if (threadIdx.x == 0) {
        double* dst = (double*)a.part + ((((size_t)j * a.n + i) * a.B + b) * a.nblk + blockIdx.x) * 12;
#pragma unroll
        for (int e = 0; e < 12; ++e) dst[e] = sum[e];
      }
    }
  }
  if (!BACKWARD) {
    float v[2] = {dsum, psum};
    block_sum<2>(v, scratch);
    if (threadIdx.x == 0) {
      float* dst = a.part + (((size_t)i * a.B + b) * a.nblk + blockIdx.x) * 2;
      dst[0] = v[0];
      dst[1] = v[1];
    }
  }
}

// One block: per prediction, fixed-order sums of the partials, then the
// reference's weighting (supervised_loss.py:263-277, :318-325, :364-369).
__global__ __launch_bounds__(256) void sup_finalize_kernel(SupArgs a, float* __restrict__ out) {
  __shared__ float scratch[2 * 4];
  const int per = a.B * a.nblk;
  const float npx = (float)((double)a.B * a.H * a.W);
  float depth_loss = 0.f, pose_loss = 0.f;
  for (int i = 0; i < a.n; ++i) {
    float v[2] = {0.f, 0.f};
    for (int k = threadIdx.x; k < per; k += blockDim.x) {
      const float* src = a.part + ((size_t)i * per + k) * 2;
      v[0] += src[0];
      v[1] += src[1];
    }
    block_sum<2>(v, scratch);
    if (threadIdx.x == 0) {
      const float w = decay_weight(i, a.n);
      depth_loss += w * (v[0] / npx);
      pose_loss += w * ((v[1] / (2.f * npx)) / (float)a.N);
    }
  }
  if (threadIdx.x == 0) {
    out[0] = depth_loss + pose_loss;
    out[1] = depth_loss;
    out[2] = pose_loss;
  }
}

static int sup_setup(const float* gt_inv, const float* inv, const float* K, const float* ref_K,
                     const float* gt_pose, const float* pose, int pose_mode, int B, int N, int n,
                     int H, int W, float min_depth, float max_depth, void* workspace, SupArgs& a) {
  if (!gt_inv || !inv || !K || !ref_K || !gt_pose || !pose || !workspace) {
    set_error("supervised_loss: NULL pointer");
    return DRO_E_NULL;
  }
  if (B < 1 || N < 1 || n < 1 || H < 2 || W < 2 || B > 65535 || n > 65535 ||
      (long long)H * W > (1LL << 30)) {
    set_error("supervised_loss: sizes out of range (need B,N,n >= 1, H,W >= 2)");
    return DRO_E_SHAPE;
  }
  if (pose_mode != DRO_POSE_EULER && pose_mode != DRO_POSE_MATRIX) {
    set_error("supervised_loss: unknown pose_mode");
    return DRO_E_MODE;
  }
  if (!(min_depth > 0.f) || !(max_depth > min_depth)) {
    set_error("supervised_loss: need 0 < min_depth < max_depth");
    return DRO_E_SHAPE;
  }
  a.gt_inv = gt_inv;
  a.inv = inv;
  a.K = K;
  a.ref_K = ref_K;
  a.gt_pose = gt_pose;
  a.pose = pose;
  a.pose_mode = pose_mode;
  a.B = B;
  a.N = N;
  a.n = n;
  a.H = H;
  a.W = W;
  // the reference compares fp32 tensors with Python doubles cast to fp32
  a.lo_disp = (float)(1.0 / (double)max_depth);
  a.hi_disp = (float)(1.0 / (double)min_depth);
  a.min_d = min_depth;
  a.max_d4 = (float)((double)max_depth / 4.0);
  a.nblk = (H * W + kPxBlock - 1) / kPxBlock;
  a.part = (float*)workspace;
  return DRO_OK;
}

}  // namespace dro

using namespace dro;

extern "C" size_t dro_supervised_workspace_bytes(int B, int N, int n, int H, int W) {
  const size_t nblk = ((size_t)H * W + kPxBlock - 1) / kPxBlock;
  // forward: float partials; backward: fp64 pose partials
  const size_t fwd = (size_t)n * B * nblk * 2 * sizeof(float);
  const size_t bwd = (size_t)N * n * B * nblk * 12 * sizeof(double);
  return fwd > bwd ? fwd : bwd;
}

extern "C" int dro_supervised_forward(const float* gt_inv, const float* inv_depths, const float* K,
                                      const float* ref_K, const float* gt_pose, const float* pose,
                                      int pose_mode, int B, int N, int n, int H, int W,
                                      float min_depth, float max_depth, float* out,
                                      void* workspace, void* stream) {
  SupArgs a;
  int st = sup_setup(gt_inv, inv_depths, K, ref_K, gt_pose, pose, pose_mode, B, N, n, H, W,
                     min_depth, max_depth, workspace, a);
  if (st) return st;
  if (!out) {
    set_error("supervised_forward: NULL out");
    return DRO_E_NULL;
  }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sup_loss_kernel<false>, dim3(a.nblk, B, n), dim3(kSupThreads), 0, s, a,
                     nullptr, nullptr);
  if ((st = launch_status("sup_loss_kernel<fwd> launch failed"))) return st;
  hipLaunchKernelGGL(sup_finalize_kernel, dim3(1), dim3(256), 0, s, a, out);
  return launch_status("sup_finalize_kernel launch failed");
}

extern "C" int dro_supervised_backward(const float* gt_inv, const float* inv_depths,
                                       const float* K, const float* ref_K, const float* gt_pose,
                                       const float* pose, int pose_mode, int B, int N, int n,
                                       int H, int W, float min_depth, float max_depth,
                                       const float* grad_out, float* grad_inv_depths,
                                       float* grad_pose, void* workspace, void* stream) {
  SupArgs a;
  int st = sup_setup(gt_inv, inv_depths, K, ref_K, gt_pose, pose, pose_mode, B, N, n, H, W,
                     min_depth, max_depth, workspace, a);
  if (st) return st;
  if (!grad_out || !grad_inv_depths || !grad_pose) {
    set_error("supervised_backward: NULL grad_out/grad_inv_depths/grad_pose");
    return DRO_E_NULL;
  }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sup_loss_kernel<true>, dim3(a.nblk, B, n), dim3(kSupThreads), 0, s, a,
                     grad_out, grad_inv_depths);
  if ((st = launch_status("sup_loss_kernel<bwd> launch failed"))) return st;
  return launch_pose_finalize((const double*)a.part, a.nblk, N * n * B, pose, pose_mode, grad_pose, s);
}
