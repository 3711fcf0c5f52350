// Device helpers shared by the gfx950 kernels: pinhole geometry, pose
// algebra, bilinear taps and wave/block reductions.  Arithmetic order follows
// the reference's PyTorch expressions (cited per function) so fp32 results
// track the reference to rounding.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/dro_amd.h"

namespace dro {

constexpr int kWave = 64;

// ---------------------------------------------------------------- error state
void set_error(const char* msg);
int launch_status(const char* what);
// zero n floats on stream s with a (graph-capturable) kernel launch
int launch_zero(float* p, size_t n, hipStream_t s);
// Sums per-workgroup pose partials [npose, nblk, 12] (dL/dR row-major, dL/dt)
// in a fixed order and writes the pose gradient in its own encoding.
int launch_pose_finalize(const double* partial, int nblk, int npose, const float* pose,
                         int pose_mode, float* gpose, hipStream_t s);

// ---------------------------------------------------------------- intrinsics
// Camera.scaled -> scale_intrinsics (geometry/camera_utils.py:13-19); only
// fx, fy, cx, cy change; skew and the last row are kept as given.
__device__ __forceinline__ void scaled_K(const float* __restrict__ K, float s, bool do_scale,
                                         float k[9]) {
#pragma unroll
  for (int i = 0; i < 9; ++i) k[i] = K[i];
  if (do_scale) {
    k[0] *= s;
    k[4] *= s;
    k[2] = (k[2] + 0.5f) * s - 0.5f;
    k[5] = (k[5] + 0.5f) * s - 0.5f;
  }
}

// Camera.Kinv (geometry/camera.py:70-79): a clone of K with the four pinhole
// entries replaced; every other entry is copied from K.
__device__ __forceinline__ void K_inverse(const float k[9], float ki[9]) {
#pragma unroll
  for (int i = 0; i < 9; ++i) ki[i] = k[i];
  ki[0] = 1.f / k[0];
  ki[4] = 1.f / k[4];
  ki[2] = (-1.f * k[2]) / k[0];
  ki[5] = (-1.f * k[5]) / k[4];
}

// ---------------------------------------------------------------- pose
// euler2mat (geometry/pose_utils.py:40-69): R = Rx(x) * Ry(y) * Rz(z).
__device__ __forceinline__ void euler_to_R(float ax, float ay, float az, float R[9]) {
  float sx, cx, sy, cy, sz, cz;
  sincosf(ax, &sx, &cx);
  sincosf(ay, &sy, &cy);
  sincosf(az, &sz, &cz);
  // Rx*Ry
  const float a10 = sx * sy, a12 = -sx * cy, a20 = -cx * sy, a22 = cx * cy;
  R[0] = cy * cz;
  R[1] = -(cy * sz);
  R[2] = sy;
  R[3] = a10 * cz + cx * sz;
  R[4] = a10 * (-sz) + cx * cz;
  R[5] = a12;
  R[6] = a20 * cz + sx * sz;
  R[7] = a20 * (-sz) + sx * cz;
  R[8] = a22;
}

__device__ __forceinline__ void load_pose(const float* __restrict__ p, int mode, float R[9],
                                          float t[3]) {
  if (mode == DRO_POSE_EULER) {
    t[0] = p[0];
    t[1] = p[1];
    t[2] = p[2];
    euler_to_R(p[3], p[4], p[5], R);
  } else {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      R[3 * r + 0] = p[4 * r + 0];
      R[3 * r + 1] = p[4 * r + 1];
      R[3 * r + 2] = p[4 * r + 2];
      t[r] = p[4 * r + 3];
    }
  }
}

template <typename T>
__device__ __forceinline__ void mat3_mul(const T A[9], const T B[9], T C[9]) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

// Gradient of a pose given dL/dR (row-major 3x3) and dL/dt, written in the
// pose's own encoding.  Euler: dL/dangle_k = <dL/dR, dR/dangle_k>.
__device__ __forceinline__ void store_pose_grad(const float* __restrict__ p, int mode,
                                                const float gR[9], const float gt[3],
                                                float* __restrict__ out) {
  if (mode == DRO_POSE_EULER) {
    out[0] = gt[0];
    out[1] = gt[1];
    out[2] = gt[2];
    float sx, cx, sy, cy, sz, cz;
    sincosf(p[3], &sx, &cx);
    sincosf(p[4], &sy, &cy);
    sincosf(p[5], &sz, &cz);
    const float Rx[9] = {1, 0, 0, 0, cx, -sx, 0, sx, cx};
    const float Ry[9] = {cy, 0, sy, 0, 1, 0, -sy, 0, cy};
    const float Rz[9] = {cz, -sz, 0, sz, cz, 0, 0, 0, 1};
    const float dRx[9] = {0, 0, 0, 0, -sx, -cx, 0, cx, -sx};
    const float dRy[9] = {-sy, 0, cy, 0, 0, 0, -cy, 0, -sy};
    const float dRz[9] = {-sz, -cz, 0, cz, -sz, 0, 0, 0, 0};
    float T0[9], T1[9], D[9];
    mat3_mul(dRx, Ry, T0);
    mat3_mul(T0, Rz, D);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 9; ++i) s += gR[i] * D[i];
    out[3] = s;
    mat3_mul(Rx, dRy, T0);
    mat3_mul(T0, Rz, D);
    s = 0.f;
#pragma unroll
    for (int i = 0; i < 9; ++i) s += gR[i] * D[i];
    out[4] = s;
    mat3_mul(Rx, Ry, T1);
    mat3_mul(T1, dRz, D);
    s = 0.f;
#pragma unroll
    for (int i = 0; i < 9; ++i) s += gR[i] * D[i];
    out[5] = s;
  } else {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      out[4 * r + 0] = gR[3 * r + 0];
      out[4 * r + 1] = gR[3 * r + 1];
      out[4 * r + 2] = gR[3 * r + 2];
      out[4 * r + 3] = gt[r];
    }
  }
}

// fp64 variant: the contraction of the summed R-gradient with dR/d(euler)
// cancels (see block_sum_d); sums and chain in double, stored as float.
__device__ __forceinline__ void store_pose_grad_d(const float* __restrict__ p, int mode,
                                                  const double gR[9], const double gt[3],
                                                float* __restrict__ out) {
  if (mode == DRO_POSE_EULER) {
    out[0] = (float)gt[0];
    out[1] = (float)gt[1];
    out[2] = (float)gt[2];
    double sx, cx, sy, cy, sz, cz;
    sincos((double)p[3], &sx, &cx);
    sincos((double)p[4], &sy, &cy);
    sincos((double)p[5], &sz, &cz);
    const double Rx[9] = {1, 0, 0, 0, cx, -sx, 0, sx, cx};
    const double Ry[9] = {cy, 0, sy, 0, 1, 0, -sy, 0, cy};
    const double Rz[9] = {cz, -sz, 0, sz, cz, 0, 0, 0, 1};
    const double dRx[9] = {0, 0, 0, 0, -sx, -cx, 0, cx, -sx};
    const double dRy[9] = {-sy, 0, cy, 0, 0, 0, -cy, 0, -sy};
    const double dRz[9] = {-sz, -cz, 0, cz, -sz, 0, 0, 0, 0};
    double T0[9], T1[9], D[9];
    mat3_mul(dRx, Ry, T0);
    mat3_mul(T0, Rz, D);
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i) s += gR[i] * D[i];
    out[3] = (float)s;
    mat3_mul(Rx, dRy, T0);
    mat3_mul(T0, Rz, D);
    s = 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i) s += gR[i] * D[i];
    out[4] = (float)s;
    mat3_mul(Rx, Ry, T1);
    mat3_mul(T1, dRz, D);
    s = 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i) s += gR[i] * D[i];
    out[5] = (float)s;
  } else {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      out[4 * r + 0] = (float)gR[3 * r + 0];
      out[4 * r + 1] = (float)gR[3 * r + 1];
      out[4 * r + 2] = (float)gR[3 * r + 2];
      out[4 * r + 3] = (float)gt[r];
    }
  }
}

__host__ __device__ constexpr int pose_stride(int mode) { return mode == DRO_POSE_EULER ? 6 : 12; }

// ---------------------------------------------------------------- depth
// Metric depth from the caller's encoding, and d(depth)/d(input).
//   inv2depth (utils/depth.py:102-121): 1/clamp(x,1e-6), 0 where x <= 0
//   disp_to_depth (networks/layers/resnet/layers.py:11-20): x' = a + (b-a)*x
__device__ __forceinline__ float decode_depth(float x, int mode, float min_disp, float span,
                                              float* ddx) {
  if (mode == DRO_DEPTH_METRIC) {
    *ddx = 1.f;
    return x;
  }
  float sd = x, dsd = 1.f;
  if (mode == DRO_DEPTH_DISP) {
    sd = min_disp + span * x;
    dsd = span;
  }
  if (sd <= 0.f) {
    *ddx = 0.f;
    return 0.f;
  }
  const float c = fmaxf(sd, 1e-6f);
  const float d = 1.f / c;
  *ddx = (sd >= 1e-6f) ? (-dsd / (c * c)) : 0.f;
  return d;
}

// ---------------------------------------------------------------- projection
// Camera.reconstruct (camera.py:111-147) of pixel (u,v) at `depth` with the
// identity Tcw, then Camera(ref_K, Tcw=pose).project(normalize=True)
// (camera.py:149-194) and grid_sample's align_corners unnormalisation.
struct Proj {
  float xn[3];  // Kinv * [u, v, 1]
  float X[3];   // xn * depth  (world == target camera frame)
  float x[3];   // ref_K * (R X + t)   (x[2] before the clamp)
  float Z;      // clamp(x[2], min=1e-5)
  float ix, iy; // sampling position in pixels of the reference map
};

__device__ __forceinline__ void project(const float ki[9], const float kr[9], const float R[9],
                                        const float t[3], float u, float v, float depth, int h,
                                        int w, Proj& q) {
  q.xn[0] = ki[0] * u + ki[1] * v + ki[2];
  q.xn[1] = ki[3] * u + ki[4] * v + ki[5];
  q.xn[2] = ki[6] * u + ki[7] * v + ki[8];
  q.X[0] = q.xn[0] * depth;
  q.X[1] = q.xn[1] * depth;
  q.X[2] = q.xn[2] * depth;
  float P[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) P[r] = R[3 * r] * q.X[0] + R[3 * r + 1] * q.X[1] + R[3 * r + 2] * q.X[2] + t[r];
#pragma unroll
  for (int r = 0; r < 3; ++r) q.x[r] = kr[3 * r] * P[0] + kr[3 * r + 1] * P[1] + kr[3 * r + 2] * P[2];
  q.Z = fmaxf(q.x[2], 1e-5f);
  const float wm1 = (float)(w - 1), hm1 = (float)(h - 1);
  const float xnorm = 2.f * (q.x[0] / q.Z) / wm1 - 1.f;
  const float ynorm = 2.f * (q.x[1] / q.Z) / hm1 - 1.f;
  q.ix = ((xnorm + 1.f) / 2.f) * wm1;
  q.iy = ((ynorm + 1.f) / 2.f) * hm1;
}

// Chain dL/d(ix,iy) back through the projection.  Accumulates dL/dR, dL/dt
// and returns dL/d(depth).  (ix == x0/Z and iy == x1/Z up to rounding: the
// grid normalisation and grid_sample's unnormalisation cancel.)
__device__ __forceinline__ float project_backward(const Proj& q, const float kr[9], const float R[9],
                                                  float gix, float giy, float gR[9], float gt[3]) {
  const float iz = 1.f / q.Z;
  float gx0 = gix * iz, gx1 = giy * iz;
  float gZ = -(gix * q.x[0] + giy * q.x[1]) * iz * iz;
  float gx2 = (q.x[2] >= 1e-5f) ? gZ : 0.f;
  float gP[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) gP[c] = kr[c] * gx0 + kr[3 + c] * gx1 + kr[6 + c] * gx2;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    gt[r] += gP[r];
    gR[3 * r + 0] += gP[r] * q.X[0];
    gR[3 * r + 1] += gP[r] * q.X[1];
    gR[3 * r + 2] += gP[r] * q.X[2];
  }
  float gd = 0.f;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float gX = R[c] * gP[0] + R[3 + c] * gP[1] + R[6 + c] * gP[2];
    gd += gX * q.xn[c];
  }
  return gd;
}

// project_backward, with dL/d(depth) in the parallax form.  With x = depth *
// (Kr R xn) + Kr t and u = x0 / x2, du/d(depth) = ((Kr R xn)_0 - u (Kr R xn)_2)
// / x2, and since x0 - u x2 = 0 the two terms of that difference are equal
// up to -((Kr t)_0 - u (Kr t)_2) / depth: the chain through gP above forms
// them separately and cancels them in fp32 (measured: 1.6e-4 relative at
// image-border pixels, where |xn| is largest, against 1.5e-5 for fp32
// autograd), this form takes the small difference from t directly.  Same
// value in exact arithmetic; the chain form where x2 is clamped or depth ~ 0.
__device__ __forceinline__ float project_backward_pt(const Proj& q, const float kr[9], const float R[9],
                                                     const float t[3], float depth, float gix, float giy,
                                                     float gR[9], float gt[3]) {
  const float gd_chain = project_backward(q, kr, R, gix, giy, gR, gt);
  if (!(q.x[2] >= 1e-5f) || !(depth > 1e-12f)) return gd_chain;
  const float kt0 = kr[0] * t[0] + kr[1] * t[1] + kr[2] * t[2];
  const float kt1 = kr[3] * t[0] + kr[4] * t[1] + kr[5] * t[2];
  const float kt2 = kr[6] * t[0] + kr[7] * t[1] + kr[8] * t[2];
  const float iz = 1.f / q.Z;
  const float u = q.x[0] * iz, v = q.x[1] * iz;
  return -(gix * (kt0 - u * kt2) + giy * (kt1 - v * kt2)) * iz / depth;
}

// ---------------------------------------------------------------- bilinear
// grid_sample(mode='bilinear', padding_mode='zeros', align_corners=True) taps
// in ATen's corner order nw, ne, sw, se.  Out-of-range corners have valid=0.
struct Taps {
  int idx[4];
  float wgt[4];
  bool ok[4];
  float tx, ty;  // ix - floor(ix), iy - floor(iy)
};

__device__ __forceinline__ void bilinear_taps(float ix, float iy, int h, int w, Taps& T) {
  const float fx = floorf(ix), fy = floorf(iy);
  const float ix_se = fx + 1.f, iy_se = fy + 1.f;
  T.wgt[0] = (ix_se - ix) * (iy_se - iy);  // nw
  T.wgt[1] = (ix - fx) * (iy_se - iy);     // ne
  T.wgt[2] = (ix_se - ix) * (iy - fy);     // sw
  T.wgt[3] = (ix - fx) * (iy - fy);        // se
  T.tx = ix - fx;
  T.ty = iy - fy;
  // range-check in float before the integer conversion (|ix| may be huge)
  const bool x0 = (fx >= 0.f) && (fx <= (float)(w - 1));
  const bool x1 = (fx >= -1.f) && (fx <= (float)(w - 2));
  const bool y0 = (fy >= 0.f) && (fy <= (float)(h - 1));
  const bool y1 = (fy >= -1.f) && (fy <= (float)(h - 2));
  const int xi = (x0 || x1) ? (int)fx : 0;
  const int yi = (y0 || y1) ? (int)fy : 0;
  T.ok[0] = x0 && y0;
  T.ok[1] = x1 && y0;
  T.ok[2] = x0 && y1;
  T.ok[3] = x1 && y1;
  T.idx[0] = yi * w + xi;
  T.idx[1] = T.idx[0] + 1;
  T.idx[2] = T.idx[0] + w;
  T.idx[3] = T.idx[2] + 1;
}

// Test hook (parity tests): the bilinear cell (floor(ix), floor(iy)) a kernel
// took, packed as ((y0 + 32768) << 16) | (x0 + 32768) with each coordinate
// clamped to [-32767, 32766] (cells that far out have no in-image tap either
// way); -1 (0xffffffff) is never produced and marks "not recorded".  A
// coordinate within rounding of an integer is where grid_sample's derivative
// jumps between two cells: the oracle takes the recorded cell so that fp32
// and fp64 evaluations are compared on the same branch.
__device__ __forceinline__ int pack_cell(float ix, float iy) {
  const float fx = fminf(fmaxf(floorf(ix), -32767.f), 32766.f);
  const float fy = fminf(fmaxf(floorf(iy), -32767.f), 32766.f);
  return (int)(((unsigned)((int)fy + 32768) << 16) | (unsigned)((int)fx + 32768));
}

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Block-wide sum of NV values per thread; result valid in thread 0.
// `scratch` must hold NV * (blockDim.x / 64) floats.
template <int NV>
__device__ __forceinline__ void block_sum(float (&v)[NV], float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) scratch[k * nw + wid] = v[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      float s = 0.f;
      for (int i = 0; i < nw; ++i) s += scratch[k * nw + i];
      v[k] = s;
    }
  }
  __syncthreads();
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Block-wide sum of NV per-thread values accumulated in fp64 (pose-gradient
// partials: the per-pixel terms R-gradient = sum_p gP X^T cancel heavily, and
// the euler chain contracts them again -- fp32 sums of ~10^4 terms put
// errors of ~1e-3 of the largest component on the small ones).  Result in
// `out` of thread 0.  `scratch` holds NV * (blockDim.x / 64) doubles.
template <int NV>
__device__ __forceinline__ void block_sum_d(const float (&v)[NV], double (&out)[NV], double* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) out[k] = wave_sum_d((double)v[k]);
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) scratch[k * nw + wid] = out[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      double s = 0.0;
      for (int i = 0; i < nw; ++i) s += scratch[k * nw + i];
      out[k] = s;
    }
  }
  __syncthreads();
}

// host: an integer tuning override from the environment (A/B runs), or dflt
inline int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e && *e ? atoi(e) : dflt;
}

}  // namespace dro
