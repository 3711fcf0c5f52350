// Fused inverse warp + squared feature cost for the DRO recurrent optimizer.
//
// Replaces the ATen chain of DepthPoseNet.get_cost_each / depth_cost_calc
// (dro_sfm/networks/depth_pose/DepthPoseNet.py:76-105): Pose.from_vec,
// 2x Camera.scaled, Kinv, 3 bmm (reconstruct / transform / project), clamp,
// normalise, grid_sampler_2d, sub, pow, stack, mean -- ~40 launches per call
// in the reference -- with ONE launch over every reference view.
//
// Layout: all maps dense NCHW fp32.  A 256-thread workgroup covers 64
// consecutive pixels (one per lane, so every per-channel access of a wave is a
// 256-B coalesced row segment) x 4 channel groups (one per wave); each thread
// walks CPT channels.  The projection (~60 flops, 6 sincos) is recomputed per
// wave instead of being staged: it is far cheaper than a round trip.
//
// Roofline: HBM/L2 bound.  Algorithmic bytes per forward call:
//   P * ((N+2) * 4C + 4)   [fmap + N ref maps read once, cost written once,
//                           depth read once]; backward ~ P * (5*4C + 8) per ref.
#include <hip/hip_runtime.h>

#include "dro_common.hpp"

namespace dro {

#ifndef DRO_WARP_CPT
#define DRO_WARP_CPT 4
#endif
constexpr int kCPT = DRO_WARP_CPT;   // channels per thread
constexpr int kGroups = 4;     // channel groups (waves) per workgroup
constexpr int kGeoThreads = 256;

struct WarpArgs {
  const float* fmap;
  const float* fmap_ref;
  const float* depth;
  const float* K;
  const float* ref_K;
  const float* pose;
  int depth_mode, pose_mode;
  float min_disp, span;
  float scale;
  int do_scale;
  int B, N, C, h, w;
  int reduce_mean;
  int acc_fmap;      // backward: add into grad_fmap
  int acc_depth;     // backward: add into grad_depth
  int* cells;        // backward test hook: bilinear cell per (n, b, p) (pack_cell), or NULL
  int merge;         // backward: merge runs of lanes sharing a cell before the scatter (default 1;
                     // DRO_WARP_NOMERGE=1 for A/B measurements)
};

__device__ __forceinline__ void cams(const WarpArgs& a, int b, float ki[9], float kr[9]) {
  float k[9];
  scaled_K(a.K + 9 * b, a.scale, a.do_scale, k);
  K_inverse(k, ki);
  scaled_K(a.ref_K + 9 * b, a.scale, a.do_scale, kr);
}

// ------------------------------------------------------------------ forward
// SAMPLE = false: cost = (fmap - warped)^2 (mean over refs with reduce_mean);
// SAMPLE = true: the warped map itself (view_synthesis, camera_utils.py:23-56;
// fmap unused, out [N,B,C,h,w]).
template <bool SAMPLE>
__global__ __launch_bounds__(256) void warp_cost_fwd_kernel(WarpArgs a, float* __restrict__ cost) {
  const int P = a.h * a.w;
  const int p = blockIdx.x * kWave + (threadIdx.x & 63);
  const int b = blockIdx.z;
  const int c0 = (blockIdx.y * kGroups + (threadIdx.x >> 6)) * kCPT;
  if (p >= P || c0 >= a.C) return;
  const int cn = min(kCPT, a.C - c0);

  float ki[9], kr[9];
  cams(a, b, ki, kr);
  float dd;
  const float depth = decode_depth(a.depth[b * P + p], a.depth_mode, a.min_disp, a.span, &dd);
  const float u = (float)(p % a.w), v = (float)(p / a.w);

  float f[kCPT], acc[kCPT];
  const float* fm = SAMPLE ? nullptr : a.fmap + ((size_t)b * a.C + c0) * P + p;
#pragma unroll
  for (int c = 0; c < kCPT; ++c) {
    f[c] = (!SAMPLE && c < cn) ? fm[(size_t)c * P] : 0.f;
    acc[c] = 0.f;
  }
  const int ps = pose_stride(a.pose_mode);
  for (int n = 0; n < a.N; ++n) {
    float R[9], t[3];
    load_pose(a.pose + (size_t)(n * a.B + b) * ps, a.pose_mode, R, t);
    Proj q;
    project(ki, kr, R, t, u, v, depth, a.h, a.w, q);
    Taps T;
    bilinear_taps(q.ix, q.iy, a.h, a.w, T);
    const float* fr = a.fmap_ref + (((size_t)n * a.B + b) * a.C + c0) * P;
#pragma unroll
    for (int c = 0; c < kCPT; ++c) {
      if (c < cn) {
        const float* pl = fr + (size_t)c * P;
        float val = 0.f;
        if (T.ok[0]) val += pl[T.idx[0]] * T.wgt[0];
        if (T.ok[1]) val += pl[T.idx[1]] * T.wgt[1];
        if (T.ok[2]) val += pl[T.idx[2]] * T.wgt[2];
        if (T.ok[3]) val += pl[T.idx[3]] * T.wgt[3];
        if (SAMPLE) {
          cost[(((size_t)n * a.B + b) * a.C + c0 + c) * P + p] = val;
          continue;
        }
        const float d = f[c] - val;
        if (a.reduce_mean) {
          acc[c] += d * d;
        } else {
          cost[(((size_t)n * a.B + b) * a.C + c0 + c) * P + p] = d * d;
        }
      }
    }
  }
  if (!SAMPLE && a.reduce_mean) {
    float* out = cost + ((size_t)b * a.C + c0) * P + p;
    const float invN = (float)a.N;
#pragma unroll
    for (int c = 0; c < kCPT; ++c)
      if (c < cn) out[(size_t)c * P] = acc[c] / invN;
  }
}

// ------------------------------------------------------------------ backward: feature side
// d/dfmap, d/dfmap_ref (bilinear scatter, fp32 atomics) and the per-pixel
// sampling-position gradient gxy[n,b,p] = sum_c dL/dwarped * dwarped/d(ix,iy).
// SAMPLE: gcost is dL/dwarped [N,B,C,h,w] (view synthesis), no fmap.
template <bool SAMPLE>
__global__ __launch_bounds__(256) void warp_cost_bwd_feat_kernel(
    WarpArgs a, const float* __restrict__ gcost, float* __restrict__ gfmap,
    float* __restrict__ gfref, float* __restrict__ gxy) {
  // the block's kGroups waves share 64 pixels: their sampling-position
  // gradients are summed through LDS (fixed wave order) before one atomic pair
  // per pixel and block, instead of one per wave (those all hit one address)
  __shared__ float red[kGroups][kWave][2];
  const int P = a.h * a.w;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int p = blockIdx.x * kWave + lane;
  const int b = blockIdx.z;
  const int c0 = (blockIdx.y * kGroups + wave) * kCPT;
  const bool active = p < P && c0 < a.C;   // inactive lanes still join the block's barriers
  const int pp = active ? p : 0;
  const int cn = active ? min(kCPT, a.C - c0) : 0;
  const int cb = c0 < a.C ? c0 : 0;

  float ki[9], kr[9];
  cams(a, b, ki, kr);
  float dd;
  const float depth = decode_depth(a.depth[b * P + pp], a.depth_mode, a.min_disp, a.span, &dd);
  const float u = (float)(pp % a.w), v = (float)(pp / a.w);
  const float scaleN = a.reduce_mean ? 1.f / (float)a.N : 1.f;

  float f[kCPT], gf[kCPT], g[kCPT];
  const float* fm = SAMPLE ? nullptr : a.fmap + ((size_t)b * a.C + cb) * P + pp;
#pragma unroll
  for (int c = 0; c < kCPT; ++c) {
    f[c] = (!SAMPLE && c < cn) ? fm[(size_t)c * P] : 0.f;
    gf[c] = 0.f;
  }
  if (!SAMPLE && a.reduce_mean) {
    const float* gp = gcost + ((size_t)b * a.C + cb) * P + pp;
#pragma unroll
    for (int c = 0; c < kCPT; ++c) g[c] = (c < cn) ? gp[(size_t)c * P] * scaleN : 0.f;
  }
  const int ps = pose_stride(a.pose_mode);
  for (int n = 0; n < a.N; ++n) {
    if (SAMPLE || !a.reduce_mean) {
      const float* gp = gcost + (((size_t)n * a.B + b) * a.C + cb) * P + pp;
#pragma unroll
      for (int c = 0; c < kCPT; ++c) g[c] = (c < cn) ? gp[(size_t)c * P] : 0.f;
    }
    float R[9], t[3];
    load_pose(a.pose + (size_t)(n * a.B + b) * ps, a.pose_mode, R, t);
    Proj q;
    project(ki, kr, R, t, u, v, depth, a.h, a.w, q);
    Taps T;
    bilinear_taps(q.ix, q.iy, a.h, a.w, T);
    if (a.cells && blockIdx.y == 0 && wave == 0 && active)
      a.cells[(size_t)(n * a.B + b) * P + p] = pack_cell(q.ix, q.iy);
    const float* fr = a.fmap_ref + (((size_t)n * a.B + b) * a.C + cb) * P;
    float* gr = gfref ? gfref + (((size_t)n * a.B + b) * a.C + cb) * P : nullptr;
    const float omy = 1.f - T.ty, omx = 1.f - T.tx;
    float gix = 0.f, giy = 0.f;
    // Scatter contention: where the warp compresses the image (consecutive
    // pixels of the wave sampling one cell of the reference), up to 64 lanes'
    // atomics hit the same four addresses and serialise in L2 (measured: the
    // same launch 8 -> 69 us with the state of the network).  Lanes are
    // consecutive pixels, so lanes sharing a cell form runs: when the wave has
    // any, each run's contributions are summed by a segmented suffix scan
    // over the lanes and only the run's first lane issues the atomics.
    const bool taps_in = T.ok[0] || T.ok[1] || T.ok[2] || T.ok[3];
    // the cell (floor ix, floor iy) in [-1, w-1] x [-1, h-1] when any tap is in
    // the image; T.idx[0] alone is not unique there: cell (-1, y+1) and cell
    // (w-1, y) share it, and a row's last and the next row's first pixel are
    // neighbouring lanes that hit exactly that pair at the image's side borders
    const int key = (taps_in && cn > 0)
                        ? ((int)floorf(q.iy) + 1) * (a.w + 1) + (int)floorf(q.ix) + 1 : -(lane + 1);
    const int key_next = __shfl_down(key, 1, kWave);
    const int key_prev = __shfl_up(key, 1, kWave);
    const bool run_cont = lane < kWave - 1 && key_next == key;    // the run goes on past this lane
    const bool merge = a.merge && gr != nullptr && __any(run_cont);
    const bool head = lane == 0 || key_prev != key;
    unsigned addm = 0u;                                            // scan steps that add the next partial
    if (merge) {
      bool e = !run_cont;
#pragma unroll
      for (int s_ = 0; s_ < 6; ++s_) {
        const bool en = __shfl_down((int)e, 1 << s_, kWave) != 0;
        if (!e) {
          addm |= 1u << s_;
          e = en;
        }
      }
    }
#pragma unroll
    for (int c = 0; c < kCPT; ++c) {
      float gw = 0.f;
      if (c < cn) {
        const float* pl = fr + (size_t)c * P;
        const float v0 = T.ok[0] ? pl[T.idx[0]] : 0.f;
        const float v1 = T.ok[1] ? pl[T.idx[1]] : 0.f;
        const float v2 = T.ok[2] ? pl[T.idx[2]] : 0.f;
        const float v3 = T.ok[3] ? pl[T.idx[3]] : 0.f;
        const float val = v0 * T.wgt[0] + v1 * T.wgt[1] + v2 * T.wgt[2] + v3 * T.wgt[3];
        const float gd = SAMPLE ? 0.f : 2.f * (f[c] - val) * g[c];  // d cost / d fmap
        gf[c] += gd;
        gw = SAMPLE ? g[c] : -gd;                     // d loss / d warped
        if (gr && !merge) {
          float* gpl = gr + (size_t)c * P;
          if (T.ok[0]) atomicAdd(gpl + T.idx[0], gw * T.wgt[0]);
          if (T.ok[1]) atomicAdd(gpl + T.idx[1], gw * T.wgt[1]);
          if (T.ok[2]) atomicAdd(gpl + T.idx[2], gw * T.wgt[2]);
          if (T.ok[3]) atomicAdd(gpl + T.idx[3], gw * T.wgt[3]);
        }
        gix += gw * ((v1 - v0) * omy + (v3 - v2) * T.ty);
        giy += gw * ((v2 - v0) * omx + (v3 - v1) * T.tx);
      }
      if (merge) {                                    // wave-uniform: every lane shuffles
        float w4[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) w4[q] = gw * T.wgt[q];
#pragma unroll
        for (int s_ = 0; s_ < 6; ++s_) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float o = __shfl_down(w4[q], 1 << s_, kWave);
            if (addm & (1u << s_)) w4[q] += o;
          }
        }
        if (head && c < cn) {
          float* gpl = gr + (size_t)c * P;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (T.ok[q]) atomicAdd(gpl + T.idx[q], w4[q]);
        }
      }
    }
    if (gxy) {
      red[wave][lane][0] = gix;
      red[wave][lane][1] = giy;
      __syncthreads();
      if (wave == 0 && p < P) {
        float sx = 0.f, sy = 0.f;
#pragma unroll
        for (int w = 0; w < kGroups; ++w) {
          sx += red[w][lane][0];
          sy += red[w][lane][1];
        }
        float* dst = gxy + ((size_t)(n * a.B + b) * P + p) * 2;
        atomicAdd(dst, sx);
        atomicAdd(dst + 1, sy);
      }
      __syncthreads();
    }
  }
  if (!SAMPLE && gfmap) {
    float* out = gfmap + ((size_t)b * a.C + cb) * P + pp;
#pragma unroll
    for (int c = 0; c < kCPT; ++c)
      if (c < cn) out[(size_t)c * P] = a.acc_fmap ? out[(size_t)c * P] + gf[c] : gf[c];
  }
}

// ------------------------------------------------------------------ channels-last reference maps
// The same cost and backward with the reference maps channel-contiguous
// ([N,B,h,w,C], ref_layout 1).  The NCHW kernels above put one pixel on each
// lane: a tap gather (and a scatter atomic) of a wave is coalesced only where
// neighbouring pixels sample neighbouring reference pixels.  Where the warp
// shears or folds the reference -- a state the untrained recurrence reaches
// within a few steps -- every lane's tap lands on its own cache line, and the
// backward went from 12 to 90 us per launch at the metric config
// (tools/warp_state_probe.py: pixels per occupied cell 1.7, no compression,
// only the locality is gone).  Here the lanes span 64 channels of ONE pixel:
// each tap gather is one 256-B row and each scatter instruction one coalesced
// row of atomics, whatever the geometry.  The target-side maps (fmap, the
// incoming gradient, cost, d fmap) stay NCHW and pass through an LDS tile of
// kClTP pixels x 64 channels with pixel-contiguous (coalesced) global accesses.
// The projection is computed once per (pixel, ref) by the tile's first kClTP
// threads; tap weights of out-of-image taps are 0 with clamped indices (the
// sum is bit-identical to the guarded one, fma(x, 0, v) == v).
#ifndef DRO_WARP_CL_TP
#define DRO_WARP_CL_TP 8
#endif
// pixels per block (kClTP / 4 per wave).  Measured on recorded training states
// (tools/ab_warp_tile.sh, rocprof per launch): 4 / 8 / 16 / 32 pixels ->
// backward 17.8 / 11.0-11.5 / 13.6 / 22.8 us, forward 12.3 / 9.3-9.4 / 10.7 / 14.6 us
constexpr int kClTP = DRO_WARP_CL_TP;
constexpr int kClCH = kWave;              // channels per block (one per lane)
constexpr int kClPPW = kClTP / 4;         // pixels per wave
constexpr int kClNC = 4;                  // refs whose taps one phase computes (kClNC * kClTP threads)

struct ClTaps {
  int idx[kClTP][4];
  float wgt[kClTP][4];
  float tx[kClTP], ty[kClTP];
  int key[kClTP];                         // bilinear cell, -1 - j when no tap is in the image
  int ok[kClTP];                          // in-image taps (bit e), a property of the cell
};

// taps of refs n0 .. n0 + nc - 1: thread t < nc * kClTP takes (n0 + t / kClTP, pixel t % kClTP)
__device__ __forceinline__ void cl_taps(const WarpArgs& a, int b, int n0, int nc, int p0, int pn,
                                        int cells_block, ClTaps* L) {
  const int t = threadIdx.x;
  if (t >= nc * kClTP) return;
  const int dn = t / kClTP, j = t - dn * kClTP, n = n0 + dn;
  const int P = a.h * a.w;
  int key = -1 - j;
  float wg[4] = {0.f, 0.f, 0.f, 0.f}, tx = 0.f, ty = 0.f;
  int ix4[4] = {0, 0, 0, 0}, okm = 0;
  if (j < pn) {
    const int p = p0 + j;
    float ki[9], kr[9];
    cams(a, b, ki, kr);
    float dd;
    const float depth = decode_depth(a.depth[b * P + p], a.depth_mode, a.min_disp, a.span, &dd);
    float R[9], tt[3];
    load_pose(a.pose + (size_t)(n * a.B + b) * pose_stride(a.pose_mode), a.pose_mode, R, tt);
    Proj q;
    project(ki, kr, R, tt, (float)(p % a.w), (float)(p / a.w), depth, a.h, a.w, q);
    Taps T;
    bilinear_taps(q.ix, q.iy, a.h, a.w, T);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      ix4[e] = T.ok[e] ? T.idx[e] : 0;
      wg[e] = T.ok[e] ? T.wgt[e] : 0.f;
      okm |= T.ok[e] ? 1 << e : 0;
    }
    tx = T.tx;
    ty = T.ty;
    if (okm) key = ((int)floorf(q.iy) + 1) * (a.w + 1) + (int)floorf(q.ix) + 1;
    if (a.cells && cells_block) a.cells[(size_t)(n * a.B + b) * P + p] = pack_cell(q.ix, q.iy);
  }
  ClTaps& Ln = L[dn];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    Ln.idx[j][e] = ix4[e];
    Ln.wgt[j][e] = wg[e];
  }
  Ln.tx[j] = tx;
  Ln.ty[j] = ty;
  Ln.key[j] = key;
  Ln.ok[j] = okm;
}

// tile[c][j] <- src[c * P + j] (c < cn, j < pn; 0 elsewhere), scaled
template <int CB = kClCH>
__device__ __forceinline__ void cl_load_tile(float (*tile)[kClTP + 1], const float* __restrict__ src, int P,
                                             int cn, int pn, float scale) {
  for (int i = threadIdx.x; i < CB * kClTP; i += blockDim.x) {
    const int c = i / kClTP, j = i - c * kClTP;
    tile[c][j] = (c < cn && j < pn) ? src[(size_t)c * P + j] * scale : 0.f;
  }
}

template <int CB = kClCH>
__device__ __forceinline__ void cl_store_tile(float (*tile)[kClTP + 1], float* __restrict__ dst, int P, int cn,
                                              int pn, bool add) {
  for (int i = threadIdx.x; i < CB * kClTP; i += blockDim.x) {
    const int c = i / kClTP, j = i - c * kClTP;
    if (c < cn && j < pn) {
      float* o = dst + (size_t)c * P + j;
      *o = add ? *o + tile[c][j] : tile[c][j];
    }
  }
}

// Sums of 8 per-lane values over the wave in 10 shuffles (a reduce-scatter
// butterfly: halve the value set at lane distances 32, 16, 8, then sum within
// 8 lanes): lane l ends with the total of value l >> 3 when (l & 7) == 0.
__device__ __forceinline__ float wave_sum8(const float (&v)[8]) {
  const int lane = threadIdx.x & 63;
  float a4[4], a2[2], a1;
  const bool u32 = lane & 32, u16 = lane & 16, u8 = lane & 8;
#pragma unroll
  for (int i = 0; i < 4; ++i) {             // keep 0..3 (lower half) or 4..7 (upper)
    const float send = u32 ? v[i] : v[i + 4];
    const float mine = u32 ? v[i + 4] : v[i];
    a4[i] = mine + __shfl_xor(send, 32, kWave);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float send = u16 ? a4[i] : a4[i + 2];
    const float mine = u16 ? a4[i + 2] : a4[i];
    a2[i] = mine + __shfl_xor(send, 16, kWave);
  }
  {
    const float send = u8 ? a2[0] : a2[1];
    const float mine = u8 ? a2[1] : a2[0];
    a1 = mine + __shfl_xor(send, 8, kWave);
  }
#pragma unroll
  for (int o = 4; o >= 1; o >>= 1) a1 += __shfl_xor(a1, o, kWave);
  return a1;
}

__global__ __launch_bounds__(256) void warp_cost_fwd_cl_kernel(WarpArgs a, float* __restrict__ cost) {
  __shared__ float f_l[kClCH][kClTP + 1];
  __shared__ float o_l[kClCH][kClTP + 1];
  __shared__ ClTaps L[kClNC];
  const int P = a.h * a.w;
  const int p0 = blockIdx.x * kClTP, c0 = blockIdx.y * kClCH, b = blockIdx.z;
  const int cn = min(kClCH, a.C - c0), pn = min(kClTP, P - p0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  cl_load_tile(f_l, a.fmap + ((size_t)b * a.C + c0) * P + p0, P, cn, pn, 1.f);
  float acc[kClPPW];
#pragma unroll
  for (int k = 0; k < kClPPW; ++k) acc[k] = 0.f;
  for (int n0 = 0; n0 < a.N; n0 += kClNC) {
    const int nc = min(kClNC, a.N - n0);
    __syncthreads();                        // previous taps / output tile consumed
    cl_taps(a, b, n0, nc, p0, pn, 0, L);
    __syncthreads();
    for (int dn = 0; dn < nc; ++dn) {
      const int n = n0 + dn;
      const ClTaps& T = L[dn];
      const float* fr = a.fmap_ref + ((size_t)(n * a.B + b) * P) * a.C + c0 + lane;
#pragma unroll
      for (int k = 0; k < kClPPW; ++k) {
        const int j = wave * kClPPW + k;
        if (j < pn && lane < cn) {
          float val = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e)   // in-image taps only (zeros padding: an Inf / NaN elsewhere stays out)
            if ((T.ok[j] >> e) & 1) val += fr[(size_t)T.idx[j][e] * a.C] * T.wgt[j][e];
          const float d = f_l[lane][j] - val;
          if (a.reduce_mean)
            acc[k] += d * d;
          else
            o_l[lane][j] = d * d;
        }
      }
      if (!a.reduce_mean) {
        __syncthreads();
        cl_store_tile(o_l, cost + (((size_t)n * a.B + b) * a.C + c0) * P + p0, P, cn, pn, false);
        __syncthreads();
      }
    }
  }
  if (a.reduce_mean) {
    const float invN = (float)a.N;
#pragma unroll
    for (int k = 0; k < kClPPW; ++k) o_l[lane][wave * kClPPW + k] = acc[k] / invN;
    __syncthreads();
    cl_store_tile(o_l, cost + ((size_t)b * a.C + c0) * P + p0, P, cn, pn, false);
  }
}

// d/dfmap (NCHW, through the tile), d/dfmap_ref (channels-last, coalesced
// atomics; consecutive pixels of a wave that share a bilinear cell are summed
// in registers first) and the sampling-position gradient (the channel sums of
// a wave's pixels in one butterfly).  A block covers NCH x 64 channels.
// GEO (every channel in the block, C <= NCH * 64): the sampling-position
// gradient of each pixel is complete in the block, so it is chained through
// the projection right here -- d depth per pixel (summed over the refs) and
// fp64 pose partials per (ref, image, block) -- with no gxy buffer, zero-fill,
// atomics or geometry launch.  Otherwise gxy gets one atomic per value and
// channel block and warp_cost_bwd_geo_kernel follows.
template <int NCH, bool GEO>
__global__ __launch_bounds__(256) void warp_cost_bwd_feat_cl_kernel(WarpArgs a, const float* __restrict__ gcost,
                                                                    float* __restrict__ gfmap,
                                                                    float* __restrict__ gfref,
                                                                    float* __restrict__ gxy,
                                                                    float* __restrict__ gdepth,
                                                                    double* __restrict__ partial) {
  constexpr int CB = NCH * kClCH;           // channels per block
  __shared__ float f_l[CB][kClTP + 1];
  __shared__ float g_l[kClNC][CB][kClTP + 1];
  __shared__ ClTaps L[kClNC];
  __shared__ float gx_l[GEO ? kClNC : 1][kClTP][2];
  __shared__ float gd_l[GEO ? kClNC : 1][kClTP];
  const int P = a.h * a.w;
  const int p0 = blockIdx.x * kClTP, c0 = blockIdx.y * CB, b = blockIdx.z;
  const int cn = min(CB, a.C - c0), pn = min(kClTP, P - p0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  cl_load_tile<CB>(f_l, a.fmap + ((size_t)b * a.C + c0) * P + p0, P, cn, pn, 1.f);
  if (a.reduce_mean)
    cl_load_tile<CB>(g_l[0], gcost + ((size_t)b * a.C + c0) * P + p0, P, cn, pn, 1.f / (float)a.N);
  float gf[kClPPW][NCH];
#pragma unroll
  for (int k = 0; k < kClPPW; ++k)
#pragma unroll
    for (int h = 0; h < NCH; ++h) gf[k][h] = 0.f;
  float gdep = 0.f;                         // GEO: thread j < kClTP, d loss / d depth of pixel j
  for (int n0 = 0; n0 < a.N; n0 += kClNC) {
    const int nc = min(kClNC, a.N - n0);
    __syncthreads();
    if (!a.reduce_mean)
      for (int dn = 0; dn < nc; ++dn)
        cl_load_tile<CB>(g_l[dn], gcost + (((size_t)(n0 + dn) * a.B + b) * a.C + c0) * P + p0, P, cn, pn, 1.f);
    cl_taps(a, b, n0, nc, p0, pn, blockIdx.y == 0, L);
    __syncthreads();
    for (int dn = 0; dn < nc; ++dn) {
      const ClTaps& T = L[dn];
      const float (*g_t)[kClTP + 1] = g_l[a.reduce_mean ? 0 : dn];
      const size_t img = (size_t)((n0 + dn) * a.B + b) * P;
      const float* fr = a.fmap_ref + img * a.C + c0 + lane;
      float* gr = gfref ? gfref + img * a.C + c0 + lane : nullptr;
      int pkey = -1;                        // cell of the pending scatter (wave-uniform)
      int pidx[4] = {0, 0, 0, 0}, pok = 0;
      float pend[NCH][4];
#pragma unroll
      for (int h = 0; h < NCH; ++h)
#pragma unroll
        for (int e = 0; e < 4; ++e) pend[h][e] = 0.f;
      float gxyv[2 * kClPPW];
#pragma unroll
      for (int k = 0; k < kClPPW; ++k) {
        const int j = wave * kClPPW + k;
        float gw[NCH], sx = 0.f, sy = 0.f;
        const float ty = T.ty[j], tx = T.tx[j];
#pragma unroll
        for (int h = 0; h < NCH; ++h) {
          const int cl = h * kClCH + lane;
          const bool live = cl < cn && j < pn;
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)   // out-of-image taps read 0 (their values enter d/d(ix,iy))
            v[e] = (live && ((T.ok[j] >> e) & 1)) ? fr[(size_t)T.idx[j][e] * a.C + h * kClCH] : 0.f;
          gw[h] = 0.f;
          if (live) {
            // one expression, as warp_cost_bwd_feat_kernel (the same contraction)
            const float val = v[0] * T.wgt[j][0] + v[1] * T.wgt[j][1] + v[2] * T.wgt[j][2] + v[3] * T.wgt[j][3];
            const float gd = 2.f * (f_l[cl][j] - val) * g_t[cl][j];
            gf[k][h] += gd;
            gw[h] = -gd;
          }
          sx += gw[h] * ((v[1] - v[0]) * (1.f - ty) + (v[3] - v[2]) * ty);
          sy += gw[h] * ((v[2] - v[0]) * (1.f - tx) + (v[3] - v[1]) * tx);
        }
        gxyv[2 * k] = sx;
        gxyv[2 * k + 1] = sy;
        if (gr && j < pn) {
          const int key = T.key[j];
          if (key != pkey) {                // flush the previous cell's sums
            if (pkey >= 0) {
#pragma unroll
              for (int h = 0; h < NCH; ++h)
                if (h * kClCH + lane < cn)
#pragma unroll
                  for (int e = 0; e < 4; ++e)
                    if ((pok >> e) & 1) atomicAdd(gr + (size_t)pidx[e] * a.C + h * kClCH, pend[h][e]);
            }
            pkey = key;
            pok = T.ok[j];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              pidx[e] = T.idx[j][e];
#pragma unroll
              for (int h = 0; h < NCH; ++h) pend[h][e] = 0.f;
            }
          }
#pragma unroll
          for (int h = 0; h < NCH; ++h)
#pragma unroll
            for (int e = 0; e < 4; ++e) pend[h][e] += gw[h] * T.wgt[j][e];
        }
      }
      if (gr && pkey >= 0) {
#pragma unroll
        for (int h = 0; h < NCH; ++h)
          if (h * kClCH + lane < cn)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if ((pok >> e) & 1) atomicAdd(gr + (size_t)pidx[e] * a.C + h * kClCH, pend[h][e]);
      }
      if (GEO || gxy) {   // 8 values (4 pixels x (ix, iy)) per butterfly
#pragma unroll
        for (int g0 = 0; g0 < 2 * kClPPW; g0 += 8) {
          float v8[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) v8[i] = g0 + i < 2 * kClPPW ? gxyv[g0 + i] : 0.f;
          const float sum = wave_sum8(v8);
          const int vi = g0 + (lane >> 3), j = wave * kClPPW + (vi >> 1);
          if ((lane & 7) == 0 && vi < 2 * kClPPW && j < pn) {
            if (GEO)
              gx_l[dn][j][vi & 1] = sum;
            else
              atomicAdd(gxy + (img + p0 + j) * 2 + (vi & 1), sum);
          }
        }
      }
    }
    if (GEO) {
      __syncthreads();                      // every ref's gx_l of this chunk written
      // thread t = dn * kClTP + j: pixel j's sampling-position gradient for ref
      // n0 + dn chained through the projection (as warp_cost_bwd_geo_kernel)
      const int t = threadIdx.x, dn = t / kClTP, j = t - dn * kClTP;
      if (t < kClNC * kClTP) {              // whole 8-lane groups (wave 0) join the shuffles
        float acc[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) acc[k] = 0.f;
        float gd = 0.f;
        if (dn < nc && j < pn) {
          const int p = p0 + j, n = n0 + dn;
          float ki[9], kr[9];
          cams(a, b, ki, kr);
          float dd;
          const float depth = decode_depth(a.depth[b * P + p], a.depth_mode, a.min_disp, a.span, &dd);
          float R[9], tt[3];
          load_pose(a.pose + (size_t)(n * a.B + b) * pose_stride(a.pose_mode), a.pose_mode, R, tt);
          Proj q;
          project(ki, kr, R, tt, (float)(p % a.w), (float)(p / a.w), depth, a.h, a.w, q);
          gd = project_backward_pt(q, kr, R, tt, depth, gx_l[dn][j][0], gx_l[dn][j][1], acc, acc + 9);
        }
        if (dn < nc) gd_l[dn][j] = gd;
        if (partial) {                      // the ref's 8 pixels in fixed order (lanes j of the group)
          double d12[12];
#pragma unroll
          for (int k = 0; k < 12; ++k) {
            double v = acc[k];
#pragma unroll
            for (int o = 1; o < kClTP; o <<= 1) v += __shfl_xor(v, o, kWave);
            d12[k] = v;
          }
          if (j == 0 && dn < nc) {
            double* dst = partial + ((size_t)((n0 + dn) * a.B + b) * gridDim.x + blockIdx.x) * 12;
#pragma unroll
            for (int k = 0; k < 12; ++k) dst[k] = d12[k];
          }
        }
      }
      __syncthreads();
      if (t < kClTP)
        for (int d2 = 0; d2 < nc; ++d2) gdep += gd_l[d2][t];   // refs in order
    }
  }
  if (GEO && gdepth && threadIdx.x < pn) {
    float dd;
    decode_depth(a.depth[b * P + p0 + threadIdx.x], a.depth_mode, a.min_disp, a.span, &dd);
    float* gq = gdepth + b * P + p0 + threadIdx.x;
    *gq = a.acc_depth ? *gq + gdep * dd : gdep * dd;
  }
  if (gfmap) {
    __syncthreads();                        // f_l reused as the output tile
#pragma unroll
    for (int k = 0; k < kClPPW; ++k)
#pragma unroll
      for (int h = 0; h < NCH; ++h) f_l[h * kClCH + lane][wave * kClPPW + k] = gf[k][h];
    __syncthreads();
    cl_store_tile<CB>(f_l, gfmap + ((size_t)b * a.C + c0) * P + p0, P, cn, pn, a.acc_fmap != 0);
  }
}

// ------------------------------------------------------------------ backward: geometry side
// One thread per (b, pixel): chain gxy through the projection to the depth
// input (summed over refs, no atomics) and to per-workgroup pose partials.
__global__ __launch_bounds__(kGeoThreads) void warp_cost_bwd_geo_kernel(
    WarpArgs a, const float* __restrict__ gxy, float* __restrict__ gdepth,
    double* __restrict__ partial) {
  __shared__ double scratch[12 * (kGeoThreads / kWave)];
  const int P = a.h * a.w;
  const int p = blockIdx.x * kGeoThreads + threadIdx.x;
  const int b = blockIdx.y;
  const bool live = p < P;
  float ki[9], kr[9];
  cams(a, b, ki, kr);
  float dd = 0.f, depth = 0.f;
  if (live) depth = decode_depth(a.depth[b * P + p], a.depth_mode, a.min_disp, a.span, &dd);
  const float u = live ? (float)(p % a.w) : 0.f, v = live ? (float)(p / a.w) : 0.f;
  const int ps = pose_stride(a.pose_mode);
  float gd_total = 0.f;
  for (int n = 0; n < a.N; ++n) {
    float R[9], t[3];
    load_pose(a.pose + (size_t)(n * a.B + b) * ps, a.pose_mode, R, t);
    float acc[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) acc[k] = 0.f;
    if (live) {
      Proj q;
      project(ki, kr, R, t, u, v, depth, a.h, a.w, q);
      const float* g = gxy + ((size_t)(n * a.B + b) * P + p) * 2;
      gd_total += project_backward_pt(q, kr, R, t, depth, g[0], g[1], acc, acc + 9);
    }
    if (partial) {
      double sum[12];
      block_sum_d<12>(acc, sum, scratch);
      if (threadIdx.x == 0) {
        double* dst = partial + (((size_t)n * a.B + b) * gridDim.x + blockIdx.x) * 12;
#pragma unroll
        for (int k = 0; k < 12; ++k) dst[k] = sum[k];
      }
    }
  }
  if (gdepth && live) gdepth[b * P + p] = a.acc_depth ? gdepth[b * P + p] + gd_total * dd : gd_total * dd;
}

// One 256-thread block per pose: threads 0..239 = 20 row groups x 12
// components stride over the pose's [nblk][12] partials (coalesced), then the
// 20 group sums are added in a fixed order (deterministic).  The fused cost
// backward and the photometric loss hand in 240 partials per pose: with 5
// groups of one wave each group walked a 48-load dependent chain.
__global__ __launch_bounds__(256) void pose_finalize_kernel(const double* __restrict__ partial, int nblk,
                                                            int npose, const float* __restrict__ pose,
                                                            int pose_mode, float* __restrict__ gpose) {
  constexpr int G = 20;   // row groups
  __shared__ double sh[G * 12];
  __shared__ double s[12];
  const int i = blockIdx.x, t = threadIdx.x;
  if (i >= npose) return;
  if (t < G * 12) {
    const int comp = t % 12, g = t / 12;
    const double* src = partial + (size_t)i * nblk * 12 + comp;
    double v = 0.0;
    for (int j = g; j < nblk; j += G) v += src[(size_t)j * 12];
    sh[t] = v;
  }
  __syncthreads();
  if (t < 12) {
    double v = 0.0;
#pragma unroll
    for (int g = 0; g < G; ++g) v += sh[g * 12 + t];
    s[t] = v;
  }
  __syncthreads();
  if (t == 0) {
    double r[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) r[k] = s[k];
    const int ps = pose_stride(pose_mode);
    store_pose_grad_d(pose + (size_t)i * ps, pose_mode, r, r + 9, gpose + (size_t)i * ps);
  }
}

// ------------------------------------------------------------------ plane sweep (forward only)
// Sweep kernel: lanes run along 64 consecutive pixels (every tap gather of a
// wave touches consecutive addresses, every store is a 256-B row segment),
// each of the 4 waves owns kSweepCPT channels of one (b, plane).  The
// projection is computed once per pixel for all of a wave's channels; tap
// loads are unconditional from clamped indices with zero weights for
// out-of-image taps (fma(x, 0, v) == v: the sum equals the guarded one bit
// for bit), issued 8 channels at a time.  HBM bound: the volume write
// (4*B*D*C*P bytes) dominates the traffic.
constexpr int kSweepCPT = 32;

__global__ __launch_bounds__(256) void plane_sweep_wide_kernel(WarpArgs a, const float* __restrict__ disp,
                                                               int D, float* __restrict__ cost) {
  const int P = a.h * a.w;
  const int p = blockIdx.x * kWave + (threadIdx.x & 63);
  const int b = blockIdx.z / D, d = blockIdx.z - (blockIdx.z / D) * D;
  const int c0 = (blockIdx.y * 4 + (threadIdx.x >> 6)) * kSweepCPT;
  if (p >= P || c0 >= a.C) return;
  const int cn = min(kSweepCPT, a.C - c0);
  float ki[9], kr[9];
  cams(a, b, ki, kr);
  float dd;
  const float depth = decode_depth(disp[d], DRO_DEPTH_DISP, a.min_disp, a.span, &dd);
  float R[9], t[3];
  load_pose(a.pose + (size_t)b * pose_stride(a.pose_mode), a.pose_mode, R, t);
  Proj pr;
  project(ki, kr, R, t, (float)(p % a.w), (float)(p / a.w), depth, a.h, a.w, pr);
  Taps T;
  bilinear_taps(pr.ix, pr.iy, a.h, a.w, T);
  int idx[4];
  float wgt[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    idx[e] = T.ok[e] ? T.idx[e] : 0;
    wgt[e] = T.ok[e] ? T.wgt[e] : 0.f;
  }
  const float* fm = a.fmap + ((size_t)b * a.C + c0) * P + p;
  const float* fr = a.fmap_ref + ((size_t)b * a.C + c0) * P;
  float* out = cost + (((size_t)b * D + d) * a.C + c0) * P + p;
  for (int cb = 0; cb < cn; cb += 8) {
    float f[8], v[8][4];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int cc = min(cb + c, cn - 1);
      const float* pl = fr + (size_t)cc * P;
      f[c] = fm[(size_t)cc * P];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[c][e] = pl[idx[e]];
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float val = 0.f;
      val += v[c][0] * wgt[0];
      val += v[c][1] * wgt[1];
      val += v[c][2] * wgt[2];
      val += v[c][3] * wgt[3];
      const float df = f[c] - val;
      // streaming volume: non-temporal stores keep it out of L2's way
      if (cb + c < cn) __builtin_nontemporal_store(df * df, out + (size_t)(cb + c) * P);
    }
  }
}

// LDS variant (round 4): a block owns CG channels of one batch image and DG
// planes.  The CG reference channel planes (CG * h * w floats, <= 64 KB) are
// staged into LDS once with 16-B loads and serve every plane and pixel of the
// block, so the tap gathers are ds_read_b32 instead of global gathers; each
// thread takes 4 consecutive pixels (one projection each per plane), reads the
// target features as one 16-B load per channel and writes the 4 costs as one
// 16-B non-temporal store.  Same arithmetic as plane_sweep_wide_kernel (taps
// in nw, ne, sw, se order; zero weights for out-of-image taps), so the volume
// is bit-identical to one warp_cost call per plane.
typedef float v4f __attribute__((ext_vector_type(4)));

template <int CG, bool NT>
__global__ __launch_bounds__(1024) void plane_sweep_lds_kernel(WarpArgs a, const float* __restrict__ disp, int D,
                                                              int DG, float* __restrict__ cost) {
  extern __shared__ float4 lds4[];
  float* fr_l = reinterpret_cast<float*>(lds4);
  const int P = a.h * a.w, P4 = P >> 2;
  const int ncg = a.C / CG, ndg = (D + DG - 1) / DG;
  // block -> (b, plane group, channel group); channel groups of one plane
  // group are adjacent (they share the projections' inputs in L2)
  int blk = blockIdx.x;
  const int cg = blk % ncg;
  blk /= ncg;
  const int dg = blk % ndg;
  const int b = blk / ndg;
  const int c0 = cg * CG;
  {   // stage fref[b, c0 .. c0+CG) (contiguous) into LDS
    const float4* src = reinterpret_cast<const float4*>(a.fmap_ref + ((size_t)b * a.C + c0) * P);
    for (int i = threadIdx.x; i < CG * P4; i += blockDim.x) lds4[i] = src[i];
  }
  __syncthreads();
  float ki[9], kr[9];
  cams(a, b, ki, kr);
  float R[9], t[3];
  load_pose(a.pose + (size_t)b * pose_stride(a.pose_mode), a.pose_mode, R, t);
  const float4* fm4 = reinterpret_cast<const float4*>(a.fmap + ((size_t)b * a.C + c0) * P);
  const int d_end = min(D, (dg + 1) * DG);
  // 1024-thread blocks: two planes side by side, 512 threads each
  const int lanes = blockDim.x > 512 ? 512 : blockDim.x, pp = threadIdx.x / lanes, tq = threadIdx.x - pp * lanes;
  const int pstep = blockDim.x / lanes;
  for (int d = dg * DG + pp; d < d_end; d += pstep) {
    float dd;
    const float depth = decode_depth(disp[d], DRO_DEPTH_DISP, a.min_disp, a.span, &dd);
    v4f* out4 = reinterpret_cast<v4f*>(cost + (((size_t)b * D + d) * a.C + c0) * P);
    for (int q = tq; q < P4; q += lanes) {
      int idx[4][4];
      float wgt[4][4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = 4 * q + k;
        Proj pr;
        project(ki, kr, R, t, (float)(p % a.w), (float)(p / a.w), depth, a.h, a.w, pr);
        Taps T;
        bilinear_taps(pr.ix, pr.iy, a.h, a.w, T);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          idx[k][e] = T.ok[e] ? T.idx[e] : 0;
          wgt[k][e] = T.ok[e] ? T.wgt[e] : 0.f;
        }
      }
#pragma unroll 2
      for (int c = 0; c < CG; ++c) {
        const float* pl = fr_l + c * P;
        const float4 f = fm4[(size_t)c * P4 + q];
        const float fv[4] = {f.x, f.y, f.z, f.w};
        float o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float val = 0.f;
          val += pl[idx[k][0]] * wgt[k][0];
          val += pl[idx[k][1]] * wgt[k][1];
          val += pl[idx[k][2]] * wgt[k][2];
          val += pl[idx[k][3]] * wgt[k][3];
          const float df = fv[k] - val;
          o[k] = df * df;
        }
        const v4f ov = {o[0], o[1], o[2], o[3]};
        if (NT)
          __builtin_nontemporal_store(ov, out4 + (size_t)c * P4 + q);
        else
          out4[(size_t)c * P4 + q] = ov;
      }
    }
  }
}

int launch_pose_finalize(const double* partial, int nblk, int npose, const float* pose,
                         int pose_mode, float* gpose, hipStream_t s) {
  if (npose <= 0) return 0;
  hipLaunchKernelGGL(pose_finalize_kernel, dim3(npose), dim3(256), 0, s, partial, nblk,
                     npose, pose, pose_mode, gpose);
  return launch_status("pose_finalize_kernel launch failed");
}

static int check_common(const float* fmap, const float* fmap_ref, const float* K,
                        const float* ref_K, const float* pose, int pose_mode, int B, int N, int C,
                        int h, int w) {
  if (!fmap || !fmap_ref || !K || !ref_K || !pose) {
    set_error("warp_cost: NULL input pointer");
    return DRO_E_NULL;
  }
  if (B < 1 || N < 1 || C < 1 || h < 2 || w < 2 || (long long)h * w > (1LL << 30)) {
    set_error("warp_cost: sizes out of range (need B,N,C >= 1, h,w >= 2)");
    return DRO_E_SHAPE;
  }
  if (pose_mode != DRO_POSE_EULER && pose_mode != DRO_POSE_MATRIX) {
    set_error("warp_cost: unknown pose_mode");
    return DRO_E_MODE;
  }
  return DRO_OK;
}

static WarpArgs make_args(const float* fmap, const float* fmap_ref, const float* depth,
                          int depth_mode, float min_disp, float max_disp, const float* K,
                          const float* ref_K, float scale, const float* pose, int pose_mode, int B,
                          int N, int C, int h, int w, int reduce_mean) {
  WarpArgs a;
  a.acc_fmap = 0;
  a.acc_depth = 0;
  a.cells = nullptr;
  a.fmap = fmap;
  a.fmap_ref = fmap_ref;
  a.depth = depth;
  a.K = K;
  a.ref_K = ref_K;
  a.pose = pose;
  a.depth_mode = depth_mode;
  a.pose_mode = pose_mode;
  a.min_disp = min_disp;
  a.span = max_disp - min_disp;
  a.scale = scale;
  a.do_scale = scale != 1.0f;
  a.B = B;
  a.N = N;
  a.C = C;
  a.h = h;
  a.w = w;
  a.reduce_mean = reduce_mean;
  return a;
}

}  // namespace dro

using namespace dro;

extern "C" size_t dro_warp_cost_workspace_bytes(int B, int N, int h, int w) {
  const size_t P = (size_t)h * w;
  const size_t nblk = (P + kGeoThreads - 1) / kGeoThreads;
  // gxy (float), then the fp64 pose partials (8-byte aligned: N*B*P*2 floats is even);
  // the fused channels-last backward: fp64 pose partials per pixel tile only
  const size_t split = (size_t)N * B * P * 2 * sizeof(float) + (size_t)N * B * nblk * 12 * sizeof(double);
  const size_t fused = (size_t)N * B * ((P + kClTP - 1) / kClTP) * 12 * sizeof(double);
  return split > fused ? split : fused;
}

extern "C" int dro_warp_cost_forward(const float* fmap, const float* fmap_ref, const float* depth,
                                     int depth_mode, float min_disp, float max_disp,
                                     const float* K, const float* ref_K, float scale,
                                     const float* pose, int pose_mode, int B, int N, int C, int h,
                                     int w, int reduce_mean, int ref_layout, float* cost, void* stream) {
  int st = check_common(fmap, fmap_ref, K, ref_K, pose, pose_mode, B, N, C, h, w);
  if (st) return st;
  if (!depth || !cost) {
    set_error("warp_cost_forward: NULL depth/cost");
    return DRO_E_NULL;
  }
  if (depth_mode < DRO_DEPTH_METRIC || depth_mode > DRO_DEPTH_DISP) {
    set_error("warp_cost_forward: unknown depth_mode");
    return DRO_E_MODE;
  }
  if (ref_layout != 0 && ref_layout != 1) {
    set_error("warp_cost_forward: ref_layout must be 0 (NCHW) or 1 (channels-last)");
    return DRO_E_MODE;
  }
  WarpArgs a = make_args(fmap, fmap_ref, depth, depth_mode, min_disp, max_disp, K, ref_K, scale,
                         pose, pose_mode, B, N, C, h, w, reduce_mean);
  const int P = h * w;
  if (ref_layout == 1) {
    dim3 grid((P + kClTP - 1) / kClTP, (C + kClCH - 1) / kClCH, B);
    hipLaunchKernelGGL(warp_cost_fwd_cl_kernel, grid, dim3(256), 0, (hipStream_t)stream, a, cost);
    return launch_status("warp_cost_fwd_cl_kernel launch failed");
  }
  dim3 grid((P + kWave - 1) / kWave, (C + kGroups * kCPT - 1) / (kGroups * kCPT), B);
  hipLaunchKernelGGL(warp_cost_fwd_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, a, cost);
  return launch_status("warp_cost_fwd_kernel launch failed");
}

// shared backward of the cost (SAMPLE = false) and of view synthesis (true)
template <bool SAMPLE>
static int warp_backward(WarpArgs a, const float* grad_out, float* grad_fmap, float* grad_fmap_ref,
                         float* grad_depth, float* grad_pose, int accumulate, void* workspace, int* cells,
                         int ref_layout, hipStream_t s) {
  const int B = a.B, N = a.N, C = a.C, h = a.h, w = a.w;
  const bool geo = grad_depth || grad_pose;
  if (geo && !workspace) {
    set_error("warp backward: workspace required for depth/pose gradients");
    return DRO_E_NULL;
  }
  if (accumulate < 0 || accumulate > 7) {
    set_error("warp backward: accumulate must be 0..7");
    return DRO_E_MODE;
  }
  int st;
  a.acc_fmap = accumulate & 1;
  a.acc_depth = (accumulate >> 2) & 1;
  a.cells = cells;
  static const int nomerge = env_int("DRO_WARP_NOMERGE", 0);
  a.merge = nomerge ? 0 : 1;
  const int P = h * w;
  if (grad_fmap_ref && !(accumulate & 2) &&
      (st = launch_zero(grad_fmap_ref, (size_t)N * B * C * P, s)))
    return st;
  // channels-last maps of <= 256 channels: one block per pixel tile holds every
  // channel, and the depth / pose chain runs in the same launch (GEO)
  const int nch = (C + kClCH - 1) / kClCH;
  if (ref_layout == 1 && nch <= 4) {
    if (!(grad_fmap || grad_fmap_ref || geo || cells)) return DRO_OK;
    dim3 grid((P + kClTP - 1) / kClTP, 1, B);
    double* partial = grad_pose ? (double*)workspace : nullptr;
#define DRO_CLF(NCH_, GEO_)                                                                            \
  hipLaunchKernelGGL((warp_cost_bwd_feat_cl_kernel<NCH_, GEO_>), grid, dim3(256), 0, s, a, grad_out, \
                     grad_fmap, grad_fmap_ref, (float*)nullptr, grad_depth, partial)
    if (nch == 1) {
      if (geo) DRO_CLF(1, true); else DRO_CLF(1, false);
    } else if (nch == 2) {
      if (geo) DRO_CLF(2, true); else DRO_CLF(2, false);
    } else {
      if (geo) DRO_CLF(4, true); else DRO_CLF(4, false);
    }
#undef DRO_CLF
    if ((st = launch_status("warp_cost_bwd_feat_cl_kernel launch failed"))) return st;
    if (grad_pose)
      return launch_pose_finalize(partial, (int)grid.x, N * B, a.pose, a.pose_mode, grad_pose, s);
    return DRO_OK;
  }
  float* gxy = geo ? (float*)workspace : nullptr;
  const int nblk = (P + kGeoThreads - 1) / kGeoThreads;
  double* partial = (geo && grad_pose) ? (double*)(gxy + (size_t)N * B * P * 2) : nullptr;
  if (gxy && (st = launch_zero(gxy, (size_t)N * B * P * 2, s))) return st;
  if (ref_layout == 1 && (grad_fmap || grad_fmap_ref || gxy || cells)) {
    dim3 grid((P + kClTP - 1) / kClTP, nch, B);
    hipLaunchKernelGGL((warp_cost_bwd_feat_cl_kernel<1, false>), grid, dim3(256), 0, s, a, grad_out, grad_fmap,
                       grad_fmap_ref, gxy, (float*)nullptr, (double*)nullptr);
    if ((st = launch_status("warp_cost_bwd_feat_cl_kernel launch failed"))) return st;
  } else if (grad_fmap || grad_fmap_ref || gxy || cells) {
    dim3 grid((P + kWave - 1) / kWave, (C + kGroups * kCPT - 1) / (kGroups * kCPT), B);
    hipLaunchKernelGGL(warp_cost_bwd_feat_kernel<SAMPLE>, grid, dim3(256), 0, s, a, grad_out, grad_fmap,
                       grad_fmap_ref, gxy);
    if ((st = launch_status("warp_cost_bwd_feat_kernel launch failed"))) return st;
  }
  if (geo) {
    hipLaunchKernelGGL(warp_cost_bwd_geo_kernel, dim3(nblk, B), dim3(kGeoThreads), 0, s, a, gxy,
                       grad_depth, partial);
    if ((st = launch_status("warp_cost_bwd_geo_kernel launch failed"))) return st;
  }
  if (grad_pose) {
    if ((st = launch_pose_finalize(partial, nblk, N * B, a.pose, a.pose_mode, grad_pose, s))) return st;
  }
  return DRO_OK;
}

extern "C" int dro_warp_cost_backward(const float* fmap, const float* fmap_ref, const float* depth,
                                      int depth_mode, float min_disp, float max_disp,
                                      const float* K, const float* ref_K, float scale,
                                      const float* pose, int pose_mode, int B, int N, int C,
                                      int h, int w, int reduce_mean, int ref_layout, const float* grad_cost,
                                      float* grad_fmap, float* grad_fmap_ref, float* grad_depth,
                                      float* grad_pose, int accumulate, void* workspace, int* cells,
                                      void* stream) {
  int st = check_common(fmap, fmap_ref, K, ref_K, pose, pose_mode, B, N, C, h, w);
  if (st) return st;
  if (!depth || !grad_cost) {
    set_error("warp_cost_backward: NULL depth/grad_cost");
    return DRO_E_NULL;
  }
  if (ref_layout != 0 && ref_layout != 1) {
    set_error("warp_cost_backward: ref_layout must be 0 (NCHW) or 1 (channels-last)");
    return DRO_E_MODE;
  }
  WarpArgs a = make_args(fmap, fmap_ref, depth, depth_mode, min_disp, max_disp, K, ref_K, scale,
                         pose, pose_mode, B, N, C, h, w, reduce_mean);
  return warp_backward<false>(a, grad_cost, grad_fmap, grad_fmap_ref, grad_depth, grad_pose, accumulate,
                              workspace, cells, ref_layout, (hipStream_t)stream);
}

extern "C" int dro_view_synthesis_forward(const float* ref_image, const float* depth, int depth_mode,
                                          float min_disp, float max_disp, const float* K, const float* ref_K,
                                          float scale, const float* pose, int pose_mode, int B, int N, int C,
                                          int H, int W, float* warped, void* stream) {
  // check_common wants a non-NULL fmap: view synthesis has none (ref_image stands in)
  int st = check_common(ref_image, ref_image, K, ref_K, pose, pose_mode, B, N, C, H, W);
  if (st) return st;
  if (!depth || !warped) {
    set_error("view_synthesis_forward: NULL depth/warped");
    return DRO_E_NULL;
  }
  if (depth_mode < DRO_DEPTH_METRIC || depth_mode > DRO_DEPTH_DISP) {
    set_error("view_synthesis_forward: unknown depth_mode");
    return DRO_E_MODE;
  }
  WarpArgs a = make_args(nullptr, ref_image, depth, depth_mode, min_disp, max_disp, K, ref_K, scale, pose,
                         pose_mode, B, N, C, H, W, 0);
  const int P = H * W;
  dim3 grid((P + kWave - 1) / kWave, (C + kGroups * kCPT - 1) / (kGroups * kCPT), B);
  hipLaunchKernelGGL(warp_cost_fwd_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, a, warped);
  return launch_status("warp_cost_fwd_kernel<sample> launch failed");
}

extern "C" int dro_view_synthesis_backward(const float* ref_image, const float* depth, int depth_mode,
                                           float min_disp, float max_disp, const float* K, const float* ref_K,
                                           float scale, const float* pose, int pose_mode, int B, int N, int C,
                                           int H, int W, const float* grad_warped, float* grad_ref_image,
                                           float* grad_depth, float* grad_pose, void* workspace, int* cells,
                                           void* stream) {
  int st = check_common(ref_image, ref_image, K, ref_K, pose, pose_mode, B, N, C, H, W);
  if (st) return st;
  if (!depth || !grad_warped) {
    set_error("view_synthesis_backward: NULL depth/grad_warped");
    return DRO_E_NULL;
  }
  WarpArgs a = make_args(nullptr, ref_image, depth, depth_mode, min_disp, max_disp, K, ref_K, scale, pose,
                         pose_mode, B, N, C, H, W, 0);
  return warp_backward<true>(a, grad_warped, nullptr, grad_ref_image, grad_depth, grad_pose, 0, workspace,
                             cells, 0, (hipStream_t)stream);
}

extern "C" int dro_plane_sweep_forward(const float* fmap, const float* fmap_ref, const float* disp,
                                       int D, float min_disp, float max_disp, const float* K,
                                       const float* ref_K, float scale, const float* pose,
                                       int pose_mode, int B, int C, int h, int w, float* cost,
                                       void* stream) {
  int st = check_common(fmap, fmap_ref, K, ref_K, pose, pose_mode, B, 1, C, h, w);
  if (st) return st;
  if (!disp || !cost) {
    set_error("plane_sweep_forward: NULL disp/cost");
    return DRO_E_NULL;
  }
  if (D < 1 || (long long)B * D > 65535) {
    set_error("plane_sweep_forward: D out of range");
    return DRO_E_SHAPE;
  }
  WarpArgs a = make_args(fmap, fmap_ref, nullptr, DRO_DEPTH_DISP, min_disp, max_disp, K, ref_K,
                         scale, pose, pose_mode, B, 1, C, h, w, 0);
  const int P = h * w;
  // LDS path: 4-pixel vectors need P % 4 == 0 (and 16-B aligned maps); the
  // channel group's reference planes must fit 64 KB of LDS
  const bool aligned = ((reinterpret_cast<uintptr_t>(fmap) | reinterpret_cast<uintptr_t>(fmap_ref) |
                         reinterpret_cast<uintptr_t>(cost)) & 15) == 0;
  // tuning overrides (A/B runs, tools/bench_sweep.py): DRO_SWEEP_CG = largest
  // channel group (default 8), DRO_SWEEP_BLOCKS = minimum grid (default 512),
  // DRO_SWEEP_WIDE = 1 forces plane_sweep_wide_kernel, DRO_SWEEP_NT = 0 plain stores
  static const int cg_max = env_int("DRO_SWEEP_CG", 8);
  static const int min_blocks = env_int("DRO_SWEEP_BLOCKS", 512);
  static const bool wide = env_int("DRO_SWEEP_WIDE", 0) != 0;
  static const bool nt = env_int("DRO_SWEEP_NT", 1) != 0;      // non-temporal volume stores
  static const int threads = [] {   // 512: 16 waves per CU (46.7 -> 43.5 us); 1024: two planes at once
    const int t = env_int("DRO_SWEEP_THREADS", 512);
    return t == 256 || t == 1024 ? t : 512;
  }();
  int CG = cg_max;
  while (CG > 1 && (C % CG != 0 || (size_t)CG * P * sizeof(float) > 65536)) CG >>= 1;
  if (!wide && aligned && P % 4 == 0 && C % CG == 0 && (size_t)CG * P * sizeof(float) <= 65536) {
    // planes per block: enough blocks to fill the chip at least twice
    const int per_dg = B * (C / CG);
    int DG = 1;
    while (DG < D && per_dg * ((D + 2 * DG - 1) / (2 * DG)) >= min_blocks) DG *= 2;
    const int nblk = per_dg * ((D + DG - 1) / DG);
    const size_t lds = (size_t)CG * P * sizeof(float);
    hipStream_t s = (hipStream_t)stream;
#define DRO_SWEEP_LAUNCH(CG_)                                                                                  \
  do {                                                                                                         \
    if (nt)                                                                                                    \
      hipLaunchKernelGGL((plane_sweep_lds_kernel<CG_, true>), dim3(nblk), dim3(threads), lds, s, a, disp, D, DG, cost); \
    else                                                                                                       \
      hipLaunchKernelGGL((plane_sweep_lds_kernel<CG_, false>), dim3(nblk), dim3(threads), lds, s, a, disp, D, DG, cost); \
  } while (0)
    switch (CG) {
      case 8: DRO_SWEEP_LAUNCH(8); break;
      case 4: DRO_SWEEP_LAUNCH(4); break;
      case 2: DRO_SWEEP_LAUNCH(2); break;
      default: DRO_SWEEP_LAUNCH(1);
    }
#undef DRO_SWEEP_LAUNCH
    return launch_status("plane_sweep_lds_kernel launch failed");
  }
  dim3 grid((P + kWave - 1) / kWave, (C + 4 * kSweepCPT - 1) / (4 * kSweepCPT), B * D);
  hipLaunchKernelGGL(plane_sweep_wide_kernel, grid, dim3(256), 0, (hipStream_t)stream, a, disp, D,
                     cost);
  return launch_status("plane_sweep_wide_kernel launch failed");
}
