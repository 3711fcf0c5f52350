// Fused multi-view photometric decay loss + edge-aware smoothness (fwd + bwd).
//
// Replaces MultiViewPhotometricDecayLoss.forward
// (dro_sfm/losses/multiview_photometric_loss_mf.py:303-361) for the
// configuration every reference yaml uses (padding 'zeros', full-resolution
// predictions) and clip_loss >= 0 (the reference constructor's default 0.5:
// two forward passes around per-map thresholds, photo_clip_stats_kernel): per (prediction i, ref j) view_synthesis
// (geometry/camera_utils.py:23-56), SSIM 3x3 with reflection padding (:15-54),
// 0.85*SSIM + 0.15*L1 channel means (:194-229), automask (:346-351), min (or
// mean) reduction over the 2N maps with 0.85^(n-i-1) decay (:231-269), and the
// smoothness term (:273-299, utils/depth.py:147-199).  The reference runs
// ~25 ATen kernels per (i, j) pair forward (18 pairs for KITTI it8) plus the
// automask pass per (i, j); here the whole loss is 3 launches forward (the
// automask maps once per (ref, batch), the tile kernel, a one-block finalize)
// and 2 backward.
//
// Tiling: a workgroup owns an 8x64 output tile of one (prediction, batch).
// The warped reference is synthesised once per tile into LDS with a 1-pixel
// (forward) or 2-pixel (backward) reflected halo, so the 3x3 SSIM windows
// read LDS only.  The backward re-synthesises instead of storing warped
// images, keeps the per-pixel min selection from the forward (1 byte/px), and
// turns the 3x3 average-pool transposes into a gather over a per-pixel
// (dL/dmu_x, dL/dE[x^2], dL/dE[xy]) LDS image -- reflection padding makes the
// adjoint of the pool non-local at the borders, which the gather handles by
// counting the reflected taps explicitly.
//
// Roofline: HBM bound.  Algorithmic bytes: 32*HW per
// (i, j) pair, 28*HW per automask map, 8N*HW per prediction for the min
// reduce, 16*HW per prediction for smoothness.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "dro_common.hpp"

// Built with -ffp-contract=off (Makefile): the SSIM statistics and their
// adjoint difference nearly equal products, and fusing one product of a pair
// into an FMA unbalances the roundings (round 5: 1e-4 relative on the
// inverse-depth gradient at zero-padding-band pixels; 1.9e-5 uncontracted).

namespace dro {

constexpr int TH = 8, TW = 64;
constexpr int H1 = TH + 2, W1 = TW + 2;  // 1-pixel halo
constexpr int H2 = TH + 4, W2 = TW + 4;  // 2-pixel halo
constexpr int kThreads = 256;
constexpr int kPxPerThread = (TH * TW) / kThreads;

struct PhotoArgs {
  const float* image;
  const float* context;
  const float* inv;
  const float* K;
  const float* ref_K;
  const float* pose;
  int pose_mode;
  int B, N, n, H, W;
  float ssim_w, l1_w, C1, C2, smooth_w;
  int automask, reduce_min;
  int tiles_x, tiles_y;
  // workspace views
  unsigned char* sel;
  float* am;        // [N,B,HW] automask (unwarped) photometric maps, once per (ref, batch)
  float* part_inv;  // [n,B,tiles] sums of the inverse depth (its mean normalises smoothness)
  float* mean;      // [n,B]
  float* U;         // [n,B,2]
  float* part_ph;   // [n,B,tiles]
  float* part_sm;   // [n,B,tiles,2]
  double* part_pose; // [N,n,B,tiles,12] fp64 (block_sum_d)
  int* cells;        // backward test hook: bilinear cell per (j, i, b, pixel) (pack_cell), or NULL
  // clip_loss > 0 (multiview_photometric_loss_mf.py:223-227): every candidate
  // map is clamped from above at float(mean + clip * std) of itself
  float clip;
  float* pm;         // clip: [N,n,B,HW] warped photometric maps (forward pass 1)
  float* thr;        // clip: [N*n] warped + [N] unwarped clamp thresholds
  signed char* l1s;  // backward test hook: sign of est - tgt per (j, i, b, c, pixel) the L1 term used
                     // (1 / -1, 2 = zero), or NULL
};

__device__ __forceinline__ int reflect_idx(int y, int H) {
  y = y < 0 ? -y : y;
  y = y >= H ? 2 * (H - 1) - y : y;
  return min(max(y, 0), H - 1);
}

// Stage the tile's inverse depth with a HALO-pixel reflected ring into LDS
// (pitch PW): read once per block, shared by every reference j and by the
// smoothness term (in-range neighbours of the reflected ring equal the image).
template <int PL, int PW, int HALO>
__device__ __forceinline__ void stage_inv(const float* __restrict__ invp, int x0, int y0, int H, int W,
                                          float* __restrict__ invt) {
  for (int k = threadIdx.x; k < PL; k += kThreads) {
    const int gy = reflect_idx(y0 + k / PW - HALO, H), gx = reflect_idx(x0 + k % PW - HALO, W);
    invt[k] = invp[(size_t)gy * W + gx];
  }
}

// Synthesise the warped reference (view_synthesis, camera_utils.py:23-56) of
// context (j, b) over the LDS tile [PL] (pitch PW, reflected ring HALO) into
// est[3][PL].  The per-thread iterations are unrolled so every bilinear
// gather of the thread is in flight at once (the phase is bound by the
// gathers' latency, not by arithmetic).  Arithmetic order as synth().
template <int PL, int PW, int HALO>
__device__ __forceinline__ void stage_warp(const PhotoArgs& a, const float* __restrict__ ctx,
                                           const float* __restrict__ invt, const float ki[9],
                                           const float kr[9], const float R[9], const float t[3],
                                           int x0, int y0, float* __restrict__ est) {
  constexpr int IT = (PL + kThreads - 1) / kThreads;
  constexpr int CH = 2;  // iterations whose gathers are in flight together (VGPR budget)
  const size_t HW = (size_t)a.H * a.W;
#pragma unroll
  for (int i0 = 0; i0 < IT; i0 += CH) {
    Taps T[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int k = min((int)threadIdx.x + (i0 + u) * kThreads, PL - 1);  // tail: computed, not stored
      const int gy = reflect_idx(y0 + k / PW - HALO, a.H), gx = reflect_idx(x0 + k % PW - HALO, a.W);
      float dd;
      const float depth = decode_depth(invt[k], DRO_DEPTH_INV, 0.f, 0.f, &dd);
      Proj q;
      project(ki, kr, R, t, (float)gx, (float)gy, depth, a.H, a.W, q);
      bilinear_taps(q.ix, q.iy, a.H, a.W, T[u]);
    }
    float v[CH][3][4];
#pragma unroll
    for (int u = 0; u < CH; ++u)
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int q = 0; q < 4; ++q) v[u][c][q] = ctx[c * HW + (T[u].ok[q] ? T[u].idx[q] : 0)];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int k = threadIdx.x + (i0 + u) * kThreads;
      if (i0 + u >= IT || k >= PL) continue;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (T[u].ok[q]) s += v[u][c][q] * T[u].wgt[q];
        est[c * PL + k] = s;
      }
    }
  }
}

// Backward staging: est over the 2-px-halo tile exactly as stage_warp<PL2,
// W2, 2> computes it, with this thread's own interior pixels (ly = tid / TW +
// r * (kThreads / TW), lx = tid % TW) among the pixels it stages, so the
// bilinear derivative terms d est_c / d ix, d est_c / d iy of those pixels
// come from the same four gathers (a second projection + 12 gathers per pixel
// otherwise).  Ring pixels (the 2-px halo, 304 of them) are spread over the
// threads after the interior ones.
__device__ __forceinline__ void stage_warp_bwd(const PhotoArgs& a, const float* __restrict__ ctx,
                                               const float* __restrict__ invt, const float ki[9],
                                               const float kr[9], const float R[9], const float t[3],
                                               int x0, int y0, float* __restrict__ est,
                                               float (&dxc)[kPxPerThread][3], float (&dyc)[kPxPerThread][3],
                                               int* __restrict__ cells) {
  constexpr int PW = W2, PL = H2 * W2, HALO = 2;
  constexpr int NRING = PL - TH * TW;
  constexpr int NR = (NRING + kThreads - 1) / kThreads;
  static_assert(kPxPerThread == 2 && NR == 2, "two interior + two ring slots per thread");
  const size_t HW = (size_t)a.H * a.W;
  auto ring_k = [](int h) {
    if (h < 2 * PW) return h;                                   // rows 0, 1
    h -= 2 * PW;
    if (h < 2 * PW) return (H2 - 2) * PW + h;                   // rows H2-2, H2-1
    h -= 2 * PW;                                                // rows 2..H2-3, cols 0, 1, PW-2, PW-1
    const int row = 2 + h / 4, c4 = h % 4;
    return row * PW + (c4 < 2 ? c4 : PW - 4 + c4);
  };
  // one group of U pixels at a time: their gathers are in flight together
  // (interior pixels one by one -- their derivative terms stay live after)
  auto group = [&](auto u_c, const int (&kk)[decltype(u_c)::value], const bool (&valid)[decltype(u_c)::value],
                   int slot0, bool interior) {
    constexpr int U = decltype(u_c)::value;
    Taps T[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = kk[u];
      const int gy = reflect_idx(y0 + k / PW - HALO, a.H), gx = reflect_idx(x0 + k % PW - HALO, a.W);
      float dd;
      const float depth = decode_depth(invt[k], DRO_DEPTH_INV, 0.f, 0.f, &dd);
      Proj q;
      project(ki, kr, R, t, (float)gx, (float)gy, depth, a.H, a.W, q);
      bilinear_taps(q.ix, q.iy, a.H, a.W, T[u]);
      // the cell of an interior pixel is the one its derivative terms use
      if (interior && cells && y0 + k / PW - HALO < a.H && x0 + k % PW - HALO < a.W)
        cells[(size_t)gy * a.W + gx] = pack_cell(q.ix, q.iy);
    }
    float v[U][3][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int q = 0; q < 4; ++q) v[u][c][q] = ctx[c * HW + (T[u].ok[q] ? T[u].idx[q] : 0)];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!valid[u]) continue;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (T[u].ok[q]) s += v[u][c][q] * T[u].wgt[q];
        est[c * PL + kk[u]] = s;
        if (interior) {
          float z[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) z[q] = T[u].ok[q] ? v[u][c][q] : 0.f;
          const float omy = 1.f - T[u].ty, omx = 1.f - T[u].tx;
          dxc[slot0 + u][c] = (z[1] - z[0]) * omy + (z[3] - z[2]) * T[u].ty;
          dyc[slot0 + u][c] = (z[2] - z[0]) * omx + (z[3] - z[1]) * T[u].tx;
        }
      }
    }
  };
#pragma unroll
  for (int r = 0; r < kPxPerThread; ++r) {
    const int ly = threadIdx.x / TW + r * (kThreads / TW), lx = threadIdx.x % TW;
    const int kk[1] = {(ly + HALO) * PW + lx + HALO};
    const bool valid[1] = {true};
    group(std::integral_constant<int, 1>{}, kk, valid, r, true);
  }
  {
    int kk[2];
    bool valid[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int h = threadIdx.x + u * kThreads;
      valid[u] = h < NRING;
      kk[u] = ring_k(valid[u] ? h : 0);
    }
    group(std::integral_constant<int, 2>{}, kk, valid, 0, false);
  }
}

// one synthesised RGB sample of context (j, b) at target pixel (x, y)
__device__ __forceinline__ void synth(const PhotoArgs& a, const float* __restrict__ ctx,
                                      const float ki[9], const float kr[9], const float R[9],
                                      const float t[3], int x, int y, float invd, float out[3],
                                      Proj* qo, Taps* to) {
  float dd;
  const float depth = decode_depth(invd, DRO_DEPTH_INV, 0.f, 0.f, &dd);
  Proj q;
  project(ki, kr, R, t, (float)x, (float)y, depth, a.H, a.W, q);
  Taps T;
  bilinear_taps(q.ix, q.iy, a.H, a.W, T);
  const size_t HW = (size_t)a.H * a.W;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float* pl = ctx + c * HW;
    float v = 0.f;
    if (T.ok[0]) v += pl[T.idx[0]] * T.wgt[0];
    if (T.ok[1]) v += pl[T.idx[1]] * T.wgt[1];
    if (T.ok[2]) v += pl[T.idx[2]] * T.wgt[2];
    if (T.ok[3]) v += pl[T.idx[3]] * T.wgt[3];
    out[c] = v;
  }
  if (qo) *qo = q;
  if (to) *to = T;
}

// SSIM (multiview_photometric_loss_mf.py:15-54) of one channel from a 3x3
// window of two LDS images with row pitch `pitch`, centred at offset o.
// (Round 5: moments about the window's centre value and a centred adjoint were
// measured -- no change in any parity margin, photometric backward 8 % slower;
// not kept.)
struct SsimStats {
  float mx, my, sxx, syy, sxy;  // pooled E[x], E[y], E[x^2], E[y^2], E[xy]
};

__device__ __forceinline__ SsimStats pool3(const float* __restrict__ X, const float* __restrict__ Y,
                                           int o, int pitch) {
  float sx = 0.f, sy = 0.f, sxx = 0.f, syy = 0.f, sxy = 0.f;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) {
      const float xv = X[o + dy * pitch + dx], yv = Y[o + dy * pitch + dx];
      sx += xv;
      sy += yv;
      sxx += xv * xv;
      syy += yv * yv;
      sxy += xv * yv;
    }
  SsimStats s;
  s.mx = sx / 9.f;
  s.my = sy / 9.f;
  s.sxx = sxx / 9.f;
  s.syy = syy / 9.f;
  s.sxy = sxy / 9.f;
  return s;
}

__device__ __forceinline__ float ssim_value(const SsimStats& s, float C1, float C2) {
  const float mxy = s.mx * s.my, mxx = s.mx * s.mx, myy = s.my * s.my;
  const float sig_x = s.sxx - mxx, sig_y = s.syy - myy, sig_xy = s.sxy - mxy;
  const float v1 = 2.f * sig_xy + C2, v2 = sig_x + sig_y + C2;
  const float num = (2.f * mxy + C1) * v1;
  const float den = (mxx + myy + C1) * v2;
  return num / den;
}

// torch.clamp(v, max=thr) with its NaN handling: a NaN value or a NaN bound
// gives NaN (fminf would return the other operand)
__device__ __forceinline__ float clamp_max(float v, float thr) {
  return (v > thr || thr != thr) ? thr : v;
}

__device__ __forceinline__ float clamp_ssim_loss(float ssim) {
  return fminf(fmaxf((1.f - ssim) / 2.f, 0.f), 1.f);
}

// photometric map value from 3 channels' SSIM and L1 (calc_photometric_loss)
__device__ __forceinline__ float photo_value(const PhotoArgs& a, const float* X, const float* Y,
                                             int o, int pitch, int plane) {
  float ls = 0.f, l1 = 0.f;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const SsimStats s = pool3(X + c * plane, Y + c * plane, o, pitch);
    ls += clamp_ssim_loss(ssim_value(s, a.C1, a.C2));
    l1 += fabsf(X[c * plane + o] - Y[c * plane + o]);
  }
  return a.ssim_w * (ls / 3.f) + a.l1_w * (l1 / 3.f);
}

__device__ __forceinline__ void cams_full(const PhotoArgs& a, int b, float ki[9], float kr[9]) {
  float k[9];
  scaled_K(a.K + 9 * b, 1.f, false, k);
  K_inverse(k, ki);
  scaled_K(a.ref_K + 9 * b, 1.f, false, kr);
}

// ------------------------------------------------------------------ automask maps
// The unwarped-reference photometric map (multiview_photometric_loss_mf.py:346-351)
// depends on (ref j, batch b) only; the reference recomputes it for every
// prediction, the forward kernel reads it from here (same arithmetic, same values).
__global__ __launch_bounds__(kThreads) void photo_automask_kernel(PhotoArgs a) {
  constexpr int PL = H1 * W1;
  __shared__ float tgt[3 * PL];
  __shared__ float raw[3 * PL];
  const int jb = blockIdx.z, j = jb / a.B, b = jb % a.B;
  const int y0 = blockIdx.y * TH, x0 = blockIdx.x * TW;
  const int H = a.H, W = a.W;
  const size_t HW = (size_t)H * W;
  const float* img = a.image + (size_t)b * 3 * HW;
  const float* ctx = a.context + ((size_t)j * a.B + b) * 3 * HW;
  for (int k = threadIdx.x; k < PL; k += kThreads) {
    const int gy = reflect_idx(y0 + k / W1 - 1, H), gx = reflect_idx(x0 + k % W1 - 1, W);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      tgt[c * PL + k] = img[c * HW + (size_t)gy * W + gx];
      raw[c * PL + k] = ctx[c * HW + (size_t)gy * W + gx];
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kPxPerThread; ++r) {
    const int ly = threadIdx.x / TW + r * (kThreads / TW), lx = threadIdx.x % TW;
    if (y0 + ly >= H || x0 + lx >= W) continue;
    const int o = (ly + 1) * W1 + (lx + 1);
    a.am[(size_t)jb * HW + (size_t)(y0 + ly) * W + x0 + lx] = photo_value(a, raw, tgt, o, W1, PL);
  }
}

// XCD-aware block order.  Workgroups are dispatched round-robin over the 8
// XCDs (linear id % 8), each with its own 4 MB L2.  With the natural order
// every XCD sees every tile of every (prediction, batch) and the context
// images all n predictions gather from (2 refs x B x 1.5 MB at 192x640) miss
// its L2.  When the tile count divides by 8, XCD x gets a contiguous band of
// tile rows for all (i, b) instead: the band's context rows are gathered by
// n predictions from one L2.  (1-D grid of tiles * planes blocks.)
__device__ __forceinline__ void block_tile(const PhotoArgs& a, int& tile, int& plane) {
  const int L = blockIdx.x, tiles = a.tiles_x * a.tiles_y;
  if (tiles % 8 == 0) {
    const int per = tiles / 8, x = L % 8, k = L / 8;
    tile = x * per + k % per;
    plane = k / per;
  } else {
    tile = L % tiles;
    plane = L / tiles;
  }
}

// ------------------------------------------------------------------ forward tile kernel
// MODE 0: the whole forward (clip_loss == 0).  With clip_loss > 0 the
// thresholds depend on whole maps, so the forward runs in two passes around
// photo_clip_stats_kernel: MODE 1 synthesises the warped maps and stores them
// (pm), MODE 2 reads them back clamped (no second warp) and reduces as MODE 0.
enum { kPhotoFull = 0, kPhotoStore = 1, kPhotoSelect = 2 };

template <int MODE>
__global__ __launch_bounds__(kThreads) void photo_fwd_kernel(PhotoArgs a) {
  constexpr int PL = H1 * W1;
  __shared__ float tgt[3 * PL];
  __shared__ float est[3 * PL];
  __shared__ float invt[PL];
  __shared__ float scratch[4 * (kThreads / kWave)];

  int tile, ib;
  block_tile(a, tile, ib);
  const int i = ib / a.B, b = ib % a.B;
  const int y0 = (tile / a.tiles_x) * TH, x0 = (tile % a.tiles_x) * TW;
  const int H = a.H, W = a.W;
  const size_t HW = (size_t)H * W;
  const float* img = a.image + (size_t)b * 3 * HW;
  const float* invp = a.inv + (size_t)ib * HW;

  for (int k = threadIdx.x; k < PL; k += kThreads) {
    const int gy = reflect_idx(y0 + k / W1 - 1, H), gx = reflect_idx(x0 + k % W1 - 1, W);
#pragma unroll
    for (int c = 0; c < 3; ++c) tgt[c * PL + k] = img[c * HW + (size_t)gy * W + gx];
  }
  stage_inv<PL, W1, 1>(invp, x0, y0, H, W, invt);
  __syncthreads();

  float ki[9], kr[9];
  cams_full(a, b, ki, kr);
  const int M = a.automask ? 2 * a.N : a.N;
  float best[kPxPerThread], accm[kPxPerThread];
  int arg[kPxPerThread];
#pragma unroll
  for (int r = 0; r < kPxPerThread; ++r) {
    best[r] = 0.f;
    accm[r] = 0.f;
    arg[r] = -1;
  }
  const int ps = pose_stride(a.pose_mode);
  for (int j = 0; j < a.N; ++j) {
    float R[9], t[3];
    load_pose(a.pose + ((size_t)(j * a.n + i) * a.B + b) * ps, a.pose_mode, R, t);
    const float* ctx = a.context + ((size_t)j * a.B + b) * 3 * HW;
    if (MODE != kPhotoSelect) {
      if (j) __syncthreads();  // previous j's readers are done with est
      stage_warp<PL, W1, 1>(a, ctx, invt, ki, kr, R, t, x0, y0, est);
      __syncthreads();
    }
    float* pmj = MODE != kPhotoFull ? a.pm + ((size_t)(j * a.n + i) * a.B + b) * HW : nullptr;
#pragma unroll
    for (int r = 0; r < kPxPerThread; ++r) {
      const int ly = threadIdx.x / TW + r * (kThreads / TW), lx = threadIdx.x % TW;
      if (y0 + ly >= H || x0 + lx >= W) continue;
      const int o = (ly + 1) * W1 + (lx + 1);
      const size_t gp = (size_t)(y0 + ly) * W + x0 + lx;
      float vw;
      if (MODE == kPhotoSelect) {
        vw = clamp_max(pmj[gp], a.thr[j * a.n + i]);      // torch.clamp(max=...)
      } else {
        vw = photo_value(a, est, tgt, o, W1, PL);
        if (MODE == kPhotoStore) {
          pmj[gp] = vw;
          continue;
        }
      }
      // candidate order of torch.cat(losses, 1): [warped_0, unwarped_0, warped_1, ...]
      const int kw = a.automask ? 2 * j : j;
      if (a.reduce_min) {
        if (arg[r] < 0 || vw < best[r]) {
          best[r] = vw;
          arg[r] = kw;
        }
      } else {
        accm[r] += vw;
      }
      if (a.automask) {
        float vu = a.am[((size_t)j * a.B + b) * HW + gp];
        if (MODE == kPhotoSelect) vu = clamp_max(vu, a.thr[a.N * a.n + j]);
        if (a.reduce_min) {
          if (vu < best[r]) {
            best[r] = vu;
            arg[r] = kw + 1;
          }
        } else {
          accm[r] += vu;
        }
      }
    }
  }
  if (MODE == kPhotoStore) return;

  // selection map + tile partials of the reduced photometric map, the
  // smoothness sums (unnormalised: the mean of the inverse depth is a common
  // positive factor, divided out in photo_finalize_kernel) and the inverse depth
  float v3[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < kPxPerThread; ++r) {
    const int ly = threadIdx.x / TW + r * (kThreads / TW), lx = threadIdx.x % TW;
    const int gy = y0 + ly, gx = x0 + lx;
    if (gy >= H || gx >= W) continue;
    const size_t gp = (size_t)gy * W + gx;
    if (a.reduce_min) {
      a.sel[(size_t)ib * HW + gp] = (unsigned char)arg[r];
      v3[0] += best[r];
    } else {
      v3[0] += accm[r];
    }
    // smoothness (utils/depth.py:166-199): normalised inv-depth gradients
    // weighted by exp(-mean_c |image gradient|)
    const int o = (ly + 1) * W1 + (lx + 1);
    const float d0 = invt[o];
    v3[3] += d0;
    if (gx < W - 1) {
      const float g = d0 - invt[o + 1];
      const float gi = (fabsf(tgt[o] - tgt[o + 1]) + fabsf(tgt[PL + o] - tgt[PL + o + 1]) +
                        fabsf(tgt[2 * PL + o] - tgt[2 * PL + o + 1])) / 3.f;
      v3[1] += fabsf(g * expf(-gi));
    }
    if (gy < H - 1) {
      const float g = d0 - invt[o + W1];
      const float gi = (fabsf(tgt[o] - tgt[o + W1]) + fabsf(tgt[PL + o] - tgt[PL + o + W1]) +
                        fabsf(tgt[2 * PL + o] - tgt[2 * PL + o + W1])) / 3.f;
      v3[2] += fabsf(g * expf(-gi));
    }
  }
  (void)M;
  block_sum<4>(v3, scratch);
  if (threadIdx.x == 0) {
    const int tiles = a.tiles_x * a.tiles_y;
    a.part_ph[(size_t)ib * tiles + tile] = v3[0];
    a.part_sm[((size_t)ib * tiles + tile) * 2 + 0] = v3[1];
    a.part_sm[((size_t)ib * tiles + tile) * 2 + 1] = v3[2];
    a.part_inv[(size_t)ib * tiles + tile] = v3[3];
  }
}

// ------------------------------------------------------------------ clip thresholds (clip_loss > 0)
// One block per candidate map (N*n warped from pm, then N unwarped from am):
// mean and unbiased std over its B*H*W values in fp64 (two passes, fixed
// reduction order), rounded to fp32, and the threshold formed in fp32 as the
// reference does: float(mean + clip_loss * std) of fp32 tensors
// (multiview_photometric_loss_mf.py:225-227; no fused multiply-add).
__device__ __forceinline__ double block_sum_1d(double v, double* red) {
  v = wave_sum_d(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
  __syncthreads();
  return s;
}

__global__ __launch_bounds__(1024) void photo_clip_stats_kernel(PhotoArgs a) {
  __shared__ double red[16];
  const int m = blockIdx.x;
  const size_t M = (size_t)a.B * a.H * a.W;
  const float* src = m < a.N * a.n ? a.pm + (size_t)m * M : a.am + (size_t)(m - a.N * a.n) * M;
  double s = 0.0;
  for (size_t k = threadIdx.x; k < M; k += blockDim.x) s += src[k];
  const double mean = block_sum_1d(s, red) / (double)M;
  double q = 0.0;
  for (size_t k = threadIdx.x; k < M; k += blockDim.x) {
    const double d = (double)src[k] - mean;
    q += d * d;
  }
  const double var = block_sum_1d(q, red) / (double)(M - 1);
  if (threadIdx.x == 0) {
    const float mean32 = (float)mean, std32 = (float)sqrt(var);
    a.thr[m] = __fadd_rn(mean32, __fmul_rn(a.clip, std32));
  }
}

// ------------------------------------------------------------------ forward finalize (1 block)
// Per (i,b) one wave sums the tile partials (strided lanes, then a fixed
// shuffle tree: deterministic); the inverse-depth mean (inv_depths_normalize,
// utils/depth.py:147-163: clamp 1e-6) normalises the smoothness sums.

__global__ __launch_bounds__(1024) void photo_finalize_kernel(PhotoArgs a, float* __restrict__ out) {
  __shared__ double ph[64], sx[64], sy[64];
  const int tiles = a.tiles_x * a.tiles_y;
  const int nb = a.n * a.B;
  const double HWd = (double)a.H * a.W;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int ib = wid; ib < nb; ib += nw) {
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    for (int k = lane; k < tiles; k += 64) {
      s0 += a.part_ph[(size_t)ib * tiles + k];
      s1 += a.part_sm[((size_t)ib * tiles + k) * 2 + 0];
      s2 += a.part_sm[((size_t)ib * tiles + k) * 2 + 1];
      s3 += a.part_inv[(size_t)ib * tiles + k];
    }
    s0 = wave_sum_d(s0);
    s1 = wave_sum_d(s1);
    s2 = wave_sum_d(s2);
    s3 = wave_sum_d(s3);
    if (lane == 0) {
      const float mean = (float)(s3 / HWd);
      const double mc = (double)fmaxf(mean, 1e-6f);
      a.mean[ib] = mean;
      a.U[ib * 2 + 0] = (float)(s1 / mc);
      a.U[ib * 2 + 1] = (float)(s2 / mc);
      ph[ib] = s0;
      sx[ib] = s1 / mc;
      sy[ib] = s2 / mc;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int M = a.automask ? 2 * a.N : a.N;
    double photo = 0.0, smooth = 0.0;
    for (int i = 0; i < a.n; ++i) {
      double p = 0.0, qx = 0.0, qy = 0.0;
      for (int b = 0; b < a.B; ++b) {
        p += ph[i * a.B + b];
        qx += sx[i * a.B + b];
        qy += sy[i * a.B + b];
      }
      double li = p / (a.B * HWd);
      if (!a.reduce_min) li /= M;
      photo += pow(0.85, (double)(a.n - i - 1)) * li;
      const double mx = qx / ((double)a.B * a.H * (a.W - 1));
      const double my = qy / ((double)a.B * (a.H - 1) * a.W);
      smooth += (mx + my) / pow(2.0, (double)i);
    }
    smooth = a.smooth_w * (smooth / a.n);
    out[0] = (float)(photo + smooth);
    out[1] = (float)photo;
    out[2] = (float)smooth;
  }
}

// ------------------------------------------------------------------ backward tile kernel
// REC: the test hooks (bilinear cells, L1 signs) are compiled in; the
// production instantiation carries neither (their address arithmetic costs
// registers in a kernel at its 128-VGPR budget)
#ifndef DRO_PHOTO_BWD_WAVES
#define DRO_PHOTO_BWD_WAVES 4   // waves per SIMD the register budget targets (4: 128 VGPRs)
#endif
template <bool REC>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(DRO_PHOTO_BWD_WAVES))) void photo_bwd_kernel(PhotoArgs a, const float* __restrict__ gout,
                                                             float* __restrict__ ginv) {
  constexpr int PL2 = H2 * W2;  // est / tgt with 2-px halo
  constexpr int PL1 = H1 * W1;  // adjoint image with 1-px halo
  __shared__ float tgt[3 * PL2];
  __shared__ float est[3 * PL2];
  __shared__ float adj[3 * PL1];  // one channel: dL/dmu_x, dL/dE[x^2], dL/dE[xy]
  __shared__ unsigned char selt[PL1];
  __shared__ unsigned char ont[PL1];    // this ref's warped candidate passes a gradient at the pixel
  __shared__ float invt[PL2];
  __shared__ double dscratch[12 * (kThreads / kWave)];

  int tile, ib;
  block_tile(a, tile, ib);
  const int i = ib / a.B, b = ib % a.B;
  const int y0 = (tile / a.tiles_x) * TH, x0 = (tile % a.tiles_x) * TW;
  const int H = a.H, W = a.W;
  const size_t HW = (size_t)H * W;
  const float* img = a.image + (size_t)b * 3 * HW;
  const float* invp = a.inv + (size_t)ib * HW;
  const float g = gout[0];
  const int M = a.automask ? 2 * a.N : a.N;
  const float wi = (float)pow(0.85, (double)(a.n - i - 1));
  const float gsel = g * wi / (float)((double)a.B * HW * (a.reduce_min ? 1 : M));

  for (int k = threadIdx.x; k < PL2; k += kThreads) {
    const int gy = reflect_idx(y0 + k / W2 - 2, H), gx = reflect_idx(x0 + k % W2 - 2, W);
#pragma unroll
    for (int c = 0; c < 3; ++c) tgt[c * PL2 + k] = img[c * HW + (size_t)gy * W + gx];
  }
  for (int k = threadIdx.x; k < PL1; k += kThreads) {
    const int gy = y0 + k / W1 - 1, gx = x0 + k % W1 - 1;
    const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
    selt[k] = (in && a.reduce_min) ? a.sel[(size_t)ib * HW + (size_t)gy * W + gx] : 255;
  }
  stage_inv<PL2, W2, 2>(invp, x0, y0, H, W, invt);
  __syncthreads();

  float ki[9], kr[9];
  cams_full(a, b, ki, kr);
  float gdep[kPxPerThread];
#pragma unroll
  for (int r = 0; r < kPxPerThread; ++r) gdep[r] = 0.f;
  const int ps = pose_stride(a.pose_mode);
  const int tiles = a.tiles_x * a.tiles_y;

  for (int j = 0; j < a.N; ++j) {
    float R[9], t[3];
    load_pose(a.pose + ((size_t)(j * a.n + i) * a.B + b) * ps, a.pose_mode, R, t);
    const float* ctx = a.context + ((size_t)j * a.B + b) * 3 * HW;
    const int kw = a.automask ? 2 * j : j;
    // a ref none of whose candidates is selected in the tile's 1-px ring adds
    // nothing (every adjoint and L1 term of the tile is zero): skip it
    if (a.reduce_min) {
      int any = 0;
      for (int k = threadIdx.x; k < PL1; k += kThreads) any |= selt[k] == kw;
      if (!__syncthreads_or(any)) {
        if (a.part_pose && threadIdx.x < 12)
          a.part_pose[(((size_t)(j * a.n + i) * a.B + b) * tiles + tile) * 12 + threadIdx.x] = 0.0;
        continue;
      }
    } else if (j) {
      __syncthreads();
    }
    {
      // per pixel of the tile + ring: does ref j's warped candidate pass a
      // gradient -- selected (min) or in the image (mean), and with clip_loss
      // not clamped (clamp(x, max=t)' = [x <= t])
      const float* pmj = a.clip > 0.f ? a.pm + ((size_t)(j * a.n + i) * a.B + b) * HW : nullptr;
      const float tj = a.clip > 0.f ? a.thr[j * a.n + i] : 0.f;
      for (int k = threadIdx.x; k < PL1; k += kThreads) {
        const int gy = y0 + k / W1 - 1, gx = x0 + k % W1 - 1;
        const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
        bool on = a.reduce_min ? selt[k] == kw : in;
        if (pmj && on) on = pmj[(size_t)gy * W + gx] <= tj;
        ont[k] = on;
      }
    }
    // (1) the warped tile and, from the same gathers, the bilinear derivative
    // terms of the thread's own pixels (the projection is recomputed for the
    // chain rule in (3))
    float dxc[kPxPerThread][3], dyc[kPxPerThread][3];
    stage_warp_bwd(a, ctx, invt, ki, kr, R, t, x0, y0, est, dxc, dyc,
                   REC && a.cells ? a.cells + ((size_t)(j * a.n + i) * a.B + b) * HW : nullptr);
    __syncthreads();
    float gix[kPxPerThread], giy[kPxPerThread];
#pragma unroll
    for (int r = 0; r < kPxPerThread; ++r) gix[r] = giy[r] = 0.f;
    // one channel at a time: its adjoint plane (3 x PL1 floats of LDS instead
    // of 9 x PL1 for all three: 4 blocks per CU instead of 3), then the
    // gather of every real pixel's d(loss)/d(warped value) of that channel
#pragma unroll 1
    for (int c = 0; c < 3; ++c) {
      if (c) __syncthreads();                  // the previous channel's gathers are done
      // adjoint of the SSIM term of channel c at every real pixel of the tile + 1-px ring
      for (int k = threadIdx.x; k < PL1; k += kThreads) {
        const int ly = k / W1, lx = k % W1;
        const bool on = ont[k];
        const int o2 = (ly + 1) * W2 + (lx + 1);
        float A = 0.f, Bv = 0.f, Cv = 0.f;
        if (on) {
          const SsimStats s = pool3(est + c * PL2, tgt + c * PL2, o2, W2);
          const float mxy = s.mx * s.my, mxx = s.mx * s.mx, myy = s.my * s.my;
          const float v1 = 2.f * (s.sxy - mxy) + a.C2;
          const float v2 = (s.sxx - mxx) + (s.syy - myy) + a.C2;
          const float num = (2.f * mxy + a.C1) * v1, den = (mxx + myy + a.C1) * v2;
          const float rden = 1.f / den;
          const float ssim = num * rden;
          const float lval = (1.f - ssim) / 2.f;
          const float S = (lval >= 0.f && lval <= 1.f) ? gsel * (a.ssim_w / 3.f) * -0.5f : 0.f;
          const float dn = S * rden, dd = -S * ssim * rden;
          const float g_v1 = dn * (2.f * mxy + a.C1);
          const float g_v2 = dd * (mxx + myy + a.C1);
          const float g_mxy = dn * 2.f * v1 - g_v1 * 2.f;
          const float g_mxx = dd * v2 - g_v2;
          A = 2.f * s.mx * g_mxx + s.my * g_mxy;
          Bv = g_v2;
          Cv = 2.f * g_v1;
        }
        adj[0 * PL1 + k] = A;
        adj[1 * PL1 + k] = Bv;
        adj[2 * PL1 + k] = Cv;
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kPxPerThread; ++r) {
        const int ly = threadIdx.x / TW + r * (kThreads / TW), lx = threadIdx.x % TW;
        const int gy = y0 + ly, gx = x0 + lx;
        if (gy >= H || gx >= W) continue;
        const int o2 = (ly + 2) * W2 + (lx + 2);
        const int o1 = (ly + 1) * W1 + (lx + 1);
        // (2) adjoint of the 3x3 average pools: sum over the real pixels whose
        // (reflected) windows tap this pixel.  Pixels >= 2 from every border
        // see exactly the 3x3 neighbourhood (same summation order as the
        // general path, which handles the reflected taps explicitly).
        float s0 = 0.f, s1 = 0.f, s2 = 0.f;
        auto tap = [&](int kk) {
          s0 += adj[0 * PL1 + kk];
          s1 += adj[1 * PL1 + kk];
          s2 += adj[2 * PL1 + kk];
        };
        if (gy >= 2 && gy <= H - 3 && gx >= 2 && gx <= W - 3) {
#pragma unroll
          for (int u = 0; u < 3; ++u)
#pragma unroll
            for (int v = 0; v < 3; ++v) tap((ly + u) * W1 + (lx + v));
        } else {
          int rows[4], nr = 0, cols[4], nc = 0;
          for (int d = -1; d <= 1; ++d) {
            if (gy + d >= 0 && gy + d < H) rows[nr++] = ly + 1 + d;
            if (gx + d >= 0 && gx + d < W) cols[nc++] = lx + 1 + d;
          }
          if (gy == 1) rows[nr++] = ly;              // row 0's tap at -1 reflects to 1
          if (gy == H - 2) rows[nr++] = ly + 2;      // row H-1's tap at H reflects to H-2
          if (gx == 1) cols[nc++] = lx;
          if (gx == W - 2) cols[nc++] = lx + 2;
          for (int u = 0; u < nr; ++u)
            for (int v = 0; v < nc; ++v) tap(rows[u] * W1 + cols[v]);
        }
        const float xv = est[c * PL2 + o2], yv = tgt[c * PL2 + o2];
        float ge = (s0 + 2.f * xv * s1 + yv * s2) * (1.f / 9.f);
        if (ont[o1]) {
          const float df = xv - yv;
          const float sg = df > 0.f ? 1.f : (df < 0.f ? -1.f : 0.f);
          ge += gsel * (a.l1_w / 3.f) * sg;
          if (REC && a.l1s)
            a.l1s[(((size_t)(j * a.n + i) * a.B + b) * 3 + c) * HW + (size_t)gy * W + gx] =
                (signed char)(df > 0.f ? 1 : (df < 0.f ? -1 : 2));
        }
        // (3a) chain through the bilinear sample, channel by channel
        gix[r] += ge * dxc[r][c];
        giy[r] += ge * dyc[r][c];
      }
    }
    // (3b) chain through the projection
    float acc[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) acc[k] = 0.f;
#pragma unroll
    for (int r = 0; r < kPxPerThread; ++r) {
      const int ly = threadIdx.x / TW + r * (kThreads / TW), lx = threadIdx.x % TW;
      const int gy = y0 + ly, gx = x0 + lx;
      if (gy >= H || gx >= W) continue;
      float dd;
      const float depth = decode_depth(invt[(ly + 2) * W2 + (lx + 2)], DRO_DEPTH_INV, 0.f, 0.f, &dd);
      Proj q;
      project(ki, kr, R, t, (float)gx, (float)gy, depth, H, W, q);
      gdep[r] += project_backward_pt(q, kr, R, t, depth, gix[r], giy[r], acc, acc + 9);
    }
    if (a.part_pose) {
      double sum[12];
      block_sum_d<12>(acc, sum, dscratch);
      if (threadIdx.x == 0) {
        double* dst = a.part_pose + (((size_t)(j * a.n + i) * a.B + b) * tiles + tile) * 12;
#pragma unroll
        for (int k = 0; k < 12; ++k) dst[k] = sum[k];
      }
    }
  }

  // inverse depth gradient: photometric (through inv2depth) + smoothness
  const float m = a.mean[ib];
  const float mc = fmaxf(m, 1e-6f);
  const double p2 = pow(2.0, (double)i);
  const float cx = (float)((double)g * a.smooth_w / (a.n * p2 * a.B * (double)a.H * (a.W - 1)));
  const float cy = (float)((double)g * a.smooth_w / (a.n * p2 * a.B * (double)(a.H - 1) * a.W));
  const float mterm = (m >= 1e-6f) ? (cx * a.U[ib * 2] + cy * a.U[ib * 2 + 1]) / (mc * (float)HW) : 0.f;
  __syncthreads();
  // reuse est plane 0 as the target image with 1-px halo is still in tgt (2-px halo)
#pragma unroll
  for (int r = 0; r < kPxPerThread; ++r) {
    const int ly = threadIdx.x / TW + r * (kThreads / TW), lx = threadIdx.x % TW;
    const int gy = y0 + ly, gx = x0 + lx;
    if (gy >= H || gx >= W) continue;
    const size_t gp = (size_t)gy * W + gx;
    const int o = (ly + 2) * W2 + (lx + 2);
    const float iv = invt[o];
    float dd;
    decode_depth(iv, DRO_DEPTH_INV, 0.f, 0.f, &dd);
    float gy_n = 0.f;  // dL/d(normalised inv) at this pixel
    const float yq = iv / mc;
    auto wgt = [&](int oa, int ob) {
      return expf(-((fabsf(tgt[oa] - tgt[ob]) + fabsf(tgt[PL2 + oa] - tgt[PL2 + ob]) +
                     fabsf(tgt[2 * PL2 + oa] - tgt[2 * PL2 + ob])) / 3.f));
    };
    auto sgn = [](float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); };
    // neighbours read from the staged tile only where they are real pixels
    if (gx < W - 1) gy_n += cx * sgn((yq - invt[o + 1] / mc) * wgt(o, o + 1)) * wgt(o, o + 1);
    if (gx > 0) gy_n -= cx * sgn((invt[o - 1] / mc - yq) * wgt(o - 1, o)) * wgt(o - 1, o);
    if (gy < H - 1) gy_n += cy * sgn((yq - invt[o + W2] / mc) * wgt(o, o + W2)) * wgt(o, o + W2);
    if (gy > 0) gy_n -= cy * sgn((invt[o - W2] / mc - yq) * wgt(o - W2, o)) * wgt(o - W2, o);
    ginv[(size_t)ib * HW + gp] = gdep[r] * dd + gy_n / mc - mterm;
  }
}

}  // namespace dro

using namespace dro;

namespace {
struct PhotoLayout {
  size_t sel, am, part_inv, mean, U, part_ph, part_sm, part_pose, pm, thr, total;
};

PhotoLayout photo_layout(int B, int N, int n, int H, int W, bool clip) {
  const size_t HW = (size_t)H * W;
  const size_t tiles = (size_t)((W + TW - 1) / TW) * ((H + TH - 1) / TH);
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  PhotoLayout L;
  size_t off = 0;
  L.sel = off;
  off = al(off + (size_t)n * B * HW);
  L.am = off;
  off = al(off + sizeof(float) * N * B * HW);
  L.part_inv = off;
  off = al(off + sizeof(float) * n * B * tiles);
  L.mean = off;
  off = al(off + sizeof(float) * n * B);
  L.U = off;
  off = al(off + sizeof(float) * n * B * 2);
  L.part_ph = off;
  off = al(off + sizeof(float) * n * B * tiles);
  L.part_sm = off;
  off = al(off + sizeof(float) * n * B * tiles * 2);
  L.part_pose = off;
  off = al(off + sizeof(double) * N * n * B * tiles * 12);
  L.pm = off;
  if (clip) off = al(off + sizeof(float) * N * n * B * HW);
  L.thr = off;
  if (clip) off = al(off + sizeof(float) * (N * n + N));
  L.total = off;
  return L;
}

int photo_setup(PhotoArgs& a, const float* image, const float* context, const float* inv_depths,
                const float* K, const float* ref_K, const float* pose, int pose_mode, int B, int N,
                int n, int H, int W, float ssim_w, float C1, float C2, float smooth_w,
                int automask, int reduce_min, float clip_loss, void* workspace) {
  if (!image || !context || !inv_depths || !K || !ref_K || !pose || !workspace) {
    set_error("photometric: NULL pointer argument");
    return DRO_E_NULL;
  }
  if (B < 1 || N < 1 || n < 1 || H < 3 || W < 3 || n * B > 64 || N * (automask ? 2 : 1) > 254) {
    set_error("photometric: sizes out of range (B,N,n >= 1; H,W >= 3; n*B <= 64)");
    return DRO_E_SHAPE;
  }
  if (pose_mode != DRO_POSE_EULER && pose_mode != DRO_POSE_MATRIX) {
    set_error("photometric: unknown pose_mode");
    return DRO_E_MODE;
  }
  if (automask && !reduce_min) {
    set_error("photometric: automask requires the min reduction (multiview_photometric_loss_mf.py:117-119)");
    return DRO_E_MODE;
  }
  if (!(clip_loss == clip_loss)) {
    set_error("photometric: clip_loss is NaN");
    return DRO_E_MODE;
  }
  const bool clip = clip_loss > 0.f;     // the reference clips only for clip_loss > 0 (:223)
  PhotoLayout L = photo_layout(B, N, n, H, W, clip);
  char* ws = (char*)workspace;
  a.image = image;
  a.context = context;
  a.inv = inv_depths;
  a.K = K;
  a.ref_K = ref_K;
  a.pose = pose;
  a.pose_mode = pose_mode;
  a.B = B;
  a.N = N;
  a.n = n;
  a.H = H;
  a.W = W;
  a.ssim_w = ssim_w;
  a.l1_w = (float)(1.0 - (double)ssim_w);
  a.C1 = C1;
  a.C2 = C2;
  a.smooth_w = smooth_w;
  a.automask = automask;
  a.reduce_min = reduce_min;
  a.tiles_x = (W + TW - 1) / TW;
  a.tiles_y = (H + TH - 1) / TH;
  a.sel = (unsigned char*)(ws + L.sel);
  a.am = (float*)(ws + L.am);
  a.part_inv = (float*)(ws + L.part_inv);
  a.mean = (float*)(ws + L.mean);
  a.U = (float*)(ws + L.U);
  a.part_ph = (float*)(ws + L.part_ph);
  a.part_sm = (float*)(ws + L.part_sm);
  a.part_pose = (double*)(ws + L.part_pose);
  a.cells = nullptr;
  a.clip = clip ? clip_loss : 0.f;
  a.pm = clip ? (float*)(ws + L.pm) : nullptr;
  a.thr = clip ? (float*)(ws + L.thr) : nullptr;
  a.l1s = nullptr;
  return DRO_OK;
}
}  // namespace

extern "C" size_t dro_photometric_workspace_bytes(int B, int N, int n, int H, int W, float clip_loss) {
  return photo_layout(B, N, n, H, W, clip_loss > 0.f).total;
}

extern "C" size_t dro_photometric_clip_offset(int B, int N, int n, int H, int W, int which) {
  const PhotoLayout L = photo_layout(B, N, n, H, W, true);
  return which ? L.thr : L.pm;
}

extern "C" int dro_photometric_forward(const float* image, const float* context,
                                       const float* inv_depths, const float* K, const float* ref_K,
                                       const float* pose, int pose_mode, int B, int N, int n, int H,
                                       int W, float ssim_w, float C1, float C2, float smooth_w,
                                       int automask, int reduce_min, float clip_loss, float* out,
                                       void* workspace, void* stream) {
  PhotoArgs a;
  int st = photo_setup(a, image, context, inv_depths, K, ref_K, pose, pose_mode, B, N, n, H, W,
                       ssim_w, C1, C2, smooth_w, automask, reduce_min, clip_loss, workspace);
  if (st) return st;
  if (!out) {
    set_error("photometric_forward: NULL out");
    return DRO_E_NULL;
  }
  hipStream_t s = (hipStream_t)stream;
  if (automask) {
    hipLaunchKernelGGL(photo_automask_kernel, dim3(a.tiles_x, a.tiles_y, N * B), dim3(kThreads), 0, s, a);
    if ((st = launch_status("photo_automask_kernel launch failed"))) return st;
  }
  const dim3 tgrid(a.tiles_x * a.tiles_y * n * B);
  if (a.clip > 0.f) {
    hipLaunchKernelGGL(photo_fwd_kernel<kPhotoStore>, tgrid, dim3(kThreads), 0, s, a);
    if ((st = launch_status("photo_fwd_kernel (store) launch failed"))) return st;
    hipLaunchKernelGGL(photo_clip_stats_kernel, dim3(N * n + (automask ? N : 0)), dim3(1024), 0, s, a);
    if ((st = launch_status("photo_clip_stats_kernel launch failed"))) return st;
    hipLaunchKernelGGL(photo_fwd_kernel<kPhotoSelect>, tgrid, dim3(kThreads), 0, s, a);
  } else {
    hipLaunchKernelGGL(photo_fwd_kernel<kPhotoFull>, tgrid, dim3(kThreads), 0, s, a);
  }
  if ((st = launch_status("photo_fwd_kernel launch failed"))) return st;
  hipLaunchKernelGGL(photo_finalize_kernel, dim3(1), dim3(1024), 0, s, a, out);
  return launch_status("photo_finalize_kernel launch failed");
}

extern "C" int dro_photometric_backward(const float* image, const float* context,
                                        const float* inv_depths, const float* K,
                                        const float* ref_K, const float* pose, int pose_mode,
                                        int B, int N, int n, int H, int W, float ssim_w, float C1,
                                        float C2, float smooth_w, int automask, int reduce_min,
                                        float clip_loss, const float* grad_out, float* grad_inv_depths,
                                        float* grad_pose, void* workspace, int* cells,
                                        signed char* l1_signs, void* stream) {
  PhotoArgs a;
  int st = photo_setup(a, image, context, inv_depths, K, ref_K, pose, pose_mode, B, N, n, H, W,
                       ssim_w, C1, C2, smooth_w, automask, reduce_min, clip_loss, workspace);
  if (st) return st;
  if (!grad_out || !grad_inv_depths) {
    set_error("photometric_backward: NULL grad_out/grad_inv_depths");
    return DRO_E_NULL;
  }
  if (!grad_pose) a.part_pose = nullptr;
  a.cells = cells;
  a.l1s = l1_signs;
  hipStream_t s = (hipStream_t)stream;
  if (cells || l1_signs)
    hipLaunchKernelGGL(photo_bwd_kernel<true>, dim3(a.tiles_x * a.tiles_y * n * B), dim3(kThreads), 0, s, a,
                       grad_out, grad_inv_depths);
  else
    hipLaunchKernelGGL(photo_bwd_kernel<false>, dim3(a.tiles_x * a.tiles_y * n * B), dim3(kThreads), 0, s, a,
                     grad_out, grad_inv_depths);
  if ((st = launch_status("photo_bwd_kernel launch failed"))) return st;
  if (grad_pose) {
    const int npose = N * n * B;
    return launch_pose_finalize(a.part_pose, a.tiles_x * a.tiles_y, npose, pose, pose_mode,
                                grad_pose, s);
  }
  return DRO_OK;
}
