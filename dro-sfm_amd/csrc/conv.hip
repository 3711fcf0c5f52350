// Implicit-GEMM convolutions on f32 MFMA (v_mfma_f32_32x32x2_f32) for the
// recurrent update blocks of the DRO optimizer (dro_sfm/networks/optim/
// update.py): SepConvGRU 1x5 / 5x1 gates, projection encoders, heads.
//
// Why not MIOpen: at these shapes (3840..7680 output pixels, 1..576 channels)
// every MIOpen call is a separate launch plus NCHW<->NHWC transposes, bias /
// activation / concat are separate ATen kernels, and its forward is not
// run-to-run deterministic.  Here:
//   * inputs are a VIRTUAL channel concatenation of up to 4 tensor slices (no
//     torch.cat); a source may be a [B,C,1,1] map broadcast over the image
//     (the pose map of ProjectionInputPose);
//   * bias + activation run in the epilogue, plus two SepConvGRU epilogues:
//     the z|r gate conv also writes r*h, and the q conv writes the blended
//     state h' = (1-z)h + zq; results land in a channel slice of a tensor;
//   * f32 MFMA is exact f32 (a k-ordered fmaf chain): no TF32-style loss;
//   * no atomics: split reductions go through a workspace and are summed in a
//     fixed order, so every result is bitwise run-to-run deterministic.
//
// GEMM view (forward): rows = output channels, cols = pixels (B*H*W flattened),
// K = (tap, input channel) flattened TAP-MAJOR (k = tap*Cin + c), 32-deep
// chunks.  Each K row of a chunk is staged by one wave, so its (tap, channel,
// source) decode is wave-uniform scalar work; lanes run along pixels.
// Data gradient: the same kernel with rows = input channels, K = (tap, output
// channel), the tap offset negated and the weight read transposed.
// Weight gradient: rows = output channels, cols = (tap, input channel) plus a
// ones column that yields the bias gradient, K = pixels split over gridDim.y
// into per-split partials.
// Staging: every load of a chunk is issued unconditionally from a clamped
// address (a load under a branch, or one whose value is consumed at once,
// serialises the chunk), global -> registers for chunk c+1 before the MFMAs of
// chunk c, two LDS buffers, one barrier per chunk.  Tiles are remapped so that
// blocks sharing a pixel tile run on the same XCD (same L2).  Shapes with few
// output tiles and a long K split K over gridDim.y (partials + finish).
//
// Roofline: MFMA(f32) at 157 TF/s; FLOPs per launch = 2 * Cout * P * Cin * KH * KW.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <type_traits>

#include "conv_common.hpp"
#include "dro_common.hpp"

namespace dro {


// ------------------------------------------------------------------ forward / data gradient
// MODE 0: out[o, p]  = sum_{tap, c} W[o, c, tap] * X[c, p + d(tap)]   (+ epilogue)
// MODE 1: din[c, p]  = sum_{tap, o} W[o, c, tap] * G[o, p - d(tap)]
// Tile BM rows x 64 pixels, 4 waves: BM = 64 -> 2x2 waves of 32x32;
// BM = 32 -> 2 pixel halves x 2 K halves (summed through LDS at the end).
template <int BM, int MODE, int ACT, int EPI>
__global__ __launch_bounds__(256) void igemm_kernel(IgArgs a) {
  constexpr int WM = BM / 32;
  constexpr int KSTEPS = (WM == 2) ? 16 : 8;          // MFMA k-steps per wave per chunk
  __shared__ float Ws[2][kBK][BM + 1];
  __shared__ float Xs[2][kBK][kBN];
  const int cb1 = a.cbase[1], cb2 = a.cbase[2], cb3 = a.cbase[3];
  const int H = a.g.H, W = a.g.W, KW = a.g.KW, PH = a.g.PH, PW = a.g.PW;
  const int Hsrc = a.Hs, Wsrc = a.Ws, sh = a.sshift;   // staged operand size, log2 stride
  const unsigned HWs = (unsigned)Hsrc * (unsigned)Wsrc;
  const int Cin = a.g.Cin, Cout = a.g.Cout, rows = a.rows, kch = a.kch, K = a.K;
  const FastDiv kdiv = a.kdiv, kwdiv = a.kwdiv;
  const float* __restrict__ Wt = a.weight;
  const float* __restrict__ Gp = a.G;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int rt = tile % a.row_tiles, pt = tile / a.row_tiles;
  const int row0 = rt * BM;
  const long long p0 = (long long)pt * kBN;
  const size_t HW = (size_t)H * W;
  const long long P = (long long)a.g.B * HW;
  const int T = a.g.KH * KW;
  // Parity classes (stride-2 data gradient): din[c, 2Y+cy, 2X+cx] takes only
  // the taps with (cy + PH - ty) and (cx + PW - tx) even -- ty = ty0 + 2 iy,
  // tx = tx0 + 2 ix -- so the block's columns are the pixels of one class and
  // its K runs over (class tap, channel): the exact FLOPs, where the masked
  // form multiplies every tap of every pixel (3/4 of them by zero)
  const bool pcl = MODE == 1 && a.pclass;
  const int cy = pcl ? (int)(blockIdx.z >> 1) : 0, cx = pcl ? (int)(blockIdx.z & 1) : 0;
  const int ty0 = pcl ? (cy + PH) & 1 : 0, tx0 = pcl ? (cx + PW) & 1 : 0;
  const int ntx = pcl ? (KW - tx0 + 1) >> 1 : KW;
  const int nty = pcl ? (a.g.KH - ty0 + 1) >> 1 : a.g.KH;
  const int Hc = pcl ? (H - cy + 1) >> 1 : H, Wc = pcl ? (W - cx + 1) >> 1 : W;
  const long long HWc = (long long)Hc * Wc, Pc = (long long)a.g.B * HWc;
  const int Kc = pcl ? nty * ntx * kch : K;
  auto real_tap = [&](int tc) {   // class tap -> tap of the kernel
    if (!pcl) return tc;
    const int iy = tc / ntx;
    return (ty0 + 2 * iy) * KW + tx0 + 2 * (tc - iy * ntx);
  };
  const int nchunks = (Kc + kBK - 1) / kBK;
  const int cbeg = blockIdx.y * a.chunks_per_split;
  const int cend = min(nchunks, cbeg + a.chunks_per_split);

  // staging roles: X column (pixel) fixed; W k-lane fixed
  const int col = tid & 63, krow = tid >> 6;
  const long long pg = p0 + col;
  const bool pv = pg < Pc;
  const int pb = pv ? (int)(pg / HWc) : 0;
  const int prem = pv ? (int)(pg - (long long)pb * HWc) : 0;
  int py = prem / Wc, px = prem - py * Wc;
  if (pcl) {
    py = 2 * py + cy;
    px = 2 * px + cx;
  }
  const int wkl = tid & 31, wrow = tid >> 5;

  float xr[8], wv[BM / 8];
  unsigned xmask = 0, wmask = 0;
  auto load = [&](int chunk) {
    const int k0 = chunk * kBK;
    xmask = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      // row decode: wave-uniform (scalar)
      const int k = __builtin_amdgcn_readfirstlane(k0 + krow + 4 * i);
      const bool kv = k < Kc;
      const int kk = kv ? k : 0;
      const int tc = fdiv(kk, kdiv), ch = kk - tc * kch;
      const int tap = real_tap(tc);
      const int ty = fdiv(tap, kwdiv), dy = ty - PH, dx = tap - ty * KW - PW;
      // per lane.  Stride 2^sh: the forward reads input (S*y + dy, S*x + dx);
      // the data gradient of input pixel y takes G at (y - dy) / S where exact
      const int ny = MODE == 0 ? (py << sh) + dy : py - dy, nx = MODE == 0 ? (px << sh) + dx : px - dx;
      const bool onp = MODE == 0 || ((ny | nx) & ((1 << sh) - 1)) == 0;
      const int yy = MODE == 0 ? ny : (ny >> sh), xx = MODE == 0 ? nx : (nx >> sh);
      const bool ok = kv && pv && onp && (unsigned)yy < (unsigned)Hsrc && (unsigned)xx < (unsigned)Wsrc;
      const unsigned pix = (unsigned)(yy * Wsrc + xx);
      xmask |= ok ? (1u << i) : 0u;
      if (MODE == 0) {
        const RowDesc d = row_desc(cb1, cb2, cb3, ch, HWs);
        const unsigned e = (unsigned)pb * d.A + d.Bc + (d.M ? pix : 0u);
        xr[i] = d.p[ok ? e : 0u];
      } else {
        const unsigned e = ((unsigned)pb * (unsigned)Cout + (unsigned)ch) * HWs + pix;
        xr[i] = Gp[ok ? e : 0u];
      }
    }
    const int k = k0 + wkl;
    const bool kv = k < Kc;
    const int tc = kv ? fdiv(k, kdiv) : 0, ch = kv ? k - tc * kch : 0;
    const int tap = real_tap(tc);
    wmask = 0;
#pragma unroll
    for (int i = 0; i < BM / 8; ++i) {
      const int r = row0 + wrow + 8 * i;
      const bool ok = kv && r < rows;
      wmask |= ok ? (1u << i) : 0u;
      const unsigned idx = MODE == 0 ? ((unsigned)r * Cin + ch) * T + tap : ((unsigned)ch * Cin + r) * T + tap;
      wv[i] = Wt[ok ? idx : 0u];
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 8; ++i) Xs[buf][krow + 4 * i][col] = (xmask >> i) & 1u ? xr[i] : 0.f;
#pragma unroll
    for (int i = 0; i < BM / 8; ++i) Ws[buf][wkl][wrow + 8 * i] = (wmask >> i) & 1u ? wv[i] : 0.f;
  };

  const int wr = (WM == 2) ? (wave & 1) : 0;
  const int wc = (WM == 2) ? (wave >> 1) : (wave & 1);
  const int wk = (WM == 2) ? 0 : (wave >> 1);
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

  if (cbeg < cend) {
    load(cbeg);
    store(0);
  }
  __syncthreads();
  for (int c = cbeg; c < cend; ++c) {
    const int buf = (c - cbeg) & 1;
    const bool more = c + 1 < cend;
    if (more) load(c + 1);
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      const int kk = (wk * KSTEPS + s) * 2 + (lane >> 5);
      acc = mfma32(Ws[buf][kk][wr * 32 + (lane & 31)], Xs[buf][kk][wc * 32 + (lane & 31)], acc);
    }
    if (more) store(buf ^ 1);
    __syncthreads();
  }
  if (WM == 1) {   // sum the two K halves (LDS reused after the final barrier)
    float* red = &Xs[0][0][0];   // [2 pixel halves][16][64]
    if (wk == 1) {
#pragma unroll
      for (int r = 0; r < 16; ++r) red[(wc * 16 + r) * 64 + lane] = acc[r];
    }
    __syncthreads();
    if (wk == 1) return;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] += red[(wc * 16 + r) * 64 + lane];
  }

  const long long pe = p0 + wc * 32 + (lane & 31);
  if (pe >= Pc) return;
  if (a.part) {   // split-K partial: [split][rows][P]; parity classes [split][class][rows][pcmax]
    const long long PS = pcl ? a.pcmax : P;
    float* dst = a.part + ((size_t)blockIdx.y * (pcl ? 4 : 1) + (pcl ? blockIdx.z : 0)) * rows * PS + pe;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = row0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < rows) dst[(size_t)row * PS] = acc[r];
    }
    return;
  }
  const int eb = (int)(pe / HWc);
  size_t epix = (size_t)(pe - (long long)eb * HWc);
  if (pcl) {
    const int Y = (int)(epix / (unsigned)Wc), X = (int)epix - Y * Wc;
    epix = (size_t)(2 * Y + cy) * W + 2 * X + cx;
  }
  epi_tile<MODE, ACT, EPI>(a, acc, row0 + wr * 32 + 4 * (lane >> 5), eb, epix, HW);
}

// ------------------------------------------------------------------ halo-tiled direct conv
// Same GEMM as igemm_kernel, but a block's 64 pixels are a TH x TW tile of one
// image and each K chunk is CK channels x ALL taps: the CK x (TH+KH-1) x
// (TW+KW-1) input patch is staged once (each element loaded once, instead of
// once per tap) and the B operand of tap (ty, tx) is a shifted LDS read.
// The weight chunk is copied as the contiguous runs it has in global memory:
// forward: BM rows x (CK*T) floats (odd LDS row stride, so the
// A-operand reads, one row per lane, are bank-conflict free); data gradient:
// CK output channels x (BM*T) floats.  Staging address math is chunk
// independent except for one scalar per row, and all loads are unconditional
// (weights from clamped addresses: padded rows/channels only ever meet zero
// inputs or discarded outputs).
// MODE 0 forward, MODE 1 data gradient (tap flipped).  BM = 64: 2x2 waves of
// 32x32; BM = 32: 2 pixel halves x 2 channel halves (LDS reduction).
// Static LDS: 2 stages of (weight tile + CK*HPAD) floats (HaloShape).
// Compile-time shape of the halo kernel: kernel (KH, KW) -> pixel tile and
// channels per chunk.  1x5: 4x16 tiles (halo 4x20); 5x1, 3x3 and 1x1: 8x8
// tiles (halo 12x8 / 10x10 / none).  CK: 16 (BM 32) / 8 (BM 64), halved for
// 3x3, doubled for 1x1, so a thread stages <= 16 weights per chunk.
template <int BM, int KH, int KW>
struct HaloShape {
  static constexpr int T = KH * KW;
  static constexpr int TH = KW == 1 || (KH == 3 && KW == 3) ? 8 : 4;
  static constexpr int TW = 64 / TH;
  static constexpr int HWd = TW + KW - 1;
  static constexpr int HALO = (TH + KH - 1) * HWd;
  static constexpr int HPAD = HALO + ((32 - HALO % 64) + 64) % 64;   // channel stride = 32 mod 64 banks
  static constexpr int NJ = (HALO + 63) / 64;
  static constexpr int CK = (BM == 32 ? 16 : 8) * (T == 1 ? 2 : 1) / (T > 5 ? 2 : 1);
  static constexpr int RUN0 = CK * T, RUN1 = BM * T;                 // weight runs (fwd / dgrad)
  static constexpr int WS0 = RUN0 | 1, WS1 = RUN1 | 1;               // odd LDS strides
  static constexpr int WTOT = BM * CK * T;
  static constexpr int WPER = (WTOT + 255) / 256;
  static constexpr int WSZ0 = BM * WS0, WSZ1 = CK * WS1;
  static constexpr int STAGE = (WSZ0 > WSZ1 ? WSZ0 : WSZ1) + CK * HPAD;
  static constexpr int LDS = 2 * STAGE > 2 * 16 * 64 ? 2 * STAGE : 2 * 16 * 64;   // floats
  static_assert(NJ <= 4 && WPER <= 16 && CK % 4 == 0 && TH * TW == 64, "halo shape");
};

// ---- BatchNorm statistics in the conv epilogue (EPI 5 / 6, BnFuse)
// One arrival at a self-resetting counter: true in the block that arrives
// last (the counter is back at 0 for the next launch / graph replay).
// The partial sums go through agent-coherent accesses (bn_put / bn_get:
// written through to, and read from, the coherence point past the XCDs'
// L2s), so before the arrival every wave only waits for its own stores to be
// acknowledged (s_waitcnt 0) -- no agent-scope release fence, which writes
// back the whole L2 of the block's XCD in every block.
__device__ __forceinline__ bool last_arrival(unsigned* c, unsigned n, unsigned* flag) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = old == n - 1u;
    if (old == n - 1u) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return *flag != 0u;
}

__device__ __forceinline__ void bn_put(double2* p, double a, double b) {
  double* q = reinterpret_cast<double*>(p);
  __hip_atomic_store(q, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 1, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double2 bn_get(const double2* p) {
  double* q = const_cast<double*>(reinterpret_cast<const double*>(p));
  return make_double2(__hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                      __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// After a block wrote its tile's partials (part[pt][row]): the last block of
// each level-1 group of g1 pixel tiles folds the group (fixed order) into
// part2, and the last group of the row tile finalises its channels --
// batchnorm.hip's formulas (EPI 5: mean, biased variance, invstd, running
// statistics with the unbiased variance; EPI 6: mean(g), mean(g xhat),
// dgamma, dbeta).
// Sum of items p < n (item p of row r at base[p * rows + r]) by the T
// consecutive threads of row r: thread j loads items j, j + T, ... eight at a
// time (the agent-coherent loads in flight together), then the T lanes
// combine by a fixed butterfly -- a fixed order, every lane gets the sum.
__device__ __forceinline__ double2 bn_fold(const double2* base, int n, int rows, int r, int j, int T) {
  double s1 = 0.0, s2 = 0.0;
  for (int p0 = j; p0 < n; p0 += 8 * T) {
    double2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int p = p0 + u * T;
      v[u] = p < n ? bn_get(base + (size_t)p * rows + r) : make_double2(0.0, 0.0);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      s1 += v[u].x;
      s2 += v[u].y;
    }
  }
  for (int o = 1; o < T; o <<= 1) {
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  return make_double2(s1, s2);
}

// Channel r's statistics from its sums over the batch: batchnorm.hip's
// formulas (EPI 5: mean, biased variance, invstd, running statistics with the
// unbiased variance; EPI 6: mean(g), mean(g xhat), dgamma, dbeta)
template <int EPI>
__device__ __forceinline__ void bn_finalize_row(const BnFuse& f, int r, int rows, long long L, double s1, double s2) {
  if (EPI == 5) {
    const double mean = s1 / (double)L;
    double var = s2 / (double)L - mean * mean;
    var = var > 0.0 ? var : 0.0;
    const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
    const float mu = (float)mean;
    f.coef[r] = (f.gamma ? f.gamma[r] : 1.f) * invstd;
    f.coef[rows + r] = mu;
    f.coef[2 * rows + r] = f.beta ? f.beta[r] : 0.f;
    f.save_mean[r] = mu;
    f.save_invstd[r] = invstd;
    if (f.rmean) {
      const double unb = L > 1 ? var * (double)L / (double)(L - 1) : var;
      f.rmean[r] = (1.f - f.momentum) * f.rmean[r] + f.momentum * mu;
      f.rvar[r] = (1.f - f.momentum) * f.rvar[r] + f.momentum * (float)unb;
    }
    if (r == 0 && f.nbt) *f.nbt += 1;
  } else {   // the data-gradient staging coefficients of the producer (XF 3)
    const float invstd = f.invstd[r];
    f.coef[r] = (f.gamma ? f.gamma[r] : 1.f) * invstd;
    f.coef[rows + r] = (float)(s1 / (double)L);
    f.coef[2 * rows + r] = (float)(s2 / (double)L);
    f.coef[3 * rows + r] = f.mean[r];
    f.coef[4 * rows + r] = invstd;
    if (f.dgamma) f.dgamma[r] = (float)s2;
    if (f.dbeta) f.dbeta[r] = (float)s1;
  }
}

// In-kernel fold (BnFuse::inkernel, env DRO_BN_FOLD=kernel): after a block
// wrote its tile's partials (part[pt][row]), the last block of each level-1
// group of g1 pixel tiles folds the group (fixed order) into part2, and the
// last group of the row tile finalises its channels.  Measured slower in the
// training step than bn_finalize_kernel (the per-block store drain before
// each arrival and the serial tail under the other stream's load).
template <int EPI>
__device__ void bn_finish(const IgArgs& a, int pt, int rt, int row0, int bm) {
  __shared__ unsigned flag;
  const BnFuse& f = a.bn;
  if (f.dbg & 1) return;
  const int rows = a.rows, ptiles = a.g.B * a.tiles_img;
  const int grp = pt / f.g1, lo = grp * f.g1, n1 = min(f.g1, ptiles - lo);
  if (!last_arrival(f.cnt + (size_t)rt * f.ngroups + grp, (unsigned)n1, &flag)) return;
  // T threads per row (blockDim / bm: 4 .. 32, inside one wave)
  const int T = (int)blockDim.x / bm, rl = (int)threadIdx.x / T, j = (int)threadIdx.x - rl * T;
  const int r = row0 + rl;
  const bool live = r < rows;
  {
    const double2 v = bn_fold(f.part + (size_t)lo * rows, live ? n1 : 0, rows, live ? r : 0, j, T);
    if (live && j == 0) bn_put(f.part2 + (size_t)grp * rows + r, v.x, v.y);
  }
  if (!last_arrival(f.cnt + (size_t)a.row_tiles * f.ngroups + rt, (unsigned)f.ngroups, &flag)) return;
  const double2 v = bn_fold(f.part2, live ? f.ngroups : 0, rows, live ? r : 0, j, T);
  if (!live || j != 0) return;
  bn_finalize_row<EPI>(f, r, rows, (long long)a.g.B * a.g.H * a.g.W, v.x, v.y);
}

// The default: one small launch after the conv (kernel boundary: the
// partials are visible, no atomics or store drains in the conv's blocks).
// Block r folds channel r's ptiles partials: thread t sums tiles t, t + 256,
// ... in order, then a fixed tree over the block.
template <int EPI>
__global__ __launch_bounds__(256) void bn_finalize_kernel(BnFuse f, int rows, int ptiles, long long L) {
  __shared__ double red[2][4];
  const int r = blockIdx.x;
  double s1 = 0.0, s2 = 0.0;
  for (int p = threadIdx.x; p < ptiles; p += 256) {
    const double2 v = f.part[(size_t)p * rows + r];
    s1 += v.x;
    s2 += v.y;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = s1;
    red[1][w] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    bn_finalize_row<EPI>(f, r, rows, L, (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]),
                         (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]));
}

// KS > 1: intra-block K split.  The block is KS groups of 4 waves; group g
// stages and multiplies chunks g, g+KS, ... in its own LDS region, and the
// groups' accumulators are summed in group order at the end (more waves per
// tile to hide the staging latency, no split-K partials or finish launch).
template <int BM, int KH, int KW, int MODE, int ACT, int EPI, int KS, int XF = 0>
__global__ __launch_bounds__(256 * KS) void dconv_kernel(IgArgs a) {
  using S = HaloShape<BM, KH, KW>;
  {   // diagnostics: kernel entry of wave 0 (slot 10) and of the block's last wave (slot 11)
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (a.stamps && (threadIdx.x == 0 || threadIdx.x == blockDim.x - 64))
      a.stamps[(size_t)blockIdx.x * 16 + (threadIdx.x == 0 ? 10 : 11)] = t0;
  }
  // staging prefetch distance: 2 chunks when the register budget allows
  // (<= 8 waves per CU); 4 wave groups per block run at 128 VGPRs with 1
  constexpr int PF = KS <= 2 ? 2 : 1;
  static_assert(KS == 1 || S::LDS >= 4 * 16 * 64, "cross-group reduction area");
  constexpr int T = S::T, TH = S::TH, TW = S::TW, HWd = S::HWd, HALO = S::HALO, HPAD = S::HPAD;
  constexpr int CK = S::CK, NJ = S::NJ, XPER = CK / 4;
  constexpr int RUN = MODE == 0 ? S::RUN0 : S::RUN1, WS = MODE == 0 ? S::WS0 : S::WS1;
  constexpr int WSZ = MODE == 0 ? S::WSZ0 : S::WSZ1, STAGE = S::STAGE;
  constexpr int WM = BM / 32;
  constexpr int PH = KH / 2, PW = KW / 2;
  __shared__ float smem_all[KS * S::LDS];
  const int cb1 = a.cbase[1], cb2 = a.cbase[2], cb3 = a.cbase[3];
  const int H = a.g.H, W = a.g.W;
  const int Cin = a.g.Cin, Cout = a.g.Cout, rows = a.rows, kch = a.kch;
  const int CinT = Cin * T;
  const float* __restrict__ Wt = a.weight;
  const float* __restrict__ Gp = a.G;
  const int tid = threadIdx.x & 255, lane = tid & 63;
  const int grp = KS == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 8);
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave in the group (scalar)
  float* smem = smem_all + grp * S::LDS;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int pt = (int)udiv((unsigned)tile, a.rt_div), rt = tile - pt * a.row_tiles;
  const int row0 = rt * BM;
  const int b = (int)udiv((unsigned)pt, a.ti_div), trem = pt - b * a.tiles_img;
  const int tyi = (int)udiv((unsigned)trem, a.tx_div);
  const int ty0 = tyi * TH, tx0 = (trem - tyi * a.tiles_x) * TW;
  const size_t HW = (size_t)H * W;
  const unsigned HWu = (unsigned)HW;
  const int nck = (kch + CK - 1) / CK;
  const int cbeg = blockIdx.y * a.chunks_per_split;
  const int cend = min(nck, cbeg + a.chunks_per_split);

  // X staging: wave w stages the XPER consecutive channels w*XPER.. of a chunk;
  // lanes run over the halo in NJ passes whose byte offsets are chunk
  // independent (lanes outside the image read pixel 0 and are zeroed when staged)
  unsigned xpb[NJ];
  bool xok[NJ], own[NJ];
  static_assert(XF == 0 || ((MODE == 0) == (XF != 3) && ACT == 0), "BN staging transforms: XF 1/2 forward, 3 data gradient");
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int e = lane + 64 * j;
    const int hy = e / HWd, hx = e - hy * HWd;
    const int yy = ty0 - PH + hy, xx = tx0 - PW + hx;
    xok[j] = e < HALO && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
    xpb[j] = xok[j] ? 4u * (unsigned)(yy * W + xx) : 0u;
    // XF: the transformed source is stored at the pixels of the block's own
    // tile, for the chunks whose index is its row tile modulo the row tiles
    // (prep: Stage::ownc) -- every element exactly once, spread over the blocks
    own[j] = XF != 0 && xok[j] && hy >= PH && hy < PH + TH && hx >= PW && hx < PW + TW;
  }
  const unsigned wlast = (unsigned)Cout * CinT - 1;

  // Source table in SGPRs (built once): channel ch of source s starts at byte
  // address sQ[s] + ch * sR[s] (+ 4 * pixel unless broadcast: sM[s] = 0).  Per
  // channel the staging adds the deltas of the sources the channel has passed
  // (masks from three compares): scalar arithmetic, no branches, so the loads
  // share a basic block with the MFMAs
  unsigned long long sQ[4];
  unsigned sR[4], sM[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (MODE == 0) {
      sQ[t] = a.sq0[t] + (unsigned long long)b * a.sqb[t];
      sR[t] = a.sr[t];
      sM[t] = a.sm[t];
    } else {
      sQ[t] = reinterpret_cast<unsigned long long>(Gp) + 4ull * (unsigned long long)b * Cout * HW;
      sR[t] = 4u * HWu;
      sM[t] = ~0u;
    }
  }
  const unsigned long long dQ1 = sQ[1] - sQ[0], dQ2 = sQ[2] - sQ[1], dQ3 = sQ[3] - sQ[2];
  const unsigned dR1 = sR[1] - sR[0], dR2 = sR[2] - sR[1], dR3 = sR[3] - sR[2];
  const unsigned dM1 = sM[1] - sM[0], dM2 = sM[2] - sM[1], dM3 = sM[3] - sM[2];
  // second staged stream at the same offsets: the folded activation's y
  // (FOLD), the skip (XF 2) or the BN input z (XF 3); XF owner stores go to yout
  const long long sbase = MODE == 0 ? reinterpret_cast<long long>(a.src[0].p) : reinterpret_cast<long long>(Gp);
  const long long yshift = reinterpret_cast<long long>(XF == 2 ? a.bn.skip : XF == 3 ? a.bn.z : a.gy) - sbase;
  const long long oshift = reinterpret_cast<long long>(a.bn.yout) - sbase;

  // MODE 1 with ACT != 0: the activation derivative is folded into G staging
  constexpr bool FOLD = MODE == 1 && ACT != 0;
  constexpr bool Y2 = FOLD || XF == 2 || XF == 3;
  constexpr int NXC = XF == 3 ? 5 : 3;   // BN coefficients per staged channel
  const float galpha = a.galpha;
  // weights are staged as float4 runs (a run never crosses a weight row: RUN %
  // 4 == 0); starts need only dword alignment; per-thread offsets are chunk
  // independent.  Tensors of < 4 weights take the flat path (plan_igemm).
  constexpr int W4 = S::WTOT / 4, WPER4 = (W4 + 255) / 256;
  constexpr int WREG = 4 * WPER4;
  static_assert(S::WTOT % 4 == 0 && RUN % 4 == 0, "float4 weight runs");
  unsigned woff[WPER4];
  int wdst[WPER4];
#pragma unroll
  for (int i = 0; i < WPER4; ++i) {
    const int e = 4 * (tid + 256 * i);
    const int run = e / RUN, rem = e - run * RUN;
    woff[i] = (unsigned)run * CinT + (unsigned)rem;
    wdst[i] = (W4 % 256 == 0 || e < S::WTOT) ? run * WS + rem : -1;
  }
  // one chunk's staging registers; with PF == 2 two sets alternate so the
  // loads of chunk c+2 are in flight while chunk c is multiplied
  typedef __attribute__((address_space(1))) char* GWPtr;
  struct Stage {
    float xr[XPER * NJ], yr[Y2 ? XPER * NJ : 1], wv[WREG];
    unsigned cmask;   // scalar: bit i = channel i of this wave exists
    unsigned ownc;    // XF, scalar: this block stores this chunk's transformed values
    float xc[XF ? NXC * XPER : 1];   // XF: the staged channels' BN coefficients (scalar)
    GWPtr yo[XF ? XPER : 1];         // XF: owner-store rows
  };
  // a chunk's loads: scalar set-up (weight base, one row address per channel),
  // then NVM independent load items that the MFMA loop can interleave
  typedef __attribute__((address_space(1))) const char* GPtr;   // global, not flat
  typedef __attribute__((address_space(1))) const float* GFPtr;
  struct Rows {
    unsigned gbase;
    GPtr rowp[XPER], yrow[XPER];
    unsigned M[XPER];
  };
  constexpr int NVM = WPER4 + XPER * NJ;
  auto prep = [&](Stage& st, int chunk, Rows& r) {
    const int c0 = chunk * CK;
    r.gbase = MODE == 0 ? (unsigned)row0 * CinT + (unsigned)c0 * T : (unsigned)c0 * CinT + (unsigned)row0 * T;
    unsigned cm = 0;
#pragma unroll
    for (int i = 0; i < XPER; ++i) {
      const int ch = c0 + wave * XPER + i;          // scalar
      const bool cok = ch < kch;
      cm |= cok ? (1u << i) : 0u;
      const int cc = cok ? ch : 0;
      const unsigned long long k1 = MODE == 0 ? 0ull - (unsigned long long)(cc >= cb1) : 0ull;
      const unsigned long long k2 = MODE == 0 ? 0ull - (unsigned long long)(cc >= cb2) : 0ull;
      const unsigned long long k3 = MODE == 0 ? 0ull - (unsigned long long)(cc >= cb3) : 0ull;
      const unsigned j1 = (unsigned)k1, j2 = (unsigned)k2, j3 = (unsigned)k3;
      const unsigned long long Q = sQ[0] + (dQ1 & k1) + (dQ2 & k2) + (dQ3 & k3);
      const unsigned R = sR[0] + (dR1 & j1) + (dR2 & j2) + (dR3 & j3);
      r.M[i] = sM[0] + (dM1 & j1) + (dM2 & j2) + (dM3 & j3);
      const unsigned long long rq = Q + (unsigned long long)(unsigned)cc * R;
      r.rowp[i] = reinterpret_cast<GPtr>(rq);
      r.yrow[i] = reinterpret_cast<GPtr>(rq + (unsigned long long)yshift);
      if (XF) {
        st.yo[i] = reinterpret_cast<GWPtr>(rq + (unsigned long long)oshift);
#pragma unroll
        for (int k = 0; k < NXC; ++k) st.xc[k * XPER + i] = a.bn.xcoef[k * kch + cc];
      }
    }
    st.cmask = cm;
    if (XF) st.ownc = (unsigned)(chunk % a.row_tiles) == (unsigned)rt ? ~0u : 0u;
  };
  auto item = [&](Stage& st, const Rows& r, int k) {
    if (k < WPER4) {
      const unsigned g = r.gbase + woff[k];
      const float4 v = *reinterpret_cast<const float4*>(Wt + (g < wlast - 3 ? g : wlast - 3));
      st.wv[4 * k] = v.x;
      st.wv[4 * k + 1] = v.y;
      st.wv[4 * k + 2] = v.z;
      st.wv[4 * k + 3] = v.w;
    } else {
      const int q = k - WPER4, i = q / NJ, j = q - i * NJ;
      const unsigned o = xpb[j] & r.M[i];
      st.xr[q] = *reinterpret_cast<GFPtr>(r.rowp[i] + o);
      if (Y2) st.yr[q] = *reinterpret_cast<GFPtr>(r.yrow[i] + o);
    }
  };
  auto load = [&](Stage& st, int chunk) {
    Rows r;
    prep(st, chunk, r);
#pragma unroll
    for (int k = 0; k < NVM; ++k) item(st, r, k);
  };
  auto store = [&](const Stage& st, int buf) {
    const float(&xr)[XPER * NJ] = st.xr;
    const float(&yr)[Y2 ? XPER * NJ : 1] = st.yr;
    const float(&wv)[WREG] = st.wv;
    float* Ws = smem + buf * STAGE;
    float* Xs = Ws + WSZ + wave * XPER * HPAD + lane;
    auto xval = [&](int i, int j) {
      const bool ok = ((st.cmask >> i) & 1u) && xok[j];
      float v = ok ? xr[i * NJ + j] : 0.f;
      if (XF == 1 || XF == 2) {   // BN (+ skip) + ReLU of the producer (batchnorm.hip bn_fused_fwd_kernel)
        const float r = fmaf(v - st.xc[XPER + i], st.xc[i], st.xc[2 * XPER + i]) + (XF == 2 ? yr[i * NJ + j] : 0.f);
        v = ok ? fmaxf(r, 0.f) : 0.f;
      } else if (XF == 3) {       // BN backward (bn_fused_bwd_kernel): dz from g and z
        const float xh = (yr[i * NJ + j] - st.xc[3 * XPER + i]) * st.xc[4 * XPER + i];
        const float r = st.xc[i] * (v - st.xc[XPER + i] - xh * st.xc[2 * XPER + i]);
        v = ok ? r : 0.f;
      }
      if (XF && own[j] && ((st.cmask & st.ownc) >> i & 1u)) *reinterpret_cast<__attribute__((address_space(1))) float*>(st.yo[i] + xpb[j]) = v;
      if (MODE == 1) v *= galpha;
      if (FOLD) v *= act_bwd(yr[i * NJ + j], ACT);
      return v;
    };
    constexpr int JF = NJ * 64 <= HPAD ? NJ : NJ - 1;   // passes that fit the channel stride
#pragma unroll
    for (int i = 0; i < XPER; ++i) {
#pragma unroll
      for (int j = 0; j < JF; ++j) Xs[i * HPAD + 64 * j] = xval(i, j);
    }
    if (JF < NJ && lane + 64 * (NJ - 1) < HPAD) {   // (XF owners: e < HALO <= HPAD, all inside)
#pragma unroll
      for (int i = 0; i < XPER; ++i) Xs[i * HPAD + 64 * (NJ - 1)] = xval(i, NJ - 1);
    }
#pragma unroll
    for (int i = 0; i < WPER4; ++i) {
      if (W4 % 256 == 0 || wdst[i] >= 0) {
        float* d = Ws + wdst[i];   // odd row stride: 4 dword writes
        d[0] = wv[4 * i];
        d[1] = wv[4 * i + 1];
        d[2] = wv[4 * i + 2];
        d[3] = wv[4 * i + 3];
      }
    }
  };

  const int wr = (WM == 2) ? (wave & 1) : 0;
  const int wc = (WM == 2) ? (wave >> 1) : (wave & 1);
  const int wk = (WM == 2) ? 0 : (wave >> 1);
  const int q = wc * 32 + (lane & 31);          // this lane's pixel in the tile (MFMA column)
  const int qy = q / TW, qx = q - qy * TW;
  const int qoff = qy * HWd + qx;
  const int hi = lane >> 5;
  const int arow = wr * 32 + (lane & 31);       // this lane's A row in the tile
  constexpr int NS = (WM == 2) ? CK / 2 : CK / 4;   // channel pairs per wave per tap
  const int s_lo = (WM == 2) ? 0 : wk * NS;
  constexpr int ASTEP = MODE == 0 ? 2 * T : 2 * WS;  // A offset per channel pair
  const int abase = (MODE == 0 ? arow * WS + hi * T : hi * WS + arow * T) + s_lo * ASTEP;
  const int bbase = hi * HPAD + qoff + 2 * s_lo * HPAD;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

  // group grp handles chunks cbeg + grp, cbeg + grp + KS, ...; every group
  // runs the same number of iterations (barriers are block wide)
  const int nit = (cend - cbeg + KS - 1) / KS;
  auto chunk_of = [&](int it) { return cbeg + it * KS + grp; };
  unsigned long long* const stp = a.stamps ? a.stamps + (size_t)blockIdx.x * 16 : nullptr;
  auto stamp = [&](int k) {   // slots: 10/11 entry, 0 set-up done, 12 first chunk staged, 1
                                // prologue, 2.. K iterations (<= 8), 13 reductions, 14 epilogue
    if (stp && threadIdx.x == 0 && k < 15) stp[k] = __builtin_amdgcn_s_memtime();
  };
  stamp(0);
  // slot 15: start of the block's last wave (intra-block launch spread)
  if (stp && threadIdx.x == blockDim.x - 64) stp[15] = __builtin_amdgcn_s_memtime();
  // MFMAs over one staged chunk; with `st` the next chunk's load items are
  // issued one after each MFMA (sched_barrier keeps MFMAs and global loads in
  // this order and lets LDS reads / ALU move): issued as a burst ahead of the
  // MFMAs, the loads of all 16 waves queued at the texture unit and held every
  // wave's first MFMA back (profiles/r1_conv_phase_stamps.txt)
  auto mma_ld = [&](int buf, Stage* st, const Rows* r) {
    const float* wa = smem + buf * STAGE + abase;
    const float* xb = smem + buf * STAGE + WSZ + bbase;
    constexpr int NMF = T * NS, PD = 2;   // MFMAs per chunk; LDS operand prefetch distance
    auto aoff = [](int k) { return (k / NS) + (k % NS) * ASTEP; };
    auto boff = [](int k) {
      const int tap = k / NS, s = k % NS, ty = tap / KW, tx = tap % KW;
      return (MODE == 0 ? ty * HWd + tx : (KH - 1 - ty) * HWd + (KW - 1 - tx)) + 2 * s * HPAD;
    };
    float av[PD + 1], bv[PD + 1];
#pragma unroll
    for (int k = 0; k < PD && k < NMF; ++k) {
      av[k] = wa[aoff(k)];
      bv[k] = xb[boff(k)];
    }
#pragma unroll
    for (int k = 0; k < NMF; ++k) {
      if (k + PD < NMF) {
        av[(k + PD) % (PD + 1)] = wa[aoff(k + PD)];
        bv[(k + PD) % (PD + 1)] = xb[boff(k + PD)];
      }
      acc = mfma32(av[k % (PD + 1)], bv[k % (PD + 1)], acc);
      if (st) {
        if (k < NVM) item(*st, *r, k);
        // MFMAs, LDS reads and global loads stay in this order; ALU may move
        __builtin_amdgcn_sched_barrier(0x0006);
      }
    }
    if (st) {
#pragma unroll
      for (int k = NMF; k < NVM; ++k) item(*st, *r, k);
    }
  };
  auto mma = [&](int buf) { mma_ld(buf, nullptr, nullptr); };
  Stage sa, sb;
  if (chunk_of(0) < cend) {
    load(sa, chunk_of(0));
    store(sa, 0);
  }
  stamp(12);   // wave 0's first chunk landed in LDS
  if (PF == 2 && chunk_of(1) < cend) load(sb, chunk_of(1));
  __syncthreads();
  stamp(1);
  const int dbg = ablation_flags(a.dbg);
  if (PF == 1) {
    for (int it = 0; it < nit; ++it) {
      const int buf = it & 1;
      const bool more = chunk_of(it + 1) < cend;
      if (more && !(dbg & 3)) {
        Rows r;
        prep(sa, chunk_of(it + 1), r);
        mma_ld(buf, &sa, &r);
      } else {
        if (more && !(dbg & 1)) load(sa, chunk_of(it + 1));
        if ((KS == 1 || chunk_of(it) < cend) && !(dbg & 2)) mma(buf);
      }
      if (more && !(dbg & 4)) store(sa, buf ^ 1);
      __syncthreads();
      if (it < 8) stamp(2 + it);
    }
  } else {
    // registers: sb holds chunk it+1 (stored into LDS at the end of
    // iteration it), sa receives chunk it+2
    for (int it = 0; it < nit; it += 2) {
      if (chunk_of(it + 2) < cend) load(sa, chunk_of(it + 2));
      if (chunk_of(it) < cend) mma(0);
      if (chunk_of(it + 1) < cend) store(sb, 1);
      __syncthreads();
      if (it < 8) stamp(2 + it);
      if (it + 1 >= nit) break;
      if (chunk_of(it + 3) < cend) load(sb, chunk_of(it + 3));
      if (chunk_of(it + 1) < cend) mma(1);
      if (chunk_of(it + 2) < cend) store(sa, 0);
      __syncthreads();
      if (it < 7) stamp(3 + it);
    }
  }
  // Reduction + epilogue spread over ALL waves of the block: every wave parks
  // its accumulator (one partial set per (group, K half)) in LDS, then each
  // thread sums a few tile elements over the sets in a fixed order and runs
  // the epilogue for them -- instead of one or two waves doing the whole tile
  // (that serial tail cost as much as the K loop; profiles/r1_conv_phase_stamps.txt).
  constexpr int NSET = (WM == 1 ? 2 : 1) * KS;
  static_assert(NSET * BM * 64 <= KS * S::LDS, "reduction sets fit in the staging LDS");
  {
    const int set = grp * (WM == 1 ? 2 : 1) + (WM == 1 ? wk : 0);
    float* red = smem_all + (size_t)set * BM * 64;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rl = wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      red[rl * 64 + wc * 32 + (lane & 31)] = acc[r];
    }
  }
  __syncthreads();
  stamp(13);
  const long long P = (long long)a.g.B * HW;
  if constexpr (EPI >= 5) {
    // BN statistics of the tile: each thread finishes its elements (output /
    // g stored) and parks the value the statistics need in LDS at the
    // element's set-0 slot (only this thread reads that element's sets);
    // then one thread per row sums the row's 64 pixels in order (fp64) --
    // EPI 6 in two passes (g, then g * xhat, kept in registers meanwhile)
    constexpr int NIT = BM * 64 / (256 * KS);
    float second[EPI == 6 ? NIT : 1];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int e = (int)threadIdx.x + it * 256 * KS;
      const int rl = e >> 6, pl = e & 63;
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < KS; ++g) {
        if (WM == 1)
          v += smem_all[((size_t)(2 * g) * BM + rl) * 64 + pl] + smem_all[((size_t)(2 * g + 1) * BM + rl) * 64 + pl];
        else
          v += smem_all[((size_t)g * BM + rl) * 64 + pl];
      }
      const int row = row0 + rl;
      const int py = pl / TW, px = pl - py * TW;
      const int oy = ty0 + py, ox = tx0 + px;
      float first = 0.f;
      if (EPI == 6) second[it] = 0.f;
      if (row < rows && oy < H && ox < W) {
        const size_t epix = (size_t)oy * W + ox;
        if (EPI == 5) {
          first = v + (a.bias ? a.bias[row] : 0.f);
          a.out[((size_t)b * a.out_ctot + a.out_coff + row) * HW + epix] = first;
        } else {
          const size_t idx = ((size_t)b * rows + row) * HW + epix;
          first = a.bn.y[idx] > 0.f ? v : 0.f;
          const float xh = (a.bn.z[idx] - a.bn.mean[row]) * a.bn.invstd[row];
          a.gsrc[0][idx] = first;
          second[it] = first * xh;
        }
      }
      smem_all[e] = first;
    }
    __syncthreads();
    const int rl = threadIdx.x, row = row0 + rl;
    const bool rowt = rl < BM && row < rows && !(a.bn.dbg & 4);
    double s1 = 0.0, s2 = 0.0;
    if (rowt) {
#pragma unroll 16
      for (int p = 0; p < 64; ++p) {
        const double v = smem_all[rl * 64 + p];
        s1 += v;
        if (EPI == 5) s2 += v * v;
      }
    }
    if (EPI == 6) {
      __syncthreads();
#pragma unroll
      for (int it = 0; it < NIT; ++it) smem_all[(int)threadIdx.x + it * 256 * KS] = second[EPI == 6 ? it : 0];
      __syncthreads();
      if (rowt) {
#pragma unroll 16
        for (int p = 0; p < 64; ++p) s2 += (double)smem_all[rl * 64 + p];
      }
    }
    if (rowt && !(a.bn.dbg & 2)) bn_put(a.bn.part + (size_t)pt * rows + row, s1, s2);
    if (a.bn.inkernel) bn_finish<EPI>(a, pt, rt, row0, BM);
    stamp(14);
    return;
  }
  for (int e = threadIdx.x; e < BM * 64; e += 256 * KS) {
    const int rl = e >> 6, pl = e & 63;
    float v = 0.f;
#pragma unroll
    for (int g = 0; g < KS; ++g) {
      if (WM == 1)
        v += smem_all[((size_t)(2 * g) * BM + rl) * 64 + pl] + smem_all[((size_t)(2 * g + 1) * BM + rl) * 64 + pl];
      else
        v += smem_all[((size_t)g * BM + rl) * 64 + pl];
    }
    const int row = row0 + rl;
    const int py = pl / TW, px = pl - py * TW;
    const int oy = ty0 + py, ox = tx0 + px;
    if (row >= rows || oy >= H || ox >= W) continue;
    const size_t epix = (size_t)oy * W + ox;
    if (a.part)   // split-K partial: [split][rows][P]
      a.part[(size_t)blockIdx.y * rows * P + (size_t)row * P + (size_t)b * HW + epix] = v;
    else
      epi_store<MODE, ACT, EPI>(a, row, b, epix, HW, v);
  }
  stamp(14);
}


// ------------------------------------------------------------------ weight (+ bias) gradient
// dW[o, n] = sum_p G[o, p] * X[c(n), p + d(tap(n))] with n = tap*Cin + c, and
// column n = NK (= Cin*T) of X all ones, giving db[o] = sum_p G[o, p].
// rows = o (64), cols = n (64), K = the pixels of split blockIdx.y in chunks
// of 64.  Lane = pixel; wave w stages rows o0+16w.. and columns n0+16w.., so
// every row / column decode is wave-uniform.  Writes per-split partials
// [split][Cout][NK+1].
// One LDS stage (33 KB, 4 blocks per CU) with the next chunk held in
// registers: the double-buffered 66 KB allowed 2 blocks per CU, too few waves
// to cover the gathers' latency (the stems' weight gradients ran at 18-23 TF/s).
__global__ __launch_bounds__(256) void wgrad_kernel(IgArgs a) {
  constexpr int NB = 1;
  __shared__ float Gs[NB][kWP][64 + 1];
  __shared__ float Xs[NB][kWP][64 + 1];
  const int cb1 = a.cbase[1], cb2 = a.cbase[2], cb3 = a.cbase[3];
  const int H = a.g.H, W = a.g.W, KW = a.g.KW, PH = a.g.PH, PW = a.g.PW;
  const int Hsrc = a.Hs, Wsrc = a.Ws, sh = a.sshift;   // input size, log2 stride
  const unsigned HWs = (unsigned)Hsrc * (unsigned)Wsrc;
  const int Cin = a.g.Cin, Cout = a.g.Cout;
  const float* __restrict__ Gp = a.G;
  const FastDiv cindiv = a.cindiv, kwdiv = a.kwdiv;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int t = blockIdx.x;
  const int ot = t % a.otiles, nt = t / a.otiles;
  const int o0 = ot * 64, n0 = nt * 64;
  const int NK = a.K;                         // Cin * T; column NK = bias
  const int NC = a.gbias ? NK + 1 : NK;       // columns computed
  const size_t HW = (size_t)H * W;
  const unsigned HWu = (unsigned)HW;
  const long long P = (long long)a.g.B * HW;
  const long long pbeg = (long long)blockIdx.y * a.pchunk;
  const long long pend = pbeg + a.pchunk < P ? pbeg + a.pchunk : P;
  float gr[16], xr[16];
  unsigned gmask = 0, xmask = 0, omask = 0;

  auto load = [&](long long q0) {
    const long long p = q0 + lane;
    const bool v = p < pend;
    const int b = v ? (int)(p / (long long)HW) : 0;
    const int pix = v ? (int)(p - (long long)b * HW) : 0;
    const int py = pix / W, px = pix - py * W;
    gmask = 0;
    xmask = 0;
    omask = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int o = o0 + wave * 16 + j;        // wave-uniform
      const bool gok = v && o < Cout;
      gmask |= gok ? (1u << j) : 0u;
      gr[j] = Gp[gok ? ((unsigned)b * Cout + o) * HWu + pix : 0u];
      const int n = __builtin_amdgcn_readfirstlane(n0 + wave * 16 + j);
      const bool nv = n < NK;
      const int tap = nv ? fdiv(n, cindiv) : 0, ch = nv ? n - tap * Cin : 0;
      const int ty = fdiv(tap, kwdiv), dy = ty - PH, dx = tap - ty * KW - PW;
      const int yy = (py << sh) + dy, xx = (px << sh) + dx;
      const bool ok = v && nv && (unsigned)yy < (unsigned)Hsrc && (unsigned)xx < (unsigned)Wsrc;
      const unsigned spix = (unsigned)(yy * Wsrc + xx);
      xmask |= ok ? (1u << j) : 0u;
      omask |= (v && n == NK) ? (1u << j) : 0u;
      const RowDesc d = row_desc(cb1, cb2, cb3, ch, HWs);
      const unsigned e = (unsigned)b * d.A + d.Bc + (d.M ? spix : 0u);
      xr[j] = d.p[ok ? e : 0u];
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      Gs[buf][lane][wave * 16 + j] = (gmask >> j) & 1u ? gr[j] : 0.f;
      Xs[buf][lane][wave * 16 + j] = (xmask >> j) & 1u ? xr[j] : ((omask >> j) & 1u ? 1.f : 0.f);
    }
  };

  const int wo = wave & 1, wc = wave >> 1;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  if (pbeg < pend) {
    load(pbeg);
    store(0);
  }
  __syncthreads();
  int buf = 0;
  for (long long q0 = pbeg; q0 < pend; q0 += kWP) {
    const bool more = q0 + kWP < pend;
    if (more) load(q0 + kWP);
#pragma unroll
    for (int s = 0; s < kWP / 2; ++s) {
      const int kk = s * 2 + (lane >> 5);
      acc = mfma32(Gs[buf][kk][wo * 32 + (lane & 31)], Xs[buf][kk][wc * 32 + (lane & 31)], acc);
    }
    if (NB == 1) __syncthreads();          // every wave is done reading the stage
    if (more) store(NB == 1 ? 0 : buf ^ 1);
    __syncthreads();
    buf = NB == 1 ? 0 : buf ^ 1;
  }
  float* wp = a.part + (size_t)blockIdx.y * Cout * (NK + 1);
  const int n = n0 + wc * 32 + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int o = o0 + wo * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (o < Cout && n < NC) wp[(size_t)o * (NK + 1) + n] = acc[r];
  }
}

// ------------------------------------------------------------------ batched weight gradient
// One weight used by up to kMaxUse convolutions of a training step (the
// recurrent update blocks apply every weight once per iteration): the weight
// gradient of all uses is ONE launch whose pixel tiles run over
// (use, image, tile).  Each use brings its own sources, output gradient and
// saved activation output, read from this table in the kernel-argument
// segment with a wave-uniform use index.
constexpr int kMaxUse = 16;
struct WgMulti {
  IgArgs a;               // geometry, cbase, weight-gradient targets, plan (a.src = use 0)
  int nuse;
  int use_tiles;          // pixel tiles per use = B * tiles_img
  Slice usrc[kMaxUse][kMaxSrc];
  const float* uG[kMaxUse];
  const float* uy[kMaxUse];
};

template <bool MULTI>
struct WgParam {
  typedef IgArgs T;
  static __device__ __forceinline__ const IgArgs& ig(const IgArgs& x) { return x; }
};
template <>
struct WgParam<true> {
  typedef WgMulti T;
  static __device__ __forceinline__ const IgArgs& ig(const WgMulti& x) { return x.a; }
};

typedef const float* FPtr;
typedef __attribute__((address_space(4))) const FPtr* KFPtr;

__device__ __forceinline__ __attribute__((address_space(4))) const char* kernarg_base() {
  return (__attribute__((address_space(4))) const char*)__builtin_amdgcn_kernarg_segment_ptr();
}

// ------------------------------------------------------------------ halo-tiled weight gradient
// dW[o, c, tap] = sum_p G[o, p] X[c, p + d(tap)] for (KH, KW) in {1x5, 5x1, 3x3}:
// block = 64 output channels x 32 input channels x all taps, K = the pixels of
// a run of TH x TW pixel tiles.  Per tile the G tile [64 px][64 o] and the X
// patch [32 c][halo] are staged once; tap (ty, tx) reads the patch shifted.
// Waves: 2 (o halves) x 2, the second pair splitting either the taps (3x3:
// 5 + 4 per wave, no reduction) or the pixels (T = 5: summed through LDS at
// the end, one tap at a time).  Blocks of channel tile 0 also sum G over their
// pixels for the bias.  Partials: weights [split][Cout][Cin][T], bias [split][Cout].
template <int KH, int KW>
struct HaloShapeW {
  static constexpr int T = KH * KW;
  // 3x3: taps split 5 + 4 over the wave pairs (all 9 taps per wave over half
  // the pixels measured no faster and needs 512 registers per lane)
  static constexpr bool TAPSPLIT = T == 9;
  static constexpr int TPW = TAPSPLIT ? 5 : T;   // accumulators (taps) per wave
  static constexpr int TH = HaloShape<32, KH, KW>::TH, TW = 64 / TH;
  static constexpr int HWd = TW + KW - 1;
  static constexpr int HALO = (TH + KH - 1) * HWd;
  static constexpr int HPAD = HALO | 1;          // odd: lanes read 32 channels at stride HPAD
  static constexpr int NJ = (HALO + 63) / 64;
  static constexpr int BC = 32;                  // input channels per block
  static constexpr int GPAD = 65;                // [px][o] row stride
  static constexpr int STAGE = 64 * GPAD + BC * HPAD;
  static constexpr int LDS = 2 * STAGE > 2 * 16 * 64 * 2 ? 2 * STAGE : 2 * 16 * 64 * 2;
  static_assert(NJ <= 2 && TW % 2 == 0, "halo shape");
};

template <int KH, int KW, int GACT, bool MULTI>
__global__ __launch_bounds__(256) void wgrad_halo_kernel(typename WgParam<MULTI>::T P) {
  const IgArgs& a = WgParam<MULTI>::ig(P);
  using S = HaloShapeW<KH, KW>;
  constexpr int T = S::T, TH = S::TH, TW = S::TW, HWd = S::HWd, HALO = S::HALO, HPAD = S::HPAD;
  constexpr int NJ = S::NJ, BC = S::BC, GPAD = S::GPAD, STAGE = S::STAGE, TPW = S::TPW;
  constexpr bool TAPSPLIT = S::TAPSPLIT;
  constexpr int PH = KH / 2, PW = KW / 2;
  __shared__ float smem[S::LDS];
  const int cb1 = a.cbase[1], cb2 = a.cbase[2], cb3 = a.cbase[3];
  const int H = a.g.H, W = a.g.W, Cin = a.g.Cin, Cout = a.g.Cout;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int t = blockIdx.x;
  const int ot = t % a.otiles, ct = t / a.otiles;
  const int o0 = ot * 64, c0 = ct * BC;
  const size_t HW = (size_t)H * W;
  const unsigned HWu = (unsigned)HW;
  int ntiles = a.g.B * a.tiles_img;
  if constexpr (MULTI) ntiles = P.use_tiles * P.nuse;
  const int tbeg = blockIdx.y * a.chunks_per_split;
  const int tend = min(ntiles, tbeg + a.chunks_per_split);
  const bool do_bias = a.gbias && ct == 0;
  const float galpha = a.galpha;
  float gr[16], yr[GACT ? 16 : 1], xr[8 * NJ], bsum[16];
  unsigned gmask = 0, xmask = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) bsum[j] = 0.f;
  auto load = [&](int tile) {
    const float* __restrict__ Gp = a.G;
    const float* __restrict__ Yp = a.gy;
    KSlice sbase = kernarg_srcs();
    if constexpr (MULTI) {   // wave-uniform use index: its sources, G and y from the kernarg table
      const int u = tile / P.use_tiles;
      tile -= u * P.use_tiles;
      Gp = *(KFPtr)(kernarg_base() + offsetof(WgMulti, uG) + u * sizeof(FPtr));
      if (GACT) Yp = *(KFPtr)(kernarg_base() + offsetof(WgMulti, uy) + u * sizeof(FPtr));
      sbase = (KSlice)(kernarg_base() + offsetof(WgMulti, usrc)) + u * kMaxSrc;
    }
    const int b = tile / a.tiles_img, trem = tile - b * a.tiles_img;
    const int ty0 = (trem / a.tiles_x) * TH, tx0 = (trem % a.tiles_x) * TW;
    // G tile: lane = pixel of the tile, wave w -> output channels o0 + 16w + j
    const int qy = lane / TW, qx = lane - qy * TW;
    const int oy = ty0 + qy, ox = tx0 + qx;
    const bool pin = oy < H && ox < W;
    const unsigned pix = pin ? (unsigned)(oy * W + ox) : 0u;
    gmask = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int o = o0 + wave * 16 + j;        // scalar
      const bool ok = pin && o < Cout;
      gmask |= ok ? (1u << j) : 0u;
      const unsigned off = ok ? ((unsigned)b * Cout + o) * HWu + pix : 0u;
      gr[j] = Gp[off];
      if (GACT) yr[j] = Yp[off];
    }
    // X patch: wave w -> channels c0 + w + 4i, lanes over the halo
    // every channel's descriptor first (independent scalar loads, one wait),
    // then the patch loads
    RowDesc ds[8];
    bool real[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int ch = c0 + wave + 4 * i;          // scalar
      real[i] = ch < Cin;
      ds[i] = row_desc_at(sbase, cb1, cb2, cb3, real[i] ? ch : 0, HWu);
    }
    xmask = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const unsigned xbase = (unsigned)b * ds[i].A + ds[i].Bc;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int e = lane + 64 * j;
        const int hy = e / HWd, hx = e - hy * HWd;
        const int yy = ty0 - PH + hy, xx = tx0 - PW + hx;
        const bool ok = real[i] && e < HALO && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
        xmask |= ok ? (1u << (i * NJ + j)) : 0u;
        xr[i * NJ + j] = ds[i].p[ok ? xbase + (ds[i].M ? (unsigned)(yy * W + xx) : 0u) : 0u];
      }
    }
  };
  auto store = [&](int buf) {
    float* Gs = smem + buf * STAGE;
    float* Xs = Gs + 64 * GPAD;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      float g = (gmask >> j) & 1u ? galpha * gr[j] : 0.f;
      if (GACT) g *= act_bwd(yr[j], GACT);
      Gs[lane * GPAD + wave * 16 + j] = g;
      if (do_bias) bsum[j] += g;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int e = lane + 64 * j;
        if (e < HPAD) Xs[(wave + 4 * i) * HPAD + e] = (xmask >> (i * NJ + j)) & 1u ? xr[i * NJ + j] : 0.f;
      }
    }
  };

  const int wo = wave & 1, w2 = wave >> 1;       // o half; tap group (3x3) or pixel half
  const int hi = lane >> 5;
  const int tap0 = TAPSPLIT ? w2 * 5 : 0;         // first tap of this wave
  const int ntap = TAPSPLIT ? (w2 == 0 ? 5 : 4) : T;
  f32x16 acc[TPW];
#pragma unroll
  for (int tp = 0; tp < TPW; ++tp)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[tp][r] = 0.f;

  unsigned long long* const stp = a.stamps ? a.stamps + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 : nullptr;
  auto stamp = [&](int k) {   // diagnostics (dro_debug_conv_stamps): 0 set-up, 12 first tile
                                // staged, 1 prologue, 2.. tile iterations (<= 8), 13 loop done, 14 end
    if (stp && threadIdx.x == 0 && k < 15) stp[k] = __builtin_amdgcn_s_memtime();
  };
  const int dbg = ablation_flags(a.dbg);      // 1 skip the loop's loads, 2 its MFMAs, 4 its LDS stores (invalid results)
  stamp(0);
  if (tbeg < tend) {
    load(tbeg);
    store(0);
  }
  stamp(12);
  __syncthreads();
  stamp(1);
  for (int tl = tbeg; tl < tend; ++tl) {
    const int buf = (tl - tbeg) & 1;
    const bool more = tl + 1 < tend;
    if (more && !(dbg & 1)) load(tl + 1);
    const float* Gs = smem + buf * STAGE;
    const float* Xs = Gs + 64 * GPAD;
    const float* ga = Gs + hi * GPAD + wo * 32 + (lane & 31);
    const float* xb = Xs + (lane & 31) * HPAD + hi;
    constexpr int KS = TAPSPLIT ? 32 : 16;        // k-steps (pixel pairs) per wave
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (dbg & 2) break;
      const int pp = 2 * ((TAPSPLIT ? 0 : w2 * 16) + s);   // even pixel of this k-step
      const float av = ga[pp * GPAD];
      const int poff = (pp / TW) * HWd + (pp % TW);
#pragma unroll
      for (int k = 0; k < TPW; ++k) {
        if (k < ntap) {
          const int tap = tap0 + k;
          const int ty = tap / KW, tx = tap - ty * KW;
          acc[k] = mfma32(av, xb[poff + ty * HWd + tx], acc[k]);
        }
      }
    }
    if (more && !(dbg & 4)) store(buf ^ 1);
    __syncthreads();
    if (tl - tbeg < 8) stamp(2 + tl - tbeg);
  }
  stamp(13);
  float* wpart = a.part + (size_t)blockIdx.y * Cout * Cin * T;
  const int c = c0 + (lane & 31);
  if (TAPSPLIT) {
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      if (k < ntap) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int o = o0 + wo * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (o < Cout && c < Cin) wpart[((size_t)o * Cin + c) * T + tap0 + k] = acc[k][r];
        }
      }
    }
  } else {   // sum the pixel halves one tap at a time
    float* red = smem;   // [2 o halves][16][64]
#pragma unroll
    for (int tp = 0; tp < T; ++tp) {
      if (w2 == 1) {
#pragma unroll
        for (int r = 0; r < 16; ++r) red[(wo * 16 + r) * 64 + lane] = acc[tp][r];
      }
      __syncthreads();
      if (w2 == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int o = o0 + wo * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (o < Cout && c < Cin)
            wpart[((size_t)o * Cin + c) * T + tp] = acc[tp][r] + red[(wo * 16 + r) * 64 + lane];
        }
      }
      __syncthreads();
    }
  }
  if (do_bias) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float v = wave_sum(bsum[j]);
      const int o = o0 + wave * 16 + j;
      if (lane == 0 && o < Cout) a.bpart[(size_t)blockIdx.y * Cout + o] = v;
    }
  }
  stamp(14);
}

// ------------------------------------------------------------------ weight gradient v2
// dW[o, c, tap] = sum_p G[o, p] X[c, p + d(tap)]: block = 64 output x 64 input
// channels x all taps, 8 waves (2 per SIMD), K = the pixels of a run of TH x TW
// tiles.  Against wgrad_halo_kernel (64 x 32 channels, 4 waves): G is staged
// once per 64 input channels instead of per 32 (half the G / y re-reads) and
// two waves per SIMD hide the LDS -> MFMA latency the single wave left
// exposed (profiles/r3_conv_roofline.json: 25 % of the f32 MFMA peak, 195 MB
// fetched per 4.5 GFLOP launch).  Wave w: o half w & 1, c half (w >> 1) & 1,
// group w >> 2 = tap group (3x3: taps 0-4 / 5-8) or pixel half (T <= 5:
// summed through LDS at the end).  Same partials as wgrad_halo_kernel
// ([split][Cout][Cin][T], bias [split][Cout]) and the same finish kernel.
template <int KH, int KW, int TG>
struct HaloShapeW2 {
  static constexpr int T = KH * KW;
  // TG == 3 (3x3 only): a block computes one kernel ROW (3 taps) of its
  // (o, c) tile; the pixel halves of the block reduce through LDS as for the
  // 1-D shapes.  TG == 1 for a 3x3: all 9 taps, split 5 | 4 over wave groups.
  static constexpr bool TAPSPLIT = T == 9 && TG == 1;
  static constexpr int TPW = TAPSPLIT ? 5 : (TG == 3 ? 3 : T);
  static constexpr int TH = HaloShape<32, KH, KW>::TH, TW = 64 / TH;
  static constexpr int HWd = TW + KW - 1;
  static constexpr int HALO = (TH + KH - 1) * HWd;
  static constexpr int HPAD = HALO | 1;
  static constexpr int NJ = (HALO + 63) / 64;
  static constexpr int BC = 64, GPAD = 65;
  static constexpr int STAGE = 64 * GPAD + BC * HPAD;
  static constexpr int RED = TAPSPLIT ? 0 : 4 * 16 * 64;        // pixel-half reduction (one tap)
  static constexpr int LDS = 2 * STAGE > RED ? 2 * STAGE : RED;
  static_assert(NJ <= 2 && TW % 2 == 0, "halo shape");
};

template <int KH, int KW, int GACT, bool MULTI, int TG>
__global__ __launch_bounds__(512) void wgrad2_kernel(typename WgParam<MULTI>::T P) {
  static_assert(TG == 1 || (TG == 3 && KH == 3 && KW == 3), "tap groups: 3x3 rows");
  const IgArgs& a = WgParam<MULTI>::ig(P);
  using S = HaloShapeW2<KH, KW, TG>;
  constexpr int T = S::T, TH = S::TH, TW = S::TW, HWd = S::HWd, HALO = S::HALO, HPAD = S::HPAD;
  constexpr int NJ = S::NJ, BC = S::BC, GPAD = S::GPAD, STAGE = S::STAGE, TPW = S::TPW;
  constexpr bool TAPSPLIT = S::TAPSPLIT;
  constexpr int PH = KH / 2, PW = KW / 2;
  __shared__ float smem[S::LDS];
  const int cb1 = a.cbase[1], cb2 = a.cbase[2], cb3 = a.cbase[3];
  const int H = a.g.H, W = a.g.W, Cin = a.g.Cin, Cout = a.g.Cout;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // 0..7
  const int noc = a.otiles * ((Cin + BC - 1) / BC);
  // XCD-aware block order: the blocks of consecutive splits (adjacent pixel
  // runs: their halo rows share cache lines) and the channel tiles of one split
  // (they stage the same G / X tiles) land on the same XCD, i.e. the same L2
  const int nbx = (int)gridDim.x;
  const int lin = xcd_remap((int)(blockIdx.x + blockIdx.y * gridDim.x), (int)(gridDim.x * gridDim.y));
  const int bx = lin % nbx, by = lin / nbx;
  const int tg = TG == 1 ? 0 : bx / noc;    // kernel row of this block (TG == 3)
  const int t = bx - tg * noc;
  const int ot = t % a.otiles, ct = t / a.otiles;
  const int o0 = ot * 64, c0 = ct * BC;
  const size_t HW = (size_t)H * W;
  const unsigned HWu = (unsigned)HW;
  int ntiles = a.g.B * a.tiles_img;
  if constexpr (MULTI) ntiles = P.use_tiles * P.nuse;
  const int tbeg = by * a.chunks_per_split;
  const int tend = min(ntiles, tbeg + a.chunks_per_split);
  const bool do_bias = a.gbias && ct == 0 && tg == 0;
  const float galpha = a.galpha;
  float gr[8], yr[GACT ? 8 : 1], xr[8 * NJ], bsum[8];
  unsigned gmask = 0, xmask = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) bsum[j] = 0.f;
  auto load = [&](int tile) {
    const float* __restrict__ Gp = a.G;
    const float* __restrict__ Yp = a.gy;
    KSlice sbase = kernarg_srcs();
    if constexpr (MULTI) {
      const int u = tile / P.use_tiles;
      tile -= u * P.use_tiles;
      Gp = *(KFPtr)(kernarg_base() + offsetof(WgMulti, uG) + u * sizeof(FPtr));
      if (GACT) Yp = *(KFPtr)(kernarg_base() + offsetof(WgMulti, uy) + u * sizeof(FPtr));
      sbase = (KSlice)(kernarg_base() + offsetof(WgMulti, usrc)) + u * kMaxSrc;
    }
    const int b = tile / a.tiles_img, trem = tile - b * a.tiles_img;
    const int ty0 = (trem / a.tiles_x) * TH, tx0 = (trem % a.tiles_x) * TW;
    // G tile: lane = pixel of the tile, wave w -> output channels o0 + 8w + j
    const int qy = lane / TW, qx = lane - qy * TW;
    const int oy = ty0 + qy, ox = tx0 + qx;
    const bool pin = oy < H && ox < W;
    const unsigned pix = pin ? (unsigned)(oy * W + ox) : 0u;
    gmask = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = o0 + wave * 8 + j;          // scalar
      const bool ok = pin && o < Cout;
      gmask |= ok ? (1u << j) : 0u;
      const unsigned off = ok ? ((unsigned)b * Cout + o) * HWu + pix : 0u;
      gr[j] = Gp[off];
      if (GACT) yr[j] = Yp[off];
    }
    // X patch: wave w -> channels c0 + w + 8i, lanes over the halo
    RowDesc ds[8];
    bool real[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int ch = c0 + wave + 8 * i;         // scalar
      real[i] = ch < Cin;
      ds[i] = row_desc_at(sbase, cb1, cb2, cb3, real[i] ? ch : 0, HWu);
    }
    xmask = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const unsigned xbase = (unsigned)b * ds[i].A + ds[i].Bc;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int e = lane + 64 * j;
        const int hy = e / HWd, hx = e - hy * HWd;
        const int yy = ty0 - PH + hy, xx = tx0 - PW + hx;
        const bool ok = real[i] && e < HALO && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
        xmask |= ok ? (1u << (i * NJ + j)) : 0u;
        xr[i * NJ + j] = ds[i].p[ok ? xbase + (ds[i].M ? (unsigned)(yy * W + xx) : 0u) : 0u];
      }
    }
  };
  auto store = [&](int buf) {
    float* Gs = smem + buf * STAGE;
    float* Xs = Gs + 64 * GPAD;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float g = (gmask >> j) & 1u ? galpha * gr[j] : 0.f;
      if (GACT) g *= act_bwd(yr[j], GACT);
      Gs[lane * GPAD + wave * 8 + j] = g;
      if (do_bias) bsum[j] += g;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int e = lane + 64 * j;
        if (e < HPAD) Xs[(wave + 8 * i) * HPAD + e] = (xmask >> (i * NJ + j)) & 1u ? xr[i * NJ + j] : 0.f;
      }
    }
  };

  const int wo = wave & 1, wc = (wave >> 1) & 1, wg = wave >> 2;
  const int hi = lane >> 5;
  const int tap0 = TAPSPLIT ? wg * 5 : 0;
  const int ntap = TAPSPLIT ? (wg == 0 ? 5 : 4) : T;
  f32x16 acc[TPW];
#pragma unroll
  for (int tp = 0; tp < TPW; ++tp)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[tp][r] = 0.f;

  if (tbeg < tend) {
    load(tbeg);
    store(0);
  }
  __syncthreads();
  for (int tl = tbeg; tl < tend; ++tl) {
    const int buf = (tl - tbeg) & 1;
    const bool more = tl + 1 < tend;
    if (more) load(tl + 1);
    const float* Gs = smem + buf * STAGE;
    const float* Xs = Gs + 64 * GPAD;
    const float* ga = Gs + hi * GPAD + wo * 32 + (lane & 31);
    const float* xb = Xs + (wc * 32 + (lane & 31)) * HPAD + hi + (TG == 3 ? tg * HWd : 0);
    constexpr int KS = TAPSPLIT ? 32 : 16;        // k-steps (pixel pairs) per wave
    const int pbase = TAPSPLIT ? 0 : wg * 16;
    // The tap count of a wave is a compile-time constant in each copy of the
    // loop (3x3: wave group 0 takes taps 0-4, group 1 taps 5-8): a runtime
    // `k < ntap` test put a branch into every k-step, and the compiler then
    // waited for each LDS operand right before its MFMA (round 3 ISA:
    // ds_read / s_waitcnt / v_mfma, serialised).  Without the branches the
    // scheduler batches the reads (ds_read2 pairs of adjacent taps) ahead.
    auto kloop = [&](auto nt_c, int tbase) __attribute__((always_inline)) {
      constexpr int NT = decltype(nt_c)::value;
      int toff[NT];
#pragma unroll
      for (int k = 0; k < NT; ++k) {
        const int tap = tbase + k;
        toff[k] = (tap / KW) * HWd + (tap % KW);
      }
#pragma unroll 8
      for (int s = 0; s < KS; ++s) {
        const int pp = 2 * (pbase + s), poff = (pp / TW) * HWd + (pp % TW);
        const float av = ga[pp * GPAD];
#pragma unroll
        for (int k = 0; k < NT; ++k) acc[k] = mfma32(av, xb[poff + toff[k]], acc[k]);
      }
    };
    if constexpr (TAPSPLIT) {
      if (wg == 0) kloop(std::integral_constant<int, 5>{}, 0);
      else kloop(std::integral_constant<int, 4>{}, 5);
    } else {
      kloop(std::integral_constant<int, TPW>{}, 0);
    }
    if (more) store(buf ^ 1);
    __syncthreads();
  }
  // partials [split][tap][o][c]: lanes run along c, so each store is a
  // 128-B row segment (the [o][c][tap] order of wgrad_halo_kernel scattered
  // them 36 B apart -- 7x write amplification measured at this split count)
  float* wpart = a.part + (size_t)by * Cout * Cin * T;
  const int c = c0 + wc * 32 + (lane & 31);
  const size_t tstride = (size_t)Cout * Cin;
  if (TAPSPLIT) {
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      if (k < ntap) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int o = o0 + wo * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (o < Cout && c < Cin) wpart[(tap0 + k) * tstride + (size_t)o * Cin + c] = acc[k][r];
        }
      }
    }
  } else {   // sum the pixel halves one tap at a time
    float* red = smem;   // [4 (o half, c half)][16][64]
    const int q4 = wo + 2 * wc;
#pragma unroll
    for (int tp = 0; tp < TPW; ++tp) {
      if (wg == 1) {
#pragma unroll
        for (int r = 0; r < 16; ++r) red[(q4 * 16 + r) * 64 + lane] = acc[tp][r];
      }
      __syncthreads();
      if (wg == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int o = o0 + wo * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (o < Cout && c < Cin)
            wpart[(tg * TPW + tp) * tstride + (size_t)o * Cin + c] = acc[tp][r] + red[(q4 * 16 + r) * 64 + lane];
        }
      }
      __syncthreads();
    }
  }
  if (do_bias) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = wave_sum(bsum[j]);
      const int o = o0 + wave * 8 + j;
      if (lane == 0 && o < Cout) a.bpart[(size_t)by * Cout + o] = v;
    }
  }
}


// wgrad2 partials: dW[o][c][tap] = sum_s part[s][tap][o][c]; db[o] = sum_s bpart[s][o].
// Threads walk the partials' coalesced (tap, o, c) order.  The reduction is
// latency-bound (few output elements, up to 256 partials each), so Q lanes
// of a wave share one element: lane group q sums the q-th contiguous range of
// splits (split_sum, 4 chains), and the Q range sums are combined by shuffles
// in a fixed tree -- the same order on every run.
template <int Q>
__global__ __launch_bounds__(256) void wgrad2_finish_kernel(IgArgs a, int splits) {
  constexpr int EPW = 64 / Q;                     // elements per wave
  const int Cout = a.g.Cout, Cin = a.g.Cin, T = a.g.KH * a.g.KW;
  const long long oc = (long long)Cout * Cin, total = oc * T;
  const int lane = threadIdx.x & 63, q = lane / EPW, le = lane - q * EPW;
  const int per = (splits + Q - 1) / Q;
  const int s0 = min(splits, q * per), n = min(splits, s0 + per) - s0;
  const long long wstride = (long long)gridDim.x * (blockDim.x / 64) * EPW;
  for (long long eb = ((long long)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)) * EPW; eb < total;
       eb += wstride) {
    const long long e = eb + le;
    const bool ok = e < total;
    float v = ok ? split_sum(a.part + (size_t)s0 * total + e, (size_t)total, n) : 0.f;
    // every lane shuffles (a shuffle under a lane-dependent branch would read
    // inactive lanes); a + b == b + a exactly, so each pair's sum is one value
    if (Q >= 4) v += __shfl_xor(v, 2 * EPW);      // (q0 + q2), (q1 + q3)
    if (Q >= 2) {
      const float o = __shfl_xor(v, EPW);
      v = q & 1 ? o + v : v + o;
    }
    if (ok && q == 0) {
      const int tap = (int)(e / oc);
      const long long r = e - (long long)tap * oc;        // o * Cin + c
      const size_t dst = (size_t)r * T + tap;
      a.gweight[dst] = a.wacc ? a.gweight[dst] + v : v;
    }
  }
  if (a.gbias) {
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < Cout; e += gridDim.x * blockDim.x) {
      const float bv = split_sum(a.bpart + e, (size_t)Cout, splits);
      a.gbias[e] = a.wacc ? a.gbias[e] + bv : bv;
    }
  }
}

static void launch_wgrad2_finish(const IgArgs& a, int splits, hipStream_t s) {
  const long long total = (long long)a.g.Cout * a.g.Cin * a.g.KH * a.g.KW;
  const int Q = splits >= 32 ? 4 : splits >= 8 ? 2 : 1;
  long long blocks = (total * Q + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (Q == 4) hipLaunchKernelGGL(wgrad2_finish_kernel<4>, dim3((unsigned)blocks), dim3(256), 0, s, a, splits);
  else if (Q == 2) hipLaunchKernelGGL(wgrad2_finish_kernel<2>, dim3((unsigned)blocks), dim3(256), 0, s, a, splits);
  else hipLaunchKernelGGL(wgrad2_finish_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, s, a, splits);
}

// dW[o][c][tap] = sum_s part[s][o][c][tap]; db[o] = sum_s bpart[s][o]
__global__ __launch_bounds__(256) void wgrad_halo_finish_kernel(IgArgs a, int splits) {
  const int Cout = a.g.Cout;
  const long long total = (long long)Cout * a.g.Cin * a.g.KH * a.g.KW;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    float v = 0.f;
    v = split_sum(a.part + e, (size_t)total, splits);
    a.gweight[e] = a.wacc ? a.gweight[e] + v : v;
    if (a.gbias && e < Cout) {
      float bv = 0.f;
      bv = split_sum(a.bpart + e, (size_t)Cout, splits);
      a.gbias[e] = a.wacc ? a.gbias[e] + bv : bv;
    }
  }
}

// dW[o][c][tap] = sum_s part[s][o][tap*Cin + c]; db[o] = sum_s part[s][o][NK].
// Threads walk the partials in their (coalesced) [o][n] order.
// Q lanes share an output element (lane group q sums the q-th contiguous
// range of splits, the Q range sums meet in a fixed shuffle tree, as in
// wgrad2_finish_kernel): with 240 splits one lane per element was a serial
// 240-load chain per element (9 us at the stems' 9.5 K elements)
template <int Q>
__global__ __launch_bounds__(256) void wgrad_finish_kernel(IgArgs a, int splits) {
  constexpr int EPW = 64 / Q;
  const int Cin = a.g.Cin, T = a.g.KH * a.g.KW, NK = a.K, Cout = a.g.Cout;
  const int NC = a.gbias ? NK + 1 : NK;
  const long long total = (long long)Cout * NC;
  const size_t sstride = (size_t)Cout * (NK + 1);
  const int lane = threadIdx.x & 63, q = lane / EPW, le = lane - q * EPW;
  const int per = (splits + Q - 1) / Q;
  const int s0 = min(splits, q * per), ns = min(splits, s0 + per) - s0;
  const long long wstride = (long long)gridDim.x * (blockDim.x / 64) * EPW;
  for (long long eb = ((long long)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)) * EPW; eb < total;
       eb += wstride) {
    const long long e = eb + le;
    const bool ok = e < total;
    const int o = ok ? (int)(e / NC) : 0, n = ok ? (int)(e - (long long)o * NC) : 0;
    const size_t src = (size_t)o * (NK + 1) + n;
    float v = ok ? split_sum(a.part + (size_t)s0 * sstride + src, sstride, ns) : 0.f;
    if (Q >= 4) v += __shfl_xor(v, 2 * EPW);
    if (Q >= 2) {
      const float w = __shfl_xor(v, EPW);
      v = q & 1 ? w + v : v + w;
    }
    if (!ok || q != 0) continue;
    if (n == NK) {
      a.gbias[o] = a.wacc ? a.gbias[o] + v : v;
    } else {
      const int tap = n / Cin, c = n - tap * Cin;
      float* d = a.gweight + ((size_t)o * Cin + c) * T + tap;
      *d = a.wacc ? *d + v : v;
    }
  }
}

static void launch_wgrad_finish(const IgArgs& a, int splits, hipStream_t s) {
  const long long total = (long long)a.g.Cout * (a.K + 1);
  const int Q = splits >= 32 ? 4 : splits >= 8 ? 2 : 1;
  long long blocks = (total * Q + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (Q == 4) hipLaunchKernelGGL(wgrad_finish_kernel<4>, dim3((unsigned)blocks), dim3(256), 0, s, a, splits);
  else if (Q == 2) hipLaunchKernelGGL(wgrad_finish_kernel<2>, dim3((unsigned)blocks), dim3(256), 0, s, a, splits);
  else hipLaunchKernelGGL(wgrad_finish_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, s, a, splits);
}

// ------------------------------------------------------------------ 7x7 weight gradient
// The encoders' 7x7 stems (stride 2, pad 3, 3 or 6 input channels;
// extractor.py:59 via torchvision conv1) and the update blocks' 7x7 state
// convs (stride 1, pad 3, 1 or 6 channels; update.py:77-124).  wgrad_kernel
// gathered every (tap, channel) column from global memory per 64-pixel chunk
// (25-32 TF/s on the stems).  Here a block walks 8x8 output-pixel tiles
// (tile = blockIdx.x + k * gridDim.x, rows o0 = 64 * blockIdx.y), staging per
// tile G[64 o][64 px] and the Cin x PD x PD input patch the tile reads (PD =
// 7 S + 7, zero outside the image) into LDS; the MFMA B operand of column n =
// tap * Cin + c at pixel p is the patch value at (S py + ty, S px + tx) -- one
// shifted LDS read per lane per MFMA pair (both 32-row halves of A share it).
// Wave w owns 32-column subtiles w, w + NW, ... (J of them).  The bias column
// (NK) is the per-block row sum of G.  Partials [split][Cout][NK + 1] for
// wgrad_finish_kernel (fixed order: the same finish as wgrad_kernel's).
template <int S, int CIN, int NW, int J, int GR>
__global__ __launch_bounds__(64 * NW * GR) void wgrad_k7_kernel(IgArgs a) {
  // GR wave groups per block (NW waves each) take alternate tiles of the
  // block's list with their own LDS buffers, and their accumulators are
  // summed (group order) before the one partial: more waves per CU without
  // more partials
  constexpr int PD = 7 * S + 7, PDP = PD | 1, GS = 65, NK = CIN * 49, NSUB = (NK + 31) / 32;
  constexpr int NTH = 64 * NW, PATCH = CIN * PD * PDP, NPE = CIN * PD * PD;
  constexpr int GPER = (4096 + NTH - 1) / NTH, PPER = (NPE + NTH - 1) / NTH;
  static_assert(NW * J >= NSUB && NW * GR <= 16, "subtiles per wave");
  __shared__ float Gs_all[GR][64 * GS];
  __shared__ float Ps_all[GR][PATCH + 1];    // [CIN][PD][PDP], then one zero
  __shared__ float cmb[GR > 1 ? NTH * 16 + 64 : 1];
  const int Cout = a.g.Cout, B = a.g.B, Ho = a.g.H, Wo = a.g.W;
  const int Hi = a.Hs, Wi = a.Ws;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int grp = GR == 1 ? 0 : wave / NW, wv = wave - grp * NW, tid = threadIdx.x - grp * NTH;
  float* Gs = Gs_all[grp];
  float* Ps = Ps_all[grp];
  const int o0 = blockIdx.y * 64;
  const int txs = (Wo + 7) / 8, tis = ((Ho + 7) / 8) * txs, tiles = B * tis;
  const float* __restrict__ Gp = a.G;
  const float* __restrict__ X = a.src[0].p;
  // per lane and subtile: the B operand's patch offset (the zero slot past
  // the patch for padded columns)
  int boff[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int n = (wv + j * NW) * 32 + (lane & 31);
    if (n < NK) {
      const int tap = n / CIN, c = n - tap * CIN, ty = tap / 7, tx = tap - ty * 7;
      boff[j] = (c * PD + ty) * PDP + tx;
    } else {
      boff[j] = -1;
    }
  }
  const int h = lane >> 5;
  f32x16 acc[J][2];
#pragma unroll
  for (int j = 0; j < J; ++j)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][u][r] = 0.f;
  float bsum = 0.f;                      // bias column: thread o < 64 of each group
  if (tid == 0) Ps[PATCH] = 0.f;
  // this thread's staging slots (compile-time counts): the next tile's G and
  // patch are loaded into registers while the current one is multiplied
  float gr[GPER], pr[PPER];
  auto load_tile = [&](int t) {
    const int b = t / tis, r0 = t - b * tis, tyi = r0 / txs, txi = r0 - tyi * txs;
    const int oy0 = tyi * 8, ox0 = txi * 8, iy0 = S * oy0 - 3, ix0 = S * ox0 - 3;
    const float* gb = Gp + ((size_t)b * Cout + o0) * Ho * Wo;
    const float* xb = X + (size_t)b * CIN * Hi * Wi;
#pragma unroll
    for (int i = 0; i < GPER; ++i) {
      const int e = tid + i * NTH;
      const int o = e >> 6, p = e & 63, oy = oy0 + (p >> 3), ox = ox0 + (p & 7);
      const bool ok = (GPER * NTH == 4096 || e < 4096) && o0 + o < Cout && oy < Ho && ox < Wo;
      gr[i] = ok ? gb[((size_t)o * Ho + oy) * Wo + ox] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < PPER; ++i) {
      const int e = tid + i * NTH;
      const int c = e / (PD * PD), rem = e - c * (PD * PD), yy = rem / PD, xx = rem - yy * PD;
      const int iy = iy0 + yy, ix = ix0 + xx;
      const bool ok = e < NPE && (unsigned)iy < (unsigned)Hi && (unsigned)ix < (unsigned)Wi;
      pr[i] = ok ? xb[((size_t)c * Hi + iy) * Wi + ix] : 0.f;
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < GPER; ++i) {
      const int e = tid + i * NTH;
      if (GPER * NTH == 4096 || e < 4096) Gs[(e >> 6) * GS + (e & 63)] = gr[i];
    }
#pragma unroll
    for (int i = 0; i < PPER; ++i) {
      const int e = tid + i * NTH;
      if (e < NPE) {
        const int c = e / (PD * PD), rem = e - c * (PD * PD), yy = rem / PD, xx = rem - yy * PD;
        Ps[(c * PD + yy) * PDP + xx] = pr[i];
      }
    }
  };
  // the block's tiles blockIdx.x + i * gridDim.x; group g takes i = g, g + GR, ...
  const int step = GR * gridDim.x;
  const int nblk = (int)blockIdx.x < tiles ? (tiles - (int)blockIdx.x + gridDim.x - 1) / gridDim.x : 0;
  const int iters = (nblk + GR - 1) / GR;
  const int t0 = blockIdx.x + grp * gridDim.x;
  if (t0 < tiles) {
    load_tile(t0);
    store_tile();
  }
  __syncthreads();
  for (int m = 0, t = t0; m < iters; ++m, t += step) {
    const int tn = t + step;
    const bool has = t < tiles;
    if (tn < tiles) load_tile(tn);
    if (has) {
      if (a.gbias && tid < 64) {
        float sb = 0.f;
        for (int p = 0; p < 64; ++p) sb += Gs[tid * GS + p];
        bsum += sb;
      }
      // LDS operands one step ahead of the MFMAs
      float a0n = Gs[(lane & 31) * GS + h], a1n = Gs[(32 + (lane & 31)) * GS + h];
      float bn[J];
#pragma unroll
      for (int j = 0; j < J; ++j) bn[j] = Ps[boff[j] < 0 ? PATCH : boff[j] + S * h];
#pragma unroll 8
      for (int k = 0; k < 32; ++k) {
        const float a0 = a0n, a1 = a1n;
        float bv[J];
#pragma unroll
        for (int j = 0; j < J; ++j) bv[j] = bn[j];
        if (k + 1 < 32) {
          const int p = 2 * (k + 1) + h, po = S * (p >> 3) * PDP + S * (p & 7);
          a0n = Gs[(lane & 31) * GS + p];
          a1n = Gs[(32 + (lane & 31)) * GS + p];
#pragma unroll
          for (int j = 0; j < J; ++j) bn[j] = Ps[boff[j] < 0 ? PATCH : boff[j] + po];
        }
#pragma unroll
        for (int j = 0; j < J; ++j) {
          acc[j][0] = mfma32(a0, bv[j], acc[j][0]);
          acc[j][1] = mfma32(a1, bv[j], acc[j][1]);
        }
      }
    }
    __syncthreads();                     // every wave is done with this tile
    if (tn < tiles) store_tile();
    __syncthreads();
  }
  if constexpr (GR > 1) {
    // group 1's sums into group 0's (one (j, u) accumulator at a time)
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (grp == 1) {
#pragma unroll
          for (int r = 0; r < 16; ++r) cmb[(wv * 64 + lane) * 16 + r] = acc[j][u][r];
        }
        __syncthreads();
        if (grp == 0) {
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[j][u][r] += cmb[(wv * 64 + lane) * 16 + r];
        }
        __syncthreads();
      }
    if (grp == 1 && tid < 64) cmb[NTH * 16 + tid] = bsum;
    __syncthreads();
    if (grp == 0 && tid < 64) bsum += cmb[NTH * 16 + tid];
    if (grp != 0) return;
  }
  float* part = a.part + (size_t)blockIdx.x * Cout * (NK + 1);
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int n = (wv + j * NW) * 32 + (lane & 31);
    if (n >= NK) continue;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = o0 + u * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (o < Cout) part[(size_t)o * (NK + 1) + n] = acc[j][u][r];
      }
  }
  if (a.gbias && tid < 64 && o0 + tid < Cout) part[(size_t)(o0 + tid) * (NK + 1) + NK] = bsum;
}

// The stems' forward (7x7, stride 2, pad 3, 3 or 6 input channels, no bias
// or activation: BN follows): out[o, p] = sum_k W[o, k] Xpatch[k, p], k = tap
// * Cin + c.  The weights (64 x 49 Cin) are staged in LDS once per block, a
// block walks 8x8 output tiles with the next tile's input patch loaded into
// registers while the current one is multiplied; the four waves take the
// four 32 x 32 quadrants (output-channel half x pixel half) of the tile --
// balanced over the SIMDs -- and the B operand is the patch value at
// (2 py + ty, 2 px + tx): one shifted LDS read per MFMA.  igemm_kernel
// gathered every (tap, channel) row from global memory (30 TF/s).
template <int CIN>
__global__ __launch_bounds__(256) void fwd_k7s2_kernel(IgArgs a) {
  constexpr int S = 2, PD = 7 * S + 7, PDP = PD | 1, NK = CIN * 49, KP = NK + 1;   // odd row stride
  constexpr int KSTEPS = (NK + 1) / 2, NPE = CIN * PD * PD, PPER = (NPE + 255) / 256;
  __shared__ float Ws[64 * KP];
  __shared__ float Ps[CIN * PD * PDP + 1];
  __shared__ int koff[2 * KSTEPS];      // patch offset of column k (the zero slot past NK)
  const int Cout = a.g.Cout, B = a.g.B, Ho = a.g.H, Wo = a.g.W, Hi = a.Hs, Wi = a.Ws;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int oh = wave & 1, ph = wave >> 1, h = lane >> 5;
  const int o0 = blockIdx.y * 64;
  const int txs = (Wo + 7) / 8, tis = ((Ho + 7) / 8) * txs, tiles = B * tis;
  const float* __restrict__ X = a.src[0].p;
  for (int e = tid; e < 64 * NK; e += 256) {
    const int o = e / NK, k = e - o * NK;
    // torch weight layout [o][c][ty][tx]; column k = tap * Cin + c
    const int tap = k / CIN, c = k - tap * CIN;
    Ws[o * KP + k] = o0 + o < Cout ? a.weight[((size_t)(o0 + o) * CIN + c) * 49 + tap] : 0.f;
  }
  if (tid < 64) Ws[tid * KP + NK] = 0.f;
  for (int k = tid; k < 2 * KSTEPS; k += 256) {
    const int tap = k / CIN, c = k - tap * CIN, ty = tap / 7, tx = tap - ty * 7;
    koff[k] = k < NK ? (c * PD + ty) * PDP + tx : CIN * PD * PDP;
  }
  if (tid == 0) Ps[CIN * PD * PDP] = 0.f;
  const int pl = ph * 32 + (lane & 31), py = pl >> 3, px = pl & 7;
  const int poff = S * py * PDP + S * px;
  float pr[PPER];
  auto load_tile = [&](int t) {
    const int b = t / tis, r0 = t - b * tis, tyi = r0 / txs, txi = r0 - tyi * txs;
    const int iy0 = S * tyi * 8 - 3, ix0 = S * txi * 8 - 3;
    const float* xb = X + (size_t)b * CIN * Hi * Wi;
#pragma unroll
    for (int i = 0; i < PPER; ++i) {
      const int e = tid + i * 256;
      const int c = e / (PD * PD), rem = e - c * (PD * PD), yy = rem / PD, xx = rem - yy * PD;
      const int iy = iy0 + yy, ix = ix0 + xx;
      const bool ok = e < NPE && (unsigned)iy < (unsigned)Hi && (unsigned)ix < (unsigned)Wi;
      pr[i] = ok ? xb[((size_t)c * Hi + iy) * Wi + ix] : 0.f;
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < PPER; ++i) {
      const int e = tid + i * 256;
      if (e < NPE) {
        const int c = e / (PD * PD), rem = e - c * (PD * PD), yy = rem / PD, xx = rem - yy * PD;
        Ps[(c * PD + yy) * PDP + xx] = pr[i];
      }
    }
  };
  if ((int)blockIdx.x < tiles) {
    load_tile(blockIdx.x);
    store_tile();
  }
  __syncthreads();
  const float* wrow = Ws + (oh * 32 + (lane & 31)) * KP + h;
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int tn = t + gridDim.x;
    if (tn < tiles) load_tile(tn);
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    float an = wrow[0], bn = Ps[koff[h] + poff];
#pragma unroll 8
    for (int s2 = 0; s2 < KSTEPS; ++s2) {
      const float av = an, bv = bn;
      if (s2 + 1 < KSTEPS) {
        an = wrow[2 * (s2 + 1)];
        bn = Ps[koff[2 * (s2 + 1) + h] + poff];
      }
      acc = mfma32(av, bv, acc);
    }
    const int b = t / tis, r0 = t - b * tis, tyi = r0 / txs, txi = r0 - tyi * txs;
    const int oy = tyi * 8 + py, ox = txi * 8 + px;
    if (oy < Ho && ox < Wo) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = o0 + oh * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (o < Cout) a.out[(((size_t)b * a.out_ctot + a.out_coff + o) * Ho + oy) * Wo + ox] = acc[r];
      }
    }
    __syncthreads();                     // every wave is done with this patch
    if (tn < tiles) store_tile();
    __syncthreads();
  }
}

// G = alpha * dout * act'(y) (only when act != none or alpha != 1)
// grid (pixel blocks, B * Cout planes): no 64-bit division per element
__global__ __launch_bounds__(256) void grad_pre_kernel(int act, float alpha, int Cout, int HW,
                                                       const float* __restrict__ dout,
                                                       Slice y, float* __restrict__ G) {
  const int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= HW) return;
  const int plane = blockIdx.y;                 // b * Cout + o (wave-uniform)
  const size_t i = (size_t)plane * HW + pix;
  float d = alpha * dout[i];
  if (act) {
    const int b = plane / Cout, o = plane - b * Cout;
    d *= act_bwd(y.p[((size_t)b * y.ctot + y.coff + o) * HW + pix], act);
  }
  G[i] = d;
}

}  // namespace dro

using namespace dro;

namespace {

FastDiv make_fdiv(int d) {
  FastDiv f;
  f.one = d == 1;
  f.m = d == 1 ? 0u : (unsigned)(((1ULL << 32) + (unsigned long long)d - 1) / (unsigned long long)d);
  return f;
}

// ---- launch plans (shared by the workspace query and the launches)
struct IgPlan {
  bool halo;
  int bm, row_tiles, ptiles, ksplit, chunks_per_split;
  int kin;                // intra-block K split (wave groups per tile; halo kernels)
  int TH, TW, HWd, HPAD, tiles_x, tiles_img, CK;
  size_t lds_bytes;
  size_t part_bytes;
};


IgPlan plan_igemm_flat(int rows, int kch, int KH, int KW, int B, int H, int W);

template <int BM, int KH, int KW>
void halo_fill(IgPlan& pl) {
  using S = HaloShape<BM, KH, KW>;
  pl.TH = S::TH;
  pl.TW = S::TW;
  pl.HWd = S::HWd;
  pl.HPAD = S::HPAD;
  pl.CK = S::CK;
  pl.lds_bytes = S::LDS * sizeof(float);
}

IgPlan plan_igemm(int rows, int kch, int KH, int KW, int B, int H, int W) {
  const bool shape_ok = (KH == 1 && KW == 5) || (KH == 5 && KW == 1) || (KH == 3 && KW == 3) ||
                        (KH == 1 && KW == 1);
  // the halo kernel stages weights as float4 runs: tensors of < 4 weights go flat
  if (!shape_ok || (long long)rows * kch * KH * KW < 4) return plan_igemm_flat(rows, kch, KH, KW, B, H, W);
  IgPlan pl = {};
  const long long P = (long long)B * H * W;
  pl.halo = true;
  const int TH = (KW == 1 || (KH == 3 && KW == 3)) ? 8 : 4, TW = 64 / TH;
  pl.tiles_x = (W + TW - 1) / TW;
  pl.tiles_img = ((H + TH - 1) / TH) * pl.tiles_x;
  pl.ptiles = B * pl.tiles_img;
  const int t64 = (rows + 63) / 64;
  pl.bm = (long long)t64 * pl.ptiles >= 480 ? 64 : 32;
  pl.row_tiles = (rows + pl.bm - 1) / pl.bm;
  if (pl.bm == 32) {
    if (KH == 1 && KW == 1) halo_fill<32, 1, 1>(pl);
    else if (KH == 1) halo_fill<32, 1, 5>(pl);
    else if (KW == 1) halo_fill<32, 5, 1>(pl);
    else halo_fill<32, 3, 3>(pl);
  } else {
    if (KH == 1 && KW == 1) halo_fill<64, 1, 1>(pl);
    else if (KH == 1) halo_fill<64, 1, 5>(pl);
    else if (KW == 1) halo_fill<64, 5, 1>(pl);
    else halo_fill<64, 3, 3>(pl);
  }
  const int nchunks = (kch + pl.CK - 1) / pl.CK;
  const long long blocks = (long long)pl.row_tiles * pl.ptiles;
  // K split inside the block first (4 or 2 wave groups per tile: no partials,
  // no finish launch), over blocks only when the grid is still very short
  static const long long t2 = [] {   // tuning: grids below this many tiles use 2 wave groups
    const char* e = getenv("DRO_CONV_KIN2_BELOW");
    return e ? atoll(e) : 512LL;
  }();
  int kin = blocks < 256 ? 4 : (blocks < t2 ? 2 : 1);
  static const int kin_env = [] {   // tuning override: DRO_CONV_KIN=1|2|4
    const char* e = getenv("DRO_CONV_KIN");
    const int v = e ? atoi(e) : 0;
    return (v == 1 || v == 2 || v == 4) ? v : 0;
  }();
  if (kin_env) kin = kin_env;
  while (kin > 1 && kin > nchunks) kin >>= 1;
  pl.kin = kin;
  int ks = 1;
  if (blocks < 120) {
    ks = (int)((480 + blocks * kin - 1) / (blocks * kin));
    if (ks > 16) ks = 16;
    if (ks > nchunks / kin) ks = nchunks / kin;
    if (ks < 1) ks = 1;
  }
  pl.chunks_per_split = (nchunks + ks - 1) / ks;
  pl.ksplit = (nchunks + pl.chunks_per_split - 1) / pl.chunks_per_split;
  pl.part_bytes = pl.ksplit > 1 ? align256((size_t)pl.ksplit * rows * P * sizeof(float)) : 0;
  return pl;
}

// the flattened-pixel implicit GEMM (1x1 and large kernels)
IgPlan plan_igemm_flat(int rows, int kch, int KH, int KW, int B, int H, int W) {
  IgPlan pl = {};
  const int T = KH * KW;
  const long long P = (long long)B * H * W;
  pl.halo = false;
  pl.kin = 1;
  pl.ptiles = (int)((P + kBN - 1) / kBN);
  const int t64 = (rows + 63) / 64;
  pl.bm = (long long)t64 * pl.ptiles >= 448 ? 64 : 32;
  pl.row_tiles = (rows + pl.bm - 1) / pl.bm;
  const int nchunks = (kch * T + kBK - 1) / kBK;
  const long long blocks = (long long)pl.row_tiles * pl.ptiles;
  static const long long below = env_int("DRO_FLAT_BELOW", 960), target = env_int("DRO_FLAT_TARGET", 480);
  int ks = 1;
  if (blocks < below) {
    ks = (int)((target + blocks - 1) / blocks);
    if (ks > 16) ks = 16;
    if (ks > nchunks / 4) ks = nchunks / 4;
    if (ks < 1) ks = 1;
  }
  pl.chunks_per_split = (nchunks + ks - 1) / ks;
  pl.ksplit = (nchunks + pl.chunks_per_split - 1) / pl.chunks_per_split;
  pl.part_bytes = pl.ksplit > 1 ? align256((size_t)pl.ksplit * rows * P * sizeof(float)) : 0;
  return pl;
}

struct WgPlan {
  int otiles, ntiles, splits;
  long long pchunk;
  size_t part_bytes;
};

WgPlan plan_wgrad(int Cin, int Cout, int T, long long P) {
  WgPlan pl;
  const int NK = Cin * T;
  pl.otiles = (Cout + 63) / 64;
  pl.ntiles = (NK + 1 + 63) / 64;
  const long long tiles = (long long)pl.otiles * pl.ntiles;
  // ~4 blocks per CU: the stems (3 or 6 input channels, 7x7: 3-5 column tiles
  // over 10^5 pixels) got 192 blocks at the old 64-split cap and ran at 18 TF/s
  static const long long target = env_int("DRO_WG_TARGET", 1024), cap = env_int("DRO_WG_MAXSPLIT", 256);
  long long splits = (target + tiles - 1) / tiles;
  static const long long minch = env_int("DRO_WG_MINCHUNKS", 1);   // pixel chunks per split, at least
  const long long maxs = (P + minch * kWP - 1) / (minch * kWP);
  if (splits > maxs) splits = maxs;
  if (splits > cap) splits = cap;
  if (splits < 1) splits = 1;
  pl.pchunk = ((P + splits - 1) / splits + kWP - 1) / kWP * kWP;
  pl.splits = (int)((P + pl.pchunk - 1) / pl.pchunk);
  pl.part_bytes = align256((size_t)pl.splits * Cout * (NK + 1) * sizeof(float));
  return pl;
}

// halo weight gradient: (KH, KW) in {1x5, 5x1, 3x3}
struct WhPlan {
  bool ok;
  int otiles, ctiles, tiles_x, tiles_img, splits, tiles_per_split;
  size_t part_bytes;
  int tgroups;   // wgrad2, 3x3: blocks per (o, c) tile along the kernel rows (1 or 3)
};

WhPlan plan_wgrad_halo(int Cin, int Cout, int KH, int KW, int B, int H, int W) {
  WhPlan pl = {};
  pl.ok = (KH == 1 && KW == 5) || (KH == 5 && KW == 1) || (KH == 3 && KW == 3) || (KH == 1 && KW == 1);
  if (!pl.ok) return pl;
  const int TH = (KW == 1 || (KH == 3 && KW == 3)) ? 8 : 4, TW = 64 / TH;
  pl.tiles_x = (W + TW - 1) / TW;
  pl.tiles_img = ((H + TH - 1) / TH) * pl.tiles_x;
  const int ntiles = B * pl.tiles_img;
  pl.otiles = (Cout + 63) / 64;
  pl.ctiles = (Cin + 31) / 32;
  const int blocks = pl.otiles * pl.ctiles;
  // ~1.5 blocks per CU (parallelism beats the partials' extra traffic here)
  static const int max_sp = [] {   // tuning override: DRO_WH_MAX_SPLITS (default 32)
    const char* e = getenv("DRO_WH_MAX_SPLITS");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 32;
  }();
  static const int target = [] {   // tuning override: DRO_WH_TARGET_BLOCKS (default 384)
    const char* e = getenv("DRO_WH_TARGET_BLOCKS");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 384;
  }();
  int sp = (target + blocks - 1) / blocks;
  if (sp > max_sp) sp = max_sp;
  if (sp > ntiles) sp = ntiles;
  if (sp < 1) sp = 1;
  pl.tiles_per_split = (ntiles + sp - 1) / sp;
  pl.splits = (ntiles + pl.tiles_per_split - 1) / pl.tiles_per_split;
  pl.part_bytes = align256((size_t)pl.splits * Cout * Cin * KH * KW * sizeof(float)) +
                  align256((size_t)pl.splits * Cout * sizeof(float));
  return pl;
}

// weight gradient v2 (wgrad2_kernel): 64 x 64 channel tiles, one block of 8
// waves per CU (85 KB LDS); splits fill ~`target` blocks with >= `min_tiles`
// pixel tiles per split (each split writes a full Cout x Cin x T partial).  DRO_WGRAD_V1=1 keeps the wgrad_halo_kernel path (A/B).
bool wgrad_v1() {
  static const bool v1 = getenv("DRO_WGRAD_V1") != nullptr;
  return v1;
}

WhPlan plan_wgrad2(int Cin, int Cout, int KH, int KW, int ntiles_total, int B, int H, int W) {
  WhPlan pl = {};
  pl.ok = (KH == 1 && KW == 5) || (KH == 5 && KW == 1) || (KH == 3 && KW == 3) || (KH == 1 && KW == 1);
  if (!pl.ok) return pl;
  const int TH = (KW == 1 || (KH == 3 && KW == 3)) ? 8 : 4, TW = 64 / TH;
  pl.tiles_x = (W + TW - 1) / TW;
  pl.tiles_img = ((H + TH - 1) / TH) * pl.tiles_x;
  const int ntiles = ntiles_total > 0 ? ntiles_total : B * pl.tiles_img;
  pl.otiles = (Cout + 63) / 64;
  pl.ctiles = (Cin + 63) / 64;
  // 3x3: one block per kernel row of a tile -- 3x the blocks at the same
  // split count, so a third of the split partials for the same occupancy
  // measured (fnet layer1 wgrad, B=6 48x160 64->64): 3 row groups 72 + 5 us
  // vs all 9 taps per block 51 + 8 us -- staging per MFMA triples; default 1
  static const int tg3 = [] {   // tuning override: DRO_WG2_TGROUPS=3 (default 1)
    const char* e = getenv("DRO_WG2_TGROUPS");
    return e && atoi(e) == 3 ? 3 : 1;
  }();
  pl.tgroups = (KH == 3 && KW == 3) ? tg3 : 1;
  const int blocks = pl.otiles * pl.ctiles * pl.tgroups;
  static const int target = [] {   // tuning override: DRO_WG2_TARGET_BLOCKS (default 256)
    const char* e = getenv("DRO_WG2_TARGET_BLOCKS");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 256;
  }();
  static const int min_tiles = [] {   // tuning override: DRO_WG2_MIN_TILES (default 1, measured best)
    const char* e = getenv("DRO_WG2_MIN_TILES");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 1;
  }();
  int sp = (target + blocks - 1) / blocks;
  if (sp > 256) sp = 256;
  if (sp > ntiles / min_tiles) sp = ntiles / min_tiles;
  if (sp < 1) sp = 1;
  pl.tiles_per_split = (ntiles + sp - 1) / sp;
  pl.splits = (ntiles + pl.tiles_per_split - 1) / pl.tiles_per_split;
  pl.part_bytes = align256((size_t)pl.splits * Cout * Cin * KH * KW * sizeof(float)) +
                  align256((size_t)pl.splits * Cout * sizeof(float));
  return pl;
}

size_t fwd_workspace(int B, int H, int W, int Cin, int Cout, int KH, int KW) {
  return std::max(plan_igemm(Cout, Cin, KH, KW, B, H, W).part_bytes,
                  xconv_part_bytes(Cout, Cin, KH, KW, B, H, W));
}

size_t bwd_workspace(int B, int H, int W, int Cin, int Cout, int KH, int KW) {
  const long long P = (long long)B * H * W;
  const int T = KH * KW;
  return align256((size_t)Cout * P * sizeof(float)) +              // pre-activation gradient
         std::max(plan_igemm(Cin, Cout, KH, KW, B, H, W).part_bytes,  // data-gradient split-K
                  xconv_part_bytes(Cin, Cout, KH, KW, B, H, W)) +
         std::max(std::max(plan_wgrad(Cin, Cout, T, P).part_bytes,  // weight-gradient partials
                           plan_wgrad_halo(Cin, Cout, KH, KW, B, H, W).part_bytes),
                  plan_wgrad2(Cin, Cout, KH, KW, 0, B, H, W).part_bytes);
}

bool too_big(long long B, long long C, long long HW) { return B * C * HW >= (1LL << 30); }

int conv_setup_geom(IgArgs& a, const dro_slice* srcs, int nsrc, int B, int H, int W, int Cout, int KH,
                    int KW) {
  ConvGeom& g = a.g;
  if (!srcs || nsrc < 1 || nsrc > kMaxSrc) {
    set_error("conv2d: need 1..4 input slices");
    return DRO_E_SHAPE;
  }
  if (B < 1 || H < 1 || W < 1 || Cout < 1 || KH < 1 || KW < 1 || (KH % 2) == 0 || (KW % 2) == 0) {
    set_error("conv2d: sizes out of range (odd kernels, 'same' padding, stride 1)");
    return DRO_E_SHAPE;
  }
  int cin = 0;
  for (int i = 0; i < nsrc; ++i) {
    if (!srcs[i].data) {
      set_error("conv2d: NULL input slice");
      return DRO_E_NULL;
    }
    if (srcs[i].channels < 1 || srcs[i].channel_offset < 0 ||
        srcs[i].channel_offset + srcs[i].channels > srcs[i].total_channels) {
      set_error("conv2d: bad input slice");
      return DRO_E_SHAPE;
    }
    if (too_big(B, srcs[i].total_channels, srcs[i].broadcast ? 1LL : (long long)H * W)) {
      set_error("conv2d: a source tensor has >= 2^30 elements (32-bit offsets)");
      return DRO_E_SHAPE;
    }
    cin += srcs[i].channels;
  }
  if (cin >= 4096 || Cout >= 4096 || (long long)cin * KH * KW >= 65535 ||
      (long long)Cout * KH * KW >= 65535 || too_big(B, cin > Cout ? cin : Cout, (long long)H * W)) {
    set_error("conv2d: sizes out of range (C < 4096, C*KH*KW < 65535, B*C*H*W < 2^30)");
    return DRO_E_SHAPE;
  }
  g.B = B;
  g.H = H;
  g.W = W;
  g.Cin = cin;
  g.Cout = Cout;
  g.KH = KH;
  g.KW = KW;
  g.PH = KH / 2;
  g.PW = KW / 2;
  int base = 0;
  for (int i = 0; i < kMaxSrc; ++i) {
    if (i < nsrc) {
      a.src[i].p = srcs[i].data;
      a.src[i].C = srcs[i].channels;
      a.src[i].ctot = srcs[i].total_channels;
      a.src[i].coff = srcs[i].channel_offset;
      a.src[i].bcast = srcs[i].broadcast;
      a.cbase[i] = base;
      base += srcs[i].channels;
    } else {
      a.src[i] = a.src[0];
      a.cbase[i] = cin;
    }
  }
  a.kwdiv = make_fdiv(KW);
  a.cindiv = make_fdiv(cin);
  a.Hs = H;
  a.Ws = W;
  a.sshift = 0;
  return DRO_OK;
}

Slice to_slice(const dro_slice* s) {
  Slice r;
  r.p = s ? s->data : nullptr;
  r.C = s ? s->channels : 0;
  r.ctot = s ? s->total_channels : 0;
  r.coff = s ? s->channel_offset : 0;
  r.bcast = s ? s->broadcast : 0;
  return r;
}

// ---------------------------------------------------------------- thin 7x7
// The 7x7 state convolutions of the projection encoders (update.py:77-124:
// convd1 1 -> hidden, convp1 6 -> hidden, the latter over a broadcast pose
// map) have <= 8 input channels: as an MFMA GEMM 26-97 % of every tile is
// padding, so they run on plain FMAs over an 8x8 pixel tile staged with its
// halo in LDS.  Forward: a block is 64 pixels x 16 output channels (thread =
// 1 pixel x 4 channels, float4 weight reads).  Data gradient: a block is 64
// pixels x all input channels, the output channels split over 4 thread
// groups and summed through LDS in a fixed order (deterministic).
constexpr int kThinK = 7, kThinT = 49, kThinHalo = 14 * 14;

template <int ACT>
__global__ __launch_bounds__(256) void thin_fwd_kernel(IgArgs a, int tiles_x) {
  __shared__ float Xs[8 * kThinHalo];
  __shared__ float4 Wv[8 * kThinT * 4];          // [ci][tap][co/4], 16 co per block
  const int H = a.g.H, W = a.g.W, Cin = a.g.Cin, Cout = a.g.Cout;
  const size_t HW = (size_t)H * W;
  const int b = blockIdx.z, co0 = blockIdx.y * 16;
  const int ty0 = (blockIdx.x / tiles_x) * 8, tx0 = (blockIdx.x % tiles_x) * 8;
  const Slice sl = a.src[0];
  for (int e = threadIdx.x; e < Cin * kThinHalo; e += 256) {
    const int ci = e / kThinHalo, r = e - ci * kThinHalo, hy = r / 14, hx = r - hy * 14;
    const int yy = ty0 - 3 + hy, xx = tx0 - 3 + hx;
    float v = 0.f;
    if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) {
      const size_t ch = (size_t)b * sl.ctot + sl.coff + ci;
      v = sl.bcast ? sl.p[ch] : sl.p[ch * HW + (size_t)yy * W + xx];
    }
    Xs[e] = v;
  }
  float* Wf = reinterpret_cast<float*>(Wv);
  for (int e = threadIdx.x; e < Cin * kThinT * 16; e += 256) {
    const int col = e & 15, q = e >> 4, tap = q % kThinT, ci = q / kThinT;
    const int co = co0 + col;
    Wf[e] = co < Cout ? a.weight[((size_t)co * Cin + ci) * kThinT + tap] : 0.f;
  }
  __syncthreads();
  const int px = threadIdx.x & 63, cg = threadIdx.x >> 6;   // 4 channels per thread
  const int py = px >> 3, pxx = px & 7;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int ci = 0; ci < Cin; ++ci) {
    const float* xb = Xs + ci * kThinHalo + py * 14 + pxx;
    const float4* wb = Wv + ci * kThinT * 4 + cg;
#pragma unroll
    for (int ky = 0; ky < kThinK; ++ky)
#pragma unroll
      for (int kx = 0; kx < kThinK; ++kx) {
        const float v = xb[ky * 14 + kx];
        const float4 w = wb[(ky * kThinK + kx) * 4];
        acc.x = fmaf(v, w.x, acc.x);
        acc.y = fmaf(v, w.y, acc.y);
        acc.z = fmaf(v, w.z, acc.z);
        acc.w = fmaf(v, w.w, acc.w);
      }
  }
  const int oy = ty0 + py, ox = tx0 + pxx;
  if (oy >= H || ox >= W) return;
  const float r[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int co = co0 + cg * 4 + j;
    if (co >= Cout) continue;
    const float v = a.alpha * act_fwd(r[j] + (a.bias ? a.bias[co] : 0.f), ACT);
    a.out[((size_t)b * a.out_ctot + a.out_coff + co) * HW + (size_t)oy * W + ox] = v;
  }
}

// data gradient w.r.t. a single source of <= 8 channels; G folded as in dconv.
// blockIdx.y takes a span of output channels (partials [split][Cin][P] summed by
// igemm_finish_kernel in a fixed order when there is more than one span)
template <int ACT, int CINP>
__global__ __launch_bounds__(256) void thin_dgrad_kernel(IgArgs a, int tiles_x, int cps) {
  constexpr int CC = 16;                          // output channels staged per pass
  __shared__ float Gs[CC * kThinHalo];
  __shared__ float Ws[CC * kThinT * CINP];        // [co][tap][ci]
  __shared__ float red[4 * 64 * CINP];
  const int H = a.g.H, W = a.g.W, Cin = a.rows, Cout = a.g.Cout;
  const size_t HW = (size_t)H * W;
  const int b = blockIdx.z;
  const int ty0 = (blockIdx.x / tiles_x) * 8, tx0 = (blockIdx.x % tiles_x) * 8;
  const int px = threadIdx.x & 63, cg = threadIdx.x >> 6;   // group cg takes 4 co per pass
  const int py = px >> 3, pxx = px & 7;
  const int co_lo = blockIdx.y * cps, co_hi = min(Cout, co_lo + cps);
  float acc[CINP];
#pragma unroll
  for (int i = 0; i < CINP; ++i) acc[i] = 0.f;
  for (int c0 = co_lo; c0 < co_hi; c0 += CC) {
    __syncthreads();
    for (int e = threadIdx.x; e < CC * kThinHalo; e += 256) {
      const int cl = e / kThinHalo, r = e - cl * kThinHalo, hy = r / 14, hx = r - hy * 14;
      const int yy = ty0 - 3 + hy, xx = tx0 - 3 + hx, co = c0 + cl;
      float v = 0.f;
      if (co < co_hi && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) {
        const size_t o = ((size_t)b * Cout + co) * HW + (size_t)yy * W + xx;
        v = a.galpha * a.G[o];
        if (ACT != 0) v *= act_bwd(a.gy[o], ACT);
      }
      Gs[e] = v;
    }
    for (int e = threadIdx.x; e < CC * kThinT * CINP; e += 256) {
      const int ci = e % CINP, q = e / CINP, tap = q % kThinT, cl = q / kThinT, co = c0 + cl;
      Ws[e] = (co < co_hi && ci < Cin) ? a.weight[((size_t)co * Cin + ci) * kThinT + tap] : 0.f;
    }
    __syncthreads();
#pragma unroll 1
    for (int j = 0; j < CC / 4; ++j) {
      const int cl = cg * (CC / 4) + j;
      const float* gb = Gs + cl * kThinHalo + py * 14 + pxx;
      const float* wb = Ws + cl * kThinT * CINP;
#pragma unroll
      for (int ky = 0; ky < kThinK; ++ky)
#pragma unroll
        for (int kx = 0; kx < kThinK; ++kx) {
          // input pixel (y, x) receives G at (y - ky + 3, x - kx + 3)
          const float g = gb[(6 - ky) * 14 + (6 - kx)];
          const int tap = ky * kThinK + kx;
          if (CINP == 8) {
            const float4 w0 = reinterpret_cast<const float4*>(wb)[tap * 2];
            const float4 w1 = reinterpret_cast<const float4*>(wb)[tap * 2 + 1];
            acc[0] = fmaf(g, w0.x, acc[0]);
            acc[1 % CINP] = fmaf(g, w0.y, acc[1 % CINP]);
            acc[2 % CINP] = fmaf(g, w0.z, acc[2 % CINP]);
            acc[3 % CINP] = fmaf(g, w0.w, acc[3 % CINP]);
            acc[4 % CINP] = fmaf(g, w1.x, acc[4 % CINP]);
            acc[5 % CINP] = fmaf(g, w1.y, acc[5 % CINP]);
            acc[6 % CINP] = fmaf(g, w1.z, acc[6 % CINP]);
            acc[7 % CINP] = fmaf(g, w1.w, acc[7 % CINP]);
          } else {
#pragma unroll
            for (int ci = 0; ci < CINP; ++ci) acc[ci] = fmaf(g, wb[tap * CINP + ci], acc[ci]);
          }
        }
    }
  }
#pragma unroll
  for (int i = 0; i < CINP; ++i) red[(cg * 64 + px) * CINP + i] = acc[i];
  __syncthreads();
  const long long P = (long long)a.g.B * HW;
  for (int e = threadIdx.x; e < 64 * CINP; e += 256) {
    const int p = e / CINP, ci = e % CINP;
    if (ci >= Cin) continue;
    const float v = (red[(0 * 64 + p) * CINP + ci] + red[(1 * 64 + p) * CINP + ci]) +
                    (red[(2 * 64 + p) * CINP + ci] + red[(3 * 64 + p) * CINP + ci]);
    const int oy = ty0 + (p / 8), ox = tx0 + (p % 8);
    if (oy >= H || ox >= W) continue;
    const size_t epix = (size_t)oy * W + ox;
    if (a.part)
      a.part[(size_t)blockIdx.y * Cin * P + (size_t)ci * P + (size_t)b * HW + epix] = v;
    else
      grad_put(a.gsrc[0], a.gsrc_ctot[0], a.gsrc_coff[0], a.gsrc_acc[0], ci, b, epix, HW, v);
  }
}

// thin path eligibility: 7x7, a single source of <= 8 channels, plain epilogue
// ---- launch log (dro_conv_log_*): algorithmic FLOPs per kernel instantiation,
// for the per-kernel roofline table (tools/conv_roofline.py).  Host side only.
bool g_conv_log = false;
std::mutex g_conv_log_mu;
std::map<std::string, std::pair<long long, double>> g_conv_log_map;

void conv_log(const char* name, double flops) {
  if (!g_conv_log) return;
  std::lock_guard<std::mutex> lk(g_conv_log_mu);
  auto& e = g_conv_log_map[name];
  e.first += 1;
  e.second += flops;
}

template <typename... Ts>
void conv_logf(double flops, const char* fmt, Ts... args) {
  if (!g_conv_log) return;
  char buf[160];
  snprintf(buf, sizeof(buf), fmt, args...);
  conv_log(buf, flops);
}

// the 7x7 path applies (weights of < 4096 floats per row, 64-row tiles)
bool k7_ok(int KH, int KW, int Cin, int pad, int stride) {
  static const bool off = getenv("DRO_K7_WGRAD_OFF") != nullptr;   // A/B: wgrad_kernel for them
  return !off && KH == 7 && KW == 7 && pad == 3 &&
         ((stride == 2 && (Cin == 3 || Cin == 6)) || (stride == 1 && (Cin == 1 || Cin == 6)));
}

// launches wgrad_k7_kernel + the finish with `splits` <= the caller's
// wgrad_kernel plan (same partial workspace)
// blocks (= partials) of the 7x7 weight gradient: >= 4 tiles per block, at
// most 256 (measured at the stems, tools/bench_k7.py: 256 blocks of 11 tiles
// 88 us for fnet's; 720 of 4 108 us -- the partials' traffic grows faster
// than the SIMD balance improves)
int k7_splits(int B, int Ho, int Wo) {
  static const int per = (int)env_int("DRO_K7_TILES_PER_BLOCK", 4);
  static const int cap = (int)env_int("DRO_K7_MAX_BLOCKS", 256);
  const int tiles = B * ((Ho + 7) / 8) * ((Wo + 7) / 8);
  int sp = (tiles + per - 1) / per;
  if (sp > cap) sp = cap;
  return sp < 1 ? 1 : sp;
}

size_t k7_part_bytes(int B, int Ho, int Wo, int Cin, int Cout) {
  return align256((size_t)k7_splits(B, Ho, Wo) * Cout * (Cin * 49 + 1) * sizeof(float));
}

int launch_wgrad_k7(IgArgs& a, int stride, int splits, hipStream_t s) {
  const int Cin = a.g.Cin, NK = Cin * 49;
  const int tiles = a.g.B * ((a.g.H + 7) / 8) * ((a.g.W + 7) / 8);
  if (splits > tiles) splits = tiles;
  if (splits < 1) splits = 1;
  const dim3 grid((unsigned)splits, (unsigned)((a.g.Cout + 63) / 64));
  conv_logf(2.0 * a.g.Cout * NK * (double)a.g.B * a.g.H * a.g.W, "wgrad_k7_kernel<%d, %d>", stride, Cin);
  // (S, CIN, waves, subtiles per wave, wave groups): 32-column subtiles of the
  // 49 Cin columns; two wave groups per block for the 3-channel stems (fnet
  // 93 -> 78 us, cnet_depth 41 -> 37 us; the 6-channel variant spills and is
  // no faster), DRO_K7_GROUPS=1|2 forces one (A/B)
  static const int forced = env_int("DRO_K7_GROUPS", 0);
  const int groups = forced == 1 || forced == 2 ? forced : (stride == 2 && Cin == 3 ? 2 : 1);
#define DRO_K7(S_, C_, NW_, J_)                                                                         \
  do {                                                                                                  \
    if (groups == 2) hipLaunchKernelGGL((wgrad_k7_kernel<S_, C_, NW_, J_, 2>), grid, dim3(128 * NW_), 0, s, a); \
    else hipLaunchKernelGGL((wgrad_k7_kernel<S_, C_, NW_, J_, 1>), grid, dim3(64 * NW_), 0, s, a);     \
  } while (0)
  if (stride == 2 && Cin == 3) DRO_K7(2, 3, 5, 1);
  else if (stride == 2 && Cin == 6) DRO_K7(2, 6, 5, 2);
  else if (stride == 1 && Cin == 1) DRO_K7(1, 1, 2, 1);
  else if (stride == 1 && Cin == 6) DRO_K7(1, 6, 5, 2);
#undef DRO_K7
  else {
    set_error("wgrad_k7: unsupported channel count");
    return DRO_E_SHAPE;
  }
  int st = launch_status("wgrad_k7_kernel launch failed");
  if (st) return st;
  a.K = NK;
  launch_wgrad_finish(a, splits, s);
  return launch_status("wgrad_finish_kernel launch failed");
}

// the stems' forward on fwd_k7s2_kernel: opt-in (env DRO_K7_FWD=1).  Its
// different (equally exact) summation order moves the golden flip step's
// gradients past the reference-fixture check (depth_head.conv2.bias 0.23 %
// from the reference's own fp32 value; the fp64-oracle check passes), so the
// default keeps igemm_kernel's order
bool k7_fwd_ok(int KH, int KW, int Cin, int pad, int stride, int act, const float* bias) {
  static const bool on = env_int("DRO_K7_FWD", 0) != 0;
  return on && KH == 7 && KW == 7 && pad == 3 && stride == 2 && (Cin == 3 || Cin == 6) && act == 0 && !bias;
}

int launch_fwd_k7(IgArgs& a, hipStream_t s) {
  const int tiles = a.g.B * ((a.g.H + 7) / 8) * ((a.g.W + 7) / 8);
  static const int per = (int)env_int("DRO_K7_FWD_TILES_PER_BLOCK", 4);
  int nb = (tiles + per - 1) / per;
  if (nb < 1) nb = 1;
  const dim3 grid((unsigned)nb, (unsigned)((a.g.Cout + 63) / 64));
  conv_logf(2.0 * a.g.Cout * a.g.Cin * 49 * (double)a.g.B * a.g.H * a.g.W, "fwd_k7s2_kernel<%d>", a.g.Cin);
  if (a.g.Cin == 3) hipLaunchKernelGGL((fwd_k7s2_kernel<3>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((fwd_k7s2_kernel<6>), grid, dim3(256), 0, s, a);
  return launch_status("fwd_k7s2_kernel launch failed");
}


template <int MODE, int EPI>
bool thin_ok(const IgArgs& a) {
  if (EPI != 0 || a.g.KH != kThinK || a.g.KW != kThinK || a.g.B > 65535) return false;
  const int cin = MODE == 0 ? a.g.Cin : a.rows;
  if (cin > 8 || a.cbase[1] < cin) return false;
  if (MODE == 1 && a.gsrc[0] == nullptr) return false;
  return true;
}

template <int MODE, int ACT>
int launch_thin(IgArgs& a, int max_splits, hipStream_t s) {
  const int tiles_x = (a.g.W + 7) / 8, tiles = tiles_x * ((a.g.H + 7) / 8);
  const double flops = 2.0 * a.rows * a.kch * a.g.KH * a.g.KW * (double)a.g.B * a.g.H * a.g.W;
  if (MODE == 0) {
    conv_logf(flops, "thin_fwd_kernel<%d>", ACT);
    hipLaunchKernelGGL((thin_fwd_kernel<ACT>), dim3(tiles, (a.g.Cout + 15) / 16, a.g.B), dim3(256), 0,
                       s, a, tiles_x);
    return launch_status("thin_fwd_kernel launch failed");
  }
  // output channels in spans of 16 over up to 4 blocks (partials in the
  // workspace the caller sized for the flat plan's split-K)
  const int splits = max_splits >= 4 ? 4 : (max_splits >= 2 ? 2 : 1);
  const int cps = (a.g.Cout + splits - 1) / splits;
  if (splits == 1) a.part = nullptr;
  const dim3 grid(tiles, splits, a.g.B);
  conv_logf(flops, "thin_dgrad_kernel<%d, %d>", ACT, a.rows == 1 ? 1 : a.rows == 2 ? 2 : a.rows <= 4 ? 4 : 8);
  if (a.rows == 1)
    hipLaunchKernelGGL((thin_dgrad_kernel<ACT, 1>), grid, dim3(256), 0, s, a, tiles_x, cps);
  else if (a.rows == 2)
    hipLaunchKernelGGL((thin_dgrad_kernel<ACT, 2>), grid, dim3(256), 0, s, a, tiles_x, cps);
  else if (a.rows <= 4)
    hipLaunchKernelGGL((thin_dgrad_kernel<ACT, 4>), grid, dim3(256), 0, s, a, tiles_x, cps);
  else
    hipLaunchKernelGGL((thin_dgrad_kernel<ACT, 8>), grid, dim3(256), 0, s, a, tiles_x, cps);
  int st = launch_status("thin_dgrad_kernel launch failed");
  if (st || splits == 1) return st;
  const long long P = (long long)a.g.B * a.g.H * a.g.W;
  const long long total = (long long)a.rows * P;
  hipLaunchKernelGGL((igemm_finish_kernel<1, 0, 0>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     s, a, splits);
  return launch_status("igemm_finish_kernel launch failed");
}

unsigned long long* g_conv_stamps = nullptr;   // dro_debug_conv_stamps

// rows / kch set by the caller; `ws` must hold plan.part_bytes
template <int MODE, int ACT, int EPI, int XF = 0>
int launch_igemm(IgArgs& a, long long P, char* ws, hipStream_t s) {
  IgPlan pl = a.flat_only ? plan_igemm_flat(a.rows, a.kch, a.g.KH, a.g.KW, a.g.B, a.g.H, a.g.W)
                          : plan_igemm(a.rows, a.kch, a.g.KH, a.g.KW, a.g.B, a.g.H, a.g.W);
  // BN fused into the conv (BnFuse): 3x3 halo kernel only, and no split-K for
  // the statistics epilogues (the blocks' own tiles are the partials)
  constexpr bool BNF = EPI >= 5 || XF != 0;
  if (BNF) {
    if (!pl.halo || a.g.KH != 3 || a.g.KW != 3 || a.flat_only) {
      set_error("conv2d: BatchNorm fusion needs a 3x3 stride-1 halo convolution");
      return DRO_E_SHAPE;
    }
    if (EPI >= 5) {
      pl.chunks_per_split = (a.kch + pl.CK - 1) / pl.CK;
      pl.ksplit = 1;
    }
  }
  a.stamps = g_conv_stamps;
  a.dbg = 0;
  if (g_conv_stamps) {
    const char* e = getenv("DRO_CONV_DBG");
    a.dbg = e ? atoi(e) : 0;
  }
  a.K = a.kch * a.g.KH * a.g.KW;
  static const bool thin_off = getenv("DRO_CONV_NO_THIN") != nullptr;   // A/B switch
  if (!BNF && !a.flat_only && !thin_off && thin_ok<MODE, EPI>(a)) {
    a.part = reinterpret_cast<float*>(ws);
    return launch_thin<MODE, ACT>(a, pl.ksplit, s);
  }
  // split-bf16 MFMA engine (xconv.hip) when the caller passed split weights
  if constexpr (EPI < 3 && !BNF) {   // (no GRU / BN epilogues in the split-bf16 engine)
    if (!a.flat_only && a.wsplit && xconv_supported(a.g.KH, a.g.KW)) return launch_xconv<MODE, ACT, EPI>(a, ws, s);
  }
  a.row_tiles = pl.row_tiles;
  a.chunks_per_split = pl.chunks_per_split;
  a.part = pl.ksplit > 1 ? reinterpret_cast<float*>(ws) : nullptr;
  const dim3 grid(pl.row_tiles * pl.ptiles, pl.ksplit);
  const double flops = 2.0 * a.rows * a.kch * a.g.KH * a.g.KW * (double)P;
  if (pl.halo)
    conv_logf(flops, "dconv_kernel<%d, %d, %d, %d, %d, %d, %d>", pl.bm, a.g.KH, a.g.KW, MODE, ACT, EPI, pl.kin);
  else
    conv_logf(flops, "igemm_kernel<%d, %d, %d, %d>", pl.bm, MODE, ACT, EPI);
  if (pl.halo) {
    a.TH = pl.TH;
    a.TW = pl.TW;
    a.HWd = pl.HWd;
    a.HPAD = pl.HPAD;
    a.tiles_x = pl.tiles_x;
    a.tiles_img = pl.tiles_img;
    a.CK = pl.CK;
    a.rt_div = make_div32(pl.row_tiles);
    a.ti_div = make_div32(pl.tiles_img);
    a.tx_div = make_div32(pl.tiles_x);
    if (MODE == 0) {
      const unsigned long long HWl = (unsigned long long)a.g.H * a.g.W;
      for (int t = 0; t < kMaxSrc; ++t) {
        const Slice& sl = a.src[t];
        const unsigned long long chs = sl.bcast ? 1ull : HWl;
        const long long cbt = t == 0 ? 0 : a.cbase[t];
        a.sq0[t] = reinterpret_cast<unsigned long long>(sl.p) +
                   4ull * (unsigned long long)(((long long)sl.coff - cbt) * (long long)chs);
        a.sqb[t] = 4ull * (unsigned long long)sl.ctot * chs;
        a.sr[t] = 4u * (unsigned)chs;
        a.sm[t] = sl.bcast ? 0u : ~0u;
      }
    }
    const int KH = a.g.KH;
    const int KW = a.g.KW;
#define DRO_DCONV(BM_, KH_, KW_)                                                                    \
    do {                                                                                            \
      if (pl.kin == 4)                                                                              \
        hipLaunchKernelGGL((dconv_kernel<BM_, KH_, KW_, MODE, ACT, EPI, 4, XF>), grid, dim3(1024), 0, s, a); \
      else if (pl.kin == 2)                                                                         \
        hipLaunchKernelGGL((dconv_kernel<BM_, KH_, KW_, MODE, ACT, EPI, 2, XF>), grid, dim3(512), 0, s, a);  \
      else                                                                                          \
        hipLaunchKernelGGL((dconv_kernel<BM_, KH_, KW_, MODE, ACT, EPI, 1, XF>), grid, dim3(256), 0, s, a);  \
    } while (0)
    if constexpr (BNF) {
      if (pl.bm == 32) DRO_DCONV(32, 3, 3);
      else DRO_DCONV(64, 3, 3);
    } else if (pl.bm == 32) {
      if (KH == 1 && KW == 1) DRO_DCONV(32, 1, 1);
      else if (KH == 1) DRO_DCONV(32, 1, 5);
      else if (KW == 1) DRO_DCONV(32, 5, 1);
      else DRO_DCONV(32, 3, 3);
    } else {
      if (KH == 1 && KW == 1) DRO_DCONV(64, 1, 1);
      else if (KH == 1) DRO_DCONV(64, 1, 5);
      else if (KW == 1) DRO_DCONV(64, 5, 1);
      else DRO_DCONV(64, 3, 3);
    }
#undef DRO_DCONV
  } else if constexpr (!BNF) {
    a.kdiv = make_fdiv(a.kch);
    if (pl.bm == 64)
      hipLaunchKernelGGL((igemm_kernel<64, MODE, ACT, EPI>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((igemm_kernel<32, MODE, ACT, EPI>), grid, dim3(256), 0, s, a);
  }
  int st = launch_status("conv kernel launch failed");
  if (st || (EPI < 5 && pl.ksplit == 1)) return st;
  if constexpr (EPI >= 5) {   // (never split; XF with split-K takes the finish below)
    if (st || a.bn.inkernel) return st;
    hipLaunchKernelGGL((bn_finalize_kernel<EPI>), dim3((unsigned)a.rows), dim3(256), 0, s, a.bn, a.rows,
                       pl.ptiles, P);
    return launch_status("bn_finalize_kernel launch failed");
  } else {
    const long long total = (long long)a.rows * P;
    long long blocks = (total + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL((igemm_finish_kernel<MODE, ACT, EPI>), dim3((unsigned)blocks), dim3(256), 0, s, a,
                       pl.ksplit);
    return launch_status("igemm_finish_kernel launch failed");
  }
}

int check_ws(const void* ws, size_t have, size_t need, const char* what) {
  if (need > 0 && (!ws || have < need)) {
    static thread_local char msg[192];
    snprintf(msg, sizeof(msg), "%s: workspace of %zu bytes is smaller than the %zu required "
             "(dro_conv2d_workspace_bytes)", what, ws ? have : (size_t)0, need);
    set_error(msg);
    return DRO_E_SHAPE;
  }
  return DRO_OK;
}

}  // namespace

#define DRO_ACT_SWITCH(act, ...)                  \
  switch (act) {                                  \
    case 0: { constexpr int A_ = 0; __VA_ARGS__; } break; \
    case 1: { constexpr int A_ = 1; __VA_ARGS__; } break; \
    case 2: { constexpr int A_ = 2; __VA_ARGS__; } break; \
    case 3: { constexpr int A_ = 3; __VA_ARGS__; } break; \
    default: set_error("conv2d: unknown activation"); return DRO_E_MODE; \
  }

extern "C" int dro_conv2d_plan(int rows, int kch, int KH, int KW, int B, int H, int W, long long* info) {
  if (!info || rows < 1 || kch < 1 || KH < 1 || KW < 1 || B < 1 || H < 1 || W < 1) {
    set_error("conv2d_plan: bad arguments");
    return DRO_E_SHAPE;
  }
  const IgPlan pl = plan_igemm(rows, kch, KH, KW, B, H, W);
  const long long v[16] = {pl.halo, pl.bm, pl.row_tiles, pl.ptiles, pl.ksplit, pl.chunks_per_split,
                           pl.TH, pl.TW, pl.HWd, pl.HPAD, pl.tiles_x, pl.tiles_img, pl.CK,
                           (long long)pl.lds_bytes, (long long)pl.part_bytes, pl.kin};
  for (int i = 0; i < 16; ++i) info[i] = v[i];
  return DRO_OK;
}

extern "C" int dro_conv_log(int enable) {
  std::lock_guard<std::mutex> lk(g_conv_log_mu);
  g_conv_log = enable != 0;
  if (enable) g_conv_log_map.clear();
  return DRO_OK;
}

extern "C" long long dro_conv_log_read(char* buf, long long cap) {
  std::lock_guard<std::mutex> lk(g_conv_log_mu);
  std::string out;
  for (const auto& kv : g_conv_log_map) {
    char line[256];
    snprintf(line, sizeof(line), "%s\t%lld\t%.17g\n", kv.first.c_str(), kv.second.first, kv.second.second);
    out += line;
  }
  const long long n = (long long)out.size();
  if (buf && cap > 0) {
    const long long m = n < cap - 1 ? n : cap - 1;
    memcpy(buf, out.data(), (size_t)m);
    buf[m] = 0;
  }
  return n;
}

extern "C" int dro_debug_conv_stamps(void* buffer) {
  g_conv_stamps = static_cast<unsigned long long*>(buffer);
  return DRO_OK;
}

extern "C" size_t dro_conv2d_workspace_bytes(int B, int H, int W, int Cin, int Cout, int KH, int KW) {
  if (B < 1 || H < 1 || W < 1 || Cin < 1 || Cout < 1 || KH < 1 || KW < 1) return 0;
  const size_t f = fwd_workspace(B, H, W, Cin, Cout, KH, KW);
  const size_t b = bwd_workspace(B, H, W, Cin, Cout, KH, KW);
  return f > b ? f : b;
}

extern "C" int dro_conv2d_forward(const dro_slice* srcs, int nsrc, const float* weight, const float* bias,
                                  int B, int H, int W, int Cout, int KH, int KW, int act, float alpha,
                                  float* out, int out_ctot, int out_coff, const void* wsplit,
                                  void* workspace, size_t workspace_bytes, void* stream) {
  IgArgs a = {};
  a.wsplit = static_cast<const char*>(wsplit);
  int st = conv_setup_geom(a, srcs, nsrc, B, H, W, Cout, KH, KW);
  if (st) return st;
  if (!weight || !out || out_coff < 0 || out_coff + Cout > out_ctot || too_big(B, out_ctot, (long long)H * W)) {
    set_error("conv2d_forward: NULL weight/out or bad output slice");
    return DRO_E_NULL;
  }
  if (alpha != 1.f && act != 0) {
    set_error("conv2d_forward: alpha != 1 requires act none");
    return DRO_E_MODE;
  }
  if ((st = check_ws(workspace, workspace_bytes, fwd_workspace(B, H, W, a.g.Cin, Cout, KH, KW),
                     "conv2d_forward")))
    return st;
  a.weight = weight;
  a.bias = bias;
  a.alpha = alpha;
  a.out = out;
  a.out_ctot = out_ctot;
  a.out_coff = out_coff;
  a.rows = Cout;
  a.kch = a.g.Cin;
  const long long P = (long long)B * H * W;
  hipStream_t s = (hipStream_t)stream;
  char* ws = static_cast<char*>(workspace);
  DRO_ACT_SWITCH(act, st = (launch_igemm<0, A_, 0>(a, P, ws, s)));
  return st;
}

// ---- BatchNorm fused into the 3x3 convs (ABI 10): per-site state layout
// [counters | part: ptiles x C double2 | part2: groups x C double2 | coef: 5 x C]
namespace {
struct BnLayout {
  int ptiles, g1, ngroups;
  size_t cnt, part, part2, coef, bytes;
};

BnLayout bn_layout(int B, int H, int W, int C) {
  BnLayout l;
  l.ptiles = B * ((H + 7) / 8) * ((W + 7) / 8);   // the 3x3 halo kernel's 8 x 8 pixel tiles
  l.g1 = 32;
  l.ngroups = (l.ptiles + l.g1 - 1) / l.g1;
  const int rtmax = (C + 31) / 32;                  // row tiles (BM >= 32)
  l.cnt = 0;
  l.part = align256((size_t)rtmax * (l.ngroups + 1) * sizeof(unsigned));
  l.part2 = l.part + align256((size_t)l.ptiles * C * sizeof(double2));
  l.coef = l.part2 + align256((size_t)l.ngroups * C * sizeof(double2));
  l.bytes = l.coef + align256((size_t)5 * C * sizeof(float));
  return l;
}

void bn_bind(BnFuse& f, void* state, const BnLayout& l) {
  char* b = static_cast<char*>(state);
  f.cnt = reinterpret_cast<unsigned*>(b + l.cnt);
  f.part = reinterpret_cast<double2*>(b + l.part);
  f.part2 = reinterpret_cast<double2*>(b + l.part2);
  f.coef = reinterpret_cast<float*>(b + l.coef);
  f.g1 = l.g1;
  f.ngroups = l.ngroups;
  static const int dbg = [] {
    const char* e = getenv("DRO_BN_ABLATE");
    return e ? atoi(e) : 0;
  }();
  static const int inkernel = [] {   // DRO_BN_FOLD=kernel: the last block folds (A/B)
    const char* e = getenv("DRO_BN_FOLD");
    return e && strcmp(e, "kernel") == 0 ? 1 : 0;
  }();
  f.dbg = dbg;
  f.inkernel = inkernel;
}

const float* bn_coef(const void* state, const BnLayout& l) {
  return reinterpret_cast<const float*>(static_cast<const char*>(state) + l.coef);
}

bool bn_dims_ok(int B, int H, int W, int Cin, int Cout) {
  return B >= 1 && H >= 1 && W >= 1 && Cin >= 1 && Cout >= 1 && Cin < 4096 && Cout < 4096 &&
         !too_big(B, Cin > Cout ? Cin : Cout, (long long)H * W);
}
}  // namespace

extern "C" size_t dro_bn_state_bytes(int B, int H, int W, int C) {
  if (!bn_dims_ok(B, H, W, C, C)) return 0;
  return bn_layout(B, H, W, C).bytes;
}

// y = relu(fmaf(x - mean, k, beta) [+ skip]) from the coefficients a producing
// conv's statistics epilogue left in a BN state (bn_fused_fwd_kernel's
// arithmetic): the BN output of a site whose consumer is not a 3x3 halo conv
namespace {
template <bool VEC>
__global__ __launch_bounds__(256) void bn_coef_apply_kernel(const float* __restrict__ x, const float* __restrict__ skip,
                                                            const float* __restrict__ coef, int relu, int C, int HW,
                                                            float* __restrict__ y) {
  const int plane = blockIdx.y, c = plane % C;
  const float k = coef[c], mu = coef[C + c], o = coef[2 * C + c];
  const long long base = (long long)plane * HW;
  auto f = [&](float v, float s) {
    const float r = fmaf(v - mu, k, o) + s;
    return relu ? fmaxf(r, 0.f) : r;
  };
  const int hw4 = VEC ? (HW & ~3) : 0;
  for (int i = 4 * (blockIdx.x * 256 + threadIdx.x); i < hw4; i += 4 * 256 * gridDim.x) {
    const float4 v = *reinterpret_cast<const float4*>(x + base + i);
    const float4 s = skip ? *reinterpret_cast<const float4*>(skip + base + i) : make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(y + base + i) = make_float4(f(v.x, s.x), f(v.y, s.y), f(v.z, s.z), f(v.w, s.w));
  }
  for (int i = hw4 + blockIdx.x * 256 + threadIdx.x; i < HW; i += 256 * gridDim.x)
    y[base + i] = f(x[base + i], skip ? skip[base + i] : 0.f);
}

// dz = k (g - mean(g) - xhat mean(g xhat)), xhat = (z - mean) invstd, from
// the coefficients a consumer's data gradient (EPI 6) left in the backward
// state: the BN backward's apply where the producer's data gradient does not
// stage it (XF 3 re-reads z once per row tile: dearer than this pass beyond
// one row tile)
template <bool VEC>
__global__ __launch_bounds__(256) void bn_bwd_coef_apply_kernel(const float* __restrict__ g, const float* __restrict__ z,
                                                                const float* __restrict__ coef, int C, int HW,
                                                                float* __restrict__ dz) {
  const int plane = blockIdx.y, c = plane % C;
  const float k = coef[c], mg = coef[C + c], mgx = coef[2 * C + c], mu = coef[3 * C + c], is = coef[4 * C + c];
  const long long base = (long long)plane * HW;
  auto f = [&](float gv, float zv) {
    const float xh = (zv - mu) * is;
    return k * (gv - mg - xh * mgx);
  };
  const int hw4 = VEC ? (HW & ~3) : 0;
  for (int i = 4 * (blockIdx.x * 256 + threadIdx.x); i < hw4; i += 4 * 256 * gridDim.x) {
    const float4 a = *reinterpret_cast<const float4*>(g + base + i);
    const float4 b = *reinterpret_cast<const float4*>(z + base + i);
    *reinterpret_cast<float4*>(dz + base + i) = make_float4(f(a.x, b.x), f(a.y, b.y), f(a.z, b.z), f(a.w, b.w));
  }
  for (int i = hw4 + blockIdx.x * 256 + threadIdx.x; i < HW; i += 256 * gridDim.x) dz[base + i] = f(g[base + i], z[base + i]);
}
}  // namespace

extern "C" int dro_bn_backward_apply(const float* g, const float* z, int B, int C, int H, int W,
                                     const void* state, float* dz, void* stream) {
  if (!bn_dims_ok(B, H, W, C, C) || (long long)B * C > 65535) {
    set_error("bn_backward_apply: sizes out of range");
    return DRO_E_SHAPE;
  }
  if (!g || !z || !dz || !state) {
    set_error("bn_backward_apply: NULL g/z/dz/state");
    return DRO_E_NULL;
  }
  const int HW = H * W;
  const float* coef = bn_coef(state, bn_layout(B, H, W, C));
  long long per = (2048 + (long long)B * C - 1) / ((long long)B * C);
  const long long need = (HW + 1023) / 1024;
  if (per > need) per = need;
  if (per < 1) per = 1;
  const dim3 grid((unsigned)per, (unsigned)(B * C));
  auto al = [](const void* p) { return (reinterpret_cast<size_t>(p) & 15) == 0; };
  hipStream_t s = (hipStream_t)stream;
  if ((HW & 3) == 0 && al(g) && al(z) && al(dz))
    hipLaunchKernelGGL(bn_bwd_coef_apply_kernel<true>, grid, dim3(256), 0, s, g, z, coef, C, HW, dz);
  else
    hipLaunchKernelGGL(bn_bwd_coef_apply_kernel<false>, grid, dim3(256), 0, s, g, z, coef, C, HW, dz);
  return launch_status("bn_bwd_coef_apply_kernel launch failed");
}

extern "C" int dro_bn_apply(const float* x, const float* skip, int relu, int B, int C, int H, int W,
                            const void* state, float* y, void* stream) {
  if (!bn_dims_ok(B, H, W, C, C) || (long long)B * C > 65535) {
    set_error("bn_apply: sizes out of range");
    return DRO_E_SHAPE;
  }
  if (!x || !y || !state) {
    set_error("bn_apply: NULL x/y/state");
    return DRO_E_NULL;
  }
  if (relu != 0 && relu != 1) {
    set_error("bn_apply: relu must be 0 or 1");
    return DRO_E_MODE;
  }
  const int HW = H * W;
  const float* coef = bn_coef(state, bn_layout(B, H, W, C));
  long long per = (2048 + (long long)B * C - 1) / ((long long)B * C);
  const long long need = (HW + 1023) / 1024;
  if (per > need) per = need;
  if (per < 1) per = 1;
  const dim3 grid((unsigned)per, (unsigned)(B * C));
  auto al = [](const void* p) { return p == nullptr || (reinterpret_cast<size_t>(p) & 15) == 0; };
  hipStream_t s = (hipStream_t)stream;
  if ((HW & 3) == 0 && al(x) && al(skip) && al(y))
    hipLaunchKernelGGL(bn_coef_apply_kernel<true>, grid, dim3(256), 0, s, x, skip, coef, relu, C, HW, y);
  else
    hipLaunchKernelGGL(bn_coef_apply_kernel<false>, grid, dim3(256), 0, s, x, skip, coef, relu, C, HW, y);
  return launch_status("bn_coef_apply_kernel launch failed");
}

extern "C" int dro_conv2d_bn_forward(const float* x, int B, int H, int W, int Cin, const float* weight, int Cout,
                                     const void* in_state, const float* in_skip, float* in_y,
                                     const dro_bn_params* bn, void* out_state, float* out, void* workspace,
                                     size_t workspace_bytes, void* stream) {
  if (!bn_dims_ok(B, H, W, Cin, Cout)) {
    set_error("conv2d_bn_forward: sizes out of range");
    return DRO_E_SHAPE;
  }
  if (!x || !weight || !out || (!in_state) != (!in_y) || (in_skip && !in_state) || (!bn) != (!out_state) ||
      (bn && (!bn->save_mean || !bn->save_invstd || (!bn->running_mean) != (!bn->running_var)))) {
    set_error("conv2d_bn_forward: NULL pointer (x/weight/out; in_y with in_state; out_state and "
              "save_mean/save_invstd with bn)");
    return DRO_E_NULL;
  }
  const dro_slice sl{x, Cin, Cin, 0, 0};
  IgArgs a = {};
  int st = conv_setup_geom(a, &sl, 1, B, H, W, Cout, 3, 3);
  if (st) return st;
  if ((st = check_ws(workspace, workspace_bytes, fwd_workspace(B, H, W, Cin, Cout, 3, 3), "conv2d_bn_forward")))
    return st;
  a.weight = weight;
  a.alpha = 1.f;
  a.out = out;
  a.out_ctot = Cout;
  a.out_coff = 0;
  a.rows = Cout;
  a.kch = Cin;
  if (in_state) {
    a.bn.xcoef = bn_coef(in_state, bn_layout(B, H, W, Cin));
    a.bn.skip = in_skip;
    a.bn.yout = in_y;
  }
  if (bn) {
    bn_bind(a.bn, out_state, bn_layout(B, H, W, Cout));
    a.bn.gamma = bn->gamma;
    a.bn.beta = bn->beta;
    a.bn.rmean = bn->running_mean;
    a.bn.rvar = bn->running_var;
    a.bn.nbt = bn->num_batches_tracked;
    a.bn.eps = bn->eps;
    a.bn.momentum = bn->momentum;
    a.bn.save_mean = bn->save_mean;
    a.bn.save_invstd = bn->save_invstd;
  }
  const long long P = (long long)B * H * W;
  hipStream_t s = (hipStream_t)stream;
  char* ws = static_cast<char*>(workspace);
  const int xf = in_state ? (in_skip ? 2 : 1) : 0;
  if (bn) {
    if (xf == 2) return launch_igemm<0, 0, 5, 2>(a, P, ws, s);
    if (xf == 1) return launch_igemm<0, 0, 5, 1>(a, P, ws, s);
    return launch_igemm<0, 0, 5, 0>(a, P, ws, s);
  }
  if (xf == 2) return launch_igemm<0, 0, 0, 2>(a, P, ws, s);
  if (xf == 1) return launch_igemm<0, 0, 0, 1>(a, P, ws, s);
  return launch_igemm<0, 0, 0, 0>(a, P, ws, s);
}

extern "C" int dro_conv2d_bn_backward_data(const float* weight, int B, int H, int W, int Cin, int Cout,
                                           const float* dout, const void* gin_state, const float* gin_z,
                                           float* gin_dz, const dro_bn_grad_params* src_bn, void* src_state,
                                           float* grad_x, int grad_x_accumulate, void* workspace,
                                           size_t workspace_bytes, void* stream) {
  if (!bn_dims_ok(B, H, W, Cin, Cout)) {
    set_error("conv2d_bn_backward_data: sizes out of range");
    return DRO_E_SHAPE;
  }
  if (!weight || !dout || !grad_x || (gin_state && (!gin_z || !gin_dz)) || (!src_bn) != (!src_state) ||
      (src_bn && (!src_bn->y || !src_bn->z || !src_bn->save_mean || !src_bn->save_invstd))) {
    set_error("conv2d_bn_backward_data: NULL pointer (weight/dout/grad_x; gin_z/gin_dz with gin_state; "
              "src_state and y/z/save_mean/save_invstd with src_bn)");
    return DRO_E_NULL;
  }
  if (src_bn && grad_x_accumulate) {
    set_error("conv2d_bn_backward_data: grad_x receives g with src_bn (no accumulation)");
    return DRO_E_MODE;
  }
  if (gin_state && src_bn) {
    set_error("conv2d_bn_backward_data: gin_state and src_bn in one call are not supported");
    return DRO_E_MODE;
  }
  const dro_slice sl{grad_x, Cin, Cin, 0, 0};   // geometry only (the data gradient stages dout)
  IgArgs a = {};
  int st = conv_setup_geom(a, &sl, 1, B, H, W, Cout, 3, 3);
  if (st) return st;
  if ((st = check_ws(workspace, workspace_bytes, plan_igemm(Cin, Cout, 3, 3, B, H, W).part_bytes,
                     "conv2d_bn_backward_data")))
    return st;
  a.weight = weight;
  a.G = dout;
  a.galpha = 1.f;
  a.gsrc[0] = grad_x;
  a.gsrc_ctot[0] = Cin;
  a.gsrc_coff[0] = 0;
  a.gsrc_acc[0] = grad_x_accumulate ? 1 : 0;
  a.rows = Cin;
  a.kch = Cout;
  if (gin_state) {
    a.bn.xcoef = bn_coef(gin_state, bn_layout(B, H, W, Cout));
    a.bn.z = gin_z;
    a.bn.yout = gin_dz;
  }
  if (src_bn) {
    bn_bind(a.bn, src_state, bn_layout(B, H, W, Cin));
    a.bn.y = src_bn->y;
    a.bn.z = src_bn->z;
    a.bn.gamma = src_bn->gamma;
    a.bn.mean = src_bn->save_mean;
    a.bn.invstd = src_bn->save_invstd;
    a.bn.dgamma = src_bn->grad_gamma;
    a.bn.dbeta = src_bn->grad_beta;
  }
  const long long P = (long long)B * H * W;
  hipStream_t s = (hipStream_t)stream;
  char* ws = static_cast<char*>(workspace);
  if (src_bn) return launch_igemm<1, 0, 6, 0>(a, P, ws, s);
  if (gin_state) return launch_igemm<1, 0, 0, 3>(a, P, ws, s);
  return launch_igemm<1, 0, 0, 0>(a, P, ws, s);
}

extern "C" int dro_convgru_gates_forward(const dro_slice* srcs, int nsrc, const float* weight,
                                         const float* bias, int B, int H, int W, int hd, int KH, int KW,
                                         float* zr, float* rh, const void* wsplit, void* workspace,
                                         size_t workspace_bytes, void* stream) {
  IgArgs a = {};
  a.wsplit = static_cast<const char*>(wsplit);
  int st = conv_setup_geom(a, srcs, nsrc, B, H, W, 2 * hd, KH, KW);
  if (st) return st;
  if (!weight || !zr || !rh) {
    set_error("convgru_gates_forward: NULL weight/zr/rh");
    return DRO_E_NULL;
  }
  if (srcs[0].channels != hd || srcs[0].broadcast) {
    set_error("convgru_gates_forward: source 0 must be the dense hidden state (hd channels)");
    return DRO_E_SHAPE;
  }
  if ((st = check_ws(workspace, workspace_bytes, fwd_workspace(B, H, W, a.g.Cin, 2 * hd, KH, KW),
                     "convgru_gates_forward")))
    return st;
  a.weight = weight;
  a.bias = bias;
  a.alpha = 1.f;
  a.out = zr;
  a.out_ctot = 2 * hd;
  a.out_coff = 0;
  a.h = to_slice(srcs);
  a.aux = rh;
  a.hd = hd;
  a.rows = 2 * hd;
  a.kch = a.g.Cin;
  return launch_igemm<0, 2, 2>(a, (long long)B * H * W, static_cast<char*>(workspace), (hipStream_t)stream);
}

extern "C" int dro_convgru_blend_forward(const dro_slice* srcs, int nsrc, const float* weight,
                                         const float* bias, int B, int H, int W, int Cout, int KH, int KW,
                                         const dro_slice* z, const dro_slice* h, float* q_out, float* out,
                                         int out_ctot, int out_coff, const void* wsplit, void* workspace,
                                         size_t workspace_bytes, void* stream) {
  IgArgs a = {};
  a.wsplit = static_cast<const char*>(wsplit);
  int st = conv_setup_geom(a, srcs, nsrc, B, H, W, Cout, KH, KW);
  if (st) return st;
  if (!weight || !out || !q_out || !z || !h || !z->data || !h->data) {
    set_error("convgru_blend_forward: NULL weight/out/q/z/h");
    return DRO_E_NULL;
  }
  if ((st = check_ws(workspace, workspace_bytes, fwd_workspace(B, H, W, a.g.Cin, Cout, KH, KW),
                     "convgru_blend_forward")))
    return st;
  a.weight = weight;
  a.bias = bias;
  a.alpha = 1.f;
  a.out = out;
  a.out_ctot = out_ctot;
  a.out_coff = out_coff;
  a.z = to_slice(z);
  a.h = to_slice(h);
  a.aux = q_out;
  a.rows = Cout;
  a.kch = a.g.Cin;
  return launch_igemm<0, 3, 1>(a, (long long)B * H * W, static_cast<char*>(workspace),
                               (hipStream_t)stream);
}

// SepConvGRU stage 2 folded into the candidate conv's data gradient (EPI 3)
// kind 3: stage 2 of this half in the candidate conv (source 0 = r*h);
// kind 4: stage 1 of the previous half in this half's gate conv (source 0 = h,
// its finished gradient is the previous half's dh')
struct GruFold {
  int kind;
  const float* zr;
  const float* h;
  float* dzr;
  float* dh;
  const float* q;
  float* dq;
  int dh_acc;
};

static int conv2d_backward_impl(const dro_slice* srcs, int nsrc, const float* weight, int B, int H, int W,
                                int Cout, int KH, int KW, int act, float alpha, const dro_slice* y,
                                const float* dout, float* const* grad_srcs, const int* grad_ctot,
                                const int* grad_coff, const int* grad_accumulate, float* grad_weight,
                                float* grad_bias, int grad_weight_accumulate, const void* wsplit,
                                void* workspace, size_t workspace_bytes, void* stream, const GruFold* gf) {
  IgArgs a = {};
  a.wsplit = static_cast<const char*>(wsplit);   // transposed layout: the data gradient
  int st = conv_setup_geom(a, srcs, nsrc, B, H, W, Cout, KH, KW);
  if (st) return st;
  const bool pre = act != 0 || alpha != 1.f;
  if (!weight || !dout || (act != 0 && (!y || !y->data))) {
    set_error("conv2d_backward: NULL weight/dout/y");
    return DRO_E_NULL;
  }
  if (act < 0 || act > 3) {
    set_error("conv2d_backward: unknown activation");
    return DRO_E_MODE;
  }
  if (grad_bias && !grad_weight) {
    set_error("conv2d_backward: grad_bias requires grad_weight");
    return DRO_E_NULL;
  }
  if ((st = check_ws(workspace, workspace_bytes, bwd_workspace(B, H, W, a.g.Cin, Cout, KH, KW),
                     "conv2d_backward")))
    return st;
  for (int i = 0; i < nsrc; ++i) {
    a.gsrc[i] = grad_srcs ? grad_srcs[i] : nullptr;
    a.gsrc_ctot[i] = grad_ctot ? grad_ctot[i] : srcs[i].channels;
    a.gsrc_coff[i] = grad_coff ? grad_coff[i] : 0;
    a.gsrc_acc[i] = grad_accumulate ? grad_accumulate[i] : 0;
    if (a.gsrc[i] && too_big(B, a.gsrc_ctot[i], (long long)H * W)) {
      set_error("conv2d_backward: gradient target too large (32-bit offsets)");
      return DRO_E_SHAPE;
    }
  }
  if (gf && gf->kind == 3) {   // source 0 is r*h (Cout channels): its gradient feeds stage 2, not a buffer
    if (!gf->zr || !gf->h || !gf->dzr || !gf->dh) {
      set_error("convgru_candidate_backward: NULL zr/h/dzr/dh");
      return DRO_E_NULL;
    }
    if (srcs[0].channels != Cout || act != 0 || alpha != 1.f || grad_weight || too_big(B, 2 * Cout, (long long)H * W)) {
      set_error("convgru_candidate_backward: source 0 must be r*h with Cout channels (no activation, no weight gradient)");
      return DRO_E_SHAPE;
    }
    a.z = Slice{gf->zr, Cout, 2 * Cout, Cout, 0};
    a.h = Slice{gf->h, Cout, Cout, 0, 0};
    a.aux = gf->dzr;
    a.hd = Cout;
    a.gsrc[0] = gf->dh;
    a.gsrc_ctot[0] = Cout;
    a.gsrc_coff[0] = 0;
    a.gsrc_acc[0] = 1;
    a.wsplit = nullptr;   // the split-bf16 engine has no GRU epilogues
  } else if (gf) {   // kind 4: source 0 is this half's h (hd = Cout / 2 channels), accumulated
    const int hd = Cout / 2;
    if (!gf->zr || !gf->h || !gf->dzr || !gf->dh || !gf->q || !gf->dq || !a.gsrc[0]) {
      set_error("convgru_gates_backward: NULL zr/h/q/dq/dzr/dh or d h target");
      return DRO_E_NULL;
    }
    if (Cout % 2 || srcs[0].channels != hd || act != 0 || alpha != 1.f || grad_weight ||
        a.gsrc_ctot[0] != hd || a.gsrc_coff[0] != 0 || too_big(B, Cout, (long long)H * W)) {
      set_error("convgru_gates_backward: source 0 must be h with Cout / 2 channels and a dense d h target "
                "(no activation, no weight gradient)");
      return DRO_E_SHAPE;
    }
    a.z = Slice{gf->zr, hd, Cout, 0, 0};
    a.h = Slice{gf->h, hd, hd, 0, 0};
    a.aux = gf->dzr;
    a.hd = hd;
    a.g1q = gf->q;
    a.g1dq = gf->dq;
    a.g1dh = gf->dh;
    a.g1acc = gf->dh_acc ? 1 : 0;
    a.gsrc_acc[0] = 1;
    a.wsplit = nullptr;
  }
  a.weight = weight;
  a.gweight = grad_weight;
  a.gbias = grad_bias;
  a.wacc = grad_weight_accumulate ? 1 : 0;
  hipStream_t s = (hipStream_t)stream;
  const size_t HW = (size_t)H * W;
  const long long P = (long long)B * HW;
  const int T = KH * KW;
  char* ws = static_cast<char*>(workspace);
  char* ws_pre = ws;
  char* ws_ig = ws_pre + align256((size_t)Cout * P * sizeof(float));
  char* ws_wg = ws_ig + std::max(plan_igemm(a.g.Cin, Cout, KH, KW, B, H, W).part_bytes,
                                 xconv_part_bytes(a.g.Cin, Cout, KH, KW, B, H, W));
  // fold the activation derivative into the halo kernels' G staging when both
  // gradients run there (dense y); otherwise form G first
  const WhPlan wh = plan_wgrad_halo(a.g.Cin, Cout, KH, KW, B, H, W);
  const bool halo_dgrad = plan_igemm(a.g.Cin, Cout, KH, KW, B, H, W).halo;
  // the thin data gradient (7x7 over <= 8 input channels, one source) folds
  // as well; a call without a weight gradient (the trainer queues those)
  // needs only its data-gradient kernel to fold
  static const bool thin_off = getenv("DRO_CONV_NO_THIN") != nullptr;
  const bool thin_dgrad = KH == kThinK && KW == kThinK && nsrc == 1 && a.g.Cin <= 8 && B <= 65535 && !thin_off;
  const bool fold = pre && (halo_dgrad || thin_dgrad) && (wh.ok || !grad_weight) &&
                    (act == 0 || (y->total_channels == Cout && y->channel_offset == 0));
  a.galpha = fold ? alpha : 1.f;
  a.gy = (fold && act) ? y->data : nullptr;
  if (pre && !fold) {
    if ((long long)B * Cout > 65535 || HW >= ((size_t)1 << 31)) {
      set_error("conv2d_backward: B * Cout or H * W out of range for the gradient pre-pass");
      return DRO_E_SHAPE;
    }
    float* G = reinterpret_cast<float*>(ws_pre);
    hipLaunchKernelGGL(grad_pre_kernel, dim3((unsigned)((HW + 255) / 256), (unsigned)(B * Cout)), dim3(256), 0, s,
                       act, alpha, Cout, (int)HW, dout, to_slice(y), G);
    if ((st = launch_status("grad_pre_kernel launch failed"))) return st;
    a.G = G;
  } else {
    a.G = dout;
  }
  bool any_dgrad = false;
  for (int i = 0; i < nsrc; ++i) any_dgrad |= a.gsrc[i] != nullptr;
  if (any_dgrad) {
    a.rows = a.g.Cin;
    a.kch = Cout;
    const int gact = fold ? act : 0;
    if (gf && gf->kind == 3)
      st = launch_igemm<1, 0, 3>(a, P, ws_ig, s);
    else if (gf)
      st = launch_igemm<1, 0, 4>(a, P, ws_ig, s);
    else
      DRO_ACT_SWITCH(gact, st = (launch_igemm<1, A_, 0>(a, P, ws_ig, s)));
    if (st) return st;
  }
  if (grad_weight && wh.ok && !wgrad_v1()) {
    const WhPlan w2 = plan_wgrad2(a.g.Cin, Cout, KH, KW, 0, B, H, W);
    a.otiles = w2.otiles;
    a.tiles_x = w2.tiles_x;
    a.tiles_img = w2.tiles_img;
    a.chunks_per_split = w2.tiles_per_split;
    a.part = reinterpret_cast<float*>(ws_wg);
    a.bpart = reinterpret_cast<float*>(ws_wg + align256((size_t)w2.splits * Cout * a.g.Cin * T * sizeof(float)));
    const dim3 grid((unsigned)(w2.otiles * w2.ctiles * w2.tgroups), (unsigned)w2.splits);
    const int gact = fold ? act : 0;
    conv_logf(2.0 * Cout * a.g.Cin * T * (double)P, "wgrad2_kernel<%d, %d, %d, false, %d>", KH, KW, gact,
              w2.tgroups);
#define DRO_WG2(KH_, KW_, TG_) DRO_ACT_SWITCH(gact, hipLaunchKernelGGL((wgrad2_kernel<KH_, KW_, A_, false, TG_>), grid, dim3(512), 0, s, a))
    if (KH == 1 && KW == 1) { DRO_WG2(1, 1, 1); }
    else if (KH == 1) { DRO_WG2(1, 5, 1); }
    else if (KW == 1) { DRO_WG2(5, 1, 1); }
    else if (w2.tgroups == 3) { DRO_WG2(3, 3, 3); }
    else { DRO_WG2(3, 3, 1); }
#undef DRO_WG2
    if ((st = launch_status("wgrad2_kernel launch failed"))) return st;
    launch_wgrad2_finish(a, w2.splits, s);
    if ((st = launch_status("wgrad_halo_finish_kernel launch failed"))) return st;
  } else if (grad_weight && wh.ok) {
    a.otiles = wh.otiles;
    a.tiles_x = wh.tiles_x;
    a.tiles_img = wh.tiles_img;
    a.chunks_per_split = wh.tiles_per_split;
    a.part = reinterpret_cast<float*>(ws_wg);
    a.bpart = reinterpret_cast<float*>(ws_wg + align256((size_t)wh.splits * Cout * a.g.Cin * T * sizeof(float)));
    const dim3 grid((unsigned)(wh.otiles * wh.ctiles), (unsigned)wh.splits);
    const int gact = fold ? act : 0;
    conv_logf(2.0 * Cout * a.g.Cin * T * (double)P, "wgrad_halo_kernel<%d, %d, %d, false>", KH, KW, gact);
#define DRO_WH(KH_, KW_) DRO_ACT_SWITCH(gact, hipLaunchKernelGGL((wgrad_halo_kernel<KH_, KW_, A_, false>), grid, dim3(256), 0, s, a))
    if (KH == 1 && KW == 1) { DRO_WH(1, 1); }
    else if (KH == 1) { DRO_WH(1, 5); }
    else if (KW == 1) { DRO_WH(5, 1); }
    else { DRO_WH(3, 3); }
#undef DRO_WH
    if ((st = launch_status("wgrad_halo_kernel launch failed"))) return st;
    const long long total = (long long)Cout * a.g.Cin * T;
    long long blocks = (total + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(wgrad_halo_finish_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, wh.splits);
    if ((st = launch_status("wgrad_halo_finish_kernel launch failed"))) return st;
  } else if (grad_weight) {
    const WgPlan pl = plan_wgrad(a.g.Cin, Cout, T, P);
    a.K = a.g.Cin * T;
    a.otiles = pl.otiles;
    a.pchunk = pl.pchunk;
    a.part = reinterpret_cast<float*>(ws_wg);
    if (nsrc == 1 && !srcs[0].broadcast && srcs[0].channel_offset == 0 && srcs[0].total_channels == srcs[0].channels &&
        k7_ok(KH, KW, a.g.Cin, KH / 2, 1)) {
      // the update blocks' 7x7 state convs (stride 1, one dense source)
      a.Hs = H;
      a.Ws = W;
      return launch_wgrad_k7(a, 1, pl.splits, s);
    }
    conv_log("wgrad_kernel(", 2.0 * Cout * a.g.Cin * T * (double)P);
    hipLaunchKernelGGL(wgrad_kernel, dim3((unsigned)(pl.otiles * pl.ntiles), (unsigned)pl.splits),
                       dim3(256), 0, s, a);
    if ((st = launch_status("wgrad_kernel launch failed"))) return st;
    launch_wgrad_finish(a, pl.splits, s);
    if ((st = launch_status("wgrad_finish_kernel launch failed"))) return st;
  }
  return DRO_OK;
}

extern "C" int dro_conv2d_backward(const dro_slice* srcs, int nsrc, const float* weight, int B, int H,
                                   int W, int Cout, int KH, int KW, int act, float alpha,
                                   const dro_slice* y, const float* dout, float* const* grad_srcs,
                                   const int* grad_ctot, const int* grad_coff,
                                   const int* grad_accumulate, float* grad_weight, float* grad_bias,
                                   int grad_weight_accumulate, const void* wsplit, void* workspace,
                                   size_t workspace_bytes, void* stream) {
  return conv2d_backward_impl(srcs, nsrc, weight, B, H, W, Cout, KH, KW, act, alpha, y, dout, grad_srcs,
                              grad_ctot, grad_coff, grad_accumulate, grad_weight, grad_bias,
                              grad_weight_accumulate, wsplit, workspace, workspace_bytes, stream, nullptr);
}

extern "C" int dro_convgru_candidate_backward(const dro_slice* srcs, int nsrc, const float* weight, int B,
                                              int H, int W, int hd, int KH, int KW, const float* dq,
                                              const float* zr, const float* h, float* dzr, float* dh,
                                              float* const* grad_srcs, const int* grad_ctot,
                                              const int* grad_coff, const int* grad_accumulate,
                                              void* workspace, size_t workspace_bytes, void* stream) {
  if (!srcs || nsrc < 1) {
    set_error("convgru_candidate_backward: need the r*h source");
    return DRO_E_NULL;
  }
  const GruFold gf = {3, zr, h, dzr, dh, nullptr, nullptr, 0};
  return conv2d_backward_impl(srcs, nsrc, weight, B, H, W, hd, KH, KW, 0, 1.f, nullptr, dq, grad_srcs, grad_ctot,
                              grad_coff, grad_accumulate, nullptr, nullptr, 0, nullptr, workspace, workspace_bytes,
                              stream, &gf);
}

extern "C" int dro_convgru_gates_backward(const dro_slice* srcs, int nsrc, const float* weight, int B, int H,
                                          int W, int hd, int KH, int KW, const float* dzr_in,
                                          float* const* grad_srcs, const int* grad_ctot, const int* grad_coff,
                                          const int* grad_accumulate, const float* prev_zr, const float* prev_q,
                                          const float* prev_h, float* prev_dq, float* prev_dzr, float* prev_dh,
                                          int prev_dh_accumulate, void* workspace, size_t workspace_bytes,
                                          void* stream) {
  if (!srcs || nsrc < 1 || !grad_srcs) {
    set_error("convgru_gates_backward: need the h source and its gradient target");
    return DRO_E_NULL;
  }
  const GruFold gf = {4, prev_zr, prev_h, prev_dzr, prev_dh, prev_q, prev_dq, prev_dh_accumulate};
  return conv2d_backward_impl(srcs, nsrc, weight, B, H, W, 2 * hd, KH, KW, 0, 1.f, nullptr, dzr_in, grad_srcs,
                              grad_ctot, grad_coff, grad_accumulate, nullptr, nullptr, 0, nullptr, workspace,
                              workspace_bytes, stream, &gf);
}

// split-K partials of the parity-class data gradient, [split][class][rows][pcmax]
// -> the strided input gradient (fixed split order: deterministic)
__global__ __launch_bounds__(256) void igemm_class_finish_kernel(IgArgs a, int ksplit) {
  // grid (pixel blocks of the largest class, 4 * rows): class and row are
  // block-uniform, 32-bit index arithmetic (4 * rows * pcmax < 2^31, checked
  // by the launcher)
  const int H = a.g.H, W = a.g.W;
  const size_t HW = (size_t)H * W;
  const unsigned pcm = (unsigned)a.pcmax, rows = (unsigned)a.rows;
  const unsigned zr = blockIdx.y, z = zr / rows, row = zr - z * rows;
  const int cy = (int)(z >> 1), cx = (int)(z & 1);
  const unsigned Hc = (unsigned)((H - cy + 1) >> 1), Wc = (unsigned)((W - cx + 1) >> 1), HWc = Hc * Wc;
  const unsigned pe = blockIdx.x * blockDim.x + threadIdx.x;
  if (pe >= (unsigned)a.g.B * HWc) return;
  const size_t total = (size_t)4 * rows * pcm;
  const float v = split_sum(a.part + (size_t)zr * pcm + pe, total, ksplit);
  const unsigned eb = pe / HWc, q = pe - eb * HWc, Y = q / Wc, X = q - Y * Wc;
  epi_store<1, 0, 0>(a, (int)row, (int)eb, (size_t)(2 * Y + cy) * W + 2 * X + cx, HW, v);
}

// ------------------------------------------------------------------ strided convolutions
// The ResNet encoders' stride-2 convolutions (extractor.py:7-107 /
// torchvision BasicBlock + stem): 7x7/s2 pad 3 stems, 3x3/s2 pad 1 stage
// entries, 1x1/s2 downsamples; one dense NCHW input, no bias / activation
// needed there (BN follows) but both are supported in the forward.  They run
// on the flattened implicit GEMM (igemm_kernel: per-tap gathers, so any
// kernel size and stride) and the generic weight-gradient kernel
// (wgrad_kernel), with the staged operand's own size and the stride:
//   forward      out[o, y, x] = sum W[o, c, t] * X[c, S*y + ty - P, S*x + tx - P]
//   data grad    dX[c, y, x]  = sum W[o, c, t] * G[o, (y + P - ty) / S, (x + P - tx) / S]  (exact only)
//   weight grad  dW[o, c, t]  = sum G[o, y, x] * X[c, S*y + ty - P, S*x + tx - P]
namespace {
int strided_setup(IgArgs& a, const float* x, int B, int Hi, int Wi, int Cin, int Cout, int KH, int KW,
                  int stride, int pad, int& Ho, int& Wo) {
  if (!x) {
    set_error("conv2d_strided: NULL input");
    return DRO_E_NULL;
  }
  if (B < 1 || Hi < 1 || Wi < 1 || Cin < 1 || Cout < 1 || KH < 1 || KW < 1 || pad < 0 ||
      (stride != 1 && stride != 2) || Cin >= 4096 || Cout >= 4096 || (long long)Cin * KH * KW >= 65535 ||
      (long long)Cout * KH * KW >= 65535) {
    set_error("conv2d_strided: sizes out of range (stride 1 or 2, C < 4096, C*KH*KW < 65535)");
    return DRO_E_SHAPE;
  }
  Ho = (Hi + 2 * pad - KH) / stride + 1;
  Wo = (Wi + 2 * pad - KW) / stride + 1;
  if (Ho < 1 || Wo < 1 || too_big(B, Cin, (long long)Hi * Wi) || too_big(B, Cout, (long long)Ho * Wo)) {
    set_error("conv2d_strided: empty output or a tensor of >= 2^30 elements");
    return DRO_E_SHAPE;
  }
  const dro_slice src = {x, Cin, Cin, 0, 0};
  // geometry of the output (the forward's GEMM columns); 'same' checks skipped
  ConvGeom& g = a.g;
  g.B = B;
  g.H = Ho;
  g.W = Wo;
  g.Cin = Cin;
  g.Cout = Cout;
  g.KH = KH;
  g.KW = KW;
  g.PH = pad;
  g.PW = pad;
  for (int i = 0; i < kMaxSrc; ++i) {
    a.src[i].p = src.data;
    a.src[i].C = Cin;
    a.src[i].ctot = Cin;
    a.src[i].coff = 0;
    a.src[i].bcast = 0;
    a.cbase[i] = i == 0 ? 0 : Cin;
  }
  a.kwdiv = make_fdiv(KW);
  a.cindiv = make_fdiv(Cin);
  a.Hs = Hi;
  a.Ws = Wi;
  a.sshift = stride == 2 ? 1 : 0;
  a.flat_only = 1;
  return DRO_OK;
}
}  // namespace

// parity-class data gradient plan (stride 2): tiles over the largest class,
// K split over grid.y until ~4 blocks per CU
struct ClassPlan {
  int bm, row_tiles, ptiles, ksplit, chunks_per_split;
  long long pcmax;
  size_t part_bytes;
};

static ClassPlan plan_class_dgrad(int B, int Hi, int Wi, int Cin, int Cout, int KH, int KW) {
  ClassPlan cp = {};
  cp.pcmax = (long long)B * ((Hi + 1) / 2) * ((Wi + 1) / 2);
  cp.ptiles = (int)((cp.pcmax + kBN - 1) / kBN);
  cp.bm = (long long)((Cin + 63) / 64) * cp.ptiles * 4 >= 448 ? 64 : 32;
  cp.row_tiles = (Cin + cp.bm - 1) / cp.bm;
  const int nck = (((KH + 1) / 2) * ((KW + 1) / 2) * Cout + kBK - 1) / kBK;   // the largest class
  const long long blocks = 4LL * cp.row_tiles * cp.ptiles;
  static const long long target = env_int("DRO_CLASS_TARGET", 1024);
  int ks = 1;
  if (blocks < target) {
    ks = (int)((target + blocks - 1) / blocks);
    if (ks > 16) ks = 16;
    if (ks > nck / 4) ks = nck / 4;      // >= 4 chunks per split
    if (ks < 1) ks = 1;
  }
  cp.chunks_per_split = (nck + ks - 1) / ks;
  cp.ksplit = (nck + cp.chunks_per_split - 1) / cp.chunks_per_split;
  cp.part_bytes = cp.ksplit > 1 ? align256((size_t)cp.ksplit * 4 * Cin * cp.pcmax * sizeof(float)) : 0;
  return cp;
}

extern "C" size_t dro_conv2d_strided_workspace_bytes(int B, int Hi, int Wi, int Cin, int Cout, int KH, int KW,
                                                     int stride, int pad) {
  if (stride < 1) return 0;
  const int Ho = (Hi + 2 * pad - KH) / stride + 1, Wo = (Wi + 2 * pad - KW) / stride + 1;
  if (Ho < 1 || Wo < 1) return 0;
  const size_t fwd = plan_igemm_flat(Cout, Cin, KH, KW, B, Ho, Wo).part_bytes;
  const size_t dg = std::max(plan_igemm_flat(Cin, Cout, KH, KW, B, Hi, Wi).part_bytes,
                             stride == 2 ? plan_class_dgrad(B, Hi, Wi, Cin, Cout, KH, KW).part_bytes : (size_t)0);
  size_t wg = plan_wgrad(Cin, Cout, KH * KW, (long long)B * Ho * Wo).part_bytes;
  if (k7_ok(KH, KW, Cin, pad, stride)) wg = std::max(wg, k7_part_bytes(B, Ho, Wo, Cin, Cout));
  return std::max(fwd, align256(dg) + wg);
}

extern "C" int dro_conv2d_strided_forward(const float* x, const float* weight, const float* bias, int B, int Hi,
                                          int Wi, int Cin, int Cout, int KH, int KW, int stride, int pad,
                                          int act, float* out, void* workspace, size_t workspace_bytes,
                                          void* stream) {
  IgArgs a = {};
  int Ho, Wo;
  int st = strided_setup(a, x, B, Hi, Wi, Cin, Cout, KH, KW, stride, pad, Ho, Wo);
  if (st) return st;
  if (!weight || !out) {
    set_error("conv2d_strided_forward: NULL weight/out");
    return DRO_E_NULL;
  }
  if ((st = check_ws(workspace, workspace_bytes,
                     dro_conv2d_strided_workspace_bytes(B, Hi, Wi, Cin, Cout, KH, KW, stride, pad),
                     "conv2d_strided_forward")))
    return st;
  a.weight = weight;
  a.bias = bias;
  a.alpha = 1.f;
  a.out = out;
  a.out_ctot = Cout;
  a.out_coff = 0;
  a.rows = Cout;
  a.kch = Cin;
  const long long P = (long long)B * Ho * Wo;
  hipStream_t s = (hipStream_t)stream;
  if (k7_fwd_ok(KH, KW, Cin, pad, stride, act, bias)) return launch_fwd_k7(a, s);   // the stems
  DRO_ACT_SWITCH(act, st = (launch_igemm<0, A_, 0>(a, P, static_cast<char*>(workspace), s)));
  return st;
}

extern "C" int dro_conv2d_strided_backward(const float* x, const float* weight, const float* dout, int B, int Hi,
                                           int Wi, int Cin, int Cout, int KH, int KW, int stride, int pad,
                                           float* grad_x, int grad_x_accumulate, float* grad_weight,
                                           float* grad_bias, int grad_weight_accumulate, void* workspace,
                                           size_t workspace_bytes, void* stream) {
  IgArgs a = {};
  int Ho, Wo;
  int st = strided_setup(a, x, B, Hi, Wi, Cin, Cout, KH, KW, stride, pad, Ho, Wo);
  if (st) return st;
  if (!weight || !dout || (grad_bias && !grad_weight)) {
    set_error("conv2d_strided_backward: NULL weight/dout, or grad_bias without grad_weight");
    return DRO_E_NULL;
  }
  if ((st = check_ws(workspace, workspace_bytes,
                     dro_conv2d_strided_workspace_bytes(B, Hi, Wi, Cin, Cout, KH, KW, stride, pad),
                     "conv2d_strided_backward")))
    return st;
  hipStream_t s = (hipStream_t)stream;
  char* ws = static_cast<char*>(workspace);
  a.weight = weight;
  a.G = dout;
  a.galpha = 1.f;
  if (grad_x) {
    // data gradient: GEMM columns = input pixels, staged operand = G (output size)
    IgArgs d = a;
    d.g.H = Hi;
    d.g.W = Wi;
    d.Hs = Ho;
    d.Ws = Wo;
    d.rows = Cin;
    d.kch = Cout;
    d.gsrc[0] = grad_x;
    d.gsrc_ctot[0] = Cin;
    d.gsrc_coff[0] = 0;
    d.gsrc_acc[0] = grad_x_accumulate ? 1 : 0;
    static const bool masked = env_int("DRO_STRIDED_MASKED", 0) != 0;   // A/B: the 4x-masked form
    if (stride == 2 && !masked) {
      // parity classes: grid.z = class, columns = that class's pixels (at most
      // ceil(Hi/2) x ceil(Wi/2) per image), K = its taps x Cout, split over
      // grid.y when the grid is short (partials + class-aware finish)
      const ClassPlan cp = plan_class_dgrad(B, Hi, Wi, Cin, Cout, KH, KW);
      d.pclass = 1;
      d.pcmax = cp.pcmax;
      d.kdiv = make_fdiv(Cout);
      d.K = Cout * KH * KW;
      d.row_tiles = cp.row_tiles;
      d.chunks_per_split = cp.chunks_per_split;
      d.part = cp.ksplit > 1 ? reinterpret_cast<float*>(ws) : nullptr;
      const dim3 grid((unsigned)(cp.row_tiles * cp.ptiles), (unsigned)cp.ksplit, 4);
      conv_logf(2.0 * Cin * Cout * KH * KW * (double)B * Ho * Wo, "igemm_kernel<%d, 1, 0, 0> parity classes", cp.bm);
      if (cp.bm == 64) hipLaunchKernelGGL((igemm_kernel<64, 1, 0, 0>), grid, dim3(256), 0, s, d);
      else hipLaunchKernelGGL((igemm_kernel<32, 1, 0, 0>), grid, dim3(256), 0, s, d);
      if ((st = launch_status("igemm_kernel (parity classes) launch failed"))) return st;
      if (cp.ksplit > 1) {
        // the finish indexes one split's [class][rows][pcmax] slab in 32 bits
        if (4LL * Cin * (long long)cp.pcmax >= (1LL << 31)) {
          set_error("conv2d_strided: data-gradient partial slab exceeds 32-bit indexing");
          return DRO_E_SHAPE;
        }
        const dim3 fgrid((unsigned)((cp.pcmax + 255) / 256), (unsigned)(4 * Cin));
        hipLaunchKernelGGL(igemm_class_finish_kernel, fgrid, dim3(256), 0, s, d, cp.ksplit);
        if ((st = launch_status("igemm_class_finish_kernel launch failed"))) return st;
      }
    } else if ((st = launch_igemm<1, 0, 0>(d, (long long)B * Hi * Wi, ws, s))) {
      return st;
    }
  }
  if (grad_weight) {
    const long long P = (long long)B * Ho * Wo;
    const int T = KH * KW;
    const WgPlan pl = plan_wgrad(Cin, Cout, T, P);
    a.gweight = grad_weight;
    a.gbias = grad_bias;
    a.wacc = grad_weight_accumulate ? 1 : 0;
    a.K = Cin * T;
    a.otiles = pl.otiles;
    a.pchunk = pl.pchunk;
    a.part = reinterpret_cast<float*>(
        ws + align256(std::max(plan_igemm_flat(Cin, Cout, KH, KW, B, Hi, Wi).part_bytes,
                               stride == 2 ? plan_class_dgrad(B, Hi, Wi, Cin, Cout, KH, KW).part_bytes : (size_t)0)));
    if (k7_ok(KH, KW, Cin, pad, stride)) return launch_wgrad_k7(a, stride, k7_splits(B, Ho, Wo), s);   // the stems
    conv_log("wgrad_kernel(", 2.0 * Cout * Cin * T * (double)P);
    hipLaunchKernelGGL(wgrad_kernel, dim3((unsigned)(pl.otiles * pl.ntiles), (unsigned)pl.splits), dim3(256), 0,
                       s, a);
    if ((st = launch_status("wgrad_kernel launch failed"))) return st;
    launch_wgrad_finish(a, pl.splits, s);
    if ((st = launch_status("wgrad_finish_kernel launch failed"))) return st;
  }
  return DRO_OK;
}

// ------------------------------------------------------------------ batched weight gradient (host)
// Split policy for a whole training step's uses of one weight: ~2 blocks per
// CU, at least 4 pixel tiles per split, at most 64 splits.
static WhPlan plan_wgrad_multi(int Cin, int Cout, int KH, int KW, int nuse, int B, int H, int W) {
  WhPlan pl = plan_wgrad_halo(Cin, Cout, KH, KW, B, H, W);
  if (!pl.ok) return pl;
  const int ntiles = nuse * B * pl.tiles_img;
  const int blocks = pl.otiles * pl.ctiles;
  static const int target = [] {   // tuning override: DRO_WHM_TARGET_BLOCKS (default 512)
    const char* e = getenv("DRO_WHM_TARGET_BLOCKS");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 512;
  }();
  static const int max_sp = [] {   // tuning override: DRO_WHM_MAX_SPLITS (default 64)
    const char* e = getenv("DRO_WHM_MAX_SPLITS");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 64;
  }();
  int sp = (target + blocks - 1) / blocks;
  if (sp > max_sp) sp = max_sp;
  if (sp > ntiles / 4) sp = ntiles / 4;
  if (sp < 1) sp = 1;
  pl.tiles_per_split = (ntiles + sp - 1) / sp;
  pl.splits = (ntiles + pl.tiles_per_split - 1) / pl.tiles_per_split;
  pl.part_bytes = align256((size_t)pl.splits * Cout * Cin * KH * KW * sizeof(float)) +
                  align256((size_t)pl.splits * Cout * sizeof(float));
  return pl;
}

extern "C" size_t dro_conv2d_weight_grad_multi_workspace_bytes(int nuse, int B, int H, int W, int Cin,
                                                              int Cout, int KH, int KW) {
  if (nuse < 1) nuse = 1;
  if (!wgrad_v1()) {
    const WhPlan t = plan_wgrad_halo(Cin, Cout, KH, KW, B, H, W);
    return plan_wgrad2(Cin, Cout, KH, KW, nuse * B * t.tiles_img, B, H, W).part_bytes;
  }
  return plan_wgrad_multi(Cin, Cout, KH, KW, nuse, B, H, W).part_bytes;
}

extern "C" int dro_conv2d_weight_grad_multi(const dro_wgrad_use* uses, int nuse, int nsrc, int B, int H,
                                            int W, int Cout, int KH, int KW, int act, float alpha,
                                            float* grad_weight, float* grad_bias, int accumulate,
                                            void* workspace, size_t workspace_bytes, void* stream) {
  if (!uses || !grad_weight) {
    set_error("conv2d_weight_grad_multi: NULL uses/grad_weight");
    return DRO_E_NULL;
  }
  if (nuse < 1 || nuse > kMaxUse) {
    set_error("conv2d_weight_grad_multi: need 1..16 uses per call");
    return DRO_E_SHAPE;
  }
  if (act < 0 || act > 3) {
    set_error("conv2d_weight_grad_multi: unknown activation");
    return DRO_E_MODE;
  }
  WgMulti m = {};
  int st;
  for (int u = 0; u < nuse; ++u) {
    IgArgs t = {};
    if ((st = conv_setup_geom(t, uses[u].srcs, nsrc, B, H, W, Cout, KH, KW))) return st;
    if (!uses[u].dout || (act != 0 && !uses[u].y)) {
      set_error("conv2d_weight_grad_multi: NULL dout (or y with an activation)");
      return DRO_E_NULL;
    }
    if (u == 0) {
      m.a = t;
    } else {
      for (int i = 0; i < kMaxSrc; ++i)
        if (t.cbase[i] != m.a.cbase[i]) {
          set_error("conv2d_weight_grad_multi: uses split the input channels differently");
          return DRO_E_SHAPE;
        }
    }
    for (int i = 0; i < kMaxSrc; ++i) m.usrc[u][i] = t.src[i];
    m.uG[u] = uses[u].dout;
    m.uy[u] = act ? uses[u].y : nullptr;
  }
  const int Cin = m.a.g.Cin, T = KH * KW;
  const bool v2 = !wgrad_v1();
  const int ntiles_all = nuse * B * plan_wgrad_halo(Cin, Cout, KH, KW, B, H, W).tiles_img;
  const WhPlan wh = v2 ? plan_wgrad2(Cin, Cout, KH, KW, ntiles_all, B, H, W)
                       : plan_wgrad_multi(Cin, Cout, KH, KW, nuse, B, H, W);
  if (!wh.ok) {
    set_error("conv2d_weight_grad_multi: kernel shape not supported (1x1, 1x5, 5x1, 3x3)");
    return DRO_E_SHAPE;
  }
  if ((st = check_ws(workspace, workspace_bytes, wh.part_bytes, "conv2d_weight_grad_multi"))) return st;
  IgArgs& a = m.a;
  a.G = uses[0].dout;
  a.gy = m.uy[0];
  a.galpha = alpha;
  a.gweight = grad_weight;
  a.gbias = grad_bias;
  a.wacc = accumulate ? 1 : 0;
  a.otiles = wh.otiles;
  a.tiles_x = wh.tiles_x;
  a.tiles_img = wh.tiles_img;
  a.chunks_per_split = wh.tiles_per_split;
  char* ws = static_cast<char*>(workspace);
  a.part = reinterpret_cast<float*>(ws);
  a.bpart = reinterpret_cast<float*>(ws + align256((size_t)wh.splits * Cout * Cin * T * sizeof(float)));
  m.nuse = nuse;
  m.use_tiles = B * wh.tiles_img;
  a.stamps = g_conv_stamps;
  a.dbg = 0;
  if (g_conv_stamps) {
    const char* e = getenv("DRO_CONV_DBG");
    a.dbg = e ? atoi(e) : 0;
  }
  hipStream_t s = (hipStream_t)stream;
  const int tgroups = v2 ? wh.tgroups : 1;
  const dim3 grid((unsigned)(wh.otiles * wh.ctiles * tgroups), (unsigned)wh.splits);
  if (v2)
    conv_logf(2.0 * Cout * Cin * T * (double)B * H * W * nuse, "wgrad2_kernel<%d, %d, %d, true, %d>", KH, KW,
              act, tgroups);
  else
    conv_logf(2.0 * Cout * Cin * T * (double)B * H * W * nuse, "wgrad_halo_kernel<%d, %d, %d, true>", KH, KW,
              act);
  if (v2) {
#define DRO_WG2M(KH_, KW_, TG_) DRO_ACT_SWITCH(act, hipLaunchKernelGGL((wgrad2_kernel<KH_, KW_, A_, true, TG_>), grid, dim3(512), 0, s, m))
    if (KH == 1 && KW == 1) { DRO_WG2M(1, 1, 1); }
    else if (KH == 1) { DRO_WG2M(1, 5, 1); }
    else if (KW == 1) { DRO_WG2M(5, 1, 1); }
    else if (tgroups == 3) { DRO_WG2M(3, 3, 3); }
    else { DRO_WG2M(3, 3, 1); }
#undef DRO_WG2M
  } else {
#define DRO_WHM(KH_, KW_) DRO_ACT_SWITCH(act, hipLaunchKernelGGL((wgrad_halo_kernel<KH_, KW_, A_, true>), grid, dim3(256), 0, s, m))
    if (KH == 1 && KW == 1) { DRO_WHM(1, 1); }
    else if (KH == 1) { DRO_WHM(1, 5); }
    else if (KW == 1) { DRO_WHM(5, 1); }
    else { DRO_WHM(3, 3); }
#undef DRO_WHM
  }
  if ((st = launch_status("wgrad_halo_kernel<multi> launch failed"))) return st;
  const long long total = (long long)Cout * Cin * T;
  long long blocks = (total + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (v2)
    launch_wgrad2_finish(a, wh.splits, s);
  else
    hipLaunchKernelGGL(wgrad_halo_finish_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, wh.splits);
  return launch_status("wgrad_halo_finish_kernel launch failed");
}

// ------------------------------------------------------------------ SepConvGRU elementwise backward
// update.py:67-70 (and :74-77): h' = (1-z) h + z q, q = tanh(.), z, r = sigmoid(.).
// Outputs are gradients w.r.t. the PRE-activations, ready for the conv backward:
// stage 1: dq~ = dh' z (1-q^2);  dz~ = dh' (q-h) z (1-z);  dh = dh' (1-z)
// stage 2 (after the q-gate backward, drh = dL/d(r*h)):  dr~ = drh h r (1-r);  dh += drh r
// z = zr[:, :hd], r = zr[:, hd:], dz~ / dr~ written into dzr likewise.
namespace dro {
// grid (pixel blocks over hd * HW, B): no 64-bit division per element
__global__ __launch_bounds__(256) void gru_elem_kernel(int stage, int hd, int HW,
                                                       const float* __restrict__ dhn,
                                                       const float* __restrict__ zr,
                                                       const float* __restrict__ q,
                                                       const float* __restrict__ h,
                                                       const float* __restrict__ drh,
                                                       float* __restrict__ dq,
                                                       float* __restrict__ dzr,
                                                       float* __restrict__ dh) {
  const int n = hd * HW;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const size_t b = blockIdx.y;
  const size_t i = b * n + j;
  const size_t zi = b * 2 * n + j, ri = zi + n;
  if (stage == 1) {
    const float gn = dhn[i], z = zr[zi], qv = q[i], hv = h[i];
    dq[i] = gn * z * (1.f - qv * qv);
    dzr[zi] = gn * (qv - hv) * z * (1.f - z);
    dh[i] = gn * (1.f - z);
  } else {
    const float d = drh[i], r = zr[ri];
    dzr[ri] = d * h[i] * r * (1.f - r);
    dh[i] += d * r;
  }
}
}  // namespace dro

extern "C" int dro_gru_backward_elem(int stage, int B, int hd, int H, int W, const float* dhn,
                                     const float* zr, const float* q, const float* h,
                                     const float* drh, float* dq, float* dzr, float* dh,
                                     void* stream) {
  if (B < 1 || hd < 1 || H < 1 || W < 1 || (stage != 1 && stage != 2)) {
    set_error("gru_backward_elem: bad sizes/stage");
    return DRO_E_SHAPE;
  }
  if (!zr || !h || !dzr || !dh || (stage == 1 && (!dhn || !q || !dq)) || (stage == 2 && !drh)) {
    set_error("gru_backward_elem: NULL pointer");
    return DRO_E_NULL;
  }
  if (B > 65535 || (long long)hd * H * W >= (1LL << 31)) {
    set_error("gru_backward_elem: sizes out of range");
    return DRO_E_SHAPE;
  }
  const int n = hd * H * W;
  hipLaunchKernelGGL(gru_elem_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)B), dim3(256), 0,
                     (hipStream_t)stream, stage, hd, H * W, dhn, zr, q, h, drh, dq, dzr, dh);
  return launch_status("gru_elem_kernel launch failed");
}
