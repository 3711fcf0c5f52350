// Implicit-GEMM convolutions on f32 MFMA (v_mfma_f32_32x32x2_f32) for the
// recurrent update blocks of the DRO optimizer (dro_sfm/networks/optim/
// update.py): SepConvGRU 1x5 / 5x1 gates, projection encoders, heads.
//
// Why not MIOpen: at these shapes (3840..7680 output pixels, 1..576 channels)
// every MIOpen call is a separate launch plus NCHW<->NHWC transposes, bias /
// activation / concat are separate ATen kernels, and its forward is not
// run-to-run deterministic.  Here:
//   * inputs are a VIRTUAL channel concatenation of up to 4 tensor slices (no
//     torch.cat), optionally with source 0 multiplied elementwise by another
//     slice (the GRU's r*h) while it is staged; a source may be a [B,C,1,1]
//     map broadcast over the image (the pose map);
//   * bias + activation (+ the GRU blend h' = (1-z)h + zq) run in the epilogue,
//     and the result lands in a channel slice of a bigger tensor;
//   * f32 MFMA is exact f32 (a k-ordered fmaf chain): no TF32-style loss;
//   * no atomics: split reductions go through a workspace and are summed in a
//     fixed order, so every result is bitwise run-to-run deterministic.
//
// GEMM view (forward): rows = output channels, cols = pixels (B*H*W flattened),
// K = (tap, input channel) flattened TAP-MAJOR (k = tap*Cin + c), 32-deep
// chunks.  Each K row of a chunk is staged by one wave, so its (tap, channel,
// source) decode is wave-uniform; lanes run along pixels (coalesced).
// Data gradient: the same kernel with rows = input channels, K = (tap, output
// channel), the tap offset negated and the weight read transposed.
// Weight gradient: rows = output channels, cols = (tap, input channel),
// K = pixels split over gridDim.y into per-split partials.
// Pipeline: global -> registers for chunk c+1 is issued before the MFMAs of
// chunk c (two LDS buffers, one barrier per chunk).  Tiles are remapped so
// that blocks sharing a pixel tile run on the same XCD (same L2).  Shapes with
// few output tiles and a long K split K over gridDim.y (partials + finish).
//
// Roofline: MFMA(f32) at 157 TF/s; FLOPs per launch = 2 * Cout * P * Cin * KH * KW.
#include <hip/hip_runtime.h>

#include "dro_common.hpp"

namespace dro {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kBN = 64;   // pixels per tile (forward / data gradient)
constexpr int kBK = 32;   // reduction chunk
constexpr int kMaxSrc = 4;

struct Slice {            // channels [coff, coff+C) of a [B, ctot, H, W] tensor
  const float* p;
  int C, ctot, coff;
  int bcast;              // 1: a [B, ctot, 1, 1] tensor broadcast over H x W
};

// exact n / d for 0 <= n < 2^16, 1 <= d < 2^12: (n * ceil(2^32/d)) >> 32
struct FastDiv {
  unsigned long long m;
};
__device__ __forceinline__ int fdiv(int n, FastDiv f) {
  return (int)(((unsigned long long)(unsigned)n * f.m) >> 32);
}

struct ConvGeom {
  int B, H, W, Cin, Cout, KH, KW, PH, PW;
};

struct IgArgs {
  ConvGeom g;
  Slice src[kMaxSrc];     // forward inputs (virtual concat)
  int cbase[kMaxSrc];     // first virtual channel of each source (Cin for unused)
  Slice scale0;           // optional multiplier of source 0 (p == nullptr: none)
  const float* weight;    // [Cout][Cin][KH][KW]
  const float* bias;      // [Cout] or nullptr
  float alpha;            // output scale (act none only)
  float* out;             // forward output slice base
  int out_ctot, out_coff;
  Slice z, h;             // GRU blend epilogue: out = (1-z) h + z q, q = tanh(acc+b)
  float* q_out;           // optional: q saved for the backward
  int q_ctot, q_coff;
  const float* G;         // [B, Cout, H, W] gradient w.r.t. the pre-activation
  float* gsrc[kMaxSrc];   // data-gradient targets per source (nullable)
  int gsrc_ctot[kMaxSrc], gsrc_coff[kMaxSrc], gsrc_acc[kMaxSrc];
  float* gweight;         // [Cout][Cin][KH][KW]
  float* gbias;           // [Cout]
  int rows;               // GEMM rows: Cout (forward) / Cin (data gradient)
  int kch;                // channels reduced per tap: Cin (forward) / Cout (data gradient)
  int K;                  // kch * KH * KW
  FastDiv kdiv, kwdiv, cindiv;
  int row_tiles;          // tile = pixel_tile * row_tiles + row_tile
  int chunks_per_split;   // split-K (gridDim.y > 1): partials to `part`
  float* part;            // [ksplit][rows][P] (igemm) / [splits][Cout][Cin*T] (wgrad)
  float* bpart;           // [splits][Cout] (wgrad bias)
  int otiles;             // weight gradient: output-channel tiles
  long long pchunk;       // weight gradient: pixels per split
};

__device__ __forceinline__ float act_fwd(float v, int act) {
  switch (act) {
    case 1: return fmaxf(v, 0.f);
    case 2: return 1.f / (1.f + expf(-v));
    case 3: return tanhf(v);
    default: return v;
  }
}

// d act / d pre, expressed through the saved activation output y
__device__ __forceinline__ float act_bwd(float y, int act) {
  switch (act) {
    case 1: return y > 0.f ? 1.f : 0.f;
    case 2: return y * (1.f - y);
    case 3: return 1.f - y * y;
    default: return 1.f;
  }
}

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// Blocks that share a pixel tile get consecutive logical ids on one XCD
// (hardware dispatch is round-robin over the 8 XCDs by block id).
__device__ __forceinline__ int xcd_remap(int id, int total) {
  const int xcd = id & 7, local = id >> 3, per = total >> 3, rem = total & 7;
  return (xcd < rem ? xcd * (per + 1) : rem * (per + 1) + (xcd - rem) * per) + local;
}

// one source's value (channel cl of slice s)
__device__ __forceinline__ float slice_val(const Slice& s, int cl, int b, size_t HW, size_t off) {
  const size_t ci = (size_t)b * s.ctot + s.coff + cl;
  return s.bcast ? s.p[ci] : s.p[ci * HW + off];
}

// virtual input at channel ch, image b, pixel offset off (caller checks
// padding).  One branch (and load) per source with constant indices: a
// select-then-load form gets rewritten into a dynamically indexed copy of the
// kernel arguments in scratch.
__device__ __forceinline__ float src_val(const IgArgs& a, int ch, int b, size_t HW, size_t off) {
  if (ch < a.cbase[1]) {
    float v = slice_val(a.src[0], ch, b, HW, off);
    if (a.scale0.p) v *= a.scale0.p[((size_t)b * a.scale0.ctot + a.scale0.coff + ch) * HW + off];
    return v;
  }
  if (ch < a.cbase[2]) return slice_val(a.src[1], ch - a.cbase[1], b, HW, off);
  if (ch < a.cbase[3]) return slice_val(a.src[2], ch - a.cbase[2], b, HW, off);
  return slice_val(a.src[3], ch - a.cbase[3], b, HW, off);
}

__device__ __forceinline__ void grad_put(float* dst, int ctot, int coff, int accf, int cl, int eb,
                                         size_t epix, size_t HW, float v) {
  if (!dst) return;
  float* q = dst + ((size_t)eb * ctot + coff + cl) * HW + epix;
  *q = accf ? (*q + v) : v;
}

// final value of GEMM element (row, pixel) -> destination
template <int MODE, int ACT, int EPI>
__device__ __forceinline__ void epi_store(const IgArgs& a, int row, int eb, size_t epix, size_t HW,
                                          float acc) {
  if (MODE == 0) {
    float v = acc + (a.bias ? a.bias[row] : 0.f);
    v = a.alpha * act_fwd(v, ACT);
    if (EPI == 1) {
      const float z = a.z.p[((size_t)eb * a.z.ctot + a.z.coff + row) * HW + epix];
      const float hv = a.h.p[((size_t)eb * a.h.ctot + a.h.coff + row) * HW + epix];
      if (a.q_out) a.q_out[((size_t)eb * a.q_ctot + a.q_coff + row) * HW + epix] = v;
      v = (1.f - z) * hv + z * v;
    }
    a.out[((size_t)eb * a.out_ctot + a.out_coff + row) * HW + epix] = v;
  } else {
    if (row < a.cbase[1]) grad_put(a.gsrc[0], a.gsrc_ctot[0], a.gsrc_coff[0], a.gsrc_acc[0], row, eb, epix, HW, acc);
    else if (row < a.cbase[2])
      grad_put(a.gsrc[1], a.gsrc_ctot[1], a.gsrc_coff[1], a.gsrc_acc[1], row - a.cbase[1], eb, epix, HW, acc);
    else if (row < a.cbase[3])
      grad_put(a.gsrc[2], a.gsrc_ctot[2], a.gsrc_coff[2], a.gsrc_acc[2], row - a.cbase[2], eb, epix, HW, acc);
    else
      grad_put(a.gsrc[3], a.gsrc_ctot[3], a.gsrc_coff[3], a.gsrc_acc[3], row - a.cbase[3], eb, epix, HW, acc);
  }
}

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
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int rt = tile % a.row_tiles, pt = tile / a.row_tiles;
  const int row0 = rt * BM;
  const long long p0 = (long long)pt * kBN;
  const size_t HW = (size_t)g.H * g.W;
  const long long P = (long long)g.B * HW;
  const int T = g.KH * g.KW;
  const int nchunks = (a.K + kBK - 1) / kBK;
  const int cbeg = blockIdx.y * a.chunks_per_split;
  const int cend = min(nchunks, cbeg + a.chunks_per_split);

  // staging roles: X column (pixel) fixed; W k-lane fixed
  const int col = tid & 63, krow = tid >> 6;
  const long long pg = p0 + col;
  const bool pv = pg < P;
  const int pb = pv ? (int)(pg / (long long)HW) : 0;
  const int prem = pv ? (int)(pg - (long long)pb * HW) : 0;
  const int py = prem / g.W, px = prem - py * g.W;
  const int wkl = tid & 31, wrow = tid >> 5;

  float xr[8], wv[BM / 8];
  auto load = [&](int chunk) {
    const int k0 = chunk * kBK;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = __builtin_amdgcn_readfirstlane(k0 + krow + 4 * i);
      float v = 0.f;
      if (k < a.K) {
        const int tap = fdiv(k, a.kdiv), ch = k - tap * a.kch;
        const int ty = fdiv(tap, a.kwdiv), dy = ty - g.PH, dx = tap - ty * g.KW - g.PW;
        const int yy = MODE == 0 ? py + dy : py - dy, xx = MODE == 0 ? px + dx : px - dx;
        if (pv && (unsigned)yy < (unsigned)g.H && (unsigned)xx < (unsigned)g.W) {
          const size_t off = (size_t)yy * g.W + xx;
          if (MODE == 0) v = src_val(a, ch, pb, HW, off);
          else v = a.G[((size_t)pb * g.Cout + ch) * HW + off];
        }
      }
      xr[i] = v;
    }
    const int k = k0 + wkl;
    const bool kv = k < a.K;
    const int tap = kv ? fdiv(k, a.kdiv) : 0, ch = k - tap * a.kch;
#pragma unroll
    for (int i = 0; i < BM / 8; ++i) {
      const int r = row0 + wrow + 8 * i;
      float v = 0.f;
      if (kv && r < a.rows)
        v = MODE == 0 ? a.weight[((size_t)r * g.Cin + ch) * T + tap]
                      : a.weight[((size_t)ch * g.Cin + r) * T + tap];
      wv[i] = v;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 8; ++i) Xs[buf][krow + 4 * i][col] = xr[i];
#pragma unroll
    for (int i = 0; i < BM / 8; ++i) Ws[buf][wkl][wrow + 8 * i] = wv[i];
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
  if (pe >= P) return;
  if (a.part) {   // split-K partial: [split][rows][P]
    float* dst = a.part + (size_t)blockIdx.y * a.rows * P + pe;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = row0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < a.rows) dst[(size_t)row * P] = acc[r];
    }
    return;
  }
  const int eb = (int)(pe / (long long)HW);
  const size_t epix = (size_t)(pe - (long long)eb * HW);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = row0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (row < a.rows) epi_store<MODE, ACT, EPI>(a, row, eb, epix, HW, acc[r]);
  }
}

// split-K finish: sum the partials in split order, then the epilogue
template <int MODE, int ACT, int EPI>
__global__ __launch_bounds__(256) void igemm_finish_kernel(IgArgs a, int ksplit) {
  const size_t HW = (size_t)a.g.H * a.g.W;
  const long long P = (long long)a.g.B * HW;
  const long long total = (long long)a.rows * P;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    float v = 0.f;
    for (int s = 0; s < ksplit; ++s) v += a.part[(size_t)s * total + i];
    const int row = (int)(i / P);
    const long long p = i - (long long)row * P;
    const int eb = (int)(p / (long long)HW);
    epi_store<MODE, ACT, EPI>(a, row, eb, (size_t)(p - (long long)eb * HW), HW, v);
  }
}

// ------------------------------------------------------------------ weight (+ bias) gradient
// dW[o, n] = sum_p G[o, p] * X[c(n), p + d(tap(n))] with n = tap*Cin + c:
// rows = o (64), cols = n (64), K = the pixels of split blockIdx.y (chunks of
// 32).  Writes per-split partials [split][Cout][Cin*T]; blocks of column tile
// 0 also write the bias partials sum_p G[o, p].
__global__ __launch_bounds__(256) void wgrad_kernel(IgArgs a) {
  __shared__ float Gs[2][kBK][64 + 1];
  __shared__ float Xs[2][kBK][64 + 1];
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int t = blockIdx.x;
  const int ot = t % a.otiles, nt = t / a.otiles;
  const int o0 = ot * 64, n0 = nt * 64;
  const int NK = a.K;     // Cin * T
  const size_t HW = (size_t)g.H * g.W;
  const long long P = (long long)g.B * HW;
  const long long pbeg = (long long)blockIdx.y * a.pchunk;
  const long long pend = pbeg + a.pchunk < P ? pbeg + a.pchunk : P;
  const bool do_bias = a.bpart && nt == 0;
  // staging: 32 lanes along pixels (coalesced), 8 row / column groups
  const int kp = tid & 31, hi = tid >> 5;
  int cdy[8], cdx[8], cch[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int n = n0 + hi + 8 * i;
    const int tap = n < NK ? fdiv(n, a.cindiv) : 0;
    const int ty = fdiv(tap, a.kwdiv);
    cch[i] = n < NK ? n - tap * g.Cin : -1;
    cdy[i] = ty - g.PH;
    cdx[i] = tap - ty * g.KW - g.PW;
  }
  float gr[8], xr[8], bsum[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) bsum[i] = 0.f;

  auto load = [&](long long q0) {
    const long long p = q0 + kp;
    const bool v = p < pend;
    const int b = v ? (int)(p / (long long)HW) : 0;
    const int pix = v ? (int)(p - (long long)b * HW) : 0;
    const int py = pix / g.W, px = pix - py * g.W;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int o = o0 + hi + 8 * i;
      gr[i] = (v && o < g.Cout) ? a.G[((size_t)b * g.Cout + o) * HW + pix] : 0.f;
      const int yy = py + cdy[i], xx = px + cdx[i];
      xr[i] = (v && cch[i] >= 0 && (unsigned)yy < (unsigned)g.H && (unsigned)xx < (unsigned)g.W)
                  ? src_val(a, cch[i], b, HW, (size_t)yy * g.W + xx) : 0.f;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      Gs[buf][kp][hi + 8 * i] = gr[i];
      Xs[buf][kp][hi + 8 * i] = xr[i];
      if (do_bias) bsum[i] += gr[i];
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
  for (long long q0 = pbeg; q0 < pend; q0 += kBK) {
    const bool more = q0 + kBK < pend;
    if (more) load(q0 + kBK);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int kk = s * 2 + (lane >> 5);
      acc = mfma32(Gs[buf][kk][wo * 32 + (lane & 31)], Xs[buf][kk][wc * 32 + (lane & 31)], acc);
    }
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  float* wp = a.part + (size_t)blockIdx.y * g.Cout * NK;
  const int n = n0 + wc * 32 + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int o = o0 + wo * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (o < g.Cout && n < NK) wp[(size_t)o * NK + n] = acc[r];
  }
  if (do_bias) {
    // lanes kp = 0..31 of each half-wave hold the same 8 output channels
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float v = bsum[i];
#pragma unroll
      for (int m = 16; m > 0; m >>= 1) v += __shfl_xor(v, m, 32);
      const int o = o0 + hi + 8 * i;
      if (kp == 0 && o < g.Cout) a.bpart[(size_t)blockIdx.y * g.Cout + o] = v;
    }
  }
}

// dW[o][c][tap] = sum_s part[s][o][tap*Cin + c]; db[o] = sum_s bpart[s][o]
__global__ __launch_bounds__(256) void wgrad_finish_kernel(IgArgs a, int splits) {
  const ConvGeom& g = a.g;
  const int T = g.KH * g.KW, NK = a.K;
  const long long total = (long long)g.Cout * NK;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    const int o = (int)(e / NK), rem = (int)(e - (long long)o * NK);
    const int c = rem / T, tap = rem - c * T;
    const size_t src = (size_t)o * NK + (size_t)tap * g.Cin + c;
    float v = 0.f;
    for (int s = 0; s < splits; ++s) v += a.part[(size_t)s * total + src];
    a.gweight[e] = v;
    if (a.gbias && e < g.Cout) {
      float bv = 0.f;
      for (int s = 0; s < splits; ++s) bv += a.bpart[(size_t)s * g.Cout + e];
      a.gbias[e] = bv;
    }
  }
}

// G = alpha * dout * act'(y) (only when act != none or alpha != 1)
__global__ __launch_bounds__(256) void grad_pre_kernel(int act, float alpha, int Cout, size_t HW,
                                                       size_t total, const float* __restrict__ dout,
                                                       Slice y, float* __restrict__ G) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    float d = alpha * dout[i];
    if (act) {
      const size_t b = i / ((size_t)Cout * HW), rem = i - b * Cout * HW;
      const size_t o = rem / HW, pix = rem - o * HW;
      d *= act_bwd(y.p[(b * y.ctot + y.coff + o) * HW + pix], act);
    }
    G[i] = d;
  }
}

}  // namespace dro

using namespace dro;

namespace {

FastDiv make_fdiv(int d) {
  FastDiv f;
  f.m = ((1ULL << 32) + (unsigned long long)d - 1) / (unsigned long long)d;
  return f;
}

size_t align256(size_t n) { return (n + 255) & ~(size_t)255; }

// ---- launch plans (shared by the workspace query and the launches)
struct IgPlan {
  int bm, row_tiles, ptiles, ksplit, chunks_per_split;
  size_t part_bytes;
};

IgPlan plan_igemm(int rows, int kch, int T, long long P) {
  IgPlan pl;
  pl.ptiles = (int)((P + kBN - 1) / kBN);
  const int t64 = (rows + 63) / 64;
  pl.bm = (long long)t64 * pl.ptiles >= 448 ? 64 : 32;
  pl.row_tiles = (rows + pl.bm - 1) / pl.bm;
  const int nchunks = (kch * T + kBK - 1) / kBK;
  const long long blocks = (long long)pl.row_tiles * pl.ptiles;
  int ks = 1;
  if (blocks < 240) {   // under one block per CU: split K, >= 4 chunks per split
    ks = (int)((480 + blocks - 1) / blocks);
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
  size_t part_bytes, bpart_bytes;
};

WgPlan plan_wgrad(int Cin, int Cout, int T, long long P) {
  WgPlan pl;
  pl.otiles = (Cout + 63) / 64;
  pl.ntiles = (Cin * T + 63) / 64;
  const long long tiles = (long long)pl.otiles * pl.ntiles;
  long long splits = (640 + tiles - 1) / tiles;
  const long long maxs = (P + 4 * kBK - 1) / (4 * kBK);   // >= 4 chunks per split
  if (splits > maxs) splits = maxs;
  if (splits > 64) splits = 64;
  if (splits < 1) splits = 1;
  pl.pchunk = ((P + splits - 1) / splits + kBK - 1) / kBK * kBK;
  pl.splits = (int)((P + pl.pchunk - 1) / pl.pchunk);
  pl.part_bytes = align256((size_t)pl.splits * Cout * Cin * T * sizeof(float));
  pl.bpart_bytes = align256((size_t)pl.splits * Cout * sizeof(float));
  return pl;
}

size_t fwd_workspace(int B, int H, int W, int Cin, int Cout, int KH, int KW) {
  return plan_igemm(Cout, Cin, KH * KW, (long long)B * H * W).part_bytes;
}

size_t bwd_workspace(int B, int H, int W, int Cin, int Cout, int KH, int KW) {
  const long long P = (long long)B * H * W;
  const int T = KH * KW;
  const WgPlan wp = plan_wgrad(Cin, Cout, T, P);
  return align256((size_t)Cout * P * sizeof(float)) +              // pre-activation gradient
         plan_igemm(Cin, Cout, T, P).part_bytes +                   // data-gradient split-K
         wp.part_bytes + wp.bpart_bytes;                            // weight-gradient partials
}

int conv_setup_geom(IgArgs& a, const dro_slice* srcs, int nsrc, int B, int H, int W, int Cout, int KH,
                    int KW) {
  ConvGeom& g = a.g;
  if (!srcs || nsrc < 1 || nsrc > kMaxSrc) {
    set_error("conv2d: need 1..4 input slices");
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
    cin += srcs[i].channels;
  }
  if (B < 1 || H < 1 || W < 1 || Cout < 1 || KH < 1 || KW < 1 || (KH % 2) == 0 || (KW % 2) == 0 ||
      (long long)B * H * W > (1LL << 30) || cin >= 4096 || Cout >= 4096 ||
      (long long)cin * KH * KW >= 65536 || (long long)Cout * KH * KW >= 65536) {
    set_error("conv2d: sizes out of range (odd kernels, stride 1, C*KH*KW < 65536, C < 4096)");
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

// rows / kch set by the caller; `ws` must hold plan.part_bytes
template <int MODE, int ACT, int EPI>
int launch_igemm(IgArgs& a, long long P, char* ws, hipStream_t s) {
  const IgPlan pl = plan_igemm(a.rows, a.kch, a.g.KH * a.g.KW, P);
  a.K = a.kch * a.g.KH * a.g.KW;
  a.kdiv = make_fdiv(a.kch);
  a.row_tiles = pl.row_tiles;
  a.chunks_per_split = pl.chunks_per_split;
  a.part = pl.ksplit > 1 ? reinterpret_cast<float*>(ws) : nullptr;
  const dim3 grid(pl.row_tiles * pl.ptiles, pl.ksplit);
  if (pl.bm == 64)
    hipLaunchKernelGGL((igemm_kernel<64, MODE, ACT, EPI>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((igemm_kernel<32, MODE, ACT, EPI>), grid, dim3(256), 0, s, a);
  int st = launch_status("igemm_kernel launch failed");
  if (st || pl.ksplit == 1) return st;
  const long long total = (long long)a.rows * P;
  long long blocks = (total + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL((igemm_finish_kernel<MODE, ACT, EPI>), dim3((unsigned)blocks), dim3(256), 0, s, a,
                     pl.ksplit);
  return launch_status("igemm_finish_kernel launch failed");
}

int check_ws(size_t have, size_t need, const char* what) {
  if (have < need) {
    static thread_local char msg[160];
    snprintf(msg, sizeof(msg), "%s: workspace of %zu bytes is smaller than the %zu required "
             "(dro_conv2d_workspace_bytes)", what, have, need);
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

extern "C" size_t dro_conv2d_workspace_bytes(int B, int H, int W, int Cin, int Cout, int KH, int KW) {
  if (B < 1 || H < 1 || W < 1 || Cin < 1 || Cout < 1 || KH < 1 || KW < 1) return 0;
  const size_t f = fwd_workspace(B, H, W, Cin, Cout, KH, KW);
  const size_t b = bwd_workspace(B, H, W, Cin, Cout, KH, KW);
  return f > b ? f : b;
}

extern "C" int dro_conv2d_forward(const dro_slice* srcs, int nsrc, const dro_slice* scale0,
                                  const float* weight, const float* bias, int B, int H, int W,
                                  int Cout, int KH, int KW, int act, float alpha, float* out,
                                  int out_ctot, int out_coff, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  IgArgs a = {};
  int st = conv_setup_geom(a, srcs, nsrc, B, H, W, Cout, KH, KW);
  if (st) return st;
  if (!weight || !out || out_coff < 0 || out_coff + Cout > out_ctot) {
    set_error("conv2d_forward: NULL weight/out or bad output slice");
    return DRO_E_NULL;
  }
  if (alpha != 1.f && act != 0) {
    set_error("conv2d_forward: alpha != 1 requires act none");
    return DRO_E_MODE;
  }
  if ((st = check_ws(workspace ? workspace_bytes : 0, fwd_workspace(B, H, W, a.g.Cin, Cout, KH, KW),
                     "conv2d_forward")))
    return st;
  a.scale0 = to_slice(scale0);
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

extern "C" int dro_convgru_blend_forward(const dro_slice* srcs, int nsrc, const dro_slice* scale0,
                                         const float* weight, const float* bias, int B, int H,
                                         int W, int Cout, int KH, int KW, const dro_slice* z,
                                         const dro_slice* h, float* q_out, int q_ctot, int q_coff,
                                         float* out, int out_ctot, int out_coff, void* workspace,
                                         size_t workspace_bytes, void* stream) {
  IgArgs a = {};
  int st = conv_setup_geom(a, srcs, nsrc, B, H, W, Cout, KH, KW);
  if (st) return st;
  if (!weight || !out || !z || !h || !z->data || !h->data) {
    set_error("convgru_blend_forward: NULL weight/out/z/h");
    return DRO_E_NULL;
  }
  if ((st = check_ws(workspace ? workspace_bytes : 0, fwd_workspace(B, H, W, a.g.Cin, Cout, KH, KW),
                     "convgru_blend_forward")))
    return st;
  a.scale0 = to_slice(scale0);
  a.weight = weight;
  a.bias = bias;
  a.alpha = 1.f;
  a.out = out;
  a.out_ctot = out_ctot;
  a.out_coff = out_coff;
  a.z = to_slice(z);
  a.h = to_slice(h);
  a.q_out = q_out;
  a.q_ctot = q_ctot;
  a.q_coff = q_coff;
  a.rows = Cout;
  a.kch = a.g.Cin;
  return launch_igemm<0, 3, 1>(a, (long long)B * H * W, static_cast<char*>(workspace),
                               (hipStream_t)stream);
}

extern "C" int dro_conv2d_backward(const dro_slice* srcs, int nsrc, const dro_slice* scale0,
                                   const float* weight, int B, int H, int W, int Cout, int KH,
                                   int KW, int act, float alpha, const dro_slice* y,
                                   const float* dout, float* const* grad_srcs,
                                   const int* grad_ctot, const int* grad_coff,
                                   const int* grad_accumulate, float* grad_weight,
                                   float* grad_bias, void* workspace, size_t workspace_bytes,
                                   void* stream) {
  IgArgs a = {};
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
  if ((st = check_ws(workspace ? workspace_bytes : 0, bwd_workspace(B, H, W, a.g.Cin, Cout, KH, KW),
                     "conv2d_backward")))
    return st;
  for (int i = 0; i < nsrc; ++i) {
    a.gsrc[i] = grad_srcs ? grad_srcs[i] : nullptr;
    a.gsrc_ctot[i] = grad_ctot ? grad_ctot[i] : srcs[i].channels;
    a.gsrc_coff[i] = grad_coff ? grad_coff[i] : 0;
    a.gsrc_acc[i] = grad_accumulate ? grad_accumulate[i] : 0;
  }
  a.scale0 = to_slice(scale0);
  a.weight = weight;
  a.gweight = grad_weight;
  a.gbias = grad_bias;
  hipStream_t s = (hipStream_t)stream;
  const size_t HW = (size_t)H * W;
  const long long P = (long long)B * HW;
  const int T = KH * KW;
  char* ws = static_cast<char*>(workspace);
  char* ws_pre = ws;
  char* ws_ig = ws_pre + align256((size_t)Cout * P * sizeof(float));
  char* ws_wg = ws_ig + plan_igemm(a.g.Cin, Cout, T, P).part_bytes;
  if (pre) {
    const size_t total = (size_t)Cout * P;
    size_t blocks = (total + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    float* G = reinterpret_cast<float*>(ws_pre);
    hipLaunchKernelGGL(grad_pre_kernel, dim3((unsigned)blocks), dim3(256), 0, s, act, alpha, Cout, HW,
                       total, dout, to_slice(y), G);
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
    if ((st = launch_igemm<1, 0, 0>(a, P, ws_ig, s))) return st;
  }
  if (grad_weight) {
    const WgPlan pl = plan_wgrad(a.g.Cin, Cout, T, P);
    a.K = a.g.Cin * T;
    a.otiles = pl.otiles;
    a.pchunk = pl.pchunk;
    a.part = reinterpret_cast<float*>(ws_wg);
    a.bpart = grad_bias ? reinterpret_cast<float*>(ws_wg + pl.part_bytes) : nullptr;
    hipLaunchKernelGGL(wgrad_kernel, dim3((unsigned)(pl.otiles * pl.ntiles), (unsigned)pl.splits),
                       dim3(256), 0, s, a);
    if ((st = launch_status("wgrad_kernel launch failed"))) return st;
    const long long total = (long long)Cout * a.K;
    long long blocks = (total + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(wgrad_finish_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, pl.splits);
    if ((st = launch_status("wgrad_finish_kernel launch failed"))) return st;
  }
  return DRO_OK;
}

// ------------------------------------------------------------------ SepConvGRU elementwise backward
// update.py:67-70 (and :74-77): h' = (1-z) h + z q, q = tanh(.), z, r = sigmoid(.).
// Outputs are gradients w.r.t. the PRE-activations, ready for the conv backward:
// stage 1: dq~ = dh' z (1-q^2);  dz~ = dh' (q-h) z (1-z);  dh = dh' (1-z)
// stage 2 (after the q-gate backward, drh = dL/d(r*h)):  dr~ = drh h r (1-r);  dh += drh r
// z = zr[:, :hd], r = zr[:, hd:], dz~ / dr~ written into dzr likewise.
namespace dro {
__global__ __launch_bounds__(256) void gru_elem_kernel(int stage, int hd, size_t HW, size_t total,
                                                       const float* __restrict__ dhn,
                                                       const float* __restrict__ zr,
                                                       const float* __restrict__ q,
                                                       const float* __restrict__ h,
                                                       const float* __restrict__ drh,
                                                       float* __restrict__ dq,
                                                       float* __restrict__ dzr,
                                                       float* __restrict__ dh) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const size_t b = i / ((size_t)hd * HW), rem = i - b * hd * HW;
    const size_t zi = b * 2 * hd * HW + rem, ri = zi + (size_t)hd * HW;
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
  const size_t HW = (size_t)H * W, total = (size_t)B * hd * HW;
  size_t blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(gru_elem_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     stage, hd, HW, total, dhn, zr, q, h, drh, dq, dzr, dh);
  return launch_status("gru_elem_kernel launch failed");
}
