// Shared definitions of the convolution engines (conv.hip: f32 MFMA;
// xconv.hip: split-bf16 MFMA): launch arguments, virtual-concat source
// descriptors, activation helpers, the epilogue and the split-K finish.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

#include "dro_common.hpp"

namespace dro {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kBN = 64;   // pixels per tile (forward / data gradient)
constexpr int kBK = 32;   // reduction chunk (forward / data gradient)
constexpr int kWP = 64;   // pixels per weight-gradient chunk
constexpr int kMaxSrc = 4;

struct Slice {            // channels [coff, coff+C) of a [B, ctot, H, W] tensor
  const float* p;
  int C, ctot, coff;
  int bcast;              // 1: a [B, ctot, 1, 1] tensor broadcast over H x W
};

// exact n / d for 0 <= n < 2^16, 1 <= d < 2^12: umulhi(n, ceil(2^32/d)), d = 1 apart
struct FastDiv {
  unsigned m;
  int one;
};
__device__ __forceinline__ int fdiv(int n, FastDiv f) {
  return f.one ? n : (int)__umulhi((unsigned)n, f.m);
}

// exact n / d for any 32-bit n, d >= 1: m = floor((2^32 - 1) / d) leaves the
// mulhi estimate at most 2 low (host-computed; a few scalar ops per division)
struct Div32 {
  unsigned m, d;
};
__device__ __forceinline__ unsigned udiv(unsigned n, Div32 f) {
  unsigned q = __umulhi(n, f.m);
  unsigned r = n - q * f.d;
  if (r >= f.d) {
    ++q;
    r -= f.d;
  }
  if (r >= f.d) ++q;
  return q;
}

struct ConvGeom {
  int B, H, W, Cin, Cout, KH, KW, PH, PW;
};

// Training-mode BatchNorm fused into the halo conv (3x3, stride 1) of the
// ResNet-18 encoders: conv -> BN [+ skip] -> ReLU -> conv (batchnorm.hip's
// arithmetic, fixed-order fp64 statistics).
//   EPI 5 (forward): the conv's output z is the BN input; the epilogue writes
//     per-(pixel tile, channel) partial sums of z and z^2, and the last block
//     to finish folds them (two fixed-order levels, self-resetting counters)
//     into mean / invstd, the running statistics and xcoef-style coefficients
//     `coef` = [k = gamma * invstd | mean | beta] per channel.
//   EPI 6 (data gradient): the conv's data gradient dy is the gradient of the
//     BN's ReLU output y; the epilogue writes g = dy [y > 0] and the partial
//     sums of g and g * xhat (xhat from z, mean, invstd), folded as above into
//     `coef` = [mean(g) | mean(g xhat)] and dgamma / dbeta.
//   XF 1 / 2 (forward staging): the source read is z, staged as
//     relu(fmaf(z - mean, k, beta) [+ skip]) from `xcoef`; the block that owns
//     a pixel (row tile 0, the pixel inside its tile) stores that value to
//     `yout` -- the BN output is materialised by its consumer, not by a launch.
//   XF 3 (data-gradient staging): the gradient read is g, staged as
//     dz = k (g - mean(g) - xhat mean(g xhat)) from `xcoef` = [k | mean(g) |
//     mean(g xhat) | mean | invstd] and z; owners store dz to `yout` (the
//     weight gradient's input).
// Sources / gradients / skip / yout / z / y are dense [B, C, H, W] tensors.
struct BnFuse {
  double2* part;          // [ptiles][C]
  double2* part2;         // [ngroups][C]
  unsigned* cnt;          // [row_tiles][ngroups] level-1 counters, then [row_tiles] level-2
  int g1, ngroups;        // pixel tiles per level-1 group, groups
  const float* gamma;     // nullable (1)
  const float* beta;      // nullable (0)
  float* rmean;           // nullable (no running statistics)
  float* rvar;
  long long* nbt;         // nullable
  float eps, momentum;
  float* save_mean;       // EPI 5 outputs
  float* save_invstd;
  float* coef;            // EPI 5: [3][C]; EPI 6: [2][C]
  const float* y;         // EPI 6: the BN's ReLU output (mask)
  const float* z;         // EPI 6 / XF 3: the BN input
  const float* mean;      // EPI 6: saved mean / invstd
  const float* invstd;
  float* dgamma;          // EPI 6 outputs (nullable)
  float* dbeta;
  const float* xcoef;     // XF: coefficients of the staged source's BN
  const float* skip;      // XF 2
  float* yout;            // XF: owner stores of the transformed source
  int inkernel;           // 1: the last block folds the partials (bn_finish), else bn_finalize_kernel
  int dbg;                // timing ablations (env DRO_BN_ABLATE, results invalid): 1 no arrival /
                          // fold, 2 no partial stores, 4 no row sums
};

struct IgArgs {
  ConvGeom g;
  Slice src[kMaxSrc];     // forward inputs (virtual concat); read by index from the kernarg segment
  int cbase[kMaxSrc];     // first virtual channel of each source (Cin for unused)
  const float* weight;    // [Cout][Cin][KH][KW]
  const float* bias;      // [Cout] or nullptr
  float alpha;            // output scale (act none only)
  float* out;             // forward output slice base
  int out_ctot, out_coff;
  Slice z, h;             // EPI 1: out = (1-z) h + z q, q = tanh(acc + b); EPI 2: h for r*h
                          // MODE 1 EPI 3: z = the r gate (zr channels hd..2hd), h = the state
  float* aux;             // EPI 1: q (saved for the backward); EPI 2: r*h  (dense, [B, hd, H, W]);
                          // MODE 1 EPI 3: dzr (its r half is written)
  int hd;                 // EPI 2: rows >= hd are the r gate
  // MODE 1 EPI 4 (the gate conv's data gradient of a SepConvGRU's second half
  // runs the FIRST half's stage 1 on its finished d h): z = that half's zr (z
  // channels 0..hd), h = its input state, aux = its dzr; q, dq, dh below
  const float* g1q;
  float* g1dq;
  float* g1dh;
  int g1acc;              // 1: g1dh is added into (a gradient sink already written)
  const float* G;         // [B, Cout, H, W] gradient w.r.t. the pre-activation (or w.r.t. the
                          // output when folded: then G_pre = galpha * G * act'(gy))
  const float* gy;        // folded activation: saved output y, dense [B, Cout, H, W]
  float galpha;           // folded output scale
  float* gsrc[kMaxSrc];   // data-gradient targets per source (nullable)
  int gsrc_ctot[kMaxSrc], gsrc_coff[kMaxSrc], gsrc_acc[kMaxSrc];
  float* gweight;         // [Cout][Cin][KH][KW]
  float* gbias;           // [Cout]
  int wacc;               // 1: add into gweight / gbias instead of overwriting
  int rows;               // GEMM rows: Cout (forward) / Cin (data gradient)
  int kch;                // channels reduced per tap: Cin (forward) / Cout (data gradient)
  int K;                  // kch * KH * KW
  FastDiv kdiv, kwdiv, cindiv;
  int row_tiles;          // tile = pixel_tile * row_tiles + row_tile
  int chunks_per_split;   // split-K (gridDim.y > 1): partials to `part`
  float* part;            // [ksplit][rows][P] (igemm) / [splits][Cout][NK+1] (wgrad)
  float* bpart;           // [splits][Cout] bias partials (halo weight gradient)
  int otiles;             // weight gradient: output-channel tiles
  long long pchunk;       // weight gradient: pixels per split
  // halo-tiled direct convolution (KH*KW > 1): TH x TW pixel tiles, the input
  // tile + halo staged once per channel chunk of CK channels
  int TH, TW, HWd, HPAD, tiles_x, tiles_img, CK;
  Div32 rt_div, ti_div, tx_div;  // halo kernel: row_tiles, tiles_img, tiles_x
  // halo forward: source s channel ch of image b starts at byte address
  // sq0[s] + b * sqb[s] + ch * sr[s]; sm[s] = 0 for broadcast sources, else ~0
  unsigned long long sq0[kMaxSrc], sqb[kMaxSrc];
  unsigned sr[kMaxSrc], sm[kMaxSrc];
  // split-bf16 engine (xconv.hip): weights pre-split into 3 bf16 planes
  // (dro_weight_split), [plane][row][K] with K = (32-channel chunk, tap, channel)
  const char* wsplit;           // nullptr: the f32 engine runs
  unsigned long long wplane;    // bytes per plane
  unsigned wrow;                // bytes per row (chunks * T * 64)
  // strided convolutions (flattened implicit GEMM and generic weight gradient
  // only): the staged operand's spatial size (input for the forward and the
  // weight gradient, the output gradient for the data gradient), log2 stride
  int Hs, Ws, sshift;
  int flat_only;                // 1: the flattened implicit GEMM (no halo / thin / split-bf16 paths)
  int pclass;                   // igemm data gradient, stride 2: output pixels by parity class
                                // (blockIdx.z = 2 * (y & 1) + (x & 1)), only that class's taps
  long long pcmax;              // parity classes: pixels of the largest class (partials' row stride)
  unsigned long long* stamps;   // diagnostics (dro_debug_conv_stamps): [block][16] s_memtime
  int dbg;                      // diagnostics with stamps on (env DRO_CONV_DBG): 1 skip the K
                                // loop's loads, 2 its MFMAs, 4 its LDS stores (results invalid)
  BnFuse bn;                    // EPI 5 / 6 and the XF staging transforms (halo kernel only)
};

// The K-loop ablations exist only in a diagnostic build (-DDRO_CONV_ABLATE=1,
// for tools/conv_stamps.py and tools/wgrad_stamps.py): in the product build
// the flags fold to 0.  A runtime ablation branch cost the weight-gradient
// kernel its full unroll (1x5 multi-use launch 123 -> 176 us).
#ifndef DRO_CONV_ABLATE
#define DRO_CONV_ABLATE 0
#endif
__device__ __forceinline__ int ablation_flags(int dbg) { return DRO_CONV_ABLATE ? dbg : 0; }

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

// The source descriptors are read straight from the kernel-argument segment
// with a computed index (s_load for a wave-uniform channel).  Selecting among
// struct fields instead gets rewritten by the compiler into a dynamically
// indexed copy of the arguments in scratch.
typedef __attribute__((address_space(4))) const Slice* KSlice;

__device__ __forceinline__ KSlice kernarg_srcs() {
  return (KSlice)((__attribute__((address_space(4))) const char*)__builtin_amdgcn_kernarg_segment_ptr() +
                  offsetof(IgArgs, src));
}

// Element offset of virtual channel ch in its source is b * A + Bc + (M ? pixel : 0)
// (broadcast sources: A = ctot, M = 0).  32-bit element offsets (checked on the host).
struct RowDesc {
  const float* p;
  unsigned A, Bc;
  bool M;
};

__device__ __forceinline__ RowDesc row_desc_at(KSlice base, int cb1, int cb2, int cb3, int ch,
                                               unsigned HW) {
  const int si = (ch >= cb1) + (ch >= cb2) + (ch >= cb3);
  const KSlice ks = base + si;
  const int cl = ch - (si == 0 ? 0 : si == 1 ? cb1 : si == 2 ? cb2 : cb3);
  const int ctot = ks->ctot, coff = ks->coff, bc = ks->bcast;
  RowDesc d;
  d.p = ks->p;
  d.A = bc ? (unsigned)ctot : (unsigned)ctot * HW;
  d.Bc = bc ? (unsigned)(coff + cl) : (unsigned)(coff + cl) * HW;
  d.M = !bc;
  return d;
}

__device__ __forceinline__ RowDesc row_desc(int cb1, int cb2, int cb3, int ch, unsigned HW) {
  return row_desc_at(kernarg_srcs(), cb1, cb2, cb3, ch, HW);
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
      a.aux[((size_t)eb * a.rows + row) * HW + epix] = v;
      v = (1.f - z) * hv + z * v;
    }
    if (EPI == 2 && row >= a.hd) {
      const int c = row - a.hd;
      const float hv = a.h.p[((size_t)eb * a.h.ctot + a.h.coff + c) * HW + epix];
      a.aux[((size_t)eb * a.hd + c) * HW + epix] = v * hv;
    }
    a.out[((size_t)eb * a.out_ctot + a.out_coff + row) * HW + epix] = v;
  } else {
    if (EPI == 4 && row < a.cbase[1]) {   // finished d h -> the first half's stage 1 (gru_elem_kernel)
      float* q = a.gsrc[0] + ((size_t)eb * a.gsrc_ctot[0] + a.gsrc_coff[0] + row) * HW + epix;
      const float gn = *q + acc;
      *q = gn;
      const size_t zi = ((size_t)eb * a.z.ctot + a.z.coff + row) * HW + epix;
      const size_t i1 = ((size_t)eb * a.hd + row) * HW + epix;
      const float z = a.z.p[zi], qv = a.g1q[i1], hv = a.h.p[((size_t)eb * a.h.ctot + a.h.coff + row) * HW + epix];
      a.g1dq[i1] = gn * z * (1.f - qv * qv);
      a.aux[zi] = gn * (qv - hv) * z * (1.f - z);
      a.g1dh[i1] = a.g1acc ? a.g1dh[i1] + gn * (1.f - z) : gn * (1.f - z);
    } else if (EPI == 3 && row < a.cbase[1]) {   // SepConvGRU stage 2 on d(r*h) (gru_elem_kernel)
      const size_t zi = ((size_t)eb * a.z.ctot + a.z.coff + row) * HW + epix;
      const size_t hi = ((size_t)eb * a.h.ctot + a.h.coff + row) * HW + epix;
      const float r = a.z.p[zi];
      a.aux[zi] = acc * a.h.p[hi] * r * (1.f - r);
      float* q = a.gsrc[0] + ((size_t)eb * a.gsrc_ctot[0] + a.gsrc_coff[0] + row) * HW + epix;
      *q += acc * r;
    } else if (row < a.cbase[1])
      grad_put(a.gsrc[0], a.gsrc_ctot[0], a.gsrc_coff[0], a.gsrc_acc[0], row, eb, epix, HW, acc);
    else if (row < a.cbase[2])
      grad_put(a.gsrc[1], a.gsrc_ctot[1], a.gsrc_coff[1], a.gsrc_acc[1], row - a.cbase[1], eb, epix, HW, acc);
    else if (row < a.cbase[3])
      grad_put(a.gsrc[2], a.gsrc_ctot[2], a.gsrc_coff[2], a.gsrc_acc[2], row - a.cbase[2], eb, epix, HW, acc);
    else
      grad_put(a.gsrc[3], a.gsrc_ctot[3], a.gsrc_coff[3], a.gsrc_acc[3], row - a.cbase[3], eb, epix, HW, acc);
  }
}

// Epilogue of one 32x32 MFMA accumulator (16 rows per lane, row(r) = rbase +
// (r & 3) + 8 (r >> 2)) at pixel (eb, epix): every operand the 16 rows need
// (bias, z and h of the GRU epilogues, the old value of an accumulated
// gradient) is loaded before the first is used -- one memory round trip for
// the tile instead of one per row (measured: the per-row form spent longer
// in the epilogue than in the whole K loop).
template <int MODE, int ACT, int EPI>
__device__ __forceinline__ void epi_tile(const IgArgs& a, const f32x16& acc, int rbase, int eb,
                                         size_t epix, size_t HW) {
  const int rows = a.rows;
  if (MODE == 0) {
    float bv[16], zv[EPI == 1 ? 16 : 1], hv[EPI != 0 ? 16 : 1];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = rbase + (r & 3) + 8 * (r >> 2);
      const int rr = row < rows ? row : 0;
      bv[r] = a.bias ? a.bias[rr] : 0.f;
      if (EPI == 1) {
        zv[r] = a.z.p[((size_t)eb * a.z.ctot + a.z.coff + rr) * HW + epix];
        hv[r] = a.h.p[((size_t)eb * a.h.ctot + a.h.coff + rr) * HW + epix];
      }
      if (EPI == 2) {
        const int c = rr >= a.hd ? rr - a.hd : 0;
        hv[r] = a.h.p[((size_t)eb * a.h.ctot + a.h.coff + c) * HW + epix];
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = rbase + (r & 3) + 8 * (r >> 2);
      if (row >= rows) continue;
      float v = acc[r] + bv[r];
      v = a.alpha * act_fwd(v, ACT);
      if (EPI == 1) {
        a.aux[((size_t)eb * a.rows + row) * HW + epix] = v;
        v = (1.f - zv[r]) * hv[r] + zv[r] * v;
      }
      if (EPI == 2 && row >= a.hd)
        a.aux[((size_t)eb * a.hd + (row - a.hd)) * HW + epix] = v * hv[r];
      a.out[((size_t)eb * a.out_ctot + a.out_coff + row) * HW + epix] = v;
    }
  } else {
    float* dst[16];
    bool accf[16];
    float old[16];
    // MODE 1 EPI 3 (SepConvGRU stage 2 folded into the candidate conv's data
    // gradient): rows of source 0 are d(r*h); they write dr~ = d h r (1-r) into
    // dzr's r half and add d r to dh (gsrc[0]) instead of storing d(r*h)
    // MODE 1 EPI 4: rows of source 0 finish d h (accumulated); that value is
    // the first GRU half's dh' and its stage 1 is evaluated right here
    constexpr int NG = (EPI == 3 || EPI == 4) ? 16 : 1;
    float gr[NG], gh[NG], gq[EPI == 4 ? 16 : 1], gd[EPI == 4 ? 16 : 1];
    size_t gzi[NG], gi1[EPI == 4 ? 16 : 1];
    bool g3[NG];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = rbase + (r & 3) + 8 * (r >> 2);
      const int si = row >= rows ? -1 : (row >= a.cbase[1]) + (row >= a.cbase[2]) + (row >= a.cbase[3]);
      if (EPI == 3 || EPI == 4) {
        g3[r] = si == 0;
        const int c = si == 0 ? row : 0;
        gzi[r] = ((size_t)eb * a.z.ctot + a.z.coff + c) * HW + epix;
        gr[r] = si == 0 ? a.z.p[gzi[r]] : 0.f;
        gh[r] = si == 0 ? a.h.p[((size_t)eb * a.h.ctot + a.h.coff + c) * HW + epix] : 0.f;
        if constexpr (EPI == 4) {
          gi1[r] = ((size_t)eb * a.hd + c) * HW + epix;
          gq[r] = si == 0 ? a.g1q[gi1[r]] : 0.f;
          gd[r] = si == 0 && a.g1acc ? a.g1dh[gi1[r]] : 0.f;
        }
      }
      float* base = nullptr;
      int ctot = 0, coff = 0, cl = 0, ac = 0;
      if (si >= 0) {
        const int cb = si == 0 ? 0 : si == 1 ? a.cbase[1] : si == 2 ? a.cbase[2] : a.cbase[3];
        base = si == 0 ? a.gsrc[0] : si == 1 ? a.gsrc[1] : si == 2 ? a.gsrc[2] : a.gsrc[3];
        ctot = si == 0 ? a.gsrc_ctot[0] : si == 1 ? a.gsrc_ctot[1] : si == 2 ? a.gsrc_ctot[2] : a.gsrc_ctot[3];
        coff = si == 0 ? a.gsrc_coff[0] : si == 1 ? a.gsrc_coff[1] : si == 2 ? a.gsrc_coff[2] : a.gsrc_coff[3];
        ac = si == 0 ? a.gsrc_acc[0] : si == 1 ? a.gsrc_acc[1] : si == 2 ? a.gsrc_acc[2] : a.gsrc_acc[3];
        cl = row - cb;
      }
      dst[r] = base ? base + ((size_t)eb * ctot + coff + cl) * HW + epix : nullptr;
      accf[r] = base && (ac || ((EPI == 3 || EPI == 4) && si == 0));
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) old[r] = accf[r] ? *dst[r] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (EPI == 3 && g3[r]) {
        a.aux[gzi[r]] = acc[r] * gh[r] * gr[r] * (1.f - gr[r]);
        *dst[r] = old[r] + acc[r] * gr[r];
      } else if (EPI == 4 && g3[r]) {
        if constexpr (EPI == 4) {
          const float gn = old[r] + acc[r], z = gr[r], qv = gq[r], hv = gh[r];
          *dst[r] = gn;
          a.g1dq[gi1[r]] = gn * z * (1.f - qv * qv);
          a.aux[gzi[r]] = gn * (qv - hv) * z * (1.f - z);
          a.g1dh[gi1[r]] = a.g1acc ? gd[r] + gn * (1.f - z) : gn * (1.f - z);
        }
      } else if (dst[r]) {
        *dst[r] = accf[r] ? old[r] + acc[r] : acc[r];
      }
    }
  }
}

// sum of n partials p[0], p[stride], ... in a fixed order (4 interleaved
// chains, combined at the end): the loads are independent and issue together
__device__ __forceinline__ float split_sum(const float* __restrict__ p, size_t stride, int n) {
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int i = 0;
  for (; i + 4 <= n; i += 4) {
    s0 += p[(size_t)i * stride];
    s1 += p[(size_t)(i + 1) * stride];
    s2 += p[(size_t)(i + 2) * stride];
    s3 += p[(size_t)(i + 3) * stride];
  }
  for (; i < n; ++i) s0 += p[(size_t)i * stride];
  return (s0 + s1) + (s2 + s3);
}

// split-K finish: sum the partials in split order, then the epilogue
template <int MODE, int ACT, int EPI>
__global__ __launch_bounds__(256) void igemm_finish_kernel(IgArgs a, int ksplit) {
  const size_t HW = (size_t)a.g.H * a.g.W;
  const long long P = (long long)a.g.B * HW;
  const long long total = (long long)a.rows * P;
  const long long stride = (long long)gridDim.x * blockDim.x;
  if (total < (1LL << 31)) {   // 32-bit index arithmetic (a 64-bit division is ~4x the instructions)
    const unsigned P32 = (unsigned)P, HW32 = (unsigned)HW;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < (unsigned)total; i += (unsigned)stride) {
      const float v = split_sum(a.part + i, (size_t)total, ksplit);
      const unsigned row = i / P32, p = i - row * P32, eb = p / HW32;
      epi_store<MODE, ACT, EPI>(a, (int)row, (int)eb, (size_t)(p - eb * HW32), HW, v);
    }
    return;
  }
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    float v = 0.f;
    v = split_sum(a.part + i, (size_t)total, ksplit);
    const int row = (int)(i / P);
    const long long p = i - (long long)row * P;
    const int eb = (int)(p / (long long)HW);
    epi_store<MODE, ACT, EPI>(a, row, eb, (size_t)(p - (long long)eb * HW), HW, v);
  }
}

inline Div32 make_div32(int d) {
  Div32 f;
  f.d = (unsigned)(d > 0 ? d : 1);
  f.m = 0xFFFFFFFFu / f.d;
  return f;
}

inline size_t align256(size_t n) { return (n + 255) & ~(size_t)255; }

// ---- split-bf16 engine (xconv.hip)
// true when xconv covers this halo shape (1x5, 5x1, 3x3, 1x1)
bool xconv_supported(int KH, int KW);
// split-K partial bytes the xconv launch needs for this GEMM
size_t xconv_part_bytes(int rows, int kch, int KH, int KW, int B, int H, int W);
// MODE 0 forward / MODE 1 data gradient (a.wsplit in the matching layout);
// rows, kch, G / sources and the epilogue fields set as for the f32 engine
template <int MODE, int ACT, int EPI>
int launch_xconv(IgArgs& a, char* ws, hipStream_t s);

}  // namespace dro
