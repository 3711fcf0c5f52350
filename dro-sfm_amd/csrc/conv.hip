// Implicit-GEMM convolutions on f32 MFMA (v_mfma_f32_32x32x2_f32) for the
// recurrent update blocks of the DRO optimizer (dro_sfm/networks/optim/
// update.py): SepConvGRU 1x5 / 5x1 gates, projection encoders, heads.
//
// Why not MIOpen: at these shapes (M = B*h*w = 3840..7680 output pixels,
// 64..576 channels) every MIOpen call is a separate launch of 8-30 us plus
// NCHW<->NHWC transposes, bias/activation/concat are separate ATen kernels,
// and its training-mode batch-norm/gradient paths lose precision.
// Here:
//   * inputs are a VIRTUAL channel concatenation of up to 3 tensor slices (no
//     torch.cat), optionally with source 0 multiplied elementwise by another
//     slice (the GRU's r*h) while it is staged;
//   * bias + activation (+ the GRU blend h' = (1-z)h + zq) run in the epilogue,
//     and the result lands in a channel slice of a bigger tensor;
//   * f32 MFMA is exact-f32 (a k-ordered fmaf chain): no TF32-style loss.
// GEMM orientation: rows = output channels, cols = pixels, so the epilogue
// stores are coalesced along pixels (the MFMA C column is the lane).
//
// Roofline: MFMA(f32) bound at 157 TF/s peak for the big gates; the small
// heads are latency bound.  FLOPs per launch = 2 * Cout * P * Cin * KH * KW.
#include <hip/hip_runtime.h>

#include "dro_common.hpp"

namespace dro {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kBO = 32;   // output channels per workgroup
constexpr int kBP = 64;   // pixels per workgroup
constexpr int kBK = 16;   // reduction chunk
constexpr int kMaxSrc = 4;

struct Slice {            // channels [coff, coff+C) of a [B, ctot, H, W] tensor
  const float* p;
  int C, ctot, coff;
  int bcast;              // 1: a [B, ctot, 1, 1] tensor broadcast over H x W
};

struct ConvGeom {
  int B, H, W, Cin, Cout, KH, KW, PH, PW;
};

struct ConvFwdArgs {
  ConvGeom g;
  Slice src[kMaxSrc];
  int nsrc;
  Slice scale0;           // optional multiplier of source 0 (p == nullptr: none)
  const float* weight;    // [Cout][Cin][KH][KW]
  const float* bias;      // [Cout] or nullptr
  float alpha;            // output scale (act == none only)
  float* out;             // output slice base
  int out_ctot, out_coff;
  // GRU blend epilogue (epi == 1): out = (1-z) h + z q with q = tanh(acc+b)
  Slice z, h;
  float* q_out;           // optional: raw q saved for the backward
  int q_ctot, q_coff;
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

// value of the virtual input at channel c, pixel offset `off` of image b
// (caller checks the zero-padding bounds)
__device__ __forceinline__ float src_val(const Slice* s, int nsrc, const Slice& scale0, int c, int b,
                                         size_t HW, size_t off) {
  int base = 0;
#pragma unroll
  for (int i = 0; i < kMaxSrc; ++i) {
    if (i < nsrc && c < base + s[i].C) {
      const int cl = c - base;
      float v = s[i].bcast ? s[i].p[(size_t)b * s[i].ctot + s[i].coff + cl]
                           : s[i].p[((size_t)b * s[i].ctot + s[i].coff + cl) * HW + off];
      if (i == 0 && scale0.p) v *= scale0.p[((size_t)b * scale0.ctot + scale0.coff + cl) * HW + off];
      return v;
    }
    base += (i < nsrc) ? s[i].C : 0;
  }
  return 0.f;
}

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------ forward
// Workgroup: 4 waves; tile 32 out-channels x 64 pixels.  Wave w computes
// pixels [32*(w&1), +32) over k-half (w>>1) of every chunk; the two k-halves
// are summed through LDS before the epilogue.
template <int ACT, int EPI>
__global__ __launch_bounds__(256) void conv_fwd_kernel(ConvFwdArgs a) {
  __shared__ float Ws[kBK][kBO + 1];
  __shared__ float Xs[kBK][kBP];
  __shared__ float red[2][16][64];
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int o0 = blockIdx.y * kBO, p0 = blockIdx.x * kBP;
  const size_t HW = (size_t)g.H * g.W;
  const long long P = (long long)g.B * HW;
  const int T = g.KH * g.KW, K = g.Cin * T;

  // this thread's staging pixel (fixed for the whole K loop)
  const long long pg = p0 + (tid & 63);
  const bool pv = pg < P;
  const int pb = pv ? (int)(pg / HW) : 0;
  const int prem = pv ? (int)(pg % HW) : 0;
  const int py = prem / g.W, px = prem % g.W;

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

  const int wp = wave & 1, wk = wave >> 1;
  for (int k0 = 0; k0 < K; k0 += kBK) {
    // ---- stage X: k rows (wave-uniform) x 64 pixels
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kl = wave * 4 + i, k = k0 + kl;
      float v = 0.f;
      if (pv && k < K) {
        const int c = k / T, tap = k - c * T;
        const int yy = py + tap / g.KW - g.PH, xx = px + tap % g.KW - g.PW;
        if (yy >= 0 && yy < g.H && xx >= 0 && xx < g.W)
          v = src_val(a.src, a.nsrc, a.scale0, c, pb, HW, (size_t)yy * g.W + xx);
      }
      Xs[kl][tid & 63] = v;
    }
    // ---- stage W^T: 16 k x 32 o
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ol = tid >> 3, kl = (tid & 7) * 2 + i, o = o0 + ol, k = k0 + kl;
      Ws[kl][ol] = (o < g.Cout && k < K) ? a.weight[(size_t)o * K + k] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int kl = wk * 8 + kk * 2 + (lane >> 5);
      acc = mfma32(Ws[kl][lane & 31], Xs[kl][wp * 32 + (lane & 31)], acc);
    }
    __syncthreads();
  }
  // ---- sum the two k-halves
  if (wk == 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wp][r][lane] = acc[r];
  }
  __syncthreads();
  if (wk == 1) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] += red[wp][r][lane];

  // ---- epilogue: element (o, p) with o = row, p = lane column
  const long long pe = p0 + wp * 32 + (lane & 31);
  if (pe >= P) return;
  const int eb = (int)(pe / HW);
  const size_t epix = (size_t)(pe % HW);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int o = o0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (o >= g.Cout) continue;
    float v = acc[r] + (a.bias ? a.bias[o] : 0.f);
    v = a.alpha * act_fwd(v, ACT);
    if (EPI == 1) {
      const float z = a.z.p[((size_t)eb * a.z.ctot + a.z.coff + o) * HW + epix];
      const float hv = a.h.p[((size_t)eb * a.h.ctot + a.h.coff + o) * HW + epix];
      if (a.q_out) a.q_out[((size_t)eb * a.q_ctot + a.q_coff + o) * HW + epix] = v;
      v = (1.f - z) * hv + z * v;
    }
    a.out[((size_t)eb * a.out_ctot + a.out_coff + o) * HW + epix] = v;
  }
}

// ------------------------------------------------------------------ backward: data
// din[c, p] = sum_{o,ky,kx} W[o,c,ky,kx] * G[o, p - (ky-PH, kx-PW)],
// G = dout * act'(y).  Rows = input channels, cols = pixels, K = (o, tap).
struct ConvBwdArgs {
  ConvGeom g;
  Slice src[kMaxSrc];           // forward inputs (for wgrad) -- and grad targets below
  int nsrc;
  Slice scale0;
  const float* weight;
  const float* dout;            // [B, Cout, H, W] upstream gradient (dense)
  float alpha;                  // forward output scale
  const float* y;               // saved activation output [B, Cout, H, W] (act != 0)
  Slice y_slice;                // where y lives (dense if ctot == Cout)
  // grad targets per source (dense [B, C_i, H, W] or slices), accumulate flags
  float* gsrc[kMaxSrc];
  int gsrc_ctot[kMaxSrc], gsrc_coff[kMaxSrc], gsrc_acc[kMaxSrc];
  float* gweight;               // [Cout][Cin][KH][KW], accumulated (atomic)
  float* gbias;                 // [Cout], accumulated (atomic)
  int splits;                   // pixel splits of the weight-gradient reduction
};

__device__ __forceinline__ float grad_pre(const ConvBwdArgs& a, int act, int o, int b, size_t HW,
                                          size_t pix) {
  const float d = a.alpha * a.dout[((size_t)b * a.g.Cout + o) * HW + pix];
  if (act == 0) return d;
  const float yv = a.y_slice.p[((size_t)b * a.y_slice.ctot + a.y_slice.coff + o) * HW + pix];
  return d * act_bwd(yv, act);
}

template <int ACT>
__global__ __launch_bounds__(256) void conv_dgrad_kernel(ConvBwdArgs a) {
  __shared__ float Ws[kBK][kBO + 1];   // [k=(o,tap)][c]
  __shared__ float Gs[kBK][kBP];   // [k][p]
  __shared__ float red[2][16][64];
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c0 = blockIdx.y * kBO, p0 = blockIdx.x * kBP;
  const size_t HW = (size_t)g.H * g.W;
  const long long P = (long long)g.B * HW;
  const int T = g.KH * g.KW, K = g.Cout * T;
  const long long pg = p0 + (tid & 63);
  const bool pv = pg < P;
  const int pb = pv ? (int)(pg / HW) : 0;
  const int prem = pv ? (int)(pg % HW) : 0;
  const int py = prem / g.W, px = prem % g.W;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int wp = wave & 1, wk = wave >> 1;
  for (int k0 = 0; k0 < K; k0 += kBK) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kl = wave * 4 + i, k = k0 + kl;
      float v = 0.f;
      if (pv && k < K) {
        const int o = k / T, tap = k - o * T;
        const int yy = py - (tap / g.KW - g.PH), xx = px - (tap % g.KW - g.PW);
        if (yy >= 0 && yy < g.H && xx >= 0 && xx < g.W)
          v = grad_pre(a, ACT, o, pb, HW, (size_t)yy * g.W + xx);
      }
      Gs[kl][tid & 63] = v;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int cl = tid >> 3, kl = (tid & 7) * 2 + i, c = c0 + cl, k = k0 + kl;
      float w = 0.f;
      if (c < g.Cin && k < K) {
        const int o = k / T, tap = k - o * T;
        w = a.weight[((size_t)o * g.Cin + c) * T + tap];
      }
      Ws[kl][cl] = w;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int kl = wk * 8 + kk * 2 + (lane >> 5);
      acc = mfma32(Ws[kl][lane & 31], Gs[kl][wp * 32 + (lane & 31)], acc);
    }
    __syncthreads();
  }
  if (wk == 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wp][r][lane] = acc[r];
  }
  __syncthreads();
  if (wk == 1) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] += red[wp][r][lane];
  const long long pe = p0 + wp * 32 + (lane & 31);
  if (pe >= P) return;
  const int eb = (int)(pe / HW);
  const size_t epix = (size_t)(pe % HW);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int c = c0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (c >= g.Cin) continue;
    int base = 0, which = 0;
    for (int i = 0; i < a.nsrc; ++i) {
      if (c < base + a.src[i].C) {
        which = i;
        break;
      }
      base += a.src[i].C;
    }
    float* dst = a.gsrc[which];
    if (!dst) continue;
    float* q = dst + ((size_t)eb * a.gsrc_ctot[which] + a.gsrc_coff[which] + (c - base)) * HW + epix;
    *q = a.gsrc_acc[which] ? (*q + acc[r]) : acc[r];
  }
}

// ------------------------------------------------------------------ backward: weights
// dW[o, k=(c,tap)] = sum_p G[o,p] * X[k,p]; rows = o, cols = k, reduction over
// pixels split across gridDim.z (fp32 atomics into the zeroed dW).  Wave w:
// k columns [32*(w&1), +32), pixel half (w>>1) of every chunk.
template <int ACT>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(ConvBwdArgs a) {
  __shared__ float Gs[kBK][kBO + 1];   // [p][o]
  __shared__ float Xs[kBK][kBP + 1];   // [p][k]
  __shared__ float red[2][16][64];
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kt0 = blockIdx.x * kBP, o0 = blockIdx.y * kBO;
  const size_t HW = (size_t)g.H * g.W;
  const long long P = (long long)g.B * HW;
  const int T = g.KH * g.KW, K = g.Cin * T;
  const long long chunk = ((P + a.splits - 1) / a.splits + kBK - 1) / kBK * kBK;
  const long long pbeg = (long long)blockIdx.z * chunk;
  const long long pend = pbeg + chunk < P ? pbeg + chunk : P;
  // staging role: pixel-in-chunk pl (16 consecutive lanes = 16 consecutive
  // pixels, coalesced) and 4 fixed k columns, decoded once
  const int pl = tid & 15;
  int kc[4], kdy[4], kdx[4];
  bool kv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int kg = kt0 + (tid >> 4) * 4 + i;
    kv[i] = kg < K;
    kc[i] = kv[i] ? kg / T : 0;
    const int tap = kv[i] ? kg - kc[i] * T : 0;
    kdy[i] = tap / g.KW - g.PH;
    kdx[i] = tap % g.KW - g.PW;
  }
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int wk = wave & 1, wp = wave >> 1;
  for (long long q0 = pbeg; q0 < pend; q0 += kBK) {
    const long long p = q0 + pl;
    const bool pvld = p < pend;
    const int b = pvld ? (int)(p / HW) : 0, rem = pvld ? (int)(p % HW) : 0;
    const int py = rem / g.W, px = rem % g.W;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = 0.f;
      const int yy = py + kdy[i], xx = px + kdx[i];
      if (pvld && kv[i] && yy >= 0 && yy < g.H && xx >= 0 && xx < g.W)
        v = src_val(a.src, a.nsrc, a.scale0, kc[i], b, HW, (size_t)yy * g.W + xx);
      Xs[pl][(tid >> 4) * 4 + i] = v;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ol = (tid >> 4) * 2 + i, o = o0 + ol;
      float v = 0.f;
      if (o < g.Cout && pvld) v = grad_pre(a, ACT, o, b, HW, (size_t)rem);
      Gs[pl][ol] = v;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int pr = wp * 8 + kk * 2 + (lane >> 5);
      acc = mfma32(Gs[pr][lane & 31], Xs[pr][wk * 32 + (lane & 31)], acc);
    }
    __syncthreads();
  }
  if (wp == 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wk][r][lane] = acc[r];
  }
  __syncthreads();
  if (wp == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float v = acc[r] + red[wk][r][lane];
      const int o = o0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const int k = kt0 + wk * 32 + (lane & 31);
      if (o < g.Cout && k < K) atomicAdd(a.gweight + (size_t)o * K + k, v);
    }
  }
}

// bias gradient: db[o] = sum_p G[o,p] (one workgroup per output channel chunk)
template <int ACT>
__global__ __launch_bounds__(256) void conv_bgrad_kernel(ConvBwdArgs a) {
  __shared__ float scratch[4];
  const ConvGeom& g = a.g;
  const int o = blockIdx.x;
  const size_t HW = (size_t)g.H * g.W;
  const long long P = (long long)g.B * HW;
  float s = 0.f;
  for (long long p = (long long)blockIdx.y * blockDim.x + threadIdx.x; p < P;
       p += (long long)gridDim.y * blockDim.x)
    s += grad_pre(a, ACT, o, (int)(p / HW), HW, (size_t)(p % HW));
  float v[1] = {s};
  block_sum<1>(v, scratch);
  if (threadIdx.x == 0) atomicAdd(a.gbias + o, v[0]);
}

}  // namespace dro

using namespace dro;

namespace {

int conv_setup_geom(ConvGeom& g, const dro_slice* srcs, int nsrc, int B, int H, int W, int Cout,
                    int KH, int KW) {
  if (!srcs || nsrc < 1 || nsrc > kMaxSrc) {
    set_error("conv2d: need 1..3 input slices");
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
  if (B < 1 || H < 1 || W < 1 || Cout < 1 || KH < 1 || KW < 1 || (KH % 2) == 0 || (KW % 2) == 0) {
    set_error("conv2d: sizes out of range (odd kernels, 'same' padding, stride 1)");
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

}  // namespace

#define DRO_ACT_SWITCH(act, ...)                  \
  switch (act) {                                  \
    case 0: { constexpr int A_ = 0; __VA_ARGS__; } break; \
    case 1: { constexpr int A_ = 1; __VA_ARGS__; } break; \
    case 2: { constexpr int A_ = 2; __VA_ARGS__; } break; \
    case 3: { constexpr int A_ = 3; __VA_ARGS__; } break; \
    default: set_error("conv2d: unknown activation"); return DRO_E_MODE; \
  }

extern "C" int dro_conv2d_forward(const dro_slice* srcs, int nsrc, const dro_slice* scale0,
                                  const float* weight, const float* bias, int B, int H, int W,
                                  int Cout, int KH, int KW, int act, float alpha, float* out,
                                  int out_ctot, int out_coff, void* stream) {
  ConvFwdArgs a = {};
  int st = conv_setup_geom(a.g, srcs, nsrc, B, H, W, Cout, KH, KW);
  if (st) return st;
  if (!weight || !out || out_coff < 0 || out_coff + Cout > out_ctot) {
    set_error("conv2d_forward: NULL weight/out or bad output slice");
    return DRO_E_NULL;
  }
  for (int i = 0; i < nsrc; ++i) a.src[i] = to_slice(srcs + i);
  a.nsrc = nsrc;
  a.scale0 = to_slice(scale0);
  a.weight = weight;
  a.bias = bias;
  a.alpha = alpha;
  if (alpha != 1.f && act != 0) {
    set_error("conv2d_forward: alpha != 1 requires act none");
    return DRO_E_MODE;
  }
  a.out = out;
  a.out_ctot = out_ctot;
  a.out_coff = out_coff;
  const long long P = (long long)B * H * W;
  dim3 grid((unsigned)((P + kBP - 1) / kBP), (Cout + kBO - 1) / kBO);
  hipStream_t s = (hipStream_t)stream;
  DRO_ACT_SWITCH(act, hipLaunchKernelGGL((conv_fwd_kernel<A_, 0>), grid, dim3(256), 0, s, a));
  return launch_status("conv_fwd_kernel launch failed");
}

extern "C" int dro_convgru_blend_forward(const dro_slice* srcs, int nsrc, const dro_slice* scale0,
                                         const float* weight, const float* bias, int B, int H,
                                         int W, int Cout, int KH, int KW, const dro_slice* z,
                                         const dro_slice* h, float* q_out, int q_ctot, int q_coff,
                                         float* out, int out_ctot, int out_coff, void* stream) {
  ConvFwdArgs a = {};
  int st = conv_setup_geom(a.g, srcs, nsrc, B, H, W, Cout, KH, KW);
  if (st) return st;
  if (!weight || !out || !z || !h || !z->data || !h->data) {
    set_error("convgru_blend_forward: NULL weight/out/z/h");
    return DRO_E_NULL;
  }
  for (int i = 0; i < nsrc; ++i) a.src[i] = to_slice(srcs + i);
  a.nsrc = nsrc;
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
  const long long P = (long long)B * H * W;
  dim3 grid((unsigned)((P + kBP - 1) / kBP), (Cout + kBO - 1) / kBO);
  hipLaunchKernelGGL((conv_fwd_kernel<3, 1>), grid, dim3(256), 0, (hipStream_t)stream, a);
  return launch_status("conv_fwd_kernel<blend> launch failed");
}

extern "C" int dro_conv2d_backward(const dro_slice* srcs, int nsrc, const dro_slice* scale0,
                                   const float* weight, int B, int H, int W, int Cout, int KH,
                                   int KW, int act, float alpha, const dro_slice* y,
                                   const float* dout,
                                   float* const* grad_srcs, const int* grad_ctot,
                                   const int* grad_coff, const int* grad_accumulate,
                                   float* grad_weight, float* grad_bias, void* stream) {
  ConvBwdArgs a = {};
  int st = conv_setup_geom(a.g, srcs, nsrc, B, H, W, Cout, KH, KW);
  if (st) return st;
  if (!weight || !dout || (act != 0 && (!y || !y->data))) {
    set_error("conv2d_backward: NULL weight/dout/y");
    return DRO_E_NULL;
  }
  for (int i = 0; i < nsrc; ++i) {
    a.src[i] = to_slice(srcs + i);
    a.gsrc[i] = grad_srcs ? grad_srcs[i] : nullptr;
    a.gsrc_ctot[i] = grad_ctot ? grad_ctot[i] : srcs[i].channels;
    a.gsrc_coff[i] = grad_coff ? grad_coff[i] : 0;
    a.gsrc_acc[i] = grad_accumulate ? grad_accumulate[i] : 0;
  }
  a.nsrc = nsrc;
  a.scale0 = to_slice(scale0);
  a.weight = weight;
  a.dout = dout;
  a.alpha = alpha;
  a.y_slice = to_slice(y);
  a.gweight = grad_weight;
  a.gbias = grad_bias;
  hipStream_t s = (hipStream_t)stream;
  const long long P = (long long)B * H * W;
  const int K = a.g.Cin * KH * KW;
  bool any_dgrad = false;
  for (int i = 0; i < nsrc; ++i) any_dgrad |= a.gsrc[i] != nullptr;
  if (any_dgrad) {
    dim3 grid((unsigned)((P + kBP - 1) / kBP), (a.g.Cin + kBO - 1) / kBO);
    DRO_ACT_SWITCH(act, hipLaunchKernelGGL((conv_dgrad_kernel<A_>), grid, dim3(256), 0, s, a));
    if ((st = launch_status("conv_dgrad_kernel launch failed"))) return st;
  }
  if (grad_weight) {
    if ((st = launch_zero(grad_weight, (size_t)Cout * K, s))) return st;
    const int ktiles = (K + kBP - 1) / kBP, otiles = (Cout + kBO - 1) / kBO;
    int splits = (int)((512 + ktiles * otiles - 1) / (ktiles * otiles));
    const long long maxs = (P + 63) / 64;
    if (splits > maxs) splits = (int)maxs;
    if (splits < 1) splits = 1;
    a.splits = splits;
    dim3 grid(ktiles, otiles, splits);
    DRO_ACT_SWITCH(act, hipLaunchKernelGGL((conv_wgrad_kernel<A_>), grid, dim3(256), 0, s, a));
    if ((st = launch_status("conv_wgrad_kernel launch failed"))) return st;
  }
  if (grad_bias) {
    if ((st = launch_zero(grad_bias, (size_t)Cout, s))) return st;
    dim3 grid(Cout, 8);
    DRO_ACT_SWITCH(act, hipLaunchKernelGGL((conv_bgrad_kernel<A_>), grid, dim3(256), 0, s, a));
    if ((st = launch_status("conv_bgrad_kernel launch failed"))) return st;
  }
  return DRO_OK;
}

// ------------------------------------------------------------------ SepConvGRU elementwise backward
// update.py:67-70 (and :74-77): h' = (1-z) h + z q, q = tanh(.), rh = r * h.
// stage 1 (before the q-gate backward):  dq = dh' * z;  dz = dh' * (q - h);  dh = dh' * (1 - z)
// stage 2 (after it, drh = dL/d(r*h)):   dr = drh * h;  dh += drh * r
// z = zr[:, :hd], r = zr[:, hd:], dz / dr written into dzr likewise.
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
    const size_t b = i / ((size_t)hd * HW), rem = i % ((size_t)hd * HW);
    const size_t zi = b * 2 * hd * HW + rem, ri = zi + (size_t)hd * HW;
    if (stage == 1) {
      const float g = dhn[i], z = zr[zi];
      dq[i] = g * z;
      dzr[zi] = g * (q[i] - h[i]);
      dh[i] = g * (1.f - z);
    } else {
      const float d = drh[i];
      dzr[ri] = d * h[i];
      dh[i] += d * zr[ri];
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
