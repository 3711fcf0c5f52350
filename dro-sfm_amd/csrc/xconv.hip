// Split-bf16 MFMA convolution engine ("xconv") for the stride-1 halo
// convolutions of the recurrent update blocks (dro_sfm/networks/optim/
// update.py: SepConvGRU 1x5 / 5x1, projection encoders and heads 3x3 / 1x1).
//
// Arithmetic: every f32 operand x is split exactly-enough into three bf16
// terms x = x0 + x1 + x2 (x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 -
// x1): 24 significant bits, the whole f32 significand), and a product a*b is
// accumulated as the six terms whose magnitude is >= 2^-16 |ab|:
//   a1b1 + a0b2 + a2b0 + a0b1 + a1b0 + a0b0   (smallest first)
// on v_mfma_f32_32x32x16_bf16 with f32 accumulation.  The dropped terms
// (a1b2, a2b1, a2b2) are below 2^-24 |ab|, the rounding unit of f32: the
// result has f32 accuracy (the same error model as an f32 fmaf chain, not
// bitwise equal to it).  Six bf16 MFMAs (6 x 32 cycles per 32x32x16 step) do
// the work of eight f32 MFMAs (8 x 64 cycles): 2.67x the f32 MFMA rate
// (MI355X_MICROARCH.md: bf16 dense 2.5 PF, f32 157 TF).
//
// Operands:
//   * weights are split once per weight version by dro_weight_split into
//     [plane][row][K] bf16 with K = (32-channel chunk, tap, channel): the A
//     fragment of a 16-deep K step (8 consecutive channels of one tap per lane)
//     is one 16-byte read.  The data-gradient layout is the transposed weight
//     with the taps flipped, so the data gradient is the SAME kernel run over
//     the output gradient (MODE 1 only changes staging and the epilogue);
//   * activations are split while staged: the CK = 32 channel x halo patch of
//     a 64-pixel tile goes global -> registers -> LDS as [plane][pixel][32 ch]
//     bf16 (64 B per pixel, 16-byte slots XOR-swizzled by pixel so the
//     B-fragment reads of 16 consecutive pixels hit distinct banks).
// Tile: 32 output rows x 64 pixels (TH x TW) per 256-thread block; wave w
// computes pixel half (w & 1) over channel block (w >> 1) of every chunk, the
// two channel halves summed through LDS in the block-wide epilogue (shared with
// the f32 engine).  Two LDS stages, one register stage: the next chunk's loads
// are issued before this chunk's MFMAs.  Split-K over blocks only for short
// grids (partials + igemm_finish_kernel, fixed order: deterministic).
#include <hip/hip_runtime.h>

#include "conv_common.hpp"

namespace dro {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
// native vector (not HIP's uint4 struct: its copies went through a private
// alloca and the LDS store waited for the load at once)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x16 mfma_bf16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ unsigned short bf16_bits(__bf16 v) { return __builtin_bit_cast(unsigned short, v); }

// x -> three bf16 terms (round to nearest even at each step)
__device__ __forceinline__ void split3(float x, unsigned short& h0, unsigned short& h1, unsigned short& h2) {
  const __bf16 b0 = (__bf16)x;
  const float r1 = x - (float)b0;
  const __bf16 b1 = (__bf16)r1;
  const float r2 = r1 - (float)b1;
  const __bf16 b2 = (__bf16)r2;
  h0 = bf16_bits(b0);
  h1 = bf16_bits(b1);
  h2 = bf16_bits(b2);
}

template <int KH, int KW>
struct XShape {
  static constexpr int T = KH * KW;
  static constexpr int TH = (KH == 1 && KW > 1) ? 4 : 8;   // 1x5: 4x16 tiles; 5x1, 3x3, 1x1: 8x8
  static constexpr int TW = 64 / TH;
  static constexpr int HWd = TW + KW - 1;
  static constexpr int HALO = (TH + KH - 1) * HWd;
  static constexpr int NJ = (HALO + 63) / 64;
  static constexpr int XB = HALO * 64;                     // bytes per plane: 32 channels x 2 B per pixel
  static constexpr int RS = T * 64 + 16;                   // weight row stride in LDS (bytes)
  static constexpr int WB = 32 * RS;                       // bytes per plane
  static constexpr int STAGE = 3 * (XB + WB);
  static constexpr int RED = 2 * 32 * 64 * 4;              // epilogue: two channel halves, f32
  static constexpr int LDS = 2 * STAGE > RED ? 2 * STAGE : RED;
  static constexpr int WPIECES = 3 * 32 * T * 4;           // 16-byte weight pieces per stage
  static constexpr int WPER = (WPIECES + 255) / 256;
  static_assert(TH * TW == 64 && LDS <= 160 * 1024, "xconv shape");
};

// Epilogue of 8 results of one pixel, rows r0, r0 + 4, ..., r0 + 28 (same
// arithmetic as epi_store): all loads first, then the arithmetic and stores.
template <int MODE, int ACT, int EPI>
__device__ __forceinline__ void xepi(const IgArgs& a, const float (&v)[8], int r0, int b, size_t epix,
                                     size_t HW) {
  const int rows = a.rows;
  if (MODE == 0) {
    float bv[8], zv[EPI == 1 ? 8 : 1], hv[EPI != 0 ? 8 : 1];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = r0 + 4 * i;
      const int rr = row < rows ? row : 0;
      bv[i] = a.bias ? a.bias[rr] : 0.f;
      if (EPI == 1) {
        zv[i] = a.z.p[((size_t)b * a.z.ctot + a.z.coff + rr) * HW + epix];
        hv[i] = a.h.p[((size_t)b * a.h.ctot + a.h.coff + rr) * HW + epix];
      }
      if (EPI == 2) {
        const int c = rr >= a.hd ? rr - a.hd : 0;
        hv[i] = a.h.p[((size_t)b * a.h.ctot + a.h.coff + c) * HW + epix];
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = r0 + 4 * i;
      if (row >= rows) continue;
      float val = a.alpha * act_fwd(v[i] + bv[i], ACT);
      if (EPI == 1) {
        a.aux[((size_t)b * a.rows + row) * HW + epix] = val;
        val = (1.f - zv[i]) * hv[i] + zv[i] * val;
      }
      if (EPI == 2 && row >= a.hd) a.aux[((size_t)b * a.hd + (row - a.hd)) * HW + epix] = val * hv[i];
      a.out[((size_t)b * a.out_ctot + a.out_coff + row) * HW + epix] = val;
    }
  } else {
    float* dst[8];
    bool accf[8];
    float old[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = r0 + 4 * i;
      const int si = row >= rows ? -1 : (row >= a.cbase[1]) + (row >= a.cbase[2]) + (row >= a.cbase[3]);
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
      dst[i] = base ? base + ((size_t)b * ctot + coff + cl) * HW + epix : nullptr;
      accf[i] = base && ac;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) old[i] = accf[i] ? *dst[i] : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (dst[i]) *dst[i] = accf[i] ? old[i] + v[i] : v[i];
  }
}

template <int KH, int KW, int MODE, int ACT, int EPI>
__global__ __launch_bounds__(256) void xconv_kernel(IgArgs a) {
  using S = XShape<KH, KW>;
  constexpr int T = S::T, TW = S::TW, HWd = S::HWd, HALO = S::HALO, NJ = S::NJ;
  constexpr int XB = S::XB, RS = S::RS, WB = S::WB, STAGE = S::STAGE, WPER = S::WPER;
  constexpr int PH = KH / 2, PW = KW / 2;
  constexpr bool FOLD = MODE == 1 && ACT != 0;
  __shared__ __attribute__((aligned(16))) char smem[S::LDS];
  {   // diagnostics (dro_debug_conv_stamps): kernel entry of wave 0 (slot 10) and of the last wave (11)
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (a.stamps && (threadIdx.x == 0 || threadIdx.x == blockDim.x - 64))
      a.stamps[(size_t)blockIdx.x * 16 + (threadIdx.x == 0 ? 10 : 11)] = t0;
  }

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int pt = (int)udiv((unsigned)tile, a.rt_div), rt = tile - pt * a.row_tiles;
  const int row0 = rt * 32;
  const int b = (int)udiv((unsigned)pt, a.ti_div), trem = pt - b * a.tiles_img;
  const int tyi = (int)udiv((unsigned)trem, a.tx_div);
  const int ty0 = tyi * S::TH, tx0 = (trem - tyi * a.tiles_x) * TW;
  const int H = a.g.H, W = a.g.W;
  const size_t HW = (size_t)H * W;
  const unsigned HWu = (unsigned)HW;
  const int rows = a.rows, kch = a.kch, Cout = a.g.Cout;
  const int nck = (kch + 31) >> 5;
  const int cbeg = blockIdx.y * a.chunks_per_split;
  const int cend = min(nck, cbeg + a.chunks_per_split);

  // ---- X staging geometry: wave w stages channel groups g = w, w + 4 (4
  // channels each) of a chunk; lanes run over the halo pixels in NJ passes
  unsigned xpb[NJ];
  bool xok[NJ];
  int xoff[NJ];   // LDS byte offset of the lane's pixel row (slot of group g added at store)
  int xswz[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int e = lane + 64 * j;
    const int hy = e / HWd, hx = e - hy * HWd;
    const int yy = ty0 - PH + hy, xx = tx0 - PW + hx;
    xok[j] = e < HALO && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
    xpb[j] = xok[j] ? 4u * (unsigned)(yy * W + xx) : 0u;
    xoff[j] = e * 64;
    xswz[j] = (e >> 2) & 3;
  }
  // source table (as dconv_kernel): channel ch of source s starts at byte
  // address sQ[s] + ch * sR[s] (+ 4 * pixel unless broadcast: sM[s] = 0)
  const int cb1 = a.cbase[1], cb2 = a.cbase[2], cb3 = a.cbase[3];
  unsigned long long sQ[4];
  unsigned sR[4], sM[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (MODE == 0) {
      sQ[t] = a.sq0[t] + (unsigned long long)b * a.sqb[t];
      sR[t] = a.sr[t];
      sM[t] = a.sm[t];
    } else {
      sQ[t] = reinterpret_cast<unsigned long long>(a.G) + 4ull * (unsigned long long)b * Cout * HW;
      sR[t] = 4u * HWu;
      sM[t] = ~0u;
    }
  }
  const unsigned long long dQ1 = sQ[1] - sQ[0], dQ2 = sQ[2] - sQ[1], dQ3 = sQ[3] - sQ[2];
  const unsigned dR1 = sR[1] - sR[0], dR2 = sR[2] - sR[1], dR3 = sR[3] - sR[2];
  const unsigned dM1 = sM[1] - sM[0], dM2 = sM[2] - sM[1], dM3 = sM[3] - sM[2];
  const long long yshift = reinterpret_cast<long long>(a.gy) - reinterpret_cast<long long>(a.G);
  const float galpha = a.galpha;

  // ---- weight staging: 16-byte pieces (plane, row, piece) of the chunk's
  // T * 64-byte row runs; rows past the GEMM rows read the last row (discarded)
  const char* __restrict__ Wsp = a.wsplit;
  unsigned long long wg[WPER];
  int wd[WPER];
#pragma unroll
  for (int i = 0; i < WPER; ++i) {
    const int p = tid + 256 * i;
    const int pl = p / (32 * T * 4), rem = p - pl * (32 * T * 4);
    const int r = rem / (T * 4), pc = rem - r * (T * 4);
    const int row = min(row0 + r, rows - 1);
    const bool ok = p < S::WPIECES;
    wg[i] = ok ? (unsigned long long)pl * a.wplane + (unsigned long long)row * a.wrow + 16u * pc : 0ull;
    wd[i] = ok ? 3 * XB + pl * WB + r * RS + 16 * pc : -1;
  }

  struct Stage {
    float xr[8 * NJ], yr[FOLD ? 8 * NJ : 1];
    u32x4 wv[WPER];
    unsigned cmask;   // bit gi*4+i: channel 4g+i of this wave exists
  };
  typedef __attribute__((address_space(1))) const char* GPtr;
  typedef __attribute__((address_space(1))) const float* GFPtr;
  auto load = [&](Stage& st, int chunk) {
    const int c0 = chunk * 32;
    unsigned cm = 0;
#pragma unroll
    for (int gi = 0; gi < 2; ++gi) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ch = c0 + 4 * (wave + 4 * gi) + i;   // scalar
        const bool cok = ch < kch;
        cm |= cok ? (1u << (gi * 4 + i)) : 0u;
        const int cc = cok ? ch : 0;
        const unsigned long long k1 = MODE == 0 ? 0ull - (unsigned long long)(cc >= cb1) : 0ull;
        const unsigned long long k2 = MODE == 0 ? 0ull - (unsigned long long)(cc >= cb2) : 0ull;
        const unsigned long long k3 = MODE == 0 ? 0ull - (unsigned long long)(cc >= cb3) : 0ull;
        const unsigned j1 = (unsigned)k1, j2 = (unsigned)k2, j3 = (unsigned)k3;
        const unsigned long long Q = sQ[0] + (dQ1 & k1) + (dQ2 & k2) + (dQ3 & k3);
        const unsigned R = sR[0] + (dR1 & j1) + (dR2 & j2) + (dR3 & j3);
        const unsigned M = sM[0] + (dM1 & j1) + (dM2 & j2) + (dM3 & j3);
        const unsigned long long rq = Q + (unsigned long long)(unsigned)cc * R;
        const GPtr rowp = reinterpret_cast<GPtr>(rq);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          st.xr[(gi * 4 + i) * NJ + j] = *reinterpret_cast<GFPtr>(rowp + (xpb[j] & M));
          if (FOLD)
            st.yr[(gi * 4 + i) * NJ + j] =
                *reinterpret_cast<GFPtr>(reinterpret_cast<GPtr>(rq + (unsigned long long)yshift) + (xpb[j] & M));
        }
      }
    }
    st.cmask = cm;
    const unsigned long long cofs = (unsigned long long)chunk * (T * 64);
#pragma unroll
    for (int i = 0; i < WPER; ++i)
      if (S::WPIECES % 256 == 0 || wd[i] >= 0)
        st.wv[i] = *reinterpret_cast<const u32x4*>(Wsp + wg[i] + cofs);
  };
  auto store = [&](const Stage& st, int buf) {
    char* sb = smem + buf * STAGE;
#pragma unroll
    for (int gi = 0; gi < 2; ++gi) {
      const int g = wave + 4 * gi;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (NJ * 64 == HALO || lane + 64 * j < HALO) {
          unsigned short h0[4], h1[4], h2[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float v = (((st.cmask >> (gi * 4 + i)) & 1u) && xok[j]) ? st.xr[(gi * 4 + i) * NJ + j] : 0.f;
            if (MODE == 1) v *= galpha;
            if (FOLD) v *= act_bwd(st.yr[(gi * 4 + i) * NJ + j], ACT);
            split3(v, h0[i], h1[i], h2[i]);
          }
          const int off = xoff[j] + (((g >> 1) ^ xswz[j]) << 4) + ((g & 1) << 3);
          *reinterpret_cast<uint2*>(sb + off) =
              make_uint2(h0[0] | ((unsigned)h0[1] << 16), h0[2] | ((unsigned)h0[3] << 16));
          *reinterpret_cast<uint2*>(sb + XB + off) =
              make_uint2(h1[0] | ((unsigned)h1[1] << 16), h1[2] | ((unsigned)h1[3] << 16));
          *reinterpret_cast<uint2*>(sb + 2 * XB + off) =
              make_uint2(h2[0] | ((unsigned)h2[1] << 16), h2[2] | ((unsigned)h2[3] << 16));
        }
      }
    }
#pragma unroll
    for (int i = 0; i < WPER; ++i)
      if (S::WPIECES % 256 == 0 || wd[i] >= 0) *reinterpret_cast<u32x4*>(sb + wd[i]) = st.wv[i];
  };

  // ---- MFMA roles: wave = (channel block wk, pixel half wc)
  const int wk = wave >> 1, wc = wave & 1;
  const int hi = lane >> 5;
  const int q = wc * 32 + (lane & 31);
  const int qy = q / TW, qx = q - qy * TW;
  const int aoff = 3 * XB + (lane & 31) * RS + wk * 32 + hi * 16;   // + 64 per tap ([tap][32 ch] runs)
  const int bslot = 2 * wk + hi;
  int boff[T];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int ty = t / KW, tx = t - ty * KW;
    const int hp = (qy + ty) * HWd + qx + tx;
    boff[t] = hp * 64 + ((bslot ^ ((hp >> 2) & 3)) << 4);
  }
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  auto mma = [&](int buf) {
    const char* sb = smem + buf * STAGE;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(sb + aoff + t * 64);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(sb + aoff + WB + t * 64);
      const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(sb + aoff + 2 * WB + t * 64);
      const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(sb + boff[t]);
      const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(sb + XB + boff[t]);
      const bf16x8 b2 = *reinterpret_cast<const bf16x8*>(sb + 2 * XB + boff[t]);
      acc = mfma_bf16(a1, b1, acc);
      acc = mfma_bf16(a0, b2, acc);
      acc = mfma_bf16(a2, b0, acc);
      acc = mfma_bf16(a0, b1, acc);
      acc = mfma_bf16(a1, b0, acc);
      acc = mfma_bf16(a0, b0, acc);
    }
  };

  unsigned long long* const stp = a.stamps ? a.stamps + (size_t)blockIdx.x * 16 : nullptr;
  auto stamp = [&](int k) {   // slots: 0 set-up done, 12 first chunk staged, 1 prologue,
                                // 2.. chunk iterations (<= 8), 13 reductions, 14 epilogue
    if (stp && threadIdx.x == 0 && k < 15) stp[k] = __builtin_amdgcn_s_memtime();
  };
  stamp(0);
  if (stp && threadIdx.x == blockDim.x - 64) stp[15] = __builtin_amdgcn_s_memtime();
  const int dbg = ablation_flags(a.dbg);   // diagnostics: 1 skip the loop's loads, 2 its MFMAs, 4 its LDS stores
  // one register stage: chunk c+1 is loaded before chunk c's MFMAs and
  // stored after them.  (Measured alternative: store c+1 after the MFMAs and
  // re-issue c+2 at once -- no faster per iteration, +1.8k cycles of prologue.)
  Stage st;
  if (cbeg < cend) {
    load(st, cbeg);
    store(st, 0);
  }
  stamp(12);
  __syncthreads();
  stamp(1);
  for (int c = cbeg; c < cend; ++c) {
    const int buf = (c - cbeg) & 1;
    const bool more = c + 1 < cend;
    if (more && !(dbg & 1)) load(st, c + 1);
    if (!(dbg & 2)) mma(buf);
    if (more && !(dbg & 4)) store(st, buf ^ 1);
    __syncthreads();
    if (c - cbeg < 8) stamp(2 + c - cbeg);
  }

  // ---- block-wide reduction of the two channel halves + epilogue
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int rl = (r & 3) + 8 * (r >> 2) + 4 * hi;
    red[(wk * 32 + rl) * 64 + wc * 32 + (lane & 31)] = acc[r];
  }
  __syncthreads();
  stamp(13);
  // thread = one pixel x 8 rows (rq, rq + 4, ...): every operand of the 8
  // results is loaded before the first is used (one memory round trip)
  const int pl = tid & 63, rq = tid >> 6;
  const int py = pl / TW, px = pl - py * TW;
  const int oy = ty0 + py, ox = tx0 + px;
  if (oy < H && ox < W) {
    const size_t epix = (size_t)oy * W + ox;
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = red[(rq + 4 * i) * 64 + pl] + red[(32 + rq + 4 * i) * 64 + pl];
    if (a.part) {   // split-K partial: [split][rows][P]
      const long long P = (long long)a.g.B * HW;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = row0 + rq + 4 * i;
        if (row < rows) a.part[(size_t)blockIdx.y * rows * P + (size_t)row * P + (size_t)b * HW + epix] = v[i];
      }
    } else {
      xepi<MODE, ACT, EPI>(a, v, row0 + rq, b, epix, HW);
    }
  }
  stamp(14);
}

// ------------------------------------------------------------------ weight split
// w [Cout][Cin][KH][KW] f32 -> fwd [3][Cout][nf * T * 32] (channel padded to
// nf * 32, nf = ceil(Cin / 32)) and bwd [3][Cin][nb * T * 32] (transposed,
// taps flipped, nb = ceil(Cout / 32)); K index = (chunk, tap, channel % 32).
__global__ __launch_bounds__(256) void weight_split_kernel(const float* __restrict__ w, int Cout, int Cin,
                                                           int T, unsigned short* __restrict__ out,
                                                           int bwd) {
  const int rows = bwd ? Cin : Cout, kc = bwd ? Cout : Cin;
  const int nch = (kc + 31) >> 5;
  const long long rowlen = (long long)nch * T * 32;
  const long long total = (long long)rows * rowlen;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int row = (int)(i / rowlen);
    const int k = (int)(i - (long long)row * rowlen);
    const int chunk = k / (T * 32), r = k - chunk * (T * 32);
    const int tap = r >> 5, cl = r & 31;
    const int c = chunk * 32 + cl;
    float v = 0.f;
    if (c < kc) {
      v = bwd ? w[((size_t)c * Cin + row) * T + (T - 1 - tap)] : w[((size_t)row * Cin + c) * T + tap];
    }
    unsigned short h0, h1, h2;
    split3(v, h0, h1, h2);
    out[i] = h0;
    out[total + i] = h1;
    out[2 * total + i] = h2;
  }
}

// ------------------------------------------------------------------ host side
bool xconv_supported(int KH, int KW) {
  return (KH == 1 && KW == 5) || (KH == 5 && KW == 1) || (KH == 3 && KW == 3) || (KH == 1 && KW == 1);
}

namespace {

struct XPlan {
  int row_tiles, ptiles, tiles_x, tiles_img, nck, ksplit, chunks_per_split;
  size_t part_bytes;
};

XPlan plan_xconv(int rows, int kch, int KH, int KW, int B, int H, int W) {
  XPlan pl = {};
  const int TH = (KH == 1 && KW > 1) ? 4 : 8, TW = 64 / TH;
  pl.tiles_x = (W + TW - 1) / TW;
  pl.tiles_img = ((H + TH - 1) / TH) * pl.tiles_x;
  pl.ptiles = B * pl.tiles_img;
  pl.row_tiles = (rows + 31) / 32;
  pl.nck = (kch + 31) / 32;
  const long long blocks = (long long)pl.row_tiles * pl.ptiles;
  int ks = 1;
  static const long long short_grid = [] {   // tuning: grids below this many tiles split K over blocks
    const char* e = getenv("DRO_XCONV_SPLIT_BELOW");
    return e ? atoll(e) : 128LL;
  }();
  if (blocks < short_grid) {
    ks = (int)((256 + blocks - 1) / blocks);
    if (ks > 16) ks = 16;
    if (ks > pl.nck) ks = pl.nck;
    if (ks < 1) ks = 1;
  }
  pl.chunks_per_split = (pl.nck + ks - 1) / ks;
  pl.ksplit = (pl.nck + pl.chunks_per_split - 1) / pl.chunks_per_split;
  const long long P = (long long)B * H * W;
  pl.part_bytes = pl.ksplit > 1 ? align256((size_t)pl.ksplit * rows * P * sizeof(float)) : 0;
  return pl;
}

}  // namespace

size_t xconv_part_bytes(int rows, int kch, int KH, int KW, int B, int H, int W) {
  if (!xconv_supported(KH, KW)) return 0;
  return plan_xconv(rows, kch, KH, KW, B, H, W).part_bytes;
}

template <int MODE, int ACT, int EPI>
int launch_xconv(IgArgs& a, char* ws, hipStream_t s) {
  const int KH = a.g.KH, KW = a.g.KW;
  if (!xconv_supported(KH, KW) || !a.wsplit) {
    set_error("xconv: unsupported shape or missing split weights");
    return DRO_E_SHAPE;
  }
  const XPlan pl = plan_xconv(a.rows, a.kch, KH, KW, a.g.B, a.g.H, a.g.W);
  const int T = KH * KW;
  a.wrow = (unsigned)pl.nck * T * 64;
  a.wplane = (unsigned long long)a.rows * a.wrow;
  a.row_tiles = pl.row_tiles;
  a.tiles_x = pl.tiles_x;
  a.tiles_img = pl.tiles_img;
  a.rt_div = make_div32(pl.row_tiles);
  a.ti_div = make_div32(pl.tiles_img);
  a.tx_div = make_div32(pl.tiles_x);
  a.chunks_per_split = pl.chunks_per_split;
  a.part = pl.ksplit > 1 ? reinterpret_cast<float*>(ws) : nullptr;
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
  const dim3 grid((unsigned)(pl.row_tiles * pl.ptiles), (unsigned)pl.ksplit);
  if (KH == 1 && KW == 5)
    hipLaunchKernelGGL((xconv_kernel<1, 5, MODE, ACT, EPI>), grid, dim3(256), 0, s, a);
  else if (KH == 5)
    hipLaunchKernelGGL((xconv_kernel<5, 1, MODE, ACT, EPI>), grid, dim3(256), 0, s, a);
  else if (KH == 3)
    hipLaunchKernelGGL((xconv_kernel<3, 3, MODE, ACT, EPI>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((xconv_kernel<1, 1, MODE, ACT, EPI>), grid, dim3(256), 0, s, a);
  int st = launch_status("xconv_kernel launch failed");
  if (st || pl.ksplit == 1) return st;
  const long long total = (long long)a.rows * a.g.B * a.g.H * a.g.W;
  long long blocks = (total + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL((igemm_finish_kernel<MODE, ACT, EPI>), dim3((unsigned)blocks), dim3(256), 0, s, a,
                     pl.ksplit);
  return launch_status("igemm_finish_kernel launch failed");
}

// the (MODE, ACT, EPI) combinations the C ABI reaches
template int launch_xconv<0, 0, 0>(IgArgs&, char*, hipStream_t);
template int launch_xconv<0, 1, 0>(IgArgs&, char*, hipStream_t);
template int launch_xconv<0, 2, 0>(IgArgs&, char*, hipStream_t);
template int launch_xconv<0, 3, 0>(IgArgs&, char*, hipStream_t);
template int launch_xconv<0, 2, 2>(IgArgs&, char*, hipStream_t);
template int launch_xconv<0, 3, 1>(IgArgs&, char*, hipStream_t);
template int launch_xconv<1, 0, 0>(IgArgs&, char*, hipStream_t);
template int launch_xconv<1, 1, 0>(IgArgs&, char*, hipStream_t);
template int launch_xconv<1, 2, 0>(IgArgs&, char*, hipStream_t);
template int launch_xconv<1, 3, 0>(IgArgs&, char*, hipStream_t);

}  // namespace dro

using namespace dro;

extern "C" size_t dro_weight_split_bytes(int Cout, int Cin, int KH, int KW, int transposed) {
  if (Cout < 1 || Cin < 1 || KH < 1 || KW < 1) return 0;
  const int rows = transposed ? Cin : Cout, kc = transposed ? Cout : Cin;
  return (size_t)3 * rows * ((kc + 31) / 32) * KH * KW * 32 * sizeof(unsigned short);
}

extern "C" int dro_weight_split(const float* weight, int Cout, int Cin, int KH, int KW, void* fwd, void* bwd,
                                void* stream) {
  if (!weight || (!fwd && !bwd)) {
    set_error("weight_split: NULL weight or outputs");
    return DRO_E_NULL;
  }
  if (Cout < 1 || Cin < 1 || KH < 1 || KW < 1 || Cout >= 4096 || Cin >= 4096 || KH * KW > 49) {
    set_error("weight_split: sizes out of range");
    return DRO_E_SHAPE;
  }
  hipStream_t s = (hipStream_t)stream;
  const int T = KH * KW;
  for (int which = 0; which < 2; ++which) {
    void* out = which ? bwd : fwd;
    if (!out) continue;
    const long long n = (long long)dro_weight_split_bytes(Cout, Cin, KH, KW, which) / 6;
    long long blocks = (n + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(weight_split_kernel, dim3((unsigned)blocks), dim3(256), 0, s, weight, Cout, Cin, T,
                       static_cast<unsigned short*>(out), which);
    int st = launch_status("weight_split_kernel launch failed");
    if (st) return st;
  }
  return DRO_OK;
}
