// PNG decoding on the GPU: the image-decode step of the training data pipeline
// (SURVEY.md §8(f)2).  Replaces, for the frames KITTIDataset reads
// (dro_sfm/datasets/kitti_dataset.py:354, :387 -> utils/image.py:13-27
// load_image = PIL.Image.open) and its ground-truth depth PNGs
// (kitti_dataset.py:38-44 read_png_depth), Pillow's PNG decoder: zlib inflate
// of the concatenated IDAT payload (RFC 1950/1951: stored, fixed and dynamic
// Huffman blocks) and the per-row PNG filters (None, Sub, Up, Average, Paeth),
// for non-interlaced 8-bit grey / RGB / RGBA and 16-bit grey images.  Output
// bit-identical to Pillow (tests/test_png.py): uint8 [N, H, W, 3] frames (grey
// replicated, alpha dropped -- PIL .convert("RGB")) or, for 16-bit depth PNGs,
// float32 [N, H, W] = value / 256 with -1 where the value is 0 (read_png_depth).
//
// Host side (dro_sfm_amd/datasets/png.py): chunk parsing only (IHDR, IDAT
// concatenation); the compressed bytes go to the device as they are.
//
// Kernels (one 64-lane workgroup per image each; N images per launch):
//   png_inflate_kernel  -- the DEFLATE bit stream is serial: every lane runs the
//     same Huffman decode (wave-uniform state, no divergence); the compressed
//     bytes are staged through a 4 KB LDS window by all lanes, the tables are
//     canonical-Huffman with a 10-bit direct lookup (built by all lanes, one
//     entry each), and LZ77 copies run across the 64 lanes out of a 32 KB LDS
//     history window (byte k of a match of distance d is the byte d back, k mod d
//     into the run: every lane's source precedes the match, so overlapping
//     matches copy in parallel too).  Output: the filtered scanlines.
//   png_unfilter_kernel -- PNG filters depend on the left pixel and the row above:
//     64 rows at a time, lane l on row r0 + l, skewed one pixel per lane (lane l
//     reconstructs pixel t - l at step t), the row above's two latest pixels
//     passed down by one lane shuffle each; W + 63 steps per band of 64 rows.
// Roofline: neither HBM nor MFMA -- the inflate is a serial dependency chain of
// table lookups per image (latency bound); throughput comes from decoding many
// images at once (one CU each).  Algorithmic bytes per image: compressed size +
// H (1 + W bpp) filtered bytes written and read + the output.
#include <hip/hip_runtime.h>

#include "dro_common.hpp"

namespace dro {
namespace {

constexpr int kPngThreads = 64;
constexpr int kWinBits = 15, kWin = 1 << kWinBits;   // DEFLATE's 32 KB history
constexpr int kInWords = 1024;                        // 4 KB staged input
constexpr int kFastBits = 10;

enum PngErr {
  kOk = 0,
  kBadHeader = 1,
  kBadBlock = 2,
  kBadLengths = 3,
  kBadSymbol = 4,
  kBadDistance = 5,
  kOutOverrun = 6,
  kInOverrun = 7,
  kBadFilter = 8,
  kShortOutput = 9,
};

struct Huff {
  unsigned short count[16];
  unsigned short symbol[288];
  unsigned short fast[1 << kFastBits];   // (symbol << 4) | length; 0: longer than kFastBits
};

__constant__ unsigned short kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                            31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ unsigned char kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                            2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ unsigned short kDistBase[30] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,
                                             33,   49,   65,   97,   129,  193,   257,   385,   513, 769,
                                             1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ unsigned char kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                             6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ unsigned char kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// One wave per image: LDS writes and reads of the wave's lanes are ordered by
// program order alone (the LDS executes a wave's operations in issue order).
// A compiler-only barrier replaces __syncthreads(), whose release fence would
// also wait for every byte the wave has stored to global memory (measured:
// 261 ms per KITTI frame with it, the waits serialising every match copy).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The whole decoder state is wave-uniform: every lane holds the same copy.
struct Inflater {
  const unsigned* src;        // the image's stream, 4-byte aligned
  long long n;                // stream bytes
  long long ip;               // next byte to move into the bit buffer
  long long lo;               // stream offset of in[0] (multiple of 4)
  unsigned long long bb;      // bit buffer (LSB first)
  int bc;                     // valid bits in bb
  int err;
  unsigned* in;               // LDS: stream bytes [lo, lo + 4096)
};

__device__ __forceinline__ unsigned in_word(const Inflater& s, long long w) {
  // word w of the stream (0 past the end; the load itself always in bounds)
  const long long nw = (s.n + 3) >> 2;
  const unsigned v = s.src[w < nw ? w : nw - 1];
  return w < nw ? v : 0u;
}

// stream words [w0, w0 + kInWords) into the LDS window (all lanes: every
// lane's 16 loads in flight together, then the 16 LDS stores).  Out of line:
// the decode loop stays small (one wave per CU runs it, so instruction-cache
// misses of a sprawling inlined loop are fully exposed).
__device__ __noinline__ void load_window(unsigned* __restrict__ in, const unsigned* __restrict__ src, long long n,
                                         long long w0) {
  wave_sync();
  const long long nw = (n + 3) >> 2;
  constexpr int PER = kInWords / kPngThreads;
  unsigned w[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const long long wi = w0 + threadIdx.x + k * kPngThreads;
    const unsigned v = src[wi < nw ? wi : nw - 1];
    w[k] = wi < nw ? v : 0u;
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) in[threadIdx.x + k * kPngThreads] = w[k];
  wave_sync();
}

// make stream bytes [ip, ip + 8) resident in the LDS window
__device__ __forceinline__ void stage(Inflater& s) {
  if (s.ip >= s.lo && s.ip + 8 <= s.lo + 4 * kInWords) return;
  s.lo = s.ip & ~3LL;
  load_window(s.in, s.src, s.n, s.lo >> 2);
}

__device__ __forceinline__ long long rfl64(long long v) {
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((unsigned long long)v >> 32));
  return (long long)(((unsigned long long)hi << 32) | lo);
}

// the bit reader's state, re-asserted wave-uniform (SGPRs): the compiler's
// divergence analysis cannot see that every lane runs the same decode
__device__ __forceinline__ void uniform(Inflater& s) {
  s.bb = (unsigned long long)rfl64((long long)s.bb);
  s.bc = __builtin_amdgcn_readfirstlane(s.bc);
  s.ip = rfl64(s.ip);
  s.lo = rfl64(s.lo);
}

__device__ __forceinline__ void refill(Inflater& s) {
  if (s.bc > 32) return;
  stage(s);
  const long long r = s.ip - s.lo;      // byte offset in the window, < 4096 - 8
  // readfirstlane: the decoder state is wave-uniform; held in SGPRs its
  // branches are scalar (as LDS results in VGPRs, every test became exec-mask
  // flow and each symbol walked dozens of such blocks)
  const unsigned w0 = __builtin_amdgcn_readfirstlane(s.in[r >> 2]);
  const unsigned w1 = __builtin_amdgcn_readfirstlane(s.in[(r >> 2) + 1]);
  const int sh = (int)(r & 3) * 8;
  const unsigned w = sh ? (w0 >> sh) | (w1 << (32 - sh)) : w0;
  s.bb |= (unsigned long long)w << s.bc;
  s.bc += 32;
  s.ip += 4;
}

__device__ __forceinline__ unsigned take(Inflater& s, int nbits) {
  if (nbits == 0) return 0;
  refill(s);
  const unsigned v = (unsigned)(s.bb & ((1ull << nbits) - 1));
  s.bb >>= nbits;
  s.bc -= nbits;
  return v;
}

// bytes of the stream consumed so far (bits read, rounded up at byte boundaries)
__device__ __forceinline__ long long consumed(const Inflater& s) { return s.ip - s.bc / 8; }

// Canonical Huffman code from code lengths (puff.c's construction); returns
// < 0 for an over-subscribed set.  The direct table: entry e decodes the next
// kFastBits stream bits e; each lane fills its own entries by walking the code.
__device__ __noinline__ int build(Huff& h, const unsigned char* len, int n) {
  wave_sync();
  const int lane = threadIdx.x;
  // lane l < 16 counts the codes of length l and places them in symbol order
  // (every lane reads the same length byte each step: an LDS broadcast)
  if (lane < 16) {
    int cnt = 0;
    for (int s = 0; s < n; ++s) cnt += len[s] == lane;
    h.count[lane] = (unsigned short)cnt;
  }
  wave_sync();
  if (lane >= 1 && lane < 16) {
    int o = 0;
    for (int l = 1; l < lane; ++l) o += h.count[l];
    for (int s = 0; s < n; ++s)
      if (len[s] == lane) h.symbol[o++] = (unsigned short)s;
  }
  wave_sync();
  int left = 1;
  for (int l = 1; l < 16; ++l) {
    left <<= 1;
    left -= __builtin_amdgcn_readfirstlane(h.count[l]);
    if (left < 0) return -1;
  }
  for (int e = threadIdx.x; e < (1 << kFastBits); e += kPngThreads) {
    int code = 0, first = 0, index = 0;
    unsigned short v = 0;
    for (int l = 1; l <= kFastBits; ++l) {
      code |= (e >> (l - 1)) & 1;
      const int count = h.count[l];
      if (code - count < first) {
        v = (unsigned short)((h.symbol[index + (code - first)] << 4) | l);
        break;
      }
      index += count;
      first += count;
      first <<= 1;
      code <<= 1;
    }
    h.fast[e] = v;
  }
  wave_sync();
  return left;
}

__device__ __forceinline__ int decode(Inflater& s, const Huff& h) {
  refill(s);
  const unsigned e = __builtin_amdgcn_readfirstlane(h.fast[s.bb & ((1u << kFastBits) - 1)]);
  if (e) {
    const int l = (int)(e & 15);
    if (l > s.bc) {
      s.err = kInOverrun;
      return -1;
    }
    s.bb >>= l;
    s.bc -= l;
    return (int)(e >> 4);
  }
  int code = 0, first = 0, index = 0;
  for (int l = 1; l < 16; ++l) {
    if (l > s.bc) break;
    code |= (int)((s.bb >> (l - 1)) & 1);
    const int count = __builtin_amdgcn_readfirstlane(h.count[l]);
    if (code - count < first) {
      s.bb >>= l;
      s.bc -= l;
      return __builtin_amdgcn_readfirstlane(h.symbol[index + (code - first)]);
    }
    index += count;
    first += count;
    first <<= 1;
    code <<= 1;
  }
  s.err = kBadSymbol;
  return -1;
}

__global__ __launch_bounds__(kPngThreads) void png_inflate_kernel(const unsigned char* __restrict__ zdata,
                                                                  const long long* __restrict__ zoff,
                                                                  unsigned char* __restrict__ filt,
                                                                  long long flen, int* __restrict__ status) {
  __shared__ unsigned char win[kWin];
  __shared__ unsigned inw[kInWords];
  __shared__ Huff hl, hd;
  __shared__ unsigned char lens[320];
  const int img = blockIdx.x, lane = threadIdx.x;
  Inflater s;
  s.src = reinterpret_cast<const unsigned*>(zdata + zoff[img]);
  s.n = zoff[img + 1] - zoff[img];
  s.ip = 0;
  s.lo = -(1LL << 40);
  s.bb = 0;
  s.bc = 0;
  s.err = kOk;
  s.in = inw;
  unsigned char* out = filt + (long long)img * flen;
  auto fail = [&](int code) {
    if (lane == 0) status[img] = code;
  };
  // zlib header (RFC 1950): deflate, 32 KB window, no preset dictionary
  const unsigned cmf = take(s, 8), flg = take(s, 8);
  if ((cmf & 15) != 8 || (cmf >> 4) > 7 || ((cmf << 8) | flg) % 31 != 0 || (flg & 32)) {
    fail(kBadHeader);
    return;
  }
  // Output goes to the LDS history window only; whole spans of it are copied
  // to global memory (`flush`) every 16 KB and at the end.  A global store per
  // symbol made every later s_waitcnt vmcnt(0) of the decode loop (the input
  // staging's) wait for all of them: 260 ms per KITTI frame.
  long long pos = 0, flushed = 0;
  auto flush = [&]() {
    wave_sync();
    for (long long k = flushed + lane; k < pos; k += kPngThreads) out[k] = win[k & (kWin - 1)];
    flushed = pos;
  };
  int last = 0;
  while (!last) {
    last = (int)take(s, 1);
    const int type = (int)take(s, 2);
    if (type == 0) {                                   // stored block
      const int drop = s.bc & 7;
      s.bb >>= drop;
      s.bc -= drop;
      const unsigned ln = take(s, 16), nln = take(s, 16);
      if ((ln ^ 0xffffu) != nln) {
        fail(kBadBlock);
        return;
      }
      // un-read the whole bytes left in the bit buffer, copy straight from the stream
      s.ip -= s.bc / 8;
      s.bb = 0;
      s.bc = 0;
      if (s.ip + ln > s.n) {
        fail(kInOverrun);
        return;
      }
      if (pos + ln > flen) {
        fail(kOutOverrun);
        return;
      }
      flush();
      const unsigned char* sb = zdata + zoff[img] + s.ip;
      for (unsigned k = lane; k < ln; k += kPngThreads) {
        const unsigned char b = sb[k];
        win[(pos + k) & (kWin - 1)] = b;
        out[pos + k] = b;
      }
      pos += ln;
      flushed = pos;
      s.ip += ln;
      wave_sync();
      continue;
    }
    if (type == 3) {
      fail(kBadBlock);
      return;
    }
    if (type == 1) {                                   // fixed Huffman codes
      wave_sync();
      for (int k = lane; k < 320; k += kPngThreads)
        lens[k] = k < 144 ? 8 : k < 256 ? 9 : k < 280 ? 7 : k < 288 ? 8 : 5;
      if (build(hl, lens, 288) < 0 || build(hd, lens + 288, 30) < 0) {
        fail(kBadLengths);
        return;
      }
    } else {                                           // dynamic Huffman codes
      const int nlen = (int)take(s, 5) + 257, ndist = (int)take(s, 5) + 1, ncode = (int)take(s, 4) + 4;
      if (nlen > 286 || ndist > 30) {
        fail(kBadLengths);
        return;
      }
      wave_sync();
      if (lane < 19) lens[lane] = 0;
      wave_sync();
      for (int k = 0; k < ncode; ++k) {
        const unsigned v = take(s, 3);
        if (lane == 0) lens[kClOrder[k]] = (unsigned char)v;
      }
      if (build(hl, lens, 19) != 0) {                  // the code-length code must be complete
        fail(kBadLengths);
        return;
      }
      // the literal/length and distance code lengths, straight into LDS (every
      // lane decodes, the lanes write the runs)
      int k = 0, prev = 0;
      while (k < nlen + ndist) {
        const int sym = decode(s, hl);
        if (sym < 0) {
          fail(s.err);
          return;
        }
        int v = sym, rep = 1;
        if (sym == 16) {
          if (k == 0) {
            fail(kBadLengths);
            return;
          }
          v = prev;
          rep = 3 + (int)take(s, 2);
        } else if (sym == 17) {
          v = 0;
          rep = 3 + (int)take(s, 3);
        } else if (sym == 18) {
          v = 0;
          rep = 11 + (int)take(s, 7);
        }
        if (k + rep > nlen + ndist) {
          fail(kBadLengths);
          return;
        }
        for (int j = lane; j < rep; j += kPngThreads) lens[k + j] = (unsigned char)v;
        k += rep;
        prev = v;
      }
      wave_sync();
      if (__builtin_amdgcn_readfirstlane(lens[256]) == 0) {   // no end-of-block code
        fail(kBadLengths);
        return;
      }
      // incomplete codes are allowed only for a single distance code (puff.c)
      const int ll = build(hl, lens, nlen);
      const int dl = build(hd, lens + nlen, ndist);
      const int z0 = __builtin_amdgcn_readfirstlane(hl.count[0]), z1 = __builtin_amdgcn_readfirstlane(hd.count[0]);
      if (ll < 0 || (ll > 0 && nlen - z0 != 1) || dl < 0 || (dl > 0 && ndist - z1 != 1)) {
        fail(kBadLengths);
        return;
      }
    }
    // the block's symbols
    for (;;) {
      uniform(s);
      pos = rfl64(pos);
      flushed = rfl64(flushed);
      if (pos - flushed >= kWin / 2) flush();          // unflushed bytes stay < 32 KB
      // Literal runs first: a tight loop over direct-table literal hits (the
      // measured cost of the general path was ~75 instructions per literal,
      // SQ counters of a literal-only stream, tools/png_pmc_probe.py)
      {
        const long long lim = flushed + kWin / 2 < flen ? flushed + kWin / 2 : flen;
        while (pos < lim) {
          if (s.bc < 16) refill(s);
          const unsigned e = __builtin_amdgcn_readfirstlane(hl.fast[s.bb & ((1u << kFastBits) - 1)]);
          const int l = (int)(e & 15);
          if (e == 0 || (e >> 4) > 255 || l > s.bc) break;
          s.bb >>= l;
          s.bc -= l;
          if (lane == 0) win[pos & (kWin - 1)] = (unsigned char)(e >> 4);
          ++pos;
        }
        if (pos - flushed >= kWin / 2) continue;       // flush before the next symbol
      }
      const int sym = decode(s, hl);
      if (sym < 0) {
        fail(s.err);
        return;
      }
      if (sym < 256) {
        if (pos >= flen) {
          fail(kOutOverrun);
          return;
        }
        if (lane == 0) win[pos & (kWin - 1)] = (unsigned char)sym;
        ++pos;
        continue;
      }
      if (sym == 256) break;
      const int li = sym - 257;
      if (li >= 29) {
        fail(kBadSymbol);
        return;
      }
      const int len = kLenBase[li] + (int)take(s, kLenExtra[li]);
      const int dsym = decode(s, hd);
      if (dsym < 0 || dsym >= 30) {
        fail(dsym < 0 ? s.err : kBadSymbol);
        return;
      }
      const int dist = kDistBase[dsym] + (int)take(s, kDistExtra[dsym]);
      if (dist > pos) {
        fail(kBadDistance);
        return;
      }
      if (pos + len > flen) {
        fail(kOutOverrun);
        return;
      }
      wave_sync();                                 // earlier single-lane window writes
      for (int k = lane; k < len; k += kPngThreads) {
        const int kk = k < dist ? k : k % dist;
        const unsigned char b = win[(pos - dist + kk) & (kWin - 1)];
        win[(pos + k) & (kWin - 1)] = b;
      }
      pos += len;
      wave_sync();
    }
    if (s.err) {
      fail(s.err);
      return;
    }
  }
  flush();
  if (pos != flen) {
    fail(kShortOutput);
    return;
  }
  if (consumed(s) > s.n) {
    fail(kInOverrun);
    return;
  }
  if (lane == 0) status[img] = kOk;
}

__device__ __forceinline__ int paeth(int a, int b, int c) {
  const int p = a + b - c;
  const int pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
  return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

// kind: 0 grey8 -> RGB, 2 RGB8, 6 RGBA8 -> RGB (alpha dropped), 16 grey16 -> depth
template <int BPP, int KIND>
__global__ __launch_bounds__(kPngThreads) void png_unfilter_kernel(const unsigned char* __restrict__ filt,
                                                                   long long flen, int H, int W,
                                                                   void* __restrict__ outp,
                                                                   int* __restrict__ status) {
  __shared__ unsigned char above[8192 * 2];     // the previous band's last row (W * BPP <= 16 K)
  const int img = blockIdx.x, lane = threadIdx.x;
  if (status[img] != kOk) return;               // the inflate failed: leave its code
  const long long stride = 1 + (long long)W * BPP;
  const unsigned char* f = filt + (long long)img * flen;
  for (int k = lane; k < W * BPP; k += kPngThreads) above[k] = 0;   // the row above row 0 is zeros
  __syncthreads();
  int bad = 0;
  for (int r0 = 0; r0 < H; r0 += kPngThreads) {
    const int r = r0 + lane;
    const bool live = r < H;
    const unsigned char* row = f + (long long)(live ? r : 0) * stride;
    const int ftype = live ? row[0] : 0;
    bad |= ftype > 4;
    unsigned char h1[BPP], h2[BPP];             // this row's pixels x-1 and x-2 (own steps t-1, t-2)
#pragma unroll
    for (int k = 0; k < BPP; ++k) h1[k] = h2[k] = 0;
    const int nsteps = W + kPngThreads - 1;
    for (int t = 0; t < nsteps; ++t) {
      const int x = t - lane;
      // the row above: lane l-1's pixels x (its step t-1) and x-1 (step t-2)
      unsigned char b[BPP], c[BPP];
#pragma unroll
      for (int k = 0; k < BPP; ++k) {
        const int ub = __shfl_up((int)h1[k], 1, kPngThreads);
        const int uc = __shfl_up((int)h2[k], 1, kPngThreads);
        b[k] = (unsigned char)ub;
        c[k] = (unsigned char)uc;
      }
      const bool on = live && x >= 0 && x < W;
      if (lane == 0 && on) {
#pragma unroll
        for (int k = 0; k < BPP; ++k) {
          b[k] = above[x * BPP + k];
          c[k] = x > 0 ? above[(x - 1) * BPP + k] : 0;
        }
      }
      unsigned char v[BPP];
#pragma unroll
      for (int k = 0; k < BPP; ++k) {
        const int a = x > 0 ? h1[k] : 0, bb = b[k], cc = x > 0 ? c[k] : 0;
        const int raw = on ? row[1 + x * BPP + k] : 0;
        int p;
        switch (ftype) {
          case 1: p = a; break;
          case 2: p = bb; break;
          case 3: p = (a + bb) >> 1; break;
          case 4: p = paeth(a, bb, cc); break;
          default: p = 0; break;
        }
        v[k] = (unsigned char)(raw + p);
      }
      if (on) {
        if (KIND == 16) {
          const int d = ((int)v[0] << 8) | v[1];        // big-endian 16-bit grey
          reinterpret_cast<float*>(outp)[((long long)img * H + r) * W + x] = d == 0 ? -1.f : (float)d / 256.f;
        } else {
          unsigned char* o = reinterpret_cast<unsigned char*>(outp) + (((long long)img * H + r) * W + x) * 3;
          o[0] = v[0];
          o[1] = KIND == 0 ? v[0] : v[1];
          o[2] = KIND == 0 ? v[0] : v[2];
        }
#pragma unroll
        for (int k = 0; k < BPP; ++k) {
          h2[k] = h1[k];
          h1[k] = v[k];
        }
      } else {
#pragma unroll
        for (int k = 0; k < BPP; ++k) {
          h2[k] = h1[k];
          h1[k] = 0;
        }
      }
      // the band's last row feeds the next band's first (its pixel x is read
      // by lane 0 at step x of the next band; written here at step x + 63)
      if (lane == kPngThreads - 1 && on) {
#pragma unroll
        for (int k = 0; k < BPP; ++k) above[x * BPP + k] = v[k];
      }
    }
    // a short last band: its last live row, not lane 63, is the row above nothing
    __syncthreads();
  }
  if (__any(bad) && lane == 0) status[img] = kBadFilter;
}

}  // namespace
}  // namespace dro

using namespace dro;

extern "C" size_t dro_png_filtered_bytes(int H, int W, int bpp) {
  return (size_t)H * (1 + (size_t)W * bpp);
}

extern "C" int dro_png_decode(const unsigned char* zdata, const long long* zoff, int N, int H, int W, int kind,
                              unsigned char* filtered, void* out, int* status, void* stream) {
  if (!zdata || !zoff || !filtered || !out || !status) {
    set_error("png_decode: NULL pointer");
    return DRO_E_NULL;
  }
  const int bpp = kind == 0 ? 1 : kind == 2 ? 3 : kind == 6 ? 4 : kind == 16 ? 2 : 0;
  if (!bpp) {
    set_error("png_decode: kind must be 0 (grey8), 2 (RGB8), 6 (RGBA8) or 16 (grey16)");
    return DRO_E_MODE;
  }
  if (N < 1 || N > 65535 || H < 1 || W < 1 || (long long)W * bpp > 16384 || (long long)H * W >= (1LL << 31)) {
    set_error("png_decode: sizes out of range (row bytes <= 16384)");
    return DRO_E_SHAPE;
  }
  hipStream_t s = (hipStream_t)stream;
  const long long flen = (long long)dro_png_filtered_bytes(H, W, bpp);
  hipLaunchKernelGGL(png_inflate_kernel, dim3(N), dim3(kPngThreads), 0, s, zdata, zoff, filtered, flen, status);
  int st = launch_status("png_inflate_kernel launch failed");
  if (st) return st;
  switch (kind) {
    case 0: hipLaunchKernelGGL((png_unfilter_kernel<1, 0>), dim3(N), dim3(kPngThreads), 0, s, filtered, flen, H, W, out, status); break;
    case 2: hipLaunchKernelGGL((png_unfilter_kernel<3, 2>), dim3(N), dim3(kPngThreads), 0, s, filtered, flen, H, W, out, status); break;
    case 6: hipLaunchKernelGGL((png_unfilter_kernel<4, 6>), dim3(N), dim3(kPngThreads), 0, s, filtered, flen, H, W, out, status); break;
    default: hipLaunchKernelGGL((png_unfilter_kernel<2, 16>), dim3(N), dim3(kPngThreads), 0, s, filtered, flen, H, W, out, status); break;
  }
  return launch_status("png_unfilter_kernel launch failed");
}
