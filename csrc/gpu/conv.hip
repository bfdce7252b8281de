// Weight gradient of the DCGAN discriminator's 4x4 / stride-2 / pad-1
// convolutions on channels-last bf16 activations, on the MFMA units.
//
//   dW[co][kh][kw][ci] = sum over pixels m = (n, oh, ow) of
//                        dY[m][co] * X[n][2oh-1+kh][2ow-1+kw][ci]
//
// As a GEMM: C[co][kc] = sum_m A[co][m] * B[m][kc], kc = (kh*4 + kw)*Cin + ci.
// Both operands have the reduction index m as their OUTER (row) dimension in
// memory (NHWC rows of channels), while the MFMA wants 8 consecutive m per
// lane: the tiles are staged row-major in LDS exactly as loaded (16-byte
// vectors, no scatter) and fed to v_mfma_f32_16x16x32_bf16 with
// ds_read_b64_tr_b16, the gfx950 transposing LDS read (each 16-lane group
// reads 4 rows x 16 columns and gets them column-major).
//
// A kc tile of 128 never straddles a kh row when Cin % 32 == 0, and a kh row
// of the im2col matrix is contiguous in X ((kw, ci) runs over 4 neighbouring
// input pixels), so every 16-byte chunk of the B tile is one aligned load --
// or zero at an image border.
//
// Work split: blocks = tiles (Cout/64 x KC/128) x S pixel slices; each block
// reduces its slice into a 64 x 128 fp32 tile of partial[S][Cout][KC]
// (plain stores, no atomics), and conv_wgrad_reduce sums the S partials into
// the fp32 weight gradient in the parameter's own memory layout.  Block ids
// are remapped so the tiles of one slice (which read the same dY rows and
// overlapping X rows) share an XCD and its L2.
//
// Reference role: the gradient PyTorch/MIOpen computes for nn.Conv2d in the
// reference's densityopt discriminator (examples/densityopt/densityopt.py:
// 139-190); MIOpen's bf16 NHWC path spends 2 zero-fills + an atomic igemm +
// a cast kernel per layer on it (profiles/r2/disc_mtrace_kernels.txt).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace btn {
namespace gpu {
namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int kThreads = 256;   // 4 waves: 2 (co) x 2 (kc), a 32 x 64 sub-tile each
constexpr int BCO = 64;         // output channels per block
constexpr int BKC = 128;        // im2col columns per block
constexpr int BPX = 32;         // pixels per k-step (the MFMA's K)
constexpr int DY_ROW = BCO * 2;             // 128-byte LDS rows
constexpr int X_ROW = BKC * 2;              // 256-byte LDS rows
constexpr int DY_TILE = BPX * DY_ROW;       // 4 KiB
constexpr int X_TILE = BPX * X_ROW;         // 8 KiB
constexpr int STAGE = DY_TILE + X_TILE;     // one pipeline stage

// LDS images are row-major [pixel][channel]; the 32-byte windows of a row are
// XOR-swizzled so that the 8 rows one 32-lane half reads with a transposing
// read (rows 8g+q and 8g+8+q, q = 0..3, same columns) land on 8 different
// bank windows.  X rows are 256 B (one full bank row, 8 windows); dY rows are
// 128 B (two rows share a bank row, 4 windows each).
__device__ __forceinline__ int x_off(int r, int byte) {
  const int f = (r & 3) | (((r >> 3) & 1) << 2);
  return r * X_ROW + ((((byte >> 5) ^ f) << 5) | (byte & 31));
}
__device__ __forceinline__ int dy_off(int r, int byte) {
  const int f = ((r >> 1) & 1) | (((r >> 3) & 1) << 1);
  return r * DY_ROW + ((((byte >> 5) ^ f) << 5) | (byte & 31));
}

__device__ __forceinline__ s16x4 tr_read(const char* lds, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + off));
}

// 8-element MFMA fragment: rows (pixels) 8g .. 8g+7 of 16 columns starting at
// `col` (elements); lane 4q+p of each 16-lane group addresses row q, columns
// col+4p .. col+4p+3 (T10 of the CDNA guide), lane i gets column col+i.
template <bool IS_X>
__device__ __forceinline__ bf16x8 frag(const char* img, int lane, int col) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int byte = (col + 4 * p) * 2;
  const int r0 = 8 * g + q;
  const s16x4 lo = tr_read(img, IS_X ? x_off(r0, byte) : dy_off(r0, byte));
  const s16x4 hi = tr_read(img, IS_X ? x_off(r0 + 4, byte) : dy_off(r0 + 4, byte));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// Bounds-checked 16-byte loads through a buffer descriptor: a lane whose
// chunk lies outside the image (padding) or past the last pixel passes an
// offset beyond the descriptor's range and gets zeros from the hardware --
// no branch around the load, so the next tile's loads stay in flight across
// the MFMAs (a masked or branched load makes hipcc wait vmcnt(0) for it).
constexpr uint32_t kOOB = 0x80000000u;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, int(bytes), 0x00020000);
}
__device__ __forceinline__ uint4 bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, int(off), 0, 0);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// frag() with a precomputed lane offset: rows r0 (off) and r0 + 4 (off + row4)
__device__ __forceinline__ bf16x8 frag_at(const char* img, int off, int row4) {
  const s16x4 lo = tr_read(img, off);
  const s16x4 hi = tr_read(img, off + row4);
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

struct PixelCursor {   // (n, oh, ow) of pixel m, advanced by BPX per k-step
  int n, oh, ow;
  __device__ void init(int m, int Ho, int Wo) {
    const int hw = Ho * Wo;
    n = m / hw;
    const int r = m - n * hw;
    oh = r / Wo;
    ow = r - oh * Wo;
  }
  __device__ void advance(int Ho, int Wo) {
    ow += BPX;
    while (ow >= Wo) {
      ow -= Wo;
      if (++oh == Ho) oh = 0, ++n;
    }
  }
};

__global__ __launch_bounds__(kThreads) void conv_wgrad_kernel(ConvWgradParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int t = int(threadIdx.x), lane = t & 63, wave = t >> 6;
  const int KC = 16 * p.Cin, KT = KC / BKC, T = (p.Cout / BCO) * KT;

  // XCD-aware bijective remap: consecutive work ids share an XCD (blockIdx % 8)
  const int nwg = int(gridDim.x), b = int(blockIdx.x);
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int w = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int slice = w / T, tile = w - slice * T;
  const int co0 = (tile / KT) * BCO, kt = tile - (tile / KT) * KT;
  // all index math in 32 bits (the host guarantees every byte offset < 2^31):
  // 64-bit address arithmetic made this kernel VALU-bound (9.5 VALU per MFMA)
  const int m_begin = slice * int(p.px_per_slice);
  const int m_end = m_begin + int(p.px_per_slice) < int(p.M) ? m_begin + int(p.px_per_slice) : int(p.M);
  const int nsteps = m_end > m_begin ? (m_end - m_begin + BPX - 1) / BPX : 0;

  // this thread's staging work: one dY chunk, two X chunks per k-step
  const int dpx = t >> 3, dch = t & 7;                 // dY: pixel, 16-byte chunk
  const int xpx0 = t >> 4, xch = t & 15;               // X: pixels xpx0, xpx0+16, chunk
  const int kc = kt * BKC + xch * 8;
  const int kh = kc / (4 * p.Cin);
  const int rem = kc - kh * 4 * p.Cin;
  const int kw = rem / p.Cin, ci = rem - kw * p.Cin;
  PixelCursor c0, c1;
  c0.init(m_begin + xpx0, p.Ho, p.Wo);
  c1.init(m_begin + xpx0 + 16, p.Ho, p.Wo);

  const __amdgpu_buffer_rsrc_t rs_x = make_rsrc(p.x, int64_t(p.N) * p.H * p.W * p.Cin * 2);
  const __amdgpu_buffer_rsrc_t rs_dy = make_rsrc(p.dy, p.M * p.Cout * 2);
  // Stage loads run kDepth stages ahead of the MFMAs in a register ring (one
  // block per CU: nothing else would hide the ~0.8 us load latency).  Stages
  // past the slice load out of range (zeros, no memory traffic), so the loop
  // has no tail and the compiler keeps counted vmcnt waits.
  constexpr int kDepth = 4;
  struct Stage {
    uint4 dy, x0, x1;
  };
  Stage ring[kDepth];
  int md = m_begin + dpx;                                           // this thread's dY pixel
  uint32_t dy_byte = uint32_t(md) * uint32_t(p.Cout * 2) + uint32_t((co0 + dch * 8) * 2);
  const uint32_t dy_step = uint32_t(BPX * p.Cout * 2);
  int mx = m_begin + xpx0;                                          // X pixels mx, mx + 16
  const int row_elems = p.W * p.Cin;
  auto xload = [&](const PixelCursor& c, int m) {
    const int ih = 2 * c.oh - 1 + kh, iw = 2 * c.ow - 1 + kw;
    const bool ok = m < m_end && unsigned(ih) < unsigned(p.H) && unsigned(iw) < unsigned(p.W);
    const int e = (c.n * p.H + ih) * row_elems + iw * p.Cin + ci;
    return bload(rs_x, ok ? uint32_t(e) * 2u : kOOB);
  };
  auto load = [&](Stage& r) {
    r.dy = bload(rs_dy, md < m_end ? dy_byte : kOOB);
    r.x0 = xload(c0, mx);
    r.x1 = xload(c1, mx + 16);
    md += BPX;
    dy_byte += dy_step;
    mx += BPX;
    c0.advance(p.Ho, p.Wo);
    c1.advance(p.Ho, p.Wo);
  };
  const int st_dy = dy_off(dpx, dch * 16), st_x0 = DY_TILE + x_off(xpx0, xch * 16),
            st_x1 = DY_TILE + x_off(xpx0 + 16, xch * 16);
  auto store = [&](const Stage& r, int buf) {
    char* base = smem + buf * STAGE;
    *reinterpret_cast<uint4*>(base + st_dy) = r.dy;
    *reinterpret_cast<uint4*>(base + st_x0) = r.x0;
    *reinterpret_cast<uint4*>(base + st_x1) = r.x1;
  };

  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int wco = (wave >> 1) * 32, wkc = (wave & 1) * 64;
  // per-lane transposed-read offsets (loop invariant): row 8g+q, columns col+4p
  int ra[2], rb[4];
  {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
#pragma unroll
    for (int i = 0; i < 2; ++i) ra[i] = dy_off(8 * g + q, (wco + 16 * i + 4 * pp) * 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) rb[j] = x_off(8 * g + q, (wkc + 16 * j + 4 * pp) * 2);
  }
#pragma unroll
  for (int u = 0; u < kDepth; ++u) load(ring[u]);
  const int padded = (nsteps + kDepth - 1) / kDepth * kDepth;
  for (int s0 = 0; s0 < padded; s0 += kDepth) {
#pragma unroll
    for (int u = 0; u < kDepth; ++u) {
      const int buf = u & 1;   // kDepth is even: (s0 + u) & 1
      store(ring[u], buf);     // waits for this stage's loads only (counted vmcnt)
      // LDS-only barrier: the ring's later stages stay in flight across it
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      load(ring[u]);           // stage s + kDepth
      const char* base = smem + buf * STAGE;
      bf16x8 a[2], bm[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = frag_at(base, ra[i], 4 * DY_ROW);
#pragma unroll
      for (int j = 0; j < 4; ++j) bm[j] = frag_at(base + DY_TILE, rb[j], 4 * X_ROW);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bm[j], acc[i][j], 0, 0, 0);
    }
  }

  // C/D map of 16x16x32: column = lane & 15 (kc), row = 4 * (lane >> 4) + reg (co)
  float* out = p.partial + int64_t(slice) * p.Cout * KC;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wco + 16 * i + 4 * (lane >> 4) + r;
        const int col = kt * BKC + wkc + 16 * j + (lane & 15);
        out[int64_t(co) * KC + col] = acc[i][j][r];
      }
}

// Sum the S slices into fp32 dW[co][kh][kw][ci] at the parameter's strides.
// blockIdx.y takes a group of kSliceGroup slices and each lane four
// consecutive elements (one 16-byte load per slice, all of a group's loads
// independent and in flight together); groups add into the zeroed output
// with float atomics (S / kSliceGroup adds per element).  One lane per
// element walking all S slices serially was latency-bound (17 us at S = 64).
constexpr int kSliceGroup = 8;

__global__ __launch_bounds__(kThreads) void conv_wgrad_reduce_kernel(const float* __restrict__ partial, int S,
                                                                     int Cout, int Cin, float* __restrict__ out,
                                                                     int64_t s_co, int64_t s_ci, int64_t s_kh,
                                                                     int64_t s_kw) {
  const int KC = 16 * Cin;
  const int total = Cout * KC;
  const int e0 = (int(blockIdx.x) * kThreads + int(threadIdx.x)) * 4;
  if (e0 >= total) return;
  const int k0 = int(blockIdx.y) * kSliceGroup;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int k = 0; k < kSliceGroup; ++k) {
    if (k0 + k < S) {
      const float4 v = *reinterpret_cast<const float4*>(partial + int64_t(k0 + k) * total + e0);
      acc.x += v.x, acc.y += v.y, acc.z += v.z, acc.w += v.w;
    }
  }
  const float vals[4] = {acc.x, acc.y, acc.z, acc.w};
  const bool single = S <= kSliceGroup;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = e0 + j;
    const int co = e / KC, kc = e - co * KC;
    const int tap = kc / Cin, ci = kc - tap * Cin;
    float* dst = out + co * s_co + ci * s_ci + (tap >> 2) * s_kh + (tap & 3) * s_kw;
    if (single) *dst = vals[j];
    else atomicAdd(dst, vals[j]);
  }
}


// ---------------------------------------------------------------------------
// Forward: y[m][co] = sum_kc X_im2col[m][kc] * W[co][kc], with the BatchNorm
// statistics of y (per-channel sum and sum of squares of the bf16-rounded
// outputs) reduced in the epilogue into one partial row per pixel tile -- the
// rows bn_finalize folds, so the separate BN reduction pass over y is gone.
// Both MFMA operands have K (kc) contiguous in memory here (an im2col row is
// 4 neighbouring input pixels' channels; a channels-last weight row is
// [kh][kw][ci]), so tiles are staged as plain 128-byte LDS rows (16-byte
// chunks XOR-swizzled by row) and read with ds_read_b128.

constexpr int FBM = 128;   // pixels per block
constexpr int FBN = 64;    // output channels per block
constexpr int FBK = 64;    // kc per k-step
constexpr int F_ROW = FBK * 2;                  // 128-byte LDS rows
constexpr int FA_TILE = FBM * F_ROW;            // 16 KiB
constexpr int FB_TILE = FBN * F_ROW;            // 8 KiB
constexpr int F_STAGE = FA_TILE + FB_TILE;

__device__ __forceinline__ int f_off(int r, int chunk) { return r * F_ROW + ((chunk ^ (r & 7)) << 4); }

__global__ __launch_bounds__(kThreads) void conv_fwd_kernel(ConvFwdParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * F_STAGE + 2 * 2 * FBN * 4];
  float* red = reinterpret_cast<float*>(smem + 2 * F_STAGE);   // [2 waves in m][2][FBN]
  const int t = int(threadIdx.x), lane = t & 63, wave = t >> 6;
  const int K = 16 * p.Cin, NT = p.Cout / FBN;
  const int64_t MT = (p.M + FBM - 1) / FBM;

  const int nwg = int(gridDim.x), b = int(blockIdx.x);
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int w = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int mt = w / NT, co0 = (w - mt * NT) * FBN;
  const int64_t m0 = int64_t(mt) * FBM;

  // staging: A chunks rows ar + 32j (j = 0..3), B chunks rows ar + 32j (j = 0, 1); chunk ac
  const int ar = t >> 3, ac = t & 7;
  int pn[4], poh[4], pow_[4];
  bool pin[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t m = m0 + ar + 32 * j;
    pin[j] = m < p.M;
    const int64_t mm = pin[j] ? m : 0;
    const int64_t hw = int64_t(p.Ho) * p.Wo;
    pn[j] = int(mm / hw);
    const int r = int(mm - int64_t(pn[j]) * hw);
    poh[j] = r / p.Wo;
    pow_[j] = r - poh[j] * p.Wo;
  }
  const __amdgpu_buffer_rsrc_t rs_x = make_rsrc(p.x, int64_t(p.N) * p.H * p.W * p.Cin * 2);
  uint4 ra[4], rb0, rb1;
  auto load = [&](int ks) {
    const int kc = ks * FBK + ac * 8;
    const int kh = kc / (4 * p.Cin), rem = kc - kh * 4 * p.Cin;
    const int kw = rem / p.Cin, ci = rem - kw * p.Cin;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ih = 2 * poh[j] - 1 + kh, iw = 2 * pow_[j] - 1 + kw;
      const bool ok = pin[j] && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
      ra[j] = bload(rs_x, ok ? uint32_t((((int64_t(pn[j]) * p.H + ih) * p.W + iw) * p.Cin + ci) * 2) : kOOB);
    }
    rb0 = *reinterpret_cast<const uint4*>(p.w + int64_t(co0 + ar) * K + kc);
    rb1 = *reinterpret_cast<const uint4*>(p.w + int64_t(co0 + ar + 32) * K + kc);
  };
  auto store = [&](int buf) {
    char* ai = smem + buf * F_STAGE;
    char* bi = ai + FA_TILE;
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<uint4*>(ai + f_off(ar + 32 * j, ac)) = ra[j];
    *reinterpret_cast<uint4*>(bi + f_off(ar, ac)) = rb0;
    *reinterpret_cast<uint4*>(bi + f_off(ar + 32, ac)) = rb1;
  };

  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wm = wave >> 1, wn = wave & 1;
  const int nsteps = K / FBK;
  load(0);
  store(0);
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    if (s + 1 < nsteps) load(s + 1);
    const char* ai = smem + (s & 1) * F_STAGE;
    const char* bi = ai + FA_TILE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = 4 * kk + (lane >> 4);
      bf16x8 a[4], bb[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 64 + 16 * i + (lane & 15);
        a[i] = *reinterpret_cast<const bf16x8*>(ai + f_off(r, chunk));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wn * 32 + 16 * j + (lane & 15);
        bb[j] = *reinterpret_cast<const bf16x8*>(bi + f_off(r, chunk));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bb[j], acc[i][j], 0, 0, 0);
    }
    if (s + 1 < nsteps) store((s + 1) & 1);
    __syncthreads();
  }

  // epilogue: bf16 y (RNE), and BN sums of the rounded values per channel
  float sum[2] = {0.f, 0.f}, sq[2] = {0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm * 64 + 16 * i + 4 * (lane >> 4) + r;
        const int co = co0 + wn * 32 + 16 * j + (lane & 15);
        const float v = acc[i][j][r];
        uint32_t u = __float_as_uint(v);
        u += 0x7FFFu + ((u >> 16) & 1u);               // round to nearest even (finite values)
        const uint16_t h = uint16_t(u >> 16);
        if (m < p.M) {
          p.y[m * p.Cout + co] = h;
          const float vr = __uint_as_float(uint32_t(h) << 16);
          sum[j] += vr;
          sq[j] += vr * vr;
        }
      }
  if (p.stats) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {   // lanes l, l^16, l^32, l^48 hold the same channel
      sum[j] += __shfl_xor(sum[j], 16);
      sum[j] += __shfl_xor(sum[j], 32);
      sq[j] += __shfl_xor(sq[j], 16);
      sq[j] += __shfl_xor(sq[j], 32);
    }
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        red[(wm * 2 + 0) * FBN + wn * 32 + 16 * j + lane] = sum[j];
        red[(wm * 2 + 1) * FBN + wn * 32 + 16 * j + lane] = sq[j];
      }
    }
    __syncthreads();
    if (t < 2 * FBN) {
      const int which = t / FBN, c = t - which * FBN;   // 0: sum, 1: sum of squares
      const float v = red[which * FBN + c] + red[(2 + which) * FBN + c];
      p.stats[int64_t(mt) * 2 * p.Cout + which * p.Cout + co0 + c] = v;
    }
  }
  (void)MT;
}

}  // namespace

bool conv_wgrad_supported(int Cin, int Cout) { return Cin >= 32 && Cin % 32 == 0 && Cout >= 64 && Cout % 64 == 0; }

int conv_wgrad_slices(int64_t M, int Cin, int Cout, int target_blocks) {
  if (!conv_wgrad_supported(Cin, Cout) || M <= 0) return 0;
  const int64_t tiles = int64_t(Cout / BCO) * (16 * Cin / BKC);
  int64_t s = (target_blocks + tiles - 1) / tiles;
  const int64_t max_s = (M + BPX - 1) / BPX;
  s = s < 1 ? 1 : (s > max_s ? max_s : s);
  return int(s);
}

hipError_t conv_wgrad(const ConvWgradParams& p, float* out, int64_t s_co, int64_t s_ci, int64_t s_kh, int64_t s_kw,
                      hipStream_t stream) {
  if (!conv_wgrad_supported(p.Cin, p.Cout) || p.slices <= 0 || !p.x || !p.dy || !p.partial || !out)
    return hipErrorInvalidValue;
  if (p.Ho != (p.H + 2 - 4) / 2 + 1 || p.Wo != (p.W + 2 - 4) / 2 + 1 || p.M != int64_t(p.N) * p.Ho * p.Wo)
    return hipErrorInvalidValue;   // 4x4 / stride 2 / pad 1 only
  if (p.px_per_slice <= 0 || p.px_per_slice % BPX != 0 || int64_t(p.slices) * p.px_per_slice < p.M)
    return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(p.x) | reinterpret_cast<uintptr_t>(p.dy)) & 15) return hipErrorInvalidValue;
  if (int64_t(p.N) * p.H * p.W * p.Cin * 2 >= int64_t(kOOB) || p.M * p.Cout * 2 >= int64_t(kOOB))
    return hipErrorInvalidValue;   // 32-bit buffer offsets
  const int64_t tiles = int64_t(p.Cout / BCO) * (16 * p.Cin / BKC);
  const int64_t blocks = tiles * p.slices;
  if (blocks > (int64_t(1) << 31) - 1) return hipErrorInvalidValue;
  conv_wgrad_kernel<<<unsigned(blocks), kThreads, 0, stream>>>(p);
  const int64_t total = int64_t(p.Cout) * 16 * p.Cin;   // multiple of 4 * kThreads? not needed: lanes past it return
  if (p.slices > kSliceGroup) {
    // groups add atomically: start from zero (out is dense: contiguous or channels-last)
    const hipError_t e = hipMemsetAsync(out, 0, size_t(total) * sizeof(float), stream);
    if (e != hipSuccess) return e;
  }
  const dim3 rgrid(unsigned((total / 4 + kThreads - 1) / kThreads), unsigned((p.slices + kSliceGroup - 1) / kSliceGroup));
  conv_wgrad_reduce_kernel<<<rgrid, kThreads, 0, stream>>>(p.partial, p.slices, p.Cout, p.Cin, out, s_co, s_ci,
                                                           s_kh, s_kw);
  return hipGetLastError();
}

bool conv_fwd_supported(int Cin, int Cout) { return Cin >= 8 && Cin % 8 == 0 && (16 * Cin) % FBK == 0 && Cout % FBN == 0; }

int64_t conv_fwd_tiles(int64_t M) { return (M + FBM - 1) / FBM; }

hipError_t conv_fwd(const ConvFwdParams& p, hipStream_t stream) {
  if (!conv_fwd_supported(p.Cin, p.Cout) || !p.x || !p.w || !p.y) return hipErrorInvalidValue;
  if (p.Ho != (p.H + 2 - 4) / 2 + 1 || p.Wo != (p.W + 2 - 4) / 2 + 1 || p.M != int64_t(p.N) * p.Ho * p.Wo)
    return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(p.x) | reinterpret_cast<uintptr_t>(p.w)) & 15) return hipErrorInvalidValue;
  if (int64_t(p.N) * p.H * p.W * p.Cin * 2 >= int64_t(kOOB)) return hipErrorInvalidValue;   // 32-bit buffer offsets
  const int64_t blocks = conv_fwd_tiles(p.M) * (p.Cout / FBN);
  if (blocks > (int64_t(1) << 31) - 1) return hipErrorInvalidValue;
  conv_fwd_kernel<<<unsigned(blocks), kThreads, 0, stream>>>(p);
  return hipGetLastError();
}

}  // namespace gpu
}  // namespace btn
