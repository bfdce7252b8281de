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

#include <algorithm>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <type_traits>
#include <vector>

#include "adam_sched.h"
#include "bn_fold.h"
#include "kernels.h"
#include "wgrad_reduce.h"

namespace btn {
namespace gpu {
namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
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

// (base and size are block-uniform at every call site; readfirstlane makes
// that visible to the compiler -- where its divergence analysis could not
// prove it (the first layer's `lut ? 1 : 2` byte size), every buffer load of
// the kernel became a waterfall loop with a full memory wait)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int64_t bytes) {
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(b)), hi = __builtin_amdgcn_readfirstlane(uint32_t(b >> 32));
  const int n = __builtin_amdgcn_readfirstlane(int(bytes));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((uint64_t(hi) << 32) | lo), 0, n, 0x00020000);
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

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint2 bload8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, int(off), 0, 0);
  return make_uint2(v[0], v[1]);
}
__device__ __forceinline__ uint32_t bload4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, int(off), 0, 0);
}

// First layer fed the RAW u8 RGBA frames (decode fused into the convolution):
// a pixel's 4 bytes become 4 bf16 values through the decode's value table,
// RNE-rounded to bf16 ([4][256], 2 KB, staged in LDS per block) -- exactly
// what the decode kernel writes for a bf16 NHWC RGBA output.  Padding pixels
// stay zero (not table[0]).
constexpr int kLutBytes = 4 * 256 * 2;
__device__ __forceinline__ void stage_lut(const uint16_t* lut, char* lds) {
  const int t = int(threadIdx.x);   // 256 threads x 8 bytes (threads past 256: nothing)
  if (t < 256) *reinterpret_cast<uint2*>(lds + 8 * t) = *reinterpret_cast<const uint2*>(lut + 4 * t);
}
__device__ __forceinline__ uint2 lut_px(const char* lds, uint32_t w, bool ok) {
  const uint16_t* l = reinterpret_cast<const uint16_t*>(lds);
  if (!ok) return make_uint2(0u, 0u);
  return make_uint2(uint32_t(l[w & 255u]) | (uint32_t(l[256 + ((w >> 8) & 255u)]) << 16),
                    uint32_t(l[512 + ((w >> 16) & 255u)]) | (uint32_t(l[768 + (w >> 24)]) << 16));
}

// The slice-reduce adds slice groups atomically into the gradient, which must
// start at zero: the weight-gradient kernel clears it (every block a share,
// plain stores) -- the reduce runs after it on the stream, so no separate
// memset launch is needed.
__device__ __forceinline__ int main_blocks(const ConvWgradParams& p) {
  return p.main_blocks > 0 ? p.main_blocks : int(gridDim.x);
}

// bid: the block's index in the weight gradient's own grid (blockIdx.x, or its
// place in a launch shared with a data gradient: dgrad_wgrad_kernel)
__device__ __forceinline__ void zero_output(const ConvWgradParams& p, int bid) {
  if (!p.zero_out) return;
  const int per = (p.zero_count + main_blocks(p) - 1) / main_blocks(p);
  const int e0 = bid * per, e1 = e0 + per < p.zero_count ? e0 + per : p.zero_count;
  for (int e = e0 + int(threadIdx.x); e < e1; e += int(blockDim.x)) p.zero_out[e] = 0.f;
}
__device__ __forceinline__ void zero_output(const ConvWgradParams& p) { zero_output(p, int(blockIdx.x)); }

// Sum the S slices into fp32 dW[co][kh][kw][ci] at the parameter's strides.
// blockIdx.y takes a group of kSliceGroup slices and each lane four
// consecutive elements (one 16-byte load per slice, all of a group's loads
// independent and in flight together); groups add into the zeroed output
// with float atomics (S / kSliceGroup adds per element).  One lane per
// element walking all S slices serially was latency-bound (17 us at S = 64).
constexpr int kSliceGroup = 8;   // (groups of 32 for the first layer's 512 slices -- 16 atomics per
                                 // element instead of 64 -- measured slower: 8.4 -> 11.0 us)

// The ordered form (r.sub > 0, the default; BT_WGRAD_ORDERED=0: the atomic
// groups above): bit-identical gradients run to run.  Lane groups of `sub`
// (a power of two <= 64, <= S) share 4 elements; lane `part` of a group sums
// slices part, part + sub, ... in that order, 8 loads in flight, then the
// group adds its lanes with a fixed xor-shuffle tree (commutative adds: every
// lane ends with the same bits) and lane 0 stores.  Same bytes read as the
// atomic form, no zeroing of the output, no atomics (wgrad_reduce.h).
__device__ __forceinline__ void wgrad_reduce_ordered(const ConvWgradParams::Reduce& r, int bx) {
  wgrad_slice_sum<kThreads, kSliceGroup>(r, bx, [&](int e0, float4 acc) {
    const int Cin = r.Cin, KC = 16 * Cin;
    const float vals[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = e0 + j;
      const int co = e / KC, kc = e - co * KC;
      const int tap = kc / Cin, ci = kc - tap * Cin;
      if (ci >= r.cin_out) continue;
      r.out[co * r.s_co + ci * r.s_ci + (tap >> 2) * r.s_kh + (tap & 3) * r.s_kw] = vals[j];
    }
  });
}

__device__ __forceinline__ void wgrad_reduce_block(const ConvWgradParams::Reduce& r, int bx, int by) {
  if (r.sub > 0) {
    wgrad_reduce_ordered(r, bx);
    return;
  }
  const float* __restrict__ partial = r.partial;
  const int S = r.S, Cin = r.Cin, cin_out = r.cin_out;
  float* __restrict__ out = r.out;
  const int KC = 16 * Cin;
  const int total = r.Cout * KC;
  if (int(threadIdx.x) >= kThreads) return;   // (a side job of a wider block: 256 lanes do it)
  const int e0 = (bx * kThreads + int(threadIdx.x)) * 4;
  if (e0 >= total) return;
  const int k0 = by * kSliceGroup;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  // all of the group's loads in flight at once (past the last slice: re-read
  // slice k0, not added); a guarded load per slice compiled to a branch and a
  // memory wait each -- 8 round trips
  float4 v[kSliceGroup];
#pragma unroll
  for (int k = 0; k < kSliceGroup; ++k)
    v[k] = *reinterpret_cast<const float4*>(partial + int64_t(k0 + k < S ? k0 + k : k0) * total + e0);
#pragma unroll
  for (int k = 0; k < kSliceGroup; ++k)
    if (k0 + k < S) acc.x += v[k].x, acc.y += v[k].y, acc.z += v[k].z, acc.w += v[k].w;
  const float vals[4] = {acc.x, acc.y, acc.z, acc.w};
  const bool single = S <= kSliceGroup;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = e0 + j;
    const int co = e / KC, kc = e - co * KC;
    const int tap = kc / Cin, ci = kc - tap * Cin;
    if (ci >= cin_out) continue;   // padded input channel (4-channel first layer)
    float* dst = out + co * r.s_co + ci * r.s_ci + (tap >> 2) * r.s_kh + (tap & 3) * r.s_kw;
    if (single) *dst = vals[j];
    else atomicAdd(dst, vals[j]);
  }
}

// job: an attached Adam schedule (adam_sched.h), run by the first lane
__global__ __launch_bounds__(kThreads) void conv_wgrad_reduce_kernel(ConvWgradParams::Reduce r, AdamSchedJob job) {
  if (job.step && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) adam_schedule_run(job);
  wgrad_reduce_block(r, int(blockIdx.x), int(blockIdx.y));
}

namespace {
AdamSchedJob g_sched_job;     // attached, not yet launched
int g_sched_device = -1;      // the optimizer's device and stream: the only launches that take it
hipStream_t g_sched_stream = nullptr;
bool g_sched_taken = false;   // a launch ran the attached job
// BT_SCHED_EARLY (default on): the first fused data + weight gradient launch takes the job
// (dgrad_wgrad_kernel), 0: the slice reduce
bool sched_early() {
  static const bool on = [] {
    const char* v = std::getenv("BT_SCHED_EARLY");
    return !v || v[0] != '0';
  }();
  return on;
}
AdamSchedJob take_sched_job(hipStream_t stream) {
  if (!g_sched_job.step || stream != g_sched_stream) return AdamSchedJob();
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev != g_sched_device) return AdamSchedJob();
  AdamSchedJob j = g_sched_job;
  g_sched_taken = true;
  g_sched_job = AdamSchedJob();
  return j;
}
}  // namespace

// (conv_attach_adam_schedule / _taken / _detach: after this file's internal namespace)

// blocks past the main grid: a previous layer's deferred reduce (the side
// job), then -- one block -- the BN statistics fold the preceding data
// gradient's epilogue accumulated (ConvWgradParams::fold)
__device__ __forceinline__ bool run_side(const ConvWgradParams& p, char* lds, int bid) {
  int b = bid - main_blocks(p);
  if (b < 0) return false;
  const int nred = p.side.partial ? p.side.rx * p.side.ry : 0;
  if (b < nred) {
    wgrad_reduce_block(p.side, b % p.side.rx, b / p.side.rx);
    return true;
  }
  BnFold f;
  f.acc = p.fold.acc, f.R = p.fold.R, f.C = p.fold.C, f.M = p.fold.M, f.bwd = 1;
  f.o0 = p.fold.db, f.o1 = p.fold.dw;
  bn_fold_block(f, reinterpret_cast<double*>(lds));
  return true;
}
__device__ __forceinline__ bool run_side(const ConvWgradParams& p, char* lds) {
  return run_side(p, lds, int(blockIdx.x));
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

// One X pixel's im2col source for a thread's fixed (kh, kw, ci), advanced BPX
// output pixels per k-step: the element offset moves by constant jumps (next
// column block, next row, next image), so a k-step costs a few adds and
// selects -- recomputing (n, ih, iw) -> offset with multiplies, and the
// divergent while loop of PixelCursor, made this kernel VALU-bound.
struct XCursor {
  int oh, ow, e;
  __device__ void init(int m, const ConvWgradParams& p, int kh, int kw, int ci) {
    const int hw = p.Ho * p.Wo;
    const int n = m / hw, r = m - n * hw;
    oh = r / p.Wo;
    ow = r - oh * p.Wo;
    e = (n * p.H + 2 * oh - 1 + kh) * (p.W * p.Cin) + (2 * ow - 1 + kw) * p.Cin + ci;
  }
  // col = 2 BPX Cin, row = 2 W Cin - 2 Wo Cin, img = (H - 2 Ho) W Cin;
  // single: Wo >= BPX (block-uniform), so at most one row wrap per step
  __device__ void advance(int Ho, int Wo, int col, int row, int img, bool single) {
    ow += BPX;
    e += col;
    if (single) {
      const bool wr = ow >= Wo;
      ow = wr ? ow - Wo : ow;
      e = wr ? e + row : e;
      oh += wr ? 1 : 0;
      const bool wi = oh == Ho;
      oh = wi ? 0 : oh;
      e = wi ? e + img : e;
    } else {
      while (ow >= Wo) {
        ow -= Wo;
        e += row;
        if (++oh == Ho) oh = 0, e += img;
      }
    }
  }
};

// BND: the BN backward applied to dY (ConvWgradParams::bn_dy) -- its
// coefficients and ring cost ~80 VGPRs, so the plain variant stays lean.
// PIPE: the next step's fragments are read right after the barrier that
// publishes them, while this step's MFMAs run (two fragment sets, +24 VGPRs):
// without it every step waited out barrier -> LDS read latency -> MFMAs in turn.
constexpr int kWgradLds = 2 * STAGE;
template <bool BND, bool PIPE = false>
__device__ __forceinline__ void conv_wgrad_body(const ConvWgradParams& p, char* smem, int bid) {
  if (run_side(p, smem, bid)) return;
  const int t = int(threadIdx.x), lane = t & 63, wave = t >> 6;
  const int KC = 16 * p.Cin, KT = KC / BKC, T = (p.Cout / BCO) * KT;

  // XCD-aware bijective remap: consecutive work ids share an XCD (blockIdx % 8)
  const int nwg = main_blocks(p), b = bid;
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
  // X: one pixel per thread, its chunks xch and xch + 8 (im2col columns kc
  // and kc + 64): one pixel cursor feeds both loads
  const int xpx = t >> 3, xch = t & 7;
  const int kc = kt * BKC + xch * 8, kc1 = kc + 64;
  int kh, kw, ci, kh1, kw1, ci1;
  if ((p.Cin & (p.Cin - 1)) == 0) {   // power-of-two channels (block-uniform): shifts, not divisions
    const int cs = __builtin_ctz(unsigned(p.Cin));
    kh = kc >> (cs + 2), kw = (kc >> cs) & 3, ci = kc & (p.Cin - 1);
    kh1 = kc1 >> (cs + 2), kw1 = (kc1 >> cs) & 3, ci1 = kc1 & (p.Cin - 1);
  } else {
    kh = kc / (4 * p.Cin);
    const int rem = kc - kh * 4 * p.Cin;
    kw = rem / p.Cin, ci = rem - kw * p.Cin;
    kh1 = kc1 / (4 * p.Cin);
    const int rem1 = kc1 - kh1 * 4 * p.Cin;
    kw1 = rem1 / p.Cin, ci1 = rem1 - kw1 * p.Cin;
  }
  const int dkh = kh1 - kh, dkw = kw1 - kw;
  const int de = (dkh * p.W + dkw) * p.Cin + (ci1 - ci);   // element offset of the second chunk
  XCursor c0;
  c0.init(m_begin + xpx, p, kh, kw, ci);
  const int j_col = 2 * BPX * p.Cin, j_row = 2 * (p.W - p.Wo) * p.Cin, j_img = (p.H - 2 * p.Ho) * p.W * p.Cin;
  const bool single = p.Wo >= BPX;

  const __amdgpu_buffer_rsrc_t rs_x = make_rsrc(p.x, int64_t(p.N) * p.H * p.W * p.Cin * 2);
  const __amdgpu_buffer_rsrc_t rs_dy = make_rsrc(p.dy, p.M * p.Cout * 2);
  // bn_dy: dy is the gradient of the BatchNorm+LeakyReLU that follows this
  // layer; its backward (BnBwdCoef, the apply kernel's arithmetic) is applied
  // to the staged dY chunk, which the first column tile's blocks also store
  // to gx_out (the next data gradient's operand)
  constexpr bool bnd = BND;
  BnBwdCoef bc[8];
  if (bnd) {   // (LDS scratch: the staging area, free until the loop)
    bn_dy_coefs(p.bn_dy, p.Cout, p.M, co0 + dch * 8, reinterpret_cast<double*>(smem),
                reinterpret_cast<int*>(smem + 4096), unsigned(b), unsigned(nwg), bc);
    __syncthreads();
  }
  const __amdgpu_buffer_rsrc_t rs_by = make_rsrc(bnd ? p.bn_dy.y : p.dy, p.M * p.Cout * 2);
  uint16_t* const gx_out = bnd && kt == 0 ? p.bn_dy.gx_out : nullptr;
  // Stage loads run kDepth stages ahead of the MFMAs in a register ring (one
  // block per CU: nothing else would hide the ~0.8 us load latency).  Stages
  // past the slice load out of range (zeros, no memory traffic), so the loop
  // has no tail and the compiler keeps counted vmcnt waits.
  constexpr int kDepth = 4;
  struct Stage {
    uint4 dy, x0, x1, y;   // y: the BN input at the dY chunk (bn_dy)
    uint32_t off;          // the dY chunk's byte offset, kOOB past the slice
  };
  Stage ring[kDepth];
  int md = m_begin + dpx;                                           // this thread's dY pixel
  uint32_t dy_byte = uint32_t(md) * uint32_t(p.Cout * 2) + uint32_t((co0 + dch * 8) * 2);
  const uint32_t dy_step = uint32_t(BPX * p.Cout * 2);
  // X needs no slice-end test: a pixel past the slice pairs with a zero dY
  // chunk (out-of-range dY loads return 0), and past the tensor the X load is
  // out of range too
  auto load = [&](Stage& r) {
    r.off = md < m_end ? dy_byte : kOOB;
    r.dy = bload(rs_dy, r.off);
    if (bnd) r.y = bload(rs_by, r.off);
    const int ih = 2 * c0.oh - 1 + kh, iw = 2 * c0.ow - 1 + kw;
    const bool ok0 = unsigned(ih) < unsigned(p.H) && unsigned(iw) < unsigned(p.W);
    const bool ok1 = unsigned(ih + dkh) < unsigned(p.H) && unsigned(iw + dkw) < unsigned(p.W);
    r.x0 = bload(rs_x, ok0 ? uint32_t(c0.e) * 2u : kOOB);
    r.x1 = bload(rs_x, ok1 ? uint32_t(c0.e + de) * 2u : kOOB);
    md += BPX;
    dy_byte += dy_step;
    c0.advance(p.Ho, p.Wo, j_col, j_row, j_img, single);
  };
  const int st_dy = dy_off(dpx, dch * 16), st_x0 = DY_TILE + x_off(xpx, xch * 16),
            st_x1 = DY_TILE + x_off(xpx, (xch + 8) * 16);
  const float slope = p.bn_dy.slope;
  auto store = [&](const Stage& r, int buf) {
    char* base = smem + buf * STAGE;
    uint4 d = r.dy;
    if (bnd) {   // gx of the 8 channels (rows past the slice stay zero, not gx(0, 0))
      if (r.off != kOOB) {
        const uint32_t gw[4] = {r.dy.x, r.dy.y, r.dy.z, r.dy.w}, yw[4] = {r.y.x, r.y.y, r.y.z, r.y.w};
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x2 pr = {bc[2 * q].gx(__uint_as_float(yw[q] << 16), __uint_as_float(gw[q] << 16), slope),
                            bc[2 * q + 1].gx(__uint_as_float(yw[q] & 0xFFFF0000u),
                                             __uint_as_float(gw[q] & 0xFFFF0000u), slope)};
          o[q] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pr, bf16x2));
        }
        d = make_uint4(o[0], o[1], o[2], o[3]);
        if (gx_out) *reinterpret_cast<uint4*>(reinterpret_cast<char*>(gx_out) + r.off) = d;
      }
    }
    *reinterpret_cast<uint4*>(base + st_dy) = d;
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
  auto frags = [&](int buf, bf16x8 (&a)[2], bf16x8 (&bm)[4]) {
    const char* base = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < 2; ++i) a[i] = frag_at(base, ra[i], 4 * DY_ROW);
#pragma unroll
    for (int j = 0; j < 4; ++j) bm[j] = frag_at(base + DY_TILE, rb[j], 4 * X_ROW);
  };
  auto mma = [&](const bf16x8 (&a)[2], const bf16x8 (&bm)[4]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bm[j], acc[i][j], 0, 0, 0);
  };
  if constexpr (PIPE) {
    // ring slot k holds step s0 + k; iteration (s0, u) stores step s0 + u + 1,
    // refills its slot with step s0 + u + 1 + kDepth, reads its fragments and
    // runs step s0 + u's MFMAs (fragments read one iteration earlier).  The
    // lgkmcnt(0) before each barrier also retires every wave's fragment reads
    // of the buffer the next store overwrites.  Past the slice the steps are
    // zeros (and the final extra store / load is never multiplied in).
    bf16x8 ac[2], bc4[4], an[2], bn[4];
    store(ring[0], 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    load(ring[0]);   // step kDepth
    frags(0, ac, bc4);
    for (int s0 = 0; s0 < padded; s0 += kDepth) {
#pragma unroll
      for (int u = 0; u < kDepth; ++u) {
        Stage& nx = ring[(u + 1) % kDepth];
        store(nx, (u + 1) & 1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        load(nx);
        frags((u + 1) & 1, an, bn);
        mma(ac, bc4);
#pragma unroll
        for (int i = 0; i < 2; ++i) ac[i] = an[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) bc4[j] = bn[j];
      }
    }
  } else {
    for (int s0 = 0; s0 < padded; s0 += kDepth) {
#pragma unroll
      for (int u = 0; u < kDepth; ++u) {
        const int buf = u & 1;   // kDepth is even: (s0 + u) & 1
        store(ring[u], buf);     // waits for this stage's loads only (counted vmcnt)
        // LDS-only barrier: the ring's later stages stay in flight across it
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        load(ring[u]);           // stage s + kDepth
        bf16x8 a[2], bm[4];
        frags(buf, a, bm);
        mma(a, bm);
      }
    }
  }

  // C/D map of 16x16x32: column = lane & 15 (kc), row = 4 * (lane >> 4) + reg (co)
  zero_output(p, bid);
  // 32-bit offsets from the lane's first element (the slice's partial block
  // is < 2^31 elements): one add per store instead of 64-bit address math
  float* out = p.partial + int64_t(slice) * p.Cout * KC + (co0 + wco + 4 * (lane >> 4)) * KC +
               (kt * BKC + wkc + (lane & 15));
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(16 * i + r) * KC + 16 * j] = acc[i][j][r];
}

// 128-channel tiles (BT_WGRAD_CO128, layers with Cout % 128 == 0): a block's
// tile is 128 output channels x 128 im2col columns, 4 waves of 64 x 64 (16
// MFMAs per wave and 32-pixel step instead of 8).  Every staged X chunk then
// feeds twice the channels: per FLOP the block stages 2/3 of the bytes of the
// 64 x 128 tile (16 KiB per step for 2 MFLOP against 12 KiB for 1), and the
// L2 -> LDS fills are what the tap-gather GEMMs of this file wait on (the
// MFMAs of a step are 128 cycles per wave).  Plain variant only (no BN on dY).
constexpr int BCO2 = 128;
constexpr int DY2_ROW = BCO2 * 2;             // 256-byte LDS rows (x_off's swizzle)
constexpr int DY2_TILE = BPX * DY2_ROW;       // 8 KiB
constexpr int STAGE_CO2 = DY2_TILE + X_TILE;     // 16 KiB
constexpr int kWgrad2Lds = 2 * STAGE_CO2;

template <int kDepth = 2>
__device__ __forceinline__ void conv_wgrad_co128_body(const ConvWgradParams& p, char* smem, int bid) {
  if (run_side(p, smem, bid)) return;
  const int t = int(threadIdx.x), lane = t & 63, wave = t >> 6;
  const int KC = 16 * p.Cin, KT = KC / BKC, T = (p.Cout / BCO2) * KT;
  const int nwg = main_blocks(p), b = bid;
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int w = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int slice = w / T, tile = w - slice * T;
  const int co0 = (tile / KT) * BCO2, kt = tile - (tile / KT) * KT;
  const int m_begin = slice * int(p.px_per_slice);
  const int m_end = m_begin + int(p.px_per_slice) < int(p.M) ? m_begin + int(p.px_per_slice) : int(p.M);
  const int nsteps = m_end > m_begin ? (m_end - m_begin + BPX - 1) / BPX : 0;
  // staging: dY chunks of pixels dpx and dpx + 16 (16 chunks per 128-channel row), X as the 64-channel body
  const int dpx = t >> 4, dch = t & 15;
  const int xpx = t >> 3, xch = t & 7;
  const int kc = kt * BKC + xch * 8, kc1 = kc + 64;
  const int cs = __builtin_ctz(unsigned(p.Cin));   // (power-of-two channels: the host checks)
  const int kh = kc >> (cs + 2), kw = (kc >> cs) & 3, ci = kc & (p.Cin - 1);
  const int kh1 = kc1 >> (cs + 2), kw1 = (kc1 >> cs) & 3, ci1 = kc1 & (p.Cin - 1);
  const int dkh = kh1 - kh, dkw = kw1 - kw;
  const int de = (dkh * p.W + dkw) * p.Cin + (ci1 - ci);
  XCursor c0;
  c0.init(m_begin + xpx, p, kh, kw, ci);
  const int j_col = 2 * BPX * p.Cin, j_row = 2 * (p.W - p.Wo) * p.Cin, j_img = (p.H - 2 * p.Ho) * p.W * p.Cin;
  const bool single = p.Wo >= BPX;
  const __amdgpu_buffer_rsrc_t rs_x = make_rsrc(p.x, int64_t(p.N) * p.H * p.W * p.Cin * 2);
  const __amdgpu_buffer_rsrc_t rs_dy = make_rsrc(p.dy, p.M * p.Cout * 2);
  // (a 4-deep ring holds the fused launch at 2 waves per SIMD: 150 VGPRs + 88 AGPRs)
  static_assert(kDepth % 2 == 0, "even ring depth: step parity picks the LDS buffer");
  struct Stage {
    uint4 dy0, dy1, x0, x1;
  };
  Stage ring[kDepth];
  int md = m_begin + dpx;
  uint32_t dy_byte = uint32_t(md) * uint32_t(p.Cout * 2) + uint32_t((co0 + dch * 8) * 2);
  const uint32_t dy_step = uint32_t(BPX * p.Cout * 2), dy_half = uint32_t(16 * p.Cout * 2);
  auto load = [&](Stage& r) {
    r.dy0 = bload(rs_dy, md < m_end ? dy_byte : kOOB);
    r.dy1 = bload(rs_dy, md + 16 < m_end ? dy_byte + dy_half : kOOB);
    const int ih = 2 * c0.oh - 1 + kh, iw = 2 * c0.ow - 1 + kw;
    const bool ok0 = unsigned(ih) < unsigned(p.H) && unsigned(iw) < unsigned(p.W);
    const bool ok1 = unsigned(ih + dkh) < unsigned(p.H) && unsigned(iw + dkw) < unsigned(p.W);
    r.x0 = bload(rs_x, ok0 ? uint32_t(c0.e) * 2u : kOOB);
    r.x1 = bload(rs_x, ok1 ? uint32_t(c0.e + de) * 2u : kOOB);
    md += BPX;
    dy_byte += dy_step;
    c0.advance(p.Ho, p.Wo, j_col, j_row, j_img, single);
  };
  const int st_dy0 = x_off(dpx, dch * 16), st_dy1 = x_off(dpx + 16, dch * 16);
  const int st_x0 = DY2_TILE + x_off(xpx, xch * 16), st_x1 = DY2_TILE + x_off(xpx, (xch + 8) * 16);
  auto store = [&](const Stage& r, int buf) {
    char* base = smem + buf * STAGE_CO2;
    *reinterpret_cast<uint4*>(base + st_dy0) = r.dy0;
    *reinterpret_cast<uint4*>(base + st_dy1) = r.dy1;
    *reinterpret_cast<uint4*>(base + st_x0) = r.x0;
    *reinterpret_cast<uint4*>(base + st_x1) = r.x1;
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wco = (wave >> 1) * 64, wkc = (wave & 1) * 64;
  int ra[4], rb[4];
  {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
#pragma unroll
    for (int i = 0; i < 4; ++i) ra[i] = x_off(8 * g + q, (wco + 16 * i + 4 * pp) * 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) rb[j] = DY2_TILE + x_off(8 * g + q, (wkc + 16 * j + 4 * pp) * 2);
  }
#pragma unroll
  for (int u = 0; u < kDepth; ++u) load(ring[u]);
  const int padded = (nsteps + kDepth - 1) / kDepth * kDepth;
  for (int s0 = 0; s0 < padded; s0 += kDepth) {
#pragma unroll
    for (int u = 0; u < kDepth; ++u) {
      const int buf = u & 1;
      store(ring[u], buf);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      load(ring[u]);
      const char* base = smem + buf * STAGE_CO2;
      bf16x8 bm[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bm[j] = frag_at(base, rb[j], 4 * X_ROW);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 a = frag_at(base, ra[i], 4 * X_ROW);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bm[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  zero_output(p, bid);
  float* out = p.partial + int64_t(slice) * p.Cout * KC + (co0 + wco + 4 * (lane >> 4)) * KC +
               (kt * BKC + wkc + (lane & 15));
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(16 * i + r) * KC + 16 * j] = acc[i][j][r];
}

__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(3))) void conv_wgrad_co128_kernel(ConvWgradParams p) {
  __shared__ __attribute__((aligned(16))) char smem[kWgrad2Lds];
  conv_wgrad_co128_body<>(p, smem, int(blockIdx.x));
}

template <bool BND, bool PIPE = false>
__global__ __launch_bounds__(kThreads) void conv_wgrad_kernel(ConvWgradParams p) {
  __shared__ __attribute__((aligned(16))) char smem[kWgradLds];
  conv_wgrad_body<BND, PIPE>(p, smem, int(blockIdx.x));
}

// ---------------------------------------------------------------------------
// The weight gradient with 256-column im2col tiles (BT_WGRAD_WIDE).  The
// register-staged kernel above (128 columns, waves of 32 x 64) runs one
// barrier and 12 transposing fragment reads per 8 MFMAs per wave; here the
// waves are 2 (co) x 2 (kc) tiles of 32 x 128: 16 MFMAs and 20 reads per
// barrier, half the block tiles (and slices of the same length, so the
// same MFMAs per block).  X rows are 512 bytes: 16 windows of 32 bytes whose
// low 3 bits take the same XOR swizzle as x_off (every row starts at bank 0,
// so the 8 rows of a transposing read land on 8 windows).  Each thread
// stages one dY chunk and four X chunks (im2col columns 64 apart) per step
// from one pixel cursor.  Non-BN variant (the default path).
constexpr int BKC2 = 256;
constexpr int X2_ROW = BKC2 * 2;              // 512-byte LDS rows
constexpr int X2_TILE = BPX * X2_ROW;         // 16 KiB
constexpr int STAGE2 = DY_TILE + X2_TILE;     // 20 KiB
__device__ __forceinline__ int x2_off(int r, int byte) {
  const int f = (r & 3) | (((r >> 3) & 1) << 2);
  return r * X2_ROW + ((((byte >> 5) ^ f) << 5) | (byte & 31));
}

constexpr int kWgradWideLds = 2 * STAGE2;
// bid: the block's index in the weight gradient's own grid (a launch shared with
// the 32-channel patch data gradient: dpatch_wgrad_kernel<.., true>)
__device__ __forceinline__ void conv_wgrad_wide_body(const ConvWgradParams& p, char* smem, int bid) {
  if (run_side(p, smem, bid)) return;
  const int t = int(threadIdx.x), lane = t & 63, wave = t >> 6;
  const int KC = 16 * p.Cin, KT = KC / BKC2, T = (p.Cout / BCO) * KT;
  const int nwg = main_blocks(p), b = bid;
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int w = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int slice = w / T, tile = w - slice * T;
  const int co0 = (tile / KT) * BCO, kt = tile - (tile / KT) * KT;
  const int m_begin = slice * int(p.px_per_slice);
  const int m_end = m_begin + int(p.px_per_slice) < int(p.M) ? m_begin + int(p.px_per_slice) : int(p.M);
  const int nsteps = m_end > m_begin ? (m_end - m_begin + BPX - 1) / BPX : 0;

  const int dpx = t >> 3, dch = t & 7;   // dY: pixel, 16-byte chunk
  const int xpx = t >> 3, xch = t & 7;   // X: pixel, chunks xch + 8 i (columns kc0 + 64 i)
  const int cs = __builtin_ctz(unsigned(p.Cin));   // (host: power-of-two Cin)
  const int kc0 = kt * BKC2 + xch * 8;
  int dkh[4], dkw[4], de[4];
  const int kh = kc0 >> (cs + 2), kw = (kc0 >> cs) & 3, ci = kc0 & (p.Cin - 1);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int kc = kc0 + 64 * i;
    dkh[i] = (kc >> (cs + 2)) - kh;
    dkw[i] = ((kc >> cs) & 3) - kw;
    de[i] = (dkh[i] * p.W + dkw[i]) * p.Cin + ((kc & (p.Cin - 1)) - ci);
  }
  XCursor c0;
  c0.init(m_begin + xpx, p, kh, kw, ci);
  const int j_col = 2 * BPX * p.Cin, j_row = 2 * (p.W - p.Wo) * p.Cin, j_img = (p.H - 2 * p.Ho) * p.W * p.Cin;
  const bool single = p.Wo >= BPX;
  const __amdgpu_buffer_rsrc_t rs_x = make_rsrc(p.x, int64_t(p.N) * p.H * p.W * p.Cin * 2);
  const __amdgpu_buffer_rsrc_t rs_dy = make_rsrc(p.dy, p.M * p.Cout * 2);
  constexpr int kDepth = 2;   // (4 stages of 5 chunks: 276 registers, one wave per SIMD)
  struct Stage {
    uint4 dy, x[4];
  };
  Stage ring[kDepth];
  int md = m_begin + dpx;
  uint32_t dy_byte = uint32_t(md) * uint32_t(p.Cout * 2) + uint32_t((co0 + dch * 8) * 2);
  const uint32_t dy_step = uint32_t(BPX * p.Cout * 2);
  auto load = [&](Stage& r) __attribute__((always_inline)) {
    r.dy = bload(rs_dy, md < m_end ? dy_byte : kOOB);
    const int ih = 2 * c0.oh - 1 + kh, iw = 2 * c0.ow - 1 + kw;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool ok = unsigned(ih + dkh[i]) < unsigned(p.H) && unsigned(iw + dkw[i]) < unsigned(p.W);
      r.x[i] = bload(rs_x, ok ? uint32_t(c0.e + de[i]) * 2u : kOOB);
    }
    md += BPX;
    dy_byte += dy_step;
    c0.advance(p.Ho, p.Wo, j_col, j_row, j_img, single);
  };
  const int st_dy = dy_off(dpx, dch * 16);
  int st_x[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) st_x[i] = DY_TILE + x2_off(xpx, (xch + 8 * i) * 16);
  auto store = [&](const Stage& r, int buf) __attribute__((always_inline)) {
    char* base = smem + buf * STAGE2;
    *reinterpret_cast<uint4*>(base + st_dy) = r.dy;
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<uint4*>(base + st_x[i]) = r.x[i];
  };

  f32x4 acc[2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wco = (wave >> 1) * 32, wkc = (wave & 1) * 128;
  int ra[2], rb[8];
  {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
#pragma unroll
    for (int i = 0; i < 2; ++i) ra[i] = dy_off(8 * g + q, (wco + 16 * i + 4 * pp) * 2);
#pragma unroll
    for (int j = 0; j < 8; ++j) rb[j] = x2_off(8 * g + q, (wkc + 16 * j + 4 * pp) * 2);
  }
#pragma unroll
  for (int u = 0; u < kDepth; ++u) load(ring[u]);
  const int padded = (nsteps + kDepth - 1) / kDepth * kDepth;
  for (int s0 = 0; s0 < padded; s0 += kDepth) {
#pragma unroll
    for (int u = 0; u < kDepth; ++u) {
      const int buf = u & 1;
      store(ring[u], buf);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      load(ring[u]);
      const char* base = smem + buf * STAGE2;
      bf16x8 a[2], bm[8];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = frag_at(base, ra[i], 4 * DY_ROW);
#pragma unroll
      for (int j = 0; j < 8; ++j) bm[j] = frag_at(base + DY_TILE, rb[j], 4 * X2_ROW);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bm[j], acc[i][j], 0, 0, 0);
    }
  }
  zero_output(p, bid);
  float* out = p.partial + int64_t(slice) * p.Cout * KC + (co0 + wco + 4 * (lane >> 4)) * KC +
               (kt * BKC2 + wkc + (lane & 15));
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(16 * i + r) * KC + 16 * j] = acc[i][j][r];
}

__global__ __launch_bounds__(kThreads) void conv_wgrad_wide_kernel(ConvWgradParams p) {
  __shared__ __attribute__((aligned(16))) char smem[kWgradWideLds];
  conv_wgrad_wide_body(p, smem, int(blockIdx.x));
}

// ---------------------------------------------------------------------------
// The same weight gradient with LDS-DMA staging (buffer_load ... lds) and
// 64-pixel k-steps: the register path above stages every 16-byte chunk through
// VGPRs and ds_write (the kernel's VALU and LDS-store bound: 6.4 VALU per
// MFMA, 24 us per layer in the disc step) and barriers every 8 MFMAs.
//
// LDS image per stage: COLUMN blocks -- one 16-byte chunk column (8 channels)
// of the 64 pixels, 1 KiB, padded to 1088 B -- so one wave-instruction of
// LDS-DMA (lane l -> bytes 16 l of 1 KiB) lands 64 pixels of one chunk: lane l
// is pixel l of the step, every lane keeps ONE pixel cursor, and a wave's
// instructions are whole chunk columns (wave-uniform (kh, kw, ci), scalar).
// The transposing fragment read of 4 pixels x 16 columns (two column blocks)
// is conflict-free: within 32 lanes the 8-byte pieces sit at 128 g + 16 q
// (pixel) + 64 (block, from the 1088-byte pitch) + 8 (half chunk) mod 256.
constexpr int W2_BPX = 64;                        // pixels per k-step
constexpr int W2_COL = W2_BPX * 16 + 64;          // one column block, padded
constexpr int W2_DY = (BCO / 8) * W2_COL;         // dY: 8 blocks (64 output channels)
constexpr int W2_X = (BKC / 8) * W2_COL;          // X: 16 blocks (128 im2col columns)
constexpr int W2_STAGE = W2_DY + W2_X;

__device__ __forceinline__ int w2_off(int px, int col) { return (col >> 3) * W2_COL + px * 16 + (col & 7) * 2; }

template <int NST>
__global__ __launch_bounds__(kThreads) void conv_wgrad_dma_kernel(ConvWgradParams p) {
  __shared__ __attribute__((aligned(16))) char smem[NST * W2_STAGE];
  if (run_side(p, smem)) return;
  const int t = int(threadIdx.x), lane = t & 63, wave = t >> 6;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int KC = 16 * p.Cin, KT = KC / BKC, T = (p.Cout / BCO) * KT;
  const int nwg = main_blocks(p), b = int(blockIdx.x);
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int w = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int slice = w / T, tile = w - slice * T;
  const int co0 = (tile / KT) * BCO, kt = tile - (tile / KT) * KT;
  const int m_begin = slice * int(p.px_per_slice);
  const int m_end = m_begin + int(p.px_per_slice) < int(p.M) ? m_begin + int(p.px_per_slice) : int(p.M);
  const int nsteps = m_end > m_begin ? (m_end - m_begin + W2_BPX - 1) / W2_BPX : 0;

  // this wave's chunk columns: X blocks 4 wv + j (j < 4), dY blocks 2 wv + j (j < 2);
  // (kh, kw, ci) and the element delta from the pixel's tap-(0, 0) origin are wave-uniform
  int xkh[4], xkw[4], xde[4];
  const int cs = __builtin_ctz(unsigned(p.Cin));   // Cin is a power of two (host check)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int kc = kt * BKC + (4 * wv + j) * 8;
    xkh[j] = kc >> (cs + 2);
    xkw[j] = (kc >> cs) & 3;
    xde[j] = (xkh[j] * p.W + xkw[j]) * p.Cin + (kc & (p.Cin - 1));
  }
  // lane = pixel m of the step: (oh, ow) and the element offset of its tap-(0, 0) origin
  int m = m_begin + lane;
  int oh, ow, e;
  {
    const int hw = p.Ho * p.Wo;
    const int n = m / hw, r = m - n * hw;
    oh = r / p.Wo;
    ow = r - oh * p.Wo;
    e = (n * p.H + 2 * oh - 1) * (p.W * p.Cin) + (2 * ow - 1) * p.Cin;
  }
  const int j_col = 2 * W2_BPX * p.Cin, j_row = 2 * (p.W - p.Wo) * p.Cin, j_img = (p.H - 2 * p.Ho) * p.W * p.Cin;
  const __amdgpu_buffer_rsrc_t rs_x = make_rsrc(p.x, int64_t(p.N) * p.H * p.W * p.Cin * 2);
  const __amdgpu_buffer_rsrc_t rs_dy = make_rsrc(p.dy, p.M * p.Cout * 2);
  const uint32_t dy_co = uint32_t((co0 + 2 * wv * 8) * 2);

  // one stage: 4 X + 2 dY LDS-DMA instructions per wave; stages past the slice
  // load out of range (zeros, no memory traffic), so every stage counts the same
  auto issue = [&](int buf) {
    char* st = smem + buf * W2_STAGE;
    const int ih = 2 * oh - 1, iw = 2 * ow - 1;
    const bool live = m < m_end;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool ok = live && unsigned(ih + xkh[j]) < unsigned(p.H) && unsigned(iw + xkw[j]) < unsigned(p.W);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs_x, (__attribute__((address_space(3))) void*)(st + W2_DY + (4 * wv + j) * W2_COL), 16,
          int(ok ? uint32_t(e + xde[j]) * 2u : kOOB), 0, 0, 0);
    }
    const uint32_t doff = uint32_t(m) * uint32_t(p.Cout * 2) + dy_co;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs_dy, (__attribute__((address_space(3))) void*)(st + (2 * wv + j) * W2_COL), 16,
          int(live ? doff + uint32_t(j * 16) : kOOB), 0, 0, 0);
    // advance the pixel by 64 (at most two row wraps for Wo >= 32)
    m += W2_BPX;
    ow += W2_BPX;
    e += j_col;
    while (ow >= p.Wo) {
      ow -= p.Wo;
      e += j_row;
      if (++oh == p.Ho) oh = 0, e += j_img;
    }
  };

  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wco = (wave >> 1) * 32, wkc = (wave & 1) * 64;
  // fragment read offsets (loop invariant): rows (pixels) 8 g + q (+4, +32 kk), columns col + 4 pp
  int ra[2], rb[4];
  {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
#pragma unroll
    for (int i = 0; i < 2; ++i) ra[i] = w2_off(8 * g + q, wco + 16 * i + 4 * pp);
#pragma unroll
    for (int j = 0; j < 4; ++j) rb[j] = W2_DY + w2_off(8 * g + q, wkc + 16 * j + 4 * pp);
  }
  constexpr int NL = 6;   // LDS-DMA instructions per stage per lane
  constexpr uint32_t kWaitAll = (7u << 4) | (0xFu << 8);
  constexpr uint32_t kWaitNewer = kWaitAll | uint32_t((NL * (NST - 2)) & 15) | (uint32_t((NL * (NST - 2)) >> 4) << 14);
#pragma unroll
  for (int u = 0; u < NST - 1; ++u) issue(u);
  int cur = 0;
  for (int s = 0; s < nsteps; ++s) {
    // stage s landed (the NST - 2 younger stages may stay in flight), visible
    // to every wave; every wave is done reading stage s - 1's buffer
    __builtin_amdgcn_s_waitcnt(kWaitNewer);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(cur == 0 ? NST - 1 : cur - 1);   // step s + NST - 1
    const char* base = smem + cur * W2_STAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ko = kk * 32 * 16;          // 32 pixels further down the column blocks
      bf16x8 a[2], bm[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = frag_at(base, ra[i] + ko, 4 * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) bm[j] = frag_at(base, rb[j] + ko, 4 * 16);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bm[j], acc[i][j], 0, 0, 0);
    }
    cur = cur == NST - 1 ? 0 : cur + 1;
  }
  __builtin_amdgcn_s_waitcnt(kWaitAll);   // the padding stages' DMAs are done before the block exits

  zero_output(p);
  float* out = p.partial + int64_t(slice) * p.Cout * KC + (co0 + wco + 4 * (lane >> 4)) * KC +
               (kt * BKC + wkc + (lane & 15));
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(16 * i + r) * KC + 16 * j] = acc[i][j][r];
}

// ---------------------------------------------------------------------------
// Weight gradient of the FIRST layer: 4-channel input (RGB frames decoded as
// RGBA bf16; the alpha channel's gradient is computed and discarded), Cout %
// 32 == 0.  KC = 16 taps x 4 channels = 64, one 32 x 64 tile per block and
// pixel slice.  A 16-byte chunk of an im2col row is two horizontally
// adjacent input pixels (taps kw, kw+1) -- 8-byte aligned only, and at the
// left / right image border half of it is padding -- so it is two bounds-
// checked 8-byte buffer loads.  LDS images: dY [32 px][32 co] (64-byte rows),
// X [32 px][64 kc] (128-byte rows), both read by ds_read_b64_tr_b16.
constexpr int C4_DY_ROW = 64, C4_X_ROW = 128;
constexpr int C4_DY_TILE = BPX * C4_DY_ROW, C4_X_TILE = BPX * C4_X_ROW;
constexpr int C4_STAGE = C4_DY_TILE + C4_X_TILE;

// 64-byte rows: 4 rows per bank row; the row pair 8 apart (same bank window
// otherwise) flips its 32-byte half
__device__ __forceinline__ int c4dy_off(int r, int byte) {
  return r * C4_DY_ROW + ((((byte >> 5) ^ ((r >> 3) & 1)) << 5) | (byte & 31));
}
// 128-byte rows: the dY scheme of the main kernel
__device__ __forceinline__ int c4x_off(int r, int byte) { return dy_off(r, byte); }

__global__ __launch_bounds__(kThreads) void conv_wgrad_c4_kernel(ConvWgradParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * C4_STAGE + kLutBytes];
  if (run_side(p, smem)) return;
  const bool u8in = p.lut != nullptr;   // raw u8 RGBA input, decoded through the table (see stage_lut)
  char* const lutl = smem + 2 * C4_STAGE;
  if (u8in) {
    stage_lut(p.lut, lutl);
    __syncthreads();
  }
  const int t = int(threadIdx.x), lane = t & 63, wave = t >> 6;
  const int T = p.Cout / 32;
  const int nwg = main_blocks(p), b = int(blockIdx.x);
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int w = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int slice = w / T, co0 = (w - slice * T) * 32;
  const int m_begin = slice * int(p.px_per_slice);
  const int m_end = m_begin + int(p.px_per_slice) < int(p.M) ? m_begin + int(p.px_per_slice) : int(p.M);
  const int nsteps = m_end > m_begin ? (m_end - m_begin + BPX - 1) / BPX : 0;

  const int dpx = (t & 127) >> 2, dch = t & 3;          // dY: threads < 128, 4 chunks per pixel row
  const bool dy_loader = t < 128;
  const int xpx = t >> 3, xch = t & 7;                  // X: one 2-pixel chunk per thread
  const int kh = xch >> 1, kw = (xch & 1) * 2;
  PixelCursor c;
  c.init(m_begin + xpx, p.Ho, p.Wo);
  const __amdgpu_buffer_rsrc_t rs_x = make_rsrc(p.x, int64_t(p.N) * p.H * p.W * 4 * (u8in ? 1 : 2));
  const __amdgpu_buffer_rsrc_t rs_dy = make_rsrc(p.dy, p.M * p.Cout * 2);
  // BN backward applied while staging dY (ConvWgradParams::bn_dy): the lane's
  // 8 channels are fixed, so their coefficients live in registers
  const bool bnd = p.bn_dy.y != nullptr;
  const __amdgpu_buffer_rsrc_t rs_by = make_rsrc(bnd ? p.bn_dy.y : p.dy, p.M * p.Cout * 2);
  BnBwdCoef bc[8];
  if (bnd) {
    const float invM = 1.f / float(p.M);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = co0 + dch * 8 + i;
      bc[i].init(p.bn_dy.mean[c], p.bn_dy.invstd[c], p.bn_dy.w[c], p.bn_dy.b[c], p.bn_dy.dw[c], p.bn_dy.db[c], invM);
    }
  }
  constexpr int kDepth = 4;
  struct Stage {
    uint4 dy, by;    // by: the BN input chunk (bnd)
    uint2 x0, x1;    // bf16 pixels; u8 input: x0.x / x1.x the raw bytes, x0.y / x1.y in-image flags
  };
  Stage ring[kDepth];
  int md = m_begin + dpx, mx = m_begin + xpx;
  uint32_t dy_byte = uint32_t(md) * uint32_t(p.Cout * 2) + uint32_t((co0 + dch * 8) * 2);
  const uint32_t dy_step = uint32_t(BPX * p.Cout * 2);
  auto load = [&](Stage& r) {
    const uint32_t doff = dy_loader && md < m_end ? dy_byte : kOOB;
    r.dy = bload(rs_dy, doff);
    if (bnd) r.by = bload(rs_by, doff);
    const int ih = 2 * c.oh - 1 + kh, iw = 2 * c.ow - 1 + kw;
    const bool row_ok = mx < m_end && unsigned(ih) < unsigned(p.H);
    const int e = ((c.n * p.H + ih) * p.W + iw) * 4;
    const bool ok0 = row_ok && unsigned(iw) < unsigned(p.W), ok1 = row_ok && unsigned(iw + 1) < unsigned(p.W);
    if (u8in) {   // converted when stored (the ring keeps its loads in flight)
      r.x0 = make_uint2(bload4(rs_x, ok0 ? uint32_t(e) : kOOB), ok0 ? 1u : 0u);
      r.x1 = make_uint2(bload4(rs_x, ok1 ? uint32_t(e + 4) : kOOB), ok1 ? 1u : 0u);
    } else {
      r.x0 = bload8(rs_x, ok0 ? uint32_t(e) * 2u : kOOB);
      r.x1 = bload8(rs_x, ok1 ? uint32_t(e + 4) * 2u : kOOB);
    }
    md += BPX;
    mx += BPX;
    dy_byte += dy_step;
    c.advance(p.Ho, p.Wo);
  };
  const int st_dy = c4dy_off(dpx, dch * 16), st_x = C4_DY_TILE + c4x_off(xpx, xch * 16);
  const float slope = p.bn_dy.slope;
  auto store = [&](const Stage& r, int buf) {
    char* base = smem + buf * C4_STAGE;
    if (dy_loader) {
      uint4 d = r.dy;
      if (bnd) {   // gx of the BN from its input (by) and its output gradient (dy)
        const uint32_t gw[4] = {r.dy.x, r.dy.y, r.dy.z, r.dy.w}, yw[4] = {r.by.x, r.by.y, r.by.z, r.by.w};
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float2 g = make_float2(__uint_as_float(gw[k] << 16), __uint_as_float(gw[k] & 0xFFFF0000u));
          const float2 v = make_float2(__uint_as_float(yw[k] << 16), __uint_as_float(yw[k] & 0xFFFF0000u));
          const f32x2 pr = {bc[2 * k].gx(v.x, g.x, slope), bc[2 * k + 1].gx(v.y, g.y, slope)};
          o[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pr, bf16x2));
        }
        // a row past the slice loaded zeros for both and gets a nonzero gx: its X
        // row is past the slice too and staged as zeros, so it adds nothing
        d = make_uint4(o[0], o[1], o[2], o[3]);
      }
      *reinterpret_cast<uint4*>(base + st_dy) = d;
    }
    if (u8in) {
      const uint2 a = lut_px(lutl, r.x0.x, r.x0.y != 0u), b = lut_px(lutl, r.x1.x, r.x1.y != 0u);
      *reinterpret_cast<uint4*>(base + st_x) = make_uint4(a.x, a.y, b.x, b.y);
    } else {
      *reinterpret_cast<uint4*>(base + st_x) = make_uint4(r.x0.x, r.x0.y, r.x1.x, r.x1.y);
    }
  };
  // wave: co fragment wave / 2, kc fragments 2 (wave % 2) + {0, 1}
  const int fco = (wave >> 1) * 16, fkc = (wave & 1) * 32;
  int ra, rb[2];
  {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    ra = c4dy_off(8 * g + q, (fco + 4 * pp) * 2);
#pragma unroll
    for (int j = 0; j < 2; ++j) rb[j] = C4_DY_TILE + c4x_off(8 * g + q, (fkc + 16 * j + 4 * pp) * 2);
  }
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int u = 0; u < kDepth; ++u) load(ring[u]);
  const int padded = (nsteps + kDepth - 1) / kDepth * kDepth;
  for (int s0 = 0; s0 < padded; s0 += kDepth) {
#pragma unroll
    for (int u = 0; u < kDepth; ++u) {
      const int buf = u & 1;
      store(ring[u], buf);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      load(ring[u]);
      const char* base = smem + buf * C4_STAGE;
      const bf16x8 a = frag_at(base, ra, 4 * C4_DY_ROW);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, frag_at(base, rb[j], 4 * C4_X_ROW), acc[j], 0, 0, 0);
    }
  }
  zero_output(p);
  float* out = p.partial + int64_t(slice) * p.Cout * 64;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + fco + 4 * (lane >> 4) + r;
      out[co * 64 + fkc + 16 * j + (lane & 15)] = acc[j][r];
    }
}

// ---------------------------------------------------------------------------
// The first layer's weight gradient with WAVE-PRIVATE staging.  Its 32 x 64
// tile is 2 MFMAs per wave per 32-pixel step, so the block-shared staging of
// conv_wgrad_c4_kernel spent its time in the per-step block barrier, with
// the dY loaders (128 threads) doing all of the BN-backward arithmetic while
// the other two waves waited.  Here each wave streams its own pixel steps
// (wave w takes steps w, w + 4, ...) through its own 6 KiB of LDS: no block
// barrier in the loop (a wave's LDS writes and reads are ordered by its own
// lgkmcnt), every lane stages dY (and applies the BN backward to its 8
// channels) and X, and a step is 8 MFMAs (the whole 32 x 64 tile).  The
// four waves' tiles meet in LDS at the end.  Same slices, same reduce.
constexpr int C4W_DY = BPX * C4_DY_ROW;          // 2 KiB: [32 px][32 co]
constexpr int C4W_X = BPX * C4_X_ROW;            // 4 KiB: [32 px][64 kc]
constexpr int C4W_WAVE = C4W_DY + C4W_X;
// NW waves per block (BT_C4W_WAVES, 4 or 8): the kernel is latency-bound --
// 512 blocks of 4 waves are 2 waves per SIMD, each walking ~9 pixel steps
// whose loads, LUT lookups and BN-backward arithmetic form one chain -- so 8
// waves per block double the chains in flight with the same slices (the
// same partials, the same reduce, the same per-block fold).
template <int NW>
constexpr int c4w_lds() { return NW * 32 * 64 * 4; }   // the combine: NW waves x [32][64] fp32
static_assert(4 * C4W_WAVE + kLutBytes <= c4w_lds<4>(), "staging fits the combine area");

// U8: the input is raw u8 frames read through the decode table (p.lut): a
// compile-time switch, so neither form carries the other's stage registers
// LDSC: the BN-backward coefficients (7 floats x 8 channels of a lane's dY
// chunk, 56 VGPRs) live in LDS and are read per staged stage, freeing the
// registers that held the kernel at 2 waves per SIMD (BT_C4W_LDS_COEF)
template <int NW, bool U8, bool LDSC = false>
__global__ __launch_bounds__(64 * NW) void conv_wgrad_c4w_kernel(ConvWgradParams p) {
  static_assert(NW * C4W_WAVE + kLutBytes + 32 * 8 * 4 <= c4w_lds<NW>(), "the coefficient table fits");
  __shared__ __attribute__((aligned(16))) char smem[c4w_lds<NW>()];
  if (run_side(p, smem)) return;
  constexpr bool u8in = U8;
  char* const lutl = smem + NW * C4W_WAVE;
  if (u8in) {
    stage_lut(p.lut, lutl);
    __syncthreads();
  }
  const int t = int(threadIdx.x), lane = t & 63, wave = t >> 6;
  const int T = p.Cout / 32;
  const int nwg = main_blocks(p), b = int(blockIdx.x);
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int w = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int slice = w / T, co0 = (w - slice * T) * 32;
  const int m_begin = slice * int(p.px_per_slice);
  const int m_end = m_begin + int(p.px_per_slice) < int(p.M) ? m_begin + int(p.px_per_slice) : int(p.M);
  const int nsteps = m_end > m_begin ? (m_end - m_begin + BPX - 1) / BPX : 0;
  const int mysteps = nsteps > wave ? (nsteps - wave + NW - 1) / NW : 0;   // steps wave, wave + NW, ...
  char* const ws = smem + wave * C4W_WAVE;

  // dY: lane -> channel chunk dc (8 channels), pixels dp and dp + 16 of the step
  const int dc = lane & 3, dp = lane >> 2;
  // X: lane -> pixel xp of the step, chunks xc0 .. xc0 + 3 (taps kh0, kh0 + 1 by kw 0, 2)
  const int xp = lane & 31, kh0 = (lane >> 5) * 2;
  const bool bnd = p.bn_dy.y != nullptr;
  BnBwdCoef bc[LDSC ? 1 : 8];
  float* const coefl = reinterpret_cast<float*>(smem + NW * C4W_WAVE + kLutBytes);   // [32 co][8] (LDSC)
  if (bnd) {   // (LDS scratch: the staging area, free until the loop)
    if constexpr (LDSC) {
      BnBwdCoef t8[8];
      bn_dy_coefs(p.bn_dy, p.Cout, p.M, co0 + dc * 8, reinterpret_cast<double*>(smem),
                  reinterpret_cast<int*>(smem + 4096), unsigned(b), unsigned(nwg), t8);
      if (wave == 0 && lane < 4) {   // lanes 0-3 hold the 4 chunks of the block's 32 channels
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float4* q = reinterpret_cast<float4*>(coefl + (dc * 8 + i) * 8);
          q[0] = make_float4(t8[i].is, t8[i].nm, t8[i].ww, t8[i].bb);
          q[1] = make_float4(t8[i].P, t8[i].dbm, t8[i].pdw, 0.f);
        }
      }
    } else {
      bn_dy_coefs(p.bn_dy, p.Cout, p.M, co0 + dc * 8, reinterpret_cast<double*>(smem),
                  reinterpret_cast<int*>(smem + 4096), unsigned(b), unsigned(nwg), bc);
    }
    __syncthreads();
  }
  const float slope = p.bn_dy.slope;
  const __amdgpu_buffer_rsrc_t rs_x = make_rsrc(p.x, int64_t(p.N) * p.H * p.W * 4 * (u8in ? 1 : 2));
  const __amdgpu_buffer_rsrc_t rs_dy = make_rsrc(p.dy, p.M * p.Cout * 2);
  const __amdgpu_buffer_rsrc_t rs_by = make_rsrc(bnd ? p.bn_dy.y : p.dy, p.M * p.Cout * 2);
  PixelCursor c;
  c.init(m_begin + wave * BPX + xp, p.Ho, p.Wo);
  int md = m_begin + wave * BPX + dp, mx = m_begin + wave * BPX + xp;
  uint32_t dy_byte = uint32_t(md) * uint32_t(p.Cout * 2) + uint32_t((co0 + dc * 8) * 2);
  const uint32_t dy_step = uint32_t(NW * BPX * p.Cout * 2), dy_half = uint32_t(16 * p.Cout * 2);
  constexpr int kDepth = 2;
  struct Stage {
    uint4 g[2], y[2];   // dY chunks of pixels dp, dp + 16 (y: the BN input, bnd)
    uint32_t x[4][2];   // u8: RGBA words of the 2 pixels of each chunk; bf16: low halves
    uint32_t xh[4][2];  // bf16: high halves
    uint32_t ok;        // per-pixel in-image bits (u8)
  };
  Stage ring[kDepth];
  auto load = [&](Stage& r) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t off = md + 16 * h < m_end ? dy_byte + uint32_t(h) * dy_half : kOOB;
      r.g[h] = bload(rs_dy, off);
      if (bnd) r.y[h] = bload(rs_by, off);
    }
    r.ok = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int kh = kh0 + (k >> 1), kw = (k & 1) * 2;
      const int ih = 2 * c.oh - 1 + kh, iw = 2 * c.ow - 1 + kw;
      const bool row_ok = mx < m_end && unsigned(ih) < unsigned(p.H);
      const int e = ((c.n * p.H + ih) * p.W + iw) * 4;
      const bool ok0 = row_ok && unsigned(iw) < unsigned(p.W), ok1 = row_ok && unsigned(iw + 1) < unsigned(p.W);
      if constexpr (u8in) {
        r.x[k][0] = bload4(rs_x, ok0 ? uint32_t(e) : kOOB);
        r.x[k][1] = bload4(rs_x, ok1 ? uint32_t(e + 4) : kOOB);
        r.ok |= (ok0 ? 1u : 0u) << (2 * k) | (ok1 ? 2u : 0u) << (2 * k);
      } else {
        const uint2 lo = bload8(rs_x, ok0 ? uint32_t(e) * 2u : kOOB), hi = bload8(rs_x, ok1 ? uint32_t(e + 4) * 2u : kOOB);
        r.x[k][0] = lo.x, r.xh[k][0] = lo.y, r.x[k][1] = hi.x, r.xh[k][1] = hi.y;
      }
    }
    md += NW * BPX;
    mx += NW * BPX;
    dy_byte += dy_step;
#pragma unroll
    for (int k = 0; k < NW; ++k) c.advance(p.Ho, p.Wo);   // NW x 32 pixels: this wave's next step
  };
  auto store = [&](const Stage& r) {
    uint32_t o[2][4];
    if (bnd) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {   // channels 2 k, 2 k + 1 of the chunk, both pixels
        BnBwdCoef e0, e1;
        if constexpr (LDSC) {
          const float4* q = reinterpret_cast<const float4*>(coefl + (dc * 8 + 2 * k) * 8);
          const float4 a0 = q[0], b0 = q[1], a1 = q[2], b1 = q[3];
          e0.is = a0.x, e0.nm = a0.y, e0.ww = a0.z, e0.bb = a0.w, e0.P = b0.x, e0.dbm = b0.y, e0.pdw = b0.z;
          e1.is = a1.x, e1.nm = a1.y, e1.ww = a1.z, e1.bb = a1.w, e1.P = b1.x, e1.dbm = b1.y, e1.pdw = b1.z;
        } else {
          e0 = bc[2 * k], e1 = bc[2 * k + 1];
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t gw = k == 0 ? r.g[h].x : k == 1 ? r.g[h].y : k == 2 ? r.g[h].z : r.g[h].w;
          const uint32_t yw = k == 0 ? r.y[h].x : k == 1 ? r.y[h].y : k == 2 ? r.y[h].z : r.y[h].w;
          const f32x2 pr = {e0.gx(__uint_as_float(yw << 16), __uint_as_float(gw << 16), slope),
                            e1.gx(__uint_as_float(yw & 0xFFFF0000u), __uint_as_float(gw & 0xFFFF0000u), slope)};
          o[h][k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pr, bf16x2));
        }
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // (a pixel past the slice gets a nonzero gx from its zero loads; its X
      // row is past the slice too and staged as zeros: it adds nothing)
      const uint4 d = bnd ? make_uint4(o[h][0], o[h][1], o[h][2], o[h][3]) : r.g[h];
      *reinterpret_cast<uint4*>(ws + c4dy_off(dp + 16 * h, dc * 16)) = d;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int chunk = (kh0 + (k >> 1)) * 2 + (k & 1);   // im2col columns 8 chunk .. + 7
      uint4 v;
      if constexpr (u8in) {
        const uint2 lo = lut_px(lutl, r.x[k][0], (r.ok >> (2 * k)) & 1u), hi = lut_px(lutl, r.x[k][1], (r.ok >> (2 * k + 1)) & 1u);
        v = make_uint4(lo.x, lo.y, hi.x, hi.y);
      } else {
        v = make_uint4(r.x[k][0], r.xh[k][0], r.x[k][1], r.xh[k][1]);
      }
      *reinterpret_cast<uint4*>(ws + C4W_DY + c4x_off(xp, chunk * 16)) = v;
    }
  };
  int ra[2], rb[4];
  {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
#pragma unroll
    for (int i = 0; i < 2; ++i) ra[i] = c4dy_off(8 * g + q, (16 * i + 4 * pp) * 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) rb[j] = C4W_DY + c4x_off(8 * g + q, (16 * j + 4 * pp) * 2);
  }
  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < kDepth; ++u) load(ring[u]);
  const int padded = (mysteps + kDepth - 1) / kDepth * kDepth;
  for (int s0 = 0; s0 < padded; s0 += kDepth) {
#pragma unroll
    for (int u = 0; u < kDepth; ++u) {
      asm volatile("" ::: "memory");
      store(ring[u]);                            // waits for this stage's loads (counted vmcnt)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      load(ring[u]);                             // step + 2 (past the end: out of range, zeros)
      bf16x8 a[2], bm[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = frag_at(ws, ra[i], 4 * C4_DY_ROW);
#pragma unroll
      for (int j = 0; j < 4; ++j) bm[j] = frag_at(ws, rb[j], 4 * C4_X_ROW);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bm[j], acc[i][j], 0, 0, 0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // fragments in registers before the next store
    }
  }
  // combine the NW waves' tiles: [wave][co 32][kc 64] fp32 in LDS
  __syncthreads();
  float* cmb = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        cmb[(wave * 32 + 16 * i + 4 * (lane >> 4) + r) * 64 + 16 * j + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  zero_output(p);
  float* out = p.partial + int64_t(slice) * p.Cout * 64 + co0 * 64;
  for (int e = t; e < 32 * 64; e += 64 * NW) {
    float v = cmb[e];
#pragma unroll
    for (int w = 1; w < NW; ++w) v += cmb[w * 32 * 64 + e];   // (wave order: NW = 4 sums as before)
    out[e] = v;
  }
}

// ---------------------------------------------------------------------------
// The first layer's weight gradient from a DECODED INPUT PATCH (c4p).  The
// wave-private kernel above gathers every output pixel's 16 taps straight from
// the u8 frames each step: a stride-2 4x4 window reads every input pixel 4x,
// and each read is a dword load plus 4 table lookups and a 16-byte LDS store
// of the im2col row -- 12 loads, 32 lookups and 6 stores per lane and step,
// at 206 VGPRs (2 waves per SIMD; profiles/r5/disc_roofline.md: 34 us, 1.9
// TB/s).  Here a block takes a BAND of R output rows of one image (a slice
// of R x Wo pixels), decodes the band's 2R + 2 input rows ONCE into LDS
// ([row][column + 1][4 ch] bf16, the padding columns and rows zero), and
// reads the MFMA B fragments (32 pixels x 16 im2col columns = 4 taps x 4
// channels) straight out of that image with the transposing LDS read: lane
// (q, p) of a 16-lane group addresses output pixel 8g + q at tap (kh = j, kw
// = p), i.e. input column 2 ow + p of patch row 2 orow + j -- 8 bytes, the
// pixel's 4 channels.  The 32 such reads of a half-wave hit 20 distinct
// 8-byte words of one patch row (2 q + p, overlapping lanes broadcast): no
// bank conflict.  A step then costs a lane 4 dY loads (dY and the BN input
// of 2 pixels x 8 channels), the BN backward of those 16 values, 2 LDS
// stores and 8 MFMAs; the decode is one lookup set per input pixel per band.
// Same slices-then-reduce contract as conv_wgrad_c4w_kernel (slice = band).
constexpr int kC4pMaxW = 640;                    // input width the static LDS image is sized for
constexpr int kC4pPW = kC4pMaxW + 2;             // + the two zero padding columns
template <int R>
constexpr int c4p_patch() { return (2 * R + 2) * kC4pPW * 8; }
template <int R>
constexpr int c4p_lds() {
  // patch | 4 waves x 2 A tiles (2 KiB each) | decode table; the closing combine of the 4 waves'
  // 32 x 64 fp32 tiles (32 KiB) and the BN fold's scratch alias the front
  return c4p_patch<R>() + 4 * 2 * C4W_DY + kLutBytes > 4 * 32 * 64 * 4 ? c4p_patch<R>() + 4 * 2 * C4W_DY + kLutBytes
                                                                       : 4 * 32 * 64 * 4;
}

// KD: dY ring depth (steps in flight per wave).  2 (136 VGPRs, 3 waves per SIMD):
// 4 (173 VGPRs, 2 waves) measured 29.6 against 27.8 us with the BN backward
// (profiles/r6/b4/c4w_bench.jsonl, profiles/r6/b2/c4w_bench.jsonl)
// PRE: the first decode round's loads issued before the BN fold, so their latency hides under
// the fold's accumulator reads (BT_C4P_PRE, default on; 4-row bands are LDS-limited to 2 blocks
// per CU either way)
template <int R, int KD = 2, bool PRE = false>
__global__ __launch_bounds__(kThreads) void conv_wgrad_c4p_kernel(ConvWgradParams p) {
  constexpr int PR = 2 * R + 2;
  constexpr int PATCH = c4p_patch<R>();
  __shared__ __attribute__((aligned(16))) char smem[c4p_lds<R>()];
  if (run_side(p, smem)) return;
  char* const patch = smem;
  char* const lutl = smem + PATCH + 4 * 2 * C4W_DY;
  const int t = int(threadIdx.x), lane = t & 63, wave = t >> 6;
  const int nwg = main_blocks(p), b = int(blockIdx.x);
  // neighbouring bands share their two halo input rows: keep them on one XCD (its L2)
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int band = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int bpi = p.Ho / R;
  const int n = band / bpi, oh0 = (band - n * bpi) * R;
  const int m_begin = band * R * p.Wo;
  const int spr = p.Wo / BPX, nsteps = R * spr;
  const int PW = p.W + 2;
  const int dc = lane & 3, dp = lane >> 2;
  const bool bnd = p.bn_dy.y != nullptr;
  // the band's input rows 2 oh0 - 1 .. 2 (oh0 + R) decoded once: 16-byte loads of 4 input pixels
  // (W % 64 == 0: c4p_rows_for), DQ in flight per thread and round -- a 4-row band of a 640-wide
  // frame is one round (1600 quads; 4-byte loads took 4 rounds of 8, a memory latency each) --
  // then their lookups; the first round's loads are issued before the BN fold, so their latency
  // hides under the fold's own accumulator reads
  const __amdgpu_buffer_rsrc_t rs_x = make_rsrc(p.x, int64_t(p.N) * p.H * p.W * 4);
  const int QW = p.W >> 2, nq = PR * QW, ih0 = 2 * oh0 - 1;
  constexpr int DQ = 8;
  auto issue = [&](int i0, uint4 (&wv)[DQ], bool (&ok)[DQ]) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < DQ; ++k) {
      const int i = i0 + k * kThreads + t;
      const int pr = i / QW, qc = i - pr * QW;
      const int ih = ih0 + pr;
      ok[k] = i < nq && unsigned(ih) < unsigned(p.H);
      wv[k] = bload(rs_x, ok[k] ? uint32_t(((n * p.H + ih) * p.W + 4 * qc) * 4) : kOOB);
    }
  };
  auto lookups = [&](int i0, const uint4 (&wv)[DQ], const bool (&ok)[DQ]) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < DQ; ++k) {
      const int i = i0 + k * kThreads + t;
      if (i < nq) {
        const int pr = i / QW, qc = i - pr * QW;
        uint2* d = reinterpret_cast<uint2*>(patch + (pr * PW + 4 * qc + 1) * 8);   // columns 4 qc + 1 ..
        d[0] = lut_px(lutl, wv[k].x, ok[k]);
        d[1] = lut_px(lutl, wv[k].y, ok[k]);
        d[2] = lut_px(lutl, wv[k].z, ok[k]);
        d[3] = lut_px(lutl, wv[k].w, ok[k]);
      }
    }
  };
  uint4 wv0[DQ];
  bool ok0[DQ];
  if constexpr (PRE) issue(0, wv0, ok0);
  // the decode table and the BN coefficients' inputs go out with the first decode round too: the
  // fold's accumulator reads are then the prologue's only other round trip
  const uint2 lut8 = *reinterpret_cast<const uint2*>(p.lut + 4 * t);   // (kThreads == 256: stage_lut's split)
  BnDyPre pre;
  if (bnd) pre.load(p.bn_dy, dc * 8);
  BnBwdCoef bc[8];
  unsigned rel_tk = 0;   // the accumulator release's ticket (thread 0), answered at the end
  if (bnd) {   // (LDS scratch: the front, free until the patch is written)
    bn_dy_coefs(p.bn_dy, p.Cout, p.M, dc * 8, reinterpret_cast<double*>(smem), reinterpret_cast<int*>(smem + 4096),
                unsigned(b), unsigned(nwg), bc, &rel_tk, &pre);
  }
  *reinterpret_cast<uint2*>(lutl + 8 * t) = lut8;
  __syncthreads();
  for (int i = t; i < 2 * PR; i += kThreads)   // the zero padding columns 0 and W + 1
    *reinterpret_cast<uint2*>(patch + ((i >> 1) * PW + ((i & 1) ? PW - 1 : 0)) * 8) = make_uint2(0u, 0u);
  if constexpr (PRE) lookups(0, wv0, ok0);
  for (int i0 = PRE ? DQ * kThreads : 0; i0 < nq; i0 += DQ * kThreads) {
    uint4 wv[DQ];
    bool ok[DQ];
    issue(i0, wv, ok);
    lookups(i0, wv, ok);
  }
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs_dy = make_rsrc(p.dy, p.M * p.Cout * 2);
  const __amdgpu_buffer_rsrc_t rs_by = make_rsrc(bnd ? p.bn_dy.y : p.dy, p.M * p.Cout * 2);
  const float slope = p.bn_dy.slope;
  char* const ws = smem + PATCH + wave * 2 * C4W_DY;
  int ra[2], rbl[4];
  {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
#pragma unroll
    for (int i = 0; i < 2; ++i) ra[i] = c4dy_off(8 * g + q, (16 * i + 4 * pp) * 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) rbl[j] = (j * PW + 2 * (8 * g + q) + pp) * 8;
  }
  // steps wave, wave + 4, ...; stage u of the ring holds the dY / BN-input chunks of pixels dp, dp + 16
  struct Stage {
    uint4 g[2], y[2];
  };
  Stage ring[KD];
  int s_load = wave;
  auto load = [&](Stage& r) {
    const bool live = s_load < nsteps;
    const uint32_t base = uint32_t(m_begin + s_load * BPX + dp) * uint32_t(p.Cout * 2) + uint32_t(dc * 16);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t off = live ? base + uint32_t(h * 16 * p.Cout * 2) : kOOB;
      r.g[h] = bload(rs_dy, off);
      // (unconditional, out of range without the BN: a load issued on only some paths made every
      // wait in this loop count the smaller total -- each stage's wait then took the next stage's
      // first load with it)
      r.y[h] = bload(rs_by, bnd ? off : kOOB);
      __builtin_amdgcn_sched_barrier(0);   // issue in consumption order: the waits count a FIFO
    }
    s_load += 4;
  };
  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < KD; ++u) load(ring[u]);
  // the accumulator release's ticket behind the ring's first loads: its round trip overlaps the
  // loop, and no wait before the loop counts it (taken before the table's LDS store it made that
  // store -- a wait on a path without the BN -- wait for the atomic too)
  if (bnd && p.bn_dy.acc && t == 0) rel_tk = bn_acc_ticket_take(p.bn_dy.acc, p.bn_dy.R, p.Cout, unsigned(b));
  const int mysteps = nsteps > wave ? (nsteps - wave + 3) / 4 : 0;
  const int padded = (mysteps + KD - 1) / KD * KD;
  int s = wave;
  for (int i0 = 0; i0 < padded; i0 += KD) {
#pragma unroll
    for (int u = 0; u < KD; ++u, s += 4) {
      const bool live = s < nsteps;   // (wave-uniform: false on the ring's padding steps)
      const Stage& r = ring[u];
      char* const A = ws + (u & 1) * C4W_DY;
#pragma unroll
      for (int h = 0; h < 2 && live; ++h) {
        uint4 d = r.g[h];
        if (bnd) {   // gx of BN1 from its input (y) and its output gradient (g), rounded to bf16
          const uint32_t gw[4] = {r.g[h].x, r.g[h].y, r.g[h].z, r.g[h].w}, yw[4] = {r.y[h].x, r.y[h].y, r.y[h].z, r.y[h].w};
          uint32_t o[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const f32x2 pr = {bc[2 * k].gx(__uint_as_float(yw[k] << 16), __uint_as_float(gw[k] << 16), slope),
                              bc[2 * k + 1].gx(__uint_as_float(yw[k] & 0xFFFF0000u), __uint_as_float(gw[k] & 0xFFFF0000u),
                                               slope)};
            o[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pr, bf16x2));
          }
          d = make_uint4(o[0], o[1], o[2], o[3]);
        }
        *reinterpret_cast<uint4*>(A + c4dy_off(dp + 16 * h, dc * 16)) = d;
      }
      load(ring[u]);   // KD steps ahead (past the end: out of range, zeros, never used)
      if (!live) continue;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int orow = s / spr, ow0 = (s - orow * spr) * BPX;
      const int sb = (2 * orow * PW + 2 * ow0) * 8;
      bf16x8 a[2], bm[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = frag_at(A, ra[i], 4 * C4_DY_ROW);
#pragma unroll
      for (int j = 0; j < 4; ++j) bm[j] = frag_at(patch, sb + rbl[j], 64);   // pixel + 4: column + 8
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bm[j], acc[i][j], 0, 0, 0);
    }
  }
  // combine the 4 waves' tiles: [wave][co 32][kc 64] fp32 over the patch
  __syncthreads();
  float* cmb = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        cmb[(wave * 32 + 16 * i + 4 * (lane >> 4) + r) * 64 + 16 * j + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  zero_output(p);
  float* out = p.partial + int64_t(band) * p.Cout * 64;
  for (int e = t; e < 32 * 64; e += kThreads) out[e] = cmb[e] + cmb[2048 + e] + cmb[4096 + e] + cmb[6144 + e];
  if (bnd && p.bn_dy.acc) {
    __syncthreads();   // (the flag word reuses the combine area)
    bn_acc_ticket_finish(p.bn_dy.acc, p.bn_dy.R, p.Cout, reinterpret_cast<int*>(smem), rel_tk, unsigned(b),
                         unsigned(nwg));
  }
}

// rows per band of conv_wgrad_c4p_kernel for this first layer (0: the shape does not take it)
int c4p_rows_for(int N, int H, int W, int Ho, int Wo, int Cout);

// ---------------------------------------------------------------------------
// Tap-gather GEMM: the forward convolution AND the data gradient.
//
//   out[pixel m][col] = sum over taps t, channels c of
//                       src[n][r0(m) + dr(t)][c0(m) + dc(t)][c] * w[col][wtap(t)][c]
//
// forward (16 taps):   src = x, r0 = 2a - 1, c0 = 2b - 1, (dr, dc) = (kh, kw),
//                      w = the channels-last weight [Cout][kh][kw][Cin]; out = y.
// data gradient: dx[n][ih][iw] only receives from the 2 x 2 taps whose
//   stride-2 phase matches (ih, iw), so it is 4 GEMMs (parity classes
//   (ph, pw) = blockIdx.y) of 4 taps each over the grid ih = 2a + ph,
//   iw = 2b + pw: src = dy, r0 = a, c0 = b, dr = ph - t/2, dc = pw - t%2,
//   kh = 1 - ph + 2(t/2), kw = 1 - pw + 2(t%2), and w = the weight transposed
//   to [Cin][kh][kw][Cout] (conv_weight_t).
//
// Both MFMA operands have K (tap, channel) contiguous in memory: a tap's C
// channels are one NHWC pixel, a weight row is [kh][kw][c].  Tiles stage as
// 128-byte LDS rows (16-byte chunks XOR-swizzled by row) read with
// ds_read_b128.  All index math is 32-bit and per-pixel bases are computed
// once; padding reads are range-checked buffer loads that return zeros.  The
// epilogue goes through LDS so every global store is 16 bytes; the forward
// also sums each output channel (and its square) of the bf16-rounded result
// into one partial row per pixel tile, which bn_finalize folds.

constexpr int FBM = 128;   // pixels per block
constexpr int FBN = 64;    // output channels per block
constexpr int FBK = 64;    // K per k-step
constexpr int F_ROW = FBK * 2;                  // 128-byte LDS rows
constexpr int FA_TILE = FBM * F_ROW;            // 16 KiB
constexpr int FB_TILE = FBN * F_ROW;            // 8 KiB
constexpr int F_STAGE = FA_TILE + FB_TILE;

__device__ __forceinline__ int f_off(int r, int chunk) { return r * F_ROW + ((chunk ^ (r & 7)) << 4); }

// Channels-as-rows MFMA tiles (the weights as the A operand, the pixels as B):
// a lane's accumulator then holds 4 channels of ONE pixel.  Row rho of channel
// fragment f is channel 32 (f >> 1) + 8 (rho >> 2) + 4 (f & 1) + (rho & 3), so
// fragments 2q and 2q + 1 give lane group g = lane >> 4 the 8 consecutive
// channels 32 q + 8 g .. + 7: one 16-byte store per lane and pixel.
__device__ __forceinline__ int c1_row_chan(int f, int rho) {
  return 32 * (f >> 1) + 8 * (rho >> 2) + 4 * (f & 1) + (rho & 3);
}
// The swizzle key of such a channel tile's LDS rows: the 16 rows one fragment
// read touches (c1_row_chan(f, 0..15): bits 0-1 and 3-4 vary) must land on
// 16 different 16-byte bank slots; with the pixel tiles' key (r & 7) they
// shared 4 and the reads ran 4-way conflicted (PMC: 60-124 % conflict cycles)
__device__ __forceinline__ int bkey(int r) { return ((r >> 1) & 1) | (((r >> 3) & 3) << 1); }

// Blocks of one launch wait here for each other (all of them resident: the
// caller's duty).  bar: a zero word; the last arriver resets it, the others
// spin on it with s_sleep.  No fences: what the blocks hand over is atomics
// at agent scope (the BN sums, performed past the XCD caches once this wave's
// vmcnt drains) read back with agent-scope loads -- a release / acquire per
// wave wrote back and invalidated the XCD's L2 and made the launch 4-5x slower
// (profiles/r5/b13).  A spin that outlasts ~1 s gives up (never a hung GPU),
// counts itself in g_grid_barrier_timeouts (conv_grid_barrier_timeouts) and
// raises the host-mapped flag g_grid_barrier_flag: the host polls that word
// without a HIP call (conv_grid_barrier_failed) and ops / CapturedStep raise
// on it, so BN statistics folded past a failed barrier never train silently.
__device__ unsigned g_grid_barrier_timeouts = 0;
__device__ unsigned* g_grid_barrier_flag = nullptr;   // host-mapped (conv_grid_barrier_arm)
constexpr unsigned kBarrierSpins = 1u << 22;
__device__ __forceinline__ void grid_barrier(unsigned* bar, unsigned nblk) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's atomics have been performed
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == nblk - 1) {
      __hip_atomic_store(bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned n = 0;
      while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
        __builtin_amdgcn_s_sleep(4);
        if (++n == kBarrierSpins) {
          atomicAdd(&g_grid_barrier_timeouts, 1u);
          if (unsigned* f = g_grid_barrier_flag)
            __hip_atomic_store(f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
    }
  }
  __syncthreads();
}

struct TapGemm {
  const uint16_t* src = nullptr;
  const uint16_t* w = nullptr;     // [NOUT][16][C]
  uint16_t* dst = nullptr;
  float* stats = nullptr;          // forward only (nullable)
  int N = 0, SH = 0, SW = 0, C = 0, cshift = 0;   // src [N][SH][SW][C], C = 1 << cshift
  int GH = 0, GW = 0, M = 0;       // GEMM rows: m = (n * GH + a) * GW + b
  int NOUT = 0, OH = 0, OW = 0;    // dst [N][OH][OW][NOUT]
  int wc = 0;                      // C4 mode: weight input channels (3 or 4)
  const uint16_t* lut = nullptr;   // C4 mode: src is raw u8 RGBA, decoded through this bf16 table [4][256]
  int acc_r = 0;                   // forward: > 0 = stats points at a BnAcc accumulator (fp64 [acc_r][2][NOUT])
  BnBwdFuse bn;                    // data gradient only: BN backward statistics in the epilogue (bn.part nullable)
  int cls_per_block = 1;           // data gradient: parity classes per block (1, or 4 = all; grid.y = 4 / this)
  // forward: src is the INPUT of a BatchNorm+LeakyReLU (act.on()) applied to the A tile as it is
  // staged; act_out (nullable) receives the activation itself (every input element once)
  BnActIn act;
  uint16_t* act_out = nullptr;
  // forward (tap_gemm_body OBN): the BatchNorm+LeakyReLU that consumes dst, applied by this
  // launch after a grid barrier on its statistics (acc = stats); oy receives leaky(bn(dst))
  BnActIn oact;
  uint16_t* oy = nullptr;
  // forward split-K (tap_gemm_body SPLIT = 2): the first block of a tile's pair to finish its
  // K half parks its fp32 accumulators here ([tile][FM * FN][kThreads] float4) and raises
  // split_ready[tile]; the second adds them to its own and runs the epilogue.  Both words zero
  // between launches (the second block resets them).
  float* split_part = nullptr;
  unsigned* split_ticket = nullptr;   // [2 * tiles]: ticket, ready
};

// BN = output channels per block (128 or 64, or 32 for 32-channel outputs
// such as the first layer's data gradient); 4 waves as WGM (pixels) x WGN
// (channels).  A wider BN re-reads the tap-gathered A tile for fewer channel
// tiles (the deep layers' A traffic is the bound, not the MFMAs).
// BM = pixels per block: 128, or 64 when 128-pixel tiles would leave the
// chip short of blocks (the deep-K layers: 300-600 tiles on 256 CUs).
// NST = staging: 0 = loads into a register ring then ds_write_b128 into two
// LDS buffers; 2 or 3 = LDS-DMA (buffer_load ... lds) straight into NST LDS
// stages -- the 16-byte LDS stores of the register path run at ~79 B/clk/CU
// (a third of what the fragment reads get) and were the kernel's bound.
// ACT (forward, LDS-DMA staging): the BatchNorm+LeakyReLU that produced src
// is applied here (BnActIn): every block folds the statistics accumulator in
// its prologue (overlapping its first stage's loads), and after its own
// LDS-DMA chunks of a stage have landed each thread rewrites them in place
// as leaky(bn(x)) rounded to bf16 -- before the barrier that publishes the
// stage, so no extra barrier and no register staging.  Padding chunks stay
// zero.  The chunks of the 4 centre taps (kh, kw in {1, 2}) cover every input
// element exactly once, so blocks of the first channel tile also store those
// to act_out: the activation the weight gradient reads, written without a
// pass of its own.  ACT = coefficient sets per thread: a thread's chunk is
// always the same 8 channels when C <= 64 (1), or alternates between two with
// the k-step when C = 128 (2).
// LDS of a tap GEMM block (the formulas of tap_gemm_body's STG / NBUF / RT / LUTB)
template <bool DGRAD, int BN, bool C4, int BM, int NST>
constexpr int tap_gemm_lds() {
  return ((C4 || NST == 0) ? 2 : NST) * (BM * F_ROW + BN * F_ROW) + (C4 ? 0 : BM * 16) + (C4 ? kLutBytes : 0);
}

// bx, by, nwg: the block's place in the GEMM's own grid (blockIdx.x / .y and
// gridDim.x, or its place in a launch shared with a weight gradient:
// dgrad_wgrad_kernel); smem: tap_gemm_lds() bytes
// OBN (forward, accumulator statistics, every block of the launch resident):
// the output's BatchNorm+LeakyReLU applied here too -- the block adds its
// sums, waits at a grid barrier, folds the accumulator (bn_apply_kernel's
// fold: the same mean / invstd) and writes leaky(bn(z)) of its accumulators
// to p.oy next to z (Conv1Bn has the first layer's form of the same).
// SPLIT (plain forward, LDS-DMA staging): 2 blocks per tile, each half of K; see TapGemm::split_part
template <bool DGRAD, int BN, bool C4 = false, int BM = FBM, int NST = 0, int CLS = 1, int ACT = 0, bool OBN = false,
          int SPLIT = 1>
__device__ __forceinline__ void tap_gemm_body(const TapGemm& p, char* smem, int bx, int by, int nwg) {
  static_assert(ACT == 0 || (!DGRAD && !C4 && NST >= 2), "the BN apply rides on the forward's LDS-DMA staging");
  static_assert(SPLIT == 1 || (SPLIT == 2 && !DGRAD && !C4 && NST >= 2 && ACT == 0 && !OBN), "split-K: plain forward");
  static_assert(!OBN || (!DGRAD && !C4 && ACT == 0), "the output BN: plain forward only");
  constexpr int RJ = BM / 32;                  // staged A rows per thread (ar + 32 j)
  constexpr int A_TILE = BM * F_ROW;
  constexpr int WGM = BN >= 64 ? 2 : 4, WGN = 4 / WGM;
  constexpr int RB = BN / 32;                  // staged B rows per thread (ar + 32 j)
  // epilogue tile row pitch (bytes): whole 128-byte rows at least, so the
  // 8-chunk XOR swizzle stays inside its row (a 32-channel row uses half)
  constexpr int T_ROW = BN >= 64 ? BN * 2 : F_ROW;
  constexpr int FM = BM / WGM / 16, FN = BN / WGN / 16;   // 16x16 fragments per wave
  // one stage = the A tile + a BN-row B tile; the epilogue's bf16 tile
  // ([BM][BN] bf16) and the per-wave channel sums (red, [4][2][BN])
  // reuse the staging space once the k-loop is done.  A 32-channel block
  // therefore takes 40 KiB, and four fit a CU's LDS (50 KiB fit three).
  constexpr int STG = A_TILE + BN * F_ROW;
  constexpr int E_TILE = BM * T_ROW;
  constexpr int NBUF = (C4 || NST == 0) ? 2 : NST;
  static_assert(NST == 0 || NST == 2 || NST == 3 || NST == 4, "staging: register ring, or 2-4 LDS-DMA stages");
  static_assert(NBUF * STG >= E_TILE + 4 * 2 * BN * 4, "epilogue does not fit the staging LDS");
  // the tile's row table after the staging space (not C4): {abase, vmask, obase, in range} per GEMM row
  constexpr int RT_OFF = NBUF * STG, RT = C4 ? 0 : BM * 16;
  constexpr int LUT_OFF = NBUF * STG + RT, LUTB = C4 ? kLutBytes : 0;   // C4: the u8 decode table
  static_assert(tap_gemm_lds<DGRAD, BN, C4, BM, NST>() == NBUF * STG + RT + LUTB, "tap_gemm_lds matches");
  float* red = reinterpret_cast<float*>(smem + E_TILE);   // [WGM][2][BN], after the epilogue tile
  const int t = int(threadIdx.x), lane = t & 63, wave = t >> 6;
  constexpr int NTAPS = DGRAD ? 4 : 16;
  // DIRECT (every layer but the im2col first layer): channels-as-rows tiles
  // (c1_row_chan) and an epilogue straight from the accumulators -- each lane
  // rounds its pixel's 8 channels and stores them with one 16-byte store, the
  // BatchNorm sums stay in registers.  The LDS round trip it replaces wrote
  // every value with a 2-byte ds_write (16 per lane per tile) behind a barrier.
  constexpr bool DIRECT = !C4;
  static_assert(!DIRECT || FN % 2 == 0, "channel fragments pair up");
  const int K = C4 ? FBK : NTAPS * p.C, NT = p.NOUT / BN;
  // data gradient: blockIdx.y is one stride-2 parity class (ph, pw), or with
  // p.cls_per_block == 4 the block runs all four classes of its pixel tile in
  // turn (the 32-channel layer: 4x fewer, 4x longer blocks -- its 4800
  // one-class blocks of 16 MFMAs per wave were prologue- and epilogue-bound)
  // (a compile-time count: with a runtime one the BN-backward sums stayed live
  // across the whole k-loop of every data gradient, 24 -> 32 us per layer)
  constexpr int ncls = DGRAD ? CLS : 1;
  int ph = 0, pw = 0;

  const int b = bx;
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wr = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  // split-K: consecutive work ids (one XCD) are the two K halves of one tile
  const int w = SPLIT > 1 ? wr / SPLIT : wr, khalf = SPLIT > 1 ? wr - w * SPLIT : 0;
  const int mt = w / NT, n0 = (w - mt * NT) * BN;
  const int m0 = mt * BM;
  // epilogue geometry: every thread takes whole 16-byte row chunks -- CPR
  // chunks per row, RPP rows per pass, NJ rows per thread (for BN = 32 that
  // is 2 rows of all 256 threads, not 4 rows of half of them)
  constexpr int CPR = BN / 8, RPP = kThreads / CPR, NJ = BM / RPP;
  const int ec = t % CPR;
  const bool bnf = DGRAD && p.bn.part != nullptr;
  // BN-backward sums (bnf), over every class this block runs: 8 channels per
  // 32-channel group of the wave (DIRECT), or the 8 of the lane's row chunk
  constexpr int NQ = DIRECT ? FN / 2 : 1;
  float bs[NQ][8], bq[NQ][8];
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) bs[q][e] = bq[q][e] = 0.f;
  for (int cls_i = 0; cls_i < ncls; ++cls_i) {
  if constexpr (DGRAD) {
    const int cls = by * ncls + cls_i;
    ph = cls >> 1;
    pw = cls & 1;
  }
  if (cls_i > 0) __syncthreads();   // the previous class's epilogue is done with the LDS

  // this thread's RJ GEMM rows (staging A, and the epilogue stores): ar + 32j
  const int ar = t >> 3, ac = t & 7;
  int rb[RJ], cb[RJ], base[RJ], obase[RJ];
  bool pin[RJ];
  // per row: byte offset of its tap-origin pixel (mod 2^32: border rows start
  // at -1, and only in-bounds taps are ever added to it) and a bitmask of the
  // taps that land inside the image -- the k-loop then costs one add and one
  // mask test per row instead of the full index and bounds arithmetic
  // (the mask is the outer product of the in-image tap rows and columns)
  constexpr int TW = DGRAD ? 2 : 4;   // taps per row of the tap grid
  // The in-image tap rows k (dr = k, or ph - k for the data gradient) form one
  // interval, so do the columns: two clamps each, then the interval bits are
  // spread over the tap grid with a multiply instead of a per-tap test.
  auto span = [](int lo, int hi) -> uint32_t {   // bits [lo, hi) of [0, TW)
    lo = lo < 0 ? 0 : lo;
    hi = hi > TW ? TW : hi;
    return hi > lo ? (1u << hi) - (1u << lo) : 0u;
  };
  auto tap_mask = [&](int r0, int c0) -> uint32_t {
    uint32_t rows, cols;
    if (DGRAD) {   // 0 <= rb + ph - k < SH  <=>  rb + ph - SH < k <= rb + ph
      rows = span(r0 + ph - p.SH + 1, r0 + ph + 1);
      cols = span(c0 + pw - p.SW + 1, c0 + pw + 1);
    } else {       // 0 <= rb + k < SH
      rows = span(-r0, p.SH - r0);
      cols = span(-c0, p.SW - c0);
    }
    if constexpr (TW == 4) {
      const uint32_t x = (rows | (rows << 3) | (rows << 6) | (rows << 9)) & 0x1111u;   // row k -> bit 4k
      return (x * 0xFu) & (cols * 0x1111u);
    } else {
      const uint32_t x = (rows | (rows << 1)) & 0x5u;                                   // row k -> bit 2k
      return (x * 0x3u) & (cols * 0x5u);
    }
  };
  uint32_t abase[RJ], vmask[RJ];
  if constexpr (!C4) {
    // Row table: thread t < BM works out row m0 + t once (two divisions, the
    // base offset, the tap mask, the output offset) and every thread reads
    // the RJ rows it stages from LDS.  Each row was worked out by all 8 lanes
    // that stage its chunks -- 8x the index math, most of the kernel's VALU.
    int4* rt = reinterpret_cast<int4*>(smem + RT_OFF);
    if (t < BM) {
      const int m = m0 + t;
      const bool in = m < p.M;
      const int mm = in ? m : 0;
      const int gn = mm / (p.GH * p.GW);
      const int rem = mm - gn * (p.GH * p.GW);
      const int ga = rem / p.GW, gbb = rem - ga * p.GW;
      const int r0 = DGRAD ? ga : 2 * ga - 1, c0 = DGRAD ? gbb : 2 * gbb - 1;
      const uint32_t ab = uint32_t((gn * p.SH + r0) * p.SW + c0) << (p.cshift + 1);
      const int ob = DGRAD ? ((gn * p.OH + 2 * ga + ph) * p.OW + 2 * gbb + pw) * p.NOUT : mm * p.NOUT;
      rt[t] = make_int4(int(ab), int(in ? tap_mask(r0, c0) : 0u), ob, in ? 1 : 0);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RJ; ++j) {
      const int4 r = rt[ar + 32 * j];
      abase[j] = uint32_t(r.x), vmask[j] = uint32_t(r.y), obase[j] = r.z, pin[j] = r.w != 0;
    }
  } else {
    // (n, a, b) of row ar by division, the next rows 32 GEMM rows on by stepping
    int gn, ga, gbb;
    {
      const int m = m0 + ar < p.M ? m0 + ar : 0;
      gn = m / (p.GH * p.GW);
      const int rem = m - gn * (p.GH * p.GW);
      ga = rem / p.GW;
      gbb = rem - ga * p.GW;
    }
#pragma unroll
    for (int j = 0; j < RJ; ++j) {
      const int m = m0 + ar + 32 * j;
      if (j > 0) {
        gbb += 32;
        while (gbb >= p.GW) {
          gbb -= p.GW;
          if (++ga == p.GH) ga = 0, ++gn;
        }
      }
      pin[j] = m < p.M;
      const int mm = pin[j] ? m : 0;
      rb[j] = 2 * ga - 1;
      cb[j] = 2 * gbb - 1;
      base[j] = (gn * p.SH + rb[j]) * p.SW + cb[j];
      obase[j] = mm * p.NOUT;
      abase[j] = uint32_t(base[j]) << (p.cshift + 1);
      vmask[j] = pin[j] ? tap_mask(rb[j], cb[j]) : 0u;
    }
  }
  const bool u8in = C4 && p.lut != nullptr;
  const __amdgpu_buffer_rsrc_t rs_src = make_rsrc(p.src, int64_t(p.N) * p.SH * p.SW * p.C * (u8in ? 1 : 2));
  if (u8in) {
    stage_lut(p.lut, smem + LUT_OFF);
    __syncthreads();
  }
  const __amdgpu_buffer_rsrc_t rs_w = make_rsrc(p.w, int64_t(p.NOUT) * 16 * p.C * 2);
  const uint16_t* wrow = p.w + (n0 + ar) * (16 * p.C);   // B rows ar + 32 j: 32 * 16 * C elements apart
  uint4 ra[RJ + RB];   // staged A rows, then B rows (one array: SROA keeps it in registers)
  uint4* const rbv = ra + RJ;
  auto load_c4 = [&]() {
    // first layer, 4-channel input: K = 16 taps x 4 = one k-step; chunk ac is
    // taps (kh, kw) and (kh, kw + 1) of one row -- two adjacent input pixels,
    // each checked against the border on its own
    const int kh = ac >> 1, kw = (ac & 1) * 2;
    if (u8in) {   // raw RGBA bytes -> bf16 through the LDS table (loads first, then the lookups)
      uint32_t w0[RJ], w1[RJ];
      bool k0[RJ], k1[RJ];
#pragma unroll
      for (int j = 0; j < RJ; ++j) {
        const bool rok = pin[j] && unsigned(rb[j] + kh) < unsigned(p.SH);
        const int e = (base[j] + kh * p.SW + kw) * 4;
        k0[j] = rok && unsigned(cb[j] + kw) < unsigned(p.SW);
        k1[j] = rok && unsigned(cb[j] + kw + 1) < unsigned(p.SW);
        w0[j] = bload4(rs_src, k0[j] ? uint32_t(e) : kOOB);
        w1[j] = bload4(rs_src, k1[j] ? uint32_t(e + 4) : kOOB);
      }
#pragma unroll
      for (int j = 0; j < RJ; ++j) {
        const uint2 lo = lut_px(smem + LUT_OFF, w0[j], k0[j]), hi = lut_px(smem + LUT_OFF, w1[j], k1[j]);
        ra[j] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
    } else {
#pragma unroll
      for (int j = 0; j < RJ; ++j) {
        const bool rok = pin[j] && unsigned(rb[j] + kh) < unsigned(p.SH);
        const int e = (base[j] + kh * p.SW + kw) * 4;
        const uint2 lo = bload8(rs_src, rok && unsigned(cb[j] + kw) < unsigned(p.SW) ? uint32_t(e) * 2u : kOOB);
        const uint2 hi = bload8(rs_src, rok && unsigned(cb[j] + kw + 1) < unsigned(p.SW) ? uint32_t(e + 4) * 2u : kOOB);
        ra[j] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
    }
    // weights: 4 input channels, or 3 (an RGB model fed RGBA: channel 3 gets weight 0)
    const int tap = kh * 4 + kw;
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int co = n0 + ar + 32 * j;
      if (p.wc == 4) {
        rbv[j] = *reinterpret_cast<const uint4*>(p.w + (co * 16 + tap) * 4);
      } else {
        const uint16_t* q = p.w + (co * 16 + tap) * 3;
        rbv[j] = make_uint4(uint32_t(q[0]) | (uint32_t(q[1]) << 16), uint32_t(q[2]),
                            uint32_t(q[3]) | (uint32_t(q[4]) << 16), uint32_t(q[5]));
      }
    }
  };
  const int nsteps = K / FBK / SPLIT;   // (split-K: this block's half; the host checks divisibility)
  const int ks0 = khalf * nsteps;
  auto load = [&](int ks) {
    if constexpr (C4) {
      load_c4();
      return;
    }
    // steps past the end (the ring's padding) load zeros for A -- the MFMA then
    // adds nothing -- and re-read the last step's weights (in bounds)
    const bool live = ks < nsteps;
    const int kc = (live ? ks : nsteps - 1) * FBK + ac * 8;
    const int tap = kc >> p.cshift, ch = kc & (p.C - 1);
    int dr, dc, wtap;
    if (DGRAD) {
      dr = ph - (tap >> 1);
      dc = pw - (tap & 1);
      wtap = (1 - ph + 2 * (tap >> 1)) * 4 + (1 - pw + 2 * (tap & 1));
    } else {
      dr = tap >> 2;
      dc = tap & 3;
      wtap = tap;
    }
    const uint32_t soff = uint32_t((((dr * p.SW + dc) << p.cshift) + ch) * 2);
    const uint32_t tbit = live ? 1u << tap : 0u;
#pragma unroll
    for (int j = 0; j < RJ; ++j) ra[j] = bload(rs_src, (vmask[j] & tbit) ? abase[j] + soff : kOOB);
    const int woff = wtap * p.C + ch;
#pragma unroll
    for (int j = 0; j < RB; ++j) rbv[j] = *reinterpret_cast<const uint4*>(wrow + j * (32 * 16) * p.C + woff);
  };
  const int st_a = f_off(ar, ac);   // rows ar + 32j keep the swizzle phase: (ar + 32j) & 7 == ar & 7
  // the B (channel) tile: DIRECT reads its rows in c1_row_chan order -> bkey swizzle (also ar + 32j invariant)
  const int st_b = DIRECT ? ar * F_ROW + ((ac ^ bkey(ar)) << 4) : st_a;
  auto store = [&](int buf) {
    char* ai = smem + buf * STG;
#pragma unroll
    for (int j = 0; j < RJ; ++j) *reinterpret_cast<uint4*>(ai + st_a + j * 32 * F_ROW) = ra[j];
#pragma unroll
    for (int j = 0; j < RB; ++j) *reinterpret_cast<uint4*>(ai + A_TILE + st_b + j * 32 * F_ROW) = rbv[j];
  };
  // LDS-DMA staging: one wave-instruction writes 1 KiB of LDS linearly (lane l
  // at 16 l), i.e. rows 8 w + 32 j .. + 7 of the tile, lane l on row 8 w +
  // 32 j + l / 8 at PHYSICAL chunk l & 7.  The XOR swizzle of the image
  // (logical chunk c at c ^ (row & 7)) therefore moves to the source: lane l
  // fetches logical chunk (l & 7) ^ (l / 8).  Border taps load out of range
  // (zeros).  All LDS in one array (a second __shared__ object makes hipcc
  // drain vmcnt before the fragment reads).
  const int acs = ac ^ (ar & 7);
  const int acs_b = DIRECT ? ac ^ bkey(ar) : acs;   // the B tile's logical chunk (its own swizzle)
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t wrow_b = uint32_t((n0 + ar) * 16 * p.C) * 2u;   // byte offset of B row ar
  auto issue = [&](int ks, int buf) {
    ks += ks0;
    const int kc = ks * FBK + acs * 8;
    const int tap = kc >> p.cshift, ch = kc & (p.C - 1);
    int dr, dc;
    if (DGRAD) {
      dr = ph - (tap >> 1);
      dc = pw - (tap & 1);
    } else {
      dr = tap >> 2;
      dc = tap & 3;
    }
    const int kcb = ks * FBK + acs_b * 8;
    const int tapb = kcb >> p.cshift, chb = kcb & (p.C - 1);
    const int wtap = DGRAD ? (1 - ph + 2 * (tapb >> 1)) * 4 + (1 - pw + 2 * (tapb & 1)) : tapb;
    const uint32_t soff = uint32_t((((dr * p.SW + dc) << p.cshift) + ch) * 2);
    const uint32_t tbit = 1u << tap;
    char* st = smem + buf * STG + wv * 1024;
#pragma unroll
    for (int j = 0; j < RJ; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_src, (__attribute__((address_space(3))) void*)(st + j * 4096), 16,
                                               int((vmask[j] & tbit) ? abase[j] + soff : kOOB), 0, 0, 0);
    const uint32_t woff = wrow_b + uint32_t(wtap * p.C + chb) * 2u;
#pragma unroll
    for (int j = 0; j < RB; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_w, (__attribute__((address_space(3))) void*)(st + A_TILE + j * 4096),
                                               16, int(woff + uint32_t(j * 32 * 16 * p.C) * 2u), 0, 0, 0);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wm = wave / WGN, wn = wave % WGN;
  const int row0 = wm * (BM / WGM), col0 = wn * (BN / WGN);
  // fragment read offsets (loop invariant): row r, chunk 4 kk + lane / 16
  int fa[FM][2], fb[FN][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int chunk = 4 * kk + (lane >> 4);
#pragma unroll
    for (int i = 0; i < FM; ++i) fa[i][kk] = f_off(row0 + 16 * i + (lane & 15), chunk);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int r = col0 + (DIRECT ? c1_row_chan(j, lane & 15) : 16 * j + (lane & 15));
      fb[j][kk] = A_TILE + (DIRECT ? r * F_ROW + ((chunk ^ bkey(r)) << 4) : f_off(r, chunk));
    }
  }
  auto mma = [&](int buf) {
    const char* ai = smem + buf * STG;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 a[FM], bb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i] = *reinterpret_cast<const bf16x8*>(ai + fa[i][kk]);
#pragma unroll
      for (int j = 0; j < FN; ++j) bb[j] = *reinterpret_cast<const bf16x8*>(ai + fb[j][kk]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = DIRECT ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb[j], a[i], acc[i][j], 0, 0, 0)
                             : __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bb[j], acc[i][j], 0, 0, 0);
    }
  };
  if constexpr (C4) {   // the first layer's K is one step
    load(0);
    store(0);
    __syncthreads();
    mma(0);
    __syncthreads();   // the epilogue tile overwrites stage 0
  } else if constexpr (NST > 0) {
    // NST - 1 stages in flight: at step ks wait for stage ks (the NST - 2
    // younger stages' NL loads each may stay out), barrier (stage ks is
    // visible to every wave, and every wave is done reading stage ks - 1),
    // refill stage ks - 1's buffer with step ks + NST - 1, then the MFMAs
    constexpr int NL = RJ + RB;   // LDS-DMA instructions per stage per thread
    constexpr uint32_t kWaitAll = (7u << 4) | (0xFu << 8);   // vmcnt(0), no lgkm / exp wait
    constexpr uint32_t kWaitOne = kWaitAll | uint32_t(NL & 15) | (uint32_t(NL >> 4) << 14);
    constexpr uint32_t kWaitTwo = kWaitAll | uint32_t((2 * NL) & 15) | (uint32_t((2 * NL) >> 4) << 14);
#pragma unroll
    for (int u = 0; u < NST - 1; ++u)
      if (u < nsteps) issue(u, u);
    // ACT: fold the BN statistics while the first stages load (scratch: the
    // last stage's buffer, issued only after the k-loop's first barrier)
    constexpr int NSET = ACT > 0 ? ACT : 1;
    float cis[NSET][8], cnm[NSET][8], cw[NSET][8], cb[NSET][8];
    if constexpr (ACT > 0) {
      double* part = reinterpret_cast<double*>(smem + (NST - 1) * STG);
      float* coef = reinterpret_cast<float*>(smem + (NST - 1) * STG + kThreads * 8);
      int* flag = reinterpret_cast<int*>(coef + 2 * p.C);
      bn_acc_column_sums(p.act.acc, p.act.R, 2 * p.C, part);
      BnFwdFinal f;
      f.eps = p.act.eps, f.momentum = p.act.momentum, f.mean = p.act.mean, f.invstd = p.act.invstd;
      f.rm = p.act.rm, f.rv = p.act.rv, f.tracked = p.act.tracked;
      for (int c = t; c < p.C; c += kThreads)
        bn_fwd_finalize(f, part, p.C, p.act.M, c, bx == 0, coef[c], coef[p.C + c]);
      __syncthreads();
      bn_acc_release(p.act.acc, p.act.R, p.C, flag, unsigned(bx), unsigned(nwg));
#pragma unroll
      for (int u = 0; u < NSET; ++u) {
        const int cbase = (u * FBK + acs * 8) & (p.C - 1);   // this thread's chunk channels at k-steps u, u + NSET, ...
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          cis[u][e] = coef[p.C + cbase + e];
          cnm[u][e] = -coef[cbase + e] * cis[u][e];
          cw[u][e] = p.act.w[cbase + e];
          cb[u][e] = p.act.b[cbase + e];
        }
      }
    }
    // leaky(bn(.)) of this thread's own chunks of stage ks, in place (coefficient set U)
    auto act_stage = [&](int ks, int buf, auto U) {
      constexpr int u = decltype(U)::value;
      const int kc = ks * FBK + acs * 8;
      const int tap = kc >> p.cshift, ch = kc & (p.C - 1);
      const uint32_t tbit = 1u << tap;
      const bool centre = p.act_out && n0 == 0 && unsigned((tap >> 2) - 1) < 2u && unsigned((tap & 3) - 1) < 2u;
      const uint32_t soff = uint32_t(((((tap >> 2) * p.SW + (tap & 3)) << p.cshift) + ch) * 2);
      char* st = smem + buf * STG + wv * 1024 + lane * 16;
#pragma unroll
      for (int j = 0; j < RJ; ++j) {
        if (!(vmask[j] & tbit)) continue;   // padding: stays zero
        uint4 v = *reinterpret_cast<const uint4*>(st + j * 4096);
        uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float z0 = fmaf(fmaf(__uint_as_float(w4[q] << 16), cis[u][2 * q], cnm[u][2 * q]), cw[u][2 * q],
                                cb[u][2 * q]);
          const float z1 = fmaf(fmaf(__uint_as_float(w4[q] & 0xFFFF0000u), cis[u][2 * q + 1], cnm[u][2 * q + 1]),
                                cw[u][2 * q + 1], cb[u][2 * q + 1]);
          const f32x2 pr = {z0 > 0.f ? z0 : z0 * p.act.slope, z1 > 0.f ? z1 : z1 * p.act.slope};
          w4[q] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pr, bf16x2));
        }
        v = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        *reinterpret_cast<uint4*>(st + j * 4096) = v;
        if (centre) *reinterpret_cast<uint4*>(reinterpret_cast<char*>(p.act_out) + (abase[j] + soff)) = v;
      }
    };
    int cur = 0;
    for (int ks = 0; ks < nsteps; ++ks) {
      // the stages younger than ks that were issued (the last steps issue none)
      const int younger = nsteps - 1 - ks < NST - 2 ? nsteps - 1 - ks : NST - 2;
      if (younger >= 2) __builtin_amdgcn_s_waitcnt(kWaitTwo);
      else if (younger == 1) __builtin_amdgcn_s_waitcnt(kWaitOne);
      else __builtin_amdgcn_s_waitcnt(kWaitAll);
      if constexpr (ACT == 1) {
        act_stage(ks, cur, std::integral_constant<int, 0>());
      } else if constexpr (ACT == 2) {
        if (ks & 1) act_stage(ks, cur, std::integral_constant<int, 1>());
        else act_stage(ks, cur, std::integral_constant<int, 0>());
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const int nxt = ks + NST - 1;
      if (nxt < nsteps) issue(nxt, cur == 0 ? NST - 1 : cur - 1);
      mma(cur);
      cur = cur == NST - 1 ? 0 : cur + 1;
    }
    __syncthreads();   // the epilogue reuses the staging LDS
  } else {
    // Loads run kDepth steps ahead of the MFMAs in a register ring: with one
    // step of prefetch every k-step waited out a full global-load latency, and
    // the deep-K layers (16-32 steps) were latency-bound.  The barrier is
    // LDS-only, so the ring's later stages stay in flight across it (counted
    // vmcnt waits on the stage being stored).
    constexpr int kDepth = 2;
    uint4 ring[kDepth][RJ + RB];
    int ks_next = 0;
    auto fetch = [&](int u) {
      load(ks_next++);
#pragma unroll
      for (int j = 0; j < RJ + RB; ++j) ring[u][j] = ra[j];
    };
#pragma unroll
    for (int u = 0; u < kDepth; ++u) fetch(u);
    const int padded = (nsteps + kDepth - 1) / kDepth * kDepth;
    for (int s0 = 0; s0 < padded; s0 += kDepth) {
#pragma unroll
      for (int u = 0; u < kDepth; ++u) {
        const int buf = u & 1;   // kDepth is even: (s0 + u) & 1
#pragma unroll
        for (int j = 0; j < RJ + RB; ++j) ra[j] = ring[u][j];
        store(buf);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        fetch(u);                // step s0 + u + kDepth
        mma(buf);
      }
    }
    __syncthreads();   // the epilogue reuses the staging LDS
  }

  if constexpr (SPLIT > 1) {
    // split-K: the first block of the tile's pair to get here parks its accumulators (device-scope
    // stores, written through this XCD's L2) and leaves; the second waits for them (the first is
    // running -- it took the ticket -- so the wait is bounded), adds them to its own (a + b == b + a:
    // the same bits whichever half finishes first) and runs the epilogue
    unsigned* role = reinterpret_cast<unsigned*>(smem);   // (the staging LDS is free: DIRECT epilogue)
    unsigned* tk = p.split_ticket + 2 * w;
    if (t == 0) *role = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const unsigned first = *role == 0u;
    const __amdgpu_buffer_rsrc_t rs_part =
        make_rsrc(p.split_part + int64_t(w) * (FM * FN) * kThreads * 4, int64_t(FM * FN) * kThreads * 16);
    if (first) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs_part,
                                                 ((i * FN + j) * kThreads + t) * 16, 0, 16 /* sc1 */);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t == 0) __hip_atomic_store(tk + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    if (t == 0) {
      unsigned n = 0;
      while (__hip_atomic_load(tk + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        __builtin_amdgcn_s_sleep(2);
        if (++n == kBarrierSpins) {   // (never expected: flag it like a failed grid barrier)
          atomicAdd(&g_grid_barrier_timeouts, 1u);
          if (unsigned* f = g_grid_barrier_flag) __hip_atomic_store(f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
      __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // both words zero for the next launch
      __hip_atomic_store(tk + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs_part, ((i * FN + j) * kThreads + t) * 16, 0, 16);
        acc[i][j] += __builtin_bit_cast(f32x4, v);
      }
  }

  if constexpr (DIRECT) {
    // this lane's pixel of fragment i: GEMM row row0 + 16 i + (lane & 15), its
    // output offset and range flag from the row table; its channels: 32 q + 8 g .. + 7
    const int g = lane >> 4;
    const int4* rtab = reinterpret_cast<const int4*>(smem + RT_OFF);
    int ob[FM];
    bool pv[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int4 r = rtab[row0 + 16 * i + (lane & 15)];
      ob[i] = r.z + n0 + col0 + 8 * g, pv[i] = r.w != 0;
    }
    // BN-backward fusion: the BN input at the same offsets and the lane's per-channel BN inputs, every
    // load issued before any is used, unconditionally (buffer loads; out of range without the BN or
    // past the tile: zeros).  The per-channel values as scalar loads, each consumed at once, made the
    // compiler reuse one register for all of them: 8 memory round trips in series in every data-
    // gradient block's epilogue.
    uint4 xq[FM][NQ];
    float is[NQ][8], nm[NQ][8], ww[NQ][8], bb[NQ][8];
    if constexpr (DGRAD) {
      const __amdgpu_buffer_rsrc_t rs_bx =
          make_rsrc(bnf ? static_cast<const void*>(p.bn.x) : p.dst, bnf ? int64_t(p.N) * p.OH * p.OW * p.NOUT * 2 : 0);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int q = 0; q < NQ; ++q) xq[i][q] = bload(rs_bx, pv[i] ? uint32_t(ob[i] + 32 * q) * 2u : kOOB);
      const float* src[4] = {p.bn.invstd, p.bn.mean, p.bn.w, p.bn.b};
      float4 cv[4][NQ][2];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const __amdgpu_buffer_rsrc_t rc = make_rsrc(bnf ? static_cast<const void*>(src[a]) : p.dst, bnf ? p.NOUT * 4 : 0);
#pragma unroll
        for (int q = 0; q < NQ; ++q)
#pragma unroll
          for (int h = 0; h < 2; ++h)
            cv[a][q][h] = __builtin_bit_cast(float4, bload(rc, uint32_t(n0 + col0 + 32 * q + 8 * g + 4 * h) * 4u));
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          auto pick = [&](int a) {
            const float4 f = cv[a][q][e >> 2];
            const int k = e & 3;
            return k == 0 ? f.x : k == 1 ? f.y : k == 2 ? f.z : f.w;
          };
          is[q][e] = pick(0);
          nm[q][e] = -pick(1) * is[q][e];
          ww[q][e] = pick(2);
          bb[q][e] = pick(3);
        }
    }
    float sum[NQ][8], sq[NQ][8];
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) sum[q][e] = sq[q][e] = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        uint32_t pk[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {   // channels 8 g + 2 h, + 1: fragment 2 q + (h >> 1), rows 2 (h & 1), + 1
          const f32x4& a = acc[i][2 * q + (h >> 1)];
          const f32x2 pr = {a[2 * (h & 1)], a[2 * (h & 1) + 1]};
          pk[h] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pr, bf16x2));   // RNE
        }
        if (!pv[i]) continue;
        *reinterpret_cast<uint4*>(p.dst + ob[i] + 32 * q) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        if (!DGRAD && p.stats) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float v = __uint_as_float(e & 1 ? pk[e >> 1] & 0xFFFF0000u : pk[e >> 1] << 16);
            sum[q][e] += v;
            sq[q][e] += v * v;
          }
        }
        if (bnf) {
          const uint32_t xw[4] = {xq[i][q].x, xq[i][q].y, xq[i][q].z, xq[i][q].w};
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float gv = __uint_as_float(e & 1 ? pk[e >> 1] & 0xFFFF0000u : pk[e >> 1] << 16);
            const float xh = fmaf(__uint_as_float(e & 1 ? xw[e >> 1] & 0xFFFF0000u : xw[e >> 1] << 16),
                                  is[q][e], nm[q][e]);
            const float gz = fmaf(xh, ww[q][e], bb[q][e]) > 0.f ? gv : gv * p.bn.slope;
            bs[q][e] += gz;
            bq[q][e] += gz * xh;
          }
        }
      }
    if (!DGRAD && p.stats) {
      // the 16 lanes of a group hold the same channels; then the WGN waves of a
      // row group write disjoint channel ranges of row wm
#pragma unroll
      for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e)
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) sum[q][e] += __shfl_xor(sum[q][e], o), sq[q][e] += __shfl_xor(sq[q][e], o);
      if ((lane & 15) == 0) {
#pragma unroll
        for (int q = 0; q < NQ; ++q)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            red[(wm * 2 + 0) * BN + col0 + 32 * q + 8 * g + e] = sum[q][e];
            red[(wm * 2 + 1) * BN + col0 + 32 * q + 8 * g + e] = sq[q][e];
          }
      }
      __syncthreads();
    }
    if constexpr (OBN) {
      // the block's sums (as at the end of the body otherwise), the barrier, the fold
      double* acc64 = reinterpret_cast<double*>(p.stats);
      if (t < 2 * BN) {
        const int which = t / BN, c = t - which * BN;
        float v = 0.f;
#pragma unroll
        for (int g2 = 0; g2 < WGM; ++g2) v += red[(g2 * 2 + which) * BN + c];
        unsafeAtomicAdd(acc64 + ((mt % p.acc_r) * 2 + which) * p.NOUT + n0 + c, double(v));
      }
      grid_barrier(bn_acc_barrier(acc64, p.acc_r, p.NOUT), unsigned(nwg));
      // (the staging LDS is free: the sums, then every channel's mean / invstd)
      double* part = reinterpret_cast<double*>(smem);
      float* coef = reinterpret_cast<float*>(smem + 8 * (2 * kBnFoldMaxC > kThreads ? 2 * kBnFoldMaxC : kThreads));
      static_assert(NBUF * STG >= 8 * 2 * kBnFoldMaxC + 4 * 2 * kBnFoldMaxC, "fold scratch");
      __shared__ int oflag;
      bn_acc_column_sums<true>(acc64, p.acc_r, 2 * p.NOUT, part);
      for (int c = t; c < p.NOUT; c += kThreads) {
        BnFwdFinal fin;
        fin.eps = p.oact.eps, fin.momentum = p.oact.momentum;
        fin.mean = p.oact.mean, fin.invstd = p.oact.invstd;
        fin.rm = p.oact.rm, fin.rv = p.oact.rv, fin.tracked = p.oact.tracked;
        float mu, is1;
        bn_fwd_finalize(fin, part, p.NOUT, p.oact.M, c, bx == 0 && by == 0, mu, is1);
        coef[c] = mu;
        coef[p.NOUT + c] = is1;
      }
      __syncthreads();
      bn_acc_release(acc64, p.acc_r, p.NOUT, &oflag, unsigned(bx), unsigned(nwg));
      float ois[NQ][8], onm[NQ][8], oww[NQ][8], obb[NQ][8];
#pragma unroll
      for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int c = n0 + col0 + 32 * q + 8 * g + e;
          ois[q][e] = coef[p.NOUT + c];
          onm[q][e] = -coef[c] * ois[q][e];
          oww[q][e] = p.oact.w[c];
          obb[q][e] = p.oact.b[c];
        }
      const float slope = p.oact.slope;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          if (!pv[i]) continue;
          uint32_t o[4];
#pragma unroll
          for (int h = 0; h < 4; ++h) {   // the same bf16 z as stored above, then bn_apply_kernel's arithmetic
            const f32x4& a = acc[i][2 * q + (h >> 1)];
            const f32x2 pr = {a[2 * (h & 1)], a[2 * (h & 1) + 1]};
            const uint32_t zz = __builtin_bit_cast(uint32_t, __builtin_convertvector(pr, bf16x2));
            f32x2 r;
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
              const int e = 2 * h + s2;
              const float x = s2 ? __uint_as_float(zz & 0xFFFF0000u) : __uint_as_float(zz << 16);
              const float z = fmaf(fmaf(x, ois[q][e], onm[q][e]), oww[q][e], obb[q][e]);
              r[s2] = z > 0.f ? z : z * slope;
            }
            o[h] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, bf16x2));
          }
          *reinterpret_cast<uint4*>(p.oy + ob[i] + 32 * q) = make_uint4(o[0], o[1], o[2], o[3]);
        }
    }
  } else {
  // Epilogue stores (geometry above)
  int eob[NJ];
  bool epin[NJ];
  if constexpr (BN == 64) {   // the staging rows ar + 32 j
#pragma unroll
    for (int j = 0; j < NJ; ++j) eob[j] = obase[j], epin[j] = pin[j];
  } else if constexpr (!C4) {  // rows t / CPR + RPP j: from the row table
    const int4* rt = reinterpret_cast<const int4*>(smem + RT_OFF);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int4 r = rt[t / CPR + RPP * j];
      eob[j] = r.z, epin[j] = r.w != 0;
    }
  } else {                     // (C4, forward) rows t / CPR + RPP j: divide once, then step
    const int m_first = m0 + t / CPR;
    int en = 0, ea = 0, eb = 0;
    {
      const int m = m_first < p.M ? m_first : 0;
      en = m / (p.GH * p.GW);
      const int rem = m - en * (p.GH * p.GW);
      ea = rem / p.GW;
      eb = rem - ea * p.GW;
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      if (j > 0) {
        eb += RPP;
        while (eb >= p.GW) {
          eb -= p.GW;
          if (++ea == p.GH) ea = 0, ++en;
        }
      }
      const int m = m_first + RPP * j;
      epin[j] = m < p.M;
      eob[j] = m * p.NOUT;
    }
  }
  // BN-backward fusion (below): issue the BN input loads now, so their
  // latency hides under the epilogue's LDS round trip
  uint4 xpre[NJ];
  if (bnf) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      xpre[j] = epin[j] ? *reinterpret_cast<const uint4*>(p.bn.x + eob[j] + n0 + ec * 8) : make_uint4(0, 0, 0, 0);
  }

  // epilogue: round to bf16 (RNE) into an LDS tile [BM][BN] (128-byte row
  // pitch, same swizzle), sum the rounded values per channel (forward), then
  // 16-byte stores of whole row chunks
  uint16_t* tile = reinterpret_cast<uint16_t*>(smem);
  float sum[FN], sq[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) sum[j] = sq[j] = 0.f;
  // LDS element offsets of this lane's values: row row0 + 16 i + lr + r has
  // swizzle phase (lr + r) & 7 for every i (row0 and 16 i are multiples of 8),
  // so the 4 x FN offsets are computed once and i only adds 16 rows
  const int lr = 4 * (lane >> 4);
  int toff[FN][4];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int col = col0 + 16 * j + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      toff[j][r] = (row0 + lr + r) * (T_ROW / 2) + ((((col >> 3) ^ ((lr + r) & 7)) << 4) >> 1) + (col & 7);
  }
  const bool all_rows = m0 + BM <= p.M;   // the tile holds no row past the GEMM
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      // RNE to bf16, two values per v_cvt_pk_bf16_f32
      uint32_t pk[2];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const f32x2 pr = {acc[i][j][2 * h2], acc[i][j][2 * h2 + 1]};
        pk[h2] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pr, bf16x2));
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t w2 = pk[r >> 1];
        tile[toff[j][r] + i * 16 * (T_ROW / 2)] = uint16_t(r & 1 ? w2 >> 16 : w2);
        if (!DGRAD && (all_rows || m0 + row0 + 16 * i + lr + r < p.M)) {
          const float vr = __uint_as_float(r & 1 ? w2 & 0xFFFF0000u : w2 << 16);
          sum[j] += vr;
          sq[j] += vr * vr;
        }
      }
    }
  if (!DGRAD && p.stats) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {   // lanes l, l^16, l^32, l^48 hold the same channel
      sum[j] += __shfl_xor(sum[j], 16);
      sum[j] += __shfl_xor(sum[j], 32);
      sq[j] += __shfl_xor(sq[j], 16);
      sq[j] += __shfl_xor(sq[j], 32);
    }
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        red[(wm * 2 + 0) * BN + col0 + 16 * j + lane] = sum[j];
        red[(wm * 2 + 1) * BN + col0 + 16 * j + lane] = sq[j];
      }
    }
  }
  __syncthreads();
  // data gradient feeding a BatchNorm+LeakyReLU backward (p.bn.part): the
  // stored gradient IS that backward's gy.  Per channel, sum gz and gz * xhat
  // over this tile (gz = gy * leaky'(z), z = xhat * w + b, xhat from the BN's
  // saved input at the same offsets) -- the reduction pass over gy and x the
  // BN backward would otherwise make.
  float is[8], nm[8], ww[8], bb[8];
  if (bnf) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = n0 + ec * 8 + q;
      is[q] = p.bn.invstd[c];
      nm[q] = -p.bn.mean[c] * is[q];
      ww[q] = p.bn.w[c];
      bb[q] = p.bn.b[c];
    }
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    if (!epin[j]) continue;
    const int er = t / CPR + RPP * j;
    const uint4 v = *reinterpret_cast<const uint4*>(smem + er * T_ROW + ((ec ^ (er & 7)) << 4));
    *reinterpret_cast<uint4*>(p.dst + eob[j] + n0 + ec * 8) = v;
    if (bnf) {
      const uint4 xv = xpre[j];
      const uint32_t gw[4] = {v.x, v.y, v.z, v.w}, xw[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint32_t gb = q & 1 ? gw[q >> 1] & 0xFFFF0000u : gw[q >> 1] << 16;
        const uint32_t xb = q & 1 ? xw[q >> 1] & 0xFFFF0000u : xw[q >> 1] << 16;
        const float xh = fmaf(__uint_as_float(xb), is[q], nm[q]);
        const float g = __uint_as_float(gb);
        const float gz = fmaf(xh, ww[q], bb[q]) > 0.f ? g : g * p.bn.slope;
        bs[0][q] += gz;
        bq[0][q] += gz * xh;
      }
    }
  }
  }
  }   // parity classes
  if (bnf) {
    // lanes holding the same channels fold, then the row groups through LDS
    // (the statistics area is free in backward): DIRECT -- the 16 lanes of a
    // group, waves (wm, wn) writing row wm; else lanes with the same ec, 4 waves
    constexpr int RG = DIRECT ? WGM : 4;
    if constexpr (DIRECT) {
      const int g = lane >> 4, wm = wave / WGN, col0 = (wave % WGN) * (BN / WGN);
#pragma unroll
      for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e)
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) bs[q][e] += __shfl_xor(bs[q][e], o), bq[q][e] += __shfl_xor(bq[q][e], o);
      __syncthreads();   // every wave is done with the last class's LDS
      if ((lane & 15) == 0) {
#pragma unroll
        for (int q = 0; q < NQ; ++q)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            red[(wm * 2 + 0) * BN + col0 + 32 * q + 8 * g + e] = bs[q][e];
            red[(wm * 2 + 1) * BN + col0 + 32 * q + 8 * g + e] = bq[q][e];
          }
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
#pragma unroll
        for (int o = CPR; o < 64; o <<= 1) bs[0][q] += __shfl_xor(bs[0][q], o), bq[0][q] += __shfl_xor(bq[0][q], o);
      }
      if (lane < CPR) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          red[(wave * 2 + 0) * BN + ec * 8 + q] = bs[0][q];
          red[(wave * 2 + 1) * BN + ec * 8 + q] = bq[0][q];
        }
      }
    }
    __syncthreads();
    if (t < 2 * BN) {
      const int which = t / BN, c = t - which * BN;
      float v = 0.f;
#pragma unroll
      for (int w4 = 0; w4 < RG; ++w4) v += red[(w4 * 2 + which) * BN + c];
      // channel-major [2][NOUT][rows], row = (pixel tile, parity class); or
      // added into replica row % R of an accumulator [R][2][NOUT] (bn_bwd_apply_acc folds it)
      const int row = mt * 4 + by * ncls;
      if (p.bn.acc_r > 0) {
        unsafeAtomicAdd(reinterpret_cast<double*>(p.bn.part) + ((row % p.bn.acc_r) * 2 + which) * p.NOUT + n0 + c,
                        double(v));
      } else {
        p.bn.part[(which * p.NOUT + n0 + c) * p.bn.rows + row] = v;
        for (int k = 1; k < ncls; ++k) p.bn.part[(which * p.NOUT + n0 + c) * p.bn.rows + row + k] = 0.f;
      }
    }
  }
  if (!OBN && !DGRAD && p.stats && t < 2 * BN) {
    const int which = t / BN, c = t - which * BN;   // 0: sum, 1: sum of squares
    float v = 0.f;
#pragma unroll
    for (int g = 0; g < WGM; ++g) v += red[(g * 2 + which) * BN + c];
    // channel-major [2][NOUT][tiles], the layout bn_finalize_rows folds; or
    // added into replica mt % R of an accumulator [R][2][NOUT] (bn_apply_acc folds it)
    if (p.acc_r > 0)
      unsafeAtomicAdd(reinterpret_cast<double*>(p.stats) + ((mt % p.acc_r) * 2 + which) * p.NOUT + n0 + c, double(v));
    else p.stats[(which * p.NOUT + n0 + c) * ((p.M + BM - 1) / BM) + mt] = v;
  }
}

template <bool DGRAD, int BN, bool C4 = false, int BM = FBM, int NST = 0, int CLS = 1, int ACT = 0, bool OBN = false,
          int SPLIT = 1>
__global__ __launch_bounds__(kThreads) void tap_gemm_kernel(TapGemm p) {
  __shared__ __attribute__((aligned(16))) char smem[tap_gemm_lds<DGRAD, BN, C4, BM, NST>()];
  tap_gemm_body<DGRAD, BN, C4, BM, NST, CLS, ACT, OBN, SPLIT>(p, smem, int(blockIdx.x), int(blockIdx.y),
                                                             int(gridDim.x));
}

// ---------------------------------------------------------------------------
// The first layer's forward (4-channel RGBA input, raw u8 through the decode
// table or decoded bf16; K = 16 taps x 4 channels = 64) from a decoded input
// PATCH.  As an im2col GEMM (the C4 path of tap_gemm_kernel) each output
// pixel gathers its 16 input pixels -- a stride-2 4x4 window re-reads every
// input pixel 4 times, so the LUT decode and the A-tile stores ran 4x per
// input pixel, and the kernel was VALU/LDS bound at ~51 VALU per MFMA
// (profiles/r4/disc_pmc_b2.txt).  Here a block decodes the (2 TR + 2) x 130
// input pixels under a TR x 64 output tile ONCE into LDS (8 bytes a pixel,
// rows of 1,040 bytes) and reads each MFMA operand straight out of it: the
// k-chunk (kh, kw..kw+1) of output pixel (r, c) is the 16 bytes at patch
// (2r + kh, 2c + kw), 16-byte aligned because the patch starts one pixel
// left of the tile's first input column.
//
// The weights are the MFMA's A operand (rows = output channels, held in
// registers for the whole block) and the patch the B operand (columns =
// pixels), so a lane's accumulator holds 4 channels of ONE pixel; fragment
// pairs map their rows to channels 8g..8g+7 of a 32-channel group (lane group
// g), and the lane writes them with one 16-byte store -- no LDS epilogue.
// T tiles per block: the table and weights are staged once, the next tile's
// frame loads are in flight while this tile computes, and the BatchNorm sums
// stay in registers until the block's last tile.
constexpr int kC1Cols = 64;   // output columns per tile

// KEEP > 0: the BatchNorm+LeakyReLU that consumes this layer's output is
// applied here too.  Every block keeps its KEEP tiles' bf16 outputs in
// registers, adds its BN sums into the accumulator, and waits at a grid
// barrier (every block resident: the host launches at most the occupancy
// limit); then each block folds the accumulator (as bn_apply_kernel does: the
// same mean / invstd, bit for bit), applies leaky(bn(z)) to its kept tiles and
// writes them to y.  z still goes out as before (the BN's saved input).  One
// launch and one read of z fewer than conv1 + the BN apply kernel.
struct Conv1Bn {
  BnActIn act;              // acc = p.stats (fp64 [R][2][BN]); mean / invstd / running statistics written by block 0
  uint16_t* y = nullptr;    // leaky(bn(z)), [N][OH][OW][BN] bf16
};
constexpr int kConv1Keep = 10;   // tiles per block of the BN-applying launch (80 VGPRs of kept outputs)

template <int BN, int TR, bool U8, int KEEP = 0>
__global__ __launch_bounds__(kThreads) void conv1_fwd_kernel(TapGemm p, int tiles_per_block, Conv1Bn ob) {
  constexpr int PR = 2 * TR + 2, PC = 2 * kC1Cols + 2, PX = PR * PC;
  constexpr int NL = (PX + kThreads - 1) / kThreads;   // patch pixels per thread
  constexpr int FC = BN / 16, CP = BN / 32;            // channel fragments, 32-channel groups
  constexpr int PF = TR * kC1Cols / 16 / 4;            // 16-pixel fragments per wave
  constexpr int LUT_OFF = PX * 8, RED_OFF = LUT_OFF + kLutBytes;
  static_assert(PF >= 1 && (TR * kC1Cols) % 64 == 0, "tile");
  __shared__ __attribute__((aligned(16))) char smem[RED_OFF + 4 * 2 * BN * 4];
  float* red = reinterpret_cast<float*>(smem + RED_OFF);
  const int t = int(threadIdx.x), lane = t & 63, wave = t >> 6;
  const int tiles_r = (p.OH + TR - 1) / TR, tiles_c = (p.OW + kC1Cols - 1) / kC1Cols;
  const int ntiles = p.N * tiles_r * tiles_c;
  if constexpr (KEEP > 0) tiles_per_block = KEEP;
  const int tile0 = int(blockIdx.x) * tiles_per_block;
  const int tile1 = tile0 + tiles_per_block < ntiles ? tile0 + tiles_per_block : ntiles;
  constexpr bool u8in = U8;   // raw u8 frames through the table (a template parameter: a runtime branch
                              // between the load kinds put the in-flight words in scratch)
  if (u8in) stage_lut(p.lut, smem + LUT_OFF);
  // the weights, once, as A fragments: row rho of fragment f = channel c1_row_chan(f, rho);
  // k-chunk 4 kk + (lane >> 4) = taps (kh, kw), (kh, kw + 1), kh = chunk >> 1, kw = 2 (chunk & 1)
  bf16x8 wa[FC][2];
#pragma unroll
  for (int f = 0; f < FC; ++f)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int co = c1_row_chan(f, lane & 15), chunk = 4 * kk + (lane >> 4);
      const int tap = (chunk >> 1) * 4 + (chunk & 1) * 2;
      uint4 v;
      if (p.wc == 4) {
        v = *reinterpret_cast<const uint4*>(p.w + (co * 16 + tap) * 4);
      } else {   // an RGB weight on RGBA input: channel 3 gets weight 0
        const uint16_t* q = p.w + (co * 16 + tap) * 3;
        v = make_uint4(uint32_t(q[0]) | (uint32_t(q[1]) << 16), uint32_t(q[2]),
                       uint32_t(q[3]) | (uint32_t(q[4]) << 16), uint32_t(q[5]));
      }
      wa[f][kk] = __builtin_bit_cast(bf16x8, v);
    }
  const __amdgpu_buffer_rsrc_t rs_src = make_rsrc(p.src, int64_t(p.N) * p.SH * p.SW * p.C * (u8in ? 1 : 2));
  // this thread's patch pixels u = t + 256 i: (row, column) within the patch
  int pr[NL], pc[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int u = t + kThreads * i;
    pr[i] = u < PX ? u / PC : -8;   // past the patch: never in range
    pc[i] = u - (u / PC) * PC;
  }
  uint32_t w0[NL], w1[NL];   // raw pixels in flight (u8: the RGBA word; bf16: two words)
  bool ok[NL];
  // act_out (u8 input): the decoded frame, bf16 NHWC RGBA -- each tile stores the 2 TR x 128 input
  // pixels it owns (patch rows 1 .. 2 TR, columns 1 .. 128; even sides: every pixel once), the
  // weight gradient's operand without a decode of its own
  uint32_t eo[NL];
  // Every load and store of the tile loop is issued unconditionally (buffer ops: out-of-range ones
  // read zeros / are dropped), so the compiler's memory-counter waits count exactly: a store issued
  // on only some paths made its wait for a tile's patch loads vmcnt(0) -- the previous tile's
  // output stores too, a write round trip per tile in series with the read one.  tile < 0: a dead
  // prefetch past the block's last tile.
  const __amdgpu_buffer_rsrc_t rs_dst = make_rsrc(p.dst, int64_t(p.N) * p.OH * p.OW * p.NOUT * 2);
  const __amdgpu_buffer_rsrc_t rs_act =
      make_rsrc(p.act_out, p.act_out ? int64_t(p.N) * p.SH * p.SW * 8 : 0);   // (none: every store dropped)
  auto load_patch = [&](int tile) __attribute__((always_inline)) {
    const bool live = tile >= 0;
    const int tl = live ? tile : 0;
    const int n = tl / (tiles_r * tiles_c), rem = tl - n * (tiles_r * tiles_c);
    const int r0 = 2 * (rem / tiles_c) * TR - 1, c0 = 2 * (rem % tiles_c) * kC1Cols - 1;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int ir = r0 + pr[i], ic = c0 + pc[i];
      ok[i] = live && unsigned(ir) < unsigned(p.SH) && unsigned(ic) < unsigned(p.SW);
      const uint32_t e = uint32_t(((n * p.SH + ir) * p.SW + ic) * 4);
      eo[i] = ok[i] && unsigned(pr[i] - 1) < unsigned(2 * TR) && unsigned(pc[i] - 1) < unsigned(2 * kC1Cols) ? e : ~0u;
      if constexpr (u8in) {
        w0[i] = bload4(rs_src, ok[i] ? e : kOOB);
      } else {
        const uint2 v = bload8(rs_src, ok[i] ? e * 2u : kOOB);
        w0[i] = v.x, w1[i] = v.y;
      }
    }
  };
  auto store_patch = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const uint2 v = u8in ? lut_px(smem + LUT_OFF, w0[i], ok[i]) : make_uint2(w0[i], w1[i]);
      if ((i + 1) * kThreads <= PX || t + kThreads * i < PX) *reinterpret_cast<uint2*>(smem + (t + kThreads * i) * 8) = v;
      if constexpr (u8in)
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{v.x, v.y}, rs_act, eo[i] != ~0u ? eo[i] * 2u : kOOB, 0, 0);
    }
  };
  // the B fragments' patch offsets (tile-invariant): pixel fragment j of this
  // wave = output row fi / 4, columns 16 (fi % 4) .. +15
  int boff[PF][2];
#pragma unroll
  for (int j = 0; j < PF; ++j) {
    const int fi = wave * PF + j, r = fi >> 2, c = 16 * (fi & 3) + (lane & 15);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = 4 * kk + (lane >> 4);
      boff[j][kk] = ((2 * r + (chunk >> 1)) * PC + 2 * c + 2 * (chunk & 1)) * 8;
    }
  }
  const int g = lane >> 4;
  float sum[CP][8], sq[CP][8];
#pragma unroll
  for (int q = 0; q < CP; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) sum[q][e] = sq[q][e] = 0.f;

  // KEEP: the tiles' bf16 outputs, kept for the BN apply after the grid barrier
  uint32_t keep[KEEP > 0 ? KEEP : 1][PF][CP][4];
  auto tile_body = [&](int tile, int k) __attribute__((always_inline)) {
    __syncthreads();                 // the previous tile's fragment reads are done (and, first, the table)
    store_patch();                   // decode (the table lookups wait for this tile's loads)
    load_patch(tile + 1 < tile1 ? tile + 1 : -1);   // in flight while this tile computes and stores
    __syncthreads();
    f32x4 acc[FC][PF];
#pragma unroll
    for (int f = 0; f < FC; ++f)
#pragma unroll
      for (int j = 0; j < PF; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 b[PF];
#pragma unroll
      for (int j = 0; j < PF; ++j) b[j] = *reinterpret_cast<const bf16x8*>(smem + boff[j][kk]);
#pragma unroll
      for (int f = 0; f < FC; ++f)
#pragma unroll
        for (int j = 0; j < PF; ++j)
          acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[f][kk], b[j], acc[f][j], 0, 0, 0);
    }
    const int n = tile / (tiles_r * tiles_c), rem = tile - n * (tiles_r * tiles_c);
    const int orow0 = (rem / tiles_c) * TR, ocol0 = (rem % tiles_c) * kC1Cols;
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const int fi = wave * PF + j;
      const int orow = orow0 + (fi >> 2), ocol = ocol0 + 16 * (fi & 3) + (lane & 15);
      const bool in = orow < p.OH && ocol < p.OW;
      const uint32_t ob0 = in ? uint32_t(((n * p.OH + orow) * p.OW + ocol) * p.NOUT + 8 * g) * 2u : kOOB;
#pragma unroll
      for (int q = 0; q < CP; ++q) {
        uint32_t pk[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {   // channels 8g + 2h, +1: fragment 2q + (h >> 1), rows 2 (h & 1), +1
          const f32x4& a = acc[2 * q + (h >> 1)][j];
          const f32x2 pr2 = {a[2 * (h & 1)], a[2 * (h & 1) + 1]};
          pk[h] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pr2, bf16x2));
          const float lo = in ? __uint_as_float(pk[h] << 16) : 0.f, hi = in ? __uint_as_float(pk[h] & 0xFFFF0000u) : 0.f;
          sum[q][2 * h] += lo, sq[q][2 * h] += lo * lo;
          sum[q][2 * h + 1] += hi, sq[q][2 * h + 1] += hi * hi;
          if constexpr (KEEP > 0) keep[k][j][q][h] = pk[h];
        }
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{pk[0], pk[1], pk[2], pk[3]}, rs_dst,
                                               ob0 == kOOB ? kOOB : ob0 + 64u * q, 0, 0);
      }
    }
  };
  if (tile0 < tile1) load_patch(tile0);
  // every prologue load (weights, table, the first patch) complete here, as a real waitcnt the
  // compiler's counter tracking sees: otherwise the weight fragments' loads stay "pending" through
  // the tile loop's merge and every tile's MFMAs waited for vmcnt(0) -- the NEXT tile's patch loads
  // too, which serialised the prefetch with the compute
  __builtin_amdgcn_s_waitcnt(0xF70);   // vmcnt(0)
  if constexpr (KEEP > 0) {
#pragma unroll
    for (int k = 0; k < KEEP; ++k)
      if (tile0 + k < tile1) tile_body(tile0 + k, k);
  } else {
    for (int tile = tile0; tile < tile1; ++tile) tile_body(tile, 0);
  }
  if (!p.stats) return;
  // the block's BatchNorm sums: the 16 lanes of a group hold the same 8 channels
#pragma unroll
  for (int q = 0; q < CP; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
#pragma unroll
      for (int s = 1; s < 16; s <<= 1) {
        sum[q][e] += __shfl_xor(sum[q][e], s);
        sq[q][e] += __shfl_xor(sq[q][e], s);
      }
    }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int q = 0; q < CP; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(wave * 2 + 0) * BN + 32 * q + 8 * g + e] = sum[q][e];
        red[(wave * 2 + 1) * BN + 32 * q + 8 * g + e] = sq[q][e];
      }
  }
  __syncthreads();
  if (t < 2 * BN) {
    const int which = t / BN, c = t - which * BN;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) v += red[(w * 2 + which) * BN + c];
    unsafeAtomicAdd(reinterpret_cast<double*>(p.stats) + ((int(blockIdx.x) % p.acc_r) * 2 + which) * p.NOUT + c,
                    double(v));
  }
  if constexpr (KEEP > 0) {
    double* acc = reinterpret_cast<double*>(p.stats);
    grid_barrier(bn_acc_barrier(acc, p.acc_r, BN), gridDim.x);
    // the fold, as bn_apply_kernel's (the patch area is free now: >= 2 KiB of sums, then the coefficients)
    double* part = reinterpret_cast<double*>(smem);
    float* coef = reinterpret_cast<float*>(smem + 2048);
    static_assert(PX * 8 >= 2048 + 2 * BN * 4 && 2 * BN <= kThreads, "fold scratch");
    __shared__ int flag;
    bn_acc_column_sums<true>(acc, p.acc_r, 2 * BN, part);
    if (t < BN) {
      BnFwdFinal fin;
      fin.eps = ob.act.eps, fin.momentum = ob.act.momentum;
      fin.mean = ob.act.mean, fin.invstd = ob.act.invstd;
      fin.rm = ob.act.rm, fin.rv = ob.act.rv, fin.tracked = ob.act.tracked;
      float mu, is;
      bn_fwd_finalize(fin, part, BN, ob.act.M, t, blockIdx.x == 0, mu, is);
      coef[t] = mu;
      coef[BN + t] = is;
    }
    __syncthreads();
    bn_acc_release(acc, p.acc_r, BN, &flag, blockIdx.x, gridDim.x);
    // this lane's channels 32 q + 8 g + e: xhat = v is + nm, z = xhat ww + bb (bn_apply_kernel's order)
    float is[CP][8], nm[CP][8], ww[CP][8], bb[CP][8];
#pragma unroll
    for (int q = 0; q < CP; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = 32 * q + 8 * g + e;
        is[q][e] = coef[BN + c];
        nm[q][e] = -coef[c] * is[q][e];
        ww[q][e] = ob.act.w[c];
        bb[q][e] = ob.act.b[c];
      }
    const float slope = ob.act.slope;
#pragma unroll
    for (int k = 0; k < KEEP; ++k) {
      const int tile = tile0 + k;
      if (tile >= tile1) break;
      const int n = tile / (tiles_r * tiles_c), rem = tile - n * (tiles_r * tiles_c);
      const int orow0 = (rem / tiles_c) * TR, ocol0 = (rem % tiles_c) * kC1Cols;
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const int fi = wave * PF + j;
        const int orow = orow0 + (fi >> 2), ocol = ocol0 + 16 * (fi & 3) + (lane & 15);
        if (orow >= p.OH || ocol >= p.OW) continue;
        uint16_t* out = ob.y + (int64_t(n * p.OH + orow) * p.OW + ocol) * p.NOUT + 8 * g;
#pragma unroll
        for (int q = 0; q < CP; ++q) {
          uint32_t o[4];
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            const uint32_t v = keep[k][j][q][h];
            f32x2 r;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
              const int e = 2 * h + s;
              const float x = s ? __uint_as_float(v & 0xFFFF0000u) : __uint_as_float(v << 16);
              const float z = fmaf(fmaf(x, is[q][e], nm[q][e]), ww[q][e], bb[q][e]);
              r[s] = z > 0.f ? z : z * slope;
            }
            o[h] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, bf16x2));
          }
          *reinterpret_cast<uint4*>(out + 32 * q) = make_uint4(o[0], o[1], o[2], o[3]);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// The data gradient of the 32-channel layer (conv 32 -> 64: dY 64 channels,
// dx 32) from a dY PATCH.  As a tap GEMM (tap_gemm_kernel<true, 32, ..., 4>)
// every class pixel re-stages its 4 taps x 64 channels through LDS-DMA each
// k-step: 16 x the dY tensor of LDS traffic, 5 DMA pieces per wave per 8
// MFMAs, 16 latency-bound k-steps per block (47 us, 13.9 VALU per MFMA).
// Here a block loads the (4 + 2) x (32 + 2) dY pixels under a 4 x 32 tile of
// the class grid ONCE into LDS (26 KB, 16-byte chunks XOR-swizzled by pixel so
// a 16-lane fragment read of 16 consecutive pixels hits 16 bank slots) and
// runs all four parity classes' 8 K=32 steps straight from it.  The weights
// -- a class's [32 ci][4 taps x 64 co] rows, 16 KB -- are the MFMA's A
// operand, staged in LDS once per class for all 4 waves (the next class's
// global loads are in flight while this class computes), and the patch
// pixels its B operand: a lane's accumulators hold 8 consecutive dx channels
// of one pixel (c1_row_chan), so the epilogue stores 16 bytes and sums the
// BN-backward terms from registers.  (Weights loaded into every lane's
// registers instead: 4 x the L2 traffic, 65-67 us.)
constexpr int DP_TA = 4, DP_TB = 32;                  // class-grid rows x columns per block
constexpr int DP_PR = DP_TA + 2, DP_PC = DP_TB + 2;   // the dY patch: one pixel of halo each side
constexpr int DP_C = 64, DP_NOUT = 32;                 // dY channels, dx channels
constexpr int DP_NP = DP_PR * DP_PC;                   // 204 patch pixels, 128 bytes each
constexpr int DP_PATCH = DP_NP * DP_C * 2;             // 26,112 bytes
constexpr int DP_WROW = 4 * DP_C * 2;                  // one weight row: 4 taps x 64 co, 512 bytes (32 chunks)
constexpr int DP_W = DP_NOUT * DP_WROW;                // one class's weights, 16 KiB
__device__ __forceinline__ int dp_off(int px, int q) { return px * (DP_C * 2) + ((q ^ ((px >> 1) & 7)) << 4); }
// weight row ci, chunk kc (k = 8 kc): the 16 rows a fragment reads (c1_row_chan: bits 0-1, 3-4 of ci)
// take 16 different chunk slots
__device__ __forceinline__ int dpw_off(int ci, int kc) {
  return ci * DP_WROW + ((kc ^ ((ci & 3) | (((ci >> 3) & 3) << 2))) << 4);
}

// one weight buffer (43 KB of LDS: 3 blocks per CU; double-buffered, 59 KB, fit 2 and ran slower)
constexpr int kDpatchLds = DP_PATCH + DP_W + 4 * 2 * DP_NOUT * 4;
// blk: the block's index in its own grid (blockIdx.x, or its place in a launch
// shared with the weight gradient: dpatch_wgrad_kernel)
__device__ __forceinline__ void dgrad_patch_body(const TapGemm& p, char* smem, int blk) {
  constexpr int NCH = DP_NP * 8, NL = (NCH + kThreads - 1) / kThreads;
  constexpr int WCH = DP_W / 16, WL = WCH / kThreads;   // 1024 weight chunks, 4 per thread
  char* const wl = smem + DP_PATCH;
  float* red = reinterpret_cast<float*>(smem + DP_PATCH + DP_W);
  const int t = int(threadIdx.x), lane = t & 63, wave = t >> 6, g = lane >> 4;
  const int tb = (p.GW + DP_TB - 1) / DP_TB, ta = (p.GH + DP_TA - 1) / DP_TA;
  const int n = blk / (ta * tb), rem = blk - n * (ta * tb);
  const int a0 = (rem / tb) * DP_TA, b0 = (rem % tb) * DP_TB;
  // a class's weight chunks: chunk c = t + 256 i -> row ci = c / 32, chunk kc = c % 32
  // (k = 8 kc: tap kc / 8, co 8 (kc % 8)) <- wt[ci][kh][kw][co]
  static_assert(WL == 4, "4 weight chunks per thread");
  // (four named registers, not an array: an array live across the class loop was promoted to LDS)
  uint4 wv0, wv1, wv2, wv3;
  auto wsrc = [&](int cls, int i) -> const uint4* {
    const int ph = cls >> 1, pw = cls & 1;
    const int c = t + kThreads * i, ci = c >> 5, kc = c & 31, tap = kc >> 3;
    const int kh = 1 - ph + 2 * (tap >> 1), kw = 1 - pw + 2 * (tap & 1);
    return reinterpret_cast<const uint4*>(p.w + (ci * 16 + kh * 4 + kw) * DP_C + 8 * (kc & 7));
  };
  auto load_w = [&](int cls) __attribute__((always_inline)) {
    wv0 = *wsrc(cls, 0), wv1 = *wsrc(cls, 1), wv2 = *wsrc(cls, 2), wv3 = *wsrc(cls, 3);
  };
  auto wdst = [&](int buf, int i) -> uint4* {
    const int c = t + kThreads * i;
    return reinterpret_cast<uint4*>(wl + buf * DP_W + dpw_off(c >> 5, c & 31));
  };
  auto store_w = [&](int buf) __attribute__((always_inline)) {
    *wdst(buf, 0) = wv0, *wdst(buf, 1) = wv1, *wdst(buf, 2) = wv2, *wdst(buf, 3) = wv3;
  };
  const bool bnf = p.bn.part != nullptr;
  // the BN's per-channel inputs of this lane's channels 8 g .. + 7: 16-byte loads issued first, in
  // flight with the patch (a scalar load per value, each consumed at once, made the compiler reuse
  // one register for all of them -- 8 round trips in series after the patch's); without the BN: out
  // of range, zeros
  float4 cv[4][2];
  {
    const float* src[4] = {p.bn.invstd, p.bn.mean, p.bn.w, p.bn.b};
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const __amdgpu_buffer_rsrc_t rc = make_rsrc(bnf ? static_cast<const void*>(src[a]) : p.w, bnf ? DP_NOUT * 4 : 0);
#pragma unroll
      for (int h = 0; h < 2; ++h) cv[a][h] = __builtin_bit_cast(float4, bload(rc, uint32_t(32 * g + 16 * h)));
    }
  }
  load_w(0);
  // the patch: chunk u = t + 256 i is chunk u & 7 of patch pixel u >> 3
  {
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.src, int64_t(p.N) * p.SH * p.SW * DP_C * 2);
    uint4 v[NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int u = t + kThreads * i, pix = u >> 3, q = u & 7;
      const int pr = pix / DP_PC, pc = pix - pr * DP_PC;
      const int ya = a0 - 1 + pr, yb = b0 - 1 + pc;
      const bool ok = u < NCH && unsigned(ya) < unsigned(p.SH) && unsigned(yb) < unsigned(p.SW);
      v[i] = bload(rs, ok ? uint32_t(((n * p.SH + ya) * p.SW + yb) * (DP_C * 2) + q * 16) : kOOB);
    }
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int u = t + kThreads * i;
      if ((i + 1) * kThreads <= NCH || u < NCH) *reinterpret_cast<uint4*>(smem + dp_off(u >> 3, u & 7)) = v[i];
    }
  }
  store_w(0);
  // this wave: class-grid row a0 + wave, columns b0 + 16 j + (lane & 15), j = 0, 1
  const int ra = a0 + wave;
  float is[8], nm[8], ww[8], bb[8], bs[8], bq[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    bs[e] = bq[e] = 0.f;
    auto pick = [&](int a) {
      const float4 f = cv[a][e >> 2];
      const int k = e & 3;
      return k == 0 ? f.x : k == 1 ? f.y : k == 2 ? f.z : f.w;
    };
    is[e] = pick(0);
    nm[e] = -pick(1) * is[e];
    ww[e] = pick(2);
    bb[e] = pick(3);
  }
  // A fragment offsets (class-invariant): row c1_row_chan(f, lane & 15), chunk 4 s + g
  int aoff[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) aoff[f] = c1_row_chan(f, lane & 15);
  __syncthreads();
  for (int cls = 0; cls < 4; ++cls) {
    const int ph = cls >> 1, pw = cls & 1;
    if (cls < 3) load_w(cls + 1);   // in flight while this class computes
    // the epilogue's BN inputs, also in flight during the MFMAs
    int eoff[2];
    uint4 xv[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int bcol = b0 + 16 * j + (lane & 15);
      eoff[j] = ra < p.GH && bcol < p.GW ? ((n * p.OH + 2 * ra + ph) * p.OW + 2 * bcol + pw) * DP_NOUT + 8 * g : -1;
      xv[j] = bnf && eoff[j] >= 0 ? *reinterpret_cast<const uint4*>(p.bn.x + eoff[j]) : make_uint4(0, 0, 0, 0);
    }
    const char* wb = wl;
    f32x4 acc[2][2];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int tap = s >> 1, dr = ph - (tap >> 1), dc = pw - (tap & 1);
      const int q = 4 * (s & 1) + g;
      bf16x8 wa[2], bm[2];
#pragma unroll
      for (int f = 0; f < 2; ++f) wa[f] = *reinterpret_cast<const bf16x8*>(wb + dpw_off(aoff[f], 4 * s + g));
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int px = (wave + dr + 1) * DP_PC + 16 * j + (lane & 15) + dc + 1;
        bm[j] = *reinterpret_cast<const bf16x8*>(smem + dp_off(px, q));
      }
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[f], bm[j], acc[f][j], 0, 0, 0);
    }
    // epilogue: dx pixel (2 a + ph, 2 b + pw), channels 8 g .. + 7
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (eoff[j] >= 0) {
        const int off = eoff[j];
        uint32_t pk[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {   // channels 8 g + 2 h, + 1: fragment h >> 1, rows 2 (h & 1), + 1
          const f32x4& a = acc[h >> 1][j];
          const f32x2 pr = {a[2 * (h & 1)], a[2 * (h & 1) + 1]};
          pk[h] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pr, bf16x2));
        }
        *reinterpret_cast<uint4*>(p.dst + off) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        if (bnf) {
          const uint32_t xw[4] = {xv[j].x, xv[j].y, xv[j].z, xv[j].w};
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float gv = __uint_as_float(e & 1 ? pk[e >> 1] & 0xFFFF0000u : pk[e >> 1] << 16);
            const float xh = fmaf(__uint_as_float(e & 1 ? xw[e >> 1] & 0xFFFF0000u : xw[e >> 1] << 16), is[e], nm[e]);
            const float gz = fmaf(xh, ww[e], bb[e]) > 0.f ? gv : gv * p.bn.slope;
            bs[e] += gz;
            bq[e] += gz * xh;
          }
        }
      }
    }
    if (cls < 3) {   // the next class's weights, once every wave is done with this class's
      __syncthreads();
      store_w(0);
      __syncthreads();
    }
  }
  if (!bnf) return;
  // the 16 lanes of a group hold the same channels; then the 4 waves through LDS
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) bs[e] += __shfl_xor(bs[e], o), bq[e] += __shfl_xor(bq[e], o);
  if ((lane & 15) == 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(wave * 2 + 0) * DP_NOUT + 8 * g + e] = bs[e];
      red[(wave * 2 + 1) * DP_NOUT + 8 * g + e] = bq[e];
    }
  }
  __syncthreads();
  if (t < 2 * DP_NOUT) {
    const int which = t / DP_NOUT, c = t - which * DP_NOUT;
    float v = 0.f;
#pragma unroll
    for (int w4 = 0; w4 < 4; ++w4) v += red[(w4 * 2 + which) * DP_NOUT + c];
    unsafeAtomicAdd(reinterpret_cast<double*>(p.bn.part) + ((blk % p.bn.acc_r) * 2 + which) * DP_NOUT + c,
                    double(v));
  }
}

__global__ __launch_bounds__(kThreads) void dgrad_patch_kernel(TapGemm p) {
  __shared__ __attribute__((aligned(16))) char smem[kDpatchLds];
  dgrad_patch_body(p, smem, int(blockIdx.x));
}

// ---------------------------------------------------------------------------
// The 32 -> 64 channel forward (the disc's conv2: 8 x 240 x 320 x 32 in,
// 120 x 160 x 64 out) as a PERSISTENT PATCH GEMM.  The tap GEMM gathers an
// im2col A tile per k-step through LDS-DMA (a stride-2 4x4 window stages every
// input pixel 4x) and re-stages the weights in every block: 192 KB of LDS fills
// per 128-pixel tile.  Those fills -- ~65 GB/s per CU from L2
// (MI355X_MICROARCH.md, 'gather into LDS') -- set the tap GEMMs' time, not the
// MFMAs (profiles/r6/disc_roofline.md).  Here one block per CU keeps all 64 KB
// of weights in LDS for the whole launch and walks its share of 4 x 32-pixel
// output tiles, staging each tile's (10 x 66)-pixel input patch ONCE (42 KB,
// double-buffered: the next tile's patch lands while this one computes) --
// 42 KB of fills per tile instead of 192, and no grid tail of a second wave of
// blocks (1,200 tiles over 256 persistent blocks).
//
// Patch layout: the 66 columns split by parity into two 33-pixel lines per
// row, pixel u = (row * 2 + parity) * 33 + col / 2, 64 bytes each with chunk q
// at slot q ^ ((u >> 1) & 3): the 16 pixels of an MFMA B fragment (output
// columns b..b+15 -> input columns 2b + kw, one parity) are 16 consecutive u
// and, in ds_read_b128's lane groups, on distinct 16-byte bank slots
// (/tmp-free model: scripts/lds_banks.py's groups).  Weights: row co (1 KB:
// 16 taps x 32 ci), chunk kc at kc ^ key(co) (dpw_off's key).  MFMA A = the
// weights (rows: channels in c1_row_chan order, so a lane's accumulators are 8
// consecutive channels of one pixel: 16-byte stores), B = patch pixels, K =
// one tap's 32 channels in tap order 0..15 -- the tap GEMM's accumulation
// order, the same bf16 output bit for bit.  BN sums (accumulator, acc_r > 0)
// stay in registers across the block's tiles: one fp64 add per channel per block.
constexpr int FP_CIN = 32, FP_COUT = 64;
constexpr int FP_TA = 4, FP_TB = 32;                  // output rows (one per wave) x columns per tile
constexpr int FP_PR = 2 * FP_TA + 2;                  // 10 patch rows
constexpr int FP_PL = FP_TB + 1;                      // 33 pixels per parity line
constexpr int FP_NPIX = FP_PR * 2 * FP_PL;            // 660 patch pixels of 64 bytes
constexpr int FP_PIECES = 44;                         // 1 KiB LDS-DMA pieces per patch: 11 per wave
constexpr int FP_PPW = FP_PIECES / 4;
constexpr int FP_PATCH = FP_PIECES * 1024;            // 45,056 bytes (41.25 KiB of pixels)
constexpr int FP_W = FP_COUT * 16 * FP_CIN * 2;       // 65,536 bytes
constexpr int kFwdPatchLds = FP_W + 2 * FP_PATCH + 4 * 2 * FP_COUT * 4;   // 157,696 bytes: one block per CU
static_assert(FP_NPIX * 64 <= FP_PATCH && kFwdPatchLds <= 163840, "patch GEMM LDS");
__device__ __forceinline__ int fp_off(int u, int q) { return u * 64 + ((q ^ ((u >> 1) & 3)) << 4); }
__device__ __forceinline__ int fpw_key(int co) { return (co & 3) | (((co >> 3) & 3) << 2); }

// dbg (experiments only; 0 in production): bit 0 no patch fills, bit 1 no MFMAs, bit 2 no stores
__global__ __launch_bounds__(kThreads) void conv_fwd_patch_kernel(TapGemm p, int ntiles, int dbg) {
  __shared__ __attribute__((aligned(16))) char smem[kFwdPatchLds];
  char* const wl = smem;
  char* const pb = smem + FP_W;
  float* const red = reinterpret_cast<float*>(smem + FP_W + 2 * FP_PATCH);
  const int t = int(threadIdx.x), lane = t & 63, wave = t >> 6, g = lane >> 4, lb = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int tb = (p.OW + FP_TB - 1) / FP_TB, ta = (p.OH + FP_TA - 1) / FP_TA;
  const int G = int(gridDim.x), first = int(blockIdx.x);
  const int mine = first < ntiles ? (ntiles - 1 - first) / G + 1 : 0;
  const __amdgpu_buffer_rsrc_t rs_x = make_rsrc(p.src, int64_t(p.N) * p.SH * p.SW * FP_CIN * 2);
  const __amdgpu_buffer_rsrc_t rs_w = make_rsrc(p.w, int64_t(FP_W));
  const __amdgpu_buffer_rsrc_t rs_y = make_rsrc(p.dst, int64_t(p.N) * p.OH * p.OW * FP_COUT * 2);
  typedef __attribute__((address_space(3))) void lds_void;

  // the weights, once: wave piece co = wv + 4 m; lane l lands at physical chunk l = logical l ^ key(co)
#pragma unroll
  for (int m = 0; m < FP_COUT / 4; ++m) {
    const int co = wv + 4 * m;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_w, (lds_void*)(wl + co * 1024), 16,
                                             co * 1024 + ((lane ^ fpw_key(co)) << 4), 0, 0, 0);
  }
  // this lane's patch pieces (tile-invariant): piece k = wv + 4 i, LDS byte 1024 k + 16 lane = pixel u,
  // physical slot lane & 3 = logical chunk q; patch row pr, column pc, byte offset from the patch origin
  int prow[FP_PPW], pcol[FP_PPW], prel[FP_PPW];
#pragma unroll
  for (int i = 0; i < FP_PPW; ++i) {
    const int u = (wv + 4 * i) * 16 + (lane >> 2);
    const int q = (lane & 3) ^ ((u >> 1) & 3);
    const int r = u / (2 * FP_PL), rem = u - r * (2 * FP_PL);
    const int pa = rem >= FP_PL ? 1 : 0, c = 2 * (rem - pa * FP_PL) + pa;
    prow[i] = u < FP_NPIX ? r : -1000;   // past the patch: never in range (zeros into the padding)
    pcol[i] = c;
    prel[i] = (r * p.SW + c) * (FP_CIN * 2) + q * 16;
  }
  auto tile_of = [&](int i, int& n, int& a0, int& b0) {
    const int T = first + i * G;
    n = T / (ta * tb);
    const int rem = T - n * (ta * tb);
    a0 = (rem / tb) * FP_TA;
    b0 = (rem - (rem / tb) * tb) * FP_TB;
  };
  auto issue = [&](int i) {
    int n, a0, b0;
    tile_of(i, n, a0, b0);
    if (dbg & 1) return;
    const int y0 = 2 * a0 - 1, x0 = 2 * b0 - 1;
    const int base = ((n * p.SH + y0) * p.SW + x0) * (FP_CIN * 2);   // (negative at the top-left border)
    char* const dst = pb + (i & 1) * FP_PATCH;
#pragma unroll
    for (int k = 0; k < FP_PPW; ++k) {
      const bool ok = unsigned(y0 + prow[k]) < unsigned(p.SH) && unsigned(x0 + pcol[k]) < unsigned(p.SW);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_x, (lds_void*)(dst + (wv + 4 * k) * 1024), 16,
                                               int(ok ? uint32_t(base + prel[k]) : kOOB), 0, 0, 0);
    }
  };
  // MFMA operand offsets (tile-invariant).  Weights: fragment f's row co, chunk (4 kw + g) ^ key at
  // tap (kh, kw) = chunk 16 kh + that: offset wo[f][kw] + 256 kh.  Patch: pixel u of tap (kh, kw),
  // fragment j: row 2 wave + kh, parity kw & 1, column 16 j + lb + kw / 2.
  int wo[4][4];
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const int co = c1_row_chan(f, lb);
#pragma unroll
    for (int kw = 0; kw < 4; ++kw) wo[f][kw] = co * 1024 + (((4 * kw + g) ^ fpw_key(co)) << 4);
  }
  int po[16][2];
#pragma unroll
  for (int tap = 0; tap < 16; ++tap)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int kh = tap >> 2, kw = tap & 3;
      po[tap][j] = fp_off(((2 * wave + kh) * 2 + (kw & 1)) * FP_PL + 16 * j + lb + (kw >> 1), g);
    }
  const bool stats = p.stats != nullptr;
  float sm[2][8], sq[2][8];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) sm[q][e] = sq[q][e] = 0.f;

  constexpr uint32_t kWaitAll = (7u << 4) | (0xFu << 8);   // vmcnt(0), no lgkm / exp wait
  constexpr uint32_t kWaitP = kWaitAll | uint32_t(FP_PPW);                 // the next patch's pieces out
  constexpr uint32_t kWaitPS = kWaitAll | uint32_t((FP_PPW + 4) & 15) | (uint32_t((FP_PPW + 4) >> 4) << 14);
  constexpr uint32_t kWaitS = kWaitAll | 4u;                                // the last tile's 4 stores out
  if (mine > 0) issue(0);
  for (int i = 0; i < mine; ++i) {
    const bool next = i + 1 < mine;
    if (next) issue(i + 1);
    asm volatile("" ::: "memory");
    // this tile's pieces are older than everything but the previous tile's 4 stores and the next pieces
    if (i == 0) {
      if (next) __builtin_amdgcn_s_waitcnt(kWaitP);
      else __builtin_amdgcn_s_waitcnt(kWaitAll);
    } else {
      if (next) __builtin_amdgcn_s_waitcnt(kWaitPS);
      else __builtin_amdgcn_s_waitcnt(kWaitS);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const char* const P = pb + (i & 1) * FP_PATCH;
    f32x4 acc[4][2];
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 16; ++tap) {
      if (dbg & 2) break;
      bf16x8 wa[4], bm[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) bm[j] = *reinterpret_cast<const bf16x8*>(P + po[tap][j]);
#pragma unroll
      for (int f = 0; f < 4; ++f) wa[f] = *reinterpret_cast<const bf16x8*>(wl + wo[f][tap & 3] + 256 * (tap >> 2));
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[f], bm[j], acc[f][j], 0, 0, 0);
    }
    // epilogue: pixel (a0 + wave, b0 + 16 j + lb), channels 32 q + 8 g .. + 7; 4 buffer stores per wave
    // always (out-of-range lanes store nowhere), so the wait counts above hold
    int n, a0, b0;
    tile_of(i, n, a0, b0);
    const int a = a0 + wave;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int b = b0 + 16 * j + lb;
      const bool ok = a < p.OH && b < p.OW;
      const uint32_t ob = uint32_t(((n * p.OH + a) * p.OW + b) * FP_COUT + 8 * g) * 2u;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        uint32_t pk[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {   // channels 8 g + 2 h, + 1: fragment 2 q + (h >> 1), rows 2 (h & 1), + 1
          const f32x4& av = acc[2 * q + (h >> 1)][j];
          const f32x2 pr = {av[2 * (h & 1)], av[2 * (h & 1) + 1]};
          pk[h] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pr, bf16x2));   // RNE
        }
        const u32x4 v = {pk[0], pk[1], pk[2], pk[3]};
        __builtin_amdgcn_raw_buffer_store_b128(v, rs_y, int(ok && !(dbg & 4) ? ob + uint32_t(64 * q) : kOOB), 0, 0);
        if (stats && ok) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float x = __uint_as_float(e & 1 ? pk[e >> 1] & 0xFFFF0000u : pk[e >> 1] << 16);
            sm[q][e] += x;
            sq[q][e] += x * x;
          }
        }
      }
    }
    asm volatile("" ::: "memory");
    __syncthreads();   // every wave is done with patch buffer i & 1 before tile i + 2 is issued into it
  }
  if (!stats) return;
  // the 16 lanes of a group hold the same channels; then the 4 waves through LDS; one fp64 add per
  // channel per block into replica blockIdx % acc_r of the accumulator [acc_r][2][64]
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) sm[q][e] += __shfl_xor(sm[q][e], o), sq[q][e] += __shfl_xor(sq[q][e], o);
  if (lb == 0) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(wave * 2 + 0) * FP_COUT + 32 * q + 8 * g + e] = sm[q][e];
        red[(wave * 2 + 1) * FP_COUT + 32 * q + 8 * g + e] = sq[q][e];
      }
  }
  __syncthreads();
  if (t < 2 * FP_COUT) {
    const int which = t / FP_COUT, c = t - which * FP_COUT;
    float v = 0.f;
#pragma unroll
    for (int w4 = 0; w4 < 4; ++w4) v += red[(w4 * 2 + which) * FP_COUT + c];
    unsafeAtomicAdd(reinterpret_cast<double*>(p.stats) + ((first % p.acc_r) * 2 + which) * FP_COUT + c, double(v));
  }
}

// several weights at once (blockIdx.y = tensor): the data gradients' operands for every layer in one launch
__global__ __launch_bounds__(kThreads) void weight_t_multi_kernel(WeightTParams p) {
  const int k = int(blockIdx.y);
  const int Cout = p.cout[k], Cin = p.cin[k];
  const int total = Cout * 16 * Cin;
  for (int e = int(blockIdx.x) * kThreads + int(threadIdx.x); e < total; e += int(gridDim.x) * kThreads) {
    const int ci = e % Cin, tap = (e / Cin) % 16, co = e / (16 * Cin);
    p.dst[k][(ci * 16 + tap) * Cout + co] = p.src[k][e];
  }
}

// [Cout][kh][kw][Cin] (channels-last weight, any dtype pair) -> [Cin][kh][kw][Cout]
__global__ __launch_bounds__(kThreads) void weight_t_kernel(const uint16_t* __restrict__ w, uint16_t* __restrict__ wt,
                                                            int Cout, int Cin) {
  const int total = Cout * 16 * Cin;
  for (int e = int(blockIdx.x) * kThreads + int(threadIdx.x); e < total; e += int(gridDim.x) * kThreads) {
    const int ci = e % Cin, tap = (e / Cin) % 16, co = e / (16 * Cin);
    wt[(ci * 16 + tap) * Cout + co] = w[e];
  }
}

}  // namespace

void conv_attach_adam_schedule(const AdamSchedJob& j, int device, hipStream_t stream) {
  g_sched_job = j;
  g_sched_device = device, g_sched_stream = stream;
  g_sched_taken = false;
}
bool conv_adam_schedule_taken() {
  const bool t = g_sched_taken;
  g_sched_taken = false;
  return t;
}
void conv_detach_adam_schedule() {
  g_sched_job = AdamSchedJob();
  g_sched_taken = false;
}

namespace {
// weight-gradient staging: 0 = register ring (conv_wgrad_kernel, default), 2 /
// 3 = LDS-DMA stages of 64 pixels (conv_wgrad_dma_kernel: 33 us against 24 us
// per layer in the disc step, profiles/r4/disc_kernels.md); BT_WGRAD_STAGING
int g_dgrad_patch = -1;   // the 32-channel data gradient from a dY patch (BT_DGRAD_PATCH, default on: 47 -> 36.5 us)
int dgrad_patch() {
  if (g_dgrad_patch < 0) {
    const char* v = std::getenv("BT_DGRAD_PATCH");
    g_dgrad_patch = v ? (std::atoi(v) ? 1 : 0) : 1;
  }
  return g_dgrad_patch;
}
// the patch data gradient held for a shared launch with the weight gradient
// (dpatch_wgrad_kernel) when conv_dgrad_hold is on; BT_FUSE_PATCH=0: never
int fuse_patch() {
  static const int v = [] {
    const char* e = std::getenv("BT_FUSE_PATCH");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return v;
}
int g_wgrad_wide = -1;   // register-staged weight gradient over 256-column tiles (BT_WGRAD_WIDE)
int wgrad_wide() {
  if (g_wgrad_wide < 0) {
    const char* v = std::getenv("BT_WGRAD_WIDE");
    g_wgrad_wide = v ? (std::atoi(v) ? 1 : 0) : 0;
  }
  return g_wgrad_wide;
}
// the wide kernel's layers: power-of-two Cin with whole 256-column tiles, plain dY
bool wgrad_wide_ok(int Cin, int Cout) { return wgrad_wide() && Cin >= 16 && (Cin & (Cin - 1)) == 0 && Cout % BCO == 0; }
int g_wgrad_pipe = -1;   // register-staged weight gradient: fragments read a step ahead (BT_WGRAD_PIPE)
// BT_DGRAD_BN128 (default 0): the held data gradient of a layer with Cin % 128 == 0 takes 128-channel
// tiles in the fused data + weight gradient launch (with the 128-channel weight-gradient tiles)
int g_dgrad_bn128 = -1;
bool dgrad_bn128() {
  if (g_dgrad_bn128 < 0) {
    const char* v = std::getenv("BT_DGRAD_BN128");
    g_dgrad_bn128 = v ? (std::atoi(v) ? 1 : 0) : 0;
  }
  return g_dgrad_bn128 == 1;
}
// BT_WGRAD_CO128 (default 1): 128-channel weight-gradient tiles (conv_wgrad_co128_body) where Cout % 128 == 0
int g_wgrad_co128 = -1;
bool wgrad_co128_ok(int Cin, int Cout) {
  if (g_wgrad_co128 < 0) {
    // default on: the step's 64->128 pair 49.5 -> 41.6 us, 21.1-21.4k -> 21.9-22.0k img/s
    // (profiles/r6/b3/disc_co*.jsonl, disc_step_sequence*.txt)
    const char* v = std::getenv("BT_WGRAD_CO128");
    g_wgrad_co128 = v ? (std::atoi(v) ? 1 : 0) : 1;
  }
  return g_wgrad_co128 == 1 && Cout % BCO2 == 0 && Cin >= 16 && (Cin & (Cin - 1)) == 0;
}
int wgrad_pipe() {
  if (g_wgrad_pipe < 0) {
    const char* v = std::getenv("BT_WGRAD_PIPE");
    g_wgrad_pipe = v ? (std::atoi(v) ? 1 : 0) : 0;
  }
  return g_wgrad_pipe;
}
// the ordered (deterministic) slice reduce (wgrad_reduce_ordered); BT_WGRAD_ORDERED=0: atomic groups
int g_wgrad_ordered = -1;
bool wgrad_ordered() {
  if (g_wgrad_ordered < 0) {
    const char* v = std::getenv("BT_WGRAD_ORDERED");
    g_wgrad_ordered = v && v[0] == '0' ? 0 : 1;
  }
  return g_wgrad_ordered == 1;
}
int g_wgrad_staging = -1;
int wgrad_staging() {
  if (g_wgrad_staging < 0) {
    const char* v = std::getenv("BT_WGRAD_STAGING");
    const int e = v ? std::atoi(v) : 0;
    g_wgrad_staging = e == 0 || e == 2 || e == 3 ? e : 0;
  }
  return g_wgrad_staging;
}
}  // namespace

namespace {
int g_c4w = -1;   // first-layer weight gradient: 1 = wave-private staging (default), 0 = block-shared; BT_C4_WAVE
int g_c4w_waves = -1;   // waves per block of the first layer's weight gradient; -1: BT_C4W_WAVES or the default
int c4w_waves() {
  if (g_c4w_waves < 0) {
    const char* e = std::getenv("BT_C4W_WAVES");
    const int v = e ? std::atoi(e) : 4;
    g_c4w_waves = v == 8 ? 8 : 4;
  }
  return g_c4w_waves;
}

// BT_C4W_PATCH (default 1): the first layer's weight gradient from a decoded input patch
// (conv_wgrad_c4p_kernel) when the shape takes it; BT_C4P_ROWS: output rows per band (1, 2, 4)
// default on: 21.55k / 21.54k against 21.27k / 21.45k img/s (profiles/r6/b6/disc_*.jsonl); BT_C4P_PRE=0: off
bool c4p_pre() {
  static const bool on = !(std::getenv("BT_C4P_PRE") && std::getenv("BT_C4P_PRE")[0] == '0');
  return on;
}
int g_c4p_override = -1;   // conv_set_c4p_rows (tests / benches): -1 = the environment's choice
int c4p_rows_for(int N, int H, int W, int Ho, int Wo, int Cout) {
  static const int env_rows = [] {
    const char* v = std::getenv("BT_C4W_PATCH");
    if (v && v[0] == '0') return 0;
    // 4 rows: 27.8 us with the BN backward against 31.3 at 2 rows, 40.8 at 1 and 31.0 for the
    // wave-private kernel (profiles/r6/b2/c4w_bench.jsonl)
    const char* r = std::getenv("BT_C4P_ROWS");
    const int k = r ? std::atoi(r) : 4;
    return k == 1 || k == 2 || k == 4 ? k : 4;
  }();
  const int rows = g_c4p_override >= 0 ? g_c4p_override : env_rows;
  if (rows == 0 || Cout != 32 || W > kC4pMaxW || W != 2 * Wo || H != 2 * Ho || Wo % BPX != 0 || Ho % rows != 0 ||
      N <= 0)
    return 0;
  return rows;
}

bool c4_wave_private() {
  if (g_c4w < 0) {
    const char* v = std::getenv("BT_C4_WAVE");
    g_c4w = v ? (std::atoi(v) != 0 ? 1 : 0) : 1;
  }
  return g_c4w == 1;
}
}  // namespace

void conv_set_c4_wave_private(int on) { g_c4w = on < 0 ? -1 : (on ? 1 : 0); }
void conv_set_c4w_waves(int nw) { g_c4w_waves = nw == 4 || nw == 8 ? nw : -1; }

void conv_set_dgrad_patch(int on) { g_dgrad_patch = on < 0 ? -1 : (on ? 1 : 0); }
void conv_set_wgrad_wide(int on) { g_wgrad_wide = on < 0 ? -1 : (on ? 1 : 0); }
void conv_set_wgrad_pipe(int on) { g_wgrad_pipe = on < 0 ? -1 : (on ? 1 : 0); }
void conv_set_wgrad_ordered(int on) { g_wgrad_ordered = on < 0 ? -1 : (on ? 1 : 0); }

void conv_set_wgrad_staging(int staging) { g_wgrad_staging = staging == 0 || staging == 2 || staging == 3 ? staging : -1; }

bool conv_wgrad_supported(int Cin, int Cout) {
  return (Cin >= 32 && Cin % 32 == 0 && Cout >= 64 && Cout % 64 == 0) || (Cin == 4 && Cout % 32 == 0 && Cout > 0);
}

int conv_c4p_rows(int N, int H, int W, int Ho, int Wo, int Cout) { return c4p_rows_for(N, H, W, Ho, Wo, Cout); }
void conv_set_dgrad_bn128(int on) { g_dgrad_bn128 = on < 0 ? -1 : (on ? 1 : 0); }
void conv_set_wgrad_co128(int on) { g_wgrad_co128 = on < 0 ? -1 : (on ? 1 : 0); }
void conv_set_c4p_rows(int rows) { g_c4p_override = rows == 0 || rows == 1 || rows == 2 || rows == 4 ? rows : -1; }

int conv_wgrad_slices(int64_t M, int Cin, int Cout, int target_blocks) {
  if (!conv_wgrad_supported(Cin, Cout) || M <= 0) return 0;
  const int64_t tiles = Cin == 4 ? Cout / 32 : wgrad_co128_ok(Cin, Cout) ? int64_t(Cout / BCO2) * (16 * Cin / BKC)
                                          : int64_t(Cout / BCO) * (16 * Cin / (wgrad_wide_ok(Cin, Cout) ? BKC2 : BKC));
  // 128-channel tiles: half the blocks by default (each stages twice the channels; the same
  // partial volume, [slices][Cout][KC], as the 64-channel tiles at the full target)
  static const int co128_div = [] {
    const char* v = std::getenv("BT_WGRAD_CO128_DIV");
    const int d = v ? std::atoi(v) : 2;
    return d >= 1 ? d : 2;
  }();
  if (Cin != 4 && wgrad_co128_ok(Cin, Cout)) target_blocks = (target_blocks + co128_div - 1) / co128_div;
  int64_t s = (target_blocks + tiles - 1) / tiles;
  const int64_t max_s = (M + BPX - 1) / BPX;
  s = s < 1 ? 1 : (s > max_s ? max_s : s);
  return int(s);
}

hipError_t conv_wgrad_reduce(const ConvWgradParams::Reduce& r, hipStream_t stream) {
  if (!r.partial || !r.out || r.S <= 0 || r.rx <= 0 || r.ry <= 0) return hipErrorInvalidValue;
  conv_wgrad_reduce_kernel<<<dim3(unsigned(r.rx), unsigned(r.ry)), kThreads, 0, stream>>>(r, take_sched_job(stream));
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// A layer's data gradient and weight gradient in ONE launch.  Both are
// latency-bound at 3 blocks per CU (tap GEMM: 16-64 k-steps of LDS-DMA
// stages; weight gradient: ~40 pixel steps per slice), and both read the
// same dY: sharing the CUs fills each other's memory waits, and the kernel
// boundary between them goes away.  Blocks alternate in runs of 8 (a data-
// gradient run, then a weight-gradient run, ... then the longer kind's
// rest), so each part's XCD-aware tile order still sees consecutive ids on
// one XCD.  The weight-gradient part may carry its chain's deferred reduce
// (its side blocks) but not a BN fold: the fold would read the accumulator
// this launch's data gradient is still filling (the BN backward then folds
// it in its own apply).  conv_dgrad holds its tap-GEMM launch while
// conv_dgrad_hold(1) is set; the next conv_wgrad on that stream launches
// both, or conv_dgrad_flush launches the data gradient alone.
// DBN: the data gradient's output-channel tile (64, or 128 with BT_DGRAD_BN128 where Cin % 128 == 0:
// each tap-gathered dY tile then feeds twice the channels)
// (a 4-deep dY / X ring in the 128-channel weight-gradient blocks -- 184 VGPRs, 2 waves per SIMD --
// ran the step at 20.2 / 20.6k against 21.4 / 21.5k img/s, profiles/r6/b10/)
template <int BM, bool PIPE, bool W2 = false, int DBN = 64>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(W2 ? 3 : 1))) void dgrad_wgrad_kernel(TapGemm g, ConvWgradParams q, int gx, int nd, int nw) {
  constexpr int TL = tap_gemm_lds<true, DBN, false, BM, 2>();
  constexpr int WL = W2 ? kWgrad2Lds : kWgradLds;
  __shared__ __attribute__((aligned(16))) char smem[TL > WL ? TL : WL];
  const int b = int(blockIdx.x);
  const int nd8 = (nd + 7) & ~7, nw8 = (nw + 7) & ~7, m8 = nd8 < nw8 ? nd8 : nw8;
  int kind, idx;
  if (b < 2 * m8) {
    const int run = b >> 3;
    kind = run & 1;
    idx = ((run >> 1) << 3) | (b & 7);
  } else {
    kind = nd8 > nw8 ? 0 : 1;
    idx = m8 + (b - 2 * m8);
  }
  if (kind == 0) {
    if (idx >= nd) return;   // (padding of the run: block-uniform, before any barrier)
    tap_gemm_body<true, DBN, false, BM, 2, 1, 0>(g, smem, idx % gx, idx / gx, gx);
    // the attached Adam schedule (block 0: the first tile; the update launch may take the
    // backward's last slice reduce, so the schedule cannot wait for that launch)
    if (b == 0 && q.job.step && threadIdx.x == 0) adam_schedule_run(q.job);
  } else {
    if (idx >= nw) return;
    if constexpr (W2) conv_wgrad_co128_body<>(q, smem, idx);
    else conv_wgrad_body<false, PIPE>(q, smem, idx);
  }
}

// the same for the 32-channel layer's patch data gradient (dgrad_patch_body)
// WIDE: the weight gradient's 256-column tiles (conv_wgrad_wide_body; 32 x 128 per wave)
template <bool PIPE, bool WIDE = false>
__global__ __launch_bounds__(kThreads) void dpatch_wgrad_kernel(
    TapGemm g, ConvWgradParams q, int nd, int nw) {
  constexpr int WL = WIDE ? kWgradWideLds : kWgradLds;
  __shared__ __attribute__((aligned(16))) char smem[kDpatchLds > WL ? kDpatchLds : WL];
  const int b = int(blockIdx.x);
  const int nd8 = (nd + 7) & ~7, nw8 = (nw + 7) & ~7, m8 = nd8 < nw8 ? nd8 : nw8;
  int kind, idx;
  if (b < 2 * m8) {
    const int run = b >> 3;
    kind = run & 1;
    idx = ((run >> 1) << 3) | (b & 7);
  } else {
    kind = nd8 > nw8 ? 0 : 1;
    idx = m8 + (b - 2 * m8);
  }
  if (kind == 0) {
    if (idx >= nd) return;
    dgrad_patch_body(g, smem, idx);
    if (b == 0 && q.job.step && threadIdx.x == 0) adam_schedule_run(q.job);   // (dgrad_wgrad_kernel)
  } else {
    if (idx >= nw) return;
    if constexpr (WIDE) conv_wgrad_wide_body(q, smem, idx);
    else conv_wgrad_body<false, PIPE>(q, smem, idx);
  }
}

namespace {
struct HeldDgrad {
  bool on = false;
  bool patch = false;   // dgrad_patch_kernel's grid (gx blocks), else the tap GEMM's (gx x 4 classes)
  TapGemm g;
  int bm = 0;
  int bn = 64;          // the data gradient's channel tile (128: BT_DGRAD_BN128)
  unsigned gx = 0;   // the data gradient's x grid (4 parity classes in y)
  hipStream_t s = nullptr;
};
HeldDgrad g_held;
bool g_hold = false;
}  // namespace

bool conv_dgrad_held() { return g_held.on; }

hipError_t conv_wgrad(const ConvWgradParams& p, float* out, int64_t s_co, int64_t s_ci, int64_t s_kh, int64_t s_kw,
                      hipStream_t stream, ConvWgradParams::Reduce* defer, const ConvWgradParams::Reduce* side) {
  if (!conv_wgrad_supported(p.Cin, p.Cout) || p.slices <= 0 || !p.x || !p.dy || !p.partial || !out ||
      p.cin_out < 0 || p.cin_out > p.Cin)
    return hipErrorInvalidValue;
  if (p.Ho != (p.H + 2 - 4) / 2 + 1 || p.Wo != (p.W + 2 - 4) / 2 + 1 || p.M != int64_t(p.N) * p.Ho * p.Wo)
    return hipErrorInvalidValue;   // 4x4 / stride 2 / pad 1 only
  if (p.px_per_slice <= 0 || p.px_per_slice % BPX != 0 || int64_t(p.slices) * p.px_per_slice < p.M)
    return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(p.x) | reinterpret_cast<uintptr_t>(p.dy)) & 15) return hipErrorInvalidValue;
  if (p.lut && (p.Cin != 4 || (reinterpret_cast<uintptr_t>(p.lut) & 7))) return hipErrorInvalidValue;
  if (p.bn_dy.y) {
    const bool given = p.bn_dy.dw && p.bn_dy.db;                               // folded elsewhere
    const bool folds = p.bn_dy.acc && p.bn_dy.R > 0 && p.bn_dy.dw_out && p.bn_dy.db_out;   // folded here
    if ((reinterpret_cast<uintptr_t>(p.bn_dy.y) | reinterpret_cast<uintptr_t>(p.bn_dy.gx_out)) & 15 ||
        !p.bn_dy.mean || !p.bn_dy.invstd || !p.bn_dy.w || !p.bn_dy.b || given == folds || p.fold.acc ||
        (p.Cin != 4 && !folds) || (p.Cin == 4 && p.bn_dy.gx_out) || 2 * p.Cout > 512)   // fold scratch: 4 KiB
      return hipErrorInvalidValue;
  }
  if (int64_t(p.N) * p.H * p.W * p.Cin * 2 >= int64_t(kOOB) || p.M * p.Cout * 2 >= int64_t(kOOB))
    return hipErrorInvalidValue;   // 32-bit buffer offsets
  const bool c4 = p.Cin == 4;
  // 256-column tiles (BT_WGRAD_WIDE): the plain register-staged path only
  // 128-channel tiles: the plain path only (its slices were counted with them: conv_wgrad_slices)
  const bool co128 = !c4 && wgrad_co128_ok(p.Cin, p.Cout) && !p.bn_dy.y;
  const bool wide = !c4 && !co128 && wgrad_wide_ok(p.Cin, p.Cout) && !p.bn_dy.y && wgrad_staging() == 0;
  const int64_t tiles = c4 ? p.Cout / 32 : co128 ? int64_t(p.Cout / BCO2) * (16 * p.Cin / BKC)
                                               : int64_t(p.Cout / BCO) * (16 * p.Cin / (wide ? BKC2 : BKC));
  const int64_t blocks = tiles * p.slices;
  if (blocks > (int64_t(1) << 31) - 1) return hipErrorInvalidValue;
  ConvWgradParams q = p;
  q.job = AdamSchedJob();
  if (p.slices > kSliceGroup && !wgrad_ordered()) {   // groups add atomically: the main kernel zeroes out first
    q.zero_out = out;
    q.zero_count = p.Cout * 16 * (p.cin_out > 0 ? p.cin_out : p.Cin);
  }
  int64_t grid = blocks;
  q.main_blocks = int(blocks);
  if (side) {
    if (!side->partial || !side->out || side->S <= 0 || side->rx <= 0 || side->ry <= 0) return hipErrorInvalidValue;
    q.side = *side;
    grid += int64_t(side->rx) * side->ry;
  } else {
    q.side = ConvWgradParams::Reduce();
  }
  if (p.fold.acc) {   // + one block: the BN fold (its LDS: 2 C doubles of the kernel's staging array)
    if (c4 || p.fold.R <= 0 || p.fold.C <= 0 || 2 * p.fold.C * 8 > 2 * STAGE || !p.fold.dw || !p.fold.db)
      return hipErrorInvalidValue;
    grid += 1;
  }
  // (a BN backward folded in-kernel: the wave-private first-layer kernel or the register-staged one)
  const bool bn_folds = p.bn_dy.acc != nullptr;
  bool fused = false;
  if (g_held.on) {   // a held data gradient: one launch for both when this is the plain kernel's case
    const bool dma = (wgrad_staging() == 2 || wgrad_staging() == 3) && (p.Cin & (p.Cin - 1)) == 0 && p.Wo >= 32;
    // (256-column tiles fuse with the patch data gradient; the tap GEMM's launch takes 128-column
    // or 128-channel tiles)
    const bool plain = !c4 && !bn_folds && !p.bn_dy.y && !p.fold.acc && !dma && (!wide || g_held.patch) &&
                       (!co128 || !wgrad_pipe()) && (g_held.bn == 64 || co128);
    const int64_t nd = int64_t(g_held.gx) * (g_held.patch ? 1 : 4);
    if (plain && stream == g_held.s && nd + grid + 16 < (int64_t(1) << 31)) {
      if (sched_early()) q.job = take_sched_job(stream);
      const unsigned total = unsigned(((nd + 7) & ~int64_t(7)) + ((grid + 7) & ~int64_t(7)));
      const int gx = int(g_held.gx), ndi = int(nd), nwi = int(grid);
      if (g_held.patch && wide)
        dpatch_wgrad_kernel<false, true><<<total, kThreads, 0, stream>>>(g_held.g, q, ndi, nwi);
      else if (g_held.patch && wgrad_pipe())
        dpatch_wgrad_kernel<true><<<total, kThreads, 0, stream>>>(g_held.g, q, ndi, nwi);
      else if (g_held.patch)
        dpatch_wgrad_kernel<false><<<total, kThreads, 0, stream>>>(g_held.g, q, ndi, nwi);
      else if (co128 && g_held.bn == 128 && g_held.bm == 64)
        dgrad_wgrad_kernel<64, false, true, 128><<<total, kThreads, 0, stream>>>(g_held.g, q, gx, ndi, nwi);
      else if (co128 && g_held.bn == 128)
        dgrad_wgrad_kernel<FBM, false, true, 128><<<total, kThreads, 0, stream>>>(g_held.g, q, gx, ndi, nwi);
      else if (co128 && g_held.bm == 64)
        dgrad_wgrad_kernel<64, false, true><<<total, kThreads, 0, stream>>>(g_held.g, q, gx, ndi, nwi);
      else if (co128)
        dgrad_wgrad_kernel<FBM, false, true><<<total, kThreads, 0, stream>>>(g_held.g, q, gx, ndi, nwi);
      else if (g_held.bm == 64 && wgrad_pipe())
        dgrad_wgrad_kernel<64, true><<<total, kThreads, 0, stream>>>(g_held.g, q, gx, ndi, nwi);
      else if (g_held.bm == 64)
        dgrad_wgrad_kernel<64, false><<<total, kThreads, 0, stream>>>(g_held.g, q, gx, ndi, nwi);
      else if (wgrad_pipe())
        dgrad_wgrad_kernel<FBM, true><<<total, kThreads, 0, stream>>>(g_held.g, q, gx, ndi, nwi);
      else
        dgrad_wgrad_kernel<FBM, false><<<total, kThreads, 0, stream>>>(g_held.g, q, gx, ndi, nwi);
      g_held.on = false;
      fused = true;
    } else {
      const hipError_t e = conv_dgrad_flush();
      if (e != hipSuccess) return e;
    }
  }
  const int c4p = c4 && p.lut ? c4p_rows_for(p.N, p.H, p.W, p.Ho, p.Wo, p.Cout) : 0;
  if (fused) {
  } else if (c4p > 0 && p.px_per_slice == int64_t(c4p) * p.Wo && int64_t(p.slices) * p.px_per_slice == p.M) {
    if (c4p == 1) conv_wgrad_c4p_kernel<1><<<unsigned(grid), kThreads, 0, stream>>>(q);
    else if (c4p == 2) conv_wgrad_c4p_kernel<2><<<unsigned(grid), kThreads, 0, stream>>>(q);
    else if (c4p_pre()) conv_wgrad_c4p_kernel<4, 2, true><<<unsigned(grid), kThreads, 0, stream>>>(q);
    else conv_wgrad_c4p_kernel<4><<<unsigned(grid), kThreads, 0, stream>>>(q);
  } else if (c4 && (c4_wave_private() || bn_folds)) {
    const bool u8 = p.lut != nullptr;
    static const bool ldsc = std::getenv("BT_C4W_LDS_COEF") && std::getenv("BT_C4W_LDS_COEF")[0] == '1';
    if (c4w_waves() == 8 && u8) conv_wgrad_c4w_kernel<8, true><<<unsigned(grid), 512, 0, stream>>>(q);
    else if (c4w_waves() == 8) conv_wgrad_c4w_kernel<8, false><<<unsigned(grid), 512, 0, stream>>>(q);
    else if (u8 && ldsc) conv_wgrad_c4w_kernel<4, true, true><<<unsigned(grid), kThreads, 0, stream>>>(q);
    else if (u8) conv_wgrad_c4w_kernel<4, true><<<unsigned(grid), kThreads, 0, stream>>>(q);
    else if (ldsc) conv_wgrad_c4w_kernel<4, false, true><<<unsigned(grid), kThreads, 0, stream>>>(q);
    else conv_wgrad_c4w_kernel<4, false><<<unsigned(grid), kThreads, 0, stream>>>(q);
  }
  else if (c4) conv_wgrad_c4_kernel<<<unsigned(grid), kThreads, 0, stream>>>(q);
  else if (co128) conv_wgrad_co128_kernel<<<unsigned(grid), kThreads, 0, stream>>>(q);
  else if (bn_folds && wgrad_pipe()) conv_wgrad_kernel<true, true><<<unsigned(grid), kThreads, 0, stream>>>(q);
  else if (bn_folds) conv_wgrad_kernel<true><<<unsigned(grid), kThreads, 0, stream>>>(q);
  else if (wgrad_staging() == 2 && (p.Cin & (p.Cin - 1)) == 0 && p.Wo >= 32)
    conv_wgrad_dma_kernel<2><<<unsigned(grid), kThreads, 0, stream>>>(q);
  else if (wgrad_staging() == 3 && (p.Cin & (p.Cin - 1)) == 0 && p.Wo >= 32)
    conv_wgrad_dma_kernel<3><<<unsigned(grid), kThreads, 0, stream>>>(q);
  else if (wide) conv_wgrad_wide_kernel<<<unsigned(grid), kThreads, 0, stream>>>(q);
  else if (wgrad_pipe()) conv_wgrad_kernel<false, true><<<unsigned(grid), kThreads, 0, stream>>>(q);
  else conv_wgrad_kernel<false><<<unsigned(grid), kThreads, 0, stream>>>(q);
  const int64_t total = int64_t(p.Cout) * 16 * p.Cin;   // partial elements per slice
  ConvWgradParams::Reduce r;
  r.partial = p.partial, r.S = p.slices, r.Cout = p.Cout, r.Cin = p.Cin;
  r.cin_out = p.cin_out > 0 ? p.cin_out : p.Cin;
  r.out = out, r.s_co = s_co, r.s_ci = s_ci, r.s_kh = s_kh, r.s_kw = s_kw;
  if (wgrad_ordered()) {
    // lanes per 4 elements: each walks <= rounds x 8 slices (rounds of 8 loads in flight);
    // BT_REDUCE_ROUNDS (default 2; 1: twice the lanes, one round)
    static const int rounds = [] {
      const char* v = std::getenv("BT_REDUCE_ROUNDS");
      const int k = v ? std::atoi(v) : 2;
      return k >= 1 && k <= 8 ? k : 2;
    }();
    int sub = 1;
    while (sub < 64 && (p.slices + sub - 1) / sub > rounds * kSliceGroup) sub <<= 1;
    r.sub = sub;
    r.rx = int((total / 4 * sub + kThreads - 1) / kThreads);
    r.ry = 1;
  } else {
    r.rx = int((total / 4 + kThreads - 1) / kThreads);
    r.ry = (p.slices + kSliceGroup - 1) / kSliceGroup;
  }
  if (defer) {
    *defer = r;
    return hipGetLastError();
  }
  conv_wgrad_reduce_kernel<<<dim3(unsigned(r.rx), unsigned(r.ry)), kThreads, 0, stream>>>(r, take_sched_job(stream));
  return hipGetLastError();
}

namespace {
int ilog2_exact(int v) {
  int k = 0;
  while ((1 << k) < v) ++k;
  return (1 << k) == v ? k : -1;
}
}  // namespace

bool conv_fwd_supported(int Cin, int Cout) {
  return (Cin == 4 || (Cin >= 8 && ilog2_exact(Cin) >= 0 && (16 * Cin) % FBK == 0)) && Cout % 32 == 0;
}

bool conv_dgrad_supported(int Cin, int Cout) {
  return Cout >= 16 && ilog2_exact(Cout) >= 0 && (4 * Cout) % FBK == 0 && Cin % 32 == 0;
}

namespace {
template <bool DGRAD, int BM, int NST>
void launch_tap_gemm_bm(const TapGemm& g, int bn, unsigned ytiles, hipStream_t stream) {
  const int64_t blocks = (g.M + BM - 1) / BM * (g.NOUT / bn);
  const bool all_cls = DGRAD && g.cls_per_block == 4;
  const dim3 grid(unsigned(blocks), all_cls ? 1u : ytiles);
  if (!DGRAD && g.C == 4) {
    if (bn == 64) tap_gemm_kernel<false, 64, true, BM><<<grid, kThreads, 0, stream>>>(g);
    else tap_gemm_kernel<false, 32, true, BM><<<grid, kThreads, 0, stream>>>(g);
  } else if (all_cls) {   // (the 32-channel data gradient; other widths as well for tests / sweeps)
    if (bn == 128) tap_gemm_kernel<DGRAD, 128, false, BM, NST, 4><<<grid, kThreads, 0, stream>>>(g);
    else if (bn == 64) tap_gemm_kernel<DGRAD, 64, false, BM, NST, 4><<<grid, kThreads, 0, stream>>>(g);
    else tap_gemm_kernel<DGRAD, 32, false, BM, NST, 4><<<grid, kThreads, 0, stream>>>(g);
  } else if (bn == 128) {
    tap_gemm_kernel<DGRAD, 128, false, BM, NST><<<grid, kThreads, 0, stream>>>(g);
  } else if (bn == 64) {
    tap_gemm_kernel<DGRAD, 64, false, BM, NST><<<grid, kThreads, 0, stream>>>(g);
  } else {
    tap_gemm_kernel<DGRAD, 32, false, BM, NST><<<grid, kThreads, 0, stream>>>(g);
  }
}

int g_staging = -1;   // 0 register ring, 2/3 LDS-DMA stages; -1 = BT_CONV_STAGING or the default

int staging() {
  if (g_staging < 0) {
    const char* v = std::getenv("BT_CONV_STAGING");
    const int e = v ? std::atoi(v) : 2;
    g_staging = e == 0 || e == 2 || e == 3 || e == 4 ? e : 2;
  }
  return g_staging;
}

template <bool DGRAD, int BM>
void launch_tap_gemm_st(const TapGemm& g, int bn, unsigned ytiles, hipStream_t stream) {
  switch (staging()) {
    case 0: launch_tap_gemm_bm<DGRAD, BM, 0>(g, bn, ytiles, stream); break;
    case 3: launch_tap_gemm_bm<DGRAD, BM, 3>(g, bn, ytiles, stream); break;
    case 4: launch_tap_gemm_bm<DGRAD, BM, 4>(g, bn, ytiles, stream); break;
    default: launch_tap_gemm_bm<DGRAD, BM, 2>(g, bn, ytiles, stream); break;
  }
}

// forward with the input BatchNorm applied in the staging (TapGemm::act): 2 LDS-DMA stages
template <int BM, int ACT>
void launch_tap_gemm_act(const TapGemm& g, int bn, hipStream_t stream) {
  const dim3 grid(unsigned((g.M + BM - 1) / BM * (g.NOUT / bn)));
  if (bn == 128) tap_gemm_kernel<false, 128, false, BM, 2, 1, ACT><<<grid, kThreads, 0, stream>>>(g);
  else if (bn == 64) tap_gemm_kernel<false, 64, false, BM, 2, 1, ACT><<<grid, kThreads, 0, stream>>>(g);
  else tap_gemm_kernel<false, 32, false, BM, 2, 1, ACT><<<grid, kThreads, 0, stream>>>(g);
}

template <bool DGRAD>
void launch_tap_gemm(const TapGemm& g, unsigned ytiles, hipStream_t stream) {
  const int bn = conv_tile_channels(g.NOUT, g.C == 4 && !DGRAD);
  if (!DGRAD && g.act.on()) {
    const bool two = g.C > FBK;   // a thread's chunk alternates between two channel sets (C = 128)
    if (conv_tile_pixels(g.M, g.NOUT, int(ytiles)) == 64) {
      if (two) launch_tap_gemm_act<64, 2>(g, bn, stream);
      else launch_tap_gemm_act<64, 1>(g, bn, stream);
    } else {
      if (two) launch_tap_gemm_act<FBM, 2>(g, bn, stream);
      else launch_tap_gemm_act<FBM, 1>(g, bn, stream);
    }
    return;
  }
  if (conv_tile_pixels(g.M, g.NOUT, int(ytiles)) == 64) launch_tap_gemm_st<DGRAD, 64>(g, bn, ytiles, stream);
  else launch_tap_gemm_st<DGRAD, FBM>(g, bn, ytiles, stream);
}

// tile-size overrides (0 = the automatic rule); set from tests and sweeps,
// first from BT_CONV_BM / BT_CONV_BN
int env_int(const char* name) {
  const char* v = std::getenv(name);
  return v ? std::atoi(v) : 0;
}
int g_force_bm = env_int("BT_CONV_BM");
// 128-pixel tiles unless that leaves fewer blocks than this (BT_CONV_BM64_BELOW; 512 = 2 per CU)
int g_bm64_below = env_int("BT_CONV_BM64_BELOW") > 0 ? env_int("BT_CONV_BM64_BELOW") : 512;
int g_force_bn = env_int("BT_CONV_BN");
int g_dgrad_cls = env_int("BT_CONV_DGRAD_CLS");   // 1 / 4: force the data gradient's classes per block
// first-layer forward: tiles per block of the patch kernel (0 = the im2col tap-GEMM path), output rows per tile
int g_conv1_tiles = env_int("BT_CONV1_TILES");
int g_conv1_rows = env_int("BT_CONV1_ROWS");
int conv1_tiles() { return g_conv1_tiles > 0 ? g_conv1_tiles : g_conv1_tiles < 0 ? 0 : 4; }
int conv1_rows() { return g_conv1_rows == 4 ? 4 : 2; }
// BT_CONV1_BN=0: the first layer never applies its output's BN (the apply launch does)
bool g_conv1_bn = !(std::getenv("BT_CONV1_BN") && std::getenv("BT_CONV1_BN")[0] == '0');
// blocks of the BN-applying first-layer kernel that fit on the device at once (occupancy x CUs, cached)
int conv1_bn_resident() {
  static int cap = -1;
  if (cap < 0) {
    int nb = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, conv1_fwd_kernel<32, 2, true, kConv1Keep>, kThreads, 0) !=
            hipSuccess ||
        hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      nb = cus = 0;
    cap = nb * cus;
  }
  return cap;
}
int64_t conv1_tiles_of(int N, int Ho, int Wo, int tr) {
  return int64_t(N) * ((Ho + tr - 1) / tr) * ((Wo + kC1Cols - 1) / kC1Cols);
}
// A launch whose blocks meet at grid_barrier: outside a graph capture it goes
// through hipLaunchCooperativeKernel, which checks that the whole grid is
// co-resident with what else runs on the device (another stream's kernels, another
// process) and fails instead of starting blocks that would spin into the barrier's
// timeout -- the caller (ops.conv_fwd) then runs the plain forward and the separate
// BN apply.  Inside a capture (cooperative launches are not captured) the plain
// launch, sized by the occupancy query (conv_out_bn_fits); the barrier's timeout
// flag still catches a grid that was not resident.
template <typename... A>
hipError_t launch_grid_barrier(void (*kernel)(A...), dim3 grid, hipStream_t stream, A... args) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &st) == hipSuccess && st == hipStreamCaptureStatusNone) {
    void* argv[] = {static_cast<void*>(&args)...};
    return hipLaunchCooperativeKernel(reinterpret_cast<const void*>(kernel), grid, dim3(kThreads), argv, 0, stream);
  }
  kernel<<<grid, kThreads, 0, stream>>>(args...);
  return hipGetLastError();
}

// the 32 -> 64 forward as the persistent patch GEMM (conv_fwd_patch_kernel), BT_CONV_FWD_PATCH=1; default
// the tap GEMM: alone the patch kernel is 22.5 us against 23.6, but 7.3 us of it is a fixed cost (the
// weights' 64 KB per CU and one block per CU), and in the step the tap GEMM's launch ran faster
// (20.95k vs 20.7k img/s, profiles/r6/b1/disc_*.jsonl, profiles/r6/b2/fwd_patch_bench.jsonl)
int g_fwd_patch = -1;
int g_fwd_patch_dbg = 0, g_fwd_patch_blocks = 0;   // (experiments: conv_set_fwd_patch)
bool fwd_patch() {
  if (g_fwd_patch < 0) {
    const char* v = std::getenv("BT_CONV_FWD_PATCH");
    g_fwd_patch = v && v[0] == '1' ? 1 : 0;
  }
  return g_fwd_patch == 1;
}
int device_cus() {
  static int cus = 0;
  if (cus <= 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
        hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}
// Split-K forward (tap_gemm_body SPLIT = 2, BT_CONV_FWD_SPLIT=1, opt-in): 128-channel tiles whose
// two K halves run as two blocks, for the deep layers whose grids are short of tiles (conv3: 300
// tiles of 128 x 128, conv4: 150 of 64 x 128).  A 128 x 128 tile stages 64 FLOP per byte against 43
// for the 128 x 64 tiles it replaces; the cost is the parked accumulators (64 KiB per tile, written
// through to memory and read back by the partner block).  Measured slower: conv3 28.7-29.9 vs
// 16.5-18.3 us, conv4 25.3 vs 16.7-17.4 us, the disc step 20.4-20.6k vs 21.5-21.7k img/s
// (profiles/r6/b7/): the parked accumulators are ~20 MB a layer, as many bytes as the GEMM's own.  The scratch is per device, grown outside
// a graph capture (a forward captured before an eager one of its size runs unsplit): split forwards
// of one device run one at a time -- on one stream, as a training step's graph does (torch captures
// on its own stream, warm-up runs on another: per-stream scratch would never be there to capture).
int g_fwd_split = -1;
int64_t g_fwd_split_launches = 0;   // (tests: the split path ran)
bool fwd_split_on() {
  if (g_fwd_split < 0) {
    const char* v = std::getenv("BT_CONV_FWD_SPLIT");
    g_fwd_split = v && v[0] == '1' ? 1 : 0;
  }
  return g_fwd_split == 1;
}
struct SplitScratch {
  int device = -1;
  float* part = nullptr;
  unsigned* ticket = nullptr;
  int64_t tiles = 0;
};
std::vector<SplitScratch> g_split_scratch;
SplitScratch& split_scratch() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  for (auto& s : g_split_scratch)
    if (s.device == dev) return s;
  g_split_scratch.push_back(SplitScratch{dev});
  return g_split_scratch.back();
}
// the split forward's pixel tile (64 / 128) for this GEMM, or 0: run it unsplit
int fwd_split_bm(const TapGemm& g, hipStream_t stream) {
  if (!fwd_split_on() || g.C == 4 || g.act.on() || g.oact.on() || g.NOUT % 128 || staging() != 2 ||
      (16 * g.C / FBK) % 2)
    return 0;
  const int bm = (int64_t(g.M) + FBM - 1) / FBM * (g.NOUT / 128) * 2 >= g_bm64_below ? FBM : 64;
  const int64_t tiles = (int64_t(g.M) + bm - 1) / bm * (g.NOUT / 128);
  SplitScratch& sc = split_scratch();
  if (sc.tiles < tiles) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return 0;
    if (hipDeviceSynchronize() != hipSuccess) return 0;   // (the old scratch may be in use)
    if (sc.part) (void)hipFree(sc.part);
    if (sc.ticket) (void)hipFree(sc.ticket);
    sc.part = nullptr, sc.ticket = nullptr, sc.tiles = 0;
    // (FM * FN float4 per thread: 64 KiB per 128 x 128 tile, half that for 64 x 128)
    if (hipMalloc(&sc.part, size_t(tiles * (FBM / 32) * 4 * kThreads * 16)) != hipSuccess ||
        hipMalloc(&sc.ticket, size_t(tiles) * 2 * sizeof(unsigned)) != hipSuccess ||
        hipMemset(sc.ticket, 0, size_t(tiles) * 2 * sizeof(unsigned)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
      if (sc.part) (void)hipFree(sc.part);
      if (sc.ticket) (void)hipFree(sc.ticket);
      sc.part = nullptr, sc.ticket = nullptr;
      (void)hipGetLastError();
      return 0;
    }
    sc.tiles = tiles;
  }
  return bm;
}
// BT_CONV_OUT_BN=0: the tap-GEMM forward never applies its output's BN
bool g_out_bn = !(std::getenv("BT_CONV_OUT_BN") && std::getenv("BT_CONV_OUT_BN")[0] == '0');
// blocks of the BN-applying tap-GEMM forward (64-channel tiles, 2 LDS-DMA stages) resident at once
template <int BM>
int tap_obn_resident() {
  static int cap = -1;
  if (cap < 0) {
    int nb = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, tap_gemm_kernel<false, 64, false, BM, 2, 1, 0, true>,
                                                     kThreads, 0) != hipSuccess ||
        hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      nb = cus = 0;
    cap = nb * cus;
  }
  return cap;
}
}  // namespace

// the tap-GEMM forward's tile for an output BN it applies (0: it cannot: tile, staging or grid)
int tap_obn_bm(int64_t M, int NOUT) {
  if (!g_out_bn || M <= 0 || NOUT > kBnFoldMaxC || conv_tile_channels(NOUT, false) != 64 || staging() != 2) return 0;
  const int bm = conv_tile_pixels(M, NOUT, 1);
  if (bm != 64 && bm != FBM) return 0;
  const int64_t blocks = (M + bm - 1) / bm * (NOUT / 64);
  return blocks <= (bm == 64 ? tap_obn_resident<64>() : tap_obn_resident<FBM>()) ? bm : 0;
}

bool conv_out_bn_fits(int N, int Ho, int Wo, int Cin, int Cout) {
  if (Cin == 4) return conv1_bn_apply_fits(N, Ho, Wo, Cout);
  if (N <= 0 || Ho <= 0 || Wo <= 0 || Cout % 64) return false;
  return tap_obn_bm(int64_t(N) * Ho * Wo, Cout) > 0;
}

bool conv1_bn_apply_fits(int N, int Ho, int Wo, int Cout) {
  if (!g_conv1_bn || Cout != 32 || conv1_tiles() <= 0 || conv1_rows() != 2 || N <= 0 || Ho <= 0 || Wo <= 0)
    return false;
  const int64_t blocks = (conv1_tiles_of(N, Ho, Wo, 2) + kConv1Keep - 1) / kConv1Keep;
  return blocks <= conv1_bn_resident();
}

unsigned conv_grid_barrier_timeouts() {
  unsigned v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_grid_barrier_timeouts), sizeof(v)) != hipSuccess) return ~0u;
  return v;
}

namespace {
volatile unsigned* g_barrier_host_flag = nullptr;   // host view of g_grid_barrier_flag
}

bool conv_grid_barrier_arm() {
  // once per process, outside any graph capture (a symbol copy cannot be
  // captured): the callers arm it when a grid-barrier path is first chosen
  if (g_barrier_host_flag) return true;
  void* host = nullptr;
  if (hipHostMalloc(&host, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return false;
  std::memset(host, 0, 64);
  void* dev = nullptr;
  if (hipHostGetDevicePointer(&dev, host, 0) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(g_grid_barrier_flag), &dev, sizeof(dev)) != hipSuccess) {
    (void)hipHostFree(host);
    return false;
  }
  g_barrier_host_flag = static_cast<volatile unsigned*>(host);
  return true;
}

int conv_grid_barrier_failed() {   // no HIP call: a plain read of the host-mapped word
  return g_barrier_host_flag ? int(*g_barrier_host_flag) : -1;
}

void conv_grid_barrier_clear(int value) {   // value != 0: simulate a failure (tests)
  if (g_barrier_host_flag) *g_barrier_host_flag = unsigned(value);
}

void conv_set_fwd_patch(int on, int dbg, int blocks) {
  g_fwd_patch = on < 0 ? -1 : (on ? 1 : 0);
  g_fwd_patch_dbg = dbg;
  g_fwd_patch_blocks = blocks;
}

void conv_set_conv1_tiles(int tiles, int rows) {   // tiles: > 0 patch kernel, -1 the tap-GEMM path, 0 default
  g_conv1_tiles = tiles;
  g_conv1_rows = rows;
}

int conv_dgrad_classes_per_block(int64_t M, int NOUT) {
  // one parity class per block unless that makes >= 4096 blocks (the
  // 32-channel layer: 4800); then a block runs all four (1200 blocks)
  if (g_dgrad_cls == 1 || g_dgrad_cls == 4) return g_dgrad_cls;
  const int bm = conv_tile_pixels(M, NOUT, 4);
  const int64_t blocks = (M + bm - 1) / bm * (NOUT / conv_tile_channels(NOUT, false)) * 4;
  return blocks >= 4096 ? 4 : 1;
}

void conv_set_tiles(int bm, int bn, int staging, int dgrad_cls) {
  g_force_bm = bm == 64 || bm == 128 ? bm : 0;
  g_force_bn = bn == 32 || bn == 64 || bn == 128 ? bn : 0;
  g_staging = staging == 0 || staging == 2 || staging == 3 || staging == 4 ? staging : -1;
  g_dgrad_cls = dgrad_cls == 1 || dgrad_cls == 4 ? dgrad_cls : 0;
}

int conv_tile_channels(int NOUT, bool c4) {
  // 64 by default; 128 (an override) halves how often the tap-gathered A
  // tile is re-read; 32 for 32-channel outputs.  The first layer's one-step K
  // has no use for 128.
  const int f = g_force_bn;
  if (f && NOUT % f == 0 && !(c4 && f == 128)) return f;
  return NOUT % 64 == 0 ? 64 : 32;
}

int conv_tile_pixels(int64_t M, int NOUT, int ytiles) {
  // fewer than 2 blocks per CU with 128-pixel tiles: halve the tile
  if (g_force_bm) return g_force_bm;
  const int64_t blocks = (M + FBM - 1) / FBM * (NOUT / conv_tile_channels(NOUT, false)) * ytiles;
  return blocks < g_bm64_below ? 64 : FBM;
}

int64_t conv_fwd_tiles(int64_t M, int NOUT) {
  const int bm = conv_tile_pixels(M, NOUT, 1);
  return (M + bm - 1) / bm;
}

hipError_t conv_fwd(const ConvFwdParams& p, hipStream_t stream) {
  if (!conv_fwd_supported(p.Cin, p.Cout) || !p.x || !p.w || !p.y) return hipErrorInvalidValue;
  if (p.Ho != (p.H + 2 - 4) / 2 + 1 || p.Wo != (p.W + 2 - 4) / 2 + 1 || p.M != int64_t(p.N) * p.Ho * p.Wo)
    return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(p.x) | reinterpret_cast<uintptr_t>(p.w) | reinterpret_cast<uintptr_t>(p.y)) & 15)
    return hipErrorInvalidValue;
  if (int64_t(p.N) * p.H * p.W * p.Cin * 2 >= int64_t(kOOB) || p.M * p.Cout >= int64_t(kOOB))
    return hipErrorInvalidValue;   // 32-bit offsets
  TapGemm g;
  g.src = p.x, g.w = p.w, g.dst = p.y, g.stats = p.stats;
  g.N = p.N, g.SH = p.H, g.SW = p.W, g.C = p.Cin, g.cshift = ilog2_exact(p.Cin);
  g.GH = p.Ho, g.GW = p.Wo, g.M = int(p.M);
  g.NOUT = p.Cout, g.OH = p.Ho, g.OW = p.Wo;
  g.wc = p.Cin == 4 ? (p.w_channels > 0 ? p.w_channels : 4) : p.Cin;
  g.lut = p.Cin == 4 ? p.lut : nullptr;
  if (p.lut && (p.Cin != 4 || (reinterpret_cast<uintptr_t>(p.lut) & 7))) return hipErrorInvalidValue;
  g.acc_r = p.stats ? p.acc_r : 0;
  if (g.acc_r < 0 || g.acc_r > 64) return hipErrorInvalidValue;
  if (p.act_out && !p.act.on()) {   // u8 first layer: the decoded frame as a side output (patch kernel)
    if (p.Cin != 4 || !p.lut || conv1_tiles() <= 0 || p.H % 2 || p.W % 2 || (reinterpret_cast<uintptr_t>(p.act_out) & 7) ||
        (p.stats && p.acc_r <= 0) || p.Cout != conv_tile_channels(p.Cout, true))
      return hipErrorInvalidValue;   // (the conditions of the patch kernel's dispatch below)
    g.act_out = p.act_out;
  }
  if (p.act.on()) {   // the input BN applied in the staging: C <= 128 (two coefficient sets), accumulator given
    if (p.Cin == 4 || p.Cin > 2 * FBK || !p.act.acc || p.act.R <= 0 || !p.act.b || !p.act.mean || !p.act.invstd ||
        p.act.M != int64_t(p.N) * p.H * p.W || (reinterpret_cast<uintptr_t>(p.act_out) & 15) ||
        (p.act_out && (p.H % 2 || p.W % 2)))   // the centre taps cover every input element: even sides
      return hipErrorInvalidValue;
    g.act = p.act;
    g.act_out = p.act_out;
  }
  if (p.Cin == 4 && g.wc != 3 && g.wc != 4) return hipErrorInvalidValue;
  // the first layer from a decoded input patch (conv1_fwd_kernel): BN sums
  // into an accumulator (or none), Cout 32 / 64
  const int bn1 = conv_tile_channels(p.Cout, true);
  if (p.out_act.on() && p.Cin != 4) {   // the tap GEMM applies the output's BN too (grid barrier)
    const int bm = tap_obn_bm(p.M, p.Cout);
    if (p.act.on() || !p.stats || g.acc_r <= 0 || !p.out_y || (reinterpret_cast<uintptr_t>(p.out_y) & 15) ||
        p.out_act.acc != reinterpret_cast<double*>(p.stats) || p.out_act.R != g.acc_r || p.out_act.M != p.M ||
        !p.out_act.b || !p.out_act.mean || !p.out_act.invstd || bm == 0 || p.M >= int64_t(kOOB))
      return hipErrorInvalidValue;
    g.oact = p.out_act, g.oy = p.out_y;
    const dim3 grid(unsigned((p.M + bm - 1) / bm * (p.Cout / 64)));
    if (bm == 64) return launch_grid_barrier(tap_gemm_kernel<false, 64, false, 64, 2, 1, 0, true>, grid, stream, g);
    return launch_grid_barrier(tap_gemm_kernel<false, 64, false, FBM, 2, 1, 0, true>, grid, stream, g);
  }
  if (p.out_act.on()) {   // the output's BN applied here too (grid barrier): checked again, as the caller asked
    if (p.Cin != 4 || !p.lut || !p.stats || g.acc_r <= 0 || !p.out_y || p.Cout != 32 || bn1 != 32 ||
        (reinterpret_cast<uintptr_t>(p.out_y) & 15) || p.out_act.acc != reinterpret_cast<double*>(p.stats) ||
        p.out_act.R != g.acc_r || p.out_act.M != p.M || !p.out_act.b || !p.out_act.mean || !p.out_act.invstd ||
        !conv1_bn_apply_fits(p.N, p.Ho, p.Wo, p.Cout))
      return hipErrorInvalidValue;
    Conv1Bn ob;
    ob.act = p.out_act, ob.y = p.out_y;
    const unsigned blocks = unsigned((conv1_tiles_of(p.N, p.Ho, p.Wo, 2) + kConv1Keep - 1) / kConv1Keep);
    return launch_grid_barrier(conv1_fwd_kernel<32, 2, true, kConv1Keep>, dim3(blocks), stream, g, kConv1Keep, ob);
  }
  if (p.Cin == 4 && (!p.stats || g.acc_r > 0) && p.Cout == bn1 && conv1_tiles() > 0) {
    const int tr = conv1_rows(), tpb = conv1_tiles();
    const int64_t ntiles = conv1_tiles_of(p.N, p.Ho, p.Wo, tr);
    const unsigned blocks = unsigned((ntiles + tpb - 1) / tpb);
    const dim3 grid(blocks);
    const bool u8 = g.lut != nullptr;
#define BT_CONV1(BN_, TR_)                                                   \
    do {                                                                     \
      if (u8) conv1_fwd_kernel<BN_, TR_, true><<<grid, kThreads, 0, stream>>>(g, tpb, Conv1Bn());  \
      else conv1_fwd_kernel<BN_, TR_, false><<<grid, kThreads, 0, stream>>>(g, tpb, Conv1Bn());    \
    } while (0)
    if (bn1 == 64 && tr == 4) BT_CONV1(64, 4);
    else if (bn1 == 64) BT_CONV1(64, 2);
    else if (tr == 4) BT_CONV1(32, 4);
    else BT_CONV1(32, 2);
#undef BT_CONV1
    return hipGetLastError();
  }
  if (p.Cin == FP_CIN && p.Cout == FP_COUT && fwd_patch() && !p.act.on() && !p.act_out && (!p.stats || g.acc_r > 0)) {
    // the persistent patch GEMM: one block per CU (its LDS), each walking a share of the tiles
    const int64_t ntiles = int64_t(p.N) * ((p.Ho + FP_TA - 1) / FP_TA) * ((p.Wo + FP_TB - 1) / FP_TB);
    if (ntiles < (int64_t(1) << 30)) {
      const int cus = g_fwd_patch_blocks > 0 ? g_fwd_patch_blocks : device_cus();
      const unsigned blocks = unsigned(ntiles < cus ? ntiles : cus);
      conv_fwd_patch_kernel<<<blocks, kThreads, 0, stream>>>(g, int(ntiles), g_fwd_patch_dbg);
      return hipGetLastError();
    }
  }
  if (const int sbm = fwd_split_bm(g, stream)) {
    SplitScratch& sc = split_scratch();
    g.split_part = sc.part, g.split_ticket = sc.ticket;
    ++g_fwd_split_launches;
    const dim3 grid(unsigned((g.M + sbm - 1) / sbm * (g.NOUT / 128) * 2));
    if (sbm == 64) tap_gemm_kernel<false, 128, false, 64, 2, 1, 0, false, 2><<<grid, kThreads, 0, stream>>>(g);
    else tap_gemm_kernel<false, 128, false, FBM, 2, 1, 0, false, 2><<<grid, kThreads, 0, stream>>>(g);
    return hipGetLastError();
  }
  launch_tap_gemm<false>(g, 1, stream);
  return hipGetLastError();
}

void conv_set_fwd_split(int on) { g_fwd_split = on < 0 ? -1 : (on ? 1 : 0); }
int64_t conv_fwd_split_launches() { return g_fwd_split_launches; }

hipError_t conv_weight_t(const uint16_t* w, uint16_t* wt, int Cout, int Cin, hipStream_t stream) {
  if (!w || !wt || Cout <= 0 || Cin <= 0) return hipErrorInvalidValue;
  const int total = Cout * 16 * Cin;
  const int blocks = (total + kThreads - 1) / kThreads;
  weight_t_kernel<<<blocks < 2048 ? blocks : 2048, kThreads, 0, stream>>>(w, wt, Cout, Cin);
  return hipGetLastError();
}

hipError_t conv_weight_t_multi(const WeightTParams& p, hipStream_t stream) {
  if (p.n <= 0) return hipSuccess;
  if (p.n > kMaxWeightT) return hipErrorInvalidValue;
  int most = 0;
  for (int k = 0; k < p.n; ++k) {
    if (!p.src[k] || !p.dst[k] || p.cout[k] <= 0 || p.cin[k] <= 0) return hipErrorInvalidValue;
    most = std::max(most, p.cout[k] * 16 * p.cin[k]);
  }
  const int blocks = (most + kThreads - 1) / kThreads;
  weight_t_multi_kernel<<<dim3(unsigned(blocks < 1024 ? blocks : 1024), unsigned(p.n)), kThreads, 0, stream>>>(p);
  return hipGetLastError();
}

int64_t conv_dgrad_bn_rows(int N, int H, int W, int Cin) {
  const int64_t M = int64_t(N) * (H / 2) * (W / 2);
  const int bm = conv_tile_pixels(M, Cin, 4);
  return (M + bm - 1) / bm * 4;
}

hipError_t conv_dgrad(const uint16_t* dy, const uint16_t* wt, uint16_t* dx, int N, int H, int W, int Cin, int Cout,
                      hipStream_t stream, const BnBwdFuse* bn) {
  if (!conv_dgrad_supported(Cin, Cout) || !dy || !wt || !dx || H % 2 || W % 2) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(wt) | reinterpret_cast<uintptr_t>(dx)) & 15)
    return hipErrorInvalidValue;
  const int Ho = H / 2, Wo = W / 2;
  if (int64_t(N) * Ho * Wo * Cout * 2 >= int64_t(kOOB) || int64_t(N) * H * W * Cin >= int64_t(kOOB))
    return hipErrorInvalidValue;
  TapGemm g;
  g.src = dy, g.w = wt, g.dst = dx;
  g.N = N, g.SH = Ho, g.SW = Wo, g.C = Cout, g.cshift = ilog2_exact(Cout);
  g.GH = Ho, g.GW = Wo, g.M = N * Ho * Wo;   // one parity class: every (a, b)
  g.NOUT = Cin, g.OH = H, g.OW = W;
  if (bn && bn->part) {
    if (!bn->x || !bn->mean || !bn->invstd || !bn->w || !bn->b || bn->acc_r < 0 || bn->acc_r > 64 ||
        (bn->acc_r == 0 && bn->rows != conv_dgrad_bn_rows(N, H, W, Cin)) || (reinterpret_cast<uintptr_t>(bn->x) & 15))
      return hipErrorInvalidValue;
    g.bn = *bn;
  }
  // the 32-channel layer (dY 64 channels -> dx 32): from a dY patch, all four classes per block
  // (BN-backward sums into an accumulator, or none)
  if (Cout == DP_C && Cin == DP_NOUT && dgrad_patch() && (!g.bn.part || g.bn.acc_r > 0)) {
    const int64_t blocks = int64_t(N) * ((Ho + DP_TA - 1) / DP_TA) * ((Wo + DP_TB - 1) / DP_TB);
    if (g_hold && fuse_patch()) {   // held for the weight gradient that follows (dpatch_wgrad_kernel)
      const hipError_t e = conv_dgrad_flush();
      if (e != hipSuccess) return e;
      g_held.g = g;
      g_held.patch = true;
      g_held.bm = 0;
      g_held.gx = unsigned(blocks);
      g_held.s = stream;
      g_held.on = true;
      return hipSuccess;
    }
    dgrad_patch_kernel<<<unsigned(blocks), kThreads, 0, stream>>>(g);
    return hipGetLastError();
  }
  g.cls_per_block = conv_dgrad_classes_per_block(g.M, g.NOUT);
  if (g_hold) {   // held for the weight gradient that follows (dgrad_wgrad_kernel)
    const hipError_t e = conv_dgrad_flush();
    if (e != hipSuccess) return e;
    const int bn = dgrad_bn128() && g.NOUT % 128 == 0 ? 128 : conv_tile_channels(g.NOUT, false);
    const int bm = conv_tile_pixels(g.M, g.NOUT, 4);
    if (g.cls_per_block == 1 && (bn == 64 || bn == 128) && staging() == 2 && (bm == 64 || bm == FBM)) {
      g_held.g = g;
      g_held.patch = false;
      g_held.bm = bm;
      g_held.bn = bn;
      g_held.gx = unsigned((g.M + bm - 1) / bm * (g.NOUT / bn));
      g_held.s = stream;
      g_held.on = true;
      return hipSuccess;
    }
  }
  launch_tap_gemm<true>(g, 4, stream);
  return hipGetLastError();
}

void conv_dgrad_hold(int on) { g_hold = on != 0; }

hipError_t conv_dgrad_flush() {
  if (!g_held.on) return hipSuccess;
  g_held.on = false;
  if (g_held.patch) dgrad_patch_kernel<<<g_held.gx, kThreads, 0, g_held.s>>>(g_held.g);
  else launch_tap_gemm<true>(g_held.g, 4, g_held.s);
  return hipGetLastError();
}

}  // namespace gpu
}  // namespace btn
