// gfx950 training-step kernels of the consumer models (see kernels.h):
// NHWC adaptive average pooling, BatchNorm2d + LeakyReLU (statistics,
// finalize -- per-tile rows or fp64 accumulators -- and apply, forward and
// backward), the multi-tensor dtype cast and Adam.  Split from kernels.hip
// (the image-path kernels) so the two compile in parallel.
#include <hip/hip_runtime.h>
#include <hip/amd_detail/amd_hip_unsafe_atomics.h>

#include <cstdlib>

#include "adam_sched.h"
#include "bn_fold.h"
#include "kernels.h"
#include "wgrad_reduce.h"

namespace btn {
namespace gpu {

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ uint16_t f2bf(float f) {
  // round-to-nearest-even in one v_cvt_pk_bf16_f32 (gfx950)
  return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f));
}

}  // namespace

// ---------------------------------------------------------------------------
// Adaptive average pooling, NHWC.  The pooled maps are small (the DCGAN
// consumer pools 8 x 30 x 40 x 256 bf16 down to 4 x 4), so the kernels are
// shaped for parallelism, not bandwidth: forward = one lane per output
// element, lanes of a wave walk adjacent channels (every window load is one
// coalesced 128/256-byte row segment); backward = one lane per input element
// gathering the (at most a few) output cells whose window covers it -- no
// atomics, every gradient written once.

template <int DT>
__device__ __forceinline__ float load_act(const void* p, int64_t i) {
  if constexpr (DT == OUT_BF16)
    return __uint_as_float(uint32_t(reinterpret_cast<const uint16_t*>(p)[i]) << 16);
  else
    return reinterpret_cast<const float*>(p)[i];
}

template <int DT>
__device__ __forceinline__ void store_act(void* p, int64_t i, float v) {
  if constexpr (DT == OUT_BF16)
    reinterpret_cast<uint16_t*>(p)[i] = f2bf(v);
  else
    reinterpret_cast<float*>(p)[i] = v;
}

__device__ __forceinline__ int win_start(int i, int in, int out) { return int((int64_t(i) * in) / out); }
__device__ __forceinline__ int win_end(int i, int in, int out) { return int((int64_t(i + 1) * in + out - 1) / out); }

template <int DT>
__global__ __launch_bounds__(kBlock) void avgpool_fwd_kernel(const void* __restrict__ x, void* __restrict__ y, int N,
                                                             int H, int W, int C, int OH, int OW) {
  const int64_t total = int64_t(N) * OH * OW * C;
  for (int64_t o = int64_t(blockIdx.x) * kBlock + threadIdx.x; o < total; o += int64_t(gridDim.x) * kBlock) {
    const int c = int(o % C);
    int64_t r = o / C;
    const int j = int(r % OW);
    r /= OW;
    const int i = int(r % OH);
    const int n = int(r / OH);
    const int h0 = win_start(i, H, OH), h1 = win_end(i, H, OH);
    const int w0 = win_start(j, W, OW), w1 = win_end(j, W, OW);
    float acc = 0.f;
    for (int h = h0; h < h1; ++h) {
      const int64_t row = ((int64_t(n) * H + h) * W) * C + c;
#pragma unroll 4
      for (int w = w0; w < w1; ++w) acc += load_act<DT>(x, row + int64_t(w) * C);
    }
    store_act<DT>(y, o, acc / float((h1 - h0) * (w1 - w0)));
  }
}

template <int DT>
__global__ __launch_bounds__(kBlock) void avgpool_bwd_kernel(const void* __restrict__ gy, void* __restrict__ gx, int N,
                                                             int H, int W, int C, int OH, int OW) {
  const int64_t total = int64_t(N) * H * W * C;
  for (int64_t e = int64_t(blockIdx.x) * kBlock + threadIdx.x; e < total; e += int64_t(gridDim.x) * kBlock) {
    const int c = int(e % C);
    int64_t r = e / C;
    const int w = int(r % W);
    r /= W;
    const int h = int(r % H);
    const int n = int(r / H);
    // output rows whose window covers h: floor(h*OH/H) .. ceil((h+1)*OH/H)-1
    const int i0 = int((int64_t(h) * OH) / H), i1 = int((int64_t(h + 1) * OH + H - 1) / H);
    const int j0 = int((int64_t(w) * OW) / W), j1 = int((int64_t(w + 1) * OW + W - 1) / W);
    float acc = 0.f;
    for (int i = i0; i < i1 && i < OH; ++i) {
      const int hs = win_start(i, H, OH), he = win_end(i, H, OH);
      if (h < hs || h >= he) continue;
      for (int j = j0; j < j1 && j < OW; ++j) {
        const int ws = win_start(j, W, OW), we = win_end(j, W, OW);
        if (w < ws || w >= we) continue;
        acc += load_act<DT>(gy, ((int64_t(n) * OH + i) * OW + j) * C + c) / float((he - hs) * (we - ws));
      }
    }
    store_act<DT>(gx, e, acc);
  }
}

namespace {
int pool_grid(int64_t total) {
  const int64_t blocks = (total + kBlock - 1) / kBlock;
  return int(blocks < 8192 ? (blocks < 1 ? 1 : blocks) : 8192);
}
}  // namespace

hipError_t adaptive_avgpool_nhwc(const void* x, void* y, int N, int H, int W, int C, int OH, int OW, int dtype,
                                 hipStream_t stream) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || OH <= 0 || OW <= 0) return hipErrorInvalidValue;
  const int grid = pool_grid(int64_t(N) * OH * OW * C);
  if (dtype == OUT_BF16)
    avgpool_fwd_kernel<OUT_BF16><<<grid, kBlock, 0, stream>>>(x, y, N, H, W, C, OH, OW);
  else if (dtype == OUT_F32)
    avgpool_fwd_kernel<OUT_F32><<<grid, kBlock, 0, stream>>>(x, y, N, H, W, C, OH, OW);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t adaptive_avgpool_nhwc_bwd(const void* gy, void* gx, int N, int H, int W, int C, int OH, int OW, int dtype,
                                     hipStream_t stream) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || OH <= 0 || OW <= 0) return hipErrorInvalidValue;
  const int grid = pool_grid(int64_t(N) * H * W * C);
  if (dtype == OUT_BF16)
    avgpool_bwd_kernel<OUT_BF16><<<grid, kBlock, 0, stream>>>(gy, gx, N, H, W, C, OH, OW);
  else if (dtype == OUT_F32)
    avgpool_bwd_kernel<OUT_F32><<<grid, kBlock, 0, stream>>>(gy, gx, N, H, W, C, OH, OW);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Training-mode BatchNorm2d + LeakyReLU, channels-last.  The consumer's
// BN -> LeakyReLU pairs were 7 MIOpen/PyTorch kernels per layer and step
// (mean/variance, final, normalise, leaky; and the same backwards), each a
// full pass over the activation.  Here: forward = one statistics pass + one
// normalise-and-activate pass; backward = one reduction pass + one gradient
// pass, with the activation's derivative recomputed from x (z > 0 <=> y > 0
// for a positive slope), so nothing but x is kept for backward.
//
// Reductions: a lane owns V = 16 B of channels of a row (8 bf16 / 4 fp32),
// the G = C / V lanes of one row read it as one contiguous segment and
// R = 256 / G rows are in flight per block; per-block partial sums go through
// LDS to a [blocks, 2C] scratch that one lane per channel folds in fp64.

constexpr int kBnMaxBlocks = 1024;

template <int DT>
struct BnVec {
  static constexpr int V = DT == OUT_BF16 ? 8 : 4;
  static constexpr int ES = DT == OUT_BF16 ? 2 : 4;
};

template <int DT>
__device__ __forceinline__ uint4 bn_load_raw(const void* p, int64_t e) {
  return *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(p) + e * BnVec<DT>::ES);
}

template <int DT>
__device__ __forceinline__ void bn_unpack(const uint4 raw, float (&v)[BnVec<DT>::V]) {
  const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
  if constexpr (DT == OUT_BF16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = __uint_as_float(w[i]);
  }
}

template <int DT>
__device__ __forceinline__ void bn_load(const void* p, int64_t e, float (&v)[BnVec<DT>::V]) {
  const uint4 raw = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(p) + e * BnVec<DT>::ES);
  const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
  if constexpr (DT == OUT_BF16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = __uint_as_float(w[i]);
  }
}

template <int DT>
__device__ __forceinline__ void bn_store(void* p, int64_t e, const float (&v)[BnVec<DT>::V]) {
  uint4 raw;
  if constexpr (DT == OUT_BF16) {
    raw.x = uint32_t(f2bf(v[0])) | (uint32_t(f2bf(v[1])) << 16);
    raw.y = uint32_t(f2bf(v[2])) | (uint32_t(f2bf(v[3])) << 16);
    raw.z = uint32_t(f2bf(v[4])) | (uint32_t(f2bf(v[5])) << 16);
    raw.w = uint32_t(f2bf(v[6])) | (uint32_t(f2bf(v[7])) << 16);
  } else {
    raw = make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3]));
  }
  *reinterpret_cast<uint4*>(reinterpret_cast<char*>(p) + e * BnVec<DT>::ES) = raw;
}

// BWD = false: sums of x and x^2.  BWD = true: sums of gz and gz * xhat.
template <int DT, bool BWD>
__global__ __launch_bounds__(kBlock) void bn_reduce_kernel(const void* __restrict__ x, const void* __restrict__ gy,
                                                           int64_t M, int C, int64_t rows_per_block,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ w, const float* __restrict__ b,
                                                           float slope, float* __restrict__ partial,
                                                           int acc_r = 0) {
  constexpr int V = BnVec<DT>::V;
  // partials laid out [V][kBlock + 1]: lane t's V values land in V different
  // rows at column t, so the write is bank-conflict free (a [row][C] layout
  // put the lanes' 8-float runs on the same banks)
  constexpr int LS = kBlock + 1;
  __shared__ float ls[V * LS], lq[V * LS];
  const int G = C / V, R = kBlock / G;
  const int g = int(threadIdx.x) % G, r0 = int(threadIdx.x) / G;
  const int c0 = g * V;
  float nm[V], is[V], ww[V], bb[V];   // xhat = v * is + nm, as bn_apply_kernel computes it
  if constexpr (BWD) {
#pragma unroll
    for (int i = 0; i < V; ++i)
      is[i] = invstd[c0 + i], nm[i] = -mean[c0 + i] * is[i], ww[i] = w[c0 + i], bb[i] = b[c0 + i];
  }
  float s[V], q[V];
#pragma unroll
  for (int i = 0; i < V; ++i) s[i] = 0.f, q[i] = 0.f;
  const int64_t row_begin = int64_t(blockIdx.x) * rows_per_block;
  const int64_t row_end = row_begin + rows_per_block < M ? row_begin + rows_per_block : M;
  for (int64_t r = row_begin + r0; r < row_end; r += R) {
    float v[V];
    bn_load<DT>(x, r * C + c0, v);
    if constexpr (BWD) {
      float gv[V];
      bn_load<DT>(gy, r * C + c0, gv);
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const float xh = fmaf(v[i], is[i], nm[i]);
        const float gz = fmaf(xh, ww[i], bb[i]) > 0.f ? gv[i] : gv[i] * slope;
        s[i] += gz;
        q[i] += gz * xh;
      }
    } else {
#pragma unroll
      for (int i = 0; i < V; ++i) s[i] += v[i], q[i] += v[i] * v[i];
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i) ls[i * LS + threadIdx.x] = s[i], lq[i * LS + threadIdx.x] = q[i];
  __syncthreads();
  for (int c = int(threadIdx.x); c < C; c += kBlock) {
    // channel c = group c / V, element c % V; its R partials sit in lanes r * G + c / V
    const float* ps = ls + (c % V) * LS + c / V;
    const float* pq = lq + (c % V) * LS + c / V;
    float a = 0.f, q2 = 0.f;
    for (int r = 0; r < R; ++r) a += ps[r * G], q2 += pq[r * G];
    if (acc_r > 0) {   // a BnAcc accumulator (fp64 [acc_r][2][C]): consecutive lanes, consecutive doubles
      double* row = reinterpret_cast<double*>(partial) + int64_t(int(blockIdx.x) % acc_r) * 2 * C;
      unsafeAtomicAdd(row + c, double(a));
      unsafeAtomicAdd(row + C + c, double(q2));
    } else {
      // channel-major [2C][blocks]: the fold reads each channel's partials contiguously
      partial[int64_t(c) * gridDim.x + blockIdx.x] = a;
      partial[int64_t(C + c) * gridDim.x + blockIdx.x] = q2;
    }
  }
}

// One WAVE per channel folds the per-block partials in fp64 (a single lane
// per channel walking 1024 partials serially cost ~1 ms per step; a 256-lane
// block per channel with an LDS tree and 8 barriers ~6.5 us per call).
// Partials are channel-major ([2C][nblocks]: sums, then sums of squares), so
// a wave's lanes read consecutive floats.  Lane 0 of the wave returns.
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ void bn_fold(const float* __restrict__ partial, int nblocks, int C, int c, double& s,
                                        double& q) {
  const int lane = int(threadIdx.x) & 63;
  double a = 0.0, b2 = 0.0;
  const float* ps = partial + int64_t(c) * nblocks;
  const float* pq = partial + int64_t(C + c) * nblocks;
#pragma unroll 4
  for (int b = lane; b < nblocks; b += 64) a += ps[b], b2 += pq[b];
  s = wave_sum(a);
  q = wave_sum(b2);
}

constexpr int kFoldWaves = 4;   // channels per finalize block (one wave each)

__global__ __launch_bounds__(64 * kFoldWaves) void bn_finalize_kernel(const float* __restrict__ partial, int nblocks,
                                                                      int64_t M, int C, float eps, float momentum,
                                                                      float* mean, float* invstd, float* rm,
                                                                      float* rv, int64_t* tracked) {
  const int c = int(blockIdx.x) * kFoldWaves + (int(threadIdx.x) >> 6);
  if (c >= C) return;
  double s, q;
  bn_fold(partial, nblocks, C, c, s, q);
  if ((threadIdx.x & 63) != 0) return;
  if (tracked && c == 0) tracked[0] += 1;   // BatchNorm2d.num_batches_tracked (saves a launch)
  const double mu = s / double(M);
  double var = q / double(M) - mu * mu;
  var = var < 0.0 ? 0.0 : var;
  mean[c] = float(mu);
  invstd[c] = float(1.0 / sqrt(var + double(eps)));
  if (rm) {
    rm[c] = float((1.0 - momentum) * rm[c] + momentum * mu);
    rv[c] = float((1.0 - momentum) * rv[c] + momentum * var * double(M) / double(M > 1 ? M - 1 : 1));
  }
}

__global__ __launch_bounds__(64 * kFoldWaves) void bn_bwd_finalize_kernel(const float* __restrict__ partial,
                                                                          int nblocks, int C, float* dw, float* db) {
  const int c = int(blockIdx.x) * kFoldWaves + (int(threadIdx.x) >> 6);
  if (c >= C) return;
  double s, q;
  bn_fold(partial, nblocks, C, c, s, q);
  if ((threadIdx.x & 63) != 0) return;
  db[c] = float(s);
  dw[c] = float(q);
}

// BWD = false: y = leaky(xhat * w + b).  BWD = true: gx = w * invstd * (gz - db/M - xhat * dw/M).
// The grid-stride step is a multiple of kBlock and G = C / V divides kBlock,
// so a lane keeps one channel group for the whole loop: its per-channel
// coefficients are loaded once into registers, not per element.  Each lane
// takes kBnUnroll vectors kBlock apart per pass with every load issued before
// any math: one 16-byte vector per lane per pass left the kernel waiting out a
// load latency per 16 bytes (9.9 / 12.4 us per call where the bytes take 1-4).
constexpr int kBnUnroll = 4;

// BnAcc finalize (kernels.h): ONE block folds, finalizes and clears the fp64
// accumulator (bn_fold.h).  The per-tile-row finalize this replaces walked
// ~4800 rows per channel (6-8 us a call); this is one memory latency.
constexpr int kBnAccMaxC = 512;

template <bool BWD>
__global__ __launch_bounds__(kBlock) void bn_acc_finalize_kernel(double* __restrict__ acc, int R, int64_t M, int C,
                                                                 float eps, float momentum, float* o0, float* o1,
                                                                 float* rm, float* rv, int64_t* tracked) {
  __shared__ double part[2 * kBnAccMaxC];
  BnFold f;
  f.acc = acc, f.R = R, f.C = C, f.M = M, f.bwd = BWD ? 1 : 0, f.eps = eps, f.momentum = momentum;
  f.o0 = o0, f.o1 = o1, f.rm = rm, f.rv = rv, f.tracked = tracked;
  bn_fold_block(f, part);
}

// FOLD: the coefficients come from the BnAcc accumulator the producer added
// into, folded by every block itself (bn_fold.h: bn_acc_column_sums /
// bn_acc_release) -- no finalize launch before the apply.
struct BnApplyFold {
  double* acc = nullptr;
  int R = 0;
  float eps = 0.f, momentum = 0.f;
  float* o0 = nullptr;         // forward: mean; backward: db  (block 0 writes)
  float* o1 = nullptr;         // forward: invstd; backward: dw
  float* rm = nullptr;         // forward: running statistics, num_batches_tracked
  float* rv = nullptr;
  int64_t* tracked = nullptr;
  int release = 1;             // 1: ticket taken after the fold, answered at the end; 2: whole release
                               // before the pass (BT_BN_RELEASE=2); 0: none (=0: timing diagnostics only)
};

// PF (FOLD launches, BT_BN_PREFETCH): the next pass's loads go out before this pass is applied (two
// register sets), every load a buffer load issued unconditionally (past the end: out of range, no
// traffic) so the memory-counter waits count exactly -- a pass then waits only for its own loads,
// not for the previous pass's stores or a load issued behind them
template <int DT, bool BWD, bool FOLD = false, int U = kBnUnroll, bool PF = false>
__global__ __launch_bounds__(kBlock) void bn_apply_kernel(const void* __restrict__ x, const void* __restrict__ gy,
                                                          void* __restrict__ out, int64_t M, int C,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          const float* __restrict__ w, const float* __restrict__ b,
                                                          const float* __restrict__ dw, const float* __restrict__ db,
                                                          float slope, BnApplyFold fa = BnApplyFold()) {
  constexpr int V = BnVec<DT>::V;
  const int G = C / V;
  const int64_t total = M * G;
  const float invM = 1.f / float(M);
  const int c0 = (int(threadIdx.x) % G) * V;
  // The block's first pass of loads goes out before the coefficients are
  // read, so their latencies overlap; later passes load at the end of the
  // previous one (one register set).  The loads stay raw until the apply
  // unpacks them: unpacking at load time made the compiler wait for the
  // first pass before the accumulator fold even started.
  const int64_t pass = int64_t(gridDim.x) * kBlock * U;
  int64_t idx = int64_t(blockIdx.x) * kBlock * U + threadIdx.x;
  uint4 rv[U], rg[U];
  unsigned rel_tk = 0;   // FOLD: this block's release ticket (thread 0)
  auto load_pass = [&]() {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      rv[u] = bn_load_raw<DT>(x, (idx + u * kBlock) * V);
      if constexpr (BWD) rg[u] = bn_load_raw<DT>(gy, (idx + u * kBlock) * V);
    }
  };
  // (PF) 16-byte vector e of x / gy at byte 16 e; a dead pass (i < 0) reads out of range: zeros
  const __amdgpu_buffer_rsrc_t rs_xv = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(x), 0, int(PF ? total * 16 : 0),
                                                                         0x00020000);
  const __amdgpu_buffer_rsrc_t rs_gv =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(BWD ? gy : x), 0, int(PF ? total * 16 : 0), 0x00020000);
  auto load_pass_b = [&](int64_t i, uint4 (&a)[U], uint4 (&c)[U]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t off = i >= 0 ? uint32_t((i + u * kBlock) * 16) : 0x80000000u;
      a[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs_xv, off, 0, 0));
      if constexpr (BWD) c[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs_gv, off, 0, 0));
    }
  };
  bool have = idx + (U - 1) * kBlock < total;   // a whole pass: U vectors per lane
  if constexpr (PF) load_pass_b(have ? idx : -1, rv, rg);
  else if (have) load_pass();
  // xhat = v * is + nm;  z = xhat * ww + bb;  backward: gx = P * (gz - dbm) - pdw * xhat (BnBwdCoef)
  float is[V], nm[V], ww[V], bb[V];
  BnBwdCoef bc[BWD ? V : 1];
  if constexpr (FOLD) {
    // coef holds the two folded per-channel arrays (forward: mean, invstd;
    // backward: db, dw) in a lane-major order: channel c = V g + k at
    // 4 g + k (k < 4) or 4 G + 4 g + k - 4 (bf16, V = 8), so the G lanes of a
    // row read their V channels as 16-byte vectors at consecutive 16-byte
    // slots -- conflict-free ds_read_b128 (a lane reading its 8 floats one by
    // one at a 32-byte stride ran 2-4 way conflicted: PMC 30-69 % for C >= 64)
    __shared__ double part[2 * kBnAccMaxC > kBlock ? 2 * kBnAccMaxC : kBlock];
    __shared__ __attribute__((aligned(16))) float coef[2 * kBnAccMaxC];
    auto pos = [&](int c) {
      if constexpr (V == 8) {
        const int gg = c >> 3, k = c & 7;
        return k < 4 ? 4 * gg + k : 4 * G + 4 * gg + k - 4;
      } else {
        return c;
      }
    };
    // the lane's BN weights (and backward: the forward statistics) now, in flight with the fold's reads
    float wl[V], bl[V], ml[BWD ? V : 1], il[BWD ? V : 1];
#pragma unroll
    for (int i = 0; i < V; ++i) {
      wl[i] = w[c0 + i], bl[i] = b[c0 + i];
      if constexpr (BWD) ml[i] = mean[c0 + i], il[i] = invstd[c0 + i];
    }
    bn_acc_column_sums(fa.acc, fa.R, 2 * C, part);
    const bool first = blockIdx.x == 0;
    for (int c = int(threadIdx.x); c < C; c += kBlock) {
      float c0v, c1v;
      if constexpr (BWD) {   // db = sum gz, dw = sum gz * xhat (bn_fold_block, bwd)
        c0v = float(part[c]);
        c1v = float(part[C + c]);
        if (first) fa.o0[c] = c0v, fa.o1[c] = c1v;
      } else {               // exactly bn_fold_block's forward finalize
        const double mu = part[c] / double(M);
        double var = part[C + c] / double(M) - mu * mu;
        var = var < 0.0 ? 0.0 : var;
        c0v = float(mu);
        c1v = float(1.0 / sqrt(var + double(fa.eps)));
        if (first) {
          fa.o0[c] = c0v;
          fa.o1[c] = c1v;
          if (fa.rm) {
            fa.rm[c] = float((1.0 - fa.momentum) * fa.rm[c] + fa.momentum * mu);
            fa.rv[c] = float((1.0 - fa.momentum) * fa.rv[c] +
                             fa.momentum * var * double(M) / double(M > 1 ? M - 1 : 1));
          }
          if (fa.tracked && c == 0) fa.tracked[0] += 1;
        }
      }
      coef[pos(c)] = c0v;
      coef[C + pos(c)] = c1v;
    }
    __syncthreads();
    // the release's shard ticket now (every read of the accumulator is back), its answer at the end;
    // release 2: the whole release here (round 5's form, for A/Bs)
    if (fa.release == 2) {
      __shared__ int flag2;
      bn_acc_release(fa.acc, fa.R, C, &flag2);
    } else if (fa.release && threadIdx.x == 0) {
      rel_tk = bn_acc_ticket_take(fa.acc, fa.R, C, blockIdx.x);
    }
    const int gl = int(threadIdx.x) % G;   // this lane's channel group: channels V gl .. + V - 1
    float a0[V], a1[V];
#pragma unroll
    for (int h = 0; h < V / 4; ++h) {
      const float4 x0 = *reinterpret_cast<const float4*>(coef + 4 * h * G + 4 * gl);
      const float4 x1 = *reinterpret_cast<const float4*>(coef + C + 4 * h * G + 4 * gl);
      a0[4 * h] = x0.x, a0[4 * h + 1] = x0.y, a0[4 * h + 2] = x0.z, a0[4 * h + 3] = x0.w;
      a1[4 * h] = x1.x, a1[4 * h + 1] = x1.y, a1[4 * h + 2] = x1.z, a1[4 * h + 3] = x1.w;
    }
#pragma unroll
    for (int i = 0; i < V; ++i) {
      if constexpr (BWD) {
        bc[i].init(ml[i], il[i], wl[i], bl[i], a1[i], a0[i], invM);
      } else {
        is[i] = a1[i];
        nm[i] = -a0[i] * is[i];
        ww[i] = wl[i];
        bb[i] = bl[i];
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const int c = c0 + i;
      if constexpr (BWD) {
        bc[i].init(mean[c], invstd[c], w[c], b[c], dw[c], db[c], invM);
      } else {
        is[i] = invstd[c];
        nm[i] = -mean[c] * is[i];
        ww[i] = w[c];
        bb[i] = b[c];
      }
    }
  }
  auto apply = [&](const float (&v)[V], const float (&gv)[V], float (&o)[V]) {
    if constexpr (BWD) {
#pragma unroll
      for (int i = 0; i < V; ++i) o[i] = bc[i].gx(v[i], gv[i], slope);
    } else {
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const float z = fmaf(fmaf(v[i], is[i], nm[i]), ww[i], bb[i]);
        o[i] = z > 0.f ? z : z * slope;
      }
    }
  };
  while (have) {
    if constexpr (PF) {
      const int64_t nidx = idx + pass;
      const bool nhave = nidx + (U - 1) * kBlock < total;
      uint4 nv[U], ng[U];
      load_pass_b(nhave ? nidx : -1, nv, ng);   // in flight while this pass is applied
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float v[V], gv[V], o[V];
        bn_unpack<DT>(rv[u], v);
        if constexpr (BWD) bn_unpack<DT>(rg[u], gv);
        apply(v, gv, o);
        bn_store<DT>(out, (idx + u * kBlock) * V, o);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        rv[u] = nv[u];
        if constexpr (BWD) rg[u] = ng[u];
      }
      idx = nidx;
      have = nhave;
      continue;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float v[V], gv[V], o[V];
      bn_unpack<DT>(rv[u], v);
      if constexpr (BWD) bn_unpack<DT>(rg[u], gv);
      apply(v, gv, o);
      bn_store<DT>(out, (idx + u * kBlock) * V, o);
    }
    idx += pass;
    have = idx + (U - 1) * kBlock < total;
    if (have) load_pass();
  }
  for (; idx < total; idx += kBlock) {   // the tail: at most U - 1 vectors per lane
    float v[V], gv[V], o[V];
    bn_load<DT>(x, idx * V, v);
    if constexpr (BWD) bn_load<DT>(gy, idx * V, gv);
    apply(v, gv, o);
    bn_store<DT>(out, idx * V, o);
  }
  if constexpr (FOLD) {
    __shared__ int flag;
    if (fa.release == 1) bn_acc_ticket_finish(fa.acc, fa.R, C, &flag, rel_tk, blockIdx.x, gridDim.x);
  }
}

namespace {
bool bn_shape_ok(int64_t M, int C, int dtype) {
  if (M <= 0 || C <= 0 || (dtype != OUT_F32 && dtype != OUT_BF16)) return false;
  const int V = dtype == OUT_BF16 ? 8 : 4;
  return C % V == 0 && kBlock % (C / V) == 0;
}

void bn_blocks(int64_t M, int C, int dtype, int& nblocks, int64_t& rows_per_block) {
  const int V = dtype == OUT_BF16 ? 8 : 4;
  const int R = kBlock / (C / V);
  const int64_t want = (M + R - 1) / R;
  nblocks = int(want < kBnMaxBlocks ? want : kBnMaxBlocks);
  rows_per_block = (M + nblocks - 1) / nblocks;
}

int bn_grid(int64_t work, int unroll = kBnUnroll) {   // work = 16-byte vectors; `unroll` per lane per pass
  const int64_t blocks = (work + kBlock * unroll - 1) / (kBlock * unroll);
  return int(blocks < 4096 ? (blocks < 1 ? 1 : blocks) : 4096);
}

// apply launches that fold their accumulator: every block reads the 16 KB of
// replicas once, so fewer, longer-running blocks -- at most 512 (2 per CU),
// sized so every block runs the same number of passes (a cap of 1024 left
// 1.17 passes per block on the 1200-block second layer, i.e. 2 passes for
// some blocks and 1 for the rest).  Disc step: 18.8k -> 19.1-19.3k img/s,
// forward applies 42.2 -> 37.3 us (profiles/r4/b33/).  BT_BN_FOLD_GRID: the
// cap; BT_BN_FOLD_BALANCE=0: plain capping.
int bn_fold_cap() {
  static const int cap = [] {
    const char* e = std::getenv("BT_BN_FOLD_GRID");
    const int v = e ? std::atoi(e) : 512;
    return v > 0 ? v : 512;
  }();
  return cap;
}
// Vectors per lane and pass of the folding applies (BT_BN_UNROLL=8: twice the bytes in flight per
// lane).  4: 8 measured no faster alone (bn3 fwd 7.41 vs 7.47 us, bn2 fwd 10.51 vs 9.78, bn2 bwd
// 14.88 vs 13.06) and slower in the step (21.5-21.7k vs 21.9k img/s, profiles/r6/b7/): the applies'
// excess over the plain pass is the fold's latency (2.0-3.1 us a launch), not the bytes in flight.
int bn_fold_unroll(int64_t) {
  static const int u = [] {
    const char* e = std::getenv("BT_BN_UNROLL");
    return e && std::atoi(e) == 8 ? 8 : 4;
  }();
  return u;
}
// the folding applies' next-pass prefetch (bn_apply_kernel PF): BT_BN_PREFETCH=0 turns it off; only
// where the tensor's bytes fit a buffer resource's 32-bit range
int bn_prefetch(int64_t work) {
  static const bool on = !(std::getenv("BT_BN_PREFETCH") && std::getenv("BT_BN_PREFETCH")[0] == '0');
  return on && work * 16 < (int64_t(1) << 31);
}
int bn_fold_grid(int64_t work, int unroll = kBnUnroll) {
  const int cap = bn_fold_cap();
  static const bool balance = [] {
    const char* e = std::getenv("BT_BN_FOLD_BALANCE");
    return !(e && e[0] == '0');
  }();
  const int g = bn_grid(work, unroll);
  if (g <= cap) return g;
  if (!balance) return cap;
  const int passes = (g + cap - 1) / cap;
  return (g + passes - 1) / passes;
}
}  // namespace

int64_t bn_partial_floats(int64_t M, int C, int dtype) {
  if (!bn_shape_ok(M, C, dtype)) return -1;
  int nb;
  int64_t rpb;
  bn_blocks(M, C, dtype, nb, rpb);
  return int64_t(nb) * 2 * C;
}

hipError_t bn_stats(const void* x, int64_t M, int C, int dtype, float* partial, hipStream_t stream) {
  if (!bn_shape_ok(M, C, dtype)) return hipErrorInvalidValue;
  int nb;
  int64_t rpb;
  bn_blocks(M, C, dtype, nb, rpb);
  if (dtype == OUT_BF16)
    bn_reduce_kernel<OUT_BF16, false><<<nb, kBlock, 0, stream>>>(x, nullptr, M, C, rpb, nullptr, nullptr, nullptr,
                                                                 nullptr, 0.f, partial);
  else
    bn_reduce_kernel<OUT_F32, false><<<nb, kBlock, 0, stream>>>(x, nullptr, M, C, rpb, nullptr, nullptr, nullptr,
                                                                nullptr, 0.f, partial);
  return hipGetLastError();
}

hipError_t bn_finalize(const float* partial, int64_t M, int C, int dtype, float eps, float momentum, float* mean,
                       float* invstd, float* running_mean, float* running_var, hipStream_t stream,
                       int64_t* num_batches_tracked) {
  if (!bn_shape_ok(M, C, dtype)) return hipErrorInvalidValue;
  int nb;
  int64_t rpb;
  bn_blocks(M, C, dtype, nb, rpb);
  bn_finalize_kernel<<<(C + kFoldWaves - 1) / kFoldWaves, 64 * kFoldWaves, 0, stream>>>(partial, nb, M, C, eps, momentum, mean, invstd, running_mean,
                                                running_var, num_batches_tracked);
  return hipGetLastError();
}

hipError_t bn_finalize_rows(const float* partial, int nblocks, int64_t M, int C, float eps, float momentum,
                            float* mean, float* invstd, float* running_mean, float* running_var, hipStream_t stream,
                            int64_t* num_batches_tracked) {
  if (nblocks <= 0 || M <= 0 || C <= 0 || !partial || !mean || !invstd) return hipErrorInvalidValue;
  bn_finalize_kernel<<<(C + kFoldWaves - 1) / kFoldWaves, 64 * kFoldWaves, 0, stream>>>(partial, nblocks, M, C, eps, momentum, mean, invstd, running_mean,
                                                running_var, num_batches_tracked);
  return hipGetLastError();
}

hipError_t bn_apply(const void* x, void* y, int64_t M, int C, int dtype, const float* mean, const float* invstd,
                    const float* w, const float* b, float slope, hipStream_t stream) {
  if (!bn_shape_ok(M, C, dtype)) return hipErrorInvalidValue;
  const int V = dtype == OUT_BF16 ? 8 : 4;
  const int grid = bn_grid(M * (C / V));
  if (dtype == OUT_BF16)
    bn_apply_kernel<OUT_BF16, false><<<grid, kBlock, 0, stream>>>(x, nullptr, y, M, C, mean, invstd, w, b, nullptr,
                                                                  nullptr, slope);
  else
    bn_apply_kernel<OUT_F32, false><<<grid, kBlock, 0, stream>>>(x, nullptr, y, M, C, mean, invstd, w, b, nullptr,
                                                                 nullptr, slope);
  return hipGetLastError();
}

hipError_t bn_bwd_reduce(const void* x, const void* gy, int64_t M, int C, int dtype, const float* mean,
                         const float* invstd, const float* w, const float* b, float slope, float* partial,
                         hipStream_t stream) {
  if (!bn_shape_ok(M, C, dtype)) return hipErrorInvalidValue;
  int nb;
  int64_t rpb;
  bn_blocks(M, C, dtype, nb, rpb);
  if (dtype == OUT_BF16)
    bn_reduce_kernel<OUT_BF16, true><<<nb, kBlock, 0, stream>>>(x, gy, M, C, rpb, mean, invstd, w, b, slope, partial);
  else
    bn_reduce_kernel<OUT_F32, true><<<nb, kBlock, 0, stream>>>(x, gy, M, C, rpb, mean, invstd, w, b, slope, partial);
  return hipGetLastError();
}

hipError_t bn_bwd_finalize(const float* partial, int64_t M, int C, int dtype, float* dw, float* db,
                           hipStream_t stream) {
  if (!bn_shape_ok(M, C, dtype)) return hipErrorInvalidValue;
  int nb;
  int64_t rpb;
  bn_blocks(M, C, dtype, nb, rpb);
  bn_bwd_finalize_kernel<<<(C + kFoldWaves - 1) / kFoldWaves, 64 * kFoldWaves, 0, stream>>>(partial, nb, C, dw, db);
  return hipGetLastError();
}

hipError_t bn_bwd_finalize_rows(const float* partial, int rows, int C, float* dw, float* db, hipStream_t stream) {
  if (rows <= 0 || C <= 0 || !partial || !dw || !db) return hipErrorInvalidValue;
  bn_bwd_finalize_kernel<<<(C + kFoldWaves - 1) / kFoldWaves, 64 * kFoldWaves, 0, stream>>>(partial, rows, C, dw, db);
  return hipGetLastError();
}

int bn_acc_replicas(int C) {
  // 2 C R <= 2048 floats (8 KB) folded per apply block; up to 32 replicas
  // spread the producers' atomics (a tile of the 614k-pixel first layer is one
  // of ~4800 adders per channel)
  if (C <= 0 || C > kBnAccMaxC || C % 2) return 0;
  const int r = 1024 / C;
  return r > 32 ? 32 : r;   // 2 C R is a multiple of 4 and <= 2048
}

int64_t bn_acc_elems(int C) {
  // [R][2][C] replicas + the apply launches' ticket words, one 128-byte line
  // each (bn_fold.h: 8 shards + the top counter)
  const int r = bn_acc_replicas(C);
  return r > 0 ? int64_t(2) * C * r + (kBnTicketShards * kBnTicketStride + 1 + 1) / 2 : -1;
}

namespace {
// BT_BN_RELEASE=0: the accumulator apply kernels skip the release (tickets and
// clear) -- wrong for a second use of the accumulator; for the per-phase timing
// of scripts/bn_apply_bench.py only
int bn_release_env() {
  static const int v = [] {
    const char* e = std::getenv("BT_BN_RELEASE");
    return e && e[0] == '0' ? 0 : e && e[0] == '2' ? 2 : 1;
  }();
  return v;
}
}  // namespace

hipError_t bn_apply_acc(const void* x, void* y, int64_t M, int C, int dtype, BnAcc acc, float eps, float momentum,
                        float* mean, float* invstd, float* running_mean, float* running_var, int64_t* tracked,
                        const float* w, const float* b, float slope, hipStream_t stream) {
  if (!bn_shape_ok(M, C, dtype) || !acc.acc || acc.R != bn_acc_replicas(C) || !mean || !invstd || !w || !b)
    return hipErrorInvalidValue;
  // every apply block folds the accumulator itself (bn_fold.h): no finalize launch
  BnApplyFold fa;
  fa.acc = acc.acc, fa.R = acc.R, fa.eps = eps, fa.momentum = momentum;
  fa.o0 = mean, fa.o1 = invstd, fa.rm = running_mean, fa.rv = running_var, fa.tracked = tracked;
  fa.release = bn_release_env();
  const int V = dtype == OUT_BF16 ? 8 : 4;
  const int u = bn_fold_unroll(M * (C / V));
  const int grid = bn_fold_grid(M * (C / V), u);
  const bool pf = bn_prefetch(M * (C / V));
#define BT_BN_FWD(DT_, U_, PF_) \
  bn_apply_kernel<DT_, false, true, U_, PF_><<<grid, kBlock, 0, stream>>>(x, nullptr, y, M, C, nullptr, nullptr, w, b, \
                                                                          nullptr, nullptr, slope, fa)
  if (dtype == OUT_BF16 && u == 8) BT_BN_FWD(OUT_BF16, 8, false);
  else if (dtype == OUT_BF16 && pf) BT_BN_FWD(OUT_BF16, 4, true);
  else if (dtype == OUT_BF16) BT_BN_FWD(OUT_BF16, 4, false);
  else if (u == 8) BT_BN_FWD(OUT_F32, 8, false);
  else if (pf) BT_BN_FWD(OUT_F32, 4, true);
  else BT_BN_FWD(OUT_F32, 4, false);
#undef BT_BN_FWD
  return hipGetLastError();
}

hipError_t bn_bwd_apply_acc(const void* x, const void* gy, void* gx, int64_t M, int C, int dtype, BnAcc acc,
                            const float* mean, const float* invstd, const float* w, const float* b, float* dw,
                            float* db, float slope, hipStream_t stream) {
  if (!bn_shape_ok(M, C, dtype) || !acc.acc || acc.R != bn_acc_replicas(C) || !mean || !invstd || !w || !b || !dw ||
      !db)
    return hipErrorInvalidValue;
  BnApplyFold fa;
  fa.acc = acc.acc, fa.R = acc.R, fa.o0 = db, fa.o1 = dw;
  fa.release = bn_release_env();
  const int V = dtype == OUT_BF16 ? 8 : 4;
  const int u = bn_fold_unroll(M * (C / V));
  const int grid = bn_fold_grid(M * (C / V), u);
  const bool pf = bn_prefetch(M * (C / V));
#define BT_BN_BWD(DT_, U_, PF_) \
  bn_apply_kernel<DT_, true, true, U_, PF_><<<grid, kBlock, 0, stream>>>(x, gy, gx, M, C, mean, invstd, w, b, nullptr, \
                                                                         nullptr, slope, fa)
  if (dtype == OUT_BF16 && u == 8) BT_BN_BWD(OUT_BF16, 8, false);
  else if (dtype == OUT_BF16 && pf) BT_BN_BWD(OUT_BF16, 4, true);
  else if (dtype == OUT_BF16) BT_BN_BWD(OUT_BF16, 4, false);
  else if (u == 8) BT_BN_BWD(OUT_F32, 8, false);
  else if (pf) BT_BN_BWD(OUT_F32, 4, true);
  else BT_BN_BWD(OUT_F32, 4, false);
#undef BT_BN_BWD
  return hipGetLastError();
}

hipError_t bn_bwd_reduce_acc(const void* x, const void* gy, int64_t M, int C, int dtype, const float* mean,
                             const float* invstd, const float* w, const float* b, float slope, BnAcc acc,
                             hipStream_t stream) {
  if (!bn_shape_ok(M, C, dtype) || !acc.acc || acc.R != bn_acc_replicas(C)) return hipErrorInvalidValue;
  int nb;
  int64_t rpb;
  bn_blocks(M, C, dtype, nb, rpb);
  if (dtype == OUT_BF16)
    bn_reduce_kernel<OUT_BF16, true><<<nb, kBlock, 0, stream>>>(x, gy, M, C, rpb, mean, invstd, w, b, slope, reinterpret_cast<float*>(acc.acc),
                                                                acc.R);
  else
    bn_reduce_kernel<OUT_F32, true><<<nb, kBlock, 0, stream>>>(x, gy, M, C, rpb, mean, invstd, w, b, slope, reinterpret_cast<float*>(acc.acc),
                                                               acc.R);
  return hipGetLastError();
}

hipError_t bn_bwd_apply(const void* x, const void* gy, void* gx, int64_t M, int C, int dtype, const float* mean,
                        const float* invstd, const float* w, const float* b, const float* dw, const float* db,
                        float slope, hipStream_t stream) {
  if (!bn_shape_ok(M, C, dtype)) return hipErrorInvalidValue;
  const int V = dtype == OUT_BF16 ? 8 : 4;
  const int grid = bn_grid(M * (C / V));
  if (dtype == OUT_BF16)
    bn_apply_kernel<OUT_BF16, true><<<grid, kBlock, 0, stream>>>(x, gy, gx, M, C, mean, invstd, w, b, dw, db, slope);
  else
    bn_apply_kernel<OUT_F32, true><<<grid, kBlock, 0, stream>>>(x, gy, gx, M, C, mean, invstd, w, b, dw, db, slope);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// multi-tensor cast (fp32 <-> bf16)
// ---------------------------------------------------------------------------
namespace {

// blockIdx.y = tensor, blockIdx.x strides over its elements, 4 per lane
template <int MODE>
__global__ __launch_bounds__(kBlock) void multi_cast_kernel(CastParams p) {
  const int k = int(blockIdx.y);
  const int64_t n = p.numel[k];
  for (int64_t i = (int64_t(blockIdx.x) * kBlock + threadIdx.x) * 4; i < n; i += int64_t(gridDim.x) * kBlock * 4) {
    if constexpr (MODE == CAST_F32_TO_BF16) {
      const float* s = static_cast<const float*>(p.src[k]);
      uint16_t* d = static_cast<uint16_t*>(p.dst[k]);
      for (int j = 0; j < 4 && i + j < n; ++j) {
        const float f = s[i + j];
        d[i + j] = f != f ? uint16_t(0x7FC0) : f2bf(f);   // NaN stays a quiet NaN (as torch)
      }
    } else {
      const uint16_t* s = static_cast<const uint16_t*>(p.src[k]);
      float* d = static_cast<float*>(p.dst[k]);
      for (int j = 0; j < 4 && i + j < n; ++j) d[i + j] = __uint_as_float(uint32_t(s[i + j]) << 16);
    }
  }
}

}  // namespace

hipError_t multi_cast(const CastParams& p, hipStream_t stream) {
  if (p.n <= 0) return hipSuccess;
  if (p.n > kMaxCast) return hipErrorInvalidValue;
  int64_t most = 0;
  for (int k = 0; k < p.n; ++k) {
    if (p.numel[k] < 0 || (p.numel[k] > 0 && (!p.src[k] || !p.dst[k]))) return hipErrorInvalidValue;
    most = p.numel[k] > most ? p.numel[k] : most;
  }
  const int64_t blocks = (most + 4 * kBlock - 1) / (4 * kBlock);
  const dim3 grid(unsigned(blocks < 1024 ? (blocks > 0 ? blocks : 1) : 1024), unsigned(p.n));
  if (p.mode == CAST_F32_TO_BF16) multi_cast_kernel<CAST_F32_TO_BF16><<<grid, kBlock, 0, stream>>>(p);
  else if (p.mode == CAST_BF16_TO_F32) multi_cast_kernel<CAST_BF16_TO_F32><<<grid, kBlock, 0, stream>>>(p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Adam / AdamW
// ---------------------------------------------------------------------------
namespace {

// One lane: the step counter and the bias corrections, so that the update
// kernel's blocks all read a value no block is writing (adam_sched.h).

// the schedule of step counter + off, without advancing the counter: the
// one-launch update's coming step (off 1) after the counter, lr or gradient
// scale changed on the host side; or this step's (off 0) when the lr changed
// after an attached schedule already ran
__global__ void adam_schedule_prime_kernel(const float* step, const float* hp, float* sched, float beta1, float beta2,
                                           float off) {
  if (threadIdx.x == 0) adam_schedule_write(step[0] + off, hp, sched, beta1, beta2);
}

__global__ void adam_schedule_kernel(float* step, const float* hp, float* sched, float beta1, float beta2,
                                     const float* gate) {
  if (threadIdx.x != 0) return;
  AdamSchedJob j;
  j.step = step, j.hp = hp, j.sched = sched, j.beta1 = beta1, j.beta2 = beta2, j.gate = gate;
  adam_schedule_run(j);
}

// One tensor's slot of the launch, gathered into LDS by the block's first
// lanes (one parallel read of the kernel arguments): indexing the argument
// arrays with a lane's k read them from memory one dependent load at a time
// -- ~6 round trips before any parameter load could start.
struct AdamSlot {
  float* p;
  const void* g;
  const float* g2;
  float* m;
  float* v;
  uint16_t* shadow;
  uint16_t* shadow_t;
  int64_t numel;
  int tcin, tcout;
};

// one element's update (torch.optim.Adam, non-amsgrad): both paths below
__device__ __forceinline__ void adam_elem(const AdamParams& a, float step_size, float inv_bc2, float lr, float gscale,
                                          float gin, float& p, float& m, float& v) {
  const float b1 = a.beta1, b2 = a.beta2, wd = a.weight_decay;
  float g = (a.maximize ? -gin : gin) * gscale;
  if (wd != 0.f) {
    if (a.decoupled) p *= 1.f - lr * wd;
    else g += wd * p;
  }
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  p -= step_size * m / (sqrtf(v) * inv_bc2 + a.eps);
}

// AdamParams::fr: the block sums its share of the weight's slices (the ordered
// reduce's lanes and order, wgrad_reduce.h) and the group's lane 0 updates the
// weight's elements at the gradient's strides.  The lane's parameter, moment and
// shadow accesses are scattered 4-byte ones: ~3 K elements, a few hundred lanes.
template <int SG>
__device__ __forceinline__ void adam_fused_reduce(const AdamParams& a, int bx) {
  const AdamParams::FusedReduce& r = a.fr;
  const float step_size = a.sched[0], inv_bc2 = a.sched[1], lr = a.sched[2], gscale = a.sched[3];
  const bool active = a.sched[4] != 0.f;
  wgrad_slice_sum<kBlock, SG>(r, bx, [&](int e0, float4 acc) {
    const int Cin = r.Cin, KC = 16 * Cin;
    const float vals[4] = {acc.x, acc.y, acc.z, acc.w};
    int64_t off[4];
    bool ok[4];
    float pv[4], mv[4], vv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = e0 + j;
      const int co = e / KC, kc = e - co * KC;
      const int tap = kc / Cin, ci = kc - tap * Cin;
      ok[j] = ci < r.cin_out;
      off[j] = ok[j] ? co * r.s_co + ci * r.s_ci + (tap >> 2) * r.s_kh + (tap & 3) * r.s_kw : 0;
      pv[j] = r.p[off[j]], mv[j] = r.m[off[j]], vv[j] = r.v[off[j]];   // (off 0: a valid element, unused)
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!ok[j]) continue;
      r.g[off[j]] = a.zero_grad ? 0.f : vals[j];   // the gradient, as the reduce launch left it
      if (!active) continue;
      adam_elem(a, step_size, inv_bc2, lr, gscale, vals[j], pv[j], mv[j], vv[j]);
      r.p[off[j]] = pv[j], r.m[off[j]] = mv[j], r.v[off[j]] = vv[j];
      if (r.shadow) r.shadow[off[j]] = f2bf(pv[j]);
    }
  });
}

// FR: blocks [0, fr.rx) take the weight whose slice reduce this launch took (its
// own instantiation: the slice loads' registers would cost the plain update
// occupancy -- 92 VGPRs against 48)
// FSG: the fused slice sum's loads per round (8: the reduce launch's; 4: 58 VGPRs, two round trips)
template <bool GBF16, bool FR = false, int FSG = 8>
__global__ __launch_bounds__(kBlock) void adam_update_kernel(AdamParams a) {
  __shared__ AdamSlot slot[kMaxAdam];
  __shared__ int64_t gst[kMaxAdam + 1];
  const int nfr = FR ? a.fr.rx : 0;
  if constexpr (FR) {
    if (int(blockIdx.x) < nfr) {   // (block-uniform)
      adam_fused_reduce<FSG>(a, int(blockIdx.x));
      return;
    }
  }
  const int64_t bid = int64_t(blockIdx.x) - nfr;
  {
    const int t = int(threadIdx.x);
    if (t < a.n) {
      AdamSlot sl;
      sl.p = a.p[t], sl.g = a.g[t], sl.g2 = a.g2[t], sl.m = a.m[t], sl.v = a.v[t], sl.shadow = a.shadow[t];
      sl.shadow_t = a.shadow_t[t], sl.numel = a.numel[t], sl.tcin = a.tcin[t], sl.tcout = a.tcout[t];
      slot[t] = sl;
    }
    if (t <= a.n) gst[t] = a.gstart[t];
    __syncthreads();
  }
  const int64_t q = bid * kBlock + threadIdx.x;   // 4-element group
  const bool in = q < gst[a.n];
  int k = 0;
  if (in)
    while (q >= gst[k + 1]) ++k;          // <= kMaxAdam compares (LDS), mostly uniform across a wave
  const int64_t gi = in ? q - gst[k] : 0;
  // element offset of the group.  A tensor with a transposed shadow starts
  // on a block boundary and is walked in 32 x 32 (co, ci) tiles of one tap,
  // a block per tile: lane t = row t / 8 (co), 4 input channels 4 (t % 8) --
  // 128-byte runs in, and through an LDS transpose 64-byte runs of the
  // [ci][tap][co] shadow out.
  int64_t e0 = gi * 4;
  uint16_t* T = in ? slot[k].shadow_t : nullptr;   // block-uniform (host-checked tiling)
  int tco0 = 0, ttap = 0, tci0 = 0;
  if (T) {
    const int cin = slot[k].tcin, cit = cin >> 5;
    const int tile = int(gi >> 8), t = int(threadIdx.x);
    tci0 = (tile % cit) * 32;
    ttap = (tile / cit) & 15;
    tco0 = (tile / (cit * 16)) * 32;
    e0 = (int64_t(tco0 + (t >> 3)) * 16 + ttap) * cin + tci0 + 4 * (t & 7);
  }
  const int64_t n = in ? slot[k].numel : 0;
  const bool full = e0 + 4 <= n;   // tensors are 16-byte aligned (host-checked), so a full group is one dwordx4
  float* P = in ? slot[k].p : nullptr;
  float* M = in ? slot[k].m : nullptr;
  float* V = in ? slot[k].v : nullptr;
  const void* GR = in ? slot[k].g : nullptr;
  const float* G2 = in && !GBF16 ? slot[k].g2 : nullptr;
  float pv[4] = {0.f, 0.f, 0.f, 0.f}, gv[4] = {0.f, 0.f, 0.f, 0.f}, mv[4] = {0.f, 0.f, 0.f, 0.f},
        vv[4] = {0.f, 0.f, 0.f, 0.f};
  // every load is issued before the schedule below (its fp64 math and the
  // block barrier then overlap the memory latency)
  if (in && full) {
    const float4 p4 = *reinterpret_cast<const float4*>(P + e0);
    const float4 m4 = *reinterpret_cast<const float4*>(M + e0);
    const float4 v4 = *reinterpret_cast<const float4*>(V + e0);
    pv[0] = p4.x, pv[1] = p4.y, pv[2] = p4.z, pv[3] = p4.w;
    mv[0] = m4.x, mv[1] = m4.y, mv[2] = m4.z, mv[3] = m4.w;
    vv[0] = v4.x, vv[1] = v4.y, vv[2] = v4.z, vv[3] = v4.w;
    if constexpr (GBF16) {
      const uint2 g2 = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(GR) + e0);
      gv[0] = __uint_as_float(g2.x << 16), gv[1] = __uint_as_float(g2.x & 0xFFFF0000u);
      gv[2] = __uint_as_float(g2.y << 16), gv[3] = __uint_as_float(g2.y & 0xFFFF0000u);
    } else {
      const float4 g4 = *reinterpret_cast<const float4*>(static_cast<const float*>(GR) + e0);
      gv[0] = g4.x, gv[1] = g4.y, gv[2] = g4.z, gv[3] = g4.w;
      if (G2) {   // the second contribution: g1 + g2, autograd's accumulate order
        const float4 h4 = *reinterpret_cast<const float4*>(G2 + e0);
        gv[0] += h4.x, gv[1] += h4.y, gv[2] += h4.z, gv[3] += h4.w;
      }
    }
  } else if (in) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool ok = e0 + j < n;
      pv[j] = ok ? P[e0 + j] : 0.f;
      mv[j] = ok ? M[e0 + j] : 0.f;
      vv[j] = ok ? V[e0 + j] : 0.f;
      if constexpr (GBF16)
        gv[j] = ok ? __uint_as_float(uint32_t(static_cast<const uint16_t*>(GR)[e0 + j]) << 16) : 0.f;
      else
        gv[j] = ok ? static_cast<const float*>(GR)[e0 + j] + (G2 ? G2[e0 + j] : 0.f) : 0.f;
    }
  }
  float step_size, inv_bc2, lr, gscale;
  bool active;
  if (a.step) {
    // one-launch form: the schedule of THIS step was worked out ahead -- by
    // the previous launch's last block, or adam_schedule_prime -- so a block
    // only reads it (no lane computing fp64 powers behind a barrier); the gate
    // is read directly.  The block taking the last ticket advances the counter
    // and works out the next step's schedule (below).
    step_size = a.sched[0], inv_bc2 = a.sched[1], lr = a.sched[2], gscale = a.sched[3];
    active = !a.gate || a.gate[0] != 0.f;
  } else {
    step_size = a.sched[0], inv_bc2 = a.sched[1], lr = a.sched[2], gscale = a.sched[3];
    active = a.sched[4] != 0.f;
  }
  if (in) {
    if (!GBF16 && a.zero_grad) {   // consumed (also when a closed gate skips the update)
      float* G = static_cast<float*>(const_cast<void*>(GR));
      float* H = const_cast<float*>(G2);
      if (full) {
        *reinterpret_cast<float4*>(G + e0) = make_float4(0.f, 0.f, 0.f, 0.f);
        if (H) *reinterpret_cast<float4*>(H + e0) = make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        for (int j = 0; j < 4 && e0 + j < n; ++j) {
          G[e0 + j] = 0.f;
          if (H) H[e0 + j] = 0.f;
        }
      }
    }
    if (active) {
#pragma unroll
      for (int j = 0; j < 4; ++j) adam_elem(a, step_size, inv_bc2, lr, gscale, gv[j], pv[j], mv[j], vv[j]);
      uint16_t* S = slot[k].shadow;
      if (full) {
        *reinterpret_cast<float4*>(P + e0) = make_float4(pv[0], pv[1], pv[2], pv[3]);
        *reinterpret_cast<float4*>(M + e0) = make_float4(mv[0], mv[1], mv[2], mv[3]);
        *reinterpret_cast<float4*>(V + e0) = make_float4(vv[0], vv[1], vv[2], vv[3]);
        if (S) {
          uint2 s2;
          s2.x = uint32_t(f2bf(pv[0])) | (uint32_t(f2bf(pv[1])) << 16);
          s2.y = uint32_t(f2bf(pv[2])) | (uint32_t(f2bf(pv[3])) << 16);
          *reinterpret_cast<uint2*>(S + e0) = s2;
        }
      } else {
        for (int j = 0; j < 4 && e0 + j < n; ++j) {
          P[e0 + j] = pv[j], M[e0 + j] = mv[j], V[e0 + j] = vv[j];
          if (S) S[e0 + j] = f2bf(pv[j]);
        }
      }
      if (T) {   // (co, tap, ci) -> [ci][tap][co] through LDS (T, active: block-uniform)
        __shared__ uint16_t tl[32][34];
        const int t = int(threadIdx.x), cout = slot[k].tcout;
#pragma unroll
        for (int j = 0; j < 4; ++j) tl[4 * (t & 7) + j][t >> 3] = f2bf(pv[j]);
        __syncthreads();
        const int rr = t >> 3, cc = 4 * (t & 7);
        uint2 o;
        o.x = uint32_t(tl[rr][cc]) | (uint32_t(tl[rr][cc + 1]) << 16);
        o.y = uint32_t(tl[rr][cc + 2]) | (uint32_t(tl[rr][cc + 3]) << 16);
        *reinterpret_cast<uint2*>(T + (int64_t(tci0 + rr) * 16 + ttap) * cout + tco0 + cc) = o;
      }
    }
  }
  if (a.step && threadIdx.x == 0) {
    // every block has read this step's schedule (its update used it) before its ticket
    const uint32_t tk = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tk == gridDim.x - 1) {   // (no fused reduce blocks in the one-launch form: host-checked)
      if (active) {
        const float s = a.step[0] + 1.f;
        a.step[0] = s;
        adam_schedule_write(s + 1.f, a.hp, const_cast<float*>(a.sched), a.beta1, a.beta2);
      }
      __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace

hipError_t adam_schedule_prime(const float* step, const float* hp, float* sched, float beta1, float beta2,
                               hipStream_t stream, float off) {
  if (!step || !hp || !sched) return hipErrorInvalidValue;
  adam_schedule_prime_kernel<<<1, 64, 0, stream>>>(step, hp, sched, beta1, beta2, off);
  return hipGetLastError();
}

hipError_t adam_schedule(float* step, const float* hp, float* sched, float beta1, float beta2, hipStream_t stream,
                         const float* gate) {
  if (!step || !hp || !sched) return hipErrorInvalidValue;
  adam_schedule_kernel<<<1, 64, 0, stream>>>(step, hp, sched, beta1, beta2, gate);
  return hipGetLastError();
}

namespace {
int adam_fr_sg() {   // BT_ADAM_FR_SG: 4 or 8 (default) slice loads per round in the fused reduce
  static const int v = [] {
    const char* e = std::getenv("BT_ADAM_FR_SG");
    return e && std::atoi(e) == 4 ? 4 : 8;
  }();
  return v;
}
}  // namespace

hipError_t adam_update(const AdamParams& p, hipStream_t stream) {
  if (p.n <= 0 && !p.fr.partial) return hipSuccess;
  if (p.n > kMaxAdam || (!p.sched && !p.step)) return hipErrorInvalidValue;
  if (p.step && (!p.hp || !p.ticket)) return hipErrorInvalidValue;
  if (p.zero_grad && p.grad_bf16) return hipErrorInvalidValue;
  if (p.gstart[0] != 0) return hipErrorInvalidValue;
  for (int k = 0; k < p.n; ++k) {
    // a tensor's group range may be padded (blocks never straddle tensors)
    if (p.numel[k] < 0 || p.gstart[k + 1] - p.gstart[k] < (p.numel[k] + 3) / 4) return hipErrorInvalidValue;
    if (p.numel[k] > 0 && (!p.p[k] || !p.g[k] || !p.m[k] || !p.v[k])) return hipErrorInvalidValue;
    // full groups are read and written as 16-byte (8-byte for bf16) vectors
    const uintptr_t mis = reinterpret_cast<uintptr_t>(p.p[k]) | reinterpret_cast<uintptr_t>(p.m[k]) |
                          reinterpret_cast<uintptr_t>(p.v[k]) |
                          (reinterpret_cast<uintptr_t>(p.g[k]) << (p.grad_bf16 ? 1 : 0)) |
                          (reinterpret_cast<uintptr_t>(p.shadow[k]) << 1);
    if (mis & 15) return hipErrorInvalidValue;
    // transposed shadows: whole 32 x 32 tiles, one block each
    if (p.shadow_t[k] && (p.tcout[k] <= 0 || p.tcin[k] <= 0 || p.tcout[k] % 32 || p.tcin[k] % 32 ||
                          int64_t(p.tcout[k]) * 16 * p.tcin[k] != p.numel[k] || p.gstart[k] % kBlock ||
                          p.gstart[k + 1] - p.gstart[k] != p.numel[k] / 4))
      return hipErrorInvalidValue;
  }
  int64_t nfr = 0;
  if (p.fr.partial) {
    const AdamParams::FusedReduce& r = p.fr;
    const int64_t total = int64_t(r.Cout) * 16 * r.Cin;
    if (p.step || p.grad_bf16 || r.S <= 0 || r.Cout <= 0 || r.Cin <= 0 || r.cin_out <= 0 || r.cin_out > r.Cin ||
        r.sub <= 0 || r.sub > 64 || (r.sub & (r.sub - 1)) || total % 4 || total >= (int64_t(1) << 31) ||
        int64_t(r.rx) * kBlock < total / 4 * r.sub || r.rx > 65536 || !r.g || !r.p || !r.m || !r.v)
      return hipErrorInvalidValue;
    nfr = r.rx;
  }
  const int64_t groups = p.gstart[p.n];
  if (groups == 0 && nfr == 0) return hipSuccess;
  const int64_t blocks = (groups + kBlock - 1) / kBlock + nfr;
  if (blocks > int64_t(1) << 30) return hipErrorInvalidValue;
  if (p.grad_bf16) adam_update_kernel<true><<<unsigned(blocks), kBlock, 0, stream>>>(p);
  else if (nfr && adam_fr_sg() == 4) adam_update_kernel<false, true, 4><<<unsigned(blocks), kBlock, 0, stream>>>(p);
  else if (nfr) adam_update_kernel<false, true><<<unsigned(blocks), kBlock, 0, stream>>>(p);
  else adam_update_kernel<false><<<unsigned(blocks), kBlock, 0, stream>>>(p);
  return hipGetLastError();
}

}  // namespace gpu
}  // namespace btn
