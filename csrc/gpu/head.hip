// The discriminator's head as three small kernels instead of ~20 library
// launches: AdaptiveAvgPool2d(OH x OW) -> Conv2d(C, 1, (OH, OW)) -> sigmoid ->
// binary cross-entropy (mean over the batch), forward and backward.
//
// With the pooled map exactly consumed by the last convolution, each image's
// logit is a dot product of its feature map with the pooling-folded weight:
//   logit_n = sum_{i,j,c} pooled[n][i][j][c] * w[c][i][j]
//   dL/dz[n][h][w][c] = dlogit_n * sum_{(i,j) whose window holds (h,w)} w[c][i][j] / |window(i,j)|
//   dL/dw[c][i][j] = sum_n dlogit_n * pooled[n][i][j][c],  dlogit_n = g * (sigmoid(logit_n) - y_n) / N
// (PyTorch's BCE backward reduces to the same (p - y) / N once p(1-p) > 1e-12.)
// Pooling, the dot products and the loss run in fp32 on bf16 features; the
// weight and its gradient stay fp32 (no cast).  Reference head:
// examples/densityopt/densityopt.py:139-190 (conv4x4 -> sigmoid, BCELoss).
#include <hip/hip_runtime.h>

#include <hip/amd_detail/amd_hip_unsafe_atomics.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "bn_fold.h"
#include "kernels.h"

namespace btn {
namespace gpu {
namespace {

constexpr int kHeadThreads = 256;
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__host__ __device__ __forceinline__ int wstart(int i, int in, int out) { return (i * in) / out; }
__host__ __device__ __forceinline__ int wend(int i, int in, int out) { return ((i + 1) * in + out - 1) / out; }
__device__ __forceinline__ float bf(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }

constexpr int kHeadParts = 4;   // per-wave partial logits per cell (head_fwd_act_kernel: 256 threads)
static_assert(kHeadThreads / 64 == kHeadParts, "one partial per wave");
__device__ void head_loss_wave(const HeadParams& p, bool write_through, int parts);

// one block per (pooling cell, image): pooled values of the cell and the
// cell's share of the image's logit.  Lanes own 8 channels (one 16-byte load)
// of a pixel; the PL = 256 / (C / 8) pixel lanes of a channel group stride the
// window and meet in LDS.  (One lane per channel walking the window serially
// was a chain of dependent 2-byte loads: 22 us for the bench's 8x30x40x256.)
__global__ __launch_bounds__(kHeadThreads) void head_fwd_kernel(HeadParams p) {
  __shared__ float red[kHeadThreads / 64];
  __shared__ float acc_l[kHeadThreads * 8];
  const int cell = int(blockIdx.x), n = int(blockIdx.y);
  const int i = cell / p.OW, j = cell - i * p.OW;
  const int h0 = wstart(i, p.H, p.OH), h1 = wend(i, p.H, p.OH);
  const int w0 = wstart(j, p.W, p.OW), w1 = wend(j, p.W, p.OW);
  const int ww = w1 - w0, npx = (h1 - h0) * ww;
  const float inv = 1.f / float(npx);
  const int t = int(threadIdx.x);
  float part = 0.f;
  const int G = p.C / 8;
  if (p.C % 8 == 0 && G <= kHeadThreads && kHeadThreads % G == 0 && (reinterpret_cast<uintptr_t>(p.z) & 15) == 0) {
    const int g = t % G, pl = t / G, PL = kHeadThreads / G;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // act.on(): fold the BN statistics (every block; block (0, 0) writes the
    // outputs, the last block clears the accumulator) into this lane's 8
    // channels' xhat = v is + nm, z = xhat w + b
    const bool act = p.act.on();
    float is[8], nm[8], aw[8], ab[8];
    if (act) {
      __shared__ double fold[2 * kBnFoldMaxC];
      __shared__ float coef[2 * kBnFoldMaxC];
      __shared__ int flag;
      bn_acc_column_sums(p.act.acc, p.act.R, 2 * p.C, fold);
      BnFwdFinal f;
      f.eps = p.act.eps, f.momentum = p.act.momentum, f.mean = p.act.mean, f.invstd = p.act.invstd;
      f.rm = p.act.rm, f.rv = p.act.rv, f.tracked = p.act.tracked;
      const bool first = blockIdx.x == 0 && blockIdx.y == 0;
      for (int c = t; c < p.C; c += kHeadThreads) bn_fwd_finalize(f, fold, p.C, p.act.M, c, first, coef[c], coef[p.C + c]);
      __syncthreads();
      bn_acc_release(p.act.acc, p.act.R, p.C, &flag, blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        is[q] = coef[p.C + g * 8 + q];
        nm[q] = -coef[g * 8 + q] * is[q];
        aw[q] = p.act.w[g * 8 + q];
        ab[q] = p.act.b[g * 8 + q];
      }
    }
    // leaky(bn(v)) of channels q, q + 1 rounded to bf16 (RNE, v_cvt_pk_bf16_f32) -- the
    // values the apply kernel would have stored -- added into a[q], a[q + 1]
    auto act_add = [&](uint32_t word, int q) {
      const float z0 = fmaf(fmaf(__uint_as_float(word << 16), is[q], nm[q]), aw[q], ab[q]);
      const float z1 = fmaf(fmaf(__uint_as_float(word & 0xFFFF0000u), is[q + 1], nm[q + 1]), aw[q + 1], ab[q + 1]);
      const f32x2 pr = {z0 > 0.f ? z0 : z0 * p.act.slope, z1 > 0.f ? z1 : z1 * p.act.slope};
      const uint32_t r = __builtin_bit_cast(uint32_t, __builtin_convertvector(pr, bf16x2));
      a[q] += __uint_as_float(r << 16);
      a[q + 1] += __uint_as_float(r & 0xFFFF0000u);
    };
    // 4 window pixels per lane per pass, every load issued before any add: the
    // one-pixel loop waited out a load latency per pixel (~10 per lane)
    constexpr int UN = 4;
    for (int k0 = pl; k0 < npx; k0 += UN * PL) {
      uint4 v[UN];
#pragma unroll
      for (int u = 0; u < UN; ++u) {
        const int k = k0 + u * PL;
        const int kk = k < npx ? k : k0;   // past the window: re-read the first pixel, added as 0 below
        const int h = h0 + kk / ww, w = w0 + kk % ww;
        v[u] = *reinterpret_cast<const uint4*>(p.z + (int64_t(n * p.H + h) * p.W + w) * p.C + g * 8);
      }
#pragma unroll
      for (int u = 0; u < UN; ++u) {
        if (k0 + u * PL >= npx) break;
        const uint32_t uu[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
        if (act) {
#pragma unroll
          for (int q = 0; q < 4; ++q) act_add(uu[q], 2 * q);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            a[2 * q] += __uint_as_float(uu[q] << 16);
            a[2 * q + 1] += __uint_as_float(uu[q] & 0xFFFF0000u);
          }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) acc_l[pl * p.C + g * 8 + q] = a[q];
    __syncthreads();
    for (int c = t; c < p.C; c += kHeadThreads) {
      float s = 0.f;
      for (int l = 0; l < PL; ++l) s += acc_l[l * p.C + c];
      const float pooled = s * inv;
      p.pooled[(int64_t(n) * p.OH * p.OW + cell) * p.C + c] = pooled;
      part += pooled * p.w[c * p.ws_c + i * p.ws_i + j * p.ws_j];
    }
  } else {
    for (int c = t; c < p.C; c += kHeadThreads) {
      float s = 0.f;
      for (int h = h0; h < h1; ++h) {
        const uint16_t* row = p.z + (int64_t(n * p.H + h) * p.W) * p.C + c;
        for (int w = w0; w < w1; ++w) s += bf(row[int64_t(w) * p.C]);
      }
      const float pooled = s * inv;
      p.pooled[(int64_t(n) * p.OH * p.OW + cell) * p.C + c] = pooled;
      part += pooled * p.w[c * p.ws_c + i * p.ws_i + j * p.ws_j];
    }
  }
  for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = part;
  __syncthreads();
  if (!p.ticket) {
    if (threadIdx.x == 0) {
      float v = 0.f;
      for (int k = 0; k < kHeadThreads / 64; ++k) v += red[k];
      p.partial[n * p.OH * p.OW + cell] = v;
    }
    return;
  }
  // one-launch form: lane 0 publishes the block's partial write-through,
  // waits for it, then takes a ticket; the block that takes the last ticket
  // computes the loss in its first wave, reading the partials write-through
  // (agent-scope relaxed atomics: sc1 stores and loads -- no fences)
  if (threadIdx.x >= 64) return;
  uint32_t last = 0;
  if (threadIdx.x == 0) {
    float v = 0.f;
    for (int k = 0; k < kHeadThreads / 64; ++k) v += red[k];
    __hip_atomic_store(p.partial + n * p.OH * p.OW + cell, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t tk = __hip_atomic_fetch_add(p.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = tk == gridDim.x * gridDim.y - 1;
    if (last) __hip_atomic_store(p.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (!__shfl(last, 0)) return;
  head_loss_wave(p, true, 1);
}

// The same forward with the BatchNorm applied (act.on()) and the loss ticket,
// laid out as few memory round trips as possible -- one block per (cell,
// image), so the kernel is ONE wave of ~128 blocks and its time is a block's
// latency chain, not bandwidth (round 4: 14.7 us for 4.9 MB).  head_fwd_kernel
// ran ~8 dependent round trips: the accumulator fold one column at a time,
// the release ticket, the window in passes of 4 pixels, the partial store, the
// loss ticket, the release's second counter.  Here:
//  1. every window pixel of the lane is loaded up front (KMAX 16-byte loads);
//  2. the accumulator's [R][2C] replicas are read as one flat array, 8 doubles
//     per thread, all in flight with the pixels; LDS folds the replicas;
//  3. the release's shard ticket goes out as soon as those reads are back,
//     its answer is only needed at the end;
//  4. the partial logit's store and the loss ticket (and, for the last block
//     of a shard, the release's top counter) are one more round trip.
// Same arithmetic per element as head_fwd_kernel (bit-identical pooled values
// and partials: the per-channel sums run in the same lane / pixel order).
constexpr int kHeadFlat = 8;   // accumulator doubles per thread: 2 C R = 2048 (bn_acc_replicas) over 256 threads

// BNB: also the BN's backward sums, factored through dlogit (HeadParams::bn_ab)
template <int KMAX, bool BNB = false>
__global__ __launch_bounds__(kHeadThreads) void head_fwd_act_kernel(HeadParams p) {
  // (BNB) per lane group: sums of s and s * xhat over the lane's window pixels, [pl][g][9]
  __shared__ float sa_l[BNB ? kHeadThreads * 9 : 1], sb_l[BNB ? kHeadThreads * 9 : 1];
  // per-lane-group channel sums, [pl][g][9]: 9 words per channel group (8 +
  // one of padding) so the 32 lanes of a row write 32 distinct banks (at 8 a
  // row's 8 stores each ran 8-way conflicted)
  __shared__ float acc_l[kHeadThreads * 9];
  __shared__ double fold[kHeadThreads * kHeadFlat];   // the [R][2C] replicas, then the column sums
  __shared__ __attribute__((aligned(16))) float coef[2 * kBnFoldMaxC];
  __shared__ int flags[2];
  const int cell = int(blockIdx.x), n = int(blockIdx.y);
  const int i = cell / p.OW, j = cell - i * p.OW;
  const int h0 = wstart(i, p.H, p.OH), h1 = wend(i, p.H, p.OH);
  const int w0 = wstart(j, p.W, p.OW), w1 = wend(j, p.W, p.OW);
  const int ww = w1 - w0, npx = (h1 - h0) * ww;
  const float inv = 1.f / float(npx);
  const int t = int(threadIdx.x);
  const int G = p.C / 8, g = t % G, pl = t / G, PL = kHeadThreads / G;
  // 1. the lane's window pixels (k = pl + PL u), all loads in flight
  uint4 v[KMAX];
#pragma unroll
  for (int u = 0; u < KMAX; ++u) {
    const int k = pl + u * PL;
    // past the window: a re-read of its first pixel, added as 0 below (not pixel
    // pl: with fewer window pixels than lanes per pixel group -- a 6 x 8 input
    // pooled to 4 x 4 has 4 -- that lands rows below the window, past the last
    // image's end)
    const int kk = k < npx ? k : 0;
    const int h = h0 + kk / ww, w = w0 + kk % ww;
    v[u] = *reinterpret_cast<const uint4*>(p.z + (int64_t(n * p.H + h) * p.W + w) * p.C + g * 8);
  }
  // 2. the accumulator, flat: element e = t + 256 q of [R][2C]
  const int J = 2 * p.C, RJ = p.act.R * J;
  double a8[kHeadFlat];
#pragma unroll
  for (int q = 0; q < kHeadFlat; ++q) {
    const int e = t + kHeadThreads * q;
    a8[q] = e < RJ ? p.act.acc[e] : 0.0;
  }
#pragma unroll
  for (int q = 0; q < kHeadFlat; ++q) fold[t + kHeadThreads * q] = a8[q];
  __syncthreads();
  // 3. every read of the accumulator is back: the release's shard ticket (answer used at the end)
  const unsigned nblk = gridDim.x * gridDim.y, blk = blockIdx.y * gridDim.x + blockIdx.x;
  unsigned* ticket = bn_acc_ticket(p.act.acc, p.act.R, p.C);
  const unsigned shard = blk % kBnTicketShards;
  unsigned shard_old = 0;
  if (t == 0) shard_old = atomicAdd(ticket + shard * kBnTicketStride, 1u);
  // column sums in bn_acc_column_sums' order (groups g of replicas g, g + GR, ..., then the groups in
  // order: the same fp64 values, so the same mean / invstd as the other fold sites)
  {
    const int GR = J >= kHeadThreads ? 1 : kHeadThreads / J;
    for (int c = t; c < J; c += kHeadThreads) {
      double s = 0.0;
      for (int gg = 0; gg < GR; ++gg) {
        double sg = 0.0;
        for (int r = gg; r < p.act.R; r += GR) sg += fold[r * J + c];
        s = gg == 0 ? sg : s + sg;
      }
      fold[c] = s;   // row 0 of the replicas, column c: read only by this thread (above)
    }
  }
  __syncthreads();
  BnFwdFinal f;
  f.eps = p.act.eps, f.momentum = p.act.momentum, f.mean = p.act.mean, f.invstd = p.act.invstd;
  f.rm = p.act.rm, f.rv = p.act.rv, f.tracked = p.act.tracked;
  const bool first = blockIdx.x == 0 && blockIdx.y == 0;
  // mean / invstd in a lane-major order (channel 8 g + k at 4 g + k, k < 4, or
  // 4 G + 4 g + k - 4): a lane's 8 channels are two conflict-free 16-byte reads
  for (int c = t; c < p.C; c += kHeadThreads) {
    const int gg = c >> 3, k = c & 7, pc = k < 4 ? 4 * gg + k : 4 * G + 4 * gg + k - 4;
    bn_fwd_finalize(f, fold, p.C, p.act.M, c, first, coef[pc], coef[p.C + pc]);
  }
  __syncthreads();
  float is[8], nm[8], aw[8], ab[8];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const float4 mu = *reinterpret_cast<const float4*>(coef + 4 * hh * G + 4 * g);
    const float4 iv = *reinterpret_cast<const float4*>(coef + p.C + 4 * hh * G + 4 * g);
    const float m4[4] = {mu.x, mu.y, mu.z, mu.w}, i4[4] = {iv.x, iv.y, iv.z, iv.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int q = 4 * hh + k;
      is[q] = i4[k];
      nm[q] = -m4[k] * is[q];
      aw[q] = p.act.w[g * 8 + q];
      ab[q] = p.act.b[g * 8 + q];
    }
  }
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float sa[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, sb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < KMAX; ++u) {
    if (pl + u * PL >= npx) break;
    const uint32_t uu[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float xh0 = fmaf(__uint_as_float(uu[q] << 16), is[2 * q], nm[2 * q]);
      const float xh1 = fmaf(__uint_as_float(uu[q] & 0xFFFF0000u), is[2 * q + 1], nm[2 * q + 1]);
      const float z0 = fmaf(xh0, aw[2 * q], ab[2 * q]);
      const float z1 = fmaf(xh1, aw[2 * q + 1], ab[2 * q + 1]);
      const f32x2 pr = {z0 > 0.f ? z0 : z0 * p.act.slope, z1 > 0.f ? z1 : z1 * p.act.slope};
      const uint32_t r = __builtin_bit_cast(uint32_t, __builtin_convertvector(pr, bf16x2));
      a[2 * q] += __uint_as_float(r << 16);
      a[2 * q + 1] += __uint_as_float(r & 0xFFFF0000u);
      if constexpr (BNB) {   // the LeakyReLU's derivative s at the pixel, and s * xhat
        const float s0 = z0 > 0.f ? 1.f : p.act.slope, s1 = z1 > 0.f ? 1.f : p.act.slope;
        sa[2 * q] += s0, sa[2 * q + 1] += s1;
        sb[2 * q] += s0 * xh0, sb[2 * q + 1] += s1 * xh1;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) acc_l[pl * 9 * G + g * 9 + q] = a[q];
  if constexpr (BNB) {
#pragma unroll
    for (int q = 0; q < 8; ++q) sa_l[pl * 9 * G + g * 9 + q] = sa[q], sb_l[pl * 9 * G + g * 9 + q] = sb[q];
  }
  __syncthreads();
  float part = 0.f;
  for (int c = t; c < p.C; c += kHeadThreads) {
    float s = 0.f;
    for (int l = 0; l < PL; ++l) s += acc_l[l * 9 * G + (c >> 3) * 9 + (c & 7)];
    const float pooled = s * inv;
    p.pooled[(int64_t(n) * p.OH * p.OW + cell) * p.C + c] = pooled;
    const float wc = p.w[c * p.ws_c + i * p.ws_i + j * p.ws_j];
    part += pooled * wc;
    if constexpr (BNB) {   // this window's share of A[n][c], B[n][c]: w[c][i][j] / |window| times the pixel sums
      float s0 = 0.f, s1 = 0.f;
      for (int l = 0; l < PL; ++l) s0 += sa_l[l * 9 * G + (c >> 3) * 9 + (c & 7)], s1 += sb_l[l * 9 * G + (c >> 3) * 9 + (c & 7)];
      const float m = wc * inv;
      // (fp64 atomics: the ~16 window adds of an (n, c) arrive in any order; the sum is not order-exact in
      // general, but its rounding error is ~1e-16 relative -- far below the fp32 the backward reads it as)
      __hip_atomic_fetch_add(p.bn_ab + int64_t(n) * p.C + c, double(s0 * m), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(p.bn_ab + (int64_t(p.N) + n) * p.C + c, double(s1 * m), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
  // 4. each wave's partial logit (write-through, slot 4 cell + wave: head_loss_wave adds a cell's 4
  // in wave order, the block sum it had before), then one wait for it together with the block's
  // BN adds (BNB) and the shard ticket -- one round trip where the block-summed partial's store
  // took a second -- then the loss ticket and, for the shard's last block, the release's top counter
  if ((t & 63) == 0)
    __hip_atomic_store(p.partial + (n * p.OH * p.OW + cell) * kHeadParts + (t >> 6), part, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    const unsigned in_shard = (nblk - shard + kBnTicketShards - 1) / kBnTicketShards;
    const unsigned shards = nblk < unsigned(kBnTicketShards) ? nblk : unsigned(kBnTicketShards);
    const bool shard_last = shard_old == in_shard - 1;
    const uint32_t tk = __hip_atomic_fetch_add(p.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned top_old = 0;
    if (shard_last) {
      ticket[shard * kBnTicketStride] = 0u;   // every block of this shard has taken its ticket
      top_old = atomicAdd(ticket + kBnTicketShards * kBnTicketStride, 1u);
    }
    const bool loss_last = tk == nblk - 1;
    if (loss_last) __hip_atomic_store(p.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flags[0] = shard_last && top_old == shards - 1;
    flags[1] = loss_last;
  }
  __syncthreads();
  if (flags[0]) {   // every block has read the accumulator: clear it for the next producer
    for (int e = t; e < RJ; e += kHeadThreads) p.act.acc[e] = 0.0;
    if (t == 0) ticket[kBnTicketShards * kBnTicketStride] = 0u;
  }
  if (flags[1] && t < 64) head_loss_wave(p, true, kHeadParts);
  if constexpr (BNB) {
    if (!flags[1]) return;
    // the last block: every block's A / B adds are done (they preceded its ticket),
    // dlogit is written by this block's first wave
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int NC = p.N * p.C;
    const __amdgpu_buffer_rsrc_t rdl = __builtin_amdgcn_make_buffer_rsrc(p.dlogit, 0, p.N * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rab = __builtin_amdgcn_make_buffer_rsrc(p.bn_ab, 0, 2 * NC * 8, 0x00020000);
    for (int c = t; c < p.C; c += kHeadThreads) {
      float s0 = 0.f, s1 = 0.f;
      // 8 images' values in flight at a time (write-through reads: sc1 buffer loads, what an agent-
      // scope relaxed atomic load compiles to -- as atomic loads the compiler waited out one image at
      // a time: 8 round trips in series in the launch's last block), summed in image order
      for (int n0 = 0; n0 < p.N; n0 += 8) {
        float dl[8];
        double av[8], bv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int n = n0 + u < p.N ? n0 + u : 0;
          dl[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rdl, n * 4, 0, 16));
          av[u] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rab, (n * p.C + c) * 8, 0, 16));
          bv[u] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rab, (NC + n * p.C + c) * 8, 0, 16));
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (n0 + u < p.N) {
            s0 += dl[u] * float(av[u]);
            s1 += dl[u] * float(bv[u]);
          }
      }
      p.bn_sums[c] = s0;
      p.bn_sums[p.C + c] = s1;
      for (int n = 0; n < p.N; ++n) p.bn_ab[n * p.C + c] = 0.0, p.bn_ab[NC + n * p.C + c] = 0.0;   // for the next step
    }
  }
}

// one wave: logits, sigmoid, mean BCE, and dlogit/g for the backward.  parts: partials per cell
// (head_fwd_act_kernel: kHeadParts per-wave ones, added in wave order; else 1)
__device__ void head_loss_wave(const HeadParams& p, bool wt, int parts) {
  const int cells = p.OH * p.OW;
  float total = 0.f;
  if (parts == kHeadParts) {   // 16-byte loads of a cell's 4 partials, 16 cells at a time (write-through)
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(p.partial, 0, p.N * cells * kHeadParts * 4, 0x00020000);
    for (int n = int(threadIdx.x); n < p.N; n += 64) {
      float logit = 0.f;
      const float y = p.target ? p.target[n] : p.target_value;   // (in flight with the partials)
      for (int k0 = 0; k0 < cells; k0 += 16) {
        float4 v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int k = k0 + u < cells ? k0 + u : k0;
          v[u] = __builtin_bit_cast(float4, wt ? __builtin_amdgcn_raw_buffer_load_b128(rs, (n * cells + k) * 16, 0, 16)
                                               : __builtin_amdgcn_raw_buffer_load_b128(rs, (n * cells + k) * 16, 0, 0));
        }
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (k0 + u < cells) logit += ((v[u].x + v[u].y) + v[u].z) + v[u].w;
      }
      const float pr = 1.f / (1.f + expf(-logit));
      const float lp = fmaxf(logf(pr), -100.f), lq = fmaxf(logf(1.f - pr), -100.f);
      total += -(y * lp + (1.f - y) * lq);
      p.dlogit[n] = (pr - y) / float(p.N);
      if (p.logit) p.logit[n] = logit;
    }
    for (int o = 32; o > 0; o >>= 1) total += __shfl_xor(total, o);
    if (threadIdx.x == 0) p.loss[0] = total / float(p.N);
    return;
  }
  for (int n = int(threadIdx.x); n < p.N; n += 64) {
    float logit = 0.f;
    // 16 partials at a time, every load issued before the adds (summed in cell
    // order): one cell per round trip made this wave -- the kernel's tail -- a
    // chain of `cells` write-through loads
    // (write-through reads: sc1 buffer loads -- what an agent-scope relaxed
    // atomic load compiles to, but ordinary loads the compiler keeps in flight
    // together; atomic loads it waited out one at a time)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p.partial, 0, p.N * cells * 4, 0x00020000);
    for (int k0 = 0; k0 < cells; k0 += 16) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int k = k0 + u < cells ? k0 + u : k0;
        v[u] = wt ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (n * cells + k) * 4, 0, 16))
                  : p.partial[n * cells + k];
      }
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (k0 + u < cells) logit += v[u];
    }
    const float y = p.target ? p.target[n] : p.target_value;
    const float pr = 1.f / (1.f + expf(-logit));
    const float lp = fmaxf(logf(pr), -100.f), lq = fmaxf(logf(1.f - pr), -100.f);
    total += -(y * lp + (1.f - y) * lq);
    p.dlogit[n] = (pr - y) / float(p.N);
    if (p.logit) p.logit[n] = logit;
  }
  for (int o = 32; o > 0; o >>= 1) total += __shfl_xor(total, o);
  if (threadIdx.x == 0) p.loss[0] = total / float(p.N);
}

__global__ __launch_bounds__(64) void head_loss_kernel(HeadParams p) { head_loss_wave(p, false, 1); }

// Backward in ONE launch: blocks [0, nbwd) write dz, blocks [nbwd, ...) the
// weight gradient.  dz[n][h][w][c] = g dlogit_n * M[h][w][c], where M (the
// pooling-folded head weight seen by pixel (h, w): the sum of w[c][i][j] /
// |window(i, j)| over the windows holding it) does not depend on the image:
// a dz block takes PXB consecutive pixels of one row (PXB = 256 / (C / 8)
// lanes of 8 channels each), works out its lanes' M once and walks the N
// images with all their loads in flight (one pixel per lane per image was
// the old form: window search, divisions and weight gathers per element,
// 17.5 us for 8x30x40x256 at 0.56 TB/s).
// With p.bn_acc the dz blocks also sum the producing BatchNorm+LeakyReLU
// backward's gz and gz * xhat per channel; the block folds its lanes through
// LDS and adds its 2 C sums into replica blockIdx % R of the fp64 accumulator.
constexpr int kHeadImgs = 4;   // images per pass (loads in flight per lane)

__global__ __launch_bounds__(kHeadThreads) void head_bwd_kernel(HeadParams p, int nbwd) {
  const int t = int(threadIdx.x);
  const float g = p.gscale[0];
  if (int(blockIdx.x) >= nbwd) {   // weight gradient
    const int cells = p.OH * p.OW;
    const int total = p.C * cells;
    const int nw = int(gridDim.x) - nbwd;
    for (int e = (int(blockIdx.x) - nbwd) * kHeadThreads + t; e < total; e += nw * kHeadThreads) {
      const int c = e % p.C, cell = e / p.C;
      float s = 0.f;
      // 8 images' loads in flight at a time (past the last image: image 0 re-read, multiplied by 0),
      // summed in image order; one image per iteration waited out a round trip per image (64 with
      // densityopt's batch)
      for (int n0 = 0; n0 < p.N; n0 += 8) {
        float dv[8], pv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int n = n0 + u < p.N ? n0 + u : 0;
          dv[u] = p.dlogit[n];
          pv[u] = p.pooled[(int64_t(n) * cells + cell) * p.C + c];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (n0 + u < p.N) s += dv[u] * pv[u];
      }
      const int i = cell / p.OW, j = cell - i * p.OW;
      p.dw[c * p.ws_c + i * p.ws_i + j * p.ws_j] = g * s;
    }
    return;
  }
  const int groups = p.C / 8, PXB = kHeadThreads / groups;
  const int wblocks = (p.W + PXB - 1) / PXB;
  const int h = int(blockIdx.x) / wblocks, w = (int(blockIdx.x) - h * wblocks) * PXB + t / groups;
  const int c0 = (t % groups) * 8;
  const bool live = t < PXB * groups && w < p.W;
  const bool bnf = p.bn_acc != nullptr;
  // Every per-channel input (the BN's statistics, affine and sums) as two 16-byte loads of the
  // lane's 8 channels, and each pass's images' dlogit with their BN inputs, issued together before
  // any is used and unconditionally (buffer loads; absent or past the end: zeros).  As scalar loads
  // each consumed at once they were ~14 memory round trips in series (the compiler reused one
  // register for all of them): most of this kernel's 10.6 us.
  const bool bna = p.bn_sums != nullptr;
  auto rsrc_of = [](const void* a, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a), 0, int(a ? bytes : 0), 0x00020000);
  };
  auto load8 = [&](const float* a, int n, int at, float (&o)[8]) __attribute__((always_inline)) {
    const __amdgpu_buffer_rsrc_t r = rsrc_of(a, int64_t(n) * 4);
    const float4 x = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, at * 4, 0, 0));
    const float4 y = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, at * 4 + 16, 0, 0));
    o[0] = x.x, o[1] = x.y, o[2] = x.z, o[3] = x.w, o[4] = y.x, o[5] = y.y, o[6] = y.z, o[7] = y.w;
  };
  const bool need = bnf || bna;
  float cm_[8], ci_[8], cw_[8], cb_[8], sdb[8], sdw[8];
  load8(need ? p.bn_mean : nullptr, p.C, c0, cm_);
  load8(need ? p.bn_invstd : nullptr, p.C, c0, ci_);
  load8(need ? p.bn_w : nullptr, p.C, c0, cw_);
  load8(need ? p.bn_b : nullptr, p.C, c0, cb_);
  load8(bna ? p.bn_sums : nullptr, 2 * p.C, c0, sdb);
  load8(bna ? p.bn_sums : nullptr, 2 * p.C, p.C + c0, sdw);
  const int64_t img = int64_t(p.H) * p.W * p.C;
  const int64_t off = (int64_t(h) * p.W + w) * p.C + c0;
  const __amdgpu_buffer_rsrc_t rs_x = rsrc_of(need ? p.bn_x : nullptr, int64_t(p.N) * img * 2);
  const __amdgpu_buffer_rsrc_t rs_dl = rsrc_of(p.dlogit, int64_t(p.N) * 4);
  uint4 xv[kHeadImgs];
  float dl[kHeadImgs];
  // (the next pass's loads go out before this pass is worked: with 64 images that is 16 passes,
  // one round trip each when every pass waited for its own)
  auto issue_pass = [&](int n0, uint4 (&xa)[kHeadImgs], float (&da)[kHeadImgs]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < kHeadImgs; ++u) {
      const bool in = live && n0 + u < p.N;
      xa[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                            rs_x, in ? uint32_t(((n0 + u) * img + off) * 2) : 0x80000000u, 0, 0));
      da[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_dl, in ? (n0 + u) * 4 : 0x80000000u, 0, 0));
    }
  };
  issue_pass(0, xv, dl);
  float m[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (live) {
    const int i0 = (h * p.OH) / p.H, i1 = ((h + 1) * p.OH + p.H - 1) / p.H;
    const int j0 = (w * p.OW) / p.W, j1 = ((w + 1) * p.OW + p.W - 1) / p.W;
    for (int i = i0; i < i1 && i < p.OH; ++i) {
      const int hs = wstart(i, p.H, p.OH), he = wend(i, p.H, p.OH);
      if (h < hs || h >= he) continue;
      for (int j = j0; j < j1 && j < p.OW; ++j) {
        const int ws = wstart(j, p.W, p.OW), we = wend(j, p.W, p.OW);
        if (w < ws || w >= we) continue;
        const float area = float((he - hs) * (we - ws));
#pragma unroll
        for (int k = 0; k < 8; ++k) m[k] += p.w[(c0 + k) * p.ws_c + i * p.ws_i + j * p.ws_j] / area;
      }
    }
  }
  float is[8], nm[8], bw[8], bb[8], bs[8], bq[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    bs[q] = bq[q] = 0.f;
    is[q] = ci_[q];
    nm[q] = -cm_[q] * is[q];
    bw[q] = cw_[q];
    bb[q] = cb_[q];
  }
  // the BN backward applied here (its sums worked out by the forward, HeadParams::bn_sums):
  // dz becomes the BN's input gradient gx, from the same bf16-rounded gy as the apply kernel reads
  BnBwdCoef bc[8];
  if (bna) {
    const float invM = 1.f / float(int64_t(p.N) * p.H * p.W);
#pragma unroll
    for (int q = 0; q < 8; ++q) bc[q].init(cm_[q], ci_[q], cw_[q], cb_[q], g * sdw[q], g * sdb[q], invM);
    if (blockIdx.x == 0)
      for (int c = t; c < p.C; c += kHeadThreads) p.bn_dw_out[c] = g * p.bn_sums[p.C + c], p.bn_db_out[c] = g * p.bn_sums[c];
  }
  for (int n0 = 0; live && n0 < p.N; n0 += kHeadImgs) {
    uint4 xn[kHeadImgs];
    float dn[kHeadImgs];
    issue_pass(n0 + kHeadImgs, xn, dn);   // (past the last image: out of range, no traffic)
#pragma unroll
    for (int u = 0; u < kHeadImgs; ++u) {
      if (n0 + u >= p.N) break;
      const float d = g * dl[u];
      uint32_t packed[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const f32x2 pr = {d * m[2 * k], d * m[2 * k + 1]};
        packed[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pr, bf16x2));   // RNE, v_cvt_pk_bf16_f32
      }
      if (bna) {   // gx = the BN+LeakyReLU backward of gy = the rounded dz (bn_fold.h: BnBwdCoef)
        const uint32_t xw[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const f32x2 pr = {bc[2 * k].gx(__uint_as_float(xw[k] << 16), __uint_as_float(packed[k] << 16), p.bn_slope),
                            bc[2 * k + 1].gx(__uint_as_float(xw[k] & 0xFFFF0000u),
                                             __uint_as_float(packed[k] & 0xFFFF0000u), p.bn_slope)};
          packed[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pr, bf16x2));
        }
      }
      *reinterpret_cast<uint4*>(p.dz + (n0 + u) * img + off) = make_uint4(packed[0], packed[1], packed[2], packed[3]);
      if (bnf) {   // the BN backward reads the stored (bf16) dz as its gy
        const uint32_t xw[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const uint32_t gb = q & 1 ? packed[q >> 1] & 0xFFFF0000u : packed[q >> 1] << 16;
          const uint32_t xb = q & 1 ? xw[q >> 1] & 0xFFFF0000u : xw[q >> 1] << 16;
          const float xh = fmaf(__uint_as_float(xb), is[q], nm[q]);
          const float gy = __uint_as_float(gb);
          const float gz = fmaf(xh, bw[q], bb[q]) > 0.f ? gy : gy * p.bn_slope;
          bs[q] += gz;
          bq[q] += gz * xh;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kHeadImgs; ++u) xv[u] = xn[u], dl[u] = dn[u];
  }
  if (!bnf) return;
  // fold the PXB pixel lanes of each channel group in LDS ([PXB][C] per sum,
  // PXB * C = 8 * 256); a 9-float pitch per lane spreads the 8-float runs over the banks
  __shared__ float red[2][kHeadThreads * 9];
  if (t < PXB * groups) {
#pragma unroll
    for (int q = 0; q < 8; ++q) red[0][t * 9 + q] = bs[q], red[1][t * 9 + q] = bq[q];
  }
  __syncthreads();
  double* row = p.bn_acc + int64_t(int(blockIdx.x) % p.bn_acc_r) * 2 * p.C;
  for (int c = t; c < p.C; c += kHeadThreads) {
    const int gq = c >> 3, q = c & 7;
    float s0 = 0.f, s1 = 0.f;
    for (int l = 0; l < PXB; ++l) s0 += red[0][(l * groups + gq) * 9 + q], s1 += red[1][(l * groups + gq) * 9 + q];
    unsafeAtomicAdd(row + c, double(s0));
    unsafeAtomicAdd(row + p.C + c, double(s1));
  }
}

// BT_HEAD_FWD=0 (or head_set_fast(0)): round 4's head_fwd_kernel for the BN-applying forward too (A/B)
int g_head_fast = -1;
bool head_fwd_fast() {
  if (g_head_fast < 0) {
    const char* e = std::getenv("BT_HEAD_FWD");
    g_head_fast = (e && e[0] == '0') ? 0 : 1;
  }
  return g_head_fast != 0;
}

}  // namespace

void head_set_fast(int on) { g_head_fast = on < 0 ? -1 : (on ? 1 : 0); }

bool head_bn_bwd_supported(int N, int H, int W, int C, int OH, int OW, int R) {
  // the lean forward's conditions (head_forward below), which the BN-backward sums ride in
  if (N <= 0 || C <= 0 || C % 8 || C / 8 > kHeadThreads || kHeadThreads % (C / 8) || C > kBnFoldMaxC ||
      OH <= 0 || OW <= 0 || H < OH || W < OW || !head_fwd_fast() || int64_t(2) * C * R > kHeadThreads * kHeadFlat)
    return false;
  int most = 0;
  for (int i = 0; i < OH; ++i)
    for (int j = 0; j < OW; ++j) most = std::max(most, (wend(i, H, OH) - wstart(i, H, OH)) * (wend(j, W, OW) - wstart(j, W, OW)));
  return most <= 16 * (kHeadThreads / (C / 8));
}

hipError_t head_forward(const HeadParams& p, hipStream_t stream) {
  if (p.N <= 0 || p.C <= 0 || p.OH <= 0 || p.OW <= 0 || p.H < p.OH || p.W < p.OW || !p.z || !p.w || !p.pooled ||
      !p.partial || !p.loss || !p.dlogit)
    return hipErrorInvalidValue;
  if (p.act.on()) {   // the fast path only: C / 8 lane groups tiling the block, 16-byte aligned rows
    const int G = p.C / 8;
    if (p.C % 8 || G > kHeadThreads || kHeadThreads % G || (reinterpret_cast<uintptr_t>(p.z) & 15) ||
        p.C > kBnFoldMaxC || !p.act.acc || p.act.R <= 0 || !p.act.b || !p.act.mean || !p.act.invstd ||
        p.act.M != int64_t(p.N) * p.H * p.W)
      return hipErrorInvalidValue;
  }
  const dim3 grid(unsigned(p.OH * p.OW), unsigned(p.N));
  if (p.bn_ab && (!p.bn_sums || !p.act.on() || !p.ticket ||
                  !head_bn_bwd_supported(p.N, p.H, p.W, p.C, p.OH, p.OW, p.act.R)))
    return hipErrorInvalidValue;
  if (p.act.on() && p.ticket && head_fwd_fast() && int64_t(2) * p.C * p.act.R <= kHeadThreads * kHeadFlat) {
    // the round-trip-lean form: every window pixel of a lane loaded up front
    int most = 0;   // the largest pooling window
    for (int i = 0; i < p.OH; ++i)
      for (int j = 0; j < p.OW; ++j)
        most = std::max(most, (wend(i, p.H, p.OH) - wstart(i, p.H, p.OH)) * (wend(j, p.W, p.OW) - wstart(j, p.W, p.OW)));
    const int pl = kHeadThreads / (p.C / 8);
    if (most <= 16 * pl) {
      if (p.bn_ab) head_fwd_act_kernel<16, true><<<grid, kHeadThreads, 0, stream>>>(p);
      else head_fwd_act_kernel<16><<<grid, kHeadThreads, 0, stream>>>(p);
      return hipGetLastError();
    }
  }
  head_fwd_kernel<<<grid, kHeadThreads, 0, stream>>>(p);
  if (!p.ticket) head_loss_kernel<<<1, 64, 0, stream>>>(p);
  return hipGetLastError();
}

hipError_t head_backward(const HeadParams& p, hipStream_t stream) {
  if (p.C % 8 || !p.dz || !p.dw || !p.gscale || !p.dlogit || !p.pooled) return hipErrorInvalidValue;
  if (p.OH <= 0 || p.OW <= 0 || p.H < p.OH || p.W < p.OW) return hipErrorInvalidValue;   // <= 2 windows per pixel and dimension
  if (reinterpret_cast<uintptr_t>(p.dz) & 15) return hipErrorInvalidValue;
  const int64_t total = int64_t(p.N) * p.H * p.W * (p.C / 8);
  if (total >= (int64_t(1) << 31) - int64_t(kHeadThreads) * 4096) return hipErrorInvalidValue;
  const int groups = p.C / 8;
  if (p.bn_acc) {   // lanes keep one channel group: the block stride must be a multiple of C / 8
    if (p.bn_acc_r <= 0 || !p.bn_x || !p.bn_mean ||
        !p.bn_invstd || !p.bn_w || !p.bn_b || (reinterpret_cast<uintptr_t>(p.bn_x) & 15))
      return hipErrorInvalidValue;
  }
  if (p.bn_sums && (p.bn_acc || !p.bn_x || !p.bn_mean || !p.bn_invstd || !p.bn_w || !p.bn_b || !p.bn_dw_out ||
                    !p.bn_db_out || (reinterpret_cast<uintptr_t>(p.bn_x) & 15)))
    return hipErrorInvalidValue;   // (the BN backward applied here, or its sums summed here: not both)
  if (groups > kHeadThreads) return hipErrorInvalidValue;
  const int pxb = kHeadThreads / groups;
  const int nbwd = p.H * ((p.W + pxb - 1) / pxb);   // one row segment of pxb pixels per block, all images
  const int wtotal = p.C * p.OH * p.OW;
  const int nw = (wtotal + kHeadThreads - 1) / kHeadThreads;
  head_bwd_kernel<<<unsigned(nbwd + nw), kHeadThreads, 0, stream>>>(p, nbwd);
  return hipGetLastError();
}

}  // namespace gpu
}  // namespace btn
