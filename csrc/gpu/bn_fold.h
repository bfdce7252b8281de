// Fold of a BatchNorm statistics accumulator (kernels.h: BnAcc) by ONE
// 256-thread block: lane (j, g) -- j a (sum, channel) column of [R][2C], g one
// of G = 256 / 2C replica groups -- loads its R / G replicas with every load
// in flight at once (one memory latency), sums them in fp64 and clears them
// for the next producer; the G group sums meet in LDS in a fixed order (the
// same fold whichever block runs it); one lane per channel finalizes.
// Used by bn_acc_finalize_kernel (train.hip) and, as an extra block of the
// weight-gradient launch that follows the producing data gradient, by
// conv_wgrad_kernel (conv.hip) -- the backward then has no finalize launch.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace btn {
namespace gpu {

constexpr int kBnFoldMaxC = 512;

struct BnFold {
  double* acc = nullptr;   // [R][2][C] fp64
  int R = 0, C = 0;
  int64_t M = 0;
  int bwd = 0;             // 0: o0 = mean, o1 = invstd (+ running statistics); 1: o0 = db, o1 = dw
  float eps = 0.f, momentum = 0.f;
  float* o0 = nullptr;
  float* o1 = nullptr;
  float* rm = nullptr;
  float* rv = nullptr;
  int64_t* tracked = nullptr;
};

// every thread of the block; part: >= max(256, 2 C) doubles of LDS
__device__ inline void bn_fold_block(const BnFold& f, double* part) {
  const int t = int(threadIdx.x), nt = int(blockDim.x);
  const int J = 2 * f.C;
  const int G = J >= nt ? 1 : nt / J;
  for (int u = t; u < G * J; u += nt) {
    const int j = u % J, g = u / J;
    // every replica load issued unconditionally (an out-of-range one re-reads
    // replica 0 and adds 0.0): a guarded load per replica compiled to a branch
    // and a full memory wait each -- 8 round trips instead of one
    double v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = g + G * i;
      v[i] = f.acc[int64_t(r < f.R ? r : 0) * J + j];
    }
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += g + G * i < f.R ? v[i] : 0.0;
    for (int r = g + 8 * G; r < f.R; r += G) s += f.acc[int64_t(r) * J + j];   // R > 8 G: not with R = 1024 / C
    for (int r = g; r < f.R; r += G) f.acc[int64_t(r) * J + j] = 0.0;          // read: cleared for the next producer
    part[g * J + j] = s;
  }
  __syncthreads();
  for (int c = t; c < f.C; c += nt) {
    double s0 = 0.0, s1 = 0.0;
    for (int g = 0; g < G; ++g) s0 += part[g * J + c], s1 += part[g * J + f.C + c];
    if (f.bwd) {
      f.o0[c] = float(s0);
      f.o1[c] = float(s1);
    } else {
      const double mu = s0 / double(f.M);
      double var = s1 / double(f.M) - mu * mu;
      var = var < 0.0 ? 0.0 : var;
      f.o0[c] = float(mu);
      f.o1[c] = float(1.0 / sqrt(var + double(f.eps)));
      if (f.rm) {
        f.rm[c] = float((1.0 - f.momentum) * f.rm[c] + f.momentum * mu);
        f.rv[c] = float((1.0 - f.momentum) * f.rv[c] + f.momentum * var * double(f.M) / double(f.M > 1 ? f.M - 1 : 1));
      }
      if (f.tracked && c == 0) f.tracked[0] += 1;
    }
  }
}

// BatchNorm + LeakyReLU backward for one element, given the BN input v and
// the gradient g of the activation's output: gx = P (gz - db / M) - P dw / M
// xhat, xhat = v is + nm, gz = g leaky'(xhat w + b).  ONE definition for the
// apply kernel (train.hip) and the first layer's weight gradient, which
// computes its dY operand this way instead of reading a materialised gx
// (conv.hip, ConvWgradParams::bn_dy): both round the same fp32 value to bf16.
struct BnBwdCoef {
  float is, nm, ww, bb, P, dbm, pdw;
  __device__ void init(float mean, float invstd, float w, float b, float dw, float db, float invM) {
    is = invstd;
    nm = -mean * is;
    ww = w;
    bb = b;
    P = ww * is;
    dbm = db * invM;
    pdw = P * dw * invM;
  }
  __device__ float gx(float v, float g, float slope) const {
    const float xh = fmaf(v, is, nm);
    const float gz = fmaf(xh, ww, bb) > 0.f ? g : g * slope;
    return fmaf(P, gz - dbm, -pdw * xh);
  }
};

// The apply kernels' own fold (bn_apply_fold_kernel, train.hip): EVERY block
// of the apply launch folds the accumulator it consumes -- one memory latency
// at the block's start, overlapped with its first pass of loads -- so no
// one-block finalize launch (and its kernel boundary) sits between the
// producer and the apply.  The accumulator is cleared for the next producer
// by whichever block arrives last (a ticket word after the [R][2][C]
// replicas: blocks take a ticket only once their reads have returned, so the
// last ticket holder clears after every reader), and block 0 writes the
// finalized outputs (mean / invstd and running statistics, or dw / db).
//
// Sums of column j of [R][J] (J = 2C) over the replicas into part[j] (every
// thread of the block; part: >= max(nt, J) doubles of LDS).  COH: the replicas
// were added into by other blocks of THIS launch (read behind a grid barrier):
// loads at agent scope, past this XCD's caches.
template <bool COH = false>
__device__ inline double bn_acc_load(const double* p) {
  if constexpr (COH) {
    return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  } else {
    return *p;
  }
}
template <bool COH = false>
__device__ inline void bn_acc_column_sums(const double* acc, int R, int J, double* part) {
  const int t = int(threadIdx.x), nt = int(blockDim.x);
  const int G = J >= nt ? 1 : nt / J;
  for (int u = t; u < G * J; u += nt) {
    const int j = u % J, g = u / J;
    double v[8];   // (unconditional loads, as bn_fold_block)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = g + G * i;
      v[i] = bn_acc_load<COH>(acc + int64_t(r < R ? r : 0) * J + j);
    }
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += g + G * i < R ? v[i] : 0.0;
    for (int r = g + 8 * G; r < R; r += G) s += bn_acc_load<COH>(acc + int64_t(r) * J + j);
    part[g * J + j] = s;
  }
  __syncthreads();
  // fold the G groups into part[j] (column j is owned by one thread: no race)
  for (int j = t; j < J; j += nt) {
    double s = part[j];
    for (int g = 1; g < G; ++g) s += part[g * J + j];
    part[j] = s;
  }
  __syncthreads();
}

// The ticket words of a [R][2][C] accumulator (kernels.h: bn_acc_elems leaves
// room for them): 8 shard counters, then the top counter.  One counter for
// every block of a 1,024-block apply launch serialised ~1,000 returning
// atomics on one word (~88 per us): ~12 us of a 25 us kernel.  Blocks take a
// ticket on the shard of their blockIdx % 8 (8 words, 8 channels in
// parallel); the last block of each shard takes one on the top counter.
constexpr int kBnTicketShards = 8;
constexpr int kBnTicketStride = 32;   // words: one 128-byte line per counter (atomics contend per line)
__device__ inline unsigned* bn_acc_ticket(double* acc, int R, int C) {
  return reinterpret_cast<unsigned*>(acc + int64_t(R) * 2 * C);
}
// The word after the top counter (spare in bn_acc_elems): a grid barrier of
// the producing launch (conv.hip grid_barrier), zero between uses.
__device__ inline unsigned* bn_acc_barrier(double* acc, int R, int C) {
  return bn_acc_ticket(acc, R, C) + kBnTicketShards * kBnTicketStride + 1;
}

// After every reader of this block has its values (call after the block's
// last use of them, behind a barrier): take a ticket; the block with the
// last one clears the replicas and resets the tickets.  `flag`: one int of
// LDS.  `blk` / `nblk`: this block's linear index and the grid's block count.
__device__ inline void bn_acc_release(double* acc, int R, int C, int* flag, unsigned blk, unsigned nblk) {
  const int t = int(threadIdx.x), nt = int(blockDim.x);
  unsigned* ticket = bn_acc_ticket(acc, R, C);
  if (t == 0) {
    const unsigned G = nblk, s = blk % kBnTicketShards;
    const unsigned in_shard = (G - s + kBnTicketShards - 1) / kBnTicketShards;   // blocks s, s + 8, ...
    const unsigned shards = G < unsigned(kBnTicketShards) ? G : unsigned(kBnTicketShards);
    int last = 0;
    if (atomicAdd(ticket + s * kBnTicketStride, 1u) == in_shard - 1) {
      ticket[s * kBnTicketStride] = 0u;   // every block of this shard has taken its ticket
      last = atomicAdd(ticket + kBnTicketShards * kBnTicketStride, 1u) == shards - 1 ? 1 : 0;
    }
    *flag = last;
  }
  __syncthreads();
  if (*flag) {
    const int n = R * 2 * C;
    for (int i = t; i < n; i += nt) acc[i] = 0.0;
    if (t == 0) ticket[kBnTicketShards * kBnTicketStride] = 0u;
  }
}
__device__ inline void bn_acc_release(double* acc, int R, int C, int* flag) {   // 1-D grids
  bn_acc_release(acc, R, C, flag, blockIdx.x, gridDim.x);
}

// bn_acc_release in two halves, for a block with more work after its reads (bn_apply_kernel): thread
// 0 takes the shard ticket as soon as the block's reads are back (behind a barrier) and keeps the
// answer in a register; the block's remaining loads and stores then overlap that atomic's round
// trip, and at the end (every thread) the shard's last block takes the top ticket and the device's
// last block clears.  Waiting for the shard ticket before the apply pass cost 0.9-1.4 us a launch
// (profiles/r6/b8/bn_apply_norel.jsonl against bn_apply.jsonl).
__device__ inline unsigned bn_acc_ticket_take(double* acc, int R, int C, unsigned blk) {   // thread 0
  // (+ the lane id, 0 here: with an address the compiler sees as uniform, its atomic optimizer
  // folds the wave's lanes through the returned value right away -- a wait for the round trip)
  return atomicAdd(bn_acc_ticket(acc, R, C) + (blk % kBnTicketShards) * kBnTicketStride + __lane_id(), 1u);
}
__device__ inline void bn_acc_ticket_finish(double* acc, int R, int C, int* flag, unsigned tk, unsigned blk,
                                            unsigned nblk) {
  const int t = int(threadIdx.x), nt = int(blockDim.x);
  unsigned* ticket = bn_acc_ticket(acc, R, C);
  if (t == 0) {
    const unsigned s = blk % kBnTicketShards;
    const unsigned in_shard = (nblk - s + kBnTicketShards - 1) / kBnTicketShards;
    const unsigned shards = nblk < unsigned(kBnTicketShards) ? nblk : unsigned(kBnTicketShards);
    int last = 0;
    if (tk == in_shard - 1) {
      ticket[s * kBnTicketStride] = 0u;
      last = atomicAdd(ticket + kBnTicketShards * kBnTicketStride, 1u) == shards - 1 ? 1 : 0;
    }
    *flag = last;
  }
  __syncthreads();
  if (*flag) {
    const int n = R * 2 * C;
    for (int i = t; i < n; i += nt) acc[i] = 0.0;
    if (t == 0) ticket[kBnTicketShards * kBnTicketStride] = 0u;
  }
}

// The forward finalize of a folded accumulator (part[c] = sum, part[C + c] =
// sum of squares over M elements; bn_acc_column_sums), exactly as
// bn_fold_block computes it: mean and invstd of channel c; the block that
// passes `first` also writes the outputs and running statistics.
struct BnFwdFinal {
  float eps = 0.f, momentum = 0.f;
  float* mean = nullptr;
  float* invstd = nullptr;
  float* rm = nullptr;
  float* rv = nullptr;
  int64_t* tracked = nullptr;
};
__device__ inline void bn_fwd_finalize(const BnFwdFinal& f, const double* part, int C, int64_t M, int c, bool first,
                                       float& mean, float& invstd) {
  const double mu = part[c] / double(M);
  double var = part[C + c] / double(M) - mu * mu;
  var = var < 0.0 ? 0.0 : var;
  mean = float(mu);
  invstd = float(1.0 / sqrt(var + double(f.eps)));
  if (first) {
    f.mean[c] = mean;
    f.invstd[c] = invstd;
    if (f.rm) {
      f.rm[c] = float((1.0 - f.momentum) * f.rm[c] + f.momentum * mu);
      f.rv[c] = float((1.0 - f.momentum) * f.rv[c] + f.momentum * var * double(M) / double(M > 1 ? M - 1 : 1));
    }
    if (f.tracked && c == 0) f.tracked[0] += 1;
  }
}

// Coefficients of a BatchNorm+LeakyReLU backward applied by the weight
// gradient that stages its dY (ConvWgradParams::BnDy), for channels chan0 ..
// chan0 + 7: with an accumulator the block folds it here (every thread of the
// block; part: >= max(nt, 2 C) doubles of LDS, flag: one int; blk / nblk:
// this block among the nblk that fold), block 0 writes db / dw, the last
// block clears it; else dw / db are read as given.  M: elements per channel.
// The forward statistics and affine parameters of channels chan0 .. chan0 + 7, loaded ahead (at a
// kernel's start, in flight with its other first loads) for bn_dy_coefs: otherwise they are a
// memory round trip of their own after the fold's
struct BnDyPre {
  float m[8], is[8], w[8], b[8];
  template <class BnDy>
  __device__ void load(const BnDy& d, int chan0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) m[i] = d.mean[chan0 + i], is[i] = d.invstd[chan0 + i], w[i] = d.w[chan0 + i], b[i] = d.b[chan0 + i];
  }
};

// tk (nullable): no release here -- the caller takes the release's ticket (bn_acc_ticket_take, any
// time after this returns) and finishes it at its end (bn_acc_ticket_finish).  pre (nullable):
// BnDyPre of chan0, loaded ahead.
template <class BnDy>
__device__ inline void bn_dy_coefs(const BnDy& d, int C, int64_t M, int chan0, double* part, int* flag, unsigned blk,
                                   unsigned nblk, BnBwdCoef (&bc)[8], unsigned* tk = nullptr,
                                   const BnDyPre* pre = nullptr) {
  const float invM = 1.f / float(M);
  if (d.acc) {
    bn_acc_column_sums(d.acc, d.R, 2 * C, part);   // part[c] = db = sum gz, part[C + c] = dw = sum gz xhat
    if (blk == 0) {
      for (int c = int(threadIdx.x); c < C; c += int(blockDim.x)) {
        d.db_out[c] = float(part[c]);
        d.dw_out[c] = float(part[C + c]);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = chan0 + i;
      if (pre) bc[i].init(pre->m[i], pre->is[i], pre->w[i], pre->b[i], float(part[C + c]), float(part[c]), invM);
      else bc[i].init(d.mean[c], d.invstd[c], d.w[c], d.b[c], float(part[C + c]), float(part[c]), invM);
    }
    __syncthreads();
    if (!tk) bn_acc_release(d.acc, d.R, C, flag, blk, nblk);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = chan0 + i;
      bc[i].init(d.mean[c], d.invstd[c], d.w[c], d.b[c], d.dw[c], d.db[c], invM);
    }
  }
}

}  // namespace gpu
}  // namespace btn
