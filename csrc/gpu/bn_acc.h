// Producer-side finalize of a BnAcc accumulator (kernels.h): the kernel that
// adds a BatchNorm's statistics into the accumulator -- conv_fwd's or
// conv_dgrad's epilogue, the fused head backward -- also finalizes them in
// the block that finishes last, so no separate finalize launch sits between
// it and the BN's apply kernel.
//
// Hand-off: every block's adds are fp64 atomics, executed at the memory side;
// each lane waits for its own (vmcnt(0)), the block barrier collects them,
// one lane takes a ticket; the block that takes the last ticket reads the
// accumulator with returning atomic exchanges (memory side as well: fresh
// whatever any L2 holds, and cleared for the next producer in the same
// instruction), folds the R replicas in fp64 and writes the outputs.  It then
// resets the ticket.  acc and the ticket must be zero when the kernel starts;
// every producer leaves them so.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace btn {
namespace gpu {

struct BnFin {
  double* acc = nullptr;   // [R][2][C] fp64, then the ticket word (acc + 2 C R)
  int R = 0, C = 0;
  int64_t M = 0;           // elements per channel (forward: the batch statistics' count)
  int bwd = 0;             // 0: o0 = mean, o1 = invstd (+ running stats); 1: o0 = db, o1 = dw
  float eps = 0.f, momentum = 0.f;
  float* o0 = nullptr;
  float* o1 = nullptr;
  float* rm = nullptr;
  float* rv = nullptr;
  int64_t* tracked = nullptr;
};

// Called by EVERY thread of each of the nb blocks that add into the
// accumulator, after its atomic adds.  lds: at least max(256, 2 C) doubles of
// the block's (free) LDS, and one int at flag outside them.
__device__ inline void bn_fin_tail_n(const BnFin& f, double* lds, int* flag, uint32_t nb) {
  const int t = int(threadIdx.x), nt = int(blockDim.x);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this lane's adds are done at memory
  __syncthreads();
  const int J = 2 * f.C;
  if (t == 0) {
    uint32_t* ticket = reinterpret_cast<uint32_t*>(f.acc + int64_t(J) * f.R);
    const uint32_t tk = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = tk == nb - 1;
    if (tk == nb - 1) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!*flag) return;
  // G lane groups over the replicas (every lane <= 8 exchanges in flight at once)
  const int G = J >= nt ? 1 : nt / J;
  for (int u = t; u < G * J; u += nt) {
    const int j = u % J, g = u / J;
    double v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = g + G * i;
      v[i] = r < f.R ? __hip_atomic_exchange(f.acc + int64_t(r) * J + j, 0.0, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)
                     : 0.0;
    }
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[i];
    for (int r = g + 8 * G; r < f.R; r += G)   // R > 8 G (not with bn_acc_replicas' R): serial rest
      s += __hip_atomic_exchange(f.acc + int64_t(r) * J + j, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    lds[g * J + j] = s;
  }
  __syncthreads();
  for (int c = t; c < f.C; c += nt) {
    double s0 = 0.0, s1 = 0.0;
    for (int g = 0; g < G; ++g) s0 += lds[g * J + c], s1 += lds[g * J + f.C + c];
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

// every block of the grid adds
__device__ inline void bn_fin_tail(const BnFin& f, double* lds, int* flag) {
  bn_fin_tail_n(f, lds, flag, gridDim.x * gridDim.y * gridDim.z);
}

}  // namespace gpu
}  // namespace btn
