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
    double v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = g + G * i;
      v[i] = r < f.R ? f.acc[int64_t(r) * J + j] : 0.0;
    }
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[i];
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

}  // namespace gpu
}  // namespace btn
