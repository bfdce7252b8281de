// The ordered weight-gradient slice sum, shared by the slice-reduce launch
// (conv.hip wgrad_reduce_ordered) and the Adam update that takes the backward's
// last reduce into its own launch (train.hip, AdamParams::fr).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace btn {
namespace gpu {

// Lane groups of `sub` (a power of two <= 64, <= S) share 4 consecutive elements of
// the [Cout][16 Cin] slice; lane `part` of a group sums slices part, part + sub, ...
// in that order, two rounds of SG loads in flight at once, then the group adds its
// lanes with a fixed xor-shuffle tree (commutative adds: every lane ends with the
// same bits) and its lane 0 calls emit(e0, sum) -- bit-identical run to run.  R: any
// struct with partial, S, sub, Cin, Cout.  NT: the lanes of the block that take part.
template <int NT, int SG, class R, class Emit>
__device__ __forceinline__ void wgrad_slice_sum(const R& r, int bx, Emit&& emit) {
  if (int(threadIdx.x) >= NT) return;   // (wave-uniform: a side job of a wider block)
  const float* __restrict__ partial = r.partial;
  const int S = r.S, sub = r.sub;
  const int total = r.Cout * 16 * r.Cin;
  const int gl = bx * NT + int(threadIdx.x);
  const int part = gl & (sub - 1);
  const int e0 = (gl / sub) * 4;
  const bool live = e0 < total;   // (group-uniform: all sub lanes of a group share e0)
  const int64_t base = live ? e0 : 0;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  // two rounds of SG loads in flight at once (the default heuristic gives a lane <= 2
  // rounds: one round trip instead of two); the sums stay in slice order
  for (int k0 = part; k0 < S; k0 += 2 * SG * sub) {
    float4 v[2 * SG];
#pragma unroll
    for (int j = 0; j < 2 * SG; ++j) {   // past the last slice: re-read slice `part` (< S), not added
      const int k = k0 + j * sub;
      v[j] = *reinterpret_cast<const float4*>(partial + int64_t(k < S ? k : part) * total + base);
    }
#pragma unroll
    for (int j = 0; j < 2 * SG; ++j)
      if (k0 + j * sub < S) acc.x += v[j].x, acc.y += v[j].y, acc.z += v[j].z, acc.w += v[j].w;
  }
  for (int o = sub >> 1; o > 0; o >>= 1) {
    acc.x += __shfl_xor(acc.x, o);
    acc.y += __shfl_xor(acc.y, o);
    acc.z += __shfl_xor(acc.z, o);
    acc.w += __shfl_xor(acc.w, o);
  }
  if (!live || part != 0) return;
  emit(e0, acc);
}

}  // namespace gpu
}  // namespace btn
