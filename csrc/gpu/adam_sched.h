// The Adam step schedule (step counter, bias corrections) as a one-lane job:
// run by adam_schedule_kernel (train.hip) or, attached by the optimizer ahead
// of the backward, by the first lane of the weight gradient's slice-reduce
// launch (conv_wgrad_reduce_kernel, conv.hip) -- one launch fewer per step.
#pragma once

#include <hip/hip_runtime.h>

#include "kernels.h"

namespace btn {
namespace gpu {

// (AdamSchedJob and the host attach API: kernels.h)

// the schedule of step s (bias corrections in fp64, as torch.optim.Adam)
__device__ inline void adam_schedule_write(float s, const float* hp, float* sched, float beta1, float beta2) {
  const float lr = hp[0];
  const double bc1 = 1.0 - pow(double(beta1), double(s));
  const double bc2 = 1.0 - pow(double(beta2), double(s));
  sched[0] = float(double(lr) / bc1);
  sched[1] = float(1.0 / sqrt(bc2));
  sched[2] = lr;
  sched[3] = hp[1];   // gradient scale (e.g. 1 / world after a summing all-reduce)
}

// one lane: a closed gate (gate[0] == 0, computed on the device earlier in
// the same stream / graph) makes the whole step a no-op (counter, moments, weights)
__device__ inline void adam_schedule_run(const AdamSchedJob& j) {
  const bool active = !j.gate || j.gate[0] != 0.f;
  j.sched[4] = active ? 1.f : 0.f;
  if (!active) return;
  const float s = j.step[0] + 1.f;
  j.step[0] = s;
  adam_schedule_write(s, j.hp, j.sched, j.beta1, j.beta2);
}

}  // namespace gpu
}  // namespace btn
