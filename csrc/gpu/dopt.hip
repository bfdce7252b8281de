// densityopt's per-iteration control math as two gfx950 kernels: the
// discriminator gate and the simulation-parameter (S) step.
//
// The reference (examples/densityopt/densityopt.py:257-316) does this part
// of the loop in eager PyTorch with host round trips: D_real / D_sim means
// (.item()), the gate `D_real - D_sim < 0.7`, then for the S step the
// per-sample BCE against label 1, a LogNormal ProbModel's log_prob indexed by
// the returned shape ids, `mean(log_prob * (err - b))`, its autograd
// backward to the 4 parameters (mean and log-std of m1 and m2), Adam, the
// moving-average baseline and `pm.sample(B)` for the next images.  On the GPU
// that was ~150 elementwise / reduce launches of ~4 us and ~87 device copies
// per iteration (profiles/r5/b2/dopt_iteration_kernels.txt).  Here:
//
//  * dopt_gate_kernel: D_real / D_sim as the means of sigmoid(logits) over
//    the batch, the gate, written where FusedAdam.step(gate=) reads it;
//  * dopt_sstep_kernel: one block; per sample err = -max(log sigmoid(l),
//    -100) (BCELoss(reduction='none'), target 1), the score-function
//    gradient in closed form
//        d/dmu_k  = mean_i (err_i - b) (log x_ki - mu_k) / s_k^2
//        d/drho_k = mean_i (err_i - b) ((log x_ki - mu_k)^2 / s_k^2 - 1)
//    (s_k = exp(rho_k): the derivatives of the LogNormal log-density), the
//    gated Adam update of the 4 parameters (FusedAdam's arithmetic), the
//    baseline / first-step bookkeeping, and the next samples
//    x = exp(mu + s * z), z ~ N(0, 1) from a counter-based Philox4x32-10
//    keyed by (seed, iteration counter, index) -- every rank draws the same
//    samples, so data parallelism needs no broadcast.  The rank's chunk of the
//    samples, the parameters, the D statistics and both gates go straight to
//    host-mapped memory: the host's per-iteration fetch is a wait, not a copy.
//
// Sums run in a fixed order (per-thread strided partial, fixed shuffle tree,
// fixed wave order): bit-identical run to run.  With data parallelism the
// kernel runs in two phases around one RCCL all-reduce (average) of the 5
// per-rank means [err, g_mu1, g_mu2, g_rho1, g_rho2].
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace btn {
namespace gpu {
namespace {

constexpr int kDoptThreads = 256;

__device__ __forceinline__ float sigmoidf(float x) { return 1.f / (1.f + expf(-x)); }

// block-wide sum of V values per thread, fixed order: xor tree in the wave, then waves in order
template <int V>
__device__ __forceinline__ void block_sum(float (&v)[V], float* lds) {
  const int lane = int(threadIdx.x) & 63, wave = int(threadIdx.x) >> 6;
#pragma unroll
  for (int k = 0; k < V; ++k)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < V; ++k) lds[wave * V + k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < V; ++k) {
    float s = 0.f;
    for (int w = 0; w < kDoptThreads / 64; ++w) s += lds[w * V + k];
    v[k] = s;
  }
  __syncthreads();
}

// Philox4x32-10 (Salmon et al., SC'11): 4 uniform 32-bit words per (key, counter)
__device__ __forceinline__ void philox(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                       uint32_t (&out)[4]) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t h0 = __umulhi(M0, c0), l0 = M0 * c0;
    const uint32_t h1 = __umulhi(M1, c2), l1 = M1 * c2;
    const uint32_t n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
    c0 = n0, c1 = l1, c2 = n2, c3 = l0;
    k0 += W0, k1 += W1;
  }
  out[0] = c0, out[1] = c1, out[2] = c2, out[3] = c3;
}

// u in (0, 1]
__device__ __forceinline__ float u01(uint32_t x) { return (float(x >> 8) + 1.f) * (1.f / 16777216.f); }

__global__ __launch_bounds__(kDoptThreads) void dopt_gate_kernel(DoptParams p, int phase) {
  __shared__ float lds[kDoptThreads / 64 * 2];
  // phase 0: means and gate; 1: per-rank means only (averaged over ranks next); 2: gate from the averaged stats
  if (phase != 2) {
    float v[2] = {0.f, 0.f};
    for (int i = int(threadIdx.x); i < p.B; i += kDoptThreads) {
      v[0] += sigmoidf(p.logit_real[i]);
      v[1] += sigmoidf(p.logit_sim[i]);
    }
    block_sum<2>(v, lds);
    if (threadIdx.x == 0) {
      p.stats[0] = v[0] / float(p.B);
      p.stats[1] = v[1] / float(p.B);
    }
    if (phase == 1) return;
  }
  if (threadIdx.x == 0) {
    const float dr = p.stats[0], ds = p.stats[1];   // (phase 0: this thread just wrote them)
    p.gate_d[0] = dr - ds < p.threshold ? 1.f : 0.f;
  }
}

__global__ __launch_bounds__(kDoptThreads) void dopt_sstep_kernel(DoptParams p, int phase) {
  __shared__ float lds[kDoptThreads / 64 * 5];
  __shared__ float par[4];   // mu1, mu2, s1, s2 after the update
  const int t = int(threadIdx.x);
  // phase 0: all; 1: the per-rank means into red[5] (averaged over ranks next); 2: the update from red
  // (phase 3: the samples only -- the first draw, before any simulated batch exists)
  float gm[5] = {0.f, 0.f, 0.f, 0.f, 0.f};   // [err, g_mu1, g_mu2, g_rho1, g_rho2]: this rank's means, or every rank's
  if (phase == 2) {
#pragma unroll
    for (int k = 0; k < 5; ++k) gm[k] = p.red[k];
  } else if (phase != 3) {
    const float mu0 = p.mean[0], mu1 = p.mean[1];
    const float iv0 = expf(-2.f * p.log_std[0]), iv1 = expf(-2.f * p.log_std[1]);
    const float b = p.b[0];
    float v[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int i = t; i < p.B; i += kDoptThreads) {
      const float pr = sigmoidf(p.logit_s[i]);
      const float err = -fmaxf(logf(pr), -100.f);
      int64_t sid = p.sid[i];
      sid = sid < 0 ? 0 : (sid >= p.N ? p.N - 1 : sid);   // (the host validates them; never read out of bounds)
      const float d0 = logf(p.samples[sid]) - mu0, d1 = logf(p.samples[p.N + sid]) - mu1;
      const float w = err - b;
      v[0] += err;
      v[1] += w * d0 * iv0;
      v[2] += w * d1 * iv1;
      v[3] += w * (d0 * d0 * iv0 - 1.f);
      v[4] += w * (d1 * d1 * iv1 - 1.f);
    }
    block_sum<5>(v, lds);   // (ends with a barrier: every read of the current samples is done)
#pragma unroll
    for (int k = 0; k < 5; ++k) gm[k] = v[k] / float(p.B);
    if (phase == 1) {
      if (t < 5) p.red[t] = gm[t];
      return;
    }
  }
  if (t == 0) {
    const float gd = p.gate_d[0], first = p.first[0];
    float gs = (1.f - first) + (1.f - gd);
    gs = gs > 1.f ? 1.f : gs;
    if (phase == 3) gs = p.gate_s[0];
    else p.gate_s[0] = gs;
    float* prm[4] = {p.mean, p.mean + 1, p.log_std, p.log_std + 1};
    if (gs > 0.f && phase != 3) {
      // FusedAdam's update (ops/adam.py _step_reference), the step counter on the device
      const float s = p.adam_step[0] + 1.f;
      p.adam_step[0] = s;
      const float step_size = p.lr / (1.f - powf(p.b1, s));
      const float inv_bc2 = 1.f / sqrtf(1.f - powf(p.b2, s));
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float g = gm[1 + k];
        const float m = p.b1 * p.exp_avg[k] + (1.f - p.b1) * g;
        const float v2 = p.b2 * p.exp_avg_sq[k] + (1.f - p.b2) * g * g;
        p.exp_avg[k] = m;
        p.exp_avg_sq[k] = v2;
        *prm[k] -= step_size * m / (sqrtf(v2) * inv_bc2 + p.eps);
      }
      const float em = gm[0];
      const float bn = first > 0.f ? em : p.alpha * em + (1.f - p.alpha) * p.b[0];
      p.b[0] = bn;
      p.first[0] = first * (1.f - gs);
    }
    par[0] = *prm[0], par[1] = *prm[1], par[2] = expf(*prm[2]), par[3] = expf(*prm[3]);
#pragma unroll
    for (int k = 0; k < 4; ++k) p.params_out[k] = par[k];
    if (p.host) {   // host-mapped: [2][B] this rank's samples (below), params[4], stats[2], gate_d, gate_s
      float* h = p.host + 2 * p.B;
#pragma unroll
      for (int k = 0; k < 4; ++k) h[k] = par[k];
      h[4] = p.stats[0], h[5] = p.stats[1], h[6] = gd, h[7] = gs;
    }
  }
  __syncthreads();
  const uint32_t ctr = p.counter[0];
  for (int i = t; 2 * i < 2 * p.N; i += kDoptThreads) {   // 2 normals per Philox call: samples i of rows 0 and 1
    uint32_t r[4];
    philox(uint32_t(p.seed), uint32_t(p.seed >> 32), uint32_t(i), ctr, 0x5eedu, 0u, r);
    const float rad = sqrtf(-2.f * logf(u01(r[0])));
    float sn, cs;
    sincosf(6.2831853071795864f * u01(r[1]), &sn, &cs);
    const float x0 = expf(par[0] + par[2] * rad * cs), x1 = expf(par[1] + par[3] * rad * sn);
    p.samples[i] = x0;
    p.samples[p.N + i] = x1;
    const int j = i - p.rank * p.B;
    if (p.host && j >= 0 && j < p.B) p.host[j] = x0, p.host[p.B + j] = x1;
  }
  __syncthreads();
  if (t == 0) p.counter[0] = ctr + 1u;
}

}  // namespace

void* host_mapped_alloc(size_t bytes, void** dev) {
  void* host = nullptr;
  *dev = nullptr;
  if (hipHostMalloc(&host, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return nullptr;
  if (hipHostGetDevicePointer(dev, host, 0) != hipSuccess) {
    (void)hipHostFree(host);
    return nullptr;
  }
  return host;
}

void host_mapped_free(void* host) {
  if (host) (void)hipHostFree(host);
}

hipError_t dopt_gate(const DoptParams& p, int phase, hipStream_t stream) {
  if (!p.logit_real || !p.logit_sim || !p.stats || !p.gate_d || p.B <= 0 || phase < 0 || phase > 2)
    return hipErrorInvalidValue;
  dopt_gate_kernel<<<1, kDoptThreads, 0, stream>>>(p, phase);
  return hipGetLastError();
}

hipError_t dopt_sstep(const DoptParams& p, int phase, hipStream_t stream) {
  if (((phase == 0 || phase == 1) && (!p.logit_s || !p.sid)) || !p.samples || !p.mean || !p.log_std || !p.exp_avg ||
      !p.exp_avg_sq || !p.adam_step || !p.b || !p.first || !p.gate_s || !p.gate_d || !p.stats || !p.params_out ||
      !p.counter || !p.red || p.B <= 0 || p.N < p.B || p.world <= 0 || p.rank < 0 || (p.rank + 1) * p.B > p.N ||
      phase < 0 || phase > 3)
    return hipErrorInvalidValue;
  dopt_sstep_kernel<<<1, kDoptThreads, 0, stream>>>(p, phase);
  return hipGetLastError();
}

}  // namespace gpu
}  // namespace btn
