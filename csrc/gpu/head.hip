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

#include <cstdint>

#include "kernels.h"

namespace btn {
namespace gpu {
namespace {

constexpr int kHeadThreads = 256;
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int wstart(int i, int in, int out) { return (i * in) / out; }
__device__ __forceinline__ int wend(int i, int in, int out) { return ((i + 1) * in + out - 1) / out; }
__device__ __forceinline__ float bf(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }

__device__ void head_loss_wave(const HeadParams& p, bool write_through);

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
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          a[2 * q] += __uint_as_float(uu[q] << 16);
          a[2 * q + 1] += __uint_as_float(uu[q] & 0xFFFF0000u);
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
  head_loss_wave(p, true);
}

// one wave: logits, sigmoid, mean BCE, and dlogit/g for the backward
__device__ void head_loss_wave(const HeadParams& p, bool wt) {
  const int cells = p.OH * p.OW;
  float total = 0.f;
  for (int n = int(threadIdx.x); n < p.N; n += 64) {
    float logit = 0.f;
    for (int k = 0; k < cells; ++k)
      logit += wt ? __hip_atomic_load(p.partial + n * cells + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                  : p.partial[n * cells + k];
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

__global__ __launch_bounds__(64) void head_loss_kernel(HeadParams p) { head_loss_wave(p, false); }

// Backward in ONE launch: blocks [0, nbwd) write dz (8 channels of one pixel
// per lane, one 16-byte store), blocks [nbwd, ...) the weight gradient.
// With p.bn_acc the dz blocks also sum the producing BatchNorm+LeakyReLU
// backward's gz and gz * xhat per channel: a lane keeps one channel group
// over the whole grid-stride loop (the stride is a multiple of C / 8), the
// block folds its lanes through LDS and adds its 2 C sums into replica
// blockIdx % R of the fp64 accumulator.
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
      for (int n = 0; n < p.N; ++n) s += p.dlogit[n] * p.pooled[(int64_t(n) * cells + cell) * p.C + c];
      const int i = cell / p.OW, j = cell - i * p.OW;
      p.dw[c * p.ws_c + i * p.ws_i + j * p.ws_j] = g * s;
    }
    return;
  }
  // 32-bit index math (the host checks N*H*W*C/8 < 2^31): 64-bit division
  // and modulo made this an ALU-bound kernel
  const int groups = p.C / 8;
  const int total = p.N * p.H * p.W * groups;
  const bool bnf = p.bn_acc != nullptr;
  const int c0l = (t % groups) * 8;   // this lane's channel group (fixed: the stride is a multiple of groups)
  float is[8], nm[8], bw[8], bb[8], bs[8], bq[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    bs[q] = bq[q] = 0.f;
    if (bnf) {
      is[q] = p.bn_invstd[c0l + q];
      nm[q] = -p.bn_mean[c0l + q] * is[q];
      bw[q] = p.bn_w[c0l + q];
      bb[q] = p.bn_b[c0l + q];
    }
  }
  for (int e = int(blockIdx.x) * kHeadThreads + t; e < total; e += nbwd * kHeadThreads) {
    int r = e / groups;
    const int c0 = (e - r * groups) * 8;
    const int pix = r;
    r /= p.W;
    const int w = pix - r * p.W;
    const int n = r / p.H;
    const int h = r - n * p.H;
    const float d = g * p.dlogit[n];
    uint4 xv = make_uint4(0, 0, 0, 0);
    if (bnf) xv = *reinterpret_cast<const uint4*>(p.bn_x + (int64_t(pix) * p.C + c0));
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int i0 = (h * p.OH) / p.H, i1 = ((h + 1) * p.OH + p.H - 1) / p.H;
    const int j0 = (w * p.OW) / p.W, j1 = ((w + 1) * p.OW + p.W - 1) / p.W;
    for (int i = i0; i < i1 && i < p.OH; ++i) {
      const int hs = wstart(i, p.H, p.OH), he = wend(i, p.H, p.OH);
      if (h < hs || h >= he) continue;
      for (int j = j0; j < j1 && j < p.OW; ++j) {
        const int ws = wstart(j, p.W, p.OW), we = wend(j, p.W, p.OW);
        if (w < ws || w >= we) continue;
        const float inv = d / float((he - hs) * (we - ws));
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += inv * p.w[(c0 + k) * p.ws_c + i * p.ws_i + j * p.ws_j];
      }
    }
    uint32_t packed[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const f32x2 pr = {acc[2 * k], acc[2 * k + 1]};
      packed[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pr, bf16x2));   // RNE, v_cvt_pk_bf16_f32
    }
    *reinterpret_cast<uint4*>(p.dz + ((int64_t(n * p.H + h) * p.W + w) * p.C + c0)) =
        make_uint4(packed[0], packed[1], packed[2], packed[3]);
    if (bnf) {   // the BN backward reads the stored (bf16) dz as its gy
      const uint32_t xw[4] = {xv.x, xv.y, xv.z, xv.w};
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
  if (!bnf) return;
  // fold the lanes of each channel group (lanes t, t + groups, ...) in LDS
  __shared__ float red[2][kHeadThreads * 8];   // [PL][C] per sum, PL * C = 8 * 256
  const int PL = kHeadThreads / groups;
#pragma unroll
  for (int q = 0; q < 8; ++q) red[0][(t / groups) * p.C + c0l + q] = bs[q], red[1][(t / groups) * p.C + c0l + q] = bq[q];
  __syncthreads();
  double* row = p.bn_acc + int64_t(int(blockIdx.x) % p.bn_acc_r) * 2 * p.C;
  for (int c = t; c < p.C; c += kHeadThreads) {
    float s0 = 0.f, s1 = 0.f;
    for (int l = 0; l < PL; ++l) s0 += red[0][l * p.C + c], s1 += red[1][l * p.C + c];
    unsafeAtomicAdd(row + c, double(s0));
    unsafeAtomicAdd(row + p.C + c, double(s1));
  }
}

}  // namespace

hipError_t head_forward(const HeadParams& p, hipStream_t stream) {
  if (p.N <= 0 || p.C <= 0 || p.OH <= 0 || p.OW <= 0 || p.H < p.OH || p.W < p.OW || !p.z || !p.w || !p.pooled ||
      !p.partial || !p.loss || !p.dlogit)
    return hipErrorInvalidValue;
  head_fwd_kernel<<<dim3(unsigned(p.OH * p.OW), unsigned(p.N)), kHeadThreads, 0, stream>>>(p);
  if (!p.ticket) head_loss_kernel<<<1, 64, 0, stream>>>(p);
  return hipGetLastError();
}

hipError_t head_backward(const HeadParams& p, hipStream_t stream) {
  if (p.C % 8 || !p.dz || !p.dw || !p.gscale || !p.dlogit || !p.pooled) return hipErrorInvalidValue;
  if (reinterpret_cast<uintptr_t>(p.dz) & 15) return hipErrorInvalidValue;
  const int64_t total = int64_t(p.N) * p.H * p.W * (p.C / 8);
  if (total >= (int64_t(1) << 31) - int64_t(kHeadThreads) * 4096) return hipErrorInvalidValue;
  const int groups = p.C / 8;
  if (p.bn_acc) {   // lanes keep one channel group: the block stride must be a multiple of C / 8
    if (groups > kHeadThreads || kHeadThreads % groups || p.bn_acc_r <= 0 || !p.bn_x || !p.bn_mean ||
        !p.bn_invstd || !p.bn_w || !p.bn_b || (reinterpret_cast<uintptr_t>(p.bn_x) & 15))
      return hipErrorInvalidValue;
  }
  const int64_t blocks = (total + kHeadThreads - 1) / kHeadThreads;
  // BN-fused: one block per CU, lanes loop -- each block adds 2 C fp64 sums
  // into the accumulator, so fewer, fuller blocks keep that traffic small
  const int cap = p.bn_acc ? 256 : 2048;
  const int nbwd = int(blocks < cap ? blocks : cap);
  const int wtotal = p.C * p.OH * p.OW;
  const int nw = (wtotal + kHeadThreads - 1) / kHeadThreads;
  head_bwd_kernel<<<unsigned(nbwd + nw), kHeadThreads, 0, stream>>>(p, nbwd);
  return hipGetLastError();
}

}  // namespace gpu
}  // namespace btn
