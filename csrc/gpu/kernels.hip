// gfx950 kernels for the blendtorch image path (see kernels.h).
//
// decode: pure streaming op (~1.2 MB read, 3.7 MB fp32 written per 640x480
// RGBA image), so it is shaped for HBM, not ALU:
//   * every lane handles PPT consecutive pixels of ONE row, so the HWC->CHW
//     de-interleave happens in registers: one 16-byte load per lane for RGBA
//     (12/24 bytes for RGB) and one 16-byte store per output plane -- the
//     "transpose" needs no LDS round trip because each output plane is a
//     contiguous run of the same pixels;
//   * PPT is picked per output dtype so every plane store is exactly 16 B
//     (f32: 4 px, bf16/f16: 8 px, u8: 16 px);
//   * gamma + scale + per-channel mean/std: the host verifies an arithmetic
//     form of the fp32 reference table (fma, or mul/sub[/div] rounded like
//     numpy) per channel, so the kernel computes the value; only the u8 gamma
//     table is looked up, from a lane-private LDS copy (every lane of a
//     ds_read group owns a bank: no conflicts, whatever the pixel values).
//     Bit-exact with the fp32 reference (kernels.h: lut);
//   * the vertical flip (GL lower-left readback) is a source-row remap.
// color4x4: per-pixel 4x4 affine transform on the matrix cores with
//   v_mfma_f32_4x4x1_16b_f32 (16 independent 4x4 blocks per wave, exact f32):
//   block = 4 pixels x 4 output channels, K = input channel, 16 MFMAs per
//   256 pixels; lane l ends up holding output channel (l & 3) of sixteen
//   consecutive pixels -> four 16-byte stores per lane, plane-contiguous.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "kernels.h"

namespace btn {
namespace gpu {

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ uint16_t f2bf(float f) {
  // round-to-nearest-even in one v_cvt_pk_bf16_f32 (gfx950)
  return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f));
}

__device__ __forceinline__ uint16_t f2h(float f) {
  _Float16 h = (_Float16)f;
  return *reinterpret_cast<uint16_t*>(&h);
}

// Base of image b's output (elements of type T): per-image pointer when the
// launch coalesces several batches, else the b-th slab of one dense tensor.
template <typename T, typename P>
__device__ __forceinline__ T* image_out(const P& p, int b, int64_t img_elems) {
  return p.ndsts ? reinterpret_cast<T*>(p.dsts[b]) : reinterpret_cast<T*>(p.dst) + int64_t(b) * img_elems;
}

template <int PPT, int CIN>
struct Pixels {
  uint8_t v[PPT * CIN];
};

// Load PPT pixels (PPT*CIN bytes) with the widest aligned accesses.
template <int PPT, int CIN>
__device__ __forceinline__ void load_pixels(const uint8_t* p, Pixels<PPT, CIN>& px) {
  constexpr int NB = PPT * CIN;
  if constexpr (NB % 16 == 0) {
#pragma unroll
    for (int i = 0; i < NB / 16; ++i) *reinterpret_cast<uint4*>(&px.v[16 * i]) = reinterpret_cast<const uint4*>(p)[i];
  } else if constexpr (NB % 8 == 0) {
#pragma unroll
    for (int i = 0; i < NB / 8; ++i) *reinterpret_cast<uint2*>(&px.v[8 * i]) = reinterpret_cast<const uint2*>(p)[i];
  } else {
#pragma unroll
    for (int i = 0; i < NB / 4; ++i) *reinterpret_cast<uint32_t*>(&px.v[4 * i]) = reinterpret_cast<const uint32_t*>(p)[i];
  }
}

// ---- value transform (kernels.h: lut) --------------------------------------
// LDS holds either the fp32 table (mode 0, <= 4 KiB) or R copies of the u8
// gamma table: word (v >> 2) * R + (lane % R) packs gamma[v & ~3 .. v | 3],
// so with R = 32 lane l of a 32-lane ds_read group always hits bank l (8 KiB).
constexpr int kTabWords = 2048;

struct Xf {
  int arith;               // 0: fp32 table lookups; 1: arithmetic
  const float* lut;        // LDS fp32 table [c][256] (arith == 0)
  const uint8_t* g;        // this lane's column of the LDS gamma table
  int gshift;              // log2 of a gamma row's bytes (4 * copies)
  int gam[4], op[4];
  float a[4], b[4], d[4], r[4];
};

// Read the header (uniform: scalar loads) and stage the table; caller syncs.
__device__ __forceinline__ Xf stage_xf(const float* T, uint32_t* tab, int nch) {
  Xf x;
  x.arith = T[kXfHeader] != 0.f;
  x.lut = reinterpret_cast<const float*>(tab);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    x.gam[c] = T[kXfHeader + 2 + c] != 0.f;
    x.op[c] = int(T[kXfHeader + 6 + c]);
    x.a[c] = T[kXfHeader + 10 + c];
    x.b[c] = T[kXfHeader + 14 + c];
    x.d[c] = T[kXfHeader + 18 + c];
    x.r[c] = T[kXfHeader + 22 + c];
  }
  // gamma copies R (16 or 32): lane l reads copy l % R.  32 = every lane of a
  // ds_read group owns a bank; 16 = half the fill, lanes l and l+16 share a
  // bank (a 2-way conflict only when their values differ in the same column)
  const int rep = int(T[kXfHeader + 1]);
  x.gshift = rep == 32 ? 7 : 6;                 // bytes per gamma row: 4 * R
  x.g = reinterpret_cast<const uint8_t*>(tab) + (threadIdx.x & (rep - 1)) * 4;
  if (!x.arith) {
    for (int i = threadIdx.x; i < nch * 256; i += blockDim.x) reinterpret_cast<float*>(tab)[i] = T[i];
  } else if (rep > 0) {
    // 16-byte stores: the 4 words of a quad sit in one row (same gamma dword)
    const uint32_t* gw = reinterpret_cast<const uint32_t*>(T + kXfGamma);
    const int qshift = rep == 32 ? 3 : 2;       // quads per row: R / 4
    for (int i = threadIdx.x; i < 16 * rep; i += blockDim.x) {
      const uint32_t w = gw[i >> qshift];
      reinterpret_cast<uint4*>(tab)[i] = make_uint4(w, w, w, w);
    }
  }
  return x;
}

// op 1 / op 2 must round every operation on its own (numpy's float32 order),
// never contract the multiply into an fma
__device__ __forceinline__ float xf_mulsub(float x, float a, float b) {
#pragma clang fp contract(off)
  return x * a - b;
}

// op 3: the quotient by the rounded reciprocal plus one fma correction --
// the host proved it equals the correctly rounded division for every input
__device__ __forceinline__ float xf_recip_div(float t, float d, float r) {
  const float q = t * r;
  return __builtin_fmaf(__builtin_fmaf(-q, d, t), r, q);
}

__device__ __forceinline__ float xf_apply(int op, float x, float a, float b, float d, float r) {
  if (op == 0) return __builtin_fmaf(x, a, b);
  const float t = xf_mulsub(x, a, b);
  if (op == 1) return t;
  return op == 3 ? xf_recip_div(t, d, r) : t / d;   // op 2: correctly rounded fp32 division (HIP default)
}

__device__ __forceinline__ float xf_source(const Xf& xf, int c, uint32_t v) {
  return xf.gam[c] ? float(xf.g[((v >> 2) << xf.gshift) + (v & 3)]) : float(v);
}

// Value of output channel c for input byte v (scalar paths).
__device__ __forceinline__ float xf_value(const Xf& xf, int c, uint32_t v) {
  if (!xf.arith) return xf.lut[c * 256 + v];
  return xf_apply(xf.op[c], xf_source(xf, c, v), xf.a[c], xf.b[c], xf.d[c], xf.r[c]);
}

// Output channel c from input channel IC for the lane's PPT pixels.  The
// channel map is a runtime value, but it is uniform across the wave: `lookup`
// branches on it once (scalar branch) into a fully static body, so every
// byte of `px` is addressed with a compile-time index and `px` stays in
// VGPRs (a dynamically indexed byte array would be spilled to scratch).
template <int PPT, int CIN, int IC>
__device__ __forceinline__ void lookup_static(const Pixels<PPT, CIN>& px, const Xf& xf, int c, float (&o)[PPT]) {
  if (!xf.arith) {
    const float* l = xf.lut + c * 256;
#pragma unroll
    for (int i = 0; i < PPT; ++i) o[i] = l[px.v[i * CIN + IC]];
    return;
  }
  float x[PPT];
  if (xf.gam[c]) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const uint32_t v = px.v[i * CIN + IC];
      x[i] = float(xf.g[((v >> 2) << xf.gshift) + (v & 3)]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < PPT; ++i) x[i] = float(px.v[i * CIN + IC]);
  }
  const float a = xf.a[c], b = xf.b[c], d = xf.d[c], r = xf.r[c];
  if (xf.op[c] == 0) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) o[i] = __builtin_fmaf(x[i], a, b);
  } else if (xf.op[c] == 1) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) o[i] = xf_mulsub(x[i], a, b);
  } else if (xf.op[c] == 3) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) o[i] = xf_recip_div(xf_mulsub(x[i], a, b), d, r);
  } else {
#pragma unroll
    for (int i = 0; i < PPT; ++i) o[i] = xf_mulsub(x[i], a, b) / d;
  }
}

template <int PPT, int CIN>
__device__ __forceinline__ void lookup(const Pixels<PPT, CIN>& px, int ic, const Xf& xf, int c, float (&o)[PPT]) {
  switch (ic) {
    case 0: lookup_static<PPT, CIN, 0>(px, xf, c, o); break;
    case 1: if constexpr (CIN > 1) lookup_static<PPT, CIN, 1>(px, xf, c, o); break;
    case 2: if constexpr (CIN > 2) lookup_static<PPT, CIN, 2>(px, xf, c, o); break;
    default: if constexpr (CIN > 3) lookup_static<PPT, CIN, 3>(px, xf, c, o); break;
  }
}

template <int PPT, int CIN, int OUTT, int COUT>
__device__ __forceinline__ void store_nhwc(const DecodeParams& p, const Xf& xf, const int* cm,
                                           const Pixels<PPT, CIN>& px, int b, int64_t q, int64_t HW) {
  constexpr int N = PPT * COUT;
  const int64_t off = q * COUT;   // within image b (NHWC)
  float v[COUT][PPT];
#pragma unroll
  for (int c = 0; c < COUT; ++c) lookup<PPT, CIN>(px, cm[c], xf, c, v[c]);
  if constexpr (OUTT == OUT_F32) {
    float o[N];
#pragma unroll
    for (int i = 0; i < PPT; ++i)
#pragma unroll
      for (int c = 0; c < COUT; ++c) o[i * COUT + c] = v[c][i];
    float4* d = reinterpret_cast<float4*>(image_out<float>(p, b, HW * COUT) + off);
#pragma unroll
    for (int i = 0; i < N / 4; ++i) d[i] = make_float4(o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]);
  } else if constexpr (OUTT == OUT_BF16 || OUTT == OUT_F16) {
    uint16_t o[N];
#pragma unroll
    for (int i = 0; i < PPT; ++i)
#pragma unroll
      for (int c = 0; c < COUT; ++c) o[i * COUT + c] = OUTT == OUT_BF16 ? f2bf(v[c][i]) : f2h(v[c][i]);
    uint4* d = reinterpret_cast<uint4*>(image_out<uint16_t>(p, b, HW * COUT) + off);
#pragma unroll
    for (int i = 0; i < N / 8; ++i) d[i] = *reinterpret_cast<const uint4*>(&o[8 * i]);
  } else {
    uint8_t o[N];
#pragma unroll
    for (int i = 0; i < PPT; ++i)
#pragma unroll
      for (int c = 0; c < COUT; ++c) o[i * COUT + c] = uint8_t(v[c][i]);
    uint4* d = reinterpret_cast<uint4*>(image_out<uint8_t>(p, b, HW * COUT) + off);
#pragma unroll
    for (int i = 0; i < N / 16; ++i) d[i] = *reinterpret_cast<const uint4*>(&o[16 * i]);
  }
}

// Where one lane's group of PPT pixels comes from / goes to.
struct Group {
  int b;                 // image
  int64_t q;             // first pixel (row-major) in the image
  const uint8_t* src;    // first source byte (flip applied)
};

// (image, first pixel, row, column) of pixel group g.  32-bit division when
// the launch's group count fits (every real frame batch): a 64-bit divide is a
// ~100-instruction sequence, two per lane and group.
template <int PPT>
__device__ __forceinline__ void split_group(int64_t g, int64_t groups_per_img, int W, bool small, int& b, int64_t& q,
                                            int& y, int& x) {
  if (small) {
    const uint32_t g32 = uint32_t(g), gpi = uint32_t(groups_per_img);
    const uint32_t b32 = g32 / gpi;
    const uint32_t q32 = (g32 - b32 * gpi) * uint32_t(PPT);
    const uint32_t y32 = q32 / uint32_t(W);
    b = int(b32), q = int64_t(q32), y = int(y32), x = int(q32 - y32 * uint32_t(W));
  } else {
    b = int(g / groups_per_img);
    q = (g - int64_t(b) * groups_per_img) * PPT;
    y = int(q / W);
    x = int(q - int64_t(y) * W);
  }
}

template <int PPT, int CIN>
__device__ __forceinline__ Group locate(const DecodeParams& p, int64_t g, int64_t groups_per_img, int64_t HW,
                                        bool small) {
  Group r;
  int y, x;
  split_group<PPT>(g, groups_per_img, p.W, small, r.b, r.q, y, x);
  const int b = r.b;
  const bool flip = p.flip_all || (p.flip && p.flip[b]) || (b < 256 && ((p.flip_bits[b >> 6] >> (b & 63)) & 1));
  const int sy = flip ? p.H - 1 - y : y;
  const uint8_t* img = p.nsrcs ? p.srcs[b] : p.src + (p.src_offsets ? p.src_offsets[b] : int64_t(b) * HW * CIN);
  r.src = img + (int64_t(sy) * p.W + x) * CIN;
  return r;
}

template <int PPT, int CIN, int OUTT, int LAYOUT>
__device__ __forceinline__ void emit(const DecodeParams& p, const Xf& xf, const int* cm, int cout, int64_t HW,
                                     const Group& gr, const Pixels<PPT, CIN>& px) {
  const int b = gr.b;
  const int64_t q = gr.q;
  if constexpr (LAYOUT == NCHW) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c >= cout) break;
      float v[PPT];
      lookup<PPT, CIN>(px, cm[c], xf, c, v);
      const int64_t off = int64_t(c) * HW + q;   // within image b (NCHW)
      if constexpr (OUTT == OUT_F32) {
        float* d = image_out<float>(p, b, HW * cout) + off;
#pragma unroll
        for (int i = 0; i < PPT / 4; ++i) reinterpret_cast<float4*>(d)[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
      } else if constexpr (OUTT == OUT_BF16 || OUTT == OUT_F16) {
        uint16_t o[PPT];
#pragma unroll
        for (int i = 0; i < PPT; ++i) o[i] = OUTT == OUT_BF16 ? f2bf(v[i]) : f2h(v[i]);
        uint16_t* d = image_out<uint16_t>(p, b, HW * cout) + off;
#pragma unroll
        for (int i = 0; i < PPT / 8; ++i) reinterpret_cast<uint4*>(d)[i] = *reinterpret_cast<const uint4*>(&o[8 * i]);
      } else {
        uint8_t o[PPT];
#pragma unroll
        for (int i = 0; i < PPT; ++i) o[i] = uint8_t(v[i]);
        uint8_t* d = image_out<uint8_t>(p, b, HW * cout) + off;
#pragma unroll
        for (int i = 0; i < PPT / 16; ++i) reinterpret_cast<uint4*>(d)[i] = *reinterpret_cast<const uint4*>(&o[16 * i]);
      }
    }
  } else {
    // NHWC (channels_last): PPT*COUT contiguous elements, assembled in
    // registers and written as 16-byte stores (PPT*sizeof(T) == 16).
    switch (cout) {
      case 1: store_nhwc<PPT, CIN, OUTT, 1>(p, xf, cm, px, b, q, HW); break;
      case 2: store_nhwc<PPT, CIN, OUTT, 2>(p, xf, cm, px, b, q, HW); break;
      case 3: store_nhwc<PPT, CIN, OUTT, 3>(p, xf, cm, px, b, q, HW); break;
      default: store_nhwc<PPT, CIN, OUTT, 4>(p, xf, cm, px, b, q, HW); break;
    }
  }
}

// Grid-stride over pixel groups; U groups per lane per iteration: all U loads
// are issued before the first table lookup, so each lane keeps U requests in
// flight (memory-level parallelism once the grid is smaller than the work).
template <int PPT, int CIN, int OUTT, int LAYOUT, int U>
__global__ __launch_bounds__(kBlock) void decode_vec_kernel(DecodeParams p) {
  __shared__ uint32_t tab[kTabWords];
  const Xf xf = stage_xf(p.lut, tab, p.Cout);
  __syncthreads();

  const int64_t HW = int64_t(p.H) * p.W;
  const int64_t groups_per_img = HW / PPT;
  const int64_t total = groups_per_img * p.B;
  const int cout = p.Cout;
  int cm[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) cm[c] = p.cmap[c];
  const int64_t stride = int64_t(gridDim.x) * kBlock;
  const bool small = total + U * stride < (int64_t(1) << 31) && HW < (int64_t(1) << 31);

  for (int64_t g0 = int64_t(blockIdx.x) * kBlock + threadIdx.x; g0 < total; g0 += U * stride) {
    const Group gr0 = locate<PPT, CIN>(p, g0, groups_per_img, HW, small);
    Pixels<PPT, CIN> px0;
    load_pixels<PPT, CIN>(gr0.src, px0);
    if constexpr (U == 2) {
      const int64_t g1 = g0 + stride;
      const bool has1 = g1 < total;
      // second group's load goes out before the first group's lookups
      const Group gr1 = locate<PPT, CIN>(p, has1 ? g1 : g0, groups_per_img, HW, small);
      Pixels<PPT, CIN> px1;
      load_pixels<PPT, CIN>(gr1.src, px1);
      emit<PPT, CIN, OUTT, LAYOUT>(p, xf, cm, cout, HW, gr0, px0);
      if (has1) emit<PPT, CIN, OUTT, LAYOUT>(p, xf, cm, cout, HW, gr1, px1);
    } else {
      emit<PPT, CIN, OUTT, LAYOUT>(p, xf, cm, cout, HW, gr0, px0);
    }
  }
}

// Key-frame delta, launch 1: every image starts as its producer's decoded
// key frame (16-byte copies, HBM to HBM).
__global__ __launch_bounds__(kBlock) void tile_fill_kernel(DecodeParams p, TileParams t) {
  const int64_t per = t.out_img_bytes / 16;
  const int64_t total = per * p.B;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < total; i += int64_t(gridDim.x) * kBlock) {
    const int b = int(i / per);
    const int64_t j = i - int64_t(b) * per;
    uint8_t* d = p.ndsts ? static_cast<uint8_t*>(p.dsts[b]) : static_cast<uint8_t*>(p.dst) + int64_t(b) * t.out_img_bytes;
    reinterpret_cast<uint4*>(d)[j] = reinterpret_cast<const uint4*>(t.fills[b])[j];
  }
}

// Key-frame delta, launch 2: decode the payload tiles over the filled images.
// LPT = 256 / PPT lanes per 16x16 tile (64 for f32, 32 bf16/f16, 16 u8); lane
// `idx` of a tile takes PPT pixels of tile row idx / (16 / PPT).
template <int PPT, int CIN, int OUTT, int LAYOUT>
__global__ __launch_bounds__(kBlock) void tile_scatter_kernel(DecodeParams p, TileParams t) {
  __shared__ uint32_t tab[kTabWords];
  const Xf xf = stage_xf(p.lut, tab, p.Cout);
  __syncthreads();
  constexpr int T = 16, LPT = T * T / PPT, LPR = T / PPT;
  const int64_t HW = int64_t(p.H) * p.W;
  const int ntx = p.W / T;
  const int64_t total = int64_t(t.tile_start[p.B]) * LPT;
  const int cout = p.Cout;
  int cm[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) cm[c] = p.cmap[c];
  for (int64_t g = int64_t(blockIdx.x) * kBlock + threadIdx.x; g < total; g += int64_t(gridDim.x) * kBlock) {
    const int gt = int(g / LPT), idx = int(g - int64_t(gt) * LPT);
    int b = 0;
    while (b + 1 < p.B && gt >= t.tile_start[b + 1]) ++b;
    const int k = gt - t.tile_start[b];
    const uint8_t* enc = p.srcs[b];
    // independent loads: the tile's position and its pixels
    const uint32_t pos = reinterpret_cast<const uint32_t*>(enc)[1 + k];
    Pixels<PPT, CIN> px;
    load_pixels<PPT, CIN>(enc + t.payload_off + (int64_t(k) * T * T + int64_t(idx) * PPT) * CIN, px);
    const int r = idx / LPR, col = (idx - r * LPR) * PPT;
    const int sy = int(pos / ntx) * T + r, x = int(pos % ntx) * T + col;
    const bool flip = p.flip_all || (p.flip && p.flip[b]) || (b < 256 && ((p.flip_bits[b >> 6] >> (b & 63)) & 1));
    Group gr;
    gr.b = b;
    gr.q = int64_t(flip ? p.H - 1 - sy : sy) * p.W + x;
    gr.src = nullptr;
    emit<PPT, CIN, OUTT, LAYOUT>(p, xf, cm, cout, HW, gr, px);
  }
}

// Generic fallback: one pixel per thread (any W, any alignment).
template <int OUTT>
__global__ __launch_bounds__(kBlock) void decode_scalar_kernel(DecodeParams p) {
  __shared__ uint32_t tab[kTabWords];
  const Xf xf = stage_xf(p.lut, tab, p.Cout);
  __syncthreads();
  const int64_t HW = int64_t(p.H) * p.W;
  const int64_t total = HW * p.B;
  for (int64_t g = int64_t(blockIdx.x) * kBlock + threadIdx.x; g < total; g += int64_t(gridDim.x) * kBlock) {
    const int b = int(g / HW);
    const int64_t q = g - int64_t(b) * HW;
    const int y = int(q / p.W), x = int(q - int64_t(y) * p.W);
    const bool flip = p.flip_all || (p.flip && p.flip[b]) || (b < 256 && ((p.flip_bits[b >> 6] >> (b & 63)) & 1));
    const int sy = flip ? p.H - 1 - y : y;
    const uint8_t* img = p.nsrcs ? p.srcs[b] : p.src + (p.src_offsets ? p.src_offsets[b] : int64_t(b) * HW * p.Cin);
    const uint8_t* s = img + (int64_t(sy) * p.W + x) * p.Cin;
    for (int c = 0; c < p.Cout; ++c) {
      const float v = xf_value(xf, c, s[p.cmap[c]]);
      const int64_t off = p.layout == NCHW ? int64_t(c) * HW + q : q * p.Cout + c;   // within image b
      const int64_t ie = HW * p.Cout;
      if constexpr (OUTT == OUT_F32) image_out<float>(p, b, ie)[off] = v;
      else if constexpr (OUTT == OUT_BF16) image_out<uint16_t>(p, b, ie)[off] = f2bf(v);
      else if constexpr (OUTT == OUT_F16) image_out<uint16_t>(p, b, ie)[off] = f2h(v);
      else image_out<uint8_t>(p, b, ie)[off] = uint8_t(v);
    }
  }
}

int grid_for(int64_t work, int cap = 0) {
  // Measured on MI355X (profiles/decode_unroll_sweep.txt): up to ~4k blocks
  // of work, one resident wave of 2048 blocks (256 CUs x 8) is best; for
  // large batches a grid of 8192 blocks keeps more stores in flight
  // (64 x 640x480 RGBA -> f32: 74.7 us at 2048 blocks, 63.3 us at 8192).
  int64_t blocks = (work + kBlock - 1) / kBlock;
  if (cap <= 0) cap = blocks > 4096 ? 8192 : 2048;
  return int(blocks < cap ? (blocks > 0 ? blocks : 1) : cap);
}

template <typename T>
bool dsts_ok(T* const* dsts, int n, int B, uintptr_t align) {
  if (n != B) return false;
  for (int b = 0; b < n; ++b)
    if (!dsts[b] || (reinterpret_cast<uintptr_t>(dsts[b]) % align) != 0) return false;
  return true;
}

bool srcs_ok(const uint8_t* const* srcs, int n, int B, uintptr_t align) {
  if (n != B) return false;
  for (int b = 0; b < n; ++b)
    if (!srcs[b] || (reinterpret_cast<uintptr_t>(srcs[b]) % align) != 0) return false;
  return true;
}

template <int PPT, int CIN, int OUTT, int U>
void launch_vec_u(const DecodeParams& p, int grid, hipStream_t s) {
  if (p.layout == NCHW)
    decode_vec_kernel<PPT, CIN, OUTT, NCHW, U><<<grid, kBlock, 0, s>>>(p);
  else
    decode_vec_kernel<PPT, CIN, OUTT, NHWC, U><<<grid, kBlock, 0, s>>>(p);
}

template <int PPT, int CIN, int OUTT>
hipError_t launch_vec(const DecodeParams& p, hipStream_t s) {
  int64_t work = int64_t(p.B) * p.H * p.W / PPT;
  // launch-shape overrides for sweeps (BT_DECODE_MAXGRID / BT_DECODE_UNROLL)
  static const int env_grid = std::getenv("BT_DECODE_MAXGRID") ? std::atoi(std::getenv("BT_DECODE_MAXGRID")) : 0;
  static const int env_unroll = std::getenv("BT_DECODE_UNROLL") ? std::atoi(std::getenv("BT_DECODE_UNROLL")) : 0;
  const int grid = grid_for(work, p.max_grid > 0 ? p.max_grid : env_grid);
  // U=2 (two groups' loads in flight per lane) measured no faster than U=1
  // at 8 or 64 frames once the grid is sized right; kept as an option
  const int req = p.unroll > 0 ? p.unroll : env_unroll;
  const int u = req > 0 ? req : 1;
  if (u >= 2)
    launch_vec_u<PPT, CIN, OUTT, 2>(p, grid, s);
  else
    launch_vec_u<PPT, CIN, OUTT, 1>(p, grid, s);
  return hipGetLastError();
}

template <int OUTT>
hipError_t launch_out(const DecodeParams& p, hipStream_t s) {
  constexpr int PPT = OUTT == OUT_F32 ? 4 : (OUTT == OUT_U8 ? 16 : 8);
  // vector path: a lane's PPT pixels sit in one row and its loads are aligned
  const bool src_aligned = p.nsrcs ? srcs_ok(p.srcs, p.nsrcs, p.B, 16)
                                   : (reinterpret_cast<uintptr_t>(p.src) % 16) == 0 && (p.src_offsets == nullptr || p.src_offsets_aligned);
  const bool dst_aligned = p.ndsts ? dsts_ok(p.dsts, p.ndsts, p.B, 16) : (reinterpret_cast<uintptr_t>(p.dst) % 16) == 0;
  bool aligned = (p.W % PPT) == 0 && (int64_t(p.H) * p.W * p.Cin) % 16 == 0 && dst_aligned && src_aligned;
  if constexpr (OUTT == OUT_U8) {
    // RGBA -> RGBA u8 NHWC read from HOST memory (the scatter root's raw
    // frames): 4 pixels per lane, one 16-byte load and one 16-byte store, so
    // 4x the lanes of the 16-pixel shape keep PCIe read requests in flight
    // (the 16-pixel shape read host frames at ~36 GB/s against ~50)
    if (p.nsrcs && p.layout == NHWC && p.Cin == 4 && p.Cout == 4 && aligned && (p.W % 4) == 0)
      return launch_vec<4, 4, OUTT>(p, s);
  }
  if (aligned && p.Cin == 4) return launch_vec<PPT, 4, OUTT>(p, s);
  if (aligned && p.Cin == 3) return launch_vec<PPT, 3, OUTT>(p, s);
  int64_t work = int64_t(p.B) * p.H * p.W;
  decode_scalar_kernel<OUTT><<<grid_for(work, p.max_grid), kBlock, 0, s>>>(p);
  return hipGetLastError();
}

}  // namespace

template <int PPT, int CIN, int OUTT>
void launch_tiles(const DecodeParams& p, const TileParams& t, int grid, hipStream_t s) {
  if (p.layout == NCHW)
    tile_scatter_kernel<PPT, CIN, OUTT, NCHW><<<grid, kBlock, 0, s>>>(p, t);
  else
    tile_scatter_kernel<PPT, CIN, OUTT, NHWC><<<grid, kBlock, 0, s>>>(p, t);
}

template <int OUTT>
void launch_tiles_out(const DecodeParams& p, const TileParams& t, hipStream_t s) {
  constexpr int PPT = OUTT == OUT_F32 ? 4 : (OUTT == OUT_U8 ? 16 : 8);
  const int64_t work = int64_t(t.tile_start[p.B]) * (256 / PPT);
  if (work <= 0) return;
  const int grid = grid_for(work, p.max_grid);
  if (p.Cin == 4)
    launch_tiles<PPT, 4, OUTT>(p, t, grid, s);
  else
    launch_tiles<PPT, 3, OUTT>(p, t, grid, s);
}

hipError_t decode(const DecodeParams& p, hipStream_t stream) {
  if (p.B <= 0 || p.H <= 0 || p.W <= 0) return hipSuccess;
  if (p.Cout < 1 || p.Cout > 4 || p.Cin < 1 || p.Cin > 4) return hipErrorInvalidValue;
  if (p.nsrcs && (p.nsrcs != p.B || p.nsrcs > kMaxSrcs || !srcs_ok(p.srcs, p.nsrcs, p.B, 1))) return hipErrorInvalidValue;
  if (p.ndsts && (p.ndsts != p.B || p.ndsts > kMaxSrcs || !dsts_ok(p.dsts, p.ndsts, p.B, 1))) return hipErrorInvalidValue;
  for (int c = 0; c < p.Cout; ++c)
    if (p.cmap[c] < 0 || p.cmap[c] >= p.Cin) return hipErrorInvalidValue;
  switch (p.out_dtype) {
    case OUT_F32: return launch_out<OUT_F32>(p, stream);
    case OUT_BF16: return launch_out<OUT_BF16>(p, stream);
    case OUT_F16: return launch_out<OUT_F16>(p, stream);
    case OUT_U8: return launch_out<OUT_U8>(p, stream);
  }
  return hipErrorInvalidValue;
}

hipError_t decode_tiles(const DecodeParams& p, const TileParams& t, hipStream_t stream) {
  if (p.B <= 0) return hipSuccess;
  const int ppt = p.out_dtype == OUT_F32 ? 4 : (p.out_dtype == OUT_U8 ? 16 : 8);
  const size_t elem = p.out_dtype == OUT_F32 ? 4 : (p.out_dtype == OUT_U8 ? 1 : 2);
  if (p.B > kMaxSrcs || p.nsrcs != p.B || p.H % 16 != 0 || p.W % 16 != 0 || (p.Cin != 3 && p.Cin != 4) ||
      p.Cout < 1 || p.Cout > 4 || p.W % ppt != 0 || t.payload_off % 16 != 0 || t.out_img_bytes % 16 != 0 ||
      t.out_img_bytes != int64_t(p.H) * p.W * p.Cout * int64_t(elem) || !srcs_ok(p.srcs, p.nsrcs, p.B, 16) ||
      (p.ndsts ? !dsts_ok(p.dsts, p.ndsts, p.B, 16) : (reinterpret_cast<uintptr_t>(p.dst) % 16) != 0) ||
      t.tile_start[0] != 0)
    return hipErrorInvalidValue;
  const int64_t ntiles = int64_t(p.H / 16) * (p.W / 16);
  for (int b = 0; b < p.B; ++b)
    if (!t.fills[b] || (reinterpret_cast<uintptr_t>(t.fills[b]) % 16) != 0 || t.tile_start[b + 1] < t.tile_start[b] ||
        t.tile_start[b + 1] - t.tile_start[b] > ntiles)
      return hipErrorInvalidValue;
  for (int c = 0; c < p.Cout; ++c)
    if (p.cmap[c] < 0 || p.cmap[c] >= p.Cin) return hipErrorInvalidValue;
  const int64_t chunks = t.out_img_bytes / 16 * p.B;
  tile_fill_kernel<<<grid_for(chunks, 0), kBlock, 0, stream>>>(p, t);
  switch (p.out_dtype) {
    case OUT_F32: launch_tiles_out<OUT_F32>(p, t, stream); break;
    case OUT_BF16: launch_tiles_out<OUT_BF16>(p, t, stream); break;
    case OUT_F16: launch_tiles_out<OUT_F16>(p, t, stream); break;
    case OUT_U8: launch_tiles_out<OUT_U8>(p, t, stream); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// fused replay sample: Philox index draw + gather + decode + metadata gather
// ---------------------------------------------------------------------------
namespace {

// Philox4x32-10 (Salmon et al., SC'11), first output word.
__device__ __forceinline__ uint32_t philox_word(uint64_t seed, uint64_t ctr, uint32_t b) {
  uint32_t c0 = b, c1 = uint32_t(ctr), c2 = uint32_t(ctr >> 32), c3 = 0;
  uint32_t k0 = uint32_t(seed), k1 = uint32_t(seed >> 32);
#pragma unroll
  for (int round = 0; round < 10; ++round) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    c0 = hi1 ^ c1 ^ k0;
    c1 = lo1;
    c2 = hi0 ^ c3 ^ k1;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c0;
}

// Block prologue shared by both replay kernels: the table, this launch's B
// frame indices (drawn or given) in LDS, and the counter hand-over.
struct ReplayShared {
  uint32_t tab[kTabWords];
  int64_t idx[kMaxReplayB];
  uint64_t ctr;
};

__device__ Xf replay_prologue(const DecodeParams& p, const ReplayParams& r, ReplayShared& sh) {
  const Xf xf = stage_xf(p.lut, sh.tab, p.Cout);
  if (threadIdx.x == 0) sh.ctr = r.index_in ? 0 : (r.counter ? r.counter[0] : r.ctr_value);
  __syncthreads();
  for (int b = threadIdx.x; b < p.B; b += kBlock) {
    const int64_t i = r.index_in ? r.index_in[b]
                                 : int64_t((uint64_t(philox_word(r.seed, sh.ctr, uint32_t(b))) * uint64_t(r.count)) >> 32);
    sh.idx[b] = i;
    if (blockIdx.x == 0 && r.index_out) r.index_out[b] = i;
  }
  __syncthreads();
  return xf;
}

// The counter moves on in a one-lane kernel queued right behind the sample:
// every block of the sample reads it, so no block may advance it in-kernel
// without a grid-wide handshake -- and a per-block atomic (or fence) on one
// address serialises thousands of blocks (measured 68 -> 517 us).
__global__ void replay_advance_kernel(uint64_t* counter, int B) { counter[0] += uint64_t(B); }

// metadata unit m of the launch: 4-byte words of 4-byte-multiple columns,
// single bytes otherwise
__device__ __forceinline__ void replay_meta(const ReplayParams& r, const ReplayShared& sh, int B, int64_t m) {
  for (int k = 0; k < r.nmeta; ++k) {
    const int nb = r.meta_bytes[k];
    const int w = (nb % 4 == 0) ? 4 : 1;
    const int64_t per = nb / w, units = per * B;
    if (m < units) {
      const int b = int(m / per);
      const int64_t j = (m - int64_t(b) * per) * w;
      const uint8_t* s = r.meta_src[k] + sh.idx[b] * nb + j;
      uint8_t* d = r.meta_dst[k] + int64_t(b) * nb + j;
      if (w == 4) *reinterpret_cast<uint32_t*>(d) = *reinterpret_cast<const uint32_t*>(s);
      else *d = *s;
      return;
    }
    m -= units;
  }
}

template <int PPT, int CIN, int OUTT, int LAYOUT>
__global__ __launch_bounds__(kBlock) void replay_vec_kernel(DecodeParams p, ReplayParams r, int64_t meta_units) {
  __shared__ ReplayShared sh;
  const int64_t HW = int64_t(p.H) * p.W;
  const int64_t groups_per_img = HW / PPT;
  const int64_t groups = groups_per_img * p.B;
  const int cout = p.Cout;
  int cm[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) cm[c] = p.cmap[c];
  const int64_t stride = int64_t(gridDim.x) * kBlock;
  const bool small = groups + meta_units + stride < (int64_t(1) << 31);
  // Every lane draws the frame index of its own first group (the same Philox
  // word the block's table holds) and issues that group's pixel loads before
  // the LUT staging and the block barrier: the HBM latency of the first
  // loads overlaps the prologue instead of following it (one launch round
  // for a batch of 8).
  const uint64_t ctr = r.index_in ? 0 : (r.counter ? r.counter[0] : r.ctr_value);
  auto frame_of = [&](int b) -> int64_t {
    return r.index_in ? r.index_in[b]
                      : int64_t((uint64_t(philox_word(r.seed, ctr, uint32_t(b))) * uint64_t(r.count)) >> 32);
  };
  const int64_t g0 = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  Group gr0;
  Pixels<PPT, CIN> px0;
  if (g0 < groups) {
    int y, x;
    split_group<PPT>(g0, groups_per_img, p.W, small, gr0.b, gr0.q, y, x);
    const int sy = p.flip_all ? p.H - 1 - y : y;
    gr0.src = p.src + frame_of(gr0.b) * r.frame_bytes + (int64_t(sy) * p.W + x) * CIN;
    load_pixels<PPT, CIN>(gr0.src, px0);
  }
  const Xf xf = stage_xf(p.lut, sh.tab, p.Cout);
  for (int b = threadIdx.x; b < p.B; b += kBlock) {
    const int64_t i = frame_of(b);
    sh.idx[b] = i;
    if (blockIdx.x == 0 && r.index_out) r.index_out[b] = i;
  }
  __syncthreads();
  for (int64_t g = g0; g < groups + meta_units; g += stride) {
    if (g >= groups) {
      replay_meta(r, sh, p.B, g - groups);
      continue;
    }
    if (g == g0) {
      emit<PPT, CIN, OUTT, LAYOUT>(p, xf, cm, cout, HW, gr0, px0);
      continue;
    }
    Group gr;
    int y, x;
    split_group<PPT>(g, groups_per_img, p.W, small, gr.b, gr.q, y, x);
    const int sy = p.flip_all ? p.H - 1 - y : y;
    gr.src = p.src + sh.idx[gr.b] * r.frame_bytes + (int64_t(sy) * p.W + x) * CIN;
    Pixels<PPT, CIN> px;
    load_pixels<PPT, CIN>(gr.src, px);
    emit<PPT, CIN, OUTT, LAYOUT>(p, xf, cm, cout, HW, gr, px);
  }
}

// any shape / alignment: one pixel per lane
template <int OUTT>
__global__ __launch_bounds__(kBlock) void replay_scalar_kernel(DecodeParams p, ReplayParams r, int64_t meta_units) {
  __shared__ ReplayShared sh;
  const Xf xf = replay_prologue(p, r, sh);
  const int64_t HW = int64_t(p.H) * p.W;
  const int64_t total = HW * p.B;
  const int64_t ie = HW * p.Cout;
  for (int64_t g = int64_t(blockIdx.x) * kBlock + threadIdx.x; g < total + meta_units; g += int64_t(gridDim.x) * kBlock) {
    if (g >= total) {
      replay_meta(r, sh, p.B, g - total);
      continue;
    }
    const int b = int(g / HW);
    const int64_t q = g - int64_t(b) * HW;
    const int y = int(q / p.W), x = int(q - int64_t(y) * p.W);
    const int sy = p.flip_all ? p.H - 1 - y : y;
    const uint8_t* s = p.src + sh.idx[b] * r.frame_bytes + (int64_t(sy) * p.W + x) * p.Cin;
    for (int c = 0; c < p.Cout; ++c) {
      const float v = xf_value(xf, c, s[p.cmap[c]]);
      const int64_t off = p.layout == NCHW ? int64_t(c) * HW + q : q * p.Cout + c;
      if constexpr (OUTT == OUT_F32) reinterpret_cast<float*>(p.dst)[int64_t(b) * ie + off] = v;
      else if constexpr (OUTT == OUT_BF16) reinterpret_cast<uint16_t*>(p.dst)[int64_t(b) * ie + off] = f2bf(v);
      else if constexpr (OUTT == OUT_F16) reinterpret_cast<uint16_t*>(p.dst)[int64_t(b) * ie + off] = f2h(v);
      else reinterpret_cast<uint8_t*>(p.dst)[int64_t(b) * ie + off] = uint8_t(v);
    }
  }
}

template <int OUTT>
hipError_t launch_replay(const DecodeParams& p, const ReplayParams& r, int64_t meta_units, hipStream_t s) {
  constexpr int PPT = OUTT == OUT_F32 ? 4 : (OUTT == OUT_U8 ? 16 : 8);
  const bool vec = (p.W % PPT) == 0 && r.frame_bytes % 16 == 0 && (p.Cin == 3 || p.Cin == 4) &&
                   (reinterpret_cast<uintptr_t>(p.src) % 16) == 0 && (reinterpret_cast<uintptr_t>(p.dst) % 16) == 0 &&
                   (int64_t(p.H) * p.W * p.Cin) % 16 == 0;
  if (vec) {
    const int grid = grid_for(int64_t(p.B) * p.H * p.W / PPT + meta_units, p.max_grid);
#define BT_REPLAY(CIN, LAY) replay_vec_kernel<PPT, CIN, OUTT, LAY><<<grid, kBlock, 0, s>>>(p, r, meta_units)
    if (p.Cin == 4) {
      if (p.layout == NCHW) BT_REPLAY(4, NCHW);
      else BT_REPLAY(4, NHWC);
    } else {
      if (p.layout == NCHW) BT_REPLAY(3, NCHW);
      else BT_REPLAY(3, NHWC);
    }
#undef BT_REPLAY
  } else {
    replay_scalar_kernel<OUTT><<<grid_for(int64_t(p.B) * p.H * p.W + meta_units, p.max_grid), kBlock, 0, s>>>(
        p, r, meta_units);
  }
  return hipGetLastError();
}

}  // namespace

hipError_t replay_sample(const DecodeParams& p, const ReplayParams& r, hipStream_t stream) {
  if (p.B <= 0) return hipSuccess;
  if (p.B > kMaxReplayB || p.H <= 0 || p.W <= 0 || p.Cin < 1 || p.Cin > 4 || p.Cout < 1 || p.Cout > 4 || !p.src ||
      !p.dst || !p.lut || r.frame_bytes != int64_t(p.H) * p.W * p.Cin || r.nmeta < 0 || r.nmeta > kMaxMeta)
    return hipErrorInvalidValue;
  if (!r.index_in && (r.count < 1 || r.count > (int64_t(1) << 32))) return hipErrorInvalidValue;
  for (int c = 0; c < p.Cout; ++c)
    if (p.cmap[c] < 0 || p.cmap[c] >= p.Cin) return hipErrorInvalidValue;
  int64_t meta_units = 0;
  for (int k = 0; k < r.nmeta; ++k) {
    const int nb = r.meta_bytes[k];
    if (nb <= 0 || !r.meta_src[k] || !r.meta_dst[k]) return hipErrorInvalidValue;
    if (nb % 4 == 0 && ((reinterpret_cast<uintptr_t>(r.meta_src[k]) | reinterpret_cast<uintptr_t>(r.meta_dst[k])) % 4))
      return hipErrorInvalidValue;
    meta_units += int64_t(p.B) * (nb % 4 == 0 ? nb / 4 : nb);
  }
  hipError_t e = hipErrorInvalidValue;
  switch (p.out_dtype) {
    case OUT_F32: e = launch_replay<OUT_F32>(p, r, meta_units, stream); break;
    case OUT_BF16: e = launch_replay<OUT_BF16>(p, r, meta_units, stream); break;
    case OUT_F16: e = launch_replay<OUT_F16>(p, r, meta_units, stream); break;
    case OUT_U8: e = launch_replay<OUT_U8>(p, r, meta_units, stream); break;
  }
  if (e != hipSuccess || r.index_in || !r.counter) return e;
  replay_advance_kernel<<<1, 1, 0, stream>>>(r.counter, p.B);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// color4x4 on MFMA (v_mfma_f32_4x4x1_16b_f32)
// ---------------------------------------------------------------------------
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Each wave owns 256 consecutive pixels of one image per iteration.
// Operand map of the 16-block 4x4x1 MFMA (lane l = 4*blk + i):
//   A[row i][0] of block blk, B[0][col i] of block blk, D[reg r][col i].
// Row i of block blk at sub-step s (0..3) is pixel 64*i + 4*blk + s, so each
// lane's A operands over the four sub-steps are 4 consecutive pixels -> ONE
// 16-byte load.  K (input channel) accumulates over 4 MFMAs, B = M[i][k].
// Lane (blk, i) receives in reg r the output channel i of pixel
// 64*r + 4*blk + s; over s that is 4 consecutive pixels -> one float4 per
// reg, and for a fixed reg the 16 lanes of one channel cover 64 contiguous
// pixels: every store instruction writes four 256-byte plane runs.
__global__ __launch_bounds__(kBlock) void color4x4_kernel(Color4x4Params p) {
  __shared__ uint32_t tab[kTabWords];
  const Xf xf = stage_xf(p.lut, tab, 4);   // indexed by INPUT channel here
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int j = lane & 3;
  float bm[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) bm[k] = p.M[j * 4 + k];
  const float bj = p.bias[j];
  const int64_t HW = int64_t(p.H) * p.W;
  const int64_t segs_per_img = HW / 256;   // host guarantees HW % 256 == 0
  const int64_t total = segs_per_img * p.B;
  const int64_t stride = int64_t(gridDim.x) * (kBlock / 64);
  for (int64_t g = int64_t(blockIdx.x) * (kBlock / 64) + wave; g < total; g += stride) {
    const int b = int(g / segs_per_img);
    const int64_t q0 = (g - int64_t(b) * segs_per_img) * 256;
    // lane's 4 pixels share a row (W % 4 == 0); the segment may span rows
    const int blk = lane >> 2;
    const int64_t pl = q0 + 64 * j + 4 * blk;
    const int y = int(pl / p.W), x = int(pl - int64_t(y) * p.W);
    const bool flip = p.flip_all || (p.flip && p.flip[b]) || (b < 256 && ((p.flip_bits[b >> 6] >> (b & 63)) & 1));
    const int sy = flip ? p.H - 1 - y : y;
    const uint8_t* img = p.nsrcs ? p.srcs[b] : p.src + (p.src_offsets ? p.src_offsets[b] : int64_t(b) * HW * 4);
    const uint4 v4 = *reinterpret_cast<const uint4*>(img + (int64_t(sy) * p.W + x) * 4);
    const uint32_t w[4] = {v4.x, v4.y, v4.z, v4.w};
    f32x4 acc[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const uint32_t px = w[s];
      const float a0 = xf_value(xf, 0, px & 0xff), a1 = xf_value(xf, 1, (px >> 8) & 0xff);
      const float a2 = xf_value(xf, 2, (px >> 16) & 0xff), a3 = xf_value(xf, 3, px >> 24);
      f32x4 c = {bj, bj, bj, bj};
      c = __builtin_amdgcn_mfma_f32_4x4x1f32(a0, bm[0], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_4x4x1f32(a1, bm[1], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_4x4x1f32(a2, bm[2], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_4x4x1f32(a3, bm[3], c, 0, 0, 0);
      acc[s] = c;
    }
    if (j < p.Cout) {
      // pixel 64*r + 4*blk + s  <-  acc[s][r]
      float* d = image_out<float>(p, b, HW * p.Cout) + int64_t(j) * HW + q0 + 4 * blk;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        *reinterpret_cast<float4*>(d + 64 * r) = make_float4(acc[0][r], acc[1][r], acc[2][r], acc[3][r]);
    }
  }
}

__global__ void project_kernel(const float* pts, int64_t N, const float* PV, const float* V, int W, int H,
                               int upper_left, float* out_px, float* out_depth) {
  __shared__ float m[32];
  if (threadIdx.x < 16) m[threadIdx.x] = PV[threadIdx.x];
  else if (threadIdx.x < 32) m[threadIdx.x] = V[threadIdx.x - 16];
  __syncthreads();
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < N; i += int64_t(gridDim.x) * blockDim.x) {
    const float x = pts[3 * i], y = pts[3 * i + 1], z = pts[3 * i + 2];
    float c[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) c[r] = m[4 * r] * x + m[4 * r + 1] * y + m[4 * r + 2] * z + m[4 * r + 3];
    const float nx = c[0] / c[3], ny = c[1] / c[3];
    float px = (nx + 1.f) * 0.5f, py = (ny + 1.f) * 0.5f;
    if (upper_left) py = 1.f - py;
    out_px[2 * i] = px * W;
    out_px[2 * i + 1] = py * H;
    if (out_depth) out_depth[i] = -(m[16 + 8] * x + m[16 + 9] * y + m[16 + 10] * z + m[16 + 11]);
  }
}

}  // namespace

hipError_t color4x4(const Color4x4Params& p, hipStream_t stream) {
  if (p.B <= 0) return hipSuccess;
  if ((int64_t(p.H) * p.W) % 256 != 0 || p.W % 4 != 0 || p.Cout < 1 || p.Cout > 4 ||
      (p.ndsts ? !dsts_ok(p.dsts, p.ndsts, p.B, 16) : (reinterpret_cast<uintptr_t>(p.dst) % 16) != 0) ||
      (p.nsrcs ? !srcs_ok(p.srcs, p.nsrcs, p.B, 16) : (reinterpret_cast<uintptr_t>(p.src) % 16) != 0))
    return hipErrorInvalidValue;
  int64_t waves = int64_t(p.B) * p.H * p.W / 256;
  int64_t blocks = (waves + 3) / 4;
  int grid = int(blocks < 4096 ? blocks : 4096);
  color4x4_kernel<<<grid, kBlock, 0, stream>>>(p);
  return hipGetLastError();
}

hipError_t project(const float* pts, int64_t N, const float* PV, const float* V, int W, int H, int upper_left,
                   float* out_px, float* out_depth, hipStream_t stream) {
  if (N <= 0) return hipSuccess;
  int64_t blocks = (N + kBlock - 1) / kBlock;
  int grid = int(blocks < 1024 ? blocks : 1024);
  project_kernel<<<grid, kBlock, 0, stream>>>(pts, N, PV, V, W, H, upper_left, out_px, out_depth);
  return hipGetLastError();
}

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
                                                           float slope, float* __restrict__ partial) {
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
    // channel-major [2C][blocks]: the fold reads each channel's partials contiguously
    partial[int64_t(c) * gridDim.x + blockIdx.x] = a;
    partial[int64_t(C + c) * gridDim.x + blockIdx.x] = q2;
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

template <int DT, bool BWD>
__global__ __launch_bounds__(kBlock) void bn_apply_kernel(const void* __restrict__ x, const void* __restrict__ gy,
                                                          void* __restrict__ out, int64_t M, int C,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          const float* __restrict__ w, const float* __restrict__ b,
                                                          const float* __restrict__ dw, const float* __restrict__ db,
                                                          float slope) {
  constexpr int V = BnVec<DT>::V, U = kBnUnroll;
  const int G = C / V;
  const int64_t total = M * G;
  const float invM = 1.f / float(M);
  const int c0 = (int(threadIdx.x) % G) * V;
  // xhat = v * is + nm;  z = xhat * ww + bb;  backward: gx = P * (gz - dbm) - pdw * xhat
  float is[V], nm[V], ww[V], bb[V], P[V], dbm[V], pdw[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = c0 + i;
    is[i] = invstd[c];
    nm[i] = -mean[c] * is[i];
    ww[i] = w[c];
    bb[i] = b[c];
    if constexpr (BWD) {
      P[i] = ww[i] * is[i];
      dbm[i] = db[c] * invM;
      pdw[i] = P[i] * dw[c] * invM;
    }
  }
  auto apply = [&](const float (&v)[V], const float (&gv)[V], float (&o)[V]) {
    if constexpr (BWD) {
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const float xh = fmaf(v[i], is[i], nm[i]);
        const float gz = fmaf(xh, ww[i], bb[i]) > 0.f ? gv[i] : gv[i] * slope;
        o[i] = fmaf(P[i], gz - dbm[i], -pdw[i] * xh);
      }
    } else {
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const float z = fmaf(fmaf(v[i], is[i], nm[i]), ww[i], bb[i]);
        o[i] = z > 0.f ? z : z * slope;
      }
    }
  };
  const int64_t pass = int64_t(gridDim.x) * kBlock * U;
  int64_t idx = int64_t(blockIdx.x) * kBlock * U + threadIdx.x;
  for (; idx + (U - 1) * kBlock < total; idx += pass) {   // whole passes: U loads in flight
    float v[U][V], gv[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      bn_load<DT>(x, (idx + u * kBlock) * V, v[u]);
      if constexpr (BWD) bn_load<DT>(gy, (idx + u * kBlock) * V, gv[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float o[V];
      apply(v[u], gv[u], o);
      bn_store<DT>(out, (idx + u * kBlock) * V, o);
    }
  }
  for (; idx < total; idx += kBlock) {   // the tail: at most U - 1 vectors per lane
    float v[V], gv[V], o[V];
    bn_load<DT>(x, idx * V, v);
    if constexpr (BWD) bn_load<DT>(gy, idx * V, gv);
    apply(v, gv, o);
    bn_store<DT>(out, idx * V, o);
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

int bn_grid(int64_t work) {   // work = 16-byte vectors; kBnUnroll per lane per pass
  const int64_t blocks = (work + kBlock * kBnUnroll - 1) / (kBlock * kBnUnroll);
  return int(blocks < 4096 ? (blocks < 1 ? 1 : blocks) : 4096);
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
// kernel's blocks all read a value no block is writing.
__global__ void adam_schedule_kernel(float* step, const float* hp, float* sched, float beta1, float beta2,
                                     const float* gate) {
  if (threadIdx.x != 0) return;
  // a closed gate (gate[0] == 0, computed on the device earlier in the same
  // stream/graph) makes the whole step a no-op: counter, moments and weights
  const bool active = !gate || gate[0] != 0.f;
  sched[4] = active ? 1.f : 0.f;
  if (!active) return;
  const float s = step[0] + 1.f;
  step[0] = s;
  const float lr = hp[0];
  const double bc1 = 1.0 - pow(double(beta1), double(s));
  const double bc2 = 1.0 - pow(double(beta2), double(s));
  sched[0] = float(double(lr) / bc1);
  sched[1] = float(1.0 / sqrt(bc2));
  sched[2] = lr;
  sched[3] = hp[1];   // gradient scale (e.g. 1 / world after a summing all-reduce)
}

template <bool GBF16>
__global__ __launch_bounds__(kBlock) void adam_update_kernel(AdamParams a) {
  const int64_t q = int64_t(blockIdx.x) * kBlock + threadIdx.x;   // 4-element group
  if (q >= a.gstart[a.n] || a.sched[4] == 0.f) return;
  int k = 0;
  while (q >= a.gstart[k + 1]) ++k;     // <= kMaxAdam compares, mostly uniform across a wave
  const int64_t e0 = (q - a.gstart[k]) * 4;
  const int64_t n = a.numel[k];
  const float step_size = a.sched[0], inv_bc2 = a.sched[1], lr = a.sched[2], gscale = a.sched[3];
  const float b1 = a.beta1, b2 = a.beta2, wd = a.weight_decay;
  float* P = a.p[k];
  float* M = a.m[k];
  float* V = a.v[k];
  float pv[4], gv[4], mv[4], vv[4];
  const bool full = e0 + 4 <= n;   // tensors are 16-byte aligned (host-checked), so a full group is one dwordx4
  if (full) {
    const float4 p4 = *reinterpret_cast<const float4*>(P + e0);
    const float4 m4 = *reinterpret_cast<const float4*>(M + e0);
    const float4 v4 = *reinterpret_cast<const float4*>(V + e0);
    pv[0] = p4.x, pv[1] = p4.y, pv[2] = p4.z, pv[3] = p4.w;
    mv[0] = m4.x, mv[1] = m4.y, mv[2] = m4.z, mv[3] = m4.w;
    vv[0] = v4.x, vv[1] = v4.y, vv[2] = v4.z, vv[3] = v4.w;
    if constexpr (GBF16) {
      const uint2 g2 = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(a.g[k]) + e0);
      gv[0] = __uint_as_float(g2.x << 16), gv[1] = __uint_as_float(g2.x & 0xFFFF0000u);
      gv[2] = __uint_as_float(g2.y << 16), gv[3] = __uint_as_float(g2.y & 0xFFFF0000u);
    } else {
      const float4 g4 = *reinterpret_cast<const float4*>(static_cast<const float*>(a.g[k]) + e0);
      gv[0] = g4.x, gv[1] = g4.y, gv[2] = g4.z, gv[3] = g4.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool in = e0 + j < n;
      pv[j] = in ? P[e0 + j] : 0.f;
      mv[j] = in ? M[e0 + j] : 0.f;
      vv[j] = in ? V[e0 + j] : 0.f;
      if constexpr (GBF16)
        gv[j] = in ? __uint_as_float(uint32_t(static_cast<const uint16_t*>(a.g[k])[e0 + j]) << 16) : 0.f;
      else
        gv[j] = in ? static_cast<const float*>(a.g[k])[e0 + j] : 0.f;
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float g = (a.maximize ? -gv[j] : gv[j]) * gscale;
    if (wd != 0.f) {
      if (a.decoupled) pv[j] *= 1.f - lr * wd;
      else g += wd * pv[j];
    }
    mv[j] = b1 * mv[j] + (1.f - b1) * g;
    vv[j] = b2 * vv[j] + (1.f - b2) * g * g;
    pv[j] -= step_size * mv[j] / (sqrtf(vv[j]) * inv_bc2 + a.eps);
  }
  uint16_t* S = a.shadow[k];
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
}

}  // namespace

hipError_t adam_schedule(float* step, const float* hp, float* sched, float beta1, float beta2, hipStream_t stream,
                         const float* gate) {
  if (!step || !hp || !sched) return hipErrorInvalidValue;
  adam_schedule_kernel<<<1, 64, 0, stream>>>(step, hp, sched, beta1, beta2, gate);
  return hipGetLastError();
}

hipError_t adam_update(const AdamParams& p, hipStream_t stream) {
  if (p.n <= 0) return hipSuccess;
  if (p.n > kMaxAdam || !p.sched) return hipErrorInvalidValue;
  if (p.gstart[0] != 0) return hipErrorInvalidValue;
  for (int k = 0; k < p.n; ++k) {
    if (p.numel[k] < 0 || p.gstart[k + 1] - p.gstart[k] != (p.numel[k] + 3) / 4) return hipErrorInvalidValue;
    if (p.numel[k] > 0 && (!p.p[k] || !p.g[k] || !p.m[k] || !p.v[k])) return hipErrorInvalidValue;
    // full groups are read and written as 16-byte (8-byte for bf16) vectors
    const uintptr_t mis = reinterpret_cast<uintptr_t>(p.p[k]) | reinterpret_cast<uintptr_t>(p.m[k]) |
                          reinterpret_cast<uintptr_t>(p.v[k]) |
                          (reinterpret_cast<uintptr_t>(p.g[k]) << (p.grad_bf16 ? 1 : 0)) |
                          (reinterpret_cast<uintptr_t>(p.shadow[k]) << 1);
    if (mis & 15) return hipErrorInvalidValue;
  }
  const int64_t groups = p.gstart[p.n];
  if (groups == 0) return hipSuccess;
  const int64_t blocks = (groups + kBlock - 1) / kBlock;
  if (blocks > int64_t(1) << 30) return hipErrorInvalidValue;
  if (p.grad_bf16) adam_update_kernel<true><<<unsigned(blocks), kBlock, 0, stream>>>(p);
  else adam_update_kernel<false><<<unsigned(blocks), kBlock, 0, stream>>>(p);
  return hipGetLastError();
}

}  // namespace gpu
}  // namespace btn
