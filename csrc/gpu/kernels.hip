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

// PPT pixels of CIN u8 channels as 32-bit words; byte j is read by shifts (j a compile-time index
// in every use).  (A byte array written through 16-byte stores and read bytewise was kept on the
// stack in the replay kernels: 64-272 bytes of scratch per lane.)
template <int PPT, int CIN>
struct Pixels {
  static constexpr int NW = (PPT * CIN + 3) / 4;
  uint32_t w[NW];
  __device__ __forceinline__ uint32_t v(int j) const { return (w[j >> 2] >> (8 * (j & 3))) & 0xFFu; }
};

// Load PPT pixels (PPT*CIN bytes) with the widest aligned accesses.
template <int PPT, int CIN>
__device__ __forceinline__ void load_pixels(const uint8_t* p, Pixels<PPT, CIN>& px) {
  constexpr int NB = PPT * CIN;
  if constexpr (NB % 16 == 0) {
#pragma unroll
    for (int i = 0; i < NB / 16; ++i) {
      const uint4 q = reinterpret_cast<const uint4*>(p)[i];
      px.w[4 * i] = q.x, px.w[4 * i + 1] = q.y, px.w[4 * i + 2] = q.z, px.w[4 * i + 3] = q.w;
    }
  } else if constexpr (NB % 8 == 0) {
#pragma unroll
    for (int i = 0; i < NB / 8; ++i) {
      const uint2 q = reinterpret_cast<const uint2*>(p)[i];
      px.w[2 * i] = q.x, px.w[2 * i + 1] = q.y;
    }
  } else {
#pragma unroll
    for (int i = 0; i < NB / 4; ++i) px.w[i] = reinterpret_cast<const uint32_t*>(p)[i];
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
    // every load first (4 x 256 threads cover the 4 x 256 table): a
    // load-store loop waited out one round trip per 256 entries
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = int(threadIdx.x) + u * int(blockDim.x);
      v[u] = T[i < nch * 256 ? i : 0];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = int(threadIdx.x) + u * int(blockDim.x);
      if (i < nch * 256) reinterpret_cast<float*>(tab)[i] = v[u];
    }
    for (int i = int(threadIdx.x) + 4 * int(blockDim.x); i < nch * 256; i += blockDim.x)   // (blocks < 256 threads)
      reinterpret_cast<float*>(tab)[i] = T[i];
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
template <int PPT, int CIN, int IC, int TBL = 0>
__device__ __forceinline__ void lookup_static(const Pixels<PPT, CIN>& px, const Xf& xf, int c, float (&o)[PPT]) {
  if constexpr (TBL == 2) {   // one table for every output channel, 32 copies: xf.lut is this lane's copy
#pragma unroll
    for (int i = 0; i < PPT; ++i) o[i] = xf.lut[px.v(i * CIN + IC) * 32u];
    return;
  }
  if (TBL || !xf.arith) {   // TBL: the host promised a table-mode value table (no arithmetic code at all)
    const float* l = xf.lut + c * 256;
#pragma unroll
    for (int i = 0; i < PPT; ++i) o[i] = l[px.v(i * CIN + IC)];
    return;
  }
  float x[PPT];
  if (xf.gam[c]) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const uint32_t v = px.v(i * CIN + IC);
      x[i] = float(xf.g[((v >> 2) << xf.gshift) + (v & 3)]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < PPT; ++i) x[i] = float(px.v(i * CIN + IC));
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

template <int PPT, int CIN, int TBL = 0>
__device__ __forceinline__ void lookup(const Pixels<PPT, CIN>& px, int ic, const Xf& xf, int c, float (&o)[PPT]) {
  switch (ic) {
    case 0: lookup_static<PPT, CIN, 0, TBL>(px, xf, c, o); break;
    case 1: if constexpr (CIN > 1) lookup_static<PPT, CIN, 1, TBL>(px, xf, c, o); break;
    case 2: if constexpr (CIN > 2) lookup_static<PPT, CIN, 2, TBL>(px, xf, c, o); break;
    default: if constexpr (CIN > 3) lookup_static<PPT, CIN, 3, TBL>(px, xf, c, o); break;
  }
}

template <int PPT, int CIN, int OUTT, int COUT, int TBL = 0>
__device__ __forceinline__ void store_nhwc(const DecodeParams& p, const Xf& xf, const int* cm,
                                           const Pixels<PPT, CIN>& px, int b, int64_t q, int64_t HW) {
  constexpr int N = PPT * COUT;
  const int64_t off = q * COUT;   // within image b (NHWC)
  float v[COUT][PPT];
#pragma unroll
  for (int c = 0; c < COUT; ++c) lookup<PPT, CIN, TBL>(px, cm[c], xf, c, v[c]);
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

// NT: streaming (non-temporal) stores -- output written once and read by a
// later kernel, kept out of the L2's write-back set (replay sample A/B)
template <int PPT, int CIN, int OUTT, int LAYOUT, int TBL = 0, bool NT = false>
__device__ __forceinline__ void emit(const DecodeParams& p, const Xf& xf, const int* cm, int cout, int64_t HW,
                                     const Group& gr, const Pixels<PPT, CIN>& px) {
  const int b = gr.b;
  const int64_t q = gr.q;
  if constexpr (LAYOUT == NCHW) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c >= cout) break;
      float v[PPT];
      lookup<PPT, CIN, TBL>(px, cm[c], xf, c, v);
      const int64_t off = int64_t(c) * HW + q;   // within image b (NCHW)
      if constexpr (OUTT == OUT_F32) {
        float* d = image_out<float>(p, b, HW * cout) + off;
        if constexpr (NT) {
          typedef float f4v __attribute__((ext_vector_type(4)));
#pragma unroll
          for (int i = 0; i < PPT / 4; ++i)
            __builtin_nontemporal_store(f4v{v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]},
                                        reinterpret_cast<f4v*>(d) + i);
        } else {
#pragma unroll
          for (int i = 0; i < PPT / 4; ++i) reinterpret_cast<float4*>(d)[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
        }
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
      case 1: store_nhwc<PPT, CIN, OUTT, 1, TBL>(p, xf, cm, px, b, q, HW); break;
      case 2: store_nhwc<PPT, CIN, OUTT, 2, TBL>(p, xf, cm, px, b, q, HW); break;
      case 3: store_nhwc<PPT, CIN, OUTT, 3, TBL>(p, xf, cm, px, b, q, HW); break;
      default: store_nhwc<PPT, CIN, OUTT, 4, TBL>(p, xf, cm, px, b, q, HW); break;
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
template <int TW>
struct ReplaySharedT {
  uint32_t tab[TW];
  uint32_t idx[kMaxReplayB];   // frame indices (< 2^32: replay_sample checks the count)
  uint64_t ctr;
};
using ReplayShared = ReplaySharedT<kTabWords>;

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
template <class Shared>
__device__ __forceinline__ void replay_meta(const ReplayParams& r, const Shared& sh, int B, int64_t m) {
  for (int k = 0; k < r.nmeta; ++k) {
    const int nb = r.meta_bytes[k];
    const int w = (nb % 4 == 0) ? 4 : 1;
    const int64_t per = nb / w, units = per * B;
    if (m < units) {
      const int b = int(m / per);
      const int64_t j = (m - int64_t(b) * per) * w;
      const uint8_t* s = r.meta_src[k] + int64_t(sh.idx[b]) * nb + j;
      uint8_t* d = r.meta_dst[k] + int64_t(b) * nb + j;
      if (w == 4) *reinterpret_cast<uint32_t*>(d) = *reinterpret_cast<const uint32_t*>(s);
      else *d = *s;
      return;
    }
    m -= units;
  }
}

// TBL: the value table is in table mode (p.xf_table_only): the lookups are
// plain LDS reads and the kernel carries none of the arithmetic-form code
// (whose registers cut the general kernel to 4 waves per SIMD).  TBL 2: every
// output channel has the same table (xf_table_only 2) -- staged as 32 copies
// interleaved by word, [value][copy], and lane l reads copy l % 32: the 32
// lanes of a ds_read group always hit 32 distinct banks (one 1 KiB table read
// at random bytes ran ~3.4-way conflicted)
constexpr int kUniWords = 256 * 32;
constexpr int kUniU = 4;   // groups in flight per lane (TBL 2)
template <int PPT, int CIN, int OUTT, int LAYOUT, int TBL, bool NT = false>
__global__ __launch_bounds__(kBlock) void replay_vec_kernel(DecodeParams p, ReplayParams r, int64_t meta_units) {
  __shared__ ReplaySharedT<TBL == 2 ? kUniWords : kTabWords> sh;
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
  // TBL 2 runs a grid of few blocks (the table staging is per block): each
  // lane keeps kUniU groups' loads in flight per pass
  Group gru[kUniU];
  Pixels<PPT, CIN> pxu[kUniU];
#define BT_UNI_ISSUE(GB, FIRST)                                                                   \
  _Pragma("unroll") for (int u = 0; u < kUniU; ++u) {                                             \
    const int64_t g_ = (GB) + u * stride;                                                         \
    int y_ = 0, x_ = 0;                                                                           \
    split_group<PPT>(g_ < groups ? g_ : 0, groups_per_img, p.W, small, gru[u].b, gru[u].q, y_, x_); \
    const int sy_ = p.flip_all ? p.H - 1 - y_ : y_;                                               \
    const int64_t fi_ = (FIRST) ? frame_of(gru[u].b) : int64_t(sh.idx[gru[u].b]);                \
    gru[u].src = p.src + fi_ * r.frame_bytes + (int64_t(sy_) * p.W + x_) * CIN;                   \
    load_pixels<PPT, CIN>(gru[u].src, pxu[u]);                                                    \
  }
  // (a group past the end re-reads group 0 and is not emitted: no branch around the loads)
  if constexpr (TBL == 2) {
    BT_UNI_ISSUE(g0, true)
  } else if (g0 < groups) {
    int y, x;
    split_group<PPT>(g0, groups_per_img, p.W, small, gr0.b, gr0.q, y, x);
    const int sy = p.flip_all ? p.H - 1 - y : y;
    gr0.src = p.src + frame_of(gr0.b) * r.frame_bytes + (int64_t(sy) * p.W + x) * CIN;
    load_pixels<PPT, CIN>(gr0.src, px0);
  }
  Xf xf;
  if constexpr (TBL == 2) {
    // header scalars as stage_xf reads them; the table expanded into its 32
    // copies (word w = 32 value + copy: consecutive lanes, consecutive words)
    xf.arith = 0;
    float v[kUniWords / kBlock];
#pragma unroll
    for (int i = 0; i < kUniWords / kBlock; ++i) v[i] = p.lut[(int(threadIdx.x) + kBlock * i) >> 5];
#pragma unroll
    for (int i = 0; i < kUniWords / kBlock; ++i) sh.tab[int(threadIdx.x) + kBlock * i] = __float_as_uint(v[i]);
    xf.lut = reinterpret_cast<const float*>(sh.tab) + (threadIdx.x & 31);
  } else {
    xf = stage_xf(p.lut, sh.tab, p.Cout);
  }
  for (int b = threadIdx.x; b < p.B; b += kBlock) {
    const int64_t i = frame_of(b);
    sh.idx[b] = i;
    if (blockIdx.x == 0 && r.index_out) r.index_out[b] = i;
  }
  __syncthreads();
  if constexpr (TBL == 2) {
    for (int64_t gb = g0; gb < groups; gb += kUniU * stride) {
      if (gb != g0) {
        BT_UNI_ISSUE(gb, false)
      }
#pragma unroll
      for (int u = 0; u < kUniU; ++u)
        if (gb + u * stride < groups) emit<PPT, CIN, OUTT, LAYOUT, TBL, NT>(p, xf, cm, cout, HW, gru[u], pxu[u]);
    }
    for (int64_t g = g0; g < groups + meta_units; g += stride)
      if (g >= groups) replay_meta(r, sh, p.B, g - groups);
    return;
  }
#undef BT_UNI_ISSUE
  for (int64_t g = g0; g < groups + meta_units; g += stride) {
    if (g >= groups) {
      replay_meta(r, sh, p.B, g - groups);
      continue;
    }
    if (g == g0) {
      emit<PPT, CIN, OUTT, LAYOUT, TBL, NT>(p, xf, cm, cout, HW, gr0, px0);
      continue;
    }
    Group gr;
    int y, x;
    split_group<PPT>(g, groups_per_img, p.W, small, gr.b, gr.q, y, x);
    const int sy = p.flip_all ? p.H - 1 - y : y;
    gr.src = p.src + int64_t(sh.idx[gr.b]) * r.frame_bytes + (int64_t(sy) * p.W + x) * CIN;
    Pixels<PPT, CIN> px;
    load_pixels<PPT, CIN>(gr.src, px);
    emit<PPT, CIN, OUTT, LAYOUT, TBL, NT>(p, xf, cm, cout, HW, gr, px);
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
    const uint8_t* s = p.src + int64_t(sh.idx[b]) * r.frame_bytes + (int64_t(sy) * p.W + x) * p.Cin;
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
    int grid = grid_for(int64_t(p.B) * p.H * p.W / PPT + meta_units, p.max_grid);
    // fp32 NCHW table-mode output through non-temporal stores: batch 64 of
    // 640x480 58.5 us against 62.8 (profiles/r5/b6; BT_REPLAY_NT=0: plain stores)
    static const bool nt_env = !(std::getenv("BT_REPLAY_NT") && std::getenv("BT_REPLAY_NT")[0] == '0');
    const bool nt = nt_env && OUTT == OUT_F32 && p.layout == NCHW && p.xf_table_only;
    // one table for all channels (xf_table_only 2): the 32-copy conflict-free
    // form with BT_REPLAY_UNI=1 -- 0 % bank conflicts (PMC) but 83.4 us against
    // 58.4 per batch of 64 (profiles/r5/b8): its 32 KiB table per block halves
    // the resident waves and every one of the 8192 blocks stages it
    static const bool uni_env = std::getenv("BT_REPLAY_UNI") && std::getenv("BT_REPLAY_UNI")[0] == '1';
    const bool uni = uni_env && p.xf_table_only == 2;
    if (uni && p.max_grid <= 0) {   // 4 blocks per CU, the table staged once per block (BT_REPLAY_UNI_GRID)
      static const int ug = std::getenv("BT_REPLAY_UNI_GRID") ? std::atoi(std::getenv("BT_REPLAY_UNI_GRID")) : 1024;
      grid = std::min(grid, ug > 0 ? ug : 1024);
    }
#define BT_REPLAY(CIN, LAY)                                                                  \
  do {                                                                                       \
    if (uni && nt) replay_vec_kernel<PPT, CIN, OUTT, LAY, 2, true><<<grid, kBlock, 0, s>>>(p, r, meta_units); \
    else if (uni) replay_vec_kernel<PPT, CIN, OUTT, LAY, 2><<<grid, kBlock, 0, s>>>(p, r, meta_units); \
    else if (nt) replay_vec_kernel<PPT, CIN, OUTT, LAY, 1, true><<<grid, kBlock, 0, s>>>(p, r, meta_units); \
    else if (p.xf_table_only) replay_vec_kernel<PPT, CIN, OUTT, LAY, 1><<<grid, kBlock, 0, s>>>(p, r, meta_units); \
    else replay_vec_kernel<PPT, CIN, OUTT, LAY, 0><<<grid, kBlock, 0, s>>>(p, r, meta_units);               \
  } while (0)
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
// Row j (output channel) of image b's affine transform, by p.mat_mode.
__device__ __forceinline__ void color_row(const Color4x4Params& p, int b, int j, float bm[4], float& bj) {
  if (p.mat_mode == kColorJitter) {
    const float br = p.jit[b][0], c = p.jit[b][1], s = p.jit[b][2];
    float sn, cs;
    __sincosf(6.283185307179586f * p.jit[b][3], &sn, &cs);
    // row j of the hue rotation about the grey axis (rows sum to 1)
    float h0, h1, h2;
    if (j == 0) h0 = 0.213f + cs * 0.787f - sn * 0.213f, h1 = 0.715f - cs * 0.715f - sn * 0.715f,
                h2 = 0.072f - cs * 0.072f + sn * 0.928f;
    else if (j == 1) h0 = 0.213f - cs * 0.213f + sn * 0.143f, h1 = 0.715f + cs * 0.285f + sn * 0.140f,
                     h2 = 0.072f - cs * 0.072f - sn * 0.283f;
    else h0 = 0.213f - cs * 0.213f - sn * 0.787f, h1 = 0.715f - cs * 0.715f + sn * 0.715f,
         h2 = 0.072f + cs * 0.928f + sn * 0.072f;
    // (Hue . Sat)[j][k] = s * Hue[j][k] + (1 - s) * w[k]  (Hue's rows sum to 1)
    const float bc = br * c, t = 1.f - s;
    if (j < 3) {
      bm[0] = bc * (s * h0 + t * 0.213f), bm[1] = bc * (s * h1 + t * 0.715f), bm[2] = bc * (s * h2 + t * 0.072f);
      bm[3] = 0.f;
      bj = (1.f - c) * p.pivot;
    } else {
      bm[0] = bm[1] = bm[2] = 0.f, bm[3] = 1.f, bj = 0.f;
    }
    return;
  }
  const float* M = p.mat_mode == kColorPos ? p.Ms + 20 * int(p.mat_pos[b])
                   : p.mat_mode == kColorEach ? p.Ms + 20 * int64_t(b) : p.M;
  const float* bias = p.mat_mode == kColorOne ? p.bias : M + 16;
#pragma unroll
  for (int k = 0; k < 4; ++k) bm[k] = M[j * 4 + k];
  bj = bias[j];
}

__global__ __launch_bounds__(kBlock) void color4x4_kernel(Color4x4Params p) {
  __shared__ uint32_t tab[kTabWords];
  const Xf xf = stage_xf(p.lut, tab, 4);   // indexed by INPUT channel here
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int j = lane & 3;
  float bm[4];
  float bj = 0.f;
  int mat_b = -1;   // the image whose matrix row bm / bj hold
  const int64_t HW = int64_t(p.H) * p.W;
  const int64_t segs_per_img = HW / 256;   // host guarantees HW % 256 == 0
  const int64_t total = segs_per_img * p.B;
  const int64_t stride = int64_t(gridDim.x) * (kBlock / 64);
  for (int64_t g = int64_t(blockIdx.x) * (kBlock / 64) + wave; g < total; g += stride) {
    const int b = int(g / segs_per_img);
    const int64_t q0 = (g - int64_t(b) * segs_per_img) * 256;
    if (b != mat_b) {   // wave-uniform: a new image's row j of its transform
      mat_b = b;
      color_row(p, b, j, bm, bj);
    }
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
  if ((p.mat_mode == kColorPos || p.mat_mode == kColorJitter) && p.B > kMaxSrcs) return hipErrorInvalidValue;
  if ((p.mat_mode == kColorPos || p.mat_mode == kColorEach) && !p.Ms) return hipErrorInvalidValue;
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

}  // namespace gpu
}  // namespace btn
