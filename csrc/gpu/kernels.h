// gfx950 (CDNA4) kernels for the blendtorch image path.  Host-callable
// launchers; every pointer is a device pointer, every launch is async on the
// given stream.
//
// The ops are the array ops the reference performs with numpy on the CPU
// (SURVEY.md §2.5):
//   * K-flip   np.flipud to upper-left origin      (btb/offscreen.py:95-96)
//   * K-gamma  u8(255*(x/255)^(1/g)) on RGB        (btb/offscreen.py:105-112)
//   * K-unpack RGBA -> RGB channel select          (btb/offscreen.py:57-62)
//   * K-normalize + HWC->CHW                       (examples/densityopt/densityopt.py:117-119)
//   * K-collate (stack B items)                    (torch default_collate)
// fused into ONE pass (`decode`), plus a per-pixel 4x4 colour transform on
// the matrix cores (`color4x4`) and batched pinhole projection (`project`,
// btb/camera.py:84-162).
#pragma once

#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace btn {
namespace gpu {

enum OutDType : int { OUT_F32 = 0, OUT_BF16 = 1, OUT_F16 = 2, OUT_U8 = 3 };
enum Layout : int { NCHW = 0, NHWC = 1 };

// Decode a batch of B u8 HWC images into a float/bf16/f16/u8 tensor.
//   src         B images; image b starts at src + src_offsets[b] (bytes) when
//               src_offsets != nullptr (device int64[B]: a gather, e.g. random
//               replay from an HBM-resident frame store), else at src + b*H*W*Cin.
//   src_offsets_aligned  caller's promise that every src_offsets[b] is a
//               multiple of 16 (frame-strided stores): keeps the vector path.
//   lut         device value table (kTableFloats floats, layout below): for
//               every (output channel c, input u8 v) the fp32 value, plus an
//               arithmetic form of the same table the kernels use instead of
//               reading 1-KiB fp32 tables from LDS:
//                 x = gamma[v] (channels fed by colour inputs when a gamma is
//                     set) or v, then per channel one of
//                 op 0: fma(x, a, b)   op 1: x*a - b   op 2: (x*a - b) / d
//                 op 3: t = x*a - b, q = t*r, fma(fma(-q, d, t), r, q)
//                 (each operation rounded separately, like numpy's float32;
//                 csrc/codec/xform_fit.h).
//               The host picks, per channel, an op it has VERIFIED to
//               reproduce the fp32 table bit for bit for all 256 inputs
//               (blendtorch.ops.build_table); mode 0 keeps the table lookup.
//               The gamma bytes sit in LDS as a lane-private table (each of
//               the 32 lanes of a ds_read_b32 group reads its own bank), so
//               the data-dependent lookup is free of bank conflicts; without
//               a gamma nothing is read from LDS at all.
//   cmap[c]     input channel feeding output channel c (c < Cout).
//   flip        nullable device u8[B]; 1 = image stored lower-left (GL order).
//   flip_all    applies to every image (OR-ed with flip[b]).
//   flip_bits   per-image flip bitmask for b < 256 (kernel-argument copy, so
//               the stream loader needs no per-batch flag upload).
//   srcs[b]     when nsrcs == B: per-image source pointers (kernel-argument
//               copy).  They may point at pinned / registered HOST memory: the
//               kernel then streams the frames over PCIe itself (zero-copy
//               fused read, no staging copy and no DMA-engine round).
//   max_grid    0: default grid cap; >0 overrides it (launch-shape sweeps).
constexpr int kMaxSrcs = 64;
// value-table layout (floats): [0, 1024) fp32 table [4][256]; header at
// kXfHeader: mode, gamma_used, gam[4], op[4], a[4], b[4], d[4], r[4]; gamma u8[256]
// packed little-endian at kXfGamma (64 floats' worth of bytes)
constexpr int kXfHeader = 1024;
constexpr int kXfGamma = 1088;
constexpr int kTableFloats = 1152;
struct DecodeParams {
  const uint8_t* src = nullptr;
  const int64_t* src_offsets = nullptr;
  int src_offsets_aligned = 0;
  const uint8_t* srcs[kMaxSrcs] = {};
  int nsrcs = 0;
  // dsts[b] when ndsts == B: per-image output base (image b's Cout*H*W
  // elements, contiguous in either layout) -- one launch can then decode
  // images belonging to several consumer batches (launch coalescing).
  void* dsts[kMaxSrcs] = {};
  int ndsts = 0;
  int max_grid = 0;
  int unroll = 0;   // pixel groups in flight per lane (0: auto, 1 or 2)
  void* dst = nullptr;
  const float* lut = nullptr;
  const uint8_t* flip = nullptr;
  int B = 0, H = 0, W = 0, Cin = 4, Cout = 3;
  int cmap[4] = {0, 1, 2, 3};
  int flip_all = 0;
  uint64_t flip_bits[4] = {0, 0, 0, 0};   // per-image flip for b < 256
  int out_dtype = OUT_F32;
  int layout = NCHW;
  int xf_table_only = 0;   // 1: the caller built `lut` in table mode (header mode 0); replay picks its table-only kernel
};
hipError_t decode(const DecodeParams& p, hipStream_t stream);

// Key-frame delta frames (csrc/codec/tiledelta.h), decoded in two launches
// on `stream` with the same table, channel map, dtype and layout as decode():
//   1. output image b <- fills[b]: its producer's key frame, already decoded
//      (decode() of the key frame, B = 1, the image's flip) and kept in HBM;
//   2. the payload tiles of image b (p.srcs[b]: the encoded frame, usually
//      host memory mapped for the device) are decoded over it.  One wave
//      slice per 16x16 tile: the tile's position and its pixels are
//      independent loads, and a tile's bytes are one contiguous run.
// tile_start[b] .. tile_start[b + 1] are image b's payload tiles (prefix sums
// over the launch, tile_start[B] = total).  Needs p.nsrcs == B, H % 16 ==
// W % 16 == 0, Cin 3 or 4, and out_img_bytes % 16 == 0.
struct TileParams {
  const void* fills[kMaxSrcs] = {};
  int tile_start[kMaxSrcs + 1] = {};
  int64_t out_img_bytes = 0;
  int64_t payload_off = 0;   // tiledelta::payload_offset(H, W)
};
hipError_t decode_tiles(const DecodeParams& p, const TileParams& t, hipStream_t stream);

// Fused replay sample (DeviceReplayBuffer.sample / gather) in ONE launch:
//   * draw B frame indices in [0, count) on the device with Philox4x32-10
//     (key = seed, counter = (b, C)).  C is ctr_value (eager callers keep the
//     count on the host: one launch), or *counter when counter != nullptr --
//     then a one-lane kernel queued behind the sample advances *counter by B,
//     so a captured HIP graph draws fresh indices on every replay;
//     or take the indices from index_in (gather of given frames);
//   * decode frame idx[b] of the HBM-resident u8 store (p.src, stride
//     frame_bytes) exactly as decode() does (p.lut, cmap, dtype, layout,
//     flip_all) into the dense output p.dst;
//   * copy row idx[b] of every fixed-size metadata column (meta_src[k]:
//     [capacity, meta_bytes[k]]) to meta_dst[k][b].
// p.B <= kMaxReplayB.  counter: nullable device u64 (Philox counter);
// index_out (nullable) receives the int64 indices.
constexpr int kMaxReplayB = 1024;
constexpr int kMaxMeta = 8;
struct ReplayParams {
  int64_t count = 0;
  int64_t frame_bytes = 0;
  uint64_t seed = 0;
  uint64_t* counter = nullptr;
  uint64_t ctr_value = 0;
  const int64_t* index_in = nullptr;
  int64_t* index_out = nullptr;
  int nmeta = 0;
  const uint8_t* meta_src[kMaxMeta] = {};
  uint8_t* meta_dst[kMaxMeta] = {};
  int meta_bytes[kMaxMeta] = {};
};
hipError_t replay_sample(const DecodeParams& p, const ReplayParams& r, hipStream_t stream);

// Per-pixel affine colour transform on the MFMA units:
//   out[b, c, y, x] = sum_k M[c][k] * lut[k][in[b, y, x, k]] + bias[c]
// for RGBA u8 HWC input (Cin = 4), f32 NCHW output with Cout <= 4 channels;
// H*W % 256 == 0 and W % 4 == 0 (one wave = 256 consecutive pixels).
// `lut` is the same folded per-channel table decode() uses (identity for raw
// values); M is row-major 4x4 f32, bias f32[4] (device pointers).
struct Color4x4Params {
  const uint8_t* src = nullptr;
  const int64_t* src_offsets = nullptr;
  const uint8_t* srcs[kMaxSrcs] = {};   // as DecodeParams::srcs
  int nsrcs = 0;
  float* dsts[kMaxSrcs] = {};           // as DecodeParams::dsts
  int ndsts = 0;
  float* dst = nullptr;
  const float* lut = nullptr;
  const float* M = nullptr;
  const float* bias = nullptr;
  const uint8_t* flip = nullptr;
  int B = 0, H = 0, W = 0, Cout = 4;
  int flip_all = 0;
  uint64_t flip_bits[4] = {0, 0, 0, 0};
  // Per-image transforms (photometric augmentation), by mat_mode:
  //   kColorOne     one matrix for every image (M, bias)
  //   kColorPos     Ms + 20 * mat_pos[b]  (16 matrix + 4 bias floats; B <= kMaxSrcs)
  //   kColorEach    Ms + 20 * b
  //   kColorJitter  built in the kernel from jit[b] = (brightness, contrast,
  //                 saturation, hue in turns) about `pivot` (B <= kMaxSrcs):
  //                 rgb' = bc * (Hue(h) . Sat(s)) rgb + (1 - c) * pivot, alpha kept,
  //                 Sat(s) = s I + (1 - s) 1 w^T and Hue the rotation about the grey
  //                 axis with luminance w = (0.213, 0.715, 0.072) (ops.color_jitter_matrix)
  int mat_mode = 0;
  const float* Ms = nullptr;
  uint8_t mat_pos[kMaxSrcs] = {};
  float jit[kMaxSrcs][4] = {};
  float pivot = 0.5f;
};
enum { kColorOne = 0, kColorPos = 1, kColorEach = 2, kColorJitter = 3 };
hipError_t color4x4(const Color4x4Params& p, hipStream_t stream);

// Batched pinhole projection (btb.Camera.world_to_ndc + ndc_to_pixel):
//   xyzw = [p, 1];  clip = xyzw . (P*V)^T;  ndc = clip.xyz / clip.w
//   pixel = ((ndc.xy + 1) / 2) * [W, H], y flipped when upper_left.
//   depth = -(xyzw . V^T).z  (linear camera-space depth)
// pts: f32 [N,3]; PV, V: f32 row-major 4x4 (device); out_px f32 [N,2];
// out_depth nullable f32 [N].
hipError_t project(const float* pts, int64_t N, const float* PV, const float* V, int W, int H,
                   int upper_left, float* out_px, float* out_depth, hipStream_t stream);

// Adaptive average pooling over channels-last (NHWC) activations, the
// consumer model's pooling layer (nn.AdaptiveAvgPool2d semantics: output
// cell (i, j) averages input rows [floor(i*H/OH), ceil((i+1)*H/OH)) and the
// same for columns).  dtype: OUT_F32 or OUT_BF16 (fp32 accumulation, RNE).
// forward: x [N,H,W,C] -> y [N,OH,OW,C]; backward: gy [N,OH,OW,C] -> gx [N,H,W,C].
hipError_t adaptive_avgpool_nhwc(const void* x, void* y, int N, int H, int W, int C, int OH, int OW, int dtype,
                                 hipStream_t stream);
hipError_t adaptive_avgpool_nhwc_bwd(const void* gy, void* gx, int N, int H, int W, int C, int OH, int OW,
                                     int dtype, hipStream_t stream);

// Training-mode BatchNorm2d fused with LeakyReLU over channels-last
// activations (x: [M = N*H*W, C], dtype OUT_F32 or OUT_BF16; C % 8 == 0 and
// C / (16 / sizeof(dtype)) must divide 256).  fp32 statistics.
//   forward:  bn_stats (per-block partial sums) -> bn_finalize (mean, invstd,
//             running stats) -> bn_apply (y = leaky((x-mean)*invstd*w+b))
//   backward: bn_bwd_reduce (partial sum(gz), sum(gz*xhat)) -> bn_bwd_finalize
//             (dw, db) -> bn_bwd_apply (gx)
// `partial` is scratch of bn_partial_floats(M, C) floats.
int64_t bn_partial_floats(int64_t M, int C, int dtype);
hipError_t bn_stats(const void* x, int64_t M, int C, int dtype, float* partial, hipStream_t stream);
// num_batches_tracked (nullable): the module's int64 counter, incremented on the device.
hipError_t bn_finalize(const float* partial, int64_t M, int C, int dtype, float eps, float momentum, float* mean,
                       float* invstd, float* running_mean, float* running_var, hipStream_t stream,
                       int64_t* num_batches_tracked = nullptr);
hipError_t bn_apply(const void* x, void* y, int64_t M, int C, int dtype, const float* mean, const float* invstd,
                    const float* w, const float* b, float slope, hipStream_t stream);
hipError_t bn_bwd_reduce(const void* x, const void* gy, int64_t M, int C, int dtype, const float* mean,
                         const float* invstd, const float* w, const float* b, float slope, float* partial,
                         hipStream_t stream);
hipError_t bn_bwd_finalize(const float* partial, int64_t M, int C, int dtype, float* dw, float* db, hipStream_t stream);
// bn_bwd_finalize over `rows` channel-major partials produced elsewhere (conv_dgrad's BnBwdFuse epilogue)
hipError_t bn_bwd_finalize_rows(const float* partial, int rows, int C, float* dw, float* db, hipStream_t stream);
hipError_t bn_bwd_apply(const void* x, const void* gy, void* gx, int64_t M, int C, int dtype, const float* mean,
                        const float* invstd, const float* w, const float* b, const float* dw, const float* db,
                        float slope, hipStream_t stream);

// Accumulator form of the statistics hand-off.  The producer -- conv_fwd's
// or conv_dgrad's epilogue, or bn_bwd_reduce -- adds each tile's channel sums
// into acc [R][2][C] with fp64 atomics (replica = tile % R, R =
// bn_acc_replicas(C); fp64 so the sums do not depend on the adders' order
// at fp32 precision), and ONE finalize block folds the R replicas, writes the
// finalized outputs (forward: mean, invstd, running stats,
// num_batches_tracked; backward: dw, db) and clears acc for the next
// producer.  acc must be all-zero when the producer runs: allocate it zeroed
// (bn_acc_elems(C) doubles) and let the finalize keep it that way.
int bn_acc_replicas(int C);
int64_t bn_acc_elems(int C);
struct BnAcc {
  double* acc = nullptr;
  int R = 0;
};
hipError_t bn_apply_acc(const void* x, void* y, int64_t M, int C, int dtype, BnAcc acc, float eps, float momentum,
                        float* mean, float* invstd, float* running_mean, float* running_var,
                        int64_t* num_batches_tracked, const float* w, const float* b, float slope,
                        hipStream_t stream);
hipError_t bn_bwd_apply_acc(const void* x, const void* gy, void* gx, int64_t M, int C, int dtype, BnAcc acc,
                            const float* mean, const float* invstd, const float* w, const float* b, float* dw,
                            float* db, float slope, hipStream_t stream);
// bn_bwd_reduce adding into an accumulator (bn_bwd_apply_acc consumes it)
hipError_t bn_bwd_reduce_acc(const void* x, const void* gy, int64_t M, int C, int dtype, const float* mean,
                             const float* invstd, const float* w, const float* b, float slope, BnAcc acc,
                             hipStream_t stream);

// Multi-tensor dtype cast in ONE launch (the consumer step's weight casts
// for bf16 compute and the cast of the bf16 weight gradients back to fp32 --
// a dozen tiny launches otherwise).  mode CAST_F32_TO_BF16 (RNE) or
// CAST_BF16_TO_F32; tensor k has numel[k] elements (contiguous).
constexpr int kMaxCast = 32;
enum CastMode : int { CAST_F32_TO_BF16 = 0, CAST_BF16_TO_F32 = 1 };
struct CastParams {
  const void* src[kMaxCast] = {};
  void* dst[kMaxCast] = {};
  int64_t numel[kMaxCast] = {};
  int n = 0;
  int mode = CAST_F32_TO_BF16;
};
hipError_t multi_cast(const CastParams& p, hipStream_t stream);

// The Adam step schedule as a one-lane job (adam_sched.h): run by
// adam_schedule, or attached ahead of the backward to the first fused data +
// weight gradient launch (block 0's first lane, after its tile) or else the
// next weight-gradient slice-reduce launch.  taken() reports -- and clears --
// whether a launch ran the attached job; detach drops an unused one
// (conv_attach_adam_schedule below).
struct AdamSchedJob {
  float* step = nullptr;        // null: no job
  const float* hp = nullptr;    // lr, gradient scale
  float* sched = nullptr;       // step size, 1 / sqrt(bc2), lr, gradient scale, active
  float beta1 = 0.f, beta2 = 0.f;
  const float* gate = nullptr;  // optional: 0 closes the step
};

// Adam / AdamW over a list of fp32 parameters in ONE launch, graph-capturable:
// the step counter and the bias corrections live on the device.
//   adam_schedule (one lane): step += 1; sched = {lr / (1 - b1^step),
//                             1 / sqrt(1 - b2^step), lr, grad_scale, 1}
//                             (hp = {lr, grad_scale}).  With a device `gate`
//                             whose gate[0] == 0 nothing advances and
//                             sched[4] = 0 turns the update into a no-op.
//   adam_update: per element, PyTorch's Adam arithmetic
//       g = grad * grad_scale (+ wd * p unless decoupled); decoupled: p *= 1 - lr * wd
//       m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g^2
//       p -= sched[0] * m / (sqrt(v) * sched[1] + eps)
//     grads fp32 or bf16 (grad_bf16); optional bf16 shadow copy of the new
//     weights (shadow[k] != nullptr), what a bf16 forward reads next step.
// The tensors' 4-element groups are laid end to end: tensor k owns groups
// [gstart[k], gstart[k+1]); each lane updates one group.
constexpr int kMaxAdam = 32;
struct AdamParams {
  float* p[kMaxAdam] = {};
  const void* g[kMaxAdam] = {};
  float* m[kMaxAdam] = {};
  float* v[kMaxAdam] = {};
  uint16_t* shadow[kMaxAdam] = {};
  int64_t numel[kMaxAdam] = {};
  int64_t gstart[kMaxAdam + 1] = {};
  int n = 0;
  int grad_bf16 = 0;
  int decoupled = 0;   // AdamW
  int maximize = 0;
  float beta1 = 0.9f, beta2 = 0.999f, eps = 1e-8f, weight_decay = 0.f;
  const float* sched = nullptr;   // device [5], written by adam_schedule
  // One-launch form (no adam_schedule): with step != nullptr, sched holds
  // THIS step's schedule, worked out ahead (adam_schedule_prime, then each
  // launch's last block); every block reads it and the gate, and the block
  // that takes the last ticket (*ticket, zero between launches) advances the
  // counter and writes the next step's schedule from hp.
  float* step = nullptr;
  const float* hp = nullptr;
  const float* gate = nullptr;
  uint32_t* ticket = nullptr;
  // zero_grad: clear each gradient after reading it (also when a gate closes
  // the step), so a training loop with persistent gradient buffers needs no
  // separate zero-fill launch before its next backward.  fp32 grads only.
  int zero_grad = 0;
  // shadow_t[k] (nullable): a bf16 copy of the new weight transposed from
  // channels-last [tcout][4][4][tcin] to [tcin][4][4][tcout] (a 4x4
  // convolution's data-gradient operand, conv_weight_t).
  uint16_t* shadow_t[kMaxAdam] = {};
  // g2[k] (nullable, fp32 grads): a second gradient contribution of the same step
  // (a second backward pass, GradBuckets(second_sinks=True)) added to g[k] here --
  // what autograd's AccumulateGrad kernel would have done, without its launch
  const float* g2[kMaxAdam] = {};
  int tcout[kMaxAdam] = {};
  int tcin[kMaxAdam] = {};
  // fr.partial != nullptr: one more convolution weight, NOT in the lists, whose
  // gradient is not given but summed here from the backward's last weight-gradient
  // slices (the deferred ordered slice reduce, ConvWgradParams::Reduce fields;
  // ops.FusedAdam.attach_reduce): blocks [0, fr.rx) of the launch sum it
  // (wgrad_reduce.h) and update p / m / v / shadow at the gradient's strides
  // themselves, and write the gradient (0 with zero_grad) to g -- the reduce
  // launch goes away.  fp32 gradients, not the one-launch form.
  struct FusedReduce {
    const float* partial = nullptr;
    int S = 0, Cout = 0, Cin = 0, cin_out = 0, sub = 0, rx = 0;
    int64_t s_co = 0, s_ci = 0, s_kh = 0, s_kw = 0;
    float* g = nullptr;
    float* p = nullptr;
    float* m = nullptr;
    float* v = nullptr;
    uint16_t* shadow = nullptr;
  } fr;
};
// Weight gradient of a 4x4 / stride-2 / pad-1 convolution over channels-last
// bf16 activations on the MFMA units (conv.hip): x [N][H][W][Cin],
// dy [N][Ho][Wo][Cout] -> fp32 dW written at the given element strides of
// (co, ci, kh, kw).  Cin % 32 == 0, Cout % 64 == 0.  `partial` is scratch of
// slices * Cout * 16 * Cin floats; slices * px_per_slice >= M, px_per_slice % 32 == 0.
struct ConvWgradParams {
  const uint16_t* x = nullptr;
  const uint16_t* dy = nullptr;
  float* partial = nullptr;
  int N = 0, H = 0, W = 0, Cin = 0, Ho = 0, Wo = 0, Cout = 0;
  int64_t M = 0;
  int slices = 0;
  int64_t px_per_slice = 0;
  int cin_out = 0;   // dW input channels written (0: Cin); 3 for a 4-channel (RGBA-fed) first layer
  const uint16_t* lut = nullptr;   // Cin == 4: x is raw u8 RGBA decoded through this bf16 table (ConvFwdParams)
  float* zero_out = nullptr;   // set by conv_wgrad: the kernel clears the output for the atomic reduce
  int zero_count = 0;
  // set by conv_wgrad: blocks [0, main_blocks) compute this layer, blocks
  // [main_blocks, grid) run `side`, a previous layer's deferred slice reduce
  int main_blocks = 0;
  struct Reduce {
    const float* partial = nullptr;
    int S = 0, Cout = 0, Cin = 0, cin_out = 0;
    float* out = nullptr;
    int64_t s_co = 0, s_ci = 0, s_kh = 0, s_kw = 0;
    int rx = 0, ry = 0;   // its grid: element blocks x slice groups
    // sub > 0: the ordered (deterministic) reduce -- ry == 1, sub lanes per
    // 4 elements each sum a fixed subset of the slices in a fixed order, then
    // a fixed xor-shuffle tree; one plain store per element (no atomics)
    int sub = 0;
  } side;
  // fold.acc != nullptr (not the 4-channel first layer): one more block folds
  // the BatchNorm backward accumulator the preceding data gradient's epilogue
  // filled (bn_fold.h) into db = sum gz, dw = sum gz * xhat, and clears it --
  // the BN backward then needs no finalize launch
  struct Fold {
    double* acc = nullptr;
    int R = 0, C = 0;
    int64_t M = 0;
    float* dw = nullptr;
    float* db = nullptr;
  } fold;
  // bn_dy.y != nullptr: dy is NOT the
  // convolution's output gradient but the gradient of the BatchNorm +
  // LeakyReLU that follows it, whose input is bn_dy.y ([M][Cout] bf16); the
  // kernel applies that BN's backward while staging dY (bn_fold.h BnBwdCoef,
  // bit-identical to bn_bwd_apply), so no bn_bwd_apply pass runs.  dw / db:
  // the BN's folded backward sums (db = sum gz, dw = sum gz * xhat).
  // With bn_dy.acc (any layer): dw / db are not given but folded by every
  // block from the BN's backward accumulator (fp64 [R][2][Cout], filled by
  // the following layer's data-gradient epilogue); block 0 writes them to
  // dw_out / db_out (the BN's parameter gradients), the last block clears the
  // accumulator; gx_out (nullable) receives the BN's input gradient gx (the
  // blocks of the first column tile store their staged dY chunks: every
  // element once) -- the operand of this layer's data gradient, which then
  // runs after this kernel.  Not the DMA-staged kernel.
  struct BnDy {
    const uint16_t* y = nullptr;
    const float* mean = nullptr;
    const float* invstd = nullptr;
    const float* w = nullptr;
    const float* b = nullptr;
    const float* dw = nullptr;
    const float* db = nullptr;
    float slope = 0.f;
    double* acc = nullptr;
    int R = 0;
    float* dw_out = nullptr;
    float* db_out = nullptr;
    uint16_t* gx_out = nullptr;
  } bn_dy;
  // set by conv_wgrad (null: none): the attached Adam schedule, run by block 0
  // of a fused data + weight gradient launch (BT_SCHED_EARLY, default on)
  AdamSchedJob job;
};
// Cin % 32 == 0 with Cout % 64 == 0, or Cin == 4 (the first layer) with Cout % 32 == 0.
bool conv_wgrad_supported(int Cin, int Cout);
int conv_wgrad_slices(int64_t M, int Cin, int Cout, int target_blocks);
// the u8 first layer's weight gradient from a decoded input patch (conv_wgrad_c4p_kernel): output rows
// per band -- its slices must then be bands, px_per_slice = rows * Wo -- or 0 when the shape does not take it
int conv_c4p_rows(int N, int H, int W, int Ho, int Wo, int Cout);
void conv_set_c4p_rows(int rows);       // 0: off, 1 / 2 / 4 rows, else back to BT_C4W_PATCH / BT_C4P_ROWS
void conv_set_wgrad_co128(int on);      // 128-channel weight-gradient tiles: 1 on, 0 off, -1 BT_WGRAD_CO128
void conv_set_dgrad_bn128(int on);      // 128-channel tiles for the held (fused) data gradient: 1 / 0 / -1 env
void conv_set_fwd_split(int on);        // split-K forward of the 128-channel layers: 1 / 0 / -1 BT_CONV_FWD_SPLIT
int64_t conv_fwd_split_launches();      // forwards launched split so far (this process)
// Weight-gradient staging (not the 4-channel layer): 0 = register ring,
// 2 / 3 = LDS-DMA stages of 64 pixels (default 0; -1 = BT_WGRAD_STAGING or default).
void conv_set_fwd_patch(int on, int dbg = 0, int blocks = 0);       // 1 the 32->64 forward's persistent patch GEMM, 0 the tap GEMM, -1 env
void conv_set_wgrad_ordered(int on);   // 1 ordered (deterministic) slice reduce, 0 atomic groups, -1 env
void conv_set_wgrad_staging(int staging);
// Register-staged weight gradient: 1 = read the next step's fragments while this step's MFMAs run
// (two fragment sets), 0 = one set (default), -1 = BT_WGRAD_PIPE / default.
void conv_set_wgrad_pipe(int on);
// Register-staged weight gradient over 256-column im2col tiles (waves of 32 x 128): 1 on, 0 off (default), -1 env.
void conv_set_wgrad_wide(int on);
// The 32-channel data gradient (dY 64 -> dx 32): 1 = from a dY patch (default), 0 = the tap GEMM, -1 = BT_DGRAD_PATCH.
void conv_set_dgrad_patch(int on);
// First-layer weight gradient: 1 = wave-private staging (default), 0 = block-shared, -1 = BT_C4_WAVE / default.
void conv_set_c4_wave_private(int on);
void conv_set_c4w_waves(int nw);   // first-layer weight gradient: 4 or 8 waves per block (-1: BT_C4W_WAVES / default)
// The slice reduce normally follows the main kernel as its own launch.
// defer != nullptr: it is NOT launched but described in *defer, for the
// next conv_wgrad to run as extra blocks of its own launch (`side`; the
// partial scratch must stay alive until then) -- a layer chain then pays one
// reduce launch in all, the last layer's.  The deferred output was already
// cleared by its main kernel.
hipError_t conv_wgrad(const ConvWgradParams& p, float* out, int64_t s_co, int64_t s_ci, int64_t s_kh, int64_t s_kw,
                      hipStream_t stream, ConvWgradParams::Reduce* defer = nullptr,
                      const ConvWgradParams::Reduce* side = nullptr);
// a deferred reduce on its own (a chain that ends without another conv_wgrad)
hipError_t conv_wgrad_reduce(const ConvWgradParams::Reduce& r, hipStream_t stream);

// Forward 4x4 / stride-2 / pad-1 convolution on the MFMA units (conv.hip):
// x [N][H][W][Cin] bf16, w [Cout][4][4][Cin] bf16 (channels-last weight) ->
// y [N][Ho][Wo][Cout] bf16.  stats (nullable): [2][Cout][conv_fwd_tiles(M, Cout)]
// fp32 per-tile sum / sum of squares of the rounded y (channel-major) -- the
// partials bn_finalize_rows folds into BatchNorm statistics.
// A training BatchNorm+LeakyReLU applied by its CONSUMER as it reads the BN's
// input (the conv forward's operand staging, its weight gradient's re-read,
// the head's pooling): no apply pass and no activation tensor.  The batch
// statistics sit in the BnAcc accumulator the producer added into (acc,
// fp64 [R][2][C]); every consumer block folds them, block 0 writes mean /
// invstd and the running statistics, and the last block clears the
// accumulator (bn_fold.h).  With acc == nullptr the consumer reads mean /
// invstd as given (the weight gradient, after the forward wrote them).
struct BnActIn {
  double* acc = nullptr;
  int R = 0;
  int64_t M = 0;                   // elements per channel
  float eps = 0.f, momentum = 0.f;
  const float* w = nullptr;        // affine weight / bias, fp32 [C]
  const float* b = nullptr;
  float slope = 0.f;
  float* mean = nullptr;           // fp32 [C]: written (acc) or read
  float* invstd = nullptr;
  float* rm = nullptr;             // running statistics (nullable)
  float* rv = nullptr;
  int64_t* tracked = nullptr;
  __host__ __device__ bool on() const { return w != nullptr; }
};

struct ConvFwdParams {
  const uint16_t* x = nullptr;
  const uint16_t* w = nullptr;
  uint16_t* y = nullptr;
  float* stats = nullptr;
  int N = 0, H = 0, W = 0, Cin = 0, Ho = 0, Wo = 0, Cout = 0;
  int64_t M = 0;
  int w_channels = 0;   // Cin == 4 (first layer): 3 = an RGB weight [Cout][4][4][3], input channel 3 ignored
  // Cin == 4: x is the RAW u8 RGBA frames [N][H][W][4] and lut their decode
  // table as bf16 [4][256] (RNE of the fp32 table): the decode runs inside
  // the convolution's tile loads (padding stays 0)
  const uint16_t* lut = nullptr;
  int acc_r = 0;        // > 0: stats points at a bn_apply_acc accumulator (fp64 [acc_r][2][Cout], atomic adds)
  // act.on(): x is the input of a BatchNorm+LeakyReLU applied inside this
  // convolution's operand staging (Cin <= 128); act_out (nullable) receives
  // that activation, [N][H][W][Cin] bf16 -- written by the convolution, no
  // apply pass (BnActIn)
  BnActIn act;
  uint16_t* act_out = nullptr;
  // out_act.on() (first layer, u8 frames, accumulator statistics): the
  // BatchNorm+LeakyReLU that consumes y is applied by this launch too (a grid
  // barrier after its statistics); out_y receives leaky(bn(y)), y is still
  // written.  Only where conv1_bn_apply_fits says so.
  BnActIn out_act;
  uint16_t* out_y = nullptr;
};
// True when conv_fwd can apply the output's BatchNorm+LeakyReLU itself on a
// first layer of this shape (every block of the launch resident at once).
// Needs the GPU (occupancy query); BT_CONV1_BN=0 turns it off.
bool conv1_bn_apply_fits(int N, int Ho, int Wo, int Cout);
// The same for any layer (Cin == 4: conv1_bn_apply_fits; else the tap-GEMM
// forward: 64-channel tiles, its whole grid resident; BT_CONV_OUT_BN=0 off).
bool conv_out_bn_fits(int N, int Ho, int Wo, int Cin, int Cout);
// Grid-barrier waits that gave up (should stay 0; see conv.hip grid_barrier).
unsigned conv_grid_barrier_timeouts();
// host-mapped failure flag of the grid barrier: arm once (outside capture), poll without a HIP call
bool conv_grid_barrier_arm();
int conv_grid_barrier_failed();   // -1 not armed, 0 ok, 1 a barrier gave up
void conv_grid_barrier_clear(int value);
// Cin a power of two >= 8, or Cin == 4 (first layer, RGBA-decoded frames); Cout % 32 == 0.
bool conv_fwd_supported(int Cin, int Cout);
int64_t conv_fwd_tiles(int64_t M, int Cout);
// pixels per tap-GEMM tile (64 or 128) for a GEMM of M rows, NOUT outputs and
// `ytiles` parity classes, and output channels per tile (32, 64 or 128).
int conv_tile_pixels(int64_t M, int NOUT, int ytiles);
int conv_tile_channels(int NOUT, bool first_layer);
// Force the tile sizes (0 = automatic; initially BT_CONV_BM / BT_CONV_BN) and
// the staging (0 = register ring, 2 / 3 = LDS-DMA stages; -1 = default,
// BT_CONV_STAGING).
// Row counts of the statistics buffers follow the tile size: change it only
// between steps, never between sizing a buffer and the launch that fills it.
void conv_set_tiles(int bm, int bn, int staging = -1, int dgrad_cls = 0);
// Parity classes per data-gradient block (1, or 4 when one class per block
// would give >= 4096 blocks; BT_CONV_DGRAD_CLS / conv_set_tiles force it).
int conv_dgrad_classes_per_block(int64_t M, int NOUT);
// First-layer (4-channel) forward: 128-pixel tiles per block of the multi-tile
// kernel (default 1 = the one-tile tap-GEMM path; BT_CONV1_TILES).
void conv_set_conv1_tiles(int tiles, int rows);
hipError_t conv_fwd(const ConvFwdParams& p, hipStream_t stream);
// Data gradient of the same convolution (same tap-gather GEMM kernel, four
// stride-2 parity classes in one launch): dy [N][H/2][W/2][Cout] bf16,
// wt = conv_weight_t(w) [Cin][4][4][Cout] bf16 -> dx [N][H][W][Cin] bf16.
// Cout a power of two >= 16, Cin % 64 == 0, H and W even.
bool conv_dgrad_supported(int Cin, int Cout);
hipError_t conv_weight_t(const uint16_t* w, uint16_t* wt, int Cout, int Cin, hipStream_t stream);
constexpr int kMaxWeightT = 8;
struct WeightTParams {   // conv_weight_t for several weights in one launch
  const uint16_t* src[kMaxWeightT] = {};
  uint16_t* dst[kMaxWeightT] = {};
  int cout[kMaxWeightT] = {};
  int cin[kMaxWeightT] = {};
  int n = 0;
};
hipError_t conv_weight_t_multi(const WeightTParams& p, hipStream_t stream);
// bn (nullable, part != null to enable): dx is the gy of a BatchNorm+LeakyReLU
// backward whose saved input x ([N][H][W][Cin] bf16), batch mean / invstd,
// affine w / b (fp32 [Cin]) and slope are given; the epilogue writes that
// backward's per-tile sums of gz and gz * xhat, channel-major
// [2][Cin][conv_dgrad_bn_rows(N, H, W, Cin)] fp32, for bn_backward_from_stats.
struct BnBwdFuse {
  const uint16_t* x = nullptr;
  const float* mean = nullptr;
  const float* invstd = nullptr;
  const float* w = nullptr;
  const float* b = nullptr;
  float slope = 0.f;
  float* part = nullptr;
  int rows = 0;
  int acc_r = 0;   // > 0: part points at a bn_bwd_apply_acc accumulator (fp64 [acc_r][2][Cin], atomic adds), rows unused
};
int64_t conv_dgrad_bn_rows(int N, int H, int W, int Cin);

hipError_t conv_dgrad(const uint16_t* dy, const uint16_t* wt, uint16_t* dx, int N, int H, int W, int Cin, int Cout,
                      hipStream_t stream, const BnBwdFuse* bn = nullptr);
// Hold the next tap-GEMM data gradient (on) for the weight gradient that
// follows on its stream: conv_wgrad launches both in one kernel
// (dgrad_wgrad_kernel) when it is the plain weight-gradient kernel's case,
// else launches the held one first.  conv_dgrad_flush launches a held data
// gradient alone; conv_dgrad_held reports whether one is held.
void conv_dgrad_hold(int on);
hipError_t conv_dgrad_flush();
bool conv_dgrad_held();
// bn_finalize over `nblocks` partial rows produced elsewhere (conv_fwd's epilogue)
hipError_t bn_finalize_rows(const float* partial, int nblocks, int64_t M, int C, float eps, float momentum,
                            float* mean, float* invstd, float* running_mean, float* running_var, hipStream_t stream,
                            int64_t* num_batches_tracked);

// Discriminator head (head.hip): AdaptiveAvgPool2d(OH, OW) -> Conv2d(C, 1,
// (OH, OW), no bias) -> sigmoid -> mean binary cross-entropy against target
// (per-image tensor, or target_value when target is null), forward and
// backward in three launches each way.  z: bf16 [N][H][W][C] (channels-last);
// w: fp32, element (c, i, j) at c*ws_c + i*ws_i + j*ws_j.  Forward writes
// pooled [N][OH][OW][C], partial [N][OH*OW], loss [1], dlogit [N] (= (p-y)/N),
// logit [N] (nullable).  Backward scales by gscale[0] (the loss's incoming
// gradient, on the device) and writes dz (bf16, like z) and dw (fp32, like w).
struct HeadParams {
  const uint16_t* z = nullptr;
  const float* w = nullptr;
  int64_t ws_c = 0, ws_i = 0, ws_j = 0;
  int N = 0, H = 0, W = 0, C = 0, OH = 0, OW = 0;
  const float* target = nullptr;
  float target_value = 1.f;
  float* pooled = nullptr;
  float* partial = nullptr;
  float* loss = nullptr;
  float* dlogit = nullptr;
  float* logit = nullptr;
  const float* gscale = nullptr;
  uint16_t* dz = nullptr;
  float* dw = nullptr;
  // forward: with ticket (a zeroed word) the pooling blocks hand their
  // partial logits to the block that finishes last, which computes the loss
  // (one launch instead of two)
  uint32_t* ticket = nullptr;
  // backward: bn_acc (nullable) = the BnAcc accumulator of the BatchNorm +
  // LeakyReLU that produced z: the dz pass also sums that backward's gz and
  // gz * xhat (x = the BN's saved input) -- no bn_bwd_reduce launch
  const uint16_t* bn_x = nullptr;
  const float* bn_mean = nullptr;
  const float* bn_invstd = nullptr;
  const float* bn_w = nullptr;
  const float* bn_b = nullptr;
  float bn_slope = 0.f;
  double* bn_acc = nullptr;
  int bn_acc_r = 0;
  // forward: z is the INPUT of the BatchNorm+LeakyReLU whose output the head
  // pools (act.on()): the pooling reads leaky(bn(z)) rounded to bf16
  BnActIn act;
  // forward with act.on() and bn_ab (the BN's backward worked out in the head,
  // head_fwd_act_kernel): dz = g dlogit_n M[h][w][c] factors, so the BN
  // backward's sums are sum_n dlogit_n A[n][c] (db) and sum_n dlogit_n B[n][c]
  // (dw), A / B = sum over the pixels of M s (s = the LeakyReLU slope at the
  // pixel) and M s xhat.  bn_ab: [2][N][C] fp64 scratch (order-free sums), zero before the launch
  // and cleared again by it; bn_sums: [2][C] the two sums (db, dw) before the
  // backward's loss gradient g
  double* bn_ab = nullptr;
  float* bn_sums = nullptr;
  // backward with bn_sums: write the BN's INPUT gradient gx (not dz) into dz,
  // and the BN's dw / db (g times the sums) into bn_dw_out / bn_db_out
  float* bn_dw_out = nullptr;
  float* bn_db_out = nullptr;
};
hipError_t head_forward(const HeadParams& p, hipStream_t stream);
// whether head_forward can work out the BN backward's sums (HeadParams::bn_ab) for this shape
bool head_bn_bwd_supported(int N, int H, int W, int C, int OH, int OW, int R);
void head_set_fast(int on);   // BN-applying forward: 1 the round-trip-lean kernel (default), 0 round 4's, -1 BT_HEAD_FWD
hipError_t head_backward(const HeadParams& p, hipStream_t stream);

hipError_t adam_schedule(float* step, const float* hp, float* sched, float beta1, float beta2, hipStream_t stream,
                         const float* gate = nullptr);
hipError_t adam_update(const AdamParams& p, hipStream_t stream);
hipError_t adam_schedule_prime(const float* step, const float* hp, float* sched, float beta1, float beta2,
                               hipStream_t stream, float off = 1.f);

// keyed by the optimizer's device and stream: only a launch on that stream of that
// device takes it (another device's or a side stream's launch does not)
void conv_attach_adam_schedule(const AdamSchedJob& j, int device, hipStream_t stream);
bool conv_adam_schedule_taken();
void conv_detach_adam_schedule();


// densityopt's gate and S step (dopt.hip): per-iteration control math on the device
struct DoptParams {
  const float* logit_real = nullptr;   // [B] discriminator logits of the target batch
  const float* logit_sim = nullptr;    // [B] ... of the simulated batch (before the D update)
  const float* logit_s = nullptr;      // [B] ... of the simulated batch after the D update (S step)
  float* stats = nullptr;              // [2] D_real, D_sim: mean sigmoid(logits)
  float* gate_d = nullptr;             // [1] D_real - D_sim < threshold
  float threshold = 0.7f;
  const int64_t* sid = nullptr;        // [B] global sample ids of the simulated images (device or host-mapped)
  float* samples = nullptr;            // [2][N] m1, m2 of every rank (read, then the next ones written)
  float* mean = nullptr;               // [2] ProbModel.m1m2_mean (updated in place)
  float* log_std = nullptr;            // [2] ProbModel.m1m2_log_std
  float* exp_avg = nullptr;            // [4] Adam moments of (mean, log_std)
  float* exp_avg_sq = nullptr;         // [4]
  float* adam_step = nullptr;          // [1]
  float lr = 5e-2f, b1 = 0.7f, b2 = 0.999f, eps = 1e-8f;
  float* b = nullptr;                  // [1] baseline
  float* first = nullptr;              // [1] 1 until the first S step
  float* gate_s = nullptr;             // [1]
  float alpha = 0.9f;
  float* params_out = nullptr;         // [4] mu1, mu2, std1, std2 after the step
  float* red = nullptr;                // [5] per-rank means (data parallel: averaged between phases 1 and 2)
  float* host = nullptr;               // host-mapped [2B + 8]: this rank's samples, params, stats, gates (nullable)
  uint32_t* counter = nullptr;         // [1] iteration counter of the sampler
  uint64_t seed = 0;
  int B = 0, N = 0, rank = 0, world = 1;
};
hipError_t dopt_gate(const DoptParams& p, int phase, hipStream_t stream);    // phase 0 all, 1 stats, 2 gate
// phase 0 all, 1 partials, 2 update, 3 samples only
hipError_t dopt_sstep(const DoptParams& p, int phase, hipStream_t stream);
// host-mapped pinned memory (hipHostMalloc mapped + coherent): (host pointer, device pointer)
void* host_mapped_alloc(size_t bytes, void** dev);
void host_mapped_free(void* host);
}  // namespace gpu
}  // namespace btn
