// Arithmetic form of a decode value table (csrc/gpu/kernels.h: lut).
//
// The reference normalises pixels with numpy float32 ops, each rounded on
// its own: y = (x * scale - mean) / std (x = the gamma'd u8 value).  The
// decode kernels compute y instead of looking it up in an fp32 table in LDS
// (whose data-dependent reads bank-conflict), so the host picks, per
// channel, the cheapest form it has VERIFIED to reproduce the table bit for
// bit over all 256 inputs:
//   op 0: fma(x, a, b)                           (1 VALU)
//   op 1: x*a - b                                (2)
//   op 3: t = x*a - b; q = t*r; fma(fma(-q, d, t), r, q)   (5; r = 1/d rounded:
//         one Newton correction of the reciprocal product -- exact for these
//         256 values, which the check proves)
//   op 2: (x*a - b) / d                          (correctly rounded division)
#pragma once

namespace btn {
namespace codec {

struct XfChannel {
  int op = 2;
  float a = 1.f, b = 0.f, d = 1.f, r = 1.f;
};

// y: the fp32 table of one output channel; x: its inputs (gamma table or
// identity, as floats).  normalize = false: y == x expected (op 0, a 1, b 0).
// Returns false when no form reproduces y exactly.
bool fit_channel(const float* x, const float* y, float scale, float mean, float std, bool normalize, XfChannel* out);

// The same forms on the host (for tests and the checks above).
float apply_channel(const XfChannel& c, float x);

}  // namespace codec
}  // namespace btn
