// Host-side fit of the decode kernels' arithmetic value transform (see
// xform_fit.h).  Every operation is rounded on its own: the file is built
// with -ffp-contract=off, and fmas are explicit (std::fmaf: correctly
// rounded, like v_fma_f32).
#include "xform_fit.h"

#include <cmath>
#include <cstring>

namespace btn {
namespace codec {

float apply_channel(const XfChannel& c, float x) {
  switch (c.op) {
    case 0:
      return std::fmaf(x, c.a, c.b);
    case 1:
      return x * c.a - c.b;
    case 3: {
      const float t = x * c.a - c.b;
      const float q = t * c.r;
      return std::fmaf(std::fmaf(-q, c.d, t), c.r, q);
    }
    default:
      return (x * c.a - c.b) / c.d;
  }
}

namespace {

bool exact(const XfChannel& c, const float* x, const float* y) {
  for (int v = 0; v < 256; ++v) {
    const float z = apply_channel(c, x[v]);
    if (std::memcmp(&z, &y[v], sizeof(float)) != 0) return false;
  }
  return true;
}

}  // namespace

bool fit_channel(const float* x, const float* y, float scale, float mean, float std, bool normalize, XfChannel* out) {
  XfChannel c;
  if (!normalize) {
    c.op = 0, c.a = 1.f, c.b = 0.f;
    if (exact(c, x, y)) return *out = c, true;
    return false;
  }
  // op 0: the reference's own constants first, then a small ulp search
  // around (scale / std, -mean / std)
  const float a0 = scale / std, b0 = -mean / std;
  for (int da = -4; da <= 4; ++da) {
    for (int db = -4; db <= 4; ++db) {
      float a = a0, b = b0;
      for (int k = 0; k < (da < 0 ? -da : da); ++k) a = std::nextafter(a, da > 0 ? INFINITY : -INFINITY);
      for (int k = 0; k < (db < 0 ? -db : db); ++k) b = std::nextafter(b, db > 0 ? INFINITY : -INFINITY);
      c.op = 0, c.a = a, c.b = b;
      if (exact(c, x, y)) return *out = c, true;
    }
  }
  c.a = scale, c.b = mean, c.d = std, c.r = 1.f / std;
  if (std == 1.f) {
    c.op = 1;
    if (exact(c, x, y)) return *out = c, true;
  }
  c.op = 3;
  if (exact(c, x, y)) return *out = c, true;
  c.op = 2;
  if (exact(c, x, y)) return *out = c, true;
  return false;
}

}  // namespace codec
}  // namespace btn
