// Headless CPU renderer (see raster.h).  The static background (ground plane
// lit by the point light, world colour) is shaded once per Renderer; each
// frame copies it, span-fills the boxes' projected shadow hulls and scan-
// converts the boxes' front faces (two triangles each) with Gouraud-
// interpolated point-light Lambert shading and, for several boxes, a
// perspective-correct 1/z buffer.  ~0.3-0.4 ms per 640x480 frame; a buffer
// rendered into repeatedly (a shm ring slot) restores only the rectangle its
// previous frame touched (DirtyRect).
#include "raster.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>

#include <immintrin.h>

namespace btn {
namespace sim {

namespace {
constexpr double kPi = 3.14159265358979323846;

inline Vec3 add(const Vec3& a, const Vec3& b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline Vec3 sub(const Vec3& a, const Vec3& b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline Vec3 scale(const Vec3& a, double s) { return {a.x * s, a.y * s, a.z * s}; }
inline double dot(const Vec3& a, const Vec3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

// linear radiance -> display 8 bit (power 1/2.2), 4096-entry table over [0,1]
struct ToneLut {
  uint8_t v[4097];
  uint32_t gray4[4097];   // v[i] in R, G and B, alpha 255: one load per pixel of a grey box
  ToneLut() {
    for (int i = 0; i <= 4096; ++i) {
      double x = i / 4096.0;
      v[i] = uint8_t(std::min(255.0, std::floor(255.0 * std::pow(x, 1.0 / 2.2) + 0.5)));
      gray4[i] = uint32_t(v[i]) * 0x010101u | 0xff000000u;
    }
  }
  inline uint8_t operator()(double x) const {
    if (!(x > 0)) return 0;
    if (x >= 1) return 255;
    return v[int(x * 4096.0)];
  }
};
// floor / ceil to int without a libm call (exact for |v| < 2^31; the
// arguments are clamped to a range far outside any image first)
inline int ifloor(float v) {
  v = std::min(std::max(v, -1e9f), 1e9f);
  const int i = int(v);
  return i - (v < float(i));
}
inline int iceil(float v) { return -ifloor(-v); }

const ToneLut& tone() {
  static ToneLut t;
  return t;
}

// Ray/oriented-box overlap for t in (tmin, tmax).
bool ray_hits_box(const Box& b, const Vec3& o, const Vec3& d, double tmin, double tmax) {
  Vec3 lo = mul_t(b.rot, sub(o, b.center));
  Vec3 ld = mul_t(b.rot, d);
  const double ov[3] = {lo.x, lo.y, lo.z}, dv[3] = {ld.x, ld.y, ld.z};
  const double hv[3] = {b.half.x, b.half.y, b.half.z};
  for (int a = 0; a < 3; ++a) {
    if (std::fabs(dv[a]) < 1e-12) {
      if (ov[a] < -hv[a] || ov[a] > hv[a]) return false;
      continue;
    }
    double inv = 1.0 / dv[a];
    double t0 = (-hv[a] - ov[a]) * inv, t1 = (hv[a] - ov[a]) * inv;
    if (t0 > t1) std::swap(t0, t1);
    tmin = std::max(tmin, t0);
    tmax = std::min(tmax, t1);
    if (tmin > tmax) return false;
  }
  return true;
}

inline double light_scale(const Light& l) { return l.power / (4.0 * kPi * kPi); }

}  // namespace

Mat3 euler_xyz(double rx, double ry, double rz) {
  double cx = std::cos(rx), sx = std::sin(rx), cy = std::cos(ry), sy = std::sin(ry);
  double cz = std::cos(rz), sz = std::sin(rz);
  // R = Rz * Ry * Rx
  return Mat3{cz * cy, cz * sy * sx - sz * cx, cz * sy * cx + sz * sx,
              sz * cy, sz * sy * sx + cz * cx, sz * sy * cx - cz * sx,
              -sy,     cy * sx,                cy * cx};
}

Vec3 mul(const Mat3& m, const Vec3& v) {
  return {m[0] * v.x + m[1] * v.y + m[2] * v.z, m[3] * v.x + m[4] * v.y + m[5] * v.z,
          m[6] * v.x + m[7] * v.y + m[8] * v.z};
}

Vec3 mul_t(const Mat3& m, const Vec3& v) {
  return {m[0] * v.x + m[3] * v.y + m[6] * v.z, m[1] * v.x + m[4] * v.y + m[7] * v.z,
          m[2] * v.x + m[5] * v.y + m[8] * v.z};
}

double Camera::focal_px() const { return lens_mm / sensor_mm * double(std::max(width, height)); }

bool Camera::project(const Vec3& w, double* px, double* py, double* depth) const {
  Vec3 c = mul_t(rot, sub(w, loc));
  if (depth) *depth = -c.z;
  if (c.z >= -1e-12) return false;
  double f = focal_px();
  *px = 0.5 * width + f * c.x / (-c.z);
  *py = 0.5 * height - f * c.y / (-c.z);
  return true;
}

std::array<Vec3, 8> Box::corners() const {
  // Blender default cube vertex order
  static const int s[8][3] = {{1, 1, 1}, {1, 1, -1}, {1, -1, 1}, {1, -1, -1},
                              {-1, 1, 1}, {-1, 1, -1}, {-1, -1, 1}, {-1, -1, -1}};
  std::array<Vec3, 8> out;
  for (int i = 0; i < 8; ++i) {
    Vec3 l{s[i][0] * half.x, s[i][1] * half.y, s[i][2] * half.z};
    out[i] = add(center, mul(rot, l));
  }
  return out;
}

Scene cube_scene() {
  Scene s;
  s.cam.width = 640;
  s.cam.height = 480;
  s.cam.loc = {7.358891, -6.925791, 4.958309};
  s.cam.rot = euler_xyz(1.109319, 0.0, 0.814928);
  s.light.loc = {4.076245, 1.005454, 5.903862};
  s.light.power = 1000.0;
  Box b;
  b.rot = euler_xyz(0, 0, 0);
  s.boxes.push_back(b);
  return s;
}

Scene falling_cubes_scene() {
  Scene s = cube_scene();
  s.cam.loc = {14.5, -15.712, 16.754};
  // look at the origin: -Z toward target, +Y up
  Vec3 dir = sub(Vec3{0, 0, 0}, s.cam.loc);
  double n = std::sqrt(dot(dir, dir));
  dir = scale(dir, 1.0 / n);
  double pitch = std::acos(-dir.z);             // rotation about x from looking down
  double yaw = std::atan2(-dir.x, dir.y);   // Rz maps +Y to (-sin, cos)
  s.cam.rot = euler_xyz(pitch, 0.0, yaw);
  s.light.loc = {4.0, 1.0, 14.0};
  s.light.power = 6000.0;
  s.boxes.assign(7, Box());
  return s;
}

namespace {

// 2-D convex hull (monotone chain), counter-clockwise, no repeated end point.
using P2 = std::array<double, 2>;
int convex_hull(P2* p, int n, P2* h) {
  std::sort(p, p + n, [](const P2& a, const P2& b) {
    return a[0] < b[0] || (a[0] == b[0] && a[1] < b[1]);
  });
  auto cross = [](const P2& o, const P2& a, const P2& b) {
    return (a[0] - o[0]) * (b[1] - o[1]) - (a[1] - o[1]) * (b[0] - o[0]);
  };
  int k = 0;
  for (int i = 0; i < n; ++i) {
    while (k >= 2 && cross(h[k - 2], h[k - 1], p[i]) <= 0) --k;
    h[k][0] = p[i][0];
    h[k][1] = p[i][1];
    ++k;
  }
  for (int i = n - 2, t = k + 1; i >= 0; --i) {
    while (k >= t && cross(h[k - 2], h[k - 1], p[i]) <= 0) --k;
    h[k][0] = p[i][0];
    h[k][1] = p[i][1];
    ++k;
  }
  return k - 1;
}

}  // namespace

Renderer::Renderer(const Scene& s, int channels, bool lower_left)
    : W_(s.cam.width), H_(s.cam.height), C_(channels), lower_left_(lower_left) {
  const Camera& cam = s.cam;
  const double f = cam.focal_px();
  const ToneLut& T = tone();
  const Vec3 o = cam.loc;
  const Vec3 X{cam.rot[0], cam.rot[3], cam.rot[6]};
  const Vec3 Y{cam.rot[1], cam.rot[4], cam.rot[7]};
  const Vec3 Z{cam.rot[2], cam.rot[5], cam.rot[8]};
  const double ls = light_scale(s.light);
  const Vec3 L = s.light.loc;
  background_.assign(size_t(W_) * H_ * C_, 255);
  plane_xy_.assign(size_t(W_) * H_ * 2, std::numeric_limits<float>::quiet_NaN());
  for (int c = 0; c < 3; ++c) shadow_rgb_[c] = T(s.plane_albedo[c] * s.ambient);
  for (int y = 0; y < H_; ++y) {
    const double cy = -((y + 0.5) - 0.5 * H_) / f;
    for (int x = 0; x < W_; ++x) {
      const double cx = ((x + 0.5) - 0.5 * W_) / f;
      const Vec3 d{cx * X.x + cy * Y.x - Z.x, cx * X.y + cy * Y.y - Z.y, cx * X.z + cy * Y.z - Z.z};
      const int row = lower_left_ ? (H_ - 1 - y) : y;
      uint8_t* px = &background_[(size_t(row) * W_ + x) * C_];
      double t = d.z < 0 ? (s.plane_z - o.z) / d.z : -1.0;
      if (t > 0) {
        const double hx = o.x + t * d.x, hy = o.y + t * d.y;
        if (std::fabs(hx) <= s.plane_half && std::fabs(hy) <= s.plane_half) {
          const Vec3 l = sub(L, Vec3{hx, hy, s.plane_z});
          const double d2 = dot(l, l);
          const double e = std::max(0.0, ls * (l.z / std::sqrt(d2)) / d2);
          for (int c = 0; c < 3; ++c) px[c] = T(s.plane_albedo[c] * (s.ambient + e));
          plane_xy_[(size_t(y) * W_ + x) * 2] = float(hx);
          plane_xy_[(size_t(y) * W_ + x) * 2 + 1] = float(hy);
          continue;
        }
      }
      for (int c = 0; c < 3; ++c) px[c] = T(s.world[c]);
    }
  }
  // a row is a line on the ground plane and the plane is a square: its
  // covered pixels form one interval (checked, not assumed)
  plane_x0_.assign(H_, 0), plane_x1_.assign(H_, -1), plane_dense_.assign(H_, 1);
  for (int y = 0; y < H_; ++y) {
    const float* pxy = &plane_xy_[size_t(y) * W_ * 2];
    int lo = W_, hi = -1;
    for (int x = 0; x < W_; ++x)
      if (pxy[2 * x] == pxy[2 * x]) lo = std::min(lo, x), hi = std::max(hi, x);
    for (int x = lo; x <= hi; ++x)
      if (pxy[2 * x] != pxy[2 * x]) plane_dense_[y] = 0;
    plane_x0_[y] = lo, plane_x1_[y] = hi;
  }
}

inline void Renderer::put(uint8_t* out, int x, int y, float r, float g, float b) const {
  const ToneLut& T = tone();
  const int row = lower_left_ ? (H_ - 1 - y) : y;
  uint8_t* p = out + (size_t(row) * W_ + x) * C_;
  p[0] = T(r);
  p[1] = T(g);
  p[2] = T(b);
}

namespace {

// Scan conversion of a convex polygon in pixel coordinates: calls
// span(y, x0, x1) for every row segment of pixel centres inside (top-left
// style half-open rule on y, [xl, xr) on x).
template <class F>
void scan_convex(const double* px, const double* py, int n, int W, int H, F&& span) {
  double ymin = py[0], ymax = py[0];
  for (int i = 1; i < n; ++i) ymin = std::min(ymin, py[i]), ymax = std::max(ymax, py[i]);
  const int y0 = std::max(0, int(std::ceil(ymin - 0.5))), y1 = std::min(H - 1, int(std::ceil(ymax - 0.5)) - 1);
  for (int y = y0; y <= y1; ++y) {
    const double yc = y + 0.5;
    double xl = 1e300, xr = -1e300;
    for (int i = 0; i < n; ++i) {
      const int j = (i + 1) % n;
      const double ya = py[i], yb = py[j];
      if ((ya <= yc && yc < yb) || (yb <= yc && yc < ya)) {
        const double x = px[i] + (yc - ya) * (px[j] - px[i]) / (yb - ya);
        xl = std::min(xl, x), xr = std::max(xr, x);
      }
    }
    if (xl > xr) continue;
    const int x0 = std::max(0, int(std::ceil(xl - 0.5))), x1 = std::min(W - 1, int(std::ceil(xr - 0.5)) - 1);
    if (x0 <= x1) span(y, x0, x1);
  }
}

// Affine screen-space plane v(x, y) = a x + b y + c through three samples.
struct Plane2 {
  double a = 0, b = 0, c = 0;
  bool fit(const double* x, const double* y, const double* v) {
    const double d = (x[1] - x[0]) * (y[2] - y[0]) - (x[2] - x[0]) * (y[1] - y[0]);
    if (std::fabs(d) < 1e-12) return false;
    a = ((v[1] - v[0]) * (y[2] - y[0]) - (v[2] - v[0]) * (y[1] - y[0])) / d;
    b = ((x[1] - x[0]) * (v[2] - v[0]) - (x[2] - x[0]) * (v[1] - v[0])) / d;
    c = v[0] - a * x[0] - b * y[0];
    return true;
  }
};

}  // namespace

void Renderer::render(const Scene& s, uint8_t* out, DirtyRect* dirty) {
  const Camera& cam = s.cam;
  const int W = W_, H = H_, C = C_;
  const Vec3 o = cam.loc;
  const double ls = light_scale(s.light);
  const Vec3 L = s.light.loc;
  const double amb = s.ambient;
  const ToneLut& T = tone();

  auto row_ptr = [&](int y) { return out + size_t(lower_left_ ? (H - 1 - y) : y) * W * C; };
  if (dirty && dirty->known) {
    // only the previous frame's boxes and shadows differ from the background
    if (!dirty->empty()) {
      const bool rows = dirty->lo.size() == size_t(H);
      for (int y = dirty->y0; y <= dirty->y1; ++y) {
        const int a = rows ? dirty->lo[size_t(y)] : dirty->x0, b = rows ? dirty->hi[size_t(y)] : dirty->x1;
        if (a > b) continue;
        uint8_t* r = row_ptr(y);
        const size_t off = size_t(a) * C;
        std::memcpy(r + off, background_.data() + (r - out) + off, size_t(b - a + 1) * C);
      }
    }
  } else {
    std::memcpy(out, background_.data(), background_.size());
  }
  DirtyRect touched;
  if (dirty) {   // reuse the previous record's row arrays (no allocation per frame)
    touched.lo.swap(dirty->lo);
    touched.hi.swap(dirty->hi);
    touched.lo.assign(size_t(H), 1 << 30);
    touched.hi.assign(size_t(H), -1);
  }

  // ---- shadows: each box's shadow hull on the ground plane, projected to
  // the image (a projective map keeps it convex) and span-filled ----
  for (const Box& b : s.boxes) {
    auto cs = b.corners();
    P2 pts[8], hull[17];
    bool above = true;
    for (int i = 0; i < 8; ++i) {
      if (cs[i].z >= L.z - 1e-9) above = false;
      const double t = (s.plane_z - L.z) / (cs[i].z - L.z);
      pts[i][0] = L.x + t * (cs[i].x - L.x);
      pts[i][1] = L.y + t * (cs[i].y - L.y);
    }
    if (!above) continue;   // light inside/below the box: no ground shadow
    const int nh = convex_hull(pts, 8, hull);
    if (nh < 3) continue;
    double hx[17], hy[17];
    bool visible = true;
    for (int i = 0; i < nh && visible; ++i)
      visible = cam.project(Vec3{hull[i][0], hull[i][1], s.plane_z}, &hx[i], &hy[i]);
    if (!visible) continue;
    scan_convex(hx, hy, nh, W, H, [&](int y, int x0, int x1) {
      touched.add(y, x0, x1);
      const float* pxy = &plane_xy_[size_t(y) * W * 2];
      uint8_t* r = row_ptr(y);
      if (plane_dense_[y]) {
        const int a = std::max(x0, plane_x0_[y]), b = std::min(x1, plane_x1_[y]);
        if (C == 4) {
          // alpha is 255 in the background: one 32-bit pattern per pixel
          const uint32_t v = uint32_t(shadow_rgb_[0]) | uint32_t(shadow_rgb_[1]) << 8 |
                             uint32_t(shadow_rgb_[2]) << 16 | 0xff000000u;
          for (int x = a; x <= b; ++x) std::memcpy(r + size_t(x) * 4, &v, 4);
        } else {
          for (int x = a; x <= b; ++x) {
            uint8_t* p = r + size_t(x) * C;
            p[0] = shadow_rgb_[0], p[1] = shadow_rgb_[1], p[2] = shadow_rgb_[2];
          }
        }
        return;
      }
      for (int x = x0; x <= x1; ++x) {
        if (pxy[2 * x] != pxy[2 * x]) continue;   // not on the ground plane
        uint8_t* p = r + size_t(x) * C;
        p[0] = shadow_rgb_[0];
        p[1] = shadow_rgb_[1];
        p[2] = shadow_rgb_[2];
      }
    });
  }

  // ---- boxes: front faces as two triangles each, Gouraud-interpolated
  // point-light Lambert, perspective-correct depth test for several boxes ----
  const bool need_depth = s.boxes.size() > 1;
  if (need_depth) {
    // stores 1/depth, 0 = far; only the last frame's box spans are non-zero
    if (depth_.size() != size_t(W) * H) {
      depth_.assign(size_t(W) * H, 0.f);
    } else if (!depth_rect_.empty()) {
      for (int y = depth_rect_.y0; y <= depth_rect_.y1; ++y)
        std::fill_n(&depth_[size_t(y) * W + depth_rect_.x0], depth_rect_.x1 - depth_rect_.x0 + 1, 0.f);
    }
    depth_rect_.reset();
  }
  for (size_t bi = 0; bi < s.boxes.size(); ++bi) {
    const Box& b = s.boxes[bi];
    const double hv[3] = {b.half.x, b.half.y, b.half.z};
    for (int axis = 0; axis < 3; ++axis) {
      for (int sign = -1; sign <= 1; sign += 2) {
        Vec3 nl{0, 0, 0};
        (axis == 0 ? nl.x : axis == 1 ? nl.y : nl.z) = sign;
        const Vec3 n = mul(b.rot, nl);
        const Vec3 fc = add(b.center, scale(n, hv[axis]));
        if (dot(n, sub(o, fc)) <= 0) continue;   // back face
        const int j = (axis + 1) % 3, k = (axis + 2) % 3;
        Vec3 ej{0, 0, 0}, ek{0, 0, 0};
        (j == 0 ? ej.x : j == 1 ? ej.y : ej.z) = hv[j];
        (k == 0 ? ek.x : k == 1 ? ek.y : ek.z) = hv[k];
        const Vec3 wj = mul(b.rot, ej), wk = mul(b.rot, ek);
        const Vec3 q[4] = {add(fc, add(wj, wk)), add(fc, sub(wk, wj)), sub(fc, add(wj, wk)),
                           add(fc, sub(wj, wk))};
        double px[4], py[4], dep[4], inten[4], invd[4];
        bool vis = true;
        for (int i = 0; i < 4; ++i) {
          vis &= cam.project(q[i], &px[i], &py[i], &dep[i]);
          invd[i] = dep[i] > 0 ? 1.0 / dep[i] : 0.0;
          const Vec3 l = sub(L, q[i]);
          const double d2 = dot(l, l);
          double e = ls * std::max(0.0, dot(n, l) / std::sqrt(d2)) / d2;
          if (e > 0 && s.boxes.size() > 1)
            for (size_t oi = 0; oi < s.boxes.size(); ++oi)
              if (oi != bi && ray_hits_box(s.boxes[oi], q[i], l, 1e-6, 1.0)) {
                e = 0;
                break;
              }
          inten[i] = amb + e;
        }
        if (!vis) continue;
        // grey albedo (the Cube scene's): the three channels share one table index
        const bool gray = b.albedo[0] == b.albedo[1] && b.albedo[1] == b.albedo[2];
        const float a0 = b.albedo[0] * 4096.f, a1 = b.albedo[1] * 4096.f, a2 = b.albedo[2] * 4096.f;
        static const int tri[2][3] = {{0, 1, 2}, {0, 2, 3}};
        for (const auto& t : tri) {
          const double tx[3] = {px[t[0]], px[t[1]], px[t[2]]}, ty[3] = {py[t[0]], py[t[1]], py[t[2]]};
          const double ti[3] = {inten[t[0]], inten[t[1]], inten[t[2]]};
          const double tz[3] = {invd[t[0]], invd[t[1]], invd[t[2]]};
          Plane2 ip, zp;
          if (!ip.fit(tx, ty, ti) || !zp.fit(tx, ty, tz)) continue;
          scan_convex(tx, ty, 3, W, H, [&](int y, int x0, int x1) {
            touched.add(y, x0, x1);
            if (need_depth) depth_rect_.add(y, x0, x1);
            uint8_t* r = row_ptr(y);
            const double yc = y + 0.5;
            const float I0 = float(ip.a * (x0 + 0.5) + ip.b * yc + ip.c), dI = float(ip.a);
            const float Z0 = float(zp.a * (x0 + 0.5) + zp.b * yc + zp.c), dZ = float(zp.a);
            float* zrow = need_depth ? &depth_[size_t(y) * W] : nullptr;
            // chunks of the span: the tone-table indices of 4 pixels per SSE
            // op first (I = I0 + dI * k, clamped to [0, 4096]), then the
            // lookups and stores
            constexpr int kChunk = 64;
            alignas(16) int i0[kChunk], i1[kChunk], i2[kChunk];
            const __m128 vI0 = _mm_set1_ps(I0), vdI = _mm_set1_ps(dI), lo = _mm_setzero_ps();
            const __m128 hi = _mm_set1_ps(4096.f), va0 = _mm_set1_ps(a0), va1 = _mm_set1_ps(a1);
            const __m128 va2 = _mm_set1_ps(a2), four = _mm_set1_ps(4.f);
            for (int xb = x0; xb <= x1; xb += kChunk) {
              const int n = std::min(kChunk, x1 - xb + 1);
              const float kb = float(xb - x0);
              __m128 kv = _mm_add_ps(_mm_set1_ps(kb), _mm_setr_ps(0.f, 1.f, 2.f, 3.f));
              for (int k = 0; k < n; k += 4, kv = _mm_add_ps(kv, four)) {
                const __m128 I = _mm_add_ps(vI0, _mm_mul_ps(vdI, kv));
                _mm_store_si128(reinterpret_cast<__m128i*>(i0 + k),
                                _mm_cvttps_epi32(_mm_min_ps(_mm_max_ps(_mm_mul_ps(va0, I), lo), hi)));
                if (gray) continue;
                _mm_store_si128(reinterpret_cast<__m128i*>(i1 + k),
                                _mm_cvttps_epi32(_mm_min_ps(_mm_max_ps(_mm_mul_ps(va1, I), lo), hi)));
                _mm_store_si128(reinterpret_cast<__m128i*>(i2 + k),
                                _mm_cvttps_epi32(_mm_min_ps(_mm_max_ps(_mm_mul_ps(va2, I), lo), hi)));
              }
              uint8_t* p = r + size_t(xb) * C;
              if (zrow) {
                float* zr = zrow + xb;
                for (int k = 0; k < n; ++k, p += C) {
                  const float Z = Z0 + dZ * (kb + float(k));
                  if (Z <= zr[k]) continue;
                  zr[k] = Z;
                  if (gray) p[0] = p[1] = p[2] = T.v[i0[k]];
                  else p[0] = T.v[i0[k]], p[1] = T.v[i1[k]], p[2] = T.v[i2[k]];
                }
              } else if (C == 4 && gray) {
                for (int k = 0; k < n; ++k) std::memcpy(p + size_t(k) * 4, &T.gray4[i0[k]], 4);
              } else if (C == 4) {
                for (int k = 0; k < n; ++k) {
                  const uint32_t v = uint32_t(T.v[i0[k]]) | uint32_t(T.v[i1[k]]) << 8 |
                                     uint32_t(T.v[i2[k]]) << 16 | 0xff000000u;
                  std::memcpy(p + size_t(k) * 4, &v, 4);
                }
              } else if (gray) {
                for (int k = 0; k < n; ++k, p += C) p[0] = p[1] = p[2] = T.v[i0[k]];
              } else {
                for (int k = 0; k < n; ++k, p += C) p[0] = T.v[i0[k]], p[1] = T.v[i1[k]], p[2] = T.v[i2[k]];
              }
            }
          });
        }
      }
    }
  }
  if (dirty) {
    touched.known = true;
    *dirty = std::move(touched);
  }
}

void render(const Scene& s, uint8_t* out, int channels, bool lower_left) {
  Renderer r(s, channels, lower_left);
  r.render(s, out);
}

void render_mesh(const Camera& cam, const std::vector<float>& verts, const std::vector<int>& tris,
                 const MeshStyle& style, uint8_t* out, int channels, bool lower_left) {
  const int W = cam.width, H = cam.height;
  const ToneLut& T = tone();
  const size_t nv = verts.size() / 3;
  // project every vertex once (Camera::project's arithmetic, focal length
  // hoisted), and keep the range of pixel-centre columns / rows each vertex
  // bounds: a triangle's candidate pixels are then integer min/max of its
  // corners' ranges (rounding is monotone, so this equals rounding the
  // triangle's float bounding box)
  // (branch-free loops over flat arrays: the compiler vectorises both)
  // per-thread scratch, reused across calls (every entry is written below)
  thread_local std::vector<float> sx, sy, sz;
  thread_local std::vector<int> cx0, cx1, cy0, cy1;
  thread_local std::vector<uint8_t> ok;
  for (auto* v : {&sx, &sy, &sz}) v->resize(nv);
  for (auto* v : {&cx0, &cx1, &cy0, &cy1}) v->resize(nv);
  ok.resize(nv);
  const double f = cam.focal_px(), hw = 0.5 * W, hh = 0.5 * H;
  const Mat3& R = cam.rot;
  const double lx = cam.loc.x, ly = cam.loc.y, lz = cam.loc.z;
  for (size_t i = 0; i < nv; ++i) {
    const double wx = double(verts[3 * i]) - lx, wy = double(verts[3 * i + 1]) - ly, wz = double(verts[3 * i + 2]) - lz;
    const double cx = R[0] * wx + R[3] * wy + R[6] * wz;   // mul_t(rot, w - loc)
    const double cy = R[1] * wx + R[4] * wy + R[7] * wz;
    const double cz = R[2] * wx + R[5] * wy + R[8] * wz;
    ok[i] = cz < -1e-12;
    sz[i] = float(-cz);
    const double d = ok[i] ? -cz : 1.0;   // behind the camera: any finite value, never used
    sx[i] = float(hw + f * cx / d), sy[i] = float(hh - f * cy / d);
  }
  for (size_t i = 0; i < nv; ++i) {
    const float px = std::min(std::max(sx[i] - 0.5f, -1e9f), 1e9f);
    const float py = std::min(std::max(sy[i] - 0.5f, -1e9f), 1e9f);
    const int fx = int(px), fy = int(py);   // truncation, then floor / ceil fix-ups
    cx1[i] = fx - (px < float(fx)), cx0[i] = fx + (px > float(fx));
    cy1[i] = fy - (py < float(fy)), cy0[i] = fy + (py > float(fy));
  }
  thread_local std::vector<float> depth, shade;
  depth.assign(size_t(W) * H, std::numeric_limits<float>::infinity());
  shade.assign(size_t(W) * H, -1.f);
  Vec3 L = style.light_dir;
  const double ln = std::sqrt(dot(L, L));
  L = scale(L, -1.0 / ln);   // towards the light
  for (size_t t = 0; t + 2 < tris.size(); t += 3) {
    const int a = tris[t], b = tris[t + 1], c = tris[t + 2];
    if (!ok[a] || !ok[b] || !ok[c]) continue;
    // pixel centres (x + 0.5, y + 0.5) inside the triangle's bounding box; a
    // dense mesh seen at 64x64 has mostly sub-pixel triangles that cover no
    // centre at all -- they are rejected before any shading work
    const int x0 = std::max(0, std::min({cx0[a], cx0[b], cx0[c]}));
    const int x1 = std::min(W - 1, std::max({cx1[a], cx1[b], cx1[c]}));
    if (x0 > x1) continue;
    const int y0 = std::max(0, std::min({cy0[a], cy0[b], cy0[c]}));
    const int y1 = std::min(H - 1, std::max({cy1[a], cy1[b], cy1[c]}));
    if (y0 > y1) continue;
    const float area = (sx[b] - sx[a]) * (sy[c] - sy[a]) - (sx[c] - sx[a]) * (sy[b] - sy[a]);
    if (std::fabs(area) < 1e-12f) continue;
    const float inv = 1.f / area;
    float lam = -1.f;   // face shading, computed on the first covered pixel
    for (int y = y0; y <= y1; ++y) {
      const float py = y + 0.5f;
      for (int x = x0; x <= x1; ++x) {
        const float px = x + 0.5f;
        const float w0 = ((sx[b] - px) * (sy[c] - py) - (sx[c] - px) * (sy[b] - py)) * inv;
        const float w1 = ((sx[c] - px) * (sy[a] - py) - (sx[a] - px) * (sy[c] - py)) * inv;
        const float w2 = 1.f - w0 - w1;
        if (w0 < 0.f || w1 < 0.f || w2 < 0.f) continue;
        const float z = w0 * sz[a] + w1 * sz[b] + w2 * sz[c];
        float& zb = depth[size_t(y) * W + x];
        if (z >= zb) continue;
        if (lam < 0.f) {
          // face normal (world) for shading, two-sided
          const Vec3 A{verts[3 * a], verts[3 * a + 1], verts[3 * a + 2]};
          const Vec3 B{verts[3 * b], verts[3 * b + 1], verts[3 * b + 2]};
          const Vec3 C{verts[3 * c], verts[3 * c + 1], verts[3 * c + 2]};
          const Vec3 e1 = sub(B, A), e2 = sub(C, A);
          Vec3 n{e1.y * e2.z - e1.z * e2.y, e1.z * e2.x - e1.x * e2.z, e1.x * e2.y - e1.y * e2.x};
          const double nn = std::sqrt(dot(n, n));
          if (nn < 1e-18) goto next_triangle;   // degenerate in 3-D: never drawn
          n = scale(n, 1.0 / nn);
          lam = float(std::fabs(dot(n, L)));
        }
        zb = z;
        shade[size_t(y) * W + x] = lam;
      }
    }
  next_triangle:;
  }
  for (int y = 0; y < H; ++y) {
    const int row = lower_left ? (H - 1 - y) : y;
    for (int x = 0; x < W; ++x) {
      uint8_t* p = out + (size_t(row) * W + x) * channels;
      const float s = shade[size_t(y) * W + x];
      for (int k = 0; k < 3; ++k)
        p[k] = s < 0.f ? T(style.background[k]) : T(style.albedo[k] * (float(style.ambient) + (1.f - float(style.ambient)) * s));
      if (channels == 4) p[3] = 255;
    }
  }
}

}  // namespace sim
}  // namespace btn
