// RigidWorld implementation (see physics.h).
#include "physics.h"

#include <algorithm>
#include <cmath>

namespace btn {
namespace sim {

namespace {

Vec3 add(Vec3 a, Vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
Vec3 sub(Vec3 a, Vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
Vec3 scl(Vec3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
double dot(Vec3 a, Vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
Vec3 cross(Vec3 a, Vec3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
double norm(Vec3 a) { return std::sqrt(dot(a, a)); }

Mat3 matmul(const Mat3& a, const Mat3& b) {
  Mat3 c{};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) c[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
  return c;
}

// Rotation by angle |w| about w (Rodrigues).
Mat3 rotation(Vec3 w) {
  const double th = norm(w);
  if (th < 1e-12) return {1, 0, 0, 0, 1, 0, 0, 0, 1};
  const Vec3 k = scl(w, 1.0 / th);
  const double c = std::cos(th), s = std::sin(th), t = 1 - c;
  return {t * k.x * k.x + c,       t * k.x * k.y - s * k.z, t * k.x * k.z + s * k.y,
          t * k.x * k.y + s * k.z, t * k.y * k.y + c,       t * k.y * k.z - s * k.x,
          t * k.x * k.z - s * k.y, t * k.y * k.z + s * k.x, t * k.z * k.z + c};
}

// Gram-Schmidt on the columns (keeps R a rotation under repeated updates).
void orthonormalize(Mat3& r) {
  Vec3 c0{r[0], r[3], r[6]}, c1{r[1], r[4], r[7]};
  c0 = scl(c0, 1.0 / norm(c0));
  c1 = sub(c1, scl(c0, dot(c0, c1)));
  c1 = scl(c1, 1.0 / norm(c1));
  const Vec3 c2 = cross(c0, c1);
  r = {c0.x, c1.x, c2.x, c0.y, c1.y, c2.y, c0.z, c1.z, c2.z};
}

// World-space inverse inertia applied to a vector: R * diag(inv_local) * R^T * x.
Vec3 inv_inertia_world(const Mat3& R, Vec3 inv_local, Vec3 x) {
  Vec3 l = mul_t(R, x);
  l = {l.x * inv_local.x, l.y * inv_local.y, l.z * inv_local.z};
  return mul(R, l);
}

}  // namespace

RigidWorld::RigidWorld(double plane_z, RigidParams p) : plane_z_(plane_z), p_(p) {}

void RigidWorld::reset(const std::vector<Box>& boxes) {
  bodies_.assign(boxes.size(), Body());
  for (size_t i = 0; i < boxes.size(); ++i) {
    const Vec3 h = boxes[i].half;
    const double m = 8.0 * h.x * h.y * h.z;   // density 1
    Body& s = bodies_[i];
    s.inv_mass = 1.0 / m;
    // solid box: I = m/3 * (hy^2 + hz^2, ...) with half extents h
    s.inv_inertia = {3.0 / (m * (h.y * h.y + h.z * h.z)), 3.0 / (m * (h.x * h.x + h.z * h.z)),
                     3.0 / (m * (h.x * h.x + h.y * h.y))};
  }
}

void RigidWorld::contact_plane(Box& b, Body& s, double h) {
  const Vec3 n{0, 0, 1};
  auto corners = b.corners();
  double deepest = 0;
  for (const Vec3& c : corners) {
    const double pen = plane_z_ - c.z;
    if (pen <= 0) continue;
    deepest = std::max(deepest, pen);
    const Vec3 r = sub(c, b.center);
    const Vec3 vc = add(s.v, cross(s.w, r));
    const double vn = dot(vc, n);
    if (vn >= 0) continue;
    const Vec3 rn = cross(r, n);
    const double kn = s.inv_mass + dot(cross(inv_inertia_world(b.rot, s.inv_inertia, rn), r), n);
    // no bounce for slow contacts (resting)
    const double e = vn < -1.0 ? p_.restitution : 0.0;
    const double jn = -(1 + e) * vn / kn;
    Vec3 J = scl(n, jn);
    // Coulomb friction on the tangential slip
    const Vec3 vt = sub(vc, scl(n, vn));
    const double vts = norm(vt);
    if (vts > 1e-9) {
      const Vec3 t = scl(vt, 1.0 / vts);
      const Vec3 rt = cross(r, t);
      const double kt = s.inv_mass + dot(cross(inv_inertia_world(b.rot, s.inv_inertia, rt), r), t);
      const double jt = std::max(-vts / kt, -p_.friction * jn);
      J = add(J, scl(t, jt));
    }
    s.v = add(s.v, scl(J, s.inv_mass));
    s.w = add(s.w, inv_inertia_world(b.rot, s.inv_inertia, cross(r, J)));
  }
  (void)h;
  if (deepest > 0) b.center.z += 0.8 * deepest;   // positional projection out of the plane
}

void RigidWorld::contact_pair(Box& a, Body& sa, Box& b, Body& sb) {
  // bounding-sphere proxy (radius = mean half extent): cheap separation
  const double ra = (a.half.x + a.half.y + a.half.z) / 3.0, rb = (b.half.x + b.half.y + b.half.z) / 3.0;
  Vec3 d = sub(b.center, a.center);
  const double dist = norm(d);
  const double pen = ra + rb - dist;
  if (pen <= 0 || dist < 1e-9) return;
  const Vec3 n = scl(d, 1.0 / dist);
  const double vn = dot(sub(sb.v, sa.v), n);
  const double wsum = sa.inv_mass + sb.inv_mass;
  if (vn < 0) {
    const double j = -(1 + p_.restitution) * vn / wsum;
    sa.v = sub(sa.v, scl(n, j * sa.inv_mass));
    sb.v = add(sb.v, scl(n, j * sb.inv_mass));
  }
  const double corr = 0.8 * pen / wsum;
  a.center = sub(a.center, scl(n, corr * sa.inv_mass));
  b.center = add(b.center, scl(n, corr * sb.inv_mass));
}

void RigidWorld::step(std::vector<Box>& boxes, double dt) {
  if (bodies_.size() != boxes.size()) reset(boxes);
  const double h = dt / std::max(1, p_.substeps);
  const double ld = std::exp(-p_.linear_damping * h), ad = std::exp(-p_.angular_damping * h);
  for (int sub_i = 0; sub_i < p_.substeps; ++sub_i) {
    for (size_t i = 0; i < boxes.size(); ++i) {
      Body& s = bodies_[i];
      s.v.z += p_.gravity * h;
      s.v = scl(s.v, ld);
      s.w = scl(s.w, ad);
    }
    for (int it = 0; it < p_.iterations; ++it) {
      for (size_t i = 0; i < boxes.size(); ++i) contact_plane(boxes[i], bodies_[i], h);
      for (size_t i = 0; i < boxes.size(); ++i)
        for (size_t j = i + 1; j < boxes.size(); ++j) contact_pair(boxes[i], bodies_[i], boxes[j], bodies_[j]);
    }
    for (size_t i = 0; i < boxes.size(); ++i) {
      Box& b = boxes[i];
      Body& s = bodies_[i];
      b.center = add(b.center, scl(s.v, h));
      b.rot = matmul(rotation(scl(s.w, h)), b.rot);
      orthonormalize(b.rot);
    }
  }
}

double RigidWorld::kinetic_energy(const std::vector<Box>& boxes) const {
  double e = 0;
  for (size_t i = 0; i < boxes.size() && i < bodies_.size(); ++i) {
    const Body& s = bodies_[i];
    const Vec3 wl = mul_t(boxes[i].rot, s.w);
    e += 0.5 * dot(s.v, s.v) / s.inv_mass + 0.5 * (wl.x * wl.x / s.inv_inertia.x + wl.y * wl.y / s.inv_inertia.y +
                                                   wl.z * wl.z / s.inv_inertia.z);
  }
  return e;
}

}  // namespace sim
}  // namespace btn
