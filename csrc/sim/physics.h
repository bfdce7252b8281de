// Rigid-body dynamics for the falling-cubes stand-in producer.
//
// The reference's examples/datagen/falling_cubes.blend.py drops 7 cubes from
// random poses (z in [6, 12]) in `pre_animation` and lets Blender's Bullet
// rigid-body world settle them on the ground plane over the 100-frame
// episode.  Blender is not part of this stack, so cubesim steps this small
// solver instead: gravity, semi-implicit Euler with exponential-map rotation
// updates, box-plane contact resolved with sequential impulses at the
// penetrating corners (restitution + Coulomb friction, positional projection),
// and cube-cube contact approximated by bounding spheres.  It is a stand-in
// for Bullet, good enough that the rendered cubes fall, tumble, collide and
// come to rest; it is not meant to reproduce Bullet trajectories.
#pragma once

#include <vector>

#include "raster.h"

namespace btn {
namespace sim {

struct RigidParams {
  double gravity = -9.81;
  double restitution = 0.3;
  double friction = 0.5;
  double linear_damping = 0.02;    // per second
  double angular_damping = 0.1;    // per second
  int substeps = 8;
  int iterations = 4;              // contact solver passes per substep
};

class RigidWorld {
 public:
  RigidWorld(double plane_z, RigidParams p = RigidParams());
  // Zero velocities (start of an episode); masses from box volumes (density 1).
  void reset(const std::vector<Box>& boxes);
  // Advance the boxes by dt seconds.
  void step(std::vector<Box>& boxes, double dt);
  // Kinetic energy of all bodies (tests: settling).
  double kinetic_energy(const std::vector<Box>& boxes) const;

 private:
  struct Body {
    Vec3 v, w;             // linear / angular velocity (world)
    double inv_mass = 1;
    Vec3 inv_inertia;      // local principal axes (box)
  };
  void contact_plane(Box& b, Body& s, double h);
  void contact_pair(Box& a, Body& sa, Box& b, Body& sb);
  double plane_z_;
  RigidParams p_;
  std::vector<Body> bodies_;
};

}  // namespace sim
}  // namespace btn
