// Headless CPU renderer for the blendtorch stand-in producers.
//
// Blender/Eevee is not available in this stack, so the producers that feed
// the benchmark and the tests render their scenes here instead.  The scene
// model covers what the reference's example scenes contain
// (reference: examples/datagen/cube.blend, falling_cubes.blend -- camera,
// point light, ground plane, one or more boxes):
//   * a pinhole camera with Blender's conventions (looks down its local -Z,
//     +Y up, sensor_fit AUTO, focal length in pixels = lens/sensor * max(W,H));
//   * a point light with inverse-square falloff plus ambient term;
//   * an infinite-ish ground plane (square of half-size `plane_half`) that
//     receives box shadows (shadow rays against each oriented box);
//   * convex boxes drawn by rasterising their front faces with per-pixel
//     Lambert shading.
// Projection helpers follow btb.Camera (reference: pkg_blender/blendtorch/btb/
// camera.py:84-162): NDC in [-1,1], pixel = (ndc+1)/2 * [W,H] with the y axis
// flipped for the upper-left origin -- no half-pixel offset.
#pragma once

#include <array>
#include <cstdint>
#include <vector>

namespace btn {
namespace sim {

struct Vec3 {
  double x = 0, y = 0, z = 0;
};

using Mat3 = std::array<double, 9>;   // row major

Mat3 euler_xyz(double rx, double ry, double rz);   // Blender 'XYZ' euler: Rz*Ry*Rx
Vec3 mul(const Mat3& m, const Vec3& v);
Vec3 mul_t(const Mat3& m, const Vec3& v);          // m^T v

struct Camera {
  int width = 640, height = 480;
  double lens_mm = 50.0, sensor_mm = 36.0;
  double clip_start = 0.1, clip_end = 100.0;
  Vec3 loc;
  Mat3 rot;      // camera-to-world rotation
  double focal_px() const;
  // world -> pixel (upper-left origin); returns false if behind the camera.
  bool project(const Vec3& w, double* px, double* py, double* depth = nullptr) const;
};

struct Box {
  Vec3 center;
  Vec3 half{1, 1, 1};
  Mat3 rot;                                   // local-to-world
  std::array<float, 3> albedo{0.8f, 0.8f, 0.8f};
  // The 8 corners in Blender's default-cube vertex order.
  std::array<Vec3, 8> corners() const;
};

struct Light {
  Vec3 loc;
  double power = 1000.0;   // W-ish; scaled so the default scene is well exposed
};

struct Scene {
  Camera cam;
  Light light;
  double ambient = 0.08;
  double plane_z = -2.0;
  double plane_half = 10.0;
  std::array<float, 3> plane_albedo{0.8f, 0.8f, 0.8f};
  std::array<float, 3> world{0.051f, 0.051f, 0.051f};
  std::vector<Box> boxes;
};

// The default-cube scene of examples/datagen/cube.blend (640x480, camera at
// (7.359,-6.926,4.958) with Blender's default rotation, light at
// (4.076,1.005,5.904), ground plane at z=-2).
Scene cube_scene();
// examples/datagen/falling_cubes.blend stand-in: 7 boxes, raised camera.
Scene falling_cubes_scene();

// Bounding rectangle (image coordinates, row 0 = top, inclusive) of every
// pixel a frame wrote over the background.  A buffer that is rendered into
// again and again (a shared-memory ring slot) keeps the rectangle its last
// frame left; the next render restores the background inside it only,
// instead of copying the whole background.  `known` false = the buffer's
// content is unknown (fresh slot): full background copy.
// With `lo` / `hi` sized to the image height, each row also keeps the span
// it wrote (a box and its shadow cover ~57 % of their bounding rectangle, so
// a restore over the row spans moves that much less memory).
struct DirtyRect {
  int x0 = 1 << 30, y0 = 1 << 30, x1 = -1, y1 = -1;
  bool known = false;
  std::vector<int> lo, hi;   // per image row [lo, hi]; empty = rectangle only
  bool empty() const { return x1 < x0 || y1 < y0; }
  void reset() { x0 = y0 = 1 << 30, x1 = y1 = -1; }
  void add(int y, int a, int b) {
    y0 = y < y0 ? y : y0, y1 = y > y1 ? y : y1;
    x0 = a < x0 ? a : x0, x1 = b > x1 ? b : x1;
    if (!lo.empty()) {
      int& l = lo[static_cast<unsigned>(y)];
      int& h = hi[static_cast<unsigned>(y)];
      l = a < l ? a : l, h = b > h ? b : h;
    }
  }
};

// Frame renderer.  Camera, light and ground plane are static for the life of
// a Renderer, so their shading (the whole background) is computed once and
// cached together with each pixel's ground-plane hit point; a frame then costs
// one background copy, span fills of the boxes' projected shadow hulls and
// scan conversion of the boxes' front faces.
// Output: H*W*channels bytes, row-major HWC uint8, channels 3 or 4 (alpha =
// 255); `lower_left` stores row 0 = bottom image row (OpenGL readback order).
class Renderer {
 public:
  Renderer(const Scene& s, int channels, bool lower_left);
  // dirty: the rectangle `out`'s previous frame left (updated to this
  // frame's); nullptr = `out` holds anything, copy the whole background
  void render(const Scene& s, uint8_t* out, DirtyRect* dirty = nullptr);
  int width() const { return W_; }
  int height() const { return H_; }
  int channels() const { return C_; }
  // the stored bytes of a frame without boxes (what a DirtyRect restores)
  const std::vector<uint8_t>& background() const { return background_; }

 private:
  void put(uint8_t* out, int x, int y, float r, float g, float b) const;
  int W_, H_, C_;
  bool lower_left_;
  std::vector<uint8_t> background_;     // final HWC bytes, boxes absent
  std::vector<float> plane_xy_;         // per pixel ground hit (x,y); NaN = no hit
  // per image row: the ground plane covers pixels [plane_x0_, plane_x1_] and
  // nothing else (plane_dense_ = 1), or the row needs the per-pixel test
  std::vector<int> plane_x0_, plane_x1_;
  std::vector<uint8_t> plane_dense_;
  uint8_t shadow_rgb_[3];
  std::vector<float> depth_;             // 1/depth per pixel, zero outside depth_rect_
  DirtyRect depth_rect_;                // pixels of depth_ the last frame wrote
};

// Triangle-mesh rendering (z-buffered, two-sided Lambert from a directional
// light + ambient) over a uniform background -- used for parametric shapes
// (the densityopt supershapes).  verts: N x 3 world coordinates; tris:
// M x 3 vertex indices.  Output HWC u8 (linear values tone-mapped like the
// box renderer), row 0 = top unless lower_left.
struct MeshStyle {
  std::array<float, 3> albedo{0.8f, 0.8f, 0.8f};
  std::array<float, 3> background{0.05f, 0.05f, 0.05f};
  Vec3 light_dir{-0.4, -0.6, -0.7};   // direction the light travels
  double ambient = 0.15;
};
void render_mesh(const Camera& cam, const std::vector<float>& verts, const std::vector<int>& tris,
                 const MeshStyle& style, uint8_t* out, int channels, bool lower_left);

// One-shot convenience wrapper (builds a Renderer per call).
void render(const Scene& s, uint8_t* out, int channels, bool lower_left);

}  // namespace sim
}  // namespace btn
