// supershapesim -- headless stand-in for a Blender instance running
// examples/densityopt/supershape.blend.py (reference: :8-59).
//
//   supershapesim [--] -btid I -btseed S -btsockets DATA=... CTRL=... [--no-gamma]
//                 [--uv N] [--size PX]
//
// Per frame: non-blocking receive on the CTRL duplex (PAIR, bound; messages
// {'btid','btmid','shape_params': f4[N,2,6], 'shape_ids': i8[N]}, sent by
// btt.DuplexChannel).  A new message replaces the pending work; while work is
// pending, one supershape per frame is meshed on a uv grid, rendered 64x64
// (SOLID-style shading, gamma 2.2 as OffScreenRenderer(gamma_coeff=2.2)) and
// published on DATA as {'btid', 'image': u1[64,64,3], 'shape_id': int}.
//
// Supershape (3-D superformula, cheind/supershape convention): row k of the
// params is (m, a, b, n1, n2, n3) and
//   r(phi) = (|cos(m phi / 4) / a|^n2 + |sin(m phi / 4) / b|^n3)^(-1/n1)
//   x = r1(u) cos u r2(v) cos v,  y = r1(u) sin u r2(v) cos v,  z = r2(v) sin v
// with u in [-pi, pi] (longitude, params row 0) and v in [-pi/2, pi/2].
#include <atomic>
#include <chrono>
#include <cmath>
#include <csignal>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../codec/pickle_codec.h"
#include "../transport/zmtp.h"
#include "raster.h"

using namespace btn;

namespace {

std::atomic<bool> g_stop{false};
void on_signal(int) { g_stop = true; }

double superformula(const float* p, double phi) {
  const double m = p[0], a = p[1], b = p[2], n1 = p[3], n2 = p[4], n3 = p[5];
  const double t1 = std::pow(std::fabs(std::cos(m * phi / 4.0) / a), n2);
  const double t2 = std::pow(std::fabs(std::sin(m * phi / 4.0) / b), n3);
  const double s = t1 + t2;
  return s > 0 ? std::pow(s, -1.0 / n1) : 0.0;
}

void supershape_mesh(const float* params, int uv, std::vector<float>& verts, std::vector<int>& tris) {
  const double pi = 3.14159265358979323846;
  verts.resize(size_t(uv) * uv * 3);
  std::vector<double> r1(uv), r2(uv), cu(uv), su(uv), cv(uv), sv(uv);
  for (int i = 0; i < uv; ++i) {
    const double u = -pi + 2 * pi * i / (uv - 1);
    const double v = -pi / 2 + pi * i / (uv - 1);
    r1[i] = superformula(params, u);
    r2[i] = superformula(params + 6, v);
    cu[i] = std::cos(u), su[i] = std::sin(u), cv[i] = std::cos(v), sv[i] = std::sin(v);
  }
  for (int i = 0; i < uv; ++i)       // latitude rows
    for (int j = 0; j < uv; ++j) {   // longitude columns
      float* p = &verts[(size_t(i) * uv + j) * 3];
      p[0] = float(r1[j] * cu[j] * r2[i] * cv[i]);
      p[1] = float(r1[j] * su[j] * r2[i] * cv[i]);
      p[2] = float(r2[i] * sv[i]);
    }
  if (tris.empty()) {
    for (int i = 0; i + 1 < uv; ++i)
      for (int j = 0; j + 1 < uv; ++j) {
        const int a = i * uv + j, b = a + 1, c = a + uv, d = c + 1;
        tris.insert(tris.end(), {a, b, d, a, d, c});
      }
  }
}

}  // namespace

int main(int argc, char** argv) {
  std::vector<std::string> v;
  int start = 1;
  for (int i = 1; i < argc; ++i)
    if (std::strcmp(argv[i], "--") == 0) {
      start = i + 1;
      break;
    }
  for (int i = start; i < argc; ++i) v.push_back(argv[i]);
  int btid = 0, uv = 100, size = 64;
  int bench = 0;   // --bench N: render N pseudo-random shapes, print ms/shape + checksum, exit
  bool gamma = true;
  std::map<std::string, std::string> sockets;
  for (size_t i = 0; i < v.size(); ++i) {
    if (v[i] == "-btid" && i + 1 < v.size()) btid = std::stoi(v[++i]);
    else if (v[i] == "-btseed" && i + 1 < v.size()) ++i;
    else if (v[i] == "-btsockets") {
      while (i + 1 < v.size() && v[i + 1].rfind("-", 0) != 0) {
        ++i;
        auto eq = v[i].find('=');
        if (eq != std::string::npos) sockets[v[i].substr(0, eq)] = v[i].substr(eq + 1);
      }
    } else if (v[i] == "--no-gamma") gamma = false;
    else if (v[i] == "--uv" && i + 1 < v.size()) uv = std::stoi(v[++i]);
    else if (v[i] == "--size" && i + 1 < v.size()) size = std::stoi(v[++i]);
    else if (v[i] == "--bench" && i + 1 < v.size()) bench = std::stoi(v[++i]);
  }
  if (!bench && (!sockets.count("DATA") || !sockets.count("CTRL"))) {
    std::fprintf(stderr, "supershapesim: needs -btsockets DATA=... CTRL=...\n");
    return 2;
  }
  std::signal(SIGTERM, on_signal);
  std::signal(SIGINT, on_signal);
  sim::Camera cam;
  cam.width = cam.height = size;
  cam.lens_mm = 150.0;
  cam.loc = {10.0, -10.0, 6.0};
  {
    // look at the origin (-Z forward, +Y up)
    const double dx = -cam.loc.x, dy = -cam.loc.y, dz = -cam.loc.z;
    const double n = std::sqrt(dx * dx + dy * dy + dz * dz);
    const double pitch = std::acos(-dz / n), yaw = std::atan2(-dx / n, dy / n);
    cam.rot = sim::euler_xyz(pitch, 0.0, yaw);
  }
  sim::MeshStyle style;
  if (bench > 0) {
    std::vector<float> verts;
    std::vector<int> tris;
    std::vector<uint8_t> img(size_t(size) * size * 3);
    uint64_t h = 1469598103934665603ull;
    uint32_t rs = 12345;
    auto rnd = [&] { rs = rs * 1664525u + 1013904223u; return float(rs >> 8) / float(1u << 24); };
    double mesh_ms = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < bench; ++k) {
      float p[12] = {1 + 9 * rnd(), 1, 1, 1 + 4 * rnd(), 1 + 4 * rnd(), 1 + 4 * rnd(),
                     1 + 9 * rnd(), 1, 1, 1 + 4 * rnd(), 1 + 4 * rnd(), 1 + 4 * rnd()};
      const auto m0 = std::chrono::steady_clock::now();
      supershape_mesh(p, uv, verts, tris);
      mesh_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - m0).count();
      sim::render_mesh(cam, verts, tris, style, img.data(), 3, false);
      for (uint8_t b : img) h = (h ^ b) * 1099511628211ull;
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    std::printf("supershapesim bench: %d shapes, %.3f ms/shape (mesh %.3f), checksum %016llx\n", bench,
                ms / bench, mesh_ms / bench, (unsigned long long)h);
    return 0;
  }

  auto pub = zmtp::Context::global().socket(zmtp::PUSH);
  pub->setsockopt(zmtp::SNDHWM, 10);
  pub->setsockopt(zmtp::LINGER, 0);
  pub->setsockopt(zmtp::IMMEDIATE, 1);
  pub->bind(sockets["DATA"]);
  auto ctrl = zmtp::Context::global().socket(zmtp::PAIR);
  ctrl->setsockopt(zmtp::LINGER, 0);
  ctrl->setsockopt(zmtp::RCVHWM, 10);
  ctrl->setsockopt(zmtp::SNDHWM, 10);
  ctrl->bind(sockets["CTRL"]);
  const zmtp::Socket::Interrupt intr = [] { return g_stop.load(); };

  std::vector<uint8_t> glut(256);
  for (int i = 0; i < 256; ++i)
    glut[i] = gamma ? uint8_t(255.0f * std::pow(float(i) / 255.0f, float(1.0 / 2.2))) : uint8_t(i);

  struct Work {
    std::vector<float> params;   // n * 12
    std::vector<int64_t> ids;
    size_t next = 0;
  };
  std::deque<Work> pending;      // a new message replaces the current work
  std::vector<float> verts;
  std::vector<int> tris;
  codec::Bytes storage;

  while (!g_stop) {
    // pre_frame: duplex.recv(timeoutms=0)
    bool got = false;
    for (;;) {
      zmtp::Message m;
      try {
        m = ctrl->recv(zmtp::DONTWAIT);
      } catch (const zmtp::Error&) {
        break;
      }
      std::vector<uint8_t> bytes(m[0].data(), m[0].data() + m[0].size);
      codec::VPtr root;
      try {
        root = codec::parse(bytes.data(), bytes.size());
      } catch (const std::exception&) {
        continue;
      }
      const codec::Value* sp = root->get("shape_params");
      const codec::Value* si = root->get("shape_ids");
      if (!sp || !si || sp->kind != codec::Value::NDARRAY || si->kind != codec::Value::NDARRAY) continue;
      Work w;
      const int64_t n = sp->numel() / 12;
      w.params.resize(size_t(n) * 12);
      if (sp->dtype == "<f4") {
        std::memcpy(w.params.data(), bytes.data() + sp->off, size_t(n) * 12 * 4);
      } else if (sp->dtype == "<f8") {
        for (int64_t k = 0; k < n * 12; ++k) {
          double d;
          std::memcpy(&d, bytes.data() + sp->off + 8 * k, 8);
          w.params[size_t(k)] = float(d);
        }
      } else {
        continue;
      }
      w.ids.resize(size_t(si->numel()));
      for (int64_t k = 0; k < si->numel(); ++k) {
        if (si->dtype == "<i8") std::memcpy(&w.ids[size_t(k)], bytes.data() + si->off + 8 * k, 8);
        else {
          int32_t x;
          std::memcpy(&x, bytes.data() + si->off + 4 * k, 4);
          w.ids[size_t(k)] = x;
        }
      }
      pending.clear();
      pending.push_back(std::move(w));
      got = true;
    }
    if (pending.empty() || pending.front().next >= pending.front().ids.size()) {
      pending.clear();
      // idle: block until the next parameters arrive (a 500 us sleep between
      // polls added 0-0.5 ms to the start of every densityopt iteration).
      // The reference's Blender keeps animating and polls once per frame
      // (supershape.blend.py:26-36); a headless producer has no frame to draw
      if (!got) {
        try {
          (void)zmtp::Socket::poll({{ctrl.get(), zmtp::POLLIN}}, 100, intr);
        } catch (const zmtp::Error&) {
          break;   // interrupted: g_stop
        }
      }
      continue;
    }
    Work& w = pending.front();
    const size_t k = w.next++;
    supershape_mesh(&w.params[k * 12], uv, verts, tris);

    // post_frame: render + publish
    codec::Writer wr(4, std::move(storage));
    wr.begin_dict();
    wr.key("btid");
    wr.integer(btid);
    wr.key("image");
    const size_t off = wr.ndarray("u1", {size, size, 3}, nullptr, 64);
    wr.key("shape_id");
    wr.integer(w.ids[k]);
    wr.end_dict();
    auto& buf = wr.finish();
    sim::render_mesh(cam, verts, tris, style, buf.data() + off, 3, false);
    for (size_t i = 0; i < size_t(size) * size * 3; ++i) buf[off + i] = glut[buf[off + i]];
    zmtp::Message msg;
    msg.push_back(zmtp::Frame::copy_of(buf.data(), buf.size()));
    storage = std::move(buf);
    try {
      pub->send(std::move(msg), 0, intr);
    } catch (const zmtp::Error&) {
      break;
    }
  }
  pub->close(0);
  ctrl->close(0);
  return 0;
}
