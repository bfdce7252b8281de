// cubesim -- headless stand-in for a Blender instance running
// examples/datagen/cube.blend.py (or falling_cubes.blend.py).
//
// Launch contract is the one BlenderLauncher hands to Blender scripts
// (reference: pkg_pytorch/blendtorch/btt/launcher.py:114-122, parsed by
// pkg_blender/blendtorch/btb/arguments.py:5-47):
//
//   cubesim [--] -btid I -btseed S -btsockets DATA=tcp://host:port [script args]
//
// Script args:  --scene cube|falling_cubes   --mode rgb|rgba   --origin
// upper-left|lower-left   --frame-range A B   --frames N (-1 = forever)
// --sndhwm N   --linger MS   --fps F (0 = unthrottled)   --socket NAME
// --fault none|exit|stall|garbage --fault-after N   --rotation RX RY RZ   --verbose
// --resolution WxH   --stamp (integrity tests: btid/seq in the first 16 image bytes)
// --lease-ms N       shm ring lease (default 30000): unclaimed slots reclaimed after starving N ms
// --shm N (render into an N-slot shared-memory ring, send descriptors only)
// --codec tile16 (shm frames as key-frame deltas, csrc/codec/tiledelta.h)
// --bench N (no sockets: render N frames into 8 rotating buffers, full vs
// incremental (DirtyRect) rendering, and report the byte mismatches -- 0)
//
// Every frame it publishes, on a bound PUSH socket with SNDHWM/LINGER/
// IMMEDIATE as btb.DataPublisher does (reference: btb/publisher.py:21-43),
// the pickled dict {'btid', 'image' (HxWxC u8), 'xy' (8*nboxes x 2 f8),
// 'frameid'} -- the same keys cube.blend.py publishes (reference:
// examples/datagen/cube.blend.py:17-24).  Pixels are rendered straight into
// the pickle payload, so a frame costs one render and zero extra copies
// before the kernel socket buffer.
#include <atomic>
#include <chrono>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <unistd.h>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../codec/pickle_codec.h"
#include "../codec/tiledelta.h"
#include "../transport/shmring.h"
#include "../transport/zmtp.h"
#include "physics.h"
#include "raster.h"

using namespace btn;

namespace {

std::atomic<bool> g_stop{false};
void on_signal(int) { g_stop = true; }

struct Args {
  int btid = 0;
  long long btseed = 0;
  std::map<std::string, std::string> sockets;
  std::string scene = "cube";
  std::string mode = "rgb";
  std::string origin = "upper-left";
  std::string socket = "DATA";
  int frame_start = 0, frame_end = 100;
  long long frames = -1;
  int sndhwm = 10;
  long linger = 0;
  double fps = 0;
  std::string fault = "none";
  long long fault_after = -1;
  bool verbose = false;
  int shm_slots = 0;        // >0: images go through a shared-memory ring
  std::string codec = "none";   // shm frames: none (raw HWC) | tile16 (key-frame delta, tiledelta.h)
  bool fixed_rotation = false;
  double rot[3] = {0, 0, 0};
  int width = 0, height = 0;   // 0: the scene's resolution (640x480)
  bool stamp = false;          // integrity tests: (btid, seq) written into the first image row
  long lease_ms = 30000;       // shm ring: reclaim unclaimed slots after starving this long (shmring.h)
  long long bench = 0;         // >0: offline render benchmark / incremental-render check
};

[[noreturn]] void usage(const char* msg) {
  std::fprintf(stderr, "cubesim: %s\n", msg);
  std::exit(2);
}

Args parse(int argc, char** argv) {
  Args a;
  // BlenderLauncher(shm_slots=N) exports BLENDTORCH_SHM_SLOTS; --shm overrides
  if (const char* e = std::getenv("BLENDTORCH_SHM_SLOTS")) a.shm_slots = std::atoi(e);
  if (const char* e = std::getenv("BLENDTORCH_SHM_CODEC")) a.codec = e;   // BlenderLauncher(shm_codec=...)
  if (const char* e = std::getenv("BLENDTORCH_SHM_CODEC")) a.codec = e;
  std::vector<std::string> v;
  int start = 1;
  for (int i = 1; i < argc; ++i)
    if (std::strcmp(argv[i], "--") == 0) {
      start = i + 1;
      break;
    }
  for (int i = start; i < argc; ++i) v.push_back(argv[i]);
  auto need = [&](size_t i) {
    if (i + 1 >= v.size()) usage(("missing value for " + v[i]).c_str());
    return v[i + 1];
  };
  for (size_t i = 0; i < v.size(); ++i) {
    const std::string& k = v[i];
    if (k == "-btid") a.btid = std::stoi(need(i)), ++i;
    else if (k == "-btseed") a.btseed = std::stoll(need(i)), ++i;
    else if (k == "-btsockets") {
      while (i + 1 < v.size() && v[i + 1].rfind("-", 0) != 0) {
        ++i;
        auto eq = v[i].find('=');
        if (eq == std::string::npos) usage("-btsockets expects NAME=ADDRESS");
        a.sockets[v[i].substr(0, eq)] = v[i].substr(eq + 1);
      }
    } else if (k == "--scene") a.scene = need(i), ++i;
    else if (k == "--mode") a.mode = need(i), ++i;
    else if (k == "--origin") a.origin = need(i), ++i;
    else if (k == "--socket") a.socket = need(i), ++i;
    else if (k == "--frame-range") {
      a.frame_start = std::stoi(need(i));
      a.frame_end = std::stoi(need(i + 1));
      i += 2;
    } else if (k == "--frames") a.frames = std::stoll(need(i)), ++i;
    else if (k == "--sndhwm") a.sndhwm = std::stoi(need(i)), ++i;
    else if (k == "--linger") a.linger = std::stol(need(i)), ++i;
    else if (k == "--fps") a.fps = std::stod(need(i)), ++i;
    else if (k == "--fault") a.fault = need(i), ++i;
    else if (k == "--fault-after") a.fault_after = std::stoll(need(i)), ++i;
    else if (k == "--verbose") a.verbose = true;
    else if (k == "--stamp") a.stamp = true;
    else if (k == "--lease-ms") a.lease_ms = std::stol(need(i)), ++i;
    else if (k == "--shm") a.shm_slots = std::stoi(need(i)), ++i;
    else if (k == "--codec") a.codec = need(i), ++i;
    else if (k == "--bench") a.bench = std::stoll(need(i)), ++i;
    else if (k == "--resolution") {
      // WxH: render size (render.resolution_x/_y); the camera's field of view is kept
      const std::string r = need(i);
      const auto x = r.find('x');
      if (x == std::string::npos) usage("--resolution expects WxH");
      a.width = std::stoi(r.substr(0, x));
      a.height = std::stoi(r.substr(x + 1));
      if (a.width < 1 || a.height < 1) usage("bad --resolution");
      ++i;
    }
    else if (k == "--rotation") {
      if (i + 3 >= v.size()) usage("--rotation needs rx ry rz");
      for (int r = 0; r < 3; ++r) a.rot[r] = std::stod(v[i + 1 + r]);
      a.fixed_rotation = true;
      i += 3;
    }
    // unknown args are ignored, as Blender scripts ignore the remainder
  }
  if (a.mode != "rgb" && a.mode != "rgba") usage("--mode must be rgb or rgba");
  if (a.codec != "none" && a.codec != btn::tiledelta::kName) usage("--codec must be none or tile16");
  if (a.origin != "upper-left" && a.origin != "lower-left") usage("bad --origin");
  return a;
}

// Recycles frame storage: a sent frame's buffer returns here once the IO
// thread has written it, so steady state allocates nothing.
struct FramePool {
  std::mutex mu;
  std::vector<codec::Bytes*> free;
  codec::Bytes take() {
    std::lock_guard<std::mutex> lk(mu);
    if (free.empty()) return {};
    codec::Bytes v(std::move(*free.back()));
    delete free.back();
    free.pop_back();
    return v;
  }
  void give(codec::Bytes* v) {
    std::lock_guard<std::mutex> lk(mu);
    if (free.size() < 64) free.push_back(v);
    else delete v;
  }
};
FramePool g_pool;

zmtp::Frame frame_from_vector(codec::Bytes&& v) {
  auto* owned = new codec::Bytes(std::move(v));
  auto b = std::make_shared<Buffer>();
  b->data = owned->data();
  b->capacity = owned->size();
  b->owner = owned;
  b->release = [](void* o, Buffer*) { g_pool.give(static_cast<codec::Bytes*>(o)); };
  zmtp::Frame f;
  f.size = owned->size();
  f.buf = std::move(b);
  return f;
}

// --bench N: the render loop without sockets.  Every frame is rendered twice,
// once in full into a scratch buffer and once incrementally into the next of
// 8 rotating buffers (a ring slot's life; the full renders rotate over 8
// buffers of their own); both timings and the number of
// differing bytes (must be 0) are printed.
template <class Pose>
int bench(const Args& a, sim::Scene& scene, sim::Renderer& r, Pose& pose) {
  const size_t n = size_t(r.width()) * r.height() * r.channels();
  constexpr int kSlots = 8;
  std::vector<std::vector<uint8_t>> slots(kSlots, std::vector<uint8_t>(n));
  std::vector<sim::DirtyRect> dirty(kSlots);
  std::vector<std::vector<uint8_t>> fulls(kSlots, std::vector<uint8_t>(n));   // as cold as the slots
  double t_full = 0, t_inc = 0;
  long long mismatches = 0;
  uint64_t h = 1469598103934665603ull;   // FNV-1a over every incremental frame
  int frame = a.frame_start;
  for (long long i = 0; i < a.bench; ++i) {
    pose(frame);
    frame = frame >= a.frame_end ? a.frame_start : frame + 1;
    const uint8_t* full = fulls[size_t(i % kSlots)].data();
    auto t0 = std::chrono::steady_clock::now();
    r.render(scene, fulls[size_t(i % kSlots)].data());
    auto t1 = std::chrono::steady_clock::now();
    uint8_t* out = slots[size_t(i % kSlots)].data();
    r.render(scene, out, &dirty[size_t(i % kSlots)]);
    auto t2 = std::chrono::steady_clock::now();
    t_full += std::chrono::duration<double, std::milli>(t1 - t0).count();
    t_inc += std::chrono::duration<double, std::milli>(t2 - t1).count();
    for (size_t k = 0; k < n; ++k) {
      mismatches += out[k] != full[k];
      h = (h ^ out[k]) * 1099511628211ull;
    }
  }
  std::printf("{\"frames\": %lld, \"full_ms\": %.4f, \"incremental_ms\": %.4f, \"mismatched_bytes\": %lld, "
              "\"checksum\": \"%016llx\"}\n",
              a.bench, t_full / a.bench, t_inc / a.bench, mismatches, (unsigned long long)h);
  return mismatches == 0 ? 0 : 1;
}

}  // namespace

int main(int argc, char** argv) {
  Args a = parse(argc, argv);
  if (a.bench <= 0 && !a.sockets.count(a.socket)) usage(("no -btsockets entry named " + a.socket).c_str());
  std::signal(SIGTERM, on_signal);
  std::signal(SIGINT, on_signal);

  sim::Scene scene = a.scene == "falling_cubes" ? sim::falling_cubes_scene() : sim::cube_scene();
  if (a.width > 0) scene.cam.width = a.width, scene.cam.height = a.height;
  const int W = scene.cam.width, H = scene.cam.height, C = a.mode == "rgba" ? 4 : 3;
  std::mt19937_64 rng(uint64_t(a.btseed));
  std::uniform_real_distribution<double> U(0.0, 1.0);
  const double pi = 3.14159265358979323846;
  if (a.scene == "falling_cubes") {
    for (auto& b : scene.boxes)
      b.albedo = {float(U(rng)), float(U(rng)), float(U(rng))};
  }

  sim::RigidWorld physics(scene.plane_z);
  // pre_animation / pre_frame: randomise the pose(s)
  auto pose = [&](int frame) {
    if (a.scene == "falling_cubes") {
      // pre_animation: re-drop every cube at a random pose, as
      // falling_cubes.blend.py does (xyz ~ U((-3,-3,6),(3,3,12)), euler ~ U(-pi,pi));
      // every later frame advances the rigid-body world by one scene frame
      if (frame == a.frame_start) {
        for (auto& b : scene.boxes) {
          b.center = {-3 + 6 * U(rng), -3 + 6 * U(rng), 6 + 6 * U(rng)};
          b.rot = sim::euler_xyz(-pi + 2 * pi * U(rng), -pi + 2 * pi * U(rng), -pi + 2 * pi * U(rng));
        }
        physics.reset(scene.boxes);
      } else {
        physics.step(scene.boxes, 1.0 / 60.0);
      }
    } else if (a.fixed_rotation) {
      scene.boxes[0].rot = sim::euler_xyz(a.rot[0], a.rot[1], a.rot[2]);
    } else {
      scene.boxes[0].rot = sim::euler_xyz(pi * U(rng), pi * U(rng), pi * U(rng));
    }
  };
  const bool lower_left = a.origin == "lower-left";
  sim::Renderer renderer(scene, C, lower_left);
  if (a.bench > 0) return bench(a, scene, renderer, pose);

  auto sock = zmtp::Context::global().socket(zmtp::PUSH);
  sock->setsockopt(zmtp::SNDHWM, a.sndhwm);
  sock->setsockopt(zmtp::LINGER, a.linger);
  sock->setsockopt(zmtp::IMMEDIATE, 1);
  sock->bind(a.sockets[a.socket]);

  const zmtp::Socket::Interrupt intr = [] { return g_stop.load(); };
  std::unique_ptr<shm::Segment> seg, key_seg;
  // key-frame delta codec: the background goes once into a segment of its
  // own, every frame into its slot as a tile map + the tiles that differ
  bool tiled = a.shm_slots > 0 && a.codec == tiledelta::kName && tiledelta::supported(H, W, C);
  if (a.shm_slots > 0) {
    const std::string name = "blendtorch-" + std::to_string(::getpid()) + "-" + std::to_string(a.btid);
    try {
      const size_t raw = size_t(W) * H * C;
      seg.reset(shm::Segment::create(name, uint32_t(a.shm_slots), tiled ? std::max(raw, tiledelta::max_bytes(H, W, C)) : raw));
      if (tiled) {
        key_seg.reset(shm::Segment::create(name + "-key", 1, raw));
        const int k = key_seg->acquire(0);
        std::memcpy(key_seg->slot(uint32_t(k)), renderer.background().data(), raw);
        key_seg->publish(uint32_t(k));   // stays published: consumers only read it
      }
    } catch (const std::exception& e) {
      // e.g. a small /dev/shm: fall back to inline payloads
      std::fprintf(stderr, "cubesim[%d]: shared memory disabled (%s)\n", a.btid, e.what());
      seg.reset(), key_seg.reset(), tiled = false;
    }
  }
  std::vector<uint8_t> tiled_frame(tiled ? size_t(W) * H * C : 0);   // the full frame, rendered incrementally
  sim::DirtyRect tiled_dirty;
  // what each ring slot's last frame drew over the background: a slot is
  // re-rendered by restoring that rectangle only (BLENDTORCH_FULL_RENDER=1: off)
  const char* full_env = std::getenv("BLENDTORCH_FULL_RENDER");
  const bool incremental = !(full_env && std::atoi(full_env) != 0);
  std::vector<sim::DirtyRect> slot_dirty(seg ? size_t(a.shm_slots) : 0);
  const auto t_start = std::chrono::steady_clock::now();
  auto next_due = t_start;
  long long published = 0;
  int frame = a.frame_start;
  double render_ms = 0;

  while (!g_stop && (a.frames < 0 || published < a.frames)) {
    pose(frame);

    int slot = -1;
    if (seg) {
      slot = seg->acquire(-1, &g_stop, a.lease_ms);   // blocks while every slot is with a consumer
      if (slot < 0) break;
    }
    uint32_t gen = 0;
    codec::Writer w(4, g_pool.take());
    w.begin_dict();
    w.key("btid");
    w.integer(a.btid);
    size_t img_off = 0;
    if (!seg) {
      w.key("image");
      img_off = w.ndarray("u1", {H, W, C}, nullptr, 64);   // 64-byte aligned payload: zero-copy GPU reads
    }
    w.key("xy");
    std::vector<double> xy;
    for (auto& b : scene.boxes)
      for (auto& c : b.corners()) {
        double px = 0, py = 0;
        scene.cam.project(c, &px, &py);
        xy.push_back(px);
        xy.push_back(py);
      }
    w.ndarray("f8", {int64_t(xy.size() / 2), 2}, xy.data());
    w.key("frameid");
    w.integer(frame);
    if (a.stamp) {
      w.key("seq");
      w.integer(published);
    }
    if (lower_left) {
      w.key("origin");
      w.str("lower-left");
    }
    if (seg) {
      // descriptor: (segment, slot, byte offset, H, W, C, image key, generation)
      gen = ((seg->state(uint32_t(slot)) >> 2) + 1) & 0x3fffffffu;   // publish() will bump to this
      w.key("_btshm");
      w.begin_tuple();
      w.str(seg->name());
      w.integer(slot);
      w.integer(int64_t(seg->slot_offset(uint32_t(slot))));
      w.integer(H);
      w.integer(W);
      w.integer(C);
      w.str("image");
      w.integer(gen);
      if (tiled) {   // 9th element: (codec, key segment, key generation)
        w.begin_tuple();
        w.str(tiledelta::kName);
        w.str(key_seg->name());
        w.integer(int64_t(key_seg->state(0) >> 2));
        w.end_tuple();
      }
      w.end_tuple();
    }
    w.end_dict();
    auto& buf = w.finish();
    uint8_t* pixels = seg ? seg->slot(uint32_t(slot)) : buf.data() + img_off;

    auto r0 = std::chrono::steady_clock::now();
    sim::DirtyRect* dirty = tiled ? &tiled_dirty : (seg && incremental ? &slot_dirty[size_t(slot)] : nullptr);
    uint8_t* const slot_bytes = pixels;
    if (tiled) pixels = tiled_frame.data();
    renderer.render(scene, pixels, dirty);
    if (a.stamp) {
      // bytes 0..15 of the stored image (first stored row): 'B','T', btid (u16 LE),
      // 4 zero bytes, seq (u64 LE) -- lets tests match every decoded image to its metadata
      uint8_t st[16] = {'B', 'T', uint8_t(a.btid & 0xff), uint8_t((a.btid >> 8) & 0xff), 0, 0, 0, 0};
      const uint64_t q = uint64_t(published);
      std::memcpy(st + 8, &q, 8);
      std::memcpy(pixels, st, sizeof(st));
      if (dirty) dirty->add(lower_left ? H - 1 : 0, 0, (int(sizeof(st)) + C - 1) / C - 1);
    }
    if (tiled) {
      // everything outside this frame's dirty rectangle is background
      if (tiled_dirty.empty())
        tiledelta::encode(pixels, key_seg->slot(0), H, W, C, 0, -1, 0, -1, slot_bytes);
      else if (lower_left)   // DirtyRect rows are image rows (0 = top); stored rows are flipped
        tiledelta::encode(pixels, key_seg->slot(0), H, W, C, H - 1 - tiled_dirty.y1, H - 1 - tiled_dirty.y0,
                          tiled_dirty.x0, tiled_dirty.x1, slot_bytes);
      else
        tiledelta::encode(pixels, key_seg->slot(0), H, W, C, tiled_dirty.y0, tiled_dirty.y1, tiled_dirty.x0,
                          tiled_dirty.x1, slot_bytes);
    }
    if (seg) seg->publish(uint32_t(slot));   // == gen
    render_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - r0).count();

    if (a.fault != "none" && a.fault_after >= 0 && published == a.fault_after) {
      if (a.fault == "exit") std::_Exit(3);
      if (a.fault == "stall") {
        while (!g_stop) std::this_thread::sleep_for(std::chrono::milliseconds(50));
        break;
      }
      if (a.fault == "garbage") {
        zmtp::Message m;
        m.push_back(zmtp::Frame::copy_of("\x80\x04garbage", 9));
        try {
          sock->send(std::move(m), 0, intr);
        } catch (const zmtp::Error&) {
          break;
        }
        if (seg) seg->release(uint32_t(slot), seg->publish(uint32_t(slot)));
        ++published;
        continue;
      }
    }

    zmtp::Message msg;
    msg.push_back(frame_from_vector(std::move(buf)));
    try {
      sock->send(std::move(msg), 0, intr);   // blocks at SNDHWM: backpressure
    } catch (const zmtp::Error& e) {
      if (e.code == zmtp::E_INTR) break;
      std::fprintf(stderr, "cubesim[%d]: send failed: %s\n", a.btid, e.what());
      break;
    }
    ++published;
    frame = frame >= a.frame_end ? a.frame_start : frame + 1;
    if (a.fps > 0) {
      next_due += std::chrono::microseconds(int64_t(1e6 / a.fps));
      std::this_thread::sleep_until(next_due);
    }
  }
  double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
  if (a.verbose)
    std::fprintf(stderr, "cubesim[%d]: %lld frames in %.2fs (%.1f fps, render %.3f ms/frame)\n", a.btid,
                 published, secs, published / std::max(secs, 1e-9), render_ms / std::max<long long>(published, 1));
  sock->close(g_stop ? 0 : -2);
  return 0;
}
