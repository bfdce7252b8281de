// cartpolesim -- headless stand-in for a Blender instance running
// examples/control/cartpole_gym/envs/cartpole.blend.py.
//
// It serves the remote-env protocol natively, exactly as the Blender-side
// btb.env.BaseEnv + btb.env.RemoteControlledAgent pair does (reference:
// pkg_blender/blendtorch/btb/env.py:10-252):
//
//   * REP socket bound to the GYM address (LINGER 0, SNDTIMEO/RCVTIMEO);
//   * frame loop over (1, 2147483647): frame 1 of an episode = reset,
//     every later frame first asks the agent (reply to the previous request
//     = ctx after the previous frame, then read the next request);
//   * 'reset' while the episode is still at its first frame is answered
//     immediately (the reference's recursion), otherwise it restarts;
//   * real-time mode: once running, a missing request means "keep
//     simulating without an action" (non-blocking receive);
//   * ctx dict keys/order: prev_action, done, time, [rgb_array], obs, reward.
//
// Physics replaces Blender's Bullet rigid bodies: a cart on a rail driven by
// a velocity motor (the action increments the motor target velocity by
// f / m_total / fps, cartpole.blend.py:38-43) and a uniform pole hinged on
// the cart, integrated with 10 sub-steps per frame (Blender's default rigid
// body substeps).  Observation (cart_x, pole_center_x, pole_angle), reward 0,
// done when |angle| > 0.6 or |cart_x| > 4 (cartpole.blend.py:25-36).
//
//   cartpolesim [--] -btid I -btseed S -btsockets GYM=tcp://... [--render-every N]
//               [--real-time | --no-real-time] [--fps F] [--timeoutms MS]
#include <atomic>
#include <chrono>
#include <cmath>
#include <csignal>
#include <cstdio>
#include <cstring>
#include <map>
#include <random>
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

struct Args {
  int btid = 0;
  long long btseed = 0;
  std::map<std::string, std::string> sockets;
  int render_every = 0;
  bool real_time = false;
  double fps = 0;          // 0: as fast as the agent allows
  long timeoutms = 5000;
  int sim_fps = 60;        // scene fps used by the physics / action scaling
};

Args parse(int argc, char** argv) {
  Args a;
  std::vector<std::string> v;
  int start = 1;
  for (int i = 1; i < argc; ++i)
    if (std::strcmp(argv[i], "--") == 0) {
      start = i + 1;
      break;
    }
  for (int i = start; i < argc; ++i) v.push_back(argv[i]);
  for (size_t i = 0; i < v.size(); ++i) {
    const std::string& k = v[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= v.size()) {
        std::fprintf(stderr, "cartpolesim: missing value for %s\n", k.c_str());
        std::exit(2);
      }
      return v[++i];
    };
    if (k == "-btid") a.btid = std::stoi(val());
    else if (k == "-btseed") a.btseed = std::stoll(val());
    else if (k == "-btsockets") {
      while (i + 1 < v.size() && v[i + 1].rfind("-", 0) != 0) {
        ++i;
        auto eq = v[i].find('=');
        if (eq != std::string::npos) a.sockets[v[i].substr(0, eq)] = v[i].substr(eq + 1);
      }
    } else if (k == "--render-every") a.render_every = std::stoi(val());
    else if (k == "--real-time") a.real_time = true;
    else if (k == "--no-real-time") a.real_time = false;
    else if (k == "--fps") a.fps = std::stod(val());
    else if (k == "--timeoutms") a.timeoutms = std::stol(val());
    else if (k == "--sim-fps") a.sim_fps = std::stoi(val());
  }
  return a;
}

// ---------------------------------------------------------------------------
// physics
// ---------------------------------------------------------------------------
struct Cartpole {
  // geometry / masses (cartpole.blend: cart at z=1.2, pole centre at z=2.4)
  double m_cart = 1.0, m_pole = 0.1;
  double L = 2.0;            // pole length, hinge at its lower end
  double hinge_z = 1.4;
  double g = 9.81;
  double motor_gain = 60.0;  // 1/s: how fast the motor reaches its target velocity
  // state
  double x = 0, v = 0, v_target = 0, th = 0, w = 0;

  double total_mass() const { return m_cart + m_pole; }
  void reset(double angle) {
    x = 0, v = 0, v_target = 0, th = angle, w = 0;
  }
  void apply_action(double f, int fps) { v_target += f / total_mass() / fps; }
  void step(double dt_frame, int substeps = 10) {
    const double dt = dt_frame / substeps;
    for (int s = 0; s < substeps; ++s) {
      const double a = motor_gain * (v_target - v);                 // cart acceleration
      const double alpha = 1.5 / L * (g * std::sin(th) - a * std::cos(th));
      v += a * dt;
      x += v * dt;
      w += alpha * dt;
      th += w * dt;
    }
  }
  double pole_center_x() const { return x + 0.5 * L * std::sin(th); }
};

// ---------------------------------------------------------------------------
// rendering (attach_default_renderer: rgb, gamma 2.2)
// ---------------------------------------------------------------------------
struct View {
  sim::Scene scene;
  std::vector<uint8_t> gamma;   // reference gamma table: u8(255*(x/255)^(1/2.2)), float32 math
  View() {
    scene.cam.width = 480;
    scene.cam.height = 270;
    scene.cam.loc = {0.0, -14.0, 2.2};
    scene.cam.rot = sim::euler_xyz(1.5707963, 0.0, 0.0);   // look along +Y
    scene.light.loc = {2.0, -6.0, 8.0};
    scene.light.power = 2500.0;
    scene.plane_z = 0.0;
    scene.plane_half = 12.0;
    sim::Box base;   // rail
    base.center = {0, 0, 0.5};
    base.half = {5.0, 0.2, 0.5};
    base.rot = sim::euler_xyz(0, 0, 0);
    base.albedo = {0.3f, 0.3f, 0.35f};
    sim::Box cart;
    cart.half = {0.5, 0.4, 0.2};
    cart.rot = sim::euler_xyz(0, 0, 0);
    cart.albedo = {0.8f, 0.2f, 0.1f};
    sim::Box pole;
    pole.half = {0.05, 0.05, 1.0};
    pole.albedo = {0.9f, 0.8f, 0.2f};
    scene.boxes = {base, cart, pole};
    gamma.resize(256);
    for (int i = 0; i < 256; ++i) {
      float x = float(i) / 255.0f;
      gamma[i] = uint8_t(255.0f * std::pow(x, float(1.0 / 2.2)));
    }
  }
  void place(const Cartpole& cp) {
    scene.boxes[1].center = {cp.x, 0.0, 1.2};
    scene.boxes[2].center = {cp.x + 0.5 * cp.L * std::sin(cp.th), 0.0, cp.hinge_z + 0.5 * cp.L * std::cos(cp.th)};
    scene.boxes[2].rot = sim::euler_xyz(0.0, cp.th, 0.0);
  }
  void render(std::vector<uint8_t>& out) {
    out.resize(size_t(scene.cam.width) * scene.cam.height * 3);
    sim::render(scene, out.data(), 3, false);
    for (auto& b : out) b = gamma[b];
  }
};

// ---------------------------------------------------------------------------
// ctx (the dict the agent receives)
// ---------------------------------------------------------------------------
struct Ctx {
  bool has_prev_action = false;
  codec::VPtr prev_action;   // as received
  bool done = false;
  long long time = 0;
  bool has_obs = false;
  double obs[3] = {0, 0, 0};
  double reward = 0;
  bool has_rgb = false;
  std::vector<uint8_t> rgb;
  int rgb_h = 0, rgb_w = 0;
};

void write_value(codec::Writer& w, const codec::Value& v, const uint8_t* base) {
  switch (v.kind) {
    case codec::Value::NONE: w.none(); break;
    case codec::Value::BOOL: w.boolean(v.b); break;
    case codec::Value::INT: w.integer(v.i); break;
    case codec::Value::FLOAT: w.real(v.f); break;
    case codec::Value::STR: w.str(v.s); break;
    case codec::Value::LIST:
      w.begin_list();
      for (auto& x : v.items) write_value(w, *x, base);
      w.end_list();
      break;
    case codec::Value::TUPLE:
      w.begin_tuple();
      for (auto& x : v.items) write_value(w, *x, base);
      w.end_tuple();
      break;
    default: w.none(); break;   // arrays etc. are echoed as their float value below
  }
}

codec::Bytes encode(const Ctx& c, double prev_action_value) {
  codec::Writer w(4);
  w.begin_dict();
  w.key("prev_action");
  if (!c.has_prev_action) w.none();
  else if (c.prev_action->kind == codec::Value::FLOAT || c.prev_action->kind == codec::Value::INT ||
           c.prev_action->kind == codec::Value::NONE || c.prev_action->kind == codec::Value::LIST ||
           c.prev_action->kind == codec::Value::TUPLE)
    write_value(w, *c.prev_action, nullptr);
  else w.real(prev_action_value);
  w.key("done");
  w.boolean(c.done);
  w.key("time");
  w.integer(c.time);
  if (c.has_rgb) {
    w.key("rgb_array");
    w.ndarray("u1", {c.rgb_h, c.rgb_w, 3}, c.rgb.data(), 64);
  }
  if (c.has_obs) {
    w.key("obs");
    w.begin_tuple();
    for (double o : c.obs) w.real(o);
    w.end_tuple();
    w.key("reward");
    w.real(c.reward);
  }
  w.end_dict();
  return std::move(w.finish());
}

// numeric value of an action (float, int, bool, numpy scalar, 1-element array/list)
bool action_value(const codec::Value& v, const uint8_t* base, double* out) {
  switch (v.kind) {
    case codec::Value::FLOAT: *out = v.f; return true;
    case codec::Value::INT: *out = double(v.i); return true;
    case codec::Value::BOOL: *out = v.b ? 1.0 : 0.0; return true;
    case codec::Value::NONE: return false;
    case codec::Value::LIST:
    case codec::Value::TUPLE:
      if (v.items.size() >= 1) return action_value(*v.items[0], base, out);
      return false;
    case codec::Value::NDARRAY: {
      if (v.numel() < 1) return false;
      const uint8_t* p = base + v.off;
      if (v.dtype == "<f4") {
        float f;
        std::memcpy(&f, p, 4);
        *out = f;
        return true;
      }
      if (v.dtype == "<f8") {
        std::memcpy(out, p, 8);
        return true;
      }
      if (v.dtype == "<i8") {
        int64_t i;
        std::memcpy(&i, p, 8);
        *out = double(i);
        return true;
      }
      if (v.dtype == "<i4") {
        int32_t i;
        std::memcpy(&i, p, 4);
        *out = double(i);
        return true;
      }
      return false;
    }
    default: return false;
  }
}

}  // namespace

int main(int argc, char** argv) {
  Args a = parse(argc, argv);
  if (!a.sockets.count("GYM")) {
    std::fprintf(stderr, "cartpolesim: needs -btsockets GYM=<address>\n");
    return 2;
  }
  std::signal(SIGTERM, on_signal);
  std::signal(SIGINT, on_signal);
  std::mt19937_64 rng(uint64_t(a.btseed));
  std::uniform_real_distribution<double> U(-0.6, 0.6);

  auto sock = zmtp::Context::global().socket(zmtp::REP);
  sock->setsockopt(zmtp::LINGER, 0);
  sock->setsockopt(zmtp::SNDTIMEO, a.timeoutms);
  sock->setsockopt(zmtp::RCVTIMEO, a.timeoutms);
  sock->bind(a.sockets["GYM"]);
  const zmtp::Socket::Interrupt intr = [] { return g_stop.load(); };

  Cartpole cp;
  View view;
  Ctx ctx;
  const long long start = 1, end = 2147483647;
  enum { INIT, RUN } env_state = INIT;
  enum { REQ, REP } agent_state = REQ;
  double prev_action_value = 0;
  codec::VPtr last_req;
  std::vector<uint8_t> last_req_bytes;
  const double dt = 1.0 / a.sim_fps;
  auto next_due = std::chrono::steady_clock::now();

  auto post_frame = [&](long long frame) {
    if (a.render_every > 0 && ((frame - start) % a.render_every) == 0) {
      view.place(cp);
      view.render(ctx.rgb);
      ctx.rgb_h = view.scene.cam.height;
      ctx.rgb_w = view.scene.cam.width;
      ctx.has_rgb = true;
    }
    const double angle = cp.th;
    ctx.has_obs = true;
    ctx.obs[0] = cp.x;
    ctx.obs[1] = cp.pole_center_x();
    ctx.obs[2] = angle;
    ctx.reward = 0.0;
    ctx.done = std::fabs(angle) > 0.6 || std::fabs(cp.x) > 4.0;
  };
  auto new_episode = [&]() {
    // pre_animation + pre_frame(start) + post_frame(start)
    env_state = INIT;
    ctx = Ctx();
    cp.reset(U(rng));
    ctx.time = start;
    ctx.done = ctx.done || start >= end;
    post_frame(start);
  };
  auto send_ctx = [&](int flags) -> bool {
    zmtp::Message m;
    auto bytes = encode(ctx, prev_action_value);
    m.push_back(zmtp::Frame::copy_of(bytes.data(), bytes.size()));
    try {
      sock->send(std::move(m), flags, intr);
      return true;
    } catch (const zmtp::Error& e) {
      if (e.code == zmtp::E_INTR) g_stop = true;
      return false;
    }
  };

  new_episode();
  long long frame = start;
  while (!g_stop) {
    ++frame;
    ctx.time = frame;
    ctx.done = ctx.done || frame >= end;
    // --- agent (RemoteControlledAgent.__call__) ---
    enum { STEP, RESTART } cmd = STEP;
    bool have_action = false;
    double action = 0;
    codec::VPtr action_tree;
    for (;;) {
      const int flags = (a.real_time && env_state == RUN) ? zmtp::DONTWAIT : 0;
      if (agent_state == REP) {
        if (!send_ctx(flags)) {
          if (g_stop) break;
          if (!a.real_time) {
            std::fprintf(stderr, "cartpolesim[%d]: failed to send to remote agent\n", a.btid);
            return 1;
          }
          break;   // CMD_STEP, None
        }
        agent_state = REQ;
      }
      zmtp::Message req;
      try {
        req = sock->recv(flags, intr);
      } catch (const zmtp::Error& e) {
        if (e.code == zmtp::E_INTR) g_stop = true;
        break;     // timeout / nothing pending: CMD_STEP, None
      }
      if (req.empty()) break;
      last_req_bytes.assign(req[0].data(), req[0].data() + req[0].size);
      codec::VPtr r;
      try {
        r = codec::parse(last_req_bytes.data(), last_req_bytes.size());
      } catch (const std::exception&) {
        r = nullptr;
      }
      const codec::Value* c = r ? r->get("cmd") : nullptr;
      if (!c || c->kind != codec::Value::STR || (c->s != "reset" && c->s != "step")) {
        std::fprintf(stderr, "cartpolesim[%d]: malformed request\n", a.btid);
        return 1;
      }
      agent_state = REP;
      if (c->s == "reset") {
        if (env_state == INIT) continue;   // answer right away, then read the next request
        cmd = RESTART;
        break;
      }
      const codec::Value* av = r->get("action");
      if (av && action_value(*av, last_req_bytes.data(), &action)) {
        have_action = true;
        action_tree = std::make_shared<codec::Value>(*av);
      }
      last_req = r;
      cmd = STEP;
      break;
    }
    if (g_stop) break;
    if (cmd == RESTART) {
      // rewind: the nested frame_set(start) restarts the episode; the
      // current frame is swallowed (its post_frame sees frame == start)
      frame = start;
      new_episode();
      continue;
    }
    if (have_action) {
      cp.apply_action(action, a.sim_fps);
      ctx.has_prev_action = true;
      ctx.prev_action = action_tree;
      prev_action_value = action;
    }
    env_state = RUN;
    // --- physics for this frame, then post_frame ---
    cp.step(dt);
    post_frame(frame);
    if (a.fps > 0) {
      next_due += std::chrono::microseconds(int64_t(1e6 / a.fps));
      std::this_thread::sleep_until(next_due);
    }
  }
  sock->close(0);
  return 0;
}
