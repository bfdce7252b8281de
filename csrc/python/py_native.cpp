// pybind11 bindings for the CPU-side native runtime: the ZMTP transport and
// the pickle codec.  Built as `blendtorch/_native*.so` (no HIP dependency, so
// it runs in Blender-side producer processes and CPU-only tests as well).
#include <atomic>
#include <pybind11/eval.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../codec/pickle_codec.h"
#include "../codec/xform_fit.h"
#include "../sim/physics.h"
#include "../sim/raster.h"
#include "../transport/zmtp.h"
#include "pyvalue.h"

namespace py = pybind11;
using namespace btn;
using zmtp::Frame;
using zmtp::Message;
using zmtp::Socket;
using pyconv::value_to_py;

namespace {

py::object g_error_type;

// Lets Ctrl-C interrupt a blocking native wait.
const Socket::Interrupt& signal_check() {
  static const Socket::Interrupt f = [] {
    py::gil_scoped_acquire gil;
    return PyErr_CheckSignals() != 0;
  };
  return f;
}

[[noreturn]] void raise_zmtp(const zmtp::Error& e) {
  // may be reached with the GIL released (blocking calls); error_already_set
  // captures the Python error state while we hold it here.
  py::gil_scoped_acquire gil;
  if (e.code == zmtp::E_INTR && PyErr_Occurred()) throw py::error_already_set();
  py::object err = g_error_type(e.code, e.what());
  PyErr_SetObject(g_error_type.ptr(), err.ptr());
  throw py::error_already_set();
}

template <typename F>
auto guarded(F&& f) -> decltype(f()) {
  try {
    return f();
  } catch (const zmtp::Error& e) {
    raise_zmtp(e);
  }
}

struct PyFrame {
  Frame f;
  bool more = false;
};

Frame frame_from_py(const py::handle& h) {
  if (py::isinstance<PyFrame>(h)) return h.cast<PyFrame&>().f;
  py::buffer b = py::reinterpret_borrow<py::buffer>(h);
  py::buffer_info info = b.request();
  size_t n = size_t(info.size * info.itemsize);
  return Frame::copy_of(info.ptr, n);
}

}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "blendtorch native runtime: ZMTP transport + pickle codec";

  // Exception type carrying errno; the Python layer maps it onto zmq.error.*
  py::object builtins = py::module_::import("builtins");
  g_error_type = py::reinterpret_borrow<py::object>(PyExc_Exception);
  {
    py::dict ns;
    py::exec(R"(
class NativeError(Exception):
    def __init__(self, errno, msg):
        super().__init__(msg)
        self.errno = errno
)", ns);
    g_error_type = ns["NativeError"];
    m.attr("NativeError") = g_error_type;
  }

  py::class_<PyFrame>(m, "Frame", py::buffer_protocol())
      .def_buffer([](PyFrame& f) {
        return py::buffer_info(const_cast<uint8_t*>(f.f.data()), 1,
                               py::format_descriptor<uint8_t>::format(), 1,
                               {py::ssize_t(f.f.size)}, {py::ssize_t(1)}, false);
      })
      .def("__len__", [](PyFrame& f) { return f.f.size; })
      .def_property_readonly("bytes", [](PyFrame& f) {
        return py::bytes(reinterpret_cast<const char*>(f.f.data()), f.f.size);
      })
      .def_property_readonly("more", [](PyFrame& f) { return f.more; })
      .def_property_readonly("pinned", [](PyFrame& f) { return f.f.buf && f.f.buf->pinned; });

  py::class_<zmtp::Context, std::shared_ptr<zmtp::Context>>(m, "Context")
      .def(py::init<>())
      .def("socket", [](zmtp::Context& c, int t) { return guarded([&] { return c.socket(t); }); })
      .def("term", [](zmtp::Context& c) {
        py::gil_scoped_release nogil;
        c.term();
      });

  m.def("global_context", []() {
    // never destroyed: the IO thread must outlive interpreter teardown
    static std::shared_ptr<zmtp::Context> g(&zmtp::Context::global(), [](zmtp::Context*) {});
    return g;
  });

  py::class_<Socket, std::shared_ptr<Socket>>(m, "Socket")
      .def_property_readonly("type", &Socket::type)
      .def("setsockopt", [](Socket& s, int opt, int64_t v) { guarded([&] { s.setsockopt(opt, v); }); })
      .def("setsockopt_bytes",
           [](Socket& s, int opt, const std::string& v) { guarded([&] { s.setsockopt_bytes(opt, v); }); })
      .def("getsockopt", [](Socket& s, int opt) { return guarded([&] { return s.getsockopt(opt); }); })
      .def("getsockopt_string",
           [](Socket& s, int opt) { return guarded([&] { return s.getsockopt_string(opt); }); })
      .def("bind", [](Socket& s, const std::string& a) {
        py::gil_scoped_release nogil;
        return guarded([&] { return s.bind(a); });
      })
      .def("unbind", [](Socket& s, const std::string& a) {
        py::gil_scoped_release nogil;
        guarded([&] { s.unbind(a); });
      })
      .def("connect", [](Socket& s, const std::string& a) {
        py::gil_scoped_release nogil;
        guarded([&] { s.connect(a); });
      })
      .def("disconnect", [](Socket& s, const std::string& a) {
        py::gil_scoped_release nogil;
        guarded([&] { s.disconnect(a); });
      })
      .def("send_multipart",
           [](Socket& s, const py::sequence& parts, int flags) {
             Message msg;
             msg.reserve(parts.size());
             for (auto h : parts) msg.push_back(frame_from_py(h));
             py::gil_scoped_release nogil;
             guarded([&] { s.send(std::move(msg), flags, signal_check()); });
           },
           py::arg("parts"), py::arg("flags") = 0)
      .def("recv_multipart",
           [](Socket& s, int flags) {
             Message msg;
             {
               py::gil_scoped_release nogil;
               msg = guarded([&] { return s.recv(flags, signal_check()); });
             }
             py::list out;
             for (size_t i = 0; i < msg.size(); ++i) {
               PyFrame pf;
               pf.f = std::move(msg[i]);
               pf.more = i + 1 < msg.size();
               out.append(py::cast(std::move(pf)));
             }
             return out;
           },
           py::arg("flags") = 0)
      .def("events", &Socket::events)
      .def("close",
           [](Socket& s, long linger) {
             py::gil_scoped_release nogil;
             s.close(linger);
           },
           py::arg("linger") = -2)
      .def_property_readonly("closed", &Socket::closed)
      .def("num_peers", &Socket::num_peers)
      .def("stats", [](Socket& s) {
        auto st = s.stats();
        py::dict d;
        d["msgs_in"] = st.msgs_in;
        d["msgs_out"] = st.msgs_out;
        d["bytes_in"] = st.bytes_in;
        d["bytes_out"] = st.bytes_out;
        return d;
      });

  m.def("poll",
        [](const std::vector<std::pair<std::shared_ptr<Socket>, int>>& items, long timeout_ms) {
          std::vector<std::pair<Socket*, int>> raw;
          for (auto& it : items) raw.emplace_back(it.first.get(), it.second);
          py::gil_scoped_release nogil;
          return guarded([&] { return Socket::poll(raw, timeout_ms, signal_check()); });
        });

  // One fair fan-in round over several sockets (the GPU loader's receive
  // policy): at most one message per producer pipe; list of multipart lists.
  m.def("recv_round",
        [](const std::vector<std::shared_ptr<Socket>>& socks, size_t max) {
          std::vector<Socket*> raw;
          for (auto& s : socks) raw.push_back(s.get());
          std::vector<Message> msgs;
          {
            py::gil_scoped_release nogil;
            guarded([&] { return Socket::recv_round(raw, msgs, max); });
          }
          py::list out;
          for (auto& msg : msgs) {
            py::list parts;
            for (size_t i = 0; i < msg.size(); ++i) {
              PyFrame pf;
              pf.f = std::move(msg[i]);
              pf.more = i + 1 < msg.size();
              parts.append(py::cast(std::move(pf)));
            }
            out.append(parts);
          }
          return out;
        },
        py::arg("sockets"), py::arg("max") = size_t(-1));

  m.def("greeting_bytes", [](bool as_server) { return py::bytes(zmtp::greeting_bytes(as_server)); });
  m.def("ready_command", [](int t, const std::string& id) { return py::bytes(zmtp::ready_command(t, id)); },
        py::arg("socket_type"), py::arg("identity") = "");
  m.def("socket_types_compatible", &zmtp::socket_types_compatible);

  // ---- shared-memory slot words ----
  // Atomic compare-and-swap on word `i` of a writable uint32 array mapped
  // over a ring segment (csrc/transport/shmring.h states): the Python
  // consumer claims / releases slots with the same atomics as the C++ side.
  m.def("slot_cas", [](py::array words, size_t i, uint32_t expected, uint32_t desired) {
    // no conversion: a cast copy would make the CAS act on a temporary
    if (!words.dtype().is(py::dtype::of<uint32_t>()) || !(words.flags() & py::array::c_style))
      throw py::type_error("slot_cas needs a C-contiguous uint32 array over the segment");
    auto info = words.request(true);
    if (info.ndim != 1 || i >= size_t(info.shape[0])) throw py::index_error("slot index out of range");
    auto* w = reinterpret_cast<std::atomic<uint32_t>*>(static_cast<uint32_t*>(info.ptr) + i);
    return w->compare_exchange_strong(expected, desired, std::memory_order_acq_rel);
  });

  // ---- codec ----
  m.def("pickle_describe", [](py::buffer b) {
    auto info = b.request();
    try {
      auto v = codec::parse(static_cast<const uint8_t*>(info.ptr), size_t(info.size * info.itemsize));
      return codec::describe(*v);
    } catch (const codec::Unsupported& e) {
      throw py::value_error(std::string("unsupported pickle: ") + e.what());
    }
  });
  // Zero-copy loads: ndarray values become views over `obj`'s buffer.
  // Raises ValueError for constructs outside the fast path (caller falls back
  // to pickle.loads).
  m.def("fast_loads", [](py::object obj) {
    py::buffer b = py::reinterpret_borrow<py::buffer>(obj);
    auto info = b.request();
    const uint8_t* base = static_cast<const uint8_t*>(info.ptr);
    try {
      auto v = codec::parse(base, size_t(info.size * info.itemsize));
      return value_to_py(*v, base, obj);
    } catch (const codec::Unsupported& e) {
      throw py::value_error(std::string("unsupported pickle: ") + e.what());
    }
  });
  // decode value transform: the cheapest per-channel form that reproduces
  // the fp32 table exactly (codec/xform_fit.h); None when there is none
  m.def("xform_fit",
        [](py::array_t<float, py::array::c_style | py::array::forcecast> x,
           py::array_t<float, py::array::c_style | py::array::forcecast> y, float scale, float mean, float std,
           bool normalize) -> py::object {
          if (x.size() != 256 || y.size() != 256) throw std::invalid_argument("xform_fit: x and y need 256 values");
          codec::XfChannel c;
          if (!codec::fit_channel(x.data(), y.data(), scale, mean, std, normalize, &c)) return py::none();
          return py::make_tuple(c.op, c.a, c.b, c.d, c.r);
        });
  m.def("xform_apply", [](int op, float a, float b, float d, float r, float x) {
    codec::XfChannel c;
    c.op = op, c.a = a, c.b = b, c.d = d, c.r = r;
    return codec::apply_channel(c, x);
  });
  m.def("btr_header", [](py::array_t<int64_t, py::array::c_style | py::array::forcecast> offs) {
    std::vector<int64_t> o(offs.data(), offs.data() + offs.size());
    auto h = codec::btr_header(o);
    return py::bytes(reinterpret_cast<const char*>(h.data()), h.size());
  });
  m.def("dumps_array_dict",
        [](const py::dict& d, int protocol, size_t align) {
          // Minimal writer used by tests/producers: str keys; values int, float,
          // str, bool, None or C-contiguous ndarray.
          codec::Writer w(protocol);
          w.begin_dict();
          for (auto kv : d) {
            w.key(kv.first.cast<std::string>());
            py::handle v = kv.second;
            if (v.is_none()) w.none();
            else if (py::isinstance<py::bool_>(v)) w.boolean(v.cast<bool>());
            else if (py::isinstance<py::int_>(v)) w.integer(v.cast<int64_t>());
            else if (py::isinstance<py::float_>(v)) w.real(v.cast<double>());
            else if (py::isinstance<py::str>(v)) w.str(v.cast<std::string>());
            else if (py::isinstance<py::array>(v)) {
              py::array a = py::reinterpret_borrow<py::array>(v);
              a = py::array::ensure(a, py::array::c_style);
              std::string ds = py::str(a.dtype().attr("str"));
              std::vector<int64_t> shape(a.shape(), a.shape() + a.ndim());
              w.ndarray(ds.substr(1), shape, a.data(), align);
            } else {
              throw py::type_error("dumps_array_dict: unsupported value type");
            }
          }
          w.end_dict();
          auto& out = w.finish();
          return py::bytes(reinterpret_cast<const char*>(out.data()), out.size());
        },
        py::arg("d"), py::arg("protocol") = 4, py::arg("align") = 0);

  // ---- headless renderer (used by the bpy shim's GPUOffScreen) ----
  // ---- rigid bodies (falling-cubes stand-in physics; also drives the bpy
  // shim's rigid-body world) ----
  struct PyRigid {
    sim::RigidWorld world;
    std::vector<sim::Box> boxes;
    explicit PyRigid(double plane_z) : world(plane_z) {}
  };
  py::class_<PyRigid>(m, "RigidWorld")
      .def(py::init<double>(), py::arg("plane_z"))
      .def("set_bodies",
           [](PyRigid& w, py::array_t<double, py::array::c_style | py::array::forcecast> centers,
              py::array_t<double, py::array::c_style | py::array::forcecast> rots,
              py::array_t<double, py::array::c_style | py::array::forcecast> halves) {
             const ssize_t n = centers.shape(0);
             if (centers.ndim() != 2 || centers.shape(1) != 3 || rots.ndim() != 3 || rots.shape(0) != n ||
                 rots.shape(1) != 3 || rots.shape(2) != 3 || halves.ndim() != 2 || halves.shape(0) != n ||
                 halves.shape(1) != 3)
               throw py::value_error("set_bodies: centers (n,3), rots (n,3,3), halves (n,3)");
             w.boxes.assign(size_t(n), sim::Box());
             for (ssize_t i = 0; i < n; ++i) {
               auto& b = w.boxes[size_t(i)];
               b.center = {centers.at(i, 0), centers.at(i, 1), centers.at(i, 2)};
               b.half = {halves.at(i, 0), halves.at(i, 1), halves.at(i, 2)};
               for (int k = 0; k < 9; ++k) b.rot[size_t(k)] = rots.at(i, k / 3, k % 3);
             }
             w.world.reset(w.boxes);
           })
      .def("step", [](PyRigid& w, double dt) { w.world.step(w.boxes, dt); }, py::arg("dt"))
      .def("centers",
           [](PyRigid& w) {
             py::array_t<double> out({py::ssize_t(w.boxes.size()), py::ssize_t(3)});
             auto o = out.mutable_unchecked<2>();
             for (size_t i = 0; i < w.boxes.size(); ++i) {
               o(i, 0) = w.boxes[i].center.x, o(i, 1) = w.boxes[i].center.y, o(i, 2) = w.boxes[i].center.z;
             }
             return out;
           })
      .def("rotations",
           [](PyRigid& w) {
             py::array_t<double> out({py::ssize_t(w.boxes.size()), py::ssize_t(3), py::ssize_t(3)});
             auto o = out.mutable_unchecked<3>();
             for (size_t i = 0; i < w.boxes.size(); ++i)
               for (int k = 0; k < 9; ++k) o(i, k / 3, k % 3) = w.boxes[i].rot[size_t(k)];
             return out;
           })
      .def("min_corner_z",
           [](PyRigid& w) {
             double z = 1e300;
             for (auto& b : w.boxes)
               for (auto& c : b.corners()) z = std::min(z, c.z);
             return z;
           })
      .def("kinetic_energy", [](PyRigid& w) { return w.world.kinetic_energy(w.boxes); });

  m.def("render_boxes",
        [](int width, int height, int channels, bool lower_left, std::vector<double> cam_loc,
           std::vector<double> cam_rot, double lens, double sensor, std::vector<double> light_loc,
           double light_power, double plane_z, double plane_half, const py::list& boxes) {
          if (cam_loc.size() != 3 || cam_rot.size() != 9 || light_loc.size() != 3)
            throw py::value_error("render_boxes: bad camera/light vectors");
          if (channels != 3 && channels != 4) throw py::value_error("render_boxes: channels must be 3 or 4");
          sim::Scene sc;
          sc.cam.width = width;
          sc.cam.height = height;
          sc.cam.lens_mm = lens;
          sc.cam.sensor_mm = sensor;
          sc.cam.loc = {cam_loc[0], cam_loc[1], cam_loc[2]};
          for (int i = 0; i < 9; ++i) sc.cam.rot[i] = cam_rot[i];
          sc.light.loc = {light_loc[0], light_loc[1], light_loc[2]};
          sc.light.power = light_power;
          sc.plane_z = plane_z;
          sc.plane_half = plane_half;
          for (auto h : boxes) {
            auto t = h.cast<py::tuple>();
            auto c = t[0].cast<std::vector<double>>();
            auto hf = t[1].cast<std::vector<double>>();
            auto r = t[2].cast<std::vector<double>>();
            auto a = t[3].cast<std::vector<double>>();
            sim::Box b;
            b.center = {c[0], c[1], c[2]};
            b.half = {hf[0], hf[1], hf[2]};
            for (int i = 0; i < 9; ++i) b.rot[i] = r[i];
            b.albedo = {float(a[0]), float(a[1]), float(a[2])};
            sc.boxes.push_back(b);
          }
          py::array_t<uint8_t> out({height, width, channels});
          {
            py::gil_scoped_release nogil;
            sim::render(sc, out.mutable_data(), channels, lower_left);
          }
          return out;
        });

  // ---- batched remote-env client (VectorRemoteEnv fast path) ----
  // N REQ sockets (RELAXED + CORRELATE, like btt.env.RemoteEnv); step()
  // fans the requests out before gathering any reply, all with the GIL
  // released, and decodes numeric obs/reward/done/time straight into arrays.
  struct VecReq {
    // own IO threads (declared first: destroyed after the sockets); several
    // threads let the per-message wake-ups of N envs proceed in parallel
    std::vector<std::unique_ptr<zmtp::Context>> ctxs;
    std::vector<std::shared_ptr<Socket>> socks;
    std::vector<int64_t> times;
    std::vector<bool> has_time;
    std::vector<std::vector<uint8_t>> last;   // raw last replies (for info dicts)
  };
  py::class_<VecReq, std::shared_ptr<VecReq>>(m, "VecReq")
      .def(py::init([](const std::vector<std::string>& addresses, long timeoutms, int io_threads) {
             auto v = std::make_shared<VecReq>();
             // measured on MI355X hosts (profiles/results_r1_gpu.jsonl): 4 IO threads give
             // 8 envs 61k -> 76k and 32 envs 68k -> 126k steps/s over 1 thread; 8 are no better
             const int n_io = io_threads > 0 ? io_threads : std::max(1, std::min(4, int(addresses.size()) / 2));
             for (int k = 0; k < n_io; ++k) v->ctxs.emplace_back(new zmtp::Context());
             for (size_t j = 0; j < addresses.size(); ++j) {
               const auto& a = addresses[j];
               auto s = v->ctxs[j % v->ctxs.size()]->socket(zmtp::REQ);
               s->setsockopt(zmtp::LINGER, 0);
               s->setsockopt(zmtp::SNDTIMEO, timeoutms * 10);
               s->setsockopt(zmtp::RCVTIMEO, timeoutms);
               s->setsockopt(zmtp::REQ_RELAXED, 1);
               s->setsockopt(zmtp::REQ_CORRELATE, 1);
               s->connect(a);
               v->socks.push_back(s);
             }
             v->times.assign(addresses.size(), 0);
             v->has_time.assign(addresses.size(), false);
             v->last.resize(addresses.size());
             return v;
           }),
           py::arg("addresses"), py::arg("timeoutms") = 10000, py::arg("io_threads") = 0)
      .def("__len__", [](VecReq& v) { return v.socks.size(); })
      .def("exchange",
           [](VecReq& v, const std::vector<int>& which, const std::string& cmd,
              py::array_t<double, py::array::c_style | py::array::forcecast> actions, int obs_dim, int phase) {
             // phase 0: send all requests, then gather all replies; 1: send only
             // (step_async); 2: gather only (step_wait) -- cmd/actions unused
             const size_t n = which.size();
             if (phase != 2 && cmd == "step" && size_t(actions.size()) < n) throw py::value_error("one action per env");
             std::vector<double> act(actions.data(), actions.data() + actions.size());
             py::array_t<double> obs(std::vector<py::ssize_t>{py::ssize_t(n), py::ssize_t(obs_dim)});
             py::array_t<double> rew(std::vector<py::ssize_t>{py::ssize_t(n)});
             py::array_t<bool> done(std::vector<py::ssize_t>{py::ssize_t(n)});
             double* po = obs.mutable_data();
             double* pr = rew.mutable_data();
             bool* pd = done.mutable_data();
             std::string err;
             {
               py::gil_scoped_release nogil;
               try {
                 for (size_t k = 0; k < n && phase != 2; ++k) {
                   const int i = which[k];
                   codec::Writer w(4);
                   w.begin_dict();
                   w.key("cmd");
                   w.str(cmd);
                   if (cmd == "step") {
                     w.key("action");
                     w.real(act[k]);
                   }
                   w.key("time");
                   if (v.has_time[size_t(i)]) w.integer(v.times[size_t(i)]);
                   else w.none();
                   w.end_dict();
                   auto& b = w.finish();
                   Message m;
                   m.push_back(Frame::copy_of(b.data(), b.size()));
                   v.socks[size_t(i)]->send(std::move(m));
                 }
                 for (size_t k = 0; k < n && phase != 1; ++k) {
                   const int i = which[k];
                   Message r = v.socks[size_t(i)]->recv();
                   auto& raw = v.last[size_t(i)];
                   raw.assign(r[0].data(), r[0].data() + r[0].size);
                   auto root = codec::parse(raw.data(), raw.size());
                   auto num = [&](const codec::Value* x, double dflt) {
                     if (!x) return dflt;
                     if (x->kind == codec::Value::FLOAT) return x->f;
                     if (x->kind == codec::Value::INT) return double(x->i);
                     if (x->kind == codec::Value::BOOL) return x->b ? 1.0 : 0.0;
                     return dflt;
                   };
                   const codec::Value* o = root->get("obs");
                   for (int d = 0; d < obs_dim; ++d) {
                     double val = 0;
                     if (o && (o->kind == codec::Value::TUPLE || o->kind == codec::Value::LIST) &&
                         size_t(d) < o->items.size())
                       val = num(o->items[size_t(d)].get(), 0.0);
                     else if (o && o->kind == codec::Value::NDARRAY && d < o->numel()) {
                       if (o->dtype == "<f8") std::memcpy(&val, o->ptr(reinterpret_cast<const uint8_t*>(raw.data())) + 8 * size_t(d), 8);
                       else if (o->dtype == "<f4") {
                         float f;
                         std::memcpy(&f, o->ptr(reinterpret_cast<const uint8_t*>(raw.data())) + 4 * size_t(d), 4);
                         val = f;
                       }
                     } else if (o && d == 0)
                       val = num(o, 0.0);
                     po[k * size_t(obs_dim) + size_t(d)] = val;
                   }
                   pr[k] = num(root->get("reward"), 0.0);
                   const codec::Value* dn = root->get("done");
                   pd[k] = dn && ((dn->kind == codec::Value::BOOL && dn->b) || (dn->kind == codec::Value::INT && dn->i));
                   const codec::Value* t = root->get("time");
                   if (t && t->kind == codec::Value::INT) {
                     v.times[size_t(i)] = t->i;
                     v.has_time[size_t(i)] = true;
                   }
                 }
               } catch (const zmtp::Error& e) {
                 err = e.code == zmtp::E_AGAIN ? "Failed to receive from remote environment" : e.what();
               } catch (const std::exception& e) {
                 err = e.what();
               }
             }
             if (!err.empty()) throw py::value_error(err);
             return py::make_tuple(obs, rew, done);
           },
           py::arg("which"), py::arg("cmd"), py::arg("actions"), py::arg("obs_dim"), py::arg("phase") = 0)
      .def("roundtrip",
           [](VecReq& v, int i, py::bytes request) {
             // one pickled request -> the raw reply frame, GIL released
             // (btt.env.RemoteEnv on the native client: N = 1)
             if (i < 0 || size_t(i) >= v.socks.size()) throw py::index_error("env index");
             std::string req = request;
             std::string err;
             Message r;
             {
               py::gil_scoped_release nogil;
               try {
                 Message m;
                 m.push_back(Frame::copy_of(req.data(), req.size()));
                 try {
                   v.socks[size_t(i)]->send(std::move(m));
                 } catch (const zmtp::Error& e) {
                   throw std::runtime_error(e.code == zmtp::E_AGAIN ? "Failed to send to remote environment"
                                                                    : e.what());
                 }
                 try {
                   r = v.socks[size_t(i)]->recv();
                 } catch (const zmtp::Error& e) {
                   throw std::runtime_error(e.code == zmtp::E_AGAIN ? "Failed to receive from remote environment"
                                                                    : e.what());
                 }
               } catch (const std::exception& e) {
                 err = e.what();
               }
             }
             if (!err.empty()) throw py::value_error(err);
             if (r.size() != 1) throw py::value_error("expected a single-frame reply");
             v.last[size_t(i)].assign(r[0].data(), r[0].data() + r[0].size);
             return py::bytes(reinterpret_cast<const char*>(r[0].data()), r[0].size);
           },
           py::arg("i"), py::arg("request"))
      .def("last_reply", [](VecReq& v, int i) {
        // full reply dict of env i (info, rgb_array, ...), decoded lazily
        auto& raw = v.last[size_t(i)];
        py::bytearray owner(reinterpret_cast<const char*>(raw.data()), raw.size());
        const uint8_t* base = reinterpret_cast<const uint8_t*>(PyByteArray_AsString(owner.ptr()));
        auto root = codec::parse(base, raw.size());
        return value_to_py(*root, base, owner);
      })
      .def("close", [](VecReq& v) {
        py::gil_scoped_release nogil;
        for (auto& s : v.socks) s->close(0);
        v.socks.clear();
        v.ctxs.clear();
      });
}
