// pybind11 bindings of the GPU side: gfx950 kernels (pointer-level, the
// Python layer passes torch tensors' data_ptr() and stream handles) and the
// StreamLoader.  Built as `blendtorch/_hip*.so` by hipcc for gfx950; it links
// the HIP runtime torch already loaded (same soname), so device pointers and
// streams are shared with torch.
#include <hip/hip_runtime_api.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <chrono>
#include <tuple>
#include <cstring>
#include <stdexcept>
#include <string>
#include <sys/mman.h>

#include "../python/pyvalue.h"
#include "comm.h"
#include "kernels.h"
#include "loader.h"

namespace py = pybind11;
using namespace btn;
using namespace btn::gpu;

namespace {

template <typename T>
T* ptr(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}

// BnActIn from Python: None, or (acc, R, M, eps, momentum, w, b, slope, mean, invstd, rm, rv, tracked) --
// integers are device pointers (0 = none)
BnActIn act_from(const py::object& o, const char* what) {
  BnActIn a;
  if (o.is_none()) return a;
  const py::tuple f = o.cast<py::tuple>();
  if (f.size() != 13)
    throw std::invalid_argument(std::string(what) +
                                ": act is (acc, R, M, eps, momentum, w, b, slope, mean, invstd, rm, rv, tracked)");
  a.acc = ptr<double>(f[0].cast<uintptr_t>());
  a.R = f[1].cast<int>();
  a.M = f[2].cast<int64_t>();
  a.eps = f[3].cast<float>();
  a.momentum = f[4].cast<float>();
  a.w = ptr<const float>(f[5].cast<uintptr_t>());
  a.b = ptr<const float>(f[6].cast<uintptr_t>());
  a.slope = f[7].cast<float>();
  a.mean = ptr<float>(f[8].cast<uintptr_t>());
  a.invstd = ptr<float>(f[9].cast<uintptr_t>());
  a.rm = ptr<float>(f[10].cast<uintptr_t>());
  a.rv = ptr<float>(f[11].cast<uintptr_t>());
  a.tracked = ptr<int64_t>(f[12].cast<uintptr_t>());
  if (!a.w) throw std::invalid_argument(std::string(what) + ": act needs the BN weight");
  return a;
}

hipStream_t stream_of(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// Native default_collate of a batch's metadata: for every key of the first
// item's dict, values of one scalar kind become one numpy array (int ->
// int64, float -> float64, bool -> bool, numpy scalars keep their dtype),
// same-shape C-order ndarrays are stacked into one [B, ...] array; anything
// else (strings, nested containers, ragged arrays, missing keys) comes back
// as a list of per-item Python values.  torch.from_numpy on the arrays gives
// what torch.utils.data.default_collate would, without per-item objects.
py::dict collate_meta(const std::vector<BatchMeta>& items) {
  using K = codec::Value;
  py::dict out;
  if (items.empty() || !items[0].tree || items[0].tree->kind != K::DICT) return out;
  const size_t B = items.size();
  const K& first = *items[0].tree;
  for (size_t k = 0; k + 1 < first.items.size(); k += 2) {
    if (first.items[k]->kind != K::STR) continue;
    const std::string& key = first.items[k]->s;
    std::vector<const K*> vals(B, nullptr);
    bool all = true;
    for (size_t i = 0; i < B && all; ++i) {
      vals[i] = items[i].tree ? items[i].tree->get(key) : nullptr;
      all = vals[i] != nullptr;
    }
    const K* v0 = all ? vals[0] : nullptr;
    auto same = [&](auto pred) {
      for (auto* v : vals)
        if (!pred(*v)) return false;
      return true;
    };
    py::object col;
    if (v0 && !v0->np_scalar && v0->kind == K::INT &&
        same([](const K& v) { return v.kind == K::INT && !v.np_scalar; })) {
      py::array_t<int64_t> a(static_cast<py::ssize_t>(B));
      for (size_t i = 0; i < B; ++i) a.mutable_at(i) = vals[i]->i;
      col = a;
    } else if (v0 && !v0->np_scalar && v0->kind == K::FLOAT &&
               same([](const K& v) { return v.kind == K::FLOAT && !v.np_scalar; })) {
      py::array_t<double> a(static_cast<py::ssize_t>(B));
      for (size_t i = 0; i < B; ++i) a.mutable_at(i) = vals[i]->f;
      col = a;
    } else if (v0 && !v0->np_scalar && v0->kind == K::BOOL &&
               same([](const K& v) { return v.kind == K::BOOL && !v.np_scalar; })) {
      py::array_t<bool> a(static_cast<py::ssize_t>(B));
      for (size_t i = 0; i < B; ++i) a.mutable_at(i) = vals[i]->b;
      col = a;
    } else if (v0 && (v0->kind == K::NDARRAY || v0->np_scalar) &&
               same([&](const K& v) {
                 return (v.kind == K::NDARRAY || v.np_scalar) && v.np_scalar == v0->np_scalar && !v.fortran &&
                        v.dtype == v0->dtype && v.shape == v0->shape;
               })) {
      std::vector<py::ssize_t> shape{py::ssize_t(B)};
      if (!v0->np_scalar) shape.insert(shape.end(), v0->shape.begin(), v0->shape.end());
      py::array a{py::dtype(v0->dtype), shape};
      const size_t nb = v0->np_scalar ? v0->itemsize() : size_t(v0->numel()) * v0->itemsize();
      auto* dst = static_cast<uint8_t*>(a.mutable_data());
      for (size_t i = 0; i < B; ++i) std::memcpy(dst + i * nb, vals[i]->ptr(items[i].bytes.data()), nb);
      col = a;
    } else {
      py::list l;
      for (size_t i = 0; i < B; ++i) {
        if (!vals[i]) {
          l.append(py::none());
          continue;
        }
        py::bytearray owner(reinterpret_cast<const char*>(items[i].bytes.data()), items[i].bytes.size());
        const uint8_t* base = reinterpret_cast<const uint8_t*>(PyByteArray_AsString(owner.ptr()));
        l.append(pyconv::value_to_py(*vals[i], base, owner));
      }
      col = l;
    }
    out[py::str(key)] = col;
  }
  return out;
}

void fill_cmap(int* dst, const std::vector<int>& cmap) {
  for (size_t i = 0; i < 4; ++i) dst[i] = i < cmap.size() ? cmap[i] : int(i);
}

}  // namespace

// a deferred weight-gradient slice reduce (ConvWgradParams::Reduce) as a
// plain tuple: (partial, S, Cout, Cin, cin_out, out, s_co, s_ci, s_kh, s_kw, rx, ry, sub)
py::tuple reduce_to_tuple(const ConvWgradParams::Reduce& r) {
  return py::make_tuple(reinterpret_cast<uintptr_t>(r.partial), r.S, r.Cout, r.Cin, r.cin_out,
                        reinterpret_cast<uintptr_t>(r.out), r.s_co, r.s_ci, r.s_kh, r.s_kw, r.rx, r.ry, r.sub);
}

ConvWgradParams::Reduce reduce_from_tuple(const py::tuple& t) {
  if (t.size() != 13) throw std::invalid_argument("conv_wgrad: a deferred reduce is a 13-tuple");
  ConvWgradParams::Reduce r;
  r.partial = reinterpret_cast<const float*>(t[0].cast<uintptr_t>());
  r.S = t[1].cast<int>(), r.Cout = t[2].cast<int>(), r.Cin = t[3].cast<int>(), r.cin_out = t[4].cast<int>();
  r.out = reinterpret_cast<float*>(t[5].cast<uintptr_t>());
  r.s_co = t[6].cast<int64_t>(), r.s_ci = t[7].cast<int64_t>(), r.s_kh = t[8].cast<int64_t>();
  r.s_kw = t[9].cast<int64_t>(), r.rx = t[10].cast<int>(), r.ry = t[11].cast<int>();
  r.sub = t[12].cast<int>();
  return r;
}


// densityopt gate / S step: the parameters as a dict of device pointers (ints) and scalars
DoptParams dopt_from_dict(const py::dict& d) {
  DoptParams p;
  auto ptr = [&](const char* k) -> uintptr_t { return d.contains(k) ? d[k].cast<uintptr_t>() : 0; };
  auto f32 = [&](const char* k, float dflt) { return d.contains(k) ? d[k].cast<float>() : dflt; };
  auto i32 = [&](const char* k, int dflt) { return d.contains(k) ? d[k].cast<int>() : dflt; };
  p.logit_real = reinterpret_cast<const float*>(ptr("logit_real"));
  p.logit_sim = reinterpret_cast<const float*>(ptr("logit_sim"));
  p.logit_s = reinterpret_cast<const float*>(ptr("logit_s"));
  p.stats = reinterpret_cast<float*>(ptr("stats"));
  p.gate_d = reinterpret_cast<float*>(ptr("gate_d"));
  p.threshold = f32("threshold", 0.7f);
  p.sid = reinterpret_cast<const int64_t*>(ptr("sid"));
  p.samples = reinterpret_cast<float*>(ptr("samples"));
  p.mean = reinterpret_cast<float*>(ptr("mean"));
  p.log_std = reinterpret_cast<float*>(ptr("log_std"));
  p.exp_avg = reinterpret_cast<float*>(ptr("exp_avg"));
  p.exp_avg_sq = reinterpret_cast<float*>(ptr("exp_avg_sq"));
  p.adam_step = reinterpret_cast<float*>(ptr("adam_step"));
  p.lr = f32("lr", 5e-2f), p.b1 = f32("b1", 0.7f), p.b2 = f32("b2", 0.999f), p.eps = f32("eps", 1e-8f);
  p.b = reinterpret_cast<float*>(ptr("b"));
  p.first = reinterpret_cast<float*>(ptr("first"));
  p.gate_s = reinterpret_cast<float*>(ptr("gate_s"));
  p.alpha = f32("alpha", 0.9f);
  p.params_out = reinterpret_cast<float*>(ptr("params_out"));
  p.red = reinterpret_cast<float*>(ptr("red"));
  p.host = reinterpret_cast<float*>(ptr("host"));
  p.counter = reinterpret_cast<uint32_t*>(ptr("counter"));
  p.seed = d.contains("seed") ? d["seed"].cast<uint64_t>() : 0;
  p.B = i32("B", 0), p.N = i32("N", 0), p.rank = i32("rank", 0), p.world = i32("world", 1);
  return p;
}

PYBIND11_MODULE(_hip, m) {
  m.doc() = "blendtorch gfx950 kernels + GPU stream loader";

  m.def("runtime_version", [] {
    int v = 0;
    hipRuntimeGetVersion(&v);
    return v;
  });
  m.def("device_count", [] {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });
  m.def("pci_bus_id", [](int dev) {
    char buf[64] = {0};
    check(hipDeviceGetPCIBusId(buf, int(sizeof(buf)), dev), "hipDeviceGetPCIBusId");
    return std::string(buf);
  });
  m.def("device_arch", [](int dev) {
    hipDeviceProp_t p;
    check(hipGetDeviceProperties(&p, dev), "hipGetDeviceProperties");
    return std::string(p.gcnArchName);
  });

  m.def("decode",
        [](uintptr_t src, uintptr_t src_offsets, uintptr_t dst, uintptr_t lut, uintptr_t flip, int B, int H, int W,
           int Cin, int Cout, std::vector<int> cmap, int flip_all, int out_dtype, int layout, uintptr_t stream,
           bool src_offsets_aligned) {
          DecodeParams p;
          p.src = ptr<const uint8_t>(src);
          p.src_offsets = ptr<const int64_t>(src_offsets);
          p.src_offsets_aligned = src_offsets_aligned;
          p.dst = ptr<void>(dst);
          p.lut = ptr<const float>(lut);
          p.flip = ptr<const uint8_t>(flip);
          p.B = B, p.H = H, p.W = W, p.Cin = Cin, p.Cout = Cout;
          fill_cmap(p.cmap, cmap);
          p.flip_all = flip_all;
          p.out_dtype = out_dtype;
          p.layout = layout;
          check(decode(p, stream_of(stream)), "decode");
        },
        py::arg("src"), py::arg("src_offsets"), py::arg("dst"), py::arg("lut"), py::arg("flip"), py::arg("B"),
        py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("Cout"), py::arg("cmap"), py::arg("flip_all"),
        py::arg("out_dtype"), py::arg("layout"), py::arg("stream"), py::arg("src_offsets_aligned") = false);

  m.def("replay_sample",
        [](uintptr_t store, int64_t count, uintptr_t dst, uintptr_t lut, int B, int H, int W, int Cin, int Cout,
           std::vector<int> cmap, int flip_all, int out_dtype, int layout, uint64_t seed, uintptr_t counter,
           uint64_t ctr_value, uintptr_t index_in, uintptr_t index_out, std::vector<uintptr_t> meta_src, std::vector<uintptr_t> meta_dst,
           std::vector<int> meta_bytes, uintptr_t stream, int xf_table_only) {
          DecodeParams p;
          p.xf_table_only = xf_table_only;
          p.src = ptr<const uint8_t>(store);
          p.dst = ptr<void>(dst);
          p.lut = ptr<const float>(lut);
          p.B = B, p.H = H, p.W = W, p.Cin = Cin, p.Cout = Cout;
          fill_cmap(p.cmap, cmap);
          p.flip_all = flip_all;
          p.out_dtype = out_dtype;
          p.layout = layout;
          ReplayParams r;
          r.count = count;
          r.frame_bytes = int64_t(H) * W * Cin;
          r.seed = seed;
          r.counter = ptr<uint64_t>(counter);
          r.ctr_value = ctr_value;
          r.index_in = ptr<const int64_t>(index_in);
          r.index_out = ptr<int64_t>(index_out);
          if (meta_src.size() != meta_dst.size() || meta_src.size() != meta_bytes.size() ||
              meta_src.size() > size_t(kMaxMeta))
            throw std::invalid_argument("replay_sample: metadata columns mismatch or > kMaxMeta");
          r.nmeta = int(meta_src.size());
          for (int k = 0; k < r.nmeta; ++k) {
            r.meta_src[k] = ptr<const uint8_t>(meta_src[size_t(k)]);
            r.meta_dst[k] = ptr<uint8_t>(meta_dst[size_t(k)]);
            r.meta_bytes[k] = meta_bytes[size_t(k)];
          }
          check(replay_sample(p, r, stream_of(stream)), "replay_sample");
        },
        py::arg("store"), py::arg("count"), py::arg("dst"), py::arg("lut"), py::arg("B"), py::arg("H"), py::arg("W"),
        py::arg("Cin"), py::arg("Cout"), py::arg("cmap"), py::arg("flip_all"), py::arg("out_dtype"), py::arg("layout"),
        py::arg("seed"), py::arg("counter"), py::arg("ctr_value"), py::arg("index_in"), py::arg("index_out"), py::arg("meta_src"),
        py::arg("meta_dst"), py::arg("meta_bytes"), py::arg("stream"), py::arg("xf_table_only") = 0);

  m.def("multi_cast",
        [](std::vector<uintptr_t> src, std::vector<uintptr_t> dst, std::vector<int64_t> numel, int mode,
           uintptr_t stream) {
          if (src.size() != dst.size() || src.size() != numel.size() || src.size() > size_t(kMaxCast))
            throw std::invalid_argument("multi_cast: list lengths differ or exceed kMaxCast");
          CastParams p;
          p.n = int(src.size());
          p.mode = mode;
          for (int k = 0; k < p.n; ++k) {
            p.src[k] = ptr<const void>(src[size_t(k)]);
            p.dst[k] = ptr<void>(dst[size_t(k)]);
            p.numel[k] = numel[size_t(k)];
          }
          check(multi_cast(p, stream_of(stream)), "multi_cast");
        });

  m.def("conv_wgrad_slices", &conv_wgrad_slices);
  m.def("conv_c4p_rows", &conv_c4p_rows);
  m.def("conv_set_c4p_rows", &conv_set_c4p_rows);
  m.def("conv_set_wgrad_co128", &conv_set_wgrad_co128);
  m.def("conv_set_dgrad_bn128", &conv_set_dgrad_bn128);
  m.def("conv_set_fwd_split", &conv_set_fwd_split);
  m.def("conv_fwd_split_launches", &conv_fwd_split_launches);
  m.def("conv_dgrad_hold", [](int on) { conv_dgrad_hold(on); });
  m.def("conv_dgrad_flush", []() { check(conv_dgrad_flush(), "conv_dgrad_flush"); });
  m.def("conv_dgrad_held", []() { return conv_dgrad_held(); });
  m.def("conv_wgrad",
        [](uintptr_t x, uintptr_t dy, uintptr_t partial, int N, int H, int W, int Cin, int Ho, int Wo, int Cout,
           int slices, int64_t px_per_slice, uintptr_t out, int64_t s_co, int64_t s_ci, int64_t s_kh, int64_t s_kw,
           uintptr_t stream, int cin_out, bool defer, py::object side, uintptr_t lut, py::object fold,
           py::object bn_dy) -> py::object {
          ConvWgradParams p;
          p.cin_out = cin_out;
          if (!bn_dy.is_none()) {   // (y, mean, invstd, w, b, dw, db, slope[, acc, R, dw_out, db_out, gx_out])
            const py::tuple f = bn_dy.cast<py::tuple>();
            if (f.size() != 8 && f.size() != 13)
              throw std::invalid_argument(
                  "conv_wgrad: bn_dy is (y, mean, invstd, w, b, dw, db, slope[, acc, R, dw_out, db_out, gx_out])");
            if (f.size() == 13) {
              p.bn_dy.acc = ptr<double>(f[8].cast<uintptr_t>());
              p.bn_dy.R = f[9].cast<int>();
              p.bn_dy.dw_out = ptr<float>(f[10].cast<uintptr_t>());
              p.bn_dy.db_out = ptr<float>(f[11].cast<uintptr_t>());
              p.bn_dy.gx_out = ptr<uint16_t>(f[12].cast<uintptr_t>());
            }
            p.bn_dy.y = ptr<const uint16_t>(f[0].cast<uintptr_t>());
            p.bn_dy.mean = ptr<const float>(f[1].cast<uintptr_t>());
            p.bn_dy.invstd = ptr<const float>(f[2].cast<uintptr_t>());
            p.bn_dy.w = ptr<const float>(f[3].cast<uintptr_t>());
            p.bn_dy.b = ptr<const float>(f[4].cast<uintptr_t>());
            p.bn_dy.dw = ptr<const float>(f[5].cast<uintptr_t>());
            p.bn_dy.db = ptr<const float>(f[6].cast<uintptr_t>());
            p.bn_dy.slope = f[7].cast<float>();
          }
          if (!fold.is_none()) {   // (acc, R, C, M, dw, db)
            const py::tuple f = fold.cast<py::tuple>();
            if (f.size() != 6) throw std::invalid_argument("conv_wgrad: fold is (acc, R, C, M, dw, db)");
            p.fold.acc = reinterpret_cast<double*>(f[0].cast<uintptr_t>());
            p.fold.R = f[1].cast<int>(), p.fold.C = f[2].cast<int>(), p.fold.M = f[3].cast<int64_t>();
            p.fold.dw = reinterpret_cast<float*>(f[4].cast<uintptr_t>());
            p.fold.db = reinterpret_cast<float*>(f[5].cast<uintptr_t>());
          }
          p.lut = ptr<const uint16_t>(lut);
          p.x = ptr<const uint16_t>(x);
          p.dy = ptr<const uint16_t>(dy);
          p.partial = ptr<float>(partial);
          p.N = N, p.H = H, p.W = W, p.Cin = Cin, p.Ho = Ho, p.Wo = Wo, p.Cout = Cout;
          p.M = int64_t(N) * Ho * Wo;
          p.slices = slices;
          p.px_per_slice = px_per_slice;
          ConvWgradParams::Reduce sd, df;
          const bool has_side = !side.is_none();
          if (has_side) sd = reduce_from_tuple(side.cast<py::tuple>());
          check(conv_wgrad(p, ptr<float>(out), s_co, s_ci, s_kh, s_kw, stream_of(stream), defer ? &df : nullptr,
                           has_side ? &sd : nullptr),
                "conv_wgrad");
          if (!defer) return py::none();
          return reduce_to_tuple(df);
        },
        py::arg("x"), py::arg("dy"), py::arg("partial"), py::arg("N"), py::arg("H"), py::arg("W"), py::arg("Cin"),
        py::arg("Ho"), py::arg("Wo"), py::arg("Cout"), py::arg("slices"), py::arg("px_per_slice"), py::arg("out"),
        py::arg("s_co"), py::arg("s_ci"), py::arg("s_kh"), py::arg("s_kw"), py::arg("stream"), py::arg("cin_out") = 0,
        py::arg("defer") = false, py::arg("side") = py::none(), py::arg("lut") = 0, py::arg("fold") = py::none(),
        py::arg("bn_dy") = py::none());
  // a deferred slice reduce on its own (a weight-gradient chain that ended early)
  m.def("conv_wgrad_reduce", [](py::tuple r, uintptr_t stream) {
    check(conv_wgrad_reduce(reduce_from_tuple(r), stream_of(stream)), "conv_wgrad_reduce");
  });

  m.def("conv_fwd_tiles", &conv_fwd_tiles);
  m.def("conv_set_tiles", &conv_set_tiles, py::arg("bm") = 0, py::arg("bn") = 0, py::arg("staging") = -1,
        py::arg("dgrad_cls") = 0);
  m.def("conv_dgrad_classes_per_block", &conv_dgrad_classes_per_block);
  m.def("conv_set_fwd_patch", &conv_set_fwd_patch, py::arg("on"), py::arg("dbg") = 0, py::arg("blocks") = 0);
  m.def("dopt_gate", [](const py::dict& d, int phase, uintptr_t stream) {
    check(dopt_gate(dopt_from_dict(d), phase, reinterpret_cast<hipStream_t>(stream)), "dopt_gate");
  });
  m.def("dopt_sstep", [](const py::dict& d, int phase, uintptr_t stream) {
    check(dopt_sstep(dopt_from_dict(d), phase, reinterpret_cast<hipStream_t>(stream)), "dopt_sstep");
  });
  m.def("host_mapped_alloc", [](size_t bytes) {
    void* dev = nullptr;
    void* host = host_mapped_alloc(bytes, &dev);
    if (!host) throw std::runtime_error("host_mapped_alloc: hipHostMalloc(mapped) failed");
    return py::make_tuple(reinterpret_cast<uintptr_t>(host), reinterpret_cast<uintptr_t>(dev));
  });
  m.def("host_mapped_free", [](uintptr_t host) { host_mapped_free(reinterpret_cast<void*>(host)); });
  m.def("conv_set_wgrad_ordered", &conv_set_wgrad_ordered);
  m.def("conv_set_wgrad_staging", &conv_set_wgrad_staging);
  m.def("conv_set_wgrad_pipe", &conv_set_wgrad_pipe);
  m.def("conv_set_wgrad_wide", &conv_set_wgrad_wide);
  m.def("conv_set_dgrad_patch", &conv_set_dgrad_patch);
  m.def("conv_set_conv1_tiles", &conv_set_conv1_tiles, py::arg("tiles"), py::arg("rows") = 0);
  m.def("conv_set_c4_wave_private", &conv_set_c4_wave_private);
  m.def("conv_set_c4w_waves", &conv_set_c4w_waves);
  m.def("head_set_fast", &head_set_fast);
  m.def("conv_tile_pixels", &conv_tile_pixels);
  m.def("conv_tile_channels", &conv_tile_channels);
  m.def("conv_dgrad_supported", &conv_dgrad_supported);
  m.def("conv_weight_t", [](uintptr_t w, uintptr_t wt, int Cout, int Cin, uintptr_t stream) {
    check(conv_weight_t(ptr<const uint16_t>(w), ptr<uint16_t>(wt), Cout, Cin, stream_of(stream)), "conv_weight_t");
  });
  m.def("conv_weight_t_multi", [](std::vector<uintptr_t> src, std::vector<uintptr_t> dst, std::vector<int> cout,
                                  std::vector<int> cin, uintptr_t stream) {
    const size_t n = src.size();
    if (dst.size() != n || cout.size() != n || cin.size() != n || n > size_t(kMaxWeightT))
      throw std::invalid_argument("conv_weight_t_multi: list lengths differ or exceed kMaxWeightT");
    WeightTParams p;
    p.n = int(n);
    for (size_t k = 0; k < n; ++k) {
      p.src[k] = ptr<const uint16_t>(src[k]);
      p.dst[k] = ptr<uint16_t>(dst[k]);
      p.cout[k] = cout[k];
      p.cin[k] = cin[k];
    }
    check(conv_weight_t_multi(p, stream_of(stream)), "conv_weight_t_multi");
  });
  m.def(
      "conv_dgrad",
      [](uintptr_t dy, uintptr_t wt, uintptr_t dx, int N, int H, int W, int Cin, int Cout, uintptr_t stream,
         uintptr_t bn_x, uintptr_t bn_mean, uintptr_t bn_invstd, uintptr_t bn_w, uintptr_t bn_b, float bn_slope,
         uintptr_t bn_part, int bn_rows, int bn_acc_r) {
        BnBwdFuse bn;
        bn.acc_r = bn_acc_r;
        bn.x = ptr<const uint16_t>(bn_x);
        bn.mean = ptr<const float>(bn_mean);
        bn.invstd = ptr<const float>(bn_invstd);
        bn.w = ptr<const float>(bn_w);
        bn.b = ptr<const float>(bn_b);
        bn.slope = bn_slope;
        bn.part = ptr<float>(bn_part);
        bn.rows = bn_rows;
        check(conv_dgrad(ptr<const uint16_t>(dy), ptr<const uint16_t>(wt), ptr<uint16_t>(dx), N, H, W, Cin, Cout,
                         stream_of(stream), bn_part ? &bn : nullptr),
              "conv_dgrad");
      },
      py::arg("dy"), py::arg("wt"), py::arg("dx"), py::arg("N"), py::arg("H"), py::arg("W"), py::arg("Cin"),
      py::arg("Cout"), py::arg("stream"), py::arg("bn_x") = 0, py::arg("bn_mean") = 0, py::arg("bn_invstd") = 0,
      py::arg("bn_w") = 0, py::arg("bn_b") = 0, py::arg("bn_slope") = 0.f, py::arg("bn_part") = 0,
      py::arg("bn_rows") = 0, py::arg("bn_acc_r") = 0);
  m.def("conv_dgrad_bn_rows", &conv_dgrad_bn_rows);
  m.def("bn_backward_from_stats",
        [](uintptr_t x, uintptr_t gy, uintptr_t gx, int64_t M, int C, int dtype, uintptr_t part, int rows,
           uintptr_t mean, uintptr_t invstd, uintptr_t w, uintptr_t b, uintptr_t dw, uintptr_t db, float slope,
           uintptr_t stream) {
          hipStream_t s = stream_of(stream);
          check(bn_bwd_finalize_rows(ptr<const float>(part), rows, C, ptr<float>(dw), ptr<float>(db), s),
                "bn_bwd_finalize_rows");
          check(bn_bwd_apply(ptr<const void>(x), ptr<const void>(gy), ptr<void>(gx), M, C, dtype,
                             ptr<const float>(mean), ptr<const float>(invstd), ptr<const float>(w),
                             ptr<const float>(b), ptr<const float>(dw), ptr<const float>(db), slope, s),
                "bn_bwd_apply");
        });
  m.def("conv_fwd",
        [](uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats, int N, int H, int W, int Cin, int Ho, int Wo,
           int Cout, uintptr_t stream, int w_channels, int acc_r, uintptr_t lut, py::object act,
           uintptr_t act_out, py::object out_act, uintptr_t out_y) {
          ConvFwdParams p;
          p.act = act_from(act, "conv_fwd");
          p.act_out = ptr<uint16_t>(act_out);
          p.out_act = act_from(out_act, "conv_fwd(out_act)");
          p.out_y = ptr<uint16_t>(out_y);
          p.lut = ptr<const uint16_t>(lut);
          p.w_channels = w_channels;
          p.acc_r = acc_r;
          p.x = ptr<const uint16_t>(x);
          p.w = ptr<const uint16_t>(w);
          p.y = ptr<uint16_t>(y);
          p.stats = ptr<float>(stats);
          p.N = N, p.H = H, p.W = W, p.Cin = Cin, p.Ho = Ho, p.Wo = Wo, p.Cout = Cout;
          p.M = int64_t(N) * Ho * Wo;
          check(conv_fwd(p, stream_of(stream)), "conv_fwd");
        },
        py::arg("x"), py::arg("w"), py::arg("y"), py::arg("stats"), py::arg("N"), py::arg("H"), py::arg("W"),
        py::arg("Cin"), py::arg("Ho"), py::arg("Wo"), py::arg("Cout"), py::arg("stream"), py::arg("w_channels") = 0,
        py::arg("acc_r") = 0, py::arg("lut") = 0, py::arg("act") = py::none(), py::arg("act_out") = 0,
        py::arg("out_act") = py::none(), py::arg("out_y") = 0);
  m.def("conv1_bn_apply_fits", &conv1_bn_apply_fits);
  m.def("conv_out_bn_fits", &conv_out_bn_fits);
  m.def("conv_grid_barrier_timeouts", &conv_grid_barrier_timeouts);
  m.def("conv_grid_barrier_arm", &conv_grid_barrier_arm);
  m.def("conv_grid_barrier_failed", &conv_grid_barrier_failed);
  m.def("conv_grid_barrier_clear", &conv_grid_barrier_clear, pybind11::arg("value") = 0);
  // BatchNorm+LeakyReLU forward from conv_fwd's per-tile statistics: finalize + apply
  m.def("bn_forward_from_stats",
        [](uintptr_t x, uintptr_t y, int64_t M, int C, int dtype, uintptr_t stats, int nrows, float eps,
           float momentum, uintptr_t mean, uintptr_t invstd, uintptr_t rm, uintptr_t rv, uintptr_t w, uintptr_t b,
           float slope, uintptr_t stream, uintptr_t tracked) {
          hipStream_t s = stream_of(stream);
          check(bn_finalize_rows(ptr<const float>(stats), nrows, M, C, eps, momentum, ptr<float>(mean),
                                 ptr<float>(invstd), ptr<float>(rm), ptr<float>(rv), s, ptr<int64_t>(tracked)),
                "bn_finalize_rows");
          check(bn_apply(ptr<const void>(x), ptr<void>(y), M, C, dtype, ptr<const float>(mean),
                         ptr<const float>(invstd), ptr<const float>(w), ptr<const float>(b), slope, s),
                "bn_apply");
        });

  m.def("head_forward",
        [](uintptr_t z, uintptr_t w, int64_t ws_c, int64_t ws_i, int64_t ws_j, int N, int H, int W, int C, int OH,
           int OW, uintptr_t target, float target_value, uintptr_t pooled, uintptr_t partial, uintptr_t loss,
           uintptr_t dlogit, uintptr_t logit, uintptr_t stream, uintptr_t ticket, py::object act, uintptr_t bn_ab,
           uintptr_t bn_sums) {
          HeadParams p;
          p.act = act_from(act, "head_forward");
          p.bn_ab = ptr<double>(bn_ab);
          p.bn_sums = ptr<float>(bn_sums);
          p.ticket = ptr<uint32_t>(ticket);
          p.z = ptr<const uint16_t>(z);
          p.w = ptr<const float>(w);
          p.ws_c = ws_c, p.ws_i = ws_i, p.ws_j = ws_j;
          p.N = N, p.H = H, p.W = W, p.C = C, p.OH = OH, p.OW = OW;
          p.target = ptr<const float>(target);
          p.target_value = target_value;
          p.pooled = ptr<float>(pooled);
          p.partial = ptr<float>(partial);
          p.loss = ptr<float>(loss);
          p.dlogit = ptr<float>(dlogit);
          p.logit = ptr<float>(logit);
          check(head_forward(p, stream_of(stream)), "head_forward");
        },
        py::arg("z"), py::arg("w"), py::arg("ws_c"), py::arg("ws_i"), py::arg("ws_j"), py::arg("N"), py::arg("H"),
        py::arg("W"), py::arg("C"), py::arg("OH"), py::arg("OW"), py::arg("target"), py::arg("target_value"),
        py::arg("pooled"), py::arg("partial"), py::arg("loss"), py::arg("dlogit"), py::arg("logit"),
        py::arg("stream"), py::arg("ticket") = 0, py::arg("act") = py::none(), py::arg("bn_ab") = 0,
        py::arg("bn_sums") = 0);
  m.def("head_bn_bwd_supported", &head_bn_bwd_supported);
  m.def("head_backward",
        [](uintptr_t w, int64_t ws_c, int64_t ws_i, int64_t ws_j, int N, int H, int W, int C, int OH, int OW,
           uintptr_t pooled, uintptr_t dlogit, uintptr_t gscale, uintptr_t dz, uintptr_t dw, uintptr_t stream,
           uintptr_t bn_x, uintptr_t bn_mean, uintptr_t bn_invstd, uintptr_t bn_w, uintptr_t bn_b, float bn_slope,
           uintptr_t bn_acc, int bn_acc_r, uintptr_t bn_sums, uintptr_t bn_dw_out, uintptr_t bn_db_out) {
          HeadParams p;
          p.bn_sums = ptr<float>(bn_sums);
          p.bn_dw_out = ptr<float>(bn_dw_out);
          p.bn_db_out = ptr<float>(bn_db_out);
          p.bn_x = ptr<const uint16_t>(bn_x);
          p.bn_mean = ptr<const float>(bn_mean);
          p.bn_invstd = ptr<const float>(bn_invstd);
          p.bn_w = ptr<const float>(bn_w);
          p.bn_b = ptr<const float>(bn_b);
          p.bn_slope = bn_slope;
          p.bn_acc = ptr<double>(bn_acc);
          p.bn_acc_r = bn_acc_r;
          p.w = ptr<const float>(w);
          p.ws_c = ws_c, p.ws_i = ws_i, p.ws_j = ws_j;
          p.N = N, p.H = H, p.W = W, p.C = C, p.OH = OH, p.OW = OW;
          p.pooled = ptr<float>(pooled);
          p.dlogit = ptr<float>(dlogit);
          p.gscale = ptr<const float>(gscale);
          p.dz = ptr<uint16_t>(dz);
          p.dw = ptr<float>(dw);
          check(head_backward(p, stream_of(stream)), "head_backward");
        },
        py::arg("w"), py::arg("ws_c"), py::arg("ws_i"), py::arg("ws_j"), py::arg("N"), py::arg("H"), py::arg("W"),
        py::arg("C"), py::arg("OH"), py::arg("OW"), py::arg("pooled"), py::arg("dlogit"), py::arg("gscale"),
        py::arg("dz"), py::arg("dw"), py::arg("stream"), py::arg("bn_x") = 0, py::arg("bn_mean") = 0,
        py::arg("bn_invstd") = 0, py::arg("bn_w") = 0, py::arg("bn_b") = 0, py::arg("bn_slope") = 0.f,
        py::arg("bn_acc") = 0, py::arg("bn_acc_r") = 0, py::arg("bn_sums") = 0, py::arg("bn_dw_out") = 0,
        py::arg("bn_db_out") = 0);

  // direct RCCL on the caller's stream (comm.h); the GIL is released while
  // RCCL enqueues (a group end may block until peers have posted theirs)
  m.def("rccl_load", [](const std::string& path) { comm::load(path); });
  m.def("rccl_loaded", [] { return comm::loaded(); });
  m.def("rccl_count", [](uintptr_t c) { return comm::comm_count(c); });
  m.def("rccl_rank", [](uintptr_t c) { return comm::comm_rank(c); });
  m.def("rccl_async_error", [](uintptr_t c) { return comm::async_error(c); });
  m.def(
      "rccl_all_reduce",
      [](uintptr_t send, uintptr_t recv, size_t count, int dtype, int op, uintptr_t c, uintptr_t stream) {
        comm::all_reduce(ptr<const void>(send), ptr<void>(recv), count, dtype, op, c, stream_of(stream));
      },
      py::call_guard<py::gil_scoped_release>());
  m.def(
      "rccl_broadcast",
      [](uintptr_t send, uintptr_t recv, size_t count, int dtype, int root, uintptr_t c, uintptr_t stream) {
        comm::broadcast(ptr<const void>(send), ptr<void>(recv), count, dtype, root, c, stream_of(stream));
      },
      py::call_guard<py::gil_scoped_release>());
  // one group of point-to-point transfers: ops = [(is_send, ptr, count, dtype, peer)]
  m.def(
      "rccl_p2p",
      [](std::vector<std::tuple<int, uintptr_t, size_t, int, int>> ops, uintptr_t c, uintptr_t stream) {
        comm::group_start();
        try {
          for (auto& [is_send, p, count, dtype, peer] : ops) {
            if (is_send) comm::send(ptr<const void>(p), count, dtype, peer, c, stream_of(stream));
            else comm::recv(ptr<void>(p), count, dtype, peer, c, stream_of(stream));
          }
        } catch (...) {
          try {
            comm::group_end();
          } catch (...) {
          }
          throw;
        }
        comm::group_end();
      },
      py::call_guard<py::gil_scoped_release>());

  m.def("adam_schedule",
        [](uintptr_t step, uintptr_t hp, uintptr_t sched, float beta1, float beta2, uintptr_t stream,
           uintptr_t gate) {
          check(adam_schedule(ptr<float>(step), ptr<const float>(hp), ptr<float>(sched), beta1, beta2,
                              stream_of(stream), ptr<const float>(gate)),
                "adam_schedule");
        },
        py::arg("step"), py::arg("hp"), py::arg("sched"), py::arg("beta1"), py::arg("beta2"), py::arg("stream"),
        py::arg("gate") = 0);

  m.def("adam_schedule_prime",
        [](uintptr_t step, uintptr_t hp, uintptr_t sched, float beta1, float beta2, uintptr_t stream, float off) {
          check(adam_schedule_prime(ptr<const float>(step), ptr<const float>(hp), ptr<float>(sched), beta1, beta2,
                                    stream_of(stream), off),
                "adam_schedule_prime");
        },
        py::arg("step"), py::arg("hp"), py::arg("sched"), py::arg("beta1"), py::arg("beta2"), py::arg("stream"),
        py::arg("off") = 1.0f);
  // the Adam schedule attached to the next weight-gradient slice-reduce launch (adam_sched.h)
  m.def("adam_attach_schedule",
        [](uintptr_t step, uintptr_t hp, uintptr_t sched, float beta1, float beta2, int device, uintptr_t stream) {
          AdamSchedJob j;
          j.step = ptr<float>(step), j.hp = ptr<const float>(hp), j.sched = ptr<float>(sched);
          j.beta1 = beta1, j.beta2 = beta2;
          conv_attach_adam_schedule(j, device, stream_of(stream));
        },
        py::arg("step"), py::arg("hp"), py::arg("sched"), py::arg("beta1"), py::arg("beta2"), py::arg("device"),
        py::arg("stream"));
  m.def("adam_schedule_taken", []() { return conv_adam_schedule_taken(); });
  m.def("adam_detach_schedule", []() { conv_detach_adam_schedule(); });

  m.def("adam_update",
        [](std::vector<uintptr_t> params, std::vector<uintptr_t> grads, std::vector<uintptr_t> exp_avg,
           std::vector<uintptr_t> exp_avg_sq, std::vector<uintptr_t> shadow, std::vector<int64_t> numel,
           uintptr_t sched, int grad_bf16, float beta1, float beta2, float eps, float weight_decay, int decoupled,
           int maximize, uintptr_t stream, uintptr_t step, uintptr_t hp, uintptr_t gate, uintptr_t ticket,
           int zero_grad, std::vector<uintptr_t> shadow_t, std::vector<int> tcout, std::vector<int> tcin,
           std::vector<uintptr_t> grads2, py::object fused_reduce, std::vector<uintptr_t> fr_tensors) {
          const size_t n = params.size();
          if (grads.size() != n || exp_avg.size() != n || exp_avg_sq.size() != n || shadow.size() != n ||
              numel.size() != n || n > size_t(kMaxAdam))
            throw std::invalid_argument("adam_update: list lengths differ or exceed kMaxAdam");
          if (!shadow_t.empty() && (shadow_t.size() != n || tcout.size() != n || tcin.size() != n))
            throw std::invalid_argument("adam_update: shadow_t / tcout / tcin must match params");
          AdamParams a;
          a.n = int(n);
          for (size_t k = 0; k < n; ++k) {
            a.p[k] = ptr<float>(params[k]);
            a.g[k] = ptr<const void>(grads[k]);
            a.m[k] = ptr<float>(exp_avg[k]);
            a.v[k] = ptr<float>(exp_avg_sq[k]);
            a.shadow[k] = ptr<uint16_t>(shadow[k]);
            a.numel[k] = numel[k];
            // every tensor starts on a 256-group block boundary (transposed
            // shadows are walked a block per tile; the padding groups are no-ops)
            a.gstart[k + 1] = (a.gstart[k] + (numel[k] + 3) / 4 + 255) / 256 * 256;
          }
          if (!grads2.empty()) {
            if (grads2.size() != n || grad_bf16) throw std::invalid_argument("adam_update: grads2 (fp32) must match params");
            for (size_t k = 0; k < n; ++k) a.g2[k] = ptr<const float>(grads2[k]);
          }
          for (size_t k = 0; k < shadow_t.size(); ++k) {
            a.shadow_t[k] = ptr<uint16_t>(shadow_t[k]);
            a.tcout[k] = tcout[k];
            a.tcin[k] = tcin[k];
          }
          a.sched = ptr<const float>(sched);
          a.step = ptr<float>(step);
          a.hp = ptr<const float>(hp);
          a.gate = ptr<const float>(gate);
          a.ticket = ptr<uint32_t>(ticket);
          a.zero_grad = zero_grad;
          a.grad_bf16 = grad_bf16, a.decoupled = decoupled, a.maximize = maximize;
          a.beta1 = beta1, a.beta2 = beta2, a.eps = eps, a.weight_decay = weight_decay;
          if (!fused_reduce.is_none()) {   // a deferred slice reduce (conv_wgrad defer=1) + (g, p, m, v, shadow)
            const ConvWgradParams::Reduce r = reduce_from_tuple(fused_reduce.cast<py::tuple>());
            if (fr_tensors.size() != 5 || r.ry != 1 || r.sub <= 0)
              throw std::invalid_argument("adam_update: fused_reduce needs an ordered reduce and 5 tensors");
            AdamParams::FusedReduce& f = a.fr;
            f.partial = r.partial, f.S = r.S, f.Cout = r.Cout, f.Cin = r.Cin, f.cin_out = r.cin_out;
            f.sub = r.sub, f.rx = r.rx;
            f.s_co = r.s_co, f.s_ci = r.s_ci, f.s_kh = r.s_kh, f.s_kw = r.s_kw;
            f.g = ptr<float>(fr_tensors[0]), f.p = ptr<float>(fr_tensors[1]), f.m = ptr<float>(fr_tensors[2]);
            f.v = ptr<float>(fr_tensors[3]), f.shadow = ptr<uint16_t>(fr_tensors[4]);
          }
          check(adam_update(a, stream_of(stream)), "adam_update");
        },
        py::arg("params"), py::arg("grads"), py::arg("exp_avg"), py::arg("exp_avg_sq"), py::arg("shadow"),
        py::arg("numel"), py::arg("sched"), py::arg("grad_bf16"), py::arg("beta1"), py::arg("beta2"), py::arg("eps"),
        py::arg("weight_decay"), py::arg("decoupled"), py::arg("maximize"), py::arg("stream"), py::arg("step") = 0,
        py::arg("hp") = 0, py::arg("gate") = 0, py::arg("ticket") = 0, py::arg("zero_grad") = 0,
        py::arg("shadow_t") = std::vector<uintptr_t>(), py::arg("tcout") = std::vector<int>(),
        py::arg("tcin") = std::vector<int>(), py::arg("grads2") = std::vector<uintptr_t>(),
        py::arg("fused_reduce") = py::none(), py::arg("fr_tensors") = std::vector<uintptr_t>());

  m.def("color4x4",
        [](uintptr_t src, uintptr_t dst, uintptr_t lut, uintptr_t M, uintptr_t bias, uintptr_t flip, int B, int H,
           int W, int Cout, int flip_all, uintptr_t stream, int mat_mode, uintptr_t Ms, std::vector<float> jitter,
           float pivot) {
          Color4x4Params p;
          p.src = ptr<const uint8_t>(src);
          p.dst = ptr<float>(dst);
          p.lut = ptr<const float>(lut);
          p.M = ptr<const float>(M);
          p.bias = ptr<const float>(bias);
          p.flip = ptr<const uint8_t>(flip);
          p.B = B, p.H = H, p.W = W, p.Cout = Cout;
          p.flip_all = flip_all;
          p.mat_mode = mat_mode;
          p.Ms = ptr<const float>(Ms);
          p.pivot = pivot;
          if (mat_mode == kColorJitter) {
            if (B > kMaxSrcs || jitter.size() != size_t(4) * size_t(B))
              throw std::invalid_argument("color4x4: jitter needs 4 factors per image, B <= 64");
            for (int b = 0; b < B; ++b)
              for (int k = 0; k < 4; ++k) p.jit[b][k] = jitter[size_t(b) * 4 + size_t(k)];
          }
          check(color4x4(p, stream_of(stream)), "color4x4");
        },
        py::arg("src"), py::arg("dst"), py::arg("lut"), py::arg("M"), py::arg("bias"), py::arg("flip"), py::arg("B"),
        py::arg("H"), py::arg("W"), py::arg("Cout"), py::arg("flip_all"), py::arg("stream"), py::arg("mat_mode") = 0,
        py::arg("Ms") = 0, py::arg("jitter") = std::vector<float>(), py::arg("pivot") = 0.5f);

  m.def("project",
        [](uintptr_t pts, int64_t N, uintptr_t PV, uintptr_t V, int W, int H, int upper_left, uintptr_t out_px,
           uintptr_t out_depth, uintptr_t stream) {
          check(project(ptr<const float>(pts), N, ptr<const float>(PV), ptr<const float>(V), W, H, upper_left,
                        ptr<float>(out_px), ptr<float>(out_depth), stream_of(stream)),
                "project");
        });

  m.def("adaptive_avgpool_nhwc",
        [](uintptr_t x, uintptr_t y, int N, int H, int W, int C, int OH, int OW, int dtype, uintptr_t stream) {
          check(adaptive_avgpool_nhwc(ptr<const void>(x), ptr<void>(y), N, H, W, C, OH, OW, dtype, stream_of(stream)),
                "adaptive_avgpool_nhwc");
        });
  m.def("adaptive_avgpool_nhwc_bwd",
        [](uintptr_t gy, uintptr_t gx, int N, int H, int W, int C, int OH, int OW, int dtype, uintptr_t stream) {
          check(adaptive_avgpool_nhwc_bwd(ptr<const void>(gy), ptr<void>(gx), N, H, W, C, OH, OW, dtype,
                                          stream_of(stream)),
                "adaptive_avgpool_nhwc_bwd");
        });

  // fused training BatchNorm2d + LeakyReLU (channels-last); pointers are device addresses
  m.def("bn_partial_floats", [](int64_t M, int C, int dtype) { return bn_partial_floats(M, C, dtype); });
  m.def("bn_forward",
        [](uintptr_t x, uintptr_t y, int64_t M, int C, int dtype, uintptr_t partial, float eps, float momentum,
           uintptr_t mean, uintptr_t invstd, uintptr_t rm, uintptr_t rv, uintptr_t w, uintptr_t b, float slope,
           uintptr_t stream, uintptr_t tracked) {
          hipStream_t s = stream_of(stream);
          check(bn_stats(ptr<const void>(x), M, C, dtype, ptr<float>(partial), s), "bn_stats");
          check(bn_finalize(ptr<const float>(partial), M, C, dtype, eps, momentum, ptr<float>(mean), ptr<float>(invstd),
                            ptr<float>(rm), ptr<float>(rv), s, ptr<int64_t>(tracked)),
                "bn_finalize");
          check(bn_apply(ptr<const void>(x), ptr<void>(y), M, C, dtype, ptr<const float>(mean),
                         ptr<const float>(invstd), ptr<const float>(w), ptr<const float>(b), slope, s),
                "bn_apply");
        },
        py::arg("x"), py::arg("y"), py::arg("M"), py::arg("C"), py::arg("dtype"), py::arg("partial"), py::arg("eps"),
        py::arg("momentum"), py::arg("mean"), py::arg("invstd"), py::arg("rm"), py::arg("rv"), py::arg("w"),
        py::arg("b"), py::arg("slope"), py::arg("stream"), py::arg("tracked") = 0);
  m.def("bn_backward",
        [](uintptr_t x, uintptr_t gy, uintptr_t gx, int64_t M, int C, int dtype, uintptr_t partial, uintptr_t mean,
           uintptr_t invstd, uintptr_t w, uintptr_t b, uintptr_t dw, uintptr_t db, float slope, uintptr_t stream) {
          hipStream_t s = stream_of(stream);
          check(bn_bwd_reduce(ptr<const void>(x), ptr<const void>(gy), M, C, dtype, ptr<const float>(mean),
                              ptr<const float>(invstd), ptr<const float>(w), ptr<const float>(b), slope,
                              ptr<float>(partial), s),
                "bn_bwd_reduce");
          check(bn_bwd_finalize(ptr<const float>(partial), M, C, dtype, ptr<float>(dw), ptr<float>(db), s),
                "bn_bwd_finalize");
          check(bn_bwd_apply(ptr<const void>(x), ptr<const void>(gy), ptr<void>(gx), M, C, dtype,
                             ptr<const float>(mean), ptr<const float>(invstd), ptr<const float>(w),
                             ptr<const float>(b), ptr<const float>(dw), ptr<const float>(db), slope, s),
                "bn_bwd_apply");
        });

  // the BN backward's apply pass alone (dw, db folded elsewhere: conv_wgrad fold=)
  m.def("bn_bwd_apply",
        [](uintptr_t x, uintptr_t gy, uintptr_t gx, int64_t M, int C, int dtype, uintptr_t mean, uintptr_t invstd,
           uintptr_t w, uintptr_t b, uintptr_t dw, uintptr_t db, float slope, uintptr_t stream) {
          check(bn_bwd_apply(ptr<const void>(x), ptr<const void>(gy), ptr<void>(gx), M, C, dtype,
                             ptr<const float>(mean), ptr<const float>(invstd), ptr<const float>(w),
                             ptr<const float>(b), ptr<const float>(dw), ptr<const float>(db), slope,
                             stream_of(stream)),
                "bn_bwd_apply");
        });
  // the BN forward's apply pass alone (mean, invstd given)
  m.def("bn_fwd_apply",
        [](uintptr_t x, uintptr_t y, int64_t M, int C, int dtype, uintptr_t mean, uintptr_t invstd, uintptr_t w,
           uintptr_t b, float slope, uintptr_t stream) {
          check(bn_apply(ptr<const void>(x), ptr<void>(y), M, C, dtype, ptr<const float>(mean),
                         ptr<const float>(invstd), ptr<const float>(w), ptr<const float>(b), slope, stream_of(stream)),
                "bn_apply");
        });
  // accumulator hand-off (kernels.h BnAcc): no finalize launches
  m.def("bn_acc_replicas", &bn_acc_replicas);
  m.def("bn_acc_elems", &bn_acc_elems);
  m.def("bn_forward_acc",
        [](uintptr_t x, uintptr_t y, int64_t M, int C, int dtype, uintptr_t acc, int R, float eps, float momentum,
           uintptr_t mean, uintptr_t invstd, uintptr_t rm, uintptr_t rv, uintptr_t w, uintptr_t b, float slope,
           uintptr_t stream, uintptr_t tracked) {
          BnAcc a;
          a.acc = ptr<double>(acc), a.R = R;
          check(bn_apply_acc(ptr<const void>(x), ptr<void>(y), M, C, dtype, a, eps, momentum, ptr<float>(mean),
                             ptr<float>(invstd), ptr<float>(rm), ptr<float>(rv), ptr<int64_t>(tracked),
                             ptr<const float>(w), ptr<const float>(b), slope, stream_of(stream)),
                "bn_apply_acc");
        });
  m.def("bn_backward_acc",
        [](uintptr_t x, uintptr_t gy, uintptr_t gx, int64_t M, int C, int dtype, uintptr_t acc, int R, uintptr_t mean,
           uintptr_t invstd, uintptr_t w, uintptr_t b, uintptr_t dw, uintptr_t db, float slope, uintptr_t stream,
           bool reduce) {
          // reduce: sum gz, gz * xhat here first (no producer epilogue did)
          BnAcc a;
          a.acc = ptr<double>(acc), a.R = R;
          hipStream_t s = stream_of(stream);
          if (reduce)
            check(bn_bwd_reduce_acc(ptr<const void>(x), ptr<const void>(gy), M, C, dtype, ptr<const float>(mean),
                                    ptr<const float>(invstd), ptr<const float>(w), ptr<const float>(b), slope, a, s),
                  "bn_bwd_reduce_acc");
          check(bn_bwd_apply_acc(ptr<const void>(x), ptr<const void>(gy), ptr<void>(gx), M, C, dtype, a,
                                 ptr<const float>(mean), ptr<const float>(invstd), ptr<const float>(w),
                                 ptr<const float>(b), ptr<float>(dw), ptr<float>(db), slope, s),
                "bn_bwd_apply_acc");
        });

  // Diagnostics: H2D bandwidth of one `nbytes` copy repeated `iters` times
  // from host memory of the given kind ("hostmalloc", "register", "pageable").
  m.def("bench_h2d", [](const std::string& kind, size_t nbytes, int iters, int chunks) {
    py::gil_scoped_release nogil;
    void* host = nullptr;
    bool reg = false;
    if (kind == "hostmalloc") {
      check(hipHostMalloc(&host, nbytes * chunks, hipHostMallocDefault), "hipHostMalloc");
    } else {
      host = mmap(nullptr, nbytes * chunks, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
      std::memset(host, 1, nbytes * chunks);
      if (kind == "register") {
        check(hipHostRegister(host, nbytes * chunks, hipHostRegisterDefault), "hipHostRegister");
        reg = true;
      }
    }
    void* dev = nullptr;
    check(hipMalloc(&dev, nbytes * chunks), "hipMalloc");
    hipStream_t s;
    check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "stream");
    auto run = [&] {
      for (int c = 0; c < chunks; ++c)
        check(hipMemcpyAsync(static_cast<char*>(dev) + c * nbytes, static_cast<char*>(host) + c * nbytes, nbytes,
                             hipMemcpyHostToDevice, s), "memcpy");
    };
    run();
    check(hipStreamSynchronize(s), "sync");
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i) run();
    check(hipStreamSynchronize(s), "sync");
    double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    (void)hipStreamDestroy(s);
    (void)hipFree(dev);
    if (kind == "hostmalloc") (void)hipHostFree(host);
    else {
      if (reg) (void)hipHostUnregister(host);
      munmap(host, nbytes * chunks);
    }
    return double(nbytes) * chunks * iters / sec / 1e9;   // GB/s
  });

  // Host-resident frames -> decoded batch, two ways (returns us per batch):
  //   mode "copy":   B hipMemcpyAsync into a device staging buffer + decode
  //                  (the DMA-engine path);
  //   mode "direct": decode reads the B host frames itself over PCIe
  //                  (zero-copy fused read; srcs[] = host pointers).
  // `kind` picks the host memory: "hostmalloc" (hipHostMalloc) or
  // "register" (mmap + hipHostRegister, like the producers' shm ring).
  // Each iteration rewrites one byte per frame on the host first, and the
  // result of the last iteration is checked, so a stale GPU-cached read of
  // host memory would show up as a mismatch (returned as `stale`).
  m.def("bench_frames_to_device",
        [](const std::string& mode, const std::string& kind, int B, int H, int W, int Cin, int iters, int max_grid,
           int copy_streams, bool pipelined) {
          py::gil_scoped_release nogil;
          const size_t img = size_t(H) * W * Cin;
          const size_t slot = (img + 4095) & ~size_t(4095);
          uint8_t* host = nullptr;
          if (kind == "hostmalloc") {
            check(hipHostMalloc(reinterpret_cast<void**>(&host), slot * B, hipHostMallocDefault), "hipHostMalloc");
          } else {
            // "register": shared mapping (like the producers' shm ring, 4 KiB pages);
            // "register_thp": private anonymous mapping with MADV_HUGEPAGE (2 MiB pages)
            const bool thp = kind == "register_thp";
            host = static_cast<uint8_t*>(mmap(nullptr, slot * B, PROT_READ | PROT_WRITE,
                                              (thp ? MAP_PRIVATE : MAP_SHARED) | MAP_ANONYMOUS, -1, 0));
            if (thp) (void)madvise(host, slot * B, MADV_HUGEPAGE);
            std::memset(host, 0, slot * B);   // fault the pages in (huge where possible)
            check(hipHostRegister(host, slot * B, hipHostRegisterMapped), "hipHostRegister");
          }
          for (size_t i = 0; i < slot * size_t(B); ++i) host[i] = uint8_t(i * 7);
          uint8_t* dev_host = nullptr;
          check(hipHostGetDevicePointer(reinterpret_cast<void**>(&dev_host), host, 0), "hipHostGetDevicePointer");
          uint8_t* stage = nullptr;
          float *dst = nullptr, *lut = nullptr;
          check(hipMalloc(reinterpret_cast<void**>(&stage), img * B), "hipMalloc");
          check(hipMalloc(reinterpret_cast<void**>(&dst), size_t(B) * 3 * H * W * sizeof(float)), "hipMalloc");
          std::vector<float> hl(kTableFloats, 0.f);   // identity table, mode 0 header
          for (int i = 0; i < 4 * 256; ++i) hl[size_t(i)] = float(i & 255);
          check(hipMalloc(reinterpret_cast<void**>(&lut), hl.size() * sizeof(float)), "hipMalloc");
          check(hipMemcpy(lut, hl.data(), hl.size() * sizeof(float), hipMemcpyHostToDevice), "lut");
          hipStream_t s;
          check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "stream");
          // copy mode over K streams: frame b on stream b % K (each its own
          // hardware queue, so several SDMA engines pull concurrently); the
          // decode stream joins them with one event per stream
          const int K = copy_streams < 1 ? 1 : (copy_streams > 4 ? 4 : copy_streams);
          std::vector<hipStream_t> cs(size_t(K), nullptr);
          std::vector<hipEvent_t> ce(size_t(K), nullptr);
          for (int k = 1; k < K; ++k) {
            check(hipStreamCreateWithFlags(&cs[size_t(k)], hipStreamNonBlocking), "stream");
            check(hipEventCreateWithFlags(&ce[size_t(k)], hipEventDisableTiming), "event");
          }
          cs[0] = s;
          hipEvent_t kdone;
          check(hipEventCreateWithFlags(&kdone, hipEventDisableTiming), "event");
          // pipelined: two staging buffers, no host sync between batches (the
          // copies of batch i+1 overlap the decode of batch i)
          uint8_t* stage2 = nullptr;
          if (pipelined) check(hipMalloc(reinterpret_cast<void**>(&stage2), img * B), "hipMalloc");
          DecodeParams p;
          p.dst = dst;
          p.lut = lut;
          p.B = B, p.H = H, p.W = W, p.Cin = Cin, p.Cout = 3;
          p.max_grid = max_grid;
          // "hybrid:<n>": the first n frames of a batch are read over PCIe by the
          // decode kernel itself, the rest are DMA'd to staging first (both
          // paths pulling over the link at once)
          const bool hybrid = mode.rfind("hybrid:", 0) == 0;
          const int ndirect = hybrid ? std::max(0, std::min(B, std::stoi(mode.substr(7)))) : 0;
          const bool direct = mode == "direct";
          if (hybrid) {
            p.nsrcs = B;
          } else if (direct) {
            p.nsrcs = B;
            for (int b = 0; b < B; ++b) p.srcs[b] = dev_host + size_t(b) * slot;
          } else {
            p.src = stage;
          }
          auto run = [&](int it, bool rewrite) {
            if (rewrite)
              for (int b = 0; b < B; ++b) host[size_t(b) * slot] = uint8_t(it);   // fresh content per batch
            uint8_t* st = (pipelined && (it & 1)) ? stage2 : stage;
            if (hybrid)
              for (int b = 0; b < B; ++b) p.srcs[b] = b < ndirect ? dev_host + size_t(b) * slot : st + size_t(b) * img;
            if (!direct) {
              p.src = st;
              for (int k = 1; k < K; ++k) check(hipStreamWaitEvent(cs[size_t(k)], kdone, 0), "wait");   // staging free
              for (int b = ndirect; b < B; ++b)
                check(hipMemcpyAsync(st + size_t(b) * img, host + size_t(b) * slot, img, hipMemcpyHostToDevice,
                                     cs[size_t(b % K)]),
                      "memcpy");
              for (int k = 1; k < K; ++k) {
                check(hipEventRecord(ce[size_t(k)], cs[size_t(k)]), "record");
                check(hipStreamWaitEvent(s, ce[size_t(k)], 0), "wait");
              }
            }
            check(decode(p, s), "decode");
            check(hipEventRecord(kdone, s), "record");
          };
          for (int i = 0; i < 5; ++i) {
            run(i, true);
            check(hipStreamSynchronize(s), "sync");
          }
          auto t0 = std::chrono::steady_clock::now();
          for (int i = 0; i < iters; ++i) {
            if (!pipelined) check(hipStreamSynchronize(s), "sync");   // host rewrites only after the last read
            const bool last = i == iters - 1;
            if (pipelined && last) check(hipStreamSynchronize(s), "sync");
            run(100 + i, !pipelined || last);
          }
          check(hipStreamSynchronize(s), "sync");
          double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
          // check pixel 0 (channel 0) of every image of the last batch
          int stale = 0;
          for (int b = 0; b < B; ++b) {
            float v = 0;
            check(hipMemcpy(&v, dst + size_t(b) * 3 * H * W, sizeof(float), hipMemcpyDeviceToHost), "d2h");
            if (v != float(uint8_t(100 + iters - 1))) ++stale;
          }
          for (int k = 1; k < K; ++k) {
            (void)hipStreamDestroy(cs[size_t(k)]);
            (void)hipEventDestroy(ce[size_t(k)]);
          }
          (void)hipEventDestroy(kdone);
          if (stage2) (void)hipFree(stage2);
          (void)hipStreamDestroy(s);
          (void)hipFree(stage);
          (void)hipFree(dst);
          (void)hipFree(lut);
          if (kind == "hostmalloc") (void)hipHostFree(host);
          else {
            (void)hipHostUnregister(host);
            munmap(host, slot * B);
          }
          // us/batch, GB/s of frame bytes, stale (std::tuple: converted after the GIL is re-taken)
          return std::make_tuple(us, double(img) * B / us / 1e3, stale);
        },
        py::arg("mode"), py::arg("kind"), py::arg("B"), py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("iters"),
        py::arg("max_grid") = 0, py::arg("copy_streams") = 1, py::arg("pipelined") = false);

  // Kernel-only timing (no Python launch overhead): `iters` back-to-back
  // decode launches between two HIP events; returns microseconds per launch.
  m.def("bench_decode",
        [](uintptr_t src, uintptr_t dst, uintptr_t lut, int B, int H, int W, int Cin, int Cout, std::vector<int> cmap,
           int out_dtype, int layout, int iters) {
          py::gil_scoped_release nogil;
          DecodeParams p;
          p.src = ptr<const uint8_t>(src);
          p.dst = ptr<void>(dst);
          p.lut = ptr<const float>(lut);
          p.B = B, p.H = H, p.W = W, p.Cin = Cin, p.Cout = Cout;
          fill_cmap(p.cmap, cmap);
          p.out_dtype = out_dtype;
          p.layout = layout;
          hipStream_t s;
          check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "stream");
          hipEvent_t a, b;
          check(hipEventCreate(&a), "event");
          check(hipEventCreate(&b), "event");
          for (int i = 0; i < 10; ++i) check(decode(p, s), "decode");
          check(hipEventRecord(a, s), "record");
          for (int i = 0; i < iters; ++i) check(decode(p, s), "decode");
          check(hipEventRecord(b, s), "record");
          check(hipEventSynchronize(b), "sync");
          float ms = 0;
          check(hipEventElapsedTime(&ms, a, b), "elapsed");
          (void)hipEventDestroy(a);
          (void)hipEventDestroy(b);
          (void)hipStreamDestroy(s);
          return double(ms) * 1000.0 / iters;
        });

  // Kernel-only timing of the MFMA colour transform (see bench_decode).
  m.def("bench_color4x4",
        [](uintptr_t src, uintptr_t dst, uintptr_t lut, uintptr_t M, uintptr_t bias, int B, int H, int W, int Cout,
           int iters) {
          py::gil_scoped_release nogil;
          Color4x4Params p;
          p.src = ptr<const uint8_t>(src);
          p.dst = ptr<float>(dst);
          p.lut = ptr<const float>(lut);
          p.M = ptr<const float>(M);
          p.bias = ptr<const float>(bias);
          p.B = B, p.H = H, p.W = W, p.Cout = Cout;
          hipStream_t s;
          check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "stream");
          hipEvent_t a, b;
          check(hipEventCreate(&a), "event");
          check(hipEventCreate(&b), "event");
          for (int i = 0; i < 10; ++i) check(color4x4(p, s), "color4x4");
          check(hipEventRecord(a, s), "record");
          for (int i = 0; i < iters; ++i) check(color4x4(p, s), "color4x4");
          check(hipEventRecord(b, s), "record");
          check(hipEventSynchronize(b), "sync");
          float ms = 0;
          check(hipEventElapsedTime(&ms, a, b), "elapsed");
          (void)hipEventDestroy(a);
          (void)hipEventDestroy(b);
          (void)hipStreamDestroy(s);
          return double(ms) * 1000.0 / iters;
        });

  py::class_<StreamLoader>(m, "StreamLoader")
      .def(py::init([](std::vector<std::string> addresses, int batch_size, std::string image_key, int rcvhwm,
                       int io_threads, int device, int64_t max_batches, size_t max_frame_bytes, int pool_slots,
                       int staging_depth, bool skip_bad, int cout, std::vector<int> cmap, int flip_all,
                       int out_dtype, int layout, std::vector<float> lut, std::vector<float> matrix,
                       std::vector<float> bias, bool direct, int launch_depth, int copy_streams, bool host_sync,
                       std::vector<float> matrices, std::vector<float> jitter, uint64_t jitter_seed) {
             LoaderConfig c;
             c.direct = direct;
             c.host_sync = host_sync;
             c.copy_streams = copy_streams;
             c.launch_depth = launch_depth;
             c.addresses = std::move(addresses);
             c.batch_size = batch_size;
             c.image_key = std::move(image_key);
             c.rcvhwm = rcvhwm;
             c.io_threads = io_threads;
             c.device = device;
             c.max_batches = max_batches;
             c.max_frame_bytes = max_frame_bytes;
             c.pool_slots = pool_slots;
             c.staging_depth = staging_depth;
             c.skip_bad = skip_bad;
             c.cout = cout;
             fill_cmap(c.cmap, cmap);
             c.flip_all = flip_all;
             c.out_dtype = out_dtype;
             c.layout = layout;
             c.lut = std::move(lut);
             c.color_matrix = !matrix.empty();
             c.matrix = std::move(matrix);
             c.bias = std::move(bias);
             // per-batch-position matrices (B x (16 + 4)) or random colour jitter
             // (4 ranges + pivot), both on the MFMA colour kernel
             if (!matrices.empty() || !jitter.empty()) c.color_matrix = true;
             c.matrices = std::move(matrices);
             if (!jitter.empty()) {
               if (jitter.size() != 5) throw std::invalid_argument("StreamLoader: jitter = 4 ranges + pivot");
               c.jitter = true;
               for (int k = 0; k < 4; ++k) c.jitter_range[k] = jitter[size_t(k)];
               c.pivot = jitter[4];
               c.jitter_seed = jitter_seed;
             }
             return new StreamLoader(c);
           }),
           py::arg("addresses"), py::arg("batch_size"), py::arg("image_key"), py::arg("rcvhwm"),
           py::arg("io_threads"), py::arg("device"), py::arg("max_batches"), py::arg("max_frame_bytes"),
           py::arg("pool_slots"), py::arg("staging_depth"), py::arg("skip_bad"), py::arg("cout"), py::arg("cmap"),
           py::arg("flip_all"), py::arg("out_dtype"), py::arg("layout"), py::arg("lut"), py::arg("matrix"),
           py::arg("bias"), py::arg("direct") = true, py::arg("launch_depth") = 2,
           py::arg("copy_streams") = 2, py::arg("host_sync") = true, py::arg("matrices") = std::vector<float>(),
           py::arg("jitter") = std::vector<float>(), py::arg("jitter_seed") = 0)
      .def("start", &StreamLoader::start)
      .def("wait_shape",
           [](StreamLoader& l, long timeout_ms) -> py::object {
             int H = 0, W = 0, C = 0;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = l.wait_shape(timeout_ms, &H, &W, &C);
             }
             if (!ok) return py::none();
             return py::make_tuple(H, W, C);
           })
      .def("post",
           [](StreamLoader& l, uintptr_t dst, uintptr_t stream) {
             py::gil_scoped_release nogil;
             l.post(ptr<void>(dst), stream_of(stream));
           })
      .def("next",
           [](StreamLoader& l, uintptr_t stream, long timeout_ms) -> py::object {
             ReadyBatch rb;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = l.next(&rb, stream_of(stream), timeout_ms);
             }
             if (!ok) return py::none();                 // timeout
             if (rb.index < 0) return py::make_tuple(-1, py::list(), 0.0);   // exhausted
             py::list metas;
             for (auto& it : rb.items) {
               py::bytearray owner(reinterpret_cast<const char*>(it.bytes.data()), it.bytes.size());
               const uint8_t* base = reinterpret_cast<const uint8_t*>(PyByteArray_AsString(owner.ptr()));
               metas.append(pyconv::value_to_py(*it.tree, base, owner));
             }
             return py::make_tuple(rb.index, metas, rb.recv_ms);
           })
      .def("next_collated",
           [](StreamLoader& l, uintptr_t stream, long timeout_ms) -> py::object {
             ReadyBatch rb;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = l.next(&rb, stream_of(stream), timeout_ms);
             }
             if (!ok) return py::none();
             if (rb.index < 0) return py::make_tuple(-1, py::dict(), 0.0);
             py::dict meta = collate_meta(rb.items);
             if (!rb.jitter.empty()) {   // the colour-jitter factors each image was decoded with
               py::array_t<float> f({py::ssize_t(rb.jitter.size() / 4), py::ssize_t(4)});
               std::memcpy(f.mutable_data(), rb.jitter.data(), rb.jitter.size() * sizeof(float));
               meta["color_jitter"] = f;
             }
             return py::make_tuple(rb.index, meta, rb.recv_ms);
           })
      .def("stop",
           [](StreamLoader& l) {
             py::gil_scoped_release nogil;
             l.stop();
           })
      .def("stats", [](StreamLoader& l) {
        auto s = l.stats();
        py::dict d;
        d["frames"] = s.frames;
        d["batches"] = s.batches;
        d["bytes"] = s.bytes;
        d["bad"] = s.bad;
        d["pool_fallbacks"] = s.pool_fallbacks;
        d["h2d_issue_ms"] = s.h2d_issue_ms;
        d["shm_frames"] = s.shm_frames;
        d["shm_torn"] = s.shm_torn;
        d["shm_stale"] = s.shm_stale;
        d["direct_batches"] = s.direct_batches;
        d["launches"] = s.launches;
        d["image_bytes"] = s.image_bytes;
        d["tiled_frames"] = s.tiled_frames;
        d["timed_launches"] = s.timed_launches;
        d["timed_images"] = s.timed_images;
        d["timed_gpu_ms"] = s.timed_gpu_ms;
        d["keys_evicted"] = s.keys_evicted;
        d["passthrough_batches"] = s.passthrough_batches;
        d["staged_frames"] = s.staged_frames;
        d["ring_slots"] = s.ring_slots;
        d["ring_published"] = s.ring_published;
        d["ring_held"] = s.ring_held;
        d["cpu_poll_ms"] = s.cpu_poll_ms;
        d["cpu_recv_ms"] = s.cpu_recv_ms;
        d["cpu_launch_ms"] = s.cpu_launch_ms;
        d["cpu_reap_ms"] = s.cpu_reap_ms;
        d["worker_tid"] = s.worker_tid;
        py::dict per;
        for (const auto& kv : s.frames_per_btid) per[py::int_(kv.first)] = kv.second;
        d["frames_per_btid"] = per;
        return d;
      });
}
