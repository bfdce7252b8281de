// Conversion of a parsed pickle value tree (codec::Value) to Python objects.
// ndarray payloads become zero-copy numpy views over `base`, kept alive by
// `owner`.  Shared by the _native (CPU) and _hip (GPU loader) modules.
#pragma once

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include "../codec/pickle_codec.h"

namespace btn {
namespace pyconv {

namespace py = pybind11;

// Keeps a value's decoded (`owned`) payload alive for numpy views over it.
inline py::object owned_keeper(const codec::Value& v) {
  auto* keep = new std::shared_ptr<const codec::Bytes>(v.owned);
  return py::capsule(keep, [](void* p) { delete static_cast<std::shared_ptr<const codec::Bytes>*>(p); });
}

inline py::object value_to_py(const codec::Value& v, const uint8_t* base, const py::object& owner) {
  using K = codec::Value;
  const uint8_t* data = v.ptr(base);
  if (v.np_scalar) {
    // numpy scalar (e.g. np.float32): 0-d view, then index -> scalar copy
    py::array a(py::dtype(v.dtype), std::vector<py::ssize_t>{}, std::vector<py::ssize_t>{},
                const_cast<uint8_t*>(data), v.owned ? owned_keeper(v) : owner);
    return a[py::tuple()];
  }
  if (v.kind == K::BYTES && v.bytearray)
    return py::reinterpret_steal<py::object>(
        PyByteArray_FromStringAndSize(reinterpret_cast<const char*>(data), py::ssize_t(v.len)));
  switch (v.kind) {
    case K::NONE: return py::none();
    case K::BOOL: return py::bool_(v.b);
    case K::INT: return py::int_(v.i);
    case K::FLOAT: return py::float_(v.f);
    case K::STR: return py::str(v.s);
    case K::BYTES: return py::bytes(reinterpret_cast<const char*>(data), v.len);
    case K::LIST: {
      py::list l;
      for (auto& x : v.items) l.append(value_to_py(*x, base, owner));
      return l;
    }
    case K::TUPLE: {
      py::tuple t(v.items.size());
      for (size_t i = 0; i < v.items.size(); ++i) t[i] = value_to_py(*v.items[i], base, owner);
      return t;
    }
    case K::SET: {
      py::set s;
      for (auto& x : v.items) s.add(value_to_py(*x, base, owner));
      return s;
    }
    case K::DICT: {
      py::dict d;
      for (size_t i = 0; i + 1 < v.items.size(); i += 2)
        d[value_to_py(*v.items[i], base, owner)] = value_to_py(*v.items[i + 1], base, owner);
      return d;
    }
    case K::NDARRAY: {
      py::dtype dt(v.dtype);
      std::vector<py::ssize_t> shape(v.shape.begin(), v.shape.end());
      std::vector<py::ssize_t> strides(shape.size());
      py::ssize_t st = py::ssize_t(v.itemsize());
      if (v.fortran) {
        for (size_t i = 0; i < shape.size(); ++i) {
          strides[i] = st;
          st *= shape[i];
        }
      } else {
        for (size_t i = shape.size(); i-- > 0;) {
          strides[i] = st;
          st *= shape[i];
        }
      }
      // zero-copy view; `owner` keeps the receive buffer alive
      return py::array(dt, shape, strides, const_cast<uint8_t*>(data), v.owned ? owned_keeper(v) : owner);
    }
    default: throw codec::Unsupported("value kind");
  }
}

}  // namespace pyconv
}  // namespace btn
