// Zero-copy pickle scanner / writer for blendtorch message frames.
//
// Producers publish `{'btid': int, 'image': ndarray, ...}` dicts pickled with
// protocol 3/4/5 (reference: pkg_blender/blendtorch/btb/publisher.py:42-43,
// pyzmq send_pyobj).  The scanner interprets the pickle opcode stream without
// materialising Python objects: ndarray payloads are reported as
// (offset, nbytes, dtype, shape) *inside the received frame*, so the GPU
// loader can DMA image bytes straight from the pinned receive buffer.
// Anything the scanner does not understand raises `Unsupported` and the
// caller falls back to CPython's pickle.
//
// The writer emits the same structure (numpy 1.x `numpy.core.multiarray`
// module path, readable by numpy 1.x and 2.x) and lets the caller render
// pixels directly into the reserved payload region.
#pragma once

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace btn {
namespace codec {

// Allocator whose value-construction is a no-op: resizing a byte buffer that
// is about to be overwritten (pixel payloads) skips the memset.
template <class T>
struct default_init_allocator : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = default_init_allocator<U>;
  };
  default_init_allocator() = default;
  template <class U>
  default_init_allocator(const default_init_allocator<U>&) noexcept {}
  template <class U>
  void construct(U* p) noexcept {
    ::new (static_cast<void*>(p)) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
};
using Bytes = std::vector<uint8_t, default_init_allocator<uint8_t>>;

class Unsupported : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

struct Value;
using VPtr = std::shared_ptr<Value>;

struct Value {
  enum Kind {
    NONE, BOOL, INT, FLOAT, STR, BYTES, LIST, TUPLE, DICT, NDARRAY,
    // internal
    GLOBAL, DTYPE, MARK_, SET
  };
  Kind kind = NONE;
  bool b = false;
  int64_t i = 0;
  double f = 0.0;
  std::string s;                  // STR text, GLOBAL "module.name", DTYPE code
  size_t off = 0, len = 0;        // BYTES / NDARRAY payload within the frame
  std::vector<VPtr> items;        // LIST/TUPLE elements; DICT: k0,v0,k1,v1,...
  // NDARRAY
  std::string dtype;              // numpy dtype.str e.g. "|u1", "<f8"
  std::vector<int64_t> shape;
  bool fortran = false;
  char byteorder = '=';           // DTYPE
  bool np_scalar = false;         // INT/FLOAT/BOOL decoded from a numpy scalar
  bool bytearray = false;         // BYTES that were a bytearray (protocol 5)
  // BYTES / NDARRAY whose payload is not a byte range of the frame (protocol
  // 2 writes bytes as _codecs.encode(latin-1 text)): the decoded bytes live
  // here and `off` is relative to them
  std::shared_ptr<const Bytes> owned;

  // payload start: inside the frame (`base`) or in `owned`
  const uint8_t* ptr(const uint8_t* base) const { return owned ? owned->data() + off : base + off; }

  const Value* get(const std::string& key) const;   // DICT lookup by str key
  int64_t numel() const;
  size_t itemsize() const;
};

// Parses a pickle; throws Unsupported on unknown constructs.
VPtr parse(const uint8_t* data, size_t n);

// Render a value tree as a short human readable string (tests/debug).
std::string describe(const Value& v);

// --------------------------------------------------------------------------
// Writer
// --------------------------------------------------------------------------
class Writer {
 public:
  explicit Writer(int protocol = 4);
  // Reuse `storage`'s capacity (cleared first) -- producers recycle frame
  // buffers instead of allocating ~1 MB per message.
  Writer(int protocol, Bytes&& storage);
  // Dict building (keys are str).  Values written in call order.
  void begin_dict();
  void key(const std::string& k);
  void end_dict();      // emits SETITEMS for the pending pairs
  void none();
  void boolean(bool v);
  void integer(int64_t v);
  void real(double v);
  void str(const std::string& v);
  void bytes(const void* p, size_t n);
  void begin_tuple();
  void end_tuple();
  void begin_list();
  void end_list();
  // ndarray in C order.  dtype like "u1", "f8", "f4", "i8"; byteorder '|' for
  // single-byte types, '<' otherwise.  Returns the payload offset; the caller
  // writes `nbytes` at out.data() + offset (after finish()).
  // align > 1: pad with pickle no-ops (NONE+POP, BININT1+POP) so that the
  // payload starts at a multiple of `align` from the start of the pickle --
  // a receiver that lands the frame body at an aligned address (the GPU
  // loader's pinned slots) can then hand the payload to vector loads as is.
  // The unpickled value is unchanged.
  size_t ndarray(const std::string& dtype, const std::vector<int64_t>& shape,
                 const void* data = nullptr, size_t align = 0);
  Bytes& finish();
  Bytes& buffer() { return out_; }

 private:
  void op(uint8_t c) { out_.push_back(c); }
  void raw(const void* p, size_t n);
  void u32le(uint32_t v);
  void u64le(uint64_t v);
  void short_str(const std::string& s);
  void global(const std::string& mod, const std::string& name);
  int protocol_;
  Bytes out_;
  std::vector<size_t> marks_;
};

// Exact bytes of `pickle.dumps(np.full(capacity, -1, np.int64), protocol=3)`
// as numpy 1.x writes it (module path numpy.core.multiarray) with the given
// offsets filled in -- the `.btr` recording header
// (reference: pkg_pytorch/blendtorch/btt/file.py:56-74).
std::vector<uint8_t> btr_header(const std::vector<int64_t>& offsets);

}  // namespace codec
}  // namespace btn
