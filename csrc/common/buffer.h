// Reference-counted byte buffers with pluggable allocation.
//
// Every frame that crosses the native transport lives in a `Buffer`.  The
// allocator hook is what lets the GPU loader land socket payloads directly in
// pinned (hipHostMalloc'd) slots: the transport never knows whether the bytes
// it reads into are pageable heap or DMA-able host memory.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>

namespace btn {

struct Buffer {
  uint8_t* data = nullptr;
  size_t capacity = 0;
  // Opaque owner cookie (e.g. pinned slot index); released by `release`.
  void (*release)(void* owner, Buffer* self) = nullptr;
  void* owner = nullptr;
  int64_t tag = -1;       // allocator-defined (pinned slot id, ...)
  bool pinned = false;    // true if the bytes are DMA-able host memory

  Buffer() = default;
  Buffer(const Buffer&) = delete;
  Buffer& operator=(const Buffer&) = delete;
  ~Buffer() {
    if (release) release(owner, this);
  }
};

using BufPtr = std::shared_ptr<Buffer>;

inline void heap_release(void*, Buffer* b) { std::free(b->data); }

inline BufPtr heap_buffer(size_t n) {
  auto b = std::make_shared<Buffer>();
  b->data = static_cast<uint8_t*>(std::malloc(n ? n : 1));
  if (!b->data) throw std::bad_alloc();
  b->capacity = n;
  b->release = heap_release;
  return b;
}

// Allocation policy for receive buffers.  `alloc` may return nullptr to
// request the heap fallback.
class Allocator {
 public:
  virtual ~Allocator() = default;
  virtual BufPtr alloc(size_t n) = 0;
};

}  // namespace btn
