// POSIX shared-memory frame slots (see shmring.h).
#include "shmring.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace btn {
namespace shm {

namespace {
std::string shm_path(const std::string& name) { return name[0] == '/' ? name : "/" + name; }
size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
}  // namespace

std::atomic<uint32_t>* Segment::states() const {
  return reinterpret_cast<std::atomic<uint32_t>*>(base_ + sizeof(Header));
}

Segment* Segment::create(const std::string& name, uint32_t nslots, size_t slot_bytes) {
  if (nslots == 0 || slot_bytes == 0) throw std::invalid_argument("shm: empty segment");
  const std::string path = shm_path(name);
  int fd = ::shm_open(path.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("shm_open(create) failed for " + path + ": " + std::strerror(errno));
  slot_bytes = round_up(slot_bytes, 4096);
  const size_t data_off = round_up(sizeof(Header) + sizeof(uint32_t) * nslots, 4096);
  const size_t size = data_off + slot_bytes * nslots;
  // reserve the pages now: a too-small /dev/shm fails here with ENOSPC
  // instead of SIGBUS on first touch later
  if (::ftruncate(fd, off_t(size)) != 0 || ::posix_fallocate(fd, 0, off_t(size)) != 0) {
    ::close(fd);
    ::shm_unlink(path.c_str());
    throw std::runtime_error("shm: cannot reserve " + std::to_string(size >> 20) + " MiB in /dev/shm");
  }
  void* p = ::mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    ::close(fd);
    ::shm_unlink(path.c_str());
    throw std::runtime_error("shm: mmap failed");
  }
  auto* s = new Segment();
  s->name_ = name;
  s->fd_ = fd;
  s->base_ = static_cast<uint8_t*>(p);
  s->size_ = size;
  s->owner_ = true;
  s->hdr_ = reinterpret_cast<Header*>(p);
  s->hdr_->version = 1;
  s->hdr_->nslots = nslots;
  s->hdr_->slot_bytes = slot_bytes;
  s->hdr_->data_offset = data_off;
  for (uint32_t i = 0; i < nslots; ++i) new (&s->states()[i]) std::atomic<uint32_t>(FREE);
  std::atomic_thread_fence(std::memory_order_release);
  s->hdr_->magic = kMagic;
  return s;
}

Segment* Segment::open(const std::string& name) {
  const std::string path = shm_path(name);
  int fd = ::shm_open(path.c_str(), O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("shm_open failed for " + path + ": " + std::strerror(errno));
  struct stat st;
  if (::fstat(fd, &st) != 0 || size_t(st.st_size) < sizeof(Header)) {
    ::close(fd);
    throw std::runtime_error("shm: bad segment " + path);
  }
  void* p = ::mmap(nullptr, size_t(st.st_size), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    ::close(fd);
    throw std::runtime_error("shm: mmap failed for " + path);
  }
  auto* s = new Segment();
  s->name_ = name;
  s->fd_ = fd;
  s->base_ = static_cast<uint8_t*>(p);
  s->size_ = size_t(st.st_size);
  s->hdr_ = reinterpret_cast<Header*>(p);
  if (s->hdr_->magic != kMagic || s->hdr_->data_offset + s->hdr_->slot_bytes * s->hdr_->nslots > s->size_) {
    delete s;
    throw std::runtime_error("shm: " + path + " is not a blendtorch segment");
  }
  return s;
}

Segment::~Segment() {
  if (base_) ::munmap(base_, size_);
  if (fd_ >= 0) ::close(fd_);
  if (owner_) ::shm_unlink(shm_path(name_).c_str());
}

namespace {
int64_t now_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
}  // namespace

int Segment::acquire(long timeout_ms, const std::atomic<bool>* stop, long lease_ms) {
  const int64_t t0 = now_us();
  const uint32_t n = hdr_->nslots;
  if (published_at_.size() != n) published_at_.assign(n, 0);
  int spins = 0;
  for (;;) {
    for (uint32_t k = 0; k < n; ++k) {
      const uint32_t i = (next_ + k) % n;
      const uint32_t w = states()[i].load(std::memory_order_acquire);
      if ((w & 3u) == FREE) {
        states()[i].store((w & ~3u) | WRITING, std::memory_order_relaxed);
        next_ = (i + 1) % n;
        return int(i);
      }
    }
    if (stop && stop->load()) return -1;
    const int64_t waited = now_us() - t0;
    if (timeout_ms >= 0 && waited >= timeout_ms * 1000) return -1;
    if (lease_ms > 0 && waited >= lease_ms * 1000) {
      // reclaim the slot published longest ago (its message was dropped);
      // held slots only after a much longer stall (their consumer died)
      const bool take_held = waited >= lease_ms * 1000 * kHeldLeaseFactor;
      uint32_t best = n;
      for (uint32_t i = 0; i < n; ++i) {
        const uint32_t st = state(i) & 3u;
        if ((st == PUBLISHED || (take_held && st == HELD)) &&
            (best == n || published_at_[i] < published_at_[best]))
          best = i;
      }
      if (best < n) {
        uint32_t w = state(best);
        const uint32_t st = w & 3u;
        if ((st == PUBLISHED || (take_held && st == HELD)) &&
            states()[best].compare_exchange_strong(w, (w & ~3u) | WRITING, std::memory_order_acq_rel)) {
          ++reclaimed_;
          next_ = (best + 1) % n;
          return int(best);
        }
      }
    }
    // every slot is with a consumer: backpressure, like a full SNDHWM
    if (++spins < 64) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
}

uint32_t Segment::publish(uint32_t i) {
  const uint32_t w = states()[i].load(std::memory_order_relaxed);
  const uint32_t gen = ((w >> 2) + 1) & 0x3fffffffu;
  if (published_at_.size() == hdr_->nslots) published_at_[i] = now_us();
  states()[i].store((gen << 2) | PUBLISHED, std::memory_order_release);
  return gen;
}

bool Segment::claim(uint32_t i, uint32_t gen) {
  if (i >= hdr_->nslots) return false;
  uint32_t expect = (gen << 2) | PUBLISHED;
  return states()[i].compare_exchange_strong(expect, (gen << 2) | HELD, std::memory_order_acq_rel);
}

void Segment::release(uint32_t i, uint32_t gen) {
  if (i >= hdr_->nslots) return;
  uint32_t expect = (gen << 2) | HELD;
  if (states()[i].compare_exchange_strong(expect, gen << 2 | FREE, std::memory_order_acq_rel)) return;
  expect = (gen << 2) | PUBLISHED;   // never claimed (a dropped descriptor)
  states()[i].compare_exchange_strong(expect, gen << 2 | FREE, std::memory_order_acq_rel);
}

bool Segment::valid(uint32_t i, uint32_t gen) const {
  if (i >= hdr_->nslots) return false;
  const uint32_t w = state(i);
  return w == ((gen << 2) | PUBLISHED) || w == ((gen << 2) | HELD);
}

uint32_t Segment::count(SlotState st) const {
  uint32_t c = 0;
  for (uint32_t i = 0; i < hdr_->nslots; ++i) c += (state(i) & 3u) == uint32_t(st);
  return c;
}

uint32_t Segment::state(uint32_t i) const { return states()[i].load(std::memory_order_acquire); }

uint32_t Segment::free_count() const { return count(FREE); }

}  // namespace shm
}  // namespace btn
