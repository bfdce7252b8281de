// StreamLoader implementation (see loader.h).
#include "loader.h"

#include <pthread.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include "../codec/tiledelta.h"
#include "../common/trace.h"

#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <stdexcept>

namespace btn {
namespace gpu {

namespace {

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Remove the image entry from the dict and shift every payload offset that
// lies behind the cut so the tree indexes the compacted metadata bytes.
void shift_offsets(codec::Value& v, size_t cut, size_t len) {
  if ((v.kind == codec::Value::BYTES || v.kind == codec::Value::NDARRAY || v.np_scalar) && !v.owned) {
    if (v.off >= cut + len) v.off -= len;
  }
  for (auto& c : v.items)
    if (c) shift_offsets(*c, cut, len);
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    (void)hipGetDevice(&prev);
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
  }
};

}  // namespace

// ---------------------------------------------------------------------------
// PinnedPool
// ---------------------------------------------------------------------------
PinnedPool::PinnedPool(size_t slot_bytes, int nslots) : slot_bytes_(slot_bytes), nslots_(nslots) {
  check(hipHostMalloc(reinterpret_cast<void**>(&base_), slot_bytes_ * size_t(nslots_), hipHostMallocDefault),
        "hipHostMalloc(pinned pool)");
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&dev_base_), base_, 0) != hipSuccess) dev_base_ = nullptr;
  free_.reserve(size_t(nslots_));
  for (int i = nslots_ - 1; i >= 0; --i) free_.push_back(i);
}

PinnedPool::~PinnedPool() {
  if (base_) (void)hipHostFree(base_);
}

int PinnedPool::free_slots() {
  std::lock_guard<std::mutex> lk(mu_);
  return int(free_.size());
}

BufPtr PinnedPool::alloc(size_t n) {
  if (n > slot_bytes_) {
    fallbacks_++;
    return nullptr;
  }
  int id;
  {
    std::unique_lock<std::mutex> lk(mu_);
    if (free_.empty() && wait_ms_ > 0)
      cv_.wait_for(lk, std::chrono::milliseconds(wait_ms_), [&] { return !free_.empty(); });
    if (free_.empty()) {
      fallbacks_++;
      return nullptr;
    }
    id = free_.back();
    free_.pop_back();
  }
  auto b = std::make_shared<Buffer>();
  b->data = base_ + size_t(id) * slot_bytes_;
  b->capacity = slot_bytes_;
  b->owner = this;
  b->tag = id;
  b->pinned = true;
  b->release = &PinnedPool::release;
  return b;
}

BufPtr PinnedPool::try_alloc(size_t n) {
  if (n > slot_bytes_) return nullptr;
  int id;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (free_.empty()) return nullptr;
    id = free_.back();
    free_.pop_back();
  }
  auto b = std::make_shared<Buffer>();
  b->data = base_ + size_t(id) * slot_bytes_;
  b->capacity = slot_bytes_;
  b->owner = this;
  b->tag = id;
  b->pinned = true;
  b->release = &PinnedPool::release;
  return b;
}

void PinnedPool::release(void* owner, Buffer* b) {
  auto* self = static_cast<PinnedPool*>(owner);
  {
    std::lock_guard<std::mutex> lk(self->mu_);
    self->free_.push_back(int(b->tag));
  }
  self->cv_.notify_one();
}

// ---------------------------------------------------------------------------
// StreamLoader
// ---------------------------------------------------------------------------
StreamLoader::StreamLoader(const LoaderConfig& cfg) : cfg_(cfg) {
  if (cfg_.addresses.empty()) throw std::invalid_argument("StreamLoader: no addresses");
  if (cfg_.batch_size < 1) throw std::invalid_argument("StreamLoader: batch_size < 1");
  // the value table (kernels.h): a bare [4][256] fp32 table is padded with a
  // zero header (mode 0: table lookups)
  if (cfg_.lut.size() == 4 * 256) cfg_.lut.resize(kTableFloats, 0.f);
  if (cfg_.lut.size() != size_t(kTableFloats))
    throw std::invalid_argument("StreamLoader: lut must hold 4*256 or kTableFloats floats");
  if (cfg_.cout < 1 || cfg_.cout > 4) throw std::invalid_argument("StreamLoader: cout must be 1..4");
  if (cfg_.color_matrix && !cfg_.jitter && cfg_.matrices.empty() && (cfg_.matrix.size() != 16 || cfg_.bias.size() != 4))
    throw std::invalid_argument("StreamLoader: colour matrix needs 16 + 4 floats");
  if (!cfg_.matrices.empty() && cfg_.matrices.size() != size_t(cfg_.batch_size) * 20)
    throw std::invalid_argument("StreamLoader: per-position colour matrices need batch_size x (16 + 4) floats");
  if ((cfg_.jitter || !cfg_.matrices.empty()) && cfg_.batch_size > kMaxSrcs)
    throw std::invalid_argument("StreamLoader: per-image colour transforms need batch_size <= 64");
  jit_state_ = cfg_.jitter_seed * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
  int k = std::max(1, std::min<int>(cfg_.io_threads, int(cfg_.addresses.size())));
  for (int i = 0; i < k; ++i) {
    ctxs_.emplace_back(new zmtp::Context());
    auto s = ctxs_.back()->socket(zmtp::PULL);
    s->setsockopt(zmtp::RCVHWM, cfg_.rcvhwm);
    s->setsockopt(zmtp::LINGER, 0);
    socks_.push_back(s);
  }
  for (size_t i = 0; i < cfg_.addresses.size(); ++i) socks_[i % socks_.size()]->connect(cfg_.addresses[i]);
}

namespace {
uint64_t thread_cpu_ns() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}
// Host-ordered hand-off (host_sync): with BT_LOADER_BLOCKING=1 the events
// that mark a batch's device work are blocking-sync events, and a worker that
// cannot go on until the oldest launched batch completes (every posted
// buffer in use) sleeps in hipEventSynchronize instead of polling it every
// few microseconds.
bool blocking_waits() {
  static const bool on = [] {
    const char* e = std::getenv("BT_LOADER_BLOCKING");
    return e && e[0] == '1';
  }();
  return on;
}
unsigned completion_event_flags() {
  return hipEventDisableTiming | (blocking_waits() ? hipEventBlockingSync : 0u);
}
// BT_LOADER_CPU=1: the worker accounts its thread CPU per loop stage (the
// thread clock is a system call, ~0.3 us, a few per loop turn: off by default)
bool cpu_accounting() {
  static const bool on = [] {
    const char* e = std::getenv("BT_LOADER_CPU");
    return e && e[0] == '1';
  }();
  return on;
}
// adds the calling thread's CPU time over its scope to one counter
struct CpuScope {
  std::atomic<uint64_t>& acc;
  const bool on = cpu_accounting();
  const uint64_t t0 = on ? thread_cpu_ns() : 0;
  explicit CpuScope(std::atomic<uint64_t>& a) : acc(a) {}
  ~CpuScope() {
    if (on) acc.fetch_add(thread_cpu_ns() - t0, std::memory_order_relaxed);
  }
};
// Completion polling grain of the worker thread while launched batches are in
// flight (BT_LOADER_POLL_US, default 10): finer hands batches over sooner,
// coarser costs less CPU per delivered frame.
std::chrono::microseconds poll_grain() {
  static const long us = [] {
    const char* e = std::getenv("BT_LOADER_POLL_US");
    const long v = e ? std::atol(e) : 10;
    return v > 0 ? v : 10;
  }();
  return std::chrono::microseconds(us);
}
}  // namespace

StreamLoader::~StreamLoader() { stop(); }

void StreamLoader::start() {
  if (worker_.joinable()) return;
  worker_ = std::thread([this] {
    pthread_setname_np(pthread_self(), "bt-loader");
    worker_tid_ = int64_t(syscall(SYS_gettid));
    try {
      run();
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> lk(mu_);
      error_ = e.what();
    }
    cv_.notify_all();
  });
}

bool StreamLoader::wait_shape(long timeout_ms, int* H, int* W, int* C) {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return have_shape_ || !error_.empty(); });
  if (!error_.empty()) throw std::runtime_error(error_);
  if (!have_shape_) return false;
  *H = H_;
  *W = W_;
  *C = C_;
  return true;
}

void StreamLoader::post(void* dst, hipStream_t consumer) {
  DeviceGuard g(cfg_.device);
  hipEvent_t ev;
  check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
  check(hipEventRecord(ev, consumer), "hipEventRecord(post)");
  {
    std::lock_guard<std::mutex> lk(mu_);
    posted_.push_back({dst, ev});
  }
  cv_.notify_all();
}

bool StreamLoader::next(ReadyBatch* out, hipStream_t consumer, long timeout_ms) {
  trace::Range tr("btn.loader.next");
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms),
               [&] { return !ready_.empty() || !error_.empty() || exhausted_; });
  if (ready_.empty()) {
    if (!error_.empty()) throw std::runtime_error(error_);
    if (exhausted_) {
      out->index = -1;
      return true;
    }
    return false;
  }
  *out = std::move(ready_.front());
  ready_.pop_front();
  lk.unlock();
  if (out->done) {   // host_sync = false: the consumer stream waits on the device
    DeviceGuard g(cfg_.device);
    check(hipStreamWaitEvent(consumer, out->done, 0), "hipStreamWaitEvent");
    (void)hipEventDestroy(out->done);
    out->done = nullptr;
  }
  out->pending.reset();
  return true;
}

// host_sync: hand out, in order, the launched batches whose device work the
// host has seen complete (worker thread).  Their shm slots are re-validated
// first: a HELD slot a dead-consumer lease took back while the DMA read it
// fails the stream BEFORE the batch reaches the consumer (reap() counts it).
// Without host_sync the batch is handed out at launch and the same check in
// reap() raises on the consumer's next next() call.
void StreamLoader::promote_ready() {
  bool any = false;
  while (!unready_.empty() && unready_.front().pending->done()) {
    ReadyBatch& rb = unready_.front();
    // a launch reap() has retired was validated there (before its slots were
    // handed back: they may already belong to new frames); otherwise the
    // slots are still held by this loader and are checked here
    const bool torn = rb.launch_no > retired_launch_ &&
                      std::any_of(rb.slots.begin(), rb.slots.end(),
                                  [](const ReadyBatch::SlotRef& s) { return !s.seg->valid(s.slot, s.gen); });
    std::lock_guard<std::mutex> lk(mu_);
    if ((torn || !error_.empty()) && !cfg_.skip_bad) {   // reap() may have failed the stream already
      if (error_.empty())
        error_ = "StreamLoader: shared-memory slot(s) were reclaimed by their producer while a batch read them";
      stop_ = true;
      any = true;
      break;
    }
    rb.slots.clear();
    ready_.push_back(std::move(rb));
    unready_.pop_front();
    any = true;
  }
  if (any) cv_.notify_all();
}

void StreamLoader::host_wait(hipEvent_t ev) {
  while (hipEventQuery(ev) == hipErrorNotReady && !stop_) {
    promote_ready();
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

void StreamLoader::stop() {
  stop_ = true;
  cv_.notify_all();
  if (worker_.joinable()) worker_.join();
  drain_sockets();
  for (auto& s : socks_) s->close(0);
  socks_.clear();
  ctxs_.clear();   // joins IO threads; queued frames are released
  DeviceGuard g(cfg_.device);
  for (auto cs : copy_streams_) {
    (void)hipStreamSynchronize(cs);
    (void)hipStreamDestroy(cs);
  }
  copy_streams_.clear();
  for (auto ev : copy_done_) (void)hipEventDestroy(ev);
  copy_done_.clear();
  if (stream_) {
    (void)hipStreamSynchronize(stream_);
    reap(true);                            // drop pinned refs of finished copies
    (void)hipStreamDestroy(stream_);
    stream_ = nullptr;
  }
  for (auto ev : stage_free_)
    if (ev) (void)hipEventDestroy(ev);
  stage_free_.clear();
  for (auto& it : cur_)
    if (it.seg) it.seg->release(it.slot, it.gen);
  cur_.clear();
  for (auto& b : pending_) {
    for (auto& it : b.items)
      if (it.seg) it.seg->release(it.slot, it.gen);
    if (b.ready) (void)hipEventDestroy(b.ready);
  }
  pending_.clear();
  pending_images_ = 0;
  for (auto& kv : segments_) (void)hipHostUnregister(kv.second.seg->base());
  segments_.clear();
  for (auto& kv : keys_) {
    if (kv.second.dev) (void)hipFree(kv.second.dev);
    for (void* d : kv.second.decoded)
      if (d) (void)hipFree(d);
  }
  keys_.clear();
  {
    std::lock_guard<std::mutex> lk(mu_);
    seg_list_.clear();
    for (auto& p : posted_) (void)hipEventDestroy(p.ready);
    posted_.clear();
    for (auto& r : ready_)
      if (r.done) (void)hipEventDestroy(r.done);
    ready_.clear();
  }
  unready_.clear();
  for (auto* p : staging_) (void)hipFree(p);
  staging_.clear();
  if (d_lut_) (void)hipFree(d_lut_);
  if (d_mat_) (void)hipFree(d_mat_);
  d_lut_ = d_mat_ = nullptr;
  pool_.reset();
}

// Descriptors still queued in the sockets when the loader stops would pin
// their producers' ring slots until the lease reclaims them: hand them back
// (the reference's PULL socket simply drops queued messages on close).
void StreamLoader::drain_sockets() {
  for (auto& s : socks_) {
    for (int n = 0; n < 4096; ++n) {
      zmtp::Message m;
      try {
        if (!s->try_recv(m)) break;
      } catch (const zmtp::Error&) {
        break;
      }
      release_descriptor(m);
    }
  }
}

// A received but unprocessed shm descriptor: hand its (still PUBLISHED) slot
// back to the producer.  Anything else needs nothing.
void StreamLoader::release_descriptor(const zmtp::Message& m) {
  if (m.size() != 1) return;
  try {
    codec::VPtr root = codec::parse(m[0].data(), m[0].size);
    if (!root || root->kind != codec::Value::DICT) return;
    const codec::Value* d = root->get("_btshm");
    if (!d || d->kind != codec::Value::TUPLE || d->items.size() < 8 || d->items[0]->kind != codec::Value::STR) return;
    const uint32_t slot = uint32_t(d->items[1]->i), gen = uint32_t(d->items[7]->i);
    auto it = segments_.find(d->items[0]->s);
    if (it != segments_.end()) {
      it->second.seg->release(slot, gen);
    } else {
      std::unique_ptr<shm::Segment> seg(shm::Segment::open(d->items[0]->s));
      seg->release(slot, gen);
    }
  } catch (const std::exception&) {
    // producer gone / not a descriptor: nothing to hand back
  }
}

LoaderStats StreamLoader::stats() {
  std::lock_guard<std::mutex> lk(mu_);
  LoaderStats s = stats_;
  s.cpu_poll_ms = double(cpu_ns_[kCpuPoll].load()) * 1e-6;
  s.cpu_recv_ms = double(cpu_ns_[kCpuRecv].load()) * 1e-6;
  s.cpu_launch_ms = double(cpu_ns_[kCpuLaunch].load()) * 1e-6;
  s.cpu_reap_ms = double(cpu_ns_[kCpuReap].load()) * 1e-6;
  s.worker_tid = worker_tid_.load();
  s.pool_fallbacks = pool_ ? pool_->fallbacks() : 0;
  s.ring_slots = s.ring_published = s.ring_held = 0;
  for (const shm::Segment* g : seg_list_) {
    s.ring_slots += g->nslots();
    s.ring_published += g->count(shm::PUBLISHED);
    s.ring_held += g->count(shm::HELD);
  }
  return s;
}

void StreamLoader::run() {
  check(hipSetDevice(cfg_.device), "hipSetDevice");
  check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
  for (int k = 0; cfg_.copy_streams > 1 && k < std::min(cfg_.copy_streams, 4); ++k) {
    hipStream_t cs;
    hipEvent_t ev;
    check(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking), "hipStreamCreate(copy)");
    check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate(copy)");
    copy_streams_.push_back(cs);
    copy_done_.push_back(ev);
  }
  std::vector<std::pair<zmtp::Socket*, int>> items;
  for (auto& s : socks_) items.emplace_back(s.get(), zmtp::POLLIN);
  std::vector<zmtp::Socket*> ready;
  std::vector<zmtp::Message> round;
  const auto intr = [this] { return stop_.load(); };
  const int64_t max_frames = cfg_.max_batches < 0 ? -1 : cfg_.max_batches * cfg_.batch_size;
  int64_t taken = 0;
  while (!stop_) {
    {
      CpuScope cs(cpu_ns_[kCpuReap]);
      promote_ready();
      reap();
    }
    if (max_frames >= 0 && taken >= max_frames) break;
    std::vector<int> ev;
    try {
      CpuScope cs(cpu_ns_[kCpuPoll]);
      // with copies in flight, wake up often enough to recycle their slots
      // promptly (producers / IO threads may be waiting for them)
      trace::Range tp("btn.loader.poll");
      ev = zmtp::Socket::poll(items, inflight_.empty() && pending_.empty() && unready_.empty() ? 100 : (unready_.empty() ? 1 : 0),
                              intr);
      if (!unready_.empty() && std::none_of(ev.begin(), ev.end(), [](int e) { return e != 0; }))
        std::this_thread::sleep_for(poll_grain());   // nothing to receive: poll completions
    } catch (const zmtp::Error& e) {
      if (e.code == zmtp::E_INTR) break;
      throw;
    }
    CpuScope cs(cpu_ns_[kCpuRecv]);
    flush_pending(max_frames >= 0 && taken >= max_frames);
    ready.clear();
    for (size_t i = 0; i < ev.size(); ++i)
      if (ev[i] & zmtp::POLLIN) ready.push_back(socks_[i].get());
    // Fair fan-in (the reference's PULL contract, examples/datagen/Readme.md:
    // 168-177): every round takes at most ONE message per producer pipe,
    // across all IO sockets, whatever the producer -> socket spread (5
    // producers on 4 sockets put 2 on one).  Draining a socket at a time let
    // a lone producer's socket deliver twice its share.  Rounds repeat until
    // one comes back empty or ~64 frames were taken (amortises the poll).
    size_t woke = 0;
    while (!stop_ && !ready.empty() && woke < 64) {
      const size_t room = max_frames >= 0 ? size_t(std::max<int64_t>(0, max_frames - taken)) : size_t(-1);
      if (room == 0) break;
      round.clear();
      if (zmtp::Socket::recv_round(ready, round, room) == 0) break;
      woke += round.size();
      for (auto& m : round) {
        if (stop_) {
          release_descriptor(m);   // the stream failed / stopped mid-round: hand its shm slot back
          continue;
        }
        if (process(std::move(m))) ++taken;
      }
    }
  }
  if (!stop_) flush_pending(true);   // stream complete: nothing more will join the pending batches
  while (!stop_ && !unready_.empty()) {
    unready_.front().pending->wait();
    promote_ready();
  }
  std::lock_guard<std::mutex> lk(mu_);
  exhausted_ = true;
}

bool StreamLoader::process(zmtp::Message&& msg) {
  trace::Range tr("btn.loader.process");
  auto bad = [&](const std::string& why) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stats_.bad++;
      if (!cfg_.skip_bad && error_.empty()) error_ = "StreamLoader: bad message: " + why;
    }
    cv_.notify_all();
    if (!cfg_.skip_bad) stop_ = true;
    return false;
  };
  if (msg.size() != 1) return bad("expected a single-frame message");
  Item it;
  // a claimed shm slot (and the key-frame reference of a tile16 frame) goes
  // back on every exit that does not hand the item to cur_ -- the bad()
  // returns and the throws alike: a rejected descriptor must not pin a ring
  // slot for the HELD lease (minutes) nor keep a replaced key frame alive
  struct ClaimGuard {
    Item& it;
    bool armed = false;
    ~ClaimGuard() {
      if (!armed) return;
      it.seg->release(it.slot, it.gen);
      if (it.key) it.key->refs--;
      it.key = nullptr;
    }
  } guard{it};
  it.frame = std::move(msg[0]);
  const uint8_t* data = it.frame.data();
  const size_t n = it.frame.size;
  codec::VPtr root;
  try {
    root = codec::parse(data, n);
  } catch (const std::exception& e) {
    return bad(std::string("unparseable pickle (") + e.what() + ")");
  }
  if (!root || root->kind != codec::Value::DICT) return bad("payload is not a dict");
  size_t img_idx = size_t(-1), shm_idx = size_t(-1);
  for (size_t i = 0; i + 1 < root->items.size(); i += 2) {
    if (root->items[i]->kind != codec::Value::STR) continue;
    if (root->items[i]->s == cfg_.image_key) img_idx = i;
    else if (root->items[i]->s == "_btshm") shm_idx = i;
  }
  int h, w, c;
  size_t cut = 0, len = 0;
  if (shm_idx != size_t(-1)) {
    // descriptor (segment, slot, byte offset, H, W, C, key): image in shared memory
    const codec::Value& d = *root->items[shm_idx + 1];
    if (d.kind != codec::Value::TUPLE || d.items.size() < 8 || d.items[0]->kind != codec::Value::STR)
      return bad("malformed _btshm descriptor");
    uint8_t* dev_base = nullptr;
    try {
      MappedSegment& ms = segment(d.items[0]->s);
      it.seg = ms.seg.get();
      dev_base = ms.dev_base;
    } catch (const std::exception& e) {
      return bad(e.what());
    }
    it.slot = uint32_t(d.items[1]->i);
    it.gen = uint32_t(d.items[7]->i);
    const int64_t off = d.items[2]->i;
    h = int(d.items[3]->i), w = int(d.items[4]->i), c = int(d.items[5]->i);
    const bool has_codec = d.items.size() >= 9 && d.items[8]->kind == codec::Value::TUPLE;
    if (it.slot >= it.seg->nslots() || off < 0 || (!has_codec && size_t(off) + size_t(h) * w * c > it.seg->size()))
      return bad("_btshm descriptor out of range");
    if (!it.seg->claim(it.slot, it.gen)) {
      // the producer reclaimed the slot (lease expired while this descriptor
      // sat in a queue): its bytes are another frame's now -- drop it.  Once
      // claimed (HELD) the slot is ours until reap() hands it back.
      std::lock_guard<std::mutex> lk(mu_);
      stats_.shm_stale++;
      return false;
    }
    guard.armed = true;   // claimed: every exit but the hand-over to cur_ gives it back
    it.src = it.seg->base() + off;
    if (dev_base) it.dsrc = dev_base + off;
    if (d.items.size() >= 9 && d.items[8]->kind == codec::Value::TUPLE) {
      // 9th element (codec, key segment, key generation): key-frame delta
      const codec::Value& cd = *d.items[8];
      if (cd.items.size() < 3 || cd.items[0]->kind != codec::Value::STR || cd.items[0]->s != tiledelta::kName ||
          cd.items[1]->kind != codec::Value::STR)
        return bad("unknown _btshm codec");
      if (!tiledelta::supported(h, w, c)) return bad("tile16 frame size must be a multiple of 16");
      // the tile count and every position must stay inside this slot and
      // frame: the scatter kernel trusts them when it reads host memory
      const size_t slot_end = it.seg->slot_offset(it.slot) + it.seg->slot_bytes();
      if (size_t(off) < it.seg->slot_offset(it.slot) || size_t(off) + 4 > slot_end)
        return bad("_btshm tile16 frame out of range");
      const long ntiles = tiledelta::check(it.src, h, w, c, slot_end - size_t(off));
      if (ntiles < 0) return bad("malformed tile16 frame");
      it.ntiles = int(ntiles);
      try {
        KeyFrame& kf = key_frame(cd.items[1]->s, size_t(h) * w * c);
        kf.refs++;
        it.key = &kf;
        it.key_host = kf.seg->slot(0);
      } catch (const std::exception& e) {
        return bad(e.what());
      }
      it.tiled = true;
    }
    root->items.erase(root->items.begin() + long(shm_idx), root->items.begin() + long(shm_idx) + 2);
  } else {
    if (img_idx == size_t(-1)) return bad("no '" + cfg_.image_key + "' entry");
    const codec::Value& img = *root->items[img_idx + 1];
    if (img.kind != codec::Value::NDARRAY || img.dtype != "|u1" || img.fortran)
      return bad("image must be a C-contiguous uint8 ndarray");
    if (img.shape.size() == 3) {
      h = int(img.shape[0]), w = int(img.shape[1]), c = int(img.shape[2]);
    } else if (img.shape.size() == 2) {
      h = int(img.shape[0]), w = int(img.shape[1]), c = 1;
    } else {
      return bad("image must be HxW or HxWxC");
    }
    if (img.owned) {
      // protocol-2 frame: the pixels were decoded out of latin-1 text, they
      // are not a byte range of the frame -- take them by the copy path
      it.expanded.assign(img.owned->begin() + long(img.off), img.owned->begin() + long(img.off + img.len));
      it.src = it.expanded.data();
    } else {
      it.src = data + img.off;
      if (pool_ && it.frame.buf && it.frame.buf->pinned && it.frame.buf->owner == pool_.get())
        it.dsrc = pool_->device_ptr(it.src);
      cut = img.off, len = img.len;
    }
  }
  if (c < 1 || c > 4) return bad("image channels must be 1..4");
  if (const codec::Value* o = root->get("origin"))
    it.flip = o->kind == codec::Value::STR && o->s == "lower-left";

  if (!have_shape_) {
    for (int k = 0; k < cfg_.cout; ++k)
      if (cfg_.cmap[k] >= c) throw std::runtime_error("StreamLoader: channel map exceeds image channels");
    if (cfg_.color_matrix && (c != 4 || (int64_t(h) * w) % 256 != 0 || w % 4 != 0))
      throw std::runtime_error("StreamLoader: colour matrix needs RGBA input with H*W % 256 == 0, W % 4 == 0");
    img_bytes_ = size_t(h) * w * c;
    passthrough_ = cfg_.out_dtype == OUT_U8 && cfg_.layout == NHWC && cfg_.cout == c && !cfg_.flip_all &&
                   !cfg_.color_matrix;
    for (int k = 0; passthrough_ && k < c; ++k) {
      passthrough_ = cfg_.cmap[k] == k;
      for (int v = 0; passthrough_ && v < 256; ++v) passthrough_ = cfg_.lut[size_t(k) * 256 + size_t(v)] == float(v);
    }
    // sized for an inline frame of this image even when the first message is a
    // shared-memory descriptor (a few hundred bytes): in a mixed fleet the
    // inline producers' frames must fit the slots, or they land on the heap
    // and their batches fall off the direct path
    const size_t inline_bytes = std::max(n, size_t(h) * w * c + n + 1024);
    size_t slot = cfg_.max_frame_bytes ? cfg_.max_frame_bytes : size_t(double(inline_bytes) * 1.05) + 4096;
    slot = (slot + 4095) & ~size_t(4095);
    int nslots = cfg_.pool_slots;
    if (nslots <= 0) {
      // every pipe may hold RCVHWM queued + 1 partial frame; the worker holds
      // the batch being assembled plus the batches whose copies are in flight
      nslots = int(cfg_.addresses.size()) * (cfg_.rcvhwm + 2) + (cfg_.staging_depth + 12) * cfg_.batch_size;
      nslots = std::max(64, nslots + nslots / 2);
      const size_t cap = size_t(4) << 30;   // <= 4 GiB pinned
      if (size_t(nslots) * slot > cap) nslots = int(std::max<size_t>(16, cap / slot));
    }
    pool_ = std::make_shared<PinnedPool>(slot, nslots);
    // every image-bearing frame goes to a pinned slot (small images too: a
    // frame below 64 KB used to be heap-received and took its batch to the
    // copy path); descriptor-only messages stay on the heap
    for (auto& s : socks_) s->set_allocator(pool_, std::min<size_t>(64 * 1024, size_t(h) * w * c));
    for (int k = 0; k < std::max(2, cfg_.staging_depth); ++k) {
      uint8_t* p = nullptr;
      check(hipMalloc(reinterpret_cast<void**>(&p), img_bytes_ * size_t(cfg_.batch_size)), "hipMalloc(staging)");
      staging_.push_back(p);
    }
    check(hipMalloc(reinterpret_cast<void**>(&d_lut_), kTableFloats * sizeof(float)), "hipMalloc(lut)");
    check(hipMemcpy(d_lut_, cfg_.lut.data(), kTableFloats * sizeof(float), hipMemcpyHostToDevice), "upload lut");
    if (cfg_.color_matrix && !cfg_.jitter) {
      std::vector<float> mb(cfg_.matrices);
      if (mb.empty()) {
        mb = cfg_.matrix;
        mb.insert(mb.end(), cfg_.bias.begin(), cfg_.bias.end());
      }
      check(hipMalloc(reinterpret_cast<void**>(&d_mat_), mb.size() * sizeof(float)), "hipMalloc(matrix)");
      check(hipMemcpy(d_mat_, mb.data(), mb.size() * sizeof(float), hipMemcpyHostToDevice), "upload matrix");
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      H_ = h, W_ = w, C_ = c;
      have_shape_ = true;
    }
    cv_.notify_all();
  } else if (h != H_ || w != W_ || c != C_) {
    return bad("image shape changed within the stream");
  }
  // metadata: the frame minus the image payload, tree re-based onto it
  it.meta.bytes.reserve(n - len);
  it.meta.bytes.insert(it.meta.bytes.end(), data, data + cut);
  it.meta.bytes.insert(it.meta.bytes.end(), data + cut + len, data + n);
  if (len) {
    for (size_t i = 0; i + 1 < root->items.size(); i += 2)
      if (root->items[i]->kind == codec::Value::STR && root->items[i]->s == cfg_.image_key) {
        root->items.erase(root->items.begin() + long(i), root->items.begin() + long(i) + 2);
        break;
      }
    shift_offsets(*root, cut, len);
  }
  it.meta.tree = root;

  if (cfg_.jitter) {
    // splitmix64: brightness, contrast, saturation in [max(0, 1 - r), 1 + r], hue in [-r, r] turns
    for (int k = 0; k < 4; ++k) {
      uint64_t z = (jit_state_ += 0x9E3779B97F4A7C15ull);
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      z ^= z >> 31;
      const float u = float(z >> 40) * (1.f / 16777216.f);   // [0, 1)
      const float r = cfg_.jitter_range[k];
      const float lo = k < 3 ? std::max(0.f, 1.f - r) : -r, hi = k < 3 ? 1.f + r : r;
      it.jit[k] = lo + (hi - lo) * u;
    }
  }
  if (cur_.empty()) batch_t0_ = now_ms();
  {
    std::lock_guard<std::mutex> lk(mu_);
    stats_.frames++;
    stats_.bytes += n;
    if (it.tiled) {
      stats_.image_bytes += 4 * (size_t(it.ntiles) + 1) + size_t(it.ntiles) * tiledelta::tile_bytes(c);
      stats_.tiled_frames++;
    } else {
      stats_.image_bytes += img_bytes_;
    }
    if (it.seg) stats_.shm_frames++;
    if (const codec::Value* b = root->get("btid"))
      if (b->kind == codec::Value::INT) stats_.frames_per_btid[b->i]++;
  }
  guard.armed = false;
  cur_.push_back(std::move(it));
  if (int(cur_.size()) == cfg_.batch_size) launch();
  return true;
}

StreamLoader::KeyFrame& StreamLoader::key_frame(const std::string& name, size_t bytes) {
  auto it = keys_.find(name);
  if (it != keys_.end()) return it->second;
  KeyFrame kf;
  kf.seg.reset(shm::Segment::open(name));
  if (kf.seg->nslots() < 1 || kf.seg->slot_bytes() < bytes || kf.seg->state(0) % 4 != shm::PUBLISHED)
    throw std::runtime_error("tile16 key segment " + name + " is not a published key frame");
  // once per producer: the key frame stays in HBM for the stream's lifetime
  check(hipMalloc(reinterpret_cast<void**>(&kf.dev), bytes), "hipMalloc(key frame)");
  check(hipMemcpy(kf.dev, kf.seg->slot(0), bytes, hipMemcpyHostToDevice), "upload key frame");
  return keys_[name] = std::move(kf);
}

const void* StreamLoader::decoded_key(KeyFrame& kf, bool flip, size_t out_img_bytes) {
  void*& d = kf.decoded[flip ? 1 : 0];
  if (d) return d;
  // the key frame through this loader's own decode (table, channels, dtype,
  // layout, flip): every tiled image of this producer starts as a copy of it
  check(hipMalloc(&d, out_img_bytes), "hipMalloc(decoded key)");
  DecodeParams dp;
  dp.src = kf.dev;
  dp.dst = d;
  dp.lut = d_lut_;
  dp.B = 1, dp.H = H_, dp.W = W_, dp.Cin = C_, dp.Cout = cfg_.cout;
  std::memcpy(dp.cmap, cfg_.cmap, sizeof(dp.cmap));
  dp.flip_all = cfg_.flip_all || flip;
  dp.out_dtype = cfg_.out_dtype;
  dp.layout = cfg_.layout;
  check(decode(dp, stream_), "decode(key frame)");
  return d;
}

void StreamLoader::materialize(Item& it) {
  if (!it.tiled) return;
  it.expanded.resize(img_bytes_);
  tiledelta::expand(it.src, it.key_host, H_, W_, C_, it.expanded.data());
  it.src = it.expanded.data();
  it.dsrc = nullptr;
  it.tiled = false;
  if (it.key) it.key->refs--;   // rebuilt on the host: the HBM key is not read for it
  it.key = nullptr;
}

StreamLoader::MappedSegment& StreamLoader::segment(const std::string& name) {
  auto it = segments_.find(name);
  if (it != segments_.end()) return it->second;
  MappedSegment ms;
  ms.seg.reset(shm::Segment::open(name));
  // pin + map the producer's ring: the DMA engine (copy path) or the decode
  // kernel itself (direct path) reads the slots in place
  check(hipHostRegister(ms.seg->base(), ms.seg->size(), hipHostRegisterMapped), "hipHostRegister(shm)");
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&ms.dev_base), ms.seg->base(), 0) != hipSuccess)
    ms.dev_base = nullptr;
  {
    std::lock_guard<std::mutex> lk(mu_);
    seg_list_.push_back(ms.seg.get());   // ring occupancy in stats()
  }
  return segments_[name] = std::move(ms);
}

void StreamLoader::reap(bool wait_all) {
  // drop the frames of batches whose H2D copies completed: their pinned
  // slots return to the pool (and unblock an IO thread waiting for one)
  // (diagnostic BT_LOADER_REAP_US: at most one completion query per interval)
  static const long reap_us = [] {
    const char* e = std::getenv("BT_LOADER_REAP_US");
    return e ? std::atol(e) : 0L;
  }();
  if (reap_us > 0 && !wait_all && !inflight_.empty()) {
    const double t = now_ms();
    if (t - last_reap_ms_ < reap_us * 1e-3) return;
    last_reap_ms_ = t;
  }
  while (!inflight_.empty()) {
    Inflight& f = inflight_.front();
    if (wait_all) f.copied->wait();
    else if (!f.copied->done()) break;
    f.copied.reset();
    if (f.t0) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, f.t0, f.t1) == hipSuccess) {
        std::lock_guard<std::mutex> lk(mu_);
        stats_.timed_launches++;
        stats_.timed_images += uint64_t(f.images);
        stats_.timed_gpu_ms += ms;
      }
      (void)hipEventDestroy(f.t0);
      (void)hipEventDestroy(f.t1);
    }
    uint64_t torn = 0;
    for (auto& s : f.slots) {
      if (!s.seg->valid(s.slot, s.gen)) torn++;   // a HELD slot taken back (dead-consumer lease)
      s.seg->release(s.slot, s.gen);
    }
    if (torn) {
      // the batch went out with another frame's pixels under its metadata:
      // never deliver that silently (skip_bad only counts it)
      {
        std::lock_guard<std::mutex> lk(mu_);
        stats_.shm_torn += torn;
        if (!cfg_.skip_bad && error_.empty())
          error_ = "StreamLoader: " + std::to_string(torn) +
                   " shared-memory slot(s) were reclaimed by their producer while a batch read them";
      }
      cv_.notify_all();
      if (!cfg_.skip_bad) stop_ = true;
    }
    retired_launch_ = f.launch_no;
    inflight_.pop_front();
  }
  evict_keys();
}

// Key frames a producer replaced (set_key_frame) are never referenced again:
// free their HBM copies once no queued batch and no in-flight launch uses them.
void StreamLoader::evict_keys() {
  for (auto it = keys_.begin(); it != keys_.end();) {
    KeyFrame& kf = it->second;
    if (kf.refs == 0 && kf.last_launch <= retired_launch_ && launch_no_ - kf.last_launch > kKeyIdleLaunches) {
      if (kf.dev) (void)hipFree(kf.dev);
      for (void* d : kf.decoded)
        if (d) (void)hipFree(d);
      {
        std::lock_guard<std::mutex> lk(mu_);
        stats_.keys_evicted++;
      }
      it = keys_.erase(it);
    } else {
      ++it;
    }
  }
}

// One batch of B frames is complete: bind it to the next consumer-posted
// output buffer and queue it for launch.
void StreamLoader::launch() {
  trace::Range tr("btn.loader.assemble");
  Posted p{nullptr, nullptr};
  {
    std::unique_lock<std::mutex> lk(mu_);
    while (posted_.empty() && !stop_) {
      lk.unlock();
      // out of output buffers: the consumer is waiting for batches, so
      // holding assembled ones back for coalescing would only stall it
      flush_pending(true);
      promote_ready();
      lk.lock();
      if (!posted_.empty() || stop_) break;
      if (!unready_.empty()) {
        // the consumer is most likely waiting for one of these: keep
        // promoting at a fine grain instead of sleeping through a post
        // (blocking: sleep until the oldest completes, then promote it)
        lk.unlock();
        if (blocking_waits()) unready_.front().pending->wait();
        else std::this_thread::sleep_for(poll_grain());
        lk.lock();
        continue;
      }
      cv_.wait_for(lk, std::chrono::milliseconds(2));
    }
    if (stop_) return;
    p = posted_.front();
    posted_.pop_front();
  }
  Pending pb;
  pb.dst = p.dst;
  pb.ready = p.ready;
  pb.t0 = batch_t0_;
  auto aligned = [](const Item& it) { return it.dsrc && (reinterpret_cast<uintptr_t>(it.dsrc) % 16) == 0; };
  const bool direct = cfg_.direct && int(cur_.size()) <= kMaxSrcs;
  // a batch of key-frame deltas only decodes as such (fill + tile scatter);
  // in any other batch (copy path, MFMA colour kernel, mixed producers) they
  // are rebuilt on the host
  pb.tiled = direct && !cfg_.color_matrix &&
             std::all_of(cur_.begin(), cur_.end(), [&](const Item& it) { return it.tiled && aligned(it); });
  if (!pb.tiled)
    for (auto& it : cur_) materialize(it);
  // mixed batches stay on the direct path: a frame the kernel cannot read in
  // place (heap-received: dry pool, rebuilt on the host, unaligned) is copied
  // into a free pinned slot here, and the rest are still read where they lie
  if (direct && !pb.tiled && pool_)
    for (auto& it : cur_) {
      if (aligned(it)) continue;
      BufPtr b = pool_->try_alloc(img_bytes_);
      if (!b) break;   // no slot free now: this batch takes the copy path
      std::memcpy(b->data, it.src, img_bytes_);
      it.src = b->data;
      it.dsrc = pool_->device_ptr(b->data);
      it.staged = std::move(b);
      std::lock_guard<std::mutex> lk(mu_);
      stats_.staged_frames++;
    }
  pb.direct = direct && std::all_of(cur_.begin(), cur_.end(), aligned);
  pb.items = std::move(cur_);
  cur_.clear();
  pending_images_ += int(pb.items.size());
  pending_.push_back(std::move(pb));
  flush_pending(false);
}

// Launch coalescing: a direct-path batch launches at once while fewer than
// kMaxInflight launches are queued on the loader stream; otherwise it waits,
// and when a launch retires every waiting batch goes out in ONE kernel
// (per-image source/destination pointers).  When the GPU side is the
// bottleneck the launches therefore grow -- fewer ramp-up/tail phases per
// image -- and when the producers are, every batch still launches at once.
void StreamLoader::flush_pending(bool force) {
  if (pending_.empty()) return;
  reap();
  const bool room = int(inflight_.size()) < cfg_.launch_depth;
  const bool full = pending_images_ + cfg_.batch_size > kMaxSrcs;
  const bool copy_waiting = std::any_of(pending_.begin(), pending_.end(), [](const Pending& b) { return !b.direct; });
  if (!(force || room || full || copy_waiting)) return;
  // maximal runs of direct batches go out together; copy-path batches one by one
  std::vector<Pending> group;
  auto emit = [&] {
    if (!group.empty()) launch_group(group);
    group.clear();
  };
  while (!pending_.empty()) {
    Pending b = std::move(pending_.front());
    pending_.pop_front();
    if (!b.direct) {
      emit();
      group.push_back(std::move(b));
      emit();
    } else {
      if (!group.empty() && group.front().tiled != b.tiled) emit();   // one kernel family per launch
      group.push_back(std::move(b));
    }
  }
  emit();
  pending_images_ = 0;
}

void StreamLoader::launch_group(std::vector<Pending>& group) {
  trace::Range tr("btn.loader.launch");
  CpuScope cpu(cpu_ns_[kCpuLaunch]);
  const double t_issue = now_ms();
  const bool direct = group.front().direct;
  int total = 0;
  for (auto& b : group) {
    if (cfg_.host_sync) host_wait(b.ready);   // the consumer is done with the buffer
    else check(hipStreamWaitEvent(stream_, b.ready, 0), "hipStreamWaitEvent(post)");
    (void)hipEventDestroy(b.ready);
    total += int(b.items.size());
  }
  const size_t elem = cfg_.color_matrix ? 4 : (cfg_.out_dtype == OUT_F32 ? 4 : (cfg_.out_dtype == OUT_U8 ? 1 : 2));
  const int cout = cfg_.cout;   // (colour kernel: 4, or 3 for RGB jitter)
  const size_t out_img_bytes = size_t(H_) * W_ * cout * elem;
  uint64_t flips[4] = {0, 0, 0, 0};
  std::vector<const Item*> all;
  all.reserve(size_t(total));
  for (auto& b : group)
    for (auto& it : b.items) all.push_back(&it);
  for (int i = 0; i < total; ++i)
    if (all[size_t(i)]->flip) {
      if (i >= 256) throw std::runtime_error("StreamLoader: per-image flip supports batch <= 256");
      flips[i >> 6] |= uint64_t(1) << (i & 63);
    }
  // sampled GPU timing: events bracket this launch's copies + kernel (the
  // stream has already passed the consumers' post events here)
  hipEvent_t t0 = nullptr, t1 = nullptr;
  const int64_t launch_no = ++launch_no_;
  // skip the cold first launches (allocation, code-object load, page faults)
  if (launch_no > kTimedSkip && launch_no % kTimedEvery == 0 && hipEventCreate(&t0) == hipSuccess) {
    if (hipEventCreate(&t1) != hipSuccess || hipEventRecord(t0, stream_) != hipSuccess) {
      (void)hipEventDestroy(t0);
      if (t1) (void)hipEventDestroy(t1);
      t0 = t1 = nullptr;
    }
  }
  uint8_t* stage = nullptr;
  const size_t stage_idx = size_t(batch_index_) % staging_.size();
  const bool passthrough = !direct && passthrough_ &&
                           std::none_of(all.begin(), all.end(), [](const Item* it) { return it->flip; });
  auto copied = std::make_shared<EventSet>();
  auto add_event = [&](hipStream_t st) {
    hipEvent_t ev;
    check(hipEventCreateWithFlags(&ev, completion_event_flags()), "hipEventCreate(copied)");
    check(hipEventRecord(ev, st), "hipEventRecord(copied)");
    copied->ev.push_back(ev);
  };
  if (passthrough && cfg_.host_sync) {
    // identity decode, host-ordered: the buffer is free (post event seen
    // complete), so the frames go by DMA straight into the consumer's tensor
    // over the copy streams with no stream waits at all; one event per
    // stream marks both the slots' release and the batch's readiness
    const size_t K = std::max<size_t>(1, copy_streams_.size());
    int i = 0;
    for (auto& b : group)
      for (size_t k = 0; k < b.items.size(); ++k, ++i) {
        hipStream_t cs = copy_streams_.empty() ? stream_ : copy_streams_[size_t(i) % K];
        check(hipMemcpyAsync(static_cast<uint8_t*>(b.dst) + k * img_bytes_, all[size_t(i)]->src, img_bytes_,
                             hipMemcpyHostToDevice, cs),
              "hipMemcpyAsync(H2D passthrough)");
      }
    for (size_t k = 0; k < K && k < size_t(total); ++k) add_event(copy_streams_.empty() ? stream_ : copy_streams_[k]);
  } else if (passthrough) {
    // identity decode: the frames go by DMA straight into the consumer's
    // tensor (its post event already gates stream_; the copy streams wait on
    // stream_'s progress through it), and no kernel is launched
    hipEvent_t gate;
    check(hipEventCreateWithFlags(&gate, hipEventDisableTiming), "hipEventCreate(gate)");
    check(hipEventRecord(gate, stream_), "hipEventRecord(gate)");
    const size_t K = std::max<size_t>(1, copy_streams_.size());
    int i = 0;
    for (auto& b : group)
      for (size_t k = 0; k < b.items.size(); ++k, ++i) {
        hipStream_t cs = copy_streams_.empty() ? stream_ : copy_streams_[size_t(i) % K];
        if (cs != stream_ && size_t(i) < K) check(hipStreamWaitEvent(cs, gate, 0), "hipStreamWaitEvent(gate)");
        check(hipMemcpyAsync(static_cast<uint8_t*>(b.dst) + k * img_bytes_, all[size_t(i)]->src, img_bytes_,
                             hipMemcpyHostToDevice, cs),
              "hipMemcpyAsync(H2D passthrough)");
      }
    for (size_t k = 0; k < copy_streams_.size() && k < size_t(total); ++k) {
      check(hipEventRecord(copy_done_[k], copy_streams_[k]), "hipEventRecord(copy)");
      check(hipStreamWaitEvent(stream_, copy_done_[k], 0), "hipStreamWaitEvent(copy)");
    }
    (void)hipEventDestroy(gate);
  } else if (!direct) {   // copy path: exactly one batch per launch
    stage = staging_[stage_idx];
    if (copy_streams_.empty()) {
      for (int i = 0; i < total; ++i)
        check(hipMemcpyAsync(stage + size_t(i) * img_bytes_, all[size_t(i)]->src, img_bytes_, hipMemcpyHostToDevice,
                             stream_),
              "hipMemcpyAsync(H2D)");
    } else {
      // frames round-robin over the copy streams (separate hardware queues,
      // so several DMA engines read host memory at once); each copy stream
      // first waits until the kernel that last read this staging buffer is done
      const size_t K = copy_streams_.size();
      hipEvent_t freed = stage_idx < stage_free_.size() ? stage_free_[stage_idx] : nullptr;
      for (size_t k = 0; k < K && k < size_t(total); ++k) {
        if (freed) check(hipStreamWaitEvent(copy_streams_[k], freed, 0), "hipStreamWaitEvent(stage)");
        for (int i = int(k); i < total; i += int(K))
          check(hipMemcpyAsync(stage + size_t(i) * img_bytes_, all[size_t(i)]->src, img_bytes_,
                               hipMemcpyHostToDevice, copy_streams_[k]),
                "hipMemcpyAsync(H2D)");
        check(hipEventRecord(copy_done_[k], copy_streams_[k]), "hipEventRecord(copy)");
        check(hipStreamWaitEvent(stream_, copy_done_[k], 0), "hipStreamWaitEvent(copy)");
      }
    }
  }
  // `copied` marks the last device read of the host slots: after the copies,
  // or (direct) after the kernel that reads them
  const bool host_passthrough = passthrough && cfg_.host_sync;
  if (!direct && !host_passthrough) add_event(stream_);
  const bool per_image_dst = group.size() > 1;
  hipError_t e = hipSuccess;
  if (passthrough) {
    // nothing to launch: the DMA wrote the output
  } else if (cfg_.color_matrix) {
    Color4x4Params cp;
    cp.src = stage;
    cp.dst = static_cast<float*>(group.front().dst);
    if (direct) {
      cp.nsrcs = total;
      for (int i = 0; i < total; ++i) cp.srcs[i] = all[size_t(i)]->dsrc;
    }
    if (per_image_dst) {
      cp.ndsts = total;
      int i = 0;
      for (auto& b : group)
        for (size_t k = 0; k < b.items.size(); ++k)
          cp.dsts[i++] = reinterpret_cast<float*>(static_cast<uint8_t*>(b.dst) + k * out_img_bytes);
    }
    cp.lut = d_lut_;
    if (cfg_.jitter) {
      cp.mat_mode = kColorJitter;
      cp.pivot = cfg_.pivot;
      for (int i = 0; i < total; ++i) std::memcpy(cp.jit[i], all[size_t(i)]->jit, sizeof(cp.jit[i]));
    } else if (!cfg_.matrices.empty()) {
      cp.mat_mode = kColorPos;
      cp.Ms = d_mat_;
      int i = 0;
      for (auto& b : group)
        for (size_t k = 0; k < b.items.size(); ++k) cp.mat_pos[i++] = uint8_t(k);
    } else {
      cp.M = d_mat_;
      cp.bias = d_mat_ + 16;
    }
    cp.B = total, cp.H = H_, cp.W = W_, cp.Cout = cfg_.cout;
    cp.flip_all = cfg_.flip_all;
    std::memcpy(cp.flip_bits, flips, sizeof(flips));
    e = color4x4(cp, stream_);
  } else {
    DecodeParams dp;
    dp.src = stage;
    dp.dst = group.front().dst;
    if (direct) {
      dp.nsrcs = total;
      for (int i = 0; i < total; ++i) dp.srcs[i] = all[size_t(i)]->dsrc;
    }
    if (per_image_dst) {
      dp.ndsts = total;
      int i = 0;
      for (auto& b : group)
        for (size_t k = 0; k < b.items.size(); ++k) dp.dsts[i++] = static_cast<uint8_t*>(b.dst) + k * out_img_bytes;
    }
    dp.lut = d_lut_;
    dp.B = total, dp.H = H_, dp.W = W_, dp.Cin = C_, dp.Cout = cfg_.cout;
    std::memcpy(dp.cmap, cfg_.cmap, sizeof(dp.cmap));
    dp.flip_all = cfg_.flip_all;
    std::memcpy(dp.flip_bits, flips, sizeof(flips));
    dp.out_dtype = cfg_.out_dtype;
    dp.layout = cfg_.layout;
    if (group.front().tiled) {
      TileParams tp;
      tp.out_img_bytes = int64_t(out_img_bytes);
      tp.payload_off = int64_t(tiledelta::payload_offset(H_, W_));
      for (int i = 0; i < total; ++i) {
        const Item& it = *all[size_t(i)];
        it.key->refs--;
        it.key->last_launch = launch_no;
        tp.fills[i] = decoded_key(*it.key, cfg_.flip_all || it.flip, out_img_bytes);
        tp.tile_start[i + 1] = tp.tile_start[i] + it.ntiles;
      }
      e = decode_tiles(dp, tp, stream_);
    } else {
      e = decode(dp, stream_);
    }
  }
  check(e, "decode kernel launch");
  if (direct) add_event(stream_);
  if (!direct && !passthrough && !copy_streams_.empty()) {
    if (stage_free_.size() < staging_.size()) stage_free_.resize(staging_.size(), nullptr);
    if (!stage_free_[stage_idx])
      check(hipEventCreateWithFlags(&stage_free_[stage_idx], hipEventDisableTiming), "hipEventCreate(stage)");
    check(hipEventRecord(stage_free_[stage_idx], stream_), "hipEventRecord(stage)");
  }
  if (t0 && host_passthrough) {   // the copies ran on other streams: nothing on stream_ to time
    (void)hipEventDestroy(t0);
    (void)hipEventDestroy(t1);
    t0 = t1 = nullptr;
  }
  if (t0) check(hipEventRecord(t1, stream_), "hipEventRecord(t1)");
  Inflight fl;
  fl.launch_no = launch_no;
  fl.t0 = t0, fl.t1 = t1, fl.images = total;
  fl.frames.reserve(size_t(total));
  std::vector<ReadyBatch> done;
  for (auto& b : group) {
    ReadyBatch rb;
    rb.index = batch_index_++;
    rb.launch_no = launch_no;
    rb.items.reserve(b.items.size());
    for (auto& it : b.items) {
      fl.frames.push_back(std::move(it.frame));
      if (it.seg) {
        fl.slots.push_back({it.seg, it.slot, it.gen});
        if (cfg_.host_sync) rb.slots.push_back({it.seg, it.slot, it.gen});
      }
      if (!it.expanded.empty()) fl.expanded.push_back(std::move(it.expanded));
      if (cfg_.jitter) rb.jitter.insert(rb.jitter.end(), it.jit, it.jit + 4);
      if (it.staged) fl.staged.push_back(std::move(it.staged));
      rb.items.push_back(std::move(it.meta));
    }
    if (host_passthrough) {
      rb.pending = copied;        // the DMA is all the batch's device work
    } else if (cfg_.host_sync) {
      auto fin = std::make_shared<EventSet>();
      hipEvent_t ev;
      check(hipEventCreateWithFlags(&ev, completion_event_flags()), "hipEventCreate(done)");
      check(hipEventRecord(ev, stream_), "hipEventRecord(done)");
      fin->ev.push_back(ev);
      rb.pending = fin;
    } else {
      check(hipEventCreateWithFlags(&rb.done, hipEventDisableTiming), "hipEventCreate(done)");
      check(hipEventRecord(rb.done, stream_), "hipEventRecord(done)");
    }
    rb.recv_ms = t_issue - b.t0;
    done.push_back(std::move(rb));
  }
  fl.copied = copied;
  inflight_.push_back(std::move(fl));
  {
    std::lock_guard<std::mutex> lk(mu_);
    stats_.batches += group.size();
    stats_.launches++;
    if (direct) stats_.direct_batches += group.size();
    if (passthrough) stats_.passthrough_batches += group.size();
    stats_.h2d_issue_ms += now_ms() - t_issue;
    if (!cfg_.host_sync)
      for (auto& rb : done) ready_.push_back(std::move(rb));
  }
  if (cfg_.host_sync) {
    for (auto& rb : done) unready_.push_back(std::move(rb));
    promote_ready();
  }
  cv_.notify_all();
}

}  // namespace gpu
}  // namespace btn
