// StreamLoader: producer frames -> decoded batch in HBM.
//
// Replaces the reference's receive path (pkg_pytorch/blendtorch/btt/
// dataset.py:64-117 PULL socket per DataLoader worker + pickle.loads +
// default_collate + worker->main shared-memory copy) with one native
// pipeline per GPU rank:
//
//   producers --PUSH/ZMTP--> K PULL sockets (K IO threads, fair-queued)
//     -> the image is either in the producer's shared-memory ring (the
//        message carries a `_btshm` descriptor; the ring is hipHostRegister'ed
//        and mapped once) or inline, read by the IO thread straight into
//        hipHostMalloc'd slots (PinnedPool is the socket allocator)
//     -> worker thread: zero-copy pickle scan locates the image payload,
//        copies only the small non-image bytes (metadata) out
//     -> B items + the next consumer-posted output buffer form a batch;
//        direct path (default, every frame device-visible and 16-byte
//        aligned): the fused decode kernel reads the host frames over PCIe
//        itself, and batches that wait while `launch_depth` launches are
//        queued go out together in one launch; copy path: hipMemcpyAsync of
//        every image into a device staging ring first, then the kernel
//     -> the kernel (flip/gamma/unpack/normalize/CHW|NHWC) writes the
//        consumer's tensor on a private non-blocking HIP stream; an event
//        after the last host read lets the worker hand slots back (no host
//        callback in the stream); a per-batch event marks it ready
//     -> consumer (Python) takes batch j; its torch stream waits on the event.
//
// Backpressure is preserved end to end: when the consumer stops posting
// output buffers the worker stops receiving, each pipe fills to RCVHWM, the
// TCP window closes and the producers block at SNDHWM -- exactly the
// behaviour the reference's PUSH/PULL + HWM gives (btb/publisher.py:21-28).
#pragma once

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../codec/pickle_codec.h"
#include "../common/buffer.h"
#include "../transport/shmring.h"
#include "../transport/zmtp.h"
#include "kernels.h"

namespace btn {
namespace gpu {

// Fixed-size pinned host slots handed to the transport as its frame
// allocator.  A slot returns to the pool when the last reference to its
// Buffer drops (after the H2D copy that reads it has completed).
class PinnedPool : public Allocator, public std::enable_shared_from_this<PinnedPool> {
 public:
  PinnedPool(size_t slot_bytes, int nslots);
  ~PinnedPool() override;
  // Blocks up to `wait_ms` for a free slot (backpressure on the IO thread),
  // then returns nullptr (heap fallback) if the pool is still dry.
  BufPtr alloc(size_t n) override;
  // A free slot now or nullptr: no wait, not counted as a fallback (the
  // worker stages a heap-received frame into it, StreamLoader::launch)
  BufPtr try_alloc(size_t n);
  void set_wait_ms(int ms) { wait_ms_ = ms; }
  size_t slot_bytes() const { return slot_bytes_; }
  int nslots() const { return nslots_; }
  int free_slots();
  uint64_t fallbacks() const { return fallbacks_.load(); }
  // Device-visible address of a host byte inside the pool (kernels may read
  // the slots directly over PCIe), or nullptr if `host` is not in the pool.
  const uint8_t* device_ptr(const uint8_t* host) const {
    if (!dev_base_ || host < base_ || host >= base_ + slot_bytes_ * size_t(nslots_)) return nullptr;
    return dev_base_ + (host - base_);
  }

 private:
  static void release(void* owner, Buffer* b);
  size_t slot_bytes_;
  int nslots_;
  uint8_t* base_ = nullptr;
  uint8_t* dev_base_ = nullptr;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<int> free_;
  std::atomic<uint64_t> fallbacks_{0};
  int wait_ms_ = 50;
};

struct LoaderConfig {
  std::vector<std::string> addresses;
  int batch_size = 8;
  std::string image_key = "image";
  int rcvhwm = 10;
  int io_threads = 1;
  int device = 0;
  int64_t max_batches = -1;          // -1: stream forever
  size_t max_frame_bytes = 0;        // 0: infer from first frame (x1.05 + 4 KiB)
  int pool_slots = 0;                // 0: auto
  int staging_depth = 3;
  bool skip_bad = false;             // drop malformed messages instead of failing
  // true: when every frame of a batch sits in device-visible pinned host
  // memory (pool slot or registered shm ring) with 16-byte alignment, the
  // decode kernel reads the frames itself over PCIe (zero-copy fused read,
  // ~45 GB/s vs ~35 GB/s for per-frame DMA copies + decode on MI355X);
  // false: always DMA into the device staging ring first.
  bool direct = true;
  // Copy path: a batch's frames are spread over this many HIP streams so
  // several DMA engines pull from host memory concurrently (1: all on the
  // loader stream).  Bounded by the runtime's hardware queues.
  int copy_streams = 2;
  // Direct-path launches queued on the loader stream before new batches wait
  // and coalesce into one launch (0: always hold until 64 images or stream end).
  int launch_depth = 2;
  // Order the loader's work against the consumer on the HOST: a posted
  // buffer is written only once the host has seen its post event complete,
  // and a batch is handed out only once the host has seen all its device
  // work (copies / kernel) complete -- no cross-stream hipStreamWaitEvent in
  // either direction.  Each such wait costs 28-430 us of host time on ROCm
  // 7 (profiles/r2/hip_api_cost.json), and issuing them per batch from the
  // loader thread held up the consumer's graph launches (~0.2 ms per step of
  // the disc consumer).  false: the GPU-side waits of round 1.
  bool host_sync = true;
  // decode parameters (src/dst/B/H/W/Cin filled per batch)
  int cout = 3;
  int cmap[4] = {0, 1, 2, 3};
  int flip_all = 0;
  int out_dtype = OUT_F32;
  int layout = NCHW;
  std::vector<float> lut;            // 4*256 floats (host)
  bool color_matrix = false;         // use the MFMA colour-transform kernel
  std::vector<float> matrix, bias;   // 16 + 4 floats
  // per-image transforms on the same kernel (photometric augmentation):
  // matrices: batch_size x (16 + 4) floats, the transform of each batch position;
  // jitter: every image draws (brightness, contrast, saturation, hue) uniformly from
  // [1 - r, 1 + r] (hue: [-r, r] turns) with a seeded splitmix64 stream in arrival
  // order, and the batch reports the factors it was decoded with
  std::vector<float> matrices;
  bool jitter = false;
  float jitter_range[4] = {0.f, 0.f, 0.f, 0.f};
  float pivot = 0.5f;
  uint64_t jitter_seed = 0;
};

// One delivered batch: metadata of each item (non-image bytes of the frame,
// re-based) and the event that completes its device work.
struct BatchMeta {
  std::vector<uint8_t> bytes;        // frame with the image payload cut out
  codec::VPtr tree;                  // parse tree over `bytes` (image entry removed)
};

// Events owned jointly by an in-flight launch (slot release) and the batches
// waiting for completion (host_sync); destroyed with the last owner.
struct EventSet {
  std::vector<hipEvent_t> ev;
  EventSet() = default;
  EventSet(const EventSet&) = delete;
  EventSet& operator=(const EventSet&) = delete;
  ~EventSet() {
    for (auto e : ev) (void)hipEventDestroy(e);
  }
  // all complete? (errors count as complete: the stream reports them later)
  bool done() const {
    for (auto e : ev)
      if (hipEventQuery(e) == hipErrorNotReady) return false;
    return true;
  }
  void wait() const {
    for (auto e : ev) (void)hipEventSynchronize(e);
  }
};

struct ReadyBatch {
  int64_t index = -1;
  std::vector<BatchMeta> items;
  hipEvent_t done = nullptr;         // GPU-side completion (host_sync = false)
  std::shared_ptr<EventSet> pending; // host-side completion (host_sync): ready once done()
  double recv_ms = 0;                // wall time spent assembling the batch
  struct SlotRef {
    shm::Segment* seg;
    uint32_t slot, gen;
  };
  std::vector<SlotRef> slots;        // host_sync: shm slots re-validated before hand-out
  int64_t launch_no = 0;             // host_sync: the launch that read them
  std::vector<float> jitter;         // colour jitter: 4 factors per image (LoaderConfig::jitter)
};

struct LoaderStats {
  uint64_t frames = 0, batches = 0, bytes = 0, bad = 0, pool_fallbacks = 0;
  uint64_t shm_frames = 0, shm_torn = 0;   // via shared memory / slot reclaimed during the copy
  uint64_t shm_stale = 0;                  // descriptors dropped: slot already reclaimed on arrival
  uint64_t direct_batches = 0;             // decoded straight from host memory (no staging copy)
  uint64_t launches = 0;                   // decode kernel launches (< batches when coalesced)
  uint64_t image_bytes = 0;                // image bytes that crossed host -> device
  uint64_t tiled_frames = 0;               // key-frame delta frames (tiledelta.h)
  double h2d_issue_ms = 0;
  // GPU time of every kTimedEvery-th launch (timing events around its H2D
  // copies + decode kernel): per-image device cost without timing every launch
  uint64_t timed_launches = 0, timed_images = 0;
  double timed_gpu_ms = 0;
  uint64_t keys_evicted = 0;               // replaced tile16 key frames freed from HBM
  // producer rings at the time of stats(): slots, frames published and not
  // yet claimed (waiting in queues), frames claimed by this loader
  uint64_t ring_slots = 0, ring_published = 0, ring_held = 0;
  uint64_t passthrough_batches = 0;        // copy path, identity decode: DMA only, no kernel
  uint64_t staged_frames = 0;              // heap-received frames copied into a pinned slot (batch kept direct)
  std::map<int64_t, uint64_t> frames_per_btid;   // provenance: frames per producer id
  // worker-thread CPU (thread clock, ms) per stage of its loop -- where the
  // consumer process's CPU per delivered frame goes: socket poll, receive +
  // descriptor parse + batch assembly, decode launches (a subset of the
  // previous), completion checks (reap + promote)
  double cpu_poll_ms = 0, cpu_recv_ms = 0, cpu_launch_ms = 0, cpu_reap_ms = 0;
  int64_t worker_tid = 0;
};

class StreamLoader {
 public:
  explicit StreamLoader(const LoaderConfig& cfg);
  ~StreamLoader();

  void start();
  // Blocks until the first frame fixed H, W, Cin (or timeout -> false).
  bool wait_shape(long timeout_ms, int* H, int* W, int* C);
  // Queue an output buffer for the next batch.  An event recorded on
  // `consumer` now is waited on by the loader stream before it writes, so
  // the caching allocator's reuse of `dst` is safe.
  void post(void* dst, hipStream_t consumer);
  // Next completed batch (in order).  Makes `consumer` wait on its event.
  // Returns false on timeout; throws std::runtime_error on a loader error
  // or when the stream is exhausted (max_batches reached -> index == -1).
  bool next(ReadyBatch* out, hipStream_t consumer, long timeout_ms);
  void stop();
  LoaderStats stats();

 private:
  struct KeyFrame;
  struct Item {
    zmtp::Frame frame;
    const uint8_t* src = nullptr;      // image bytes: in the frame or in a shm slot
    const uint8_t* dsrc = nullptr;     // device-visible alias of `src` (pinned + mapped), or null
    shm::Segment* seg = nullptr;       // shared-memory slot to hand back, if any
    uint32_t slot = 0, gen = 0;
    bool flip = false;
    // key-frame delta (csrc/codec/tiledelta.h): `src`/`dsrc` point at the
    // encoded frame (ntiles payload tiles); the key frame is at key_host (shm)
    bool tiled = false;
    int ntiles = 0;
    KeyFrame* key = nullptr;
    const uint8_t* key_host = nullptr;
    std::vector<uint8_t> expanded;     // copy path: the frame rebuilt on the host
    BufPtr staged;                     // pinned slot a heap-received image was copied into (direct path)
    float jit[4] = {1.f, 1.f, 1.f, 0.f};   // colour-jitter factors (LoaderConfig::jitter)
    BatchMeta meta;
  };
  void materialize(Item& it);
  struct Posted {
    void* dst;
    hipEvent_t ready;
  };
  void run();
  bool process(zmtp::Message&& msg);
  struct Pending {                    // assembled batch waiting for launch
    std::vector<Item> items;
    void* dst = nullptr;
    hipEvent_t ready = nullptr;
    double t0 = 0;
    bool direct = false;
    bool tiled = false;               // every image a key-frame delta: fill + tile scatter
  };
  void launch();
  void flush_pending(bool force);
  void launch_group(std::vector<Pending>& group);
  void reap(bool wait_all = false);   // release pinned slots of completed H2D copies
  void evict_keys();
  void drain_sockets();               // stop(): hand back ring slots of still-queued descriptors
  void release_descriptor(const zmtp::Message& m);   // an unprocessed descriptor: slot back to its producer

  LoaderConfig cfg_;
  std::vector<std::unique_ptr<zmtp::Context>> ctxs_;
  std::vector<std::shared_ptr<zmtp::Socket>> socks_;
  std::shared_ptr<PinnedPool> pool_;
  std::thread worker_;
  std::atomic<bool> stop_{false};
  // LoaderStats::cpu_*_ms, in ns (written by the worker, read by stats())
  enum CpuStage { kCpuPoll, kCpuRecv, kCpuLaunch, kCpuReap, kCpuStages };
  std::atomic<uint64_t> cpu_ns_[kCpuStages] = {};
  std::atomic<int64_t> worker_tid_{0};

  std::mutex mu_;
  std::condition_variable cv_;
  bool have_shape_ = false;
  int H_ = 0, W_ = 0, C_ = 0;
  size_t img_bytes_ = 0;
  std::deque<Posted> posted_;
  std::deque<ReadyBatch> ready_;
  std::string error_;
  bool exhausted_ = false;

  // worker-thread state
  hipStream_t stream_ = nullptr;
  std::vector<uint8_t*> staging_;
  float* d_lut_ = nullptr;
  float* d_mat_ = nullptr;   // 16 matrix + 4 bias (or batch_size x 20: LoaderConfig::matrices)
  uint64_t jit_state_ = 0;   // splitmix64 state of the colour-jitter draws
  std::vector<Item> cur_;
  std::deque<Pending> pending_;
  int pending_images_ = 0;
  static constexpr int kTimedEvery = 4;
  static constexpr int kTimedSkip = 8;         // cold launches never sampled
  static constexpr int64_t kKeyIdleLaunches = 64;
  int64_t launch_no_ = 0, retired_launch_ = 0;
  double last_reap_ms_ = 0;
  std::vector<hipStream_t> copy_streams_;      // copy path fan-out (cfg_.copy_streams > 1)
  std::vector<hipEvent_t> copy_done_;          // one per copy stream, reused
  std::vector<hipEvent_t> stage_free_;         // per staging buffer: last kernel reading it
  std::vector<shm::Segment*> seg_list_;        // mapped rings, for stats() (guarded by mu_)
  // the configured decode is the identity on the frame bytes (u8, NHWC, all
  // channels in order, identity table, no flip): copy-path batches are then
  // DMA'd straight into the consumer's tensor and no kernel runs at all
  bool passthrough_ = false;
  void promote_ready();                 // host_sync: completed batches -> ready_
  void host_wait(hipEvent_t ev);        // host_sync: poll an event, promoting meanwhile
  std::deque<ReadyBatch> unready_;      // host_sync: launched, device work not yet seen complete
  struct Inflight {
    int64_t launch_no = 0;
    std::shared_ptr<EventSet> copied;
    hipEvent_t t0 = nullptr, t1 = nullptr;   // sampled launch timing (or null)
    int images = 0;
    std::vector<zmtp::Frame> frames;
    struct Slot {
      shm::Segment* seg;
      uint32_t slot, gen;
    };
    std::vector<Slot> slots;
    std::vector<std::vector<uint8_t>> expanded;   // pageable copy sources, alive until `copied`
    std::vector<BufPtr> staged;                   // pinned slots of staged heap frames, alive until `copied`
  };
  struct MappedSegment {
    std::unique_ptr<shm::Segment> seg;
    uint8_t* dev_base = nullptr;   // device-visible alias of seg->base()
  };
  MappedSegment& segment(const std::string& name);
  std::map<std::string, MappedSegment> segments_;   // mapped + hipHostRegister'ed
  struct KeyFrame {
    std::unique_ptr<shm::Segment> seg;
    uint8_t* dev = nullptr;          // HBM copy, made on first use
    void* decoded[2] = {nullptr, nullptr};   // decoded for this loader (upper-left, flipped)
    int refs = 0;                    // items holding it that have not launched yet
    int64_t last_launch = 0;         // last launch that read it
  };
  KeyFrame& key_frame(const std::string& name, size_t bytes);
  const void* decoded_key(KeyFrame& kf, bool flip, size_t out_img_bytes);
  std::map<std::string, KeyFrame> keys_;
  std::deque<Inflight> inflight_;   // H2D copies not yet known complete
  int64_t batch_index_ = 0;
  double batch_t0_ = 0;
  LoaderStats stats_;
};

}  // namespace gpu
}  // namespace btn
