// Same-host zero-copy frame slots in POSIX shared memory.
//
// A producer that runs on the consumer's host can place its large payloads
// (rendered images) in a shared-memory ring instead of pushing the bytes
// through a socket: it renders straight into a free slot and sends only a
// small descriptor over the normal ZMTP socket (key "_btshm" in the message
// dict: (segment name, slot, byte offset, H, W, C, image key)).  The GPU
// loader maps the segment once, registers it as pinned host memory with the
// HIP runtime, DMAs the image out of the slot in place and hands the slot
// back; the CPU dataset path copies the image out and hands it back.  This
// removes both kernel socket copies of every frame.
//
// Layout: [Header | word[nslots] (uint32) | pad to 4 KiB | slot 0 | slot 1 ...]
// Slot word = generation << 2 | state.  States: FREE (0) -> WRITING (1,
// producer) -> PUBLISHED (2, generation bumped) -> HELD (3, a consumer took
// the descriptor: CAS on the exact published word) -> FREE (consumer, after
// its last read of the slot completed).  Descriptors carry the generation, so
// a consumer can tell whether a slot was reclaimed before it claimed it.
// Lease: a message dropped without being consumed (a consumer that died with
// frames still queued) would pin its slot forever; when the producer has
// found no free slot for `lease_ms`, it reclaims the longest-PUBLISHED slot
// (counted in reclaimed()).  A claimed (HELD) slot is never taken back while
// its consumer may still read it -- a paused consumer (eval pass, checkpoint,
// breakpoint) only stalls the producer, exactly like a full SNDHWM -- unless
// the stall lasts kHeldLeaseFactor x lease_ms (a consumer that died holding
// slots); the consumer then sees valid() fail and reports the batch torn.
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace btn {
namespace shm {

constexpr uint64_t kMagic = 0x6d68735f7462746eull;   // "ntbt_shm"
enum SlotState : uint32_t { FREE = 0, WRITING = 1, PUBLISHED = 2, HELD = 3 };
constexpr long kHeldLeaseFactor = 20;

struct Header {
  uint64_t magic;
  uint32_t version;
  uint32_t nslots;
  uint64_t slot_bytes;
  uint64_t data_offset;
};

class Segment {
 public:
  // Producer: create (and own / unlink on destruction) a new segment.
  static Segment* create(const std::string& name, uint32_t nslots, size_t slot_bytes);
  // Consumer: map an existing segment.
  static Segment* open(const std::string& name);
  ~Segment();

  const std::string& name() const { return name_; }
  uint32_t nslots() const { return hdr_->nslots; }
  size_t slot_bytes() const { return hdr_->slot_bytes; }
  uint8_t* base() const { return base_; }
  size_t size() const { return size_; }
  uint8_t* slot(uint32_t i) const { return base_ + hdr_->data_offset + size_t(i) * hdr_->slot_bytes; }
  size_t slot_offset(uint32_t i) const { return hdr_->data_offset + size_t(i) * hdr_->slot_bytes; }

  // Producer: claim a FREE slot, waiting up to timeout_ms (-1 forever);
  // returns -1 on timeout or when `stop` becomes true.
  int acquire(long timeout_ms, const std::atomic<bool>* stop = nullptr, long lease_ms = 30000);
  uint32_t publish(uint32_t i);        // returns the slot's new generation
  // Consumer: take the descriptor's slot (PUBLISHED -> HELD).  False when the
  // producer reclaimed it first: the descriptor is stale and must be dropped.
  bool claim(uint32_t i, uint32_t gen);
  // Consumer: hand a slot back, claimed or not (no-op if it was reclaimed meanwhile).
  void release(uint32_t i, uint32_t gen);
  // Consumer: is the slot still holding generation `gen` (published or held)?
  bool valid(uint32_t i, uint32_t gen) const;
  uint32_t count(SlotState st) const;   // slots currently in state `st`
  uint32_t state(uint32_t i) const;
  uint32_t free_count() const;
  uint64_t reclaimed() const { return reclaimed_; }

 private:
  Segment() = default;
  std::atomic<uint32_t>* states() const;
  std::string name_;
  int fd_ = -1;
  uint8_t* base_ = nullptr;
  size_t size_ = 0;
  Header* hdr_ = nullptr;
  bool owner_ = false;
  uint32_t next_ = 0;
  uint64_t reclaimed_ = 0;
  std::vector<int64_t> published_at_;   // producer-private publish times (us)
};

}  // namespace shm
}  // namespace btn
