// Concurrency stress test of the shared-memory frame ring (shmring), built
// with ThreadSanitizer / AddressSanitizer by tests/test_sanitizers.py.
//
// P producer threads each own a segment (as each cubesim process does) and
// publish frames whose bytes are a function of (producer, sequence). They
// hand descriptors (segment, slot, generation, sequence) to C consumer threads
// through a queue that stands in for the ZMTP socket. Each consumer maps the
// segments itself (Segment::open, as the GPU loader does), claims the slot at
// the descriptor's generation (PUBLISHED -> HELD; a failed claim is a stale
// descriptor), verifies every byte, re-checks the generation (torn-read
// detection), and hands the slot back. A fraction of descriptors is dropped
// without release (a consumer that went away): the producers must recover
// those slots through the lease and keep going. Another fraction is held for
// twice the lease before it is read (a paused consumer): a held slot must
// never be reclaimed under it.
//
// Exit 0 and "verified=N corrupt=0 torn=0" when every claimed frame carried
// exactly the producer's bytes and none was taken back while held.
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include "../transport/shmring.h"

using namespace btn;

namespace {

struct Desc {
  int producer;
  uint32_t slot, gen;
  int seq;
};

std::mutex qmu;
std::condition_variable qcv;
std::deque<Desc> queue;
std::atomic<int> producers_done{0};

uint8_t pattern(int p, int seq, size_t k) { return uint8_t((k * 131 + size_t(seq) * 7 + size_t(p) * 29) & 0xff); }

}  // namespace

int main(int argc, char** argv) {
  const int P = 4, C = 3, per_producer = 400, nslots = 6;
  const size_t bytes = 20000;
  const long lease_ms = 500;
  const std::string tag = std::to_string(::getpid());
  std::vector<std::string> names;
  for (int p = 0; p < P; ++p) names.push_back("bt-stress-" + tag + "-" + std::to_string(p));
  std::vector<std::unique_ptr<shm::Segment>> segs;
  for (auto& n : names) segs.emplace_back(shm::Segment::create(n, nslots, bytes));

  std::vector<std::thread> threads;
  std::atomic<uint64_t> reclaimed{0};
  for (int p = 0; p < P; ++p)
    threads.emplace_back([&, p] {
      shm::Segment& seg = *segs[size_t(p)];
      for (int seq = 0; seq < per_producer; ++seq) {
        const int slot = seg.acquire(20000, nullptr, lease_ms);
        if (slot < 0) {
          std::fprintf(stderr, "producer %d: no slot\n", p);
          std::exit(3);
        }
        uint8_t* d = seg.slot(uint32_t(slot));
        for (size_t k = 0; k < bytes; ++k) d[k] = pattern(p, seq, k);
        const uint32_t gen = seg.publish(uint32_t(slot));
        {
          std::lock_guard<std::mutex> lk(qmu);
          queue.push_back({p, uint32_t(slot), gen, seq});
        }
        qcv.notify_one();
      }
      reclaimed += seg.reclaimed();
      producers_done++;
      qcv.notify_all();
    });

  std::atomic<int> verified{0}, corrupt{0}, stale{0}, dropped{0}, torn{0}, paused{0};
  for (int c = 0; c < C; ++c)
    threads.emplace_back([&, c] {
      std::map<int, std::unique_ptr<shm::Segment>> mapped;   // consumer-side mappings
      unsigned rnd = 12345u + unsigned(c);
      for (;;) {
        Desc d;
        {
          std::unique_lock<std::mutex> lk(qmu);
          qcv.wait(lk, [&] { return !queue.empty() || producers_done.load() == P; });
          if (queue.empty()) return;
          d = queue.front();
          queue.pop_front();
        }
        auto& m = mapped[d.producer];
        if (!m) m.reset(shm::Segment::open(names[size_t(d.producer)]));
        rnd = rnd * 1103515245u + 12345u;
        if ((rnd >> 16) % 20 == 0) {   // ~5%: message lost, slot never released
          dropped++;
          continue;
        }
        if (!m->claim(d.slot, d.gen)) {   // reclaimed while queued: drop it
          stale++;
          continue;
        }
        if ((rnd >> 16) % 50 == 1) {      // ~2%: consumer pauses past the lease
          paused++;
          std::this_thread::sleep_for(std::chrono::milliseconds(2 * lease_ms));
        }
        const uint8_t* s = m->slot(d.slot);
        bool ok = true;
        for (size_t k = 0; k < bytes; ++k) ok &= s[k] == pattern(d.producer, d.seq, k);
        if (m->valid(d.slot, d.gen)) {   // not reclaimed while we read
          if (ok) verified++;
          else corrupt++;
        } else {
          torn++;
        }
        m->release(d.slot, d.gen);
      }
    });
  for (auto& t : threads) t.join();
  std::printf("verified=%d corrupt=%d torn=%d stale=%d dropped=%d paused=%d reclaimed=%llu\n", verified.load(),
              corrupt.load(), torn.load(), stale.load(), dropped.load(), paused.load(),
              (unsigned long long)reclaimed.load());
  segs.clear();   // unlinks
  return corrupt.load() == 0 && torn.load() == 0 && verified.load() > 0 ? 0 : 1;
}
