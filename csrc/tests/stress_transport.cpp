// Concurrency stress test of the native transport + codec, built with
// -fsanitize=thread or -fsanitize=address by tests/test_sanitizers.py
// (race detection for the host runtime).
//
// N producer threads, each with its own PUSH socket (own context for half of
// them, the shared global context for the rest), stream pickled frames with
// a checksummed payload into one PULL socket whose large frames go through a
// recycling slot allocator (the same hook the GPU loader's pinned pool uses).
// A consumer thread verifies every frame; a second consumer thread polls and
// a third closes/reopens a REQ/REP pair concurrently.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../codec/pickle_codec.h"
#include "../transport/zmtp.h"

using namespace btn;

namespace {

class SlotAllocator : public Allocator {
 public:
  SlotAllocator(size_t slot, int n) : slot_(slot), mem_(slot * size_t(n)) {
    for (int i = 0; i < n; ++i) free_.push_back(i);
  }
  BufPtr alloc(size_t n) override {
    std::lock_guard<std::mutex> lk(mu_);
    if (n > slot_ || free_.empty()) {
      fallbacks++;
      return nullptr;
    }
    int id = free_.back();
    free_.pop_back();
    auto b = std::make_shared<Buffer>();
    b->data = mem_.data() + size_t(id) * slot_;
    b->capacity = slot_;
    b->tag = id;
    b->owner = this;
    b->release = [](void* o, Buffer* self) {
      auto* a = static_cast<SlotAllocator*>(o);
      std::lock_guard<std::mutex> lk(a->mu_);
      a->free_.push_back(int(self->tag));
    };
    return b;
  }
  std::atomic<int> fallbacks{0};

 private:
  size_t slot_;
  std::vector<uint8_t> mem_;
  std::mutex mu_;
  std::vector<int> free_;
};

uint64_t checksum(const uint8_t* p, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}

}  // namespace

int main(int argc, char** argv) {
  const int producers = 6, per_producer = 150;
  const int base_port = argc > 1 ? std::atoi(argv[1]) : 39100;
  const bool churn = argc > 2 && std::strcmp(argv[2], "--churn") == 0;
  std::vector<std::unique_ptr<zmtp::Context>> own;
  std::vector<std::shared_ptr<zmtp::Socket>> pushes;
  for (int p = 0; p < producers; ++p) {
    zmtp::Context* ctx = &zmtp::Context::global();
    if (p % 2) {
      own.emplace_back(new zmtp::Context());
      ctx = own.back().get();
    }
    auto s = ctx->socket(zmtp::PUSH);
    s->setsockopt(zmtp::SNDHWM, 4);
    s->setsockopt(zmtp::LINGER, 5000);
    s->bind("tcp://127.0.0.1:" + std::to_string(base_port + p));
    pushes.push_back(s);
  }
  zmtp::Context rx;
  auto pull = rx.socket(zmtp::PULL);
  pull->setsockopt(zmtp::RCVHWM, 3);
  pull->setsockopt(zmtp::RCVTIMEO, 20000);
  auto alloc = std::make_shared<SlotAllocator>(96 * 1024, 24);
  pull->set_allocator(alloc, 16 * 1024);
  for (int p = 0; p < producers; ++p) pull->connect("tcp://127.0.0.1:" + std::to_string(base_port + p));

  std::vector<std::thread> threads;
  for (int p = 0; p < producers; ++p) {
    threads.emplace_back([&, p] {
      for (int i = 0; i < per_producer; ++i) {
        const int64_t n = 1000 + (i * 7919 + p * 104729) % 60000;
        codec::Writer w(4);
        w.begin_dict();
        w.key("btid");
        w.integer(p);
        w.key("seq");
        w.integer(i);
        w.key("image");
        size_t off = w.ndarray("u1", {n});
        w.key("sum");
        size_t sum_off = w.ndarray("u8", {1});
        w.end_dict();
        auto& buf = w.finish();
        for (int64_t k = 0; k < n; ++k) buf[off + size_t(k)] = uint8_t((k * 31 + i + p) & 0xff);
        uint64_t h = checksum(buf.data() + off, size_t(n));
        std::memcpy(buf.data() + sum_off, &h, 8);
        zmtp::Message m;
        m.push_back(zmtp::Frame::copy_of(buf.data(), buf.size()));
        pushes[size_t(p)]->send(std::move(m));
      }
    });
  }
  std::atomic<bool> done{false};
  std::thread side([&] {
    // optional concurrent REQ/REP socket churn while the stream runs
    int k = 0;
    zmtp::Context c;
    while (churn && !done) {
      auto rep = c.socket(zmtp::REP);
      std::string ep = rep->bind("tcp://127.0.0.1:*");
      auto req = zmtp::Context::global().socket(zmtp::REQ);
      req->setsockopt(zmtp::RCVTIMEO, 5000);
      req->connect(ep);
      zmtp::Message m;
      m.push_back(zmtp::Frame::copy_of("ping", 4));
      req->send(std::move(m));
      auto r = rep->recv();
      rep->send(std::move(r));
      auto back = req->recv();
      if (back.size() != 1 || back[0].size != 4) {
        std::fprintf(stderr, "REQ/REP echo broken\n");
        std::exit(3);
      }
      req->close(0);
      rep->close(0);
      ++k;
    }
  });
  std::vector<int> last(producers, -1);
  int received = 0, bad = 0;
  for (int i = 0; i < producers * per_producer; ++i) {
    zmtp::Message m = pull->recv();
    auto v = codec::parse(m[0].data(), m[0].size);
    const auto* img = v->get("image");
    const auto* sum = v->get("sum");
    int p = int(v->get("btid")->i), s = int(v->get("seq")->i);
    uint64_t h;
    std::memcpy(&h, m[0].data() + sum->off, 8);
    if (checksum(m[0].data() + img->off, img->len) != h) ++bad;
    if (s != last[size_t(p)] + 1) ++bad;   // per-producer order is preserved
    last[size_t(p)] = s;
    ++received;
  }
  done = true;
  side.join();
  for (auto& t : threads) t.join();
  for (auto& s : pushes) s->close(0);
  pull->close(0);
  std::printf("received=%d bad=%d fallbacks=%d\n", received, bad, alloc->fallbacks.load());
  return bad == 0 && received == producers * per_producer ? 0 : 1;
}
