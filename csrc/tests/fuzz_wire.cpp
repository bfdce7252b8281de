// Hostile-input fuzz of the two parsers that read peer-controlled bytes,
// built with AddressSanitizer (+UBSan) by tests/test_sanitizers.py:
//
//  1. the pickle codec: valid producer frames (protocols 3-5, with and without
//     aligned payloads) mutated at random -- flipped bytes, 1/4/8-byte length
//     fields overwritten with huge or wrapping values, truncation.  parse()
//     must either throw codec::Unsupported or return a tree whose every
//     payload range lies inside the frame;
//  2. the ZMTP engine: raw TCP peers complete the handshake with a bound PULL
//     socket and then send malformed frames (zero-size commands, a name
//     length past the frame, 64-bit command / data sizes, random garbage).
//     Each offender's connection may be dropped, the process must survive,
//     and a well-behaved PUSH peer must still get its message through.
//
// Exit 0 with "codec_cases=N bad_ranges=0 wire_cases=M delivered=1".
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../codec/pickle_codec.h"
#include "../transport/zmtp.h"

using namespace btn;

namespace {

codec::Bytes frame(int protocol, size_t align, std::mt19937_64& rng) {
  codec::Writer w(protocol);
  w.begin_dict();
  w.key("btid");
  w.integer(int64_t(rng() % 100));
  w.key("image");
  const int h = 4 + int(rng() % 8), wd = 4 + int(rng() % 8), c = 3 + int(rng() % 2);
  std::vector<uint8_t> px(size_t(h * wd * c), uint8_t(rng()));
  w.ndarray("u1", {h, wd, c}, px.data(), align);
  w.key("xy");
  std::vector<double> xy(16, 0.5);
  w.ndarray("f8", {8, 2}, xy.data());
  w.key("name");
  w.str("frame");
  w.end_dict();
  return w.finish();
}

int check_ranges(const codec::Value& v, size_t n) {
  int bad = 0;
  if ((v.kind == codec::Value::BYTES || v.kind == codec::Value::NDARRAY || v.np_scalar) && !v.owned &&
      (v.off > n || v.len > n - v.off))
    ++bad;
  if (v.owned && (v.off > v.owned->size() || v.len > v.owned->size() - v.off)) ++bad;
  for (const auto& c : v.items)
    if (c) bad += check_ranges(*c, n);
  return bad;
}

void put_le(uint8_t* p, uint64_t v, int nb) {
  for (int i = 0; i < nb; ++i) p[i] = uint8_t(v >> (8 * i));
}

int fuzz_codec(int cases, int* bad_ranges) {
  std::mt19937_64 rng(1234);
  const uint64_t nasty[] = {0, 1, 0xFF, 0xFFFF, 0x7FFFFFFF, 0xFFFFFFFF, 0x7FFFFFFFFFFFFFFFull,
                            0xFFFFFFFFFFFFFFFFull, 0xFFFFFFFFFFFFFFF0ull, 0x8000000000000000ull};
  int parsed = 0;
  for (int k = 0; k < cases; ++k) {
    codec::Bytes b = frame(3 + int(rng() % 3), (rng() & 1) ? 16 : 0, rng);
    const int edits = 1 + int(rng() % 4);
    for (int e = 0; e < edits && !b.empty(); ++e) {
      const size_t at = size_t(rng() % b.size());
      switch (rng() % 4) {
        case 0: b[at] ^= uint8_t(1u << (rng() % 8)); break;
        case 1: if (at + 4 <= b.size()) put_le(&b[at], nasty[rng() % 10], 4); break;
        case 2: if (at + 8 <= b.size()) put_le(&b[at], nasty[rng() % 10], 8); break;
        default: b.resize(at); break;   // truncation
      }
    }
    try {
      codec::VPtr v = codec::parse(b.data(), b.size());
      ++parsed;
      if (v) *bad_ranges += check_ranges(*v, b.size());
    } catch (const codec::Unsupported&) {
    } catch (const std::length_error&) {   // a huge (but in-range) count refused by the allocator
    } catch (const std::bad_alloc&) {
    }
  }
  return parsed;
}

int raw_connect(int port) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(uint16_t(port));
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0) {
    ::close(fd);
    return -1;
  }
  return fd;
}

void send_all(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    ssize_t n = ::send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
    if (n <= 0) return;   // peer dropped us: expected for hostile input
    off += size_t(n);
  }
}

std::string handshake() {
  std::string g = zmtp::greeting_bytes(false);
  return g + zmtp::ready_command(zmtp::PUSH, "");
}

std::string hostile(std::mt19937_64& rng, int kind) {
  std::string s;
  auto u64be = [&](uint64_t v) {
    for (int i = 7; i >= 0; --i) s.push_back(char(v >> (8 * i)));
  };
  switch (kind) {
    case 0: s = std::string("\x04\x00", 2) + "PINGPINGPINGPING"; break;            // zero-size command
    case 1: s = std::string("\x04\x03\xc8", 3) + std::string(64, 'x'); break;      // name past the frame
    case 2: s.push_back('\x06'); u64be(0xFFFFFFFFFFFFFFFBull); s += "\x04PING" + std::string(32, '\0'); break;
    case 3: s.push_back('\x02'); u64be(uint64_t(1) << 62); s += std::string(64, '\0'); break;   // huge data frame
    case 4: s.push_back('\x06'); u64be(0); break;                                   // long command, size 0
    default:
      for (int i = 0; i < 256; ++i) s.push_back(char(rng()));                       // garbage
  }
  return s;
}

}  // namespace

int main(int argc, char** argv) {
  const int port = argc > 1 ? std::atoi(argv[1]) : 47123;
  int bad_ranges = 0;
  const int codec_cases = 20000;
  fuzz_codec(codec_cases, &bad_ranges);

  zmtp::Context ctx;
  auto pull = ctx.socket(zmtp::PULL);
  pull->setsockopt(zmtp::RCVTIMEO, 3000);
  pull->bind("tcp://127.0.0.1:" + std::to_string(port));
  std::mt19937_64 rng(99);
  int wire_cases = 0;
  for (int round = 0; round < 8; ++round)
    for (int kind = 0; kind < 6; ++kind) {
      int fd = raw_connect(port);
      if (fd < 0) continue;
      send_all(fd, handshake());
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
      send_all(fd, hostile(rng, kind));
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
      ::close(fd);
      ++wire_cases;
    }
  // a well-behaved peer still gets through
  auto push = ctx.socket(zmtp::PUSH);
  push->connect("tcp://127.0.0.1:" + std::to_string(port));
  zmtp::Message m;
  m.push_back(zmtp::Frame::copy_of("still-alive", 11));
  push->send(std::move(m));
  // (random garbage may well contain complete, legal data frames: those are
  // delivered like any message and skipped here)
  int delivered = 0;
  try {
    for (int n = 0; n < 1000 && !delivered; ++n) {
      zmtp::Message r = pull->recv();
      delivered = r.size() == 1 && r[0].size == 11 && std::memcmp(r[0].data(), "still-alive", 11) == 0;
    }
  } catch (const zmtp::Error&) {
  }
  push->close(0);
  pull->close(0);
  std::printf("codec_cases=%d bad_ranges=%d wire_cases=%d delivered=%d\n", codec_cases, bad_ranges, wire_cases,
              delivered);
  return bad_ranges == 0 && delivered == 1 ? 0 : 1;
}
