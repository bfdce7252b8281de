// Native ZMTP/3.0 engine -- see zmtp.h for the design notes.
#include "zmtp.h"

#include <pthread.h>

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <future>
#include <random>
#include <sstream>

namespace btn {
namespace zmtp {

using Clock = std::chrono::steady_clock;

// --------------------------------------------------------------------------
// Wire helpers
// --------------------------------------------------------------------------
enum : uint8_t { F_MORE = 1, F_LONG = 2, F_COMMAND = 4 };

const char* socket_type_name(int type) {
  switch (type) {
    case PAIR: return "PAIR";
    case PUB: return "PUB";
    case SUB: return "SUB";
    case REQ: return "REQ";
    case REP: return "REP";
    case DEALER: return "DEALER";
    case ROUTER: return "ROUTER";
    case PULL: return "PULL";
    case PUSH: return "PUSH";
  }
  return "UNKNOWN";
}

static int socket_type_from_name(const std::string& n) {
  static const char* names[] = {"PAIR", "PUB", "SUB", "REQ", "REP",
                                "DEALER", "ROUTER", "PULL", "PUSH"};
  for (int i = 0; i < 9; ++i)
    if (n == names[i]) return i;
  return -1;
}

bool socket_types_compatible(int a, int b) {
  switch (a) {
    case PAIR: return b == PAIR;
    case PUB: return b == SUB;
    case SUB: return b == PUB;
    case REQ: return b == REP || b == ROUTER;
    case REP: return b == REQ || b == DEALER;
    case DEALER: return b == REP || b == DEALER || b == ROUTER;
    case ROUTER: return b == REQ || b == DEALER || b == ROUTER;
    case PULL: return b == PUSH;
    case PUSH: return b == PULL;
  }
  return false;
}

std::string greeting_bytes(bool as_server) {
  std::string g(64, '\0');
  g[0] = '\xff';
  g[9] = '\x7f';
  g[10] = 3;   // major
  g[11] = 0;   // minor: ZMTP 3.0 (libzmq 4.x peers negotiate down to it)
  std::memcpy(&g[12], "NULL", 4);
  g[32] = as_server ? 1 : 0;
  return g;
}

static void put_u32be(std::string& s, uint32_t v) {
  s.push_back(char((v >> 24) & 0xff));
  s.push_back(char((v >> 16) & 0xff));
  s.push_back(char((v >> 8) & 0xff));
  s.push_back(char(v & 0xff));
}

static std::string encode_command(const std::string& name, const std::string& body) {
  std::string payload;
  payload.push_back(char(name.size()));
  payload += name;
  payload += body;
  std::string out;
  if (payload.size() > 255) {
    out.push_back(char(F_COMMAND | F_LONG));
    uint64_t n = payload.size();
    for (int i = 7; i >= 0; --i) out.push_back(char((n >> (8 * i)) & 0xff));
  } else {
    out.push_back(char(F_COMMAND));
    out.push_back(char(payload.size()));
  }
  return out + payload;
}

std::string ready_command(int socket_type, const std::string& identity) {
  std::string props;
  auto prop = [&](const std::string& k, const std::string& v) {
    props.push_back(char(k.size()));
    props += k;
    put_u32be(props, uint32_t(v.size()));
    props += v;
  };
  prop("Socket-Type", socket_type_name(socket_type));
  if (socket_type == REQ || socket_type == DEALER || socket_type == ROUTER)
    prop("Identity", identity);
  return encode_command("READY", props);
}

static size_t frame_header(uint8_t* hdr, size_t size, bool more) {
  if (size > 255) {
    hdr[0] = uint8_t(F_LONG | (more ? F_MORE : 0));
    uint64_t n = size;
    for (int i = 0; i < 8; ++i) hdr[1 + i] = uint8_t((n >> (8 * (7 - i))) & 0xff);
    return 9;
  }
  hdr[0] = uint8_t(more ? F_MORE : 0);
  hdr[1] = uint8_t(size);
  return 2;
}

Frame Frame::copy_of(const void* p, size_t n) {
  Frame f;
  f.buf = heap_buffer(n);
  if (n) std::memcpy(f.buf->data, p, n);
  f.size = n;
  return f;
}

Frame Frame::empty() { return copy_of(nullptr, 0); }

// --------------------------------------------------------------------------
// Endpoint parsing
// --------------------------------------------------------------------------
std::string Endpoint::str() const {
  if (kind == IPC) return "ipc://" + host;
  return "tcp://" + host + ":" + std::to_string(port);
}

Endpoint Endpoint::parse(const std::string& addr) {
  Endpoint ep;
  auto pos = addr.find("://");
  if (pos == std::string::npos) throw Error(E_INVAL, "invalid endpoint: " + addr);
  std::string proto = addr.substr(0, pos), rest = addr.substr(pos + 3);
  if (proto == "ipc") {
    ep.kind = IPC;
    ep.host = rest;
    return ep;
  }
  if (proto != "tcp") throw Error(E_INVAL, "unsupported transport: " + proto);
  auto c = rest.rfind(':');
  if (c == std::string::npos) throw Error(E_INVAL, "missing port: " + addr);
  ep.host = rest.substr(0, c);
  std::string port = rest.substr(c + 1);
  if (!ep.host.empty() && ep.host.front() == '[' && ep.host.back() == ']')
    ep.host = ep.host.substr(1, ep.host.size() - 2);
  ep.port = (port == "*" || port == "0") ? -1 : std::stoi(port);
  return ep;
}

struct SockAddr {
  sockaddr_storage ss{};
  socklen_t len = 0;
  int family = AF_INET;
};

static SockAddr resolve(const Endpoint& ep, bool for_bind) {
  SockAddr sa;
  if (ep.kind == Endpoint::IPC) {
    auto* un = reinterpret_cast<sockaddr_un*>(&sa.ss);
    un->sun_family = AF_UNIX;
    if (ep.host.size() >= sizeof(un->sun_path)) throw Error(E_INVAL, "ipc path too long");
    std::memcpy(un->sun_path, ep.host.data(), ep.host.size());
    if (!ep.host.empty() && ep.host[0] == '@') un->sun_path[0] = '\0';  // abstract
    sa.len = socklen_t(offsetof(sockaddr_un, sun_path) + ep.host.size() +
                       (ep.host[0] == '@' ? 0 : 1));
    sa.family = AF_UNIX;
    return sa;
  }
  std::string host = ep.host;
  int port = ep.port < 0 ? 0 : ep.port;
  if (host == "*" || host.empty()) {
    auto* in = reinterpret_cast<sockaddr_in*>(&sa.ss);
    in->sin_family = AF_INET;
    in->sin_addr.s_addr = htonl(INADDR_ANY);
    in->sin_port = htons(uint16_t(port));
    sa.len = sizeof(sockaddr_in);
    return sa;
  }
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  if (for_bind) hints.ai_flags = AI_PASSIVE;
  int rc = getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res);
  if (rc != 0 || !res) throw Error(E_HOSTUNREACH, "cannot resolve host " + host);
  std::memcpy(&sa.ss, res->ai_addr, res->ai_addrlen);
  sa.len = socklen_t(res->ai_addrlen);
  sa.family = res->ai_family;
  freeaddrinfo(res);
  return sa;
}

// --------------------------------------------------------------------------
// Pipe: one stream connection to a peer
// --------------------------------------------------------------------------
struct Pipe : std::enable_shared_from_this<Pipe> {
  enum State { IDLE, CONNECTING, HANDSHAKE, ACTIVE, DEAD };

  Context* ctx = nullptr;
  std::weak_ptr<Socket> sock;
  int fd = -1;
  bool outbound = false;   // created by connect()
  Endpoint ep;
  SockAddr addr;
  std::atomic<State> state{IDLE};   // written by the IO thread, read by senders
  bool attached = false;   // member of Socket::pipes_ (mu_)
  bool gone = false;       // permanently finished (mu_)
  uint64_t id = 0;
  std::string router_id;   // ROUTER routing identity

  // handshake
  std::string hs_out;
  size_t hs_off = 0;
  uint8_t greet_in[64];
  size_t greet_got = 0;
  bool ready_in = false;
  int peer_type = -1;
  std::string peer_identity;

  // read path (IO thread)
  std::vector<uint8_t> rbuf = std::vector<uint8_t>(128 * 1024);
  size_t rpos = 0, rlen = 0;
  BufPtr body;
  size_t body_size = 0, body_got = 0;
  bool body_more = false;
  Message partial;
  bool read_paused = false;    // mu_
  bool resume_posted = false;  // mu_

  // queues (mu_)
  std::deque<Message> inq;
  std::deque<Message> outq;
  bool write_scheduled = false;  // mu_
  bool wactive = false;          // mu_ (an in-flight message exists)

  // write path (IO thread)
  Message wmsg;
  size_t wframe = 0, woff = 0;   // woff counts header+body bytes of wframe
  uint8_t whdr[9];
  size_t whdr_len = 0;
  bool epollout = false;
  uint32_t cur_events = 0;
  bool registered = false;
};

static std::atomic<uint64_t> g_pipe_ids{1};

// --------------------------------------------------------------------------
// PollHub
// --------------------------------------------------------------------------
void PollHub::bump() {
  {
    std::lock_guard<std::mutex> lk(mu);
    ++generation;
  }
  cv.notify_all();
}

PollHub& PollHub::instance() {
  static PollHub* hub = new PollHub();
  return *hub;
}

// --------------------------------------------------------------------------
// Context
// --------------------------------------------------------------------------
Context::Context() {
  epfd_ = epoll_create1(EPOLL_CLOEXEC);
  evfd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (epfd_ < 0 || evfd_ < 0) throw Error(errno, "epoll/eventfd failed");
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = evfd_;
  epoll_ctl(epfd_, EPOLL_CTL_ADD, evfd_, &ev);
  running_ = true;
  thread_ = std::thread([this] {
    pthread_setname_np(pthread_self(), "bt-zmtp-io");   // per-thread CPU reports (bench.py)
    loop();
  });
}

Context::~Context() { term(); }

Context& Context::global() {
  // Intentionally leaked: sockets may outlive static destruction order.
  static Context* ctx = new Context();
  return *ctx;
}

std::shared_ptr<Socket> Context::socket(int type) {
  if (!running_) throw Error(E_TERM, "context terminated");
  auto s = std::make_shared<Socket>(this, type);
  std::lock_guard<std::mutex> lk(sockets_mu_);
  sockets_.push_back(s);
  return s;
}

void Context::term() {
  if (!running_) return;
  std::vector<std::shared_ptr<Socket>> live;
  {
    std::lock_guard<std::mutex> lk(sockets_mu_);
    for (auto& w : sockets_)
      if (auto s = w.lock()) live.push_back(s);
    sockets_.clear();
  }
  for (auto& s : live)
    if (!s->closed()) s->close(-2);
  running_ = false;
  wake();
  if (thread_.joinable()) thread_.join();
  if (epfd_ >= 0) ::close(epfd_);
  if (evfd_ >= 0) ::close(evfd_);
  epfd_ = evfd_ = -1;
}

bool Context::on_io_thread() const { return std::this_thread::get_id() == thread_id_.load(std::memory_order_acquire); }

void Context::wake() {
  uint64_t one = 1;
  ssize_t r = ::write(evfd_, &one, sizeof(one));
  (void)r;
}

void Context::post(std::function<void()> fn) {
  {
    std::lock_guard<std::mutex> lk(cmd_mu_);
    cmds_.push_back(std::move(fn));
  }
  wake();
}

void Context::post_sync(std::function<void()> fn) {
  if (on_io_thread()) {
    fn();
    return;
  }
  auto done = std::make_shared<std::promise<void>>();
  auto fut = done->get_future();
  post([fn, done] {
    fn();
    done->set_value();
  });
  fut.wait();
}

void Context::loop() {
  thread_id_.store(std::this_thread::get_id(), std::memory_order_release);
  std::vector<epoll_event> evs(256);
  while (running_) {
    int timeout = 1000;
    auto now = Clock::now();
    for (auto& t : timers_) {
      auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(t.at - now).count();
      timeout = std::max<int>(0, std::min<int>(timeout, int(ms)));
    }
    int n = epoll_wait(epfd_, evs.data(), int(evs.size()), timeout);
    if (n < 0 && errno != EINTR) break;
    for (int i = 0; i < n; ++i) {
      int fd = evs[i].data.fd;
      uint32_t e = evs[i].events;
      if (fd == evfd_) {
        uint64_t v;
        while (::read(evfd_, &v, sizeof(v)) > 0) {
        }
        continue;
      }
      auto li = listeners_.find(fd);
      if (li != listeners_.end()) {
        handle_accept(fd);
        continue;
      }
      auto pi = fd_pipes_.find(fd);
      if (pi == fd_pipes_.end()) continue;
      auto p = pi->second;
      if (p->state == Pipe::CONNECTING) {
        if (e & (EPOLLOUT | EPOLLERR | EPOLLHUP)) io_connected(p);
        continue;
      }
      if (e & (EPOLLIN | EPOLLERR | EPOLLHUP)) io_read(p);
      if (p->fd >= 0 && p->state != Pipe::DEAD && (e & EPOLLOUT)) io_write(p);
    }
    // commands
    std::vector<std::function<void()>> cmds;
    {
      std::lock_guard<std::mutex> lk(cmd_mu_);
      cmds.swap(cmds_);
    }
    for (auto& c : cmds) c();
    // timers
    if (!timers_.empty()) {
      now = Clock::now();
      std::vector<Timer> due, keep;
      for (auto& t : timers_) (t.at <= now ? due : keep).push_back(t);
      timers_.swap(keep);
      for (auto& t : due)
        if (t.pipe->state == Pipe::IDLE) start_connect(t.pipe);
    }
  }
  // Drain remaining commands so post_sync callers never hang.
  std::vector<std::function<void()>> cmds;
  {
    std::lock_guard<std::mutex> lk(cmd_mu_);
    cmds.swap(cmds_);
  }
  for (auto& c : cmds) c();
  for (auto& kv : listeners_) ::close(kv.first);
  listeners_.clear();
  for (auto& kv : fd_pipes_) ::close(kv.first);
  fd_pipes_.clear();
}

void Context::add_listener(int fd, Endpoint ep, std::shared_ptr<Socket> s) {
  Listener l{fd, ep, s};
  listeners_[fd] = l;
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = fd;
  epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev);
}

void Context::remove_listeners_of(Socket* s, const std::string* only_ep) {
  for (auto it = listeners_.begin(); it != listeners_.end();) {
    auto sp = it->second.sock.lock();
    bool mine = !sp || sp.get() == s;
    if (mine && (!only_ep || it->second.ep.str() == *only_ep)) {
      epoll_ctl(epfd_, EPOLL_CTL_DEL, it->first, nullptr);
      ::close(it->first);
      if (it->second.ep.kind == Endpoint::IPC && !it->second.ep.host.empty() &&
          it->second.ep.host[0] != '@')
        ::unlink(it->second.ep.host.c_str());
      it = listeners_.erase(it);
    } else {
      ++it;
    }
  }
}

static void tune_fd(int fd, bool tcp, int sndkb, int rcvkb) {
  if (tcp) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  }
  if (sndkb > 0) {
    int v = sndkb * 1024;
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &v, sizeof(v));
  }
  if (rcvkb > 0) {
    int v = rcvkb * 1024;
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &v, sizeof(v));
  }
}

void Context::register_pipe(const std::shared_ptr<Pipe>& p, uint32_t events) {
  epoll_event ev{};
  ev.events = events;
  ev.data.fd = p->fd;
  if (p->registered)
    epoll_ctl(epfd_, EPOLL_CTL_MOD, p->fd, &ev);
  else
    epoll_ctl(epfd_, EPOLL_CTL_ADD, p->fd, &ev);
  p->registered = true;
  p->cur_events = events;
  fd_pipes_[p->fd] = p;
}

void Context::update_pipe_events(Pipe* p) {
  if (p->fd < 0 || !p->registered) return;
  uint32_t ev = 0;
  bool paused;
  {
    auto s = p->sock.lock();
    if (s) {
      std::lock_guard<std::mutex> lk(s->mu_);
      paused = p->read_paused;
    } else {
      paused = false;
    }
  }
  if (p->state == Pipe::CONNECTING) {
    ev = EPOLLOUT;
  } else {
    if (!paused) ev |= EPOLLIN;
    if (p->epollout) ev |= EPOLLOUT;
  }
  if (ev == p->cur_events) return;
  epoll_event e{};
  e.events = ev;
  e.data.fd = p->fd;
  epoll_ctl(epfd_, EPOLL_CTL_MOD, p->fd, &e);
  p->cur_events = ev;
}

void Context::handle_accept(int lfd) {
  auto& l = listeners_[lfd];
  auto s = l.sock.lock();
  for (;;) {
    int fd = accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (fd < 0) break;
    if (!s || s->closing_) {
      ::close(fd);
      continue;
    }
    tune_fd(fd, l.ep.kind == Endpoint::TCP, s->sndbuf_kb_, s->rcvbuf_kb_);
    auto p = std::make_shared<Pipe>();
    p->ctx = this;
    p->sock = s;
    p->fd = fd;
    p->outbound = false;
    p->ep = l.ep;
    p->id = g_pipe_ids++;
    p->state = Pipe::HANDSHAKE;
    p->hs_out = greeting_bytes(false) + ready_command(s->type_, s->identity_);
    register_pipe(p, EPOLLIN | EPOLLOUT);
    p->epollout = true;
  }
}

void Context::start_connect(const std::shared_ptr<Pipe>& p) {
  auto s = p->sock.lock();
  if (!s || s->closing_ || p->gone) return;
  int fd = ::socket(p->addr.family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0) {
    schedule_reconnect(p);
    return;
  }
  tune_fd(fd, p->ep.kind == Endpoint::TCP, s->sndbuf_kb_, s->rcvbuf_kb_);
  int rc = ::connect(fd, reinterpret_cast<sockaddr*>(&p->addr.ss), p->addr.len);
  if (rc < 0 && errno != EINPROGRESS) {
    ::close(fd);
    schedule_reconnect(p);
    return;
  }
  p->fd = fd;
  p->state = Pipe::CONNECTING;
  p->registered = false;
  register_pipe(p, EPOLLOUT);
  if (rc == 0) io_connected(p);
}

void Context::schedule_reconnect(const std::shared_ptr<Pipe>& p) {
  auto s = p->sock.lock();
  if (!s || s->closing_ || p->gone) return;
  p->state = Pipe::IDLE;
  int ivl = std::max(1, s->reconnect_ivl_);
  timers_.push_back({Clock::now() + std::chrono::milliseconds(ivl), p});
}

void Context::io_connected(const std::shared_ptr<Pipe>& p) {
  int err = 0;
  socklen_t len = sizeof(err);
  getsockopt(p->fd, SOL_SOCKET, SO_ERROR, &err, &len);
  if (err != 0) {
    epoll_ctl(epfd_, EPOLL_CTL_DEL, p->fd, nullptr);
    fd_pipes_.erase(p->fd);
    ::close(p->fd);
    p->fd = -1;
    p->registered = false;
    schedule_reconnect(p);
    return;
  }
  auto s = p->sock.lock();
  if (!s) {
    close_pipe(p, false);
    return;
  }
  p->state = Pipe::HANDSHAKE;
  p->hs_out = greeting_bytes(false) + ready_command(s->type_, s->identity_);
  p->hs_off = 0;
  p->greet_got = 0;
  p->ready_in = false;
  p->rpos = p->rlen = 0;
  p->body.reset();
  p->partial.clear();
  p->epollout = true;
  update_pipe_events(p.get());
  io_write(p);
}

void Context::close_pipe(const std::shared_ptr<Pipe>& p, bool allow_reconnect) {
  if (p->fd >= 0) {
    if (p->registered) epoll_ctl(epfd_, EPOLL_CTL_DEL, p->fd, nullptr);
    fd_pipes_.erase(p->fd);
    ::shutdown(p->fd, SHUT_RDWR);
    ::close(p->fd);
    p->fd = -1;
  }
  p->registered = false;
  p->epollout = false;
  p->body.reset();
  p->partial.clear();
  p->rpos = p->rlen = 0;
  auto s = p->sock.lock();
  bool reconnect = allow_reconnect && p->outbound && s && !s->closing_ && !p->gone;
  if (s) {
    std::lock_guard<std::mutex> lk(s->mu_);
    if (p->wactive) {
      // restart the interrupted message after reconnect (at-least-once)
      if (reconnect) p->outq.push_front(std::move(p->wmsg));
      p->wmsg.clear();
      p->wactive = false;
    }
    p->write_scheduled = false;
    p->read_paused = false;
    p->resume_posted = false;
    if (!reconnect || s->immediate_) {
      if (!reconnect) {
        p->outq.clear();
        p->gone = true;
        p->state = Pipe::DEAD;
      }
      if (p->attached && p->inq.empty()) s->detach_pipe_locked(p.get());
    }
    s->cv_.notify_all();
  }
  PollHub::instance().bump();
  if (reconnect) {
    p->state = Pipe::IDLE;
    schedule_reconnect(p);
  } else {
    p->state = Pipe::DEAD;
  }
}

void Context::io_write(const std::shared_ptr<Pipe>& p) {
  auto s = p->sock.lock();
  if (!s || p->fd < 0) return;
  // 1) handshake bytes
  while (p->hs_off < p->hs_out.size()) {
    ssize_t n = ::send(p->fd, p->hs_out.data() + p->hs_off, p->hs_out.size() - p->hs_off,
                       MSG_NOSIGNAL);
    if (n < 0) {
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        if (!p->epollout) {
          p->epollout = true;
          update_pipe_events(p.get());
        }
        return;
      }
      close_pipe(p, true);
      return;
    }
    p->hs_off += size_t(n);
  }
  if (p->state != Pipe::ACTIVE) {
    if (p->epollout) {
      p->epollout = false;
      update_pipe_events(p.get());
    }
    return;
  }
  // 2) data messages
  for (int rounds = 0; rounds < 64; ++rounds) {
    if (!p->wmsg.size()) {
      std::lock_guard<std::mutex> lk(s->mu_);
      if (p->outq.empty()) {
        p->write_scheduled = false;
        p->wactive = false;
        break;
      }
      p->wmsg = std::move(p->outq.front());
      p->outq.pop_front();
      p->wactive = true;
      p->wframe = 0;
      p->woff = 0;
      // space became available for blocked senders
      s->cv_.notify_all();
      PollHub::instance().bump();
    }
    // gather iovecs for the rest of this message
    iovec iov[64];
    uint8_t hdrs[32][9];
    int niov = 0;
    int k = 0;
    for (size_t f = p->wframe; f < p->wmsg.size() && niov < 62 && k < 32; ++f, ++k) {
      const Frame& fr = p->wmsg[f];
      size_t hl = frame_header(hdrs[k], fr.size, f + 1 < p->wmsg.size());
      size_t skip = (f == p->wframe) ? p->woff : 0;
      if (skip < hl) {
        iov[niov++] = {hdrs[k] + skip, hl - skip};
        if (fr.size) iov[niov++] = {const_cast<uint8_t*>(fr.data()), fr.size};
      } else {
        size_t off = skip - hl;
        if (fr.size > off) iov[niov++] = {const_cast<uint8_t*>(fr.data()) + off, fr.size - off};
      }
    }
    msghdr mh{};
    mh.msg_iov = iov;
    mh.msg_iovlen = size_t(niov);
    ssize_t n = niov ? ::sendmsg(p->fd, &mh, MSG_NOSIGNAL) : 0;
    if (n < 0) {
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        if (!p->epollout) {
          p->epollout = true;
          update_pipe_events(p.get());
        }
        return;
      }
      close_pipe(p, true);
      return;
    }
    // advance
    size_t adv = size_t(n) + p->woff;
    size_t f = p->wframe;
    while (f < p->wmsg.size()) {
      uint8_t tmp[9];
      size_t total = frame_header(tmp, p->wmsg[f].size, f + 1 < p->wmsg.size()) + p->wmsg[f].size;
      if (adv >= total) {
        adv -= total;
        ++f;
      } else {
        break;
      }
    }
    p->wframe = f;
    p->woff = adv;
    if (f >= p->wmsg.size()) {
      size_t bytes = 0;
      for (auto& fr : p->wmsg) bytes += fr.size;
      p->wmsg.clear();
      std::lock_guard<std::mutex> lk(s->mu_);
      p->wactive = false;
      s->stats_.msgs_out++;
      s->stats_.bytes_out += bytes;
      s->cv_.notify_all();
    } else {
      // partial write: wait for EPOLLOUT
      if (!p->epollout) {
        p->epollout = true;
        update_pipe_events(p.get());
      }
      return;
    }
  }
  bool more;
  {
    std::lock_guard<std::mutex> lk(s->mu_);
    more = !p->outq.empty();
    if (more) p->write_scheduled = true;
  }
  if (more) {
    // yield to other pipes; continue on next loop iteration
    auto self = p;
    post([this, self] { io_write(self); });
  } else if (p->epollout) {
    p->epollout = false;
    update_pipe_events(p.get());
  }
}

// Parses the peer's READY command; returns false on protocol violation.
static bool parse_ready(Pipe* p, const uint8_t* d, size_t n) {
  size_t i = 0;
  while (i < n) {
    size_t kl = d[i++];
    if (i + kl + 4 > n) return false;
    std::string k(reinterpret_cast<const char*>(d + i), kl);
    i += kl;
    uint32_t vl = (uint32_t(d[i]) << 24) | (uint32_t(d[i + 1]) << 16) |
                  (uint32_t(d[i + 2]) << 8) | uint32_t(d[i + 3]);
    i += 4;
    if (i + vl > n) return false;
    std::string v(reinterpret_cast<const char*>(d + i), vl);
    i += vl;
    std::string kk = k;
    std::transform(kk.begin(), kk.end(), kk.begin(), ::tolower);
    if (kk == "socket-type") p->peer_type = socket_type_from_name(v);
    if (kk == "identity") p->peer_identity = v;
  }
  return true;
}

void Context::io_read(const std::shared_ptr<Pipe>& p) {
  auto s = p->sock.lock();
  if (!s) {
    close_pipe(p, false);
    return;
  }
  size_t budget_frames = 64, budget_bytes = 16u << 20;
  for (;;) {
    if (p->fd < 0) return;
    // direct body read for large frames
    if (p->body) {
      ssize_t n = ::recv(p->fd, p->body->data + p->body_got, p->body_size - p->body_got, 0);
      if (n == 0) {
        close_pipe(p, true);
        return;
      }
      if (n < 0) {
        if (errno == EAGAIN || errno == EWOULDBLOCK) return;
        close_pipe(p, true);
        return;
      }
      p->body_got += size_t(n);
      if (budget_bytes > size_t(n)) budget_bytes -= size_t(n); else budget_bytes = 0;
      if (p->body_got < p->body_size) continue;
      Frame fr;
      fr.buf = std::move(p->body);
      fr.size = p->body_size;
      p->body.reset();
      p->partial.push_back(std::move(fr));
      if (!p->body_more) goto deliver;
      continue;
    }
    {
      size_t avail = p->rlen - p->rpos;
      // Decide how many bytes the next parse step needs.
      size_t need;
      if (p->state == Pipe::HANDSHAKE && p->greet_got < 64) {
        need = 1;
      } else if (avail >= 1) {
        need = (p->rbuf[p->rpos] & F_LONG) ? 9 : 2;
        if (avail >= need) {
          const uint8_t* h = &p->rbuf[p->rpos];
          uint64_t sz = 0;
          if (h[0] & F_LONG) {
            for (int i = 0; i < 8; ++i) sz = (sz << 8) | h[1 + i];
          } else {
            sz = h[1];
          }
          if (h[0] & F_COMMAND) {             // commands must be whole in rbuf
            if (sz > (64u << 20)) {            // (and a 64-bit size must not wrap `need`)
              close_pipe(p, true);
              return;
            }
            need += sz;
          }
        }
      } else {
        need = 1;
      }
      if (need > p->rbuf.size()) {
        if (need > (64u << 20)) {
          close_pipe(p, true);
          return;
        }
        p->rbuf.resize(need);
      }
      if (avail < need) {
        if (p->rpos > 0) {
          std::memmove(p->rbuf.data(), p->rbuf.data() + p->rpos, avail);
          p->rpos = 0;
          p->rlen = avail;
        }
        ssize_t n = ::recv(p->fd, p->rbuf.data() + p->rlen, p->rbuf.size() - p->rlen, 0);
        if (n == 0) {
          close_pipe(p, true);
          return;
        }
        if (n < 0) {
          if (errno == EAGAIN || errno == EWOULDBLOCK) return;
          close_pipe(p, true);
          return;
        }
        p->rlen += size_t(n);
        continue;
      }
      // --- greeting ---
      if (p->state == Pipe::HANDSHAKE && p->greet_got < 64) {
        size_t take = std::min(avail, 64 - p->greet_got);
        std::memcpy(p->greet_in + p->greet_got, &p->rbuf[p->rpos], take);
        p->greet_got += take;
        p->rpos += take;
        if (p->greet_got >= 10 && (p->greet_in[0] != 0xff || p->greet_in[9] != 0x7f)) {
          close_pipe(p, false);
          return;
        }
        if (p->greet_got == 64) {
          if (p->greet_in[10] < 3 || std::memcmp(p->greet_in + 12, "NULL", 4) != 0) {
            close_pipe(p, false);
            return;
          }
        }
        continue;
      }
      // --- frame ---
      const uint8_t* h = &p->rbuf[p->rpos];
      uint8_t flags = h[0];
      size_t hl = (flags & F_LONG) ? 9 : 2;
      uint64_t sz = 0;
      if (flags & F_LONG) {
        for (int i = 0; i < 8; ++i) sz = (sz << 8) | h[1 + i];
      } else {
        sz = h[1];
      }
      if (flags & F_COMMAND) {
        const uint8_t* c = h + hl;
        // a command is name-length byte + name + body: reject frames too short
        // for their own name before reading any of it (a peer may send sz 0)
        if (sz < 1 || size_t(c[0]) > sz - 1) {
          close_pipe(p, false);
          return;
        }
        size_t nl = c[0];
        std::string name(reinterpret_cast<const char*>(c + 1), std::min<size_t>(nl, sz - 1));
        const uint8_t* body = c + 1 + nl;
        size_t bl = sz - 1 - nl;
        p->rpos += hl + sz;
        if (name == "READY" && p->state == Pipe::HANDSHAKE) {
          if (!parse_ready(p.get(), body, bl) || !socket_types_compatible(s->type_, p->peer_type)) {
            std::string err = encode_command("ERROR", std::string("\x1b") + "Invalid socket type pair.");
            ssize_t r = ::send(p->fd, err.data(), err.size(), MSG_NOSIGNAL);
            (void)r;
            close_pipe(p, false);
            return;
          }
          p->ready_in = true;
          // PAIR accepts exactly one peer.
          bool reject = false;
          {
            std::lock_guard<std::mutex> lk(s->mu_);
            if (s->type_ == PAIR) {
              for (auto& q : s->pipes_)
                if (q.get() != p.get() && q->state == Pipe::ACTIVE) reject = true;
            }
            if (!reject) {
              p->state = Pipe::ACTIVE;
              s->attach_pipe_locked(p);
              if (!p->outq.empty()) p->write_scheduled = true;
            }
          }
          if (reject) {
            close_pipe(p, false);
            return;
          }
          PollHub::instance().bump();
          io_write(p);
          if (p->fd < 0) return;
        } else if (name == "PING") {
          // reply PONG with the ping context (ZMTP 3.1)
          std::string ctxb = bl > 2 ? std::string(reinterpret_cast<const char*>(body + 2), bl - 2) : "";
          std::string pong = encode_command("PONG", ctxb);
          ssize_t r = ::send(p->fd, pong.data(), pong.size(), MSG_NOSIGNAL);
          (void)r;
        } else if (name == "ERROR") {
          close_pipe(p, false);
          return;
        }
        continue;
      }
      if (p->state != Pipe::ACTIVE) {
        close_pipe(p, false);
        return;
      }
      if (sz > (uint64_t(2) << 30)) {   // > 2 GiB: a corrupt or hostile length, not a frame
        close_pipe(p, true);
        return;
      }
      bool more = flags & F_MORE;
      size_t inbuf = avail - hl;
      BufPtr buf;
      if (sz >= s->alloc_threshold_) {
        std::shared_ptr<Allocator> a;
        {
          std::lock_guard<std::mutex> lk(s->mu_);
          a = s->allocator_;
        }
        if (a) buf = a->alloc(sz);
      }
      if (!buf) buf = heap_buffer(sz);
      if (sz <= inbuf) {
        if (sz) std::memcpy(buf->data, h + hl, sz);
        p->rpos += hl + sz;
        Frame fr;
        fr.buf = std::move(buf);
        fr.size = sz;
        p->partial.push_back(std::move(fr));
        if (!more) goto deliver;
        continue;
      }
      // large: copy what we have, then read the rest straight into buf
      if (inbuf) std::memcpy(buf->data, h + hl, inbuf);
      p->rpos = p->rlen = 0;
      p->body = std::move(buf);
      p->body_size = sz;
      p->body_got = inbuf;
      p->body_more = more;
      continue;
    }
  deliver : {
    Message m = std::move(p->partial);
    p->partial.clear();
    size_t bytes = 0;
    for (auto& f : m) bytes += f.size;
    bool paused = false;
    {
      std::lock_guard<std::mutex> lk(s->mu_);
      if (p->attached && !s->closing_) {
        p->inq.push_back(std::move(m));
        s->stats_.msgs_in++;
        s->stats_.bytes_in += bytes;
        if (s->rcvhwm_ > 0 && p->inq.size() >= size_t(s->rcvhwm_)) {
          p->read_paused = true;
          paused = true;
        }
        s->on_message_locked(p.get());
      }
    }
    PollHub::instance().bump();
    if (paused) {
      update_pipe_events(p.get());
      return;
    }
    if (--budget_frames == 0 || budget_bytes == 0) return;   // fairness: let others run
  }
  }
}

// --------------------------------------------------------------------------
// Socket
// --------------------------------------------------------------------------
Socket::Socket(Context* ctx, int type) : ctx_(ctx), type_(type) {
  if (type < 0 || type > PUSH || type == PUB || type == SUB)
    throw Error(E_INVAL, "unsupported socket type");
  std::random_device rd;
  req_id_ = rd();
}

Socket::~Socket() {
  if (!closed_) {
    try {
      close(0);
    } catch (...) {
    }
  }
}

void Socket::setsockopt(int opt, int64_t v) {
  std::lock_guard<std::mutex> lk(mu_);
  switch (opt) {
    case SNDHWM: sndhwm_ = int(v); break;
    case RCVHWM: rcvhwm_ = int(v); break;
    case LINGER: linger_ = long(v); break;
    case SNDTIMEO: sndtimeo_ = long(v); break;
    case RCVTIMEO: rcvtimeo_ = long(v); break;
    case IMMEDIATE: immediate_ = v != 0; break;
    case REQ_CORRELATE: req_correlate_ = v != 0; break;
    case REQ_RELAXED: req_relaxed_ = v != 0; break;
    case RECONNECT_IVL: reconnect_ivl_ = int(v); break;
    case BT_SNDBUF_KB: sndbuf_kb_ = int(v); break;
    case BT_RCVBUF_KB: rcvbuf_kb_ = int(v); break;
    case BT_ALLOC_THRESHOLD: alloc_threshold_ = size_t(v); break;
    default: throw Error(E_INVAL, "unsupported socket option " + std::to_string(opt));
  }
}

void Socket::setsockopt_bytes(int opt, const std::string& v) {
  std::lock_guard<std::mutex> lk(mu_);
  if (opt == IDENTITY) {
    identity_ = v;
    return;
  }
  throw Error(E_INVAL, "unsupported bytes option " + std::to_string(opt));
}

int64_t Socket::getsockopt(int opt) {
  std::lock_guard<std::mutex> lk(mu_);
  switch (opt) {
    case SNDHWM: return sndhwm_;
    case RCVHWM: return rcvhwm_;
    case LINGER: return linger_;
    case SNDTIMEO: return sndtimeo_;
    case RCVTIMEO: return rcvtimeo_;
    case IMMEDIATE: return immediate_;
    case REQ_CORRELATE: return req_correlate_;
    case REQ_RELAXED: return req_relaxed_;
    case RECONNECT_IVL: return reconnect_ivl_;
    case TYPE: return type_;
    case RCVMORE: return 0;
    case BT_ALLOC_THRESHOLD: return int64_t(alloc_threshold_);
  }
  throw Error(E_INVAL, "unsupported socket option " + std::to_string(opt));
}

std::string Socket::getsockopt_string(int opt) {
  std::lock_guard<std::mutex> lk(mu_);
  if (opt == LAST_ENDPOINT) return last_endpoint_;
  if (opt == IDENTITY) return identity_;
  throw Error(E_INVAL, "unsupported string option " + std::to_string(opt));
}

void Socket::set_allocator(std::shared_ptr<Allocator> a, size_t threshold) {
  std::lock_guard<std::mutex> lk(mu_);
  allocator_ = std::move(a);
  alloc_threshold_ = threshold;
}

std::string Socket::bind(const std::string& addr) {
  if (closing_) throw Error(E_TERM, "socket closed");
  Endpoint ep = Endpoint::parse(addr);
  SockAddr sa = resolve(ep, true);
  int fd = ::socket(sa.family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0) throw Error(errno, "socket() failed");
  if (ep.kind == Endpoint::TCP) {
    int one = 1;
    ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  } else if (!ep.host.empty() && ep.host[0] != '@') {
    ::unlink(ep.host.c_str());
  }
  if (::bind(fd, reinterpret_cast<sockaddr*>(&sa.ss), sa.len) < 0) {
    int e = errno;
    ::close(fd);
    throw Error(e == EADDRINUSE ? E_ADDRINUSE : e, "bind failed for " + addr + ": " + strerror(e));
  }
  if (::listen(fd, 128) < 0) {
    int e = errno;
    ::close(fd);
    throw Error(e, "listen failed");
  }
  if (ep.kind == Endpoint::TCP && ep.port < 0) {
    sockaddr_storage ss{};
    socklen_t l = sizeof(ss);
    getsockname(fd, reinterpret_cast<sockaddr*>(&ss), &l);
    ep.port = ntohs(ss.ss_family == AF_INET6 ? reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port
                                              : reinterpret_cast<sockaddr_in*>(&ss)->sin_port);
  }
  if (ep.kind == Endpoint::TCP && (ep.host.empty())) ep.host = "0.0.0.0";
  std::string conc = ep.str();
  {
    std::lock_guard<std::mutex> lk(mu_);
    last_endpoint_ = conc;
    binds_.push_back(conc);
  }
  auto self = shared_from_this();
  ctx_->post_sync([this, fd, ep, self] { ctx_->add_listener(fd, ep, self); });
  return conc;
}

void Socket::unbind(const std::string& addr) {
  std::string a = addr;
  ctx_->post_sync([this, a] { ctx_->remove_listeners_of(this, &a); });
}

void Socket::connect(const std::string& addr) {
  if (closing_) throw Error(E_TERM, "socket closed");
  auto p = std::make_shared<Pipe>();
  p->ctx = ctx_;
  p->sock = shared_from_this();
  p->outbound = true;
  p->ep = Endpoint::parse(addr);
  p->addr = resolve(p->ep, false);
  p->id = g_pipe_ids++;
  {
    std::lock_guard<std::mutex> lk(mu_);
    connects_.push_back(addr);
    last_endpoint_ = addr;
    if (!immediate_) attach_pipe_locked(p);   // messages may queue before connected
  }
  PollHub::instance().bump();
  ctx_->post([this, p] { ctx_->start_connect(p); });
}

void Socket::disconnect(const std::string& addr) {
  auto self = shared_from_this();
  ctx_->post_sync([this, addr, self] {
    std::vector<std::shared_ptr<Pipe>> victims;
    for (auto& kv : ctx_->fd_pipes_) {
      auto s = kv.second->sock.lock();
      if (s.get() == this && kv.second->outbound && kv.second->ep.str() == Endpoint::parse(addr).str())
        victims.push_back(kv.second);
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (auto& q : pipes_)
        if (q->outbound && q->ep.str() == Endpoint::parse(addr).str()) {
          q->gone = true;
          victims.push_back(q);
        }
    }
    for (auto& v : victims) {
      v->gone = true;
      ctx_->close_pipe(v, false);
      std::lock_guard<std::mutex> lk(mu_);
      if (v->attached) detach_pipe_locked(v.get());
    }
  });
}

void Socket::attach_pipe_locked(const std::shared_ptr<Pipe>& p) {
  if (p->attached) return;
  p->attached = true;
  if (type_ == ROUTER) {
    if (!p->peer_identity.empty()) {
      p->router_id = p->peer_identity;
    } else {
      uint32_t id = next_router_id_++;
      p->router_id = std::string(1, '\0') + std::string(reinterpret_cast<char*>(&id), 4);
    }
    router_map_[p->router_id] = p;
  }
  pipes_.push_back(p);
  cv_.notify_all();
}

void Socket::detach_pipe_locked(Pipe* p) {
  p->attached = false;
  for (size_t i = 0; i < pipes_.size(); ++i) {
    if (pipes_[i].get() == p) {
      pipes_.erase(pipes_.begin() + long(i));
      break;
    }
  }
  if (type_ == ROUTER) router_map_.erase(p->router_id);
  if (!pipes_.empty()) {
    rr_in_ %= pipes_.size();
    rr_out_ %= pipes_.size();
  } else {
    rr_in_ = rr_out_ = 0;
  }
  cv_.notify_all();
}

void Socket::on_message_locked(Pipe*) { cv_.notify_all(); }

static bool pipe_writable(const Pipe* p, int hwm) {
  if (!p->attached || p->gone) return false;
  if (p->state == Pipe::DEAD) return false;
  return hwm <= 0 || p->outq.size() < size_t(hwm);
}

std::shared_ptr<Pipe> Socket::pick_out_pipe_locked() {
  size_t n = pipes_.size();
  for (size_t k = 0; k < n; ++k) {
    size_t i = (rr_out_ + k) % n;
    if (pipe_writable(pipes_[i].get(), sndhwm_)) {
      rr_out_ = (i + 1) % n;
      return pipes_[i];
    }
  }
  return nullptr;
}

bool Socket::can_send_locked() {
  switch (type_) {
    case REP: {
      auto p = rep_pipe_.lock();
      return rep_replying_ && (!p || pipe_writable(p.get(), sndhwm_) || !p->attached);
    }
    case ROUTER: return true;
    case PULL: return false;
    default:
      for (auto& p : pipes_)
        if (pipe_writable(p.get(), sndhwm_)) return true;
      return false;
  }
}

void Socket::resume_reads_locked(Pipe* p) {
  if (p->read_paused && !p->resume_posted &&
      (rcvhwm_ <= 0 || p->inq.size() < size_t(rcvhwm_))) {
    p->resume_posted = true;
    auto sp = p->shared_from_this();
    ctx_->post([sp] {
      auto s = sp->sock.lock();
      if (!s) return;
      {
        std::lock_guard<std::mutex> lk(s->mu_);
        sp->read_paused = false;
        sp->resume_posted = false;
      }
      sp->ctx->update_pipe_events(sp.get());
      if (sp->fd >= 0 && sp->state == Pipe::ACTIVE) sp->ctx->io_read(sp);
    });
  }
}

// Pops one routable message; applies REQ/REP envelope rules.
bool Socket::try_recv_locked(Message& out) {
  // purge drained pipes of dead peers
  for (size_t i = 0; i < pipes_.size();) {
    Pipe* p = pipes_[i].get();
    if (p->gone && p->inq.empty() && p->state == Pipe::DEAD) {
      detach_pipe_locked(p);
      continue;
    }
    ++i;
  }
  size_t n = pipes_.size();
  if (type_ == REQ) {
    if (!req_expect_reply_) return false;
    auto rp = req_reply_pipe_.lock();
    // discard anything that is not from the pipe we sent the request to
    for (auto& p : pipes_) {
      if (p != rp && !p->inq.empty()) {
        p->inq.clear();
        resume_reads_locked(p.get());
      }
    }
    if (!rp) return false;
    while (!rp->inq.empty()) {
      Message m = std::move(rp->inq.front());
      rp->inq.pop_front();
      resume_reads_locked(rp.get());
      size_t i = 0;
      if (req_correlate_) {
        if (m.size() < 1 || m[0].size != 4 || std::memcmp(m[0].data(), &req_id_, 4) != 0) continue;
        i = 1;
      }
      if (m.size() <= i || m[i].size != 0) continue;   // missing delimiter
      out.assign(std::make_move_iterator(m.begin() + long(i) + 1), std::make_move_iterator(m.end()));
      req_expect_reply_ = false;
      return true;
    }
    return false;
  }
  for (size_t k = 0; k < n; ++k) {
    size_t idx = (rr_in_ + k) % n;
    auto p = pipes_[idx];
    if (p->inq.empty()) continue;
    Message m = std::move(p->inq.front());
    p->inq.pop_front();
    rr_in_ = (idx + 1) % n;
    resume_reads_locked(p.get());
    if (type_ == REP) {
      size_t d = 0;
      while (d < m.size() && m[d].size != 0) ++d;
      if (d >= m.size()) {   // malformed: no delimiter -> drop
        --k;
        continue;
      }
      rep_envelope_.assign(m.begin(), m.begin() + long(d) + 1);
      out.assign(std::make_move_iterator(m.begin() + long(d) + 1), std::make_move_iterator(m.end()));
      rep_pipe_ = p;
      rep_replying_ = true;
    } else if (type_ == ROUTER) {
      out.clear();
      out.push_back(Frame::copy_of(p->router_id.data(), p->router_id.size()));
      for (auto& f : m) out.push_back(std::move(f));
    } else {
      out = std::move(m);
    }
    if (p->gone && p->inq.empty() && p->state == Pipe::DEAD) detach_pipe_locked(p.get());
    return true;
  }
  return false;
}

bool Socket::can_recv_locked() {
  if (type_ == PUSH) return false;
  if (type_ == REQ) {
    if (!req_expect_reply_) return false;
    auto rp = req_reply_pipe_.lock();
    return rp && !rp->inq.empty();
  }
  if (type_ == REP && rep_replying_) return false;
  for (auto& p : pipes_)
    if (!p->inq.empty()) return true;
  return false;
}

long Socket::deadline_ms(int flags, bool sending) {
  if (flags & DONTWAIT) return 0;
  return sending ? sndtimeo_ : rcvtimeo_;
}

void Socket::send(Message&& msg, int flags, const Interrupt& intr) {
  std::unique_lock<std::mutex> lk(mu_);
  if (closing_) throw Error(E_TERM, "socket closed");
  if (type_ == PULL) throw Error(E_INVAL, "PULL sockets cannot send");
  if (type_ == REQ) {
    if (req_expect_reply_ && !req_relaxed_) throw Error(E_FSM, "REQ: must recv before next send");
    Message env;
    ++req_id_;
    if (req_correlate_) env.push_back(Frame::copy_of(&req_id_, 4));
    env.push_back(Frame::empty());
    for (auto& f : msg) env.push_back(std::move(f));
    msg = std::move(env);
  }
  if (type_ == REP) {
    if (!rep_replying_) throw Error(E_FSM, "REP: must recv before send");
    Message env = rep_envelope_;
    for (auto& f : msg) env.push_back(std::move(f));
    msg = std::move(env);
  }
  long to = deadline_ms(flags, true);
  auto deadline = Clock::now() + std::chrono::milliseconds(to < 0 ? 0 : to);
  std::shared_ptr<Pipe> target;
  auto ready = [&]() -> bool {
    if (type_ == REP) {
      target = rep_pipe_.lock();
      if (!target || !target->attached || target->gone) return true;   // dropped below
      return pipe_writable(target.get(), sndhwm_);
    }
    target = pick_out_pipe_locked();
    return bool(target);
  };
  if (type_ == ROUTER) {
    if (msg.empty()) throw Error(E_INVAL, "ROUTER: missing identity frame");
    std::string id(reinterpret_cast<const char*>(msg[0].data()), msg[0].size);
    auto it = router_map_.find(id);
    target = it == router_map_.end() ? nullptr : it->second.lock();
    msg.erase(msg.begin());
    if (!target || !pipe_writable(target.get(), sndhwm_)) return;   // unroutable/full: drop
  } else {
    for (;;) {
      if (closing_) throw Error(E_TERM, "socket closed");
      if (ready()) break;
      if (to == 0) throw Error(E_AGAIN, "Resource temporarily unavailable");
      wait_slice(lk, to < 0 ? nullptr : &deadline, intr);
      if (to >= 0 && Clock::now() >= deadline) {
        if (ready()) break;
        throw Error(E_AGAIN, "Resource temporarily unavailable");
      }
    }
    if (type_ == REP && (!target || !target->attached || target->gone)) {
      // peer vanished: libzmq silently drops the reply
      rep_replying_ = false;
      rep_envelope_.clear();
      return;
    }
  }
  target->outq.push_back(std::move(msg));
  if (type_ == REQ) {
    req_expect_reply_ = true;
    req_reply_pipe_ = target;
  }
  if (type_ == REP) {
    rep_replying_ = false;
    rep_envelope_.clear();
  }
  bool schedule = target->state == Pipe::ACTIVE && !target->write_scheduled;
  if (schedule) target->write_scheduled = true;
  lk.unlock();
  if (schedule) {
    auto ctx = ctx_;
    ctx_->post([ctx, target] { ctx->io_write(target); });
  }
}

Message Socket::recv(int flags, const Interrupt& intr) {
  std::unique_lock<std::mutex> lk(mu_);
  if (closing_) throw Error(E_TERM, "socket closed");
  if (type_ == PUSH) throw Error(E_INVAL, "PUSH sockets cannot recv");
  if (type_ == REQ && !req_expect_reply_) throw Error(E_FSM, "REQ: must send before recv");
  if (type_ == REP && rep_replying_) throw Error(E_FSM, "REP: must send reply before next recv");
  long to = deadline_ms(flags, false);
  auto deadline = Clock::now() + std::chrono::milliseconds(to < 0 ? 0 : to);
  Message out;
  for (;;) {
    if (try_recv_locked(out)) return out;
    if (closing_) throw Error(E_TERM, "socket closed");
    if (to == 0) throw Error(E_AGAIN, "Resource temporarily unavailable");
    wait_slice(lk, to < 0 ? nullptr : &deadline, intr);
    if (to >= 0 && Clock::now() >= deadline) {
      if (try_recv_locked(out)) return out;
      throw Error(E_AGAIN, "Resource temporarily unavailable");
    }
  }
}

bool Socket::try_recv(Message& out) {
  std::lock_guard<std::mutex> lk(mu_);
  if (closing_) throw Error(E_TERM, "socket closed");
  if (type_ == PUSH) throw Error(E_INVAL, "PUSH sockets cannot recv");
  if (type_ == REQ && !req_expect_reply_) throw Error(E_FSM, "REQ: must send before recv");
  if (type_ == REP && rep_replying_) throw Error(E_FSM, "REP: must send reply before next recv");
  return try_recv_locked(out);
}

size_t Socket::recv_round(std::vector<Message>& out, size_t max) {
  std::lock_guard<std::mutex> lk(mu_);
  if (closing_) throw Error(E_TERM, "socket closed");
  if (type_ != PULL && type_ != PAIR && type_ != DEALER) throw Error(E_INVAL, "recv_round: PULL/PAIR/DEALER only");
  // purge drained pipes of dead peers (as try_recv_locked does)
  for (size_t i = 0; i < pipes_.size();) {
    Pipe* p = pipes_[i].get();
    if (p->gone && p->inq.empty() && p->state == Pipe::DEAD) {
      detach_pipe_locked(p);
      continue;
    }
    ++i;
  }
  const size_t n = pipes_.size();
  size_t got = 0;
  std::vector<Pipe*> dead;
  const size_t start = rr_in_;
  for (size_t k = 0; k < n && got < max; ++k) {
    const size_t idx = (start + k) % n;
    Pipe* p = pipes_[idx].get();
    if (p->inq.empty()) continue;
    out.push_back(std::move(p->inq.front()));
    p->inq.pop_front();
    resume_reads_locked(p);
    ++got;
    if (p->gone && p->inq.empty() && p->state == Pipe::DEAD) dead.push_back(p);
    // the next round starts behind the last pipe served: a round cut short
    // by `max` continues where it stopped instead of favouring pipe 0
    rr_in_ = (idx + 1) % n;
  }
  for (Pipe* p : dead) detach_pipe_locked(p);
  return got;
}

size_t Socket::recv_round(const std::vector<Socket*>& socks, std::vector<Message>& out, size_t max) {
  size_t got = 0;
  for (Socket* s : socks) {
    if (got >= max) break;
    got += s->recv_round(out, max - got);
  }
  return got;
}

void Socket::wait_slice(std::unique_lock<std::mutex>& lk, const Clock::time_point* deadline,
                        const Interrupt& intr) {
  auto until = Clock::now() + std::chrono::milliseconds(intr ? 100 : 1000);
  if (deadline && *deadline < until) until = *deadline;
  cv_.wait_until(lk, until);
  if (intr) {
    lk.unlock();
    bool stop = intr();
    lk.lock();
    if (stop) throw Error(E_INTR, "interrupted");
  }
}

int Socket::events() {
  std::lock_guard<std::mutex> lk(mu_);
  int e = 0;
  if (can_recv_locked()) e |= POLLIN;
  if (can_send_locked()) e |= POLLOUT;
  return e;
}

std::vector<int> Socket::poll(const std::vector<std::pair<Socket*, int>>& items, long timeout_ms,
                              const Interrupt& intr) {
  auto& hub = PollHub::instance();
  auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms < 0 ? 0 : timeout_ms);
  std::vector<int> res(items.size(), 0);
  auto scan = [&] {
    bool any = false;
    for (size_t i = 0; i < items.size(); ++i) {
      res[i] = items[i].first->closed() ? 0 : (items[i].first->events() & items[i].second);
      any |= res[i] != 0;
    }
    return any;
  };
  for (;;) {
    uint64_t gen;
    {
      std::lock_guard<std::mutex> lk(hub.mu);
      gen = hub.generation;
    }
    if (scan() || timeout_ms == 0) return res;
    auto until = Clock::now() + std::chrono::milliseconds(intr ? 100 : 1000);
    if (timeout_ms > 0 && deadline < until) until = deadline;
    {
      std::unique_lock<std::mutex> lk(hub.mu);
      hub.cv.wait_until(lk, until, [&] { return hub.generation != gen; });
    }
    if (intr && intr()) throw Error(E_INTR, "interrupted");
    if (timeout_ms > 0 && Clock::now() >= deadline) {
      scan();
      return res;
    }
  }
}

void Socket::close(long linger_ms) {
  if (closed_) return;
  std::unique_lock<std::mutex> lk(mu_);
  if (closing_) {
    lk.unlock();
    return;
  }
  long linger = linger_ms == -2 ? linger_ : linger_ms;
  auto pending = [&] {
    for (auto& p : pipes_)
      if (!p->gone && (!p->outq.empty() || p->wactive)) return true;
    return false;
  };
  if (linger != 0 && !ctx_->on_io_thread()) {
    if (linger < 0) {
      cv_.wait(lk, [&] { return !pending(); });
    } else {
      cv_.wait_until(lk, Clock::now() + std::chrono::milliseconds(linger), [&] { return !pending(); });
    }
  }
  closing_ = true;
  std::vector<std::shared_ptr<Pipe>> mine = pipes_;
  lk.unlock();
  cv_.notify_all();
  auto cleanup = [this, mine] {
    ctx_->remove_listeners_of(this, nullptr);
    std::vector<std::shared_ptr<Pipe>> victims = mine;
    for (auto& kv : ctx_->fd_pipes_) {
      auto s = kv.second->sock.lock();
      if (!s || s.get() == this) victims.push_back(kv.second);
    }
    for (auto& t : ctx_->timers_) {
      auto s = t.pipe->sock.lock();
      if (!s || s.get() == this) victims.push_back(t.pipe);
    }
    ctx_->timers_.erase(std::remove_if(ctx_->timers_.begin(), ctx_->timers_.end(),
                                       [this](const Context::Timer& t) {
                                         auto s = t.pipe->sock.lock();
                                         return !s || s.get() == this;
                                       }),
                        ctx_->timers_.end());
    for (auto& v : victims) {
      v->gone = true;
      if (v->fd >= 0) {
        if (v->registered) epoll_ctl(ctx_->epfd_, EPOLL_CTL_DEL, v->fd, nullptr);
        ctx_->fd_pipes_.erase(v->fd);
        ::close(v->fd);
        v->fd = -1;
        v->registered = false;
      }
      v->state = Pipe::DEAD;
    }
  };
  if (ctx_->on_io_thread() || !ctx_->running_) {
    if (ctx_->on_io_thread()) cleanup();
  } else {
    ctx_->post_sync(cleanup);
  }
  {
    std::lock_guard<std::mutex> lk2(mu_);
    for (auto& p : pipes_) {
      p->inq.clear();
      p->outq.clear();
      p->attached = false;
    }
    pipes_.clear();
    router_map_.clear();
  }
  closed_ = true;
  PollHub::instance().bump();
}

size_t Socket::num_peers() {
  std::lock_guard<std::mutex> lk(mu_);
  size_t n = 0;
  for (auto& p : pipes_)
    if (p->state == Pipe::ACTIVE) ++n;
  return n;
}

Socket::Stats Socket::stats() {
  std::lock_guard<std::mutex> lk(mu_);
  return stats_;
}

}  // namespace zmtp
}  // namespace btn
