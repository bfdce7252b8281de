// Direct RCCL calls on the caller's stream (see comm.h).
#include "comm.h"

#include <dlfcn.h>

#include <mutex>
#include <stdexcept>

namespace btn {
namespace comm {
namespace {

using Result = int;   // ncclResult_t: 0 = success
using Comm = void*;   // ncclComm_t

struct Api {
  Result (*all_reduce)(const void*, void*, size_t, int, int, Comm, hipStream_t) = nullptr;
  Result (*broadcast)(const void*, void*, size_t, int, int, Comm, hipStream_t) = nullptr;
  Result (*send)(const void*, size_t, int, int, Comm, hipStream_t) = nullptr;
  Result (*recv)(void*, size_t, int, int, Comm, hipStream_t) = nullptr;
  Result (*group_start)() = nullptr;
  Result (*group_end)() = nullptr;
  Result (*count)(Comm, int*) = nullptr;
  Result (*user_rank)(Comm, int*) = nullptr;
  Result (*async_error)(Comm, Result*) = nullptr;
  const char* (*error_string)(Result) = nullptr;
};

Api g_api;
std::mutex g_mu;
bool g_loaded = false;

template <typename F>
void resolve(void* h, const char* name, F& fn) {
  fn = reinterpret_cast<F>(dlsym(h, name));
  if (!fn) throw std::runtime_error(std::string("rccl: missing symbol ") + name);
}

void check(Result r, const char* what) {
  if (r == 0) return;
  const char* msg = g_api.error_string ? g_api.error_string(r) : "unknown";
  throw std::runtime_error(std::string("rccl ") + what + " failed: " + msg + " (" + std::to_string(r) + ")");
}

const Api& api() {
  if (!g_loaded) throw std::runtime_error("rccl: entry points not loaded (comm.load)");
  return g_api;
}

Comm as_comm(uintptr_t c) {
  if (!c) throw std::invalid_argument("rccl: null communicator");
  return reinterpret_cast<Comm>(c);
}

void check_count(size_t count) {
  // counts are element counts of one device buffer; a negative value cast
  // from Python shows up as a huge size_t
  if (count > (size_t(1) << 40)) throw std::invalid_argument("rccl: implausible element count");
}

}  // namespace

void load(const std::string& path) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_loaded) return;
  void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD);
  if (!h) h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!h) throw std::runtime_error(std::string("rccl: dlopen failed: ") + dlerror());
  Api a;
  resolve(h, "ncclAllReduce", a.all_reduce);
  resolve(h, "ncclBroadcast", a.broadcast);
  resolve(h, "ncclSend", a.send);
  resolve(h, "ncclRecv", a.recv);
  resolve(h, "ncclGroupStart", a.group_start);
  resolve(h, "ncclGroupEnd", a.group_end);
  resolve(h, "ncclCommCount", a.count);
  resolve(h, "ncclCommUserRank", a.user_rank);
  resolve(h, "ncclCommGetAsyncError", a.async_error);
  resolve(h, "ncclGetErrorString", a.error_string);
  g_api = a;
  g_loaded = true;
}

bool loaded() { return g_loaded; }

int comm_count(uintptr_t c) {
  int n = 0;
  check(api().count(as_comm(c), &n), "ncclCommCount");
  return n;
}

int comm_rank(uintptr_t c) {
  int r = 0;
  check(api().user_rank(as_comm(c), &r), "ncclCommUserRank");
  return r;
}

void all_reduce(const void* send, void* recv, size_t count, int dtype, int op, uintptr_t c, hipStream_t s) {
  check_count(count);
  check(api().all_reduce(send, recv, count, dtype, op, as_comm(c), s), "ncclAllReduce");
}

void broadcast(const void* send, void* recv, size_t count, int dtype, int root, uintptr_t c, hipStream_t s) {
  check_count(count);
  check(api().broadcast(send, recv, count, dtype, root, as_comm(c), s), "ncclBroadcast");
}

void send(const void* buf, size_t count, int dtype, int peer, uintptr_t c, hipStream_t s) {
  check_count(count);
  check(api().send(buf, count, dtype, peer, as_comm(c), s), "ncclSend");
}

void recv(void* buf, size_t count, int dtype, int peer, uintptr_t c, hipStream_t s) {
  check_count(count);
  check(api().recv(buf, count, dtype, peer, as_comm(c), s), "ncclRecv");
}

void group_start() { check(api().group_start(), "ncclGroupStart"); }
void group_end() { check(api().group_end(), "ncclGroupEnd"); }

std::string async_error(uintptr_t c) {
  Result r = 0;
  check(api().async_error(as_comm(c), &r), "ncclCommGetAsyncError");
  if (r == 0) return "";
  return std::string(g_api.error_string(r)) + " (" + std::to_string(r) + ")";
}

}  // namespace comm
}  // namespace btn
