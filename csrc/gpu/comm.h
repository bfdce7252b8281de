// Direct RCCL calls on the caller's HIP stream.
//
// torch.distributed's ProcessGroupNCCL runs every collective on its own
// internal stream: an event on the compute stream, a cross-stream wait, the
// collective, an event back.  Inside a captured training step that turns the
// graph into a fork/join DAG, which ROCm 7 executes node by node with ~10 us
// between kernels instead of as one back-to-back queue (profiles/r3/
// dp_tax.md); eagerly each hipStreamWaitEvent costs 28-590 us of host time
// (profiles/r2/hip_api_cost.json).  These entry points take the communicator
// torch already built (ProcessGroupNCCL._comm_ptr()) and enqueue the RCCL
// kernel straight onto the compute stream, so a captured step stays one linear
// queue and an eager step pays no cross-stream synchronisation.
//
// The RCCL entry points are resolved with dlsym from the librccl.so torch has
// loaded (the caller passes its path): a communicator must only ever be used
// with the library instance that created it.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>
#include <string>

namespace btn {
namespace comm {

// nccl.h enum values (stable across RCCL 2.x)
enum DType : int { I8 = 0, U8 = 1, I32 = 2, U32 = 3, I64 = 4, U64 = 5, F16 = 6, F32 = 7, F64 = 8, BF16 = 9 };
enum RedOp : int { SUM = 0, PROD = 1, MAX = 2, MIN = 3, AVG = 4 };

// Loads the entry points from `path` (dlopen of an already-loaded library
// returns that instance).  Throws with the dlerror text on failure.
void load(const std::string& path);
bool loaded();

int comm_count(uintptr_t comm);
int comm_rank(uintptr_t comm);

void all_reduce(const void* send, void* recv, size_t count, int dtype, int op, uintptr_t comm, hipStream_t s);
void broadcast(const void* send, void* recv, size_t count, int dtype, int root, uintptr_t comm, hipStream_t s);
void send(const void* buf, size_t count, int dtype, int peer, uintptr_t comm, hipStream_t s);
void recv(void* buf, size_t count, int dtype, int peer, uintptr_t comm, hipStream_t s);
void group_start();
void group_end();
// Asynchronous error state of a communicator ("" when healthy).
std::string async_error(uintptr_t comm);

}  // namespace comm
}  // namespace btn
