// aql.hpp — the engine's kernels dispatched as AQL packets on a user-mode HSA queue
// (crane_queue_*, crane_dyn_step_keys_queue in include/crane_dyn.h).
//
// A HIP launch costs the enqueuing thread 2.1-5.2 us on this image, box to box (the runtime's
// command objects, locks and argument handling; profiles/r05/kernarg_probe.txt), so a config-3
// batch (three kernels) costs ~9-15 us of host time, about the GPU's ~11 us per batch with four
// in flight.  Writing the packet ourselves costs 0.2-0.6 us (profiles/r05/aql_probe.txt): the
// host stays under the GPU's rate on every box.  While a queue is installed on the calling thread (tl_aql),
// klaunch (kernels.hpp) packs the kernel's arguments by the AMDGPU kernarg rules (each by-value
// argument at its natural alignment, then the code-object-v5 implicit arguments the kernel
// reads: block counts, group sizes, grid dimensions, dynamic LDS size) into the queue's
// kernarg ring and writes a kernel-dispatch packet.  Every packet has the barrier bit (a
// queue is in order, like a stream); a step's packets become visible to the packet processor
// together (aql_commit: headers in order, one doorbell), the last one carrying the queue's
// completion signal, which counts the committed steps still running.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstring>

struct crane_queue;
struct crane_dyn;

namespace crane {

constexpr size_t kAqlMaxArgs = 3072;  // explicit argument bytes (K1's are ~1.3 KiB)

// the queue this thread's klaunch calls go to (set for one step on a queue), else HIP
extern thread_local crane_queue* tl_aql;

hipError_t aql_launch(crane_queue* q, const void* host_fn, dim3 grid, dim3 block, uint32_t dyn_lds,
                      const unsigned char* args, size_t explicit_bytes);
// make the packets written since the last commit visible, the last one counted on the
// queue's completion signal
hipError_t aql_commit(crane_queue* q);
// commit, then wait until every committed packet has completed
hipError_t aql_wait(crane_queue* q);
// commits (steps) made visible on the queue so far, and how many of them have completed (in
// order: a queue runs its packets one after the other) — what a host thread polls to order work
// after a step without a device-side wait
uint64_t aql_commits(const crane_queue* q);
uint64_t aql_completed(const crane_queue* q);
const char* aql_error(const crane_queue* q);
// Engines that put steps on a queue register with it (crane_dyn_step_keys_queue), so whichever of
// the two is destroyed first can tell the other: a queue's destroy hands itself back to every
// registered engine (engine_drop_queue, engine.hip), an engine's destroy waits for the queues it
// used and unregisters.
void aql_add_user(crane_queue* q, crane_dyn* h);
void aql_remove_user(crane_queue* q, crane_dyn* h);
void engine_drop_queue(crane_dyn* h, crane_queue* q);
// (group.cpp) engine h shares engine from's shard inputs (engine.hip: ShardData)
int engine_share_shard(crane_dyn* h, crane_dyn* from);

template <typename T>
inline void aql_pack(unsigned char* buf, size_t& off, const T& v) {
    off = (off + alignof(T) - 1) & ~(alignof(T) - 1);
    std::memcpy(buf + off, &v, sizeof(T));
    off += sizeof(T);
}

}  // namespace crane
