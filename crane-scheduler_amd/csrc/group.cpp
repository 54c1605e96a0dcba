// group.cpp — one process driving N devices: the node-shard engine behind the C ABI
// (crane_dyn_group_* in include/crane_dyn.h).
//
// Reference: the scheduler is ONE Go process (cmd/scheduler/main.go:18-32) holding ONE plugin
// instance (NewDynamicScheduler, pkg/plugins/dynamic/plugins.go:105-120), so the node-shard
// path SURVEY §8(b)/(e) describes — nodes split across the GPUs of one node, each shard's
// best (score, node) packed into an int64 and max-combined over xGMI — has to be reachable
// from a single caller through the C ABI.  A group holds, per shard (a contiguous node range on
// one device), `depth` engines (crane_dyn, one per batch in flight) that SHARE the shard's inputs
// (engine.hip ShardData: the annotation SoA and the binding log or heap, one copy per shard) and
// keep only their own scratch; their HIP streams and dispatch queues; and one RCCL communicator
// per device from ncclCommInitAll.  A batch runs the shard step (K2 hot values + K1 node pass +
// K3 Filter/Score/argmax, engine.hip) on every device; the keys are then max-combined by an
// in-place ncclAllReduce(int64, ncclMax): per batch (crane_dyn_group_step_keys_async, on the
// slot's stream), or once per group of G batches over their keys [G][P]
// (crane_dyn_group_step_keys_batch, on a collective stream per device, issued by the enqueueing
// thread once it sees the slots' dispatch queues complete the window's steps).
//
// The shard's state changes go to the shard's slot-0 engine (its slots follow, engine.hip
// adopt), routed by global node index: the controller's patches (update_nodes /
// update_node_steps), nodes joining and leaving (resize_nodes: the cluster's node range grows or
// shrinks at its end, i.e. in the last shard), the BindingRecords heap (each device runs the same
// heap over the same stream of bindings — its order depends on timestamps only — with the nodes of
// other shards mapped to "no node"), and the drop-in's answer tables (node_steps).
//
// Enqueueing: a step costs the host ~9 us of HIP kernel launches per device (~4 us on the
// dispatch queues, aql.cpp), so one thread feeding eight devices would leave them idle.  With
// more than one device each device has a worker thread (spinning briefly, then sleeping) that
// takes the batch descriptors the caller pushes and enqueues its device's step and its part of
// the all-reduce on its own communicator (RCCL's one-thread-per-device usage); the caller only
// pushes descriptors.  Option "threads" 0 instead enqueues everything from the caller's thread,
// the collective inside ncclGroupStart / ncclGroupEnd (RCCL's one-thread-many-devices usage).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/crane_dyn.h"
#include "aql.hpp"

namespace {

// Job kinds: one batch's shard step (+ its own all-reduce when per_batch_coll), or the
// collective over a group of batches' keys (after the slots' last batches of the group)
enum : int { kJobStep = 0, kJobGroupColl = 1 };

struct Job {
    int kind = kJobStep;
    int64_t now = 0, hv_ts = 0, P = 0;
    const int64_t* d_now = nullptr;
    const uint8_t* d_flags = nullptr;
    int64_t* d_keys = nullptr;
    int slot = 0;
    bool qmode = false;           // the step's kernels on the slot's dispatch queue
    bool per_batch_coll = false;  // an all-reduce of this batch's keys on the slot's stream
    uint64_t slots = 0;           // kJobGroupColl: the slots whose last batches it follows (bit mask)
    int64_t count = 0;            // kJobGroupColl: keys reduced in place at d_keys
};

inline void cpu_relax() { __builtin_ia32_pause(); }

}  // namespace

struct GroupWorker;

// What the thread that enqueues for a shard (its worker, or the caller) keeps per shard
struct DevCtx {
    hipStream_t cstream = nullptr;    // the group collective's stream
    std::vector<hipEvent_t> slot_ev;  // [slot] after the slot's last batch (HIP-stream steps)
    // group collectives after batches on dispatch queues, not issued yet: issued (in order) once
    // the host sees every slot's queue complete the steps the window committed on it (a queue is
    // ordered with no HIP stream; a device-side wait on a flag the queue writes,
    // hipStreamWaitValue64, runs as a polling kernel that holds the GPU meanwhile: measured
    // 0.0125 -> 0.026 ms per batch at config 3 on one device)
    struct PendColl {
        int64_t* keys;
        int64_t count;
        std::vector<uint64_t> target;  // [slot] commits of the slot's queue to complete (0: none)
        std::chrono::steady_clock::time_point t0;
    };
    std::deque<PendColl> pcoll;
    struct Pending {                  // a group collective in flight over [p, p + bytes)
        const char* p;
        size_t bytes;
        hipEvent_t ev;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> free_ev;
};

struct crane_dyn_group {
    std::mutex mu;  // serialises the ABI calls on the group
    std::string err;
    int n = 0, depth = 1;
    std::vector<int> dev;
    std::vector<std::vector<crane_dyn*>> eng;  // [slot][shard]; a shard's slots share its inputs
    std::vector<std::vector<hipStream_t>> st;  // [slot][shard]
    std::vector<ncclComm_t> comm;              // [shard], created on first use
    std::vector<int64_t> lo, hi;               // node range of each shard
    std::vector<DevCtx> ctx;                   // [shard]
    int64_t N = -1;
    int collective = 1;  // 0: never (a host max combines), 1: when n > 1, 2: always (tests at n = 1)
    int threads = -1;    // -1: worker threads when n > 1, 0: the caller's thread, 1: worker threads
    // 0: the steps' kernels on the slots' HIP streams; 1: on user-mode AQL queues (crane_queue, one
    // per slot and shard, created on first use); -1: queues, except with the per-batch collective
    // (crane_dyn_group_step_keys_async / _schedule with the collective on: RCCL follows each batch
    // on its stream).  ring_kind of their kernargs
    int dispatch = -1, ring_kind = 0;
    int defer = 1;  // engine option step_defer on the queues' engines (a step's K3s in the slot's next launch)
    std::vector<std::vector<crane_queue*>> q;  // [slot][shard]
    bool comm_broken = false;
    uint64_t batch = 0;
    uint64_t synced = 0;  // batch at the last wait_all: the slots used since are the ones to wait for
    std::vector<std::unique_ptr<GroupWorker>> workers;
    // crane_dyn_group_schedule's device buffers per shard, and its pinned key staging
    std::vector<int64_t*> b_now, b_keys;
    std::vector<uint8_t*> b_flags;
    size_t b_cap = 0;
    int64_t* h_keys = nullptr;
    size_t h_cap = 0;
    // host scratch of the routed calls
    std::vector<int64_t> r_idx, r_pos;
    std::vector<double> r_val, r_hv;
    std::vector<int64_t> r_ts, r_hvts;
    std::vector<int32_t> r_node;

    int fail(int code, const std::string& m) {
        err = m;
        return code;
    }
    int hipfail(hipError_t e, const char* what) {
        err = std::string(what) + ": " + hipGetErrorString(e);
        return CRANE_E_HIP;
    }
    int ncclfail(ncclResult_t r, const char* what) {
        err = std::string(what) + ": " + ncclGetErrorString(r);
        return CRANE_E_HIP;
    }
    bool use_coll() const { return collective == 2 || (collective == 1 && n > 1); }
    crane_queue* queue(int slot, int i) const { return q.empty() ? nullptr : q[(size_t)slot][(size_t)i]; }
    bool use_workers() const { return threads == 1 || (threads < 0 && n > 1); }
};

namespace {

int engine_err(crane_dyn_group* g, crane_dyn* e, int rc, int i) {
    g->err = std::string("shard ") + std::to_string(i) + " (device " + std::to_string(g->dev[(size_t)i]) +
             "): " + crane_dyn_last_error(e);
    return rc;
}

// the collective stream of shard i waits for slot s's work so far on its HIP stream (steps
// launched through HIP); called by the thread enqueueing for the shard
hipError_t order_after_slot(crane_dyn_group* g, int i, int s) {
    DevCtx& c = g->ctx[(size_t)i];
    hipError_t e = hipEventRecord(c.slot_ev[(size_t)s], g->st[(size_t)s][(size_t)i]);
    return e == hipSuccess ? hipStreamWaitEvent(c.cstream, c.slot_ev[(size_t)s], 0) : e;
}

// a group collective after steps on dispatch queues: held until the queues completed them
void pcoll_push(crane_dyn_group* g, int i, const Job& j) {
    DevCtx::PendColl pc{j.d_keys, j.count, std::vector<uint64_t>((size_t)g->depth, 0),
                        std::chrono::steady_clock::now()};
    for (int sl = 0; sl < g->depth; ++sl)
        if (j.slots >> sl & 1)
            if (crane_queue* qq = g->queue(sl, i)) pc.target[(size_t)sl] = crane::aql_commits(qq);
    g->ctx[(size_t)i].pcoll.push_back(std::move(pc));
}

// 1: the oldest held collective of shard i may be issued, 0: not yet, <0: its steps did not finish
// within 60 s (a fault or a hang: reported, not waited for forever)
int pcoll_ready(crane_dyn_group* g, int i) {
    const DevCtx::PendColl& pc = g->ctx[(size_t)i].pcoll.front();
    for (int sl = 0; sl < g->depth; ++sl)
        if (pc.target[(size_t)sl] && crane::aql_completed(g->queue(sl, i)) < pc.target[(size_t)sl])
            return std::chrono::steady_clock::now() - pc.t0 > std::chrono::seconds(60) ? -1 : 0;
    return 1;
}

// a held (not yet issued) group collective of shard i over keys at [p, p + bytes)
bool held_overlap(const crane_dyn_group* g, int i, const void* p, size_t bytes) {
    const char* a = static_cast<const char*>(p);
    for (const auto& pc : g->ctx[(size_t)i].pcoll) {
        const char* k = reinterpret_cast<const char*>(pc.keys);
        if (k < a + bytes && a < k + sizeof(int64_t) * (size_t)pc.count) return true;
    }
    return false;
}

// before a batch writes keys at [p, p + bytes) on shard i: a group collective still reducing
// (in place) keys there is waited for — callers alternate key buffers, so this rarely blocks
// (a held one is issued first by the caller of this: held_overlap)
hipError_t wait_pending(crane_dyn_group* g, int i, const void* p, size_t bytes) {
    DevCtx& c = g->ctx[(size_t)i];
    const char* a = static_cast<const char*>(p);
    for (size_t k = 0; k < c.pending.size();) {
        DevCtx::Pending& pe = c.pending[k];
        if (pe.p < a + bytes && a < pe.p + pe.bytes) {
            hipError_t e = hipEventSynchronize(pe.ev);
            if (e != hipSuccess) return e;
            c.free_ev.push_back(pe.ev);
            c.pending.erase(c.pending.begin() + (long)k);
            continue;
        }
        ++k;
    }
    return hipSuccess;
}

// shard i's part of one job before its collective (worker thread or caller): the batch's shard
// step, or the collective stream's ordering after the batches
int run_job_dev(crane_dyn_group* g, int i, const Job& j, std::string* msg) {
    const std::string who = "shard " + std::to_string(i) + " (device " + std::to_string(g->dev[(size_t)i]) + ")";
    if (j.kind == kJobGroupColl) {
        if (hipError_t r = hipSetDevice(g->dev[(size_t)i])) {
            *msg = who + ": " + hipGetErrorString(r);
            return CRANE_E_HIP;
        }
        if (j.qmode) {
            // the window's deferred K3s (option step_defer) run now, so the targets pcoll_push reads
            // count them; then held until the queues completed the window
            for (int sl = 0; sl < g->depth; ++sl)
                if (j.slots >> sl & 1)
                    if (int rc = crane_dyn_step_flush(g->eng[(size_t)sl][(size_t)i])) {
                        *msg = who + ": " + crane_dyn_last_error(g->eng[(size_t)sl][(size_t)i]);
                        return rc;
                    }
            return 0;
        }
        for (int sl = 0; sl < g->depth; ++sl)
            if (j.slots >> sl & 1)
                if (hipError_t r = order_after_slot(g, i, sl)) {
                    *msg = who + ": ordering the collective: " + hipGetErrorString(r);
                    return CRANE_E_HIP;
                }
        return 0;
    }
    crane_dyn* e = g->eng[(size_t)j.slot][(size_t)i];
    hipStream_t s = g->st[(size_t)j.slot][(size_t)i];
    if (hipError_t r = wait_pending(g, i, j.d_keys, sizeof(int64_t) * (size_t)j.P)) {
        *msg = who + ": " + hipGetErrorString(r);
        return CRANE_E_HIP;
    }
    crane_queue* qq = j.qmode ? g->queue(j.slot, i) : nullptr;
    if (g->hi[(size_t)i] > g->lo[(size_t)i]) {
        const int rc = qq ? crane_dyn_step_keys_queue(e, j.now, j.hv_ts, j.P, j.d_now, j.d_flags, j.d_keys, qq)
                          : crane_dyn_step_keys_async(e, j.now, j.hv_ts, j.P, j.d_now, j.d_flags, j.d_keys, s);
        if (rc) {
            *msg = who + ": " + crane_dyn_last_error(e);
            return rc;
        }
    } else if (j.P > 0) {  // an empty shard contributes "no node"
        hipError_t r = hipSetDevice(g->dev[(size_t)i]);
        if (r == hipSuccess) r = hipMemsetAsync(j.d_keys, 0xFF, sizeof(int64_t) * (size_t)j.P, s);
        if (r == hipSuccess && qq) r = hipStreamSynchronize(s);  // (queues: wait_all waits for those only)
        if (r != hipSuccess) {
            *msg = who + ": " + hipGetErrorString(r);
            return CRANE_E_HIP;
        }
    }
    return 0;
}

// after the group collective of job j was enqueued on shard i's collective stream: its
// completion, for wait_pending
hipError_t note_pending(crane_dyn_group* g, int i, const Job& j) {
    DevCtx& c = g->ctx[(size_t)i];
    if (hipError_t e = hipSetDevice(g->dev[(size_t)i])) return e;
    hipEvent_t ev = nullptr;
    if (!c.free_ev.empty()) {
        ev = c.free_ev.back();
        c.free_ev.pop_back();
    } else if (hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) {
        return e;
    }
    hipError_t e = hipEventRecord(ev, c.cstream);
    if (e != hipSuccess) {
        c.free_ev.push_back(ev);
        return e;
    }
    c.pending.push_back({reinterpret_cast<const char*>(j.d_keys), sizeof(int64_t) * (size_t)j.count, ev});
    return hipSuccess;
}

// a held group collective issued on shard i's collective stream (ncclAllReduce, in place)
int issue_held(crane_dyn_group* g, int i, const DevCtx::PendColl& pc, std::string* msg) {
    ncclResult_t r = ncclAllReduce(pc.keys, pc.keys, (size_t)pc.count, ncclInt64, ncclMax, g->comm[(size_t)i],
                                   g->ctx[(size_t)i].cstream);
    if (r != ncclSuccess) {
        *msg = std::string("ncclAllReduce: ") + ncclGetErrorString(r);
        return CRANE_E_HIP;
    }
    Job j;
    j.d_keys = pc.keys;
    j.count = pc.count;
    if (hipError_t e = note_pending(g, i, j)) {
        *msg = hipGetErrorString(e);
        return CRANE_E_HIP;
    }
    return 0;
}

bool has_coll(const Job& j) { return (j.kind == kJobStep && j.per_batch_coll) || j.kind == kJobGroupColl; }
int64_t coll_count(const Job& j) { return j.kind == kJobStep ? j.P : j.count; }
hipStream_t coll_stream(const crane_dyn_group* g, const Job& j, int i) {
    return j.kind == kJobStep ? g->st[(size_t)j.slot][(size_t)i] : g->ctx[(size_t)i].cstream;
}

}  // namespace

struct GroupWorker {
    static constexpr uint64_t kRing = 256;
    crane_dyn_group* g = nullptr;
    int i = 0;
    std::thread th;
    Job ring[kRing];
    std::atomic<uint64_t> head{0}, tail{0};
    std::atomic<bool> stop{false};
    std::atomic<int> sleeping{0};
    std::atomic<int> held{0};  // group collectives held for their queues (DevCtx::pcoll)
    std::mutex m;
    std::condition_variable cv;
    std::mutex emu;
    std::string emsg;  // first error since the last sync
    int ecode = 0;

    void record(int code, const std::string& msg) {
        std::lock_guard<std::mutex> l(emu);
        if (!ecode) {
            ecode = code;
            emsg = msg;
        }
    }

    // One job on this device: the shard step (then, per batch, this device's part of the
    // all-reduce) or a group collective (the all-reduce is always issued once the group uses it,
    // even after a failed step: the other devices' all-reduce kernels wait for this one's)
    void run_job(const Job& j) {
        std::string msg;
        if (j.kind == kJobStep)  // (keys a held collective will reduce: it goes first)
            while (held_overlap(g, i, j.d_keys, sizeof(int64_t) * (size_t)j.P)) {
                progress();
                cpu_relax();
            }
        if (int rc = run_job_dev(g, i, j, &msg)) record(rc, msg);
        if (j.kind == kJobGroupColl && j.qmode) {  // held until the queues completed the window
            pcoll_push(g, i, j);
            progress();
            return;
        }
        if (!has_coll(j) || coll_count(j) <= 0) return;
        ncclResult_t r = ncclAllReduce(j.d_keys, j.d_keys, (size_t)coll_count(j), ncclInt64, ncclMax,
                                       g->comm[(size_t)i], coll_stream(g, j, i));
        if (r != ncclSuccess) record(CRANE_E_HIP, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
        if (j.kind == kJobGroupColl)
            if (hipError_t e = note_pending(g, i, j)) record(CRANE_E_HIP, hipGetErrorString(e));
    }

    // the held collectives whose queues completed their windows, in order (every device issues
    // its part of the same sequence); one whose steps did not finish within 60 s is dropped and
    // reported (wait_all then aborts the communicators)
    void progress() {
        auto& pc = g->ctx[(size_t)i].pcoll;
        while (!pc.empty()) {
            const int r = pcoll_ready(g, i);
            if (r == 0) break;
            std::string msg;
            if (r < 0) record(CRANE_E_HIP, "the steps before a group collective did not finish within 60 s");
            else if (int rc = issue_held(g, i, pc.front(), &msg)) record(rc, msg);
            pc.pop_front();
        }
        held.store((int)pc.size(), std::memory_order_release);
    }

    void loop() {
        (void)hipSetDevice(g->dev[i]);
        uint64_t t = tail.load(std::memory_order_relaxed);
        for (;;) {
            uint64_t h = head.load(std::memory_order_acquire);
            for (int spins = 0; h == t; h = head.load(std::memory_order_acquire)) {
                if (stop.load(std::memory_order_acquire)) return;
                if (held.load(std::memory_order_relaxed)) {  // (no sleep while collectives are held)
                    progress();
                    cpu_relax();
                    continue;
                }
                if (++spins < (1 << 14)) {
                    cpu_relax();
                    continue;
                }
                // idle: sleep until a push (Dekker with the pusher: sleeping, then head, both
                // sequentially consistent), with a timeout as a backstop
                std::unique_lock<std::mutex> l(m);
                sleeping.store(1, std::memory_order_seq_cst);
                cv.wait_for(l, std::chrono::milliseconds(2), [&] {
                    return head.load(std::memory_order_seq_cst) != t || stop.load(std::memory_order_seq_cst);
                });
                sleeping.store(0, std::memory_order_relaxed);
                spins = 0;
            }
            for (; t < h; ++t) {
                run_job(ring[t % kRing]);
                tail.store(t + 1, std::memory_order_release);
            }
        }
    }

    void push(const Job& j) {
        const uint64_t h = head.load(std::memory_order_relaxed);
        while (h - tail.load(std::memory_order_acquire) >= kRing) cpu_relax();
        ring[h % kRing] = j;
        head.store(h + 1, std::memory_order_seq_cst);
        if (sleeping.load(std::memory_order_seq_cst)) {
            std::lock_guard<std::mutex> l(m);
            cv.notify_one();
        }
    }

    void drain() const {
        while (tail.load(std::memory_order_acquire) != head.load(std::memory_order_acquire) ||
               held.load(std::memory_order_acquire))
            cpu_relax();
    }
};

namespace {

struct GLock {
    std::lock_guard<std::mutex> l;
    explicit GLock(crane_dyn_group* g) : l(g->mu) {}
};

// the communicators, on the first batch that needs them (one per device, ncclCommInitAll)
int ensure_comms(crane_dyn_group* g) {
    if (!g->use_coll() || !g->comm.empty()) return g->comm_broken ? g->fail(CRANE_E_STATE, "communicator aborted") : 0;
    // (a device listed twice — several shards on one GPU, the tests' layout — has no RCCL rank
    // layout: those groups combine on the host, "collective" 0)
    for (int i = 0; i < g->n; ++i)
        for (int k = 0; k < i; ++k)
            if (g->dev[(size_t)k] == g->dev[(size_t)i])
                return g->fail(CRANE_E_INVALID, "the collective needs distinct devices (set \"collective\" 0)");
    std::vector<ncclComm_t> c((size_t)g->n, nullptr);
    ncclResult_t r = ncclCommInitAll(c.data(), g->n, g->dev.data());
    if (r != ncclSuccess) return g->ncclfail(r, "ncclCommInitAll");
    g->comm = c;
    return 0;
}

// the group collective's streams, flags and events, on first use
int ensure_ctx(crane_dyn_group* g) {
    for (int i = 0; i < g->n; ++i) {
        DevCtx& c = g->ctx[(size_t)i];
        if (c.cstream) continue;
        hipError_t e = hipSetDevice(g->dev[(size_t)i]);
        c.slot_ev.assign((size_t)g->depth, nullptr);
        for (int s = 0; s < g->depth && e == hipSuccess; ++s)
            e = hipEventCreateWithFlags(&c.slot_ev[(size_t)s], hipEventDisableTiming);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&c.cstream, hipStreamNonBlocking);
        if (e != hipSuccess) return g->hipfail(e, "collective stream / events");
    }
    return 0;
}

// the caller's thread (threads 0): the held collectives whose queues completed, on every device at
// once (grouped), in order
int progress_here(crane_dyn_group* g) {
    int rc = 0;
    for (;;) {
        bool all = true, late = false;
        for (int i = 0; i < g->n && all; ++i) {
            if (g->ctx[(size_t)i].pcoll.empty()) return rc;
            const int r = pcoll_ready(g, i);
            all = r != 0;
            late = late || r < 0;
        }
        if (!all) return rc;
        if (late) {
            if (!rc) rc = g->fail(CRANE_E_HIP, "the steps before a group collective did not finish within 60 s");
        } else {
            ncclResult_t r = ncclGroupStart();
            std::string msg;
            for (int i = 0; i < g->n && r == ncclSuccess; ++i) {
                const auto& pc = g->ctx[(size_t)i].pcoll.front();
                r = ncclAllReduce(pc.keys, pc.keys, (size_t)pc.count, ncclInt64, ncclMax, g->comm[(size_t)i],
                                  g->ctx[(size_t)i].cstream);
            }
            const ncclResult_t r2 = ncclGroupEnd();
            if (r != ncclSuccess && !rc) rc = g->ncclfail(r, "ncclAllReduce");
            if (r2 != ncclSuccess && !rc) rc = g->ncclfail(r2, "ncclGroupEnd");
            for (int i = 0; i < g->n; ++i) {
                Job j;
                j.d_keys = g->ctx[(size_t)i].pcoll.front().keys;
                j.count = g->ctx[(size_t)i].pcoll.front().count;
                if (hipError_t e = note_pending(g, i, j))
                    if (!rc) rc = g->hipfail(e, "collective event");
            }
        }
        for (int i = 0; i < g->n; ++i) g->ctx[(size_t)i].pcoll.pop_front();
    }
}

// wait for every pushed job, the used slots' streams and queues and the collective streams; the
// first error since the last wait
int wait_all(crane_dyn_group* g) {
    int rc = 0;
    if (g->workers.empty()) {  // (caller's thread: its held collectives, issued as their queues finish)
        for (bool held = true; held;) {
            if (int r = progress_here(g)) {
                if (!rc) rc = r;
                for (auto& c : g->ctx) c.pcoll.clear();
            }
            held = false;
            for (auto& c : g->ctx) held = held || !c.pcoll.empty();
            if (held) cpu_relax();
        }
    }
    for (auto& w : g->workers) {
        w->drain();
        std::lock_guard<std::mutex> l(w->emu);
        if (w->ecode && !rc) {
            rc = w->ecode;
            g->err = w->emsg;
        }
        w->ecode = 0;
        w->emsg.clear();
    }
    // the slots' deferred K3s (option step_defer), from this thread: the workers are idle
    for (size_t s = 0; s < g->eng.size(); ++s)
        for (size_t i = 0; i < g->eng[s].size(); ++i)
            if (g->eng[s][i] && crane_dyn_step_flush(g->eng[s][i]) && !rc)
                rc = engine_err(g, g->eng[s][i], CRANE_E_HIP, (int)i);
    if (rc && !g->comm.empty() && !g->comm_broken) {
        // a device that failed may have left the others' all-reduce kernels waiting for it:
        // abort the communicators (their kernels see the abort flag and exit) before waiting
        for (ncclComm_t c : g->comm) (void)ncclCommAbort(c);
        g->comm.clear();
        g->comm_broken = true;
    }
    // the slots that ran batches since the last wait, oldest first (by the time the oldest is
    // done the others mostly are: a wait on every slot, idle or not, cost the short timed
    // regions a few microseconds per slot)
    const uint64_t used = std::min<uint64_t>(g->batch - g->synced, (uint64_t)g->depth);
    for (uint64_t b = g->batch - used; b < g->batch; ++b) {
        const size_t s = (size_t)(b % (uint64_t)g->depth);
        for (int i = 0; i < g->n; ++i) {
            if (crane_queue* qq = g->queue((int)s, i))
                if (crane_queue_wait(qq) && !rc) rc = g->fail(CRANE_E_HIP, std::string("queue: ") + crane_queue_last_error(qq));
            hipError_t e = hipSetDevice(g->dev[(size_t)i]);
            if (e == hipSuccess) e = hipStreamSynchronize(g->st[s][(size_t)i]);
            if (e != hipSuccess && !rc) rc = g->hipfail(e, "hipStreamSynchronize");
        }
    }
    for (int i = 0; i < g->n; ++i) {
        DevCtx& c = g->ctx[(size_t)i];
        if (!c.cstream) continue;
        hipError_t e = hipSetDevice(g->dev[(size_t)i]);
        if (e == hipSuccess) e = hipStreamSynchronize(c.cstream);
        if (e != hipSuccess && !rc) rc = g->hipfail(e, "collective stream");
        for (auto& pe : c.pending) c.free_ev.push_back(pe.ev);
        c.pending.clear();
    }
    g->synced = g->batch;
    return rc;
}

void stop_workers(crane_dyn_group* g) {
    for (auto& w : g->workers) {
        w->stop.store(true, std::memory_order_seq_cst);
        {
            std::lock_guard<std::mutex> l(w->m);
            w->cv.notify_one();
        }
        if (w->th.joinable()) w->th.join();
    }
    g->workers.clear();
}

void start_workers(crane_dyn_group* g) {
    if (!g->use_workers() || !g->workers.empty()) return;
    for (int i = 0; i < g->n; ++i) {
        std::unique_ptr<GroupWorker> w(new GroupWorker());
        w->g = g;
        w->i = i;
        GroupWorker* p = w.get();
        w->th = std::thread([p] { p->loop(); });
        g->workers.push_back(std::move(w));
    }
}

// one job on every shard from the caller's thread (threads 0, or crane_dyn_group_schedule):
// each shard's part, then the collective, grouped
int run_here(crane_dyn_group* g, const Job& j, const int64_t* const* d_now, const uint8_t* const* d_flags,
             int64_t* const* d_keys) {
    for (int i = 0; i < g->n; ++i) {
        Job ji = j;
        ji.d_now = d_now ? d_now[i] : nullptr;
        ji.d_flags = d_flags ? d_flags[i] : nullptr;
        ji.d_keys = d_keys[i];
        if (j.kind == kJobStep)  // (keys a held collective will reduce: it goes first)
            while (held_overlap(g, i, ji.d_keys, sizeof(int64_t) * (size_t)j.P)) {
                if (int rc = progress_here(g)) return rc;
                cpu_relax();
            }
        std::string msg;
        if (int rc = run_job_dev(g, i, ji, &msg)) {
            g->err = msg;
            return rc;
        }
        if (j.kind == kJobGroupColl && j.qmode) pcoll_push(g, i, ji);
    }
    if (j.kind == kJobGroupColl && j.qmode) return progress_here(g);
    if (!has_coll(j) || coll_count(j) <= 0) return 0;
    ncclResult_t r = ncclGroupStart();
    for (int i = 0; i < g->n && r == ncclSuccess; ++i)
        r = ncclAllReduce(d_keys[i], d_keys[i], (size_t)coll_count(j), ncclInt64, ncclMax, g->comm[(size_t)i],
                          coll_stream(g, j, i));
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess) return g->ncclfail(r, "ncclAllReduce");
    if (r2 != ncclSuccess) return g->ncclfail(r2, "ncclGroupEnd");
    if (j.kind == kJobGroupColl)
        for (int i = 0; i < g->n; ++i) {
            Job ji = j;
            ji.d_keys = d_keys[i];
            if (hipError_t e = note_pending(g, i, ji)) return g->hipfail(e, "collective event");
        }
    return 0;
}

// a job for every shard: to the workers, or run here
int dispatch_job(crane_dyn_group* g, const Job& j, const int64_t* const* d_now, const uint8_t* const* d_flags,
                 int64_t* const* d_keys) {
    if (g->use_workers()) {
        start_workers(g);
        for (int i = 0; i < g->n; ++i) {
            Job ji = j;
            ji.d_now = d_now ? d_now[i] : nullptr;
            ji.d_flags = d_flags ? d_flags[i] : nullptr;
            ji.d_keys = d_keys[i];
            g->workers[(size_t)i]->push(ji);
        }
        return 0;
    }
    return run_here(g, j, d_now, d_flags, d_keys);
}

int check_ready(crane_dyn_group* g) {
    if (g->n <= 0) return g->fail(CRANE_E_STATE, "group was not created successfully");
    if (g->N < 0) return g->fail(CRANE_E_STATE, "upload nodes before scheduling");
    return 0;
}

// (after wait_all) the dispatch queues, waited for; the engines forget them first
void free_queues(crane_dyn_group* g) {
    for (size_t s = 0; s < g->q.size(); ++s)
        for (size_t i = 0; i < g->q[s].size(); ++i)
            if (crane_queue*& qq = g->q[s][i]) {
                if (g->eng[s][i]) (void)crane_dyn_forget_queue(g->eng[s][i], qq);
                (void)crane_queue_destroy(qq);
                qq = nullptr;
            }
    g->q.clear();
}

// one queue per slot and shard, on first use; *qmode false when the runtime refuses them and
// the dispatch is automatic (HIP launches from then on)
int ensure_queues(crane_dyn_group* g, bool* qmode) {
    if (!*qmode || !g->q.empty()) return 0;
    g->q.assign((size_t)g->depth, std::vector<crane_queue*>((size_t)g->n, nullptr));
    for (int s = 0; s < g->depth; ++s)
        for (int i = 0; i < g->n; ++i) {
            crane_queue* qq = nullptr;
            if (crane_queue_create(g->dev[(size_t)i], g->ring_kind, &qq)) {
                const std::string m = std::string("crane_queue_create: ") + crane_queue_last_error(qq);
                (void)crane_queue_destroy(qq);
                free_queues(g);
                if (g->dispatch < 0) {  // (auto: a runtime that refuses the queues keeps HIP launches)
                    g->dispatch = 0;
                    *qmode = false;
                    return 0;
                }
                return g->fail(CRANE_E_HIP, m);
            }
            g->q[(size_t)s][(size_t)i] = qq;
            // the slot's K3s rides in its next step's first launch (flushed at wait_all)
            if (g->eng[(size_t)s][(size_t)i])
                (void)crane_dyn_set_option(g->eng[(size_t)s][(size_t)i], "step_defer", g->defer);
        }
    return 0;
}

// a routed call's node list: every index a node of the cluster
int check_nodes(crane_dyn_group* g, int64_t k, const int64_t* idx) {
    if (k < 0 || (k > 0 && !idx)) return g->fail(CRANE_E_INVALID, "bad node index array");
    for (int64_t j = 0; j < k; ++j)
        if (idx[j] < 0 || idx[j] >= g->N) return g->fail(CRANE_E_INVALID, "node index out of range");
    return 0;
}

// Routed update of k nodes: per shard, its nodes' local indices and columns gathered, the shard's
// slot-0 engine updated (the other slots follow), the answer rows (when asked) scattered back
int routed_update(crane_dyn_group* g, int64_t k, const int64_t* idx, const double* val, const int64_t* ts,
                  const double* hv, const int64_t* hv_ts, bool rows, int64_t t0, int64_t t1, uint8_t* n_steps,
                  int64_t* bp, int8_t* first_fail, int8_t* score) {
    if (int rc = check_ready(g)) return rc;
    if (int rc = check_nodes(g, k, idx)) return rc;
    crane_dyn* e00 = g->eng[0][0];
    const int64_t M = crane_dyn_num_metrics(e00);
    if (k > 0 && M > 0 && (!val || !ts)) return g->fail(CRANE_E_INVALID, "val/ts must not be NULL");
    if ((hv == nullptr) != (hv_ts == nullptr)) return g->fail(CRANE_E_INVALID, "hv and hv_ts must both be set or NULL");
    if (rows && k > 0 && (!n_steps || !bp || !first_fail || !score)) return g->fail(CRANE_E_INVALID, "NULL output");
    if (int rc = wait_all(g)) return rc;
    const size_t S = (size_t)crane_dyn_step_slots(e00);
    std::vector<uint8_t> ons;
    std::vector<int64_t> obp;
    std::vector<int8_t> off, osc;
    for (int i = 0; i < g->n; ++i) {
        g->r_pos.clear();
        for (int64_t j = 0; j < k; ++j)
            if (idx[j] >= g->lo[(size_t)i] && idx[j] < g->hi[(size_t)i]) g->r_pos.push_back(j);
        const size_t kk = g->r_pos.size();
        if (kk == 0) continue;
        g->r_idx.resize(kk);
        g->r_val.resize((size_t)M * kk);
        g->r_ts.resize((size_t)M * kk);
        g->r_hv.resize(kk);
        g->r_hvts.resize(kk);
        for (size_t a = 0; a < kk; ++a) {
            const int64_t j = g->r_pos[a];
            g->r_idx[a] = idx[j] - g->lo[(size_t)i];
            for (int64_t m = 0; m < M; ++m) {
                g->r_val[(size_t)m * kk + a] = val[m * k + j];
                g->r_ts[(size_t)m * kk + a] = ts[m * k + j];
            }
            if (hv) {
                g->r_hv[a] = hv[j];
                g->r_hvts[a] = hv_ts[j];
            }
        }
        crane_dyn* e = g->eng[0][(size_t)i];
        int rc;
        if (rows) {
            ons.resize(kk);
            obp.resize(kk * S);
            off.resize(kk * (S + 1));
            osc.resize(kk * (S + 1));
            rc = crane_dyn_update_node_steps(e, (int64_t)kk, g->r_idx.data(), g->r_val.data(), g->r_ts.data(),
                                             hv ? g->r_hv.data() : nullptr, hv ? g->r_hvts.data() : nullptr, t0, t1,
                                             ons.data(), obp.data(), off.data(), osc.data());
        } else {
            rc = crane_dyn_update_nodes(e, (int64_t)kk, g->r_idx.data(), g->r_val.data(), g->r_ts.data(),
                                        hv ? g->r_hv.data() : nullptr, hv ? g->r_hvts.data() : nullptr);
        }
        if (rc) return engine_err(g, e, rc, i);
        if (rows)
            for (size_t a = 0; a < kk; ++a) {
                const size_t j = (size_t)g->r_pos[a];
                n_steps[j] = ons[a];
                std::memcpy(bp + j * S, obp.data() + a * S, sizeof(int64_t) * S);
                std::memcpy(first_fail + j * (S + 1), off.data() + a * (S + 1), S + 1);
                std::memcpy(score + j * (S + 1), osc.data() + a * (S + 1), S + 1);
            }
    }
    return CRANE_OK;
}

}  // namespace

extern "C" {

int crane_shard_range(int64_t n_nodes, int32_t n_shards, int32_t shard, int64_t* lo, int64_t* hi) {
    if (n_nodes < 0 || n_shards <= 0 || shard < 0 || shard >= n_shards || !lo || !hi) return CRANE_E_INVALID;
    const int64_t q = n_nodes / n_shards, r = n_nodes % n_shards;
    *lo = (int64_t)shard * q + std::min<int64_t>(shard, r);
    *hi = *lo + q + (shard < r ? 1 : 0);
    return CRANE_OK;
}

int crane_dyn_group_create(const crane_policy* pol, int32_t n_dev, const int32_t* devices, int32_t depth,
                           crane_dyn_group** out) {
    if (!out) return CRANE_E_INVALID;
    crane_dyn_group* g = new crane_dyn_group();
    *out = g;  // returned on failure too (its error is readable); destroy it either way
    if (n_dev <= 0 || depth <= 0 || depth > 64) return g->fail(CRANE_E_INVALID, "n_dev must be > 0, depth in [1, 64]");
    int have = 0;
    hipError_t e = hipGetDeviceCount(&have);
    if (e != hipSuccess) return g->hipfail(e, "hipGetDeviceCount");
    std::vector<int> dv((size_t)n_dev);
    for (int i = 0; i < n_dev; ++i) {
        dv[(size_t)i] = devices ? devices[i] : i;
        if (dv[(size_t)i] < 0 || dv[(size_t)i] >= have)
            return g->fail(CRANE_E_INVALID, "device " + std::to_string(dv[(size_t)i]) + " not visible (" +
                                                std::to_string(have) + " devices)");
    }
    g->dev = dv;
    g->depth = depth;
    g->eng.assign((size_t)depth, std::vector<crane_dyn*>((size_t)n_dev, nullptr));
    g->st.assign((size_t)depth, std::vector<hipStream_t>((size_t)n_dev, nullptr));
    g->lo.assign((size_t)n_dev, 0);
    g->hi.assign((size_t)n_dev, 0);
    g->ctx.resize((size_t)n_dev);
    g->b_now.assign((size_t)n_dev, nullptr);
    g->b_keys.assign((size_t)n_dev, nullptr);
    g->b_flags.assign((size_t)n_dev, nullptr);
    // the slots' streams first, then the engines (each creates a stream of its own, idle here):
    // the runtime deals a device's streams round-robin over its hardware queues (4 on the box),
    // so the depth streams the batches run on get distinct queues
    for (int s = 0; s < depth; ++s)
        for (int i = 0; i < n_dev; ++i) {
            e = hipSetDevice(dv[(size_t)i]);
            if (e == hipSuccess) e = hipStreamCreateWithFlags(&g->st[(size_t)s][(size_t)i], hipStreamNonBlocking);
            if (e != hipSuccess) return g->hipfail(e, "hipStreamCreate");
        }
    for (int s = 0; s < depth; ++s)
        for (int i = 0; i < n_dev; ++i) {
            crane_dyn* eg = nullptr;
            int rc = crane_dyn_create(pol, dv[(size_t)i], &eg);
            g->eng[(size_t)s][(size_t)i] = eg;
            if (rc) {
                g->err = eg ? crane_dyn_last_error(eg) : "engine creation failed";
                return rc;
            }
            // one copy of the shard's nodes and log per shard: slot s > 0 shares slot 0's
            if (s > 0 && (rc = crane::engine_share_shard(eg, g->eng[0][(size_t)i]))) {
                g->err = crane_dyn_last_error(eg);
                return rc;
            }
        }
    g->n = n_dev;
    return CRANE_OK;
}

int crane_dyn_group_destroy(crane_dyn_group* g) {
    if (!g) return CRANE_OK;
    {
        std::lock_guard<std::mutex> l(g->mu);
        stop_workers(g);
        free_queues(g);  // (each waited for, and handed back by its engine, before the engines go)
        for (size_t i = 0; i < g->dev.size(); ++i) {
            if (hipSetDevice(g->dev[i]) == hipSuccess) (void)hipDeviceSynchronize();
        }
        for (ncclComm_t c : g->comm) (void)ncclCommDestroy(c);
        g->comm.clear();
        for (size_t s = 0; s < g->eng.size(); ++s)
            for (size_t i = 0; i < g->eng[s].size(); ++i) {
                if (g->eng[s][i]) crane_dyn_destroy(g->eng[s][i]);
                if (g->st[s][i]) {
                    (void)hipSetDevice(g->dev[i]);
                    (void)hipStreamDestroy(g->st[s][i]);
                }
            }
        for (size_t i = 0; i < g->ctx.size(); ++i) {
            DevCtx& c = g->ctx[i];
            (void)hipSetDevice(g->dev[i]);
            for (hipEvent_t ev : c.slot_ev)
                if (ev) (void)hipEventDestroy(ev);
            for (auto& pe : c.pending) (void)hipEventDestroy(pe.ev);
            for (hipEvent_t ev : c.free_ev) (void)hipEventDestroy(ev);
            if (c.cstream) (void)hipStreamDestroy(c.cstream);
        }
        for (size_t i = 0; i < g->b_now.size(); ++i) {
            (void)hipSetDevice(g->dev[i]);
            if (g->b_now[i]) (void)hipFree(g->b_now[i]);
            if (g->b_keys[i]) (void)hipFree(g->b_keys[i]);
            if (g->b_flags[i]) (void)hipFree(g->b_flags[i]);
        }
        if (g->h_keys) (void)hipHostFree(g->h_keys);
    }
    delete g;
    return CRANE_OK;
}

const char* crane_dyn_group_last_error(const crane_dyn_group* g) { return g ? g->err.c_str() : "null group"; }

int32_t crane_dyn_group_size(const crane_dyn_group* g) { return g ? g->n : 0; }

int crane_dyn_group_shard(const crane_dyn_group* g, int32_t i, int32_t* device, int64_t* lo, int64_t* hi) {
    if (!g || i < 0 || i >= g->n) return CRANE_E_INVALID;
    if (device) *device = g->dev[(size_t)i];
    if (lo) *lo = g->lo[(size_t)i];
    if (hi) *hi = g->hi[(size_t)i];
    return CRANE_OK;
}

crane_dyn* crane_dyn_group_engine(crane_dyn_group* g, int32_t i, int32_t slot) {
    if (!g || i < 0 || i >= g->n || slot < 0 || slot >= g->depth) return nullptr;
    return g->eng[(size_t)slot][(size_t)i];
}

int crane_dyn_group_set_option(crane_dyn_group* g, const char* name, int64_t value) {
    if (!g || !name) return CRANE_E_INVALID;
    GLock lk(g);
    if (g->n <= 0) return g->fail(CRANE_E_STATE, "group was not created successfully");
    const std::string nm = name;
    if (nm == "defer") {
        if (value < 0 || value > 1) return g->fail(CRANE_E_INVALID, "defer: 0 | 1");
        if (wait_all(g)) return CRANE_E_STATE;
        g->defer = (int)value;
        for (auto& row : g->eng)
            for (crane_dyn* e : row)
                if (e) (void)crane_dyn_set_option(e, "step_defer", g->q.empty() ? 0 : value);
        return 0;
    }
    if (nm == "dispatch" || nm == "dispatch_ring") {
        if (value < (nm == "dispatch" ? -1 : 0) || value > 1)
            return g->fail(CRANE_E_INVALID, nm + (nm == "dispatch" ? ": -1 | 0 | 1" : ": 0 | 1"));
        if (int rc = wait_all(g)) return rc;
        free_queues(g);  // (the engines wait for the queues they used at their next state change: none now)
        (nm == "dispatch" ? g->dispatch : g->ring_kind) = (int)value;
        return CRANE_OK;
    }
    if (nm == "collective" || nm == "threads") {
        if (int rc = wait_all(g)) return rc;
        if (nm == "collective") {
            if (value < 0 || value > 2) return g->fail(CRANE_E_INVALID, "collective: 0 | 1 | 2");
            g->collective = (int)value;
        } else {
            if (value < -1 || value > 1) return g->fail(CRANE_E_INVALID, "threads: -1 | 0 | 1");
            stop_workers(g);
            g->threads = (int)value;
        }
        return CRANE_OK;
    }
    for (auto& row : g->eng)
        for (size_t i = 0; i < row.size(); ++i)
            if (int rc = crane_dyn_set_option(row[i], name, value)) return engine_err(g, row[i], rc, (int)i);
    return CRANE_OK;
}

int crane_dyn_group_upload_nodes(crane_dyn_group* g, int64_t n_nodes, const double* val, const int64_t* ts,
                                 const double* hv, const int64_t* hv_ts) {
    if (!g) return CRANE_E_INVALID;
    GLock lk(g);
    if (g->n <= 0) return g->fail(CRANE_E_STATE, "group was not created successfully");
    if (n_nodes < 0 || n_nodes > 0xFFFFFFFFLL) return g->fail(CRANE_E_INVALID, "node count out of range");
    if ((hv == nullptr) != (hv_ts == nullptr)) return g->fail(CRANE_E_INVALID, "hv and hv_ts must both be set or NULL");
    const int64_t M = crane_dyn_num_metrics(g->eng[0][0]);
    if (n_nodes > 0 && M > 0 && (!val || !ts)) return g->fail(CRANE_E_INVALID, "val/ts must not be NULL");
    if (int rc = wait_all(g)) return rc;
    std::vector<double> v;
    std::vector<int64_t> t;
    for (int i = 0; i < g->n; ++i) {
        int64_t lo, hi;
        crane_shard_range(n_nodes, g->n, i, &lo, &hi);
        const int64_t k = hi - lo;
        // this shard's columns of the [M][N] rows, contiguous
        v.resize((size_t)(M * k));
        t.resize((size_t)(M * k));
        for (int64_t m = 0; m < M; ++m) {
            if (k == 0) break;
            std::memcpy(&v[(size_t)(m * k)], val + m * n_nodes + lo, sizeof(double) * (size_t)k);
            std::memcpy(&t[(size_t)(m * k)], ts + m * n_nodes + lo, sizeof(int64_t) * (size_t)k);
        }
        crane_dyn* e = g->eng[0][(size_t)i];  // (the shard's other slots share it)
        int rc = crane_dyn_upload_nodes(e, k, lo, v.data(), t.data(), hv ? hv + lo : nullptr,
                                        hv_ts ? hv_ts + lo : nullptr);
        if (rc) return engine_err(g, e, rc, i);
        g->lo[(size_t)i] = lo;
        g->hi[(size_t)i] = hi;
    }
    g->N = n_nodes;
    return CRANE_OK;
}

int crane_dyn_group_upload_bindings(crane_dyn_group* g, int64_t n, const int32_t* node, const int64_t* ts_s) {
    if (!g) return CRANE_E_INVALID;
    GLock lk(g);
    if (int rc = check_ready(g)) return rc;
    if (n < 0 || (n > 0 && (!node || !ts_s))) return g->fail(CRANE_E_INVALID, "bad binding arrays");
    if (int rc = wait_all(g)) return rc;
    std::vector<int32_t> bn;
    std::vector<int64_t> bt;
    for (int i = 0; i < g->n; ++i) {
        const int64_t lo = g->lo[(size_t)i], hi = g->hi[(size_t)i];
        bn.clear();
        bt.clear();
        for (int64_t b = 0; b < n; ++b)  // this shard's bindings, local indices, in log order
            if (node[b] >= lo && node[b] < hi) {
                bn.push_back((int32_t)(node[b] - lo));
                bt.push_back(ts_s[b]);
            }
        crane_dyn* e = g->eng[0][(size_t)i];
        int rc = crane_dyn_upload_bindings(e, (int64_t)bn.size(), bn.data(), bt.data());
        if (rc) return engine_err(g, e, rc, i);
    }
    return CRANE_OK;
}

int crane_dyn_group_update_nodes(crane_dyn_group* g, int64_t k, const int64_t* idx, const double* val,
                                 const int64_t* ts, const double* hv, const int64_t* hv_ts) {
    if (!g) return CRANE_E_INVALID;
    GLock lk(g);
    return routed_update(g, k, idx, val, ts, hv, hv_ts, false, 0, 0, nullptr, nullptr, nullptr, nullptr);
}

int crane_dyn_group_update_node_steps(crane_dyn_group* g, int64_t k, const int64_t* idx, const double* val,
                                      const int64_t* ts, const double* hv, const int64_t* hv_ts, int64_t t0_ns,
                                      int64_t t1_ns, uint8_t* n_steps, int64_t* bp, int8_t* first_fail, int8_t* score) {
    if (!g) return CRANE_E_INVALID;
    GLock lk(g);
    if (!(t0_ns < t1_ns)) return g->fail(CRANE_E_INVALID, "t0 must be before t1");
    return routed_update(g, k, idx, val, ts, hv, hv_ts, true, t0_ns, t1_ns, n_steps, bp, first_fail, score);
}

int crane_dyn_group_resize_nodes(crane_dyn_group* g, int64_t n) {
    if (!g) return CRANE_E_INVALID;
    GLock lk(g);
    if (int rc = check_ready(g)) return rc;
    if (n < 0 || n > 0xFFFFFFFFLL) return g->fail(CRANE_E_INVALID, "node count out of range");
    if (n == g->N) return CRANE_OK;
    if (int rc = wait_all(g)) return rc;
    // the cluster's node range changes at its end: the last shard grows; shrinking empties the
    // shards from the end (global indices stay where they are)
    for (int i = 0; i < g->n; ++i) {
        const int64_t lo = g->lo[(size_t)i];
        const int64_t nhi = i == g->n - 1 ? std::max(lo, n) : std::max(lo, std::min(g->hi[(size_t)i], n));
        if (nhi == g->hi[(size_t)i]) continue;
        crane_dyn* e = g->eng[0][(size_t)i];
        if (int rc = crane_dyn_resize_nodes(e, nhi - lo)) return engine_err(g, e, rc, i);
        g->hi[(size_t)i] = nhi;
    }
    g->N = n;
    return CRANE_OK;
}

int crane_dyn_group_binding_records(crane_dyn_group* g, int64_t size, int64_t gc_time_range_ns) {
    if (!g) return CRANE_E_INVALID;
    GLock lk(g);
    if (int rc = check_ready(g)) return rc;
    if (int rc = wait_all(g)) return rc;
    for (int i = 0; i < g->n; ++i)
        if (int rc = crane_dyn_binding_records(g->eng[0][(size_t)i], size, gc_time_range_ns))
            return engine_err(g, g->eng[0][(size_t)i], rc, i);
    return CRANE_OK;
}

int crane_dyn_group_add_bindings(crane_dyn_group* g, int64_t n, const int32_t* node, const int64_t* ts_s) {
    if (!g) return CRANE_E_INVALID;
    GLock lk(g);
    if (int rc = check_ready(g)) return rc;
    if (n < 0 || (n > 0 && (!node || !ts_s))) return g->fail(CRANE_E_INVALID, "bad binding arrays");
    if (int rc = wait_all(g)) return rc;
    // every shard takes every binding (the same heap everywhere: its order is by timestamp only,
    // binding.go:25-47), the nodes of other shards as "no node"
    g->r_node.resize((size_t)n);
    for (int i = 0; i < g->n; ++i) {
        const int64_t lo = g->lo[(size_t)i], hi = g->hi[(size_t)i];
        for (int64_t b = 0; b < n; ++b)
            g->r_node[(size_t)b] = node[b] >= lo && node[b] < hi ? (int32_t)(node[b] - lo) : -1;
        if (int rc = crane_dyn_add_bindings(g->eng[0][(size_t)i], n, g->r_node.data(), ts_s))
            return engine_err(g, g->eng[0][(size_t)i], rc, i);
    }
    return CRANE_OK;
}

int crane_dyn_group_gc_bindings(crane_dyn_group* g, int64_t now_ns) {
    if (!g) return CRANE_E_INVALID;
    GLock lk(g);
    if (int rc = check_ready(g)) return rc;
    if (int rc = wait_all(g)) return rc;
    for (int i = 0; i < g->n; ++i)
        if (int rc = crane_dyn_gc_bindings(g->eng[0][(size_t)i], now_ns)) return engine_err(g, g->eng[0][(size_t)i], rc, i);
    return CRANE_OK;
}

int64_t crane_dyn_group_binding_count(crane_dyn_group* g) {
    if (!g) return CRANE_E_INVALID;
    GLock lk(g);
    if (g->n <= 0) return g->fail(CRANE_E_STATE, "group was not created successfully");
    return crane_dyn_binding_count(g->eng[0][0]);
}

int crane_dyn_group_refresh_hot_values(crane_dyn_group* g, int64_t now_ns, int64_t hv_ts_ns) {
    if (!g) return CRANE_E_INVALID;
    GLock lk(g);
    if (int rc = check_ready(g)) return rc;
    if (int rc = wait_all(g)) return rc;
    for (int i = 0; i < g->n; ++i)
        if (int rc = crane_dyn_refresh_hot_values(g->eng[0][(size_t)i], now_ns, hv_ts_ns))
            return engine_err(g, g->eng[0][(size_t)i], rc, i);
    return CRANE_OK;
}

int crane_dyn_group_hot_values(crane_dyn_group* g, int64_t n, double* hv_out) {
    if (!g) return CRANE_E_INVALID;
    GLock lk(g);
    if (int rc = check_ready(g)) return rc;
    if (n != g->N || (n > 0 && !hv_out)) return g->fail(CRANE_E_INVALID, "hv_out must hold one value per node");
    if (int rc = wait_all(g)) return rc;
    for (int i = 0; i < g->n; ++i) {
        const int64_t lo = g->lo[(size_t)i], k = g->hi[(size_t)i] - lo;
        if (int rc = crane_dyn_hot_values(g->eng[0][(size_t)i], k, hv_out + lo))
            return engine_err(g, g->eng[0][(size_t)i], rc, i);
    }
    return CRANE_OK;
}

int crane_dyn_group_node_steps(crane_dyn_group* g, int64_t t0_ns, int64_t t1_ns, int64_t n, uint8_t* n_steps,
                               int64_t* bp, int8_t* first_fail, int8_t* score) {
    if (!g) return CRANE_E_INVALID;
    GLock lk(g);
    if (int rc = check_ready(g)) return rc;
    if (n != g->N) return g->fail(CRANE_E_INVALID, "n must be the cluster's node count");
    if (int rc = wait_all(g)) return rc;
    const int64_t S = crane_dyn_step_slots(g->eng[0][0]);
    for (int i = 0; i < g->n; ++i) {
        const int64_t lo = g->lo[(size_t)i], k = g->hi[(size_t)i] - lo;
        if (k == 0) continue;
        crane_dyn* e = g->eng[0][(size_t)i];
        if (int rc = crane_dyn_node_steps(e, t0_ns, t1_ns, k, n_steps + lo, bp + lo * S, first_fail + lo * (S + 1),
                                          score + lo * (S + 1)))
            return engine_err(g, e, rc, i);
    }
    return CRANE_OK;
}

int crane_dyn_group_step_keys_async(crane_dyn_group* g, int64_t now_ns, int64_t hv_ts_ns, int64_t n_pods,
                                    const int64_t* const* d_now, const uint8_t* const* d_flags,
                                    int64_t* const* d_keys) {
    if (!g) return CRANE_E_INVALID;
    GLock lk(g);
    if (int rc = check_ready(g)) return rc;
    if (n_pods < 0 || (n_pods > 0 && (!d_now || !d_keys))) return g->fail(CRANE_E_INVALID, "bad pod arrays");
    for (int i = 0; i < g->n && n_pods > 0; ++i)
        if (!d_now[i] || !d_keys[i]) return g->fail(CRANE_E_INVALID, "NULL device pointer");
    if (int rc = ensure_comms(g)) return rc;
    // a per-batch collective follows each batch on its HIP stream: no queues with it
    bool qmode = g->dispatch == 1 || (g->dispatch < 0 && !g->use_coll());
    if (qmode && g->use_coll())
        return g->fail(CRANE_E_STATE, "dispatch 1 (queues) with the per-batch collective: use "
                                      "crane_dyn_group_step_keys_batch, or \"dispatch\" 0");
    if (int rc = ensure_queues(g, &qmode)) return rc;
    Job j;
    j.now = now_ns;
    j.hv_ts = hv_ts_ns;
    j.P = n_pods;
    j.slot = (int)(g->batch++ % (uint64_t)g->depth);
    j.qmode = qmode;
    j.per_batch_coll = g->use_coll();
    return dispatch_job(g, j, d_now, d_flags, d_keys);
}

int crane_dyn_group_step_keys_batch(crane_dyn_group* g, int32_t n_batches, const int64_t* now_ns,
                                    const int64_t* hv_ts_ns, int64_t n_pods, const int64_t* const* d_now,
                                    const uint8_t* const* d_flags, int64_t* const* d_keys) {
    if (!g) return CRANE_E_INVALID;
    GLock lk(g);
    if (int rc = check_ready(g)) return rc;
    if (n_batches < 0 || (n_batches > 0 && (!now_ns || !hv_ts_ns)))
        return g->fail(CRANE_E_INVALID, "bad batch time arrays");
    if (n_pods < 0 || (n_pods > 0 && (!d_now || !d_keys))) return g->fail(CRANE_E_INVALID, "bad pod arrays");
    for (int i = 0; i < g->n && n_pods > 0; ++i)
        if (!d_now[i] || !d_keys[i]) return g->fail(CRANE_E_INVALID, "NULL device pointer");
    if (n_batches == 0 || n_pods == 0) return CRANE_OK;
    if (int rc = ensure_comms(g)) return rc;
    bool qmode = g->dispatch != 0;
    if (int rc = ensure_queues(g, &qmode)) return rc;
    const bool coll = g->use_coll();
    if (int rc = ensure_ctx(g)) return rc;
    const size_t P = (size_t)n_pods;
    std::vector<const int64_t*> pn((size_t)g->n);
    std::vector<const uint8_t*> pf((size_t)g->n);
    std::vector<int64_t*> pk((size_t)g->n);
    uint64_t slots = 0;
    for (int32_t b = 0; b < n_batches; ++b) {
        Job j;
        j.now = now_ns[b];
        j.hv_ts = hv_ts_ns[b];
        j.P = n_pods;
        j.slot = (int)(g->batch++ % (uint64_t)g->depth);
        j.qmode = qmode;
        slots |= 1ull << j.slot;
        for (int i = 0; i < g->n; ++i) {
            pn[(size_t)i] = d_now[i] + (size_t)b * P;
            pf[(size_t)i] = d_flags && d_flags[i] ? d_flags[i] + (size_t)b * P : nullptr;
            pk[(size_t)i] = d_keys[i] + (size_t)b * P;
        }
        if (int rc = dispatch_job(g, j, pn.data(), pf.data(), pk.data())) return rc;
    }
    if (!coll) return CRANE_OK;
    // one in-place all-reduce of the batches' keys [n_batches][P] per device, on its collective
    // stream after every slot these batches ran on
    Job c;
    c.kind = kJobGroupColl;
    c.slots = slots;
    c.qmode = qmode;
    c.count = (int64_t)n_batches * n_pods;
    return dispatch_job(g, c, nullptr, nullptr, d_keys);
}

int crane_dyn_group_sync(crane_dyn_group* g) {
    if (!g) return CRANE_E_INVALID;
    GLock lk(g);
    return wait_all(g);
}

int crane_dyn_group_schedule(crane_dyn_group* g, int64_t now_ns, int64_t hv_ts_ns, int64_t n_pods,
                             const int64_t* now_pods, const uint8_t* pod_flags, int64_t* chosen, int64_t* chosen_score) {
    if (!g) return CRANE_E_INVALID;
    GLock lk(g);
    if (int rc = check_ready(g)) return rc;
    if (n_pods < 0 || (n_pods > 0 && !now_pods)) return g->fail(CRANE_E_INVALID, "bad pod arrays");
    if (n_pods == 0) return CRANE_OK;
    if (int rc = wait_all(g)) return rc;
    if (int rc = ensure_comms(g)) return rc;
    bool qmode = g->dispatch == 1 || (g->dispatch < 0 && !g->use_coll());
    if (qmode && g->use_coll())
        return g->fail(CRANE_E_STATE, "dispatch 1 (queues) with the per-batch collective: \"dispatch\" 0");
    if (int rc = ensure_queues(g, &qmode)) return rc;
    const size_t P = (size_t)n_pods;
    if (P > g->b_cap) {
        for (int i = 0; i < g->n; ++i) {
            hipError_t e = hipSetDevice(g->dev[(size_t)i]);
            if (g->b_now[(size_t)i]) (void)hipFree(g->b_now[(size_t)i]);
            if (g->b_keys[(size_t)i]) (void)hipFree(g->b_keys[(size_t)i]);
            if (g->b_flags[(size_t)i]) (void)hipFree(g->b_flags[(size_t)i]);
            g->b_now[(size_t)i] = g->b_keys[(size_t)i] = nullptr;
            g->b_flags[(size_t)i] = nullptr;
            if (e == hipSuccess) e = hipMalloc((void**)&g->b_now[(size_t)i], sizeof(int64_t) * P);
            if (e == hipSuccess) e = hipMalloc((void**)&g->b_keys[(size_t)i], sizeof(int64_t) * P);
            if (e == hipSuccess) e = hipMalloc((void**)&g->b_flags[(size_t)i], P);
            if (e != hipSuccess) {
                g->b_cap = 0;
                return g->hipfail(e, "hipMalloc");
            }
        }
        g->b_cap = P;
    }
    const size_t hk = P * (size_t)(g->use_coll() ? 1 : g->n);
    if (hk > g->h_cap) {
        if (g->h_keys) (void)hipHostFree(g->h_keys);
        g->h_keys = nullptr;
        g->h_cap = 0;
        hipError_t e = hipHostMalloc((void**)&g->h_keys, sizeof(int64_t) * hk, hipHostMallocDefault);
        if (e != hipSuccess) return g->hipfail(e, "hipHostMalloc");
        g->h_cap = hk;
    }
    // a batch like the asynchronous ones (its slot counted in g->batch): every later wait_all —
    // this call's error path, the next call's start before it may reallocate the pod buffers —
    // waits for its streams and queues
    const int slot = (int)(g->batch++ % (uint64_t)g->depth);
    for (int i = 0; i < g->n; ++i) {
        hipStream_t s = g->st[(size_t)slot][(size_t)i];
        hipError_t e = hipSetDevice(g->dev[(size_t)i]);
        if (e == hipSuccess) e = hipMemcpyAsync(g->b_now[(size_t)i], now_pods, sizeof(int64_t) * P, hipMemcpyHostToDevice, s);
        if (e == hipSuccess)
            e = pod_flags ? hipMemcpyAsync(g->b_flags[(size_t)i], pod_flags, P, hipMemcpyHostToDevice, s)
                          : hipMemsetAsync(g->b_flags[(size_t)i], 0, P, s);
        if (e == hipSuccess && qmode) e = hipStreamSynchronize(s);  // (a queue orders with nothing)
        if (e != hipSuccess) {
            (void)wait_all(g);
            return g->hipfail(e, "pod upload");
        }
    }
    Job j;
    j.now = now_ns;
    j.hv_ts = hv_ts_ns;
    j.P = n_pods;
    j.slot = slot;
    j.qmode = qmode;
    j.per_batch_coll = g->use_coll();
    std::vector<const int64_t*> pn(g->b_now.begin(), g->b_now.end());
    std::vector<const uint8_t*> pf(g->b_flags.begin(), g->b_flags.end());
    if (int rc = run_here(g, j, pn.data(), pf.data(), g->b_keys.data())) {
        const std::string m = g->err;
        (void)wait_all(g);
        g->err = m;
        return rc;
    }
    // the combined keys from device 0; without the collective every shard's, max-combined here
    const int nk = g->use_coll() ? 1 : g->n;
    for (int i = 0; i < nk; ++i) {
        hipStream_t s = g->st[(size_t)slot][(size_t)i];
        // (the step's deferred K3s, option step_defer: run now)
        if (int rc = crane_dyn_step_flush(g->eng[(size_t)slot][(size_t)i])) return engine_err(g, g->eng[(size_t)slot][(size_t)i], rc, i);
        if (crane_queue* qq = qmode ? g->queue(slot, i) : nullptr)
            if (crane_queue_wait(qq)) return g->fail(CRANE_E_HIP, std::string("queue: ") + crane_queue_last_error(qq));
        hipError_t e = hipSetDevice(g->dev[(size_t)i]);
        if (e == hipSuccess)
            e = hipMemcpyAsync(g->h_keys + (size_t)i * P, g->b_keys[(size_t)i], sizeof(int64_t) * P,
                               hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return g->hipfail(e, "key readback");
    }
    for (size_t p = 0; p < P; ++p) {
        int64_t k = g->h_keys[p];
        for (int i = 1; i < nk; ++i) k = std::max(k, g->h_keys[(size_t)i * P + p]);
        int64_t sc = -1;
        const int64_t nd = crane_dyn_key_node(k, &sc);
        if (chosen) chosen[p] = nd;
        if (chosen_score) chosen_score[p] = sc;
    }
    return CRANE_OK;
}

}  // extern "C"
