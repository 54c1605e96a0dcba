// group.cpp — one process driving N devices: the node-shard engine behind the C ABI
// (crane_dyn_group_* in include/crane_dyn.h).
//
// Reference: the scheduler is ONE Go process (cmd/scheduler/main.go:18-32) holding ONE plugin
// instance (NewDynamicScheduler, pkg/plugins/dynamic/plugins.go:105-120), so the node-shard
// path SURVEY §8(b)/(e) describes — nodes split across the GPUs of one node, each shard's
// best (score, node) packed into an int64 and max-combined over xGMI — has to be reachable
// from a single caller through the C ABI.  A group holds, per device, `depth` engines
// (crane_dyn, one per batch in flight) over that device's contiguous node range, their HIP
// streams, and one RCCL communicator per device from ncclCommInitAll.  A batch runs the
// shard step (K2 hot values + K1 node pass + K3 Filter/Score/argmax, engine.hip) on every
// device, then an in-place ncclAllReduce(int64, ncclMax) of the per-pod keys on the same
// stream: afterwards every device holds the global choice.
//
// Enqueueing: a step costs the host ~9 us of HIP kernel launches per device (~4 us on the
// dispatch queues, aql.cpp, which the group uses unless the collective runs: RCCL's kernels are
// on HIP streams, which a queue is not ordered with), so one thread feeding eight devices would
// leave them idle.  With more than one device each device has
// a worker thread (spinning briefly, then sleeping) that takes the batch descriptors the
// caller pushes and enqueues its device's step and its part of the all-reduce on its own
// communicator (RCCL's one-thread-per-device usage); the caller only pushes descriptors.
// Option "threads" 0 instead enqueues everything from the caller's thread, the collective
// inside ncclGroupStart / ncclGroupEnd (RCCL's one-thread-many-devices usage).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/crane_dyn.h"

namespace {

struct Job {
    int64_t now, hv_ts, P;
    const int64_t* d_now;
    const uint8_t* d_flags;
    int64_t* d_keys;
    int slot;
};

inline void cpu_relax() { __builtin_ia32_pause(); }

}  // namespace

struct GroupWorker;

struct crane_dyn_group {
    std::mutex mu;  // serialises the ABI calls on the group
    std::string err;
    int n = 0, depth = 1;
    std::vector<int> dev;
    std::vector<std::vector<crane_dyn*>> eng;  // [slot][device index]
    std::vector<std::vector<hipStream_t>> st;  // [slot][device index]
    std::vector<ncclComm_t> comm;              // [device index], created on first use
    std::vector<int64_t> lo, hi;               // node shard of each device
    int64_t N = -1;
    int collective = 1;  // 0: never (a host max combines), 1: when n > 1, 2: always (tests at n = 1)
    int threads = -1;    // -1: worker threads when n > 1, 0: the caller's thread, 1: worker threads
    // 0: the steps' kernels on the slots' HIP streams; 1: on user-mode AQL queues (crane_queue, one
    // per slot and device, created on first use; no collective); -1: queues unless the collective
    // runs.  ring_kind of their kernargs
    int dispatch = -1, ring_kind = 0;
    std::vector<std::vector<crane_queue*>> q;  // [slot][device index]
    bool comm_broken = false;
    uint64_t batch = 0;
    uint64_t synced = 0;  // batch at the last wait_all: the slots used since are the ones to wait for
    std::vector<std::unique_ptr<GroupWorker>> workers;
    // crane_dyn_group_schedule's device buffers per device, and its pinned key staging
    std::vector<int64_t*> b_now, b_keys;
    std::vector<uint8_t*> b_flags;
    size_t b_cap = 0;
    int64_t* h_keys = nullptr;
    size_t h_cap = 0;

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
    bool use_queues() const { return dispatch == 1 || (dispatch < 0 && !use_coll()); }
    crane_queue* queue(int slot, int i) const { return use_queues() && !q.empty() ? q[(size_t)slot][(size_t)i] : nullptr; }
    bool use_workers() const { return threads == 1 || (threads < 0 && n > 1); }
};

struct GroupWorker {
    static constexpr uint64_t kRing = 256;
    crane_dyn_group* g = nullptr;
    int i = 0;
    std::thread th;
    Job ring[kRing];
    std::atomic<uint64_t> head{0}, tail{0};
    std::atomic<bool> stop{false};
    std::atomic<int> sleeping{0};
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

    // One batch on this device: the shard step, then this device's part of the all-reduce
    // (always issued once the group uses the collective, even after a failed step: the other
    // devices' all-reduce kernels wait for this one's).
    void run_job(const Job& j) {
        crane_dyn* e = g->eng[j.slot][i];
        hipStream_t s = g->st[j.slot][i];
        crane_queue* qq = g->queue(j.slot, i);
        if (g->hi[i] > g->lo[i]) {
            if (qq ? crane_dyn_step_keys_queue(e, j.now, j.hv_ts, j.P, j.d_now, j.d_flags, j.d_keys, qq)
                   : crane_dyn_step_keys_async(e, j.now, j.hv_ts, j.P, j.d_now, j.d_flags, j.d_keys, s))
                record(CRANE_E_HIP, std::string("device ") + std::to_string(g->dev[i]) + ": " + crane_dyn_last_error(e));
        } else if (j.P > 0) {  // an empty shard contributes "no node"
            hipError_t r = hipMemsetAsync(j.d_keys, 0xFF, sizeof(int64_t) * (size_t)j.P, s);
            if (r == hipSuccess && qq) r = hipStreamSynchronize(s);  // (queues: wait_all waits for those only)
            if (r != hipSuccess) record(CRANE_E_HIP, hipGetErrorString(r));
        }
        if (g->use_coll() && j.P > 0) {
            ncclResult_t r = ncclAllReduce(j.d_keys, j.d_keys, (size_t)j.P, ncclInt64, ncclMax, g->comm[i], s);
            if (r != ncclSuccess) record(CRANE_E_HIP, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
        }
    }

    void loop() {
        (void)hipSetDevice(g->dev[i]);
        uint64_t t = tail.load(std::memory_order_relaxed);
        for (;;) {
            uint64_t h = head.load(std::memory_order_acquire);
            for (int spins = 0; h == t; h = head.load(std::memory_order_acquire)) {
                if (stop.load(std::memory_order_acquire)) return;
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
        while (tail.load(std::memory_order_acquire) != head.load(std::memory_order_acquire)) cpu_relax();
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

// wait for every pushed batch and every stream of the group; the first error since the last wait
int wait_all(crane_dyn_group* g) {
    int rc = 0;
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
            if (crane_queue* qq = g->queue((int)s, i)) {
                if (crane_queue_wait(qq) && !rc) rc = g->fail(CRANE_E_HIP, std::string("queue: ") + crane_queue_last_error(qq));
                continue;
            }
            hipError_t e = hipSetDevice(g->dev[(size_t)i]);
            if (e == hipSuccess) e = hipStreamSynchronize(g->st[s][(size_t)i]);
            if (e != hipSuccess && !rc) rc = g->hipfail(e, "hipStreamSynchronize");
        }
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

int engine_err(crane_dyn_group* g, crane_dyn* e, int rc, int i) {
    g->err = std::string("device ") + std::to_string(g->dev[(size_t)i]) + ": " + crane_dyn_last_error(e);
    return rc;
}

// one batch on every device from the caller's thread (threads 0, or crane_dyn_group_schedule)
int step_here(crane_dyn_group* g, const Job& j, const int64_t* const* d_now, const uint8_t* const* d_flags,
              int64_t* const* d_keys) {
    for (int i = 0; i < g->n; ++i) {
        crane_dyn* e = g->eng[(size_t)j.slot][(size_t)i];
        hipStream_t s = g->st[(size_t)j.slot][(size_t)i];
        crane_queue* qq = g->queue(j.slot, i);
        if (g->hi[(size_t)i] > g->lo[(size_t)i]) {
            const uint8_t* fl = d_flags ? d_flags[i] : nullptr;
            int rc = qq ? crane_dyn_step_keys_queue(e, j.now, j.hv_ts, j.P, d_now[i], fl, d_keys[i], qq)
                        : crane_dyn_step_keys_async(e, j.now, j.hv_ts, j.P, d_now[i], fl, d_keys[i], s);
            if (rc) return engine_err(g, e, rc, i);
        } else if (j.P > 0) {
            hipError_t r = hipSetDevice(g->dev[(size_t)i]);
            if (r == hipSuccess) r = hipMemsetAsync(d_keys[i], 0xFF, sizeof(int64_t) * (size_t)j.P, s);
            if (r == hipSuccess && qq) r = hipStreamSynchronize(s);
            if (r != hipSuccess) return g->hipfail(r, "hipMemsetAsync");
        }
    }
    if (g->use_coll() && j.P > 0) {
        ncclResult_t r = ncclGroupStart();
        for (int i = 0; i < g->n && r == ncclSuccess; ++i)
            r = ncclAllReduce(d_keys[i], d_keys[i], (size_t)j.P, ncclInt64, ncclMax, g->comm[(size_t)i],
                              g->st[(size_t)j.slot][(size_t)i]);
        const ncclResult_t r2 = ncclGroupEnd();
        if (r != ncclSuccess) return g->ncclfail(r, "ncclAllReduce");
        if (r2 != ncclSuccess) return g->ncclfail(r2, "ncclGroupEnd");
    }
    return 0;
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

// dispatch 1: one queue per slot and device, on first use
int ensure_queues(crane_dyn_group* g) {
    if (!g->use_queues() || !g->q.empty()) return 0;
    if (g->use_coll())
        return g->fail(CRANE_E_STATE, "dispatch 1 (queues) has no collective: set \"collective\" 0 or \"dispatch\" 0");
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
                    return 0;
                }
                return g->fail(CRANE_E_HIP, m);
            }
            g->q[(size_t)s][(size_t)i] = qq;
        }
    return 0;
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
        for (size_t i = 0; i < g->dev.size(); ++i) {
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
            free_queues(g);  // (dispatch -1 follows the collective)
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
    std::vector<double> v, h;
    std::vector<int64_t> t, ht;
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
        for (int s = 0; s < g->depth; ++s) {
            crane_dyn* e = g->eng[(size_t)s][(size_t)i];
            int rc = crane_dyn_upload_nodes(e, k, lo, v.data(), t.data(), hv ? hv + lo : nullptr,
                                            hv_ts ? hv_ts + lo : nullptr);
            if (rc) return engine_err(g, e, rc, i);
        }
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
        for (int s = 0; s < g->depth; ++s) {
            crane_dyn* e = g->eng[(size_t)s][(size_t)i];
            int rc = crane_dyn_upload_bindings(e, (int64_t)bn.size(), bn.data(), bt.data());
            if (rc) return engine_err(g, e, rc, i);
        }
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
    if (int rc = ensure_queues(g)) return rc;
    const int slot = (int)(g->batch++ % (uint64_t)g->depth);
    Job j{now_ns, hv_ts_ns, n_pods, nullptr, nullptr, nullptr, slot};
    if (g->use_workers()) {
        start_workers(g);
        for (int i = 0; i < g->n; ++i) {
            j.d_now = d_now[i];
            j.d_flags = d_flags ? d_flags[i] : nullptr;
            j.d_keys = d_keys[i];
            g->workers[(size_t)i]->push(j);
        }
        return CRANE_OK;
    }
    return step_here(g, j, d_now, d_flags, d_keys);
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
    if (int rc = ensure_queues(g)) return rc;
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
        if (e == hipSuccess && g->queue(slot, i)) e = hipStreamSynchronize(s);  // (a queue orders with nothing)
        if (e != hipSuccess) {
            (void)wait_all(g);
            return g->hipfail(e, "pod upload");
        }
    }
    Job j{now_ns, hv_ts_ns, n_pods, nullptr, nullptr, nullptr, slot};
    std::vector<const int64_t*> pn(g->b_now.begin(), g->b_now.end());
    std::vector<const uint8_t*> pf(g->b_flags.begin(), g->b_flags.end());
    if (int rc = step_here(g, j, pn.data(), pf.data(), g->b_keys.data())) {
        const std::string m = g->err;
        (void)wait_all(g);
        g->err = m;
        return rc;
    }
    // the combined keys from device 0; without the collective every shard's, max-combined here
    const int nk = g->use_coll() ? 1 : g->n;
    for (int i = 0; i < nk; ++i) {
        hipStream_t s = g->st[(size_t)slot][(size_t)i];
        if (crane_queue* qq = g->queue(slot, i))
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
