// engine.hip — the C ABI of include/crane_dyn.h: engine lifecycle, device
// buffers, policy flattening and the pipeline K2 -> K1 -> K3 on a HIP stream.
//
// Reference mapping (/root/reference):
//   crane_dyn_create      NewDynamicScheduler      pkg/plugins/dynamic/plugins.go:105-120
//   policy flattening     getActiveDuration        pkg/plugins/dynamic/stats.go:140-150
//   crane_dyn_eval*       Filter + Score + select  plugins.go:39-98 (+ upstream selectHost)
//   refresh_hot_values    GetLastNodeBindingCount  pkg/controller/annotator/binding.go:81-97
//                         annotateNodeHotValue     pkg/controller/annotator/node.go:113-121
//   binding records       BindingRecords heap      binding.go:50-123 (bindings.hpp)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/crane_dyn.h"
#include "bindings.hpp"
#include "dyn_types.hpp"
#include "kernels.hpp"

using namespace crane;

namespace {

// A buffer replaced during a step on a dispatch queue (a first batch sizing its scratch) may
// still be read by the packets this thread put on that queue: wait for them first (hipFree
// waits for HIP's own queues only)
hipError_t before_free() { return crane::tl_aql ? crane::aql_wait(crane::tl_aql) : hipSuccess; }

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;  // elements
    hipError_t reserve(size_t want) {
        if (want <= n && p) return hipSuccess;
        if (p) {
            if (hipError_t e = before_free()) return e;
            hipError_t e = hipFree(p);
            p = nullptr;
            n = 0;
            if (e != hipSuccess) return e;
        }
        // + 64 B: a 16-byte vector load of a row's last element may run up to 12 B past it
        // (the prefetching count pass's LDS-DMA of SoA / bucket rows, kernels.hip)
        hipError_t e = hipMalloc(&p, std::max<size_t>(want, 1) * sizeof(T) + 64);
        if (e == hipSuccess) n = std::max<size_t>(want, 1);
        return e;
    }
    // staging that follows a varying size: geometric growth (an allocation syncs the device)
    hipError_t grow(size_t want) {
        if (want <= n && p) return hipSuccess;
        return reserve(std::max({want, n + n / 2, (size_t)(1 << 20) / sizeof(T)}));
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

// pinned host staging (D2H of the matrix rows, H2D of binding-record slots)
template <typename T>
struct HostBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t reserve(size_t want) {
        if (want <= n && p) return hipSuccess;
        if (p) {
            if (hipError_t e = before_free()) return e;
            hipError_t e = hipHostFree(p);
            p = nullptr;
            n = 0;
            if (e != hipSuccess) return e;
        }
        hipError_t e = hipHostMalloc((void**)&p, std::max<size_t>(want, 1) * sizeof(T), hipHostMallocDefault);
        if (e == hipSuccess) n = std::max<size_t>(want, 1);
        return e;
    }
    hipError_t grow(size_t want) {  // (pinned allocations cost ~0.1-1 ms: geometric growth)
        if (want <= n && p) return hipSuccess;
        return reserve(std::max({want, n + n / 2, (size_t)(1 << 20) / sizeof(T)}));
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
};

// Go: int64(d.Seconds()) (binding.go:85)
int64_t go_seconds_trunc(int64_t d) {
    const int64_t sec = d / 1000000000LL, nsec = d % 1000000000LL;
    const double s = (double)sec + (double)nsec / 1e9;
    if (!(s >= -9223372036854775808.0 && s < 9223372036854775808.0)) return INT64_MIN;
    return (int64_t)s;
}

int64_t floor_div(int64_t a, int64_t b) {
    int64_t q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
    return q;
}

// Engine options: fixed defaults; crane_dyn_set_option changes them per engine
// (tests and A/B tools only — nothing reads the environment).
struct Options {
    int k2_form = 0;          // 0: dedupe, the large form past its count/offset cap, the atomics form past that;
                              // 2: the atomics form (LDS hash + global atomics); 3: the large form (region
                              // pass with coarse bins + dense per-bin histograms)
    int keys_path = 0;        // 0: step path when it applies, 1: the per-pair kernel (K3m keys)
    int greedy_form = 0;      // 0: merge form when every hotValue count > 0, 1: sequential kernel
    int sel_chain = 0;        // selection windows: 0 LDS rank/select walk when it fits, 1 streaming kernel
    int step_rows = 1;        // 1: producers write per-tile record ranges for K3s (when they fit), 0: K3s searches
    int step_lds_cap = 1 << 30;  // K1: one-step records per kind staged in LDS at most (0: always st.stage)
    int step_pieces = 0;      // middle pieces cut into elementary ones per block (step_pieces): 0 when the
                              // producer blocks take more than 4 rounds of the CUs (there the producers'
                              // extra latency overlaps other blocks'; in one round it is the kernel's
                              // critical path: config 4 on one GPU K3s 0.118 -> 0.065 ms, K1 0.070 ->
                              // 0.089; a config-4 shard, one round, got slower) and the batch has
                              // >= kPieceMinTiles pod tiles (a piece is re-read once per tile), 1 always,
                              // 2 never (then no per-tile piece ranges either: K3s reads all pieces)
    bool trace = false;       // phase stamps of K2x / K1 / K3s (crane_dyn_debug_trace)
    int k1_stream = 1;        // keys-only step without dedupe-form K2 entries: the streamed step pass
                              // (k1_stream_steps, no record in registers) | 0 the fused record pass
    int k1_tail = 0;          // the streamed pass's tail: 0 on one wave when the grid has >= 4096 blocks
                              // (the other waves leave), 1 always on one wave, 4 on all four
    int k2_sorted = 1;        // a time-ordered log: K2 reads the widest window's suffix, ranks by position
    int k2_delta = 1;         // ... and, once anchored, only the bindings whose window rank changed since
                              // the anchor refresh (delta form, HotDelta); 0: every refresh re-counts
    int step_defer = 0;       // 1: a step on a dispatch queue leaves its K3s to the engine's next step,
                              // which runs it in its first launch (crane_dyn_step_flush; the group sets it)
};
// Fixed launch shapes (round 6 removed their options; the A/B sweeps that chose them are in
// profiles/ab/r03_k2_cold_*.txt and profiles/r05/config3_option_sweep_queues.txt)
constexpr int kK1Block = 256;     // K1 workgroup size (the dedupe K2 bins nodes by it)
constexpr int kK2xThreads = 512;  // dedupe K2 workgroup size
constexpr int kK2lThreads = 1024; // large K2 partition workgroup size (4096-binding regions)
constexpr int64_t kTraceWgs = 65536;  // workgroups traced per kernel

}  // namespace

struct crane_dyn;

// A node shard's inputs: the parsed annotation SoA, the binding log (or the binding heap and its
// slot log) and what describes them.  One per engine, or shared by the engines of a group's batch
// slots on one device (crane::engine_share_shard): those slots then hold one copy of the shard's
// nodes and log, and only their own derived state and scratch.  A change through any sharing
// engine bumps a version; each engine adopts the new description (and drops what it derived from
// the old) at its next call.  The engines sharing a shard are driven by one caller at a time, which
// waits for their work in flight before it changes the shard (the group: wait_all).
struct ShardData {
    int device = 0;
    uint64_t node_ver = 1, log_ver = 1;
    int64_t N = -1, node_offset = 0, B = 0;
    bool have_hv = false, log_sorted = false, heap_mode = false;
    DevBuf<double> val, hv;
    DevBuf<int64_t> ts, hv_ts;
    DevBuf<int32_t> bnode;
    DevBuf<int64_t> bts;
    HostBuf<int32_t> hnode;  // pinned mirror of the slots in heap mode
    HostBuf<int64_t> hts;
    BindingHeap heap;        // BindingRecords restatement (crane_dyn_binding_records mode)
    std::vector<int64_t> hts_copy;    // a time-ordered log's timestamps (the windows' suffixes are found here)
    std::vector<int64_t> hts_sample;  // every 64th of them: the suffix search touches one 512-byte run
    explicit ShardData(int dev) : device(dev) {}
    ~ShardData() {
        (void)hipSetDevice(device);
        val.release(); hv.release(); ts.release(); hv_ts.release(); bnode.release(); bts.release();
        hnode.release(); hts.release();
    }
};

struct EngineTimer final : KernelTimer {
    crane_dyn* h = nullptr;
    void next(const char* name, hipEvent_t* start, hipEvent_t* stop) override;
};

struct crane_dyn {
    std::mutex mu;
    std::string err;
    int device = 0;
    int n_cu = 0;  // compute units of the device
    hipStream_t stream = nullptr;
    Options opt;
    // policy
    DevPolicy dp{};
    int shape = kShape16x16;
    size_t rec_bytes = 0;
    std::vector<std::string> slot_names;
    int8_t pred_orig[kMaxPred] = {};
    std::vector<int64_t> hot_tr;  // hotValue.timeRange in policy order
    int n_pred_policy = 0;
    // shard state
    int64_t N = -1, node_offset = 0;
    bool have_hv = false;
    bool hv_from_counts = false;
    int64_t hv_ts_counts = 0;
    bool rec_dirty = true;
    bool buckets_zero = false;    // K1 consumes (zeroes) the buckets K2 filled
    bool buckets_dense = false;   // ... unless the large form wrote them whole (K1 leaves them)
    bool counts_pending = false;  // buckets hold K2 counts no node pass has consumed yet
    bool hx_pending = false;      // ... in the dedupe form: per-block entries in k2_sorted (hx_g)
    HotPart hx_g{};
    // delta form (hot_delta_locked): dense anchor counts at suffix starts dl_pos (valid for log
    // version dl_log_ver, N dl_N), the adjustments of the next node pass (zero unless dl_adj_dirty)
    bool dl_valid = false, dl_pending = false, dl_adj_dirty = true;
    bool dl_zero = false;  // this refresh has no binding in any window (K1: adjustments as the anchor)
    uint64_t dl_log_ver = 0;
    int64_t dl_N = -1, dl_B = -1;
    int64_t dl_pos[kMaxWin] = {};
    DevBuf<uint32_t> dl_base, dl_adj;
    // binding log on the device: B slots (node < 0 = empty slot)
    int64_t B = 0;
    bool heap_mode = false;
    bool log_sorted = false;            // uploaded log in non-decreasing time order (upload_bindings)
    bool pos_valid = false;             // pos_s[r]: the suffix start of window rank r for cutoffs pos_cut
    int64_t pos_cut[kMaxWin] = {};
    int64_t pos_s[kMaxWin] = {};
    // the shard's inputs (ShardData), shared by the engines of a group's batch slots on one device
    std::shared_ptr<ShardData> sd;
    uint64_t sd_node_ver = 0, sd_log_ver = 0;  // the versions this engine's derived state follows
    DevBuf<unsigned char> rec;
    DevBuf<uint32_t> buckets;
    // scratch for the host-pointer API
    DevBuf<int64_t> now;
    DevBuf<uint8_t> flags;
    DevBuf<long long> keys;
    DevBuf<int8_t> ff;
    DevBuf<int64_t> score;
    DevBuf<int8_t> score8;
    HostBuf<int8_t> stage8;
    HostBuf<long long> stagek;
    DevBuf<uint32_t> k2_sorted;  // K2 scratch
    DevBuf<double> hvc;                           // [N] binding-log hot values of the last consuming K1
    DevBuf<uint32_t> gcnt;  // greedy: per-window counts [W][N]
    DevBuf<int64_t> gbase, gchosen;
    DevBuf<uint8_t> gleaf, gflags;
    DevBuf<unsigned long long> mH, mbs;  // merge-form greedy (merge.hip)
    DevBuf<int32_t> mflag, mapos, mtk;
    DevBuf<int64_t> mFs, mIs, mgi;
    DevBuf<unsigned long long> trace;  // [3][kTraceWgs][8] phase stamps (option "trace")
    DevBuf<int32_t> sperm, scnt;  // K3 step path scratch (step.hip)
    DevBuf<int64_t> stile, spnow, sbatch;
    DevBuf<int32_t> sperm2;       // ... the second set of K3p's outputs: steps alternate (sbatch_par)
    DevBuf<int64_t> stile2, spnow2;
    int sbatch_par = 0;  // the range of sbatch and the K3p output set the next step uses (StepPlan)
    // option step_defer: the last step's K3s, not launched yet (its queue, tables, pod set, keys)
    struct PendK3s {
        bool on = false;
        crane_queue* q = nullptr;
        StepTables stt{};
        StepGeometry g{};
        const int32_t* perm = nullptr;
        const int64_t* pnow = nullptr;
        const int64_t* tiles = nullptr;
        int64_t P = 0;
        long long* keys = nullptr;
    } pend;
    DevBuf<int64_t> sel_fth, sel_win, sel_state;  // framework selection (select.hip)
    DevBuf<long long> sel_keys;
    DevBuf<unsigned char> stp_dev;  // node answer tables (crane_dyn_node_steps): bp, ns, ff, score
    HostBuf<unsigned char> stp_host;
    DevBuf<Mid> smid;
    DevBuf<Step1> sstep1;
    DevBuf<Step1> sstage;  // K1's one-step staging past its LDS (StepTables::stage)
    DevBuf<int32_t> spm1, ssm0;   // prefix / suffix key maxima of the sorted Step1 records
    DevBuf<int4> srows;           // per (pod tile, producer block): uniform keys + record ranges
    DevBuf<int2> sprow;           // ... and middle-piece ranges
    // caller streams that asynchronous work was enqueued on since the last quiesce: calls that
    // replace engine state (and the synchronous calls on the engine stream) first wait for
    // them — those streams only, not the device (another engine's batches and collectives
    // keep running).  A handle is kept only until that wait.
    std::vector<hipStream_t> busy;
    std::vector<crane_queue*> busy_q;  // the same for dispatch queues (crane_dyn_step_keys_queue)
    std::vector<crane_queue*> seen_q;  // every queue this engine is registered with (aql_add_user)
    DevBuf<unsigned char> upd_dev;   // crane_dyn_update_nodes / _node_steps_subset staging
    HostBuf<unsigned char> upd_host;
    // kernel timing (crane_dyn_set_profiling)
    bool prof = false;
    EngineTimer timer;
    std::vector<hipEvent_t> ev;           // pool, two per timed launch
    std::vector<const char*> ev_name;     // ev_name[i]: kernel of events 2i, 2i + 1
    int nk = 0;
    hipError_t timer_err = hipSuccess;

    unsigned long long* trace_region(int which) {
        return opt.trace && trace.p ? trace.p + (size_t)which * kTraceWgs * 8 : nullptr;
    }
    int fail(int code, const std::string& m) {
        err = m;
        return code;
    }
    int hipfail(hipError_t e, const char* what) {
        err = std::string(what) + ": " + hipGetErrorString(e);
        return CRANE_E_HIP;
    }
};

void EngineTimer::next(const char* name, hipEvent_t* start, hipEvent_t* stop) {
    if ((int)h->ev.size() < 2 * (h->nk + 1)) {
        for (int i = 0; i < 2; ++i) {
            hipEvent_t e;
            hipError_t r = hipEventCreate(&e);
            if (r != hipSuccess) {
                h->timer_err = r;
                return;
            }
            h->ev.push_back(e);
        }
        h->ev_name.push_back(nullptr);
    }
    h->ev_name[h->nk] = name;
    *start = h->ev[2 * h->nk];
    *stop = h->ev[2 * h->nk + 1];
    ++h->nk;
}

namespace {

// After this engine changed the shard's nodes (upload, update, resize) or its bindings (upload,
// heap): the new description for the engines sharing it; this engine's own derived state was
// updated by the change itself
void publish_nodes(crane_dyn* h) {
    ShardData& d = *h->sd;
    d.N = h->N;
    d.node_offset = h->node_offset;
    d.have_hv = h->have_hv;
    h->sd_node_ver = ++d.node_ver;
}
void publish_log(crane_dyn* h) {
    ShardData& d = *h->sd;
    d.B = h->B;
    d.log_sorted = h->log_sorted;
    d.heap_mode = h->heap_mode;
    h->sd_log_ver = ++d.log_ver;
}

// Another engine changed the shared shard: take its description and drop what was derived from
// the old one, as this engine's own upload_nodes / upload_bindings would
int adopt(crane_dyn* h) {
    ShardData& d = *h->sd;
    if (h->sd_node_ver != d.node_ver) {
        if (d.N >= 0) {
            hipError_t e = hipSetDevice(h->device);
            if (e == hipSuccess) e = h->rec.reserve((size_t)d.N * h->rec_bytes);
            if (e != hipSuccess) return h->hipfail(e, "shared shard: record buffer");
        }
        if (d.N != h->N) h->buckets_zero = false;
        h->N = d.N;
        h->node_offset = d.node_offset;
        h->have_hv = d.have_hv;
        h->hv_from_counts = false;
        h->counts_pending = false;
        h->hx_pending = false;
        h->dl_pending = false;
        h->rec_dirty = true;
        h->sd_node_ver = d.node_ver;
    }
    if (h->sd_log_ver != d.log_ver) {
        h->B = d.B;
        h->log_sorted = d.log_sorted;
        h->heap_mode = d.heap_mode;
        h->pos_valid = false;
        h->sd_log_ver = d.log_ver;
    }
    return CRANE_OK;
}

// Every ABI entry that enqueues work holds the engine mutex, takes a shared shard's changes
// (adopt; rc holds its error) and installs the engine's kernel timer on the calling thread while
// profiling is on.
int flush_pending(crane_dyn* h);

struct Locked {
    std::lock_guard<std::mutex> g;
    KernelTimer* prev;
    int rc = 0;
    // keep_pending: the caller is a step on a dispatch queue, which takes a deferred K3s into its
    // own first launch (option step_defer); every other call runs it first
    explicit Locked(crane_dyn* h, bool keep_pending = false) : g(h->mu), prev(tl_ktimer) {
        tl_ktimer = h->prof ? &h->timer : nullptr;
        if (!keep_pending && h->pend.on) rc = flush_pending(h);
        if (!rc && h->sd && (h->sd_node_ver != h->sd->node_ver || h->sd_log_ver != h->sd->log_ver)) rc = adopt(h);
    }
    ~Locked() { tl_ktimer = prev; }
};

}  // namespace

#define HIPTRY(h, expr)                                        \
    do {                                                       \
        hipError_t _e = (expr);                                \
        if (_e != hipSuccess) return (h)->hipfail(_e, #expr);  \
    } while (0)

static int flatten_policy(crane_dyn* h, const crane_policy* pol) {
    if (!pol) return h->fail(CRANE_E_INVALID, "policy is NULL");
    if (pol->n_sync < 0 || pol->n_pred < 0 || pol->n_prio < 0 || pol->n_hot < 0)
        return h->fail(CRANE_E_INVALID, "negative policy list length");
    DevPolicy& dp = h->dp;
    std::memset(&dp, 0, sizeof dp);
    auto active = [&](const char* name, int64_t* dur) -> bool {  // getActiveDuration
        for (int32_t i = 0; i < pol->n_sync; ++i)
            if (std::strcmp(pol->sync_name[i], name) == 0 && pol->sync_period_ns[i] != 0) {
                *dur = pol->sync_period_ns[i] + kExtraActiveNs;
                return true;
            }
        return false;
    };
    auto slot_of = [&](const char* name) -> int {
        for (size_t i = 0; i < h->slot_names.size(); ++i)
            if (h->slot_names[i] == name) return (int)i;
        h->slot_names.emplace_back(name);
        return (int)h->slot_names.size() - 1;
    };
    h->slot_names.clear();
    h->n_pred_policy = pol->n_pred;
    for (int32_t k = 0; k < pol->n_pred; ++k) {
        int64_t dur;
        // Filter skips predicates with no/zero active duration (plugins.go:56-61)
        if (!active(pol->pred_name[k], &dur) || dur == 0) continue;
        if (dp.npd >= kMaxPred) return h->fail(CRANE_E_INVALID, "more than 16 active predicates");
        if (k > 127) return h->fail(CRANE_E_INVALID, "predicate index > 127");
        dp.pred_slot[dp.npd] = slot_of(pol->pred_name[k]);
        dp.pred_limit[dp.npd] = pol->pred_limit[k];
        dp.pred_dur[dp.npd] = dur;
        h->pred_orig[dp.npd] = (int8_t)k;
        dp.npd++;
    }
    double wsum = 0.0;
    for (int32_t k = 0; k < pol->n_prio; ++k) {
        wsum += pol->prio_weight[k];  // accumulates even for failed terms (stats.go:131)
        int64_t dur;
        if (!active(pol->prio_name[k], &dur) || dur == 0) continue;  // term is 0 (stats.go:79-82)
        if (dp.npr >= kMaxPrio) return h->fail(CRANE_E_INVALID, "more than 16 active priorities");
        dp.prio_slot[dp.npr] = slot_of(pol->prio_name[k]);
        dp.prio_w[dp.npr] = pol->prio_weight[k];
        dp.prio_dur[dp.npr] = dur;
        dp.npr++;
    }
    if ((int)h->slot_names.size() > kMaxSlots) return h->fail(CRANE_E_INVALID, "more than 32 metric keys");
    dp.n_slots = (int32_t)h->slot_names.size();
    dp.wsum = wsum;
    {
        int e = 0;
        const double m = std::frexp(wsum, &e);  // wsum = m * 2^e
        dp.winv = (m == 0.5 || m == -0.5) && std::isnormal(wsum) && e - 1 <= 1022 ? std::ldexp(2.0 * m, 1 - e) : 0.0;
        if (dp.winv != 0.0 && dp.winv * wsum != 1.0) dp.winv = 0.0;
    }
    dp.noprio = pol->n_prio == 0;
    if (pol->n_hot > kMaxWin) return h->fail(CRANE_E_INVALID, "more than 8 hotValue windows");
    dp.n_win = pol->n_hot;
    for (int32_t w = 0; w < pol->n_hot; ++w) {
        // Go integer division by zero panics in annotateNodeHotValue (node.go:117)
        if (pol->hot_count[w] == 0) return h->fail(CRANE_E_INVALID, "hotValue count must not be 0");
        dp.win_count[w] = pol->hot_count[w];
    }
    h->hot_tr.assign(pol->hot_tr_ns, pol->hot_tr_ns + pol->n_hot);
    if (dp.npd <= 4 && dp.npr <= 6) h->shape = kShape4x6;
    else if (dp.npd <= 8 && dp.npr <= 8) h->shape = kShape8x8;
    else h->shape = kShape16x16;
    h->rec_bytes = node_rec_bytes(h->shape);
    return CRANE_OK;
}

// ------------------------------------------------------------- pipeline pieces

// Zeroes a buffer the next kernels on `st` read: on a dispatch queue (no fill kernel there) after
// the queue's packets, on the engine stream, waited for
static int zero_for(crane_dyn* h, uint32_t* p, size_t n, hipStream_t st) {
    if (tl_aql) {
        HIPTRY(h, aql_wait(tl_aql));
        HIPTRY(h, hipMemsetAsync(p, 0, n * sizeof(uint32_t), h->stream));
        HIPTRY(h, hipStreamSynchronize(h->stream));
    } else {
        HIPTRY(h, hipMemsetAsync(p, 0, n * sizeof(uint32_t), st));
    }
    return CRANE_OK;
}

// Delta form of a time-ordered log's refresh (kernels.hpp HotDelta), after the suffix search
// (h->pos_s): counts = the anchor's dense counts + the changed bindings' adjustments.  The first
// refresh after the log or the node count changed, or one whose changed bindings pass half the
// widest window's suffix, re-anchors here: the large form writes its dense counts as the new
// anchor (adjustments zero).  *done false: the form does not apply (the caller's forms run).
static int hot_delta_locked(crane_dyn* h, int64_t Bk, const HotCutoffs& pcut, hipStream_t st, const PodPrep* pods,
                            bool* pods_done, bool* done) {
    const DevPolicy& dp = h->dp;
    const int nw = dp.n_win;
    *done = false;
    if (h->N <= 0 || h->N >= (1LL << 27) || nw < 1 || nw > kDeltaMaxWin) return CRANE_OK;
    const size_t nb = (size_t)nw * (size_t)h->N;
    const bool anchored = h->dl_valid && h->dl_log_ver == h->sd_log_ver && h->dl_N == h->N && h->dl_B == h->B;
    // the changed positions: per window rank r, between the anchor's and this refresh's suffix
    // starts; merged
    HotDelta d{};
    d.n_win = nw;
    int64_t L = 0;
    if (anchored) {
        std::pair<int64_t, int64_t> rg[kMaxWin];
        int n = 0;
        for (int r = 0; r < nw; ++r) {
            d.a[r] = h->dl_pos[r];
            d.p[r] = h->pos_s[r];
            const int64_t lo = std::min(d.a[r], d.p[r]), hi = std::max(d.a[r], d.p[r]);
            if (hi > lo) rg[n++] = {lo, hi};
        }
        std::sort(rg, rg + n);
        int m = 0;
        for (int i = 0; i < n; ++i) {
            if (m > 0 && rg[i].first <= rg[m - 1].second) rg[m - 1].second = std::max(rg[m - 1].second, rg[i].second);
            else rg[m++] = rg[i];
        }
        d.n_rng = m;
        d.start[0] = 0;
        for (int k = 0; k < m; ++k) {
            d.lo[k] = rg[k].first;
            d.start[k + 1] = d.start[k] + (rg[k].second - rg[k].first);
        }
        L = d.start[m];
    }
    if (h->dl_adj.n < nb) {
        HIPTRY(h, h->dl_adj.reserve(nb));
        h->dl_adj_dirty = true;
    }
    if (h->dl_adj_dirty) {  // (an earlier refresh's adjustments no node pass consumed, or a new buffer)
        if (int rc = zero_for(h, h->dl_adj.p, h->dl_adj.n, st)) return rc;
        h->dl_adj_dirty = false;
    }
    h->dl_zero = false;
    if (Bk == 0) {
        // no binding inside any window: every count is zero — K1 reads the (clean) adjustments as
        // the anchor too; the anchor itself is kept for the next refresh
        h->dl_zero = true;
    } else if (!anchored || 2 * L > Bk) {
        const HotPart gl = hot_large_geometry(Bk, h->N, nw);
        const HotPart gf = hot_large_geometry(h->B, h->N, nw);
        if (!gl.ok) return CRANE_OK;
        HIPTRY(h, h->dl_base.reserve(nb));
        h->dl_valid = false;
        HIPTRY(h, h->k2_sorted.reserve(std::max(hot_dedupe_scratch(gl), gf.ok ? hot_dedupe_scratch(gf) : 0)));
        HIPTRY(h, launch_hot_count_large(h->sd->bnode.p + h->pos_s[0], h->sd->bts.p, Bk, h->N, pcut, gl,
                                         h->k2_sorted.p, h->dl_base.p, h->n_cu, st, kK2lThreads));
        std::memcpy(h->dl_pos, h->pos_s, sizeof(int64_t) * nw);
        h->dl_valid = true;
        h->dl_log_ver = h->sd_log_ver;
        h->dl_N = h->N;
        h->dl_B = h->B;
    } else {
        crane_dyn::PendK3s& pk = h->pend;
        if (pk.on && tl_aql && pk.q == tl_aql && pods && pods->P > 0) {
            // the previous step's K3s in this launch (option step_defer: step.hip k3s_delta_pods)
            HIPTRY(h, launch_k3s_delta_pods(h->N, h->node_offset, pk.P, pk.keys, pk.stt, pk.g, pk.perm, pk.pnow,
                                            pk.tiles, h->sd->bnode.p, h->N, d, h->dl_adj.p, *pods, st));
            pk.on = false;
        } else {
            d.trace = h->trace_region(0);  // (the delta launch stays far below kTraceWgs workgroups at
                                           // config 3; larger ones are not traced)
            if ((pods ? pods->ntiles : 0) + (L + 1023) / 1024 > kTraceWgs) d.trace = nullptr;
            HIPTRY(h, launch_hot_count_delta(h->sd->bnode.p, h->N, d, h->dl_adj.p, st, pods));
        }
        if (pods_done) *pods_done = pods != nullptr && pods->P > 0;
    }
    h->dl_adj_dirty = true;  // (until the node pass reads and zeroes the adjustments)
    h->dl_pending = true;
    *done = true;
    return CRANE_OK;
}

// pods (optional): the step path's pod preparation, launched together with K2x
// when the dedupe K2 runs (*pods_done reports whether it did).
static int hot_values_locked(crane_dyn* h, int64_t now_ns, int64_t hv_ts_ns, hipStream_t st,
                             const PodPrep* pods = nullptr, bool* pods_done = nullptr) {
    if (pods_done) *pods_done = false;
    if (h->N < 0) return h->fail(CRANE_E_STATE, "upload nodes before refreshing hot values");
    DevPolicy& dp = h->dp;
    HotCutoffs cut{};
    cut.n_win = dp.n_win;
    // time.Now().UTC().Unix() - int64(timeRange.Seconds())   (binding.go:85)
    const int64_t now_unix = floor_div(now_ns, 1000000000LL);
    int64_t c[kMaxWin];
    int order[kMaxWin];
    for (int w = 0; w < dp.n_win; ++w) {
        const int64_t trs = go_seconds_trunc(h->hot_tr[w]);
        c[w] = now_unix - trs;
        order[w] = w;
    }
    std::stable_sort(order, order + dp.n_win, [&](int a, int b) { return c[a] < c[b]; });
    for (int r = 0; r < dp.n_win; ++r) {
        cut.sorted[r] = c[order[r]];
        dp.win_pos[order[r]] = r;
        dp.win_cut_sorted[r] = c[order[r]];
        dp.win_of_rank[r] = order[r];
        const int64_t cw = dp.win_count[order[r]];
        dp.win_div_m[r] = 0;
        dp.win_div_sh[r] = 0;
        if (cw >= 1 && cw <= 0xFFFFFFFFLL) make_div_magic((uint32_t)cw, &dp.win_div_m[r], &dp.win_div_sh[r]);
    }
    h->hx_pending = false;
    h->dl_pending = false;
    h->counts_pending = true;
    h->hv_from_counts = true;
    h->hv_ts_counts = hv_ts_ns;
    h->rec_dirty = true;
    // A time-ordered log (a ring of bindings appended as they happen, checked at upload): the
    // bindings inside window w are the suffix from s_w = the first with ts > cutoff_w
    // (binding.go:85-91), found on the host copy of the timestamps.  The dedupe / large forms
    // then read only the node ids of the widest window's suffix and rank a binding by its
    // position — the same counts as the timestamp test, without the 8-byte stamps and without
    // the bindings older than every window.
    const int32_t* bn = h->sd->bnode.p;
    int64_t Bk = h->B;
    HotCutoffs pcut = cut;
    const bool by_pos = h->log_sorted && h->opt.k2_sorted && dp.n_win > 0 && (int64_t)h->sd->hts_copy.size() == h->B;
    if (by_pos) {
        // (the cutoffs move once per second: the last search's suffixes are reused until they do)
        if (!h->pos_valid || std::memcmp(h->pos_cut, cut.sorted, sizeof(int64_t) * dp.n_win) != 0) {
            // (a batch whose time advanced moves them: the sampled stamps narrow each search to one
            // 64-stamp run, ~7 + 6 probes, instead of 20 probes across the 8 MB stamp array)
            const std::vector<int64_t>& smp = h->sd->hts_sample;
            const int64_t* t0 = h->sd->hts_copy.data();
            for (int r = 0; r < dp.n_win; ++r) {
                const int64_t j = std::upper_bound(smp.begin(), smp.end(), cut.sorted[r]) - smp.begin();
                const int64_t lo = j == 0 ? 0 : 64 * (j - 1), hi = std::min<int64_t>(h->B, 64 * j);
                h->pos_s[r] = std::upper_bound(t0 + lo, t0 + hi, cut.sorted[r]) - t0;
            }
            std::memcpy(h->pos_cut, cut.sorted, sizeof(int64_t) * dp.n_win);
            h->pos_valid = true;
        }
        const int64_t s0 = h->pos_s[0];
        for (int r = 0; r < dp.n_win; ++r) pcut.sorted[r] = h->pos_s[r] - s0 - 1;
        pcut.by_pos = 1;
        bn = h->sd->bnode.p + s0;
        Bk = h->B - s0;
    }
    if (by_pos && h->opt.k2_delta && h->opt.k2_form == 0) {
        bool done = false;
        const int rc = hot_delta_locked(h, Bk, pcut, st, pods, pods_done, &done);
        if (rc || done) return rc;
    }
    HotPart gx = hot_dedupe_geometry(Bk, h->N, dp.n_win, kK1Block);
    gx.trace = gx.nblk <= kTraceWgs ? h->trace_region(0) : nullptr;
    if (h->opt.k2_form == 0 && gx.ok) {
        // one launch (+ K3p); the node pass counts its own block's entries (no buckets).  The
        // scratch is sized for the whole log, not this refresh's suffix: the suffix moves with
        // `now`, and a reallocation (hipFree waits for the device) inside a pipeline of batches
        // cost 30-55 us per batch when the batch times advanced
        const HotPart gf = hot_dedupe_geometry(h->B, h->N, dp.n_win, kK1Block);
        HIPTRY(h, h->k2_sorted.reserve(std::max(hot_dedupe_scratch(gx), gf.ok ? hot_dedupe_scratch(gf) : 0)));
        HIPTRY(h, launch_hot_count_dedupe(bn, h->sd->bts.p, Bk, h->N, by_pos ? pcut : cut, gx, h->k2_sorted.p, st, pods,
                                          kK2xThreads));
        if (pods_done) *pods_done = pods != nullptr && pods->P > 0;
        h->hx_g = gx;
        h->hx_pending = true;
        return CRANE_OK;
    }
    const size_t nb = (size_t)std::max(1, dp.n_win) * (size_t)std::max<int64_t>(h->N, 1);
    if (nb > h->buckets.n) h->buckets_zero = false;
    HIPTRY(h, h->buckets.reserve(nb));
    HotPart gl = hot_large_geometry(Bk, h->N, dp.n_win);
    gl.trace = gl.nblk <= kTraceWgs ? h->trace_region(0) : nullptr;  // (stamps per region)
    if ((h->opt.k2_form == 0 || h->opt.k2_form == 3) && gl.ok) {
        // the region pass with coarse bins + the dense per-bin histogram: every bucket row
        // is rewritten, so nothing is zeroed before and K1 leaves them
        const HotPart gf = hot_large_geometry(h->B, h->N, dp.n_win);
        HIPTRY(h, h->k2_sorted.reserve(std::max(hot_dedupe_scratch(gl), gf.ok ? hot_dedupe_scratch(gf) : 0)));
        HIPTRY(h, launch_hot_count_large(bn, h->sd->bts.p, Bk, h->N, by_pos ? pcut : cut, gl, h->k2_sorted.p,
                                         h->buckets.p, h->n_cu, st, kK2lThreads));
        h->buckets_zero = false;
        h->buckets_dense = true;
        return CRANE_OK;
    }
    h->buckets_dense = false;
    if (!h->buckets_zero && tl_aql) {
        // (on a dispatch queue: a fill is no kernel here — after the queue's packets, on the engine
        // stream, waited for)
        HIPTRY(h, aql_wait(tl_aql));
        HIPTRY(h, hipMemsetAsync(h->buckets.p, 0, nb * sizeof(uint32_t), h->stream));
        HIPTRY(h, hipStreamSynchronize(h->stream));
    } else if (!h->buckets_zero) {
        HIPTRY(h, hipMemsetAsync(h->buckets.p, 0, nb * sizeof(uint32_t), st));
    }
    // the atomics form (any size; shards past the large form's caps)
    HIPTRY(h, launch_hot_count(h->sd->bnode.p, h->sd->bts.p, h->B, h->N, cut, h->buckets.p, st));
    h->buckets_zero = false;
    return CRANE_OK;
}

// K1's workgroup size: the dedupe-form K2 bins nodes by it
static int k1_bs(const crane_dyn* h) {
    return h->hv_from_counts && h->counts_pending && h->hx_pending ? 1 << h->hx_g.bb : kK1Block;
}

// K1 (optionally with the K3 step tables fused in).  Hot values: pending K2
// counts (consumed), else the values the last consuming pass kept, else the
// uploaded annotation.
static int node_pass_locked(crane_dyn* h, hipStream_t st, uint32_t* cnt_out = nullptr, const K1Step* step = nullptr) {
    if (h->N < 0) return h->fail(CRANE_E_STATE, "upload nodes before the node pass");
    K1Args a{};
    a.pol = h->dp;
    a.N = h->N;
    a.val = h->sd->val.p;
    a.ts = h->sd->ts.p;
    // the fused keys-only step reads its records from LDS; writing them out
    // (160 B/node of the pass's 280) is left to the next pass that reads them
    const bool keep = !step;
    a.out = keep ? h->rec.p : nullptr;
    a.hv_ts_counts = h->hv_ts_counts;
    const bool consume = h->hv_from_counts && h->counts_pending;
    if (cnt_out && !consume) return h->fail(CRANE_E_STATE, "per-window counts need a hot-value refresh first");
    if (consume) {
        HIPTRY(h, h->hvc.reserve((size_t)std::max<int64_t>(h->N, 1)));
        if (h->hx_pending) {
            const HotPart& g = h->hx_g;
            a.hx_region = h->k2_sorted.p;
            a.hx_CO = h->k2_sorted.p + g.cap;
            a.hx_nblk = g.nblk;
        } else if (h->dl_pending) {
            a.buckets = h->dl_adj.p;  // read and zeroed
            a.bucket_base = h->dl_zero ? h->dl_adj.p : h->dl_base.p;
            a.buckets_keep = 0;
        } else {
            a.buckets = h->buckets.p;
            a.buckets_keep = h->buckets_dense ? 1 : 0;
        }
        a.cnt_out = cnt_out;
        a.hvc_out = h->hvc.p;
    } else if (h->hv_from_counts) {
        a.hv = h->hvc.p;  // hv_ts null: stamped hv_ts_counts
    } else if (h->have_hv) {
        a.hv = h->sd->hv.p;
        a.hv_ts = h->sd->hv_ts.p;
    }
    a.threads = k1_bs(h);
    a.trace = (h->N + a.threads - 1) / a.threads <= kTraceWgs ? h->trace_region(1) : nullptr;
    HIPTRY(h, launch_node_pass(h->shape, a, st, step, h->opt.k1_stream));
    if (consume) {
        if (h->dl_pending) h->dl_adj_dirty = false;  // K1 zeroed the adjustments
        else if (!h->hx_pending) h->buckets_zero = !h->buckets_dense;  // K1 zeroed what it read
        h->counts_pending = false;
        h->hx_pending = false;
        h->dl_pending = false;
    }
    h->rec_dirty = !keep;
    return CRANE_OK;
}

// ---- keys-only step path (step.hip): K3p -> [K1 +] K3a -> K3s
struct StepPlan {
    StepGeometry g;
    StepTables stt;
    bool fuse;  // K3a fused into the node pass (records stale)
    int64_t* batch;       // this step's time range (K3p folds it, K1 reads it)
    int64_t* batch_next;  // the other range: reset by K3p for the next step
    int32_t* perm;        // this step's K3p outputs (one of two sets, by sbatch_par)
    int64_t* pnow;
    int64_t* tiles;
};

static bool step_path_ok(const crane_dyn* h, int64_t P) {
    return h->opt.keys_path == 0 && h->N >= 0 && h->N < kStepMaxNodes && P < (1LL << 31);
}

static int step_plan(crane_dyn* h, int64_t P, StepPlan& sp) {
    sp.fuse = h->rec_dirty;
    const int32_t bs = sp.fuse ? k1_bs(h) : kStepSeg;  // producer workgroup size
    const int32_t nblk = (int32_t)((h->N + bs - 1) / bs);
    sp.g = step_geometry(P, h->N, nblk, 0);
    const StepGeometry& g = sp.g;
    HIPTRY(h, h->sperm.reserve((size_t)(g.ntiles * 1024)));
    HIPTRY(h, h->stile.reserve((size_t)(kTileStat * g.ntiles)));
    HIPTRY(h, h->sperm2.reserve((size_t)(g.ntiles * 1024)));
    HIPTRY(h, h->stile2.reserve((size_t)(kTileStat * g.ntiles)));
    HIPTRY(h, h->spnow2.reserve((size_t)(g.ntiles * 1024)));
    if (!h->sbatch.p) {  // two {tmin, tmax} ranges, alternating between steps, start empty
        HIPTRY(h, h->sbatch.reserve(4));
        // on the engine stream and waited for: a null-stream copy is not ordered with the
        // non-blocking streams K3p runs on and may land after it (a batch then saw tmin = tmax
        // = 0: every pod scored as at time 0, seen once in test_greedy_then_eval_consistent)
        static const int64_t empty[4] = {INT64_MAX, INT64_MIN, INT64_MAX, INT64_MIN};
        HIPTRY(h, hipMemcpyAsync(h->sbatch.p, empty, sizeof(empty), hipMemcpyHostToDevice, h->stream));
        HIPTRY(h, hipStreamSynchronize(h->stream));
        h->sbatch_par = 0;
    }
    // (the ranges alternate once K3p was launched: pods_ran)
    sp.batch = h->sbatch.p + 2 * h->sbatch_par;
    sp.batch_next = h->sbatch.p + 2 * (h->sbatch_par ^ 1);
    HIPTRY(h, h->spnow.reserve((size_t)(g.ntiles * 1024)));
    sp.perm = h->sbatch_par ? h->sperm2.p : h->sperm.p;
    sp.pnow = h->sbatch_par ? h->spnow2.p : h->spnow.p;
    sp.tiles = h->sbatch_par ? h->stile2.p : h->stile.p;
    HIPTRY(h, h->scnt.reserve((size_t)std::max<int32_t>(nblk, 1) * 6));  // cnt [nblk][4] + flat [nblk][2]
    // per kind and producer block: 2 * bs one-step records, bs * (breakpoints - 1) middle pieces
    const int64_t s1pad = 2 * g.npad, mstride = (int64_t)bs * (step_breakpoints(h->shape) - 1);
    const int64_t mpad = (int64_t)nblk * mstride;
    HIPTRY(h, h->sstep1.reserve((size_t)(2 * s1pad)));
    if (sp.fuse) HIPTRY(h, h->sstage.reserve((size_t)(2 * s1pad)));
    HIPTRY(h, h->spm1.reserve((size_t)(2 * s1pad)));
    HIPTRY(h, h->ssm0.reserve((size_t)(2 * s1pad)));
    HIPTRY(h, h->smid.reserve((size_t)(2 * mpad)));
    StepTables& t = sp.stt;
    t = StepTables{};
    t.cnt = h->scnt.p;
    t.flat = h->scnt.p + (size_t)nblk * 4;
    t.single = h->sstep1.p;
    t.stage = sp.fuse ? h->sstage.p : nullptr;
    t.lds_cap = h->opt.step_lds_cap;
    const bool pieces = h->opt.step_pieces == 1 ||
                        (h->opt.step_pieces == 0 && nblk > 4 * h->n_cu && g.ntiles >= kPieceMinTiles);
    t.piece_work = pieces ? 256 : INT32_MAX;
    t.pm1 = h->spm1.p;
    t.sm0 = h->ssm0.p;
    t.mid = h->smid.p;
    t.s1pad = s1pad;
    t.mpad = mpad;
    t.bs = bs;
    t.nblk = nblk;
    t.mstride = (int32_t)mstride;
    t.ntiles = (int32_t)g.ntiles;
    t.tiles = sp.tiles;
    const int64_t nrows = g.ntiles * (int64_t)nblk;
    if (h->opt.step_rows && nrows <= kStepRowsMax) {
        HIPTRY(h, h->srows.reserve((size_t)std::max<int64_t>(nrows, 1)));
        t.rows = h->srows.p;
        if (pieces) {
            HIPTRY(h, h->sprow.reserve((size_t)std::max<int64_t>(nrows, 1)));
            t.prow = h->sprow.p;
        }
    }
    t.trace = g.ngroups * g.R <= kTraceWgs ? h->trace_region(2) : nullptr;
    return CRANE_OK;
}

// K3p was launched for a step: the next step folds into the range this one reset
static void pods_ran(crane_dyn* h, int64_t P) {
    if (P > 0) h->sbatch_par ^= 1;
}

static int step_pods(crane_dyn* h, const StepPlan& sp, int64_t P, const int64_t* d_now, const uint8_t* d_flags,
                     long long* d_keys, hipStream_t st) {
    HIPTRY(h, launch_step_pods(d_now, d_flags, P, d_keys, sp.batch, sp.batch_next, sp.g, sp.perm, sp.pnow, sp.tiles,
                               st));
    pods_ran(h, P);
    return CRANE_OK;
}

static int step_rest(crane_dyn* h, const StepPlan& sp, int64_t P, long long* d_keys, hipStream_t st,
                     bool defer = false) {
    if (P == 0) return CRANE_OK;
    if (sp.fuse) {
        // (the records the fused step leaves stale serve as the streamed pass's scratch)
        const K1Step ks{sp.tiles, sp.batch, (int32_t)sp.g.ntiles, h->dp.noprio, h->dp.wsum, h->dp.winv, sp.stt,
                        h->rec.p, h->opt.k1_tail};
        int rc = node_pass_locked(h, st, nullptr, &ks);
        if (rc) return rc;
    } else {
        if (h->rec_dirty) {
            int rc = node_pass_locked(h, st);
            if (rc) return rc;
        }
        HIPTRY(h, launch_step_nodes(h->shape, h->rec.p, h->N, h->dp.wsum, h->dp.noprio, sp.stt, sp.g, sp.tiles, st));
    }
    if (defer) {  // (the next step's first launch runs it: PendK3s)
        crane_dyn::PendK3s& pk = h->pend;
        pk.on = true;
        pk.q = tl_aql;
        pk.stt = sp.stt;
        pk.g = sp.g;
        pk.perm = sp.perm;
        pk.pnow = sp.pnow;
        pk.tiles = sp.tiles;
        pk.P = P;
        pk.keys = d_keys;
        return CRANE_OK;
    }
    HIPTRY(h, launch_step_pairs(h->shape, h->N, h->node_offset, P, d_keys, sp.stt, sp.g, sp.perm, sp.pnow, sp.tiles, st));
    return CRANE_OK;
}

// option step_defer: the last step's K3s launched now on its queue (alone) and committed
namespace {
int flush_pending(crane_dyn* h) {
    crane_dyn::PendK3s& pk = h->pend;
    if (!pk.on) return CRANE_OK;
    pk.on = false;
    crane_queue* const prev = tl_aql;
    tl_aql = pk.q;
    const hipError_t e = launch_step_pairs(h->shape, h->N, h->node_offset, pk.P, pk.keys, pk.stt, pk.g, pk.perm,
                                           pk.pnow, pk.tiles, h->stream);
    const hipError_t c = aql_commit(pk.q);
    tl_aql = prev;
    if (e != hipSuccess) return h->hipfail(e, "deferred k3s_eval");
    if (c != hipSuccess) return h->fail(CRANE_E_HIP, std::string("queue: ") + aql_error(pk.q));
    return CRANE_OK;
}
}  // namespace

// The per-pair kernel (K3m): first-fail / score matrices [P][ld] and/or keys.
static int matrix_locked(crane_dyn* h, int64_t P, const int64_t* d_now, const uint8_t* d_flags, long long* d_keys,
                         int8_t* d_ff, void* d_score, bool score_i64, int64_t ld, hipStream_t st) {
    if (h->rec_dirty) {
        int rc = node_pass_locked(h, st);
        if (rc) return rc;
    }
    MatrixArgs a{};
    a.rec = h->rec.p;
    a.N = h->N;
    a.node_offset = h->node_offset;
    a.now = d_now;
    a.flags = d_flags;
    a.P = P;
    a.ld = ld;
    a.wsum = h->dp.wsum;
    a.noprio = h->dp.noprio;
    a.first_fail = d_ff;
    a.score = d_score;
    a.score_i64 = score_i64 ? 1 : 0;
    a.keys = d_keys;
    std::memcpy(a.pred_orig, h->pred_orig, sizeof a.pred_orig);
    if (d_keys && P > 0) HIPTRY(h, hipMemsetAsync(d_keys, 0xFF, sizeof(long long) * (size_t)P, st));
    HIPTRY(h, launch_matrix(h->shape, a, st));
    return CRANE_OK;
}

static int keys_locked(crane_dyn* h, int64_t P, const int64_t* d_now, const uint8_t* d_flags, long long* d_keys,
                       hipStream_t st) {
    if (h->N < 0) return h->fail(CRANE_E_STATE, "upload nodes before evaluating pods");
    if (step_path_ok(h, P)) {
        StepPlan sp;
        int rc = step_plan(h, P, sp);
        if (!rc) rc = step_pods(h, sp, P, d_now, d_flags, d_keys, st);
        if (!rc) rc = step_rest(h, sp, P, d_keys, st);
        return rc;
    }
    return matrix_locked(h, P, d_now, d_flags, d_keys, nullptr, nullptr, false, 0, st);
}

// Re-upload the dirty binding-record slots of the heap mode (pinned mirror -> device).
static int flush_heap_slots(crane_dyn* h) {
    std::vector<std::pair<int64_t, int64_t>> runs;
    h->sd->heap.take_dirty_runs(&runs);
    for (const auto& r : runs) {
        const size_t n = (size_t)(r.second - r.first);
        HIPTRY(h, hipMemcpyAsync(h->sd->bnode.p + r.first, h->sd->hnode.p + r.first, n * sizeof(int32_t),
                                 hipMemcpyHostToDevice, h->stream));
        HIPTRY(h, hipMemcpyAsync(h->sd->bts.p + r.first, h->sd->hts.p + r.first, n * sizeof(int64_t), hipMemcpyHostToDevice,
                                 h->stream));
    }
    if (!runs.empty()) HIPTRY(h, hipStreamSynchronize(h->stream));  // the mirror may change after we return
    return CRANE_OK;
}

// After enqueueing work that reads engine buffers on a caller stream: remember the stream
// (no per-call HIP call: a completion event recorded per call, round 2, put a marker packet
// between batches that cost 3 us of a config-3 batch's latency and 3 % of the in-flight rate).
static int mark_busy(crane_dyn* h, hipStream_t st) {
    if (st == h->stream) return CRANE_OK;  // engine-stream work is ordered by the stream itself
    for (hipStream_t s : h->busy)
        if (s == st) return CRANE_OK;
    h->busy.push_back(st);
    return CRANE_OK;
}

// Before changing or reallocating buffers that asynchronous calls read (node SoA, binding
// log, scratch), and before synchronous work on the engine stream: wait for the caller
// streams this engine enqueued work on since the last wait — not the device, so other
// engines' batches and collectives in flight are not drained.  State changes are per
// snapshot sync / controller tick, not per batch.
static int quiesce(crane_dyn* h) {
    if (int rc = flush_pending(h)) return rc;
    if (!h->busy_q.empty()) {
        std::vector<crane_queue*> qs;
        qs.swap(h->busy_q);
        for (crane_queue* q : qs)
            if (aql_wait(q) != hipSuccess) return h->fail(CRANE_E_HIP, std::string("queue: ") + aql_error(q));
    }
    if (h->busy.empty()) return CRANE_OK;
    // the list is cleared even when a wait fails (a stream the caller destroyed without
    // crane_dyn_forget_stream): the error is reported once, not by every later state change
    std::vector<hipStream_t> busy;
    busy.swap(h->busy);
    HIPTRY(h, hipSetDevice(h->device));
    for (hipStream_t s : busy) HIPTRY(h, hipStreamSynchronize(s));
    return CRANE_OK;
}

// A group's batch slots on one device share the shard of slot 0 (group.cpp): h drops its own
// (empty) shard inputs and takes from's; its derived state follows at its next call (adopt)
int crane::engine_share_shard(crane_dyn* h, crane_dyn* from) {
    if (!h || !from || h == from) return CRANE_E_INVALID;
    std::scoped_lock l(h->mu, from->mu);
    if (h->device != from->device || h->shape != from->shape || h->dp.n_slots != from->dp.n_slots)
        return h->fail(CRANE_E_INVALID, "a shared shard needs the same device and policy");
    if (int rc = quiesce(h)) return rc;
    h->sd = from->sd;
    h->sd_node_ver = h->sd_log_ver = 0;  // (versions start at 1: adopt at the next call)
    return CRANE_OK;
}

// a queue being destroyed hands itself back (aql.cpp; it has waited for its steps)
void crane::engine_drop_queue(crane_dyn* h, crane_queue* q) {
    std::lock_guard<std::mutex> g(h->mu);
    if (h->pend.q == q) h->pend.on = false;  // (a deferred K3s on a queue going away: not run)
    h->busy_q.erase(std::remove(h->busy_q.begin(), h->busy_q.end(), q), h->busy_q.end());
    h->seen_q.erase(std::remove(h->seen_q.begin(), h->seen_q.end(), q), h->seen_q.end());
}

extern "C" {

const char* crane_dyn_version(void) { return "crane_dyn 0.2 gfx950"; }

int64_t crane_dyn_key_node(int64_t key, int64_t* score) {
    if (key < 0) {
        if (score) *score = -1;
        return -1;
    }
    if (score) *score = key >> 32;
    return (int64_t)(0xFFFFFFFFull - ((uint64_t)key & 0xFFFFFFFFull));
}

int crane_dyn_create(const crane_policy* pol, int32_t device, crane_dyn** out) {
    if (!out) return CRANE_E_INVALID;
    *out = nullptr;
    crane_dyn* h = new crane_dyn();
    h->timer.h = h;
    // the handle is returned even on failure so the caller can read the error; it is
    // flagged unusable (N = -2) and must still be destroyed
    *out = h;
    int rc = flatten_policy(h, pol);
    if (rc) {
        h->N = -2;
        return rc;
    }
    h->device = device;
    h->sd = std::make_shared<ShardData>(device);
    h->sd_node_ver = h->sd->node_ver;
    h->sd_log_ver = h->sd->log_ver;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&h->n_cu, hipDeviceAttributeMultiprocessorCount, device);
    if (e != hipSuccess) {
        h->hipfail(e, "hipSetDevice/hipStreamCreate");
        h->N = -2;
        return CRANE_E_HIP;
    }
    return CRANE_OK;
}

int crane_dyn_destroy(crane_dyn* h) {
    if (!h) return CRANE_OK;
    // the whole device, not the remembered caller streams: a caller may have destroyed one of
    // them already (its handle is then dangling), and nothing may still read the buffers freed here
    if (h->stream) {
        (void)hipSetDevice(h->device);
        (void)hipDeviceSynchronize();
    }
    h->busy.clear();
    // the queues still registered are alive (a destroyed queue unregisters itself,
    // engine_drop_queue): wait for the ones with steps of this engine, then unregister
    {
        std::lock_guard<std::mutex> g(h->mu);
        (void)flush_pending(h);
        for (crane_queue* q : h->busy_q) (void)aql_wait(q);
        for (crane_queue* q : h->seen_q) aql_remove_user(q, h);
        h->busy_q.clear();
        h->seen_q.clear();
    }
    for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
    h->ev.clear();
    h->sd.reset();  // (the shard's inputs go with the last engine holding them)
    h->rec.release();
    h->buckets.release(); h->now.release(); h->flags.release();
    h->keys.release(); h->ff.release(); h->score.release(); h->score8.release();
    h->stage8.release(); h->stagek.release();
    h->k2_sorted.release(); h->hvc.release();
    h->gcnt.release(); h->gbase.release(); h->gchosen.release(); h->gleaf.release(); h->gflags.release();
    h->mH.release(); h->mbs.release(); h->mflag.release(); h->mapos.release(); h->mtk.release();
    h->mFs.release(); h->mIs.release(); h->mgi.release();
    h->trace.release();
    h->sperm2.release(); h->stile2.release(); h->spnow2.release();
    h->sperm.release(); h->scnt.release(); h->stile.release(); h->sbatch.release(); h->spnow.release(); h->smid.release(); h->sstep1.release(); h->sstage.release();
    h->spm1.release(); h->ssm0.release(); h->srows.release(); h->sprow.release();
    h->sel_fth.release(); h->sel_win.release(); h->sel_state.release(); h->sel_keys.release();
    h->stp_dev.release(); h->stp_host.release(); h->upd_dev.release(); h->upd_host.release();
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return CRANE_OK;
}

const char* crane_dyn_last_error(const crane_dyn* h) { return h ? h->err.c_str() : "null engine"; }

int crane_dyn_forget_stream(crane_dyn* h, void* stream) {
    if (!h) return CRANE_E_INVALID;
    std::lock_guard<std::mutex> g(h->mu);
    auto it = std::find(h->busy.begin(), h->busy.end(), (hipStream_t)stream);
    if (it == h->busy.end()) return CRANE_OK;
    h->busy.erase(it);
    HIPTRY(h, hipSetDevice(h->device));
    HIPTRY(h, hipStreamSynchronize((hipStream_t)stream));
    return CRANE_OK;
}

int crane_dyn_step_flush(crane_dyn* h) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);  // (runs a deferred K3s)
    return lk.rc;
}

int crane_dyn_forget_queue(crane_dyn* h, crane_queue* q) {
    if (!h) return CRANE_E_INVALID;
    std::lock_guard<std::mutex> g(h->mu);
    if (h->pend.on && h->pend.q == q)
        if (int rc = flush_pending(h)) return rc;
    auto sq = std::find(h->seen_q.begin(), h->seen_q.end(), q);
    if (sq != h->seen_q.end()) {
        h->seen_q.erase(sq);
        aql_remove_user(q, h);
    }
    auto it = std::find(h->busy_q.begin(), h->busy_q.end(), q);
    if (it == h->busy_q.end()) return CRANE_OK;
    h->busy_q.erase(it);
    if (aql_wait(q) != hipSuccess) return h->fail(CRANE_E_HIP, std::string("queue: ") + aql_error(q));
    return CRANE_OK;
}

int32_t crane_dyn_num_metrics(const crane_dyn* h) { return h ? (int32_t)h->slot_names.size() : 0; }

const char* crane_dyn_metric_name(const crane_dyn* h, int32_t slot) {
    if (!h || slot < 0 || slot >= (int32_t)h->slot_names.size()) return nullptr;
    return h->slot_names[slot].c_str();
}

int crane_dyn_set_option(crane_dyn* h, const char* name, int64_t value) {
    if (!h || !name) return CRANE_E_INVALID;
    std::lock_guard<std::mutex> g(h->mu);
    const std::string n = name;
    Options& o = h->opt;
    auto range = [&](int64_t lo, int64_t hi) { return value >= lo && value <= hi; };
    if (n == "k2_form" && (value == 0 || value == 2 || value == 3)) o.k2_form = (int)value;
    else if (n == "keys_path" && range(0, 1)) o.keys_path = (int)value;
    else if (n == "greedy_form" && range(0, 1)) o.greedy_form = (int)value;
    else if (n == "sel_chain" && range(0, 1)) o.sel_chain = (int)value;
    else if (n == "step_rows" && range(0, 1)) o.step_rows = (int)value;
    else if (n == "step_pieces" && range(0, 2)) o.step_pieces = (int)value;
    else if (n == "step_lds_cap" && value >= 0) o.step_lds_cap = (int)std::min<int64_t>(value, 1 << 30);
    else if (n == "k2_sorted" && range(0, 1)) o.k2_sorted = (int)value;
    else if (n == "k2_delta" && range(0, 1)) o.k2_delta = (int)value;
    else if (n == "step_defer" && range(0, 1)) o.step_defer = (int)value;
    else if (n == "k1_stream" && range(0, 1)) o.k1_stream = (int)value;
    else if (n == "k1_tail" && (value == 0 || value == 1 || value == 4)) o.k1_tail = (int)value;
    else if (n == "trace" && range(0, 1)) {
        o.trace = value != 0;
        if (o.trace) {
            hipError_t e = hipSetDevice(h->device);
            if (e == hipSuccess) e = h->trace.reserve((size_t)3 * kTraceWgs * 8);
            if (e == hipSuccess) e = hipMemsetAsync(h->trace.p, 0, sizeof(unsigned long long) * h->trace.n, h->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
            if (e != hipSuccess) return h->hipfail(e, "trace buffer");
        }
    }
    else return h->fail(CRANE_E_INVALID, "unknown option or value: " + n + "=" + std::to_string(value));
    // a pending dedupe-form count is bound to the K1 block size it was binned by
    h->rec_dirty = true;
    return CRANE_OK;
}

int64_t crane_dyn_debug_trace(crane_dyn* h, int32_t which, int64_t max, uint64_t* out) {
    if (!h || which < 0 || which > 2 || max < 0 || (max > 0 && !out)) return CRANE_E_INVALID;
    std::lock_guard<std::mutex> g(h->mu);
    if (!h->opt.trace || !h->trace.p) return h->fail(CRANE_E_STATE, "option \"trace\" is off");
    const int64_t n = std::min<int64_t>(max, kTraceWgs * 8);
    HIPTRY(h, hipSetDevice(h->device));
    HIPTRY(h, hipStreamSynchronize(h->stream));
    HIPTRY(h, hipDeviceSynchronize());
    HIPTRY(h, hipMemcpy(out, h->trace_region(which), sizeof(uint64_t) * n, hipMemcpyDeviceToHost));
    return n;
}

int crane_dyn_upload_nodes(crane_dyn* h, int64_t n, int64_t node_offset, const double* val, const int64_t* ts,
                           const double* hv, const int64_t* hv_ts) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    if (h->N == -2) return h->fail(CRANE_E_STATE, "engine was not created successfully");
    if (n < 0 || n > 0xFFFFFFFFLL || node_offset < 0 || node_offset + n > 0xFFFFFFFFLL)
        return h->fail(CRANE_E_INVALID, "node count/offset out of range (global indices must fit 32 bits)");
    const int64_t M = h->dp.n_slots;
    if (n > 0 && M > 0 && (!val || !ts)) return h->fail(CRANE_E_INVALID, "val/ts must not be NULL");
    if ((hv == nullptr) != (hv_ts == nullptr)) return h->fail(CRANE_E_INVALID, "hv and hv_ts must both be set or NULL");
    HIPTRY(h, hipSetDevice(h->device));
    if (int rc = quiesce(h)) return rc;
    HIPTRY(h, h->sd->val.reserve((size_t)(M * n)));
    HIPTRY(h, h->sd->ts.reserve((size_t)(M * n)));
    HIPTRY(h, h->sd->hv.reserve((size_t)n));
    HIPTRY(h, h->sd->hv_ts.reserve((size_t)n));
    HIPTRY(h, h->rec.reserve((size_t)n * h->rec_bytes));
    if (M * n > 0) {
        HIPTRY(h, hipMemcpyAsync(h->sd->val.p, val, sizeof(double) * M * n, hipMemcpyHostToDevice, h->stream));
        HIPTRY(h, hipMemcpyAsync(h->sd->ts.p, ts, sizeof(int64_t) * M * n, hipMemcpyHostToDevice, h->stream));
    }
    if (hv && n > 0) {
        HIPTRY(h, hipMemcpyAsync(h->sd->hv.p, hv, sizeof(double) * n, hipMemcpyHostToDevice, h->stream));
        HIPTRY(h, hipMemcpyAsync(h->sd->hv_ts.p, hv_ts, sizeof(int64_t) * n, hipMemcpyHostToDevice, h->stream));
    }
    HIPTRY(h, hipStreamSynchronize(h->stream));
    if (n != h->N) h->buckets_zero = false;
    h->N = n;
    h->node_offset = node_offset;
    h->have_hv = hv != nullptr;
    h->hv_from_counts = false;
    h->counts_pending = false;
    h->hx_pending = false;
    h->dl_pending = false;
    h->rec_dirty = true;
    publish_nodes(h);
    return CRANE_OK;
}

int crane_dyn_upload_bindings(crane_dyn* h, int64_t n, const int32_t* node, const int64_t* ts_s) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    if (h->N == -2) return h->fail(CRANE_E_STATE, "engine was not created successfully");
    if (n < 0 || (n > 0 && (!node || !ts_s))) return h->fail(CRANE_E_INVALID, "bad binding arrays");
    HIPTRY(h, hipSetDevice(h->device));
    if (int rc = quiesce(h)) return rc;
    HIPTRY(h, h->sd->bnode.reserve((size_t)n));
    HIPTRY(h, h->sd->bts.reserve((size_t)n));
    if (n > 0) {
        HIPTRY(h, hipMemcpyAsync(h->sd->bnode.p, node, sizeof(int32_t) * n, hipMemcpyHostToDevice, h->stream));
        HIPTRY(h, hipMemcpyAsync(h->sd->bts.p, ts_s, sizeof(int64_t) * n, hipMemcpyHostToDevice, h->stream));
    }
    // a ring of bindings appended in time order (the synthetic and the controller-shaped logs):
    // kept for the suffix search of every refresh
    h->pos_valid = false;
    h->log_sorted = n > 0 && std::is_sorted(ts_s, ts_s + n);
    h->sd->hts_sample.clear();
    if (h->log_sorted) {
        h->sd->hts_copy.assign(ts_s, ts_s + n);
        for (int64_t i = 0; i < n; i += 64) h->sd->hts_sample.push_back(ts_s[i]);
    } else {
        h->sd->hts_copy.clear();
    }
    HIPTRY(h, hipStreamSynchronize(h->stream));
    h->B = n;
    h->heap_mode = false;
    h->sd->heap.reset(0, 0);
    publish_log(h);
    return CRANE_OK;
}

int crane_dyn_binding_records(crane_dyn* h, int64_t size, int64_t gc_time_range_ns) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    if (h->N == -2) return h->fail(CRANE_E_STATE, "engine was not created successfully");
    // size 0 would pop an empty heap in AddBinding (binding.go:73-75); size < 0 never evicts
    if (size <= 0 || size > 0x7FFFFFFF) return h->fail(CRANE_E_INVALID, "binding heap size must be in [1, 2^31)");
    HIPTRY(h, hipSetDevice(h->device));
    if (int rc = quiesce(h)) return rc;
    HIPTRY(h, h->sd->hnode.reserve((size_t)size));
    HIPTRY(h, h->sd->hts.reserve((size_t)size));
    HIPTRY(h, h->sd->bnode.reserve((size_t)size));
    HIPTRY(h, h->sd->bts.reserve((size_t)size));
    for (int64_t i = 0; i < size; ++i) {
        h->sd->hnode.p[i] = -1;
        h->sd->hts.p[i] = 0;
    }
    HIPTRY(h, hipMemcpyAsync(h->sd->bnode.p, h->sd->hnode.p, sizeof(int32_t) * size, hipMemcpyHostToDevice, h->stream));
    HIPTRY(h, hipMemcpyAsync(h->sd->bts.p, h->sd->hts.p, sizeof(int64_t) * size, hipMemcpyHostToDevice, h->stream));
    HIPTRY(h, hipStreamSynchronize(h->stream));
    h->sd->heap.reset(size, gc_time_range_ns);
    h->sd->heap.bind(h->sd->hnode.p, h->sd->hts.p);
    h->heap_mode = true;
    h->log_sorted = false;  // heap order
    h->pos_valid = false;
    h->sd->hts_copy.clear();
    h->sd->hts_sample.clear();
    h->B = size;
    publish_log(h);
    return CRANE_OK;
}

int crane_dyn_add_bindings(crane_dyn* h, int64_t n, const int32_t* node, const int64_t* ts_s) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    if (!h->heap_mode) return h->fail(CRANE_E_STATE, "crane_dyn_binding_records first");
    if (n < 0 || (n > 0 && (!node || !ts_s))) return h->fail(CRANE_E_INVALID, "bad binding arrays");
    HIPTRY(h, hipSetDevice(h->device));
    if (int rc = quiesce(h)) return rc;
    for (int64_t i = 0; i < n; ++i) h->sd->heap.add(node[i], ts_s[i]);
    const int rc = flush_heap_slots(h);
    publish_log(h);  // (the slots changed: the sharing engines' suffix searches restart)
    return rc;
}

int crane_dyn_gc_bindings(crane_dyn* h, int64_t now_ns) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    if (!h->heap_mode) return h->fail(CRANE_E_STATE, "crane_dyn_binding_records first");
    HIPTRY(h, hipSetDevice(h->device));
    if (int rc = quiesce(h)) return rc;
    h->sd->heap.gc(floor_div(now_ns, 1000000000LL));
    const int rc = flush_heap_slots(h);
    publish_log(h);
    return rc;
}

int64_t crane_dyn_binding_count(const crane_dyn* h) {
    if (!h) return CRANE_E_INVALID;
    std::lock_guard<std::mutex> g(const_cast<crane_dyn*>(h)->mu);
    return h->heap_mode ? h->sd->heap.len() : h->B;
}

int crane_dyn_refresh_hot_values(crane_dyn* h, int64_t now_ns, int64_t hv_ts_ns) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    HIPTRY(h, hipSetDevice(h->device));
    if (int rc = quiesce(h)) return rc;
    int rc = hot_values_locked(h, now_ns, hv_ts_ns, h->stream);
    if (rc) return rc;
    HIPTRY(h, hipStreamSynchronize(h->stream));
    return CRANE_OK;
}

int crane_dyn_hot_values(crane_dyn* h, int64_t n, double* hv_out) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    if (h->N < 0) return h->fail(CRANE_E_STATE, "upload nodes before reading hot values");
    if (n != h->N || (n > 0 && !hv_out)) return h->fail(CRANE_E_INVALID, "hv_out must hold one value per node");
    if (n == 0) return CRANE_OK;
    HIPTRY(h, hipSetDevice(h->device));
    if (int rc = quiesce(h)) return rc;
    const double* src = nullptr;
    if (h->hv_from_counts) {
        if (h->counts_pending) {  // the node pass consumes the counts and keeps the values
            int rc = node_pass_locked(h, h->stream);
            if (rc) return rc;
        }
        src = h->hvc.p;
    } else if (h->have_hv) {
        src = h->sd->hv.p;
    }
    if (src) {
        HIPTRY(h, hipMemcpyAsync(hv_out, src, sizeof(double) * n, hipMemcpyDeviceToHost, h->stream));
        HIPTRY(h, hipStreamSynchronize(h->stream));
    } else {
        for (int64_t i = 0; i < n; ++i) hv_out[i] = 0.0;
    }
    return CRANE_OK;
}

int crane_dyn_refresh_hot_values_async(crane_dyn* h, int64_t now_ns, int64_t hv_ts_ns, void* stream) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    HIPTRY(h, hipSetDevice(h->device));
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    int rc = hot_values_locked(h, now_ns, hv_ts_ns, st);
    return rc ? rc : mark_busy(h, st);
}

int crane_dyn_node_pass_async(crane_dyn* h, void* stream) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    HIPTRY(h, hipSetDevice(h->device));
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    int rc = node_pass_locked(h, st);
    return rc ? rc : mark_busy(h, st);
}

int crane_dyn_eval_keys_async(crane_dyn* h, int64_t P, const int64_t* d_now, const uint8_t* d_flags,
                              int64_t* d_keys, void* stream) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    if (P < 0 || (P > 0 && (!d_now || !d_keys))) return h->fail(CRANE_E_INVALID, "bad pod arrays");
    HIPTRY(h, hipSetDevice(h->device));
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    int rc = keys_locked(h, P, d_now, d_flags, reinterpret_cast<long long*>(d_keys), st);
    return rc ? rc : mark_busy(h, st);
}

int crane_dyn_eval_matrix_async(crane_dyn* h, int64_t P, const int64_t* d_now, const uint8_t* d_flags,
                                int8_t* d_first_fail, int8_t* d_score, int64_t ld, int64_t* d_keys, void* stream) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    if (P < 0 || (P > 0 && !d_now)) return h->fail(CRANE_E_INVALID, "bad pod arrays");
    if (h->N < 0) return h->fail(CRANE_E_STATE, "upload nodes before evaluating pods");
    if ((d_first_fail || d_score) && ld < h->N) return h->fail(CRANE_E_INVALID, "ld must be >= the node count");
    HIPTRY(h, hipSetDevice(h->device));
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    int rc = matrix_locked(h, P, d_now, d_flags, reinterpret_cast<long long*>(d_keys), d_first_fail, d_score, false,
                           ld, st);
    return rc ? rc : mark_busy(h, st);
}

// kube-scheduler v1.23.3 numFeasibleNodesToFind (pkg/scheduler/core/generic_scheduler.go,
// not in the container): minFeasibleNodesToFind 100, minFeasibleNodesPercentageToFind 5,
// adaptive percentage 50 - N / 125 when percentageOfNodesToScore <= 0.
int64_t crane_num_feasible_nodes_to_find(int64_t num_all_nodes, int32_t percentage) {
    const int64_t n = num_all_nodes;
    if (n < 100 || percentage >= 100) return n;
    int64_t pct = percentage;
    if (pct <= 0) {
        pct = 50 - n / 125;
        if (pct < 5) pct = 5;
    }
    const int64_t k = n * pct / 100;
    return k < 100 ? 100 : k;
}

int crane_dyn_select(crane_dyn* h, int64_t P, const int64_t* d_now, const uint8_t* d_flags,
                     const uint8_t* d_ext_ok, const int64_t* d_ext_score, int64_t dyn_weight, int32_t percentage,
                     int64_t start, uint64_t tie_seed, int64_t* d_chosen, int64_t* d_total, int64_t* d_wstart,
                     int64_t* d_wlen, int64_t* next_start, void* stream) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    if (P < 0 || (P > 0 && (!d_now || !d_chosen))) return h->fail(CRANE_E_INVALID, "bad pod arrays");
    if (h->N < 0) return h->fail(CRANE_E_STATE, "upload nodes before evaluating pods");
    if (dyn_weight < 0 || dyn_weight > (1 << 20)) return h->fail(CRANE_E_INVALID, "dyn_weight must be in [0, 2^20]");
    if (h->N >= (1LL << 32) || h->node_offset + h->N > (1LL << 32))
        return h->fail(CRANE_E_INVALID, "selection keys hold 32-bit node indices");
    const int64_t N = h->N;
    if (start < 0 || (N > 0 && start >= N)) return h->fail(CRANE_E_INVALID, "start must be in [0, N)");
    HIPTRY(h, hipSetDevice(h->device));
    if (int rc = quiesce(h)) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    const int64_t K = crane_num_feasible_nodes_to_find(N, percentage);
    const bool window = K < N;  // otherwise every node is checked for every pod, the start stays
    if (P == 0 || N == 0) {
        if (next_start) *next_start = start;
        if (P > 0) HIPTRY(h, hipMemsetAsync(d_chosen, 0xFF, sizeof(int64_t) * (size_t)P, st));
        if (P > 0 && d_total) HIPTRY(h, hipMemsetAsync(d_total, 0xFF, sizeof(int64_t) * (size_t)P, st));
        HIPTRY(h, hipStreamSynchronize(st));
        return CRANE_OK;
    }
    if (h->rec_dirty) {
        int rc = node_pass_locked(h, st);
        if (rc) return rc;
    }
    SelArgs a{};
    a.rec = h->rec.p;
    a.N = N;
    a.node_offset = h->node_offset;
    a.now = d_now;
    a.flags = d_flags;
    a.P = P;
    a.wsum = h->dp.wsum;
    a.noprio = h->dp.noprio;
    a.ext_ok = d_ext_ok;
    a.ext_score = d_ext_score;
    a.w_dyn = dyn_weight;
    a.seed = tie_seed;
    a.kb = (uint32_t)(tie_seed * 0x9E3779B97F4A7C15ull >> 32);
    HIPTRY(h, h->sel_keys.reserve((size_t)P));
    HIPTRY(h, h->sel_state.reserve(2));  // next start, chain-form flag
    a.keys = h->sel_keys.p;
    int64_t* ws = d_wstart;
    int64_t* wl = d_wlen;
    if (window) {
        HIPTRY(h, h->sel_fth.reserve((size_t)N));
        if (!ws || !wl) {
            HIPTRY(h, h->sel_win.reserve((size_t)(2 * P)));
            if (!ws) ws = h->sel_win.p;
            if (!wl) wl = h->sel_win.p + P;
        }
        HIPTRY(h, launch_select_fth(a, h->shape, h->sel_fth.p, st));
        HIPTRY(h, launch_select_chain(a, h->sel_fth.p, K, start, ws, wl, h->sel_state.p,
                                      reinterpret_cast<int32_t*>(h->sel_state.p + 1), h->opt.sel_chain, st));
        a.wstart = ws;
        a.wlen = wl;
    }
    HIPTRY(h, hipMemsetAsync(a.keys, 0xFF, sizeof(long long) * (size_t)P, st));
    HIPTRY(h, launch_select_pairs(h->shape, a, st));
    HIPTRY(h, launch_select_decode(a, d_chosen, d_total, st));
    int64_t nxt = start;
    if (window) HIPTRY(h, hipMemcpyAsync(&nxt, h->sel_state.p, sizeof nxt, hipMemcpyDeviceToHost, st));
    HIPTRY(h, hipStreamSynchronize(st));
    if (!window) {  // every pod checked all N nodes: the start advances by N, mod N
        // on the caller's stream and waited for (a pageable hipMemcpy may return before the
        // copy lands and is not ordered with non-blocking streams)
        std::vector<int64_t> vs(d_wstart ? (size_t)P : 0, start), vl(d_wlen ? (size_t)P : 0, N);
        if (d_wstart) HIPTRY(h, hipMemcpyAsync(d_wstart, vs.data(), sizeof(int64_t) * (size_t)P, hipMemcpyHostToDevice, st));
        if (d_wlen) HIPTRY(h, hipMemcpyAsync(d_wlen, vl.data(), sizeof(int64_t) * (size_t)P, hipMemcpyHostToDevice, st));
        if (d_wstart || d_wlen) HIPTRY(h, hipStreamSynchronize(st));
    }
    if (next_start) *next_start = nxt;
    return CRANE_OK;
}

int crane_dyn_step_keys_async(crane_dyn* h, int64_t now_ns, int64_t hv_ts_ns, int64_t P, const int64_t* d_now,
                              const uint8_t* d_flags, int64_t* d_keys, void* stream) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    if (P < 0 || (P > 0 && (!d_now || !d_keys))) return h->fail(CRANE_E_INVALID, "bad pod arrays");
    if (h->N < 0) return h->fail(CRANE_E_STATE, "upload nodes before evaluating pods");
    HIPTRY(h, hipSetDevice(h->device));
    if (!h->busy_q.empty()) {  // (steps on dispatch queues before: they are not ordered with streams)
        if (int rc = quiesce(h)) return rc;
    }
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    long long* keys = reinterpret_cast<long long*>(d_keys);
    if (!step_path_ok(h, P) || P == 0) {
        int rc = hot_values_locked(h, now_ns, hv_ts_ns, st);
        if (!rc) rc = keys_locked(h, P, d_now, d_flags, keys, st);
        return rc ? rc : mark_busy(h, st);
    }
    // the refresh leaves the records stale: plan for the fused node pass; K3p rides in
    // K2x's launch when the dedupe K2 runs
    h->rec_dirty = true;
    StepPlan sp;
    int rc = step_plan(h, P, sp);
    if (rc) return rc;
    const PodPrep pp{d_now, d_flags, P, sp.g.ntiles, sp.perm, sp.pnow, sp.tiles, keys, sp.batch, sp.batch_next};
    bool pods_done = false;
    rc = hot_values_locked(h, now_ns, hv_ts_ns, st, &pp, &pods_done);
    if (pods_done) pods_ran(h, P);
    if (!rc && !pods_done) rc = step_pods(h, sp, P, d_now, d_flags, keys, st);
    if (!rc) rc = step_rest(h, sp, P, keys, st);
    return rc ? rc : mark_busy(h, st);
}

int crane_dyn_step_keys_queue(crane_dyn* h, int64_t now_ns, int64_t hv_ts_ns, int64_t P, const int64_t* d_now,
                              const uint8_t* d_flags, int64_t* d_keys, crane_queue* q) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h, true);  // (a deferred K3s goes into this step's first launch)
    if (lk.rc) return lk.rc;
    if (!q) return h->fail(CRANE_E_INVALID, "null queue");
    if (P < 0 || (P > 0 && (!d_now || !d_keys))) return h->fail(CRANE_E_INVALID, "bad pod arrays");
    if (h->N < 0) return h->fail(CRANE_E_STATE, "upload nodes before evaluating pods");
    HIPTRY(h, hipSetDevice(h->device));
    // a queue is ordered with nothing else: this engine's work on HIP streams or other queues first
    if (!h->busy.empty() || h->busy_q.size() > 1 || (h->busy_q.size() == 1 && h->busy_q[0] != q)) {
        if (int rc = quiesce(h)) return rc;
    }
    long long* keys = reinterpret_cast<long long*>(d_keys);
    if (!step_path_ok(h, P) || P == 0) {
        // (the per-pair form has fills and copies: on the engine stream after the queue, waited for)
        if (aql_wait(q) != hipSuccess) return h->fail(CRANE_E_HIP, std::string("queue: ") + aql_error(q));
        int rc = hot_values_locked(h, now_ns, hv_ts_ns, h->stream);
        if (!rc) rc = keys_locked(h, P, d_now, d_flags, keys, h->stream);
        if (!rc) HIPTRY(h, hipStreamSynchronize(h->stream));
        return rc;
    }
    struct OnQueue {  // this thread's launches go to q until the step is written
        explicit OnQueue(crane_queue* x) { tl_aql = x; }
        ~OnQueue() { tl_aql = nullptr; }
    };
    int rc = CRANE_OK;
    {
        OnQueue on(q);
        const bool defer = h->opt.step_defer != 0;
        // a deferred K3s of another queue, or one writing the keys this step writes (its K3p resets
        // them), runs first, alone
        if (h->pend.on && (h->pend.q != q || h->pend.keys == keys || !defer)) rc = flush_pending(h);
        h->rec_dirty = true;
        StepPlan sp{};
        if (!rc) rc = step_plan(h, P, sp);
        const PodPrep pp{d_now, d_flags, P, sp.g.ntiles, sp.perm, sp.pnow, sp.tiles, keys, sp.batch, sp.batch_next};
        bool pods_done = false;
        if (!rc) rc = hot_values_locked(h, now_ns, hv_ts_ns, h->stream, &pp, &pods_done);
        if (pods_done) pods_ran(h, P);
        // (not taken into the first launch: before this step's node pass rewrites its tables)
        if (!rc && h->pend.on) rc = flush_pending(h);
        if (!rc && !pods_done) rc = step_pods(h, sp, P, d_now, d_flags, keys, h->stream);
        if (!rc) rc = step_rest(h, sp, P, keys, h->stream, defer);
    }
    // (what was written runs even after an error: the packets before it are whole)
    const hipError_t ce = aql_commit(q);
    if (std::find(h->busy_q.begin(), h->busy_q.end(), q) == h->busy_q.end()) h->busy_q.push_back(q);
    if (std::find(h->seen_q.begin(), h->seen_q.end(), q) == h->seen_q.end()) {
        h->seen_q.push_back(q);
        aql_add_user(q, h);
    }
    if (rc) return rc;
    if (ce != hipSuccess) return h->fail(CRANE_E_HIP, std::string("queue: ") + aql_error(q));
    return CRANE_OK;
}

// Host-pointer evaluation: the matrices go through device scratch in pod slices of
// at most ~64M entries; chosen nodes come from the same kernel's keys.
static int eval_host(crane_dyn* h, int64_t P, const int64_t* now_ns, const uint8_t* pod_flags, int8_t* first_fail,
                     void* score, bool score_i64, int64_t* chosen, int64_t* chosen_score) {
    if (P < 0 || (P > 0 && !now_ns)) return h->fail(CRANE_E_INVALID, "bad pod arrays");
    if (h->N < 0) return h->fail(CRANE_E_STATE, "upload nodes before evaluating pods");
    HIPTRY(h, hipSetDevice(h->device));
    if (int rc = quiesce(h)) return rc;
    const int64_t N = h->N;
    const bool matrix = first_fail || score;
    int64_t pc = P;
    if (matrix && N > 0) pc = std::max<int64_t>(1, std::min<int64_t>(P, (int64_t)(64LL << 20) / N));
    if (pc <= 0) pc = 1;
    HIPTRY(h, h->now.reserve((size_t)pc));
    HIPTRY(h, h->flags.reserve((size_t)pc));
    HIPTRY(h, h->keys.reserve((size_t)pc));
    HIPTRY(h, h->stagek.reserve((size_t)pc));
    const size_t cells = (size_t)(pc * std::max<int64_t>(N, 1));
    if (first_fail) HIPTRY(h, h->ff.reserve(cells));
    if (score && score_i64) HIPTRY(h, h->score.reserve(cells));
    if (score && !score_i64) HIPTRY(h, h->score8.reserve(cells));
    const bool compact = !score_i64;  // compact rows come back through pinned staging
    if (compact && matrix) HIPTRY(h, h->stage8.reserve(2 * cells));
    for (int64_t p0 = 0; p0 < P; p0 += pc) {
        const int64_t np = std::min(pc, P - p0);
        HIPTRY(h, hipMemcpyAsync(h->now.p, now_ns + p0, sizeof(int64_t) * np, hipMemcpyHostToDevice, h->stream));
        if (pod_flags)
            HIPTRY(h, hipMemcpyAsync(h->flags.p, pod_flags + p0, np, hipMemcpyHostToDevice, h->stream));
        int rc;
        if (!matrix) {
            rc = keys_locked(h, np, h->now.p, pod_flags ? h->flags.p : nullptr, h->keys.p, h->stream);
        } else {
            void* sdev = !score ? nullptr : score_i64 ? (void*)h->score.p : (void*)h->score8.p;
            rc = matrix_locked(h, np, h->now.p, pod_flags ? h->flags.p : nullptr, h->keys.p,
                               first_fail ? h->ff.p : nullptr, sdev, score_i64, N, h->stream);
        }
        if (rc) return rc;
        HIPTRY(h, hipMemcpyAsync(h->stagek.p, h->keys.p, sizeof(long long) * np, hipMemcpyDeviceToHost, h->stream));
        const size_t cnt = (size_t)(np * N);
        if (first_fail && N > 0)
            HIPTRY(h, hipMemcpyAsync(compact ? (void*)h->stage8.p : (void*)(first_fail + p0 * N), h->ff.p, cnt,
                                     hipMemcpyDeviceToHost, h->stream));
        if (score && N > 0) {
            if (score_i64)
                HIPTRY(h, hipMemcpyAsync(static_cast<int64_t*>(score) + p0 * N, h->score.p, sizeof(int64_t) * cnt,
                                         hipMemcpyDeviceToHost, h->stream));
            else
                HIPTRY(h, hipMemcpyAsync(h->stage8.p + cells, h->score8.p, cnt, hipMemcpyDeviceToHost, h->stream));
        }
        HIPTRY(h, hipStreamSynchronize(h->stream));
        if (compact && first_fail && N > 0) std::memcpy(first_fail + p0 * N, h->stage8.p, cnt);
        if (compact && score && N > 0) std::memcpy(static_cast<int8_t*>(score) + p0 * N, h->stage8.p + cells, cnt);
        for (int64_t i = 0; i < np; ++i) {
            int64_t s;
            const int64_t nd = crane_dyn_key_node(h->stagek.p[i], &s);
            if (chosen) chosen[p0 + i] = nd;
            if (chosen_score) chosen_score[p0 + i] = s;
        }
    }
    return CRANE_OK;
}

int crane_dyn_eval(crane_dyn* h, int64_t P, const int64_t* now_ns, const uint8_t* pod_flags, int8_t* first_fail,
                   int64_t* score, int64_t* chosen, int64_t* chosen_score) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    return eval_host(h, P, now_ns, pod_flags, first_fail, score, true, chosen, chosen_score);
}

int crane_dyn_eval_compact(crane_dyn* h, int64_t P, const int64_t* now_ns, const uint8_t* pod_flags,
                           int8_t* first_fail, int8_t* score, int64_t* chosen, int64_t* chosen_score) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    return eval_host(h, P, now_ns, pod_flags, first_fail, score, false, chosen, chosen_score);
}

int32_t crane_dyn_step_slots(const crane_dyn* h) { return h && h->N != -2 ? node_step_slots(h->shape) : 0; }

int crane_dyn_node_steps(crane_dyn* h, int64_t t0_ns, int64_t t1_ns, int64_t n, uint8_t* n_steps, int64_t* bp,
                         int8_t* first_fail, int8_t* score) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    if (h->N < 0) return h->fail(CRANE_E_STATE, "upload nodes before building node tables");
    if (n != h->N) return h->fail(CRANE_E_INVALID, "the tables hold one entry per node of the shard");
    if (n > 0 && (!n_steps || !bp || !first_fail || !score)) return h->fail(CRANE_E_INVALID, "NULL output");
    if (!(t0_ns < t1_ns)) return h->fail(CRANE_E_INVALID, "t0 must be before t1");
    if (n == 0) return CRANE_OK;
    HIPTRY(h, hipSetDevice(h->device));
    // a fused step_keys_async on a caller stream may still be writing what the node pass reads
    if (int rc = quiesce(h)) return rc;
    hipStream_t st = h->stream;
    if (h->rec_dirty) {
        int rc = node_pass_locked(h, st);
        if (rc) return rc;
    }
    const size_t S = (size_t)node_step_slots(h->shape), N = (size_t)n;
    const size_t o_ns = 8 * N * S, o_ff = o_ns + N, o_sc = o_ff + N * (S + 1), total = o_sc + N * (S + 1);
    HIPTRY(h, h->stp_dev.reserve(total));
    HIPTRY(h, h->stp_host.reserve(total));
    MatrixArgs a{};
    a.rec = h->rec.p;
    a.N = h->N;
    a.node_offset = h->node_offset;
    a.wsum = h->dp.wsum;
    a.noprio = h->dp.noprio;
    std::memcpy(a.pred_orig, h->pred_orig, sizeof a.pred_orig);
    unsigned char* d = h->stp_dev.p;
    HIPTRY(h, launch_node_steps(h->shape, a, t0_ns, t1_ns, d + o_ns, reinterpret_cast<int64_t*>(d),
                                reinterpret_cast<int8_t*>(d + o_ff), reinterpret_cast<int8_t*>(d + o_sc), st));
    HIPTRY(h, hipMemcpyAsync(h->stp_host.p, d, total, hipMemcpyDeviceToHost, st));
    HIPTRY(h, hipStreamSynchronize(st));
    const unsigned char* p = h->stp_host.p;
    std::memcpy(bp, p, 8 * N * S);
    std::memcpy(n_steps, p + o_ns, N);
    std::memcpy(first_fail, p + o_ff, N * (S + 1));
    std::memcpy(score, p + o_sc, N * (S + 1));
    return CRANE_OK;
}

// k distinct local node indices in [0, N): CRANE_OK or the error
static int check_subset(crane_dyn* h, int64_t k, const int64_t* idx) {
    if (h->N < 0) return h->fail(CRANE_E_STATE, "upload nodes first");
    if (k < 0 || (k > 0 && !idx)) return h->fail(CRANE_E_INVALID, "bad node index array");
    if (k > h->N) return h->fail(CRANE_E_INVALID, "more indices than nodes");
    std::vector<int64_t> sorted(idx, idx + k);
    std::sort(sorted.begin(), sorted.end());
    for (int64_t j = 0; j < k; ++j) {
        if (sorted[j] < 0 || sorted[j] >= h->N) return h->fail(CRANE_E_INVALID, "node index out of range");
        if (j > 0 && sorted[j] == sorted[j - 1]) return h->fail(CRANE_E_INVALID, "duplicate node index");
    }
    return CRANE_OK;
}

// Table rows the fused update writes (crane_dyn_update_node_steps): outputs of k rows.
struct RowOut {
    int64_t t0, t1;
    uint8_t* n_steps;
    int64_t* bp;
    int8_t* first_fail;
    int8_t* score;
};

static int update_locked(crane_dyn* h, int64_t k, const int64_t* idx, const double* val, const int64_t* ts,
                         const double* hv, const int64_t* hv_ts, const RowOut* rows) {
    if (int rc = check_subset(h, k, idx)) return rc;
    const int64_t M = h->dp.n_slots;
    if (k > 0 && M > 0 && (!val || !ts)) return h->fail(CRANE_E_INVALID, "val/ts must not be NULL");
    if ((hv == nullptr) != (hv_ts == nullptr)) return h->fail(CRANE_E_INVALID, "hv and hv_ts must both be set or NULL");
    if (rows && k > 0 && (!rows->n_steps || !rows->bp || !rows->first_fail || !rows->score))
        return h->fail(CRANE_E_INVALID, "NULL output");
    if (rows && !(rows->t0 < rows->t1)) return h->fail(CRANE_E_INVALID, "t0 must be before t1");
    if (k == 0) return CRANE_OK;
    // CRANE_DYN_TRACE_UPD=1: each update's parts on stderr (the drop-in's slowest cycles)
    static const bool trace_upd = std::getenv("CRANE_DYN_TRACE_UPD") != nullptr;
    using TClock = std::chrono::steady_clock;
    const TClock::time_point u0 = trace_upd ? TClock::now() : TClock::time_point{};
    HIPTRY(h, hipSetDevice(h->device));
    if (int rc = quiesce(h)) return rc;
    const TClock::time_point u1 = trace_upd ? TClock::now() : TClock::time_point{};
    // the hot values come from the annotations again, as after crane_dyn_upload_nodes: records
    // built from binding-log counts are stale as a whole
    if (h->hv_from_counts) {
        h->hv_from_counts = false;
        h->counts_pending = false;
        h->hx_pending = false;
        h->dl_pending = false;
        h->rec_dirty = true;
    }
    if (hv && !h->have_hv) {  // the first hot-value annotations of the shard: the others have none
        HIPTRY(h, h->sd->hv.reserve((size_t)h->N));
        HIPTRY(h, h->sd->hv_ts.reserve((size_t)h->N));
        HIPTRY(h, hipMemsetAsync(h->sd->hv.p, 0, sizeof(double) * (size_t)h->N, h->stream));
        HIPTRY(h, launch_fill_i64(h->sd->hv_ts.p, h->N, kTsInvalid, h->stream));
        h->have_hv = true;
    }
    // staging: in idx [k] | val [M][k] | ts [M][k] | hv [k] | hv_ts [k];  out (rows) bp [k][S] | ns [k] |
    // ff [k][S+1] | sc [k][S+1]
    const size_t K = (size_t)k, S = (size_t)node_step_slots(h->shape);
    const size_t o_val = 8 * K, o_ts = o_val + 8 * (size_t)M * K, o_hv = o_ts + 8 * (size_t)M * K,
                 o_hvt = o_hv + 8 * K, o_out = o_hvt + 8 * K;
    const size_t r_ns = o_out + 8 * K * S, r_ff = r_ns + K, r_sc = r_ff + K * (S + 1), r_end = r_sc + K * (S + 1);
    const size_t total = rows ? r_end : o_out;
    HIPTRY(h, h->upd_host.grow(total));
    unsigned char* p = h->upd_host.p;
    std::memcpy(p, idx, 8 * K);
    if (M > 0) {
        std::memcpy(p + o_val, val, 8 * (size_t)M * K);
        std::memcpy(p + o_ts, ts, 8 * (size_t)M * K);
    }
    if (hv) {
        std::memcpy(p + o_hv, hv, 8 * K);
        std::memcpy(p + o_hvt, hv_ts, 8 * K);
    }
    // The kernel reads the staged columns from and writes the rows to the pinned staging itself
    // (a few KB to a few hundred): no copy-engine commands, whose first use after the device sat
    // idle for a while cost the drop-in's first changed cycle 10-15 ms (the copy engines power
    // down; a kernel's first launch after the same gap costs 0.3 ms, tools/idle_probe.py)
    unsigned char* d = nullptr;
    HIPTRY(h, hipHostGetDevicePointer(reinterpret_cast<void**>(&d), p, 0));
    UpdateArgs a{};
    a.pol = h->dp;
    a.N = h->N;
    a.k = k;
    a.idx = reinterpret_cast<const int64_t*>(d);
    a.sval = reinterpret_cast<const double*>(d + o_val);
    a.sts = reinterpret_cast<const int64_t*>(d + o_ts);
    a.shv = hv ? reinterpret_cast<const double*>(d + o_hv) : nullptr;
    a.shv_ts = hv ? reinterpret_cast<const int64_t*>(d + o_hvt) : nullptr;
    a.val = h->sd->val.p;
    a.ts = h->sd->ts.p;
    a.hv = h->have_hv ? h->sd->hv.p : nullptr;
    a.hv_ts = h->have_hv ? h->sd->hv_ts.p : nullptr;
    a.rec = h->rec_dirty ? nullptr : h->rec.p;  // current records stay current
    if (rows) {
        a.ma.wsum = h->dp.wsum;
        a.ma.noprio = h->dp.noprio;
        std::memcpy(a.ma.pred_orig, h->pred_orig, sizeof a.ma.pred_orig);
        a.t0 = rows->t0;
        a.t1 = rows->t1;
        a.bp = reinterpret_cast<int64_t*>(d + o_out);
        a.ns = d + r_ns;
        a.ff = reinterpret_cast<int8_t*>(d + r_ff);
        a.sc = reinterpret_cast<int8_t*>(d + r_sc);
    }
    const TClock::time_point u2 = trace_upd ? TClock::now() : TClock::time_point{};
    hipEvent_t ev[2] = {nullptr, nullptr};
    if (trace_upd && hipEventCreate(&ev[0]) == hipSuccess && hipEventCreate(&ev[1]) == hipSuccess)
        (void)hipEventRecord(ev[0], h->stream);
    HIPTRY(h, launch_update_nodes(h->shape, a, h->stream));
    if (ev[1]) (void)hipEventRecord(ev[1], h->stream);
    const TClock::time_point u3 = trace_upd ? TClock::now() : TClock::time_point{};
    // (waited for: the staging is reused, and work the caller enqueues next on its own
    // streams must see the new columns).  Polled for the first 2 ms, then a blocking wait: the
    // update is tens of microseconds of GPU work, and a blocking wait's wake-up is the host's
    // interrupt path, slow when every core is busy (the framework's goroutines spin meanwhile)
    long long nq = 0;
    double qmax_us = 0.0;
    {
        const TClock::time_point w0 = TClock::now();
        hipError_t q;
        for (;;) {
            const TClock::time_point a0 = trace_upd ? TClock::now() : TClock::time_point{};
            q = hipStreamQuery(h->stream);
            if (trace_upd) {
                ++nq;
                qmax_us = std::max(qmax_us, std::chrono::duration<double, std::micro>(TClock::now() - a0).count());
            }
            if (q != hipErrorNotReady || TClock::now() - w0 >= std::chrono::milliseconds(2)) break;
            __builtin_ia32_pause();
        }
        if (q == hipErrorNotReady) q = hipStreamSynchronize(h->stream);
        HIPTRY(h, q);
    }
    if (trace_upd) {
        auto us = [](TClock::time_point x, TClock::time_point y) {
            return std::chrono::duration<double, std::micro>(y - x).count();
        };
        const TClock::time_point u4 = TClock::now();
        float gpu_ms = -1.f;
        if (ev[1]) (void)hipEventElapsedTime(&gpu_ms, ev[0], ev[1]);
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        std::fprintf(stderr, "crane_dyn update k=%lld: quiesce %.1f us, staging %.1f us, launch %.1f us, "
                     "sync %.1f us (kernel between events %.1f us; %lld queries, the longest %.1f us)\n",
                     (long long)k, us(u0, u1), us(u1, u2), us(u2, u3), us(u3, u4), gpu_ms * 1000.f, nq, qmax_us);
    }
    publish_nodes(h);  // (the engines sharing the shard rebuild their records from the new columns)
    if (rows) {
        std::memcpy(rows->bp, p + o_out, 8 * K * S);
        std::memcpy(rows->n_steps, p + r_ns, K);
        std::memcpy(rows->first_fail, p + r_ff, K * (S + 1));
        std::memcpy(rows->score, p + r_sc, K * (S + 1));
    }
    return CRANE_OK;
}

// Grow or shrink the shard to n nodes in place: nodes [0, min(N, n)) keep their parsed columns,
// nodes past the old count start with no annotations (every metric and the hot value missing);
// records are rebuilt by the next pass that needs them.  (The drop-in plugin adds joining nodes
// this way and then writes their columns with crane_dyn_update_node_steps.)
int crane_dyn_resize_nodes(crane_dyn* h, int64_t n) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    if (h->N < 0) return h->fail(CRANE_E_STATE, "upload nodes before resizing the shard");
    if (n < 0 || n > 0xFFFFFFFFLL || h->node_offset + n > 0xFFFFFFFFLL)
        return h->fail(CRANE_E_INVALID, "node count out of range (global indices must fit 32 bits)");
    if (n == h->N) return CRANE_OK;
    HIPTRY(h, hipSetDevice(h->device));
    if (int rc = quiesce(h)) return rc;
    const int64_t M = h->dp.n_slots, keep = std::min(h->N, n), N0 = h->N;
    DevBuf<double> val, hv;
    DevBuf<int64_t> ts, hv_ts;
    auto fail = [&](hipError_t e, const char* what) {
        val.release(); ts.release(); hv.release(); hv_ts.release();
        return h->hipfail(e, what);
    };
    hipError_t e = val.reserve((size_t)(M * n));
    if (e == hipSuccess) e = ts.reserve((size_t)(M * n));
    if (e == hipSuccess) e = hv.reserve((size_t)n);
    if (e == hipSuccess) e = hv_ts.reserve((size_t)n);
    if (e != hipSuccess) return fail(e, "resize: hipMalloc");
    hipStream_t st = h->stream;
    if (M > 0 && keep > 0) {
        e = hipMemcpy2DAsync(val.p, sizeof(double) * n, h->sd->val.p, sizeof(double) * N0, sizeof(double) * keep, M,
                             hipMemcpyDeviceToDevice, st);
        if (e == hipSuccess)
            e = hipMemcpy2DAsync(ts.p, sizeof(int64_t) * n, h->sd->ts.p, sizeof(int64_t) * N0, sizeof(int64_t) * keep, M,
                                 hipMemcpyDeviceToDevice, st);
    }
    for (int64_t m = 0; m < M && n > keep && e == hipSuccess; ++m) {
        e = hipMemsetAsync(val.p + m * n + keep, 0, sizeof(double) * (size_t)(n - keep), st);
        if (e == hipSuccess) e = launch_fill_i64(ts.p + m * n + keep, n - keep, kTsInvalid, st);
    }
    if (h->have_hv && keep > 0 && e == hipSuccess) {
        e = hipMemcpyAsync(hv.p, h->sd->hv.p, sizeof(double) * (size_t)keep, hipMemcpyDeviceToDevice, st);
        if (e == hipSuccess)
            e = hipMemcpyAsync(hv_ts.p, h->sd->hv_ts.p, sizeof(int64_t) * (size_t)keep, hipMemcpyDeviceToDevice, st);
    }
    if (h->have_hv && n > keep && e == hipSuccess) {
        e = hipMemsetAsync(hv.p + keep, 0, sizeof(double) * (size_t)(n - keep), st);
        if (e == hipSuccess) e = launch_fill_i64(hv_ts.p + keep, n - keep, kTsInvalid, st);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return fail(e, "resize: copy");
    std::swap(h->sd->val, val);
    std::swap(h->sd->ts, ts);
    std::swap(h->sd->hv, hv);
    std::swap(h->sd->hv_ts, hv_ts);
    val.release(); ts.release(); hv.release(); hv_ts.release();
    HIPTRY(h, h->rec.reserve((size_t)n * h->rec_bytes));
    h->N = n;
    h->buckets_zero = false;
    h->hv_from_counts = false;  // binding-log hot values were per old node index
    h->counts_pending = false;
    h->hx_pending = false;
    h->dl_pending = false;
    h->rec_dirty = true;
    publish_nodes(h);
    return CRANE_OK;
}

int crane_dyn_update_nodes(crane_dyn* h, int64_t k, const int64_t* idx, const double* val, const int64_t* ts,
                           const double* hv, const int64_t* hv_ts) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    return update_locked(h, k, idx, val, ts, hv, hv_ts, nullptr);
}

int crane_dyn_update_node_steps(crane_dyn* h, int64_t k, const int64_t* idx, const double* val, const int64_t* ts,
                                const double* hv, const int64_t* hv_ts, int64_t t0_ns, int64_t t1_ns,
                                uint8_t* n_steps, int64_t* bp, int8_t* first_fail, int8_t* score) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    const RowOut rows{t0_ns, t1_ns, n_steps, bp, first_fail, score};
    return update_locked(h, k, idx, val, ts, hv, hv_ts, &rows);
}

int crane_dyn_node_steps_subset(crane_dyn* h, int64_t t0_ns, int64_t t1_ns, int64_t k, const int64_t* idx,
                                uint8_t* n_steps, int64_t* bp, int8_t* first_fail, int8_t* score) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    if (int rc = check_subset(h, k, idx)) return rc;
    if (k > 0 && (!n_steps || !bp || !first_fail || !score)) return h->fail(CRANE_E_INVALID, "NULL output");
    if (!(t0_ns < t1_ns)) return h->fail(CRANE_E_INVALID, "t0 must be before t1");
    if (k == 0) return CRANE_OK;
    HIPTRY(h, hipSetDevice(h->device));
    if (int rc = quiesce(h)) return rc;
    hipStream_t st = h->stream;
    if (h->rec_dirty) {
        int rc = node_pass_locked(h, st);
        if (rc) return rc;
    }
    // staging: out bp [k][S] | ns [k] | ff [k][S+1] | sc [k][S+1] | in idx [k]
    const size_t S = (size_t)node_step_slots(h->shape), K = (size_t)k;
    const size_t o_ns = 8 * K * S, o_ff = o_ns + K, o_sc = o_ff + K * (S + 1), o_out = o_sc + K * (S + 1);
    const size_t o_idx = (o_out + 7) & ~(size_t)7, total = o_idx + 8 * K;
    HIPTRY(h, h->upd_host.grow(total));
    HIPTRY(h, h->upd_dev.grow(total));
    std::memcpy(h->upd_host.p + o_idx, idx, 8 * K);
    unsigned char* d = h->upd_dev.p;
    HIPTRY(h, hipMemcpyAsync(d + o_idx, h->upd_host.p + o_idx, 8 * K, hipMemcpyHostToDevice, st));
    MatrixArgs a{};
    a.rec = h->rec.p;
    a.N = k;
    a.node_offset = h->node_offset;
    a.wsum = h->dp.wsum;
    a.noprio = h->dp.noprio;
    std::memcpy(a.pred_orig, h->pred_orig, sizeof a.pred_orig);
    HIPTRY(h, launch_node_steps(h->shape, a, t0_ns, t1_ns, d + o_ns, reinterpret_cast<int64_t*>(d),
                                reinterpret_cast<int8_t*>(d + o_ff), reinterpret_cast<int8_t*>(d + o_sc), st,
                                reinterpret_cast<const int64_t*>(d + o_idx)));
    HIPTRY(h, hipMemcpyAsync(h->upd_host.p, d, o_out, hipMemcpyDeviceToHost, st));
    HIPTRY(h, hipStreamSynchronize(st));
    const unsigned char* p = h->upd_host.p;
    std::memcpy(bp, p, 8 * K * S);
    std::memcpy(n_steps, p + o_ns, K);
    std::memcpy(first_fail, p + o_ff, K * (S + 1));
    std::memcpy(score, p + o_sc, K * (S + 1));
    return CRANE_OK;
}

int crane_dyn_set_profiling(crane_dyn* h, int on) {
    if (!h) return CRANE_E_INVALID;
    std::lock_guard<std::mutex> g(h->mu);
    h->prof = on != 0;
    h->nk = 0;
    h->timer_err = hipSuccess;
    return CRANE_OK;
}

int crane_dyn_stage_times(crane_dyn* h, int32_t max, const char** names, double* ms) {
    if (!h) return CRANE_E_INVALID;
    std::lock_guard<std::mutex> g(h->mu);
    if (h->timer_err != hipSuccess) {
        const hipError_t e = h->timer_err;
        h->timer_err = hipSuccess;
        h->nk = 0;
        return h->hipfail(e, "kernel timer events");
    }
    int n = 0;
    for (int i = 0; i < h->nk && n < max; ++i, ++n) {
        HIPTRY(h, hipEventSynchronize(h->ev[2 * i + 1]));
        float t = 0.f;
        HIPTRY(h, hipEventElapsedTime(&t, h->ev[2 * i], h->ev[2 * i + 1]));
        if (names) names[n] = h->ev_name[i];
        if (ms) ms[n] = t;
    }
    h->nk = 0;
    return n;
}

int crane_dyn_greedy(crane_dyn* h, int64_t P, int64_t now_ns, const uint8_t* pod_flags, int64_t* chosen) {
    if (!h) return CRANE_E_INVALID;
    Locked lk(h);
    if (lk.rc) return lk.rc;
    if (P < 0 || (P > 0 && !chosen)) return h->fail(CRANE_E_INVALID, "bad pod arrays");
    if (h->N < 0) return h->fail(CRANE_E_STATE, "upload nodes before greedy placement");
    if (h->N > kGreedyMaxNodes) return h->fail(CRANE_E_INVALID, "greedy mode supports up to 64^4 nodes");
    HIPTRY(h, hipSetDevice(h->device));
    if (int rc = quiesce(h)) return rc;
    hipStream_t st = h->stream;
    const int64_t N = h->N;
    // hot values from the binding log at `now`, annotation stamped `now` (fresh)
    int rc = hot_values_locked(h, now_ns, now_ns, st);
    if (rc) return rc;
    const int W = h->dp.n_win;
    HIPTRY(h, h->gcnt.reserve((size_t)std::max(1, W) * (size_t)std::max<int64_t>(N, 1)));
    rc = node_pass_locked(h, st, h->gcnt.p);
    if (rc) return rc;
    h->rec_dirty = true;  // records now carry the greedy batch's hot values; recompute for eval
    GreedyArgs a{};
    a.now = now_ns;
    a.wsum = h->dp.wsum;
    a.noprio = h->dp.noprio;
    a.n_win = W;
    const int64_t now_unix = floor_div(now_ns, 1000000000LL);
    for (int w = 0; w < W; ++w) {
        a.win_count[w] = h->dp.win_count[w];
        // binding.go:85-91 for Binding{Timestamp: now_unix}
        a.win_inc[w] = now_unix > now_unix - go_seconds_trunc(h->hot_tr[w]);
    }
    HIPTRY(h, h->gbase.reserve((size_t)std::max<int64_t>(N, 1)));
    HIPTRY(h, h->gleaf.reserve((size_t)std::max<int64_t>(N, 1)));
    HIPTRY(h, h->gchosen.reserve((size_t)std::max<int64_t>(P, 1)));
    HIPTRY(h, h->gflags.reserve((size_t)std::max<int64_t>(P, 1)));
    if (pod_flags && P > 0) HIPTRY(h, hipMemcpyAsync(h->gflags.p, pod_flags, P, hipMemcpyHostToDevice, st));
    // Merge form (merge.hip) when every hotValue count is positive; else the sequential kernel
    bool merge = h->opt.greedy_form == 0 && N > 0 && P > 0;
    for (int w = 0; w < W; ++w) merge = merge && a.win_count[w] > 0;
    bool done = false;
    if (merge) {
        int64_t Pd = 0;
        if (pod_flags)
            for (int64_t p = 0; p < P; ++p) Pd += pod_flags[p] & 1;
        HIPTRY(h, launch_greedy(h->shape, h->rec.p, N, h->gcnt.p, a, h->gbase.p, h->gleaf.p, P, nullptr, nullptr, st,
                                kGreedyPrep));
        MergeArgs ma{};
        ma.n_win = W;
        for (int w = 0; w < W; ++w) {
            ma.win_count[w] = a.win_count[w];
            ma.win_inc[w] = a.win_inc[w];
        }
        HIPTRY(h, h->mH.reserve(2 * 101));
        HIPTRY(h, h->mflag.reserve(1));
        HIPTRY(h, launch_merge_hist(h->gbase.p, h->gleaf.p, h->gcnt.p, N, ma, P, Pd, h->mH.p, h->mflag.p, st));
        unsigned long long Hh[2 * 101];
        int32_t flag = 1;
        HIPTRY(h, hipMemcpyAsync(Hh, h->mH.p, sizeof Hh, hipMemcpyDeviceToHost, st));
        HIPTRY(h, hipMemcpyAsync(&flag, h->mflag.p, sizeof flag, hipMemcpyDeviceToHost, st));
        HIPTRY(h, hipStreamSynchronize(st));
        if (flag == 0) {
            // cut level: the stream's first `cap` elements all have score >= vlo
            auto cut = [&](int T, int64_t cap, int* vlo) -> int64_t {
                unsigned long long cum = 0;
                *vlo = 0;
                for (int u = 100; u >= 0; --u) {
                    cum += Hh[T * 101 + u];
                    if (cum >= (unsigned long long)cap) {
                        *vlo = u;
                        return cap;
                    }
                }
                return (int64_t)cum;
            };
            int vF = 0, vI = 0;
            const int64_t nF = cut(0, P, &vF);
            const int64_t nI = Pd ? cut(1, Pd, &vI) : 0;
            HIPTRY(h, h->mbs.reserve((size_t)merge_bsum_len(N, std::min(vF, vI))));
            HIPTRY(h, h->mFs.reserve((size_t)std::max<int64_t>(nF, 1)));
            HIPTRY(h, h->mIs.reserve((size_t)std::max<int64_t>(nI, 1)));
            HIPTRY(h, h->mapos.reserve((size_t)std::max<int64_t>(Pd, 1)));
            HIPTRY(h, h->mtk.reserve((size_t)std::max<int64_t>(nI, 1)));
            HIPTRY(h, h->mgi.reserve((size_t)std::max<int64_t>(nI, 1) + 1));
            if (nF) HIPTRY(h, launch_merge_stream(h->gbase.p, h->gleaf.p, h->gcnt.p, N, ma, 0, vF, nF, h->mbs.p,
                                                  h->mFs.p, st));
            if (nI) HIPTRY(h, launch_merge_stream(h->gbase.p, h->gleaf.p, h->gcnt.p, N, ma, 1, vI, nI, h->mbs.p,
                                                  h->mIs.p, st));
            HIPTRY(h, launch_merge_assign(h->mFs.p, nF, h->mIs.p, nI, h->gflags.p, P, Pd, h->mapos.p, h->mtk.p,
                                          h->mgi.p, h->gchosen.p, st));
            done = true;
        }
    }
    if (!done)
        HIPTRY(h, launch_greedy(h->shape, h->rec.p, N, h->gcnt.p, a, h->gbase.p, h->gleaf.p, P,
                                pod_flags ? h->gflags.p : nullptr, h->gchosen.p, st, merge ? kGreedyRun : kGreedyBoth));
    if (P > 0) HIPTRY(h, hipMemcpyAsync(chosen, h->gchosen.p, sizeof(int64_t) * P, hipMemcpyDeviceToHost, st));
    HIPTRY(h, hipStreamSynchronize(st));
    for (int64_t p = 0; p < P; ++p)
        if (chosen[p] >= 0) chosen[p] += h->node_offset;
    return CRANE_OK;
}

}  // extern "C"
