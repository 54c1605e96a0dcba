// kernels.hpp — host-side launch interface of the engine's kernels.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aql.hpp"
#include "dyn_types.hpp"

namespace crane {

// NodeRec template instances (max predicates x max priorities).
enum { kShape4x6 = 0, kShape8x8 = 1, kShape16x16 = 2 };

// ---------------------------------------------------------------- launches
// Kernel timing (crane_dyn_set_profiling): while a KernelTimer is installed on
// the calling thread, every launch gets a (start, stop) event pair that the
// runtime stamps from the dispatch itself (hipExtLaunchKernel), i.e. the
// kernel's own begin -> end as rocprofv3 --kernel-trace reports it.
struct KernelTimer {
    virtual ~KernelTimer() = default;
    virtual void next(const char* name, hipEvent_t* start, hipEvent_t* stop) = 0;
};
extern thread_local KernelTimer* tl_ktimer;

// On a thread with an AQL queue installed (aql.hpp: a step on a crane_queue) the launch is a
// packet on that queue instead (no timing events there).
template <typename... KArgs, typename... Args>
inline hipError_t klaunch(const char* name, void (*kernel)(KArgs...), dim3 grid, dim3 block, size_t lds,
                          hipStream_t st, Args... args) {
    if (tl_aql) {
        static_assert((sizeof(KArgs) + ... + 0) + 16 * sizeof...(KArgs) <= kAqlMaxArgs, "kernel arguments too large");
        alignas(16) unsigned char buf[kAqlMaxArgs];
        size_t off = 0;
        (aql_pack<KArgs>(buf, off, static_cast<KArgs>(args)), ...);
        return aql_launch(tl_aql, reinterpret_cast<const void*>(kernel), grid, block, (uint32_t)lds, buf, off);
    }
    hipEvent_t a = nullptr, b = nullptr;
    if (tl_ktimer) tl_ktimer->next(name, &a, &b);
    hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)lds, st, a, b, 0u, static_cast<KArgs>(args)...);
    return hipGetLastError();
}

// Phase trace (engine option "trace", crane_dyn_debug_trace): when non-null, thread 0
// of every workgroup stores s_memrealtime stamps (100 MHz) at the kernel's phase
// boundaries into trace[8 * workgroup + k].
// (stamp 0 also records the workgroup's XCD in slot 7: HW_REG_XCC_ID, hwreg id 20)
#define CRANE_TSTAMP(tr, wg, k)                                                                      \
    do {                                                                                             \
        if ((tr) && threadIdx.x == 0) {                                                              \
            (tr)[8 * (int64_t)(wg) + (k)] = __builtin_amdgcn_s_memrealtime();                        \
            if ((k) == 0) (tr)[8 * (int64_t)(wg) + 7] = (unsigned)__builtin_amdgcn_s_getreg(63508) & 15u; \
        }                                                                                            \
    } while (0)

// One scalar load per 64-byte line of the first BYTES of this launch's kernarg segment, all in
// flight together and waited for once, so the launch's later argument reads (chains of scalar
// load -> wait -> branch, the policy words under per-term conditions) hit the scalar cache instead
// of each waiting for its own L2 round trip.  Called after a kernel's first vector loads are
// issued, so the wait overlaps theirs.
template <int BYTES>
__device__ __forceinline__ void kernarg_warm() {
    typedef const uint32_t __attribute__((address_space(4)))* kptr;
    const kptr p = (kptr)__builtin_amdgcn_kernarg_segment_ptr();
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < BYTES / 4; i += 16) x ^= p[i];
    asm volatile("" ::"s"(x));
}

struct HotCutoffs {
    int32_t n_win;
    // 0: sorted[] are the ascending cutoffs now_unix - int64(timeRange.Seconds()) and a
    // binding's window rank is #{w : ts > sorted[w]};  1 (a time-ordered log, the binding
    // array passed from its first binding inside the widest window on): sorted[w] = (the
    // first binding inside window w) - 1, relative, and the rank is the same count over the
    // binding's position — the timestamps are not read
    int32_t by_pos;
    int64_t sorted[kMaxWin];
};

// ---------------------------------------------------------------- K3m (matrix.hip)
// Per-pair Filter + Score of every (pod, node): first failing predicate and
// score matrices [P][ld] (row p, column = local node), and/or the per-pod
// packed keys (max over the shard's feasible nodes).
struct MatrixArgs {
    const void* rec;        // NodeRec [N]
    int64_t N, node_offset;
    const int64_t* now;     // [P]
    const uint8_t* flags;   // [P] or null
    int64_t P;
    int64_t ld;             // row stride of the output matrices (>= N)
    double wsum;
    int32_t noprio;
    int32_t pad;
    int8_t* first_fail;     // [P][ld] or null: -1 = Filter Success, else policy predicate index
    void* score;            // [P][ld] int8 or int64 (score_i64), or null
    int32_t score_i64;
    int32_t pad2;
    long long* keys;        // [P] or null: max-combined (atomicMax, keys must be initialised to -1)
    int8_t pred_orig[kMaxPred];  // device predicate -> policy predicate index
};
hipError_t launch_matrix(int shape, const MatrixArgs& a, hipStream_t st);
// Filter / Score of every node as step functions over [t0, t1) (crane_dyn_node_steps):
// ns[n] breakpoints bp[n * S + j], values ff / sc[n * (S + 1) + j]; S = node_step_slots(shape).
// idx non-null: row n is node idx[n], for n < a.N (crane_dyn_node_steps_subset)
int node_step_slots(int shape);
hipError_t launch_node_steps(int shape, const MatrixArgs& a, int64_t t0, int64_t t1, uint8_t* ns, int64_t* bp,
                             int8_t* ff, int8_t* sc, hipStream_t st, const int64_t* idx = nullptr);

// Scatter update of k nodes' parsed annotations (crane_dyn_update_nodes, update.hip): the
// staged columns go into the shard's SoA and, when the records are current, each changed
// node's NodeRec is recomputed in place (the same rec_metrics / rec_hot_annotation as K1).
struct UpdateArgs {
    DevPolicy pol;
    int64_t N, k;
    const int64_t* idx;     // [k] local node indices, distinct
    const double* sval;     // [M][k] staged values
    const int64_t* sts;     // [M][k] staged timestamps
    const double* shv;      // [k] staged node_hot_value or null (no annotation on these nodes)
    const int64_t* shv_ts;  // [k]
    double* val;            // [M][N] shard SoA
    int64_t* ts;
    double* hv;             // [N] or null (the shard holds no hot-value annotations)
    int64_t* hv_ts;
    void* rec;              // NodeRec [N] or null (records stale: the next node pass rebuilds them)
    // optional: the changed nodes' answer-table rows over [t0, t1) (node_steps.hpp), row j for
    // node idx[j] (ns null: none); ma carries wsum / noprio / pred_orig
    MatrixArgs ma;
    int64_t t0, t1;
    uint8_t* ns;
    int64_t* bp;
    int8_t* ff;
    int8_t* sc;
};
hipError_t launch_update_nodes(int shape, const UpdateArgs& a, hipStream_t st);
// fill [n] int64 with v (hv_ts of a shard that had no hot-value annotations)
hipError_t launch_fill_i64(int64_t* p, int64_t n, int64_t v, hipStream_t st);

// Framework-level selection (select.hip): upstream kube-scheduler's percentageOfNodesToScore
// window with a rotating start, the weighted sum of Dynamic's score and the other score
// plugins' (external), and a lowest-index or seeded tie-break.
struct SelArgs {
    const void* rec;           // NodeRec [N]
    int64_t N, node_offset;
    const int64_t* now;        // [P]
    const uint8_t* flags;      // [P] or null (bit 0: DaemonSet)
    int64_t P;
    double wsum;
    int32_t noprio;
    uint32_t kb;               // tie-hash key of the batch (seed != 0)
    const uint8_t* ext_ok;     // [N] or null: 1 = the other filter plugins pass
    const int64_t* ext_score;  // [N] or null: the other score plugins' weighted sum, in [0, 2^30)
    int64_t w_dyn;             // Dynamic's score weight, in [0, 2^20]
    const int64_t* wstart;     // [P] or null: window start (local node index) per pod
    const int64_t* wlen;       // [P]: window length (nodes in rotated order)
    uint64_t seed;             // 0: lowest index wins ties
    long long* keys;           // [P]: (total << 32) | tie, -1 = no feasible node (initialised to -1)
};
hipError_t launch_select_fth(const SelArgs& a, int shape, int64_t* fth, hipStream_t st);
// form: 0 the LDS rank/select walk when it fits (else / on overflow the streaming kernel), 1 streaming only;
// done: device flag the two forms share
hipError_t launch_select_chain(const SelArgs& a, const int64_t* fth, int64_t K, int64_t start, int64_t* wstart,
                               int64_t* wlen, int64_t* next_start, int32_t* done, int form, hipStream_t st);
hipError_t launch_select_pairs(int shape, const SelArgs& a, hipStream_t st);
hipError_t launch_select_decode(const SelArgs& a, int64_t* chosen, int64_t* total, hipStream_t st);

// Sequential greedy (greedy.hip)
constexpr int64_t kGreedyMaxNodes = 64LL * 64 * 64 * 64;
constexpr size_t kGreedyLdsBytes = 160 * 1024;
struct GreedyArgs {
    int64_t now;       // batch time, ns
    double wsum;
    int32_t noprio;
    int32_t n_win;
    int64_t win_count[kMaxWin];
    int32_t win_inc[kMaxWin];  // a binding stamped now_unix falls in window w
};
// prep = G1 only (base, leaf); run = G2 only (expects G1's outputs); both = G1 + G2
enum { kGreedyPrep = 1, kGreedyRun = 2, kGreedyBoth = 3 };
hipError_t launch_greedy(int shape, const void* rec, int64_t N, uint32_t* cnt, const GreedyArgs& a, int64_t* base,
                         uint8_t* leaf, int64_t P, const uint8_t* flags, int64_t* chosen, hipStream_t st,
                         int what = kGreedyBoth);

// Merge form of the sequential greedy (merge.hip)
struct MergeArgs {
    int32_t n_win;
    int32_t pad;
    int64_t win_count[kMaxWin];  // all > 0 (else the sequential kernel runs)
    int32_t win_inc[kMaxWin];    // a binding stamped now_unix falls in window w
};
// H [2][101] per-level element counts of the F (feasible) and I streams; flag != 0: use the sequential kernel
hipError_t launch_merge_hist(const int64_t* base, const uint8_t* leaf, const uint32_t* cnt, int64_t N,
                             const MergeArgs& a, int64_t capF, int64_t capI, unsigned long long* H, int32_t* flag,
                             hipStream_t st);
int64_t merge_bsum_len(int64_t N, int vlo);
// stream [cap] packed (level << 32 | ~node) keys of stream T (0 = F, 1 = I), levels >= vlo; bs scratch [merge_bsum_len]
hipError_t launch_merge_stream(const int64_t* base, const uint8_t* leaf, const uint32_t* cnt, int64_t N,
                               const MergeArgs& a, int T, int vlo, int64_t cap, unsigned long long* bs,
                               int64_t* stream, hipStream_t st);
// scratch: apos [Pd], q [nI], gi [nI + 1]
hipError_t launch_merge_assign(const int64_t* Fs, int64_t nF, const int64_t* Is, int64_t nI, const uint8_t* flags,
                               int64_t P, int64_t Pd, int32_t* apos, int32_t* q, int64_t* gi, int64_t* chosen,
                               hipStream_t st);

// ---------------------------------------------------------------- K2 (hotcount.hip, kernels.hip)
// LDS-hash K2 (one kernel, global atomics into the bucket matrix): the fallback of any shape.
hipError_t launch_hot_count(const int32_t* bnode, const int64_t* bts, int64_t B, int64_t N, const HotCutoffs& cut,
                            uint32_t* buckets, hipStream_t st);

// Dedupe form (default): one launch (K2x' [+ K3p]); bins = the node pass's workgroups
// (bs nodes), consumed by K1 through K1Args::hx_*.  Region stride kHxRegion entries.
struct HotPart {
    int32_t bb, nbins;  // 2^bb nodes per bin
    int64_t cap;        // region entries (nblk * reg)
    int32_t nblk;       // regions
    int32_t reg;        // bindings per region (the dedupe form: kHxRegion)
    bool ok;
    unsigned long long* trace;  // phase trace or null
};
// The step path's pod preparation (K3p, pods.hpp) for 1024-pod tiles.
constexpr int kTileStat = 8;  // int64 per tile: min/max now per kind, pods per kind, pad
struct PodPrep {
    const int64_t* now;
    const uint8_t* flags;
    int64_t P, ntiles;
    int32_t* perm;
    int64_t* pnow;
    int64_t* tile_mm;
    long long* keys;
    // the batch's time range {tmin, tmax}: every tile folds its pods' range in with one relaxed
    // atomic min / max (no tile waits for another), or null.  batch_next: the other of the two
    // ranges the engine alternates between batches, reset to {INT64_MAX, INT64_MIN} by tile 0 for
    // the next batch (the kernels that read this batch's range precede the next K3p)
    int64_t* batch;
    int64_t* batch_next;
};
constexpr int kHxRegion = 2048;
HotPart hot_dedupe_geometry(int64_t B, int64_t N, int32_t W, int32_t bs);
size_t hot_dedupe_scratch(const HotPart& g);  // uint32 entries: regions + count/offset matrix
hipError_t launch_hot_count_dedupe(const int32_t* bnode, const int64_t* bts, int64_t B, int64_t N,
                                   const HotCutoffs& cut, const HotPart& g, uint32_t* scratch, hipStream_t st,
                                   const PodPrep* pods = nullptr, int threads = 512);
// Delta form (a time-ordered log whose window cutoffs moved since an anchor refresh; at most
// kDeltaMaxWin windows): only the bindings whose window rank differs between the anchor's suffix
// starts a[] and this refresh's p[] (absolute positions, ascending by rank) are read; each changes
// the count of every window rank whose cutoff it crossed by -1 (left) or +1 (entered), in the
// adjustment matrix adj [W][N] per window rank (zero on entry; K1 reads the anchor's buckets +
// adj[b] - adj[b + 1] and zeroes adj).  The changed positions are the merged ranges
// [lo_k, lo_k + len_k), start[] their prefix lengths.  pods: K3p fused (its tiles first), as in
// the dedupe form.
constexpr int kDeltaMaxWin = 2;
struct HotDelta {
    int32_t n_win, n_rng;
    int64_t a[kMaxWin], p[kMaxWin];
    int64_t lo[kMaxWin], start[kMaxWin + 1];
    unsigned long long* trace;  // phase stamps per workgroup (K3p tiles first) or null
};
hipError_t launch_hot_count_delta(const int32_t* bnode, int64_t N, const HotDelta& d, uint32_t* adj, hipStream_t st,
                                  const PodPrep* pods);
// Large form (past the dedupe form's cap): the same region pass with coarse bins of 2^bb
// nodes (Y's LDS histogram [W][2^bb] <= kK2LargeHistBytes), then k2y_bin_hist writes the
// dense window-rank buckets [W][N] (every row of every bin: K1 reads them, nothing to zero).
// scratch: hot_dedupe_scratch(g) words.
constexpr int64_t kK2LargeHistBytes = 128 * 1024;
constexpr int32_t kK2lRegion = 4096;  // large form: bindings per region
HotPart hot_large_geometry(int64_t B, int64_t N, int32_t W);
hipError_t launch_hot_count_large(const int32_t* bnode, const int64_t* bts, int64_t B, int64_t N,
                                  const HotCutoffs& cut, const HotPart& g, uint32_t* scratch, uint32_t* buckets,
                                  int n_cu, hipStream_t st, int threads = 1024);

// ---------------------------------------------------------------- K3 step path (step.hip)
constexpr int kStepSeg = 256;                 // nodes per segment (K3a workgroup)
constexpr int64_t kStepMaxNodes = 1LL << 24;  // packed key keeps 24 bits of node index
// A node whose key changes once inside the batch: key k0 for now < bp, k1 after.
struct alignas(16) Step1 {
    int64_t bp;
    int32_t k0, k1;
};
// A middle piece of a node whose key changes more than once in the batch: the
// key on [s, e) (step_node.hpp).
struct alignas(8) Mid {
    int64_t s, e;
    int32_t key;
    int32_t pad;
};
// Step tables, one region per producer workgroup b (K1: bs = 128/256 nodes,
// K3a: 256): its flat-key maxima flat[b][kind], its record counts cnt[b][L]
// (L = 2 * kind + 0: one-step records, 1: middle pieces), its one-step records
// sorted by step time with their prefix / suffix key maxima
// (step_sort_publish) and its middle pieces.  Producers need no global
// atomics; K3s reads the producer blocks it covers.
struct StepTables {
    int32_t* cnt;    // [nblk][4]
    int32_t* flat;   // [nblk][2], -1 = no flat feasible node
    Step1* single;   // kind T, block b: 2 * bs records at s1_at(T, b), sorted by bp
    int32_t* pm1;    // same indexing: prefix max of k1 (after-step keys) over the sorted records
    int32_t* sm0;    // same indexing: suffix max of k0 (before-step keys)
    Mid* mid;        // kind T, block b: mstride pieces at T * mpad + b * mstride
    int64_t s1pad, mpad;  // per-kind strides
    int32_t bs;      // nodes per producer workgroup
    int32_t nblk;    // producer workgroups
    int32_t mstride; // middle pieces per block region (bs * (breakpoints per node - 1))
    int32_t ntiles;  // pod tiles of the batch (K3p)
    const int64_t* tiles;  // K3p's tile stats (kTileStat per tile)
    // per (pod tile t, block b) at rows[t * nblk + b], or null (K3s searches itself):
    // {uniform key kind 0, kind 1, jl0 | jh0 << 16, jl1 | jh1 << 16}; [jl, jh) = the
    // block's sorted one-step records stepping inside the tile's range of that kind
    int4* rows;
    // with rows, per (tile t, block b) at prow[t * nblk + b]: {pl0 | ph0 << 16, pl1 | ph1 << 16},
    // the block's middle pieces [pl, ph) of that kind overlapping the tile's range (0: none);
    // null: no per-tile ranges (K3s reads every piece of the block, none is ever cut)
    int2* prow;
    unsigned long long* trace;  // K3s phase trace or null
    // K1's one-step staging for blocks with more records of a kind than its LDS holds
    // (or than lds_cap, 0 = always): same indexing as single
    Step1* stage;
    int32_t lds_cap;
    // middle pieces x pod tiles from which a producer cuts a kind's pieces into elementary
    // ones (step_pieces), INT32_MAX = never
    int32_t piece_work;
};
constexpr int64_t kPieceMinTiles = 32;  // pod tiles from which step_pieces runs (engine option step_pieces 0)
constexpr int64_t kStepRowsMax = 1LL << 24;  // tile x block rows (256 MiB); larger batches: K3s searches
__host__ __device__ inline int64_t s1_at(const StepTables& st, int T, int64_t b) {
    return T * st.s1pad + b * 2 * st.bs;
}
struct StepGeometry {
    int64_t nseg, npad, ntiles, ngroups;
    int32_t R;  // K3s workgroups per 1024-pod group (raised until each covers <= kK3sMaxBlk producer blocks)
};
constexpr int kK3sMaxBlk = 256;  // producer blocks per K3s workgroup (one lane each)
int step_breakpoints(int shape);  // in-range expiries per node and kind at most: PR + 2
StepGeometry step_geometry(int64_t P, int64_t N, int32_t nblk, int32_t blk_per_wg = 0);
// The previous step's K3s (launch_step_pairs' arguments) with this step's delta form + K3p in one
// launch (step.hip k3s_delta_pods)
hipError_t launch_k3s_delta_pods(int64_t N_k3s, int64_t node_offset, int64_t P_k3s, long long* keys_k3s,
                                 const StepTables& st, const StepGeometry& g, const int32_t* perm, const int64_t* pnow,
                                 const int64_t* tile_mm, const int32_t* bnode, int64_t N, const HotDelta& d,
                                 uint32_t* adj, const PodPrep& pods, hipStream_t s);
// K3p: perm, pnow [ntiles * 1024], tile_mm [kTileStat * ntiles]; initialises keys[0..P) to -1
hipError_t launch_step_pods(const int64_t* now, const uint8_t* flags, int64_t P, long long* keys, int64_t* batch,
                            int64_t* batch_next,
                            const StepGeometry& g, int32_t* perm, int64_t* pnow, int64_t* tile_mm, hipStream_t s);
// K3a: step tables from NodeRecs in HBM (after K3p)
hipError_t launch_step_nodes(int shape, const void* rec, int64_t N, double wsum, int32_t noprio,
                             const StepTables& st, const StepGeometry& g, const int64_t* tile_mm, hipStream_t s);
// K3s: (pod, stepped node) pairs + flat maxima -> keys (after K3a or K1's STEP form)
hipError_t launch_step_pairs(int shape, int64_t N, int64_t node_offset, int64_t P, long long* keys,
                             const StepTables& st, const StepGeometry& g, const int32_t* perm, const int64_t* pnow,
                             const int64_t* tile_mm, hipStream_t s);
// K1's fused step form: the node pass also builds the step tables of a pod batch
struct K1Step {
    const int64_t* tile_mm;  // K3p's per-tile stats (kTileStat)
    const int64_t* batch;    // K3p's folded {tmin, tmax} of the batch
    int32_t ntiles;
    int32_t noprio;
    double wsum;
    double winv;             // 1 / wsum when |wsum| is a power of two, else 0 (score_at)
    StepTables st;
    void* srec;              // NodeRec [N] scratch (the streamed step pass's stepped nodes past its LDS)
    int32_t tail1;           // the streamed pass's tail on one wave (0: when the grid has >= 4096 blocks)
};

size_t node_rec_bytes(int shape);

// ---------------------------------------------------------------- K1 (kernels.hip)
// K1 node pass arguments.  Hot value source: buckets (K2 counts, consumed:
// zeroed, the value kept in hvc_out) or the dedupe-form entries (hx_*) > hv with
// hv_ts (annotation; hv_ts null: every node stamped hv_ts_counts) > none.
struct K1Args {
    DevPolicy pol;
    int64_t N;
    const double* val;      // [M][N]
    const int64_t* ts;      // [M][N]
    const double* hv;       // [N] or null
    const int64_t* hv_ts;   // [N] or null
    uint32_t* buckets;      // [W][N] K2 window-rank buckets or null
    const uint32_t* bucket_base;  // [W][N] the delta form's anchor buckets, with buckets its per-rank
                                  // adjustments (bucket b = base[b] + adj[b] - adj[b + 1]), or null
    int32_t buckets_keep;   // 1: leave them (the large form rewrites every row), 0: zero what was read
    int64_t hv_ts_counts;   // stamp of binding-log hot values
    void* out;              // NodeRec [N], or null (keys-only step: records not kept)
    uint32_t* cnt_out;      // [W][N] per-window counts (greedy) or null
    double* hvc_out;        // [N] hot values from the buckets, or null
    // dedupe-form K2 output (instead of buckets): for K1 node block b (of nb) and K2
    // region r, hx_CO[r*nb + b] = count | offset << 16 of b's entries at
    // hx_region[r*kHxRegion + offset]
    const uint32_t* hx_region;
    const uint32_t* hx_CO;
    int32_t hx_nblk;
    int32_t threads;        // workgroup size: 256
    unsigned long long* trace;  // phase trace or null
};
// step (optional): also build the K3 step tables of a pod batch (K3a fused).  stream: with step,
// no records written and no dedupe-form K2 entries, the streamed step pass (k1_stream_steps: no
// record in registers, the stepped nodes' records built in LDS)
hipError_t launch_node_pass(int shape, const K1Args& a, hipStream_t st, const K1Step* step = nullptr,
                            int stream = 0);
// the streamed step pass (k1stream.hip) for the record shape PD x PR
hipError_t launch_stream_steps(int pd, int pr, const K1Args& a, const K1Step& sa, hipStream_t st);

}  // namespace crane
