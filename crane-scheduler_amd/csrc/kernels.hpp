// kernels.hpp — host-side launch interface of kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dyn_types.hpp"

namespace crane {

// NodeRec template instances (max predicates x max priorities).
enum { kShape4x6 = 0, kShape8x8 = 1, kShape16x16 = 2 };

struct HotCutoffs {
    int32_t n_win;
    int32_t pad;
    int64_t sorted[kMaxWin];  // ascending now_unix - int64(timeRange.Seconds())
};

struct MatrixOut {
    int8_t* first_fail;  // [P][N] or null
    int64_t* score;      // [P][N] or null
    int8_t pred_orig[kMaxPred];  // device predicate -> policy predicate index
};

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

// Bin-partitioned K2 (hotcount.hip)
constexpr int kMaxBins = 4096;
struct HotBins {
    int32_t bb;       // log2(nodes per bin)
    int32_t nbins, nchunks, splits;
    int64_t chunk;    // bindings per chunk workgroup
    bool ok;          // per-bin histogram fits LDS
};
HotBins hot_bins_geometry(int64_t B, int64_t N, int32_t W);
// scratch: chunk_cnt [nbins * nchunks], bin_tot [nbins], sorted [B]
hipError_t launch_hot_count_binned(const int32_t* bnode, const int64_t* bts, int64_t B, int64_t N,
                                   const HotCutoffs& cut, uint32_t* buckets, const HotBins& g, uint32_t* chunk_cnt,
                                   uint32_t* bin_tot, uint32_t* sorted, hipStream_t st);

// Two-kernel partitioned K2 (hotcount.hip): each partition workgroup writes
// its in-window bindings bin-contiguously into its own region and publishes
// per-bin (count, offset); no global atomics besides the final bucket adds.
struct HotPart {
    int32_t bb, nbins;  // 2^bb nodes per bin
    int64_t cap;        // region entries (nblk * 2048)
    int32_t nblk;       // partition workgroups
    bool ok;
};
HotPart hot_part_geometry(int64_t B, int64_t N, int32_t W);
size_t hot_part_scratch(const HotPart& g);  // uint32 entries: region + C + O
// Adds into buckets[W][N], which must be zero on entry.  Scratch needs no initialisation.
// The step path's pod preparation (K3p) for 1024-pod tiles, as it rides in K2x's launch.
struct PodPrep {
    const int64_t* now;
    const uint8_t* flags;
    int64_t P, ntiles;
    int32_t* perm;
    int64_t* pnow;
    int64_t* tile_mm;
    long long* keys;
};
// Dedupe form: one launch (K2x' [+ K3p]); bins = the node pass's workgroups (bs
// nodes), consumed by K1 through K1Args::hx_*.  Region stride kHxRegion entries.
constexpr int kHxRegion = 2048;
HotPart hot_dedupe_geometry(int64_t B, int64_t N, int32_t W, int32_t bs);
hipError_t launch_hot_count_dedupe(const int32_t* bnode, const int64_t* bts, int64_t B, int64_t N,
                                   const HotCutoffs& cut, const HotPart& g, uint32_t* scratch, hipStream_t st,
                                   const PodPrep* pods = nullptr);
// pods (optional, with which & 1): K3p's tiles run as extra workgroups of the K2x launch
hipError_t launch_hot_count_part(const int32_t* bnode, const int64_t* bts, int64_t B, int64_t N,
                                 const HotCutoffs& cut, uint32_t* buckets, const HotPart& g, uint32_t* scratch,
                                 hipStream_t st, int which = 3, const PodPrep* pods = nullptr);  // 1: k2x, 2: k2y

// K3 step path (step.hip): per-batch node step tables + pair eval.
constexpr int kStepSeg = 256;                 // nodes per segment (K3a workgroup)
constexpr int64_t kStepMaxNodes = 1LL << 24;  // packed key keeps 24 bits of node index
// A node whose key changes once inside the batch: key k0 for now < bp, k1 after.
struct alignas(16) Step1 {
    int64_t bp;
    int32_t k0, k1;
};
// A node whose key changes more than once: cnt ascending expiries in
// (tmin, tmax], padded with INT64_MAX; key[j] holds for bp[j-1] <= now < bp[j].
template <int NB>
struct alignas(16) VRec {  // 16-byte multiple: K3s stages records with 16-byte copies
    int64_t bp[NB];
    int32_t key[NB + 1];
    int32_t cnt;
};
// Step tables, one region per producer workgroup b (K1: bs = 128 nodes, K3a:
// 256): its flat-key maxima flat[b][kind], its record counts cnt[b][L]
// (L = 2 * kind + 0: Step1, 1: VRec) and its records at b * bs + slot of each
// list.  Producers need no global atomics; K3s scans the counts of the
// producer blocks it covers.
struct StepTables {
    int32_t* cnt;    // [nblk][4]
    int32_t* flat;   // [nblk][2], -1 = no flat feasible node
    Step1* single;   // [2][npad] per pod kind
    void* multi;     // [2][npad] VRec<NB>
    int64_t npad;    // per-kind stride >= nblk * bs
    int32_t bs;      // nodes per producer workgroup
    int32_t nblk;    // producer workgroups
};
struct StepGeometry {
    int64_t nseg, npad, ntiles, ngroups;
    int32_t R;  // K3s workgroups per 256-pod group (R is raised until each covers <= kK3sMaxBlk producer blocks)
};
constexpr int kK3sMaxBlk = 1024;
size_t step_vrec_bytes(int shape);
StepGeometry step_geometry(int64_t P, int64_t N, int32_t nblk);
int k1_threads();  // K1 workgroup size (256, or 128 with CRANE_K1_THREADS=128)
// K3p: perm, pnow [ntiles * 1024], tile_mm [2 * ntiles]; initialises keys[0..P) to -1 and the step header
hipError_t launch_step_pods(const int64_t* now, const uint8_t* flags, int64_t P, long long* keys,
                            const StepTables& st, const StepGeometry& g, int32_t* perm, int64_t* pnow,
                            int64_t* tile_mm, hipStream_t s);
// K3a: step tables from NodeRecs in HBM (after K3p)
hipError_t launch_step_nodes(int shape, const void* rec, int64_t N, double wsum, int32_t noprio,
                             const StepTables& st, const StepGeometry& g, const int64_t* tile_mm, hipStream_t s);
// K3s: (pod, stepped node) pairs + flat maxima -> keys (after K3a or K1's STEP form)
hipError_t launch_step_pairs(int shape, int64_t N, int64_t node_offset, int64_t P, long long* keys,
                             const StepTables& st, const StepGeometry& g, const int32_t* perm, const int64_t* pnow,
                             hipStream_t s);
// K1's fused step form: the node pass also builds the step tables of a pod batch
struct K1Step {
    const int64_t* tile_mm;  // K3p's per-tile time range
    int32_t ntiles;
    int32_t noprio;
    double wsum;
    StepTables st;
};
int k3_variant();

size_t node_rec_bytes(int shape);
int64_t eval_chunk_nodes(int64_t P, int64_t N);

hipError_t launch_hot_count(const int32_t* bnode, const int64_t* bts, int64_t B, int64_t N, const HotCutoffs& cut,
                            uint32_t* buckets, hipStream_t st);
// K1 zeroes the buckets it consumes (so the next K2 needs no memset); with
// cnt_out it also stores the per-window counts [W][N].
// K1 node pass arguments.  Hot value source: buckets (K2 counts, consumed:
// zeroed, the value kept in hvc_out) > hv with hv_ts (annotation; hv_ts null:
// every node stamped hv_ts_counts) > none.
struct K1Args {
    DevPolicy pol;
    int64_t N;
    const double* val;      // [M][N]
    const int64_t* ts;      // [M][N]
    const double* hv;       // [N] or null
    const int64_t* hv_ts;   // [N] or null
    uint32_t* buckets;      // [W][N] K2 window-rank buckets or null
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
    int32_t threads;        // workgroup size (0: k1_threads())
};
// step (optional): also build the K3 step tables of a pod batch (K3a fused).
hipError_t launch_node_pass(int shape, const K1Args& a, hipStream_t st, const K1Step* step = nullptr);
// thr: device table of kQMax + 1 quotient thresholds (null = divide); inv_w = RN(1/wsum)
hipError_t launch_eval(int shape, const void* rec, int64_t N, int64_t node_offset, const int64_t* now,
                       const uint8_t* flags, int64_t P, double wsum, int32_t noprio, long long* keys,
                       const MatrixOut& mo, double inv_w, const double* thr, hipStream_t st);

}  // namespace crane
