// kernels.hip — CDNA4 (gfx950) kernels of the Dynamic plugin hot path.
//
//   K2 hot_count : binding records -> per-node window counts (LDS-aggregated;
//                  the fallback form, see hotcount.hip for the default)
//   K1 node_pass : parsed annotation SoA (+ K2 counts) -> NodeRec per node
//
// Numerics follow /root/reference/pkg/plugins/dynamic/stats.go and plugins.go
// bit for bit: fp64 in the reference's operation order, no FMA contraction
// (built with -ffp-contract=off), Go's float64->int conversion and wrapping
// int64 arithmetic.
#include <hip/hip_runtime.h>

#include "dyn_types.hpp"
#include "kernels.hpp"
#include "node_rec.hpp"
#include "step_node.hpp"

namespace crane {

thread_local KernelTimer* tl_ktimer = nullptr;

// ---------------------------------------------------------------- K2
// Each binding b falls into the windows whose cutoff (now_unix -
// int64(timeRange.Seconds()), binding.go:85) is < ts_b.  With cutoffs sorted
// ascending that set is a prefix 0..j-1, so one count per binding goes to
// bucket j-1 and window w's count is the suffix sum of buckets from its rank
// (done in K1).  A workgroup aggregates its slice of bindings in an LDS hash
// table keyed by node (open addressing, CAS insert) before touching global
// memory, so Zipf-hot nodes cost one global atomic per workgroup instead of
// one per binding.
constexpr int kHashSlots = 8192;  // per workgroup: load factor <= 1/2 for its 4096 bindings
constexpr int kMaxProbe = 32;
constexpr int kK2Threads = 256;
constexpr int kK2PerThread = 16;

__global__ __launch_bounds__(kK2Threads) void k2_hot_count(const int32_t* __restrict__ bnode,
                                                            const int64_t* __restrict__ bts, int64_t B,
                                                            int64_t N, HotCutoffs cut, uint32_t* __restrict__ buckets) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int W = cut.n_win;
    const bool lds = W <= kLdsWin;
    int32_t* hkey = reinterpret_cast<int32_t*>(smem);
    uint32_t* hcnt = reinterpret_cast<uint32_t*>(smem + sizeof(int32_t) * kHashSlots);  // [slot][W]
    if (lds) {
        for (int i = threadIdx.x; i < kHashSlots; i += kK2Threads) hkey[i] = -1;
        for (int i = threadIdx.x; i < kHashSlots * W; i += kK2Threads) hcnt[i] = 0;
        __syncthreads();
    }
    const int64_t per_block = (int64_t)kK2Threads * kK2PerThread;
    const int64_t b0 = (int64_t)blockIdx.x * per_block;
    const int64_t b1 = min(B, b0 + per_block);
    for (int64_t b = b0 + threadIdx.x; b < b1; b += kK2Threads) {
        const int32_t nd = bnode[b];
        const int64_t ts = bts[b];
        if (nd < 0 || (int64_t)nd >= N) continue;  // binding.go:88 — matches no node of this shard
        int j = 0;
#pragma unroll
        for (int w = 0; w < kMaxWin; ++w)
            if (w < W) j += ts > cut.sorted[w] ? 1 : 0;
        if (j == 0) continue;
        const int bucket = j - 1;
        bool done = false;
        if (lds) {
            uint32_t h = ((uint32_t)nd * 2654435761u) >> (32 - 13);
            for (int p = 0; p < kMaxProbe && !done; ++p) {
                const int32_t k = __hip_atomic_load(&hkey[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (k == nd) {
                    atomicAdd(&hcnt[h * W + bucket], 1u);
                    done = true;
                } else if (k == -1) {
                    const int32_t old = atomicCAS(&hkey[h], -1, nd);
                    if (old == -1 || old == nd) {
                        atomicAdd(&hcnt[h * W + bucket], 1u);
                        done = true;
                    }
                }
                h = (h + 1) & (kHashSlots - 1);
            }
        }
        if (!done) atomicAdd(&buckets[(int64_t)bucket * N + nd], 1u);
    }
    if (!lds) return;
    __syncthreads();
    for (int sl = threadIdx.x; sl < kHashSlots; sl += kK2Threads) {
        const int32_t nd = hkey[sl];
        if (nd < 0) continue;
        for (int w = 0; w < W; ++w) {
            const uint32_t c = hcnt[sl * W + w];
            if (c) atomicAdd(&buckets[(int64_t)w * N + nd], c);
        }
    }
}

// ---------------------------------------------------------------- K1
// Hot-value part of the record from the node's K2 window-rank buckets bc[r]
// (annotateNodeHotValue, node.go:113-121: value += count / p.Count, Go int division;
// window w counts the bindings of buckets >= its cutoff rank): one running suffix sum.
// cnt_out / hvc_out (null: not kept): the per-window counts and the value.
template <int PD, int PR>
__device__ __forceinline__ void rec_hot_counts(const DevPolicy& pol, const uint32_t (&bc)[kMaxWin], int64_t N, int64_t n,
                                               uint32_t* __restrict__ cnt_out, double* __restrict__ hvc_out,
                                               int64_t hv_ts_counts, NodeRec<PD, PR>& r) {
    int64_t v = 0;
    uint64_t suf = 0;
#pragma unroll
    for (int k = kMaxWin - 1; k >= 0; --k) {
        if (k >= pol.n_win) continue;
        suf += bc[k];
        const int w = pol.win_of_rank[k];
        if (cnt_out) cnt_out[(int64_t)w * N + n] = (uint32_t)suf;
        // Go int division (truncates toward 0): exact multiply-high division when the
        // count fits 32 bits and hotValue.count is in [1, 2^32)
        if (pol.win_div_m[k] != 0 && suf <= 0xFFFFFFFFull)
            v += (int64_t)div_magic((uint32_t)suf, pol.win_div_m[k], pol.win_div_sh[k]);
        else
            v += (int64_t)suf / pol.win_count[w];
    }
    // the plugin re-reads it via ParseFloat (exact) and rejects negatives (stats.go:71-73)
    const double h = (double)v;
    if (hvc_out) hvc_out[n] = h;  // kept for node passes after the buckets are consumed
    r.pen = go_int(h * 10.0);
    r.e_hv = v >= 0 ? sat_add(hv_ts_counts, kHotActiveNs) : kTsInvalid;
}

// One thread per node.  Reads the parsed SoA (and K2 buckets), writes the
// node's NodeRec into LDS, then the workgroup streams its records out with
// 16-byte coalesced stores.
// block size: 256 (the dedupe-form K2 bins nodes by it) or 128
// STEP: also build the K3 step tables of the pod batch (K3a fused, step.hip):
// the record is classified straight from registers.
// keys-only step: LDS staging for this many stepped records per workgroup (the sorted
// one-step records reuse it after the emit); a node past it builds its own records.
// One-step records: LDS staging for kK1S1Cap per kind (a block with more goes through
// st.stage).  With the buffers below a workgroup takes ~30 KB of LDS, five per CU.
constexpr int kK1RecCap = 112;
constexpr int kK1S1Cap = 256;

// SPLIT (with STEP; large N): classify and count only — the stepped records and queue items
// go to HBM for k3a_emit, so no LDS staging and no epilogue (short-lived workgroups, more of
// them per CU, the SoA stream is what bounds the launch).
// WPE: waves per SIMD the 4x6 shape's registers are budgeted for (5: with the fused form's ~30 KB
// of LDS, 5 workgroups per CU); HX 0: the dedupe-form K2 entries only when given, 1: never (the
// buckets / annotation forms, fewer registers).  (The split count pass's variants are engine
// option k1_count_form.)
template <int PD, int PR, int kK1Threads, bool STEP, bool SPLIT = false, int WPE = 5, int HX = 0>
__global__ __launch_bounds__(kK1Threads) __attribute__((amdgpu_waves_per_eu(PD * PR <= 24 ? WPE : 1)))
void k1_node_pass(K1Args a, K1Step step) {
    const DevPolicy& pol = a.pol;
    const int64_t N = a.N;
    const double* __restrict__ val = a.val;
    const int64_t* __restrict__ ts = a.ts;
    const double* __restrict__ hv = a.hv;
    const int64_t* __restrict__ hv_ts = a.hv_ts;
    uint32_t* __restrict__ buckets = a.buckets;
    const int64_t hv_ts_counts = a.hv_ts_counts;
    NodeRec<PD, PR>* __restrict__ out = static_cast<NodeRec<PD, PR>*>(a.out);
    uint32_t* __restrict__ cnt_out = a.cnt_out;
    using Rec = NodeRec<PD, PR>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    Rec* lrec = reinterpret_cast<Rec*>(smem);
    const int64_t blk = xcd_block(blockIdx.x, gridDim.x);  // this workgroup's block of nodes
    CRANE_TSTAMP(a.trace, blockIdx.x, 0);
    const int64_t first = blk * kK1Threads;
    const int64_t n = first + threadIdx.x;
    __shared__ StepShared ssh;
    int64_t tmin = 0, tmax = 0;
    __shared__ int32_t nq;                      // stepped (node, kind) items queued for the emit
    __shared__ uint32_t q[STEP && !SPLIT ? 2 * kK1Threads : 1];
    __shared__ int32_t qm[STEP && !SPLIT ? 2 * kK1Threads : 1];  // first middle-piece slot of queued items
    // one-step records per kind (2 per node at most, CAP staged in LDS): staging; sorted
    // copy over the records' LDS once the emit has read them (or past them when the
    // records are written out) (one buffer with the dedupe-form K2 buckets hxh below:
    // those are read before the step epilogue's first barrier, the staging is written after it)
    constexpr int CAP = kK1S1Cap < 2 * kK1Threads ? kK1S1Cap : 2 * kK1Threads;
    constexpr int kHxWords = kMaxWin * kK1Threads;
    constexpr int kUnion = (STEP && !SPLIT ? 2 * CAP * (int)sizeof(Step1) : 0) > 4 * kHxWords
                               ? 2 * CAP * (int)sizeof(Step1)
                               : 4 * kHxWords;
    __shared__ __attribute__((aligned(16))) unsigned char ush[kUnion];
    Step1* s1l = reinterpret_cast<Step1*>(ush);
    Step1* s1s = reinterpret_cast<Step1*>(smem + (out ? sizeof(Rec) * kK1Threads : 0));
    if (STEP && threadIdx.x < 4) ssh.lc[threadIdx.x >> 1][threadIdx.x & 1] = 0;
    __shared__ int32_t nrec;  // keys-only step: stepped records staged
    if (STEP && threadIdx.x == 0) nq = nrec = 0;
    auto hxh = reinterpret_cast<uint32_t(*)[kK1Threads]>(ush);  // dedupe-form K2: this block's window-rank buckets
    const bool hx = HX == 0 && a.hx_region != nullptr;
    StepSlots so;
    Rec r;
    int64_t pt[PD], qt[PR];
    double pv[PD], qv[PR];
    uint32_t bc[kMaxWin];
    double hvl = 0.0;
    int64_t hvt = kTsInvalid;
    // dedupe-form K2: the count/offset words of this block's first source
    // regions go out before the SoA loads, so the dependent entry loads below
    // wait on them, not on the whole SoA batch
    constexpr int kHxPer = 3, kHxFirst = 4, kHxRun = 8;
    uint32_t co0[kHxPer];
    // Every load is unconditional, with a clamped index (lanes past N re-read node N-1, rows
    // past npd/npr read row 0; both ignored): a load inside a branch makes the compiler wait
    // for all loads at the join (s_waitcnt vmcnt(0)), which serialised the dedupe-form chain
    // below behind the whole SoA stream.
    const int lo = (int)min((int64_t)threadIdx.x, N - 1 - first);  // lane offset, clamped
    if (hx) {
#pragma unroll
        for (int u = 0; u < kHxPer; ++u)  // (masked where used: a use here would wait for them)
            co0[u] = a.hx_CO[(int64_t)min(u * kK1Threads + (int)threadIdx.x, a.hx_nblk - 1) * gridDim.x + blk];
        for (int b = 0; b < kMaxWin; ++b) hxh[b][threadIdx.x] = 0;
    }
#pragma unroll
    for (int k = 0; k < PD; ++k) {
        pt[k] = kTsInvalid;
        pv[k] = 0.0;
    }
#pragma unroll
    for (int k = 0; k < PR; ++k) {
        qt[k] = kTsInvalid;
        qv[k] = 0.0;
    }
    if (pol.n_slots > 0) {  // (val/ts are null without metrics; uniform branch)
#pragma unroll
        for (int k = 0; k < PD; ++k) {
            const int64_t row = k < pol.npd ? pol.pred_slot[k] : 0;
            // uniform row base + lane offset (the SGPR-base load form)
            const int64_t* __restrict__ tr = ts + (row * N + first);
            const double* __restrict__ vr = val + (row * N + first);
            pt[k] = tr[lo];
            pv[k] = vr[lo];
        }
#pragma unroll
        for (int k = 0; k < PR; ++k) {
            const int64_t row = k < pol.npr ? pol.prio_slot[k] : 0;
            const int64_t* __restrict__ tr = ts + (row * N + first);
            const double* __restrict__ vr = val + (row * N + first);
            qt[k] = tr[lo];
            qv[k] = vr[lo];
        }
    }
    if (buckets) {
#pragma unroll
        for (int b = 0; b < kMaxWin; ++b)
            bc[b] = b < pol.n_win ? (buckets + first)[(int64_t)b * N + lo] : 0u;
    }
    if (!buckets && !hx && hv) {
        hvl = hv[first + lo];
        hvt = hv_ts ? hv_ts[first + lo] : hv_ts_counts;  // null: the binding-log value of an earlier pass
    }
    if (hx) {
        // this block's (node, bucket, count) entries from every K2 source region
        // (dedupe form): C/O of up to kHxPer regions per lane, then their first
        // kHxFirst entries, all loads in flight together; longer runs loop
        for (int i0 = 0; i0 < a.hx_nblk; i0 += kK1Threads * kHxPer) {
            uint32_t c[kHxPer], o[kHxPer];
#pragma unroll
            for (int u = 0; u < kHxPer; ++u) {
                const int i = i0 + u * kK1Threads + threadIdx.x;
                const uint32_t co = i0 == 0 ? co0[u] : a.hx_CO[(int64_t)min(i, a.hx_nblk - 1) * gridDim.x + blk];
                c[u] = i < a.hx_nblk ? co & 0xFFFF : 0u;
                o[u] = co >> 16;
            }
            // lanes past a run's end load entry 0 of the region array (one shared line)
            uint32_t v[kHxPer][kHxFirst];
#pragma unroll
            for (int u = 0; u < kHxPer; ++u) {
                const int64_t e0 = (int64_t)(i0 + u * kK1Threads + threadIdx.x) * kHxRegion + o[u];
#pragma unroll
                for (int k = 0; k < kHxFirst; ++k) v[u][k] = a.hx_region[(uint32_t)k < c[u] ? e0 + k : 0];
            }
            if (i0 == 0) __syncthreads();  // hxh zeroed by every thread (uniform trip count)
#pragma unroll
            for (int u = 0; u < kHxPer; ++u) {
#pragma unroll
                for (int k = 0; k < kHxFirst; ++k)
                    if ((uint32_t)k < c[u]) atomicAdd(&hxh[(v[u][k] >> 16) & 7][v[u][k] & 0xFFFF], v[u][k] >> 19);
                // long runs (the Zipf-hot blocks: ~100 entries per region) in chunks of
                // kHxRun independent loads, not one load latency per entry
                const uint32_t* src = a.hx_region + (int64_t)(i0 + u * kK1Threads + threadIdx.x) * kHxRegion + o[u];
                for (uint32_t k0 = kHxFirst; k0 < c[u]; k0 += kHxRun) {
                    uint32_t w[kHxRun];
#pragma unroll
                    for (int j = 0; j < kHxRun; ++j) w[j] = src[k0 + j < c[u] ? k0 + j : 0];
#pragma unroll
                    for (int j = 0; j < kHxRun; ++j)
                        if (k0 + j < c[u]) atomicAdd(&hxh[(w[j] >> 16) & 7][w[j] & 0xFFFF], w[j] >> 19);
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int b = 0; b < kMaxWin; ++b) bc[b] = b < pol.n_win ? hxh[b][threadIdx.x] : 0u;
    }
    CRANE_TSTAMP(a.trace, blockIdx.x, 1);
    // the batch time range partials: issued after the SoA loads, reduced after the compute
    int64_t tpre = 0;  // this thread's first tile-row bound (step_tile_rows)
    if (STEP) {
        tmin = step.batch[0];  // K3p folded the batch range
        tmax = step.batch[1];
        if (step.st.rows) tile_prefetch(step.st, &tpre);
    }
    if (n < N) {
        rec_metrics<PD, PR>(pol, pt, pv, qt, qv, r);
        if (buckets || hx) {
            if (buckets && !a.buckets_keep) {
#pragma unroll
                for (int b = 0; b < kMaxWin; ++b)  // consumed: leaves the buckets zeroed for the next K2
                    if (b < pol.n_win) (buckets + first)[(int64_t)b * N + threadIdx.x] = 0;
            }
            rec_hot_counts<PD, PR>(pol, bc, N, n, cnt_out, a.hvc_out, hv_ts_counts, r);
        } else if (hv) {
            rec_hot_annotation<PD, PR>(hvl, hvt, r);
        } else {
            r.pen = 0;
            r.e_hv = kTsInvalid;
        }
        rec_fail<PD, PR>(r);
        if (out) lrec[threadIdx.x] = r;
    }
    CRANE_TSTAMP(a.trace, blockIdx.x, 2);
    if (STEP) {
        if (!hx) __syncthreads();  // orders the lc / nq / nrec resets before the counting below
                                   // (the dedupe form's barriers above already do)
        // stepped (a few %): keys-only, the records are compacted into kK1RecCap LDS slots
        // (a node past them builds its own); the (node, kind) items go to the queue
        bool self_emit;
        if constexpr (SPLIT) {
            // every stepped node's record to HBM, every item queued in HBM; k3a_emit does the rest
            const int64_t qo = blk * 2 * kK1Threads;
            step_count_queue<PD, PR, kK1RecCap>(r, n < N, n, tmin, tmax, step.wsum, step.winv, step.noprio, true,
                                                ssh, &nrec, &nq, step.qg + qo, step.qmg + qo, lrec, so, self_emit);
            if (so.slot0 >= 0 || so.slot1 >= 0) static_cast<Rec*>(step.srec)[n] = r;
            step_publish<kK1Threads>(so, ssh, step.st, blk);  // (its barrier: nq is final)
            if (threadIdx.x == 0) step.nqg[blk] = nq;
            CRANE_TSTAMP(a.trace, blockIdx.x, 3);
            CRANE_TSTAMP(a.trace, blockIdx.x, 5);
            CRANE_TSTAMP(a.trace, blockIdx.x, 6);
            CRANE_TSTAMP(a.trace, blockIdx.x, 4);
            return;
        }
        step_count_queue<PD, PR, kK1RecCap>(r, n < N, n, tmin, tmax, step.wsum, step.winv, step.noprio,
                                            out != nullptr, ssh, &nrec, &nq, q, qm, lrec, so, self_emit);
        step_publish<kK1Threads>(so, ssh, step.st, blk);  // (its barrier also orders lrec and the queue)
        CRANE_TSTAMP(a.trace, blockIdx.x, 3);
        // one-step records staged in LDS, or (more of a kind than it holds) in st.stage
        const bool g1 = max(ssh.lc[0][0], ssh.lc[1][0]) > min(CAP, step.st.lds_cap);
        Step1* s1b = g1 ? step.st.stage + blk * 2 * step.st.bs : s1l;
        const int64_t kst = g1 ? step.st.s1pad : (int64_t)CAP;
        // (a node past the staging emits first: its record then dies before the queue's)
        if (self_emit)
            step_emit<PD, PR>(r, n, tmin, tmax, step.wsum, step.noprio, so, step.st, blk, s1b, kst, step.winv);
        // the queued items are built densely by the first lanes of the workgroup
        for (int w = threadIdx.x; w < nq; w += kK1Threads) {
            const uint32_t it = q[w];
            if (it == ~0u) continue;  // a self-emitted node's
            const int o = (int)(it & 0xFFF);
            step_emit_one<PD, PR>(lrec[it >> 24], first + o, (int)((it >> 12) & 1), (int32_t)((it >> 14) & 0x3FF),
                                  qm[w], ((it >> 13) & 1) != 0, tmin, tmax, step.wsum, step.noprio, step.st, blk,
                                  s1b, kst, step.winv);
        }
        __syncthreads();
        CRANE_TSTAMP(a.trace, blockIdx.x, 5);
        if (g1) step_sort_publish_global<kK1Threads>(ssh, step.st, blk);
        else step_sort_publish<kK1Threads, CAP>(s1l, s1s, ssh, step.st, blk);
        CRANE_TSTAMP(a.trace, blockIdx.x, 6);
        if (step.st.rows) {
            // keys-only: the middle pieces' scratch is the staged records' LDS past the sorted
            // one-step copy (dead after the emit); with the records kept there is none
            constexpr int kS1 = 2 * (int)sizeof(Step1) * CAP;
            constexpr int kDyn = (int)sizeof(Rec) * (kK1Threads < kK1RecCap ? kK1Threads : kK1RecCap);
            constexpr int kPc = kDyn > kS1 ? ((kDyn - kS1) / PieceScr::bytes_per_piece) & ~3 : 0;
            const PieceScr ps{smem + kS1, out ? 0 : (kPc < 128 ? kPc : 128)};
            step_pieces<kK1Threads>(ssh, step.st, blk, ps);
            if (g1) step_tile_rows<kK1Threads, CAP, true>(s1l, s1s, ssh, step.st, blk, &tpre, ps);
            else step_tile_rows<kK1Threads, CAP, false>(s1l, s1s, ssh, step.st, blk, &tpre, ps);
        }
    } else {
        __syncthreads();
    }
    CRANE_TSTAMP(a.trace, blockIdx.x, 4);
    if (!out) return;  // keys-only step: the records are rebuilt when a matrix/greedy pass needs them
    const int64_t nvalid = min((int64_t)kK1Threads, N - first);
    const int64_t nvec = nvalid * (int64_t)sizeof(Rec) / 16;
    const uint4* src = reinterpret_cast<const uint4*>(smem);
    uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<unsigned char*>(out) + first * (int64_t)sizeof(Rec));
    for (int64_t i = threadIdx.x; i < nvec; i += kK1Threads) dst[i] = src[i];
}

// ---------------------------------------------------------------- K1 count pass, prefetching (split form)
// The split count pass as a persistent grid (the resident workgroups: 5 per CU at the default
// policy, bound by the LDS staging): workgroup g takes the blocks g, g + grid, ... (their
// xcd_block, so each XCD keeps its contiguous run and k3a_emit finds the records in its L2).
// A block's rows — the SoA's value and stamp rows of every metric slot, the K2 bucket rows or
// the hot-value annotation rows — are staged in LDS by LDS-DMA (global_load_lds_dwordx4: 1 KiB
// per wave-instruction, no VGPR destination); each thread copies its node's values to registers,
// then the NEXT block's DMA is issued and stays in flight through this block's record,
// classification and publish.  The fused and the default count pass load a block and then work
// on it, so a workgroup's loads are in flight only a quarter of its life (phase traces,
// DESIGN 4.2); here they are in flight all the time.  All LDS is one dynamic array (a second
// __shared__ object can make hipcc wait vmcnt(0) before an LDS access) and the barriers are raw
// s_barrier after lgkmcnt(0): __syncthreads' fence would wait vmcnt(0) and drain the DMA.
struct PfGeom {
    int32_t ns;      // metric slots staged (pol.n_slots)
    int32_t hvrow;   // chunk of the hot-value annotation rows (hv: 2 chunks, hv_ts: 2) or -1
    int32_t bkrow;   // chunk of the first K2 bucket row (one chunk each) or -1
    int32_t nchunk;  // 1 KiB chunks staged per block
    int32_t grid;    // workgroups (a multiple of 8)
};
constexpr int kPfChunk = 1024;
typedef __attribute__((address_space(3))) void* lds_void_t;
typedef __attribute__((address_space(1))) void* glb_void_t;

// Workgroup barriers of the prefetching pass, in asm with a memory clobber: the builtin s_barrier
// does not order memory accesses (hipcc moved reads of the staging past it, after the next DMA),
// and __syncthreads' fence waits vmcnt(0).  pf_barrier: this wave's LDS accesses done;
// pf_barrier_dma: also its LDS-DMA and stores.
__device__ __forceinline__ void pf_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void pf_barrier_dma() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Issue the LDS-DMA of block blk's rows into stage: chunk c (1 KiB) by wave c % 4.  8-byte rows
// take two chunks per 256 nodes (2 nodes per lane), 4-byte bucket rows one (4 per lane); a lane
// wholly past N reads the row's start instead (its bytes are never used), the one straddling N
// reads up to 12 B past the row (the buffers carry 64 B of slack, engine.hip DevBuf).
__device__ __forceinline__ void pf_issue(const K1Args& a, const PfGeom& pg, int64_t blk, unsigned char* stage) {
    const int64_t N = a.N, first = blk * 256;
    const int lane = threadIdx.x & 63;
    for (int c = threadIdx.x >> 6; c < pg.nchunk; c += 4) {
        const unsigned char* src;
        if (pg.bkrow >= 0 && c >= pg.bkrow) {
            const int64_t e = first + 4 * lane;
            src = reinterpret_cast<const unsigned char*>(a.buckets + (int64_t)(c - pg.bkrow) * N + (e < N ? e : 0));
        } else {
            const int64_t e0 = first + 128 * (c & 1) + 2 * lane;
            const int64_t e = e0 < N ? e0 : 0;
            const int r = c >> 1;  // 8-byte row: val slots, ts slots, then hv, hv_ts
            if (r < pg.ns) src = reinterpret_cast<const unsigned char*>(a.val + (int64_t)r * N + e);
            else if (r < 2 * pg.ns) src = reinterpret_cast<const unsigned char*>(a.ts + (int64_t)(r - pg.ns) * N + e);
            else if (r == 2 * pg.ns) src = reinterpret_cast<const unsigned char*>(a.hv + e);
            else src = reinterpret_cast<const unsigned char*>(a.hv_ts + e);
        }
        __builtin_amdgcn_global_load_lds((glb_void_t)src, (lds_void_t)(stage + c * kPfChunk), 16, 0, 0);
    }
}

// LDS traffic of the work between two blocks (the wave totals exchanged for the slot
// assignment and the flat maxima) in inline asm: hipcc waits vmcnt(0) before every LDS access
// it sees while an LDS-DMA is in flight (it cannot tell the targets apart), which would drain the
// next block's prefetch; the asm carries its own lgkmcnt waits.
__device__ __forceinline__ uint32_t lds_off(const void* p) {
    return (uint32_t)(size_t)(const __attribute__((address_space(3))) void*)p;
}
// (addr uniform: an SGPR moved into a VGPR here, so no address VGPR lives across the loop)
__device__ __forceinline__ void asm_ds_write_b32(uint32_t addr, uint32_t v) {
    uint32_t t;
    asm volatile("v_mov_b32 %0, %1\n\tds_write_b32 %0, %2" : "=&v"(t) : "s"(addr), "v"(v) : "memory");
}
__device__ __forceinline__ uint4 asm_ds_read_b128(uint32_t addr) {
    uint4 v;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    return v;
}

template <int PD, int PR, int NCH>
// 4 waves per SIMD (128 VGPRs): at 5 the loop spills ~100 VGPRs, and every reload's vmcnt wait
// would drain the prefetch
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PD * PR <= 24 ? 4 : 1)))
void k1_count_pf(K1Args a, K1Step step, PfGeom pg) {
    using Rec = NodeRec<PD, PR>;
    constexpr int BS = 256;
    __shared__ __attribute__((aligned(16))) unsigned char stage[NCH * kPfChunk];
    // per wave: one-step records | middle pieces << 16 of kind 0 and 1, queue items, flat maxima
    __shared__ __attribute__((aligned(16))) uint32_t xch[5][4];
    const int64_t N = a.N, nb = (N + BS - 1) / BS;
    const int64_t tmin = step.batch[0], tmax = step.batch[1];  // K3p folded the batch range
    int64_t b = blockIdx.x;
    if (b < nb) pf_issue(a, pg, xcd_block(b, nb), stage);
    for (; b < nb; b += pg.grid) {
        // the thread index laundered per block: address arithmetic derived from it is redone
        // each block instead of hoisted and kept live (spilled) across the loop
        uint32_t tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const int lane = tid & 63;
        const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
        uint32_t xo = lds_off(&xch[0][0]);
        asm volatile("" : "+s"(xo));
        const int64_t blk = xcd_block(b, nb), first = blk * BS, n = first + tid;
        // the policy re-read from the kernel arguments every block through a pointer the compiler
        // cannot prove loop-invariant: hoisted out of the loop, its fields stayed live in SGPRs
        // across it (222 SGPRs spilled, and 118 VGPRs with them)
        const __attribute__((address_space(4))) K1Args* kp =
            (const __attribute__((address_space(4))) K1Args*)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(kp));
        const DevPolicy& pol = ((const K1Args*)kp)->pol;
        pf_barrier_dma();  // this block's DMA (and the last block's stores) landed
        CRANE_TSTAMP(a.trace, blk, 0);
        // the node's values out of the staging (row r of 8-byte values at chunk 2r)
        auto v8 = [&](int r) -> uint64_t {
            return *reinterpret_cast<const uint64_t*>(stage + 2 * r * kPfChunk + 8 * tid);
        };
        int64_t pt[PD], qt[PR];
        double pv[PD], qv[PR];
#pragma unroll
        for (int k = 0; k < PD; ++k) {
            const int r = k < pol.npd ? pol.pred_slot[k] : 0;
            pv[k] = __builtin_bit_cast(double, v8(r));
            pt[k] = (int64_t)v8(pg.ns + r);
        }
#pragma unroll
        for (int k = 0; k < PR; ++k) {
            const int r = k < pol.npr ? pol.prio_slot[k] : 0;
            qv[k] = __builtin_bit_cast(double, v8(r));
            qt[k] = (int64_t)v8(pg.ns + r);
        }
        uint32_t bc[kMaxWin];
        double hvl = 0.0;
        int64_t hvt = kTsInvalid;
        if (pg.bkrow >= 0) {
#pragma unroll
            for (int w = 0; w < kMaxWin; ++w)
                bc[w] = w < pol.n_win
                            ? *reinterpret_cast<const uint32_t*>(stage + (pg.bkrow + w) * kPfChunk + 4 * tid)
                            : 0u;
        } else if (pg.hvrow >= 0) {
            hvl = __builtin_bit_cast(double, v8(pg.ns * 2));
            hvt = a.hv_ts ? (int64_t)v8(pg.ns * 2 + 1) : a.hv_ts_counts;
        }
        pf_barrier();  // every value read: the staging is free
        if (b + pg.grid < nb) pf_issue(a, pg, xcd_block(b + pg.grid, nb), stage);
        CRANE_TSTAMP(a.trace, blk, 1);
        Rec r;
        const bool valid = n < N;
        if (valid) {
            rec_metrics<PD, PR>(pol, pt, pv, qt, qv, r);
            if (pg.bkrow >= 0) {
                if (!a.buckets_keep) {
#pragma unroll
                    for (int w = 0; w < kMaxWin; ++w)  // consumed: leaves the buckets zeroed for the next K2
                        if (w < pol.n_win) a.buckets[(int64_t)w * N + n] = 0;
                }
                rec_hot_counts<PD, PR>(pol, bc, N, n, a.cnt_out, a.hvc_out, a.hv_ts_counts, r);
            } else if (pg.hvrow >= 0) {
                rec_hot_annotation<PD, PR>(hvl, hvt, r);
            } else {
                r.pen = 0;
                r.e_hv = kTsInvalid;
            }
            rec_fail<PD, PR>(r);
        }
        CRANE_TSTAMP(a.trace, blk, 2);
        // classify (step_count_queue's first half: in-range expiries per kind, the flat keys)
        const int32_t s0 = score_at<PD, PR>(tmin, r, step.wsum, step.noprio, step.winv);
        int cnt1 = 0;
        int64_t mn1 = INT64_MAX, mx1 = INT64_MIN;
        auto add = [&](int64_t e, int& c, int64_t& mn, int64_t& mx) {
            const bool in = e > tmin && e <= tmax;
            c += in;
            mn = in ? min(mn, e) : mn;
            mx = in ? max(mx, e) : mx;
        };
#pragma unroll
        for (int k = 0; k < PR; ++k) add(r.e_prio[k], cnt1, mn1, mx1);
        add(r.e_hv, cnt1, mn1, mx1);
        int cnt0 = cnt1;
        int64_t mn0 = mn1, mx0 = mx1;
        add(r.e_fail, cnt0, mn0, mx0);  // DaemonSet pods bypass the Filter
        if (!valid) cnt0 = cnt1 = 0;
        const bool multi0 = cnt0 > 0 && mn0 != mx0, multi1 = cnt1 > 0 && mn1 != mx1;
        const int32_t flat0 = valid && cnt0 == 0 ? key_of<PD, PR>(0, tmin, s0, r, n) : -1;
        const int32_t flat1 = valid && cnt1 == 0 ? key_of<PD, PR>(1, tmin, s0, r, n) : -1;
        // per lane: one-step records | middle pieces << 16 per kind; queue items << 16
        const uint32_t w0 = (cnt0 ? (multi0 ? 2u : 1u) : 0u) | (multi0 ? (uint32_t)(cnt0 - 1) << 16 : 0u);
        const uint32_t w1 = (cnt1 ? (multi1 ? 2u : 1u) : 0u) | (multi1 ? (uint32_t)(cnt1 - 1) << 16 : 0u);
        const uint32_t w2 = ((cnt0 ? 1u : 0u) + (cnt1 ? 1u : 0u)) << 16;
        uint32_t e0 = wave_scan_add(w0), e1 = wave_scan_add(w1), e2 = wave_scan_add(w2);
        const int32_t f0 = wave_max(flat0), f1 = wave_max(flat1);
        // the wave's totals and flat maxima to xch[.][wave], one exchange, one barrier: every lane
        // then has the block's totals and the waves before its own (no LDS atomics)
        if (lane == 63) {
            asm_ds_write_b32(xo + 4 * (0 * 4 + wv), e0);
            asm_ds_write_b32(xo + 4 * (1 * 4 + wv), e1);
            asm_ds_write_b32(xo + 4 * (2 * 4 + wv), e2);
            asm_ds_write_b32(xo + 4 * (3 * 4 + wv), (uint32_t)f0);
            asm_ds_write_b32(xo + 4 * (4 * 4 + wv), (uint32_t)f1);
        }
        e0 -= w0;
        e1 -= w1;
        e2 -= w2;
        pf_barrier();
        uint32_t base[3], tot[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const uint4 x = asm_ds_read_b128(xo + 16 * k);
            base[k] = (wv > 0 ? x.x : 0u) + (wv > 1 ? x.y : 0u) + (wv > 2 ? x.z : 0u);
            tot[k] = x.x + x.y + x.z + x.w;
        }
        StepSlots so;
        so.slot0 = cnt0 ? (int32_t)((base[0] + e0) & 0xFFFF) : -1;
        so.mslot0 = multi0 ? (int32_t)((base[0] + e0) >> 16) : 0;
        so.slot1 = cnt1 ? (int32_t)((base[1] + e1) & 0xFFFF) : -1;
        so.mslot1 = multi1 ? (int32_t)((base[1] + e1) >> 16) : 0;
        // queue items and the stepped record to HBM (k3a_emit builds the tables from them)
        const int64_t qo = blk * 2 * BS;
        if (cnt0 | cnt1) {
            int qi = (int)((base[2] + e2) >> 16);
            if (cnt0) {
                step.qg[qo + qi] = tid | ((uint32_t)multi0 << 13) | ((uint32_t)so.slot0 << 14) |
                                   ((uint32_t)tid << 24);
                step.qmg[qo + qi] = so.mslot0;
                ++qi;
            }
            if (cnt1) {
                step.qg[qo + qi] = tid | (1u << 12) | ((uint32_t)multi1 << 13) | ((uint32_t)so.slot1 << 14) |
                                   ((uint32_t)tid << 24);
                step.qmg[qo + qi] = so.mslot1;
            }
            static_cast<Rec*>(step.srec)[n] = r;
        }
        if (tid < 6) {
            // the block's flat maxima, record counts and queued items (step_publish's outputs)
            const uint4 fx = asm_ds_read_b128(xo + 16 * (tid == 1 ? 4 : 3));
            const int32_t fm = max(max((int32_t)fx.x, (int32_t)fx.y), max((int32_t)fx.z, (int32_t)fx.w));
            if (tid < 2) {
                step.st.flat[blk * 2 + tid] = fm;
                if (tid == 0) step.nqg[blk] = (int32_t)(tot[2] >> 16);
            } else {
                const int L = tid - 2;  // [kind][one-step records, middle pieces]
                const uint32_t t = tot[L >> 1];
                step.st.cnt[blk * 4 + L] = (int32_t)((L & 1) ? t >> 16 : t & 0xFFFF);
            }
        }
        CRANE_TSTAMP(a.trace, blk, 3);
        if (a.trace && tid == 0) a.trace[8 * blk + 6] = blockIdx.x;  // (which workgroup: tools/trace_pf.py)
    }
}

template <int PD, int PR>
static hipError_t launch_count_pf(const K1Args& a, const K1Step& sa, hipStream_t st) {
    PfGeom pg{};
    pg.ns = a.pol.n_slots;
    const int rows8 = 2 * pg.ns;
    const bool bk = a.buckets != nullptr;
    const bool hvr = !bk && a.hv != nullptr;
    pg.hvrow = hvr ? 2 * rows8 : -1;
    pg.bkrow = bk ? 2 * rows8 : -1;
    pg.nchunk = 2 * rows8 + (hvr ? (a.hv_ts ? 4 : 2) : 0) + (bk ? a.pol.n_win : 0);
    // the staging's size is a template parameter: a static array beside the other LDS
    // objects, whose accesses the compiler then knows the DMA does not write (one array
    // made it wait vmcnt(0) — drain the prefetch — before every LDS atomic of the block)
    auto kern = pg.nchunk <= 16 ? k1_count_pf<PD, PR, 16> : (pg.nchunk <= 28 ? k1_count_pf<PD, PR, 28> : k1_count_pf<PD, PR, 44>);
    if (pg.nchunk > 44) return hipErrorInvalidValue;
    const size_t lds = 0;
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, 256, lds);
    if (e != hipSuccess) return e;
    const int64_t nb = (a.N + 255) / 256;
    int64_t grid = (int64_t)std::max(1, per_cu) * std::max(1, a.n_cu);
    grid = std::min<int64_t>(grid, (nb + 7) / 8 * 8);
    grid = std::max<int64_t>(8, grid / 8 * 8);
    pg.grid = (int32_t)grid;
    return klaunch("k1_node_pass+k3a_count", kern, dim3((unsigned)grid), dim3(256), lds, st, a, sa, pg);
}

// ---------------------------------------------------------------- K1 count pass, streamed (split form)
// The split count pass without the NodeRec: each node's expiries and terms are folded as its
// rows arrive into what the count pass needs — e_fail, the ordered score sum at tmin, the
// in-range count / min / max per pod kind, the hot value — so about 30 VGPRs of record never
// live (64 VGPRs: eight waves per SIMD instead of five), no LDS atomics (the waves' totals are
// exchanged once, one barrier), and no stepped records written: k3a_emit rebuilds the few
// stepped nodes' records from the SoA (k3a_emit<..., RC = true>).  Not with the dedupe-form K2
// entries (their block runs need the default pass's LDS counting).
// KEEP: the stepped nodes' records are built here and written to step.srec like the default
// count pass's, instead of rebuilt by k3a_emit: a stepped lane re-reads its node's rows (lines
// this wave just read, still in L2) once its classification is known — keeping the row values
// live to the end instead cost the occupancy the streamed form is for (83 VGPRs, five waves:
// 0.118 ms vs 0.096 cold, profiles/r04/k1_prefetch_ab.txt), and rebuilding them in k3a_emit
// after they have left the caches cost 0.022 ms of gathers.
// KEEP 2: the stepped lanes go one step further and write their one-step records (into the
// block's st.stage staging) and middle pieces themselves — step_emit, as a fused node pass's lane
// past its LDS staging does — so k3a_emit (SORT_ONLY) only sorts, publishes and writes the rows.
template <int PD, int PR, int WPE, int KEEP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
void k1_count_stream(K1Args a, K1Step step) {
    constexpr int BS = 256;
    __shared__ __attribute__((aligned(16))) uint32_t xch[5][4];
    const DevPolicy& pol = a.pol;
    const int64_t N = a.N;
    const int64_t blk = xcd_block(blockIdx.x, gridDim.x), first = blk * BS, n = first + threadIdx.x;
    CRANE_TSTAMP(a.trace, blockIdx.x, 0);
    const int lo = (int)min((int64_t)threadIdx.x, N - 1 - first);  // lane offset, clamped (K1's loads)
    int64_t pt[PD], qt[PR];
    double pv[PD], qv[PR];
#pragma unroll
    for (int k = 0; k < PD; ++k) {
        pt[k] = kTsInvalid;
        pv[k] = 0.0;
    }
#pragma unroll
    for (int k = 0; k < PR; ++k) {
        qt[k] = kTsInvalid;
        qv[k] = 0.0;
    }
    if (pol.n_slots > 0) {
#pragma unroll
        for (int k = 0; k < PD; ++k) {
            const int64_t row = k < pol.npd ? pol.pred_slot[k] : 0;
            pt[k] = (a.ts + (row * N + first))[lo];
            pv[k] = (a.val + (row * N + first))[lo];
        }
#pragma unroll
        for (int k = 0; k < PR; ++k) {
            const int64_t row = k < pol.npr ? pol.prio_slot[k] : 0;
            qt[k] = (a.ts + (row * N + first))[lo];
            qv[k] = (a.val + (row * N + first))[lo];
        }
    }
    uint32_t bc[kMaxWin];
    double hvl = 0.0;
    int64_t hvt = kTsInvalid;
    if (a.buckets) {
#pragma unroll
        for (int b = 0; b < kMaxWin; ++b) bc[b] = b < pol.n_win ? (a.buckets + first)[(int64_t)b * N + lo] : 0u;
    } else if (a.hv) {
        hvl = a.hv[first + lo];
        hvt = a.hv_ts ? a.hv_ts[first + lo] : a.hv_ts_counts;
    }
    const int64_t tmin = step.batch[0], tmax = step.batch[1];  // K3p folded the batch range
    CRANE_TSTAMP(a.trace, blockIdx.x, 1);
    const bool valid = n < N;
    // isOverLoad per predicate (stats.go:94-112): the Filter rejects iff now < e_fail
    int64_t e_fail = kTsInvalid;
#pragma unroll
    for (int k = 0; k < PD; ++k) {
        if (k < pol.npd) {
            const double u = pv[k], lim = pol.pred_limit[k];
            const bool over = pt[k] != kTsInvalid && !(u < 0.0) && lim != 0.0 && u > lim;
            if (over) e_fail = max(e_fail, sat_add(pt[k], pol.pred_dur[k]));
        }
    }
    // hot value (getNodeHotValue / the binding-log counts) -> penalty and its expiry
    NodeRec<PD, PR> hr;  // (only pen / e_hv are set and read)
    if (a.buckets) {
        if (valid && !a.buckets_keep) {
#pragma unroll
            for (int b = 0; b < kMaxWin; ++b)  // consumed: leaves the buckets zeroed for the next K2
                if (b < pol.n_win) (a.buckets + first)[(int64_t)b * N + threadIdx.x] = 0;
        }
        rec_hot_counts<PD, PR>(pol, bc, N, n, valid ? a.cnt_out : nullptr, valid ? a.hvc_out : nullptr,
                               a.hv_ts_counts, hr);
    } else if (a.hv) {
        rec_hot_annotation<PD, PR>(hvl, hvt, hr);
    } else {
        hr.pen = 0;
        hr.e_hv = kTsInvalid;
    }
    // priorities in policy order: score_at(tmin)'s ordered sum, and the in-range expiries both
    // pod kinds share (priorities, hot value); e_fail is kind 0's too (DaemonSet pods bypass the
    // Filter) — step_count_queue's classification without the record
    double s = 0.0;
    int cnt1 = 0;
    int64_t mn1 = INT64_MAX, mx1 = INT64_MIN;
    auto add = [&](int64_t e, int& c, int64_t& mn, int64_t& mx) {
        const bool in = e > tmin && e <= tmax;
        c += in;
        mn = in ? min(mn, e) : mn;
        mx = in ? max(mx, e) : mx;
    };
#pragma unroll
    for (int k = 0; k < PR; ++k) {
        int64_t e = kTsInvalid;
        double term = 0.0;
        if (k < pol.npr && qt[k] != kTsInvalid && !(qv[k] < 0.0)) {
            e = sat_add(qt[k], pol.prio_dur[k]);
            term = (1.0 - qv[k]) * pol.prio_w[k];  // getScore (stats.go:89), no FMA
            term = term * 100.0;
        }
        if (tmin < e) s += term;  // stats.go:124-133
        add(e, cnt1, mn1, mx1);
    }
    add(hr.e_hv, cnt1, mn1, mx1);
    int cnt0 = cnt1;
    int64_t mn0 = mn1, mx0 = mx1;
    add(e_fail, cnt0, mn0, mx0);
    if (!valid) cnt0 = cnt1 = 0;
    const int32_t s0 = score_of_sum(s, tmin < hr.e_hv ? hr.pen : 0, step.wsum, step.noprio, step.winv);
    const bool multi0 = cnt0 > 0 && mn0 != mx0, multi1 = cnt1 > 0 && mn1 != mx1;
    const int32_t flat0 = valid && cnt0 == 0 && !(tmin < e_fail) ? pack_key(s0, n) : -1;
    const int32_t flat1 = valid && cnt1 == 0 ? pack_key(s0, n) : -1;
    CRANE_TSTAMP(a.trace, blockIdx.x, 2);
    // slots: wave prefix sums, then the waves' totals exchanged once (one barrier, no LDS atomics)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t w0 = (cnt0 ? (multi0 ? 2u : 1u) : 0u) | (multi0 ? (uint32_t)(cnt0 - 1) << 16 : 0u);
    const uint32_t w1 = (cnt1 ? (multi1 ? 2u : 1u) : 0u) | (multi1 ? (uint32_t)(cnt1 - 1) << 16 : 0u);
    const uint32_t w2 = ((cnt0 ? 1u : 0u) + (cnt1 ? 1u : 0u)) << 16;
    uint32_t e0 = wave_scan_add(w0), e1 = wave_scan_add(w1), e2 = wave_scan_add(w2);
    const int32_t f0 = wave_max(flat0), f1 = wave_max(flat1);
    if (lane == 63) {
        xch[0][wv] = e0;
        xch[1][wv] = e1;
        xch[2][wv] = e2;
        xch[3][wv] = (uint32_t)f0;
        xch[4][wv] = (uint32_t)f1;
    }
    e0 -= w0;
    e1 -= w1;
    e2 -= w2;
    pf_barrier();  // (not __syncthreads: its fence would wait for this block's hvc / bucket stores)
    uint32_t base[3], tot[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint4 x = *reinterpret_cast<const uint4*>(xch[k]);
        base[k] = (wv > 0 ? x.x : 0u) + (wv > 1 ? x.y : 0u) + (wv > 2 ? x.z : 0u);
        tot[k] = x.x + x.y + x.z + x.w;
    }
    const int64_t qo = blk * 2 * BS;
    if (cnt0 | cnt1) {
        if constexpr (KEEP) {
            int64_t rt[PD], rq[PR];
            double rv[PD], rw[PR];
#pragma unroll
            for (int k = 0; k < PD; ++k) {
                const int64_t row = k < pol.npd ? pol.pred_slot[k] : 0;
                rt[k] = pol.n_slots > 0 ? a.ts[row * N + n] : kTsInvalid;
                rv[k] = pol.n_slots > 0 ? a.val[row * N + n] : 0.0;
            }
#pragma unroll
            for (int k = 0; k < PR; ++k) {
                const int64_t row = k < pol.npr ? pol.prio_slot[k] : 0;
                rq[k] = pol.n_slots > 0 ? a.ts[row * N + n] : kTsInvalid;
                rw[k] = pol.n_slots > 0 ? a.val[row * N + n] : 0.0;
            }
            NodeRec<PD, PR> r;
            rec_metrics<PD, PR>(pol, rt, rv, rq, rw, r);
            r.pen = hr.pen;
            r.e_hv = hr.e_hv;
            rec_fail<PD, PR>(r);
            if constexpr (KEEP == 2) {
                StepSlots so;
                so.slot0 = cnt0 ? (int32_t)((base[0] + e0) & 0xFFFF) : -1;
                so.mslot0 = multi0 ? (int32_t)((base[0] + e0) >> 16) : 0;
                so.multi0 = multi0;
                so.slot1 = cnt1 ? (int32_t)((base[1] + e1) & 0xFFFF) : -1;
                so.mslot1 = multi1 ? (int32_t)((base[1] + e1) >> 16) : 0;
                so.multi1 = multi1;
                step_emit<PD, PR>(r, n, tmin, tmax, step.wsum, step.noprio, so, step.st, blk,
                                  step.st.stage + blk * 2 * step.st.bs, step.st.s1pad, step.winv);
            } else {
                static_cast<NodeRec<PD, PR>*>(step.srec)[n] = r;
            }
        }
        const int32_t slot0 = (int32_t)((base[0] + e0) & 0xFFFF), slot1 = (int32_t)((base[1] + e1) & 0xFFFF);
        int qi = (int)((base[2] + e2) >> 16);
        if (KEEP == 2) cnt0 = cnt1 = 0;  // (nothing queued: the records are out)
        if (cnt0) {
            step.qg[qo + qi] = threadIdx.x | ((uint32_t)multi0 << 13) | ((uint32_t)slot0 << 14);
            step.qmg[qo + qi] = multi0 ? (int32_t)((base[0] + e0) >> 16) : 0;
            ++qi;
        }
        if (cnt1) {
            step.qg[qo + qi] = threadIdx.x | (1u << 12) | ((uint32_t)multi1 << 13) | ((uint32_t)slot1 << 14);
            step.qmg[qo + qi] = multi1 ? (int32_t)((base[1] + e1) >> 16) : 0;
        }
    }
    if (threadIdx.x < 6) {
        // the block's flat maxima, record counts and queued items (step_publish's outputs)
        const uint4 fx = *reinterpret_cast<const uint4*>(xch[threadIdx.x == 1 ? 4 : 3]);
        const int32_t fm = max(max((int32_t)fx.x, (int32_t)fx.y), max((int32_t)fx.z, (int32_t)fx.w));
        if (threadIdx.x < 2) {
            step.st.flat[blk * 2 + threadIdx.x] = fm;
            if (threadIdx.x == 0) step.nqg[blk] = KEEP == 2 ? 0 : (int32_t)(tot[2] >> 16);
        } else {
            const int L = threadIdx.x - 2;  // [kind][one-step records, middle pieces]
            const uint32_t t = tot[L >> 1];
            step.st.cnt[blk * 4 + L] = (int32_t)((L & 1) ? t >> 16 : t & 0xFFFF);
        }
    }
    CRANE_TSTAMP(a.trace, blockIdx.x, 3);
    CRANE_TSTAMP(a.trace, blockIdx.x, 4);
}

// A stepped node's record rebuilt from the SoA for k3a_emit after the streamed count pass
// (K1's own rec_metrics / hot-value / rec_fail, so the same bits as the record K1 builds);
// the binding-log hot value is the one the count pass kept in hvc_out.
template <int PD, int PR>
__device__ __forceinline__ NodeRec<PD, PR> rec_rebuild(const K1Args& a, int64_t n) {
    const DevPolicy& pol = a.pol;
    const int64_t N = a.N;
    int64_t pt[PD], qt[PR];
    double pv[PD], qv[PR];
#pragma unroll
    for (int k = 0; k < PD; ++k) {
        const int64_t row = k < pol.npd ? pol.pred_slot[k] : 0;
        pt[k] = pol.n_slots > 0 ? a.ts[row * N + n] : kTsInvalid;
        pv[k] = pol.n_slots > 0 ? a.val[row * N + n] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < PR; ++k) {
        const int64_t row = k < pol.npr ? pol.prio_slot[k] : 0;
        qt[k] = pol.n_slots > 0 ? a.ts[row * N + n] : kTsInvalid;
        qv[k] = pol.n_slots > 0 ? a.val[row * N + n] : 0.0;
    }
    NodeRec<PD, PR> r;
    rec_metrics<PD, PR>(pol, pt, pv, qt, qv, r);
    if (a.buckets) {
        const double h = a.hvc_out[n];  // (int64 v as double: v >= 0 iff h >= 0)
        r.pen = go_int(h * 10.0);
        r.e_hv = h >= 0.0 ? sat_add(a.hv_ts_counts, kHotActiveNs) : kTsInvalid;
    } else if (a.hv) {
        rec_hot_annotation<PD, PR>(a.hv[n], a.hv_ts ? a.hv_ts[n] : a.hv_ts_counts, r);
    } else {
        r.pen = 0;
        r.e_hv = kTsInvalid;
    }
    rec_fail<PD, PR>(r);
    return r;
}

template <int PD, int PR, int WPE, int KEEP>
static hipError_t launch_count_stream_w(const K1Args& a, const K1Step& sa, hipStream_t st) {
    const unsigned grid = (unsigned)((a.N + 255) / 256);
    return klaunch("k1_node_pass+k3a_count", k1_count_stream<PD, PR, WPE, KEEP>, dim3(grid), dim3(256), 0, st, a, sa);
}

// ---------------------------------------------------------------- K3a emit (split form)
// One workgroup per producer block of the split node pass (NODES nodes): the block's queued
// (node, kind) items are built from the stepped records in HBM (L2-resident: written by the
// node pass on the same XCD), then sorted, published and the tile rows written — the fused
// K1 epilogue.  BT threads: NODES (the block's own width), or one wave (BT = 64), whose
// barriers are free and whose small LDS (CAP one-step records per kind staged; a block with
// more goes through st.stage) lets many blocks' epilogues run on a CU at once.
// RC: the count pass was the streamed one (no stepped records written): each queued node's
// record is rebuilt from the SoA (rec_rebuild) instead of read from step.srec.
// SORT_ONLY: the count pass wrote the one-step records into st.stage and the middle pieces
// itself (count_stream_emits): no items; the staging is read by the global sort path.
template <int PD, int PR, int NODES, int BT, bool RC = false, bool SORT_ONLY = false>
__global__ __launch_bounds__(BT) void k3a_emit(K1Step step, int64_t N, K1Args a) {
    using Rec = NodeRec<PD, PR>;
    constexpr int CAP = BT == 64 ? 64 : (kK1S1Cap < 2 * NODES ? kK1S1Cap : 2 * NODES);
    __shared__ StepShared ssh;
    __shared__ __attribute__((aligned(16))) Step1 s1l[2 * CAP];
    __shared__ __attribute__((aligned(16))) Step1 s1s[2 * CAP];
    constexpr int kPieceCap = BT == 64 ? 32 : 64;
    __shared__ __attribute__((aligned(16))) unsigned char pscr[kPieceCap * PieceScr::bytes_per_piece];
    __shared__ int32_t nq;
    const int64_t nb = (N + NODES - 1) / NODES;
    const int64_t blk = xcd_block(blockIdx.x, nb);  // the node pass's mapping: same XCD
    const int64_t first = blk * NODES;
    const StepTables& st = step.st;
    if (threadIdx.x < 4) ssh.lc[threadIdx.x >> 1][threadIdx.x & 1] = st.cnt[blk * 4 + threadIdx.x];
    if (threadIdx.x < 2) {
        // the block's flat maxima (step_tile_rows folds sh.fm over the waves)
        ssh.fm[threadIdx.x][0] = st.flat[blk * 2 + threadIdx.x];
        for (int i = 1; i < BT / 64; ++i) ssh.fm[threadIdx.x][i] = -1;
    }
    if (threadIdx.x == 0) nq = step.nqg[blk];
    int64_t tpre = 0;
    if (st.rows) tile_prefetch(st, &tpre);
    const int64_t tmin = step.batch[0], tmax = step.batch[1];
    __syncthreads();
    const bool g1 = SORT_ONLY || max(ssh.lc[0][0], ssh.lc[1][0]) > min(CAP, st.lds_cap);
    Step1* s1b = g1 ? st.stage + blk * 2 * st.bs : s1l;
    const int64_t kst = g1 ? st.s1pad : (int64_t)CAP;
    const uint32_t* q = step.qg + blk * 2 * NODES;
    const int32_t* qm = step.qmg + blk * 2 * NODES;
    const Rec* rec = static_cast<const Rec*>(step.srec);
    for (int w = threadIdx.x; w < (SORT_ONLY ? 0 : nq); w += BT) {
        const uint32_t it = q[w];
        const int o = (int)(it & 0xFFF);
        const Rec r = RC ? rec_rebuild<PD, PR>(a, first + o) : rec[first + o];
        step_emit_one<PD, PR>(r, first + o, (int)((it >> 12) & 1), (int32_t)((it >> 14) & 0x3FF), qm[w],
                              ((it >> 13) & 1) != 0, tmin, tmax, step.wsum, step.noprio, st, blk, s1b, kst,
                              step.winv);
    }
    __syncthreads();
    if (g1) step_sort_publish_global<BT>(ssh, st, blk);
    else step_sort_publish<BT, CAP>(s1l, s1s, ssh, st, blk);
    if (st.rows) {
        const PieceScr ps{pscr, kPieceCap};
        step_pieces<BT>(ssh, st, blk, ps);
        if (g1) step_tile_rows<BT, CAP, true>(s1l, s1s, ssh, st, blk, &tpre, ps);
        else step_tile_rows<BT, CAP, false>(s1l, s1s, ssh, st, blk, &tpre, ps);
    }
}

template <int PD, int PR>
static hipError_t launch_emit_t(const K1Step& step, int64_t N, int32_t bs, int32_t bt, hipStream_t st,
                                const K1Args* rc, bool sort_only) {
    const int64_t nb = (N + bs - 1) / bs;
    if (nb <= 0) return hipSuccess;
    const K1Args a = rc ? *rc : K1Args{};
    if (rc) {  // after the streamed count pass (256-node blocks): rebuild, or sort only
        if (bs != 256) return hipErrorInvalidValue;
        if (sort_only) {
            if (bt == 64)
                return klaunch("k3a_emit", k3a_emit<PD, PR, 256, 64, false, true>, dim3((unsigned)nb), dim3(64), 0, st,
                               step, N, a);
            return klaunch("k3a_emit", k3a_emit<PD, PR, 256, 256, false, true>, dim3((unsigned)nb), dim3(256), 0, st,
                           step, N, a);
        }
        if (bt == 64)
            return klaunch("k3a_emit", k3a_emit<PD, PR, 256, 64, true>, dim3((unsigned)nb), dim3(64), 0, st, step, N, a);
        return klaunch("k3a_emit", k3a_emit<PD, PR, 256, 256, true>, dim3((unsigned)nb), dim3(256), 0, st, step, N, a);
    }
    if (bs == 256 && bt == 64)
        return klaunch("k3a_emit", k3a_emit<PD, PR, 256, 64>, dim3((unsigned)nb), dim3(64), 0, st, step, N, a);
    if (bs == 256) return klaunch("k3a_emit", k3a_emit<PD, PR, 256, 256>, dim3((unsigned)nb), dim3(256), 0, st, step, N, a);
    if (bs == 128) return klaunch("k3a_emit", k3a_emit<PD, PR, 128, 128>, dim3((unsigned)nb), dim3(128), 0, st, step, N, a);
    return hipErrorInvalidValue;
}

hipError_t launch_step_emit(int shape, const K1Step& step, int64_t N, int32_t bs, hipStream_t st, int32_t bt,
                            const K1Args* rc, bool sort_only) {
    switch (shape) {
        case kShape4x6: return launch_emit_t<4, 6>(step, N, bs, bt, st, rc, sort_only);
        case kShape8x8: return launch_emit_t<8, 8>(step, N, bs, bt, st, rc, sort_only);
        default: return launch_emit_t<16, 16>(step, N, bs, bt, st, rc, sort_only);
    }
}

// ---------------------------------------------------------------- launchers
bool count_stream(int count_form, const K1Args& a) {
    return count_form >= 5 && count_form <= 11 && a.threads == 256 && a.hx_region == nullptr && a.out == nullptr;
}
bool count_stream_rebuild(int count_form, const K1Args& a) { return count_stream(count_form, a) && count_form <= 7; }
bool count_stream_emits(int count_form, const K1Args& a) { return count_stream(count_form, a) && count_form >= 10; }

template <int PD, int PR>
static hipError_t launch_k1_t(const K1Args& a, const K1Step* step, hipStream_t st, int count_form) {
    if (a.N <= 0) return hipSuccess;
    const int T = a.threads;
    if (T != 128 && T != 256) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)((a.N + T - 1) / T);
    // + the sorted one-step records past the node records when both are kept (kernel above)
    // records: every node's when written out (+ the sorted one-step records past them); keys-only
    // step: kK1RecCap stepped records, the sorted one-step records over them after the emit
    const size_t s1 = step ? 2 * sizeof(Step1) * (size_t)std::min(kK1S1Cap, 2 * T) : 0;  // sorted copy
    const size_t lds = a.out ? sizeof(NodeRec<PD, PR>) * T + s1
                             : std::max(sizeof(NodeRec<PD, PR>) * (size_t)std::min(T, kK1RecCap), s1);
    if (step && !step->st.stage) return hipErrorInvalidValue;
    const K1Step sa = step ? *step : K1Step{};
    if (step && step->srec) {  // split form: no LDS staging, the epilogue is k3a_emit's
        if (a.out || !step->qg || !step->qmg || !step->nqg) return hipErrorInvalidValue;
        const char* nm = "k1_node_pass+k3a_count";
        if (count_form == 4 && T == 256 && a.hx_region == nullptr && a.pol.n_slots <= 8 && a.n_cu > 0)
            return launch_count_pf<PD, PR>(a, sa, st);
        if (count_stream(count_form, a)) {
            switch (count_form) {
                case 5: return launch_count_stream_w<PD, PR, 8, 0>(a, sa, st);
                case 6: return launch_count_stream_w<PD, PR, 7, 0>(a, sa, st);
                case 7: return launch_count_stream_w<PD, PR, 6, 0>(a, sa, st);
                case 8: return launch_count_stream_w<PD, PR, 6, 1>(a, sa, st);
                case 9: return launch_count_stream_w<PD, PR, 7, 1>(a, sa, st);
                case 10: return launch_count_stream_w<PD, PR, 6, 2>(a, sa, st);
                default: return launch_count_stream_w<PD, PR, 5, 2>(a, sa, st);
            }
        }
        if (T == 256 && PD * PR <= 24 && count_form >= 1 && count_form <= 3) {  // A/B forms of the count pass (4x6 shape)
            const bool nohx = a.hx_region == nullptr;
            switch (count_form) {
                case 1: return nohx ? klaunch(nm, k1_node_pass<PD, PR, 256, true, true, 5, 1>, dim3(grid), dim3(256), 0, st, a, sa)
                                    : klaunch(nm, k1_node_pass<PD, PR, 256, true, true, 5, 0>, dim3(grid), dim3(256), 0, st, a, sa);
                case 2: return nohx ? klaunch(nm, k1_node_pass<PD, PR, 256, true, true, 6, 1>, dim3(grid), dim3(256), 0, st, a, sa)
                                    : klaunch(nm, k1_node_pass<PD, PR, 256, true, true, 6, 0>, dim3(grid), dim3(256), 0, st, a, sa);
                default: return nohx ? klaunch(nm, k1_node_pass<PD, PR, 256, true, true, 7, 1>, dim3(grid), dim3(256), 0, st, a, sa)
                                     : klaunch(nm, k1_node_pass<PD, PR, 256, true, true, 7, 0>, dim3(grid), dim3(256), 0, st, a, sa);
            }
        }
        if (T == 256)
            return klaunch(nm, k1_node_pass<PD, PR, 256, true, true>, dim3(grid), dim3(256), 0, st, a, sa);
        return klaunch(nm, k1_node_pass<PD, PR, 128, true, true>, dim3(grid), dim3(128), 0, st, a, sa);
    }
    const char* nm = step ? "k1_node_pass+k3a_steps" : "k1_node_pass";
    if (T == 256)
        return step ? klaunch(nm, k1_node_pass<PD, PR, 256, true>, dim3(grid), dim3(256), lds, st, a, sa)
                    : klaunch(nm, k1_node_pass<PD, PR, 256, false>, dim3(grid), dim3(256), lds, st, a, sa);
    return step ? klaunch(nm, k1_node_pass<PD, PR, 128, true>, dim3(grid), dim3(128), lds, st, a, sa)
                : klaunch(nm, k1_node_pass<PD, PR, 128, false>, dim3(grid), dim3(128), lds, st, a, sa);
}

hipError_t launch_node_pass(int shape, const K1Args& a, hipStream_t st, const K1Step* step, int count_form) {
    switch (shape) {
        case kShape4x6: return launch_k1_t<4, 6>(a, step, st, count_form);
        case kShape8x8: return launch_k1_t<8, 8>(a, step, st, count_form);
        default: return launch_k1_t<16, 16>(a, step, st, count_form);
    }
}

size_t node_rec_bytes(int shape) {
    switch (shape) {
        case kShape4x6: return sizeof(NodeRec<4, 6>);
        case kShape8x8: return sizeof(NodeRec<8, 8>);
        default: return sizeof(NodeRec<16, 16>);
    }
}

hipError_t launch_hot_count(const int32_t* bnode, const int64_t* bts, int64_t B, int64_t N, const HotCutoffs& cut,
                            uint32_t* buckets, hipStream_t st) {
    if (B <= 0 || cut.n_win <= 0) return hipSuccess;
    const int64_t per_block = (int64_t)kK2Threads * kK2PerThread;
    const unsigned grid = (unsigned)((B + per_block - 1) / per_block);
    const size_t lds = cut.n_win <= kLdsWin ? (size_t)kHashSlots * (4 + 4 * cut.n_win) : 0;
    static const hipError_t attr =
        hipFuncSetAttribute((const void*)k2_hot_count, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (attr != hipSuccess) return attr;
    return klaunch("k2_hot_count", k2_hot_count, dim3(grid), dim3(kK2Threads), lds, st, bnode, bts, B, N, cut,
                   buckets);
}

}  // namespace crane
