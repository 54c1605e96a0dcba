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

// The 4x6 shape's registers are budgeted for five waves per SIMD (with the fused form's ~30 KB
// of LDS, five workgroups per CU).  Round 4's split forms of this pass (a count pass + a separate
// emit kernel, its prefetching and streamed count passes) measured no faster and were removed
// (DESIGN 4.2).
template <int PD, int PR, int kK1Threads, bool STEP>
__global__ __launch_bounds__(kK1Threads) __attribute__((amdgpu_waves_per_eu(PD * PR <= 24 ? 5 : 1)))
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
    __shared__ uint32_t q[STEP ? 2 * kK1Threads : 1];
    __shared__ int32_t qm[STEP ? 2 * kK1Threads : 1];  // first middle-piece slot of queued items
    // one-step records per kind (2 per node at most, CAP staged in LDS): staging; sorted
    // copy over the records' LDS once the emit has read them (or past them when the
    // records are written out) (one buffer with the dedupe-form K2 buckets hxh below:
    // those are read before the step epilogue's first barrier, the staging is written after it)
    constexpr int CAP = kK1S1Cap < 2 * kK1Threads ? kK1S1Cap : 2 * kK1Threads;
    constexpr int kHxWords = kMaxWin * kK1Threads;
    constexpr int kUnion = (STEP ? 2 * CAP * (int)sizeof(Step1) : 0) > 4 * kHxWords
                               ? 2 * CAP * (int)sizeof(Step1)
                               : 4 * kHxWords;
    __shared__ __attribute__((aligned(16))) unsigned char ush[kUnion];
    Step1* s1l = reinterpret_cast<Step1*>(ush);
    Step1* s1s = reinterpret_cast<Step1*>(smem + (out ? sizeof(Rec) * kK1Threads : 0));
    if (STEP && threadIdx.x < 4) ssh.lc[threadIdx.x >> 1][threadIdx.x & 1] = 0;
    __shared__ int32_t nrec;  // keys-only step: stepped records staged
    if (STEP && threadIdx.x == 0) nq = nrec = 0;
    auto hxh = reinterpret_cast<uint32_t(*)[kK1Threads]>(ush);  // dedupe-form K2: this block's window-rank buckets
    const bool hx = a.hx_region != nullptr;
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
        // the delta form's anchor counts beside the adjustments (without them: the adjustments
        // again, added as zero)
        const uint32_t* __restrict__ base = a.bucket_base ? a.bucket_base : buckets;
        uint32_t bz[kMaxWin];
#pragma unroll
        for (int b = 0; b < kMaxWin; ++b) {
            bc[b] = b < pol.n_win ? (buckets + first)[(int64_t)b * N + lo] : 0u;
            bz[b] = b < pol.n_win ? (base + first)[(int64_t)b * N + lo] : 0u;
        }
        if (a.bucket_base) {  // (rows past n_win read as 0)
#pragma unroll
            for (int b = 0; b < kMaxWin; ++b) bc[b] = bz[b] + bc[b] - (b + 1 < kMaxWin ? bc[b + 1] : 0u);
        }
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
        step_count_queue<PD, PR, kK1RecCap>(r, n < N, n, tmin, tmax, step.wsum, step.winv, step.noprio,
                                            out != nullptr, ssh, &nrec, &nq, q, qm, lrec, so, self_emit);
        step_publish<kK1Threads>(so, ssh, step.st, blk);  // (its barrier also orders lrec and the queue)
        CRANE_TSTAMP(a.trace, blockIdx.x, 3);
        // one-step records staged in LDS, or (more of a kind than it holds) in st.stage
        const bool g1 = max(ssh.lc[0][0], ssh.lc[1][0]) > min(CAP, step.st.lds_cap);
        const S1Out s1o{s1l, step.st.stage + blk * 2 * step.st.bs, g1, (int64_t)CAP, step.st.s1pad};
        // (a node past the staging emits first: its record then dies before the queue's)
        if (self_emit)
            step_emit<PD, PR>(r, n, tmin, tmax, step.wsum, step.noprio, so, step.st, blk, s1o, step.winv);
        // the queued items are built densely by the first lanes of the workgroup
        for (int w = threadIdx.x; w < nq; w += kK1Threads) {
            const uint32_t it = q[w];
            if (it == ~0u) continue;  // a self-emitted node's
            const int o = (int)(it & 0xFFF);
            step_emit_one<PD, PR>(lrec[it >> 24], first + o, (int)((it >> 12) & 1), (int32_t)((it >> 14) & 0x3FF),
                                  qm[w], ((it >> 13) & 1) != 0, tmin, tmax, step.wsum, step.noprio, step.st, blk,
                                  s1o, step.winv);
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

// ---------------------------------------------------------------- launchers
template <int PD, int PR>
static hipError_t launch_k1_t(const K1Args& a, const K1Step* step, hipStream_t st, int stream) {
    if (a.N <= 0) return hipSuccess;
    const int T = a.threads;
    if (T != 256) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)((a.N + T - 1) / T);
    // + the sorted one-step records past the node records when both are kept (kernel above)
    // records: every node's when written out (+ the sorted one-step records past them); keys-only
    // step: kK1RecCap stepped records, the sorted one-step records over them after the emit
    const size_t s1 = step ? 2 * sizeof(Step1) * (size_t)std::min(kK1S1Cap, 2 * T) : 0;  // sorted copy
    const size_t lds = a.out ? sizeof(NodeRec<PD, PR>) * T + s1
                             : std::max(sizeof(NodeRec<PD, PR>) * (size_t)std::min(T, kK1RecCap), s1);
    if (step && !step->st.stage) return hipErrorInvalidValue;
    const K1Step sa = step ? *step : K1Step{};
    const char* nm = step ? "k1_node_pass+k3a_steps" : "k1_node_pass";
    if (step && stream && !a.out && a.hx_region == nullptr && T == 256)
        return launch_stream_steps(PD, PR, a, sa, st);
    return step ? klaunch(nm, k1_node_pass<PD, PR, 256, true>, dim3(grid), dim3(256), lds, st, a, sa)
                : klaunch(nm, k1_node_pass<PD, PR, 256, false>, dim3(grid), dim3(256), lds, st, a, sa);
}

hipError_t launch_node_pass(int shape, const K1Args& a, hipStream_t st, const K1Step* step, int stream) {
    switch (shape) {
        case kShape4x6: return launch_k1_t<4, 6>(a, step, st, stream);
        case kShape8x8: return launch_k1_t<8, 8>(a, step, st, stream);
        default: return launch_k1_t<16, 16>(a, step, st, stream);
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
