// kernels.hip — CDNA4 (gfx950) kernels of the Dynamic plugin hot path.
//
//   K2 hot_count : binding records -> per-node window counts (LDS-aggregated)
//   K1 node_pass : parsed annotation SoA (+ K2 counts) -> NodeRec per node
//   K3 eval      : pods x nodes Filter + Score + per-pod argmax
//
// Numerics follow /root/reference/pkg/plugins/dynamic/stats.go and plugins.go
// bit for bit: fp64 in the reference's operation order, no FMA contraction
// (built with -ffp-contract=off), Go's float64->int conversion and wrapping
// int64 arithmetic.  Wave = 64 lanes; K3 puts 64 PODS on a wave so every node
// record is wave-uniform and arrives through scalar loads.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "dyn_types.hpp"
#include "kernels.hpp"
#include "step_node.hpp"

namespace crane {

// Go int(float64) on amd64 (CVTTSD2SQ): NaN and out-of-range -> INT64_MIN.
// Used by stats.go:135 (int(score/weight)) and plugins.go:91 (int(hv*10)).
__device__ __forceinline__ int64_t go_int(double x) {
    if (!(x >= -9223372036854775808.0 && x < 9223372036854775808.0)) return INT64_MIN;
    return (int64_t)x;
}

__device__ __forceinline__ int64_t sat_add(int64_t a, int64_t b) {
    int64_t r;
    if (__builtin_add_overflow(a, b, &r)) return b > 0 ? INT64_MAX : INT64_MIN;
    return r;
}

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
// block size: 256 by default, CRANE_K1_THREADS=128 selects the narrow variant
// STEP: also build the K3 step tables of the pod batch (K3a fused, step.hip):
// the record is classified straight from registers.
template <int PD, int PR, int kK1Threads, bool STEP>
__global__ __launch_bounds__(kK1Threads) void k1_node_pass(K1Args a, K1Step step) {
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
    const int64_t first = blk * kK1Threads;
    const int64_t n = first + threadIdx.x;
    __shared__ int64_t smn[kK1Threads / 64], smx[kK1Threads / 64];
    __shared__ StepShared ssh;
    int64_t tmin = 0, tmax = 0, pmn = 0, pmx = 0;
    __shared__ int32_t nq;                      // stepped (node, kind) items queued for the emit
    __shared__ uint32_t q[STEP ? 2 * kK1Threads : 1];
    if (STEP && threadIdx.x < 4) ssh.lc[threadIdx.x >> 1][threadIdx.x & 1] = 0;
    if (STEP && threadIdx.x == 0) nq = 0;
    __shared__ uint32_t hxh[kMaxWin][kK1Threads];  // dedupe-form K2: this block's window-rank buckets
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
    constexpr int kHxPer = 4, kHxFirst = 4, kHxRun = 8;
    uint32_t co0[kHxPer];
    if (hx) {
#pragma unroll
        for (int u = 0; u < kHxPer; ++u) {
            const int i = u * kK1Threads + threadIdx.x;
            co0[u] = i < a.hx_nblk ? a.hx_CO[(int64_t)i * gridDim.x + blk] : 0u;
        }
        for (int b = 0; b < kMaxWin; ++b) hxh[b][threadIdx.x] = 0;
    }
    if (n < N) {
        // every load first, unconditionally (rows past npd/npr read row 0 and are
        // ignored), so a wave has them all in flight at once; compute after
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
        if (pol.n_slots > 0) {  // (val/ts are null without metrics)
#pragma unroll
            for (int k = 0; k < PD; ++k) {
                const int64_t row = k < pol.npd ? pol.pred_slot[k] : 0;
                pt[k] = ts[row * N + n];
                pv[k] = val[row * N + n];
            }
#pragma unroll
            for (int k = 0; k < PR; ++k) {
                const int64_t row = k < pol.npr ? pol.prio_slot[k] : 0;
                qt[k] = ts[row * N + n];
                qv[k] = val[row * N + n];
            }
        }
        if (buckets) {
#pragma unroll
            for (int b = 0; b < kMaxWin; ++b) bc[b] = b < pol.n_win ? buckets[(int64_t)b * N + n] : 0u;
        }
        if (!buckets && !hx && hv) {
            hvl = hv[n];
            hvt = hv_ts ? hv_ts[n] : hv_ts_counts;  // null: the binding-log value of an earlier pass
        }
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
                const uint32_t co = i0 == 0 ? co0[u] : i < a.hx_nblk ? a.hx_CO[(int64_t)i * gridDim.x + blk] : 0u;
                c[u] = co & 0xFFFF;
                o[u] = co >> 16;
            }
            uint32_t v[kHxPer][kHxFirst];
#pragma unroll
            for (int u = 0; u < kHxPer; ++u) {
                const uint32_t* src = a.hx_region + (int64_t)(i0 + u * kK1Threads + threadIdx.x) * kHxRegion + o[u];
#pragma unroll
                for (int k = 0; k < kHxFirst; ++k) v[u][k] = (uint32_t)k < c[u] ? src[k] : 0u;
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
                    for (int j = 0; j < kHxRun; ++j) w[j] = k0 + j < c[u] ? src[k0 + j] : 0u;
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
    // the batch time range partials: issued after the SoA loads, reduced after the compute
    if (STEP) batch_range_load<kK1Threads>(step.tile_mm, step.ntiles, pmn, pmx);
    if (n < N) {
#pragma unroll
        for (int k = 0; k < PD; ++k) {
            int64_t e = kTsInvalid;
            if (k < pol.npd) {
                const int64_t t = pt[k];
                const double u = pv[k];
                const double lim = pol.pred_limit[k];
                // isOverLoad (stats.go:94-112): usable (stats.go:51-76), limit != 0, u > limit
                const bool over = t != kTsInvalid && !(u < 0.0) && lim != 0.0 && u > lim;
                if (over) e = sat_add(t, pol.pred_dur[k]);
            }
            r.e_pred[k] = e;
        }
#pragma unroll
        for (int k = 0; k < PR; ++k) {
            int64_t e = kTsInvalid;
            double term = 0.0;
            if (k < pol.npr) {
                const int64_t t = qt[k];
                const double u = qv[k];
                if (t != kTsInvalid && !(u < 0.0)) {
                    e = sat_add(t, pol.prio_dur[k]);
                    // getScore (stats.go:89): (1. - usage) * Weight * float64(MaxNodeScore)
                    term = (1.0 - u) * pol.prio_w[k];
                    term = term * 100.0;
                }
            }
            r.e_prio[k] = e;
            r.t[k] = term;
        }
        if (buckets || hx) {
            // annotateNodeHotValue (node.go:113-121): value += count / p.Count (Go int division)
            // window w counts the bindings of buckets >= its cutoff rank (K2)
            if (buckets) {
#pragma unroll
                for (int b = 0; b < kMaxWin; ++b)  // consumed: leaves the buckets zeroed for the next K2
                    if (b < pol.n_win) buckets[(int64_t)b * N + n] = 0;
            }
            int64_t v = 0;
#pragma unroll
            for (int w = 0; w < kMaxWin; ++w) {
                if (w >= pol.n_win) break;
                int64_t c = 0;
#pragma unroll
                for (int b = 0; b < kMaxWin; ++b) c += (b >= pol.win_pos[w] && b < pol.n_win) ? bc[b] : 0u;
                if (cnt_out) cnt_out[(int64_t)w * N + n] = (uint32_t)c;
                // Go int division (truncates toward 0); counts fit 32 bits in practice: u32 divide
                const int64_t cw = pol.win_count[w];
                if (cw > 0 && cw <= 0xFFFFFFFFLL && c <= 0xFFFFFFFFLL)
                    v += (int64_t)((uint32_t)c / (uint32_t)cw);
                else
                    v += c / cw;
            }
            // the plugin re-reads it via ParseFloat (exact) and rejects negatives (stats.go:71-73)
            const double h = (double)v;
            if (a.hvc_out) a.hvc_out[n] = h;  // kept for node passes after the buckets are consumed
            r.pen = go_int(h * 10.0);
            r.e_hv = v >= 0 ? sat_add(hv_ts_counts, kHotActiveNs) : kTsInvalid;
        } else if (hv) {
            const double h = hvl;
            const int64_t t = hvt;
            r.pen = go_int(h * 10.0);
            r.e_hv = (t != kTsInvalid && !(h < 0.0)) ? sat_add(t, kHotActiveNs) : kTsInvalid;
        } else {
            r.pen = 0;
            r.e_hv = kTsInvalid;
        }
        int64_t e_fail = kTsInvalid;
#pragma unroll
        for (int k = 0; k < PD; ++k) e_fail = max(e_fail, r.e_pred[k]);
        r.e_fail = e_fail;
        bool slow = pol.noprio != 0;
#pragma unroll
        for (int k = 0; k < PR; ++k) slow |= !(__builtin_fabs(r.t[k]) < kTermMax);  // NaN/Inf/huge
        const bool pen_fast = r.pen >= 0 && r.pen < (1LL << 30);
        slow |= r.e_hv != kTsInvalid && !pen_fast;
        r.pen32 = pen_fast ? (int32_t)r.pen : 0;
        r.flags = slow ? kRecSlow : 0;
        if (out) lrec[threadIdx.x] = r;
    }
    if (STEP) {
        batch_range_reduce<kK1Threads>(pmn, pmx, smn, smx, tmin, tmax);
        if (n < N) step_count<PD, PR>(r, n, tmin, tmax, step.wsum, step.noprio, ssh, so);
        if (so.slot0 >= 0 || so.slot1 >= 0) {  // stepped (a few %): record to LDS, items to the queue
            if (!out) lrec[threadIdx.x] = r;
            step_queue(so, &nq, q);
        }
        step_publish<kK1Threads>(so, ssh, step.st, blk);  // (its barrier also orders lrec and the queue)
        // the queued items are built densely by the first lanes of the workgroup
        for (int w = threadIdx.x; w < nq; w += kK1Threads) {
            const uint32_t it = q[w];
            const int o = (int)(it & 0xFFF);
            step_emit_one<PD, PR>(lrec[o], first + o, (int)((it >> 12) & 1), (int32_t)(it >> 14), ((it >> 13) & 1) != 0,
                                  tmin, tmax, step.wsum, step.noprio, step.st, blk);
        }
    } else {
        __syncthreads();
    }
    if (!out) return;  // keys-only step: the records are rebuilt when a matrix/greedy pass needs them
    const int64_t nvalid = min((int64_t)kK1Threads, N - first);
    const int64_t nvec = nvalid * (int64_t)sizeof(Rec) / 16;
    const uint4* src = reinterpret_cast<const uint4*>(smem);
    uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<unsigned char*>(out) + first * (int64_t)sizeof(Rec));
    for (int64_t i = threadIdx.x; i < nvec; i += kK1Threads) dst[i] = src[i];
}

// ---------------------------------------------------------------- K3
// blockIdx.x -> 256 pods (4 waves x 64), blockIdx.y -> a chunk of nodes.
// Every lane walks the chunk's nodes in ascending order keeping a packed
// 32-bit running key (score << 24 | ~local index) — max keeps the first node
// with the highest score (lowest-index tie-break) — and one 64-bit atomicMax
// per pod merges chunks.  The NodeRec address depends only on the loop
// counter, so it is wave-uniform and arrives through s_load into SGPRs.
constexpr int kK3Threads = 256;

// Exact reference semantics in 64-bit, for the rare lanes/nodes the fast
// path cannot take (non-finite usage, |score| >= 2^30, huge or NaN hot value).
template <int PD, int PR>
__device__ __attribute__((noinline)) int32_t score_exact(int64_t tnow, const NodeRec<PD, PR>& r, double wsum,
                                                         int32_t noprio) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < PR; ++k)
        if (tnow < r.e_prio[k]) s += r.t[k];  // stats.go:124-133, policy order
    const int64_t base = noprio ? 0 : go_int(s / wsum);  // stats.go:135
    const int64_t pen = tnow < r.e_hv ? r.pen : 0;
    int64_t f = (int64_t)((uint64_t)base - (uint64_t)pen);  // plugins.go:91, Go int64 wraps
    return (int32_t)(f < 0 ? 0 : (f > 100 ? 100 : f));     // NormalizeScore (utils.go:58-68)
}

// A node record's fields as the loop consumes them (wave-uniform -> SGPRs).
template <int PD, int PR>
struct RecRegs {
    int64_t e_fail, e_hv;
    int32_t pen32, flags;
    int64_t e_prio[PR];
    double t[PR];
};

template <int PD, int PR>
__device__ __forceinline__ RecRegs<PD, PR> load_rec(const NodeRec<PD, PR>& r) {
    RecRegs<PD, PR> x;
    x.e_fail = r.e_fail;
#pragma unroll
    for (int k = 0; k < PR; ++k) {
        x.e_prio[k] = r.e_prio[k];
        x.t[k] = r.t[k];
    }
    x.e_hv = r.e_hv;
    x.pen32 = r.pen32;
    x.flags = r.flags;
    return x;
}

// Filter + Score of one (pod, node) pair; returns the packed running key
// (score << 24 | 0xFFFFFF - i), or -1 when the pod may not go to the node.
template <int PD, int PR, bool DIVT = false>
__device__ __forceinline__ int32_t eval_pair(int64_t tnow, bool ds, const RecRegs<PD, PR>& x,
                                             const NodeRec<PD, PR>& r, int32_t i, double wsum, int32_t noprio,
                                             int32_t* score_out, double inv_w = 0.0, const double* thr = nullptr) {
    // Filter (plugins.go:55-66): some predicate fresh and over its limit
    const bool fail = tnow < x.e_fail;
    // getNodeScore (stats.go:124-135): fresh terms summed in policy order.
    // fma(1.0, t, s) == s + t exactly; fma(0.0, t, s) == s for finite t
    // (s is never -0.0), so a 0/1 mask replaces the select of the sum.
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < PR; ++k) {
        const double m = tnow < x.e_prio[k] ? 1.0 : 0.0;
        s = __builtin_fma(m, x.t[k], s);
    }
    int32_t base;
    bool in_range;
    if constexpr (DIVT) {
        // trunc(RN(s/W)) from q0 = RN(s * RN(1/W)): within 1, fixed by the thresholds.
        // For RN(s/W) < 1 this yields 0, which clamps to the same final score
        // as the reference's (<= 0) base since the penalty is >= 0 here.
        const double q0 = s * inv_w;
        in_range = q0 < kQFast;  // false for NaN; negative q0 clamps to k0 = 0
        int32_t k0;
        asm("v_cvt_i32_f64 %0, %1" : "=v"(k0) : "v"(q0));
        k0 = min(max(k0, 0), kQMax - 1);
        base = k0 + (s >= thr[k0 + 1] ? 1 : 0) - (s < thr[k0] ? 1 : 0);
    } else {
        const double q = s / wsum;
        in_range = __builtin_fabs(q) < kFastLim;  // false for NaN
        // v_cvt_i32_f64 truncates (saturating; lanes out of range take the exact path below)
        asm("v_cvt_i32_f64 %0, %1" : "=v"(base) : "v"(q));
    }
    // score - int(hotValue*10), NormalizeScore to [0,100] (plugins.go:91-93)
    const int32_t pen = tnow < x.e_hv ? x.pen32 : 0;
    int32_t f = min(max(base - pen, 0), 100);
    if ((x.flags & kRecSlow) || !in_range) f = score_exact<PD, PR>(tnow, r, wsum, noprio);
    if (score_out) *score_out = f;
    const bool feasible = ds || !fail;
    return feasible ? ((f << 24) | (0xFFFFFF - i)) : -1;
}

// V: 0 = plain loop, 1 = next record prefetched into SGPRs during the current
// one, 2 = two nodes per iteration.
template <int PD, int PR, bool MATRIX, int V>
__global__ __launch_bounds__(kK3Threads) void k3_eval(const NodeRec<PD, PR>* __restrict__ rec, int32_t N,
                                                      int32_t chunk, int64_t node_offset,
                                                      const int64_t* __restrict__ now, const uint8_t* __restrict__ flags,
                                                      int64_t P, double wsum, int32_t noprio,
                                                      long long* __restrict__ keys, MatrixOut mo, double inv_w,
                                                      const double* __restrict__ thr_g) {
    // V4: V3 + division-free threshold quotient (thr_g has kQMax + 1 entries)
    constexpr bool DIVT = V == 4;
    __shared__ double thr[DIVT ? kQMax + 1 : 1];
    if constexpr (DIVT) {
        for (int k = threadIdx.x; k <= kQMax; k += kK3Threads) thr[k] = thr_g[k];
        __syncthreads();
    }
    // V3: 1-D grid, XCD-aware.  Workgroups are dealt round-robin over the 8
    // XCDs (b % 8 shares an XCD), so give every XCD its own 1/8 of the node
    // chunks: each XCD's L2 then holds 1/8 of the record table.
    int64_t pg, ch;
    if constexpr (V == 3 || V == 4) {
        const int64_t b = blockIdx.x, slot = b >> 3, pgs = (P + kK3Threads - 1) / kK3Threads;
        pg = slot % pgs;
        ch = (b & 7) + 8 * (slot / pgs);
    } else {
        pg = blockIdx.x;
        ch = blockIdx.y;
    }
    const int64_t pod = pg * kK3Threads + threadIdx.x;
    const bool live = pod < P;
    const int64_t tnow = live ? now[pod] : INT64_MIN;
    const bool ds = live && flags && (flags[pod] & 1u);
    const int32_t n0 = (int32_t)min((int64_t)N, ch * chunk);
    const int32_t cnt = min(N - n0, chunk);
    const NodeRec<PD, PR>* __restrict__ r0 = rec + n0;
    int32_t best = -1;
    if constexpr (MATRIX) {
        for (int32_t i = 0; i < cnt; ++i) {
            const RecRegs<PD, PR> x = load_rec(r0[i]);
            int32_t f;
            best = max(best, eval_pair<PD, PR, DIVT>(tnow, ds, x, r0[i], i, wsum, noprio, &f, inv_w, thr));
            if (live) {
                int8_t ff = -1;
                if (!ds) {
#pragma unroll
                    for (int k = PD - 1; k >= 0; --k)
                        if (tnow < r0[i].e_pred[k]) ff = mo.pred_orig[k];
                }
                const int64_t n = n0 + i;
                if (mo.first_fail) mo.first_fail[pod * N + n] = ff;
                if (mo.score) mo.score[pod * N + n] = f;
            }
        }
    } else if constexpr (V == 1) {
        if (cnt > 0) {
            RecRegs<PD, PR> cur = load_rec(r0[0]);
            for (int32_t i = 0; i < cnt; ++i) {
                const int32_t j = i + 1 < cnt ? i + 1 : i;
                const RecRegs<PD, PR> nxt = load_rec(r0[j]);
                best = max(best, eval_pair<PD, PR>(tnow, ds, cur, r0[i], i, wsum, noprio, nullptr));
                cur = nxt;
            }
        }
    } else if constexpr (V == 2) {
        int32_t i = 0;
        for (; i + 1 < cnt; i += 2) {
            const RecRegs<PD, PR> a = load_rec(r0[i]);
            const RecRegs<PD, PR> b = load_rec(r0[i + 1]);
            const int32_t ka = eval_pair<PD, PR>(tnow, ds, a, r0[i], i, wsum, noprio, nullptr);
            const int32_t kb = eval_pair<PD, PR>(tnow, ds, b, r0[i + 1], i + 1, wsum, noprio, nullptr);
            best = max(best, max(ka, kb));
        }
        if (i < cnt) best = max(best, eval_pair<PD, PR>(tnow, ds, load_rec(r0[i]), r0[i], i, wsum, noprio, nullptr));
    } else {
        for (int32_t i = 0; i < cnt; ++i)
            best = max(best, eval_pair<PD, PR, DIVT>(tnow, ds, load_rec(r0[i]), r0[i], i, wsum, noprio, nullptr,
                                                     inv_w, thr));
    }
    if (live && best >= 0) {
        const int64_t sc = best >> 24;
        const int64_t n = n0 + (0xFFFFFF - (best & 0xFFFFFF));
        const long long key = (long long)((sc << 32) | (int64_t)(0xFFFFFFFFull - (uint64_t)(node_offset + n)));
        atomicMax(&keys[pod], key);
    }
}

// ---------------------------------------------------------------- launchers
int k1_threads() {
    // 256 by default: half the node blocks, so half the dedupe-form K2's (count,
    // offset) matrix and of K3s's producer-block scans (config 3: 0.0429 vs 0.0442 ms
    // per step); CRANE_K1_THREADS=128 selects the narrow variant
    const char* e = getenv("CRANE_K1_THREADS");
    return e && atoi(e) == 128 ? 128 : 256;
}

template <int PD, int PR>
static hipError_t launch_k1_t(const K1Args& a, const K1Step* step, hipStream_t st) {
    if (a.N <= 0) return hipSuccess;
    const int T = a.threads ? a.threads : k1_threads();
    if (T != 128 && T != 256) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)((a.N + T - 1) / T);
    const size_t lds = sizeof(NodeRec<PD, PR>) * T;
    const K1Step sa = step ? *step : K1Step{};
#define K1_LAUNCH(TT, S) hipLaunchKernelGGL((k1_node_pass<PD, PR, TT, S>), dim3(grid), dim3(TT), lds, st, a, sa)
    if (T == 256) {
        if (step) K1_LAUNCH(256, true);
        else K1_LAUNCH(256, false);
    } else {
        if (step) K1_LAUNCH(128, true);
        else K1_LAUNCH(128, false);
    }
#undef K1_LAUNCH
    return hipGetLastError();
}

hipError_t launch_node_pass(int shape, const K1Args& a, hipStream_t st, const K1Step* step) {
    switch (shape) {
        case kShape4x6: return launch_k1_t<4, 6>(a, step, st);
        case kShape8x8: return launch_k1_t<8, 8>(a, step, st);
        default: return launch_k1_t<16, 16>(a, step, st);
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
    hipLaunchKernelGGL(k2_hot_count, dim3(grid), dim3(kK2Threads), lds, st, bnode, bts, B, N, cut, buckets);
    return hipGetLastError();
}

// Tuning knobs read per launch (for A/B runs): CRANE_K3_VARIANT, CRANE_K3_ROUNDS.
static int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return e && *e ? atoi(e) : dflt;
}
int k3_variant() { return env_int("CRANE_K3_VARIANT", 5); }

int64_t eval_chunk_nodes(int64_t P, int64_t N) {
    // Size the grid to whole residency rounds: 256 CUs x 8 blocks of 4 waves
    // (8 waves/SIMD at <= 64 VGPRs) = 2048 resident blocks per round.
    int rounds = env_int("CRANE_K3_ROUNDS", 16);
    if (rounds < 1) rounds = 16;
    const int64_t pod_blocks = (P + kK3Threads - 1) / kK3Threads;
    int64_t chunks = (2048LL * rounds) / pod_blocks;
    if (chunks < 1) chunks = 1;
    int64_t chunk = (N + chunks - 1) / chunks;
    if (chunk < 64) chunk = 64;
    if (chunk > (1 << 24)) chunk = 1 << 24;  // the running key keeps 24 bits of local index
    return chunk;
}

template <int PD, int PR>
static hipError_t launch_k3_t(const void* rec, int64_t N, int64_t node_offset, const int64_t* now,
                              const uint8_t* flags, int64_t P, double wsum, int32_t noprio, long long* keys,
                              const MatrixOut& mo, double inv_w, const double* thr, hipStream_t st) {
    if (P <= 0 || N <= 0) return hipSuccess;
    if (N > 0x7FFFFFFF) return hipErrorInvalidValue;
    const int64_t chunk = eval_chunk_nodes(P, N);
    const dim3 grid((unsigned)((P + kK3Threads - 1) / kK3Threads), (unsigned)((N + chunk - 1) / chunk));
    const auto* r = static_cast<const NodeRec<PD, PR>*>(rec);
    const int32_t n32 = (int32_t)N, c32 = (int32_t)chunk;
    const bool matrix = mo.first_fail || mo.score;
    int v = k3_variant();
    if (v == 5) v = 4;  // the step path (step.hip) serves keys-only launches; matrix output uses V4
    if (v == 4 && !thr) v = 3;  // no threshold table for this policy (weight sum <= 0 or no priorities)
    if (matrix && (v == 1 || v == 2)) v = 0;
    // V3/V4 use a 1-D XCD-swizzled grid with the chunk count padded to a multiple of 8
    const unsigned chunks8 = (grid.y + 7) / 8 * 8;
    const dim3 g1(grid.x * chunks8), blk(kK3Threads);
#define K3_LAUNCH(M, V, G)                                                                                     \
    hipLaunchKernelGGL((k3_eval<PD, PR, M, V>), G, blk, 0, st, r, n32, c32, node_offset, now, flags, P, wsum, \
                       noprio, keys, mo, inv_w, thr)
    if (matrix) {
        if (v == 4) K3_LAUNCH(true, 4, g1);
        else if (v == 3) K3_LAUNCH(true, 3, g1);
        else K3_LAUNCH(true, 0, grid);
    } else {
        switch (v) {
            case 1: K3_LAUNCH(false, 1, grid); break;
            case 2: K3_LAUNCH(false, 2, grid); break;
            case 3: K3_LAUNCH(false, 3, g1); break;
            case 4: K3_LAUNCH(false, 4, g1); break;
            default: K3_LAUNCH(false, 0, grid); break;
        }
    }
#undef K3_LAUNCH
    return hipGetLastError();
}

hipError_t launch_eval(int shape, const void* rec, int64_t N, int64_t node_offset, const int64_t* now,
                       const uint8_t* flags, int64_t P, double wsum, int32_t noprio, long long* keys,
                       const MatrixOut& mo, double inv_w, const double* thr, hipStream_t st) {
    switch (shape) {
        case kShape4x6:
            return launch_k3_t<4, 6>(rec, N, node_offset, now, flags, P, wsum, noprio, keys, mo, inv_w, thr, st);
        case kShape8x8:
            return launch_k3_t<8, 8>(rec, N, node_offset, now, flags, P, wsum, noprio, keys, mo, inv_w, thr, st);
        default:
            return launch_k3_t<16, 16>(rec, N, node_offset, now, flags, P, wsum, noprio, keys, mo, inv_w, thr, st);
    }
}

}  // namespace crane
