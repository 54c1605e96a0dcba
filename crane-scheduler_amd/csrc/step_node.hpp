// step_node.hpp — per-node part of the K3 step path (step.hip), shared by the
// stand-alone step-table kernel K3a and the fused node pass K1+K3a
// (kernels.hip), which builds the step tables straight from the NodeRec it
// has just computed in registers.
//
// A node's packed key (score << 24 | 0xFFFFFF - node, -1 = the pod may not go
// there) is a step function of the pod's `now`; over a batch whose times lie
// in [tmin, tmax] only the node's expiries inside (tmin, tmax] can change it.
// A node with none is "flat": its key is the same for every pod of a kind and
// only enters the workgroup's flat max.  Otherwise the node appends a Step1
// (one step) or VRec (more) record to its kind's compact list.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "dyn_types.hpp"
#include "kernels.hpp"

namespace crane {

// Producer block of workgroup b of nb: workgroups are dispatched round-robin
// over the 8 XCDs, so XCD x gets a contiguous run of blocks (its L2 then
// shares the cache lines of neighbouring blocks' inputs).  A bijection on [0, nb).
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nb) {
    const int64_t x = b & 7, q = b >> 3, per = nb >> 3, rem = nb & 7;
    return x * per + (x < rem ? x : rem) + q;
}

__device__ __forceinline__ int32_t pack_key(int32_t f, int64_t n) { return (f << 24) | (int32_t)(0xFFFFFF - n); }

// Exact clamped Score of (pod at time t, node) — the literal int64 restatement
// of stats.go:114-138 + plugins.go:91-93, the semantics of K3's eval_pair and
// score_exact (kernels.hip).
template <int PD, int PR>
__device__ __forceinline__ int32_t score_at(int64_t t, const NodeRec<PD, PR>& r, double wsum, int32_t noprio) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < PR; ++k)
        if (t < r.e_prio[k]) s += r.t[k];  // stats.go:124-133, policy order
    int64_t base = 0;
    if (!noprio) {
        const double q = s / wsum;  // stats.go:135 int(score / weight), Go CVTTSD2SQ
        base = (q >= -9223372036854775808.0 && q < 9223372036854775808.0) ? (int64_t)q : INT64_MIN;
    }
    const int64_t pen = t < r.e_hv ? r.pen : 0;
    const int64_t f = (int64_t)((uint64_t)base - (uint64_t)pen);  // plugins.go:91, wraps like Go
    return (int32_t)(f < 0 ? 0 : (f > 100 ? 100 : f));            // NormalizeScore (utils.go:58-68)
}

// Filter (plugins.go:41-43, 55-66) + packed key for pod kind T (0: Filter applies, 1: DaemonSet)
template <int PD, int PR>
__device__ __forceinline__ int32_t key_of(int T, int64_t t, int32_t score, const NodeRec<PD, PR>& r, int64_t n) {
    return (T == 1 || !(t < r.e_fail)) ? pack_key(score, n) : -1;
}

// Batch time range [tmin, tmax] from K3p's per-tile partials, in two parts so
// a kernel can issue the loads early and reduce after its own loads:
// batch_range_load (per-thread partials), batch_range_reduce (every thread of
// the workgroup gets the result; sm*: >= BS/64 LDS entries; has a barrier).
template <int BS>
__device__ __forceinline__ void batch_range_load(const int64_t* __restrict__ tile_mm, int32_t ntiles, int64_t& mn,
                                                 int64_t& mx) {
    mn = INT64_MAX;
    mx = INT64_MIN;
    for (int i = threadIdx.x; i < ntiles; i += BS) {
        mn = min(mn, tile_mm[2 * i]);
        mx = max(mx, tile_mm[2 * i + 1]);
    }
}
template <int BS>
__device__ __forceinline__ void batch_range_reduce(int64_t mn, int64_t mx, int64_t* smn, int64_t* smx, int64_t& tmin,
                                                   int64_t& tmax) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        mn = min(mn, (int64_t)__shfl_xor((long long)mn, o));
        mx = max(mx, (int64_t)__shfl_xor((long long)mx, o));
    }
    if ((threadIdx.x & 63) == 0) {
        smn[threadIdx.x >> 6] = mn;
        smx[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    tmin = smn[0];
    tmax = smx[0];
#pragma unroll
    for (int i = 1; i < BS / 64; ++i) {
        tmin = min(tmin, smn[i]);
        tmax = max(tmax, smx[i]);
    }
}
template <int BS>
__device__ __forceinline__ void batch_range(const int64_t* __restrict__ tile_mm, int32_t ntiles, int64_t* smn,
                                            int64_t* smx, int64_t& tmin, int64_t& tmax) {
    int64_t mn, mx;
    batch_range_load<BS>(tile_mm, ntiles, mn, mx);
    batch_range_reduce<BS>(mn, mx, smn, smx, tmin, tmax);
}

// Per node and pod kind: the flat key (-1 if stepped or never feasible) and,
// for a stepped node, its slot in the workgroup's span of the kind's list.
// Phase 1 (step_count) only classifies — cheap and register-light, so it can
// run inside the node pass; phase 2 (step_emit) rebuilds the record of a
// stepped node after the workgroup has reserved its list spans.
struct StepSlots {
    int32_t flat0 = -1, flat1 = -1;
    int32_t slot0 = -1, slot1 = -1;  // >= 0: stepped
    bool multi0 = false, multi1 = false;
};

// Workgroup-shared counters of the step epilogue.
struct StepShared {
    int32_t lc[2][2];   // records per kind: [Step1, VRec]
    int32_t fm[2][16];  // per-wave flat maxima (<= 1024 threads)
};

// The node's expiries for kind T with those outside (tmin, tmax] replaced by
// INT64_MAX; returns their count and the min / max of the in-range ones.
template <int PD, int PR, int T>
__device__ __forceinline__ void step_points(const NodeRec<PD, PR>& r, int64_t tmin, int64_t tmax, int64_t* c,
                                            int& cnt, int64_t& mn, int64_t& mx) {
    constexpr int NB = PR + 2;
#pragma unroll
    for (int k = 0; k < PR; ++k) c[k] = r.e_prio[k];
    c[PR] = r.e_hv;
    c[PR + 1] = T == 0 ? r.e_fail : INT64_MIN;  // DaemonSet pods bypass the Filter
    cnt = 0;
    mn = INT64_MAX;
    mx = INT64_MIN;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        const bool in = c[j] > tmin && c[j] <= tmax;
        c[j] = in ? c[j] : INT64_MAX;
        cnt += in;
        mn = min(mn, c[j]);
        mx = in ? max(mx, c[j]) : mx;
    }
}

// Phase 1.  A node with one distinct in-range expiry (a predicate's expiry
// equals its metric's priority expiry when both use one metric) is a Step1.
template <int PD, int PR>
__device__ __forceinline__ void step_count(const NodeRec<PD, PR>& r, int64_t n, int64_t tmin, int64_t tmax,
                                           double wsum, int32_t noprio, StepShared& sh, StepSlots& o) {
    const int32_t s0 = score_at<PD, PR>(tmin, r, wsum, noprio);
    auto kind = [&](auto Tc, int32_t& flat, int32_t& slot, bool& multi) {
        constexpr int T = decltype(Tc)::value;
        int64_t c[PR + 2], mn, mx;
        int cnt;
        step_points<PD, PR, T>(r, tmin, tmax, c, cnt, mn, mx);
        flat = cnt == 0 ? key_of<PD, PR>(T, tmin, s0, r, n) : -1;
        multi = mn != mx;
        slot = cnt == 0 ? -1 : atomicAdd(&sh.lc[T][multi ? 1 : 0], 1);
    };
    kind(std::integral_constant<int, 0>{}, o.flat0, o.slot0, o.multi0);
    kind(std::integral_constant<int, 1>{}, o.flat1, o.slot1, o.multi1);
}

// Phase 2: write node n's record(s) into the workgroup's region.
template <int PD, int PR>
__device__ __forceinline__ void step_emit(const NodeRec<PD, PR>& r, int64_t n, int64_t tmin, int64_t tmax,
                                          double wsum, int32_t noprio, const StepSlots& o,
                                          const StepTables& st, int64_t blk) {
    constexpr int NB = PR + 2;
    auto kind = [&](auto Tc, int32_t slot, bool multi) {
        constexpr int T = decltype(Tc)::value;
        if (slot < 0) return;
        int64_t c[NB], mn, mx;
        int cnt;
        step_points<PD, PR, T>(r, tmin, tmax, c, cnt, mn, mx);
        const int32_t k0 = key_of<PD, PR>(T, tmin, score_at<PD, PR>(tmin, r, wsum, noprio), r, n);
        // key of the step starting at an expiry, evaluated at its first instant
        if (!multi) {
            Step1 v;
            v.bp = mn;
            v.k0 = k0;
            v.k1 = key_of<PD, PR>(T, mn, score_at<PD, PR>(mn, r, wsum, noprio), r, n);
            st.single[(int64_t)T * st.npad + blk * st.bs + slot] = v;
        } else {  // rare: sort the expiries (equal ones give equal keys)
#pragma unroll
            for (int i = 0; i < NB; ++i)  // odd-even transposition sort (static indices)
#pragma unroll
                for (int j = i & 1; j + 1 < NB; j += 2) {
                    const int64_t x = c[j], y = c[j + 1];
                    c[j] = min(x, y);
                    c[j + 1] = max(x, y);
                }
            VRec<NB> v;
            v.cnt = cnt;
            v.key[0] = k0;
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                v.bp[j] = c[j];  // INT64_MAX past cnt: never selected
                v.key[j + 1] = j < cnt ? key_of<PD, PR>(T, c[j], score_at<PD, PR>(c[j], r, wsum, noprio), r, n) : -1;
            }
            reinterpret_cast<VRec<NB>*>(st.multi)[(int64_t)T * st.npad + blk * st.bs + slot] = v;
        }
    };
    kind(std::integral_constant<int, 0>{}, o.slot0, o.multi0);
    kind(std::integral_constant<int, 1>{}, o.slot1, o.multi1);
}

// Phase 2, one (node, kind) item with the kind at run time: the fused node pass
// compacts its stepped items into a workgroup list (step_queue) so a few lanes
// of one wave build every record, instead of each wave paying both kinds' and
// both record forms' code paths whenever one of its lanes is stepped.
template <int PD, int PR>
__device__ __forceinline__ void step_emit_one(const NodeRec<PD, PR>& r, int64_t n, int T, int32_t slot, bool multi,
                                              int64_t tmin, int64_t tmax, double wsum, int32_t noprio,
                                              const StepTables& st, int64_t blk) {
    constexpr int NB = PR + 2;
    int64_t c[NB];
#pragma unroll
    for (int k = 0; k < PR; ++k) c[k] = r.e_prio[k];
    c[PR] = r.e_hv;
    c[PR + 1] = T == 0 ? r.e_fail : INT64_MIN;  // DaemonSet pods bypass the Filter
    int cnt = 0;
    int64_t mn = INT64_MAX;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        const bool in = c[j] > tmin && c[j] <= tmax;
        c[j] = in ? c[j] : INT64_MAX;
        cnt += in;
        mn = min(mn, c[j]);
    }
    auto key = [&](int64_t t) {  // key_of for the run-time kind
        const int32_t f = score_at<PD, PR>(t, r, wsum, noprio);
        return (T == 1 || !(t < r.e_fail)) ? pack_key(f, n) : -1;
    };
    const int32_t k0 = key(tmin);
    if (!multi) {
        Step1 v;
        v.bp = mn;
        v.k0 = k0;
        v.k1 = key(mn);
        st.single[(int64_t)T * st.npad + blk * st.bs + slot] = v;
    } else {
#pragma unroll
        for (int i = 0; i < NB; ++i)  // odd-even transposition sort (static indices)
#pragma unroll
            for (int j = i & 1; j + 1 < NB; j += 2) {
                const int64_t x = c[j], y = c[j + 1];
                c[j] = min(x, y);
                c[j + 1] = max(x, y);
            }
        VRec<NB> v;
        v.cnt = cnt;
        v.key[0] = k0;
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            v.bp[j] = c[j];
            v.key[j + 1] = j < cnt ? key(c[j]) : -1;
        }
        reinterpret_cast<VRec<NB>*>(st.multi)[(int64_t)T * st.npad + blk * st.bs + slot] = v;
    }
}

// Work item of the compacted emit: owner thread | kind << 12 | multi << 13 | slot << 14.
__device__ __forceinline__ void step_queue(const StepSlots& o, int32_t* nq, uint32_t* q) {
    if (o.slot0 >= 0) q[atomicAdd(nq, 1)] = threadIdx.x | ((uint32_t)o.multi0 << 13) | ((uint32_t)o.slot0 << 14);
    if (o.slot1 >= 0)
        q[atomicAdd(nq, 1)] = threadIdx.x | (1u << 12) | ((uint32_t)o.multi1 << 13) | ((uint32_t)o.slot1 << 14);
}

// Workgroup epilogue: the workgroup's flat-key maxima and record counts go to
// its own slots (producer block blk) of the step tables (plain stores, no global atomics).  Every
// thread calls it (barrier); sh.lc must have been zeroed before step_count.
template <int BS>
__device__ __forceinline__ void step_publish(const StepSlots& o, StepShared& sh, const StepTables& st, int64_t blk) {
    auto wmax = [&](int T, int32_t m) {
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) m = max(m, __shfl_xor(m, s));
        if ((threadIdx.x & 63) == 0) sh.fm[T][threadIdx.x >> 6] = m;
    };
    wmax(0, o.flat0);
    wmax(1, o.flat1);
    __syncthreads();
    if (threadIdx.x < 2) {
        const int T = threadIdx.x;
        int32_t m = sh.fm[T][0];
#pragma unroll
        for (int i = 1; i < BS / 64; ++i) m = max(m, sh.fm[T][i]);
        st.flat[blk * 2 + T] = m;
    } else if (threadIdx.x < 6) {
        const int L = threadIdx.x - 2;
        st.cnt[blk * 4 + L] = sh.lc[L >> 1][L & 1];
    }
}

}  // namespace crane
