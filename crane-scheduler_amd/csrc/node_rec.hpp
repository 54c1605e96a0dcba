// node_rec.hpp — a node's pod-invariant record (NodeRec) from its parsed
// annotations, shared by the node pass K1 (kernels.hip) and the scatter update
// of changed nodes (update.hip), so both compute it with the same instructions.
//
// Numerics follow /root/reference/pkg/plugins/dynamic/stats.go bit for bit:
// fp64 in the reference's operation order with no FMA contraction (the build
// uses -ffp-contract=off), Go's float64->int conversion and saturating expiry
// sums.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dyn_types.hpp"

namespace crane {

// Go int(float64) on amd64 (CVTTSD2SQ): NaN and out-of-range -> INT64_MIN.
// Used by stats.go:135 (int(score/weight)) and plugins.go:91 (int(hv*10)).
__device__ __forceinline__ int64_t go_int(double x) {
    if (!(x >= -9223372036854775808.0 && x < 9223372036854775808.0)) return INT64_MIN;
    return (int64_t)x;
}

__device__ __forceinline__ int64_t sat_add(int64_t a, int64_t b) {
    int64_t r;
    const bool o = __builtin_add_overflow(a, b, &r);
    return o ? (b > 0 ? INT64_MAX : INT64_MIN) : r;  // (selects: no branch around a caller's loads)
}

// Predicate and priority parts of the record from the metric rows the policy reads
// (pt / pv: predicate k's (ts, value); qt / qv: priority k's), then e_fail.
template <int PD, int PR>
__device__ __forceinline__ void rec_metrics(const DevPolicy& pol, const int64_t (&pt)[PD], const double (&pv)[PD],
                                            const int64_t (&qt)[PR], const double (&qv)[PR], NodeRec<PD, PR>& r) {
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
}

// Hot-value part from the node_hot_value annotation (getNodeHotValue, stats.go:152-166:
// no extra active period; an unusable or negative value counts as 0).
template <int PD, int PR>
__device__ __forceinline__ void rec_hot_annotation(double h, int64_t t, NodeRec<PD, PR>& r) {
    r.pen = go_int(h * 10.0);
    r.e_hv = (t != kTsInvalid && !(h < 0.0)) ? sat_add(t, kHotActiveNs) : kTsInvalid;
}

// Hot-value part of the record from the node's K2 window-rank buckets bc[r]
// (annotateNodeHotValue, node.go:113-121: value += count / p.Count, Go int division;
// window w counts the bindings of buckets >= its cutoff rank): one running suffix sum.
// cnt_out / hvc_out (null: not kept): the per-window counts and the value.
template <int PD, int PR, int NW = 0>
__device__ __forceinline__ void rec_hot_counts(const DevPolicy& pol, const uint32_t (&bc)[kMaxWin], int64_t N, int64_t n,
                                               uint32_t* __restrict__ cnt_out, double* __restrict__ hvc_out,
                                               int64_t hv_ts_counts, NodeRec<PD, PR>& r) {
    int64_t v = 0;
    uint64_t suf = 0;
#pragma unroll
    for (int k = kMaxWin - 1; k >= 0; --k) {
        if (k >= (NW ? NW : pol.n_win)) continue;  // (NW: the policy's window count, static)
        // (the rank's words read before any branch or store: one wait for the three)
        const int w = pol.win_of_rank[k];
        const uint32_t dm = pol.win_div_m[k];
        const int32_t dsh = pol.win_div_sh[k];
        suf += bc[k];
        const uint32_t q = div_magic((uint32_t)suf, dm, dsh);
        if (cnt_out) cnt_out[(int64_t)w * N + n] = (uint32_t)suf;
        // Go int division (truncates toward 0): exact multiply-high division when the
        // count fits 32 bits and hotValue.count is in [1, 2^32)
        if (dm != 0 && suf <= 0xFFFFFFFFull)
            v += (int64_t)q;
        else
            v += (int64_t)suf / pol.win_count[w];
    }
    // the plugin re-reads it via ParseFloat (exact) and rejects negatives (stats.go:71-73)
    const double h = (double)v;
    if (hvc_out) hvc_out[n] = h;  // kept for node passes after the buckets are consumed
    r.pen = go_int(h * 10.0);
    r.e_hv = v >= 0 ? sat_add(hv_ts_counts, kHotActiveNs) : kTsInvalid;
}

// The Filter rejects iff now < e_fail = max over the predicates' expiries.
template <int PD, int PR>
__device__ __forceinline__ void rec_fail(NodeRec<PD, PR>& r) {
    int64_t e_fail = kTsInvalid;
#pragma unroll
    for (int k = 0; k < PD; ++k) e_fail = max(e_fail, r.e_pred[k]);
    r.e_fail = e_fail;
}

}  // namespace crane
