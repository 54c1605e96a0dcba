// node_steps.hpp — one node's Filter / Score answers as step functions of the pod's time
// over [t0, t1) (the drop-in plugin's table rows: crane_dyn_node_steps and its subset /
// update forms).  A node's Filter (first failing predicate, plugins.go:55-66) and Score
// (stats.go:114-138 + plugins.go:91-93) change only where `now` crosses one of its
// expiries, so over [t0, t1) they are constant between the expiries inside it: the
// expiries in (t0, t1), sorted and deduplicated, and the values at t0 and at each of them
// (the same ff_at / score_at as every other path).
#pragma once
#include <hip/hip_runtime.h>

#include "dyn_types.hpp"
#include "kernels.hpp"
#include "step_node.hpp"

namespace crane {

// first failing predicate at time t, in policy order (plugins.go:55-66); -1 = none
template <int PD, int PR>
__device__ __forceinline__ int32_t ff_at(int64_t t, const NodeRec<PD, PR>& r, const MatrixArgs& a) {
    int32_t f = -1;
#pragma unroll
    for (int k = PD - 1; k >= 0; --k)
        if (t < r.e_pred[k]) f = a.pred_orig[k];
    return f;
}

// row n of the table: ns[n] breakpoints bp[n * S + j], values ff / sc[n * (S + 1) + j]
template <int PD, int PR>
__device__ __forceinline__ void node_steps_row(const NodeRec<PD, PR>& r, const MatrixArgs& a, int64_t t0, int64_t t1,
                                               int64_t n, uint8_t* __restrict__ ns, int64_t* __restrict__ bp,
                                               int8_t* __restrict__ ffv, int8_t* __restrict__ scv) {
    constexpr int S = PD + PR + 1;
    int64_t e[S];
    int c = 0;
    auto put = [&](int64_t x) {
        if (x > t0 && x < t1) e[c++] = x;
    };
#pragma unroll
    for (int k = 0; k < PD; ++k) put(r.e_pred[k]);
#pragma unroll
    for (int k = 0; k < PR; ++k) put(r.e_prio[k]);
    put(r.e_hv);
    for (int i = 1; i < c; ++i) {  // insertion sort (at most S values)
        const int64_t x = e[i];
        int j = i - 1;
        while (j >= 0 && e[j] > x) {
            e[j + 1] = e[j];
            --j;
        }
        e[j + 1] = x;
    }
    int m = 0;
    for (int i = 0; i < c; ++i)
        if (m == 0 || e[i] != e[m - 1]) e[m++] = e[i];
    ns[n] = (uint8_t)m;
    ffv[n * (S + 1)] = (int8_t)ff_at<PD, PR>(t0, r, a);
    scv[n * (S + 1)] = (int8_t)score_at<PD, PR>(t0, r, a.wsum, a.noprio);
    for (int i = 0; i < m; ++i) {
        bp[n * S + i] = e[i];
        ffv[n * (S + 1) + i + 1] = (int8_t)ff_at<PD, PR>(e[i], r, a);
        scv[n * (S + 1) + i + 1] = (int8_t)score_at<PD, PR>(e[i], r, a.wsum, a.noprio);
    }
}

}  // namespace crane
