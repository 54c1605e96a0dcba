// dyn_types.hpp — device policy table and node record shared by the host
// engine (engine.hip) and the kernels (kernels.hip).
//
// The reference evaluates Filter/Score by re-parsing node annotation strings
// on every (pod, node) call (pkg/plugins/dynamic/stats.go:51-76).  Here the
// host parses once per sync into SoA rows; the node pass (K1) then folds
// everything that does not depend on the pod into one fixed-layout NodeRec
// per node, and the pod x node kernel (K3) reads NodeRecs through the scalar
// cache (a record is uniform across the 64 pods of a wave).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace crane {

constexpr int kMaxPred = 16;   // device predicate checks
constexpr int kMaxPrio = 16;   // device priority terms
constexpr int kMaxSlots = 32;  // distinct metric keys
constexpr int kMaxWin = 8;     // hotValue windows
constexpr int kLdsWin = 4;     // windows the LDS-aggregating K2 handles
constexpr int64_t kTsInvalid = INT64_MIN;
constexpr int64_t kHotActiveNs = 5LL * 60 * 1000000000LL;    // stats.go:24
constexpr int64_t kExtraActiveNs = 5LL * 60 * 1000000000LL;  // stats.go:26

// Flattened DynamicSchedulerPolicy as the kernels see it (kernel argument).
struct DevPolicy {
    int32_t n_slots;  // metric rows in the uploaded SoA
    int32_t npd;      // predicates with an active duration (policy order kept)
    int32_t npr;      // priorities with an active duration (policy order kept)
    int32_t n_win;    // hotValue windows
    int32_t noprio;   // policy has no priorities at all -> node score 0 (stats.go:116-120)
    int32_t pad0;
    double wsum;      // sum of ALL priority weights in policy order (stats.go:131)
    double winv;      // 1 / wsum when |wsum| is a normal power of two (exact reciprocal), else 0
    int32_t pred_slot[kMaxPred];
    double pred_limit[kMaxPred];
    int64_t pred_dur[kMaxPred];   // period + 5m (getActiveDuration, stats.go:140-150)
    int32_t prio_slot[kMaxPrio];
    double prio_w[kMaxPrio];
    int64_t prio_dur[kMaxPrio];
    int32_t win_pos[kMaxWin];     // window w -> rank of its cutoff in ascending order
    int64_t win_count[kMaxWin];   // hotValue.count
    int64_t win_cut_sorted[kMaxWin];  // ascending cutoffs (set per refresh)
    // by cutoff rank r (set per refresh): the window, and hotValue.count as an exact u32
    // division by multiply-high when 1 <= count < 2^32 (win_div_m = 0: int64 division)
    int32_t win_of_rank[kMaxWin];
    uint32_t win_div_m[kMaxWin];
    int32_t win_div_sh[kMaxWin];  // sh1 | sh2 << 8
};

// n / d for the d the magic (m, sh) was made for (round-up method, exact for every
// u32 n): t = mulhi(m, n); q = (t + ((n - t) >> sh1)) >> sh2
__host__ __device__ inline uint32_t div_magic(uint32_t n, uint32_t m, int32_t sh) {
    const uint32_t t = (uint32_t)(((uint64_t)m * n) >> 32);
    return (t + ((n - t) >> (sh & 0xFF))) >> (sh >> 8);
}
// magic for 1 <= d < 2^32: l = ceil(log2 d), m = floor(2^32 (2^l - d) / d) + 1
inline void make_div_magic(uint32_t d, uint32_t* m, int32_t* sh) {
    int l = 0;
    while (l < 32 && (1ull << l) < d) ++l;
    *m = (uint32_t)((((uint64_t)1 << 32) * ((1ull << l) - d)) / d + 1);
    *sh = (l < 1 ? l : 1) | ((l - 1 > 0 ? l - 1 : 0) << 8);
}

// Pod-invariant per-node record.  All "fresh" tests become `now < expiry`,
// exactly the reference's now.Before(ts + dur) (stats.go:42-48).  An expiry of
// INT64_MIN never passes, which encodes every time-independent error (missing
// key, malformed value, negative value) and, for predicates, "not over the
// limit" — so predicate k fails iff now < e_pred[k], and the Filter rejects
// iff now < e_fail = max_k e_pred[k] (some overloaded predicate is fresh).
template <int PD, int PR>
struct alignas(16) NodeRec {
    int64_t e_fail;      // max over overloaded predicates of ts+dur, INT64_MIN if none
    int64_t e_hv;        // hot value annotation ts + 5m, INT64_MIN if unusable
    int64_t pen;         // int(hotValue * 10), plugins.go:91
    int64_t e_prio[PR];  // ts+dur of the priority's metric, INT64_MIN if unusable
    double t[PR];        // ((1 - usage) * weight) * 100, stats.go:89 (no FMA)
    int64_t e_pred[PD];  // ts+dur if usage > maxLimitPecent (and limit != 0), else INT64_MIN
};

}  // namespace crane
