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
    int32_t pred_slot[kMaxPred];
    double pred_limit[kMaxPred];
    int64_t pred_dur[kMaxPred];   // period + 5m (getActiveDuration, stats.go:140-150)
    int32_t prio_slot[kMaxPrio];
    double prio_w[kMaxPrio];
    int64_t prio_dur[kMaxPrio];
    int32_t win_pos[kMaxWin];     // window w -> rank of its cutoff in ascending order
    int64_t win_count[kMaxWin];   // hotValue.count
    int64_t win_cut_sorted[kMaxWin];  // ascending cutoffs (set per refresh)
};

// Pod-invariant per-node record.  All "fresh" tests become `now < expiry`,
// exactly the reference's now.Before(ts + dur) (stats.go:42-48).  An expiry of
// INT64_MIN never passes, which encodes every time-independent error (missing
// key, malformed value, negative value) and, for predicates, "not over the
// limit" — so predicate k fails iff now < e_pred[k], and the Filter rejects
// iff now < e_fail = max_k e_pred[k] (some overloaded predicate is fresh).
// The hot part (first) is all the pod x node kernel reads on its fast path.
template <int PD, int PR>
struct alignas(16) NodeRec {
    // --- hot
    int64_t e_fail;      // max over overloaded predicates of ts+dur, INT64_MIN if none
    int64_t e_hv;        // hot value annotation ts + 5m, INT64_MIN if unusable
    int32_t pen32;       // int(hotValue*10) when 0 <= it < 2^30 (fast path), else 0
    int32_t flags;       // kRecSlow: take the exact int64 path for this node
    int64_t e_prio[PR];  // ts+dur of the priority's metric, INT64_MIN if unusable
    double t[PR];        // ((1 - usage) * weight) * 100, stats.go:89 (no FMA)
    // --- cold (first-fail outputs and the exact path)
    int64_t pen;         // int(hotValue * 10), plugins.go:91
    int64_t e_pred[PD];  // ts+dur if usage > maxLimitPecent (and limit != 0), else INT64_MIN
};

// NodeRec.flags: a term is non-finite, pen is outside [0, 2^30), or the policy
// has no priorities.
constexpr int32_t kRecSlow = 1;
// K3 fast path: |int(score/weight)| < 2^30 and 0 <= pen < 2^30, so the
// reference's int64 "score - pen" cannot wrap and fits in int32.
constexpr double kFastLim = 1073741824.0;
// Exact int(score/weight) without a division (K3 "threshold" path, weight sum
// W > 0): T[k] = smallest double s with RN(s/W) >= k, k = 1..kQMax+1, T[0] =
// -inf.  trunc(s * RN(1/W)) is within 1 of trunc(RN(s/W)), and two compares
// against T fix it up.  Lanes with s * RN(1/W) >= kQFast take the exact path.
constexpr int kQMax = 127;
constexpr double kQFast = 125.0;
// K1 marks a node slow when a term is this large, keeping the sum finite.
constexpr double kTermMax = 1152921504606846976.0;  // 2^60

}  // namespace crane
