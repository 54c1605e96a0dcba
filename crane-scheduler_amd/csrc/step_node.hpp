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

// ---- wave primitives on DPP (VALU lane moves, no LDS round trip like ds_bpermute's
// __shfl*).  Every lane of the 64-lane wave must be active (uniform control flow).
// dpp_ctrl: quad_perm 0x00-0xFF, row_shr:k 0x110 + k, row_ror:k 0x120 + k, row_bcast:15 0x142,
// row_bcast:31 0x143; lanes whose source is outside the row keep `id` (bound_ctrl off).
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ int32_t dpp_or(int32_t id, int32_t v) {
    return __builtin_amdgcn_update_dpp(id, v, CTRL, ROWS, 0xF, false);
}
// maximum over the wave, uniform
__device__ __forceinline__ int32_t wave_max(int32_t v) {
    v = max(v, dpp_or<0xB1>(v, v));   // quad_perm [1,0,3,2]
    v = max(v, dpp_or<0x4E>(v, v));   // quad_perm [2,3,0,1]
    v = max(v, dpp_or<0x124>(v, v));  // row_ror:4
    v = max(v, dpp_or<0x128>(v, v));  // row_ror:8: every lane holds its row's maximum
    return max(max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
               max(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}
// inclusive prefix (lane order) under an associative op with identity id: Hillis-Steele
// within each row of 16, then rows 1 / 3 take row 0 / 2's total, rows 2-3 rows 0-1's
template <class Op>
__device__ __forceinline__ int32_t wave_scan(int32_t v, int32_t id, Op op) {
    v = op(v, dpp_or<0x111>(id, v));
    v = op(v, dpp_or<0x112>(id, v));
    v = op(v, dpp_or<0x114>(id, v));
    v = op(v, dpp_or<0x118>(id, v));
    v = op(v, dpp_or<0x142, 0xA>(id, v));
    v = op(v, dpp_or<0x143, 0xC>(id, v));
    return v;
}
__device__ __forceinline__ uint32_t wave_scan_add(uint32_t v) {
    return (uint32_t)wave_scan((int32_t)v, 0, [](int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); });
}
__device__ __forceinline__ int32_t wave_scan_max(int32_t v) {
    return wave_scan(v, INT32_MIN, [](int32_t a, int32_t b) { return max(a, b); });
}
// lane i takes lane (i ^ 1)'s value / lane i + 2's within its quad (lanes 0, 1 of a quad)
__device__ __forceinline__ int32_t quad_xor1(int32_t v) { return dpp_or<0xB1>(v, v); }
__device__ __forceinline__ int32_t quad_down2(int32_t v) { return dpp_or<0xEE>(v, v); }

// Exact clamped Score of (pod at time t, node) — the literal int64 restatement
// of stats.go:114-138 + plugins.go:91-93, the semantics of K3's eval_pair and
// score_exact (kernels.hip).
template <int PD, int PR>
// winv: 1 / wsum when |wsum| is a power of two (the default policy's weights sum to 2.0), else
// 0: the reciprocal is then exact and s * winv the same correctly rounded quotient as s / wsum,
// one multiply instead of the division sequence (a uniform branch).
__device__ __forceinline__ int32_t score_at(int64_t t, const NodeRec<PD, PR>& r, double wsum, int32_t noprio,
                                          double winv = 0.0);

// The score from the ordered sum s of the active priority terms and the active hot-value
// penalty pen (0 when inactive): score_at's tail, shared with the streamed count pass.
__device__ __forceinline__ int32_t score_of_sum(double s, int64_t pen, double wsum, int32_t noprio, double winv) {
    int64_t base = 0;
    if (!noprio) {
        const double q = winv != 0.0 ? s * winv : s / wsum;  // stats.go:135 int(score / weight), Go CVTTSD2SQ
        // |q| < 2^31 (every realistic score): one v_cvt_i32_f64 truncates toward zero exactly as
        // the 64-bit conversion does; otherwise the full CVTTSD2SQ restatement (NaN, overflow)
        if (__builtin_fabs(q) < 2147483648.0) base = (int64_t)(int32_t)q;
        else base = (q >= -9223372036854775808.0 && q < 9223372036854775808.0) ? (int64_t)q : INT64_MIN;
    }
    const int64_t f = (int64_t)((uint64_t)base - (uint64_t)pen);  // plugins.go:91, wraps like Go
    return (int32_t)(f < 0 ? 0 : (f > 100 ? 100 : f));            // NormalizeScore (utils.go:58-68)
}

template <int PD, int PR>
__device__ __forceinline__ int32_t score_at(int64_t t, const NodeRec<PD, PR>& r, double wsum, int32_t noprio,
                                          double winv) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < PR; ++k)
        if (t < r.e_prio[k]) s += r.t[k];  // stats.go:124-133, policy order
    return score_of_sum(s, t < r.e_hv ? r.pen : 0, wsum, noprio, winv);
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
        const int64_t* ts = tile_mm + kTileStat * i;
        mn = min(mn, min(ts[0], ts[2]));
        mx = max(mx, max(ts[1], ts[3]));
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
// Per-wave form (no LDS, no barrier): every wave reads all tile stats itself — lane l
// the tiles l, l + 64, ... — in two parts: batch_range_wave_load keeps the first two
// tiles' bounds in registers (issued early), batch_range_wave_reduce folds them, reads
// any further tiles and reduces over the wave.
struct TileBounds {
    int64_t mn[2], mx[2];
};
__device__ __forceinline__ void batch_range_wave_load(const int64_t* __restrict__ tile_mm, int32_t ntiles,
                                                      TileBounds& tb) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int i = lane + 64 * h;
        tb.mn[h] = INT64_MAX;
        tb.mx[h] = INT64_MIN;
        if (i < ntiles) {
            const int64_t* ts = tile_mm + kTileStat * i;
            tb.mn[h] = min(ts[0], ts[2]);
            tb.mx[h] = max(ts[1], ts[3]);
        }
    }
}
__device__ __forceinline__ void batch_range_wave_reduce(const int64_t* __restrict__ tile_mm, int32_t ntiles,
                                                        const TileBounds& tb, int64_t& tmin, int64_t& tmax) {
    int64_t mn = min(tb.mn[0], tb.mn[1]), mx = max(tb.mx[0], tb.mx[1]);
    for (int i = (threadIdx.x & 63) + 128; i < ntiles; i += 64) {
        const int64_t* ts = tile_mm + kTileStat * i;
        mn = min(mn, min(ts[0], ts[2]));
        mx = max(mx, max(ts[1], ts[3]));
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        mn = min(mn, (int64_t)__shfl_xor((long long)mn, o));
        mx = max(mx, (int64_t)__shfl_xor((long long)mx, o));
    }
    tmin = mn;
    tmax = mx;
}

template <int BS>
__device__ __forceinline__ void batch_range(const int64_t* __restrict__ tile_mm, int32_t ntiles, int64_t* smn,
                                            int64_t* smx, int64_t& tmin, int64_t& tmax) {
    int64_t mn, mx;
    batch_range_load<BS>(tile_mm, ntiles, mn, mx);
    batch_range_reduce<BS>(mn, mx, smn, smx, tmin, tmax);
}

// [lo, hi): the node's results are constant for every time in it (lo = latest expiry
// <= t, hi = earliest expiry > t; the comparisons are now < expiry)
template <int PD, int PR>
__device__ __forceinline__ void bracket(const NodeRec<PD, PR>& r, int64_t t, int64_t& lo, int64_t& hi) {
    lo = INT64_MIN;
    hi = INT64_MAX;
    auto upd = [&](int64_t e) {
        if (e <= t) lo = max(lo, e);
        else hi = min(hi, e);
    };
#pragma unroll
    for (int k = 0; k < PD; ++k) upd(r.e_pred[k]);
#pragma unroll
    for (int k = 0; k < PR; ++k) upd(r.e_prio[k]);
    upd(r.e_hv);
}

// exclusive workgroup scan (BT threads): wave scans + a scan of the wave totals
template <int BT = 256>
__device__ __forceinline__ uint32_t wg_excl_scan_u32(uint32_t v, uint32_t* part) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t x = wave_scan_add(v);  // (DPP lane moves: every thread of the workgroup calls this)
    if (lane == 63) part[w] = x;
    __syncthreads();
    uint32_t pre = 0;
#pragma unroll
    for (int i = 0; i < BT / 64; ++i) pre += i < w ? part[i] : 0u;
    __syncthreads();
    return pre + x - v;
}

__device__ __forceinline__ int64_t readlane64(int64_t v, int j) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, j);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), j);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Per node and pod kind: the flat key (-1 if stepped or never feasible) and,
// for a stepped node, its slots in the workgroup's spans of the kind's lists.
// Phase 1 (step_count) only classifies — cheap and register-light, so it can
// run inside the node pass; phase 2 (step_emit) rebuilds the record of a
// stepped node after the workgroup has reserved its list spans.
//
// A stepped node's key is piecewise constant over the batch: key_0 before its
// first in-range expiry c_0, key_j on [c_{j-1}, c_j), key_m from c_{m-1} on.
// It is published as pieces: two one-step records for the half-lines —
// (bp c_0: key_0 before, -1 after) and (bp c_{m-1}: -1 before, key_m after),
// or one (bp c_0: key_0 before, key_1 after) when m = 1 — and m - 1 middle
// pieces [c_j, c_{j+1}) with their keys.  The max over a node's pieces covering
// a time is its key then (a piece covers nothing outside its interval, -1).
struct StepSlots {
    int32_t flat0 = -1, flat1 = -1;
    int32_t slot0 = -1, slot1 = -1;    // >= 0: stepped (first one-step record slot)
    int32_t mslot0 = 0, mslot1 = 0;    // first middle-piece slot
    int8_t nb0 = 0, nb1 = 0;           // in-range expiries (with repeats): one-step record iff 1 distinct
    bool multi0 = false, multi1 = false;
};

// Workgroup-shared counters of the step epilogue.
struct StepShared {
    int32_t lc[2][2];   // per kind: [one-step records, middle pieces]
    int32_t fm[2][16];  // per-wave flat maxima (<= 1024 threads)
    int32_t pn[2];      // per kind: elementary pieces after step_pieces, -1 = raw pieces
};

// Phase 1.  A node with one distinct in-range expiry (a predicate's expiry
// equals its metric's priority expiry when both use one metric) is one record;
// otherwise two half-line records and cnt - 1 middle-piece slots are reserved
// (repeated expiries give empty pieces, harmless: they cover no time).
template <int PD, int PR>
__device__ __forceinline__ void step_count(const NodeRec<PD, PR>& r, int64_t n, int64_t tmin, int64_t tmax,
                                           double wsum, int32_t noprio, StepShared& sh, StepSlots& o) {
    const int32_t s0 = score_at<PD, PR>(tmin, r, wsum, noprio);
    // the in-range expiries both kinds share (priorities, hot value), then e_fail for kind 0
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
    auto kind = [&](auto Tc, int32_t& flat, int32_t& slot, int32_t& mslot, int8_t& nb, bool& multi) {
        constexpr int T = decltype(Tc)::value;
        const int cnt = T ? cnt1 : cnt0;
        const int64_t mn = T ? mn1 : mn0, mx = T ? mx1 : mx0;
        flat = cnt == 0 ? key_of<PD, PR>(T, tmin, s0, r, n) : -1;
        multi = cnt > 0 && mn != mx;  // (cnt == 0: mn = INT64_MAX, mx = INT64_MIN)
        nb = (int8_t)cnt;
        slot = cnt == 0 ? -1 : atomicAdd(&sh.lc[T][0], multi ? 2 : 1);
        mslot = multi ? atomicAdd(&sh.lc[T][1], cnt - 1) : 0;
    };
    kind(std::integral_constant<int, 0>{}, o.flat0, o.slot0, o.mslot0, o.nb0, o.multi0);
    kind(std::integral_constant<int, 1>{}, o.flat1, o.slot1, o.mslot1, o.nb1, o.multi1);
}

// Phase 2, one (node, kind): the node's one-step records go to the workgroup's
// staging (S1Out) (LDS, or st.stage when the block's records exceed the
// LDS staging; step_sort_publish writes them out sorted), its middle pieces
// straight to st.mid.
// Where a block's one-step records go: its LDS staging (lds, kind stride kl) or, when the block
// holds more of a kind than that takes (g, workgroup-uniform), st.stage (glb, stride kg).  Two
// stores with known address spaces: one store through a pointer selected between LDS and global
// is a flat store, which goes down the vector memory path even for LDS (round 5: the streamed
// pass's emit 2.6 -> 1.3 us per workgroup without them).
struct S1Out {
    Step1* lds;
    Step1* glb;
    bool g;
    int64_t kl, kg;
    __device__ __forceinline__ void put(int T, int32_t i, const Step1& v) const {
        if (g) glb[T * kg + i] = v;
        else lds[T * kl + i] = v;
    }
};

template <int PD, int PR>
__device__ __forceinline__ void step_emit_one(const NodeRec<PD, PR>& r, int64_t n, int T, int32_t slot,
                                              int32_t mslot, bool multi, int64_t tmin, int64_t tmax, double wsum,
                                              int32_t noprio, const StepTables& st, int64_t blk, const S1Out& s1o,
                                              double winv = 0.0) {
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
    auto key = [&](int64_t t) {  // key_of for the run-time kind, at the first instant of a step
        const int32_t f = score_at<PD, PR>(t, r, wsum, noprio, winv);
        return (T == 1 || !(t < r.e_fail)) ? pack_key(f, n) : -1;
    };
    const int32_t k0 = key(tmin);
    if (!multi) {
        Step1 v;
        v.bp = mn;
        v.k0 = k0;
        v.k1 = key(mn);
        s1o.put(T, slot, v);
        return;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i)  // odd-even transposition sort (static indices)
#pragma unroll
        for (int j = i & 1; j + 1 < NB; j += 2) {
            const int64_t x = c[j], y = c[j + 1];
            c[j] = min(x, y);
            c[j + 1] = max(x, y);
        }
    Mid* md = st.mid + (int64_t)T * st.mpad + blk * st.mstride + mslot;
    int32_t kprev = k0;
    int64_t last = c[0];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        if (j >= cnt) continue;
        const int32_t kj = key(c[j]);  // the key from c[j] on
        if (j + 1 < cnt) {
            Mid p;
            p.s = c[j];
            p.e = c[j + 1];
            p.key = kj;
            p.pad = 0;
            md[j] = p;
        }
        last = c[j];
        kprev = kj;
    }
    Step1 a, b;
    a.bp = c[0];
    a.k0 = k0;
    a.k1 = -1;
    b.bp = last;
    b.k0 = -1;
    b.k1 = kprev;
    s1o.put(T, slot, a);
    s1o.put(T, slot + 1, b);
}

// Phase 2 for every kind of a node (the stand-alone K3a).
template <int PD, int PR>
__device__ __forceinline__ void step_emit(const NodeRec<PD, PR>& r, int64_t n, int64_t tmin, int64_t tmax,
                                          double wsum, int32_t noprio, const StepSlots& o,
                                          const StepTables& st, int64_t blk, const S1Out& s1o,
                                          double winv = 0.0) {
    if (o.slot0 >= 0)
        step_emit_one<PD, PR>(r, n, 0, o.slot0, o.mslot0, o.multi0, tmin, tmax, wsum, noprio, st, blk, s1o, winv);
    if (o.slot1 >= 0)
        step_emit_one<PD, PR>(r, n, 1, o.slot1, o.mslot1, o.multi1, tmin, tmax, wsum, noprio, st, blk, s1o, winv);
}

// Work item of the compacted emit: owner thread | kind << 12 | multi << 13 | slot << 14 | rs << 24,
// and its first middle-piece slot in qm.
// (rs: the node's record slot in the workgroup's LDS staging, < 256; slot < 1024)
__device__ __forceinline__ void step_queue(const StepSlots& o, int32_t* nq, uint32_t* q, int32_t* qm, int rs) {
    if (o.slot0 >= 0) {
        const int i = atomicAdd(nq, 1);
        q[i] = threadIdx.x | ((uint32_t)o.multi0 << 13) | ((uint32_t)o.slot0 << 14) | ((uint32_t)rs << 24);
        qm[i] = o.mslot0;
    }
    if (o.slot1 >= 0) {
        const int i = atomicAdd(nq, 1);
        q[i] = threadIdx.x | (1u << 12) | ((uint32_t)o.multi1 << 13) | ((uint32_t)o.slot1 << 14) | ((uint32_t)rs << 24);
        qm[i] = o.mslot1;
    }
}

// K1's form of step_count + stepped-record staging + step_queue, called by every thread
// of the workgroup (valid: the thread has a node): the per-lane counts are prefix-summed
// across the wave (DPP) and one lane takes the wave's spans with one LDS atomic per
// counter, instead of a chain of per-lane returning atomics.  Slots are assigned in lane
// order (any order is a valid one: K3s takes maxima).  keep: records written out (the
// record slot is the thread's; every item queued), else the stepped records are staged in
// lrec[0, CAP) and a node past the staging builds its own (self_emit; its queue items
// are marked ~0u).
template <int PD, int PR, int CAP>
__device__ __forceinline__ void step_count_queue(const NodeRec<PD, PR>& r, bool valid, int64_t n, int64_t tmin,
                                                 int64_t tmax, double wsum, double winv, int32_t noprio,
                                                 bool keep, StepShared& sh, int32_t* nrec, int32_t* nq,
                                                 uint32_t* q, int32_t* qm, NodeRec<PD, PR>* lrec, StepSlots& o,
                                                 bool& self_emit) {
    const int32_t s0 = score_at<PD, PR>(tmin, r, wsum, noprio, winv);
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
    o.multi0 = cnt0 > 0 && mn0 != mx0;
    o.multi1 = cnt1 > 0 && mn1 != mx1;
    o.nb0 = (int8_t)cnt0;
    o.nb1 = (int8_t)cnt1;
    o.flat0 = valid && cnt0 == 0 ? key_of<PD, PR>(0, tmin, s0, r, n) : -1;
    o.flat1 = valid && cnt1 == 0 ? key_of<PD, PR>(1, tmin, s0, r, n) : -1;
    // per lane: one-step records | middle pieces << 16 per kind; stepped | queue items << 16
    const uint32_t w0 = (cnt0 ? (o.multi0 ? 2u : 1u) : 0u) | (o.multi0 ? (uint32_t)(cnt0 - 1) << 16 : 0u);
    const uint32_t w1 = (cnt1 ? (o.multi1 ? 2u : 1u) : 0u) | (o.multi1 ? (uint32_t)(cnt1 - 1) << 16 : 0u);
    const uint32_t w2 = ((cnt0 | cnt1) ? 1u : 0u) | (((cnt0 ? 1u : 0u) + (cnt1 ? 1u : 0u)) << 16);
    // exclusive prefixes and the wave's totals (lane 63's inclusive prefix)
    uint32_t e0 = wave_scan_add(w0);
    const uint32_t t0 = __builtin_amdgcn_readlane(e0, 63);
    e0 -= w0;
    uint32_t e1 = wave_scan_add(w1);
    const uint32_t t1 = __builtin_amdgcn_readlane(e1, 63);
    e1 -= w1;
    uint32_t e2 = wave_scan_add(w2);
    const uint32_t t2 = __builtin_amdgcn_readlane(e2, 63);
    e2 -= w2;
    int32_t b[6] = {0, 0, 0, 0, 0, 0};
    if ((threadIdx.x & 63) == 63) {
        if (t0) {
            b[0] = atomicAdd(&sh.lc[0][0], (int32_t)(t0 & 0xFFFF));
            b[1] = atomicAdd(&sh.lc[0][1], (int32_t)(t0 >> 16));
        }
        if (t1) {
            b[2] = atomicAdd(&sh.lc[1][0], (int32_t)(t1 & 0xFFFF));
            b[3] = atomicAdd(&sh.lc[1][1], (int32_t)(t1 >> 16));
        }
        if (t2) {
            b[4] = atomicAdd(nrec, (int32_t)(t2 & 0xFFFF));
            b[5] = atomicAdd(nq, (int32_t)(t2 >> 16));
        }
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) b[k] = __builtin_amdgcn_readlane(b[k], 63);
    o.slot0 = cnt0 ? b[0] + (int32_t)(e0 & 0xFFFF) : -1;
    o.mslot0 = o.multi0 ? b[1] + (int32_t)(e0 >> 16) : 0;
    o.slot1 = cnt1 ? b[2] + (int32_t)(e1 & 0xFFFF) : -1;
    o.mslot1 = o.multi1 ? b[3] + (int32_t)(e1 >> 16) : 0;
    self_emit = false;
    if (cnt0 | cnt1) {
        int rs = b[4] + (int32_t)(e2 & 0xFFFF);
        bool staged = true;
        if (keep) rs = threadIdx.x;
        else if (rs < CAP) lrec[rs] = r;
        else staged = false;
        int qi = b[5] + (int32_t)(e2 >> 16);
        if (cnt0) {
            q[qi] = staged ? threadIdx.x | ((uint32_t)o.multi0 << 13) | ((uint32_t)o.slot0 << 14) | ((uint32_t)rs << 24)
                           : ~0u;
            qm[qi] = o.mslot0;
            ++qi;
        }
        if (cnt1) {
            q[qi] = staged ? threadIdx.x | (1u << 12) | ((uint32_t)o.multi1 << 13) | ((uint32_t)o.slot1 << 14) |
                                 ((uint32_t)rs << 24)
                           : ~0u;
            qm[qi] = o.mslot1;
        }
        self_emit = !staged;
    }
}

// Workgroup epilogue: the workgroup's flat-key maxima and record counts go to
// its own slots (producer block blk) of the step tables (plain stores, no global atomics).  Every
// thread calls it (barrier); sh.lc must have been zeroed before step_count.
template <int BS>
__device__ __forceinline__ void step_publish(const StepSlots& o, StepShared& sh, const StepTables& st, int64_t blk) {
    auto wmax = [&](int T, int32_t m) {
        m = wave_max(m);
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

// number of the n sorted records at a[] with bp <= t (upper bound)
__device__ __forceinline__ int32_t count_le(const Step1* a, int32_t n, int64_t t) {
    int32_t lo = 0, hi = n;
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (a[mid].bp <= t) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// After every Step1 record of the workgroup is in s1l (and a barrier): per pod kind,
// the records sorted by step time bp go to the workgroup's region of st.single, with
// pm1[i] = max of k1 over sorted records 0..i (the keys after their steps) and
// sm0[i] = max of k0 over records i..n-1 (the keys before their steps).  For a pod
// tile's range [lo, hi] of a kind, the records stepping inside are [jl, jh) (jl = those
// with bp <= lo, jh = those with bp <= hi) and every pod of it takes every other
// record's key from one prefix and one suffix maximum: step_tile_rows writes that
// uniform key (with the flat maximum) and [jl, jh) per tile into st.rows (when set),
// so K3s starts from them; without rows K3s searches the records itself.
// s1l: LDS staging [2][CAP] records (CAP >= either kind's count), srt: LDS scratch
// [2][CAP]; s1l is reused for the maxima.  Every thread calls it (barriers); sh.fm
// holds the per-wave flat maxima (step_publish).
template <int BS, int CAP = 2 * BS>
__device__ __forceinline__ void step_sort_publish(Step1* s1l, Step1* srt, const StepShared& sh,
                                                  const StepTables& st, int64_t blk) {
    const int n0 = sh.lc[0][0], n1 = sh.lc[1][0];
    // rank sort (ties by slot): typically a few dozen records per kind
    for (int i = threadIdx.x; i < n0 + n1; i += BS) {
        const int T = i >= n0;
        const int k = T ? i - n0 : i;
        const int n = T ? n1 : n0;
        const Step1* a = s1l + T * CAP;
        const Step1 v = a[k];
        int rank = 0;
        int j = 0;
        for (; j + 8 <= n; j += 8) {  // 8 independent LDS reads in flight
            int64_t b[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) b[u] = a[j + u].bp;
#pragma unroll
            for (int u = 0; u < 8; ++u) rank += (b[u] < v.bp) || (b[u] == v.bp && j + u < k);
        }
        for (; j < n; ++j) {
            const int64_t b = a[j].bp;
            rank += (b < v.bp) || (b == v.bp && j < k);
        }
        srt[T * CAP + rank] = v;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n0 + n1; i += BS) {
        const int T = i >= n0;
        const int k = T ? i - n0 : i;
        st.single[s1_at(st, T, blk) + k] = srt[T * CAP + k];
    }
    // prefix max of k1 / suffix max of k0: wave T scans kind T in chunks of 64 consecutive
    // records (one per lane) with a carry; also kept in LDS (s1l is free now) for the rows
    int32_t* pmL = reinterpret_cast<int32_t*>(s1l);  // [2][CAP]
    int32_t* smL = pmL + 2 * CAP;                     // [2][CAP]
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // wave T takes kind T (a one-wave workgroup takes both in turn)
    for (int T = w; T < 2; T += (BS >= 128 ? 2 : 1)) {
        const int n = T ? n1 : n0;
        const Step1* a = srt + T * CAP;
        const int64_t base = s1_at(st, T, blk);
        int32_t carry = -1;
        for (int c0 = 0; c0 < n; c0 += 64) {
            const int i = c0 + lane;
            const int32_t v = max(wave_scan_max(i < n ? a[i].k1 : -1), carry);
            if (i < n) {
                st.pm1[base + i] = v;
                pmL[T * CAP + i] = v;
            }
            carry = __builtin_amdgcn_readlane(v, 63);
        }
        // suffix maxima: lane l takes index c0 + 63 - l, so a prefix in lane order
        carry = -1;
        for (int c0 = (n - 1) & ~63; c0 >= 0 && n > 0; c0 -= 64) {
            const int i = c0 + 63 - lane;
            const int32_t v = max(wave_scan_max(i < n ? a[i].k0 : -1), carry);
            if (i < n) {
                st.sm0[base + i] = v;
                smL[T * CAP + i] = v;
            }
            carry = __builtin_amdgcn_readlane(v, 63);
        }
    }
}

// The same for a block whose records exceed the LDS staging: staged in st.stage
// (same indexing as st.single), ranked straight into st.single, maxima into pm1 / sm0.
template <int BS>
__device__ __forceinline__ void step_sort_publish_global(const StepShared& sh, const StepTables& st, int64_t blk) {
    const int n0 = sh.lc[0][0], n1 = sh.lc[1][0];
    for (int i = threadIdx.x; i < n0 + n1; i += BS) {
        const int T = i >= n0;
        const int k = T ? i - n0 : i;
        const int n = T ? n1 : n0;
        const Step1* a = st.stage + s1_at(st, T, blk);
        const Step1 v = a[k];
        int rank = 0;
        for (int j = 0; j < n; ++j) {
            const int64_t b = a[j].bp;
            rank += (b < v.bp) || (b == v.bp && j < k);
        }
        st.single[s1_at(st, T, blk) + rank] = v;
    }
    __syncthreads();
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int T = w; T < 2; T += (BS >= 128 ? 2 : 1)) {
        const int n = T ? n1 : n0;
        const int64_t base = s1_at(st, T, blk);
        const Step1* a = st.single + base;
        int32_t carry = -1;
        for (int c0 = 0; c0 < n; c0 += 64) {
            const int i = c0 + lane;
            const int32_t v = max(wave_scan_max(i < n ? a[i].k1 : -1), carry);
            if (i < n) st.pm1[base + i] = v;
            carry = __builtin_amdgcn_readlane(v, 63);
        }
        carry = -1;
        for (int c0 = (n - 1) & ~63; c0 >= 0 && n > 0; c0 -= 64) {
            const int i = c0 + 63 - lane;
            const int32_t v = max(wave_scan_max(i < n ? a[i].k0 : -1), carry);
            if (i < n) st.sm0[base + i] = v;
            carry = __builtin_amdgcn_readlane(v, 63);
        }
    }
}

// ---- middle pieces -> disjoint elementary pieces (per block and kind, after the emit)
// A kind's raw middle pieces [s, e) (every multi-step node's: they overlap across nodes)
// are cut at every piece end into disjoint intervals, each carrying the max key of the
// pieces covering it; intervals no feasible piece covers are dropped.  At any time the
// max over the raw pieces containing it is the key of the one elementary piece containing
// it, so a pod tile needs only the pieces its time range overlaps — a contiguous range
// [pl, ph) of the sorted list (step_tile_rows writes it to st.prow; one covering the whole
// range goes into the row's uniform key) — instead of every piece of the block once per
// tile (config 4: ~32 pieces per kind and block, 98 tiles).  The list replaces the raw
// one in st.mid (and its count in st.cnt).  Kinds with more than the scratch holds, or too
// little work to pay for it (pieces x tiles < st.piece_work), stay raw: their row range is
// all pieces.
// LDS scratch per kind (pc pieces at most): sorted breakpoints bs[2pc] (i64), unsorted
// bu[2pc] (i64: s, e of piece k at 2k, 2k + 1), maxima vm[2pc] (of the interval from each
// sorted breakpoint to the next), compacted positions ix[2pc], raw keys rk[pc] (i32):
// 52 * pc bytes.
struct PieceScr {
    unsigned char* p;
    int32_t pc;  // pieces per kind the scratch holds (0: never decompose)
    __device__ int64_t* bs(int T) const { return reinterpret_cast<int64_t*>(p + (int64_t)T * 52 * pc); }
    __device__ int64_t* bu(int T) const { return reinterpret_cast<int64_t*>(p + (int64_t)T * 52 * pc + 16 * pc); }
    __device__ int32_t* vm(int T) const { return reinterpret_cast<int32_t*>(p + (int64_t)T * 52 * pc + 32 * pc); }
    __device__ int32_t* ix(int T) const { return reinterpret_cast<int32_t*>(p + (int64_t)T * 52 * pc + 40 * pc); }
    __device__ int32_t* rk(int T) const { return reinterpret_cast<int32_t*>(p + (int64_t)T * 52 * pc + 48 * pc); }
    static constexpr int bytes_per_piece = 2 * 52;  // both kinds
};
// Every thread calls it (barriers when a kind is decomposed); sh.lc final and the emit's
// pieces in st.mid (a barrier after the emit).  Sets sh.pn (read after the next barrier).
template <int BS>
__device__ __forceinline__ void step_pieces(StepShared& sh, const StepTables& st, int64_t blk, const PieceScr& ps) {
    const int32_t nm0 = sh.lc[0][1], nm1 = sh.lc[1][1];
    auto dec = [&](int32_t nm) {
        return st.prow && nm >= 2 && nm <= ps.pc && (int64_t)nm * st.ntiles >= st.piece_work;
    };
    const bool d0 = dec(nm0), d1 = dec(nm1);
    if (!d0 && !d1) {  // (workgroup-uniform)
        if (threadIdx.x < 2) sh.pn[threadIdx.x] = -1;
        return;
    }
    const int32_t a0 = d0 ? nm0 : 0, a1 = d1 ? nm1 : 0;  // pieces taken per kind
    // A: the raw pieces into LDS
    for (int i = threadIdx.x; i < a0 + a1; i += BS) {
        const int T = i >= a0, k = T ? i - a0 : i;
        const Mid m = st.mid[(int64_t)T * st.mpad + blk * st.mstride + k];
        ps.bu(T)[2 * k] = m.s;
        ps.bu(T)[2 * k + 1] = m.e;
        ps.rk(T)[k] = m.key;
    }
    __syncthreads();
    // B: every breakpoint v (s or e of a piece) in one pass over its kind's pieces: its
    // rank among the breakpoints (ties by index: its position in the sorted order) and the
    // max key of the feasible pieces covering [v, next breakpoint), i.e. with s <= v < e
    // (broadcast LDS reads, no atomics: equal breakpoints get equal maxima)
    for (int i = threadIdx.x; i < 2 * (a0 + a1); i += BS) {
        const int T = i >= 2 * a0, j = T ? i - 2 * a0 : i, n = T ? a1 : a0;
        const int64_t* b = ps.bu(T);
        const int32_t* rk = ps.rk(T);
        const int64_t v = b[j];
        int32_t r = 0, m = -1;
        for (int k = 0; k < n; ++k) {
            const int64_t s = b[2 * k], e = b[2 * k + 1];
            r += (s < v) || (s == v && 2 * k < j);
            r += (e < v) || (e == v && 2 * k + 1 < j);
            if (s <= v && v < e) m = max(m, rk[k]);
        }
        ps.bs(T)[r] = v;
        ps.vm(T)[r] = m;
    }
    __syncthreads();
    // D: wave T compacts kind T's non-empty covered intervals (in order) and publishes them
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int T = w; T < 2; T += (BS >= 128 ? 2 : 1)) {  // wave T compacts kind T (one wave: both)
        const int32_t n = 2 * (T ? a1 : a0);
        if ((T ? d1 : d0)) {
            const int64_t* bs = ps.bs(T);
            const int32_t* vm = ps.vm(T);
            Mid* out = st.mid + (int64_t)T * st.mpad + blk * st.mstride;
            uint32_t carry = 0;
            for (int32_t c0 = 0; c0 < n - 1; c0 += 64) {
                const int32_t j = c0 + lane;
                const bool f = j < n - 1 && bs[j] < bs[j + 1] && vm[j] >= 0;
                const uint32_t inc = wave_scan_add(f ? 1u : 0u);
                if (f) {
                    const int32_t pos = (int32_t)(carry + inc - 1);
                    ps.ix(T)[pos] = j;
                    Mid m;
                    m.s = bs[j];
                    m.e = bs[j + 1];
                    m.key = vm[j];
                    m.pad = 0;
                    out[pos] = m;
                }
                carry += __builtin_amdgcn_readlane(inc, 63);
            }
            if (lane == 0) {
                sh.pn[T] = (int32_t)carry;
                st.cnt[blk * 4 + 2 * T + 1] = (int32_t)carry;
            }
        } else if (lane == 0) {
            sh.pn[T] = -1;
        }
    }
}

// The tile rows (st.rows set): per pod tile t, the block's uniform key per kind and
// the range [jl, jh) of its sorted one-step records stepping inside the tile's range
// (after step_sort_publish: srt sorted, s1l holding the prefix / suffix maxima), and
// (st.prow set) the range [pl, ph) of its middle pieces overlapping it (step_pieces).
// pre: this thread's first item's bound (tile_prefetch, loaded early).  Every thread
// calls it (barrier).
__device__ __forceinline__ void tile_prefetch(const StepTables& st, int64_t* pre) {
    const int x = threadIdx.x;  // item x: tile x / 4, kind (x / 2) % 2, lo / hi
    *pre = (x >> 2) < st.ntiles ? st.tiles[kTileStat * (x >> 2) + ((x >> 1) & 1) * 2 + (x & 1)] : 0;
}
// G: the block's records went through st.stage (step_sort_publish_global): the
// searches read st.single / pm1 / sm0 instead of the LDS copies.
template <int BS, int CAP = 2 * BS, bool G = false>
__device__ __forceinline__ void step_tile_rows(const Step1* s1l, const Step1* srt, const StepShared& sh,
                                               const StepTables& st, int64_t blk, const int64_t* pre,
                                               const PieceScr& ps) {
    const int n0 = sh.lc[0][0], n1 = sh.lc[1][0];
    const int32_t* pmL = reinterpret_cast<const int32_t*>(s1l);
    const int32_t* smL = pmL + 2 * CAP;
    __syncthreads();
    int32_t fl[2];  // the block's flat maxima
#pragma unroll
    for (int T = 0; T < 2; ++T) {
        fl[T] = sh.fm[T][0];
#pragma unroll
        for (int i = 1; i < BS / 64; ++i) fl[T] = max(fl[T], sh.fm[T][i]);
    }
    // item i: tile i / 4, kind (i / 2) % 2, bound i % 2 (lo, hi): one LDS search each, the
    // four items of a tile on adjacent lanes combine by shuffles
    for (int i0 = 0; i0 < 4 * st.ntiles; i0 += BS) {
        const int i = i0 + threadIdx.x;
        const int t = i >> 2, T = (i >> 1) & 1, hi_b = i & 1;
        const int n = T ? n1 : n0;
        const int32_t pn = sh.pn[T];
        int32_t c = 0, u = -1, pc = 0;
        int64_t v = 0;
        if (t < st.ntiles) {
            v = i0 == 0 ? *pre : st.tiles[kTileStat * t + 2 * T + hi_b];
            if (G) {
                const int64_t base = s1_at(st, T, blk);
                c = count_le(st.single + base, n, v);
                if (!hi_b && c > 0) u = st.pm1[base + c - 1];
                if (hi_b && c < n) u = st.sm0[base + c];
            } else {
                c = count_le(srt + T * CAP, n, v);
                if (!hi_b && c > 0) u = pmL[T * CAP + c - 1];  // records stepped by lo: keys after
                if (hi_b && c < n) u = smL[T * CAP + c];       // records stepping after hi: keys before
            }
            // middle pieces: elementary ones ending by lo (pl) / starting by hi (ph); raw: all
            if (!st.prow) {
            } else if (pn >= 0) {
                const int64_t* bs = ps.bs(T);
                const int32_t* ix = ps.ix(T);
                int32_t lo = 0, hi = pn;
                while (lo < hi) {
                    const int32_t mid = (lo + hi) >> 1;
                    if (bs[ix[mid] + (hi_b ? 0 : 1)] <= v) lo = mid + 1;
                    else hi = mid;
                }
                pc = lo;
            } else {
                pc = hi_b ? sh.lc[T][1] : 0;
            }
        }
        const int32_t co = quad_xor1(c), uo = quad_xor1(u);
        const int32_t jl = hi_b ? co : c, jh = hi_b ? c : co;
        int32_t ukey = -1, pp = 0;
        if (st.prow) {  // (uniform)
            const int32_t pco = quad_xor1(pc);
            const int64_t vo = (int64_t)(((uint64_t)(uint32_t)quad_xor1((int32_t)((uint64_t)v >> 32)) << 32) |
                                         (uint32_t)quad_xor1((int32_t)(uint32_t)v));
            int32_t pl = hi_b ? pco : pc;
            const int32_t ph = hi_b ? pc : pco;
            if (pn >= 0 && ph - pl == 1 && t < st.ntiles) {  // one elementary piece: uniform if it covers [lo, hi]
                const int64_t lo_v = hi_b ? vo : v, hi_v = hi_b ? v : vo;
                const int32_t j = ps.ix(T)[pl];
                if (ps.bs(T)[j] <= lo_v && ps.bs(T)[j + 1] > hi_v) {
                    ukey = ps.vm(T)[j];
                    pl = ph;
                }
            }
            pp = pl < ph ? (pl | (ph << 16)) : 0;
        }
        // a kind without pods here (lo = INT64_MAX, hi = INT64_MIN) gives jl = n > jh = 0
        const int32_t um = jl > jh ? -1 : max(max(fl[T], ukey), max(u, uo)), jp = jl > jh ? 0 : (jl | (jh << 16));
        const int32_t um1 = quad_down2(um), jp1 = quad_down2(jp);
        const int32_t pp1 = st.prow ? quad_down2(pp) : 0;
        if ((i & 3) == 0 && t < st.ntiles) {
            st.rows[(int64_t)t * st.nblk + blk] = make_int4(um, um1, jp, jp1);
            if (st.prow) st.prow[(int64_t)t * st.nblk + blk] = make_int2(pp, pp1);
        }
    }
}

}  // namespace crane
