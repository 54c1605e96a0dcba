// k1stream.hip — the node pass fused with the step tables, streamed (K1 for large N).
//
// Numerics: the same per-term arithmetic as node_rec.hpp / step_node.hpp (stats.go:89-138,
// plugins.go:39-98 bit for bit, -ffp-contract=off).
#include <hip/hip_runtime.h>

#include <cstddef>

#include "dyn_types.hpp"
#include "kernels.hpp"
#include "node_rec.hpp"
#include "step_node.hpp"

namespace crane {

// The node pass fused with the step tables, without a NodeRec in registers.  Round 4 found what
// holds the fused pass at 0.41 of HBM cold: occupancy, which the 160 B record costs (96 VGPRs,
// five waves per SIMD) — a count pass that folds each row into what classification needs as it
// arrives runs at seven waves and 0.59 on its own — and every way of handing the ~3 % stepped
// nodes' records to a separate emit kernel cost more than it saved.  Here the
// hand-off stays inside the workgroup:
//   A  each lane streams its node's rows and keeps only e_fail, the hot-value penalty and
//      expiry, and per pod kind the in-range expiry count / min / max and the flat key;
//   B  wave prefix sums + one exchange of the waves' totals give every stepped node its
//      one-step / middle-piece slots and its rank among the block's stepped nodes;
//   C  in chunks of kSRec stepped nodes: each stepped lane writes its e_fail / pen / e_hv and
//      slots into an LDS record, the workgroup then gathers the chunk's priority rows from L2
//      (one (node, term) per lane: the lines this workgroup streamed microseconds earlier) and
//      writes e_prio / t with rec_metrics' arithmetic, and the first lanes emit the chunk's
//      (node, kind) items from the LDS records (step_emit_one);
//   D  the fused pass's tail: sort + publish, elementary pieces, tile rows.
// Not with the dedupe-form K2 entries (their per-block counting needs the default pass's LDS).
// step_emit_one's outputs for the stepped nodes of a chunk, spread over the lanes: node j takes
// lanes j * (PR + 2) + q, and lane q handles candidate expiry q (the priorities', the hot
// value's, e_fail) for both pod kinds at once: if it is in the batch range, its rank r in the
// kind's ascending order (with multiplicity, by ranking the candidates in registers), its key
// (one score serves both kinds: the Filter only gates kind 0's), its middle piece
// [c_r, c_{r+1}), and — r = 0 / r = cnt - 1 — the half-line records.  A node's keys are then
// computed side by side instead of one after another (round 5's first form, one lane per item
// walking its expiries in order with the record read from LDS term by term, spent 4.9 us per
// workgroup here: a chain of dependent LDS reads; a lane per (node, kind, candidate) doubled the
// emitting waves for 1 % more time).  The outputs are step_emit_one's, bit for bit.
__device__ __forceinline__ int64_t readfirstlane64(int64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// score_at for a record in LDS with its terms read one at a time (a rolled loop: two fields in
// registers at a time — the emit's keys are computed side by side, so each one's own latency
// matters less than the registers a copy of the record would hold)
template <int PD, int PR>
__device__ __forceinline__ int32_t score_at_lds(int64_t t, const NodeRec<PD, PR>& r, double wsum, int32_t noprio,
                                                double winv) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < PR; ++k)
        if (t < r.e_prio[k]) s += r.t[k];  // stats.go:124-133, policy order
    return score_of_sum(s, t < r.e_hv ? r.pen : 0, wsum, noprio, winv);
}

// K1S_SKIP (cost ablation builds only, tools/gpu_k1_ablate.sh; wrong tables): 1 no emit tasks,
// 2 no tail (sort / pieces / tile rows), 4 no record staging, 8 middle pieces left raw (no
// elementary pieces: the tables stay right, K3s reads every piece), 16 no tile rows
#ifndef K1S_SKIP
#define K1S_SKIP 0
#endif
#ifndef K1S_TAIL1  // the single-wave tail for grids of many rounds (A/B: 0 off)
#define K1S_TAIL1 1
#endif
#ifndef K1S_WAVES  // waves per SIMD the 4x6 form is built for (72 VGPRs: 7; 64: 8)
#define K1S_WAVES 7
#endif
#ifndef K1S_KWARM  // the kernarg lines warmed in the scalar cache while the rows load (A/B: 0 off)
#define K1S_KWARM 1
#endif
#ifndef K1S_FULL  // the instance for a policy of exactly 4 predicates / 6 priorities / 2 windows (A/B: 0 off)
#define K1S_FULL 1
#endif
#ifndef K1S_EMIT_SCORE  // the emit's score from the candidates in registers, terms loaded together (A/B: 0 off)
#define K1S_EMIT_SCORE 1
#endif
#ifndef K1S_PUB1  // step_publish folded into the slots' exchange (one barrier; A/B: 0 its own barrier)
#define K1S_PUB1 1
#endif
#ifndef K1S_SREC
#define K1S_SREC 64
#endif
#ifndef K1S_SCAP
#define K1S_SCAP 128
#endif
constexpr int kSRec = K1S_SREC;  // stepped records staged per chunk
constexpr int kSCap = K1S_SCAP;  // one-step records per kind staged in LDS (more: st.stage)

template <int PD, int PR>
__device__ __forceinline__ void emit_task(const NodeRec<PD, PR>& r, int64_t n, int q, const int32_t* dw, int64_t tmin,
                                          int64_t tmax, double wsum, int32_t noprio, const StepTables& st,
                                          int64_t blk, const S1Out& s1o, double winv) {
    constexpr int NB = PR + 2, F = PR + 1;  // candidate F = e_fail: kind 0's only (DaemonSet pods bypass the Filter)
    int64_t c[NB];
#pragma unroll
    for (int k = 0; k < PR; ++k) c[k] = r.e_prio[k];
    c[PR] = r.e_hv;
    c[F] = r.e_fail;
    uint32_t inm = 0;  // kind 0's in-range candidates; kind 1's are inm without F
#pragma unroll
    for (int k = 0; k < NB; ++k) inm |= (c[k] > tmin && c[k] <= tmax) ? 1u << k : 0u;
    if (!((inm >> q) & 1u)) return;  // out of range
    const int cnt0 = __builtin_popcount(inm), cnt1 = __builtin_popcount(inm & ~(1u << F));
    // c[q], its rank in the ascending order of (c, index) and the next one's value, per kind:
    // ranks among NB registers (static indices) instead of a sort
    int64_t cq = c[0];
#pragma unroll
    for (int j = 1; j < NB; ++j) cq = q == j ? c[j] : cq;
    int rk0 = 0;
    bool fb = false;  // e_fail before c[q] (kind 0 only)
    int64_t cn1 = INT64_MAX, cn0;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        const bool in = (inm >> j) & 1u;
        const bool before = in && (c[j] < cq || (c[j] == cq && j < q));
        const bool after = in && (c[j] > cq || (c[j] == cq && j > q));
        rk0 += before;
        if (j == F) {
            fb = before;
            cn0 = after ? min(cn1, c[j]) : cn1;
        } else {
            cn1 = after ? min(cn1, c[j]) : cn1;
        }
    }
    const int rk1 = rk0 - (fb ? 1 : 0);
    // one score per instant serves both kinds (the Filter only gates kind 0's key): score_at with
    // the expiries already in c[] and the terms read side by side (one LDS wait, not one per term)
#if K1S_EMIT_SCORE
    double tk[PR];
#pragma unroll
    for (int k = 0; k < PR; ++k) tk[k] = r.t[k];
    double ssum = 0.0;
#pragma unroll
    for (int k = 0; k < PR; ++k) ssum = cq < c[k] ? ssum + tk[k] : ssum;  // stats.go:124-133, policy order
    const int64_t pk = pack_key(score_of_sum(ssum, cq < c[PR] ? r.pen : 0, wsum, noprio, winv), n);
#else
    const int64_t pk = pack_key(score_at_lds<PD, PR>(cq, r, wsum, noprio, winv), n);
#endif
    // the score at tmin: phase A's, kept in the record's slot words (dw[5])
    const int64_t pk0 = pack_key(dw[5], n);
#pragma unroll
    for (int T = 0; T < 2; ++T) {
        const int32_t slot = dw[T ? 2 : 0];
        if (slot < 0 || (T == 1 && q == F)) continue;
        const int rk = T ? rk1 : rk0, cnt = T ? cnt1 : cnt0;
        const int64_t cn = T ? cn1 : cn0;
        const int32_t kq = (int32_t)((T == 1 || !(cq < r.e_fail)) ? pk : -1);    // the key from c_rk on
        const int32_t kt = (int32_t)((T == 1 || !(tmin < r.e_fail)) ? pk0 : -1); // ... before c_0
        const bool multi = ((dw[4] >> T) & 1) != 0;
        if (!multi) {  // one record: before / from the one distinct expiry
            if (rk == 0) {
                Step1 v;
                v.bp = cq;
                v.k0 = kt;
                v.k1 = kq;
                s1o.put(T, slot, v);
            }
            continue;
        }
        if (rk + 1 < cnt) {
            Mid pc;
            pc.s = cq;
            pc.e = cn;
            pc.key = kq;
            pc.pad = 0;
            (st.mid + (int64_t)T * st.mpad + blk * st.mstride + dw[T ? 3 : 1])[rk] = pc;
        }
        if (rk == 0) {
            Step1 x;
            x.bp = cq;
            x.k0 = kt;
            x.k1 = -1;
            s1o.put(T, slot, x);
        }
        if (rk == cnt - 1) {
            Step1 y;
            y.bp = cq;
            y.k0 = -1;
            y.k1 = kq;
            s1o.put(T, slot + 1, y);
        }
    }
}

// the step epilogue after the emit: sort + publish, elementary pieces, tile rows, by the BS
// threads still running (lrec: the staged records' LDS, dead now: the pieces' scratch)
template <int BS, class Rec>
__device__ __forceinline__ void tail(bool g1, Rec* lrec, Step1* s1l, Step1* srt, StepShared& ssh, const K1Step& step,
                                     int64_t blk, unsigned long long* trace) {
    if (g1) step_sort_publish_global<BS>(ssh, step.st, blk);
    else step_sort_publish<BS, kSCap>(s1l, srt, ssh, step.st, blk);
    CRANE_TSTAMP(trace, blockIdx.x, 6);
    if (step.st.rows && !(K1S_SKIP & 16)) {
        int64_t tpre = 0;  // this thread's first tile-row bound (step_tile_rows)
        tile_prefetch(step.st, &tpre);
        constexpr int kPc = ((int)(kSRec * sizeof(Rec)) / PieceScr::bytes_per_piece) & ~3;
        const PieceScr ps{reinterpret_cast<unsigned char*>(lrec), (K1S_SKIP & 8) ? 0 : (kPc < 128 ? kPc : 128)};
        step_pieces<BS>(ssh, step.st, blk, ps);
        if (g1) step_tile_rows<BS, kSCap, true>(s1l, srt, ssh, step.st, blk, &tpre, ps);
        else step_tile_rows<BS, kSCap, false>(s1l, srt, ssh, step.st, blk, &tpre, ps);
    }
    CRANE_TSTAMP(trace, blockIdx.x, 4);
}

// FULL: the policy has exactly PD predicates, PR priorities and kFullWin hot-value windows (the
// reference's shipped policy at 4 x 6): every per-term loop is static, so the policy words load
// together instead of one scalar load and wait per term under its own uniform branch
constexpr int kFullWin = 2;
template <int PD, int PR, bool FULL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PD * PR <= 24 ? K1S_WAVES : 1)))
void k1_stream_steps(K1Args a, K1Step step) {
    using Rec = NodeRec<PD, PR>;
    constexpr int BS = 256;
    const int npd = FULL ? PD : a.pol.npd, npr = FULL ? PR : a.pol.npr, nwin = FULL ? kFullWin : a.pol.n_win;
    // a staged stepped node's record: e_fail, pen, e_hv, e_prio, t (what the emit reads), and in
    // e_pred's first words its slots per kind (slot < 0: none), multi flags and the score at tmin
    __shared__ __attribute__((aligned(16))) Rec lrec[kSRec];
    __shared__ uint8_t rank_lane[BS];  // a stepped node's rank in the block -> its lane
    __shared__ __attribute__((aligned(16))) Step1 s1l[2 * kSCap];  // one-step staging, then pm / sm maxima
    __shared__ __attribute__((aligned(16))) Step1 srt[2 * kSCap];  // sorted copy
    __shared__ __attribute__((aligned(16))) uint32_t xch[5][4];
    __shared__ StepShared ssh;
    const DevPolicy& pol = a.pol;
    const int64_t N = a.N;
    const int64_t blk = xcd_block(blockIdx.x, gridDim.x), first = blk * BS, n = first + threadIdx.x;
    CRANE_TSTAMP(a.trace, blockIdx.x, 0);
    const int lo = (int)min((int64_t)threadIdx.x, N - 1 - first);  // lane offset, clamped
    // the batch range K3p folded: loaded first, so waiting for it does not wait for the rows
    const int64_t bt0 = step.batch[0], bt1 = step.batch[1];
    // ---- A: stream the rows (every load unconditional, clamped index: all in flight at once)
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
    if (FULL || pol.n_slots > 0) {  // (FULL: the policy reads metrics)
#pragma unroll
        for (int k = 0; k < PD; ++k) {
            const int64_t row = k < npd ? pol.pred_slot[k] : 0;
            pt[k] = (a.ts + (row * N + first))[lo];
            pv[k] = (a.val + (row * N + first))[lo];
        }
#pragma unroll
        for (int k = 0; k < PR; ++k) {
            const int64_t row = k < npr ? pol.prio_slot[k] : 0;
            qt[k] = (a.ts + (row * N + first))[lo];
            qv[k] = (a.val + (row * N + first))[lo];
        }
    }
    uint32_t bc[kMaxWin];
    double hvl = 0.0;
    int64_t hvt = kTsInvalid;
    if (a.buckets) {
        // (+ the delta form's anchor counts: kernels.hip)
        const uint32_t* __restrict__ base = a.bucket_base ? a.bucket_base : a.buckets;
        uint32_t bz[kMaxWin];
#pragma unroll
        for (int b = 0; b < kMaxWin; ++b) {
            bc[b] = b < nwin ? (a.buckets + first)[(int64_t)b * N + lo] : 0u;
            bz[b] = b < nwin ? (base + first)[(int64_t)b * N + lo] : 0u;
        }
        if (a.bucket_base) {  // (rows past n_win read as 0)
#pragma unroll
            for (int b = 0; b < kMaxWin; ++b) bc[b] = bz[b] + bc[b] - (b + 1 < kMaxWin ? bc[b + 1] : 0u);
        }
    } else if (a.hv) {
        hvl = a.hv[first + lo];
        hvt = a.hv_ts ? a.hv_ts[first + lo] : a.hv_ts_counts;
    }
#if K1S_KWARM
    kernarg_warm<(int)sizeof(K1Args) + (int)sizeof(K1Step)>();
#endif
    // the batch range K3p folded, uniform: kept in SGPRs
    const int64_t tmin = readfirstlane64(bt0), tmax = readfirstlane64(bt1);
    if (threadIdx.x < 4) ssh.lc[threadIdx.x >> 1][threadIdx.x & 1] = 0;
    CRANE_TSTAMP(a.trace, blockIdx.x, 1);
    const bool valid = n < N;
    // isOverLoad per predicate (stats.go:94-112): the Filter rejects iff now < e_fail
    int64_t e_fail = kTsInvalid;
    // (every policy word read unconditionally, the per-term conditions as selects: the scalar
    // loads then issue together instead of one wait per term under its own branch)
#pragma unroll
    for (int k = 0; k < PD; ++k) {
        const double u = pv[k], lim = pol.pred_limit[k];
        const int64_t e = sat_add(pt[k], pol.pred_dur[k]);
        const bool over = k < npd && pt[k] != kTsInvalid && !(u < 0.0) && lim != 0.0 && u > lim;
        e_fail = over ? max(e_fail, e) : e_fail;
    }
    // hot value (getNodeHotValue / the binding-log counts) -> penalty and its expiry
    Rec hr;  // (only pen / e_hv are set and read)
    if (a.buckets) {
        if (valid && !a.buckets_keep) {
#pragma unroll
            for (int b = 0; b < kMaxWin; ++b)  // consumed: leaves the buckets zeroed for the next K2
                if (b < nwin) (a.buckets + first)[(int64_t)b * N + threadIdx.x] = 0;
        }
        rec_hot_counts<PD, PR, FULL ? kFullWin : 0>(pol, bc, N, n, valid ? a.cnt_out : nullptr, valid ? a.hvc_out : nullptr,
                               a.hv_ts_counts, hr);
    } else if (a.hv) {
        rec_hot_annotation<PD, PR>(hvl, hvt, hr);
    } else {
        hr.pen = 0;
        hr.e_hv = kTsInvalid;
    }
    // priorities in policy order: score_at(tmin)'s ordered sum and the in-range expiries both
    // pod kinds share (priorities, hot value); e_fail is kind 0's too (DaemonSet pods bypass)
    double s = 0.0;
    int cnt1 = 0;
    int64_t mn1 = INT64_MAX, mx1 = INT64_MIN;
    auto add = [&](int64_t e, int& c, int64_t& mn, int64_t& mx) {
        const bool in = e > tmin && e <= tmax;
        c += in;
        mn = in ? min(mn, e) : mn;
        mx = in ? max(mx, e) : mx;
    };
    // the terms stay in registers (they replace the rows' ts / usage) until a stepped lane has
    // its record slot (after B): no second read of the rows
    int64_t ep[PR];
    double tp[PR];
#pragma unroll
    for (int k = 0; k < PR; ++k) {
        const bool use = k < npr && qt[k] != kTsInvalid && !(qv[k] < 0.0);
        double term = (1.0 - qv[k]) * pol.prio_w[k];  // getScore (stats.go:89), no FMA
        term = term * 100.0;
        const int64_t e = sat_add(qt[k], pol.prio_dur[k]);
        ep[k] = use ? e : kTsInvalid;
        tp[k] = use ? term : 0.0;
        s = tmin < ep[k] ? s + tp[k] : s;  // stats.go:124-133
        add(ep[k], cnt1, mn1, mx1);
    }
    add(hr.e_hv, cnt1, mn1, mx1);
    int cnt0 = cnt1;
    int64_t mn0 = mn1, mx0 = mx1;
    add(e_fail, cnt0, mn0, mx0);
    if (!valid) cnt0 = cnt1 = 0;
    const int32_t s0 = score_of_sum(s, tmin < hr.e_hv ? hr.pen : 0, step.wsum, step.noprio, step.winv);
    const bool multi0 = cnt0 > 0 && mn0 != mx0, multi1 = cnt1 > 0 && mn1 != mx1;
    StepSlots so;
    so.flat0 = valid && cnt0 == 0 && !(tmin < e_fail) ? pack_key(s0, n) : -1;
    so.flat1 = valid && cnt1 == 0 ? pack_key(s0, n) : -1;
    CRANE_TSTAMP(a.trace, blockIdx.x, 2);
    // ---- B: slots (wave prefix sums, the waves' totals exchanged once: one barrier)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t w0 = (cnt0 ? (multi0 ? 2u : 1u) : 0u) | (multi0 ? (uint32_t)(cnt0 - 1) << 16 : 0u);
    const uint32_t w1 = (cnt1 ? (multi1 ? 2u : 1u) : 0u) | (multi1 ? (uint32_t)(cnt1 - 1) << 16 : 0u);
    const uint32_t w2 = (cnt0 | cnt1) ? 1u : 0u;
    uint32_t e0 = wave_scan_add(w0), e1 = wave_scan_add(w1), e2 = wave_scan_add(w2);
#if K1S_PUB1
    // the flat maxima per wave go out with the totals (step_publish's exchange: one barrier for both)
    const int32_t fm0 = wave_max(so.flat0), fm1 = wave_max(so.flat1);
    if (lane == 0) {
        ssh.fm[0][wv] = fm0;
        ssh.fm[1][wv] = fm1;
    }
#endif
    if (lane == 63) {
        xch[0][wv] = e0;
        xch[1][wv] = e1;
        xch[2][wv] = e2;
    }
    e0 -= w0;
    e1 -= w1;
    e2 -= w2;
    __syncthreads();
    uint32_t base[3], tot[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint4 x = *reinterpret_cast<const uint4*>(xch[k]);
        base[k] = (wv > 0 ? x.x : 0u) + (wv > 1 ? x.y : 0u) + (wv > 2 ? x.z : 0u);
        tot[k] = x.x + x.y + x.z + x.w;
    }
    const int32_t slot0 = cnt0 ? (int32_t)((base[0] + e0) & 0xFFFF) : -1;
    const int32_t mslot0 = multi0 ? (int32_t)((base[0] + e0) >> 16) : 0;
    const int32_t slot1 = cnt1 ? (int32_t)((base[1] + e1) & 0xFFFF) : -1;
    const int32_t mslot1 = multi1 ? (int32_t)((base[1] + e1) >> 16) : 0;
    const int32_t rs = (int32_t)(base[2] + e2);  // rank among the block's stepped nodes
    const int32_t nst = (int32_t)tot[2];
    if (threadIdx.x == 0) {
        ssh.lc[0][0] = (int32_t)(tot[0] & 0xFFFF);
        ssh.lc[0][1] = (int32_t)(tot[0] >> 16);
        ssh.lc[1][0] = (int32_t)(tot[1] & 0xFFFF);
        ssh.lc[1][1] = (int32_t)(tot[1] >> 16);
    }
#if K1S_PUB1
    // step_publish's stores from the exchanged values (ssh.lc is read after the next barrier)
    if (threadIdx.x < 2) {
        const int T = threadIdx.x;
        step.st.flat[blk * 2 + T] = max(max(ssh.fm[T][0], ssh.fm[T][1]), max(ssh.fm[T][2], ssh.fm[T][3]));
    } else if (threadIdx.x < 6) {
        const int L = threadIdx.x - 2;  // kind L >> 1: one-step records (L & 1 = 0) / middle pieces
        step.st.cnt[blk * 4 + L] = (int32_t)((L & 1) ? tot[L >> 1] >> 16 : tot[L >> 1] & 0xFFFF);
    }
    const bool g1 = (int32_t)max(tot[0] & 0xFFFF, tot[1] & 0xFFFF) > min(kSCap, step.st.lds_cap);
    CRANE_TSTAMP(a.trace, blockIdx.x, 3);
#else
    step_publish<BS>(so, ssh, step.st, blk);  // flat maxima, counts (its barrier: ssh.lc final)
    CRANE_TSTAMP(a.trace, blockIdx.x, 3);
    // one-step records staged in LDS, or (more of a kind than it holds) in st.stage
    const bool g1 = max(ssh.lc[0][0], ssh.lc[1][0]) > min(kSCap, step.st.lds_cap);
#endif
    const S1Out s1o{s1l, step.st.stage + blk * 2 * step.st.bs, g1, (int64_t)kSCap, step.st.s1pad};
    // ---- C: the stepped nodes' records in LDS, chunk by chunk, and their (node, kind) items.
    // The first kSRec stepped nodes write their part (e_fail, pen, e_hv, slots) into the LDS
    // records now; any further ones into their node's record slot in HBM (step.srec, the node
    // records the keys-only step leaves stale anyway: the slots go in e_pred, which the emit does
    // not read), fetched chunk by chunk — no per-lane state lives across the chunks.
    const bool stepped = (cnt0 | cnt1) != 0;
    auto put = [&](Rec* r) {  // (called with an LDS and a global pointer: no flat stores)
        r->e_fail = e_fail;
        r->pen = hr.pen;
        r->e_hv = hr.e_hv;
#pragma unroll
        for (int k = 0; k < PR; ++k) {
            r->e_prio[k] = ep[k];
            r->t[k] = tp[k];
        }
        int32_t* dw = reinterpret_cast<int32_t*>(r->e_pred);
        dw[0] = slot0;
        dw[1] = mslot0;
        dw[2] = slot1;
        dw[3] = mslot1;
        dw[4] = (multi0 ? 1 : 0) | (multi1 ? 2 : 0);
        dw[5] = s0;  // score_at(tmin): the keys before a node's first step
    };
    if (stepped && !(K1S_SKIP & 4)) {
        rank_lane[rs] = (uint8_t)threadIdx.x;
        if (rs < kSRec) put(&lrec[rs]);
        else put(static_cast<Rec*>(step.srec) + n);
    }
    __syncthreads();
    // a grid of many rounds: the epilogue's single-wave phases run on wave 0 alone and the other
    // waves leave, so their slots take the next workgroups' streams — before the emit when its
    // tasks fit one wave, else before the tail; a grid of one or two rounds keeps all four waves
    // (its time is one workgroup's chain)
    const bool t1 = K1S_TAIL1 && (step.tail1 == 1 || (step.tail1 == 0 && gridDim.x >= 4096));
    const bool emit1 = t1 && nst * (PR + 2) <= 64;  // (workgroup-uniform)
    if (emit1 && threadIdx.x >= 64) return;
    const int nthr = emit1 ? 64 : BS;
    for (int32_t c0 = 0; c0 < ((K1S_SKIP & 1) ? 0 : nst); c0 += kSRec) {  // (workgroup-uniform)
        const int32_t m = min(kSRec, nst - c0);
        if (c0 > 0) {  // this chunk's records from HBM (L2: written by this workgroup)
            constexpr int W = 3 + 2 * PR + 3;  // e_fail, e_hv, pen, e_prio, t, then the slot words
            for (int i = threadIdx.x; i < m * W; i += BS) {
                const int j = i / W, f = i - j * W;
                const int64_t* src = reinterpret_cast<const int64_t*>(static_cast<const Rec*>(step.srec) + first +
                                                                      rank_lane[c0 + j]);
                reinterpret_cast<int64_t*>(&lrec[j])[f] = src[f];
            }
            __syncthreads();
        }
        {
            constexpr int NB = PR + 2;
            for (int tk = threadIdx.x; tk < m * NB; tk += nthr) {  // (node, candidate): both kinds
                const int j = tk / NB;
                int q = tk - j * NB;
                // (q = threadIdx.x % NB in every trip: without this the compiler hoists emit_task's
                // per-q lane masks out of the loop and spills them, ~30 SGPRs for the whole kernel)
                asm volatile("" : "+v"(q));
                emit_task<PD, PR>(lrec[j], first + rank_lane[c0 + j], q,
                                  reinterpret_cast<const int32_t*>(lrec[j].e_pred), tmin, tmax, step.wsum, step.noprio,
                                  step.st, blk, s1o, step.winv);
            }
        }
        __syncthreads();  // (the chunk's records are reused by the next chunk)
    }
    CRANE_TSTAMP(a.trace, blockIdx.x, 5);
    // ---- D: the fused pass's tail
    if (K1S_SKIP & 2) return;
    if (t1) {
        if (threadIdx.x >= 64) return;
        if (threadIdx.x < 2) {  // the block's flat maxima into wave 0's slot (tile rows read it)
            const int T = threadIdx.x;
            ssh.fm[T][0] = max(max(ssh.fm[T][0], ssh.fm[T][1]), max(ssh.fm[T][2], ssh.fm[T][3]));
        }
        tail<64>(g1, lrec, s1l, srt, ssh, step, blk, a.trace);
        return;
    }
    tail<BS>(g1, lrec, s1l, srt, ssh, step, blk, a.trace);
}

template <int PD, int PR, bool FULL = false>
static hipError_t launch_t(const K1Args& a, const K1Step& sa, hipStream_t st) {
    const unsigned grid = (unsigned)((a.N + 255) / 256);
    return klaunch("k1_stream_steps", k1_stream_steps<PD, PR, FULL>, dim3(grid), dim3(256), 0, st, a, sa);
}

hipError_t launch_stream_steps(int pd, int pr, const K1Args& a, const K1Step& sa, hipStream_t st) {
    if (a.N <= 0) return hipSuccess;
    if (K1S_FULL && a.pol.npd == 4 && a.pol.npr == 6 && a.pol.n_win == kFullWin) return launch_t<4, 6, true>(a, sa, st);
    if (pd <= 4 && pr <= 6) return launch_t<4, 6>(a, sa, st);
    if (pd <= 8 && pr <= 8) return launch_t<8, 8>(a, sa, st);
    return launch_t<16, 16>(a, sa, st);
}

}  // namespace crane
