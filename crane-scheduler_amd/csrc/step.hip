// step.hip — K3 "step" path: the pod x node Filter + Score + argmax with every
// pod-invariant operation hoisted into a per-batch node pass.
//
// Why it is exact.  For a fixed node, Filter (plugins.go:39-69) and Score
// (plugins.go:73-98, stats.go:114-166) depend on the pod only through `now`,
// and on `now` only through comparisons now < expiry against the node's
// expiries (e_fail, e_prio[k], e_hv; stats.go:42-48).  Over a pod batch whose
// times lie in [tmin, tmax], only expiries b with tmin < b <= tmax can split
// the batch, so the node's packed (feasible, score, index) key is a step
// function of `now` with at most PR + 2 steps.  K3a evaluates that function
// once per step with the literal int64 restatement (score_at), at the first
// instant of the step.  A node with no step inside the batch ("flat", ~95 %
// of nodes at config 3) has the same key for every pod of a kind, so its part
// of every pod's argmax is one max over the flat keys of the batch, taken once
// in K3a; K3s resolves the remaining (pod, stepped node) pairs by selecting
// each pod's step: a 64-bit compare + select + max per pair.
//
//   K3p  pods  : per 1024-pod tile, pods sorted by (kind, now) (pods.hpp),
//                key init, per-tile time range and counts per kind
//   K3a  nodes : per node, both pod kinds (Filter applies / DaemonSet bypass,
//                utils.go:17-24): flat key -> workgroup max; stepped node ->
//                its key pieces (one-step records sorted per workgroup with
//                prefix / suffix key maxima, middle pieces), step_node.hpp
//   K3s  pairs : a 1024-pod tile per workgroup, R workgroups per tile split
//                the producer blocks: binary searches find each block's
//                records stepping inside the tile's time range, one prefix and
//                one suffix maximum give the key of all others; a record inside
//                splits the tile's sorted pods of its kind into two slot ranges
//                (a middle piece cuts out one), applied as range maxima on an
//                LDS segment tree; one 64-bit atomicMax per pod per workgroup
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dyn_types.hpp"
#include "kernels.hpp"
#include "pods.hpp"
#include "lds_hash.hpp"
#include "step_node.hpp"

#ifndef K3S_BUCKETS  // slot searches through a per-kind time-bucket table (A/B: 0 plain binary search)
#define K3S_BUCKETS 1
#endif
#ifndef K3_KWARM  // the launch's kernarg lines warmed in the scalar cache first (A/B: 0 off)
#define K3_KWARM 1
#endif

namespace crane {

// ---------------------------------------------------------------- K3p
constexpr int kPodTile = 1024;

__global__ __launch_bounds__(kPodTile) void k3p_pods(PodPrep pp) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    k3p_tile<kPodTile>(blockIdx.x, pp, lds);
}

// ---------------------------------------------------------------- K3a
// Stand-alone step tables from NodeRecs already in HBM (the node pass ran
// earlier); one thread per node.  The fused form is K1's STEP variant.
template <int PD, int PR>
__global__ __launch_bounds__(kStepSeg) void k3a_steps(const NodeRec<PD, PR>* __restrict__ rec, int64_t N,
                                                      const int64_t* __restrict__ tile_mm, int32_t ntiles,
                                                      double wsum, int32_t noprio, StepTables st) {
    __shared__ int64_t smn[kStepSeg / 64], smx[kStepSeg / 64];
    __shared__ StepShared sh;
    __shared__ Step1 s1l[4 * kStepSeg], s1s[4 * kStepSeg];  // one-step records per kind: staging, sorted
    if (threadIdx.x < 4) sh.lc[threadIdx.x >> 1][threadIdx.x & 1] = 0;
    int64_t tmin, tmax;
    batch_range<kStepSeg>(tile_mm, ntiles, smn, smx, tmin, tmax);  // (its barrier orders the lc reset)
    const int64_t n = (int64_t)blockIdx.x * kStepSeg + threadIdx.x;
    StepSlots o;
    NodeRec<PD, PR> r;
    if (n < N) {
        r = rec[n];
        step_count<PD, PR>(r, n, tmin, tmax, wsum, noprio, sh, o);
    }
    step_publish<kStepSeg>(o, sh, st, blockIdx.x);
    if (n < N && (o.slot0 >= 0 || o.slot1 >= 0)) step_emit<PD, PR>(r, n, tmin, tmax, wsum, noprio, o, st, blockIdx.x, S1Out{s1l, nullptr, false, 2 * kStepSeg, 0});
    __syncthreads();
    step_sort_publish<kStepSeg>(s1l, s1s, sh, st, blockIdx.x);
    if (st.rows) {
        int64_t pre;
        tile_prefetch(st, &pre);
        // middle pieces' scratch: s1l past the prefix / suffix maxima ([2][2 * kStepSeg] int32 each)
        const PieceScr ps{reinterpret_cast<unsigned char*>(s1l) + 32 * kStepSeg,
                          ((int)sizeof(s1l) - 32 * kStepSeg) / PieceScr::bytes_per_piece & ~3};
        step_pieces<kStepSeg>(sh, st, blockIdx.x, ps);
        step_tile_rows<kStepSeg>(s1l, s1s, sh, st, blockIdx.x, &pre, ps);
    }
}

// ---------------------------------------------------------------- K3s
// Workgroup = 4 waves, one 1024-pod tile of K3p's sorted order (thread x holds
// slots u * 256 + x); kind 0 pods are slots [0, cn), kind 1 [cn, cn + cd),
// each sorted by now.  The R workgroups of a tile split the producer blocks:
// m per workgroup, LPB lanes per block (the block's leader does the searches,
// all its lanes share the record work).
// One-step records: each block's are sorted by step time bp with prefix maxima
// of the after-step key (pm1) and suffix maxima of the before-step key (sm0)
// (step_sort_publish).  For a kind's pod time range [lo, hi] the leader finds
// by two binary searches the records stepping inside (lo, hi]; every pod of
// the kind sees the key after the step of each earlier record (one prefix
// maximum) and the key before the step of each later one (one suffix maximum).
// A record inside splits the kind's slots at the first pod with now >= bp
// (binary search over the tile's times in LDS): k0 is a range maximum over the
// slots before, k1 over the slots from there on.  Middle pieces [s, e) of
// multi-step nodes: one covering [lo, hi] is uniform, one overlapping it
// partly is the range maximum over the slots with s <= now < e.  Range maxima
// go into a segment tree over the 1024 slots (<= 20 LDS atomics each); a pod's
// key is the max over its leaf's ancestors, the kind's uniform maximum and
// what the other workgroups of the tile merge: one 64-bit atomicMax per pod
// per workgroup.
// 8 waves (512 lanes, 2 pods per lane) against 4: K3s 10.6 -> 9.6 us at config 3, 65.4 ->
// 61 us at config 4 on one GPU, same box (profiles/r06/ab/k1_first_entry_rows_dropped_k3s_8waves.txt)
constexpr int kK3sWaves = 8;
constexpr int kK3sThreads = kK3sWaves * 64;
constexpr int kK3sPPL = 1024 / kK3sThreads;         // pods per lane
constexpr int kK3sPods = kK3sThreads * kK3sPPL;     // pods per workgroup (= kPodTile)
// producer blocks per workgroup aimed for (launches over kMaxWg workgroups are capped first):
// 64 -> config 3 (391 blocks) and the config-4 shard (489) take 8 workgroups per tile.  Round 3,
// same box (option k3s_blocks, tools/gpu_r03k3.sh / gpu_r03k3b.sh): shard 0.0343 -> 0.0300 ms
// per batch with 4 in flight (R 16 -> 8), config 3 unchanged (0.0120-0.0126); 32 per tile (16
// blocks) had measured 0.0128 vs 0.0123 at config 3 in round 2
constexpr int kK3sBlkPerWg = 64;  // (round 6, 8-wave K3s: 32 per workgroup within noise, 16 slower: profiles/r06/ab/k3s_blocks_per_wg.txt)
// Work lists (k3s_eval) for slices of at most kK3sListBlk blocks, holding at most this many
// straddling records / middle pieces (more: the blocks' teams).  Same-box A/B at configs 3 / 4
// (one GPU) / 4 shard against the team loops alone: K3s 0.0397 -> 0.0364 ms per batch,
// 0.122 -> 0.118 ms, 28.7 -> 24.8 us; every record and piece listed (and 4x the LDS):
// 0.0362, 0.270 ms, 52 us (tools/gpu_lib_ab.sh)
constexpr int kK3sListBlk = 64;
constexpr int kSearchBucketBits = 8, kSearchBuckets = 1 << kSearchBucketBits;  // K3S_BUCKETS: per kind
constexpr int kK3sRecList = 512;
constexpr int kK3sPieceList = 512;
static_assert(kK3sMaxBlk <= kK3sThreads, "at least one lane per producer block");
static_assert(4 * kK3sListBlk <= 256, "list entries index the item map in 8 bits");
static_assert(kK3sPods == kPodTile, "a workgroup resolves one K3p tile");

// The four counts "records of kind T with bp <= t" (t = the kind's lo, then hi)
// over a block's sorted one-step records, by a k-ary search of the block's lpb
// lanes (lanes [lead, lead + lpb) of one wave): each round every lane probes one
// record per search and a ballot narrows the range to one of lpb + 1 parts;
// the four searches' loads go out together.  Every lane of the team returns the
// counts.  (n = 0 for a kind without pods here.)
__device__ __forceinline__ void team_count_le(const Step1* __restrict__ b0, const Step1* __restrict__ b1,
                                              const int32_t n[2], const int64_t tl[2], const int64_t th[2], int sub,
                                              int lpb, int lead, int32_t out[4]) {
    const uint64_t team = lpb == 64 ? ~0ull : ((1ull << lpb) - 1ull) << lead;
    int32_t lo[4] = {0, 0, 0, 0}, hi[4] = {n[0], n[0], n[1], n[1]};
    const int64_t t[4] = {tl[0], th[0], tl[1], th[1]};
    while ((lo[0] < hi[0]) | (lo[1] < hi[1]) | (lo[2] < hi[2]) | (lo[3] < hi[3])) {  // team-uniform
        bool le[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int32_t span = hi[q] - lo[q];
            const int32_t p = lo[q] + (int32_t)((int64_t)span * (sub + 1) / (lpb + 1));  // < hi when span > 0
            le[q] = span > 0 && (q < 2 ? b0 : b1)[p].bp <= t[q];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int32_t span = hi[q] - lo[q];
            if (span <= 0) continue;
            const int k = __popcll(__ballot(le[q]) & team);  // probes with bp <= t (a prefix of the team)
            const int32_t nlo = k > 0 ? lo[q] + (int32_t)((int64_t)span * k / (lpb + 1)) + 1 : lo[q];
            const int32_t nhi = k < lpb ? lo[q] + (int32_t)((int64_t)span * (k + 1) / (lpb + 1)) : hi[q];
            lo[q] = nlo;
            hi[q] = nhi;
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) out[q] = lo[q];
}

// first slot in [lo, hi) of the sorted times tt[] with tt >= x (hi if none)
__device__ __forceinline__ int32_t slot_lower(const int64_t* tt, int32_t lo, int32_t hi, int64_t x) {
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (tt[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// key k as a range maximum over slots [a, b) of the segment tree (leaves at kK3sPods + slot)
__device__ __forceinline__ void tree_max(int32_t* tree, int32_t a, int32_t b, int32_t k) {
    for (int32_t l = a + kK3sPods, r = b + kK3sPods; l < r; l >>= 1, r >>= 1) {
        if (l & 1) atomicMax(&tree[l++], k);
        if (r & 1) atomicMax(&tree[--r], k);
    }
}

__device__ __forceinline__ void k3s_body(const int64_t b, const StepTables& st, const int32_t* __restrict__ perm,
                                         const int64_t* __restrict__ pnow, const int64_t* __restrict__ tile_mm,
                                         int64_t P, int64_t node_offset, int32_t R, long long* __restrict__ keys) {
    __shared__ int64_t tt[kK3sPods];         // the tile's pod times (sorted per kind)
    __shared__ int32_t tree[2 * kK3sPods];   // range maxima: node i covers its leaves' slots
    __shared__ int32_t umax[2];
    // work lists (slices of <= kK3sListBlk blocks): records stepping inside / middle pieces per
    // (block, kind), turned in place into their exclusive prefix (+ the total); the first record
    // stepping inside per (block, kind).  Small: K3s runs several rounds of workgroups at config 4
    // and its LDS sets how many share a CU
    __shared__ int32_t wpre[4 * kK3sListBlk + 1];
    __shared__ int32_t wjl[2 * kK3sListBlk];
    __shared__ int32_t wpl[2 * kK3sListBlk];  // the first middle piece per (block, kind)
    // item -> its entry: the list's records and pieces expanded (one LDS read per item instead of a
    // binary search of the prefix, 8 dependent reads)
    __shared__ uint8_t imap[kK3sRecList + kK3sPieceList];
#if K3S_BUCKETS
    // per kind, the first slot of each time bucket (bucket k: [lo + k 2^sh, lo + (k + 1) 2^sh)): a
    // slot search reads its bucket's two bounds and searches the few slots between them
    __shared__ int32_t sfirst[2][kSearchBuckets + 1];
#endif
    CRANE_TSTAMP(st.trace, b, 0);
    const int32_t r = (int32_t)(b % R);
    const int64_t grp = b / R;
    const int lane = threadIdx.x & 63;
    // the tile's kinds: time range and slot range (K3p's tile stats): one vector load, lane k
    // stat k, issued after this slice's and the pods' loads and broadcast once they are in (as
    // scalar loads they missed the scalar cache, and any scalar load's wait waits for all of them)
    const int64_t* ts = tile_mm + kTileStat * grp;
    // the slice's producer blocks: with R a multiple of 8, workgroup label g = r % 8 (= its
    // XCD group, blockIdx % 8) takes the blocks the node pass ran in the same group — its
    // workgroup w built block xcd_block(w) (step_node.hpp), the contiguous run of XCD w % 8 —
    // so their step tables are read from this XCD's L2; sub-slice s = r / 8 takes every S-th
    // of them (neighbouring blocks — hot nodes cluster, and with them the step records —
    // spread over the group's workgroups).  LPB lanes per block (a power of two <= 64).
    // (Placement only changes speed: the blocks covered depend on blockIdx alone.)
    int32_t xc = 0, stride = 1, k0 = 0, m = 0;
    if (R % 8 == 0) {
        const int32_t g = r & 7, S = R >> 3, s = r >> 3;
        const int32_t per = st.nblk >> 3, rem = st.nblk & 7;
        const int32_t nc = per + (g < rem ? 1 : 0);  // the group's blocks: base + k, k < nc
        xc = g * per + min(g, rem) + s;              // this sub-slice's: base + s + S j
        stride = S;
        m = nc > s ? (nc - s + S - 1) / S : 0;
    } else {
        const int32_t per = (st.nblk + R - 1) / R;
        k0 = min(st.nblk, r * per);
        m = min(st.nblk, k0 + per) - k0;
    }
    int32_t lpb = 64;
    while (lpb > 1 && lpb * m > kK3sThreads) lpb >>= 1;
    const int32_t j = threadIdx.x / lpb, sub = threadIdx.x & (lpb - 1);
    const bool own = j < m;
    const int64_t ob = xc + (int64_t)stride * (k0 + j);
    const int lead = lane - sub;  // the block's leader lane (same wave)
    // the block's team: counts (one broadcast load), the searches; the leader adds the
    // flat maxima and the prefix / suffix maxima to the uniform keys
    // this slice's loads first (counts, the tile rows), then the pods, so they overlap
    int4 c = make_int4(0, 0, 0, 0);  // [records kind 0, pieces 0, records 1, pieces 1]
    int4 row = make_int4(-1, -1, 0, 0);
    int2 prow = make_int2(0, 0);
    if (own) {
        c = reinterpret_cast<const int4*>(st.cnt)[ob];
        if (st.rows) row = st.rows[grp * st.nblk + ob];
        if (st.prow) prow = st.prow[grp * st.nblk + ob];
    }
    bool live[kK3sPPL], ds[kK3sPPL];
    int32_t pod[kK3sPPL];
    // every pod load issued before the first LDS store waits for one (unconditional, clamped
    // slot): a conditional load per pod made each store wait for its own round trip
    int32_t praw[kK3sPPL];
    int64_t pn[kK3sPPL];
#pragma unroll
    for (int u = 0; u < kK3sPPL; ++u) {
        const int64_t slot = grp * kK3sPods + u * kK3sThreads + threadIdx.x;
        live[u] = slot < P;
        const int64_t sc = live[u] ? slot : 0;
        praw[u] = perm[sc];
        pn[u] = pnow[sc];
    }
#pragma unroll
    for (int u = 0; u < kK3sPPL; ++u) {
        tt[u * kK3sThreads + threadIdx.x] = live[u] ? pn[u] : INT64_MAX;
        const int32_t pr = live[u] ? praw[u] : 0;
        ds[u] = pr < 0;
        pod[u] = pr & 0x7FFFFFFF;
    }
    const int64_t tsv = ts[lane < kTileStat ? lane : 0];
    for (int i = threadIdx.x; i < 2 * kK3sPods; i += kK3sThreads) tree[i] = -1;
    if (threadIdx.x < 2) umax[threadIdx.x] = -1;
    auto stat = [&](int k) {
        const uint32_t lo32 = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)tsv, k);
        const uint32_t hi32 = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)tsv >> 32), k);
        return (int64_t)(((uint64_t)hi32 << 32) | lo32);
    };
    const int64_t tlo[2] = {stat(0), stat(2)}, thi[2] = {stat(1), stat(3)};
    const int32_t cn = (int32_t)stat(4), cd = (int32_t)stat(5);
    const int32_t klo[2] = {0, cn}, khi[2] = {cn, cn + cd};
    const bool any[2] = {cn > 0, cd > 0};
#if K3S_BUCKETS
    int32_t sbs[2];  // bucket width 2^sbs per kind: the kind's time span in kSearchBuckets buckets
#pragma unroll
    for (int T = 0; T < 2; ++T) {
        const uint64_t span = klo[T] < khi[T] ? (uint64_t)(thi[T] - tlo[T]) : 0ull;
        const int bits = span ? 64 - __builtin_clzll(span) : 0;
        sbs[T] = bits > kSearchBucketBits ? bits - kSearchBucketBits : 0;
    }
    // first slot of kind T with tt >= x (slot_lower over [klo, khi)): its bucket's bounds, then
    // a binary search of the slots between them
    auto find = [&](int T, int64_t x) -> int32_t {
        if (klo[T] >= khi[T] || x <= tlo[T]) return klo[T];
        if (x > thi[T]) return khi[T];
        const int32_t k = (int32_t)((uint64_t)(x - tlo[T]) >> sbs[T]);
        return slot_lower(tt, sfirst[T][k], sfirst[T][k + 1], x);
    };
#else
    auto find = [&](int T, int64_t x) -> int32_t { return slot_lower(tt, klo[T], khi[T], x); };
#endif
    CRANE_TSTAMP(st.trace, b, 5);  // (pods in: the LDS stores waited for them)
    const int32_t n1[2] = {any[0] ? c.x : 0, any[1] ? c.z : 0};
    // middle pieces [pl, pl + nm) per kind: with piece ranges, those overlapping the tile (the
    // producer's elementary pieces, step_pieces), else all of them
    const int32_t pl[2] = {st.prow ? prow.x & 0xFFFF : 0, st.prow ? prow.y & 0xFFFF : 0};
    const int32_t nm[2] = {any[0] ? (st.prow ? (prow.x >> 16) - pl[0] : c.y) : 0,
                           any[1] ? (st.prow ? (prow.y >> 16) - pl[1] : c.w) : 0};
    const Step1* base[2] = {st.single + s1_at(st, 0, ob), st.single + s1_at(st, 1, ob)};
    int32_t jj[4] = {0, 0, 0, 0};  // jl[0], jh[0], jl[1], jh[1]
    int32_t um[2] = {-1, -1};
    if (st.rows) {
        // the producer wrote this tile's uniform keys and record ranges (step_sort_publish)
        if (own) {
            jj[0] = row.z & 0xFFFF;
            jj[1] = row.z >> 16;
            jj[2] = row.w & 0xFFFF;
            jj[3] = row.w >> 16;
            if (sub == 0) {
                um[0] = row.x;
                um[1] = row.y;
            }
        }
    } else {
        if (own) team_count_le(base[0], base[1], n1, tlo, thi, sub, lpb, lead, jj);
        if (own && sub == 0) {
#pragma unroll
            for (int T = 0; T < 2; ++T) {
                if (!any[T]) continue;
                const int64_t o = s1_at(st, T, ob);
                int32_t u = st.flat[ob * 2 + T];
                if (jj[2 * T] > 0) u = max(u, st.pm1[o + jj[2 * T] - 1]);
                if (jj[2 * T + 1] < n1[T]) u = max(u, st.sm0[o + jj[2 * T + 1]]);
                um[T] = u;
            }
        }
    }
    // the slice's work as lists over the workgroup's lanes, so a block with many records
    // (hot nodes) is spread over every lane instead of its team's: entries e < 2m are
    // (block, kind) one-step records stepping inside, e >= 2m (block, kind) middle pieces
    const bool lists = m <= kK3sListBlk;  // (workgroup-uniform)
    if (lists && own && sub == 0) {
        wpre[2 * j + 0] = max(0, jj[1] - jj[0]);
        wpre[2 * j + 1] = max(0, jj[3] - jj[2]);
        wpre[2 * m + 2 * j + 0] = nm[0];
        wpre[2 * m + 2 * j + 1] = nm[1];
        wjl[2 * j] = jj[0];
        wjl[2 * j + 1] = jj[2];
        wpl[2 * j] = pl[0];
        wpl[2 * j + 1] = pl[1];
    }
    __syncthreads();  // tt, tree, umax initialised; the counts in
    CRANE_TSTAMP(st.trace, b, 1);
    const int32_t E = 4 * m;
    // the bucket table (K3S_BUCKETS): lane (T, k) searches bucket k's first slot of kind T, all at
    // once (one search's time, wave 0 after its prefix), ordered by the next barrier
    auto bucket_table = [&]() {
#if K3S_BUCKETS
        static_assert(kK3sThreads == 2 * kSearchBuckets, "a lane per (kind, bucket)");
        const int T = threadIdx.x / kSearchBuckets, k = threadIdx.x % kSearchBuckets;
        if (klo[T] < khi[T]) {
            sfirst[T][k] = slot_lower(tt, klo[T], khi[T], tlo[T] + ((int64_t)k << sbs[T]));
            if (k == 0) sfirst[T][kSearchBuckets] = khi[T];
        }
#endif
    };
    int32_t nrec = 0, total = 0;
    if (lists) {
        if (threadIdx.x < 64) {  // wave 0: exclusive prefix over the entries, in place (wpre[E] = total)
            const int32_t v = lane < E ? wpre[lane] : 0;  // E <= 4 * kK3sListBlk = 256: four chunks
            int32_t carry = (int32_t)wave_scan_add((uint32_t)v);
            if (lane < E) wpre[lane] = carry - v;
            carry = __builtin_amdgcn_readlane(carry, 63);
            for (int32_t e0 = 64; e0 < E; e0 += 64) {
                const int32_t e = e0 + lane;
                const int32_t x = e < E ? wpre[e] : 0;
                const int32_t inc = (int32_t)wave_scan_add((uint32_t)x) + carry;
                if (e < E) wpre[e] = inc - x;
                carry = __builtin_amdgcn_readlane(inc, 63);
            }
            if (lane == 0) wpre[E] = carry;
        }
        bucket_table();
        __syncthreads();
        nrec = wpre[2 * m];
        total = wpre[E];
    } else if (K3S_BUCKETS) {
        bucket_table();
        __syncthreads();
    }
    const bool piece_list = lists && total - nrec <= kK3sPieceList;
    const bool rec_list = lists && nrec <= kK3sRecList;
    bool upd = false;  // this lane wrote the tree
    const int32_t i0 = rec_list ? 0 : nrec, i1 = piece_list ? total : nrec;  // (workgroup-uniform)
    if (i1 > i0) {
        // the entries' items into the map (an entry's lane writes its run; E <= 256 entries)
        for (int32_t e = threadIdx.x; e < E; e += kK3sThreads) {
            const int32_t a = max(wpre[e], i0), z = min(wpre[e + 1], i1);
            for (int32_t i = a; i < z; ++i) imap[i - i0] = (uint8_t)e;
        }
        __syncthreads();
        // every item of this lane: its entry, then its record / piece loads all in flight, then the
        // searches and the tree
        constexpr int kU = (kK3sRecList + kK3sPieceList) / kK3sThreads;
        Step1 r1[kU];
        Mid pm[kU];
        int32_t ee[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int32_t it = i0 + u * kK3sThreads + (int32_t)threadIdx.x;
            ee[u] = -1;
            if (it >= i1) continue;
            const int32_t e = imap[it - i0];
            ee[u] = e;
            const bool rec = e < 2 * m;
            const int32_t ej = rec ? e : e - 2 * m, jb = ej >> 1, T = ej & 1, idx = it - wpre[e];
            const int64_t obj = xc + (int64_t)stride * (k0 + jb);
            if (rec) r1[u] = (st.single + s1_at(st, T, obj))[wjl[2 * jb + T] + idx];
            else pm[u] = st.mid[(int64_t)T * st.mpad + obj * st.mstride + wpl[ej] + idx];
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int32_t e = ee[u];
            if (e < 0) continue;
            const bool rec = e < 2 * m;
            const int T = (rec ? e : e - 2 * m) & 1;
            if (rec) {
                // a one-step record stepping inside (lo, hi]: split the kind's slots
                const int32_t sp = find(T, r1[u].bp);
                if (r1[u].k0 >= 0) tree_max(tree, klo[T], sp, r1[u].k0);
                if (r1[u].k1 >= 0) tree_max(tree, sp, khi[T], r1[u].k1);
                upd = true;
            } else {
                // a middle piece: covering -> uniform, overlapping partly -> range maximum over
                // the slots with s <= now < e
                const Mid& q = pm[u];
                if (q.s <= tlo[T] && q.e > thi[T]) um[T] = max(um[T], q.key);
                else if (q.s <= thi[T] && q.e > tlo[T]) {
                    tree_max(tree, find(T, q.s), find(T, q.e), q.key);
                    upd = true;
                }
            }
        }
    }
    if (own && !rec_list) {
#pragma unroll
        for (int T = 0; T < 2; ++T) {
            // many records: by the block's team (consecutive records, a lane each)
            for (int32_t i = jj[2 * T] + sub; i < jj[2 * T + 1]; i += lpb) {
                const Step1 q = base[T][i];
                const int32_t sp = find(T, q.bp);
                if (q.k0 >= 0) tree_max(tree, klo[T], sp, q.k0);
                if (q.k1 >= 0) tree_max(tree, sp, khi[T], q.k1);
                upd = true;
            }
        }
    }
    CRANE_TSTAMP(st.trace, b, 6);
    if (own && !piece_list) {
#pragma unroll
        for (int T = 0; T < 2; ++T) {
            const Mid* mp = st.mid + (int64_t)T * st.mpad + ob * st.mstride + pl[T];
            for (int32_t i0 = sub; i0 < nm[T]; i0 += 4 * lpb) {
                Mid q[4];
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const int32_t i = i0 + v * lpb;
                    if (i < nm[T]) q[v] = mp[i];
                    else q[v].s = INT64_MAX;  // (matches nothing)
                }
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const Mid& pm = q[v];
                    if (pm.s <= tlo[T] && pm.e > thi[T]) um[T] = max(um[T], pm.key);
                    else if (pm.s <= thi[T] && pm.e > tlo[T]) {
                        tree_max(tree, find(T, pm.s), find(T, pm.e), pm.key);
                        upd = true;
                    }
                }
            }
        }
    }
    CRANE_TSTAMP(st.trace, b, 2);
    // uniform maxima: wave reduce, one LDS atomic per wave
#pragma unroll
    for (int T = 0; T < 2; ++T) {
        um[T] = wave_max(um[T]);
        if (lane == 0 && um[T] >= 0) atomicMax(&umax[T], um[T]);
    }
    const bool tree_used = __syncthreads_or(upd);
    CRANE_TSTAMP(st.trace, b, 3);
    // a pod's key: the max over its leaf's ancestors (every level's load issued at once, for
    // all of the lane's pods: one LDS round trip, not a dependent walk per pod)
    constexpr int kLevels = 11;  // leaves at kK3sPods + slot, root at 1
    static_assert(kK3sPods == 1 << (kLevels - 1), "a segment tree over the tile's 1024 slots");
    int32_t anc[kK3sPPL][kLevels];
    if (tree_used) {
#pragma unroll
        for (int u = 0; u < kK3sPPL; ++u)
#pragma unroll
            for (int l = 0; l < kLevels; ++l) anc[u][l] = tree[(u * kK3sThreads + threadIdx.x + kK3sPods) >> l];
    }
#pragma unroll
    for (int u = 0; u < kK3sPPL; ++u) {
        int32_t best = umax[ds[u] ? 1 : 0];
        if (tree_used) {
#pragma unroll
            for (int l = 0; l < kLevels; ++l) best = max(best, anc[u][l]);
        }
        if (live[u] && best >= 0) {
            const int64_t sc = best >> 24;
            const int64_t n = 0xFFFFFF - (best & 0xFFFFFF);
            atomicMax(&keys[pod[u]],
                      (long long)((sc << 32) | (int64_t)(0xFFFFFFFFull - (uint64_t)(node_offset + n))));
        }
    }
    CRANE_TSTAMP(st.trace, b, 4);
}

// ---------------------------------------------------------------- launchers
int step_breakpoints(int shape) {
    switch (shape) {
        case kShape4x6: return 6 + 2;
        case kShape8x8: return 8 + 2;
        default: return 16 + 2;
    }
}

__global__ __launch_bounds__(kK3sThreads) void k3s_eval(StepTables st, const int32_t* __restrict__ perm,
                                                        const int64_t* __restrict__ pnow,
                                                        const int64_t* __restrict__ tile_mm, int64_t P,
                                                        int64_t node_offset, int32_t R,
                                                        long long* __restrict__ keys) {
#if K3_KWARM
    kernarg_warm<(int)sizeof(StepTables) + 64>();
#endif
    k3s_body((int64_t)blockIdx.x, st, perm, pnow, tile_mm, P, node_offset, R, keys);
}

// The previous step's K3s and this step's first launch (the delta form's K2 + K3p's pod tiles)
// as one launch on an engine's dispatch queue (engine option step_defer, the group's slots): the
// two are independent — K3s reads the previous step's tables and pod tiles, K3p writes this
// step's (the engine alternates two sets), the delta form writes adjustments the previous K1 has
// consumed — and a queue runs its kernels one after the other, so this takes one launch and
// one kernel boundary out of each batch's chain.  Workgroups: K3s's first (its XCD placement
// follows blockIdx), then the pod tiles, then the delta's.
struct K3sArgs {
    StepTables st;
    const int32_t* perm;
    const int64_t* pnow;
    const int64_t* tile_mm;
    int64_t P, node_offset;
    int32_t R;
    long long* keys;
};
static_assert(kK3sThreads == 512, "the fused launch's workgroups are the delta form's and K3p's 512 lanes");

__global__ __launch_bounds__(kK3sThreads) void k3s_delta_pods(K3sArgs k, int32_t nk3s, const int32_t* __restrict__ bnode,
                                                              int64_t N, HotDelta d, uint32_t* __restrict__ adj,
                                                              PodPrep pp) {
#if K3_KWARM
    kernarg_warm<(int)(sizeof(K3sArgs) + 32 + sizeof(HotDelta) + 8 + sizeof(PodPrep))>();
#endif
    const int64_t b = blockIdx.x;
    if (b < nk3s) {
        k3s_body(b, k.st, k.perm, k.pnow, k.tile_mm, k.P, k.node_offset, k.R, k.keys);
        return;
    }
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn_lds[];
    if (b - nk3s < pp.ntiles) k3p_tile<kK3sThreads>(b - nk3s, pp, dyn_lds);
    else k2_delta_body<kK3sThreads>((int32_t)(b - nk3s - pp.ntiles), bnode, N, d, adj);
}

StepGeometry step_geometry(int64_t P, int64_t N, int32_t nblk, int32_t blk_per_wg) {
    StepGeometry g{};
    g.nseg = (N + kStepSeg - 1) / kStepSeg;
    g.npad = g.nseg * kStepSeg;  // >= nblk * bs for bs = 128 or 256
    g.ntiles = (P + kPodTile - 1) / kPodTile;
    g.ngroups = (P + kK3sPods - 1) / kK3sPods;
    // R workgroups per 1024-pod tile: about kK3sBlkPerWg producer blocks each while the
    // launch stays under kMaxWg workgroups (each slice costs an atomic per pod), and at
    // most kK3sMaxBlk blocks each (at least one lane per block)
    constexpr int64_t kMaxWg = 2048;
    const int32_t bpw = blk_per_wg > 0 ? blk_per_wg : kK3sBlkPerWg;
    int64_t R = (std::max<int32_t>(nblk, 1) + bpw - 1) / bpw;
    if (blk_per_wg <= 0) R = std::min<int64_t>(R, std::max<int64_t>(1, kMaxWg / std::max<int64_t>(g.ngroups, 1)));
    R = std::max<int64_t>(R, (nblk + kK3sMaxBlk - 1) / kK3sMaxBlk);
    if (nblk >= 8) {  // XCD groups (k3s_eval): a multiple of 8 (down while over kMaxWg workgroups),
                      // each group's slices <= kK3sMaxBlk blocks
        R = (R + 7) / 8 * 8;
        if (blk_per_wg <= 0 && R * g.ngroups > kMaxWg) R -= 8;
        R = std::max<int64_t>(8, R);
        while (((nblk + 7) / 8 + R / 8 - 1) / (R / 8) > kK3sMaxBlk) R += 8;
    }
    g.R = (int32_t)R;
    return g;
}

template <int PD, int PR>
static hipError_t launch_steps_t(const void* rec, int64_t N, double wsum, int32_t noprio, const StepTables& st,
                                 const StepGeometry& g, const int64_t* tile_mm, hipStream_t s) {
    return klaunch("k3a_steps", k3a_steps<PD, PR>, dim3((unsigned)g.nseg), dim3(kStepSeg), 0, s,
                   static_cast<const NodeRec<PD, PR>*>(rec), N, tile_mm, (int32_t)g.ntiles, wsum, noprio, st);
}

hipError_t launch_step_pods(const int64_t* now, const uint8_t* flags, int64_t P, long long* keys, int64_t* batch,
                            int64_t* batch_next, const StepGeometry& g, int32_t* perm, int64_t* pnow,
                            int64_t* tile_mm, hipStream_t s) {
    if (P <= 0) return hipSuccess;
    const PodPrep pp{now, flags, P, g.ntiles, perm, pnow, tile_mm, keys, batch, batch_next};
    return klaunch("k3p_pods", k3p_pods, dim3((unsigned)g.ntiles), dim3(kPodTile), kK3pLds, s, pp);
}

hipError_t launch_step_nodes(int shape, const void* rec, int64_t N, double wsum, int32_t noprio,
                             const StepTables& st, const StepGeometry& g, const int64_t* tile_mm, hipStream_t s) {
    if (N <= 0 || g.ntiles <= 0) return hipSuccess;
    if (N >= kStepMaxNodes) return hipErrorInvalidValue;
    switch (shape) {
        case kShape4x6: return launch_steps_t<4, 6>(rec, N, wsum, noprio, st, g, tile_mm, s);
        case kShape8x8: return launch_steps_t<8, 8>(rec, N, wsum, noprio, st, g, tile_mm, s);
        default: return launch_steps_t<16, 16>(rec, N, wsum, noprio, st, g, tile_mm, s);
    }
}

hipError_t launch_k3s_delta_pods(int64_t N_k3s, int64_t node_offset, int64_t P_k3s, long long* keys_k3s,
                                 const StepTables& st, const StepGeometry& g, const int32_t* perm, const int64_t* pnow,
                                 const int64_t* tile_mm, const int32_t* bnode, int64_t N, const HotDelta& d,
                                 uint32_t* adj, const PodPrep& pods, hipStream_t s) {
    if (P_k3s <= 0 || N_k3s <= 0 || d.n_win < 1 || d.n_win > kDeltaMaxWin || d.n_rng < 0 || d.n_rng > kMaxWin ||
        N >= (1LL << 27))
        return hipErrorInvalidValue;
    const int64_t nk = g.ngroups * g.R;
    const int64_t L = d.n_rng > 0 ? d.start[d.n_rng] : 0;
    const int64_t grid = nk + (pods.P > 0 ? pods.ntiles : 0) + (L + kDeltaChunk - 1) / kDeltaChunk;
    if (grid >= (1LL << 31) || nk >= (1LL << 31)) return hipErrorInvalidValue;
    PodPrep pp{};
    if (pods.P > 0) pp = pods;
    const size_t lds = std::max(kK3pLds, sizeof(uint32_t) * 2 * (size_t)kDeltaSlots +
                                             sizeof(uint16_t) * kDeltaMaxWin * kDeltaChunk);
    static const hipError_t attr = hipFuncSetAttribute((const void*)k3s_delta_pods,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (attr != hipSuccess) return attr;
    const K3sArgs k{st, perm, pnow, tile_mm, P_k3s, node_offset, g.R, keys_k3s};
    return klaunch("k3s_eval+k2_delta+k3p_pods", k3s_delta_pods, dim3((unsigned)grid), dim3(kK3sThreads), lds, s, k,
                   (int32_t)nk, bnode, N, d, adj, pp);
}

hipError_t launch_step_pairs(int shape, int64_t N, int64_t node_offset, int64_t P, long long* keys,
                             const StepTables& st, const StepGeometry& g, const int32_t* perm, const int64_t* pnow,
                             const int64_t* tile_mm, hipStream_t s) {
    (void)shape;
    if (P <= 0 || N <= 0) return hipSuccess;
    const dim3 grid((unsigned)(g.ngroups * g.R)), blk(kK3sThreads);
    return klaunch("k3s_eval", k3s_eval, grid, blk, 0, s, st, perm, pnow, tile_mm, P, node_offset, g.R, keys);
}

}  // namespace crane
