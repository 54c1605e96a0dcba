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
//   K3p  pods  : DaemonSet partition per 1024-pod tile (so waves are uniform),
//                key init, per-tile min/max of now, step-table header reset
//   K3a  nodes : per node, both pod kinds (Filter applies / DaemonSet bypass,
//                utils.go:17-24): flat key -> workgroup max; stepped node ->
//                its key pieces (one-step records sorted per workgroup with
//                prefix / suffix key maxima, middle pieces), step_node.hpp
//   K3s  pairs : a 1024-pod tile per workgroup (4 pods per lane), R workgroups
//                per tile split the producer blocks (one lane per block):
//                binary searches find the records stepping inside the tile's
//                time range, one prefix and one suffix maximum give the key of
//                all others; one 64-bit atomicMax per pod per workgroup
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dyn_types.hpp"
#include "kernels.hpp"
#include "step_node.hpp"

namespace crane {

// ---------------------------------------------------------------- K3p
constexpr int kPodTile = 1024;

__global__ __launch_bounds__(kPodTile) void k3p_pods(const int64_t* __restrict__ now,
                                                     const uint8_t* __restrict__ flags, int64_t P,
                                                     int32_t* __restrict__ perm, int64_t* __restrict__ pnow,
                                                     int64_t* __restrict__ tile_mm, long long* __restrict__ keys) {
    __shared__ int32_t cn[kPodTile / 64], cd[kPodTile / 64];
    __shared__ int64_t wmn[kPodTile / 64], wmx[kPodTile / 64];
    const int64_t t = blockIdx.x;
    const int64_t p = t * kPodTile + threadIdx.x;
    const bool live = p < P;
    const bool ds = live && flags && (flags[p] & 1u);
    const int64_t tn = live ? now[p] : 0;
    if (live) keys[p] = -1;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t mn_mask = __ballot(live && !ds), md_mask = __ballot(ds);
    const uint64_t lt = (1ull << lane) - 1ull;
    int64_t mn = live ? tn : INT64_MAX, mx = live ? tn : INT64_MIN;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        mn = min(mn, (int64_t)__shfl_xor((long long)mn, o));
        mx = max(mx, (int64_t)__shfl_xor((long long)mx, o));
    }
    if (lane == 0) {
        cn[w] = __popcll(mn_mask);
        cd[w] = __popcll(md_mask);
        wmn[w] = mn;
        wmx[w] = mx;
    }
    __syncthreads();
    int32_t pre_n = 0, pre_d = 0, tot_n = 0;
    for (int i = 0; i < kPodTile / 64; ++i) {
        if (i < w) {
            pre_n += cn[i];
            pre_d += cd[i];
        }
        tot_n += cn[i];
    }
    if (live) {
        const int32_t pos = ds ? tot_n + pre_d + __popcll(md_mask & lt) : pre_n + __popcll(mn_mask & lt);
        perm[t * kPodTile + pos] = (int32_t)p | (ds ? (int32_t)0x80000000 : 0);  // bit 31: DaemonSet
        pnow[t * kPodTile + pos] = tn;
    }
    if (threadIdx.x == 0) {
        int64_t a = INT64_MAX, b = INT64_MIN;
        for (int i = 0; i < kPodTile / 64; ++i) {
            a = min(a, wmn[i]);
            b = max(b, wmx[i]);
        }
        tile_mm[2 * t] = a;
        tile_mm[2 * t + 1] = b;
    }
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
    if (n < N && (o.slot0 >= 0 || o.slot1 >= 0)) step_emit<PD, PR>(r, n, tmin, tmax, wsum, noprio, o, st, blockIdx.x, s1l);
    __syncthreads();
    step_sort_publish<kStepSeg>(s1l, s1s, sh, st, blockIdx.x);
}

// ---------------------------------------------------------------- K3s
// Workgroup = 4 waves x 64 lanes x 4 pods per lane (one 1024-pod tile of K3p's
// partitioned order: lane l of wave w holds pods u * 256 + w * 64 + l); the R
// workgroups of a tile split the producer blocks, one lane per block.
// One-step records: each block's are sorted by step time bp with prefix maxima
// of the after-step key (pm1) and suffix maxima of the before-step key (sm0)
// (step_sort_publish).  For the tile's pod time range [lo, hi] (per pod kind)
// a lane finds by two binary searches the block's records stepping inside
// (lo, hi]; every pod of the tile sees the key after the step of each earlier
// record (one prefix maximum) and the key before the step of each later one
// (one suffix maximum).  The records inside are staged in LDS and every lane
// evaluates them for its 4 pods (64-bit compare, select, max).  Middle pieces
// [s, e) of multi-step nodes: one covering the whole range gives its key to
// every pod of the tile, one overlapping it partly is staged and evaluated per
// pod (s <= now < e).  One 64-bit atomicMax per pod per workgroup merges the
// slices.
constexpr int kK3sWaves = 4;
constexpr int kK3sThreads = kK3sWaves * 64;
constexpr int kK3sPPL = 4;                          // pods per lane
constexpr int kK3sPods = kK3sThreads * kK3sPPL;     // pods per workgroup (= kPodTile)
constexpr int kK3sS1 = 512;  // one-step records staged per round and pod kind (8 KB)
constexpr int kK3sMP = 128;  // middle pieces staged per round and pod kind
static_assert(kK3sMaxBlk <= kK3sThreads, "one lane per producer block");

// number of the n sorted step times at base[] that are <= t (upper bound)
__device__ __forceinline__ int32_t count_le(const Step1* __restrict__ base, int32_t n, int64_t t) {
    int32_t lo = 0, hi = n;
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (base[mid].bp <= t) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kK3sThreads) void k3s_eval(StepTables st, const int32_t* __restrict__ perm,
                                                        const int64_t* __restrict__ pnow, int64_t P,
                                                        int64_t node_offset, int32_t R,
                                                        long long* __restrict__ keys) {
    static_assert(kK3sWaves == 4, "per-wave partials below");
    __shared__ int4 l1[2][kK3sS1];
    __shared__ Mid lm[2][kK3sMP];
    __shared__ int32_t spart[2][kK3sWaves], mpart[2][kK3sWaves];  // straddling records / pieces per wave
    __shared__ int64_t wr[2][2][kK3sWaves];      // per kind and wave: min, max pod time
    __shared__ int32_t umax[2];
    const int64_t b = blockIdx.x;
    CRANE_TSTAMP(st.trace, b, 0);
    const int32_t r = (int32_t)(b % R);
    const int64_t grp = b / R;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // K3p wrote the pods in partitioned order: coalesced loads
    bool live[kK3sPPL], ds[kK3sPPL];
    int32_t pod[kK3sPPL];
    int64_t tnow[kK3sPPL];
#pragma unroll
    for (int u = 0; u < kK3sPPL; ++u) {
        const int64_t slot = grp * kK3sPods + u * kK3sThreads + threadIdx.x;
        live[u] = slot < P;
        const int32_t praw = live[u] ? perm[slot] : 0;
        tnow[u] = live[u] ? pnow[slot] : 0;
        ds[u] = praw < 0;
        pod[u] = praw & 0x7FFFFFFF;
    }
    // producer blocks [b0, b0 + m) of this slice; thread j < m owns block b0 + j
    const int32_t per = (st.nblk + R - 1) / R;
    const int32_t b0 = min(st.nblk, r * per), m = min(st.nblk, b0 + per) - b0;
    const bool own = (int32_t)threadIdx.x < m;
    const int64_t ob = b0 + threadIdx.x;
    int32_t cnt1[2] = {0, 0}, cntm[2] = {0, 0}, flat[2] = {-1, -1};
    if (own) {
        const int4 c = reinterpret_cast<const int4*>(st.cnt)[ob];  // [records kind 0, pieces 0, records 1, pieces 1]
        cnt1[0] = c.x;
        cntm[0] = c.y;
        cnt1[1] = c.z;
        cntm[1] = c.w;
        flat[0] = st.flat[ob * 2];
        flat[1] = st.flat[ob * 2 + 1];
    }
    bool ln = false, ld = false;  // this lane has pods of kind 0 / 1
#pragma unroll
    for (int u = 0; u < kK3sPPL; ++u) {
        ln |= live[u] && !ds[u];
        ld |= ds[u];
    }
    const bool wn = __ballot(ln) != 0, wd = __ballot(ld) != 0;
    // the workgroup's pod time range per kind
#pragma unroll
    for (int T = 0; T < 2; ++T) {
        int64_t mn = INT64_MAX, mx = INT64_MIN;
#pragma unroll
        for (int u = 0; u < kK3sPPL; ++u) {
            const bool mine = live[u] && (T ? ds[u] : !ds[u]);
            mn = mine ? min(mn, tnow[u]) : mn;
            mx = mine ? max(mx, tnow[u]) : mx;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            mn = min(mn, (int64_t)__shfl_xor((long long)mn, o));
            mx = max(mx, (int64_t)__shfl_xor((long long)mx, o));
        }
        if (lane == 0) {
            wr[T][0][w] = mn;
            wr[T][1][w] = mx;
        }
    }
    if (threadIdx.x < 2) umax[threadIdx.x] = -1;
    const bool bn = __syncthreads_or(ln), bd = __syncthreads_or(ld);  // (also orders the LDS above)
    int64_t tlo[2], thi[2];
#pragma unroll
    for (int T = 0; T < 2; ++T) {
        tlo[T] = min(min(wr[T][0][0], wr[T][0][1]), min(wr[T][0][2], wr[T][0][3]));
        thi[T] = max(max(wr[T][1][0], wr[T][1][1]), max(wr[T][1][2], wr[T][1][3]));
    }
    // one-step records of the owned block: the ones stepping inside (lo, hi], and the
    // uniform key of all others; a kind without pods here takes nothing
    int32_t s_lo[2], s_n[2];
    // this thread's share of the uniform maxima (a kind without pods here is never read)
    int32_t um0 = flat[0], um1 = flat[1];
    {
        int32_t jl[2], jh[2];
#pragma unroll
        for (int T = 0; T < 2; ++T) {  // the four searches are independent chains
            const bool any = T ? bd : bn;
            const Step1* base = st.single + s1_at(st, T, ob);
            const int32_t n = own && any ? cnt1[T] : 0;
            jl[T] = count_le(base, n, tlo[T]);
            jh[T] = count_le(base, n, thi[T]);
        }
#pragma unroll
        for (int T = 0; T < 2; ++T) {
            const int64_t base = s1_at(st, T, ob);
            const bool any = own && (T ? bd : bn);
            int32_t u = -1;
            if (any && jl[T] > 0) u = st.pm1[base + jl[T] - 1];
            if (any && jh[T] < cnt1[T]) u = max(u, st.sm0[base + jh[T]]);
            if (T) um1 = max(um1, u);
            else um0 = max(um0, u);
            if (!any) flat[T] = -1;
            s_lo[T] = jl[T];
            s_n[T] = any ? jh[T] - jl[T] : 0;
        }
    }
    // middle pieces of the owned block: covering [lo, hi] -> uniform key, overlapping
    // it partly -> counted here, staged below
    int32_t m_n[2] = {0, 0};
#pragma unroll
    for (int T = 0; T < 2; ++T) {
        const bool any = own && (T ? bd : bn);
        const Mid* mp = st.mid + (int64_t)T * st.mpad + ob * st.mstride;
        const int32_t n = any ? cntm[T] : 0;
        int32_t u = -1;
        for (int32_t i = 0; i < n; ++i) {
            const Mid p = mp[i];
            if (p.s <= tlo[T] && p.e > thi[T]) u = max(u, p.key);
            else m_n[T] += p.s <= thi[T] && p.e > tlo[T];
        }
        if (T) um1 = max(um1, u);
        else um0 = max(um0, u);
    }
    CRANE_TSTAMP(st.trace, b, 1);
    // exclusive prefix of the straddling counts over the owned blocks (per kind)
    int32_t s_off[2], s_tot[2], m_off[2], m_tot[2];
#pragma unroll
    for (int T = 0; T < 2; ++T) {
        int32_t x = s_n[T], y = m_n[T];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t xs = __shfl_up(x, o), ys = __shfl_up(y, o);
            if (lane >= o) {
                x += xs;
                y += ys;
            }
        }
        if (lane == 63) {
            spart[T][w] = x;
            mpart[T][w] = y;
        }
        s_off[T] = x - s_n[T];
        m_off[T] = y - m_n[T];
    }
    __syncthreads();
#pragma unroll
    for (int T = 0; T < 2; ++T) {
        int32_t pre = 0, tot = 0, mpre = 0, mtot = 0;
#pragma unroll
        for (int i = 0; i < kK3sWaves; ++i) {
            pre += i < w ? spart[T][i] : 0;
            tot += spart[T][i];
            mpre += i < w ? mpart[T][i] : 0;
            mtot += mpart[T][i];
        }
        s_off[T] += pre;
        s_tot[T] = tot;
        m_off[T] += mpre;
        m_tot[T] = mtot;
    }
    int32_t best_n[kK3sPPL], best_d[kK3sPPL];
#pragma unroll
    for (int u = 0; u < kK3sPPL; ++u) best_n[u] = best_d[u] = -1;
    auto walk1 = [&](int T, int32_t n1, int32_t* best) {
        int32_t i = 0;
        for (; i + 4 <= n1; i += 4) {
            int4 q[4];
#pragma unroll
            for (int v = 0; v < 4; ++v) q[v] = l1[T][i + v];  // broadcast LDS reads
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int64_t bp = (int64_t)(((uint64_t)(uint32_t)q[v].y << 32) | (uint32_t)q[v].x);
#pragma unroll
                for (int u = 0; u < kK3sPPL; ++u) best[u] = max(best[u], tnow[u] >= bp ? q[v].w : q[v].z);
            }
        }
        for (; i < n1; ++i) {
            const int4 q = l1[T][i];
            const int64_t bp = (int64_t)(((uint64_t)(uint32_t)q.y << 32) | (uint32_t)q.x);
#pragma unroll
            for (int u = 0; u < kK3sPPL; ++u) best[u] = max(best[u], tnow[u] >= bp ? q.w : q.z);
        }
    };
    // one-step records stepping inside the tile's range: rounds of kK3sS1 per kind
    for (int32_t r0 = 0; r0 < max(s_tot[0], s_tot[1]); r0 += kK3sS1) {
#pragma unroll
        for (int T = 0; T < 2; ++T) {  // the owning lane copies its records of window [r0, r0 + kK3sS1)
            const int32_t a = max(s_off[T], r0), e = min(s_off[T] + s_n[T], r0 + kK3sS1);
            const int4* src = reinterpret_cast<const int4*>(st.single + s1_at(st, T, ob)) + s_lo[T];
            for (int32_t g = a; g < e; ++g) l1[T][g - r0] = src[g - s_off[T]];
        }
        __syncthreads();
        if (wn) walk1(0, min(kK3sS1, max(0, s_tot[0] - r0)), best_n);
        if (wd) walk1(1, min(kK3sS1, max(0, s_tot[1] - r0)), best_d);
        __syncthreads();
    }
    // middle pieces overlapping the tile's range partly: rounds of kK3sMP per kind; the
    // owning lane re-reads its block's pieces and stages those of the window
    auto walkm = [&](int T, int32_t n, int32_t* best) {
        for (int32_t j = 0; j < n; ++j) {
            const Mid p = lm[T][j];
#pragma unroll
            for (int u = 0; u < kK3sPPL; ++u) best[u] = max(best[u], tnow[u] >= p.s && tnow[u] < p.e ? p.key : -1);
        }
    };
    for (int32_t r0 = 0; r0 < max(m_tot[0], m_tot[1]); r0 += kK3sMP) {
#pragma unroll
        for (int T = 0; T < 2; ++T) {
            if (m_n[T] == 0 || m_off[T] + m_n[T] <= r0 || m_off[T] >= r0 + kK3sMP) continue;
            const Mid* mp = st.mid + (int64_t)T * st.mpad + ob * st.mstride;
            int32_t g = m_off[T];
            for (int32_t i = 0; i < cntm[T]; ++i) {
                const Mid p = mp[i];
                if ((p.s <= tlo[T] && p.e > thi[T]) || !(p.s <= thi[T] && p.e > tlo[T])) continue;
                if (g >= r0 && g < r0 + kK3sMP) lm[T][g - r0] = p;
                ++g;
            }
        }
        __syncthreads();
        if (wn) walkm(0, min(kK3sMP, max(0, m_tot[0] - r0)), best_n);
        if (wd) walkm(1, min(kK3sMP, max(0, m_tot[1] - r0)), best_d);
        __syncthreads();
    }
    CRANE_TSTAMP(st.trace, b, 2);
    // uniform maxima (flat keys, prefix / suffix maxima, folded records): wave reduce, one LDS atomic per wave
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        um0 = max(um0, __shfl_xor(um0, o));
        um1 = max(um1, __shfl_xor(um1, o));
    }
    if (lane == 0) {
        if (um0 >= 0) atomicMax(&umax[0], um0);
        if (um1 >= 0) atomicMax(&umax[1], um1);
    }
    __syncthreads();
    CRANE_TSTAMP(st.trace, b, 3);
#pragma unroll
    for (int u = 0; u < kK3sPPL; ++u) {
        const int32_t best = ds[u] ? max(best_d[u], umax[1]) : max(best_n[u], umax[0]);
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

StepGeometry step_geometry(int64_t P, int64_t N, int32_t nblk) {
    StepGeometry g{};
    g.nseg = (N + kStepSeg - 1) / kStepSeg;
    g.npad = g.nseg * kStepSeg;  // >= nblk * bs for bs = 128 or 256
    g.ntiles = (P + kPodTile - 1) / kPodTile;
    g.ngroups = (P + kK3sPods - 1) / kK3sPods;
    // R workgroups per 1024-pod tile: about kTarget workgroups in all, and enough that
    // each covers at most kK3sMaxBlk producer blocks (one lane per block)
    constexpr int64_t kTarget = 256;
    int64_t R = std::max<int64_t>(1, kTarget / std::max<int64_t>(g.ngroups, 1));
    R = std::min<int64_t>(R, std::max<int32_t>(nblk, 1));
    R = std::max<int64_t>(R, (nblk + kK3sMaxBlk - 1) / kK3sMaxBlk);
    g.R = (int32_t)R;
    return g;
}

template <int PD, int PR>
static hipError_t launch_steps_t(const void* rec, int64_t N, double wsum, int32_t noprio, const StepTables& st,
                                 const StepGeometry& g, const int64_t* tile_mm, hipStream_t s) {
    return klaunch("k3a_steps", k3a_steps<PD, PR>, dim3((unsigned)g.nseg), dim3(kStepSeg), 0, s,
                   static_cast<const NodeRec<PD, PR>*>(rec), N, tile_mm, (int32_t)g.ntiles, wsum, noprio, st);
}

hipError_t launch_step_pods(const int64_t* now, const uint8_t* flags, int64_t P, long long* keys,
                            const StepGeometry& g, int32_t* perm, int64_t* pnow, int64_t* tile_mm, hipStream_t s) {
    if (P <= 0) return hipSuccess;
    return klaunch("k3p_pods", k3p_pods, dim3((unsigned)g.ntiles), dim3(kPodTile), 0, s, now, flags, P, perm, pnow,
                   tile_mm, keys);
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

hipError_t launch_step_pairs(int shape, int64_t N, int64_t node_offset, int64_t P, long long* keys,
                             const StepTables& st, const StepGeometry& g, const int32_t* perm, const int64_t* pnow,
                             hipStream_t s) {
    (void)shape;
    if (P <= 0 || N <= 0) return hipSuccess;
    const dim3 grid((unsigned)(g.ngroups * g.R)), blk(kK3sThreads);
    return klaunch("k3s_eval", k3s_eval, grid, blk, 0, s, st, perm, pnow, P, node_offset, g.R, keys);
}

}  // namespace crane
