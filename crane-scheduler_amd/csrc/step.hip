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
//                utils.go:17-24): flat key -> workgroup max -> one atomicMax
//                per workgroup; stepped node -> record appended to a compact
//                list (one atomicAdd per workgroup reserves the space)
//   K3s  pairs : 256 pods per workgroup (4 waves, one pod per lane), R
//                workgroups per pod group split the stepped lists; a slice is
//                staged in LDS and read back with broadcast reads; one 64-bit
//                atomicMax per pod per workgroup; lowest node index wins ties
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
    if (n < N && (o.slot0 >= 0 || o.slot1 >= 0)) step_emit<PD, PR>(r, n, tmin, tmax, wsum, noprio, o, st, blockIdx.x);
}

// ---------------------------------------------------------------- K3s
// Workgroup = 4 waves x 64 lanes x 4 pods per lane (one 1024-pod tile of
// K3p's partitioned order: lane l of wave w holds pods u * 256 + w * 64 + l);
// the R workgroups of a tile split the producer blocks.  A workgroup reads its
// blocks' records with coalesced loads: a one-step record whose step lies
// outside the tile's time range gives the same key to all of the tile's pods
// of its kind (one max), the others are staged in LDS and every lane walks
// them with broadcast LDS reads (per pod: 64-bit compare, select, max).  One
// 64-bit atomicMax per pod per workgroup merges the slices.
constexpr int kK3sWaves = 4;
constexpr int kK3sThreads = kK3sWaves * 64;
constexpr int kK3sPPL = 4;                          // pods per lane
constexpr int kK3sPods = kK3sThreads * kK3sPPL;     // pods per workgroup (= kPodTile)
constexpr int kK3sS1 = 512;  // Step1 records staged per round and pod kind (8 KB; 128..1024 measured slower at config 4)
constexpr int kK3sVR = 32;   // VRec records staged per round and pod kind
static_assert(kK3sS1 >= 64 && kK3sS1 % 64 == 0, "the staging rounds must make progress");
static_assert(2 * kK3sS1 * 16 + 2 * kK3sVR * 240 + 4 * 4 * (kK3sMaxBlk + 1) <= 64 * 1024, "K3s LDS budget");

// position in the per-producer-block layout of element i of the concatenation
// of blocks b0 + 0 .. m-1 (pre: exclusive prefix of their counts, pre[m] = total)
__device__ __forceinline__ int64_t blk_pos(const int32_t* pre, int32_t m, int32_t i, int32_t b0, int32_t bs) {
    int lo = 0, hi = m - 1;  // largest j with pre[j] <= i
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= i) lo = mid;
        else hi = mid - 1;
    }
    return (int64_t)(b0 + lo) * bs + (i - pre[lo]);
}

// The four stepped lists: L = 2 * kind + (0: Step1, 1: VRec).
template <int NB>
__global__ __launch_bounds__(kK3sThreads) void k3s_eval(StepTables st, const int32_t* __restrict__ perm,
                                                        const int64_t* __restrict__ pnow, int64_t P,
                                                        int64_t node_offset, int32_t R,
                                                        long long* __restrict__ keys) {
    static_assert(kK3sWaves == 4, "one wave scans each list's counts");
    static_assert(sizeof(VRec<NB>) % 16 == 0, "VRec must be a whole number of int4");
    __shared__ int4 l1[2][kK3sS1];
    __shared__ VRec<NB> lv[2][kK3sVR];
    __shared__ int32_t pre[4][kK3sMaxBlk + 1];
    __shared__ int32_t fl[2][kK3sWaves];
    __shared__ int64_t wr[2][2][kK3sWaves];  // per kind and wave: min, max pod time
    __shared__ int32_t nin[2], nvr[2], umax[2];  // staged one-step / multi-step records, uniform maximum (per kind)
    const int64_t b = blockIdx.x;
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
    // producer blocks [b0, b0 + m) of this slice: their counts, scanned per list
    // (wave w scans list w), and their flat maxima
    const int32_t per = (st.nblk + R - 1) / R;
    const int32_t b0 = min(st.nblk, r * per), m = min(st.nblk, b0 + per) - b0;
    {
        int32_t carry = 0;
        for (int32_t j0 = 0; j0 < m; j0 += 64) {
            const int32_t j = j0 + lane;
            const int32_t c = j < m ? st.cnt[(int64_t)(b0 + j) * 4 + w] : 0;
            int32_t x = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int32_t y = __shfl_up(x, o);
                if (lane >= o) x += y;
            }
            if (j < m) pre[w][j] = carry + x - c;
            carry += __shfl(x, 63);
        }
        if (lane == 0) pre[w][m] = carry;
        int32_t f = -1;
        if (w < 2)
            for (int32_t j = lane; j < m; j += 64) f = max(f, st.flat[(int64_t)(b0 + j) * 2 + w]);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) f = max(f, __shfl_xor(f, o));
        if (lane == 0 && w < 2) fl[w][0] = f;
    }
    bool ln = false, ld = false;  // this lane has pods of kind 0 / 1
#pragma unroll
    for (int u = 0; u < kK3sPPL; ++u) {
        ln |= live[u] && !ds[u];
        ld |= ds[u];
    }
    const bool wn = __ballot(ln) != 0, wd = __ballot(ld) != 0;
    // the workgroup's pod time range per kind: a record whose step lies outside it
    // gives the same key to every pod of that kind here (one max, no per-lane work)
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
    if (threadIdx.x < 2) {
        nin[threadIdx.x] = nvr[threadIdx.x] = 0;
        umax[threadIdx.x] = -1;
    }
    const bool bn = __syncthreads_or(ln), bd = __syncthreads_or(ld);  // (also orders the LDS above)
    int64_t tlo[2], thi[2];
#pragma unroll
    for (int T = 0; T < 2; ++T) {
        tlo[T] = min(min(wr[T][0][0], wr[T][0][1]), min(wr[T][0][2], wr[T][0][3]));
        thi[T] = max(max(wr[T][1][0], wr[T][1][1]), max(wr[T][1][2], wr[T][1][3]));
    }
    // the flat maxima of this slice's producer blocks hold for every pod of the kind
    int32_t best_n[kK3sPPL], best_d[kK3sPPL];
#pragma unroll
    for (int u = 0; u < kK3sPPL; ++u) {
        best_n[u] = fl[0][0];
        best_d[u] = fl[1][0];
    }
    // this workgroup's slice [lo, hi) of each list (lists of a kind without pods here: empty)
    int32_t lo[4], hi[4];
#pragma unroll
    for (int L = 0; L < 4; ++L) {
        lo[L] = 0;
        hi[L] = ((L < 2) ? bn : bd) ? pre[L][m] : 0;
    }
    int32_t um0 = -1, um1 = -1;  // this thread's share of the uniform maxima
    for (bool first = true;; first = false) {
        int32_t take[4];
#pragma unroll
        for (int L = 0; L < 4; ++L) take[L] = min((L & 1) ? kK3sVR : kK3sS1, hi[L] - lo[L]);
        if (take[0] + take[1] + take[2] + take[3] == 0) break;
        if (!first) {
            __syncthreads();  // the previous round's readers are done
            if (threadIdx.x < 2) nin[threadIdx.x] = nvr[threadIdx.x] = 0;
            __syncthreads();
        }
        // one-step records of both kinds [S1 kind 0 | S1 kind 1]: a record whose step
        // lies outside the tile's time range folds into the uniform maxima, the rest
        // are staged in LDS
        const int32_t e2 = take[0], e4 = e2 + take[2];
        for (int32_t i0 = threadIdx.x; i0 < e4; i0 += 4 * kK3sThreads) {
            const int4* src[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {  // addresses first, then 4 loads in flight
                const int32_t e = min(i0 + u * kK3sThreads, e4 - 1);  // past the end: repeat the last element
                const int T = e >= e2;
                const int32_t f = T ? e - e2 : e;
                const int32_t lo1 = T ? lo[2] : lo[0];  // selects, not indexing: keeps lo in registers
                src[u] = reinterpret_cast<const int4*>(st.single + (int64_t)T * st.npad) +
                         blk_pos(pre[2 * T], m, lo1 + f, b0, st.bs);
            }
            int4 q[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) q[u] = *src[u];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int32_t e = i0 + u * kK3sThreads;
                if (e >= e4) continue;
                const int T = e >= e2;
                const int64_t bp = (int64_t)(((uint64_t)(uint32_t)q[u].y << 32) | (uint32_t)q[u].x);
                const int64_t lo_t = T ? tlo[1] : tlo[0], hi_t = T ? thi[1] : thi[0];
                if (bp <= lo_t || bp > hi_t) {  // every pod of the kind here is on one side of the step
                    const int32_t k = bp <= lo_t ? q[u].w : q[u].z;
                    if (T) um1 = max(um1, k);
                    else um0 = max(um0, k);
                } else {
                    l1[T][atomicAdd(&nin[T], 1)] = q[u];
                }
            }
        }
        // multi-step records [VR kind 0 | VR kind 1], one thread per record: one with
        // no step inside the tile's time range folds (its key at the range start),
        // the rest are staged
        const int32_t v2 = take[1], v4 = v2 + take[3];
        for (int32_t e = threadIdx.x; e < v4; e += kK3sThreads) {
            const int T = e >= v2;
            const int32_t f = T ? e - v2 : e;
            const int32_t lov = T ? lo[3] : lo[1];
            const VRec<NB> v = reinterpret_cast<const VRec<NB>*>(st.multi)[(int64_t)T * st.npad +
                                                                       blk_pos(pre[2 * T + 1], m, lov + f, b0, st.bs)];
            const int64_t lo_t = T ? tlo[1] : tlo[0], hi_t = T ? thi[1] : thi[0];
            int32_t k = v.key[0];
            bool inside = false;
#pragma unroll
            for (int s2 = 0; s2 < NB; ++s2) {
                k = lo_t >= v.bp[s2] ? v.key[s2 + 1] : k;
                inside |= v.bp[s2] > lo_t && v.bp[s2] <= hi_t;
            }
            if (!inside) {
                if (T) um1 = max(um1, k);
                else um0 = max(um0, k);
            } else {
                lv[T][atomicAdd(&nvr[T], 1)] = v;
            }
        }
        __syncthreads();
        auto walk = [&](int T, int32_t* best) {
            const int32_t n1 = nin[T];
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
            for (int32_t j = 0; j < nvr[T]; ++j) {
                const VRec<NB>& v = lv[T][j];
#pragma unroll
                for (int u = 0; u < kK3sPPL; ++u) {
                    int32_t k = v.key[0];
#pragma unroll
                    for (int s = 0; s < NB; ++s) k = tnow[u] >= v.bp[s] ? v.key[s + 1] : k;
                    best[u] = max(best[u], k);
                }
            }
        };
        if (wn) walk(0, best_n);
        if (wd) walk(1, best_d);
#pragma unroll
        for (int L = 0; L < 4; ++L) lo[L] += take[L];
    }
    // uniform maxima: wave reduce, one LDS atomic per wave and kind
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
}

// ---------------------------------------------------------------- launchers
size_t step_vrec_bytes(int shape) {
    switch (shape) {
        case kShape4x6: return sizeof(VRec<6 + 2>);
        case kShape8x8: return sizeof(VRec<8 + 2>);
        default: return sizeof(VRec<16 + 2>);
    }
}

StepGeometry step_geometry(int64_t P, int64_t N, int32_t nblk) {
    StepGeometry g{};
    g.nseg = (N + kStepSeg - 1) / kStepSeg;
    g.npad = g.nseg * kStepSeg;  // >= nblk * bs for bs = 128 or 256
    g.ntiles = (P + kPodTile - 1) / kPodTile;
    g.ngroups = (P + kK3sPods - 1) / kK3sPods;
    // R workgroups per 1024-pod group: ~1024 workgroups in all, at most 48 per group
    // (past ~48 the per-workgroup prologue — producer counts, pod loads — outweighs the
    // shorter slices: config 3, 10 groups, R 64 -> 48 = 14.9 -> 13.6 us), and enough
    // that each covers at most kK3sMaxBlk producer blocks
    constexpr int64_t kTarget = 1024, kR = 48;
    int64_t R = std::min<int64_t>(kR, std::max<int64_t>(1, kTarget / std::max<int64_t>(g.ngroups, 1)));
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
    if (P <= 0 || N <= 0) return hipSuccess;
    const dim3 grid((unsigned)(g.ngroups * g.R)), blk(kK3sThreads);
    switch (shape) {
        case kShape4x6:
            return klaunch("k3s_eval", k3s_eval<6 + 2>, grid, blk, 0, s, st, perm, pnow, P, node_offset, g.R, keys);
        case kShape8x8:
            return klaunch("k3s_eval", k3s_eval<8 + 2>, grid, blk, 0, s, st, perm, pnow, P, node_offset, g.R, keys);
        default:
            return klaunch("k3s_eval", k3s_eval<16 + 2>, grid, blk, 0, s, st, perm, pnow, P, node_offset, g.R, keys);
    }
}

}  // namespace crane
