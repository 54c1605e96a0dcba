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
#include <cstdlib>

#include "dyn_types.hpp"
#include "kernels.hpp"
#include "step_node.hpp"

namespace crane {

// ---------------------------------------------------------------- K3p
constexpr int kPodTile = 1024;

__global__ __launch_bounds__(kPodTile) void k3p_pods(const int64_t* __restrict__ now,
                                                     const uint8_t* __restrict__ flags, int64_t P,
                                                     int32_t* __restrict__ perm, int64_t* __restrict__ pnow,
                                                     int64_t* __restrict__ tile_mm, long long* __restrict__ keys,
                                                     int32_t* __restrict__ hdr) {
    __shared__ int32_t cn[kPodTile / 64], cd[kPodTile / 64];
    __shared__ int64_t wmn[kPodTile / 64], wmx[kPodTile / 64];
    const int64_t t = blockIdx.x;
    const int64_t p = t * kPodTile + threadIdx.x;
    const bool live = p < P;
    const bool ds = live && flags && (flags[p] & 1u);
    const int64_t tn = live ? now[p] : 0;
    if (live) keys[p] = -1;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (t == 0 && threadIdx.x < kHdrLen)  // step-table header: flat maxima -1, counts 0
        hdr[threadIdx.x] = (threadIdx.x % kHdrStride) < kHdrN1 ? -1 : 0;
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
    step_reserve<kStepSeg>(o, sh, st);
    if (n < N && (o.slot0 >= 0 || o.slot1 >= 0)) step_emit<PD, PR>(r, n, tmin, tmax, wsum, noprio, sh, o, st);
}

// ---------------------------------------------------------------- K3s
// Workgroup = 4 waves x 64 pods (256 consecutive pods of K3p's partitioned
// order); the R workgroups of a pod group split each stepped list.  A
// workgroup stages its slice of the list in LDS with coalesced loads (one
// memory latency for the slice), then every wave walks the slice with
// broadcast LDS reads: per (pod, one-step node) a 64-bit compare, a select and
// a max.  One 64-bit atomicMax per pod per workgroup merges the slices.
constexpr int kK3sWaves = 4;
constexpr int kK3sThreads = kK3sWaves * 64;
constexpr int kK3sS1 = 1024;  // Step1 records staged per round (16 KB)
constexpr int kK3sVR = 64;    // VRec records staged per round

// [lo, hi) of part u of U equal parts of n
__device__ __forceinline__ void part_range(int32_t n, int32_t u, int32_t U, int32_t& lo, int32_t& hi) {
    const int32_t per = (n + U - 1) / U;
    lo = min(n, u * per);
    hi = min(n, lo + per);
}

// Exclusive prefix of the kStepSub sub-list lengths of (kind T, list k) into
// pre[0..kStepSub] (LDS); returns the total.  All threads call it.
__device__ __forceinline__ int32_t sub_prefix(const int32_t* __restrict__ hdr, int T, int k, int32_t* pre) {
    static_assert(kStepSub == 64, "one wave scans the sub-lists");
    __syncthreads();  // earlier readers of pre are done
    if (threadIdx.x < 64) {
        const int32_t c = hdr[threadIdx.x * kHdrStride + kHdrN1 + 2 * T + k];
        int32_t x = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t y = __shfl_up(x, o);
            if ((int)threadIdx.x >= o) x += y;
        }
        pre[threadIdx.x] = x - c;
        if (threadIdx.x == 63) pre[64] = x;
    }
    __syncthreads();
    return pre[64];
}

// global position in the [kStepSub][cap] layout of element i of the concatenated sub-lists
__device__ __forceinline__ int64_t sub_pos(const int32_t* pre, int32_t i, int64_t cap) {
    int lo = 0;
#pragma unroll
    for (int h = 32; h >= 1; h >>= 1)
        if (pre[lo + h] <= i) lo += h;
    return (int64_t)lo * cap + (i - pre[lo]);
}

template <int NB>
__device__ __forceinline__ int32_t k3s_kind(int T, bool any, int64_t tnow, int32_t best, const StepTables& st,
                                            int32_t r, int32_t R, int4* l1, VRec<NB>* lv, int32_t* pre) {
    const int4* __restrict__ g1 = reinterpret_cast<const int4*>(st.single + (int64_t)T * st.npad);
    const VRec<NB>* __restrict__ gv = reinterpret_cast<const VRec<NB>*>(st.multi) + (int64_t)T * st.npad;
    int32_t a0, a1;
    part_range(sub_prefix(st.hdr, T, 0, pre), r, R, a0, a1);
    // one-step records, kK3sS1 per round
    for (int32_t j0 = a0; j0 < a1; j0 += kK3sS1) {
        const int32_t n1 = min(kK3sS1, a1 - j0);
        __syncthreads();  // the previous round's readers are done
        for (int32_t i = threadIdx.x; i < n1; i += 4 * kK3sThreads) {  // 4 loads in flight per thread
            int4 q[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + u * kK3sThreads < n1) q[u] = g1[sub_pos(pre, j0 + i + u * kK3sThreads, st.cap)];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + u * kK3sThreads < n1) l1[i + u * kK3sThreads] = q[u];
        }
        __syncthreads();
        if (any) {
            int32_t i = 0;
            for (; i + 8 <= n1; i += 8) {
                int4 q[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) q[u] = l1[i + u];  // broadcast LDS reads
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int64_t bp = (int64_t)(((uint64_t)(uint32_t)q[u].y << 32) | (uint32_t)q[u].x);
                    best = max(best, tnow >= bp ? q[u].w : q[u].z);
                }
            }
            for (; i < n1; ++i) {
                const int4 q = l1[i];
                const int64_t bp = (int64_t)(((uint64_t)(uint32_t)q.y << 32) | (uint32_t)q.x);
                best = max(best, tnow >= bp ? q.w : q.z);
            }
        }
    }
    // multi-step records, kK3sVR per round (copied as int4 words)
    static_assert(sizeof(VRec<NB>) % 16 == 0, "VRec must be a whole number of int4");
    constexpr int kVRI4 = (int)(sizeof(VRec<NB>) / 16);
    int32_t m0, m1;
    part_range(sub_prefix(st.hdr, T, 1, pre), r, R, m0, m1);
    for (int32_t j0 = m0; j0 < m1; j0 += kK3sVR) {
        const int32_t nv = min(kK3sVR, m1 - j0);
        __syncthreads();
        int4* dst = reinterpret_cast<int4*>(lv);
        for (int32_t i = threadIdx.x; i < nv * kVRI4; i += kK3sThreads) {
            const int32_t e = i / kVRI4, w = i - e * kVRI4;
            dst[i] = reinterpret_cast<const int4*>(gv + sub_pos(pre, j0 + e, st.cap))[w];
        }
        __syncthreads();
        if (any)
            for (int32_t j = 0; j < nv; ++j) {
                const VRec<NB>& v = lv[j];
                int32_t k = v.key[0];
#pragma unroll
                for (int s = 0; s < NB; ++s) k = tnow >= v.bp[s] ? v.key[s + 1] : k;
                best = max(best, k);
            }
    }
    return best;
}

template <int NB>
__global__ __launch_bounds__(kK3sThreads) void k3s_eval(StepTables st, const int32_t* __restrict__ perm,
                                                        const int64_t* __restrict__ pnow, int64_t P,
                                                        int64_t node_offset, int32_t R,
                                                        long long* __restrict__ keys) {
    __shared__ int4 l1[kK3sS1];
    __shared__ VRec<NB> lv[kK3sVR];
    __shared__ int32_t pre[kStepSub + 1];
    const int64_t b = blockIdx.x;
    const int32_t r = (int32_t)(b % R);
    const int64_t grp = b / R;
    // K3p wrote the pods in partitioned order: two independent coalesced loads
    const int64_t slot = grp * kK3sThreads + threadIdx.x;
    const bool live = slot < P;
    const int32_t praw = live ? perm[slot] : 0;
    const int64_t tnow = live ? pnow[slot] : 0;
    const bool ds = praw < 0;
    const int32_t pod = praw & 0x7FFFFFFF;
    // wave-uniform "this wave has pods of the kind"; workgroup-uniform "stage the kind"
    const bool wn = __ballot(live && !ds) != 0, wd = __ballot(ds) != 0;
    const bool bn = __syncthreads_or(live && !ds), bd = __syncthreads_or(ds);
    int32_t best_n = -1, best_d = -1;
    if (r == 0) {  // the flat maxima (max over the sub-lists) enter once per pod
        int32_t fn = -1, fd = -1;
        if ((threadIdx.x & 63) < kStepSub) {
            fn = st.hdr[(threadIdx.x & 63) * kHdrStride + kHdrFlat + 0];
            fd = st.hdr[(threadIdx.x & 63) * kHdrStride + kHdrFlat + 1];
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            fn = max(fn, __shfl_xor(fn, o));
            fd = max(fd, __shfl_xor(fd, o));
        }
        best_n = fn;
        best_d = fd;
    }
    if (bn) best_n = k3s_kind<NB>(0, wn, tnow, best_n, st, r, R, l1, lv, pre);
    if (bd) best_d = k3s_kind<NB>(1, wd, tnow, best_d, st, r, R, l1, lv, pre);
    const int32_t best = ds ? best_d : best_n;
    if (live && best >= 0) {
        const int64_t sc = best >> 24;
        const int64_t n = 0xFFFFFF - (best & 0xFFFFFF);
        atomicMax(&keys[pod], (long long)((sc << 32) | (int64_t)(0xFFFFFFFFull - (uint64_t)(node_offset + n))));
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

StepGeometry step_geometry(int64_t P, int64_t N) {
    StepGeometry g{};
    g.nseg = (N + kStepSeg - 1) / kStepSeg;
    g.npad = g.nseg * kStepSeg;
    // sub-list capacity: workgroups b = s, s + kStepSub, ... of K3a (256 nodes) or K1 (128)
    g.cap = (N + kStepSub * 256 - 1) / (kStepSub * 256) * 256;
    g.npad = g.cap * kStepSub;
    g.ntiles = (P + kPodTile - 1) / kPodTile;
    g.ngroups = (P + kK3sThreads - 1) / kK3sThreads;
    // R workgroups per 256-pod group: ~512 workgroups in all, at most 64 per group
    const char* e = getenv("CRANE_K3S_BLOCKS");
    const int64_t target = e && atoi(e) > 0 ? atoi(e) : 512;
    g.R = (int32_t)std::min<int64_t>(64, std::max<int64_t>(1, target / std::max<int64_t>(g.ngroups, 1)));
    return g;
}

template <int PD, int PR>
static hipError_t launch_steps_t(const void* rec, int64_t N, double wsum, int32_t noprio, const StepTables& st,
                                 const StepGeometry& g, const int64_t* tile_mm, hipStream_t s) {
    hipLaunchKernelGGL((k3a_steps<PD, PR>), dim3((unsigned)g.nseg), dim3(kStepSeg), 0, s,
                       static_cast<const NodeRec<PD, PR>*>(rec), N, tile_mm, (int32_t)g.ntiles, wsum, noprio, st);
    return hipGetLastError();
}

hipError_t launch_step_pods(const int64_t* now, const uint8_t* flags, int64_t P, long long* keys,
                            const StepTables& st, const StepGeometry& g, int32_t* perm, int64_t* pnow,
                            int64_t* tile_mm, hipStream_t s) {
    if (P <= 0) return hipSuccess;
    hipLaunchKernelGGL(k3p_pods, dim3((unsigned)g.ntiles), dim3(kPodTile), 0, s, now, flags, P, perm, pnow, tile_mm,
                       keys, st.hdr);
    return hipGetLastError();
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
            hipLaunchKernelGGL((k3s_eval<6 + 2>), grid, blk, 0, s, st, perm, pnow, P, node_offset, g.R, keys);
            break;
        case kShape8x8:
            hipLaunchKernelGGL((k3s_eval<8 + 2>), grid, blk, 0, s, st, perm, pnow, P, node_offset, g.R, keys);
            break;
        default:
            hipLaunchKernelGGL((k3s_eval<16 + 2>), grid, blk, 0, s, st, perm, pnow, P, node_offset, g.R, keys);
    }
    return hipGetLastError();
}

}  // namespace crane
