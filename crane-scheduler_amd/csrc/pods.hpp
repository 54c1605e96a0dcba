// pods.hpp — K3p: the step path's pod-batch preparation for one 1024-pod tile,
// with a kT-thread workgroup, so it can run stand-alone (k3p_pods, step.hip,
// kT = 1024) or ride in K2x's launch (hotcount.hip).  Outputs: keys[p] = -1;
// the tile's pods sorted by (kind, now, pod) — non-DaemonSet pods first — as
// perm (pod index, bit 31 = DaemonSet) and pnow (its time); the tile's stats
// row tile_mm[kTileStat * t + i]: i = 0/1 min/max now of kind 0, 2/3 of kind 1
// (INT64_MAX / INT64_MIN for a kind without pods), 4/5 pod counts per kind.
// A tile whose times already ascend in pod order is sorted by a stable kind
// partition; any other by a bitonic sort in LDS.  K3s relies on the sort: the
// pods of one kind that a step record or a middle piece selects in a tile are
// a contiguous slot range.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace crane {

constexpr size_t kK3pLds = 1024 * (sizeof(uint64_t) + sizeof(uint32_t));  // sort keys + tags

// lexicographic (class, time, slot): class and slot live in the tag (class << 30 | slot)
__device__ __forceinline__ bool pod_gt(uint64_t ka, uint32_t va, uint64_t kb, uint32_t vb) {
    return (va >> 30) != (vb >> 30) ? va > vb : (ka != kb ? ka > kb : va > vb);
}

template <int kT>
__device__ __forceinline__ void k3p_tile(const int64_t t, const PodPrep& pp, unsigned char* lds) {
    static_assert(1024 % kT == 0 && kT >= 64, "a tile is 1024 pods");
    constexpr int kU = 1024 / kT, kG = kU * (kT / 64);  // pods per lane, (u, wave) groups
    constexpr uint64_t kSign = 1ull << 63;
    __shared__ int32_t gcn[kG], gcd[kG];
    uint64_t* ku = reinterpret_cast<uint64_t*>(lds);            // now ^ sign: unsigned order = signed order
    uint32_t* kv = reinterpret_cast<uint32_t*>(lds + 8 * 1024);  // class (0 pod, 1 DaemonSet, 2 none) << 30 | slot
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t pend = min(pp.P, (t + 1) * 1024);
    bool live[kU], ds[kU], inorder = true;
    int64_t tn[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const int64_t p = t * 1024 + u * kT + threadIdx.x;  // natural order = (u, wave, lane)
        live[u] = p < pend;
        ds[u] = live[u] && pp.flags && (pp.flags[p] & 1u);
        tn[u] = live[u] ? pp.now[p] : 0;
        if (p + 1 < pend) inorder &= tn[u] <= pp.now[p + 1];
        if (live[u]) pp.keys[p] = -1;
    }
    int32_t e0, e1;  // kind boundaries: first slot of class >= 1 and of class 2 (pod counts per kind)
    if (__syncthreads_and(inorder)) {
        // times already ascending (a queue drained in order): a stable kind partition sorts the tile
        uint64_t mnm[kU], mdm[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            mnm[u] = __ballot(live[u] && !ds[u]);
            mdm[u] = __ballot(ds[u]);
            if (lane == 0) {
                gcn[u * (kT / 64) + w] = __popcll(mnm[u]);
                gcd[u * (kT / 64) + w] = __popcll(mdm[u]);
            }
        }
        __syncthreads();
        int32_t tot_n = 0, tot_d = 0;
#pragma unroll
        for (int i = 0; i < kG; ++i) {
            tot_n += gcn[i];
            tot_d += gcd[i];
        }
        e0 = tot_n;
        e1 = tot_n + tot_d;
        const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int gi = u * (kT / 64) + w, i = u * kT + threadIdx.x;
            int32_t pre_n = 0, pre_d = 0;
            for (int k = 0; k < gi; ++k) {
                pre_n += gcn[k];
                pre_d += gcd[k];
            }
            const int pos = !live[u] ? i
                            : ds[u]  ? tot_n + pre_d + __popcll(mdm[u] & lt)
                                     : pre_n + __popcll(mnm[u] & lt);
            ku[pos] = live[u] ? (uint64_t)tn[u] ^ kSign : ~0ull;
            kv[pos] = ((live[u] ? (ds[u] ? 1u : 0u) : 2u) << 30) | (uint32_t)i;
        }
        __syncthreads();
    } else {
        e0 = e1 = 0;
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int i = u * kT + threadIdx.x;
            ku[i] = live[u] ? (uint64_t)tn[u] ^ kSign : ~0ull;
            kv[i] = ((live[u] ? (ds[u] ? 1u : 0u) : 2u) << 30) | (uint32_t)i;
            e0 += __syncthreads_count(live[u] && !ds[u]);  // (barriers: the stores above are ordered too)
            e1 += __syncthreads_count(ds[u]);
        }
        e1 += e0;
        // bitonic sort of the 1024 (key, tag) pairs in LDS: 55 compare-exchange passes
        for (int k = 2; k <= 1024; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int q = threadIdx.x; q < 512; q += kT) {
                    const int i = ((q & ~(j - 1)) << 1) | (q & (j - 1)), l = i | j;
                    const uint64_t ka = ku[i], kb = ku[l];
                    const uint32_t va = kv[i], vb = kv[l];
                    if (pod_gt(ka, va, kb, vb) == ((i & k) == 0)) {
                        ku[i] = kb;
                        ku[l] = ka;
                        kv[i] = vb;
                        kv[l] = va;
                    }
                }
                __syncthreads();
            }
        }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const int i = u * kT + threadIdx.x;
        const uint32_t v = kv[i];
        if ((v >> 30) < 2u) {
            pp.perm[t * 1024 + i] = (int32_t)(t * 1024 + (v & 1023u)) | ((v >> 30) ? (int32_t)0x80000000 : 0);
            pp.pnow[t * 1024 + i] = (int64_t)(ku[i] ^ kSign);
        }
    }
    if (threadIdx.x == 0) {
        // (e0 / e1 from the counts, not a binary search over the sorted classes: 20 dependent LDS
        // reads on the launch's critical path)
        int64_t* ts = pp.tile_mm + kTileStat * t;
        const int64_t n0 = e0 > 0 ? (int64_t)(ku[0] ^ kSign) : INT64_MAX;
        const int64_t x0 = e0 > 0 ? (int64_t)(ku[e0 - 1] ^ kSign) : INT64_MIN;
        const int64_t n1 = e1 > e0 ? (int64_t)(ku[e0] ^ kSign) : INT64_MAX;
        const int64_t x1 = e1 > e0 ? (int64_t)(ku[e1 - 1] ^ kSign) : INT64_MIN;
        ts[0] = n0;
        ts[1] = x0;
        ts[2] = n1;
        ts[3] = x1;
        ts[4] = e0;
        ts[5] = e1 - e0;
        if (pp.batch) {
            // (round 5 had the last tile to finish fold every tile's stats behind an acquire /
            // release counter: two whole-L2 cache operations on the launch's critical path)
            if (t == 0) {
                pp.batch_next[0] = INT64_MAX;
                pp.batch_next[1] = INT64_MIN;
            }
            const int64_t mn = min(n0, n1), mx = max(x0, x1);
            if (mn != INT64_MAX) __hip_atomic_fetch_min(&pp.batch[0], mn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (mx != INT64_MIN) __hip_atomic_fetch_max(&pp.batch[1], mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace crane
