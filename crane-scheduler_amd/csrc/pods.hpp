// pods.hpp — K3p's pod-batch preparation for one 1024-pod tile, with a
// 256-thread workgroup (4 pods per lane), so it can share a launch with K2x
// (hotcount.hip).  Same outputs as k3p_pods (step.hip): keys[p] = -1; the
// tile's pods partitioned non-DaemonSet first, each kind in ascending pod
// order (perm: pod index, bit 31 = DaemonSet; pnow: its time); tile_mm = the
// tile's min/max of now.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace crane {

template <int kT>
__device__ __forceinline__ void k3p_tile(const int64_t t, const PodPrep& pp) {
    static_assert(1024 % kT == 0 && kT >= 64, "a tile is 1024 pods");
    constexpr int kU = 1024 / kT, kG = kU * (kT / 64);  // pods per lane, (u, wave) groups
    __shared__ int32_t cn[kG], cd[kG];
    __shared__ int64_t wmn[kT / 64], wmx[kT / 64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t lt = (1ull << lane) - 1ull;
    int64_t tn[kU];
    bool live[kU], ds[kU];
    int64_t mn = INT64_MAX, mx = INT64_MIN;
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const int64_t p = t * 1024 + u * kT + threadIdx.x;  // pod order = (u, wave, lane)
        live[u] = p < pp.P;
        ds[u] = live[u] && pp.flags && (pp.flags[p] & 1u);
        tn[u] = live[u] ? pp.now[p] : 0;
    }
    uint64_t mnm[kU], mdm[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const int64_t p = t * 1024 + u * kT + threadIdx.x;
        if (live[u]) {
            pp.keys[p] = -1;
            mn = min(mn, tn[u]);
            mx = max(mx, tn[u]);
        }
        mnm[u] = __ballot(live[u] && !ds[u]);
        mdm[u] = __ballot(ds[u]);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        mn = min(mn, (int64_t)__shfl_xor((long long)mn, o));
        mx = max(mx, (int64_t)__shfl_xor((long long)mx, o));
    }
    if (lane == 0) {
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            cn[u * (kT / 64) + w] = __popcll(mnm[u]);
            cd[u * (kT / 64) + w] = __popcll(mdm[u]);
        }
        wmn[w] = mn;
        wmx[w] = mx;
    }
    __syncthreads();
    int32_t tot_n = 0;
#pragma unroll
    for (int i = 0; i < kG; ++i) tot_n += cn[i];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const int gi = u * (kT / 64) + w;
        int32_t pre_n = 0, pre_d = 0;
        for (int i = 0; i < gi; ++i) {
            pre_n += cn[i];
            pre_d += cd[i];
        }
        if (live[u]) {
            const int64_t p = t * 1024 + u * kT + threadIdx.x;
            const int32_t pos =
                ds[u] ? tot_n + pre_d + __popcll(mdm[u] & lt) : pre_n + __popcll(mnm[u] & lt);
            pp.perm[t * 1024 + pos] = (int32_t)p | (ds[u] ? (int32_t)0x80000000 : 0);  // bit 31: DaemonSet
            pp.pnow[t * 1024 + pos] = tn[u];
        }
    }
    if (threadIdx.x == 0) {
        int64_t a = INT64_MAX, b = INT64_MIN;
#pragma unroll
        for (int i = 0; i < kT / 64; ++i) {
            a = min(a, wmn[i]);
            b = max(b, wmx[i]);
        }
        pp.tile_mm[2 * t] = a;
        pp.tile_mm[2 * t + 1] = b;
    }
}

__device__ __forceinline__ void k3p_tile256(const int64_t t, const PodPrep& pp) { k3p_tile<256>(t, pp); }

}  // namespace crane
