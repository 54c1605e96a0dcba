// lds_hash.hpp — the LDS hash aggregation of (node, bucket) keys shared by the K2 forms
// (hotcount.hip: dedupe, large) and the delta form's body (also run inside K3s's launch by
// step.hip, k3s_delta_pods).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace crane {

constexpr int kDSlots = 4096;  // 2 slots per binding: an empty or matching slot always exists

// (Round 5 measured against these split key / count arrays, cold 4M x 16M, same boxes, reverted:
// one packed 64-bit (key << 32 | count) slot with a plain read before the CAS — k2l_partition
// 0.042 -> 0.048 ms on the ordered log, 0.063 -> 0.071 on the stamp path; a thread's four first
// probes issued back to back and waited for together — 0.042 -> 0.044, 0.061 -> 0.066: the
// hash phase is bound by the LDS atomics' throughput and bank conflicts, not their latency.)
// Adds `add` to key's count; a lane that inserts a new key also counts it in its
// bin and returns its slot (else -1).  One returning LDS atomic per probe (the CAS
// itself tells an empty, a matching and a foreign slot apart).
template <int SLOTS = kDSlots>
__device__ __forceinline__ int32_t hash_add(int32_t* hkey, uint32_t* hcnt, uint32_t* hist, int bb, int32_t key,
                                            uint32_t add) {
    constexpr int kBits = __builtin_ctz(SLOTS);
    uint32_t h = ((uint32_t)key * 2654435761u) >> (32 - kBits);
    for (;;) {  // ends: at most SLOTS / 2 distinct keys
        const int32_t old = atomicCAS(&hkey[h], -1, key);
        if (old == -1 || old == key) {
            atomicAdd(&hcnt[h], add);
            if (old == -1) {
                atomicAdd(&hist[(key >> 3) >> bb], 1u);
                return (int32_t)h;
            }
            return -1;
        }
        h = (h + 1) & (SLOTS - 1);
    }
}

// A thread's KPER keys (node * 8 + bucket, -1 = none) into the LDS hash, one wave-
// instruction per key slot: the lanes sharing the first active lane's key add once
// (the Zipf-hot node), every other lane adds its own key.  The slots of new keys go to
// the wave's own segment of uniq (KPER * 64 entries: no shared counter); returns how many
// (uniform).  (More leader rounds for the next repeated keys measured slower at config 3.)
template <int SLOTS, int KPER>
__device__ __forceinline__ uint32_t wave_aggregate(const int32_t* key, int32_t* hkey, uint32_t* hcnt, uint32_t* hist,
                                                   int bb, uint16_t* useg) {
    const int lane = threadIdx.x & 63;
    uint32_t nw = 0;
#pragma unroll
    for (int u = 0; u < KPER; ++u) {
        const bool ok = key[u] >= 0;
        const uint64_t am = __ballot(ok);
        if (am == 0) continue;
        const int lead = __ffsll((long long)am) - 1;
        const int32_t kl = __builtin_amdgcn_readlane(key[u], lead);
        const uint64_t m = __ballot(ok && key[u] == kl);
        const bool mine = lane == lead || (ok && key[u] != kl);
        const int32_t slot = mine ? hash_add<SLOTS>(hkey, hcnt, hist, bb, lane == lead ? kl : key[u],
                                                    lane == lead ? (uint32_t)__popcll(m) : 1u)
                                  : -1;
        const uint64_t nm = __ballot(slot >= 0);
        if (slot >= 0) useg[nw + __popcll(nm & ((1ull << lane) - 1ull))] = (uint16_t)slot;
        nw += __popcll(nm);
    }
    return nw;
}

// ---------------------------------------------------------------- delta form
// (kernels.hpp HotDelta.)  Per workgroup 1024 changed bindings.  A binding whose position is
// inside window rank k at one of the two times and outside at the other changes that rank's
// count by one: key (node * 8 + k) * 2 + sign (sign 1: it left, -1; 0: it entered, +1) — one key
// per crossed cutoff, at most two with two windows (the form's limit, kDeltaMaxWin).  Keys are
// aggregated in the LDS hash as the dedupe form does (a Zipf-hot node costs one global atomic per
// workgroup and rank), then one atomicAdd per distinct key into adj [W][N] — per window rank, not
// per bucket: K1 turns them into bucket adjustments (adj[b] - adj[b + 1]).  Counts are modulo
// 2^32: anchor + adjustment is the exact count.
constexpr int kDeltaChunk = 1024;
constexpr int kDeltaSlots = 4 * kDeltaChunk;  // two per key, at most two keys per binding

template <int BT>
__device__ __forceinline__ void k2_delta_body(const int32_t blk, const int32_t* __restrict__ bnode, int64_t N,
                                              const HotDelta& d, uint32_t* __restrict__ adj) {
    constexpr int kPer = kDeltaChunk / BT;
    constexpr int kKeys = kPer * kDeltaMaxWin;  // key slots per thread: (binding, rank)
    extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
    __shared__ uint32_t hist[32];  // (hash_add's bin counts: not read)
    int32_t* hkey = reinterpret_cast<int32_t*>(sh);
    uint32_t* hcnt = sh + kDeltaSlots;
    uint16_t* uniq = reinterpret_cast<uint16_t*>(hcnt + kDSlots);
    const int64_t L = d.start[d.n_rng];
    int64_t pos[kPer];
    int32_t nd[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        const int64_t t = (int64_t)blk * kDeltaChunk + u * BT + threadIdx.x;
        int k = 0;
        for (int r = 1; r < d.n_rng; ++r) k += t >= d.start[r] ? 1 : 0;
        pos[u] = d.lo[k] + (t - d.start[k]);
        nd[u] = bnode[t < L ? pos[u] : d.lo[0]];  // (unconditional load, clamped)
        if (t >= L) nd[u] = -1;
    }
    for (int i = threadIdx.x; i < kDeltaSlots; i += BT) {
        hkey[i] = -1;
        hcnt[i] = 0;
    }
    if (threadIdx.x < 32) hist[threadIdx.x] = 0;
    __syncthreads();
    int32_t key[kKeys];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        const bool ok = nd[u] >= 0 && (int64_t)nd[u] < N;  // binding.go:85-91 at both times
#pragma unroll
        for (int r = 0; r < kDeltaMaxWin; ++r) {
            const bool ia = pos[u] >= d.a[r], ip = pos[u] >= d.p[r];
            key[u * kDeltaMaxWin + r] = ok && r < d.n_win && ia != ip ? ((nd[u] * 8 + r) << 1) | (ia ? 1 : 0) : -1;
        }
    }
    uint16_t* useg = uniq + (threadIdx.x >> 6) * (kKeys * 64);
    const uint32_t nw = wave_aggregate<kDeltaSlots, kKeys>(key, hkey, hcnt, hist, 24, useg);
    __syncthreads();
    for (uint32_t i = threadIdx.x & 63; i < nw; i += 64) {  // this wave's new keys
        const int s = useg[i];
        const int32_t k = hkey[s];
        const uint32_t c = hcnt[s];
        atomicAdd(&adj[(int64_t)((k >> 1) & 7) * N + (k >> 4)], (k & 1) ? 0u - c : c);
    }
}


}  // namespace crane
