// greedy.hip — sequential-greedy batch placement (BASELINE config 5).
//
// One `now` for the batch.  Pods are placed in order; each placement is a new
// Binding{Timestamp: now_unix} on the chosen node, which raises that node's
// window counts (binding.go:85-91: now_unix > now_unix - int64(tr.Seconds())
// iff the window is positive), hence its hot value (node.go:113-121) and
// penalty int(hv*10) (plugins.go:91), before the next pod is scored.  Since
// `now` is fixed, only the chosen node's score changes per step.
//
// G1 greedy_prep: one thread per node — base = int(score/weight) at now
//    (stats.go:114-138, exact int64 path), feasibility (plugins.go:55-66) and
//    the leaf byte = final score | feasible << 7.
// G2 greedy_run: ONE workgroup.  Leaves live in LDS (N <= kGreedyLdsLeaves)
//    or global memory; above them a 64-ary max tree of (max feasible, max any)
//    score pairs in LDS.  Per pod, wave 0 descends the tree with 7-step ballot
//    argmax at the root and one ballot per lower level (lowest index wins
//    ties), then updates the chosen node's counts and leaf and re-reduces its
//    ancestors.  No float, no atomics, one wave: deterministic.
#include <hip/hip_runtime.h>

#include "dyn_types.hpp"
#include "kernels.hpp"

namespace crane {

__device__ __forceinline__ int64_t go_int_g(double x) {
    if (!(x >= -9223372036854775808.0 && x < 9223372036854775808.0)) return INT64_MIN;
    return (int64_t)x;
}

__device__ __forceinline__ int32_t final_score(int64_t base, int64_t pen) {
    const int64_t f = (int64_t)((uint64_t)base - (uint64_t)pen);  // Go int64 wraps
    return (int32_t)(f < 0 ? 0 : (f > 100 ? 100 : f));
}

// hot value of a node from its per-window counts (node.go:113-121)
__device__ __forceinline__ int64_t pen_of(const uint32_t* cnt, int64_t N, int64_t n, const GreedyArgs& a) {
    int64_t v = 0;
    for (int w = 0; w < a.n_win; ++w) {
        const uint32_t c = cnt[(int64_t)w * N + n];
        const int64_t k = a.win_count[w];
        // Go int division truncates toward zero; 32-bit unsigned division when it is the same thing
        v += (k > 0 && k <= 0xFFFFFFFFll) ? (int64_t)(c / (uint32_t)k) : (int64_t)c / k;
    }
    if (v < 0) return 0;  // a negative annotation is rejected (stats.go:71-73) -> hot value 0
    return go_int_g((double)v * 10.0);
}

template <int PD, int PR>
__global__ __launch_bounds__(256) void greedy_prep(const NodeRec<PD, PR>* __restrict__ rec, int64_t N,
                                                   const uint32_t* __restrict__ cnt, GreedyArgs a,
                                                   int64_t* __restrict__ base_out, uint8_t* __restrict__ leaf) {
    const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (n >= N) return;
    const NodeRec<PD, PR>& r = rec[n];
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < PR; ++k)
        if (a.now < r.e_prio[k]) s += r.t[k];
    const int64_t base = a.noprio ? 0 : go_int_g(s / a.wsum);
    const bool feasible = !(a.now < r.e_fail);
    base_out[n] = base;
    leaf[n] = (uint8_t)(final_score(base, pen_of(cnt, N, n, a)) | (feasible ? 0x80 : 0));
}

// ---- wave helpers (64 lanes)
__device__ __forceinline__ uint64_t ballot64(bool p) { return __ballot(p); }

// max over lanes of v in [0, 127] and the lowest lane holding it; v < 0 lanes never win
__device__ __forceinline__ int wave_argmax7(int v, int* lane_out) {
    uint64_t cand = ballot64(v >= 0);
    if (!cand) {
        *lane_out = -1;
        return -1;
    }
    int m = 0;
#pragma unroll
    for (int b = 6; b >= 0; --b) {
        const uint64_t with = cand & ballot64((v >> b) & 1);
        if (with) {
            cand = with;
            m |= 1 << b;
        }
    }
    *lane_out = __builtin_ctzll(cand);
    return m;
}

// wave max via DPP: row_shr 1,2,4,8 then row_bcast15/31 (GFX9 family) -> lane 63.
// Out-of-range source lanes return `old` = v itself, the identity of max.
__device__ __forceinline__ int wave_max_dpp(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x111, 0xF, 0xF, false));  // row_shr:1
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x112, 0xF, 0xF, false));  // row_shr:2
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x114, 0xF, 0xF, false));  // row_shr:4
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x118, 0xF, 0xF, false));  // row_shr:8
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x142, 0xA, 0xF, false));  // row_bcast:15
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x143, 0xC, 0xF, false));  // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}

constexpr int kGreedyLevels = 4;  // 64^4 = 16.7M nodes

struct Tree {
    int nlev;                     // internal levels above the leaves (>= 1)
    int64_t size[kGreedyLevels + 1];  // entries per level, level 0 = leaves
    uint16_t* lvl[kGreedyLevels + 1]; // LDS arrays for levels >= 1: lo byte max-any, hi byte max-feasible+1
};

__device__ __forceinline__ int leaf_val(uint8_t b, bool any) {
    const int sc = b & 0x7F;
    return any ? sc : ((b & 0x80) ? sc : -1);
}
__device__ __forceinline__ int ent_val(uint16_t e, bool any) { return any ? (int)(e & 0xFF) : (int)(e >> 8) - 1; }

template <int NLEV>
__global__ __launch_bounds__(256) void greedy_run(int64_t N, uint8_t* __restrict__ leaf_g, const int64_t* __restrict__ base,
                                                  uint32_t* __restrict__ cnt, GreedyArgs a, int64_t P,
                                                  const uint8_t* __restrict__ flags, int64_t* __restrict__ chosen,
                                                  int32_t leaves_in_lds) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // layout: [leaves (if in LDS)] [level 1] [level 2] ...
    // Every index into t.size / t.lvl below is a compile-time constant (loops
    // over levels are fully unrolled), so the metadata stays in registers.
    Tree t;
    t.size[0] = N;
    t.nlev = NLEV;
    {
        int64_t off = leaves_in_lds ? (N + 15) / 16 * 16 : 0, sz = N;
#pragma unroll
        for (int l = 1; l <= NLEV; ++l) {
            sz = (sz + 63) / 64;
            t.size[l] = sz;
            t.lvl[l] = reinterpret_cast<uint16_t*>(smem + off);
            off += (sz * 2 + 15) / 16 * 16;
        }
    }
    uint8_t* leaf = leaves_in_lds ? smem : leaf_g;
    if (leaves_in_lds)
        for (int64_t i = threadIdx.x; i < N; i += blockDim.x) leaf[i] = leaf_g[i];
    // Warm this XCD's L2 with the per-node state the commits touch (base, counts):
    // most placements hit a node for the first time, which would otherwise be an
    // HBM-latency miss on the serial path.  The xor keeps the loads live.
    {
        uint64_t x = 0;
        for (int64_t i = threadIdx.x; i < N; i += blockDim.x) {
            x ^= (uint64_t)base[i];
            for (int w = 0; w < a.n_win; ++w) x ^= cnt[(int64_t)w * N + i];
        }
        if (x == 0x9E3779B97F4A7C15ull && P < 0) chosen[0] = (int64_t)x;  // never true: keeps the loads
    }
    __syncthreads();
    // build level 1 from leaves, then each level from the one below
#pragma unroll
    for (int l = 1; l <= NLEV; ++l) {
        for (int64_t e = threadIdx.x; e < t.size[l]; e += blockDim.x) {
            int ma = 0, mf = -1;
            for (int j = 0; j < 64; ++j) {
                const int64_t c = e * 64 + j;
                if (c >= t.size[l - 1]) break;
                int va, vf;
                if (l == 1) {
                    va = leaf_val(leaf[c], true);
                    vf = leaf_val(leaf[c], false);
                } else {
                    va = ent_val(t.lvl[l - 1][c], true);
                    vf = ent_val(t.lvl[l - 1][c], false);
                }
                ma = max(ma, va);
                mf = max(mf, vf);
            }
            t.lvl[l][e] = (uint16_t)(ma | ((mf + 1) << 8));
        }
        __syncthreads();
    }
    if (wave != 0) return;
    constexpr int top = NLEV;
    for (int64_t p0 = 0; p0 < P; p0 += 64) {
        const int64_t pl = p0 + lane;
        // DaemonSet pods bypass Filter (plugins.go:41-43): one bit per pod of this chunk
        const uint64_t dsmask = ballot64(pl < P && flags && (flags[pl] & 1u));
        int64_t out = -1;
        const int np = (int)min((int64_t)64, P - p0);
        for (int q = 0; q < np; ++q) {
            const bool any = (dsmask >> q) & 1;
            // ---- descent: root level (<= 64 entries), then one ballot per level
            const int v = lane < t.size[top] ? ent_val(t.lvl[top][lane], any) : -1;
            const int M = wave_max_dpp(v);
            int64_t idx = -1;
            if (M >= 0) {
                idx = __builtin_ctzll(ballot64(v == M));
#pragma unroll
                for (int l = top - 1; l >= 0; --l) {
                    const int64_t c = idx * 64 + lane;
                    int w = -1;
                    if (c < t.size[l]) w = l == 0 ? leaf_val(leaf[c], any) : ent_val(t.lvl[l][c], any);
                    idx = idx * 64 + __builtin_ctzll(ballot64(w == M));
                }
            }
            if (lane == q) out = idx;
            if (idx < 0) continue;
            // ---- commit: Binding{Node: idx, Timestamp: now_unix}
            if (lane == 0) {
                // one round trip: counts and base load together, counts stored back
                uint32_t c[kMaxWin];
#pragma unroll
                for (int w = 0; w < kMaxWin; ++w)
                    if (w < a.n_win) c[w] = cnt[(int64_t)w * N + idx];
                const int64_t b = base[idx];
                int64_t v = 0;
#pragma unroll
                for (int w = 0; w < kMaxWin; ++w) {
                    if (w >= a.n_win) break;
                    c[w] += a.win_inc[w] ? 1u : 0u;
                    cnt[(int64_t)w * N + idx] = c[w];
                    const int64_t k = a.win_count[w];
                    v += (k > 0 && k <= 0xFFFFFFFFll) ? (int64_t)(c[w] / (uint32_t)k) : (int64_t)c[w] / k;
                }
                const int64_t pen = v < 0 ? 0 : go_int_g((double)v * 10.0);  // node.go:117, plugins.go:91
                const uint8_t old = leaf[idx];
                leaf[idx] = (uint8_t)(final_score(b, pen) | (old & 0x80));
            }
            // LDS instructions of one wave execute in order, so lane 0's leaf store
            // is seen by the reads below; a global leaf store is waited for.
            if (!leaves_in_lds) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            // ---- re-reduce the ancestors of idx; stop once an entry is unchanged
            int64_t child = idx;
#pragma unroll
            for (int l = 1; l <= NLEV; ++l) {
                const int64_t e = child / 64, c = e * 64 + lane;
                int va = -1, vf = -1;
                if (c < t.size[l - 1]) {
                    if (l == 1) {
                        va = leaf_val(leaf[c], true);
                        vf = leaf_val(leaf[c], false);
                    } else {
                        va = ent_val(t.lvl[l - 1][c], true);
                        vf = ent_val(t.lvl[l - 1][c], false);
                    }
                }
                const int ma = wave_max_dpp(va), mf = wave_max_dpp(vf);
                const uint16_t ne = (uint16_t)(max(ma, 0) | ((mf + 1) << 8));
                const uint16_t oe = t.lvl[l][e];
                if (ne == oe) break;
                __builtin_amdgcn_wave_barrier();
                if (lane == 0) t.lvl[l][e] = ne;
                __builtin_amdgcn_wave_barrier();
                child = e;
            }
        }
        if (lane < np) chosen[p0 + lane] = out;
    }
    if (leaves_in_lds)
        for (int64_t i = lane; i < N; i += 64) leaf_g[i] = leaf[i];
}

size_t greedy_lds_bytes(int64_t N, bool leaves_in_lds) {
    size_t off = leaves_in_lds ? (size_t)((N + 15) / 16 * 16) : 0;
    int64_t sz = N;
    int nlev = 0;
    do {
        sz = (sz + 63) / 64;
        nlev++;
        off += (size_t)((sz * 2 + 15) / 16 * 16);
    } while (sz > 64 && nlev < kGreedyLevels);
    return off;
}

template <int PD, int PR>
static hipError_t launch_greedy_t(const void* rec, int64_t N, uint32_t* cnt, const GreedyArgs& a, int64_t* base,
                                  uint8_t* leaf, int64_t P, const uint8_t* flags, int64_t* chosen, hipStream_t st,
                                  int what) {
    if (N > kGreedyMaxNodes) return hipErrorInvalidValue;
    if (N > 0 && (what & kGreedyPrep)) {
        hipError_t e = klaunch("greedy_prep", greedy_prep<PD, PR>, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st,
                               static_cast<const NodeRec<PD, PR>*>(rec), N, cnt, a, base, leaf);
        if (e != hipSuccess) return e;
    }
    if (!(what & kGreedyRun)) return hipSuccess;
    const bool in_lds = greedy_lds_bytes(N, true) <= kGreedyLdsBytes;
    const size_t lds = greedy_lds_bytes(N, in_lds);
    int nlev = 0;
    for (int64_t sz = N; nlev == 0 || sz > 64;) {
        sz = (sz + 63) / 64;
        ++nlev;
    }
#define GREEDY_LAUNCH(L)                                                                                        \
    do {                                                                                                        \
        static const hipError_t attr = hipFuncSetAttribute((const void*)greedy_run<L>,                          \
                                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
        if (attr != hipSuccess) return attr;                                                                    \
        return klaunch("greedy_run", greedy_run<L>, dim3(1), dim3(256), lds, st, N, leaf, base, cnt, a, P, flags, \
                       chosen, (int32_t)in_lds);                                                                \
    } while (0)
    switch (nlev) {
        case 1: GREEDY_LAUNCH(1);
        case 2: GREEDY_LAUNCH(2);
        case 3: GREEDY_LAUNCH(3);
        default: GREEDY_LAUNCH(4);
    }
#undef GREEDY_LAUNCH
}

hipError_t launch_greedy(int shape, const void* rec, int64_t N, uint32_t* cnt, const GreedyArgs& a, int64_t* base,
                         uint8_t* leaf, int64_t P, const uint8_t* flags, int64_t* chosen, hipStream_t st, int what) {
    switch (shape) {
        case kShape4x6: return launch_greedy_t<4, 6>(rec, N, cnt, a, base, leaf, P, flags, chosen, st, what);
        case kShape8x8: return launch_greedy_t<8, 8>(rec, N, cnt, a, base, leaf, P, flags, chosen, st, what);
        default: return launch_greedy_t<16, 16>(rec, N, cnt, a, base, leaf, P, flags, chosen, st, what);
    }
}

}  // namespace crane
