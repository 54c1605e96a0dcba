// kernels.hip — CDNA4 (gfx950) kernels of the Dynamic plugin hot path.
//
//   K2 hot_count : binding records -> per-node window counts (LDS-aggregated)
//   K1 node_pass : parsed annotation SoA (+ K2 counts) -> NodeRec per node
//   K3 eval      : pods x nodes Filter + Score + per-pod argmax
//
// Numerics follow /root/reference/pkg/plugins/dynamic/stats.go and plugins.go
// bit for bit: fp64 in the reference's operation order, no FMA contraction
// (built with -ffp-contract=off), Go's float64->int conversion and wrapping
// int64 arithmetic.  Wave = 64 lanes; K3 puts 64 PODS on a wave so every node
// record is wave-uniform and arrives through scalar loads.
#include <hip/hip_runtime.h>

#include "dyn_types.hpp"
#include "kernels.hpp"

namespace crane {

// Go int(float64) on amd64 (CVTTSD2SQ): NaN and out-of-range -> INT64_MIN.
// Used by stats.go:135 (int(score/weight)) and plugins.go:91 (int(hv*10)).
__device__ __forceinline__ int64_t go_int(double x) {
    if (!(x >= -9223372036854775808.0 && x < 9223372036854775808.0)) return INT64_MIN;
    return (int64_t)x;
}

__device__ __forceinline__ int64_t sat_add(int64_t a, int64_t b) {
    int64_t r;
    if (__builtin_add_overflow(a, b, &r)) return b > 0 ? INT64_MAX : INT64_MIN;
    return r;
}

// ---------------------------------------------------------------- K2
// Each binding b falls into the windows whose cutoff (now_unix -
// int64(timeRange.Seconds()), binding.go:85) is < ts_b.  With cutoffs sorted
// ascending that set is a prefix 0..j-1, so one count per binding goes to
// bucket j-1 and window w's count is the suffix sum of buckets from its rank
// (done in K1).  A workgroup aggregates its slice of bindings in an LDS hash
// table keyed by node (open addressing, CAS insert) before touching global
// memory, so Zipf-hot nodes cost one global atomic per workgroup instead of
// one per binding.
constexpr int kHashSlots = 4096;  // per workgroup
constexpr int kMaxProbe = 16;
constexpr int kK2Threads = 1024;
constexpr int kK2PerThread = 16;

__global__ __launch_bounds__(kK2Threads) void k2_hot_count(const int32_t* __restrict__ bnode,
                                                            const int64_t* __restrict__ bts, int64_t B,
                                                            int64_t N, HotCutoffs cut, uint32_t* __restrict__ buckets) {
    __shared__ int32_t hkey[kHashSlots];
    __shared__ uint32_t hcnt[kHashSlots * kLdsWin];
    const int W = cut.n_win;
    for (int i = threadIdx.x; i < kHashSlots; i += blockDim.x) hkey[i] = -1;
    for (int i = threadIdx.x; i < kHashSlots * kLdsWin; i += blockDim.x) hcnt[i] = 0;
    __syncthreads();
    const int64_t per_block = (int64_t)kK2Threads * kK2PerThread;
    const int64_t b0 = (int64_t)blockIdx.x * per_block;
    const int64_t b1 = min(B, b0 + per_block);
    for (int64_t b = b0 + threadIdx.x; b < b1; b += blockDim.x) {
        const int32_t nd = bnode[b];
        const int64_t ts = bts[b];
        if (nd < 0 || (int64_t)nd >= N) continue;  // binding.go:88 — matches no node of this shard
        int j = 0;
#pragma unroll
        for (int w = 0; w < kMaxWin; ++w)
            if (w < W) j += ts > cut.sorted[w] ? 1 : 0;
        if (j == 0) continue;
        const int bucket = j - 1;
        if (W > kLdsWin) {  // wide policies: straight to global
            atomicAdd(&buckets[(int64_t)bucket * N + nd], 1u);
            continue;
        }
        uint32_t h = ((uint32_t)nd * 2654435761u) >> (32 - 12);
        bool done = false;
        for (int p = 0; p < kMaxProbe && !done; ++p) {
            const int32_t k = __hip_atomic_load(&hkey[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (k == nd) {
                atomicAdd(&hcnt[h * kLdsWin + bucket], 1u);
                done = true;
            } else if (k == -1) {
                const int32_t old = atomicCAS(&hkey[h], -1, nd);
                if (old == -1 || old == nd) {
                    atomicAdd(&hcnt[h * kLdsWin + bucket], 1u);
                    done = true;
                }
            }
            h = (h + 1) & (kHashSlots - 1);
        }
        if (!done) atomicAdd(&buckets[(int64_t)bucket * N + nd], 1u);
    }
    __syncthreads();
    if (W > kLdsWin) return;
    for (int s = threadIdx.x; s < kHashSlots; s += blockDim.x) {
        const int32_t nd = hkey[s];
        if (nd < 0) continue;
        for (int w = 0; w < W; ++w) {
            const uint32_t c = hcnt[s * kLdsWin + w];
            if (c) atomicAdd(&buckets[(int64_t)w * N + nd], c);
        }
    }
}

// ---------------------------------------------------------------- K1
// One thread per node.  Reads the parsed SoA (and K2 buckets), writes the
// node's NodeRec into LDS, then the workgroup streams its records out with
// 16-byte coalesced stores.
constexpr int kK1Threads = 128;

template <int PD, int PR>
__global__ __launch_bounds__(kK1Threads) void k1_node_pass(DevPolicy pol, int64_t N, const double* __restrict__ val,
                                                           const int64_t* __restrict__ ts,
                                                           const double* __restrict__ hv,
                                                           const int64_t* __restrict__ hv_ts,
                                                           const uint32_t* __restrict__ buckets, int64_t hv_ts_counts,
                                                           NodeRec<PD, PR>* __restrict__ out) {
    using Rec = NodeRec<PD, PR>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    Rec* lrec = reinterpret_cast<Rec*>(smem);
    const int64_t first = (int64_t)blockIdx.x * kK1Threads;
    const int64_t n = first + threadIdx.x;
    if (n < N) {
        Rec r;
#pragma unroll
        for (int k = 0; k < PD; ++k) {
            int64_t e = kTsInvalid;
            if (k < pol.npd) {
                const int64_t row = pol.pred_slot[k];
                const int64_t t = ts[row * N + n];
                const double u = val[row * N + n];
                const double lim = pol.pred_limit[k];
                // isOverLoad (stats.go:94-112): usable (stats.go:51-76), limit != 0, u > limit
                const bool over = t != kTsInvalid && !(u < 0.0) && lim != 0.0 && u > lim;
                if (over) e = sat_add(t, pol.pred_dur[k]);
            }
            r.e_pred[k] = e;
        }
#pragma unroll
        for (int k = 0; k < PR; ++k) {
            int64_t e = kTsInvalid;
            double term = 0.0;
            if (k < pol.npr) {
                const int64_t row = pol.prio_slot[k];
                const int64_t t = ts[row * N + n];
                const double u = val[row * N + n];
                if (t != kTsInvalid && !(u < 0.0)) {
                    e = sat_add(t, pol.prio_dur[k]);
                    // getScore (stats.go:89): (1. - usage) * Weight * float64(MaxNodeScore)
                    term = (1.0 - u) * pol.prio_w[k];
                    term = term * 100.0;
                }
            }
            r.e_prio[k] = e;
            r.t[k] = term;
        }
        if (buckets) {
            // annotateNodeHotValue (node.go:113-121): value += count / p.Count (Go int division)
            int64_t v = 0;
            for (int w = 0; w < pol.n_win; ++w) {
                int64_t c = 0;
                for (int b = pol.win_pos[w]; b < pol.n_win; ++b) c += buckets[(int64_t)b * N + n];
                v += c / pol.win_count[w];
            }
            // the plugin re-reads it via ParseFloat (exact) and rejects negatives (stats.go:71-73)
            const double h = (double)v;
            r.pen = go_int(h * 10.0);
            r.e_hv = v >= 0 ? sat_add(hv_ts_counts, kHotActiveNs) : kTsInvalid;
        } else if (hv) {
            const double h = hv[n];
            const int64_t t = hv_ts[n];
            r.pen = go_int(h * 10.0);
            r.e_hv = (t != kTsInvalid && !(h < 0.0)) ? sat_add(t, kHotActiveNs) : kTsInvalid;
        } else {
            r.pen = 0;
            r.e_hv = kTsInvalid;
        }
        lrec[threadIdx.x] = r;
    }
    __syncthreads();
    const int64_t nvalid = min((int64_t)kK1Threads, N - first);
    const int64_t nvec = nvalid * (int64_t)sizeof(Rec) / 16;
    const uint4* src = reinterpret_cast<const uint4*>(smem);
    uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<unsigned char*>(out) + first * (int64_t)sizeof(Rec));
    for (int64_t i = threadIdx.x; i < nvec; i += kK1Threads) dst[i] = src[i];
}

// ---------------------------------------------------------------- K3
// blockIdx.x -> 256 pods (4 waves x 64), blockIdx.y -> a chunk of nodes.
// Every lane walks the chunk's nodes in ascending order keeping the first
// node with the highest score (lowest-index tie-break), then one 64-bit
// atomicMax per pod merges chunks.  The NodeRec address depends only on the
// loop counter, so it is wave-uniform and loaded with s_load into SGPRs.
constexpr int kK3Threads = 256;

template <int PD, int PR, bool MATRIX>
__global__ __launch_bounds__(kK3Threads) void k3_eval(const NodeRec<PD, PR>* __restrict__ rec, int64_t N,
                                                      int64_t chunk, int64_t node_offset,
                                                      const int64_t* __restrict__ now, const uint8_t* __restrict__ flags,
                                                      int64_t P, double wsum, int32_t noprio,
                                                      long long* __restrict__ keys, MatrixOut mo) {
    const int64_t pod = (int64_t)blockIdx.x * kK3Threads + threadIdx.x;
    const bool live = pod < P;
    const int64_t tnow = live ? now[pod] : INT64_MIN;
    const bool ds = live && flags && (flags[pod] & 1u);
    const int64_t n0 = (int64_t)blockIdx.y * chunk;
    const int64_t n1 = min(N, n0 + chunk);
    int32_t best_s = -1;
    int64_t best_n = 0;
    for (int64_t n = n0; n < n1; ++n) {
        const NodeRec<PD, PR>& r = rec[n];
        // Filter (plugins.go:55-66): some predicate fresh and over its limit
        bool fail = false;
#pragma unroll
        for (int k = 0; k < PD; ++k) fail |= tnow < r.e_pred[k];
        // getNodeScore (stats.go:124-135): fresh terms summed in policy order
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < PR; ++k) {
            const double a = s + r.t[k];
            s = tnow < r.e_prio[k] ? a : s;
        }
        const int64_t base = noprio ? 0 : go_int(s / wsum);
        // score - int(hotValue*10), NormalizeScore to [0,100] (plugins.go:91-93)
        const int64_t pen = tnow < r.e_hv ? r.pen : 0;
        int64_t f = (int64_t)((uint64_t)base - (uint64_t)pen);
        f = f < 0 ? 0 : (f > 100 ? 100 : f);
        const bool feasible = ds || !fail;
        if (feasible && (int32_t)f > best_s) {
            best_s = (int32_t)f;
            best_n = n;
        }
        if constexpr (MATRIX) {
            if (live) {
                int8_t ff = -1;
                if (!ds) {
#pragma unroll
                    for (int k = PD - 1; k >= 0; --k)
                        if (tnow < r.e_pred[k]) ff = mo.pred_orig[k];
                }
                if (mo.first_fail) mo.first_fail[pod * N + n] = ff;
                if (mo.score) mo.score[pod * N + n] = f;
            }
        }
    }
    if (live && best_s >= 0) {
        const long long key = ((long long)best_s << 32) | (long long)(0xFFFFFFFFull - (uint64_t)(node_offset + best_n));
        atomicMax(&keys[pod], key);
    }
}

// ---------------------------------------------------------------- launchers
template <int PD, int PR>
static hipError_t launch_k1_t(const DevPolicy& pol, int64_t N, const double* val, const int64_t* ts, const double* hv,
                              const int64_t* hv_ts, const uint32_t* buckets, int64_t hv_ts_counts, void* out,
                              hipStream_t st) {
    if (N <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((N + kK1Threads - 1) / kK1Threads);
    const size_t lds = sizeof(NodeRec<PD, PR>) * kK1Threads;
    hipLaunchKernelGGL((k1_node_pass<PD, PR>), dim3(grid), dim3(kK1Threads), lds, st, pol, N, val, ts, hv, hv_ts,
                       buckets, hv_ts_counts, static_cast<NodeRec<PD, PR>*>(out));
    return hipGetLastError();
}

hipError_t launch_node_pass(int shape, const DevPolicy& pol, int64_t N, const double* val, const int64_t* ts,
                            const double* hv, const int64_t* hv_ts, const uint32_t* buckets, int64_t hv_ts_counts,
                            void* out, hipStream_t st) {
    switch (shape) {
        case kShape4x6: return launch_k1_t<4, 6>(pol, N, val, ts, hv, hv_ts, buckets, hv_ts_counts, out, st);
        case kShape8x8: return launch_k1_t<8, 8>(pol, N, val, ts, hv, hv_ts, buckets, hv_ts_counts, out, st);
        default: return launch_k1_t<16, 16>(pol, N, val, ts, hv, hv_ts, buckets, hv_ts_counts, out, st);
    }
}

size_t node_rec_bytes(int shape) {
    switch (shape) {
        case kShape4x6: return sizeof(NodeRec<4, 6>);
        case kShape8x8: return sizeof(NodeRec<8, 8>);
        default: return sizeof(NodeRec<16, 16>);
    }
}

hipError_t launch_hot_count(const int32_t* bnode, const int64_t* bts, int64_t B, int64_t N, const HotCutoffs& cut,
                            uint32_t* buckets, hipStream_t st) {
    if (B <= 0 || cut.n_win <= 0) return hipSuccess;
    const int64_t per_block = (int64_t)kK2Threads * kK2PerThread;
    const unsigned grid = (unsigned)((B + per_block - 1) / per_block);
    hipLaunchKernelGGL(k2_hot_count, dim3(grid), dim3(kK2Threads), 0, st, bnode, bts, B, N, cut, buckets);
    return hipGetLastError();
}

int64_t eval_chunk_nodes(int64_t P, int64_t N) {
    // Enough workgroups to fill 256 CUs several times over, chunks of >= 64 nodes.
    const int64_t pod_blocks = (P + kK3Threads - 1) / kK3Threads;
    int64_t want_chunks = (4096 + pod_blocks - 1) / pod_blocks;
    int64_t chunk = (N + want_chunks - 1) / want_chunks;
    if (chunk < 64) chunk = 64;
    return chunk;
}

template <int PD, int PR>
static hipError_t launch_k3_t(const void* rec, int64_t N, int64_t node_offset, const int64_t* now,
                              const uint8_t* flags, int64_t P, double wsum, int32_t noprio, long long* keys,
                              const MatrixOut& mo, hipStream_t st) {
    if (P <= 0 || N <= 0) return hipSuccess;
    const int64_t chunk = eval_chunk_nodes(P, N);
    const dim3 grid((unsigned)((P + kK3Threads - 1) / kK3Threads), (unsigned)((N + chunk - 1) / chunk));
    const auto* r = static_cast<const NodeRec<PD, PR>*>(rec);
    if (mo.first_fail || mo.score)
        hipLaunchKernelGGL((k3_eval<PD, PR, true>), grid, dim3(kK3Threads), 0, st, r, N, chunk, node_offset, now,
                           flags, P, wsum, noprio, keys, mo);
    else
        hipLaunchKernelGGL((k3_eval<PD, PR, false>), grid, dim3(kK3Threads), 0, st, r, N, chunk, node_offset, now,
                           flags, P, wsum, noprio, keys, mo);
    return hipGetLastError();
}

hipError_t launch_eval(int shape, const void* rec, int64_t N, int64_t node_offset, const int64_t* now,
                       const uint8_t* flags, int64_t P, double wsum, int32_t noprio, long long* keys,
                       const MatrixOut& mo, hipStream_t st) {
    switch (shape) {
        case kShape4x6: return launch_k3_t<4, 6>(rec, N, node_offset, now, flags, P, wsum, noprio, keys, mo, st);
        case kShape8x8: return launch_k3_t<8, 8>(rec, N, node_offset, now, flags, P, wsum, noprio, keys, mo, st);
        default: return launch_k3_t<16, 16>(rec, N, node_offset, now, flags, P, wsum, noprio, keys, mo, st);
    }
}

}  // namespace crane
