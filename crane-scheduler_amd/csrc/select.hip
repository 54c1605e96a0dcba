// select.hip — framework-level selection around the Dynamic plugin (SURVEY §8f
// row 4): what kube-scheduler v1.23.3 (k8s.io/kubernetes, go.mod:26; not in the
// container, restated from its published pkg/scheduler/core/generic_scheduler.go)
// does with the plugin's Filter / Score for each pod of a queue, in order:
//
//   findNodesThatPassFilters: numNodesToFind = numFeasibleNodesToFind(N) (the
//     percentageOfNodesToScore rule, host side); nodes are checked in rotated
//     order from nextStartNodeIndex until that many pass every filter plugin,
//     then nextStartNodeIndex += processed (checked) nodes, mod N.  Upstream
//     checks with 16 goroutines and cancels once enough are found; this is its
//     sequential order (the first numNodesToFind feasible nodes of the rotation).
//   prioritizeNodes: per feasible node, sum of weight * score over the score
//     plugins: Dynamic's Score (plugins.go:73-98) times its weight (3 in the
//     shipped profile, deploy/manifests/dynamic/scheduler-config.yaml:13-15)
//     plus the other plugins' weighted sum, given per node (ext_score).
//   selectHost: the max; upstream breaks ties by reservoir sampling with the
//     global math/rand source.  Here: lowest node index (seed 0) or a seeded
//     tie-break: the tie key is a bijection of the node index (murmur3's
//     fmix32 of index ^ batch key, xor a per-pod key), so a packed key still
//     decodes to its node after a max over shards.
//
// Kernels: k_sel_fth (per node feasibility threshold: a non-DaemonSet pod
// passes every filter iff now >= fth, since Dynamic's Filter fails exactly
// while now < e_fail, the latest overloaded predicate's expiry); k_sel_chain
// (one wave walks the queue in order: per pod, 64 rotated positions per step,
// a ballot and popcounts find the numNodesToFind-th feasible node, the window =
// positions up to it, the next pod starts after it); k_sel_pairs (per (pod, node): feasible, in the
// pod's window, weighted total; lane-cached step results like K3m, matrix.hip;
// 64-bit keys, wave max, one LDS and one global atomicMax per pod per
// workgroup); k_sel_decode (key -> node, total).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dyn_types.hpp"
#include "kernels.hpp"
#include "step_node.hpp"

namespace crane {

// ---------------------------------------------------------------- tie keys
__host__ __device__ inline uint32_t tie_mix(uint32_t x) {  // murmur3 fmix32: a bijection
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    x ^= x >> 16;
    return x;
}
__host__ __device__ inline uint32_t unshift_xor(uint32_t y, int s) {  // inverse of y = x ^ (x >> s)
    uint32_t x = y;
    for (int i = s; i < 32; i += s) x = y ^ (x >> s);
    return x;
}
__host__ __device__ inline uint32_t tie_unmix(uint32_t h) {
    h = unshift_xor(h, 16);
    h *= 0x7ED1B41Du;  // 0xC2B2AE35^-1 mod 2^32
    h = unshift_xor(h, 13);
    h *= 0xA5CB9243u;  // 0x85EBCA6B^-1 mod 2^32
    h = unshift_xor(h, 16);
    return h;
}
__host__ __device__ inline uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ inline uint32_t tie_pod_key(uint64_t seed, int64_t p) {
    return seed ? (uint32_t)splitmix64(seed ^ ((uint64_t)(p + 1) * 0xD1B54A32D192ED03ull)) : 0u;
}
// the low word of a packed key for global node g (the larger wins among equal totals)
__host__ __device__ inline uint32_t tie_node(uint64_t seed, uint32_t kb, uint32_t g) {
    return seed ? tie_mix(g ^ kb) : 0xFFFFFFFFu - g;
}
__host__ __device__ inline uint32_t tie_decode(uint64_t seed, uint32_t kb, uint32_t lo, uint32_t cp) {
    return seed ? tie_unmix(lo ^ cp) ^ kb : 0xFFFFFFFFu - lo;
}

// ---------------------------------------------------------------- k_sel_fth
// fth[0][n]: a non-DaemonSet pod passes every filter iff now >= it; fth[1][n]: the
// same for DaemonSet pods (the other plugins' filters only)
template <int PD, int PR>
__global__ __launch_bounds__(256) void k_sel_fth(SelArgs a, int64_t* __restrict__ fth) {
    const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (n >= a.N) return;
    const bool ok = !a.ext_ok || a.ext_ok[n];
    fth[n] = ok ? static_cast<const NodeRec<PD, PR>*>(a.rec)[n].e_fail : INT64_MAX;
    fth[a.N + n] = ok ? INT64_MIN : INT64_MAX;
}

// ---------------------------------------------------------------- k_sel_chain
// One wave walks the queue: a pod's window is the rotated positions from the running
// start up to its numNodesToFind-th feasible node, the next pod starts right after,
// so the walk is one sequential sweep over the rotation.  64 positions per step (one
// per lane, a ballot, a popcount), kChU steps' loads in flight, no barriers.
constexpr int kChU = 8;

__global__ __launch_bounds__(64) void k_sel_chain(SelArgs a, const int64_t* __restrict__ fth, int64_t K,
                                                  int64_t start, int64_t* __restrict__ wstart,
                                                  int64_t* __restrict__ wlen, int64_t* __restrict__ next_start) {
    const int lane = threadIdx.x;
    const uint64_t lt = (1ull << lane) - 1ull;
    const int64_t N = a.N;
    int64_t s = start;
    for (int64_t p = 0; p < a.P; ++p) {
        const int64_t t = a.now[p];
        const int64_t* __restrict__ th = fth + (a.flags && (a.flags[p] & 1u) ? N : 0);
        int64_t found = 0, processed = N;
        for (int64_t base = 0; base < N; base += 64 * kChU) {
            int64_t v[kChU];
#pragma unroll
            for (int u = 0; u < kChU; ++u) {
                const int64_t pos = base + u * 64 + lane;
                int64_t n = s + pos;
                if (n >= N) n -= N;
                v[u] = pos < N ? th[n] : INT64_MAX;
            }
            bool done = false;
#pragma unroll
            for (int u = 0; u < kChU; ++u) {
                const bool f = t >= v[u];
                const uint64_t m = __ballot(f);
                const int64_t c = __popcll(m);
                if (found + c >= K) {  // the K-th feasible position is in this step (wave-uniform)
                    const bool hitl = f && found + __popcll(m & lt) + 1 == K;
                    const uint64_t hm = __ballot(hitl);
                    processed = base + u * 64 + (__ffsll((unsigned long long)hm) - 1) + 1;
                    done = true;
                    break;
                }
                found += c;
            }
            if (done) break;
        }
        if (lane == 0) {
            wstart[p] = s;
            wlen[p] = processed;
        }
        s += processed;
        if (s >= N) s -= N;
    }
    if (lane == 0) *next_start = s;
}

// ---------------------------------------------------------------- k_sel_pairs
constexpr int kSelT = 256;       // threads (one node each)
constexpr int kSelChunk = 1024;  // max pods per workgroup (LDS keys)

__device__ __forceinline__ long long wave_max64(long long v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, (long long)__shfl_xor(v, o));
    return v;
}

template <int PD, int PR>
__global__ __launch_bounds__(kSelT) void k_sel_pairs(SelArgs a, int32_t chunk, int32_t nbx, int32_t per,
                                                     int32_t ncy) {
    __shared__ unsigned long long best[kSelChunk];
    const int64_t b = blockIdx.x, q = b >> 3;  // XCD x (= workgroup id % 8) takes node blocks [x*per, (x+1)*per)
    const int32_t nb = (int32_t)((b & 7) * per + q % per), cy = (int32_t)(q / per);
    if (nb >= nbx || cy >= ncy) return;  // (whole workgroup)
    const int64_t n = (int64_t)nb * kSelT + threadIdx.x;
    const bool valid = n < a.N;
    const int64_t p0 = (int64_t)cy * chunk, p1 = min(a.P, p0 + chunk);
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < chunk; i += kSelT) best[i] = 0;  // key + 1 (0: none)
    __syncthreads();
    const NodeRec<PD, PR>* __restrict__ rec = static_cast<const NodeRec<PD, PR>*>(a.rec) + (valid ? n : 0);
    const int64_t ext = valid && a.ext_score ? a.ext_score[n] : 0;
    const bool ok = valid && (!a.ext_ok || a.ext_ok[n] != 0);
    const uint32_t tb = tie_node(a.seed, a.kb, (uint32_t)(a.node_offset + n));
    // lane cache (K3m): Filter pass (non-DaemonSet) and score at the last evaluation, valid
    // on [LO, HI); a step inside the sub-chunk: values from bp on; multi: evaluate per pod
    bool f0 = false, f1 = false, stepped = false, multi = false;
    int32_t s0 = 0, s1 = 0;
    int64_t bp = INT64_MAX, LO = INT64_MAX, HI = INT64_MIN;
    for (int64_t q0 = p0; q0 < p1; q0 += 64) {
        const int nv = (int)min((int64_t)64, p1 - q0);
        const bool pv = lane < nv;
        const int64_t tn = pv ? a.now[q0 + lane] : 0;
        const int32_t fl = pv && a.flags ? (int32_t)(a.flags[q0 + lane] & 1u) : 0;
        const int64_t ws = pv && a.wstart ? a.wstart[q0 + lane] : 0;
        const int64_t wl = pv && a.wstart ? a.wlen[q0 + lane] : a.N;
        const uint32_t cp = pv ? tie_pod_key(a.seed, q0 + lane) : 0u;
        int64_t cmin = pv ? tn : INT64_MAX, cmax = pv ? tn : INT64_MIN;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            cmin = min(cmin, (int64_t)__shfl_xor((long long)cmin, o));
            cmax = max(cmax, (int64_t)__shfl_xor((long long)cmax, o));
        }
        if (ok && !(cmin >= LO && cmax < HI)) {
            const NodeRec<PD, PR> r = *rec;
            int64_t lo, hi;
            bracket<PD, PR>(r, cmin, lo, hi);
            f0 = !(cmin < r.e_fail);
            s0 = score_at<PD, PR>(cmin, r, a.wsum, a.noprio);
            LO = lo;
            HI = hi;
            stepped = hi <= cmax;
            multi = false;
            if (stepped) {
                int64_t lo2, hi2;
                bracket<PD, PR>(r, hi, lo2, hi2);
                bp = hi;
                f1 = !(hi < r.e_fail);
                s1 = score_at<PD, PR>(hi, r, a.wsum, a.noprio);
                multi = hi2 <= cmax;
            }
        }
        for (int j = 0; j < nv; ++j) {
            const int64_t t = readlane64(tn, j);
            const bool d = __builtin_amdgcn_readlane(fl, j) != 0;
            bool f = f0;
            int32_t s = s0;
            if (ok && stepped) {
                if (multi) {
                    const NodeRec<PD, PR> r = *rec;
                    f = !(t < r.e_fail);
                    s = score_at<PD, PR>(t, r, a.wsum, a.noprio);
                } else if (t >= bp) {
                    f = f1;
                    s = s1;
                }
            }
            bool in = true;
            if (a.wstart) {  // rotated position of this node in the pod's window
                int64_t rel = n - readlane64(ws, j);
                if (rel < 0) rel += a.N;
                in = rel < readlane64(wl, j);
            }
            const bool feas = ok && in && (d || f);
            if (!__ballot(feas)) continue;  // (most waves of a pod lie outside its window)
            const uint32_t lo32 = tb ^ (uint32_t)__builtin_amdgcn_readlane((int)cp, j);
            const long long key = feas ? (long long)((((int64_t)s * a.w_dyn + ext) << 32) | (int64_t)lo32) : -1;
            const long long k = wave_max64(key);
            if (lane == 0 && k >= 0) atomicMax(&best[q0 + j - p0], (unsigned long long)k + 1ull);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < (int)(p1 - p0); i += kSelT) {
        const long long k = (long long)best[i] - 1;
        if (k >= 0) atomicMax(&a.keys[p0 + i], k);
    }
}

// ---------------------------------------------------------------- k_sel_decode
__global__ __launch_bounds__(256) void k_sel_decode(SelArgs a, int64_t* __restrict__ chosen,
                                                    int64_t* __restrict__ total) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= a.P) return;
    const long long k = a.keys[p];
    if (k < 0) {
        chosen[p] = -1;
        if (total) total[p] = -1;
        return;
    }
    const uint32_t lo = (uint32_t)(uint64_t)k;
    chosen[p] = (int64_t)tie_decode(a.seed, a.kb, lo, tie_pod_key(a.seed, p));
    if (total) total[p] = (int64_t)(k >> 32);
}

// ---------------------------------------------------------------- launchers
template <int PD, int PR>
static hipError_t fth_t(const SelArgs& a, int64_t* fth, hipStream_t st) {
    return klaunch("k_sel_fth", k_sel_fth<PD, PR>, dim3((unsigned)((a.N + 255) / 256)), dim3(256), 0, st, a, fth);
}
hipError_t launch_select_fth(const SelArgs& a, int shape, int64_t* fth, hipStream_t st) {
    if (a.N <= 0) return hipSuccess;
    switch (shape) {
        case kShape4x6: return fth_t<4, 6>(a, fth, st);
        case kShape8x8: return fth_t<8, 8>(a, fth, st);
        default: return fth_t<16, 16>(a, fth, st);
    }
}

hipError_t launch_select_chain(const SelArgs& a, const int64_t* fth, int64_t K, int64_t start, int64_t* wstart,
                               int64_t* wlen, int64_t* next_start, hipStream_t st) {
    if (a.P <= 0 || a.N <= 0) return hipSuccess;
    return klaunch("k_sel_chain", k_sel_chain, dim3(1), dim3(64), 0, st, a, fth, K, start, wstart, wlen, next_start);
}

template <int PD, int PR>
static hipError_t pairs_t(const SelArgs& a, hipStream_t st) {
    const int64_t nbx = (a.N + kSelT - 1) / kSelT;
    // about 4096 waves: pods per workgroup from the pair count (multiples of 64 once large)
    const int64_t ppw = std::max<int64_t>(1, a.P * a.N / 4096);
    int64_t chunk = std::max<int64_t>(1, ppw / 64);
    if (chunk >= 64) chunk = std::min<int64_t>(kSelChunk, (chunk + 63) / 64 * 64);
    chunk = std::min(chunk, a.P);
    const int64_t ncy = (a.P + chunk - 1) / chunk, per = (nbx + 7) / 8;
    if (8 * per * ncy > 0x7FFFFFFF) return hipErrorInvalidValue;
    return klaunch("k_sel_pairs", k_sel_pairs<PD, PR>, dim3((unsigned)(8 * per * ncy)), dim3(kSelT), 0, st, a,
                   (int32_t)chunk, (int32_t)nbx, (int32_t)per, (int32_t)ncy);
}
hipError_t launch_select_pairs(int shape, const SelArgs& a, hipStream_t st) {
    if (a.P <= 0 || a.N <= 0) return hipSuccess;
    switch (shape) {
        case kShape4x6: return pairs_t<4, 6>(a, st);
        case kShape8x8: return pairs_t<8, 8>(a, st);
        default: return pairs_t<16, 16>(a, st);
    }
}

hipError_t launch_select_decode(const SelArgs& a, int64_t* chosen, int64_t* total, hipStream_t st) {
    if (a.P <= 0) return hipSuccess;
    return klaunch("k_sel_decode", k_sel_decode, dim3((unsigned)((a.P + 255) / 256)), dim3(256), 0, st, a, chosen,
                   total);
}

}  // namespace crane
