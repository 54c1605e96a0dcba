// merge.hip — config-5 sequential greedy as a merge of per-node score staircases.
//
// Sequential greedy (greedy.hip, oracle or_greedy): with one `now` for the
// batch, pod p takes the node of highest (score, -index) among its candidates
// (all nodes for a DaemonSet pod — plugins.go:41-43 — the feasible ones
// otherwise), then a Binding{Timestamp: now} on that node raises its window
// counts (binding.go:85-91), hot value Σ_w count_w / Count_w (node.go:113-121)
// and penalty int(hv*10) (plugins.go:91).  Only the chosen node's score moves.
//
// With every Count_w > 0 the hot value, hence the penalty, is non-decreasing in
// the number k of bindings a node has received in the batch, so each node's
// score s_n(k) = clamp(base_n - 10 v_n(k), 0, 100) is a non-increasing
// staircase in k.  Taking the max head of N non-increasing lists is a k-way
// merge: the non-DaemonSet pods receive, in order, the elements of
//   F = sort_desc{ (s_n(k), -n) : n feasible, k >= 0 },
// and a DaemonSet pod takes the larger of the heads of F and of the analogous
// stream I over the infeasible nodes.  Element i of I goes to the first
// DaemonSet pod m (at pod position a_m, after the one that took i-1) with
// a_m >= T_i = i + #{j : F[j] > I[i]}, i.e. m_i = i + prefix-max(g_i - i) with
// g_i = first m with a_m >= T_i.  Every other pod p takes F[p - #(I-takers
// before p)].  Results are identical to the sequential loop; the engine falls
// back to greedy.hip when the staircase premise fails (a Count_w <= 0, or a
// base score of int(NaN) whose int64 subtraction could wrap).
//
//   M1 hist   : per node, the staircase's runs (level, length) -> per-level
//               element counts of F and I (capped at the pods that can use them)
//   M2 bsum   : per 256-node block, per level >= the cut level, element counts
//   M3 scan   : exclusive scan over (level desc, block asc)
//   M4 place  : per level, block-wide scan of each node's run length -> the
//               node's positions in F (or I); writes packed keys
//   M5 assign : DaemonSet merge (a_m compaction, binary searches, prefix max,
//               I-taker marks, pod-order scan) -> chosen node per pod
#include <hip/hip_runtime.h>

#include "dyn_types.hpp"
#include "kernels.hpp"

namespace crane {

constexpr int kMT = 256;     // node-block size of M1, M2, M4
constexpr int kM5T = 1024;   // single-workgroup kernels of M5
constexpr int kLevels = 101; // scores 0..100

// x / C and x % C for x >= 0, C > 0: 32-bit unsigned division when both fit
// (always, at realistic binding counts), 64-bit otherwise
__device__ __forceinline__ void udivmod(int64_t x, int64_t C, int64_t& q, int64_t& r) {
    if (((uint64_t)x | (uint64_t)C) <= 0xFFFFFFFFull) {
        const uint32_t xq = (uint32_t)x / (uint32_t)C;
        q = xq;
        r = (int64_t)((uint32_t)x - xq * (uint32_t)C);
    } else {
        q = x / C;
        r = x - q * C;
    }
}

// Runs of a node's staircase s(k), k = 0 .. cap-1, in order (levels non-increasing).
struct RunIter {
    int64_t base, k, cap;
    uint32_t c[kMaxWin];
    __device__ bool next(const MergeArgs& a, int& lvl, int64_t& len) {
        if (k >= cap) return false;
        // hot value sum_w (c_w + k) / C_w (node.go:117) and, per window that a binding
        // enters, the bindings until its quotient grows
        int64_t v = 0, d = INT64_MAX;
#pragma unroll
        for (int w = 0; w < kMaxWin; ++w)  // static indices: c stays in registers
            if (w < a.n_win) {
                const int64_t C = a.win_count[w];
                int64_t q, rem;
                udivmod((int64_t)c[w] + (a.win_inc[w] ? k : 0), C, q, rem);
                v += q;
                if (a.win_inc[w]) d = min(d, C - rem);
            }
        const int64_t f = base - 10 * v;  // no wrap: base >= INT64_MIN + 2^40 (M1 flag)
        lvl = (int)(f < 0 ? 0 : (f > 100 ? 100 : f));
        if (lvl == 0) d = INT64_MAX;  // clamped at 0 from here on
        len = min(d, cap - k);
        k += len;
        return true;
    }
};

__device__ __forceinline__ RunIter make_iter(const int64_t* base, const uint32_t* cnt, int64_t N, int64_t n,
                                             int64_t cap, const MergeArgs& a) {
    RunIter it;
    it.base = base[n];
    it.k = 0;
    it.cap = cap;
    for (int w = 0; w < kMaxWin; ++w) it.c[w] = w < a.n_win ? cnt[(int64_t)w * N + n] : 0u;
    return it;
}

__device__ __forceinline__ int64_t pack_level_key(int u, int64_t n) {
    return ((int64_t)u << 32) | (int64_t)(0xFFFFFFFFull - (uint64_t)n);
}

// ---------------------------------------------------------------- M1
__global__ __launch_bounds__(kMT) void m1_hist(const int64_t* __restrict__ base, const uint8_t* __restrict__ leaf,
                                               const uint32_t* __restrict__ cnt, int64_t N, MergeArgs a,
                                               int64_t capF, int64_t capI, unsigned long long* __restrict__ H,
                                               int32_t* __restrict__ flag) {
    __shared__ unsigned long long lh[2 * kLevels];
    for (int i = threadIdx.x; i < 2 * kLevels; i += kMT) lh[i] = 0;
    __syncthreads();
    const int64_t n = (int64_t)blockIdx.x * kMT + threadIdx.x;
    if (n < N) {
        if (base[n] < INT64_MIN + (1LL << 40)) atomicOr(flag, 1);  // int(NaN) base: s_n(k) may rise
        const int T = (leaf[n] & 0x80) ? 0 : 1;
        RunIter it = make_iter(base, cnt, N, n, T ? capI : capF, a);
        int lvl;
        int64_t len;
        while (it.next(a, lvl, len)) atomicAdd(&lh[T * kLevels + lvl], (unsigned long long)len);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * kLevels; i += kMT)
        if (lh[i]) atomicAdd(&H[i], lh[i]);
}

// ---------------------------------------------------------------- M2
__global__ __launch_bounds__(kMT) void m2_bsum(const int64_t* __restrict__ base, const uint8_t* __restrict__ leaf,
                                               const uint32_t* __restrict__ cnt, int64_t N, MergeArgs a, int T,
                                               int vlo, int64_t cap, unsigned long long* __restrict__ bs) {
    __shared__ unsigned long long ls[kLevels];
    for (int i = threadIdx.x; i < kLevels; i += kMT) ls[i] = 0;
    __syncthreads();
    const int64_t n = (int64_t)blockIdx.x * kMT + threadIdx.x;
    if (n < N && ((leaf[n] & 0x80) ? 0 : 1) == T) {
        RunIter it = make_iter(base, cnt, N, n, cap, a);
        int lvl;
        int64_t len;
        while (it.next(a, lvl, len) && lvl >= vlo) atomicAdd(&ls[100 - lvl], (unsigned long long)len);
    }
    __syncthreads();
    const int L = 101 - vlo;
    for (int r = threadIdx.x; r < L; r += kMT) bs[(int64_t)r * gridDim.x + blockIdx.x] = ls[r];
}

// ---------------------------------------------------------------- M3 (one workgroup)
// Exclusive scan in place.  Each thread owns a contiguous run of the array and
// reads it in batches of 8 independent loads; one workgroup scan of the run sums.
__device__ __forceinline__ unsigned long long wg_excl_scan_u64(unsigned long long v, unsigned long long* part,
                                                               unsigned long long* total = nullptr) {
    // 1024 threads: wave scans, then a scan of the 16 wave totals
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    unsigned long long x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) part[w] = x;
    __syncthreads();
    if (threadIdx.x < 64) {
        unsigned long long t = threadIdx.x < kM5T / 64 ? part[threadIdx.x] : 0ull, u = t;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned long long y = __shfl_up(u, o);
            if ((int)threadIdx.x >= o) u += y;
        }
        if (threadIdx.x < kM5T / 64) part[kM5T / 64 + threadIdx.x] = u - t;
        if (threadIdx.x == kM5T / 64 - 1) part[2 * (kM5T / 64)] = u;
    }
    __syncthreads();
    if (total) *total = part[2 * (kM5T / 64)];
    const unsigned long long r = part[kM5T / 64 + w] + x - v;
    __syncthreads();  // part is reused by the next call
    return r;
}

__global__ __launch_bounds__(kM5T) void m3_scan(unsigned long long* __restrict__ v, int64_t len) {
    // tiles of 8 x 1024 values: coalesced loads into LDS, each thread scans 8
    // consecutive values, one workgroup scan per tile, coalesced stores
    constexpr int kTile = 8 * kM5T;
    __shared__ unsigned long long part[2 * (kM5T / 64) + 1];
    __shared__ unsigned long long lv[kTile];
    unsigned long long run = 0;
    for (int64_t t0 = 0; t0 < len; t0 += kTile) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t i = t0 + u * kM5T + threadIdx.x;
            lv[u * kM5T + threadIdx.x] = i < len ? v[i] : 0ull;
        }
        __syncthreads();
        unsigned long long x[8], c = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            x[u] = lv[threadIdx.x * 8 + u];
            c += x[u];
        }
        unsigned long long tot;
        unsigned long long e = run + wg_excl_scan_u64(c, part, &tot);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            lv[threadIdx.x * 8 + u] = e;
            e += x[u];
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t i = t0 + u * kM5T + threadIdx.x;
            if (i < len) v[i] = lv[u * kM5T + threadIdx.x];
        }
        run += tot;
        __syncthreads();
    }
}

// ---------------------------------------------------------------- M4
// Each node writes its runs at their positions in the stream: position of
// (level u, node n) = off[u][block] + elements of level u from lower nodes of
// the block.  Per-wave level counts go to LDS first (one barrier); then each
// wave walks only the levels it has, with a wave scan per level (no barriers).
__global__ __launch_bounds__(kMT) void m4_place(const int64_t* __restrict__ base, const uint8_t* __restrict__ leaf,
                                                const uint32_t* __restrict__ cnt, int64_t N, MergeArgs a, int T,
                                                int vlo, int64_t cap, const unsigned long long* __restrict__ off,
                                                int64_t* __restrict__ stream) {
    __shared__ unsigned long long wc[kMT / 64][kLevels];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < (kMT / 64) * kLevels; i += kMT) (&wc[0][0])[i] = 0;
    const int64_t n = (int64_t)blockIdx.x * kMT + threadIdx.x;
    const bool mine = n < N && ((leaf[n] & 0x80) ? 0 : 1) == T;
    __syncthreads();
    {
        RunIter it = make_iter(base, cnt, N, mine ? n : 0, mine ? cap : 0, a);
        int lvl;
        int64_t len;
        while (it.next(a, lvl, len) && lvl >= vlo) atomicAdd(&wc[w][lvl], (unsigned long long)len);
    }
    __syncthreads();
    RunIter it = make_iter(base, cnt, N, mine ? n : 0, mine ? cap : 0, a);
    int lvl = -1;
    int64_t len = 0;
    bool have = mine && it.next(a, lvl, len);
    for (int u = 100; u >= vlo; --u) {
        if (wc[w][u] == 0) continue;  // wave-uniform: this wave has no element at level u
        unsigned long long c = 0;
        while (have && lvl == u) {
            c += (unsigned long long)len;
            have = it.next(a, lvl, len);
        }
        unsigned long long x = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned long long y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (c) {
            unsigned long long p0 = off[(int64_t)(100 - u) * gridDim.x + blockIdx.x] + x - c;
            for (int i = 0; i < w; ++i) p0 += wc[i][u];
            const unsigned long long p1 = min(p0 + c, (unsigned long long)cap);
            for (unsigned long long p = p0; p < p1; ++p) stream[p] = pack_level_key(u, n);
        }
    }
}

// ---------------------------------------------------------------- M5
// M5a: positions a[m] of the DaemonSet pods (pod order).  One workgroup: the
// flags go to LDS with coalesced loads (in tiles of kM5Tile pods), then each
// thread takes a contiguous run of the tile, one workgroup scan per tile.
constexpr int kM5Tile = 96 * 1024;

__global__ __launch_bounds__(kM5T) void m5a_compact(const uint8_t* __restrict__ flags, int64_t P,
                                                    int32_t* __restrict__ apos) {
    __shared__ unsigned long long part[2 * (kM5T / 64) + 1];
    __shared__ uint8_t lf[kM5Tile];
    int64_t run = 0;
    for (int64_t t0 = 0; t0 < P; t0 += kM5Tile) {
        const int32_t nt = (int32_t)min((int64_t)kM5Tile, P - t0);
#pragma unroll 8
        for (int32_t i = threadIdx.x; i < nt; i += kM5T) lf[i] = flags[t0 + i] & 1u;
        __syncthreads();
        const int32_t per = (nt + kM5T - 1) / kM5T;
        const int32_t lo = min(nt, (int32_t)threadIdx.x * per), hi = min(nt, lo + per);
        unsigned long long c = 0;
        for (int32_t i = lo; i < hi; ++i) c += lf[i];
        unsigned long long tot;
        int64_t pos = run + (int64_t)wg_excl_scan_u64(c, part, &tot);
        for (int32_t i = lo; i < hi; ++i)
            if (lf[i]) apos[pos++] = (int32_t)(t0 + i);
        run += (int64_t)tot;
        __syncthreads();  // lf is rewritten by the next tile
    }
}

// M5b: per I element i, g_i - i where g_i = first DaemonSet pod m with a_m >= T_i
__global__ __launch_bounds__(kMT) void m5b_thresholds(const int64_t* __restrict__ Fs, int64_t nF,
                                                      const int64_t* __restrict__ Is, int64_t nI,
                                                      const int32_t* __restrict__ apos, int64_t Pd,
                                                      int64_t* __restrict__ gi) {
    const int64_t i = (int64_t)blockIdx.x * kMT + threadIdx.x;
    if (i >= nI) return;
    const int64_t key = Is[i];
    int64_t lo = 0, hi = nF;  // first j with Fs[j] < key (Fs descending)
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (Fs[mid] < key) hi = mid;
        else lo = mid + 1;
    }
    const int64_t T = i + lo;
    int64_t l2 = 0, h2 = Pd;  // first m with apos[m] >= T
    while (l2 < h2) {
        const int64_t mid = (l2 + h2) >> 1;
        if ((int64_t)apos[mid] >= T) h2 = mid;
        else l2 = mid + 1;
    }
    gi[i] = l2 - i;
}

// M5c: m_i = i + prefix-max(g_i - i), strictly increasing in i; the I-takers
// are i = 0 .. K-1 (m_i < Pd), at pods q_i = a_{m_i}, increasing (one workgroup)
__global__ __launch_bounds__(kM5T) void m5c_takers(const int64_t* __restrict__ gi, int64_t nI,
                                                   const int32_t* __restrict__ apos, int64_t Pd,
                                                   int32_t* __restrict__ q, int64_t* __restrict__ K) {
    __shared__ int64_t part[kM5T];
    __shared__ unsigned long long kmax;
    if (threadIdx.x == 0) kmax = 0;
    const int64_t per = (nI + kM5T - 1) / kM5T;
    const int64_t lo = min(nI, (int64_t)threadIdx.x * per), hi = min(nI, lo + per);
    int64_t s = INT64_MIN;
    for (int64_t i = lo; i < hi; ++i) s = max(s, gi[i]);
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < kM5T; off <<= 1) {
        const int64_t y = threadIdx.x >= off ? part[threadIdx.x - off] : INT64_MIN;
        __syncthreads();
        part[threadIdx.x] = max(part[threadIdx.x], y);
        __syncthreads();
    }
    int64_t run = threadIdx.x ? part[threadIdx.x - 1] : INT64_MIN;
    for (int64_t i = lo; i < hi; ++i) {
        run = max(run, gi[i]);
        const int64_t m = i + run;
        if (m < Pd) {
            q[i] = apos[m];
            atomicMax(&kmax, (unsigned long long)(i + 1));
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) *K = (int64_t)kmax;
}

// M5d: chosen node per pod, all pods in parallel.  Pod p is I-taker i iff
// q_i = p; otherwise it takes F[p - #(I-takers before p)].
__global__ __launch_bounds__(kMT) void m5d_assign(const int64_t* __restrict__ Fs, int64_t nF,
                                                  const int64_t* __restrict__ Is, const int32_t* __restrict__ q,
                                                  const int64_t* __restrict__ Kp, int64_t P,
                                                  int64_t* __restrict__ chosen) {
    const int64_t p = (int64_t)blockIdx.x * kMT + threadIdx.x;
    if (p >= P) return;
    const int64_t K = *Kp;
    int64_t lo = 0, hi = K;  // first i with q_i >= p
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (q[mid] < p) lo = mid + 1;
        else hi = mid;
    }
    int64_t key = -1;
    if (lo < K && q[lo] == p) key = Is[lo];
    else if (p - lo < nF) key = Fs[p - lo];
    chosen[p] = key < 0 ? -1 : (int64_t)(0xFFFFFFFFull - ((uint64_t)key & 0xFFFFFFFFull));
}

// no DaemonSet pods: pod p takes F[p]
__global__ __launch_bounds__(kMT) void m5z_direct(const int64_t* __restrict__ Fs, int64_t nF, int64_t P,
                                                  int64_t* __restrict__ chosen) {
    const int64_t p = (int64_t)blockIdx.x * kMT + threadIdx.x;
    if (p >= P) return;
    chosen[p] = p < nF ? (int64_t)(0xFFFFFFFFull - ((uint64_t)Fs[p] & 0xFFFFFFFFull)) : -1;
}

// ---------------------------------------------------------------- launchers
hipError_t launch_merge_hist(const int64_t* base, const uint8_t* leaf, const uint32_t* cnt, int64_t N,
                             const MergeArgs& a, int64_t capF, int64_t capI, unsigned long long* H, int32_t* flag,
                             hipStream_t st) {
    hipError_t e = hipMemsetAsync(H, 0, sizeof(unsigned long long) * 2 * kLevels, st);
    if (e == hipSuccess) e = hipMemsetAsync(flag, 0, sizeof(int32_t), st);
    if (e != hipSuccess) return e;
    if (N <= 0) return hipSuccess;
    return klaunch("m1_hist", m1_hist, dim3((unsigned)((N + kMT - 1) / kMT)), dim3(kMT), 0, st, base, leaf, cnt, N, a,
                   capF, capI, H, flag);
}

int64_t merge_bsum_len(int64_t N, int vlo) { return (int64_t)(101 - vlo) * ((N + kMT - 1) / kMT); }

hipError_t launch_merge_stream(const int64_t* base, const uint8_t* leaf, const uint32_t* cnt, int64_t N,
                               const MergeArgs& a, int T, int vlo, int64_t cap, unsigned long long* bs,
                               int64_t* stream, hipStream_t st) {
    if (N <= 0 || cap <= 0) return hipSuccess;
    const unsigned nb = (unsigned)((N + kMT - 1) / kMT);
    hipError_t e = klaunch("m2_bsum", m2_bsum, dim3(nb), dim3(kMT), 0, st, base, leaf, cnt, N, a, T, vlo, cap, bs);
    if (e == hipSuccess) e = klaunch("m3_scan", m3_scan, dim3(1), dim3(kM5T), 0, st, bs, merge_bsum_len(N, vlo));
    if (e == hipSuccess)
        e = klaunch("m4_place", m4_place, dim3(nb), dim3(kMT), 0, st, base, leaf, cnt, N, a, T, vlo, cap,
                    (const unsigned long long*)bs, stream);
    return e;
}

hipError_t launch_merge_assign(const int64_t* Fs, int64_t nF, const int64_t* Is, int64_t nI, const uint8_t* flags,
                               int64_t P, int64_t Pd, int32_t* apos, int32_t* q, int64_t* gi, int64_t* chosen,
                               hipStream_t st) {
    if (P <= 0) return hipSuccess;
    const unsigned pb = (unsigned)((P + kMT - 1) / kMT);
    if (Pd == 0 || nI == 0) {  // no DaemonSet pod can take an infeasible node: pod p takes F[p]
        return klaunch("m5z_direct", m5z_direct, dim3(pb), dim3(kMT), 0, st, Fs, nF, P, chosen);
    }
    int64_t* K = gi + nI;  // scratch: gi [nI] then K
    hipError_t e = klaunch("m5a_compact", m5a_compact, dim3(1), dim3(kM5T), 0, st, flags, P, apos);
    if (e == hipSuccess)
        e = klaunch("m5b_thresholds", m5b_thresholds, dim3((unsigned)((nI + kMT - 1) / kMT)), dim3(kMT), 0, st, Fs, nF,
                    Is, nI, (const int32_t*)apos, Pd, gi);
    if (e == hipSuccess)
        e = klaunch("m5c_takers", m5c_takers, dim3(1), dim3(kM5T), 0, st, (const int64_t*)gi, nI,
                    (const int32_t*)apos, Pd, q, K);
    if (e == hipSuccess)
        e = klaunch("m5d_assign", m5d_assign, dim3(pb), dim3(kMT), 0, st, Fs, nF, Is, (const int32_t*)q,
                    (const int64_t*)K, P, chosen);
    return e;
}

}  // namespace crane
