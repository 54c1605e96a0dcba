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
// (one wave streams the rotated positions once for the whole queue: the next
// pod's window starts where the last one ended; ballots + a scalar scan over
// chunk counts find each pod's numNodesToFind-th feasible node); k_sel_pairs (per (pod, node): feasible, in the
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
// A non-DaemonSet pod passes every filter at node n iff now >= fth[n]; a DaemonSet
// pod (Dynamic bypassed) iff fth[n] != INT64_MAX (the other plugins pass).  Expiries
// stay below INT64_MAX / 2 + a period (timestamps saturate at INT64_MAX / 2,
// annotations.cpp), the clamp only makes the encoding unambiguous.
template <int PD, int PR>
__global__ __launch_bounds__(256) void k_sel_fth(SelArgs a, int64_t* __restrict__ fth) {
    const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (n >= a.N) return;
    const bool ok = !a.ext_ok || a.ext_ok[n];
    fth[n] = ok ? min(static_cast<const NodeRec<PD, PR>*>(a.rec)[n].e_fail, INT64_MAX - 1) : INT64_MAX;
}

// ---------------------------------------------------------------- k_sel_chain
// Pod p's window is the rotated positions from its start up to its K-th feasible
// node (at most N positions), and pod p + 1 starts right after it, so the whole
// queue is one sequential sweep over the stream of rotated positions x = 0, 1, ...
// (node (start + x) mod N), read once.  One workgroup takes the stream in rounds of
// kChR positions (the next round's loads in flight): every thread ballots its
// positions for the next kChQ pods at once (each against its own time), the masks
// go to LDS, and wave 0 resolves the pods in order from the masks alone (each
// pod's count from its window start, a wave prefix over the round's chunks, the
// K-th set bit); a round holding more than kChQ pod ends repeats the ballots for
// the next ones.
// kChQ pods' masks per ballot pass: at the config-3 queue (windows of ~5300 positions,
// 8192 a round) 2 takes 36.2 ms, 4 49.5 ms, 1 38.3 ms (same-box A/B, tools/gpu_select_ab.sh)
constexpr int kChT = 1024, kChU = 8, kChW = kChT / 64, kChQ = 2;

// position of the r-th set bit (r >= 1) of m: halving popcount search
__device__ __forceinline__ int nth_set_bit(unsigned long long m, int r) {
    int pos = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const int c = __popcll(m & ((1ull << w) - 1ull));
        if (c < r) {
            r -= c;
            m >>= w;
            pos += w;
        }
    }
    return pos;
}
constexpr int kChC = kChU * kChW;         // 64-position chunks per round (chunk c = u * kChW + wave)
constexpr int64_t kChR = 64LL * kChC;     // positions per round
static_assert(kChC == 128, "wave 0 resolves a round's chunks two per lane");
constexpr int kChPB = 1024;               // pod times cached per block

__global__ __launch_bounds__(kChT) void k_sel_chain(SelArgs a, const int64_t* __restrict__ fth, int64_t K,
                                                    int64_t start, int64_t* __restrict__ wstart,
                                                    int64_t* __restrict__ wlen, int64_t* __restrict__ next_start,
                                                    const int32_t* __restrict__ skip) {
    if (skip && *skip) return;  // k_sel_chain_rs placed the windows
    __shared__ unsigned long long msk[kChQ][kChC];
    __shared__ int64_t ptime[kChPB];
    __shared__ int8_t pds[kChPB];
    __shared__ int64_t st_p, st_pstart, st_found;
    __shared__ int32_t st_more;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t N = a.N, P = a.P;
    auto load = [&](int64_t* v, int64_t nb) {  // nb: node of the round's first position
#pragma unroll
        for (int u = 0; u < kChU; ++u) {
            int64_t n = nb + u * kChT + threadIdx.x;
            n = n < N ? n : (n - N < N ? n - N : n % N);
            v[u] = fth[n];
        }
    };
    int64_t p = 0, pstart = 0, found = 0, pb0 = -1;
    int64_t cur[kChU], nxt[kChU];
    int64_t x0 = 0, nb = start;
    load(cur, nb);
    while (p < P) {
        int64_t nb2 = nb + kChR;
        nb2 = nb2 < N ? nb2 : nb2 % N;
        load(nxt, nb2);  // the next round, in flight while this one is resolved
        bool more = true;
        while (more && p < P) {
            if (pb0 < 0 || p + kChQ > pb0 + kChPB) {  // pod times cached for [pb0, pb0 + kChPB)
                __syncthreads();
                pb0 = p;
                if (threadIdx.x < kChPB) {
                    const int64_t q = pb0 + threadIdx.x;
                    ptime[threadIdx.x] = q < P ? a.now[q] : 0;
                    pds[threadIdx.x] = q < P && a.flags ? (int8_t)(a.flags[q] & 1u) : 0;
                }
                __syncthreads();
            }
            // masks of the round's positions for pods p .. p + kChQ - 1 (positions before the
            // current pod's start are excluded; each pod's own start is applied by wave 0)
#pragma unroll
            for (int q = 0; q < kChQ; ++q) {
                const int64_t t = ptime[p - pb0 + q];
                const bool d = pds[p - pb0 + q] != 0;
#pragma unroll
                for (int u = 0; u < kChU; ++u) {
                    const int64_t pos = x0 + u * kChT + threadIdx.x;
                    const bool f = pos >= pstart && (d ? cur[u] != INT64_MAX : t >= cur[u]);
                    const unsigned long long m = __ballot(f);
                    if (lane == 0) msk[q][u * kChW + w] = m;
                }
            }
            __syncthreads();
            if (w == 0) {
                // lane L covers chunks 2L, 2L + 1 (positions x0 + 64 c .. + 63)
                int64_t ps = pstart, fnd = found, pp = p;
                bool cont = true;  // the last resolved pod ended inside this round
                for (int q = 0; q < kChQ && pp < P && cont; ++q) {
                    const int64_t lim = ps + N;  // window: positions [ps, lim)
                    int32_t cnt2[2];
                    unsigned long long mm[2];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int c = 2 * lane + h;
                        const int64_t c0 = x0 + 64LL * c;
                        unsigned long long m = msk[q][c];
                        // keep bits of positions in [ps, lim)
                        if (c0 + 64 <= ps || c0 >= lim) m = 0;
                        else {
                            if (c0 < ps) m &= ~0ull << (ps - c0);
                            if (c0 + 64 > lim) m &= (lim - c0 >= 64) ? ~0ull : ((1ull << (lim - c0)) - 1ull);
                        }
                        mm[h] = m;
                        cnt2[h] = __popcll(m);
                    }
                    // inclusive prefix over the lanes (DPP, no LDS round trips)
                    const int32_t x = (int32_t)wave_scan_add((uint32_t)(cnt2[0] + cnt2[1]));
                    const int64_t need = K - fnd;
                    const int32_t before = x - cnt2[0] - cnt2[1];  // feasible in earlier chunks
                    // the lane whose chunks hold the need-th feasible position
                    const bool mine = before < need && x >= need;
                    const unsigned long long hb = __ballot(mine);
                    int64_t end = -1;
                    if (hb) {
                        const int L = __ffsll(hb) - 1;
                        if (lane == L) {
                            int64_t r = need - before;  // rank within this lane's chunks
                            int h = cnt2[0] >= r ? 0 : 1;
                            if (h) r -= cnt2[0];
                            end = x0 + 64LL * (2 * lane + h) + nth_set_bit(mm[h], (int)r);
                        }
                        end = readlane64(end, L);
                    } else if (lim <= x0 + kChR) {
                        end = lim - 1;  // fewer than K feasible among the window's N positions
                    }
                    if (end >= 0) {
                        if (lane == 0) {
                            int64_t s0 = start + ps % N;
                            wstart[pp] = s0 >= N ? s0 - N : s0;
                            wlen[pp] = end - ps + 1;
                        }
                        ++pp;
                        ps = end + 1;
                        fnd = 0;
                    } else {
                        fnd += __builtin_amdgcn_readlane(x, 63);
                        cont = false;
                    }
                }
                if (lane == 0) {
                    st_p = pp;
                    st_pstart = ps;
                    st_found = fnd;
                    st_more = cont && pp < P && ps < x0 + kChR;  // another pod starts in this round
                }
            }
            __syncthreads();
            p = st_p;
            pstart = st_pstart;
            found = st_found;
            more = st_more != 0;
        }
#pragma unroll
        for (int u = 0; u < kChU; ++u) cur[u] = nxt[u];
        x0 += kChR;
        nb = nb2;
    }
    if (threadIdx.x == 0) {
        int64_t s0 = start + pstart % N;
        *next_start = s0 >= N ? s0 - N : s0;
    }
}

// ---------------------------------------------------------------- k_sel_chain_rs
// The same windows without streaming the rotation: for the pods of the queue (times in
// [tmin, tmax] for the non-DaemonSet ones) a node is
//   A  feasible for every non-DaemonSet pod      (fth <= tmin),
//   I  feasible from some time inside the queue  (tmin < fth <= tmax),
//   -  feasible for no non-DaemonSet pod         (fth > tmax),
//   D  feasible for a DaemonSet pod              (fth != INT64_MAX).
// The workgroup builds bit masks of A, I and D per 64-node word with prefix ranks and
// select samples (every 64th set bit's word) in LDS, plus the I nodes as a sorted list
// (node, fth).  Then one wave walks the queue: a pod's window ends at its K-th feasible
// node from its start s, i.e. at the A node of rank rank_A(s) + K - 1 unless I nodes with
// fth <= now lie before it; those candidates (the I list from rank_I(s), a few per
// window) are ranked among the A nodes (merged rank = A nodes before it + candidates
// before it), and the end is the candidate of merged rank K - 1 or else the A node of
// rank rank_A(s) + K - 1 - (candidates before it).  About ten dependent LDS round trips
// per pod instead of a stream over its ~N/20 positions.  Each I node's A rank is kept
// with the list, so a candidate chunk costs one LDS round trip (list entries), not two.
// Positions are unrolled: a window [s, s + N) wraps past node N - 1 to node 0.
// Applies while the LDS holds it (N <= 64 * kRsMaxW, |I| <= kRsIMax); else it flags the
// streaming kernel (k_sel_chain, launched behind it) to run.
constexpr int kRsT = 1024;
constexpr int kRsMaxW = 2048;  // 64-node words: N <= 131,072
constexpr int kRsIMax = 4096;  // in-range nodes

__host__ __device__ inline size_t rs_lds_bytes(int64_t W) {
    const size_t Wp = (size_t)W + 1;
    return 8 * (3 * Wp + kRsIMax) + 4 * (5 * Wp + 2 * kRsIMax);
}

struct RsView {
    const uint64_t *mA, *mI, *mD;
    const uint32_t *bA, *bI, *bD, *sA, *sD;
    int32_t W;
};

__device__ __forceinline__ int64_t rs_rank(const uint64_t* m, const uint32_t* b, int64_t n) {
    const int64_t w = n >> 6;
    const int k = (int)(n & 63);
    return (int64_t)b[w] + __popcll(m[w] & ((1ull << k) - 1ull));
}

// node of the r-th (0-based) set bit; whole wave, uniform r < total; *word = its mask word
__device__ __forceinline__ int64_t rs_select(const uint64_t* m, const uint32_t* b, const uint32_t* smp, int32_t W,
                                             int64_t r, uint64_t* word = nullptr) {
    const int lane = threadIdx.x & 63;
    int64_t w = smp[r >> 6];  // the word holding rank 64 * (r / 64) (r's word is at or after it)
    for (;;) {
        const int64_t wl = min(w + lane + 1, (int64_t)W);
        const uint64_t hb = __ballot((int64_t)b[wl] > r);
        if (hb) {
            const int64_t ww = w + __ffsll((long long)hb) - 1;
            const uint64_t mw = m[ww];
            if (word) *word = mw;
            return ww * 64 + nth_set_bit(mw, (int)(r - (int64_t)b[ww]) + 1);
        }
        w += 64;
    }
}

// the same for one lane's own rank r < total: the sample words bracket r's word, a binary
// search over the prefix ranks finds it
__device__ __forceinline__ int64_t rs_select_lane(const uint64_t* m, const uint32_t* b, const uint32_t* smp,
                                                  int32_t W, int64_t total, int64_t r) {
    const int64_t k = r >> 6;
    int32_t lo = (int32_t)smp[k];
    int32_t hi = (k + 1) * 64 < total ? (int32_t)smp[k + 1] : W - 1;
    while (lo < hi) {  // the last word with prefix rank <= r
        const int32_t mid = (lo + hi + 1) >> 1;
        if ((int64_t)b[mid] <= r) lo = mid;
        else hi = mid - 1;
    }
    return (int64_t)lo * 64 + nth_set_bit(m[lo], (int)(r - (int64_t)b[lo]) + 1);
}

__global__ __launch_bounds__(kRsT) void k_sel_chain_rs(SelArgs a, const int64_t* __restrict__ fth, int64_t K,
                                                       int64_t start, int64_t* __restrict__ wstart,
                                                       int64_t* __restrict__ wlen, int64_t* __restrict__ next_start,
                                                       int32_t* __restrict__ done) {
    extern __shared__ __attribute__((aligned(16))) uint64_t rs[];
    __shared__ int64_t red[2][kRsT / 64];
    __shared__ uint32_t part[kRsT];
    const int64_t N = a.N, P = a.P;
    const int32_t W = (int32_t)((N + 63) >> 6);
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t Wp = W + 1;
    uint64_t* mA = rs;
    uint64_t* mI = mA + Wp;
    uint64_t* mD = mI + Wp;
    int64_t* iFth = reinterpret_cast<int64_t*>(mD + Wp);
    uint32_t* bA = reinterpret_cast<uint32_t*>(iFth + kRsIMax);
    uint32_t* bI = bA + Wp;
    uint32_t* bD = bI + Wp;
    uint32_t* sA = bD + Wp;
    uint32_t* sD = sA + Wp;
    uint32_t* iPos = sD + Wp;
    uint32_t* iRA = iPos + kRsIMax;  // an in-range node's rank among the A nodes (A nodes before it)
    // the non-DaemonSet pods' time range
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    for (int64_t p = threadIdx.x; p < P; p += kRsT) {
        if (a.flags && (a.flags[p] & 1u)) continue;
        const int64_t t = a.now[p];
        lo = min(lo, t);
        hi = max(hi, t);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        lo = min(lo, (int64_t)__shfl_xor((long long)lo, o));
        hi = max(hi, (int64_t)__shfl_xor((long long)hi, o));
    }
    if (lane == 0) {
        red[0][wv] = lo;
        red[1][wv] = hi;
    }
    __syncthreads();
    int64_t tmin = INT64_MAX, tmax = INT64_MIN;
#pragma unroll
    for (int i = 0; i < kRsT / 64; ++i) {
        tmin = min(tmin, red[0][i]);
        tmax = max(tmax, red[1][i]);
    }
    for (int32_t w = wv; w < Wp; w += kRsT / 64) {
        const int64_t n = (int64_t)w * 64 + lane;
        const bool v = n < N;
        const int64_t f = fth[min(n, N - 1)];
        const uint64_t ma = __ballot(v && f <= tmin);
        const uint64_t mi = __ballot(v && f > tmin && f <= tmax);
        const uint64_t md = __ballot(v && f != INT64_MAX);
        if (lane == 0) {
            mA[w] = ma;
            mI[w] = mi;
            mD[w] = md;
        }
    }
    __syncthreads();
    // exclusive prefix ranks over the words (W + 1 entries: the last is the total)
    {
        const int per = (int)((Wp + kRsT - 1) / kRsT);
        const int w0 = min((int)Wp, (int)threadIdx.x * per), w1 = min((int)Wp, w0 + per);
        uint64_t* ms[3] = {mA, mI, mD};
        uint32_t* bs[3] = {bA, bI, bD};
        for (int x = 0; x < 3; ++x) {
            uint32_t sum = 0;
            for (int w = w0; w < w1; ++w) sum += __popcll(ms[x][w]);
            uint32_t run = wg_excl_scan_u32<kRsT>(sum, part);
            for (int w = w0; w < w1; ++w) {
                bs[x][w] = run;
                run += __popcll(ms[x][w]);
            }
            __syncthreads();
        }
    }
    const int64_t TA = bA[W], TI = bI[W], TD = bD[W];
    if (TI > kRsIMax) {  // more in-range nodes than the list holds: the streaming kernel runs
        if (threadIdx.x == 0) *done = 0;
        return;
    }
    // the in-range list and the select samples
    for (int32_t w = threadIdx.x; w < W; w += kRsT) {
        uint64_t m = mI[w];
        uint32_t b = bI[w];
        while (m) {
            const int j = __ffsll((long long)m) - 1;
            m &= m - 1;
            const int64_t n = (int64_t)w * 64 + j;
            iPos[b] = (uint32_t)n;
            iFth[b] = fth[n];
            iRA[b] = (uint32_t)rs_rank(mA, bA, n);
            ++b;
        }
        for (uint32_t k = (bA[w] + 63) >> 6; (k << 6) < bA[w + 1]; ++k) sA[k] = (uint32_t)w;
        for (uint32_t k = (bD[w] + 63) >> 6; (k << 6) < bD[w + 1]; ++k) sD[k] = (uint32_t)w;
    }
    __syncthreads();
    if (TA < K) {  // fewer nodes feasible for every pod than a window holds: position walk
        if (wv != 0) return;  // one wave walks the queue
        const uint64_t lt = (1ull << lane) - 1ull;
        int64_t s = start;
        for (int64_t p0 = 0; p0 < P; p0 += 64) {
            const int nv = (int)min((int64_t)64, P - p0);
            const int64_t tn = a.now[p0 + min(lane, nv - 1)];
            const int32_t dn = a.flags ? (int32_t)(a.flags[p0 + min(lane, nv - 1)] & 1u) : 0;
            int64_t my_ws = 0, my_wl = 0;
            for (int j = 0; j < nv; ++j) {
                const int64_t t = readlane64(tn, j);
                const bool d = __builtin_amdgcn_readlane(dn, j) != 0;
                int64_t end;  // unrolled position of the window's last node, in [s, s + N)
                if (d) {
                    if (TD < K) {
                        end = s + N - 1;
                    } else {
                        const int64_t r = rs_rank(mD, bD, s) + K - 1;
                        end = r < TD ? rs_select(mD, bD, sD, W, r) : N + rs_select(mD, bD, sD, W, r - TD);
                    }
                } else {
                    const int64_t rA0 = rs_rank(mA, bA, s), rI0 = rs_rank(mI, bI, s);
                    bool full = false;  // fewer than K feasible nodes in the whole rotation
                    if (TA < K) {
                        int64_t cnt = 0;
                        for (int64_t q0 = 0; q0 < TI; q0 += 64) {
                            const int64_t q = q0 + lane;
                            cnt += __popcll(__ballot(q < TI && iFth[min(q, TI - 1)] <= t));
                        }
                        full = TA + cnt < K;
                    }
                    if (full) {
                        end = s + N - 1;
                    } else {
                        const int64_t rT = rA0 + K - 1;
                        uint64_t wA = 0;  // the mask word holding xA (TA >= K)
                        const int64_t xA = TA < K ? s + N - 1
                                                  : (rT < TA ? rs_select(mA, bA, sA, W, rT, &wA)
                                                             : N + rs_select(mA, bA, sA, W, rT - TA, &wA));
                        // candidates: I nodes in [s, xA] with fth <= t, in position order
                        int64_t c_lt = 0, cbase = 0, hitpos = -1;
                        for (int64_t q0 = 0; q0 < TI; q0 += 64) {
                            const int64_t q = q0 + lane;
                            int64_t idx = rI0 + q;
                            const bool wrap = idx >= TI;
                            idx -= wrap ? TI : 0;
                            const int64_t ic = min(idx, TI - 1);
                            const int64_t y = (int64_t)iPos[ic] + (wrap ? N : 0);
                            const bool inr = q < TI && y <= xA;
                            const uint64_t rm = __ballot(inr);
                            if (!rm) break;
                            const bool cand = inr && iFth[ic] <= t;
                            const uint64_t cm = __ballot(cand);
                            const int64_t ra = (int64_t)iRA[ic] + (wrap ? TA : 0);  // (built with the list)
                            const int64_t mr = ra - rA0 + cbase + __popcll(cm & lt);
                            c_lt += __popcll(__ballot(cand && mr < K - 1));
                            const uint64_t eq = __ballot(cand && mr == K - 1);
                            if (eq) {
                                hitpos = readlane64(y, __ffsll((long long)eq) - 1);
                                break;
                            }
                            cbase += __popcll(cm);
                            if (rm != ~0ull) break;  // the window's last in-range node was in this chunk
                        }
                        if (hitpos >= 0) {
                            end = hitpos;
                        } else if (TA >= K && c_lt == 0) {
                            end = xA;
                        } else {
                            // the A node c_lt before xA: inside xA's word when it holds that many below it
                            const int xb = (int)((xA >= N ? xA - N : xA) & 63);  // xA's bit in its word
                            const int below = TA >= K ? __popcll(wA & ((1ull << xb) - 1ull)) : -1;
                            if (c_lt <= below) {
                                end = xA - xb + nth_set_bit(wA, below - (int)c_lt + 1);
                            } else {
                                const int64_t r = rA0 + K - 1 - c_lt;
                                end = r < TA ? rs_select(mA, bA, sA, W, r) : N + rs_select(mA, bA, sA, W, r - TA);
                            }
                        }
                    }
                }
                if (lane == j) {
                    my_ws = s;
                    my_wl = end - s + 1;
                }
                s = end + 1 >= N ? end + 1 - N : end + 1;
                s = s >= N ? s - N : s;
            }
            if (lane < nv) {
                wstart[p0 + lane] = my_ws;
                wlen[p0 + lane] = my_wl;
            }
        }
        if (lane == 0) {
            *next_start = s;
            *done = 1;
        }
        return;
    }
    // Rank-space walk (TA >= K): the chain carries (rA, rI) = the A and I nodes before the
    // pod's start, unrolled over rotations, instead of the start position.  A window that
    // ends at an A node of rank e leaves (e + 1, the I nodes before that A node); one that
    // ends at a candidate I node leaves (its A rank, its I index + 1) — no select and no
    // rank lookup on the chain, about three dependent LDS round trips per pod.  Each pod's
    // end goes out as a descriptor (A rank / I index / position, 2 tag bits) in wlen, and
    // every wave turns the descriptors into windows afterwards.  DaemonSet pods walk the
    // D nodes by position as before (their start from the previous descriptor).
    __shared__ int64_t carry;
    if (wv == 0) {
        const uint64_t lt = (1ull << lane) - 1ull;
        auto endpos = [&](int64_t dsc) -> int64_t {  // whole wave, uniform dsc
            const int64_t v = dsc >> 2;
            if ((dsc & 3) == 0) return rs_select(mA, bA, sA, W, v >= TA ? v - TA : v);
            if ((dsc & 3) == 1) return (int64_t)iPos[v >= TI ? v - TI : v];
            return v;
        };
        int64_t s = start;  // the start position, while spos
        bool spos = true;
        const int32_t TA32 = (int32_t)TA, TI32 = (int32_t)TI, K32 = (int32_t)K;
        int32_t rA = (int32_t)rs_rank(mA, bA, start), rI = (int32_t)rs_rank(mI, bI, start);
        int64_t dsc = 0;
        for (int64_t p0 = 0; p0 < P; p0 += 64) {
            const int nv = (int)min((int64_t)64, P - p0);
            const int64_t tn = a.now[p0 + min(lane, nv - 1)];
            const int32_t dn = a.flags ? (int32_t)(a.flags[p0 + min(lane, nv - 1)] & 1u) : 0;
            int64_t my_d = 0;
            for (int j = 0; j < nv; ++j) {
                const int64_t t = readlane64(tn, j);
                const bool d = __builtin_amdgcn_readlane(dn, j) != 0;
                if (d) {
                    if (!spos) {
                        const int64_t e = endpos(dsc);
                        s = e + 1 >= N ? e + 1 - N : e + 1;
                    }
                    int64_t end;
                    if (TD < K) {
                        end = s + N - 1;
                    } else {
                        const int64_t r = rs_rank(mD, bD, s) + K - 1;
                        end = r < TD ? rs_select(mD, bD, sD, W, r) : N + rs_select(mD, bD, sD, W, r - TD);
                    }
                    const int64_t en = end >= N ? end - N : end;
                    dsc = en * 4 + 2;
                    s = en + 1 >= N ? en + 1 - N : en + 1;
                    spos = true;
                    rA = (int32_t)rs_rank(mA, bA, s);
                    rI = (int32_t)rs_rank(mI, bI, s);
                } else {
                    // (32-bit ranks and indices: N <= 131,072, so unrolled ranks stay below 2^19)
                    const int32_t rT = rA + K32 - 1;  // the A-only window's last A node (unrolled rank)
                    // candidates: I nodes from index rI before A node rT (A rank <= rT) with fth <= t
                    int32_t c_lt = 0, cbase = 0, nin = 0, hit = -1, hra = 0, ra0 = 0;
                    bool one = true;  // the scan stopped in its first chunk (ra0 holds its A ranks)
                    for (int32_t q0 = 0; q0 < TI32; q0 += 64) {
                        const int32_t q = q0 + lane, h = rI + q;
                        const bool wrap = h >= TI32;
                        const int32_t ic = min(h - (wrap ? TI32 : 0), TI32 - 1);
                        const int32_t ra = (int32_t)iRA[ic] + (wrap ? TA32 : 0);
                        if (q0 == 0) ra0 = ra;
                        const bool inr = q < TI32 && ra <= rT;
                        const uint64_t rm = __ballot(inr);
                        if (!rm) break;
                        const bool cand = inr && iFth[ic] <= t;
                        const uint64_t cm = __ballot(cand);
                        const int32_t mr = ra - rA + cbase + __popcll(cm & lt);  // merged rank in the window
                        c_lt += __popcll(__ballot(cand && mr < K32 - 1));
                        const uint64_t eq = __ballot(cand && mr == K32 - 1);
                        if (eq) {
                            const int l = __ffsll((long long)eq) - 1;
                            hit = rI + q0 + l;
                            hra = __builtin_amdgcn_readlane(ra, l);
                            break;
                        }
                        cbase += __popcll(cm);
                        nin += __popcll(rm);
                        if (rm != ~0ull) break;  // the window's last in-range node was in this chunk
                        one = false;
                    }
                    if (hit >= 0) {  // the K-th feasible node is a candidate
                        dsc = (int64_t)hit * 4 + 1;
                        rA = hra;
                        rI = hit + 1;
                    } else {  // an A node: c_lt candidates took the places of the last A nodes
                        const int32_t e = rT - c_lt;
                        dsc = (int64_t)e * 4;
                        rA = e + 1;
                        if (c_lt == 0) {
                            rI += nin;
                        } else if (one) {  // the I nodes before A node e: a prefix of the first chunk
                            rI += __popcll(__ballot(lane < TI32 && ra0 <= e));
                        } else {  // ... or of the chunks from rI
                            int32_t cnt = 0;
                            for (int32_t q0 = 0; q0 < TI32; q0 += 64) {
                                const int32_t q = q0 + lane, h = rI + q;
                                const bool wrap = h >= TI32;
                                const int32_t ic = min(h - (wrap ? TI32 : 0), TI32 - 1);
                                const int32_t ra = (int32_t)iRA[ic] + (wrap ? TA32 : 0);
                                const uint64_t bm = __ballot(q < TI32 && ra <= e);
                                cnt += __popcll(bm);
                                if (bm != ~0ull) break;
                            }
                            rI += cnt;
                        }
                    }
                    if (rA >= TA32 && rI >= TI32) {  // past every A and I node of this rotation
                        rA -= TA32;
                        rI -= TI32;
                    }
                    spos = false;
                }
                if (lane == j) my_d = dsc;
            }
            if (lane < nv) wlen[p0 + lane] = my_d;
        }
        if (!spos && P > 0) {
            const int64_t e = endpos(dsc);
            s = e + 1 >= N ? e + 1 - N : e + 1;
        }
        if (lane == 0) {
            *next_start = s;
            *done = 1;
        }
    }
    __syncthreads();  // the descriptors (global, wave 0's stores) in
    // each pod's window end position -> wstart
    for (int64_t p = threadIdx.x; p < P; p += kRsT) {
        const int64_t dd = wlen[p], v = dd >> 2;
        int64_t e;
        if ((dd & 3) == 0) e = rs_select_lane(mA, bA, sA, W, TA, v >= TA ? v - TA : v);
        else if ((dd & 3) == 1) e = (int64_t)iPos[v >= TI ? v - TI : v];
        else e = v;
        wstart[p] = e;
    }
    __syncthreads();
    // windows: pod p starts after pod p - 1's end (the queue's first at `start`)
    for (int64_t c0 = 0; c0 < P; c0 += kRsT) {
        const int64_t p = c0 + threadIdx.x;
        int64_t e = 0, ep = 0;
        if (p < P) {
            e = wstart[p];
            ep = p == 0 ? start - 1 : (threadIdx.x == 0 ? carry : wstart[p - 1]);
        }
        __syncthreads();  // the chunk's ends read before they are overwritten
        if (p < P) {
            const int64_t s0 = ep + 1 >= N ? ep + 1 - N : ep + 1;
            int64_t dl = e - s0;
            if (dl < 0) dl += N;
            wstart[p] = s0;
            wlen[p] = dl + 1;
        }
        if (threadIdx.x == kRsT - 1) carry = e;
        __syncthreads();
    }
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
        // the pods whose window meets this workgroup's node block (a few % of them with
        // adaptive windows): the block's first node inside the window, or the window's first
        // position inside the block (a position past N - 1 wrapping to the block: a spare pod)
        uint64_t pm = __ballot(pv);
        if (a.wstart) {
            const int64_t nb0 = (int64_t)nb * kSelT;
            int64_t r1 = nb0 - ws, r2 = ws - nb0;
            if (r1 < 0) r1 += a.N;
            if (r2 < 0) r2 += a.N;
            pm = __ballot(pv && (r1 < wl || r2 < kSelT));
        }
        while (pm) {
            const int j = __ffsll((long long)pm) - 1;
            pm &= pm - 1;
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
                               int64_t* wlen, int64_t* next_start, int32_t* done, int form, hipStream_t st) {
    if (a.P <= 0 || a.N <= 0) return hipSuccess;
    const int64_t W = (a.N + 63) >> 6;
    const bool rs = form != 1 && W <= kRsMaxW && done;
    if (rs) {
        static const hipError_t attr = hipFuncSetAttribute(
            (const void*)k_sel_chain_rs, hipFuncAttributeMaxDynamicSharedMemorySize, (int)rs_lds_bytes(kRsMaxW));
        if (attr != hipSuccess) return attr;
        hipError_t e = klaunch("k_sel_chain_rs", k_sel_chain_rs, dim3(1), dim3(kRsT), rs_lds_bytes(W), st, a, fth, K,
                               start, wstart, wlen, next_start, done);
        if (e != hipSuccess) return e;
    }
    // the streaming form: the only one past the LDS form's size, else behind it (it exits at once
    // unless the LDS form found more in-range nodes than it holds)
    return klaunch("k_sel_chain", k_sel_chain, dim3(1), dim3(kChT), 0, st, a, fth, K, start, wstart, wlen,
                   next_start, rs ? (const int32_t*)done : nullptr);
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
