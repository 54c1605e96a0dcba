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
// once per step with the literal int64 restatement (score_exact), at a
// representative time inside the step; K3s then evaluates every (pod, node)
// pair by selecting its step: one int32 max for a node with no step inside the
// batch (most nodes), a 64-bit compare + select per step otherwise.
//
//   K3p  pods  : DaemonSet partition per 1024-pod tile (so waves are uniform),
//                key init, per-tile min/max of now
//   K3a  nodes : per-node step tables for both pod kinds (Filter applies /
//                DaemonSet bypass, utils.go:17-24), 256-node segments
//   K3s  pairs : 64 pods per wave, node keys wave-uniform through scalar loads,
//                4 waves of a workgroup split its node chunk, LDS combine, one
//                64-bit atomicMax per pod per workgroup (lowest index wins ties)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "dyn_types.hpp"
#include "kernels.hpp"

namespace crane {

// same packing as K3: (score << 24) | (0xFFFFFF - node), -1 = pod may not go there
__device__ __forceinline__ int32_t pack_key(int32_t f, int64_t n) { return (f << 24) | (int32_t)(0xFFFFFF - n); }

// Exact Filter + Score key of (pod at time t, node n) — the same semantics as
// K3's eval_pair (kernels.hip), through the literal int64 path.
template <int PD, int PR>
__device__ __attribute__((noinline)) int32_t key_at(int64_t t, bool ds, const NodeRec<PD, PR>& r, int64_t n,
                                                    double wsum, int32_t noprio) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < PR; ++k)
        if (t < r.e_prio[k]) s += r.t[k];  // stats.go:124-133, policy order
    int64_t base = 0;
    if (!noprio) {
        const double q = s / wsum;  // stats.go:135 int(score / weight), Go CVTTSD2SQ
        base = (q >= -9223372036854775808.0 && q < 9223372036854775808.0) ? (int64_t)q : INT64_MIN;
    }
    const int64_t pen = t < r.e_hv ? r.pen : 0;
    const int64_t f = (int64_t)((uint64_t)base - (uint64_t)pen);  // plugins.go:91, wraps like Go
    const int32_t fc = (int32_t)(f < 0 ? 0 : (f > 100 ? 100 : f));  // NormalizeScore (utils.go:58-68)
    const bool feasible = ds || !(t < r.e_fail);                     // plugins.go:41-43, 55-66
    return feasible ? pack_key(fc, n) : -1;
}

// ---------------------------------------------------------------- K3p
constexpr int kPodTile = 1024;

__global__ __launch_bounds__(kPodTile) void k3p_pods(const int64_t* __restrict__ now,
                                                     const uint8_t* __restrict__ flags, int64_t P,
                                                     int32_t* __restrict__ perm, int64_t* __restrict__ tile_mm,
                                                     long long* __restrict__ keys) {
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
        perm[t * kPodTile + pos] = (int32_t)p;
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
template <int PD, int PR>
__global__ __launch_bounds__(kStepSeg) void k3a_steps(const NodeRec<PD, PR>* __restrict__ rec, int64_t N,
                                                      const int64_t* __restrict__ tile_mm, int32_t ntiles,
                                                      double wsum, int32_t noprio, StepTables st) {
    constexpr int NB = PR + 2;
    using VR = VRec<NB>;
    __shared__ int64_t smn[kStepSeg / 64], smx[kStepSeg / 64];
    __shared__ int32_t vc[2];
    // batch time range [tmin, tmax] from K3p's tile partials
    int64_t mn = INT64_MAX, mx = INT64_MIN;
    for (int i = threadIdx.x; i < ntiles; i += kStepSeg) {
        mn = min(mn, tile_mm[2 * i]);
        mx = max(mx, tile_mm[2 * i + 1]);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        mn = min(mn, (int64_t)__shfl_xor((long long)mn, o));
        mx = max(mx, (int64_t)__shfl_xor((long long)mx, o));
    }
    if ((threadIdx.x & 63) == 0) {
        smn[threadIdx.x >> 6] = mn;
        smx[threadIdx.x >> 6] = mx;
    }
    if (threadIdx.x < 2) vc[threadIdx.x] = 0;
    __syncthreads();
    int64_t tmin = smn[0], tmax = smx[0];
    for (int i = 1; i < kStepSeg / 64; ++i) {
        tmin = min(tmin, smn[i]);
        tmax = max(tmax, smx[i]);
    }
    const int64_t seg = blockIdx.x;
    const int64_t n = seg * kStepSeg + threadIdx.x;
    int32_t key0[2] = {-1, -1}, cnt[2] = {0, 0};
    int64_t bp[2][NB];
    int32_t kk[2][NB];
    if (n < N) {
        const NodeRec<PD, PR> r = rec[n];
#pragma unroll
        for (int T = 0; T < 2; ++T) {
            // expiries inside (tmin, tmax], ascending (out-of-range -> INT64_MAX, sorted
            // last).  Equal expiries stay: the chain then selects equal keys twice.
            int64_t* c = bp[T];
#pragma unroll
            for (int k = 0; k < PR; ++k) c[k] = r.e_prio[k];
            c[PR] = r.e_hv;
            c[PR + 1] = T == 0 ? r.e_fail : INT64_MIN;  // DaemonSet pods bypass the Filter
            int m = 0;
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                const bool in = c[j] > tmin && c[j] <= tmax;
                c[j] = in ? c[j] : INT64_MAX;
                m += in;
            }
#pragma unroll
            for (int i = 0; i < NB; ++i)  // odd-even transposition sort, static indices
#pragma unroll
                for (int j = i & 1; j + 1 < NB; j += 2) {
                    const int64_t a = c[j], b2 = c[j + 1];
                    c[j] = min(a, b2);
                    c[j + 1] = max(a, b2);
                }
            cnt[T] = m;
            key0[T] = key_at<PD, PR>(tmin, T == 1, r, n, wsum, noprio);
#pragma unroll
            for (int j = 0; j < NB; ++j)
                kk[T][j] = j < m ? key_at<PD, PR>(c[j], T == 1, r, n, wsum, noprio) : -1;
        }
    }
    if (n < st.npad) {
#pragma unroll
        for (int T = 0; T < 2; ++T) st.flat[T * st.npad + n] = cnt[T] ? -1 : key0[T];
    }
    int32_t slot[2] = {0, 0};
#pragma unroll
    for (int T = 0; T < 2; ++T)
        if (cnt[T]) slot[T] = atomicAdd(&vc[T], 1);
#pragma unroll
    for (int T = 0; T < 2; ++T) {
        if (!cnt[T]) continue;
        VR v;
        v.cnt = cnt[T];
        v.key[0] = key0[T];
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            v.bp[j] = j < cnt[T] ? bp[T][j] : INT64_MAX;
            v.key[j + 1] = j < cnt[T] ? kk[T][j] : -1;
        }
        VR* dst = reinterpret_cast<VR*>(st.vrec) + (int64_t)T * st.npad + seg * kStepSeg + slot[T];
        *dst = v;
    }
    __syncthreads();
    if (threadIdx.x < 2) st.vcnt[threadIdx.x * st.nseg + seg] = vc[threadIdx.x];
}

// ---------------------------------------------------------------- K3s
constexpr int kK3sWaves = 4;

// Max over one 256-node segment for the 64 pods of a wave: flat keys (one
// int32 max per pair), then the segment's stepped nodes (select per step).
template <int NB>
__device__ __forceinline__ int32_t seg_max(int64_t tnow, int32_t best, const int32_t* __restrict__ flat,
                                           const int32_t* __restrict__ vcnt, const VRec<NB>* __restrict__ vrec,
                                           int64_t seg) {
    const int32_t* __restrict__ f = flat + seg * kStepSeg;
#pragma unroll 64
    for (int i = 0; i < kStepSeg; ++i) best = max(best, f[i]);
    const int32_t nv = vcnt[seg];
    const VRec<NB>* __restrict__ v = vrec + seg * kStepSeg;
    for (int32_t j = 0; j < nv; ++j) {
        const int32_t c = v[j].cnt;
        int32_t k = v[j].key[0];
        for (int32_t s = 0; s < c; ++s) k = tnow >= v[j].bp[s] ? v[j].key[s + 1] : k;
        best = max(best, k);
    }
    return best;
}

template <int NB>
__global__ __launch_bounds__(kK3sWaves * 64) void k3s_eval(StepTables st, const int32_t* __restrict__ perm,
                                                           const int64_t* __restrict__ now,
                                                           const uint8_t* __restrict__ flags, int64_t P,
                                                           int64_t node_offset, int32_t segs_per_chunk,
                                                           int32_t nchunks, long long* __restrict__ keys) {
    __shared__ int32_t red[kK3sWaves][64];
    const int64_t b = blockIdx.x;
    const int64_t chunk = b % nchunks;  // nchunks % 8 == 0 when >= 8: an XCD keeps its chunks
    const int64_t ptile = b / nchunks;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t slot = ptile * 64 + lane;
    const bool live = slot < P;
    const int32_t pod = live ? perm[slot] : 0;
    const int64_t tnow = live ? now[pod] : 0;
    const bool ds = live && flags && (flags[pod] & 1u);
    const bool any_n = __ballot(live && !ds) != 0, any_d = __ballot(ds) != 0;
    // this wave's segments of the workgroup's chunk
    const int64_t cs = chunk * segs_per_chunk;
    const int64_t ce = min((int64_t)st.nseg, cs + segs_per_chunk);
    const int64_t q = (segs_per_chunk + kK3sWaves - 1) / kK3sWaves;
    const int64_t s0 = min(ce, cs + wave * q), s1 = min(ce, s0 + q);
    const VRec<NB>* __restrict__ vr = reinterpret_cast<const VRec<NB>*>(st.vrec);
    int32_t bn = -1, bd = -1;
    if (any_n)
        for (int64_t s = s0; s < s1; ++s) bn = seg_max<NB>(tnow, bn, st.flat, st.vcnt, vr, s);
    if (any_d)
        for (int64_t s = s0; s < s1; ++s)
            bd = seg_max<NB>(tnow, bd, st.flat + st.npad, st.vcnt + st.nseg, vr + st.npad, s);
    red[wave][lane] = ds ? bd : bn;
    __syncthreads();
    if (wave == 0) {
        int32_t best = red[0][lane];
#pragma unroll
        for (int i = 1; i < kK3sWaves; ++i) best = max(best, red[i][lane]);
        if (live && best >= 0) {
            const int64_t sc = best >> 24;
            const int64_t n = 0xFFFFFF - (best & 0xFFFFFF);
            atomicMax(&keys[pod], (long long)((sc << 32) | (int64_t)(0xFFFFFFFFull - (uint64_t)(node_offset + n))));
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

StepGeometry step_geometry(int64_t P, int64_t N) {
    StepGeometry g{};
    g.nseg = (N + kStepSeg - 1) / kStepSeg;
    g.npad = g.nseg * kStepSeg;
    g.ntiles = (P + kPodTile - 1) / kPodTile;
    const int64_t ptiles = (P + 63) / 64;
    // ~4 waves per SIMD: 256 CUs x 4 SIMDs x 4 waves / 4 waves per workgroup
    const char* e = getenv("CRANE_K3S_BLOCKS");
    const int64_t target = e && atoi(e) > 0 ? atoi(e) : 4096;
    int64_t nch = std::max<int64_t>(1, target / std::max<int64_t>(ptiles, 1));
    if (nch >= 8) nch = nch / 8 * 8;
    nch = std::min<int64_t>(nch, std::max<int64_t>(g.nseg, 1));
    g.segs_per_chunk = (int32_t)((g.nseg + nch - 1) / std::max<int64_t>(nch, 1));
    if (g.segs_per_chunk < 1) g.segs_per_chunk = 1;
    g.nchunks = (int32_t)((g.nseg + g.segs_per_chunk - 1) / g.segs_per_chunk);
    if (g.nchunks < 1) g.nchunks = 1;
    g.ptiles = ptiles;
    return g;
}

template <int PD, int PR>
static hipError_t launch_step_t(const void* rec, int64_t N, int64_t node_offset, const int64_t* now,
                                const uint8_t* flags, int64_t P, double wsum, int32_t noprio, long long* keys,
                                const StepTables& st, const StepGeometry& g, int32_t* perm, int64_t* tile_mm,
                                hipStream_t s) {
    if (P <= 0) return hipSuccess;
    hipLaunchKernelGGL(k3p_pods, dim3((unsigned)g.ntiles), dim3(kPodTile), 0, s, now, flags, P, perm, tile_mm,
                       keys);
    if (N <= 0) return hipGetLastError();
    hipLaunchKernelGGL((k3a_steps<PD, PR>), dim3((unsigned)g.nseg), dim3(kStepSeg), 0, s,
                       static_cast<const NodeRec<PD, PR>*>(rec), N, tile_mm, (int32_t)g.ntiles, wsum, noprio, st);
    const unsigned blocks = (unsigned)(g.ptiles * g.nchunks);
    hipLaunchKernelGGL((k3s_eval<PR + 2>), dim3(blocks), dim3(kK3sWaves * 64), 0, s, st, perm, now, flags, P,
                       node_offset, g.segs_per_chunk, g.nchunks, keys);
    return hipGetLastError();
}

hipError_t launch_eval_step(int shape, const void* rec, int64_t N, int64_t node_offset, const int64_t* now,
                            const uint8_t* flags, int64_t P, double wsum, int32_t noprio, long long* keys,
                            const StepTables& st, const StepGeometry& g, int32_t* perm, int64_t* tile_mm,
                            hipStream_t s) {
    if (N >= kStepMaxNodes) return hipErrorInvalidValue;
    switch (shape) {
        case kShape4x6:
            return launch_step_t<4, 6>(rec, N, node_offset, now, flags, P, wsum, noprio, keys, st, g, perm, tile_mm, s);
        case kShape8x8:
            return launch_step_t<8, 8>(rec, N, node_offset, now, flags, P, wsum, noprio, keys, st, g, perm, tile_mm, s);
        default:
            return launch_step_t<16, 16>(rec, N, node_offset, now, flags, P, wsum, noprio, keys, st, g, perm, tile_mm,
                                         s);
    }
}

}  // namespace crane
