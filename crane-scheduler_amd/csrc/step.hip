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
// instant of the step; K3s then evaluates every (pod, node) pair by selecting
// its step: one int32 max for a node with no step inside the batch (most
// nodes), a 64-bit compare + select per step otherwise.
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

// Exact clamped Score of (pod at time t, node) — the literal int64 restatement
// of stats.go:114-138 + plugins.go:91-93, the semantics of K3's eval_pair and
// score_exact (kernels.hip).
template <int PD, int PR>
__device__ __forceinline__ int32_t score_at(int64_t t, const NodeRec<PD, PR>& r, double wsum, int32_t noprio) {
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
    return (int32_t)(f < 0 ? 0 : (f > 100 ? 100 : f));            // NormalizeScore (utils.go:58-68)
}

// Filter (plugins.go:41-43, 55-66) + packed key for pod kind T (0: Filter applies, 1: DaemonSet)
template <int PD, int PR>
__device__ __forceinline__ int32_t key_of(int T, int64_t t, int32_t score, const NodeRec<PD, PR>& r, int64_t n) {
    return (T == 1 || !(t < r.e_fail)) ? pack_key(score, n) : -1;
}

// ---------------------------------------------------------------- K3p
constexpr int kPodTile = 1024;

__global__ __launch_bounds__(kPodTile) void k3p_pods(const int64_t* __restrict__ now,
                                                     const uint8_t* __restrict__ flags, int64_t P,
                                                     int32_t* __restrict__ perm, int64_t* __restrict__ pnow,
                                                     int64_t* __restrict__ tile_mm, long long* __restrict__ keys) {
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
// One workgroup per 256-node segment, one thread per node.  Most nodes have no
// expiry inside the batch and only store their flat key; the rest append a
// Step1 (one step) or VRec (more) record to the segment's list for each pod
// kind, and the Step1 lists are padded to a multiple of 8 with records that
// never win, so K3s reads them eight at a time.
template <int PD, int PR>
__global__ __launch_bounds__(kStepSeg) void k3a_steps(const NodeRec<PD, PR>* __restrict__ rec, int64_t N,
                                                      const int64_t* __restrict__ tile_mm, int32_t ntiles,
                                                      double wsum, int32_t noprio, StepTables st) {
    constexpr int NB = PR + 2;
    using VR = VRec<NB>;
    __shared__ int64_t smn[kStepSeg / 64], smx[kStepSeg / 64];
    __shared__ int32_t lc[2][2];
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
    if (threadIdx.x < 4) lc[threadIdx.x >> 1][threadIdx.x & 1] = 0;
    __syncthreads();
    int64_t tmin = smn[0], tmax = smx[0];
#pragma unroll
    for (int i = 1; i < kStepSeg / 64; ++i) {
        tmin = min(tmin, smn[i]);
        tmax = max(tmax, smx[i]);
    }
    const int64_t seg = blockIdx.x;
    const int64_t n = seg * kStepSeg + threadIdx.x;
    auto in_range = [&](int64_t e) { return e > tmin && e <= tmax; };
    int32_t flat[2] = {-1, -1};
    if (n < N) {
        const NodeRec<PD, PR> r = rec[n];
        const int32_t s0 = score_at<PD, PR>(tmin, r, wsum, noprio);
        int m = in_range(r.e_hv);
#pragma unroll
        for (int k = 0; k < PR; ++k) m += in_range(r.e_prio[k]);
        const bool fail_in = in_range(r.e_fail);
        if (m == 0 && !fail_in) {
            flat[0] = key_of<PD, PR>(0, tmin, s0, r, n);
            flat[1] = key_of<PD, PR>(1, tmin, s0, r, n);
        } else {
            // stepped node (a few % of nodes): sort the in-range expiries (static indices)
#pragma unroll
            for (int T = 0; T < 2; ++T) {
                int64_t c[NB];
#pragma unroll
                for (int k = 0; k < PR; ++k) c[k] = r.e_prio[k];
                c[PR] = r.e_hv;
                c[PR + 1] = T == 0 ? r.e_fail : INT64_MIN;  // DaemonSet pods bypass the Filter
                int cnt = 0;
#pragma unroll
                for (int j = 0; j < NB; ++j) {
                    const bool in = in_range(c[j]);
                    c[j] = in ? c[j] : INT64_MAX;
                    cnt += in;
                }
                if (cnt == 0) {
                    flat[T] = key_of<PD, PR>(T, tmin, s0, r, n);
                    continue;
                }
#pragma unroll
                for (int i = 0; i < NB; ++i)  // odd-even transposition sort
#pragma unroll
                    for (int j = i & 1; j + 1 < NB; j += 2) {
                        const int64_t x = c[j], y = c[j + 1];
                        c[j] = min(x, y);
                        c[j + 1] = max(x, y);
                    }
                // key of step j+1 at its first instant c[j] (equal expiries give equal keys)
                const int32_t k0 = key_of<PD, PR>(T, tmin, s0, r, n);
                if (cnt == 1) {
                    const int32_t slot = atomicAdd(&lc[T][0], 1);
                    Step1 v;
                    v.bp = c[0];
                    v.k0 = k0;
                    v.k1 = key_of<PD, PR>(T, c[0], score_at<PD, PR>(c[0], r, wsum, noprio), r, n);
                    st.single[(int64_t)T * st.npad + seg * kStepSeg + slot] = v;
                } else {
                    const int32_t slot = atomicAdd(&lc[T][1], 1);
                    VR v;
                    v.cnt = cnt;
                    v.key[0] = k0;
#pragma unroll
                    for (int j = 0; j < NB; ++j) {
                        v.bp[j] = c[j];  // INT64_MAX past cnt: never selected
                        v.key[j + 1] =
                            j < cnt ? key_of<PD, PR>(T, c[j], score_at<PD, PR>(c[j], r, wsum, noprio), r, n) : -1;
                    }
                    reinterpret_cast<VR*>(st.multi)[(int64_t)T * st.npad + seg * kStepSeg + slot] = v;
                }
            }
        }
    }
    if (n < st.npad) {  // 16-bit segment-local form of the flat key
#pragma unroll
        for (int T = 0; T < 2; ++T)
            st.flat[T * st.npad + n] = flat[T] < 0 ? (int16_t)-1 : (int16_t)(((flat[T] >> 24) << 8) | (255 - threadIdx.x));
    }
    __syncthreads();
#pragma unroll
    for (int T = 0; T < 2; ++T) {
        const int32_t c = lc[T][0], c4 = (c + 7) & ~7;
        if ((int32_t)threadIdx.x >= c && (int32_t)threadIdx.x < c4) {
            Step1 v;
            v.bp = INT64_MAX;
            v.k0 = -1;
            v.k1 = -1;
            st.single[(int64_t)T * st.npad + seg * kStepSeg + threadIdx.x] = v;
        }
        if (threadIdx.x == 0) {
            st.cnt[((int64_t)T * st.nseg + seg) * 2] = c4;
            st.cnt[((int64_t)T * st.nseg + seg) * 2 + 1] = lc[T][1];
        }
    }
}

// ---------------------------------------------------------------- K3s
constexpr int kK3sWaves = 4;
constexpr int kK3sMaxSegs = 16;  // segments per workgroup chunk: 16 KB of LDS flat keys

// Max over one 256-node segment for the 64 pods of a wave: flat keys (one
// packed 16-bit max per two pairs), then the segment's one-step nodes eight
// records per scalar-load batch (64-bit compare + select), then the rare
// multi-step nodes.
// Pin a wave-uniform loaded value in an SGPR: keeps the compiler from turning
// "select between two loaded keys" into a per-lane gather of the selected one.
__device__ __forceinline__ int32_t sreg(int32_t x) { return __builtin_amdgcn_readfirstlane(x); }

typedef short v2i16 __attribute__((ext_vector_type(2)));

template <int NB>
__device__ __forceinline__ int32_t seg_max(int64_t tnow, int32_t best, const int4* lflat,
                                           const int32_t* __restrict__ cnt, const Step1* __restrict__ single,
                                           const VRec<NB>* __restrict__ multi, int32_t seg) {
    const int2 nc = *reinterpret_cast<const int2*>(cnt + 2 * seg);  // issued ahead of the flat loop
    // flat keys: 16-bit segment-local (score << 8 | 255 - local), two per dword,
    // one packed v_pk_max_i16 per pair of (pod, node) evaluations; read from
    // the workgroup's LDS copy with broadcast ds_read_b128 (8 keys per read)
    const int4* f = lflat;
    v2i16 b2 = {-1, -1};
#pragma unroll
    for (int i = 0; i < kStepSeg / 8; i += 16) {
        int4 k[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) k[j] = f[i + j];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            b2 = __builtin_elementwise_max(b2, __builtin_bit_cast(v2i16, k[j].x));
            b2 = __builtin_elementwise_max(b2, __builtin_bit_cast(v2i16, k[j].y));
            b2 = __builtin_elementwise_max(b2, __builtin_bit_cast(v2i16, k[j].z));
            b2 = __builtin_elementwise_max(b2, __builtin_bit_cast(v2i16, k[j].w));
        }
    }
    const int32_t m16 = max((int32_t)b2.x, (int32_t)b2.y);
    if (m16 >= 0)  // back to the global 32-bit key: (score << 24) | (0xFFFFFF - node)
        best = max(best, ((m16 >> 8) << 24) | (0xFFFFFF - (seg * kStepSeg + 255 - (m16 & 255))));
    const int4* __restrict__ s1 = reinterpret_cast<const int4*>(single + (int64_t)seg * kStepSeg);
    for (int32_t j = 0; j < nc.x; j += 8) {
        int4 q[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) q[u] = s1[j + u];
        int32_t k0[8], k1[8];
        int64_t bp[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            bp[u] = (int64_t)(((uint64_t)(uint32_t)sreg(q[u].y) << 32) | (uint32_t)sreg(q[u].x));
            k0[u] = sreg(q[u].z);
            k1[u] = sreg(q[u].w);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) best = max(best, tnow >= bp[u] ? k1[u] : k0[u]);
    }
    const VRec<NB>* __restrict__ vm = multi + (int64_t)seg * kStepSeg;
    for (int32_t j = 0; j < nc.y; ++j) {
        int32_t key[NB + 1];
        int64_t bp[NB];
#pragma unroll
        for (int s = 0; s <= NB; ++s) key[s] = sreg(vm[j].key[s]);
#pragma unroll
        for (int s = 0; s < NB; ++s) bp[s] = vm[j].bp[s];
        int32_t k = key[0];
#pragma unroll
        for (int s = 0; s < NB; ++s) k = tnow >= bp[s] ? key[s + 1] : k;
        best = max(best, k);
    }
    return best;
}

template <int NB>
__global__ __launch_bounds__(kK3sWaves * 64) void k3s_eval(StepTables st, const int32_t* __restrict__ perm,
                                                           const int64_t* __restrict__ pnow, int64_t P,
                                                           int64_t node_offset, int32_t segs_per_chunk,
                                                           int32_t nchunks, long long* __restrict__ keys) {
    const int64_t b = blockIdx.x;
    const int64_t chunk = b % nchunks;  // nchunks % 8 == 0 when >= 8: an XCD keeps its chunks
    const int64_t ptile = b / nchunks;
    // the 4 waves take 4 different 64-pod tiles over the SAME node segments, so a
    // segment's keys are fetched into the scalar cache once per workgroup
    const int64_t slot = ptile * (kK3sWaves * 64) + threadIdx.x;
    const bool live = slot < P;
    // K3p wrote the pods in partitioned order: two independent coalesced loads
    const int32_t praw = live ? perm[slot] : 0;
    const int64_t tnow = live ? pnow[slot] : 0;
    const bool ds = praw < 0;
    const int32_t pod = praw & 0x7FFFFFFF;
    const bool any_n = __ballot(live && !ds) != 0, any_d = __ballot(ds) != 0;
    const int32_t s0 = __builtin_amdgcn_readfirstlane((int32_t)chunk * segs_per_chunk);
    const int32_t s1 = __builtin_amdgcn_readfirstlane(min((int32_t)st.nseg, s0 + segs_per_chunk));
    // stage the chunk's flat keys of both pod kinds in LDS: [kind][segment][32 x int4]
    extern __shared__ int4 lds_flat[];
    constexpr int kSegI4 = kStepSeg * 2 / 16;  // int4 per segment of 16-bit keys
    const int32_t nsi4 = (s1 - s0) * kSegI4;
    for (int32_t i = threadIdx.x; i < 2 * nsi4; i += kK3sWaves * 64) {
        const int32_t T = i >= nsi4, j = i - T * nsi4;
        lds_flat[T * segs_per_chunk * kSegI4 + j] =
            reinterpret_cast<const int4*>(st.flat + T * st.npad + (int64_t)s0 * kStepSeg)[j];
    }
    __syncthreads();
    const VRec<NB>* __restrict__ vm = reinterpret_cast<const VRec<NB>*>(st.multi);
    int32_t bn = -1, bd = -1;
    if (any_n)
        for (int32_t s = s0; s < s1; ++s)
            bn = seg_max<NB>(tnow, bn, lds_flat + (s - s0) * kSegI4, st.cnt, st.single, vm, s);
    if (any_d)
        for (int32_t s = s0; s < s1; ++s)
            bd = seg_max<NB>(tnow, bd, lds_flat + (segs_per_chunk + s - s0) * kSegI4, st.cnt + 2 * st.nseg,
                             st.single + st.npad, vm + st.npad, s);
    const int32_t best = ds ? bd : bn;
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
    g.ntiles = (P + kPodTile - 1) / kPodTile;
    const int64_t ptiles = (P + kK3sWaves * 64 - 1) / (kK3sWaves * 64);
    // ~4 waves per SIMD: 256 CUs x 4 SIMDs x 4 waves / 4 waves per workgroup
    const char* e = getenv("CRANE_K3S_BLOCKS");
    const int64_t target = e && atoi(e) > 0 ? atoi(e) : 4096;
    int64_t nch = std::max<int64_t>(1, target / std::max<int64_t>(ptiles, 1));
    if (nch >= 8) nch = nch / 8 * 8;
    nch = std::min<int64_t>(nch, std::max<int64_t>(g.nseg, 1));
    g.segs_per_chunk = (int32_t)((g.nseg + nch - 1) / std::max<int64_t>(nch, 1));
    if (g.segs_per_chunk < 1) g.segs_per_chunk = 1;
    if (g.segs_per_chunk > kK3sMaxSegs) g.segs_per_chunk = kK3sMaxSegs;  // LDS copy of the flat keys
    g.nchunks = (int32_t)((g.nseg + g.segs_per_chunk - 1) / g.segs_per_chunk);
    if (g.nchunks < 1) g.nchunks = 1;
    g.ptiles = ptiles;
    return g;
}

template <int PD, int PR>
static hipError_t launch_step_t(const void* rec, int64_t N, int64_t node_offset, const int64_t* now,
                                const uint8_t* flags, int64_t P, double wsum, int32_t noprio, long long* keys,
                                const StepTables& st, const StepGeometry& g, int32_t* perm, int64_t* pnow,
                                int64_t* tile_mm, hipStream_t s) {
    if (P <= 0) return hipSuccess;
    hipLaunchKernelGGL(k3p_pods, dim3((unsigned)g.ntiles), dim3(kPodTile), 0, s, now, flags, P, perm, pnow, tile_mm,
                       keys);
    if (N <= 0) return hipGetLastError();
    hipLaunchKernelGGL((k3a_steps<PD, PR>), dim3((unsigned)g.nseg), dim3(kStepSeg), 0, s,
                       static_cast<const NodeRec<PD, PR>*>(rec), N, tile_mm, (int32_t)g.ntiles, wsum, noprio, st);
    const unsigned blocks = (unsigned)(g.ptiles * g.nchunks);
    const size_t lds = (size_t)g.segs_per_chunk * kStepSeg * 2 * sizeof(int16_t);  // both pod kinds
    hipLaunchKernelGGL((k3s_eval<PR + 2>), dim3(blocks), dim3(kK3sWaves * 64), lds, s, st, perm, pnow, P,
                       node_offset, g.segs_per_chunk, g.nchunks, keys);
    return hipGetLastError();
}

hipError_t launch_eval_step(int shape, const void* rec, int64_t N, int64_t node_offset, const int64_t* now,
                            const uint8_t* flags, int64_t P, double wsum, int32_t noprio, long long* keys,
                            const StepTables& st, const StepGeometry& g, int32_t* perm, int64_t* pnow,
                            int64_t* tile_mm, hipStream_t s) {
    if (N >= kStepMaxNodes) return hipErrorInvalidValue;
    switch (shape) {
        case kShape4x6:
            return launch_step_t<4, 6>(rec, N, node_offset, now, flags, P, wsum, noprio, keys, st, g, perm, pnow, tile_mm, s);
        case kShape8x8:
            return launch_step_t<8, 8>(rec, N, node_offset, now, flags, P, wsum, noprio, keys, st, g, perm, pnow, tile_mm, s);
        default:
            return launch_step_t<16, 16>(rec, N, node_offset, now, flags, P, wsum, noprio, keys, st, g, perm, pnow, tile_mm,
                                         s);
    }
}

}  // namespace crane
