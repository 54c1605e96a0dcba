// matrix.hip — K3m: the per-pair form of Filter + Score (plugins.go:39-98).
//
// Every (pod, node) pair's result is materialised: the first failing predicate
// (Filter: -1 = Success, else its policy index; DaemonSet pods bypass,
// plugins.go:41-43) and the clamped Score, as [P][ld] matrices — what the
// drop-in plugin's per-node Filter/Score calls read back — and/or each pod's
// packed best key (chosen node).
//
// Layout: a lane owns VEC consecutive nodes (a workgroup = 4 waves = 256 * VEC
// nodes) and walks the workgroup's chunk of pods in sub-chunks of 64.  A pod's
// time is wave-uniform (v_readlane into SGPRs), so one store instruction writes
// 64 * VEC consecutive bytes of a matrix row (byte, dword or dwordx2 stores).
//
// Why the per-pair work is small and exact: for a node, Filter and Score depend
// on the pod only through `now < expiry` comparisons (stats.go:42-48), so the
// node's (first-fail, score) is constant on [lo, hi), the interval between its
// consecutive expiries around the evaluation time.  A lane keeps its nodes'
// packed results together with the intersection [LO, HI) of their intervals;
// a sub-chunk whose pod times [cmin, cmax] lie inside it reuses them (two
// 64-bit compares per lane).  Otherwise the lane re-reads its node records and
// re-evaluates at cmin with the literal restatement (score_at, step_node.hpp);
// a node with one expiry inside (cmin, cmax] also gets its values after that
// expiry (per pod: compare + select), one with several is evaluated per pod.
//
// Keys: per pod, a lane max of (score << 24 | 0xFFFFFF - local node) over its
// nodes, a wave max, an LDS max over the workgroup's waves, and one 64-bit
// atomicMax per pod per workgroup into keys[] (initialised to -1; lowest global
// index wins ties).  In an all-flat sub-chunk the two per-kind wave maxima are
// taken once.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dyn_types.hpp"
#include "kernels.hpp"
#include "step_node.hpp"
#include "node_steps.hpp"

namespace crane {

constexpr int kMxT = 256;       // threads per workgroup
constexpr int kMxChunk = 1024;  // max pods per workgroup (LDS best keys)


__device__ __forceinline__ int32_t wave_max32(int32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

__device__ __forceinline__ uint32_t put_byte(uint32_t w, int i, int32_t b) {
    const int sh = 8 * i;
    return (w & ~(0xFFu << sh)) | (((uint32_t)b & 0xFFu) << sh);
}
__device__ __forceinline__ int32_t get_byte(uint32_t w, int i) { return (int32_t)(int8_t)(w >> (8 * i)); }

// VEC consecutive int8 values at p (VEC-byte aligned)
template <int VEC>
__device__ __forceinline__ void store_bytes(int8_t* p, const uint32_t* w) {
    if constexpr (VEC == 1) *p = (int8_t)w[0];
    else if constexpr (VEC == 4) *reinterpret_cast<uint32_t*>(p) = w[0];
    else if constexpr (VEC == 8) *reinterpret_cast<uint2*>(p) = make_uint2(w[0], w[1]);
    else *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}

template <int PD, int PR, int VEC, bool I64, bool OUT, bool KEYS>
__global__ __launch_bounds__(kMxT) void k3m_matrix(MatrixArgs a, int32_t chunk, int32_t nbx, int32_t per,
                                                   int32_t ncy) {
    static_assert(VEC == 1 || VEC == 4 || VEC == 8, "byte, dword or dwordx2 stores");
    static_assert(!I64 || VEC == 1, "int64 scores: one node per lane");
    constexpr int NW = (VEC + 3) / 4;  // packed words per lane
    __shared__ int32_t best[KEYS ? kMxChunk : 1];
    // XCD-aware: XCD x (= workgroup id % 8) takes node blocks [x*per, (x+1)*per) of every chunk,
    // so each XCD's L2 holds 1/8 of the record table
    const int64_t b = blockIdx.x, q = b >> 3;
    const int32_t nb = (int32_t)((b & 7) * per + q % per), cy = (int32_t)(q / per);
    if (nb >= nbx || cy >= ncy) return;  // (whole workgroup: no barrier is skipped by part of it)
    const int32_t loc0 = threadIdx.x * VEC;  // this lane's first node, local to the workgroup
    const int64_t n0 = (int64_t)nb * (kMxT * VEC) + loc0;
    const int nvalid = (int)max((int64_t)0, min((int64_t)VEC, a.N - n0));  // live nodes of this lane
    const int64_t p0 = (int64_t)cy * chunk, p1 = min(a.P, p0 + chunk);
    const int lane = threadIdx.x & 63;
    if (KEYS) {
        for (int i = threadIdx.x; i < chunk; i += kMxT) best[i] = -1;
        __syncthreads();
    }
    const NodeRec<PD, PR>* __restrict__ rec = static_cast<const NodeRec<PD, PR>*>(a.rec) + n0;
    // per lane: results at the last evaluation (f0, s0 packed), valid on [LO, HI); nodes with a step
    // inside the current sub-chunk: after-step values (f1, s1), the step bp, `multi` = several steps
    uint32_t f0w[NW], s0w[NW], f1w[NW], s1w[NW];
    int64_t bp[VEC];
    uint32_t stepped = 0, multi = 0;
    int64_t LO = INT64_MAX, HI = INT64_MIN;  // empty: evaluate at the first sub-chunk
    int32_t kn_l = -1, kd_l = -1;            // lane maxima of the flat keys per pod kind
#pragma unroll
    for (int w = 0; w < NW; ++w) f0w[w] = s0w[w] = f1w[w] = s1w[w] = 0;
#pragma unroll
    for (int v = 0; v < VEC; ++v) bp[v] = INT64_MAX;
    for (int64_t q0 = p0; q0 < p1; q0 += 64) {
        const int nv = (int)min((int64_t)64, p1 - q0);
        const bool pv = lane < nv;
        const int64_t tn = pv ? a.now[q0 + lane] : 0;
        const int32_t fl = pv && a.flags ? (int32_t)(a.flags[q0 + lane] & 1u) : 0;
        int64_t cmin = pv ? tn : INT64_MAX, cmax = pv ? tn : INT64_MIN;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            cmin = min(cmin, (int64_t)__shfl_xor((long long)cmin, o));
            cmax = max(cmax, (int64_t)__shfl_xor((long long)cmax, o));
        }
        if (nvalid > 0 && !(cmin >= LO && cmax < HI)) {
            // re-evaluate this lane's nodes at cmin (rare once the batch's times are covered)
            LO = INT64_MIN;
            HI = INT64_MAX;
            stepped = multi = 0;
            kn_l = kd_l = -1;
#pragma unroll
            for (int v = 0; v < VEC; ++v) {
                if (v >= nvalid) continue;
                const NodeRec<PD, PR> r = rec[v];
                int64_t lo, hi;
                bracket<PD, PR>(r, cmin, lo, hi);
                const int32_t f = ff_at<PD, PR>(cmin, r, a);
                const int32_t s = score_at<PD, PR>(cmin, r, a.wsum, a.noprio);
                f0w[v / 4] = put_byte(f0w[v / 4], v & 3, f);
                s0w[v / 4] = put_byte(s0w[v / 4], v & 3, s);
                LO = max(LO, lo);
                if (hi <= cmax) {  // a step inside the sub-chunk: the values from hi on
                    stepped |= 1u << v;
                    bp[v] = hi;
                    int64_t lo2, hi2;
                    bracket<PD, PR>(r, hi, lo2, hi2);
                    f1w[v / 4] = put_byte(f1w[v / 4], v & 3, ff_at<PD, PR>(hi, r, a));
                    s1w[v / 4] = put_byte(s1w[v / 4], v & 3, score_at<PD, PR>(hi, r, a.wsum, a.noprio));
                    if (hi2 <= cmax) multi |= 1u << v;
                }
                HI = min(HI, hi);
                const int32_t k = pack_key(s, loc0 + v);
                kd_l = max(kd_l, k);
                kn_l = max(kn_l, f < 0 ? k : -1);
            }
        }
        const bool any_stepped = __ballot(stepped != 0) != 0;
        int32_t kn = -1, kd = -1;  // wave maxima of the flat keys per pod kind
        if (KEYS && !any_stepped) {
            kn = wave_max32(kn_l);
            kd = wave_max32(kd_l);
        }
        for (int j = 0; j < nv; ++j) {
            const bool d = __builtin_amdgcn_readlane(fl, j) != 0;
            uint32_t fw[NW], sw[NW];
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                fw[w] = f0w[w];
                sw[w] = s0w[w];
            }
            int32_t kl_n = kn_l, kl_d = kd_l;
            if (any_stepped) {  // (wave-uniform)
                const int64_t t = readlane64(tn, j);
                if (stepped) {
                    kl_n = kl_d = -1;
#pragma unroll
                    for (int v = 0; v < VEC; ++v) {
                        if (v >= nvalid) continue;
                        int32_t f = get_byte(f0w[v / 4], v & 3), s = get_byte(s0w[v / 4], v & 3);
                        if (multi & (1u << v)) {
                            const NodeRec<PD, PR> r = rec[v];
                            f = ff_at<PD, PR>(t, r, a);
                            s = score_at<PD, PR>(t, r, a.wsum, a.noprio);
                        } else if ((stepped & (1u << v)) && t >= bp[v]) {
                            f = get_byte(f1w[v / 4], v & 3);
                            s = get_byte(s1w[v / 4], v & 3);
                        }
                        fw[v / 4] = put_byte(fw[v / 4], v & 3, f);
                        sw[v / 4] = put_byte(sw[v / 4], v & 3, s);
                        const int32_t k = pack_key(s, loc0 + v);
                        kl_d = max(kl_d, k);
                        kl_n = max(kl_n, f < 0 ? k : -1);
                    }
                }
            }
            if (OUT && nvalid > 0) {
                const int64_t o = (q0 + j) * a.ld + n0;
                if (a.first_fail) {
                    if (d) {
#pragma unroll
                        for (int w = 0; w < NW; ++w) fw[w] = 0xFFFFFFFFu;
                    }
                    if (nvalid == VEC) store_bytes<VEC>(a.first_fail + o, fw);
                    else
                        for (int v = 0; v < nvalid; ++v) a.first_fail[o + v] = (int8_t)get_byte(fw[v / 4], v & 3);
                }
                if (a.score) {
                    if constexpr (I64) {
                        static_cast<int64_t*>(a.score)[o] = get_byte(sw[0], 0);
                    } else {
                        int8_t* sp = static_cast<int8_t*>(a.score) + o;
                        if (nvalid == VEC) store_bytes<VEC>(sp, sw);
                        else
                            for (int v = 0; v < nvalid; ++v) sp[v] = (int8_t)get_byte(sw[v / 4], v & 3);
                    }
                }
            }
            if (KEYS) {
                const int32_t k = any_stepped ? wave_max32(d ? kl_d : kl_n) : (d ? kd : kn);
                if (lane == 0 && k >= 0) atomicMax(&best[q0 + j - p0], k);
            }
        }
    }
    if (KEYS) {
        // one 64-bit atomicMax per pod per workgroup (a last-workgroup reduction over
        // partials measured far slower: its agent-scope release fence writes back the L2)
        __syncthreads();
        for (int i = threadIdx.x; i < (int)(p1 - p0); i += kMxT) {
            const int32_t k = best[i];
            if (k < 0) continue;
            const int64_t sc = k >> 24;
            const int64_t g = a.node_offset + (int64_t)nb * (kMxT * VEC) + (0xFFFFFF - (k & 0xFFFFFF));
            atomicMax(&a.keys[p0 + i], (long long)((sc << 32) | (int64_t)(0xFFFFFFFFull - (uint64_t)g)));
        }
    }
}

// Launch geometry: VEC nodes per lane and pods per workgroup.  About four waves
// per SIMD (256 CUs x 4 SIMDs) for small batches (config 2: 5000 x 1000 best at
// one node per lane, ~19 pods per workgroup: 16.5 us vs 19-24 us for 16 or 64);
// wide lanes (8 nodes, dwordx2 stores) with 1024-pod workgroups once the batch
// is large (config 3: 0.47-0.61 ms vs 0.63-0.73 for 16 nodes per lane or 256-pod
// workgroups; tools/matrix_probe.py).
struct MatrixGeometry {
    int vec;
    int64_t chunk, nbx, ncy, per;
};

static MatrixGeometry matrix_geometry(const MatrixArgs& a, bool out) {
    const int64_t pairs = a.P * a.N;
    const int64_t want_waves = 4096;
    const int64_t ppw = std::max<int64_t>(1, pairs / want_waves);  // pairs per wave
    auto aligned = [&](int v) {
        if (!out) return true;
        if (a.score && a.score_i64) return v == 1;
        const uintptr_t m = (uintptr_t)v - 1;
        return a.ld % v == 0 && ((uintptr_t)a.first_fail & m) == 0 && ((uintptr_t)a.score & m) == 0;
    };
    MatrixGeometry g{};
    g.vec = 1;
    for (int v : {8, 4}) {
        if (aligned(v) && 64 * v * std::min<int64_t>(a.P, 64) <= ppw) {
            g.vec = v;
            break;
        }
    }
    int64_t chunk = std::max<int64_t>(1, ppw / (64 * g.vec));
    if (g.vec >= 8) chunk *= 4;
    if (chunk >= 64) chunk = std::min<int64_t>(kMxChunk, (chunk + 63) / 64 * 64);
    g.chunk = std::min(chunk, a.P);
    g.nbx = (a.N + kMxT * g.vec - 1) / (kMxT * g.vec);
    g.ncy = (a.P + g.chunk - 1) / g.chunk;
    g.per = (g.nbx + 7) / 8;
    return g;
}

template <int PD, int PR, int VEC>
static hipError_t launch_vec(const MatrixArgs& a, const MatrixGeometry& g, bool out, bool keys, hipStream_t st) {
    const int64_t grid = 8 * g.per * g.ncy;
    if (grid > 0x7FFFFFFF) return hipErrorInvalidValue;
    const dim3 gr((unsigned)grid), blk(kMxT);
    const int32_t c32 = (int32_t)g.chunk, nb32 = (int32_t)g.nbx, per32 = (int32_t)g.per, ncy32 = (int32_t)g.ncy;
    const char* nm = out ? (keys ? "k3m_matrix+keys" : "k3m_matrix") : "k3m_keys";
    if (!out) return klaunch(nm, k3m_matrix<PD, PR, VEC, false, false, true>, gr, blk, 0, st, a, c32, nb32, per32, ncy32);
    if constexpr (VEC == 1) {
        if (a.score && a.score_i64)
            return keys ? klaunch(nm, k3m_matrix<PD, PR, 1, true, true, true>, gr, blk, 0, st, a, c32, nb32, per32, ncy32)
                        : klaunch(nm, k3m_matrix<PD, PR, 1, true, true, false>, gr, blk, 0, st, a, c32, nb32, per32,
                                  ncy32);
    }
    return keys ? klaunch(nm, k3m_matrix<PD, PR, VEC, false, true, true>, gr, blk, 0, st, a, c32, nb32, per32, ncy32)
                : klaunch(nm, k3m_matrix<PD, PR, VEC, false, true, false>, gr, blk, 0, st, a, c32, nb32, per32, ncy32);
}

template <int PD, int PR>
static hipError_t launch_matrix_t(const MatrixArgs& a, hipStream_t st) {
    if (a.P <= 0 || a.N <= 0) return hipSuccess;
    const bool out = a.first_fail || a.score;
    const bool keys = a.keys != nullptr;
    if (!out && !keys) return hipSuccess;
    if (out && a.ld < a.N) return hipErrorInvalidValue;
    const MatrixGeometry g = matrix_geometry(a, out);
    if (g.nbx > 0x7FFFFFFF / 8 || g.ncy > 0x7FFFFFFF) return hipErrorInvalidValue;
    switch (g.vec) {
        case 8: return launch_vec<PD, PR, 8>(a, g, out, keys, st);
        case 4: return launch_vec<PD, PR, 4>(a, g, out, keys, st);
        default: return launch_vec<PD, PR, 1>(a, g, out, keys, st);
    }
}

hipError_t launch_matrix(int shape, const MatrixArgs& a, hipStream_t st) {
    switch (shape) {
        case kShape4x6: return launch_matrix_t<4, 6>(a, st);
        case kShape8x8: return launch_matrix_t<8, 8>(a, st);
        default: return launch_matrix_t<16, 16>(a, st);
    }
}

// ---------------------------------------------------------------- node answer tables
// The drop-in plugin's per-cycle answers as step functions of time (crane_dyn_node_steps):
// a node's Filter (first failing predicate) and Score change only where `now` crosses one
// of its expiries, so over [t0, t1) they are constant between the expiries inside it.  One
// thread per node: the expiries in (t0, t1), sorted and deduplicated, and the values at t0
// and at each of them (the same ff_at / score_at as every other path).  idx (subset form,
// crane_dyn_node_steps_subset): output row n holds node idx[n] (a.N = the subset's size).
template <int PD, int PR>
__global__ __launch_bounds__(256) void k_node_steps(MatrixArgs a, int64_t t0, int64_t t1, uint8_t* __restrict__ ns,
                                                    int64_t* __restrict__ bp, int8_t* __restrict__ ffv,
                                                    int8_t* __restrict__ scv, const int64_t* __restrict__ idx) {
    const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (n >= a.N) return;
    const NodeRec<PD, PR> r = static_cast<const NodeRec<PD, PR>*>(a.rec)[idx ? idx[n] : n];
    node_steps_row<PD, PR>(r, a, t0, t1, n, ns, bp, ffv, scv);
}

int node_step_slots(int shape) {
    switch (shape) {
        case kShape4x6: return 4 + 6 + 1;
        case kShape8x8: return 8 + 8 + 1;
        default: return 16 + 16 + 1;
    }
}

template <int PD, int PR>
static hipError_t steps_t(const MatrixArgs& a, int64_t t0, int64_t t1, uint8_t* ns, int64_t* bp, int8_t* ff,
                          int8_t* sc, const int64_t* idx, hipStream_t st) {
    return klaunch(idx ? "k_node_steps_subset" : "k_node_steps", k_node_steps<PD, PR>,
                   dim3((unsigned)((a.N + 255) / 256)), dim3(256), 0, st, a, t0, t1, ns, bp, ff, sc, idx);
}
hipError_t launch_node_steps(int shape, const MatrixArgs& a, int64_t t0, int64_t t1, uint8_t* ns, int64_t* bp,
                             int8_t* ff, int8_t* sc, hipStream_t st, const int64_t* idx) {
    if (a.N <= 0) return hipSuccess;
    switch (shape) {
        case kShape4x6: return steps_t<4, 6>(a, t0, t1, ns, bp, ff, sc, idx, st);
        case kShape8x8: return steps_t<8, 8>(a, t0, t1, ns, bp, ff, sc, idx, st);
        default: return steps_t<16, 16>(a, t0, t1, ns, bp, ff, sc, idx, st);
    }
}

}  // namespace crane
