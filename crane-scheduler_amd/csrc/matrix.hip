// matrix.hip — K3m: the per-pair form of Filter + Score (plugins.go:39-98).
//
// Every (pod, node) pair's result is materialised: the first failing predicate
// (Filter: -1 = Success, else its policy index; DaemonSet pods bypass,
// plugins.go:41-43) and the clamped Score, as [P][ld] matrices — what the
// drop-in plugin's per-node Filter/Score calls read back — and/or each pod's
// packed best key (chosen node).
//
// Layout: one lane per node (a workgroup = 256 consecutive nodes, 4 waves),
// each workgroup walks a chunk of pods in sub-chunks of 64.  A pod's time is
// wave-uniform (v_readlane into SGPRs), so every store instruction writes 64
// consecutive bytes of one matrix row.  For a node, Filter and Score depend on
// the pod only through `now < expiry` comparisons (stats.go:42-48): over a
// sub-chunk whose pod times lie in [cmin, cmax] a node with no expiry in
// (cmin, cmax] ("flat", almost every node) has one result for all 64 pods,
// computed once at cmin with the literal restatement (score_at, step_node.hpp);
// only a lane with an expiry inside evaluates per pod.  The per-pair cost is
// then the stores, and the kernel is bound by its output bytes.
//
// Keys: per pod, a wave max of (score << 24 | 0xFFFFFF - node) over its 64
// nodes, an LDS max over the workgroup's 4 waves, and one 64-bit atomicMax per
// pod per workgroup into keys[] (lowest global index wins ties).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dyn_types.hpp"
#include "kernels.hpp"
#include "step_node.hpp"

namespace crane {

constexpr int kMxT = 256;      // nodes per workgroup
constexpr int kMxChunk = 1024;  // max pods per workgroup (LDS best keys)

// first failing predicate at time t, in policy order (plugins.go:55-66); -1 = none
template <int PD, int PR>
__device__ __forceinline__ int32_t ff_at(int64_t t, const NodeRec<PD, PR>& r, const MatrixArgs& a) {
    int32_t f = -1;
#pragma unroll
    for (int k = PD - 1; k >= 0; --k)
        if (t < r.e_pred[k]) f = a.pred_orig[k];
    return f;
}

__device__ __forceinline__ int64_t readlane64(int64_t v, int j) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, j);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), j);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int32_t wave_max32(int32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

template <int PD, int PR, typename ST, bool OUT, bool KEYS>
__global__ __launch_bounds__(kMxT) void k3m_matrix(MatrixArgs a, int32_t chunk, int32_t nbx, int32_t per,
                                                   int32_t ncy) {
    __shared__ int32_t best[KEYS ? kMxChunk : 1];
    // XCD-aware: XCD x (= workgroup id % 8) takes node blocks [x*per, (x+1)*per) of every chunk,
    // so each XCD's L2 holds 1/8 of the record table
    const int64_t b = blockIdx.x, q = b >> 3;
    const int32_t nb = (int32_t)((b & 7) * per + q % per), cy = (int32_t)(q / per);
    if (nb >= nbx || cy >= ncy) return;  // (whole workgroup: no barrier is skipped by part of it)
    const int64_t n = (int64_t)nb * kMxT + threadIdx.x;
    const bool live = n < a.N;
    const int64_t p0 = (int64_t)cy * chunk, p1 = min(a.P, p0 + chunk);
    const int lane = threadIdx.x & 63;
    if (KEYS) {
        for (int i = threadIdx.x; i < chunk; i += kMxT) best[i] = -1;
        __syncthreads();
    }
    NodeRec<PD, PR> r;
    if (live) r = static_cast<const NodeRec<PD, PR>*>(a.rec)[n];
    ST* __restrict__ sout = static_cast<ST*>(a.score);
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
        // flat: no expiry of the node inside (cmin, cmax]
        bool stepped = false;
        int32_t f0 = -1, s0 = 0;
        if (live) {
            auto in = [&](int64_t e) { return e > cmin && e <= cmax; };
#pragma unroll
            for (int k = 0; k < PD; ++k) stepped |= in(r.e_pred[k]);
#pragma unroll
            for (int k = 0; k < PR; ++k) stepped |= in(r.e_prio[k]);
            stepped |= in(r.e_hv);
            f0 = ff_at<PD, PR>(cmin, r, a);
            s0 = score_at<PD, PR>(cmin, r, a.wsum, a.noprio);
        }
        const int32_t k0 = live ? pack_key(s0, threadIdx.x) : -1;
        const bool any_stepped = __ballot(stepped) != 0;
        int32_t kn = -1, kd = -1;  // wave maxima of the flat keys per pod kind
        if (KEYS && !any_stepped) {
            kn = wave_max32(f0 < 0 ? k0 : -1);
            kd = wave_max32(k0);
        }
        for (int j = 0; j < nv; ++j) {
            const bool d = __builtin_amdgcn_readlane(fl, j) != 0;
            int32_t f = f0, s = s0;
            if (stepped) {
                const int64_t t = readlane64(tn, j);
                f = ff_at<PD, PR>(t, r, a);
                s = score_at<PD, PR>(t, r, a.wsum, a.noprio);
            }
            if (OUT && live) {
                const int64_t o = (q0 + j) * a.ld + n;
                if (a.first_fail) a.first_fail[o] = (int8_t)(d ? -1 : f);
                if (sout) sout[o] = (ST)s;
            }
            if (KEYS) {
                int32_t k;
                if (any_stepped) k = wave_max32(live && (d || f < 0) ? pack_key(s, threadIdx.x) : -1);
                else k = d ? kd : kn;
                if (lane == 0 && k >= 0) atomicMax(&best[q0 + j - p0], k);
            }
        }
    }
    if (KEYS) {
        __syncthreads();
        for (int i = threadIdx.x; i < (int)(p1 - p0); i += kMxT) {
            const int32_t k = best[i];
            if (k < 0) continue;
            const int64_t sc = k >> 24;
            const int64_t g = a.node_offset + (int64_t)nb * kMxT + (0xFFFFFF - (k & 0xFFFFFF));
            atomicMax(&a.keys[p0 + i], (long long)((sc << 32) | (int64_t)(0xFFFFFFFFull - (uint64_t)g)));
        }
    }
}

template <int PD, int PR>
static hipError_t launch_matrix_t(const MatrixArgs& a, hipStream_t st) {
    if (a.P <= 0 || a.N <= 0) return hipSuccess;
    const bool out = a.first_fail || a.score;
    const bool keys = a.keys != nullptr;
    if (!out && !keys) return hipSuccess;
    if (out && a.ld < a.N) return hipErrorInvalidValue;
    const int64_t nbx = (a.N + kMxT - 1) / kMxT;
    if (nbx > 0x7FFFFFFF / 8) return hipErrorInvalidValue;
    // about two rounds of workgroups over the chip (256 CUs x 8 resident); pods per
    // workgroup a multiple of the 64-pod sub-chunk (or all of a smaller batch)
    const int64_t want_cy = std::max<int64_t>(1, 4096 / nbx);
    int64_t chunk = (a.P + want_cy - 1) / want_cy;
    chunk = a.P <= 64 ? a.P : std::min<int64_t>(kMxChunk, std::max<int64_t>(64, (chunk + 63) / 64 * 64));
    const int64_t ncy = (a.P + chunk - 1) / chunk;
    const int64_t per = (nbx + 7) / 8;
    const int64_t grid = 8 * per * ncy;
    if (grid > 0x7FFFFFFF || ncy > 0x7FFFFFFF) return hipErrorInvalidValue;
    const dim3 g((unsigned)grid), blk(kMxT);
    const int32_t c32 = (int32_t)chunk, nb32 = (int32_t)nbx, per32 = (int32_t)per, ncy32 = (int32_t)ncy;
    const char* nm = out ? (keys ? "k3m_matrix+keys" : "k3m_matrix") : "k3m_keys";
    if (!out) return klaunch(nm, k3m_matrix<PD, PR, int8_t, false, true>, g, blk, 0, st, a, c32, nb32, per32, ncy32);
    if (a.score && a.score_i64) {
        return keys ? klaunch(nm, k3m_matrix<PD, PR, int64_t, true, true>, g, blk, 0, st, a, c32, nb32, per32, ncy32)
                    : klaunch(nm, k3m_matrix<PD, PR, int64_t, true, false>, g, blk, 0, st, a, c32, nb32, per32, ncy32);
    }
    return keys ? klaunch(nm, k3m_matrix<PD, PR, int8_t, true, true>, g, blk, 0, st, a, c32, nb32, per32, ncy32)
                : klaunch(nm, k3m_matrix<PD, PR, int8_t, true, false>, g, blk, 0, st, a, c32, nb32, per32, ncy32);
}

hipError_t launch_matrix(int shape, const MatrixArgs& a, hipStream_t st) {
    switch (shape) {
        case kShape4x6: return launch_matrix_t<4, 6>(a, st);
        case kShape8x8: return launch_matrix_t<8, 8>(a, st);
        default: return launch_matrix_t<16, 16>(a, st);
    }
}

}  // namespace crane
