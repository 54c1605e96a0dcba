// hotcount.hip — K2: binding records -> per-node window counts, two forms.
//
// Each binding b counts for node n in the windows whose cutoff (now_unix -
// int64(timeRange.Seconds()), binding.go:85) is < ts_b; with the cutoffs
// sorted that set is a prefix 0..j-1, so one count per binding goes to bucket
// j-1 and K1 forms GetLastNodeBindingCount per window by suffix sums.
//
// Dedupe form (default, one launch): each 1024-thread workgroup aggregates a
//   2048-binding region per (node, bucket) in an LDS hash and writes one entry
//   per distinct pair, binned by K1 node block, plus a coalesced row of
//   (count, offset) words; K1 counts its own block's entries in LDS.  No global
//   atomics, no bucket matrix.
// Large form (past the dedupe form's count/offset cap, e.g. 4M nodes x 16M bindings): the same
//   region pass with coarse bins, then one workgroup per bin writes its rows of a dense bucket
//   matrix.  The atomics form (kernels.hip, k2_hot_count) takes any shape past the large form's caps.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dyn_types.hpp"
#include "kernels.hpp"
#include "pods.hpp"
#include "lds_hash.hpp"
#include "step_node.hpp"

namespace crane {

__device__ __forceinline__ int window_rank(int64_t ts, const HotCutoffs& cut) {
    int j = 0;
#pragma unroll
    for (int w = 0; w < kMaxWin; ++w)
        if (w < cut.n_win) j += ts > cut.sorted[w] ? 1 : 0;
    return j;  // 0: in no window
}

constexpr int kXChunk = kHxRegion;  // bindings per dedupe-form workgroup (K1 reads the regions with this stride)

// ---------------------------------------------------------------- dedupe form
// X' partition_dedupe : as X, but each workgroup first aggregates its 2048
//                bindings per (node, bucket) in an LDS hash table and writes one
//                entry per distinct pair: local node | bucket << 16 | count << 19.
//                Bins are the node pass's producer blocks (2^bb = K1's
//                workgroup size), so there is no Y: the node pass (kernels.hip,
//                K1Args::hx_*) counts its own block's entries into LDS.
// Aggregation bounds a Zipf-hot node to one entry per source region, so every
// bin's entry list stays short (the partitioned form needs 16 Y workgroups per
// bin for the hottest bins instead).

template <int BT, bool POS>
__device__ __forceinline__ void k2d_body(const int32_t blk, const int32_t* __restrict__ bnode,
                                         const int64_t* __restrict__ bts, int64_t B, int64_t N, const HotCutoffs& cut,
                                         const HotPart& g, uint32_t* __restrict__ CO, uint32_t* __restrict__ region) {
    // hkey, hcnt [kDSlots], hist, off [nbins], uniq u16 [kXChunk]
    extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
    constexpr int kPer = kXChunk / BT;  // bindings per thread
    __shared__ uint32_t part[BT];
    int32_t* hkey = reinterpret_cast<int32_t*>(sh);
    uint32_t* hcnt = sh + kDSlots;
    uint32_t* hist = hcnt + kDSlots;
    uint32_t* off = hist + g.nbins;
    uint16_t* uniq = reinterpret_cast<uint16_t*>(off + g.nbins);
    CRANE_TSTAMP(g.trace, blk, 0);
    const int64_t b0 = (int64_t)blk * kXChunk + threadIdx.x;
    int32_t nd[kPer];
    int64_t ts[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {  // unconditional loads (clamped index): all in flight at once
        const int64_t b = b0 + u * BT, bc = min(b, B - 1);
        nd[u] = bnode[bc];
        ts[u] = POS ? b : bts[bc];  // POS: the window rank from the position, no stamp loaded
        if (b >= B) nd[u] = -1;
    }
    for (int i = threadIdx.x; i < kDSlots; i += BT) {
        hkey[i] = -1;
        hcnt[i] = 0;
    }
    for (int i = threadIdx.x; i < g.nbins; i += BT) hist[i] = 0;
    __syncthreads();
    CRANE_TSTAMP(g.trace, blk, 1);
    int32_t key[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        const int j = window_rank(ts[u], cut);
        const bool ok = nd[u] >= 0 && (int64_t)nd[u] < N && j > 0;  // binding.go:85-91
        key[u] = ok ? nd[u] * 8 + (j - 1) : -1;
    }
    uint16_t* useg = uniq + (threadIdx.x >> 6) * (kPer * 64);
    const uint32_t nw = wave_aggregate<kDSlots, kPer>(key, hkey, hcnt, hist, g.bb, useg);
    __syncthreads();
    CRANE_TSTAMP(g.trace, blk, 2);
    const int per = (g.nbins + BT - 1) / BT;
    const int lo = min(g.nbins, (int)threadIdx.x * per), hi = min(g.nbins, lo + per);
    uint32_t sum = 0;
    for (int i = lo; i < hi; ++i) sum += hist[i];
    uint32_t run = wg_excl_scan_u32<BT>(sum, part);
    for (int i = lo; i < hi; ++i) {
        const uint32_t c = hist[i];
        off[i] = run;
        run += c;
    }
    __syncthreads();
    // this region's row of (count | offset << 16) per node block: coalesced (CO [nblk][nbins];
    // the column-major layout, contiguous for the readers, made this launch 10 % slower at
    // config 3 and cost K1 as much as it saved)
    for (int i = threadIdx.x; i < g.nbins; i += BT) CO[(int64_t)blk * g.nbins + i] = hist[i] | (off[i] << 16);
    __syncthreads();
    CRANE_TSTAMP(g.trace, blk, 3);
    uint32_t* reg = region + (int64_t)blk * kXChunk;
    const uint32_t mask = (1u << g.bb) - 1;
    for (uint32_t i = threadIdx.x & 63; i < nw; i += 64) {  // this wave's new keys
        const int s = useg[i];
        const int32_t k = hkey[s];
        const uint32_t p = atomicAdd(&off[(k >> 3) >> g.bb], 1u);
        reg[p] = ((uint32_t)(k >> 3) & mask) | ((uint32_t)(k & 7) << 16) | (hcnt[s] << 19);
    }
    CRANE_TSTAMP(g.trace, blk, 4);
}

// The launch is one round of workgroups at config 3, so one batch's time is one
// workgroup's dependent chain and wider workgroups shorten it; with several batches
// in flight the idle waves of the widest cost throughput.  Engine option k2x_threads,
// default 512 (config 3, one batch / 4 in flight: 1024 -> 0.0399 / 0.0168 ms per
// step, 512 -> 0.0407 / 0.0141, 256 -> 0.0446 / 0.0147; tools/inflight_sweep.sh).
template <int BT, bool POS>
__global__ __launch_bounds__(BT) void k2x_dedupe(const int32_t* __restrict__ bnode, const int64_t* __restrict__ bts,
                                                 int64_t B, int64_t N, HotCutoffs cut, HotPart g,
                                                 uint32_t* __restrict__ CO, uint32_t* __restrict__ region) {
    k2d_body<BT, POS>((int32_t)blockIdx.x, bnode, bts, B, N, cut, g, CO, region);
}

template <int BT, bool POS>
__global__ __launch_bounds__(BT) void k2x_dedupe_pods(const int32_t* __restrict__ bnode,
                                                      const int64_t* __restrict__ bts, int64_t B, int64_t N,
                                                      HotCutoffs cut, HotPart g, uint32_t* __restrict__ CO,
                                                      uint32_t* __restrict__ region, PodPrep pp) {
    // the pod tiles first: dispatched first, their sort overlaps the regions' aggregation
    // instead of trailing the launch
    if ((int64_t)blockIdx.x >= pp.ntiles) {
        k2d_body<BT, POS>((int32_t)(blockIdx.x - pp.ntiles), bnode, bts, B, N, cut, g, CO, region);
    } else {
        extern __shared__ __attribute__((aligned(16))) unsigned char k3p_lds[];
        k3p_tile<BT>((int64_t)blockIdx.x, pp, k3p_lds);
    }
}

HotPart hot_dedupe_geometry(int64_t B, int64_t N, int32_t W, int32_t bs) {
    HotPart g{};
    int bb = 0;
    while ((1 << bb) < bs) ++bb;
    g.bb = bb;
    g.nbins = (int32_t)((N + bs - 1) / bs);
    g.nblk = (int32_t)((B + kXChunk - 1) / kXChunk);
    g.reg = kXChunk;
    g.cap = (int64_t)g.nblk * kXChunk;
    // key nd*8+bucket in int32; hash + bin LDS <= 96 KiB; count/offset matrices <= 2^22 entries
    g.ok = N > 0 && B > 0 && (1 << bb) == bs && bb <= 16 && W >= 1 && W <= kMaxWin && N < (1LL << 27) &&
           g.nbins <= 8192 && (double)g.nbins * (double)g.nblk <= (double)(1 << 22);
    return g;
}

template <int BT, bool POS>
static hipError_t launch_dedupe_t(const int32_t* bnode, const int64_t* bts, int64_t B, int64_t N,
                                  const HotCutoffs& cut, const HotPart& g, uint32_t* scratch, hipStream_t st,
                                  const PodPrep* pods) {
    static const hipError_t attr = [] {
        hipError_t e = hipFuncSetAttribute((const void*)k2x_dedupe<BT, POS>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
        if (e == hipSuccess)
            e = hipFuncSetAttribute((const void*)k2x_dedupe_pods<BT, POS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    100 * 1024);
        return e;
    }();
    if (attr != hipSuccess) return attr;
    uint32_t* region = scratch;
    uint32_t* CO = scratch + g.cap;  // [nblk][nbins]
    size_t lds = sizeof(uint32_t) * (2 * (size_t)kDSlots + 2 * (size_t)g.nbins) + sizeof(uint16_t) * kXChunk;
    if (pods && pods->P > 0) lds = std::max(lds, kK3pLds);
    if (pods && pods->P > 0)
        return klaunch("k2x_dedupe+k3p_pods", k2x_dedupe_pods<BT, POS>, dim3((unsigned)(g.nblk + pods->ntiles)),
                       dim3(BT), lds, st, bnode, bts, B, N, cut, g, CO, region, *pods);
    return klaunch("k2x_dedupe", k2x_dedupe<BT, POS>, dim3((unsigned)g.nblk), dim3(BT), lds, st, bnode, bts, B, N, cut,
                   g, CO, region);
}

template <int BT>
static hipError_t launch_dedupe_p(const int32_t* bnode, const int64_t* bts, int64_t B, int64_t N,
                                  const HotCutoffs& cut, const HotPart& g, uint32_t* scratch, hipStream_t st,
                                  const PodPrep* pods) {
    return cut.by_pos ? launch_dedupe_t<BT, true>(bnode, bts, B, N, cut, g, scratch, st, pods)
                      : launch_dedupe_t<BT, false>(bnode, bts, B, N, cut, g, scratch, st, pods);
}

hipError_t launch_hot_count_dedupe(const int32_t* bnode, const int64_t* bts, int64_t B, int64_t N,
                                   const HotCutoffs& cut, const HotPart& g, uint32_t* scratch, hipStream_t st,
                                   const PodPrep* pods, int threads) {
    if (threads != 512) return hipErrorInvalidValue;  // (512: profiles/r05/config3_option_sweep_queues.txt)
    return launch_dedupe_p<512>(bnode, bts, B, N, cut, g, scratch, st, pods);
}

size_t hot_dedupe_scratch(const HotPart& g) { return (size_t)g.cap + (size_t)g.nbins * (size_t)g.nblk; }

template <int BT>
__global__ __launch_bounds__(BT) void k2_delta_pods(const int32_t* __restrict__ bnode, int64_t N, HotDelta d,
                                                    uint32_t* __restrict__ adj, PodPrep pp) {
    CRANE_TSTAMP(d.trace, blockIdx.x, 0);
    if ((int64_t)blockIdx.x >= pp.ntiles) {
        k2_delta_body<BT>((int32_t)(blockIdx.x - pp.ntiles), bnode, N, d, adj);
    } else {
        extern __shared__ __attribute__((aligned(16))) unsigned char k3p_lds[];
        k3p_tile<BT>((int64_t)blockIdx.x, pp, k3p_lds);
    }
    for (int k = 1; k <= 4; ++k) CRANE_TSTAMP(d.trace, blockIdx.x, k);  // (one phase: start -> end)
}

hipError_t launch_hot_count_delta(const int32_t* bnode, int64_t N, const HotDelta& d, uint32_t* adj, hipStream_t st,
                                  const PodPrep* pods) {
    constexpr int BT = 512;
    if (d.n_rng < 0 || d.n_rng > kMaxWin || d.n_win < 1 || d.n_win > kDeltaMaxWin || N >= (1LL << 27))
        return hipErrorInvalidValue;
    const int64_t L = d.n_rng > 0 ? d.start[d.n_rng] : 0;
    const int64_t nb = (L + kDeltaChunk - 1) / kDeltaChunk;
    PodPrep pp{};
    if (pods && pods->P > 0) pp = *pods;
    const int64_t grid = pp.ntiles + nb;
    if (grid == 0) return hipSuccess;
    if (grid >= (1LL << 31)) return hipErrorInvalidValue;
    size_t lds = sizeof(uint32_t) * 2 * (size_t)kDeltaSlots + sizeof(uint16_t) * kDeltaMaxWin * kDeltaChunk;
    if (pp.ntiles > 0) lds = std::max(lds, kK3pLds);
    return klaunch(pp.ntiles > 0 ? "k2_delta+k3p_pods" : "k2_delta", k2_delta_pods<BT>, dim3((unsigned)grid), dim3(BT),
                   lds, st, bnode, N, d, adj, pp);
}

// ---------------------------------------------------------------- large form
// When the dedupe form's count/offset matrix (K1 blocks x regions) would pass its cap
// (e.g. 4M nodes x 16M bindings: 15,625 x 7,813 words), the log goes through two kernels:
//   X  k2l_partition: the dedupe form's region pass (per region of REG bindings: LDS hash
//      aggregation per (node, bucket) — a Zipf-hot node costs one entry per region — then
//      the distinct entries binned) with COARSE bins of 2^bb nodes (16K at two windows:
//      245 bins at 4M nodes); persistent: each workgroup walks regions blockIdx, + grid, ...
//      and loads the next region's bindings while it aggregates the current one, and
//      clears only the hash slots it used;
//   Y  k2y_bin_hist: one workgroup per coarse bin gathers the bin's entries from every
//      region (the count/offset words, then the runs) into an LDS histogram [W][2^bb] and
//      writes the bin's rows of buckets [W][N] whole — no global atomics, nothing to zero
//      (K1 reads them and leaves them, K1Args::buckets_keep).
// Count/offset words: CO [nblk][nbins] (X writes its row coalesced, Y reads a column; the
// transposed layout measured no better, profiles/ab/r03_k2_cold_*.txt).
// POS: a time-ordered log ranked by position (HotCutoffs::by_pos): no timestamp loads (a
// template parameter: a load inside a run-time branch makes the compiler wait for every load
// at the join, which serialised the next region's prefetch)
template <int BT, int REG, bool POS>
__global__ __launch_bounds__(BT) __attribute__((amdgpu_waves_per_eu(BT == 1024 ? 8 : 1)))
void k2l_partition(const int32_t* __restrict__ bnode,
                                                    const int64_t* __restrict__ bts, int64_t B, int64_t N,
                                                    HotCutoffs cut, HotPart g, uint32_t* __restrict__ CO,
                                                    uint32_t* __restrict__ region) {
    constexpr int kPer = REG / BT;   // bindings per thread per region
    constexpr int kSlots = 2 * REG;  // an empty or matching slot always exists
    // hkey, hcnt [kSlots], hist, off [nbins], uniq u16 [REG]
    extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
    __shared__ uint32_t part[BT];
    int32_t* hkey = reinterpret_cast<int32_t*>(sh);
    uint32_t* hcnt = sh + kSlots;
    uint32_t* hist = hcnt + kSlots;
    uint32_t* off = hist + g.nbins;
    uint16_t* useg = reinterpret_cast<uint16_t*>(off + g.nbins) + (threadIdx.x >> 6) * (kPer * 64);
    for (int i = threadIdx.x; i < kSlots; i += BT) {
        hkey[i] = -1;
        hcnt[i] = 0;
    }
    for (int i = threadIdx.x; i < g.nbins; i += BT) hist[i] = 0;
    auto load = [&](int64_t r, int32_t* nd, int64_t* ts) {  // unconditional loads, clamped index
        const int64_t b0 = r * REG + threadIdx.x;
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int64_t b = b0 + u * BT, bc = min(b, B - 1);
            nd[u] = bnode[bc];
            ts[u] = POS ? b : bts[bc];
            if (b >= B) nd[u] = -1;
        }
    };
    int32_t nd[kPer];
    int64_t ts[kPer];
    int64_t r = blockIdx.x;  // (grid <= nblk)
    load(r, nd, ts);
    __syncthreads();
    const uint32_t mask = (1u << g.bb) - 1;
    const int per = (g.nbins + BT - 1) / BT;
    const int lo = min(g.nbins, (int)threadIdx.x * per), hi = min(g.nbins, lo + per);
    for (;;) {
        const int64_t r2 = r + gridDim.x;
        int32_t nd2[kPer];
        int64_t ts2[kPer];
        load(min(r2, (int64_t)g.nblk - 1), nd2, ts2);  // the next region, in flight meanwhile
        CRANE_TSTAMP(g.trace, r, 0);
        int32_t key[kPer];
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int j = window_rank(ts[u], cut);
            const bool ok = nd[u] >= 0 && (int64_t)nd[u] < N && j > 0;  // binding.go:85-91
            key[u] = ok ? nd[u] * 8 + (j - 1) : -1;
        }
        const uint32_t nw = wave_aggregate<kSlots, kPer>(key, hkey, hcnt, hist, g.bb, useg);
        __syncthreads();
        CRANE_TSTAMP(g.trace, r, 1);
        uint32_t sum = 0;
        for (int i = lo; i < hi; ++i) sum += hist[i];
        uint32_t run = wg_excl_scan_u32<BT>(sum, part);
        for (int i = lo; i < hi; ++i) {  // offsets + this region's count/offset words; hist cleared
            const uint32_t c = hist[i];
            off[i] = run;
            CO[r * g.nbins + i] = c | (run << 16);
            hist[i] = 0;
            run += c;
        }
        __syncthreads();
        CRANE_TSTAMP(g.trace, r, 2);
        uint32_t* reg = region + r * REG;
        for (uint32_t i = threadIdx.x & 63; i < nw; i += 64) {  // this wave's entries; its slots cleared
            const int s = useg[i];
            const int32_t k = hkey[s];
            const uint32_t cnt = hcnt[s];
            hkey[s] = -1;
            hcnt[s] = 0;
            const uint32_t p = atomicAdd(&off[(k >> 3) >> g.bb], 1u);
            reg[p] = ((uint32_t)(k >> 3) & mask) | ((uint32_t)(k & 7) << 16) | (cnt << 19);
        }
        __syncthreads();
        CRANE_TSTAMP(g.trace, r, 3);
        r = r2;
        if (r >= g.nblk) break;
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            nd[u] = nd2[u];
            ts[u] = ts2[u];
        }
    }
}

constexpr int kYThreads = 1024;
// YPER regions per lane per round (4,096-binding regions at 16M bindings: 3,907, one round of
// 4), YFIRST aligned 16-byte blocks of each run loaded in the count/offset words' round, the
// rest queued
constexpr int kYQ = 2048;    // LDS queue of the longer runs' tails

// Every load is unconditional (clamped index, result masked): conditional loads made the
// compiler wait for each one before issuing the next.
template <int kYPer, int kYFirst>
__global__ __launch_bounds__(kYThreads) void k2y_bin_hist(const uint32_t* __restrict__ region,
                                                          const uint32_t* __restrict__ CO, HotPart g, int32_t W,
                                                          int64_t N, uint32_t* __restrict__ buckets) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];  // [W][2^bb]
    __shared__ uint2 q[kYQ];  // tail of a run: {first entry index, entries left}
    __shared__ uint32_t qn;
    const int bb = g.bb, binw = 1 << bb;
    const int64_t bin = xcd_block(blockIdx.x, gridDim.x);
    const uint32_t lmask = (uint32_t)binw - 1;
    auto add = [&](uint32_t v) { atomicAdd(&hist[((v >> 16) & 7) * binw + (v & lmask)], v >> 19); };
    CRANE_TSTAMP(g.trace, bin, 4);  // (trace row = bin; the partition's rows use slots 0-3)
    for (int i0 = 0; i0 < g.nblk; i0 += kYThreads * kYPer) {
        // this bin's (count, offset) word of kYPer regions per lane, then their runs' first entries
        uint32_t c[kYPer], o[kYPer];
#pragma unroll
        for (int u = 0; u < kYPer; ++u) {
            const int i = i0 + u * kYThreads + threadIdx.x;
            const int ic = min(i, g.nblk - 1);
            const uint32_t co = CO[(int64_t)ic * g.nbins + bin];
            c[u] = i < g.nblk ? co & 0xFFFF : 0u;
            o[u] = co >> 16;
        }
        // each run as aligned 16-byte blocks: a run of up to 4 * YFIRST - 3 entries costs its
        // one or two lines in YFIRST load instructions (per-entry loads cost a line per
        // instruction: the gather was bound by the lines the loads touch); blocks past a
        // run's end load block 0 (one line shared by the wave)
        const uint4* __restrict__ region4 = reinterpret_cast<const uint4*>(region);
        uint4 v[kYPer][kYFirst];
        uint32_t a0[kYPer];
#pragma unroll
        for (int u = 0; u < kYPer; ++u) {
            const uint32_t e0 = (uint32_t)(i0 + u * kYThreads + threadIdx.x) * (uint32_t)g.reg + o[u];
            a0[u] = e0 & ~3u;
            const uint32_t nb = c[u] ? ((e0 & 3u) + c[u] + 3u) >> 2 : 0u;
#pragma unroll
            for (int k = 0; k < kYFirst; ++k) v[u][k] = region4[(uint32_t)k < nb ? (a0[u] >> 2) + k : 0u];
        }
        if (i0 == 0) {
            uint4* h4 = reinterpret_cast<uint4*>(hist);
            const int n4 = (W * binw) >> 2;
            for (int i = threadIdx.x; i < n4; i += kYThreads) h4[i] = make_uint4(0u, 0u, 0u, 0u);
        }
        if (threadIdx.x == 0) qn = 0;
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kYPer; ++u) {
            const uint32_t e0 = a0[u] + (o[u] & 3u), e1 = e0 + c[u];  // the run: [e0, e1)
#pragma unroll
            for (int k = 0; k < kYFirst; ++k) {
                const uint32_t b = a0[u] + 4u * k;
                if (b + 0 >= e0 && b + 0 < e1) add(v[u][k].x);
                if (b + 1 >= e0 && b + 1 < e1) add(v[u][k].y);
                if (b + 2 >= e0 && b + 2 < e1) add(v[u][k].z);
                if (b + 3 >= e0 && b + 3 < e1) add(v[u][k].w);
            }
            const uint32_t done = a0[u] + 4u * kYFirst;
            if (e1 > done) {  // the rest of a longer run: queued for the whole workgroup
                const uint32_t p = atomicAdd(&qn, 1u);
                if (p < (uint32_t)kYQ) {
                    q[p] = make_uint2(done, e1 - done);
                } else {  // queue full: this lane walks it
                    for (uint32_t e = done; e < e1; ++e) add(region[e]);
                }
            }
        }
        __syncthreads();
        const uint32_t nq = min(qn, (uint32_t)kYQ);
        for (uint32_t j = threadIdx.x; j < nq; j += kYThreads) {
            const uint2 it = q[j];
            for (uint32_t k0 = 0; k0 < it.y; k0 += 8) {
                uint32_t w[8];
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) w[jj] = region[k0 + jj < it.y ? (int64_t)it.x + k0 + jj : 0];
#pragma unroll
                for (int jj = 0; jj < 8; ++jj)
                    if (k0 + jj < it.y) add(w[jj]);
            }
        }
        __syncthreads();  // (qn / q reused by the next round; hist complete after the last)
    }
    CRANE_TSTAMP(g.trace, bin, 5);
    // the bin's rows, whole: lane i -> node n0 + i
    const int64_t n0 = bin << bb;
    const int nn = (int)min((int64_t)binw, N - n0);
    for (int w = 0; w < W; ++w)
        for (int i = threadIdx.x; i < nn; i += kYThreads) buckets[(int64_t)w * N + n0 + i] = hist[w * binw + i];
    CRANE_TSTAMP(g.trace, bin, 6);
}

HotPart hot_large_geometry(int64_t B, int64_t N, int32_t W) {
    HotPart g{};
    int bb = 16;  // entry format: local node in 16 bits
    while (bb > 8 && (int64_t)std::max(W, 1) * (4LL << bb) > kK2LargeHistBytes) --bb;  // Y's LDS histogram
    g.bb = bb;
    g.reg = kK2lRegion;
    g.nbins = (int32_t)((N + (1LL << bb) - 1) >> bb);
    g.nblk = (int32_t)((B + g.reg - 1) / g.reg);
    g.cap = (int64_t)g.nblk * g.reg;
    // (count <= reg < 2^13 in an entry's top bits and in a count/offset half-word)
    g.ok = N > 0 && B > 0 && W >= 1 && W <= kMaxWin && N < (1LL << 27) && B < (1LL << 31) && g.nbins <= 4096 &&
           (double)g.nbins * (double)g.nblk <= (double)(1LL << 27);
    return g;
}

template <int BT, int REG, bool POS>
static hipError_t launch_large_xp(const int32_t* bnode, const int64_t* bts, int64_t B, int64_t N,
                                  const HotCutoffs& cut, const HotPart& g, uint32_t* scratch, int n_cu,
                                  hipStream_t st) {
    const size_t lds = sizeof(uint32_t) * (4 * (size_t)REG + 2 * (size_t)g.nbins) + sizeof(uint16_t) * REG;
    static const hipError_t attr =
        hipFuncSetAttribute((const void*)k2l_partition<BT, REG, POS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            100 * 1024);
    if (attr != hipSuccess) return attr;
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k2l_partition<BT, REG, POS>, BT,
                                                               lds);
    if (e != hipSuccess) return e;
    const int64_t grid = std::min<int64_t>(g.nblk, (int64_t)std::max(1, per_cu) * std::max(1, n_cu));
    return klaunch("k2l_partition", k2l_partition<BT, REG, POS>, dim3((unsigned)grid), dim3(BT), lds, st, bnode, bts,
                   B, N, cut, g, scratch + g.cap, scratch);
}

template <int BT, int REG>
static hipError_t launch_large_x(const int32_t* bnode, const int64_t* bts, int64_t B, int64_t N,
                                 const HotCutoffs& cut, const HotPart& g, uint32_t* scratch, int n_cu,
                                 hipStream_t st) {
    return cut.by_pos ? launch_large_xp<BT, REG, true>(bnode, bts, B, N, cut, g, scratch, n_cu, st)
                      : launch_large_xp<BT, REG, false>(bnode, bts, B, N, cut, g, scratch, n_cu, st);
}

template <int kYPer, int kYFirst>
static hipError_t launch_y(const uint32_t* scratch, const HotPart& g, int32_t W, int64_t N, uint32_t* buckets,
                           hipStream_t st) {
    // (dynamic + the static tail queue stay within the CU's 160 KiB)
    static const hipError_t attr = hipFuncSetAttribute((const void*)k2y_bin_hist<kYPer, kYFirst>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)kK2LargeHistBytes);
    if (attr != hipSuccess) return attr;
    const size_t lds = sizeof(uint32_t) * (size_t)W * ((size_t)1 << g.bb);
    return klaunch("k2y_bin_hist", k2y_bin_hist<kYPer, kYFirst>, dim3((unsigned)g.nbins), dim3(kYThreads), lds, st,
                   scratch, scratch + g.cap, g, W, N, buckets);
}

hipError_t launch_hot_count_large(const int32_t* bnode, const int64_t* bts, int64_t B, int64_t N,
                                  const HotCutoffs& cut, const HotPart& g, uint32_t* scratch, uint32_t* buckets,
                                  int n_cu, hipStream_t st, int threads) {
    if (threads != 1024) return hipErrorInvalidValue;  // (1024 threads per 4096-binding region: round 3's sweep)
    hipError_t e = launch_large_x<1024, kK2lRegion>(bnode, bts, B, N, cut, g, scratch, n_cu, st);
    if (e != hipSuccess) return e;
    // kYPer = the fewest regions per lane that cover the log; kYFirst = the 16-byte blocks of each
    // run loaded in the count/offset words' round (round 4's sweep, profiles/r04/k2y_first.txt:
    // cold 4M x 16M ordered log k2y 0.019 ms at 3, 0.0165 at 6, as many as registers allow at
    // four and eight regions per lane)
    if (g.nblk > 4 * kYThreads) return launch_y<8, 2>(scratch, g, cut.n_win, N, buckets, st);
    if (g.nblk > 2 * kYThreads) return launch_y<4, 5>(scratch, g, cut.n_win, N, buckets, st);
    return launch_y<2, 6>(scratch, g, cut.n_win, N, buckets, st);
}

}  // namespace crane
