// hotcount.hip — K2 as a bin-partitioned, LDS-staged segmented count.
//
// Same result as kernels.hip's hash K2: buckets[j][n] += #bindings of node n
// whose timestamp lies in exactly the windows of sorted-cutoff ranks 0..j
// (binding.go:85-91), from which K1 forms GetLastNodeBindingCount per window.
// Instead of scattered device-scope atomics (≈17x slower than contiguous ones
// on MI355X), bindings are first partitioned by node range ("bins" of 2^BB
// nodes), then each bin is counted in a dense LDS histogram and flushed with
// contiguous atomics (lane i -> node i).
//   A  bin_count : chunk of bindings -> per-(bin, chunk) counts
//   B  bin_scan  : per bin, exclusive scan over chunks + bin total
//   C  scatter   : chunk of bindings -> bin-contiguous packed entries
//                  (local node | bucket << 24)
//   D  bin_hist  : (bin, split) -> LDS histogram [W][2^BB] -> buckets
// Order inside a bin is not deterministic; counts are.
#include <hip/hip_runtime.h>

#include "dyn_types.hpp"
#include "kernels.hpp"

namespace crane {

constexpr int kHT = 256;  // threads per workgroup in all four kernels

__device__ __forceinline__ int window_rank(int64_t ts, const HotCutoffs& cut) {
    int j = 0;
#pragma unroll
    for (int w = 0; w < kMaxWin; ++w)
        if (w < cut.n_win) j += ts > cut.sorted[w] ? 1 : 0;
    return j;  // 0: in no window
}

__global__ __launch_bounds__(kHT) void k2a_bin_count(const int32_t* __restrict__ bnode, const int64_t* __restrict__ bts,
                                                     int64_t B, int64_t N, HotCutoffs cut, HotBins g,
                                                     uint32_t* __restrict__ chunk_cnt) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];  // [nbins]
    for (int i = threadIdx.x; i < g.nbins; i += kHT) hist[i] = 0;
    __syncthreads();
    const int64_t b0 = (int64_t)blockIdx.x * g.chunk, b1 = min(B, b0 + g.chunk);
    for (int64_t b = b0 + threadIdx.x; b < b1; b += kHT) {
        const int32_t nd = bnode[b];
        if (nd < 0 || (int64_t)nd >= N || !window_rank(bts[b], cut)) continue;
        atomicAdd(&hist[nd >> g.bb], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < g.nbins; i += kHT) chunk_cnt[(int64_t)i * g.nchunks + blockIdx.x] = hist[i];
}

// exclusive scan of up to kHT*16 values in place; returns the total (block-wide)
__global__ __launch_bounds__(kHT) void k2b_bin_scan(uint32_t* __restrict__ chunk_cnt, HotBins g,
                                                    uint32_t* __restrict__ bin_tot) {
    __shared__ uint32_t part[kHT];
    uint32_t* row = chunk_cnt + (int64_t)blockIdx.x * g.nchunks;
    const int per = (g.nchunks + kHT - 1) / kHT;
    const int lo = threadIdx.x * per, hi = min(g.nchunks, lo + per);
    uint32_t s = 0;
    for (int i = lo; i < hi; ++i) s += row[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < kHT; off <<= 1) {  // Hillis-Steele inclusive scan of the partials
        const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
    for (int i = lo; i < hi; ++i) {
        const uint32_t v = row[i];
        row[i] = run;
        run += v;
    }
    if (threadIdx.x == kHT - 1) bin_tot[blockIdx.x] = part[kHT - 1];
}

// LDS exclusive scan of bin_tot[0..nbins) into base[] (nbins <= kMaxBins)
__device__ void scan_bins(const uint32_t* __restrict__ bin_tot, int nbins, uint32_t* base /*LDS*/,
                          uint32_t* part /*LDS kHT*/) {
    const int per = (nbins + kHT - 1) / kHT;
    const int lo = threadIdx.x * per, hi = min(nbins, lo + per);
    uint32_t s = 0;
    for (int i = lo; i < hi; ++i) s += bin_tot[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < kHT; off <<= 1) {
        const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
    for (int i = lo; i < hi; ++i) {
        base[i] = run;
        run += bin_tot[i];
    }
    __syncthreads();
}

__global__ __launch_bounds__(kHT) void k2c_scatter(const int32_t* __restrict__ bnode, const int64_t* __restrict__ bts,
                                                   int64_t B, int64_t N, HotCutoffs cut, HotBins g,
                                                   const uint32_t* __restrict__ chunk_off,
                                                   const uint32_t* __restrict__ bin_tot, uint32_t* __restrict__ sorted) {
    extern __shared__ __attribute__((aligned(16))) uint32_t cursor[];  // [nbins]
    __shared__ uint32_t part[kHT];
    scan_bins(bin_tot, g.nbins, cursor, part);
    for (int i = threadIdx.x; i < g.nbins; i += kHT) cursor[i] += chunk_off[(int64_t)i * g.nchunks + blockIdx.x];
    __syncthreads();
    const int64_t b0 = (int64_t)blockIdx.x * g.chunk, b1 = min(B, b0 + g.chunk);
    const uint32_t mask = (1u << g.bb) - 1;
    for (int64_t b = b0 + threadIdx.x; b < b1; b += kHT) {
        const int32_t nd = bnode[b];
        if (nd < 0 || (int64_t)nd >= N) continue;
        const int j = window_rank(bts[b], cut);
        if (!j) continue;
        const uint32_t pos = atomicAdd(&cursor[nd >> g.bb], 1u);
        sorted[pos] = ((uint32_t)nd & mask) | ((uint32_t)(j - 1) << 24);
    }
}

__global__ __launch_bounds__(kHT) void k2d_bin_hist(const uint32_t* __restrict__ sorted,
                                                    const uint32_t* __restrict__ bin_tot, HotBins g, int32_t W,
                                                    int64_t N, uint32_t* __restrict__ buckets) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];  // [W][binw]
    __shared__ uint32_t part[kHT];
    __shared__ uint32_t start_s;
    const int bin = blockIdx.x, split = blockIdx.y;
    // base of this bin = sum of the totals of the bins before it
    {
        uint32_t s = 0;
        for (int i = threadIdx.x; i < bin; i += kHT) s += bin_tot[i];
        part[threadIdx.x] = s;
        __syncthreads();
        for (int off = kHT / 2; off > 0; off >>= 1) {
            if (threadIdx.x < off) part[threadIdx.x] += part[threadIdx.x + off];
            __syncthreads();
        }
        if (threadIdx.x == 0) start_s = part[0];
    }
    const int binw = 1 << g.bb;
    for (int i = threadIdx.x; i < W * binw; i += kHT) hist[i] = 0;
    __syncthreads();
    const uint32_t len = bin_tot[bin], start = start_s;
    const uint32_t e0 = start + (uint32_t)((uint64_t)len * split / gridDim.y);
    const uint32_t e1 = start + (uint32_t)((uint64_t)len * (split + 1) / gridDim.y);
    for (uint32_t e = e0 + threadIdx.x; e < e1; e += kHT) {
        const uint32_t v = sorted[e];
        atomicAdd(&hist[(v >> 24) * binw + (v & 0xFFFFFF)], 1u);
    }
    __syncthreads();
    const int64_t n0 = (int64_t)bin << g.bb;
    for (int w = 0; w < W; ++w)
        for (int i = threadIdx.x; i < binw; i += kHT) {
            const uint32_t c = hist[w * binw + i];
            if (c && n0 + i < N) atomicAdd(&buckets[(int64_t)w * N + n0 + i], c);  // contiguous across lanes
        }
}

// ---------------------------------------------------------------- two-kernel form
// X  partition : each workgroup takes 2048 bindings (8 per thread, loads issued
//                together), counts them per node bin in LDS, reserves its run of
//                every bin region with ONE global atomic per bin, and writes
//                (local node | bucket << 24) entries into the bin regions.
//                Bin regions have capacity B, so no pre-count pass is needed.
// Y  bin_hist  : kYSplits workgroups per bin, each an LDS histogram [W][2^bb]
//                of a contiguous slice of the bin's entries, flushed with
//                contiguous atomics into the (zeroed) buckets.
// The per-bin cursors are zeroed by a memset in the same stream before X.
constexpr int kXPer = 8;     // bindings per thread in X
constexpr int kYSplits = 8;  // workgroups per bin in Y

__global__ __launch_bounds__(kHT) void k2x_partition(const int32_t* __restrict__ bnode,
                                                     const int64_t* __restrict__ bts, int64_t B, int64_t N,
                                                     HotCutoffs cut, HotPart g, uint32_t* __restrict__ cur,
                                                     uint32_t* __restrict__ region) {
    extern __shared__ __attribute__((aligned(16))) uint32_t sh[];  // hist [nbins], base [nbins]
    uint32_t* hist = sh;
    uint32_t* base = sh + g.nbins;
    for (int i = threadIdx.x; i < g.nbins; i += kHT) hist[i] = 0;
    __syncthreads();
    const int64_t b0 = (int64_t)blockIdx.x * (kHT * kXPer) + threadIdx.x;
    int32_t nd[kXPer];
    int64_t ts[kXPer];
#pragma unroll
    for (int u = 0; u < kXPer; ++u) {
        const int64_t b = b0 + u * kHT;
        nd[u] = b < B ? bnode[b] : -1;
        ts[u] = b < B ? bts[b] : INT64_MIN;
    }
    uint32_t ent[kXPer], pos[kXPer];
    int32_t bin[kXPer];
    const uint32_t mask = (1u << g.bb) - 1;
#pragma unroll
    for (int u = 0; u < kXPer; ++u) {
        const int j = window_rank(ts[u], cut);
        const bool ok = nd[u] >= 0 && (int64_t)nd[u] < N && j > 0;  // binding.go:85-91
        bin[u] = ok ? nd[u] >> g.bb : -1;
        ent[u] = ((uint32_t)nd[u] & mask) | ((uint32_t)(j - 1) << 24);
        pos[u] = ok ? atomicAdd(&hist[bin[u]], 1u) : 0u;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < g.nbins; i += kHT) {
        const uint32_t c = hist[i];
        base[i] = c ? atomicAdd(&cur[i], c) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kXPer; ++u)
        if (bin[u] >= 0) region[(int64_t)bin[u] * g.cap + base[bin[u]] + pos[u]] = ent[u];
}

__global__ __launch_bounds__(kHT) void k2y_bin_hist(const uint32_t* __restrict__ region,
                                                    const uint32_t* __restrict__ cur, HotPart g, int32_t W,
                                                    int64_t N, uint32_t* __restrict__ buckets) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];  // [W][2^bb]
    const int bin = blockIdx.x, split = blockIdx.y;
    const int binw = 1 << g.bb;
    for (int i = threadIdx.x; i < W * binw; i += kHT) hist[i] = 0;
    const uint32_t len = cur[bin];
    // contiguous 1/splits of the bin's entries: Zipf-hot bins spread over the splits
    const uint32_t lo = (uint32_t)((uint64_t)len * split / gridDim.y);
    const uint32_t hi = (uint32_t)((uint64_t)len * (split + 1) / gridDim.y);
    const uint32_t* __restrict__ r = region + (int64_t)bin * g.cap + lo;
    const uint32_t n_e = hi - lo;
    __syncthreads();
    for (uint32_t e0 = threadIdx.x; e0 < n_e; e0 += kHT * kXPer) {
        uint32_t v[kXPer];
#pragma unroll
        for (int u = 0; u < kXPer; ++u) {
            const uint32_t e = e0 + u * kHT;
            v[u] = e < n_e ? r[e] : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int u = 0; u < kXPer; ++u)
            if (v[u] != 0xFFFFFFFFu) atomicAdd(&hist[(v[u] >> 24) * binw + (v[u] & 0xFFFFFF)], 1u);
    }
    __syncthreads();
    // buckets are zero on entry (K1 zeroes what it consumes): add the non-zero
    // counts, lane i -> node i (contiguous atomics)
    const int64_t n0 = (int64_t)bin << g.bb;
    for (int w = 0; w < W; ++w)
        for (int i = threadIdx.x; i < binw; i += kHT) {
            const uint32_t c = hist[w * binw + i];
            if (c && n0 + i < N) atomicAdd(&buckets[(int64_t)w * N + n0 + i], c);
        }
}

HotPart hot_part_geometry(int64_t B, int64_t N, int32_t W) {
    HotPart g{};
    int bb = 10;
    while (((N + (1LL << bb) - 1) >> bb) > 4096) ++bb;
    g.bb = bb;
    g.nbins = (int32_t)((N + (1LL << bb) - 1) >> bb);
    g.cap = B;
    g.nblk = (int32_t)((B + kHT * kXPer - 1) / (kHT * kXPer));
    g.ok = N > 0 && B > 0 && bb <= 24 && W >= 1 && (size_t)W * ((size_t)1 << bb) * 4 <= 128 * 1024 &&
           (double)g.nbins * (double)B <= (double)(1LL << 28);
    return g;
}

hipError_t launch_hot_count_part(const int32_t* bnode, const int64_t* bts, int64_t B, int64_t N,
                                 const HotCutoffs& cut, uint32_t* buckets, const HotPart& g, uint32_t* cur,
                                 uint32_t* region, hipStream_t st, int which) {
    static const hipError_t attr =
        hipFuncSetAttribute((const void*)k2y_bin_hist, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
    if (attr != hipSuccess) return attr;
    if (which & 1)
        hipLaunchKernelGGL(k2x_partition, dim3(g.nblk), dim3(kHT), sizeof(uint32_t) * 2 * g.nbins, st, bnode, bts, B,
                           N, cut, g, cur, region);
    const size_t lds = sizeof(uint32_t) * (size_t)cut.n_win * ((size_t)1 << g.bb);
    if (which & 2)
        hipLaunchKernelGGL(k2y_bin_hist, dim3(g.nbins, kYSplits), dim3(kHT), lds, st, region, cur, g, cut.n_win, N,
                           buckets);
    return hipGetLastError();
}

HotBins hot_bins_geometry(int64_t B, int64_t N, int32_t W) {
    HotBins g{};
    int bb = 12;
    while (((N + (1LL << bb) - 1) >> bb) > kMaxBins) ++bb;
    g.bb = bb;
    g.nbins = (int32_t)((N + (1LL << bb) - 1) >> bb);
    int64_t chunk = (B + 1023) / 1024;
    chunk = (chunk + kHT - 1) / kHT * kHT;
    if (chunk < 4096) chunk = 4096;
    g.chunk = chunk;
    g.nchunks = (int32_t)((B + chunk - 1) / chunk);
    g.splits = 8;
    // usable when the per-bin histogram fits LDS
    g.ok = N > 0 && B > 0 && bb <= 24 && (size_t)W * ((size_t)1 << bb) * 4 <= 128 * 1024;
    return g;
}

hipError_t launch_hot_count_binned(const int32_t* bnode, const int64_t* bts, int64_t B, int64_t N,
                                   const HotCutoffs& cut, uint32_t* buckets, const HotBins& g, uint32_t* chunk_cnt,
                                   uint32_t* bin_tot, uint32_t* sorted, hipStream_t st) {
    if (B <= 0 || cut.n_win <= 0 || N <= 0) return hipSuccess;
    // dynamic LDS above 64 KiB must be opted into; k2d also has ~1 KiB of static LDS
    static const hipError_t attr =
        hipFuncSetAttribute((const void*)k2d_bin_hist, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
    if (attr != hipSuccess) return attr;
    const size_t lds_bins = sizeof(uint32_t) * g.nbins;
    hipLaunchKernelGGL(k2a_bin_count, dim3(g.nchunks), dim3(kHT), lds_bins, st, bnode, bts, B, N, cut, g, chunk_cnt);
    hipLaunchKernelGGL(k2b_bin_scan, dim3(g.nbins), dim3(kHT), 0, st, chunk_cnt, g, bin_tot);
    hipLaunchKernelGGL(k2c_scatter, dim3(g.nchunks), dim3(kHT), lds_bins, st, bnode, bts, B, N, cut, g, chunk_cnt,
                       bin_tot, sorted);
    const size_t lds_hist = sizeof(uint32_t) * (size_t)cut.n_win * ((size_t)1 << g.bb);
    hipLaunchKernelGGL(k2d_bin_hist, dim3(g.nbins, g.splits), dim3(kHT), lds_hist, st, sorted, bin_tot, g, cut.n_win,
                       N, buckets);
    return hipGetLastError();
}

}  // namespace crane
