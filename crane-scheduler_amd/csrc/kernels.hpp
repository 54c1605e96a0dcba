// kernels.hpp — host-side launch interface of kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dyn_types.hpp"

namespace crane {

// NodeRec template instances (max predicates x max priorities).
enum { kShape4x6 = 0, kShape8x8 = 1, kShape16x16 = 2 };

struct HotCutoffs {
    int32_t n_win;
    int32_t pad;
    int64_t sorted[kMaxWin];  // ascending now_unix - int64(timeRange.Seconds())
};

struct MatrixOut {
    int8_t* first_fail;  // [P][N] or null
    int64_t* score;      // [P][N] or null
    int8_t pred_orig[kMaxPred];  // device predicate -> policy predicate index
};

size_t node_rec_bytes(int shape);
int64_t eval_chunk_nodes(int64_t P, int64_t N);

hipError_t launch_hot_count(const int32_t* bnode, const int64_t* bts, int64_t B, int64_t N, const HotCutoffs& cut,
                            uint32_t* buckets, hipStream_t st);
hipError_t launch_node_pass(int shape, const DevPolicy& pol, int64_t N, const double* val, const int64_t* ts,
                            const double* hv, const int64_t* hv_ts, const uint32_t* buckets, int64_t hv_ts_counts,
                            void* out, hipStream_t st);
hipError_t launch_eval(int shape, const void* rec, int64_t N, int64_t node_offset, const int64_t* now,
                       const uint8_t* flags, int64_t P, double wsum, int32_t noprio, long long* keys,
                       const MatrixOut& mo, hipStream_t st);

}  // namespace crane
