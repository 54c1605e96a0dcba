// update.hip — scatter update of changed nodes (crane_dyn_update_nodes).
//
// The controller patches a node's annotations one metric at a time (each
// (node, metric) sync writes the metric and node_hot_value,
// /root/reference/pkg/controller/annotator/node.go:88-96,123-146, at every
// syncPolicy period, node.go:148-177), and the reference plugin reads the
// current annotations on every call (pkg/plugins/dynamic/stats.go:51-76).  A
// changed node's parsed columns are staged (k entries) and scattered into the
// shard's SoA here; when the node records are current, each changed node's
// record is recomputed in place with the node pass's own arithmetic
// (node_rec.hpp), so the answer tables of only those nodes need rebuilding — and the same
// launch can write those rows (node_steps.hpp: crane_dyn_update_node_steps).
//
// One thread per changed node: k is a handful per scheduling cycle, so the
// launch is latency-bound (one wave); nothing here is bandwidth-priced.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dyn_types.hpp"
#include "kernels.hpp"
#include "node_rec.hpp"
#include "node_steps.hpp"

namespace crane {

template <int PD, int PR>
__global__ __launch_bounds__(256) void k_update_nodes(UpdateArgs a) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= a.k) return;
    const DevPolicy& pol = a.pol;
    const int64_t i = a.idx[j], N = a.N, k = a.k;
    for (int m = 0; m < pol.n_slots; ++m) {
        a.val[m * N + i] = a.sval[m * k + j];
        a.ts[m * N + i] = a.sts[m * k + j];
    }
    // an update without a hot-value annotation leaves the node with none (0, unusable)
    const double h = a.shv ? a.shv[j] : 0.0;
    const int64_t ht = a.shv ? a.shv_ts[j] : kTsInvalid;
    if (a.hv) {
        a.hv[i] = h;
        a.hv_ts[i] = ht;
    }
    if (!a.rec && !a.ns) return;
    int64_t pt[PD], qt[PR];
    double pv[PD], qv[PR];
#pragma unroll
    for (int q = 0; q < PD; ++q) {
        const int64_t row = q < pol.npd ? pol.pred_slot[q] : 0;
        pt[q] = q < pol.npd ? a.sts[row * k + j] : kTsInvalid;
        pv[q] = q < pol.npd ? a.sval[row * k + j] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < PR; ++q) {
        const int64_t row = q < pol.npr ? pol.prio_slot[q] : 0;
        qt[q] = q < pol.npr ? a.sts[row * k + j] : kTsInvalid;
        qv[q] = q < pol.npr ? a.sval[row * k + j] : 0.0;
    }
    NodeRec<PD, PR> r;
    rec_metrics<PD, PR>(pol, pt, pv, qt, qv, r);
    rec_hot_annotation<PD, PR>(h, ht, r);
    rec_fail<PD, PR>(r);
    if (a.rec) static_cast<NodeRec<PD, PR>*>(a.rec)[i] = r;
    if (a.ns) node_steps_row<PD, PR>(r, a.ma, a.t0, a.t1, j, a.ns, a.bp, a.ff, a.sc);
}

__global__ __launch_bounds__(256) void k_fill_i64(int64_t* p, int64_t n, int64_t v) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = v;
}

hipError_t launch_update_nodes(int shape, const UpdateArgs& a, hipStream_t st) {
    if (a.k <= 0) return hipSuccess;
    const dim3 g((unsigned)((a.k + 255) / 256)), b(256);
    switch (shape) {
        case kShape4x6: return klaunch("k_update_nodes", k_update_nodes<4, 6>, g, b, 0, st, a);
        case kShape8x8: return klaunch("k_update_nodes", k_update_nodes<8, 8>, g, b, 0, st, a);
        default: return klaunch("k_update_nodes", k_update_nodes<16, 16>, g, b, 0, st, a);
    }
}

hipError_t launch_fill_i64(int64_t* p, int64_t n, int64_t v, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
    return klaunch("k_fill_i64", k_fill_i64, dim3((unsigned)blocks), dim3(256), 0, st, p, n, v);
}

}  // namespace crane
