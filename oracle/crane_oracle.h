/*
 * crane_oracle.h — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of crane-scheduler's Dynamic plugin hot path, written from
 * the reference's semantics (file:line citations are into /root/reference):
 *   pkg/plugins/dynamic/stats.go:18-166, plugins.go:39-98,
 *   pkg/utils/utils.go:11-12,17-24,35-45,58-68,
 *   pkg/controller/annotator/binding.go:81-97, node.go:113-146.
 *
 * Parity status: the reference ships no tests, golden vectors or fixtures for
 * this path and its Go toolchain is absent here, so parity is UNPINNED BY THE
 * REFERENCE.  The restatement is pinned instead by hand-derived known-answer
 * tests (tests/golden/kats.json) and a small golden cluster whose expected
 * outputs come from an independent pure-Python restatement
 * (tests/golden/make_golden.py).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.
 */
#ifndef CRANE_ORACLE_H
#define CRANE_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* DynamicSchedulerPolicy.Spec, flattened in policy order
 * (pkg/plugins/apis/policy/types.go:14-39). */
typedef struct {
    int32_t n_sync;
    const char *const *sync_name;
    const int64_t *sync_period_ns;
    int32_t n_pred;
    const char *const *pred_name;
    const double *pred_limit;
    int32_t n_prio;
    const char *const *prio_name;
    const double *prio_weight;
    int32_t n_hot;
    const int64_t *hot_tr_ns;
    const int64_t *hot_count;
} or_policy;

/* ---- Go stdlib semantics the path depends on (go1.17, go.mod:3) ---- */
/* strconv.ParseFloat(s, 64): 0 ok, 1 ErrSyntax, 2 ErrRange. */
int or_go_parse_float(const char *s, int64_t n, double *out);
/* time.ParseInLocation("2006-01-02T15:04:05Z", s, fixed-offset zone):
 * 0 ok (unix ns in *out), nonzero = parse error. */
int or_go_parse_time(const char *s, int64_t n, int64_t tz_offset_s, int64_t *out_ns);
/* time.ParseDuration: 0 ok. */
int or_go_parse_duration(const char *s, int64_t n, int64_t *out_ns);
/* int(float64) on amd64 (CVTTSD2SQ): NaN / out of range -> INT64_MIN. */
int64_t or_go_f64_to_int(double x);
/* int64(d.Seconds()) for a time.Duration d (binding.go:85). */
int64_t or_go_duration_seconds_trunc(int64_t d_ns);

/* ---- Plugin semantics ---- */
/* getActiveDuration (stats.go:140-150): 0 ok (*dur set, may be 0), -1 error. */
int or_active_duration(const or_policy *pol, const char *name, int64_t *dur_ns);

/* String mode: re-parses node annotations on every (pod, node, metric) call
 * exactly like getResourceUsage (stats.go:51-76).  Node n owns annotation
 * pairs [anno_off[n], anno_off[n+1]) of keys/vals.  first_fail[p*N+n] = index
 * of the first failing predicate in policy order, -1 = Success.
 * score[p*N+n] = Score() result (computed for every node).  chosen[p] = lowest
 * index of max score among feasible nodes, -1 if none.  Output pointers may be
 * NULL.  n_threads splits pods across pthreads (upstream parallelism is 16). */
int or_eval_strings(const or_policy *pol, int64_t N, const int64_t *anno_off,
                    const char *const *keys, const char *const *vals,
                    int64_t P, const int64_t *now_ns, const uint8_t *pod_ds,
                    int64_t tz_offset_s, int32_t n_threads,
                    int8_t *first_fail, int64_t *score, int64_t *chosen);

/* Parse one annotation value "<float>,<time>" into (ok, val, ts_ns);
 * ok=0 when the string is malformed (any error that does not depend on the
 * current time).  Freshness/negativity are checked at evaluation. */
void or_parse_annotation(const char *s, int64_t n, int64_t tz_offset_s,
                         uint8_t *ok, double *val, int64_t *ts_ns);

/* SoA mode: the same semantics over pre-parsed entries.  key_names[k] names
 * entry row k of ok/val/ts ([K][N]); hv_* is the node_hot_value row. */
int or_eval_soa(const or_policy *pol, int32_t K, const char *const *key_names,
                int64_t N, const uint8_t *ok, const double *val, const int64_t *ts_ns,
                const uint8_t *hv_ok, const double *hv, const int64_t *hv_ts,
                int64_t P, const int64_t *now_ns, const uint8_t *pod_ds,
                int32_t n_threads, int8_t *first_fail, int64_t *score, int64_t *chosen);

/* Hot value producer: cnt[w*N+n] = GetLastNodeBindingCount(node n, tr_w)
 * (binding.go:81-97), hv[n] = sum_w cnt_w / count_w (node.go:113-121).
 * Bindings whose node is outside [0,N) match no node.  Returns -1 if a count
 * is 0 (Go would panic with an integer divide by zero). */
int or_hot_values(const or_policy *pol, int64_t B, const int32_t *b_node,
                  const int64_t *b_ts, int64_t N, int64_t now_unix,
                  int64_t *cnt, int64_t *hv);

/* Sequential greedy: one `now` for the batch; hot values start from the
 * binding log at now (annotation fresh), each placement appends a binding
 * with Timestamp = now_unix to its node and refreshes that node's hot value
 * before the next pod is scored. */
int or_greedy(const or_policy *pol, int32_t K, const char *const *key_names,
              int64_t N, const uint8_t *ok, const double *val, const int64_t *ts_ns,
              int64_t B, const int32_t *b_node, const int64_t *b_ts,
              int64_t P, int64_t now_ns, const uint8_t *pod_ds, int64_t *chosen);

/* BindingRecords (binding.go:50-123) over go1.17 container/heap: ops[i] = 0
 * AddBinding{node[i], arg[i]}, 1 BindingsGC at unix time arg[i].  Final heap
 * slice -> out_*; -1 for size <= 0. */
int or_binding_heap(int64_t size, int64_t gc_tr_ns, int64_t n_ops, const uint8_t *ops, const int32_t *node,
                    const int64_t *arg, int64_t *out_len, int32_t *out_node, int64_t *out_ts);

#ifdef __cplusplus
}
#endif
#endif
