/*
 * crane_dyn.h — C ABI of the MI355X engine for crane-scheduler's Dynamic
 * plugin hot path (Filter + Score batched over pods x nodes, hot values,
 * selection).  Plain C types only: this is what a cgo shim in the scheduler
 * binds.  Citations are into /root/reference.
 *
 * Reference interfaces this ABI replaces:
 *   - DynamicScheduler.Filter        pkg/plugins/dynamic/plugins.go:39-69
 *   - DynamicScheduler.Score         pkg/plugins/dynamic/plugins.go:73-98
 *   - getNodeScore/isOverLoad/...    pkg/plugins/dynamic/stats.go:30-166
 *   - NewDynamicScheduler            pkg/plugins/dynamic/plugins.go:105-120
 *   - LoadPolicyFromFile/loadPolicy  pkg/plugins/dynamic/policyfile.go:11-33
 *   - BindingRecords.GetLastNodeBindingCount  pkg/controller/annotator/binding.go:81-97
 *   - BindingRecords.AddBinding / BindingsGC    binding.go:69-78, 100-123
 *   - translateEventToBinding        pkg/controller/annotator/event.go:118-145
 *   - annotateNodeHotValue           pkg/controller/annotator/node.go:113-121
 *   - upstream selectHost (argmax; lowest node index wins ties — declared
 *     deviation from upstream's random tie-break)
 *
 * Conventions: every function returns 0 on success and a negative CRANE_E_*
 * code on failure; crane_dyn_last_error() then describes it.  Callers own all
 * host arrays; the engine copies them during the call and keeps no pointer.
 * Calls on one engine are serialised by an internal mutex.  Asynchronous calls
 * (*_async) enqueue work that reads the engine's buffers on the caller's stream;
 * the calls that replace engine state (upload_nodes, update_nodes,
 * upload_bindings, binding_records, add_bindings, gc_bindings, destroy) and the
 * synchronous calls that run on the engine's own stream (eval, eval_compact,
 * node_steps, node_steps_subset, refresh_hot_values, hot_values, select, greedy)
 * first wait for the caller streams this engine enqueued asynchronous work on
 * since the last such wait — those streams only, not the device — so they never
 * change a buffer a kernel is still reading.  The engine keeps a caller stream's
 * handle until that wait: a stream passed to an *_async call must outlive the
 * engine's next state change, or be handed back first with crane_dyn_forget_stream (which waits
 * for it); destroy waits for the whole device.  Asynchronous calls on ONE engine
 * from several streams must be ordered by the caller (they share the engine's
 * scratch): use one stream per engine.  Nothing in the
 * engine reads the environment; crane_dyn_set_option (tests / A-B tools only)
 * selects alternative kernel forms of the same results.
 */
#ifndef CRANE_DYN_H
#define CRANE_DYN_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CRANE_OK 0
#define CRANE_E_INVALID -1  /* bad argument / policy */
#define CRANE_E_HIP -2      /* HIP runtime failure */
#define CRANE_E_STATE -3    /* call out of order (e.g. eval before upload) */
#define CRANE_E_PARSE -4    /* policy file could not be decoded */
#define CRANE_E_IO -5       /* policy file could not be read */

/* Sentinel timestamp for an annotation that is missing or malformed
 * (getResourceUsage errors that do not depend on the current time). */
#define CRANE_TS_INVALID INT64_MIN

/* Pod flag bits (crane_dyn_eval*). */
#define CRANE_POD_DAEMONSET 1u /* utils.IsDaemonsetPod (utils.go:17-24): Filter bypass */

/* DynamicSchedulerPolicy.Spec (pkg/plugins/apis/policy/types.go:14-39),
 * flattened in policy order.  Durations in nanoseconds. */
typedef struct crane_policy {
    int32_t n_sync;
    const char *const *sync_name;
    const int64_t *sync_period_ns;
    int32_t n_pred;
    const char *const *pred_name;
    const double *pred_limit; /* maxLimitPecent */
    int32_t n_prio;
    const char *const *prio_name;
    const double *prio_weight;
    int32_t n_hot;
    const int64_t *hot_tr_ns;  /* hotValue.timeRange */
    const int64_t *hot_count;  /* hotValue.count (must be != 0) */
} crane_policy;

/* ---------------------------------------------------------------- policy
 * Strict decoder for the DynamicSchedulerPolicy file (YAML block subset or
 * JSON), apiVersion scheduler.policy.crane.io/v1alpha1 — replaces
 * LoadPolicyFromFile/loadPolicy (policyfile.go:11-33).  Unknown or duplicate
 * fields are errors, as with the reference's strict codec
 * (policy/scheme/scheme.go:17). */
typedef struct crane_policy_doc crane_policy_doc;
int crane_policy_load_file(const char *path, crane_policy_doc **out, char *err, size_t errcap);
int crane_policy_load_bytes(const char *data, size_t n, crane_policy_doc **out, char *err, size_t errcap);
const crane_policy *crane_policy_view(const crane_policy_doc *doc);
void crane_policy_free(crane_policy_doc *doc);

/* ------------------------------------------------------------ annotations
 * Host parser for one node annotation value "<float>,<YYYY-MM-DDTHH:MM:SSZ>"
 * (written by node.go:123-146 with prometheus.go:124 / strconv.Itoa values,
 * local time per utils.go:26-45).  Follows strings.Split + time.ParseInLocation
 * + strconv.ParseFloat of getResourceUsage (stats.go:51-76).  *ts_ns is the
 * Unix time in ns or CRANE_TS_INVALID when the value is unusable at any time
 * (missing parts, bad timestamp, bad float); negative values are returned as
 * parsed — the engine rejects them like stats.go:71-73. */
int crane_tz_offset(const char *tz_name, int64_t *offset_s); /* "" or NULL = $TZ, default Asia/Shanghai */
void crane_parse_annotation(const char *s, size_t n, int64_t tz_offset_s, double *value, int64_t *ts_ns);
/* Bulk form for a whole snapshot: strs[i] (NULL = key missing) of length
 * lens[i] -> value[i], ts_ns[i]; n_threads host threads (<= 0: hardware
 * concurrency).  This is the once-per-sync parse that replaces the
 * reference's per-call parsing (stats.go:51-76). */
int crane_parse_annotations(int64_t n, const char *const *strs, const size_t *lens, int64_t tz_offset_s,
                            double *value, int64_t *ts_ns, int32_t n_threads);
/* IANA zones (utils.GetLocation = time.LoadLocation($TZ), utils.go:35-45) with
 * go1.17's semantics (tz.cpp): crane_tz_load reads the TZif file `name` from
 * zoneinfo_dir, or $ZONEINFO then /usr/share/zoneinfo, /usr/share/lib/zoneinfo,
 * /usr/lib/locale/TZ ("" and "UTC" = UTC; names with ".." or a leading '/' are
 * invalid); a wall time becomes an instant as time.Date does, including its
 * choice for skipped and repeated wall times.  The _tz parsers equal the
 * fixed-offset ones otherwise.  crane_tz_lookup = Location.lookup (offset of
 * the zone in effect at unix_s and that period [start, end)); crane_tz_date =
 * time.Date's wall clock (seconds since the epoch as if UTC) -> Unix seconds. */
typedef struct crane_tz crane_tz;
int crane_tz_load(const char *name, const char *zoneinfo_dir, crane_tz **out);
int crane_tz_load_bytes(const uint8_t *tzif, size_t n, crane_tz **out);
void crane_tz_free(crane_tz *tz);
int crane_tz_lookup(const crane_tz *tz, int64_t unix_s, int32_t *offset_s, int64_t *start_s, int64_t *end_s);
int64_t crane_tz_date(const crane_tz *tz, int64_t local_s);
void crane_parse_annotation_tz(const char *s, size_t n, const crane_tz *tz, double *value, int64_t *ts_ns);
int crane_parse_annotations_tz(int64_t n, const char *const *strs, const size_t *lens, const crane_tz *tz,
                               double *value, int64_t *ts_ns, int32_t n_threads);

/* ------------------------------------------------------------------ engine */
typedef struct crane_dyn crane_dyn;

/* NewDynamicScheduler (plugins.go:105-120) minus the policy file read: build
 * an engine for `pol` on HIP device `device`.  The policy is validated and
 * flattened into the device policy table here. */
int crane_dyn_create(const crane_policy *pol, int32_t device, crane_dyn **out);
int crane_dyn_destroy(crane_dyn *h);
const char *crane_dyn_last_error(const crane_dyn *h);
/* A caller stream that *_async calls enqueued work on is about to be destroyed: wait for it and
 * drop the engine's handle of it (the next state change would otherwise wait on a dangling
 * handle).  No-op for a stream the engine does not hold. */
int crane_dyn_forget_stream(crane_dyn *h, void *stream);

/* Metric slots: the distinct annotation keys the policy reads, in the order
 * the SoA rows of crane_dyn_upload_nodes must follow. */
int32_t crane_dyn_num_metrics(const crane_dyn *h);
const char *crane_dyn_metric_name(const crane_dyn *h, int32_t slot);

/* Upload one node shard's parsed annotations (host SoA):
 *   val[m*n_nodes + i], ts_ns[m*n_nodes + i] for metric slot m;
 *   hv[i], hv_ts_ns[i] = node_hot_value annotation (hv may be NULL: all
 *   nodes have no hot value).
 * node_offset = global index of local node 0 (node sharding across GPUs);
 * chosen-node results and packed keys use global indices. */
int crane_dyn_upload_nodes(crane_dyn *h, int64_t n_nodes, int64_t node_offset,
                           const double *val, const int64_t *ts_ns,
                           const double *hv, const int64_t *hv_ts_ns);

/* Replace the parsed annotations of k nodes of the shard, as the controller's patches change
 * them (each (node, metric) sync patches the metric and node_hot_value, node.go:88-96,123-146,
 * at every syncPolicy period, node.go:148-177) and the reference plugin reads them on its next
 * call (stats.go:51-76).  idx[j] (distinct local node indices) gets val[m*k + j], ts_ns[m*k + j]
 * for metric slot m and hv[j], hv_ts_ns[j] (hv NULL: those nodes carry no node_hot_value).
 * The result equals crane_dyn_upload_nodes of the whole shard with those nodes' columns
 * replaced (hot values come from the annotations again after a refresh from bindings); the
 * node records of the changed nodes are recomputed in place, so crane_dyn_node_steps_subset
 * of those nodes is all a table of answers needs.  Synchronous. */
int crane_dyn_update_nodes(crane_dyn *h, int64_t k, const int64_t *idx, const double *val, const int64_t *ts_ns,
                           const double *hv, const int64_t *hv_ts_ns);
/* Grow or shrink the shard to n nodes in place (global indices node_offset + i as before): nodes
 * [0, min(N, n)) keep their parsed annotations, new ones start with none (every metric and the hot
 * value missing) until crane_dyn_update_nodes writes them; hot values from the binding log revert to
 * the annotations, as after crane_dyn_upload_nodes.  The drop-in plugin grows its shard this way when
 * nodes join the cluster (the reference looks a node up per call, plugins.go:45-50,74-84: a new node
 * costs it nothing either). */
int crane_dyn_resize_nodes(crane_dyn *h, int64_t n);
/* crane_dyn_update_nodes and crane_dyn_node_steps_subset of the same nodes over [t0, t1) in one
 * call: one launch writes the columns, the records and the rows (one round trip to the device). */
int crane_dyn_update_node_steps(crane_dyn *h, int64_t k, const int64_t *idx, const double *val, const int64_t *ts_ns,
                                const double *hv, const int64_t *hv_ts_ns, int64_t t0_ns, int64_t t1_ns,
                                uint8_t *n_steps, int64_t *bp, int8_t *first_fail, int8_t *score);

/* Upload the binding records (BindingRecords heap content, binding.go:14-19):
 * node = LOCAL node index of the shard (<0 or >= n_nodes: matches no node),
 * ts_s = Binding.Timestamp (Unix seconds).  Replaces the whole log (and ends
 * the heap mode below). */
int crane_dyn_upload_bindings(crane_dyn *h, int64_t n, const int32_t *node, const int64_t *ts_s);

/* Heap mode: the engine keeps BindingRecords itself (binding.go:50-123) and the
 * controller feeds it binding by binding.
 *   crane_dyn_binding_records = NewBindingRecords(size, gcTimeRange)
 *     (controller.go:57: size = --binding-heap-size, gcTimeRange = the largest
 *     hotValue timeRange); clears the log.  size must be in [1, 2^31).
 *   crane_dyn_add_bindings    = n x AddBinding in order (a full heap pops its
 *     minimum Timestamp first, binding.go:69-78); only the changed log slots
 *     are copied to the device.
 *   crane_dyn_gc_bindings     = BindingsGC at now_ns (binding.go:100-123).
 *   crane_dyn_binding_count   = the heap's Len() (the log length outside heap mode). */
int crane_dyn_binding_records(crane_dyn *h, int64_t size, int64_t gc_time_range_ns);
int crane_dyn_add_bindings(crane_dyn *h, int64_t n, const int32_t *node, const int64_t *ts_s);
int crane_dyn_gc_bindings(crane_dyn *h, int64_t now_ns);
int64_t crane_dyn_binding_count(const crane_dyn *h);

/* Recompute every node's hot value from the uploaded bindings as the
 * controller does at `now_ns` (binding.go:81-97, node.go:113-121) and use it
 * as the node_hot_value annotation, stamped hv_ts_ns, from now on. */
int crane_dyn_refresh_hot_values(crane_dyn *h, int64_t now_ns, int64_t hv_ts_ns);

/* Controller side (annotateNodeHotValue, node.go:113-121): the hot value of
 * every node of the shard as the Score phase uses it — after a refresh, the
 * binding-log value sum_w count_w / Count_w (an integer, written by the
 * controller as strconv.Itoa); otherwise the uploaded annotation value (0 if
 * none).  hv_out holds n = the shard's node count values. */
int crane_dyn_hot_values(crane_dyn *h, int64_t n, double *hv_out);

/* Evaluate a pod batch against the current shard.  now_ns[p] is pod p's
 * time.Now(); pod_flags[p] carries CRANE_POD_* bits (NULL = 0).
 * Outputs (any may be NULL):
 *   first_fail[p*n + i]: -1 = Filter Success, else index (policy order) of the
 *                        first overloaded predicate (Unschedulable);
 *   score[p*n + i]     : Score() result in [0,100] for every node;
 *   chosen[p]          : global index of the feasible node with the highest
 *                        score, lowest index on ties; -1 = none feasible;
 *   chosen_score[p]    : that node's score (-1 when none). */
int crane_dyn_eval(crane_dyn *h, int64_t n_pods, const int64_t *now_ns, const uint8_t *pod_flags,
                   int8_t *first_fail, int64_t *score, int64_t *chosen, int64_t *chosen_score);
/* The same with the score matrix as int8 (scores lie in [0,100]): 2 bytes per
 * (pod, node) instead of 9 cross PCIe — the form the plugin shim uses per pod. */
int crane_dyn_eval_compact(crane_dyn *h, int64_t n_pods, const int64_t *now_ns, const uint8_t *pod_flags,
                           int8_t *first_fail, int8_t *score, int64_t *chosen, int64_t *chosen_score);
/* Answer tables for the drop-in plugin: a node's Filter and Score depend on `now` only
 * through `now < expiry` against its expiries, so over [t0_ns, t1_ns) each is a step
 * function.  For node i: n_steps[i] (<= S = crane_dyn_step_slots) breakpoints
 * bp[i*S + j] ascending inside (t0, t1), and first_fail / score[i*(S+1) + j] (as in
 * crane_dyn_eval, int8) on [bp[j-1], bp[j]) with bp[-1] = t0, bp[n_steps] = t1.  The
 * engine computes every value (the same kernels' arithmetic); the plugin answers a pod's
 * per-node calls at its `now` by a lookup, with no device call per pod.  Synchronous;
 * n = the shard's node count; host arrays. */
int32_t crane_dyn_step_slots(const crane_dyn *h);
int crane_dyn_node_steps(crane_dyn *h, int64_t t0_ns, int64_t t1_ns, int64_t n, uint8_t *n_steps, int64_t *bp,
                         int8_t *first_fail, int8_t *score);
/* The same answers for k distinct nodes idx[j] only, as compact rows j: n_steps[j], bp[j*S + ..],
 * first_fail / score[j*(S+1) + ..] — equal to rows idx[j] of crane_dyn_node_steps over [t0, t1).
 * What the drop-in plugin patches into its table for the nodes crane_dyn_update_nodes changed. */
int crane_dyn_node_steps_subset(crane_dyn *h, int64_t t0_ns, int64_t t1_ns, int64_t k, const int64_t *idx,
                                uint8_t *n_steps, int64_t *bp, int8_t *first_fail, int8_t *score);
/* Device-resident matrix form, asynchronous on `stream`: d_first_fail[p*ld + i]
 * and d_score[p*ld + i] (int8) as crane_dyn_eval, any may be NULL; d_keys (NULL
 * = none) as crane_dyn_eval_keys_async. */
int crane_dyn_eval_matrix_async(crane_dyn *h, int64_t n_pods, const int64_t *d_now_ns, const uint8_t *d_pod_flags,
                                int8_t *d_first_fail, int8_t *d_score, int64_t ld, int64_t *d_keys, void *stream);

/* Framework-level selection for a pod queue, in order — what kube-scheduler
 * v1.23.3 (go.mod:26; pkg/scheduler/core/generic_scheduler.go, not in the
 * repo) does around the plugin with the shipped profile
 * (deploy/manifests/dynamic/scheduler-config.yaml:7-16: the default plugins
 * plus Dynamic, score weight 3):
 *   - filter: Dynamic's Filter (DaemonSet pods bypass) and d_ext_ok[i] (the
 *     other filter plugins' verdict per node, NULL = all pass);
 *   - percentageOfNodesToScore: crane_num_feasible_nodes_to_find(N, percentage)
 *     feasible nodes are taken per pod from the rotated order starting at the
 *     running start index (first `start`), which then advances by the nodes
 *     checked (findNodesThatPassFilters, sequential order); percentage >= 100
 *     or N < 100 checks every node;
 *   - score: dyn_weight * Score() + d_ext_score[i] (the other plugins' weighted
 *     sum, in [0, 2^30); NULL = 0), dyn_weight in [0, 2^20];
 *   - selectHost: the max total; ties go to the lowest node index (tie_seed 0,
 *     a declared deviation from upstream's random reservoir) or, tie_seed != 0,
 *     to a seeded bijective hash of (node index, pod position) — decodable, so
 *     shards' packed keys still max-combine.
 * Outputs (device, [n_pods]): d_chosen global node index or -1 (no feasible
 * node: Unschedulable), d_total (NULL ok) the winning total or -1; d_wstart /
 * d_wlen (NULL ok) each pod's window (rotated start, nodes checked);
 * *next_start the start index after the queue (host).  Windows are over this
 * engine's local node order.  Synchronous on `stream`. */
int64_t crane_num_feasible_nodes_to_find(int64_t num_all_nodes, int32_t percentage_of_nodes_to_score);
int crane_dyn_select(crane_dyn *h, int64_t n_pods, const int64_t *d_now_ns, const uint8_t *d_pod_flags,
                     const uint8_t *d_ext_ok, const int64_t *d_ext_score, int64_t dyn_weight, int32_t percentage,
                     int64_t start, uint64_t tie_seed, int64_t *d_chosen, int64_t *d_total, int64_t *d_wstart,
                     int64_t *d_wlen, int64_t *next_start, void *stream);

/* Device-resident variant for batched pipelines: all pointers are device
 * pointers, work is enqueued on `stream` (hipStream_t; NULL = engine stream)
 * and the call returns without synchronising.  keys[p] = (score << 32) |
 * (0xFFFFFFFF - global_node_index) of the shard's best feasible node, or -1.
 * A max-reduction of keys across node shards (e.g. RCCL allreduce, int64,
 * max) gives the global choice. */
int crane_dyn_eval_keys_async(crane_dyn *h, int64_t n_pods, const int64_t *d_now_ns,
                              const uint8_t *d_pod_flags, int64_t *d_keys, void *stream);
/* One scheduling step, asynchronous on `stream`: hot values from the bindings
 * at now_ns (as crane_dyn_refresh_hot_values_async) then the keys-only
 * evaluation of the pod batch (as crane_dyn_eval_keys_async). */
int crane_dyn_step_keys_async(crane_dyn *h, int64_t now_ns, int64_t hv_ts_ns, int64_t n_pods,
                              const int64_t *d_now_ns, const uint8_t *d_pod_flags, int64_t *d_keys, void *stream);
/* Dispatch queues: a user-mode AQL queue on one device (HSA, the layer under HIP) to which the
 * step's kernels are written as packets by the calling thread — ~0.3 us per kernel instead of
 * HIP's 2.6-3.7 us per launch, which made a batch's three launches cost the host about the GPU's
 * time per batch.  A queue is in order (like a stream); it is not a HIP stream: work
 * on it is ordered with HIP work only through crane_queue_wait (the engine does this itself
 * around its own synchronous calls).  ring_kind 0 puts the kernel arguments in device memory
 * the host writes through the PCIe BAR (default), 1 in pinned host memory.  The handle is
 * returned on failure too (read its error, then destroy it). */
typedef struct crane_queue crane_queue;
int crane_queue_create(int32_t device, int32_t ring_kind, crane_queue **out);
/* Wait until every step enqueued on the queue has completed. */
int crane_queue_wait(crane_queue *q);
const char *crane_queue_last_error(const crane_queue *q);
/* Waits for the queue, then frees it. */
int crane_queue_destroy(crane_queue *q);
/* crane_dyn_step_keys_async with the step's kernels on `q`: d_now / d_flags must be complete on
 * the device when called (written by finished work); d_keys is complete after crane_queue_wait.
 * The engine's own state changes wait for the queues it used: a queue must outlive the engine's
 * next state change, or be handed back first with crane_dyn_forget_queue. */
int crane_dyn_step_keys_queue(crane_dyn *h, int64_t now_ns, int64_t hv_ts_ns, int64_t n_pods,
                              const int64_t *d_now_ns, const uint8_t *d_pod_flags, int64_t *d_keys, crane_queue *q);
/* option step_defer: run the last step's deferred K3s now (on its queue; then wait for the queue) */
int crane_dyn_step_flush(crane_dyn *h);
/* Hand a queue back (waits for it): the engine no longer waits for it at its state changes. */
int crane_dyn_forget_queue(crane_dyn *h, crane_queue *q);
/* Asynchronous pieces of one scheduling step on `stream`:
 * hot values from bindings (K2) and the node pass (K1). */
int crane_dyn_refresh_hot_values_async(crane_dyn *h, int64_t now_ns, int64_t hv_ts_ns, void *stream);
int crane_dyn_node_pass_async(crane_dyn *h, void *stream);

/* Kernel timing for benchmarks and profiling: while enabled, every kernel the
 * engine launches carries a start/stop event pair stamped by the dispatch
 * itself (hipExtLaunchKernel), i.e. the kernel's own duration as rocprofv3
 * reports it.  crane_dyn_stage_times() waits for them, writes up to `max`
 * (kernel name, milliseconds) pairs in launch order, returns the number of
 * kernels and clears the list.  Enabling also clears it. */
int crane_dyn_set_profiling(crane_dyn *h, int on);
int crane_dyn_stage_times(crane_dyn *h, int32_t max, const char **names, double *ms);

/* Sequential-greedy batch: one `now_ns` for the whole batch; pods are placed
 * in order and each placement appends a binding (Timestamp = now) to the
 * chosen node, refreshing its hot value before the next pod is scored.  The
 * hot values start from the uploaded bindings.  chosen[p] as above. */
int crane_dyn_greedy(crane_dyn *h, int64_t n_pods, int64_t now_ns, const uint8_t *pod_flags, int64_t *chosen);

/* Decode a packed key: returns the global node index (-1 for key < 0) and
 * stores the score in *score (-1 for key < 0) when score != NULL. */
int64_t crane_dyn_key_node(int64_t key, int64_t *score);

/* Build/version info string (static storage). */
const char *crane_dyn_version(void);

/* Alternative kernel forms of the same results, for tests and A/B tools:
 *   "k2_form" 0 dedupe (default; the large form past its count/offset cap, the atomics form past the
 *     large form's) | 2 atomics (LDS hash + global atomics, any shape) | 3 large
 *   "k2_sorted" 1 a time-ordered log (checked at upload): K2 reads the widest window's suffix only | 0 never
 *   "k2_delta" 1 ... and with k2_form 0, once anchored, only the bindings whose window rank changed since
 *     the anchor refresh (the anchor's dense counts + adjustments) | 0 every refresh re-counts the suffix
 *   "step_defer" 0 | 1: a step on a dispatch queue (crane_dyn_step_keys_queue) leaves its last kernel
 *     (K3s) to the engine's next step on that queue, which runs it inside its own first launch (one
 *     launch and one kernel boundary fewer per step); its keys are final once that launch, or
 *     crane_dyn_step_flush, or any other call on the engine, has run it and the queue completed it.
 *     The group sets it on its slots' engines and flushes at crane_dyn_group_sync
 *   "k1_stream" 1 the streamed step pass without dedupe-form K2 entries | 0 the record-holding fused pass
 *   "k1_tail" 0 its tail on one wave when the grid has >= 4096 blocks | 1 always | 4 on all four waves
 *   "keys_path" 0 step path | 1 per-pair kernel   "greedy_form" 0 merge | 1 sequential
 *   "step_rows" 1 producers index the records per pod tile | 0 K3s searches them
 *   "step_pieces" 0 auto | 1 | 2: middle pieces cut into elementary ones when it pays | always | never
 *   "step_lds_cap" one-step records per kind staged in K1's LDS at most (0: all through device memory)
 *   "sel_chain" 0 LDS rank/select walk of the selection windows (N <= 131072) | 1 streaming kernel
 *   "trace" 0 | 1: phase stamps of the step kernels (crane_dyn_debug_trace) */
int crane_dyn_set_option(crane_dyn *h, const char *name, int64_t value);
/* Phase stamps of the last K2x (which = 0), K1 (1) or K3s (2) launch with option
 * "trace" on: out[8 * workgroup + k] = s_memrealtime (100 MHz) at phase k.
 * Returns the number of entries copied (<= max). */
int64_t crane_dyn_debug_trace(crane_dyn *h, int32_t which, int64_t max, uint64_t *out);

/* ------------------------------------------------------------------ groups
 * One process, N devices (SURVEY §8(b) crane_dyn_create(..., device_count, ...), §8(e)): the
 * scheduler is one Go process with one plugin instance (cmd/scheduler/main.go:18-32,
 * plugins.go:105-120), so the node-shard path is reached through one handle.  A group holds per
 * device `depth` engines (one per batch in flight) over the device's contiguous node range
 * (crane_shard_range of the cluster over n_dev shards) — sharing ONE copy of the shard's nodes and
 * binding log, each with its own scratch —, their HIP streams and one RCCL communicator per device
 * (ncclCommInitAll).  A batch = every device's shard step
 * (crane_dyn_step_keys_async), then an in-place ncclAllReduce(int64, ncclMax) of the packed keys
 * on the same streams: every device then holds the global choice per pod.  With n_dev > 1 each
 * device has a worker thread enqueueing its part (the caller only hands over the batch).
 * Options (crane_dyn_group_set_option): "collective" 0 never (crane_dyn_group_schedule max-combines
 * on the host; the async form leaves per-shard keys) | 1 when n_dev > 1 (default) | 2 always (a
 * one-rank communicator: tests); "threads" -1 auto | 0 the caller's thread (the collective in
 * ncclGroupStart/End) | 1 worker threads; "dispatch" -1 (default) dispatch queues, except for the
 * per-batch collective (step_keys_async / schedule with the collective on) | 0 the steps' kernels
 * launched through HIP on the slots' streams | 1 on dispatch queues (crane_queue, one per slot and
 * device; the batch form crane_dyn_group_step_keys_batch orders its collective after them);
 * "dispatch_ring" 0 | 1 their ring_kind; "defer" 1 (default) | 0: engine option step_defer on the
 * queues' engines (a slot's K3s runs in its next step's first launch; crane_dyn_group_sync runs the
 * last ones — the caller alternates key buffers per slot, or the deferred K3s runs alone first);
 * any other name goes to every engine.  Either way the batch's d_now / d_flags must be
 * complete on the devices when it is handed over (the group's streams and queues are its own). */
typedef struct crane_dyn_group crane_dyn_group;
/* Contiguous balanced node range of shard `shard` of n_shards (the first n % n_shards get one more). */
int crane_shard_range(int64_t n_nodes, int32_t n_shards, int32_t shard, int64_t *lo, int64_t *hi);
/* devices NULL = 0 .. n_dev-1 (a device may be listed more than once: several shards on one GPU,
 * combined without the collective); depth in [1, 64].  The handle is returned on failure too: read
 * its error, then destroy it. */
int crane_dyn_group_create(const crane_policy *pol, int32_t n_dev, const int32_t *devices, int32_t depth,
                           crane_dyn_group **out);
int crane_dyn_group_destroy(crane_dyn_group *g);
const char *crane_dyn_group_last_error(const crane_dyn_group *g);
int crane_dyn_group_set_option(crane_dyn_group *g, const char *name, int64_t value);
int32_t crane_dyn_group_size(const crane_dyn_group *g);
/* device and node range [lo, hi) of shard i (after crane_dyn_group_upload_nodes) */
int crane_dyn_group_shard(const crane_dyn_group *g, int32_t i, int32_t *device, int64_t *lo, int64_t *hi);
/* the engine of shard i for batch slot `slot` (metric names, profiling, options) */
crane_dyn *crane_dyn_group_engine(crane_dyn_group *g, int32_t i, int32_t slot);
/* The whole cluster's SoA as crane_dyn_upload_nodes takes it ([M][n_nodes] rows, global order);
 * each device keeps its shard's columns (node_offset = its lo). */
int crane_dyn_group_upload_nodes(crane_dyn_group *g, int64_t n_nodes, const double *val, const int64_t *ts,
                                 const double *hv, const int64_t *hv_ts);
/* The whole binding log with GLOBAL node indices; each device keeps its nodes' bindings, local
 * indices, in log order (a time-ordered log stays one). */
int crane_dyn_group_upload_bindings(crane_dyn_group *g, int64_t n, const int32_t *node, const int64_t *ts_s);
/* One batch, asynchronous: d_now[i] / d_flags[i] (NULL array or entry = no flags) / d_keys[i] are
 * device pointers on device i.  Batch b (counted from the group's creation) runs on slot b % depth:
 * its engines and streams; d_keys[i] then holds the global keys (the per-shard keys with
 * "collective" 0).  A key buffer reused every `depth` batches is ordered by the slot's stream.
 * Errors of the enqueued work are reported by crane_dyn_group_sync. */
int crane_dyn_group_step_keys_async(crane_dyn_group *g, int64_t now_ns, int64_t hv_ts_ns, int64_t n_pods,
                                    const int64_t *const *d_now, const uint8_t *const *d_flags,
                                    int64_t *const *d_keys);
/* G batches at once, asynchronous, with ONE collective: batch b (b < n_batches) at now_ns[b] /
 * hv_ts_ns[b] over the pods d_now[i] + b * n_pods (device i's [n_batches][n_pods] times; d_flags[i]
 * likewise or NULL) into d_keys[i] + b * n_pods, on slot (the group's batch count) % depth, its
 * kernels on the slot's dispatch queue unless "dispatch" is 0; then, with the collective on, one
 * in-place ncclAllReduce(int64, max) of the whole [n_batches][n_pods] keys per device on a
 * collective stream of the group, issued by the thread enqueueing for the device once it sees the
 * slots' dispatch queues complete the window's steps (with HIP launches: ordered by events) — the
 * per-batch all-reduce's latency paid once per G batches, as a scheduler collecting a window of
 * batches' choices would.  A later batch that
 * writes keys where that all-reduce still works waits for it (host side): alternate two key
 * buffers.  Errors of the enqueued work are reported by crane_dyn_group_sync. */
int crane_dyn_group_step_keys_batch(crane_dyn_group *g, int32_t n_batches, const int64_t *now_ns,
                                    const int64_t *hv_ts_ns, int64_t n_pods, const int64_t *const *d_now,
                                    const uint8_t *const *d_flags, int64_t *const *d_keys);
/* wait for every batch enqueued on the group */
int crane_dyn_group_sync(crane_dyn_group *g);
/* The shard state changes of the drop-in plugin and the controller, routed by GLOBAL node index to
 * the owning shard (each shard's batch slots share one copy of its inputs and follow the change):
 *   update_nodes / update_node_steps = crane_dyn_update_nodes / _update_node_steps with global
 *     indices (rows j of the outputs for idx[j]);
 *   resize_nodes = the cluster's node count becomes n: the last shard grows (joining nodes take
 *     indices at the end, no annotations until updated), shrinking empties shards from the end;
 *     bindings uploaded with crane_dyn_group_upload_bindings for nodes past the old end need a
 *     re-upload (the heap form routes them as they come);
 *   binding_records / add_bindings / gc_bindings / binding_count = the BindingRecords heap
 *     (binding.go:50-123) with global node indices: every device runs the same heap (its order
 *     depends on timestamps only) with the other shards' nodes as "no node";
 *   refresh_hot_values / hot_values / node_steps = per shard, results at the global rows.
 * Synchronous; each first waits for the group's batches in flight. */
int crane_dyn_group_update_nodes(crane_dyn_group *g, int64_t k, const int64_t *idx, const double *val,
                                 const int64_t *ts, const double *hv, const int64_t *hv_ts);
int crane_dyn_group_update_node_steps(crane_dyn_group *g, int64_t k, const int64_t *idx, const double *val,
                                      const int64_t *ts, const double *hv, const int64_t *hv_ts, int64_t t0_ns,
                                      int64_t t1_ns, uint8_t *n_steps, int64_t *bp, int8_t *first_fail,
                                      int8_t *score);
int crane_dyn_group_resize_nodes(crane_dyn_group *g, int64_t n);
int crane_dyn_group_binding_records(crane_dyn_group *g, int64_t size, int64_t gc_time_range_ns);
int crane_dyn_group_add_bindings(crane_dyn_group *g, int64_t n, const int32_t *node, const int64_t *ts_s);
int crane_dyn_group_gc_bindings(crane_dyn_group *g, int64_t now_ns);
int64_t crane_dyn_group_binding_count(crane_dyn_group *g);
int crane_dyn_group_refresh_hot_values(crane_dyn_group *g, int64_t now_ns, int64_t hv_ts_ns);
int crane_dyn_group_hot_values(crane_dyn_group *g, int64_t n, double *hv_out);
int crane_dyn_group_node_steps(crane_dyn_group *g, int64_t t0_ns, int64_t t1_ns, int64_t n, uint8_t *n_steps,
                               int64_t *bp, int8_t *first_fail, int8_t *score);
/* One batch from host arrays, synchronous: chosen[p] = global node index or -1, chosen_score[p]
 * (either may be NULL) — the scheduler's call per pod batch. */
int crane_dyn_group_schedule(crane_dyn_group *g, int64_t now_ns, int64_t hv_ts_ns, int64_t n_pods,
                             const int64_t *now_pods, const uint8_t *pod_flags, int64_t *chosen,
                             int64_t *chosen_score);

/* ------------------------------------------------------------------ events
 * translateEventToBinding (event.go:118-145): a Scheduled event's message
 * "Successfully assigned <namespace>/<pod> to <node>" (fmt.Fscanf with two %s)
 * and its timestamps -> the Binding the controller records.  Timestamp =
 * EventTime.Unix() when count == 0, else LastTimestamp.Unix() (times in Unix
 * ns here).  On success *node / *node_len point into msg, and likewise the
 * namespace ("" for a key without '/') and pod name.  Returns CRANE_E_PARSE
 * for a message that does not scan or a key with more than one '/'
 * (cache.SplitMetaNamespaceKey). */
int crane_translate_event(const char *msg, size_t n, int32_t count, int64_t event_time_ns, int64_t last_timestamp_ns,
                          const char **node, size_t *node_len, const char **ns, size_t *ns_len, const char **pod,
                          size_t *pod_len, int64_t *ts_s);

#ifdef __cplusplus
}
#endif
#endif
