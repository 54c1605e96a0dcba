"""crane_dyn — Python binding of the MI355X Dynamic-plugin engine (libcrane_dyn.so).

A thin ctypes layer over include/crane_dyn.h.  There is no CPU fallback: if the
HIP library is missing, importing this module raises.  Build it with
``make -C crane-scheduler_amd/csrc`` (or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libcrane_dyn.so")

CRANE_TS_INVALID = -(2**63)
CRANE_POD_DAEMONSET = 1
_ERRS = {-1: "invalid argument", -2: "HIP error", -3: "bad state", -4: "policy parse error", -5: "I/O error"}


class CraneError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{_ERRS.get(code, code)}: {msg}")
        self.code = code


class _CPolicy(C.Structure):
    _fields_ = [
        ("n_sync", C.c_int32), ("sync_name", C.POINTER(C.c_char_p)), ("sync_period_ns", C.POINTER(C.c_int64)),
        ("n_pred", C.c_int32), ("pred_name", C.POINTER(C.c_char_p)), ("pred_limit", C.POINTER(C.c_double)),
        ("n_prio", C.c_int32), ("prio_name", C.POINTER(C.c_char_p)), ("prio_weight", C.POINTER(C.c_double)),
        ("n_hot", C.c_int32), ("hot_tr_ns", C.POINTER(C.c_int64)), ("hot_count", C.POINTER(C.c_int64)),
    ]


def _load():
    # PyTorch-ROCm bundles its own libamdhip64.so with the same SONAME
    # (libamdhip64.so.7).  Loading torch first makes this library bind to that
    # same HIP runtime, so device pointers and streams are shared; loading it
    # first would put two HIP runtimes in the process.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"crane_dyn: HIP library not built ({LIB_PATH}); run make -C crane-scheduler_amd/csrc")
    L = C.CDLL(LIB_PATH)
    P, vp = C.POINTER, C.c_void_p
    sig = {
        "crane_policy_load_file": (C.c_int, [C.c_char_p, P(vp), C.c_char_p, C.c_size_t]),
        "crane_policy_load_bytes": (C.c_int, [C.c_char_p, C.c_size_t, P(vp), C.c_char_p, C.c_size_t]),
        "crane_policy_view": (P(_CPolicy), [vp]),
        "crane_policy_free": (None, [vp]),
        "crane_tz_offset": (C.c_int, [C.c_char_p, P(C.c_int64)]),
        "crane_parse_annotation": (None, [C.c_char_p, C.c_size_t, C.c_int64, P(C.c_double), P(C.c_int64)]),
        "crane_parse_annotations": (C.c_int, [C.c_int64, vp, vp, C.c_int64, vp, vp, C.c_int32]),
        "crane_tz_load": (C.c_int, [C.c_char_p, C.c_char_p, P(vp)]),
        "crane_tz_load_bytes": (C.c_int, [C.c_char_p, C.c_size_t, P(vp)]),
        "crane_tz_free": (None, [vp]),
        "crane_tz_lookup": (C.c_int, [vp, C.c_int64, P(C.c_int32), P(C.c_int64), P(C.c_int64)]),
        "crane_tz_date": (C.c_int64, [vp, C.c_int64]),
        "crane_parse_annotation_tz": (None, [C.c_char_p, C.c_size_t, vp, P(C.c_double), P(C.c_int64)]),
        "crane_parse_annotations_tz": (C.c_int, [C.c_int64, vp, vp, vp, vp, vp, C.c_int32]),
        "crane_dyn_create": (C.c_int, [P(_CPolicy), C.c_int32, P(vp)]),
        "crane_dyn_destroy": (C.c_int, [vp]),
        "crane_dyn_last_error": (C.c_char_p, [vp]),
        "crane_dyn_num_metrics": (C.c_int32, [vp]),
        "crane_dyn_metric_name": (C.c_char_p, [vp, C.c_int32]),
        "crane_dyn_upload_nodes": (C.c_int, [vp, C.c_int64, C.c_int64, vp, vp, vp, vp]),
        "crane_dyn_upload_bindings": (C.c_int, [vp, C.c_int64, vp, vp]),
        "crane_dyn_binding_records": (C.c_int, [vp, C.c_int64, C.c_int64]),
        "crane_dyn_add_bindings": (C.c_int, [vp, C.c_int64, vp, vp]),
        "crane_dyn_gc_bindings": (C.c_int, [vp, C.c_int64]),
        "crane_dyn_binding_count": (C.c_int64, [vp]),
        "crane_dyn_eval_compact": (C.c_int, [vp, C.c_int64, vp, vp, vp, vp, vp, vp]),
        "crane_dyn_eval_matrix_async": (C.c_int, [vp, C.c_int64, vp, vp, vp, vp, C.c_int64, vp, vp]),
        "crane_dyn_set_option": (C.c_int, [vp, C.c_char_p, C.c_int64]),
        "crane_num_feasible_nodes_to_find": (C.c_int64, [C.c_int64, C.c_int32]),
        "crane_dyn_select": (C.c_int, [vp, C.c_int64, vp, vp, vp, vp, C.c_int64, C.c_int32, C.c_int64, C.c_uint64,
                                       vp, vp, vp, vp, P(C.c_int64), vp]),
        "crane_dyn_debug_trace": (C.c_int64, [vp, C.c_int32, C.c_int64, vp]),
        "crane_translate_event": (C.c_int, [C.c_char_p, C.c_size_t, C.c_int32, C.c_int64, C.c_int64, P(C.c_char_p),
                                            P(C.c_size_t), P(C.c_char_p), P(C.c_size_t), P(C.c_char_p),
                                            P(C.c_size_t), P(C.c_int64)]),
        "crane_dyn_refresh_hot_values": (C.c_int, [vp, C.c_int64, C.c_int64]),
        "crane_dyn_hot_values": (C.c_int, [vp, C.c_int64, vp]),
        "crane_dyn_eval": (C.c_int, [vp, C.c_int64, vp, vp, vp, vp, vp, vp]),
        "crane_dyn_eval_keys_async": (C.c_int, [vp, C.c_int64, vp, vp, vp, vp]),
        "crane_dyn_step_keys_async": (C.c_int, [vp, C.c_int64, C.c_int64, C.c_int64, vp, vp, vp, vp]),
        "crane_dyn_refresh_hot_values_async": (C.c_int, [vp, C.c_int64, C.c_int64, vp]),
        "crane_dyn_node_pass_async": (C.c_int, [vp, vp]),
        "crane_dyn_greedy": (C.c_int, [vp, C.c_int64, C.c_int64, vp, vp]),
        "crane_dyn_set_profiling": (C.c_int, [vp, C.c_int]),
        "crane_dyn_stage_times": (C.c_int, [vp, C.c_int32, P(C.c_char_p), P(C.c_double)]),
        "crane_dyn_key_node": (C.c_int64, [C.c_int64, P(C.c_int64)]),
        "crane_dyn_step_slots": (C.c_int32, [vp]),
        "crane_dyn_node_steps": (C.c_int, [vp, C.c_int64, C.c_int64, C.c_int64, vp, vp, vp, vp]),
        "crane_dyn_node_steps_subset": (C.c_int, [vp, C.c_int64, C.c_int64, C.c_int64, vp, vp, vp, vp, vp]),
        "crane_dyn_update_nodes": (C.c_int, [vp, C.c_int64, vp, vp, vp, vp, vp]),
        "crane_dyn_update_node_steps": (C.c_int, [vp, C.c_int64, vp, vp, vp, vp, vp, C.c_int64, C.c_int64, vp, vp, vp,
                                                  vp]),
        "crane_dyn_version": (C.c_char_p, []),
        "crane_dyn_forget_stream": (C.c_int, [vp, vp]),
        "crane_dyn_resize_nodes": (C.c_int, [vp, C.c_int64]),
        "crane_shard_range": (C.c_int, [C.c_int64, C.c_int32, C.c_int32, P(C.c_int64), P(C.c_int64)]),
        "crane_dyn_group_create": (C.c_int, [P(_CPolicy), C.c_int32, vp, C.c_int32, P(vp)]),
        "crane_dyn_group_destroy": (C.c_int, [vp]),
        "crane_dyn_group_last_error": (C.c_char_p, [vp]),
        "crane_dyn_group_set_option": (C.c_int, [vp, C.c_char_p, C.c_int64]),
        "crane_dyn_group_size": (C.c_int32, [vp]),
        "crane_dyn_group_shard": (C.c_int, [vp, C.c_int32, P(C.c_int32), P(C.c_int64), P(C.c_int64)]),
        "crane_dyn_group_engine": (vp, [vp, C.c_int32, C.c_int32]),
        "crane_dyn_group_upload_nodes": (C.c_int, [vp, C.c_int64, vp, vp, vp, vp]),
        "crane_dyn_group_upload_bindings": (C.c_int, [vp, C.c_int64, vp, vp]),
        "crane_dyn_group_step_keys_async": (C.c_int, [vp, C.c_int64, C.c_int64, C.c_int64, vp, vp, vp]),
        "crane_dyn_group_sync": (C.c_int, [vp]),
        "crane_dyn_group_schedule": (C.c_int, [vp, C.c_int64, C.c_int64, C.c_int64, vp, vp, vp, vp]),
        "crane_dyn_group_step_keys_batch": (C.c_int, [vp, C.c_int32, vp, vp, C.c_int64, vp, vp, vp]),
        "crane_dyn_group_update_nodes": (C.c_int, [vp, C.c_int64, vp, vp, vp, vp, vp]),
        "crane_dyn_group_update_node_steps": (C.c_int, [vp, C.c_int64, vp, vp, vp, vp, vp, C.c_int64, C.c_int64,
                                                        vp, vp, vp, vp]),
        "crane_dyn_group_resize_nodes": (C.c_int, [vp, C.c_int64]),
        "crane_dyn_group_binding_records": (C.c_int, [vp, C.c_int64, C.c_int64]),
        "crane_dyn_group_add_bindings": (C.c_int, [vp, C.c_int64, vp, vp]),
        "crane_dyn_group_gc_bindings": (C.c_int, [vp, C.c_int64]),
        "crane_dyn_group_binding_count": (C.c_int64, [vp]),
        "crane_dyn_group_refresh_hot_values": (C.c_int, [vp, C.c_int64, C.c_int64]),
        "crane_dyn_group_hot_values": (C.c_int, [vp, C.c_int64, vp]),
        "crane_dyn_group_node_steps": (C.c_int, [vp, C.c_int64, C.c_int64, C.c_int64, vp, vp, vp, vp]),
        "crane_queue_create": (C.c_int, [C.c_int32, C.c_int32, P(vp)]),
        "crane_queue_wait": (C.c_int, [vp]),
        "crane_queue_last_error": (C.c_char_p, [vp]),
        "crane_queue_destroy": (C.c_int, [vp]),
        "crane_dyn_step_keys_queue": (C.c_int, [vp, C.c_int64, C.c_int64, C.c_int64, vp, vp, vp, vp]),
        "crane_dyn_forget_queue": (C.c_int, [vp, vp]),
        "crane_dyn_step_flush": (C.c_int, [vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


lib = _load()

# The symbols include/crane_dyn.h declares (checked by tests/test_abi.py).
ABI_SYMBOLS = (
    "crane_policy_load_file", "crane_policy_load_bytes", "crane_policy_view", "crane_policy_free",
    "crane_tz_offset", "crane_parse_annotation", "crane_parse_annotations", "crane_dyn_create", "crane_dyn_destroy", "crane_dyn_last_error",
    "crane_dyn_num_metrics", "crane_dyn_metric_name", "crane_dyn_upload_nodes", "crane_dyn_upload_bindings",
    "crane_dyn_refresh_hot_values", "crane_dyn_eval", "crane_dyn_eval_keys_async", "crane_dyn_step_keys_async",
    "crane_dyn_refresh_hot_values_async", "crane_dyn_node_pass_async", "crane_dyn_greedy", "crane_dyn_key_node",
    "crane_dyn_set_profiling", "crane_dyn_stage_times", "crane_dyn_hot_values",
    "crane_dyn_version", "crane_dyn_binding_records", "crane_dyn_add_bindings", "crane_dyn_gc_bindings",
    "crane_dyn_binding_count", "crane_dyn_eval_compact", "crane_dyn_eval_matrix_async", "crane_dyn_set_option",
    "crane_translate_event", "crane_dyn_debug_trace", "crane_num_feasible_nodes_to_find", "crane_dyn_select",
    "crane_tz_load", "crane_tz_load_bytes", "crane_tz_free", "crane_tz_lookup", "crane_tz_date",
    "crane_parse_annotation_tz", "crane_parse_annotations_tz", "crane_dyn_step_slots", "crane_dyn_node_steps",
    "crane_dyn_node_steps_subset", "crane_dyn_update_nodes", "crane_dyn_update_node_steps",
    "crane_dyn_forget_stream", "crane_dyn_resize_nodes", "crane_shard_range", "crane_dyn_group_create", "crane_dyn_group_destroy",
    "crane_dyn_group_last_error", "crane_dyn_group_set_option", "crane_dyn_group_size", "crane_dyn_group_shard",
    "crane_dyn_group_engine", "crane_dyn_group_upload_nodes", "crane_dyn_group_upload_bindings",
    "crane_dyn_group_step_keys_async", "crane_dyn_group_sync", "crane_dyn_group_schedule",
    "crane_dyn_group_step_keys_batch", "crane_dyn_group_update_nodes", "crane_dyn_group_update_node_steps",
    "crane_dyn_group_resize_nodes", "crane_dyn_group_binding_records", "crane_dyn_group_add_bindings",
    "crane_dyn_group_gc_bindings", "crane_dyn_group_binding_count", "crane_dyn_group_refresh_hot_values",
    "crane_dyn_group_hot_values", "crane_dyn_group_node_steps",
    "crane_queue_create", "crane_queue_wait", "crane_queue_last_error", "crane_queue_destroy",
    "crane_dyn_step_keys_queue", "crane_dyn_forget_queue", "crane_dyn_step_flush",
)


def _ptr(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def num_feasible_nodes_to_find(n_nodes, percentage=0):
    """kube-scheduler v1.23.3 numFeasibleNodesToFind (crane_num_feasible_nodes_to_find)."""
    return lib.crane_num_feasible_nodes_to_find(int(n_nodes), int(percentage))


# ------------------------------------------------------------------ policy
class Policy:
    """A DynamicSchedulerPolicy spec (pkg/plugins/apis/policy/types.go:14-39).

    Build from a dict {"syncPolicy": [(name, period_ns)], "predicate": [(name, maxLimitPecent)],
    "priority": [(name, weight)], "hotValue": [(timeRange_ns, count)]}, or decode a policy
    file with :meth:`load_file` / :meth:`load_bytes` (strict, like LoadPolicyFromFile).
    """

    def __init__(self, spec):
        self.spec = {k: [tuple(x) for x in spec.get(k, [])] for k in ("syncPolicy", "predicate", "priority", "hotValue")}
        sp, pr, pi, hv = (self.spec[k] for k in ("syncPolicy", "predicate", "priority", "hotValue"))
        n = lambda xs: max(1, len(xs))  # noqa: E731
        self._keep = [
            (C.c_char_p * n(sp))(*[a.encode() for a, _ in sp]), (C.c_int64 * n(sp))(*[int(b) for _, b in sp]),
            (C.c_char_p * n(pr))(*[a.encode() for a, _ in pr]), (C.c_double * n(pr))(*[float(b) for _, b in pr]),
            (C.c_char_p * n(pi))(*[a.encode() for a, _ in pi]), (C.c_double * n(pi))(*[float(b) for _, b in pi]),
            (C.c_int64 * n(hv))(*[int(a) for a, _ in hv]), (C.c_int64 * n(hv))(*[int(b) for _, b in hv]),
        ]
        k = self._keep
        cp = C.POINTER
        self.c = _CPolicy(len(sp), C.cast(k[0], cp(C.c_char_p)), C.cast(k[1], cp(C.c_int64)),
                          len(pr), C.cast(k[2], cp(C.c_char_p)), C.cast(k[3], cp(C.c_double)),
                          len(pi), C.cast(k[4], cp(C.c_char_p)), C.cast(k[5], cp(C.c_double)),
                          len(hv), C.cast(k[6], cp(C.c_int64)), C.cast(k[7], cp(C.c_int64)))

    @staticmethod
    def _from_doc(doc):
        v = lib.crane_policy_view(doc).contents
        spec = {
            "syncPolicy": [(v.sync_name[i].decode(), v.sync_period_ns[i]) for i in range(v.n_sync)],
            "predicate": [(v.pred_name[i].decode(), v.pred_limit[i]) for i in range(v.n_pred)],
            "priority": [(v.prio_name[i].decode(), v.prio_weight[i]) for i in range(v.n_prio)],
            "hotValue": [(v.hot_tr_ns[i], v.hot_count[i]) for i in range(v.n_hot)],
        }
        lib.crane_policy_free(doc)
        return Policy(spec)

    @staticmethod
    def load_bytes(data: bytes | str) -> "Policy":
        if isinstance(data, str):
            data = data.encode()
        doc, err = C.c_void_p(), C.create_string_buffer(512)
        rc = lib.crane_policy_load_bytes(data, len(data), C.byref(doc), err, len(err))
        if rc:
            raise CraneError(rc, err.value.decode())
        return Policy._from_doc(doc)

    @staticmethod
    def load_file(path: str) -> "Policy":
        doc, err = C.c_void_p(), C.create_string_buffer(512)
        rc = lib.crane_policy_load_file(path.encode(), C.byref(doc), err, len(err))
        if rc:
            raise CraneError(rc, err.value.decode())
        return Policy._from_doc(doc)


def default_policy_spec():
    """deploy/manifests/dynamic/policy.yaml:1-52 (the README default policy)."""
    m = 60 * 10**9
    return {
        "syncPolicy": [("cpu_usage_avg_5m", 3 * m), ("cpu_usage_max_avg_1h", 15 * m), ("cpu_usage_max_avg_1d", 180 * m),
                       ("mem_usage_avg_5m", 3 * m), ("mem_usage_max_avg_1h", 15 * m), ("mem_usage_max_avg_1d", 180 * m)],
        "predicate": [("cpu_usage_avg_5m", 0.65), ("cpu_usage_max_avg_1h", 0.75), ("mem_usage_avg_5m", 0.65),
                      ("mem_usage_max_avg_1h", 0.75)],
        "priority": [("cpu_usage_avg_5m", 0.2), ("cpu_usage_max_avg_1h", 0.3), ("cpu_usage_max_avg_1d", 0.5),
                     ("mem_usage_avg_5m", 0.2), ("mem_usage_max_avg_1h", 0.3), ("mem_usage_max_avg_1d", 0.5)],
        "hotValue": [(5 * m, 5), (1 * m, 2)],
    }


# ------------------------------------------------------------- annotations
def tz_offset(name: str | None = None) -> int:
    off = C.c_int64()
    rc = lib.crane_tz_offset(None if name is None else name.encode(), C.byref(off))
    if rc:
        raise CraneError(rc, f"unsupported time zone {name!r}")
    return off.value


def parse_annotation(s: str, tz_offset_s: int):
    """(value, ts_ns) of one annotation value; ts_ns == CRANE_TS_INVALID when unusable."""
    b = s.encode()
    v, t = C.c_double(), C.c_int64()
    lib.crane_parse_annotation(b, len(b), tz_offset_s, C.byref(v), C.byref(t))
    return v.value, t.value


class Zone:
    """An IANA time zone with go1.17's semantics (tz.cpp): Zone(name, zoneinfo_dir) like
    time.LoadLocation, or Zone(tzif=bytes) like LoadLocationFromTZData."""

    def __init__(self, name=None, zoneinfo_dir=None, tzif=None):
        h = C.c_void_p()
        if tzif is not None:
            rc = lib.crane_tz_load_bytes(tzif, len(tzif), C.byref(h))
        else:
            rc = lib.crane_tz_load((name or "").encode(), None if zoneinfo_dir is None else zoneinfo_dir.encode(),
                                   C.byref(h))
        if rc:
            raise CraneError(rc, f"time zone {name!r} not loadable")
        self.h = h

    def lookup(self, unix_s):
        """Location.lookup: (offset_s, start_s, end_s) of the zone period holding unix_s."""
        off, st, en = C.c_int32(), C.c_int64(), C.c_int64()
        lib.crane_tz_lookup(self.h, int(unix_s), C.byref(off), C.byref(st), C.byref(en))
        return off.value, st.value, en.value

    def date(self, local_s):
        """time.Date: wall clock (seconds since the epoch as if UTC) -> Unix seconds."""
        return lib.crane_tz_date(self.h, int(local_s))

    def parse_annotation(self, s: str):
        b = s.encode()
        v, t = C.c_double(), C.c_int64()
        lib.crane_parse_annotation_tz(b, len(b), self.h, C.byref(v), C.byref(t))
        return v.value, t.value

    def close(self):
        if self.h:
            lib.crane_tz_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SnapshotStrings:
    """A node snapshot's annotation strings encoded once, row-major [M+1][N] (the
    metrics, then node_hot_value; None = key missing), for repeated bulk parses
    through crane_parse_annotations (the once-per-sync parse of SURVEY §8f row 2)."""

    def __init__(self, metric_names, nodes):
        self.M, self.N = len(metric_names), len(nodes)
        keys = list(metric_names) + ["node_hot_value"]
        self._enc = [None if x is None else x.encode() for x in (a.get(k) for k in keys for a in nodes)]
        # one contiguous buffer, as the cgo shim builds it, NULL = key missing
        self._lens = np.array([0 if x is None else len(x) for x in self._enc], dtype=np.uint64)
        self._buf = C.create_string_buffer(b"".join(x for x in self._enc if x is not None), int(self._lens.sum()) + 1)
        offs = np.concatenate(([0], np.cumsum(self._lens)[:-1])).astype(np.uint64) if len(self._enc) else self._lens
        self._strs = np.where([x is not None for x in self._enc], C.addressof(self._buf) + offs, 0).astype(np.uint64)
        self.val = np.zeros(len(self._enc))
        self.ts = np.empty(len(self._enc), np.int64)

    def __len__(self):
        return len(self._enc)

    def parse(self, tz, threads=0):
        """Parse every string into self.val / self.ts (flat [M+1][N]); tz: a fixed offset in
        seconds or a Zone; host threads <= 0 = all."""
        if isinstance(tz, Zone):
            rc = lib.crane_parse_annotations_tz(len(self._enc), _ptr(self._strs), _ptr(self._lens), tz.h,
                                                _ptr(self.val), _ptr(self.ts), threads)
        else:
            rc = lib.crane_parse_annotations(len(self._enc), _ptr(self._strs), _ptr(self._lens),
                                             tz, _ptr(self.val), _ptr(self.ts), threads)
        if rc:
            raise CraneError(rc, "bulk annotation parse")

    def soa(self):
        """(val[M][N], ts[M][N], hv[N], hv_ts[N]) from the last parse."""
        M, N = self.M, self.N
        val, ts = self.val.reshape(M + 1, N), self.ts.reshape(M + 1, N)
        return val[:M].copy(), ts[:M].copy(), val[M].copy(), ts[M].copy()


def parse_nodes(metric_names, nodes, tz_offset_s, threads=0):
    """Node annotation dicts -> SoA (val[M][N], ts[M][N], hv[N], hv_ts[N]) in one bulk parse."""
    snap = SnapshotStrings(metric_names, nodes)
    snap.parse(tz_offset_s, threads)
    return snap.soa()


def translate_event(message: str, count: int, event_time_ns: int, last_timestamp_ns: int):
    """translateEventToBinding (event.go:118-145): (namespace, pod, node, Timestamp) or None."""
    b = message.encode()
    node, ns, pod = C.c_char_p(), C.c_char_p(), C.c_char_p()
    nl, nsl, pl, ts = C.c_size_t(), C.c_size_t(), C.c_size_t(), C.c_int64()
    buf = C.create_string_buffer(b, len(b))
    rc = lib.crane_translate_event(buf, len(b), count, event_time_ns, last_timestamp_ns, C.byref(node), C.byref(nl),
                                   C.byref(ns), C.byref(nsl), C.byref(pod), C.byref(pl), C.byref(ts))
    if rc:
        return None
    base = C.addressof(buf)

    def get(p, n):
        off = C.cast(p, C.c_void_p).value - base
        return b[off:off + n.value].decode("utf-8", "surrogateescape")
    return get(ns, nsl), get(pod, pl), get(node, nl), ts.value


def key_node(key: int):
    s = C.c_int64()
    n = lib.crane_dyn_key_node(int(key), C.byref(s))
    return n, s.value


# ------------------------------------------------------------------ engine
class Engine:
    """One engine = one node shard on one HIP device (crane_dyn_create)."""

    def __init__(self, policy: Policy, device: int = 0):
        self.policy = policy
        h = C.c_void_p()
        rc = lib.crane_dyn_create(C.byref(policy.c), device, C.byref(h))
        self.h = h
        if rc:
            msg = lib.crane_dyn_last_error(h).decode() if h.value else ""
            self.close()
            raise CraneError(rc, msg)
        self.metric_names = [lib.crane_dyn_metric_name(h, i).decode() for i in range(lib.crane_dyn_num_metrics(h))]
        self.n_nodes = 0
        self.device = device

    def close(self):
        if getattr(self, "h", None) and self.h.value and lib is not None:
            lib.crane_dyn_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        self.close()

    def _check(self, rc):
        if rc:
            raise CraneError(rc, lib.crane_dyn_last_error(self.h).decode())

    def _ready(self, stream):
        """stream None = the engine's own stream, which is non-blocking: it is not ordered
        after torch's current stream, so wait for that first (tensors torch just filled must
        be written before the engine reads or overwrites them).  Results on the engine
        stream still need a synchronize before torch reads them."""
        if stream is None:
            import torch
            torch.cuda.current_stream(self.device).synchronize()

    def upload_nodes(self, val, ts, hv=None, hv_ts=None, node_offset=0):
        val = np.ascontiguousarray(val, np.float64)
        ts = np.ascontiguousarray(ts, np.int64)
        M = len(self.metric_names)
        N = val.shape[1] if val.ndim == 2 else (len(hv) if hv is not None else 0)
        if val.shape != (M, N) or ts.shape != (M, N):
            raise ValueError(f"val/ts must be [{M}][N] in engine metric order {self.metric_names}")
        if hv is not None:
            hv = np.ascontiguousarray(hv, np.float64)
            hv_ts = np.ascontiguousarray(hv_ts, np.int64)
            if hv.shape != (N,) or hv_ts.shape != (N,):
                raise ValueError("hv/hv_ts must have one entry per node")
        self._check(lib.crane_dyn_upload_nodes(self.h, N, node_offset, _ptr(val), _ptr(ts), _ptr(hv), _ptr(hv_ts)))
        self.n_nodes = N

    def upload_bindings(self, node, ts_s):
        node = np.ascontiguousarray(node, np.int32)
        ts_s = np.ascontiguousarray(ts_s, np.int64)
        if node.shape != ts_s.shape:
            raise ValueError("node/ts_s length mismatch")
        self._check(lib.crane_dyn_upload_bindings(self.h, len(node), _ptr(node), _ptr(ts_s)))

    # BindingRecords kept by the engine (binding.go:50-123)
    def binding_records(self, size, gc_time_range_ns):
        self._check(lib.crane_dyn_binding_records(self.h, int(size), int(gc_time_range_ns)))

    def add_bindings(self, node, ts_s):
        node = np.ascontiguousarray(node, np.int32)
        ts_s = np.ascontiguousarray(ts_s, np.int64)
        if node.shape != ts_s.shape:
            raise ValueError("node/ts_s length mismatch")
        self._check(lib.crane_dyn_add_bindings(self.h, len(node), _ptr(node), _ptr(ts_s)))

    def gc_bindings(self, now_ns):
        self._check(lib.crane_dyn_gc_bindings(self.h, int(now_ns)))

    def debug_trace(self, which, n_wgs):
        """Phase stamps [n_wgs][8] (100 MHz) of the last K2x (0) / K1 (1) / K3s (2) launch (option "trace")."""
        out = np.zeros(n_wgs * 8, np.uint64)
        n = lib.crane_dyn_debug_trace(self.h, which, len(out), _ptr(out))
        if n < 0:
            self._check(n)
        return out.reshape(n_wgs, 8)

    def binding_count(self):
        return lib.crane_dyn_binding_count(self.h)

    def set_option(self, name, value):
        """Alternative kernel forms of the same results (tests / A-B only), see crane_dyn.h."""
        self._check(lib.crane_dyn_set_option(self.h, name.encode(), int(value)))

    def refresh_hot_values(self, now_ns, hv_ts_ns=None):
        self._check(lib.crane_dyn_refresh_hot_values(self.h, int(now_ns), int(now_ns if hv_ts_ns is None else hv_ts_ns)))

    def hot_values(self):
        """Per-node hot value as Score uses it (controller side, node.go:113-121)."""
        out = np.empty(self.n_nodes, np.float64)
        self._check(lib.crane_dyn_hot_values(self.h, self.n_nodes, _ptr(out)))
        return out

    def eval(self, now_ns, pod_flags=None, matrix=False, compact=False):
        """Returns (first_fail[P,N] or None, score[P,N] or None, chosen[P], chosen_score[P]);
        compact: int8 scores (crane_dyn_eval_compact)."""
        now = np.ascontiguousarray(now_ns, np.int64).reshape(-1)
        P, N = len(now), self.n_nodes
        fl = None if pod_flags is None else np.ascontiguousarray(pod_flags, np.uint8).reshape(-1)
        if fl is not None and len(fl) != P:
            raise ValueError("pod_flags length mismatch")
        ff = np.empty((P, N), np.int8) if matrix else None
        sc = np.empty((P, N), np.int8 if compact else np.int64) if matrix else None
        ch = np.empty(P, np.int64)
        cs = np.empty(P, np.int64)
        fn = lib.crane_dyn_eval_compact if compact else lib.crane_dyn_eval
        self._check(fn(self.h, P, _ptr(now), _ptr(fl), _ptr(ff), _ptr(sc), _ptr(ch), _ptr(cs)))
        return ff, sc, ch, cs

    def eval_matrix_async(self, d_now, d_flags, d_ff, d_score, d_keys=None, ld=None, stream=None):
        """Device matrices (torch int8 [P][ld], either may be None) and optional keys int64[P]."""
        P = d_now.numel()
        ld = self.n_nodes if ld is None else ld
        self._ready(stream)
        vp = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
        self._check(lib.crane_dyn_eval_matrix_async(self.h, P, vp(d_now), vp(d_flags), vp(d_ff), vp(d_score), ld,
                                                    vp(d_keys), stream))

    def select(self, d_now, d_flags, d_chosen, d_total=None, d_ext_ok=None, d_ext_score=None, dyn_weight=3,
               percentage=0, start=0, tie_seed=0, d_wstart=None, d_wlen=None, stream=None):
        """Framework-level selection for the pod queue d_now (crane_dyn_select): torch device
        tensors; returns the start index after the queue."""
        P = d_now.numel()
        vp = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
        nxt = C.c_int64(0)
        self._ready(stream)
        self._check(lib.crane_dyn_select(self.h, P, vp(d_now), vp(d_flags), vp(d_ext_ok), vp(d_ext_score),
                                         int(dyn_weight), int(percentage), int(start), int(tie_seed), vp(d_chosen),
                                         vp(d_total), vp(d_wstart), vp(d_wlen), C.byref(nxt), stream))
        return nxt.value

    # device-resident pipeline (torch tensors on the engine's device)
    def refresh_hot_values_async(self, now_ns, hv_ts_ns, stream=None):
        self._ready(stream)
        self._check(lib.crane_dyn_refresh_hot_values_async(self.h, int(now_ns), int(hv_ts_ns), stream))

    def node_pass_async(self, stream=None):
        self._ready(stream)
        self._check(lib.crane_dyn_node_pass_async(self.h, stream))

    def eval_keys_async(self, d_now, d_flags, d_keys, stream=None):
        """d_now int64[P], d_flags uint8[P] or None, d_keys int64[P]: torch CUDA tensors."""
        P = d_now.numel()
        assert d_keys.numel() == P and d_now.dtype.itemsize == 8 and d_keys.dtype.itemsize == 8
        self._ready(stream)
        self._check(lib.crane_dyn_eval_keys_async(self.h, P, C.c_void_p(d_now.data_ptr()),
                                                  None if d_flags is None else C.c_void_p(d_flags.data_ptr()),
                                                  C.c_void_p(d_keys.data_ptr()), stream))

    def forget_stream(self, stream):
        """The caller is about to destroy `stream` (a raw hipStream_t handle): wait for it and drop
        the engine's handle of it (crane_dyn_forget_stream)."""
        self._check(lib.crane_dyn_forget_stream(self.h, stream))

    # stage timing: HIP events the engine records after each kernel stage
    def set_profiling(self, on=True):
        self._check(lib.crane_dyn_set_profiling(self.h, 1 if on else 0))

    def stage_times(self, max_stages=64):
        """[(stage name, ms)] of the stages enqueued since the last call (waits for them)."""
        names = (C.c_char_p * max_stages)()
        ms = (C.c_double * max_stages)()
        n = lib.crane_dyn_stage_times(self.h, max_stages, names, ms)
        if n < 0:
            self._check(n)
        return [(names[i].decode(), ms[i]) for i in range(n)]

    def step_keys_async(self, now_ns, hv_ts_ns, d_now, d_flags, d_keys, stream=None):
        """One scheduling step: hot-value refresh at now_ns + keys-only eval (torch CUDA tensors)."""
        P = d_now.numel()
        assert d_keys.numel() == P and d_now.dtype.itemsize == 8 and d_keys.dtype.itemsize == 8
        self._ready(stream)
        self._check(lib.crane_dyn_step_keys_async(self.h, int(now_ns), int(hv_ts_ns), P, C.c_void_p(d_now.data_ptr()),
                                                  None if d_flags is None else C.c_void_p(d_flags.data_ptr()),
                                                  C.c_void_p(d_keys.data_ptr()), stream))

    def step_keys_queue(self, now_ns, hv_ts_ns, d_now, d_flags, d_keys, queue):
        """step_keys_async with the kernels on a dispatch queue (Queue): the inputs must be complete
        on the device (torch.cuda.synchronize() after writing them); keys after queue.wait() (with
        engine option step_defer: after the next step on the queue or step_flush(), then the wait)."""
        P = d_now.numel()
        assert d_keys.numel() == P and d_now.dtype.itemsize == 8 and d_keys.dtype.itemsize == 8
        self._check(lib.crane_dyn_step_keys_queue(self.h, int(now_ns), int(hv_ts_ns), P, C.c_void_p(d_now.data_ptr()),
                                                  None if d_flags is None else C.c_void_p(d_flags.data_ptr()),
                                                  C.c_void_p(d_keys.data_ptr()), queue.h))

    def step_flush(self):
        """Option step_defer: run the last queue step's deferred K3s now (crane_dyn_step_flush)."""
        self._check(lib.crane_dyn_step_flush(self.h))

    def step_keys_fn(self, d_now, d_flags, d_keys, stream=None):
        """step_keys_async bound to fixed device buffers and stream: returns f(now_ns, hv_ts_ns).
        The pointer conversions happen once, so a loop of steps pays only the C call."""
        P = d_now.numel()
        assert d_keys.numel() == P and d_now.dtype.itemsize == 8 and d_keys.dtype.itemsize == 8
        fn, h = lib.crane_dyn_step_keys_async, self.h
        pn, pk = C.c_void_p(d_now.data_ptr()), C.c_void_p(d_keys.data_ptr())
        pf = None if d_flags is None else C.c_void_p(d_flags.data_ptr())
        check = self._check
        ready = self._ready if stream is None else None

        def step(now_ns, hv_ts_ns):
            if ready:
                ready(None)
            rc = fn(h, now_ns, hv_ts_ns, P, pn, pf, pk, stream)
            if rc:
                check(rc)

        return step

    def node_steps(self, t0_ns, t1_ns):
        """Every node's Filter / Score over [t0, t1) as step functions (crane_dyn_node_steps):
        (n_steps[N] u8, bp[N][S] i64, first_fail[N][S+1] i8, score[N][S+1] i8)."""
        S, N = lib.crane_dyn_step_slots(self.h), self.n_nodes
        ns = np.zeros(N, np.uint8)
        bp = np.zeros((N, S), np.int64)
        ff = np.zeros((N, S + 1), np.int8)
        sc = np.zeros((N, S + 1), np.int8)
        self._check(lib.crane_dyn_node_steps(self.h, int(t0_ns), int(t1_ns), N, _ptr(ns), _ptr(bp), _ptr(ff),
                                             _ptr(sc)))
        return ns, bp, ff, sc

    def node_steps_subset(self, t0_ns, t1_ns, idx):
        """node_steps rows of the nodes idx only (crane_dyn_node_steps_subset), as compact rows."""
        idx = np.ascontiguousarray(idx, np.int64)
        S, k = lib.crane_dyn_step_slots(self.h), len(idx)
        ns = np.zeros(k, np.uint8)
        bp = np.zeros((k, S), np.int64)
        ff = np.zeros((k, S + 1), np.int8)
        sc = np.zeros((k, S + 1), np.int8)
        self._check(lib.crane_dyn_node_steps_subset(self.h, int(t0_ns), int(t1_ns), k, _ptr(idx), _ptr(ns), _ptr(bp),
                                                    _ptr(ff), _ptr(sc)))
        return ns, bp, ff, sc

    def update_nodes(self, idx, val, ts, hv=None, hv_ts=None):
        """Replace the parsed annotations of nodes idx (crane_dyn_update_nodes): val / ts [M][k]
        in engine metric order, hv / hv_ts [k] or None (no node_hot_value on those nodes)."""
        idx = np.ascontiguousarray(idx, np.int64)
        k, M = len(idx), len(self.metric_names)
        val = np.ascontiguousarray(val, np.float64).reshape(M, k)
        ts = np.ascontiguousarray(ts, np.int64).reshape(M, k)
        if hv is not None:
            hv = np.ascontiguousarray(hv, np.float64).reshape(k)
            hv_ts = np.ascontiguousarray(hv_ts, np.int64).reshape(k)
        self._check(lib.crane_dyn_update_nodes(self.h, k, _ptr(idx), _ptr(val), _ptr(ts), _ptr(hv), _ptr(hv_ts)))

    def resize_nodes(self, n):
        """Grow / shrink the shard to n nodes (crane_dyn_resize_nodes): new nodes have no annotations."""
        self._check(lib.crane_dyn_resize_nodes(self.h, int(n)))
        self.n_nodes = int(n)

    def update_node_steps(self, idx, val, ts, hv, hv_ts, t0_ns, t1_ns):
        """update_nodes + node_steps_subset of the same nodes in one call (crane_dyn_update_node_steps)."""
        idx = np.ascontiguousarray(idx, np.int64)
        k, M = len(idx), len(self.metric_names)
        val = np.ascontiguousarray(val, np.float64).reshape(M, k)
        ts = np.ascontiguousarray(ts, np.int64).reshape(M, k)
        if hv is not None:
            hv = np.ascontiguousarray(hv, np.float64).reshape(k)
            hv_ts = np.ascontiguousarray(hv_ts, np.int64).reshape(k)
        S = lib.crane_dyn_step_slots(self.h)
        ns = np.zeros(k, np.uint8)
        bp = np.zeros((k, S), np.int64)
        ff = np.zeros((k, S + 1), np.int8)
        sc = np.zeros((k, S + 1), np.int8)
        self._check(lib.crane_dyn_update_node_steps(self.h, k, _ptr(idx), _ptr(val), _ptr(ts), _ptr(hv), _ptr(hv_ts),
                                                    int(t0_ns), int(t1_ns), _ptr(ns), _ptr(bp), _ptr(ff), _ptr(sc)))
        return ns, bp, ff, sc

    @staticmethod
    def table_lookup(tables, now_ns):
        """first_fail[N], score[N] at now_ns from node_steps tables (what the plugin does per call)."""
        ns, bp, ff, sc = tables
        j = ((bp <= now_ns) & (np.arange(bp.shape[1])[None, :] < ns[:, None])).sum(1)
        r = np.arange(len(ns))
        return ff[r, j], sc[r, j]

    def greedy(self, n_pods, now_ns, pod_flags=None):
        fl = None if pod_flags is None else np.ascontiguousarray(pod_flags, np.uint8)
        ch = np.empty(n_pods, np.int64)
        self._check(lib.crane_dyn_greedy(self.h, n_pods, int(now_ns), _ptr(fl), _ptr(ch)))
        return ch


def shard_range(n_nodes, n_shards, shard):
    """Contiguous balanced node range [lo, hi) of one shard (crane_shard_range)."""
    lo, hi = C.c_int64(), C.c_int64()
    rc = lib.crane_shard_range(int(n_nodes), int(n_shards), int(shard), C.byref(lo), C.byref(hi))
    if rc:
        raise CraneError(rc, "bad shard arguments")
    return lo.value, hi.value


class _BorrowedEngine(Engine):
    """A group's engine (crane_dyn_group_engine): the group owns and destroys it."""

    def __init__(self, h, policy, device):
        self.policy, self.h, self.device, self.n_nodes = policy, C.c_void_p(h), device, 0
        self.metric_names = [lib.crane_dyn_metric_name(self.h, i).decode()
                             for i in range(lib.crane_dyn_num_metrics(self.h))]

    def close(self):
        self.h = C.c_void_p()


class Queue:
    """A dispatch queue (crane_queue_*): a user-mode AQL queue on one device that an engine's step
    kernels are written to as packets (Engine.step_keys_queue).  ring_kind 0: kernel arguments in
    device memory, 1: in pinned host memory."""

    def __init__(self, device=0, ring_kind=0):
        h = C.c_void_p()
        rc = lib.crane_queue_create(int(device), int(ring_kind), C.byref(h))
        self.h = h
        if rc:
            msg = lib.crane_queue_last_error(h).decode() if h.value else ""
            self.close()
            raise CraneError(rc, msg)

    def wait(self):
        if lib.crane_queue_wait(self.h):
            raise CraneError(-2, lib.crane_queue_last_error(self.h).decode())

    def close(self):
        if getattr(self, "h", None) and self.h.value and lib is not None:
            lib.crane_queue_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        self.close()


class Group:
    """One process, N devices (crane_dyn_group_*): node shards over the devices, `depth` batches in
    flight, the shards' keys max-combined by an in-library RCCL all-reduce (ncclCommInitAll)."""

    def __init__(self, policy: Policy, devices=(0,), depth: int = 1):
        self.policy = policy
        self.devices = [int(d) for d in devices]
        self.depth = int(depth)
        dv = (C.c_int32 * len(self.devices))(*self.devices)
        h = C.c_void_p()
        rc = lib.crane_dyn_group_create(C.byref(policy.c), len(self.devices), C.cast(dv, C.c_void_p), self.depth,
                                        C.byref(h))
        self.h = h
        if rc:
            msg = lib.crane_dyn_group_last_error(h).decode() if h.value else ""
            self.close()
            raise CraneError(rc, msg)
        self.n_nodes = 0
        self.metric_names = self.engine(0).metric_names

    def close(self):
        if getattr(self, "h", None) and self.h.value and lib is not None:
            lib.crane_dyn_group_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        self.close()

    def _check(self, rc):
        if rc:
            raise CraneError(rc, lib.crane_dyn_group_last_error(self.h).decode())

    def engine(self, i, slot=0):
        """Shard i's engine for batch slot `slot` (borrowed: the group destroys it)."""
        p = lib.crane_dyn_group_engine(self.h, int(i), int(slot))
        if not p:
            raise CraneError(-1, "no such shard / slot")
        return _BorrowedEngine(p, self.policy, self.devices[i])

    def set_option(self, name, value):
        self._check(lib.crane_dyn_group_set_option(self.h, name.encode(), int(value)))

    def shard(self, i):
        """(device, lo, hi) of shard i."""
        d, lo, hi = C.c_int32(), C.c_int64(), C.c_int64()
        self._check(lib.crane_dyn_group_shard(self.h, int(i), C.byref(d), C.byref(lo), C.byref(hi)))
        return d.value, lo.value, hi.value

    def upload_nodes(self, val, ts, hv=None, hv_ts=None):
        val = np.ascontiguousarray(val, np.float64)
        ts = np.ascontiguousarray(ts, np.int64)
        N = val.shape[1]
        if hv is not None:
            hv = np.ascontiguousarray(hv, np.float64)
            hv_ts = np.ascontiguousarray(hv_ts, np.int64)
        self._check(lib.crane_dyn_group_upload_nodes(self.h, N, _ptr(val), _ptr(ts), _ptr(hv), _ptr(hv_ts)))
        self.n_nodes = N

    def upload_bindings(self, node, ts_s):
        node = np.ascontiguousarray(node, np.int32)
        ts_s = np.ascontiguousarray(ts_s, np.int64)
        self._check(lib.crane_dyn_group_upload_bindings(self.h, len(node), _ptr(node), _ptr(ts_s)))

    @staticmethod
    def _ptrs(ts, ctype=C.c_void_p):
        return (ctype * len(ts))(*[None if t is None else t.data_ptr() for t in ts])

    def step_keys_fn(self, d_now, d_flags, d_keys):
        """crane_dyn_group_step_keys_async bound to per-device torch tensors (lists, one per device):
        returns f(now_ns, hv_ts_ns)."""
        P = d_now[0].numel()
        pn, pk = self._ptrs(d_now), self._ptrs(d_keys)
        pf = None if d_flags is None else self._ptrs(d_flags)
        fn, h, check = lib.crane_dyn_group_step_keys_async, self.h, self._check
        an, ak = C.cast(pn, C.c_void_p), C.cast(pk, C.c_void_p)
        af = None if pf is None else C.cast(pf, C.c_void_p)
        keep = (pn, pk, pf)

        def step(now_ns, hv_ts_ns):
            _ = keep
            rc = fn(h, now_ns, hv_ts_ns, P, an, af, ak)
            if rc:
                check(rc)

        return step

    def step_keys_async(self, now_ns, hv_ts_ns, d_now, d_flags, d_keys):
        self.step_keys_fn(d_now, d_flags, d_keys)(int(now_ns), int(hv_ts_ns))

    def step_keys_batch_fn(self, d_now, d_flags, d_keys):
        """crane_dyn_group_step_keys_batch bound to per-device torch tensors [G][P] (lists, one per
        device; d_flags None or [G][P] per device): returns f(now_ns[G], hv_ts_ns[G])."""
        G, P = d_now[0].shape
        pn, pk = self._ptrs(d_now), self._ptrs(d_keys)
        pf = None if d_flags is None else self._ptrs(d_flags)
        fn, h, check = lib.crane_dyn_group_step_keys_batch, self.h, self._check
        an, ak = C.cast(pn, C.c_void_p), C.cast(pk, C.c_void_p)
        af = None if pf is None else C.cast(pf, C.c_void_p)
        tn, th = (C.c_int64 * G)(), (C.c_int64 * G)()
        keep = (pn, pk, pf, tn, th)

        def step(now_ns, hv_ts_ns):
            _ = keep
            for b in range(G):
                tn[b], th[b] = int(now_ns[b]), int(hv_ts_ns[b])
            rc = fn(h, G, C.cast(tn, C.c_void_p), C.cast(th, C.c_void_p), P, an, af, ak)
            if rc:
                check(rc)

        return step

    def step_keys_batch(self, now_ns, hv_ts_ns, d_now, d_flags, d_keys):
        self.step_keys_batch_fn(d_now, d_flags, d_keys)(now_ns, hv_ts_ns)

    def sync(self):
        self._check(lib.crane_dyn_group_sync(self.h))

    # -- shard state changes, by global node index (routed to the owning shard)
    def update_nodes(self, idx, val, ts, hv=None, hv_ts=None):
        idx = np.ascontiguousarray(idx, np.int64)
        k, M = len(idx), len(self.metric_names)
        val = np.ascontiguousarray(val, np.float64).reshape(M, k)
        ts = np.ascontiguousarray(ts, np.int64).reshape(M, k)
        if hv is not None:
            hv = np.ascontiguousarray(hv, np.float64).reshape(k)
            hv_ts = np.ascontiguousarray(hv_ts, np.int64).reshape(k)
        self._check(lib.crane_dyn_group_update_nodes(self.h, len(idx), _ptr(idx), _ptr(val), _ptr(ts), _ptr(hv),
                                                     _ptr(hv_ts)))

    def update_node_steps(self, idx, val, ts, hv, hv_ts, t0_ns, t1_ns):
        idx = np.ascontiguousarray(idx, np.int64)
        k, M = len(idx), len(self.metric_names)
        val = np.ascontiguousarray(val, np.float64).reshape(M, k)
        ts = np.ascontiguousarray(ts, np.int64).reshape(M, k)
        if hv is not None:
            hv = np.ascontiguousarray(hv, np.float64).reshape(k)
            hv_ts = np.ascontiguousarray(hv_ts, np.int64).reshape(k)
        S = lib.crane_dyn_step_slots(lib.crane_dyn_group_engine(self.h, 0, 0))
        ns = np.zeros(k, np.uint8)
        bp = np.zeros((k, S), np.int64)
        ff = np.zeros((k, S + 1), np.int8)
        sc = np.zeros((k, S + 1), np.int8)
        self._check(lib.crane_dyn_group_update_node_steps(self.h, k, _ptr(idx), _ptr(val), _ptr(ts), _ptr(hv),
                                                          _ptr(hv_ts), int(t0_ns), int(t1_ns), _ptr(ns), _ptr(bp),
                                                          _ptr(ff), _ptr(sc)))
        return ns, bp, ff, sc

    def resize_nodes(self, n):
        self._check(lib.crane_dyn_group_resize_nodes(self.h, int(n)))
        self.n_nodes = int(n)

    def binding_records(self, size, gc_time_range_ns):
        self._check(lib.crane_dyn_group_binding_records(self.h, int(size), int(gc_time_range_ns)))

    def add_bindings(self, node, ts_s):
        node = np.ascontiguousarray(node, np.int32)
        ts_s = np.ascontiguousarray(ts_s, np.int64)
        self._check(lib.crane_dyn_group_add_bindings(self.h, len(node), _ptr(node), _ptr(ts_s)))

    def gc_bindings(self, now_ns):
        self._check(lib.crane_dyn_group_gc_bindings(self.h, int(now_ns)))

    def binding_count(self):
        n = lib.crane_dyn_group_binding_count(self.h)
        if n < 0:
            self._check(n)
        return n

    def refresh_hot_values(self, now_ns, hv_ts_ns):
        self._check(lib.crane_dyn_group_refresh_hot_values(self.h, int(now_ns), int(hv_ts_ns)))

    def hot_values(self):
        out = np.empty(self.n_nodes, np.float64)
        self._check(lib.crane_dyn_group_hot_values(self.h, self.n_nodes, _ptr(out)))
        return out

    def node_steps(self, t0_ns, t1_ns):
        """Every node's answer rows over [t0, t1): (n_steps [N], bp [N][S], first_fail [N][S+1], score [N][S+1])."""
        S = lib.crane_dyn_step_slots(lib.crane_dyn_group_engine(self.h, 0, 0))
        N = self.n_nodes
        ns = np.zeros(N, np.uint8)
        bp = np.zeros((N, S), np.int64)
        ff = np.zeros((N, S + 1), np.int8)
        sc = np.zeros((N, S + 1), np.int8)
        self._check(lib.crane_dyn_group_node_steps(self.h, int(t0_ns), int(t1_ns), N, _ptr(ns), _ptr(bp), _ptr(ff),
                                                   _ptr(sc)))
        return ns, bp, ff, sc

    def schedule(self, now_ns, hv_ts_ns, pods_now, pod_flags=None):
        """One batch from host arrays: (chosen global node [P], chosen score [P])."""
        now = np.ascontiguousarray(pods_now, np.int64).reshape(-1)
        fl = None if pod_flags is None else np.ascontiguousarray(pod_flags, np.uint8).reshape(-1)
        ch = np.empty(len(now), np.int64)
        cs = np.empty(len(now), np.int64)
        self._check(lib.crane_dyn_group_schedule(self.h, int(now_ns), int(hv_ts_ns), len(now), _ptr(now), _ptr(fl),
                                                 _ptr(ch), _ptr(cs)))
        return ch, cs


def version() -> str:
    return lib.crane_dyn_version().decode()
