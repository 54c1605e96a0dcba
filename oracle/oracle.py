"""ctypes front-end of the CPU oracle (oracle/crane_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, and only as the checker / the timed CPU
baseline — never by the product path.

Policies are plain dicts in reference order (see tests/golden/pyref.py
default_policy): {"syncPolicy": [(name, period_ns)], "predicate": [(name,
limit)], "priority": [(name, weight)], "hotValue": [(timeRange_ns, count)]}.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libcrane_oracle.so")


class _Policy(C.Structure):
    _fields_ = [
        ("n_sync", C.c_int32), ("sync_name", C.POINTER(C.c_char_p)), ("sync_period_ns", C.POINTER(C.c_int64)),
        ("n_pred", C.c_int32), ("pred_name", C.POINTER(C.c_char_p)), ("pred_limit", C.POINTER(C.c_double)),
        ("n_prio", C.c_int32), ("prio_name", C.POINTER(C.c_char_p)), ("prio_weight", C.POINTER(C.c_double)),
        ("n_hot", C.c_int32), ("hot_tr_ns", C.POINTER(C.c_int64)), ("hot_count", C.POINTER(C.c_int64)),
    ]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        L.or_go_parse_float.argtypes = [C.c_char_p, C.c_int64, P(C.c_double)]
        L.or_go_parse_time.argtypes = [C.c_char_p, C.c_int64, C.c_int64, P(C.c_int64)]
        L.or_go_parse_duration.argtypes = [C.c_char_p, C.c_int64, P(C.c_int64)]
        L.or_go_f64_to_int.argtypes = [C.c_double]
        L.or_go_f64_to_int.restype = C.c_int64
        L.or_go_duration_seconds_trunc.argtypes = [C.c_int64]
        L.or_go_duration_seconds_trunc.restype = C.c_int64
        L.or_eval_strings.argtypes = [P(_Policy), C.c_int64, P(C.c_int64), P(C.c_char_p), P(C.c_char_p),
                                      C.c_int64, P(C.c_int64), P(C.c_uint8), C.c_int64, C.c_int32,
                                      P(C.c_int8), P(C.c_int64), P(C.c_int64)]
        L.or_eval_soa.argtypes = [P(_Policy), C.c_int32, P(C.c_char_p), C.c_int64, P(C.c_uint8), P(C.c_double),
                                  P(C.c_int64), P(C.c_uint8), P(C.c_double), P(C.c_int64), C.c_int64,
                                  P(C.c_int64), P(C.c_uint8), C.c_int32, P(C.c_int8), P(C.c_int64), P(C.c_int64)]
        L.or_parse_annotation.argtypes = [C.c_char_p, C.c_int64, C.c_int64, P(C.c_uint8), P(C.c_double), P(C.c_int64)]
        L.or_hot_values.argtypes = [P(_Policy), C.c_int64, P(C.c_int32), P(C.c_int64), C.c_int64, C.c_int64,
                                    P(C.c_int64), P(C.c_int64)]
        L.or_greedy.argtypes = [P(_Policy), C.c_int32, P(C.c_char_p), C.c_int64, P(C.c_uint8), P(C.c_double),
                                P(C.c_int64), C.c_int64, P(C.c_int32), P(C.c_int64), C.c_int64, C.c_int64,
                                P(C.c_uint8), P(C.c_int64)]
        L.or_binding_heap.argtypes = [C.c_int64, C.c_int64, C.c_int64, P(C.c_uint8), P(C.c_int32), P(C.c_int64),
                                      P(C.c_int64), P(C.c_int32), P(C.c_int64)]
        _lib = L
    return _lib


def _ptr(a, ct):
    return None if a is None else a.ctypes.data_as(C.POINTER(ct))


def _cstrs(names):
    arr = (C.c_char_p * max(1, len(names)))(*[n.encode() for n in names])
    return arr


class Policy:
    """Keeps the ctypes buffers of one flattened policy alive."""

    def __init__(self, pol):
        self.pol = pol
        sp, pr, pi, hv = pol["syncPolicy"], pol["predicate"], pol["priority"], pol["hotValue"]
        self._bufs = [
            _cstrs([n for n, _ in sp]), (C.c_int64 * max(1, len(sp)))(*[int(p) for _, p in sp]),
            _cstrs([n for n, _ in pr]), (C.c_double * max(1, len(pr)))(*[float(x) for _, x in pr]),
            _cstrs([n for n, _ in pi]), (C.c_double * max(1, len(pi)))(*[float(x) for _, x in pi]),
            (C.c_int64 * max(1, len(hv)))(*[int(t) for t, _ in hv]), (C.c_int64 * max(1, len(hv)))(*[int(c) for _, c in hv]),
        ]
        b = self._bufs
        self.c = _Policy(len(sp), C.cast(b[0], C.POINTER(C.c_char_p)), C.cast(b[1], C.POINTER(C.c_int64)),
                         len(pr), C.cast(b[2], C.POINTER(C.c_char_p)), C.cast(b[3], C.POINTER(C.c_double)),
                         len(pi), C.cast(b[4], C.POINTER(C.c_char_p)), C.cast(b[5], C.POINTER(C.c_double)),
                         len(hv), C.cast(b[6], C.POINTER(C.c_int64)), C.cast(b[7], C.POINTER(C.c_int64)))


# ---- Go semantics helpers --------------------------------------------------
def go_parse_float(s: str):
    v = C.c_double()
    b = s.encode()
    rc = lib().or_go_parse_float(b, len(b), C.byref(v))
    return v.value, {0: None, 1: "syntax", 2: "range"}[rc]


def go_parse_time(s: str, tz_offset_s: int):
    v = C.c_int64()
    b = s.encode()
    rc = lib().or_go_parse_time(b, len(b), tz_offset_s, C.byref(v))
    return None if rc else v.value


def go_parse_duration(s: str):
    v = C.c_int64()
    b = s.encode()
    rc = lib().or_go_parse_duration(b, len(b), C.byref(v))
    return None if rc else v.value


def go_f64_to_int(x: float) -> int:
    return lib().or_go_f64_to_int(x)


def parse_annotation(s: str, tz_offset_s: int):
    ok, v, ts = C.c_uint8(), C.c_double(), C.c_int64()
    b = s.encode()
    lib().or_parse_annotation(b, len(b), tz_offset_s, C.byref(ok), C.byref(v), C.byref(ts))
    return bool(ok.value), v.value, ts.value


# ---- evaluation ----------------------------------------------------------
def eval_strings(pol, nodes, now_ns, ds=None, tz_offset_s=8 * 3600, threads=1, want_matrix=True):
    """nodes: list of {annotation key: value} dicts."""
    P, N = len(now_ns), len(nodes)
    off = np.zeros(N + 1, np.int64)
    keys, vals = [], []
    for i, a in enumerate(nodes):
        for k, v in a.items():
            keys.append(k.encode())
            vals.append(v.encode())
        off[i + 1] = len(keys)
    ck = (C.c_char_p * max(1, len(keys)))(*keys)
    cv = (C.c_char_p * max(1, len(vals)))(*vals)
    pc = Policy(pol)
    now = np.ascontiguousarray(now_ns, np.int64)
    dsa = None if ds is None else np.ascontiguousarray(ds, np.uint8)
    ff = np.empty((P, N), np.int8) if want_matrix else None
    sc = np.empty((P, N), np.int64) if want_matrix else None
    ch = np.empty(P, np.int64)
    lib().or_eval_strings(C.byref(pc.c), N, _ptr(off, C.c_int64), ck, cv, P, _ptr(now, C.c_int64),
                          _ptr(dsa, C.c_uint8), tz_offset_s, threads, _ptr(ff, C.c_int8), _ptr(sc, C.c_int64),
                          _ptr(ch, C.c_int64))
    return ff, sc, ch


def eval_soa(pol, key_names, ok, val, ts, hv_ok, hv, hv_ts, now_ns, ds=None, threads=1, want_matrix=True):
    """ok/val/ts: [K][N] arrays for the rows named by key_names."""
    K, N = ok.shape
    P = len(now_ns)
    pc = Policy(pol)
    kn = _cstrs(list(key_names))
    ok = np.ascontiguousarray(ok, np.uint8)
    val = np.ascontiguousarray(val, np.float64)
    ts = np.ascontiguousarray(ts, np.int64)
    hv_ok = np.ascontiguousarray(hv_ok, np.uint8)
    hv = np.ascontiguousarray(hv, np.float64)
    hv_ts = np.ascontiguousarray(hv_ts, np.int64)
    now = np.ascontiguousarray(now_ns, np.int64)
    dsa = None if ds is None else np.ascontiguousarray(ds, np.uint8)
    ff = np.empty((P, N), np.int8) if want_matrix else None
    sc = np.empty((P, N), np.int64) if want_matrix else None
    ch = np.empty(P, np.int64)
    lib().or_eval_soa(C.byref(pc.c), K, kn, N, _ptr(ok, C.c_uint8), _ptr(val, C.c_double), _ptr(ts, C.c_int64),
                      _ptr(hv_ok, C.c_uint8), _ptr(hv, C.c_double), _ptr(hv_ts, C.c_int64), P, _ptr(now, C.c_int64),
                      _ptr(dsa, C.c_uint8), threads, _ptr(ff, C.c_int8), _ptr(sc, C.c_int64), _ptr(ch, C.c_int64))
    return ff, sc, ch


def hot_values(pol, b_node, b_ts, n_nodes, now_unix):
    pc = Policy(pol)
    W = len(pol["hotValue"])
    bn = np.ascontiguousarray(b_node, np.int32)
    bt = np.ascontiguousarray(b_ts, np.int64)
    cnt = np.zeros((max(W, 1), n_nodes), np.int64)
    hv = np.zeros(n_nodes, np.int64)
    rc = lib().or_hot_values(C.byref(pc.c), len(bn), _ptr(bn, C.c_int32), _ptr(bt, C.c_int64), n_nodes, now_unix,
                             _ptr(cnt, C.c_int64), _ptr(hv, C.c_int64))
    if rc:
        raise ZeroDivisionError("hotValue count is 0")
    return cnt[:W], hv


def greedy(pol, key_names, ok, val, ts, b_node, b_ts, now_ns, P, ds=None):
    K, N = ok.shape
    pc = Policy(pol)
    kn = _cstrs(list(key_names))
    ok = np.ascontiguousarray(ok, np.uint8)
    val = np.ascontiguousarray(val, np.float64)
    ts = np.ascontiguousarray(ts, np.int64)
    bn = np.ascontiguousarray(b_node, np.int32)
    bt = np.ascontiguousarray(b_ts, np.int64)
    dsa = None if ds is None else np.ascontiguousarray(ds, np.uint8)
    ch = np.empty(P, np.int64)
    rc = lib().or_greedy(C.byref(pc.c), K, kn, N, _ptr(ok, C.c_uint8), _ptr(val, C.c_double), _ptr(ts, C.c_int64),
                         len(bn), _ptr(bn, C.c_int32), _ptr(bt, C.c_int64), P, now_ns, _ptr(dsa, C.c_uint8),
                         _ptr(ch, C.c_int64))
    if rc:
        raise ZeroDivisionError("hotValue count is 0")
    return ch


def binding_heap(size, gc_tr_ns, ops, node, arg):
    """BindingRecords restated over container/heap: ops 0 = AddBinding(node, ts=arg),
    1 = BindingsGC(now_unix=arg).  Returns the final heap (node[], ts[]) in slice order."""
    ops = np.ascontiguousarray(ops, np.uint8)
    node = np.ascontiguousarray(node, np.int32)
    arg = np.ascontiguousarray(arg, np.int64)
    cap = max(int(size), 1)
    on = np.empty(cap, np.int32)
    ot = np.empty(cap, np.int64)
    n = C.c_int64()
    rc = lib().or_binding_heap(int(size), int(gc_tr_ns), len(ops), _ptr(ops, C.c_uint8), _ptr(node, C.c_int32),
                               _ptr(arg, C.c_int64), C.byref(n), _ptr(on, C.c_int32), _ptr(ot, C.c_int64))
    if rc:
        raise ValueError("binding heap size must be positive")
    return on[:n.value].copy(), ot[:n.value].copy()
