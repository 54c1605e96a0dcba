"""Independent pure-Python restatement of the Dynamic plugin hot path.

TEST INFRASTRUCTURE ONLY.  Written separately from oracle/crane_oracle.c so
the two restatements check each other; it generates the committed golden
fixtures (tests/golden/*.json) via make_golden.py.  Python floats are IEEE
binary64 with correctly rounded +,-,*,/ and no FMA contraction, matching Go on
amd64.  Citations are into /root/reference.

Parity is unpinned by the reference (no reference tests/fixtures exist for
this path; Go is absent) — these vectors are derived from the source text.
"""
from __future__ import annotations

import datetime as _dt
import math
import re
from zoneinfo import ZoneInfo

MAX_NODE_SCORE = 100  # upstream framework.MaxNodeScore
MIN_NODE_SCORE = 0
NODE_HOT_VALUE = "node_hot_value"  # stats.go:22
HOT_ACTIVE_NS = 5 * 60 * 10**9  # stats.go:24
EXTRA_ACTIVE_NS = 5 * 60 * 10**9  # stats.go:26
INT64_MIN = -(2**63)


def go_int(x: float) -> int:
    """int(float64) on amd64: NaN / out of range -> INT64_MIN."""
    if x != x or not (-(2.0**63) <= x < 2.0**63):
        return INT64_MIN
    return int(x)  # truncation toward zero


def wrap64(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= (1 << 63) else v


# --- strconv.ParseFloat(s, 64) (go1.17 atof.go) -------------------------
_DEC = re.compile(r"[+-]?([0-9_]*)(\.([0-9_]*))?([eE][+-]?[0-9][0-9_]*)?\Z")
_HEX = re.compile(r"[+-]?0[xX]([0-9a-fA-F_]*)(\.([0-9a-fA-F_]*))?[pP][+-]?[0-9][0-9_]*\Z")


def _underscore_ok(s: str) -> bool:
    saw = "^"
    i = 0
    if s[:1] in ("+", "-"):
        s = s[1:]
    hexa = False
    if len(s) >= 2 and s[0] == "0" and s[1].lower() in "box":
        i, saw, hexa = 2, "0", s[1].lower() == "x"
    while i < len(s):
        c = s[i]
        if c.isdigit() or (hexa and c.lower() in "abcdef"):
            saw = "0"
        elif c == "_":
            if saw != "0":
                return False
            saw = "_"
        else:
            if saw == "_":
                return False
            saw = "!"
        i += 1
    return saw != "_"


def go_parse_float(s: str):
    """Returns (value, err) with err in (None, 'syntax', 'range')."""
    if not s:
        return 0.0, "syntax"
    body = s[1:] if s[0] in "+-" else s
    sign = -1.0 if s[0] == "-" else 1.0
    low = body.lower()
    if s[0] not in "+-" and low == "nan":
        return math.nan, None
    if low in ("inf", "infinity"):
        return sign * math.inf, None
    if _HEX.match(s):
        m = _HEX.match(s)
        if not any(c not in "_." for c in (m.group(1) + (m.group(3) or ""))):
            return 0.0, "syntax"
        if "_" in s and not _underscore_ok(s):
            return 0.0, "syntax"
        v = float.fromhex(s.replace("_", ""))
    else:
        m = _DEC.match(s)
        if not m:
            return 0.0, "syntax"
        digits = (m.group(1) or "") + (m.group(3) or "")
        if not any(c.isdigit() for c in digits):
            return 0.0, "syntax"
        if "_" in s and not _underscore_ok(s):
            return 0.0, "syntax"
        try:
            v = float(s.replace("_", ""))
        except (ValueError, OverflowError):
            return 0.0, "syntax"
    if math.isinf(v):
        return v, "range"
    return v, None


# --- time.ParseInLocation("2006-01-02T15:04:05Z", s, loc) ----------------
_TS = re.compile(r"(\d{4})-(\d{2})-(\d{2})T(\d{1,2}):(\d{2}):(\d{2})(\.\d+)?Z\Z")


def go_parse_time(s: str, tz: str = "Asia/Shanghai"):
    """Unix ns of a local-time annotation timestamp, or None on error."""
    m = _TS.match(s)
    if not m:
        return None
    y, mo, d, h, mi, se = (int(m.group(i)) for i in range(1, 7))
    if not (1 <= mo <= 12 and h < 24 and mi < 60 and se < 60):
        return None
    frac = m.group(7)
    ns = 0
    if frac:
        digits = frac[1:10]
        ns = int(digits) * 10 ** (9 - len(digits))
    try:
        local = _dt.datetime(y, mo, d, h, mi, se, tzinfo=ZoneInfo(tz))
    except ValueError:
        return None
    off = local.utcoffset()
    days = (_dt.date(y, mo, d) - _dt.date(1970, 1, 1)).days
    return (days * 86400 + h * 3600 + mi * 60 + se - int(off.total_seconds())) * 10**9 + ns


def format_local(unix_s: int, tz: str = "Asia/Shanghai") -> str:
    """utils.GetLocalTime() format (utils.go:26-33) of a unix second."""
    t = _dt.datetime.fromtimestamp(unix_s, tz=ZoneInfo(tz))
    return t.strftime("%Y-%m-%dT%H:%M:%SZ")


# --- time.ParseDuration subset used by policies --------------------------
_UNITS = {"ns": 1, "us": 10**3, "µs": 10**3, "μs": 10**3, "ms": 10**6, "s": 10**9, "m": 60 * 10**9, "h": 3600 * 10**9}


def go_parse_duration(s: str) -> int:
    neg = s.startswith("-")
    body = s.lstrip("+-") if s[:1] in "+-" else s
    if body == "0":
        return 0
    total = 0
    for num, unit in re.findall(r"([0-9]*\.?[0-9]*)([^0-9.]+)", body):
        if unit not in _UNITS or num in ("", "."):
            raise ValueError(s)
        if "." in num:
            ip, fp = num.split(".")
            v = int(ip or "0") * _UNITS[unit]
            if fp:
                v += int(float(int(fp)) * (_UNITS[unit] / 10 ** len(fp)))
        else:
            v = int(num) * _UNITS[unit]
        total += v
    if "".join("".join(x) for x in re.findall(r"([0-9]*\.?[0-9]*)([^0-9.]+)", body)) != body:
        raise ValueError(s)
    return -total if neg else total


# --- the plugin ------------------------------------------------------------
def active_duration(policy, name):
    """getActiveDuration (stats.go:140-150)."""
    for n, period in policy["syncPolicy"]:
        if n == name and period != 0:
            return period + EXTRA_ACTIVE_NS
    return None


def resource_usage(anno, key, dur, now_ns, tz):
    """getResourceUsage (stats.go:51-76): value or None on any error."""
    if key not in anno:
        return None
    parts = anno[key].split(",")
    if len(parts) != 2:
        return None
    if len(parts[1]) < 5:
        return None
    ts = go_parse_time(parts[1], tz)
    if ts is None or not (now_ns < ts + dur):
        return None
    v, err = go_parse_float(parts[0])
    if err is not None or v < 0:
        return None
    return v


def filter_node(policy, anno, now_ns, ds=False, tz="Asia/Shanghai"):
    """DynamicScheduler.Filter (plugins.go:39-69): -1 Success or predicate index."""
    if ds:
        return -1
    for k, (name, limit) in enumerate(policy["predicate"]):
        dur = active_duration(policy, name)
        if not dur:
            continue
        u = resource_usage(anno, name, dur, now_ns, tz)
        if u is None or limit == 0:
            continue
        if u > limit:
            return k
    return -1


def node_score(policy, anno, now_ns, tz="Asia/Shanghai"):
    """getNodeScore (stats.go:114-138)."""
    if not policy["priority"]:
        return 0
    score = 0.0
    weight = 0.0
    for name, w in policy["priority"]:
        ps = 0.0
        dur = active_duration(policy, name)
        if dur:
            u = resource_usage(anno, name, dur, now_ns, tz)
            if u is not None:
                ps = (1.0 - u) * w * float(MAX_NODE_SCORE)
        weight += w
        score += ps
    try:
        q = score / weight
    except ZeroDivisionError:  # Go float division by zero: +-Inf or NaN
        q = math.nan if score == 0 or score != score else math.copysign(math.inf, score) * math.copysign(1.0, weight)
    return go_int(q)


def score_node(policy, anno, now_ns, tz="Asia/Shanghai"):
    """DynamicScheduler.Score (plugins.go:73-98)."""
    s = node_score(policy, anno, now_ns, tz)
    hv = resource_usage(anno, NODE_HOT_VALUE, HOT_ACTIVE_NS, now_ns, tz)
    if hv is None:
        hv = 0.0
    s = wrap64(s - go_int(hv * 10))
    return max(MIN_NODE_SCORE, min(MAX_NODE_SCORE, s))


def duration_seconds_trunc(d_ns: int) -> int:
    sec = int(d_ns / 10**9) if d_ns >= 0 else -int(-d_ns // 10**9)
    nsec = d_ns - sec * 10**9
    return go_int(float(sec) + float(nsec) / 1e9)


def hot_values(policy, bindings, n_nodes, now_unix):
    """GetLastNodeBindingCount x annotateNodeHotValue (binding.go:81-97, node.go:113-121)."""
    hv = [0] * n_nodes
    cnts = []
    for tr, count in policy["hotValue"]:
        timeline = now_unix - duration_seconds_trunc(tr)
        cnt = [0] * n_nodes
        for node, ts in bindings:
            if 0 <= node < n_nodes and ts > timeline:
                cnt[node] += 1
        cnts.append(cnt)
        for n in range(n_nodes):
            q = abs(cnt[n]) // abs(count)
            hv[n] += q if (cnt[n] >= 0) == (count > 0) else -q
    return cnts, hv


def default_policy():
    """deploy/manifests/dynamic/policy.yaml:1-52."""
    m = 60 * 10**9
    return {
        "syncPolicy": [
            ("cpu_usage_avg_5m", 3 * m), ("cpu_usage_max_avg_1h", 15 * m), ("cpu_usage_max_avg_1d", 180 * m),
            ("mem_usage_avg_5m", 3 * m), ("mem_usage_max_avg_1h", 15 * m), ("mem_usage_max_avg_1d", 180 * m),
        ],
        "predicate": [
            ("cpu_usage_avg_5m", 0.65), ("cpu_usage_max_avg_1h", 0.75),
            ("mem_usage_avg_5m", 0.65), ("mem_usage_max_avg_1h", 0.75),
        ],
        "priority": [
            ("cpu_usage_avg_5m", 0.2), ("cpu_usage_max_avg_1h", 0.3), ("cpu_usage_max_avg_1d", 0.5),
            ("mem_usage_avg_5m", 0.2), ("mem_usage_max_avg_1h", 0.3), ("mem_usage_max_avg_1d", 0.5),
        ],
        "hotValue": [(5 * m, 5), (1 * m, 2)],
    }
