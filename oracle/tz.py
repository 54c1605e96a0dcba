"""go1.17 time zones restated in Python — the checker of crane-scheduler_amd/csrc/tz.cpp.

TEST INFRASTRUCTURE ONLY: imported by tests/ — never by the product path.

Restates, from the published go1.17 sources (the reference's go.mod:3; Go is not
in the container): time/zoneinfo_read.go LoadLocationFromTZData, time/zoneinfo.go
Location.lookup, lookupFirstZone, tzset (tzsetName / tzsetOffset / tzsetRule /
tzsetNum, tzruleTime), and time/time.go Date's offset choice — what
utils.GetLocation + time.ParseInLocation do with the annotation stamps
(pkg/utils/utils.go:35-45, stats.go:36-40).  Parity unpinned by reference tests
(none exist for this path); tests/test_tz.py also checks the offsets against
Python's own zoneinfo.
"""
from __future__ import annotations

import struct

ALPHA, OMEGA = -(1 << 63), (1 << 63) - 1
DAY = 86400


def _days_from_civil(y, m, d):
    y -= m <= 2
    era = (y if y >= 0 else y - 399) // 400
    yoe = y - era * 400
    doy = (153 * (m + (-3 if m > 2 else 9)) + 2) // 5 + d - 1
    doe = yoe * 365 + yoe // 4 - yoe // 100 + doy
    return era * 146097 + doe - 719468


def _is_leap(y):
    return (y % 4 == 0 and y % 100 != 0) or y % 400 == 0


def _trunc_div(a, b):
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def _trunc_mod(a, b):
    return a - b * _trunc_div(a, b)


class _Parse:
    def __init__(self, s):
        self.s, self.p = s, 0

    def num(self, lo, hi):
        s, p = self.s, self.p
        if p >= len(s):
            return None
        n, i = 0, p
        while i < len(s) and s[i].isdigit():
            n = n * 10 + int(s[i])
            if n > hi:
                return None
            i += 1
        if i == p or n < lo:
            return None
        self.p = i
        return n

    def offset(self):
        s = self.s
        if self.p >= len(s):
            return None
        neg = False
        if s[self.p] in "+-":
            neg = s[self.p] == "-"
            self.p += 1
        h = self.num(0, 24 * 7)
        if h is None:
            return None
        off = h * 3600
        if self.p < len(s) and s[self.p] == ":":
            self.p += 1
            m = self.num(0, 59)
            if m is None:
                return None
            off += m * 60
            if self.p < len(s) and s[self.p] == ":":
                self.p += 1
                sec = self.num(0, 59)
                if sec is None:
                    return None
                off += sec
        return -off if neg else off

    def name(self):
        s, p = self.s, self.p
        if p >= len(s):
            return False
        if s[p] != "<":
            for i in range(p, len(s)):
                if s[i] in "0123456789,-+":
                    if i - p < 3:
                        return False
                    self.p = i
                    return True
            if len(s) - p < 3:
                return False
            self.p = len(s)
            return True
        j = s.find(">", p)
        if j < 0:
            return False
        self.p = j + 1
        return True

    def rule(self):
        s = self.s
        if self.p >= len(s):
            return None
        r = {"time": 7200}
        if s[self.p] == "J":
            self.p += 1
            d = self.num(1, 365)
            if d is None:
                return None
            r.update(kind="J", day=d)
        elif s[self.p] == "M":
            self.p += 1
            vals = []
            for k, (lo, hi) in enumerate(((1, 12), (1, 5), (0, 6))):
                v = self.num(lo, hi)
                if v is None:
                    return None
                vals.append(v)
                if k < 2:
                    if self.p >= len(s) or s[self.p] != ".":
                        return None
                    self.p += 1
            r.update(kind="M", mon=vals[0], week=vals[1], day=vals[2])
        else:
            d = self.num(0, 365)
            if d is None:
                return None
            r.update(kind="D", day=d)
        if self.p < len(s) and s[self.p] == "/":
            self.p += 1
            t = self.offset()
            if t is None:
                return None
            r["time"] = t
        return r


def _rule_time(year, r, off):
    before = [0, 31, 59, 90, 120, 151, 181, 212, 243, 273, 304, 334, 365]
    if r["kind"] == "J":
        s = (r["day"] - 1) * DAY + (DAY if _is_leap(year) and r["day"] >= 60 else 0)
    elif r["kind"] == "D":
        s = r["day"] * DAY
    else:
        mon = r["mon"]
        m1 = (mon + 9) % 12 + 1
        yy0 = year - 1 if mon <= 2 else year
        yy1, yy2 = _trunc_div(yy0, 100), _trunc_mod(yy0, 100)
        dow = _trunc_mod((26 * m1 - 2) // 10 + 1 + yy2 + _trunc_div(yy2, 4) + _trunc_div(yy1, 4) - 2 * yy1, 7)
        if dow < 0:
            dow += 7
        d = r["day"] - dow
        if d < 0:
            d += 7
        dim = before[mon] - before[mon - 1] + (1 if mon == 2 and _is_leap(year) else 0)
        for _ in range(1, r["week"]):
            if d + 7 >= dim:
                break
            d += 7
        d += before[mon - 1] + (1 if _is_leap(year) and mon > 2 else 0)
        s = d * DAY
    return s + r["time"] - off


def tzset(s, init_end, sec):
    """(offset, start, end) or None, as Go's tzset(s, initEnd, sec)."""
    p = _Parse(s)
    if not p.name():
        return None
    std = p.offset()
    if std is None:
        return None
    std = -std
    if p.p >= len(s) or s[p.p] == ",":
        return std, init_end, OMEGA
    if not p.name():
        return None
    if p.p >= len(s) or s[p.p] == ",":
        dst = std + 3600
    else:
        dst = p.offset()
        if dst is None:
            return None
        dst = -dst
    rest = s[p.p:] or ",M3.2.0,M11.1.0"
    if rest[0] not in ",;":
        return None
    q = _Parse(rest)
    q.p = 1
    sr = q.rule()
    if sr is None or q.p >= len(rest) or rest[q.p] != ",":
        return None
    q.p += 1
    er = q.rule()
    if er is None or q.p != len(rest):
        return None
    days = sec // DAY
    # civil year of the UTC day
    y = 1970 + days // 366
    while _days_from_civil(y + 1, 1, 1) <= days:
        y += 1
    while _days_from_civil(y, 1, 1) > days:
        y -= 1
    yday = days - _days_from_civil(y, 1, 1)
    ysec = yday * DAY + _trunc_mod(sec, DAY)
    abs_ = _days_from_civil(y, 1, 1) * DAY
    ss, es = _rule_time(y, sr, std), _rule_time(y, er, dst)
    so, do = std, dst
    if es < ss:
        ss, es, so, do = es, ss, do, so
    if ysec < ss:
        return so, abs_, ss + abs_
    if ysec >= es:
        return so, es + abs_, abs_ + 365 * DAY
    return do, ss + abs_, es + abs_


class Location:
    """LoadLocationFromTZData (go1.17): zones, transitions, the footer rule."""

    def __init__(self, data: bytes):
        if len(data) < 44 or data[:4] != b"TZif" or data[4:5] not in (b"\0", b"2", b"3"):
            raise ValueError("bad TZif")
        v2 = data[4:5] != b"\0"

        def counts(off):
            return struct.unpack(">6I", data[off + 20:off + 44])

        isut, isstd, leap, ntx, ntyp, nchar = counts(0)
        p, tsize = 44, 4
        if v2:
            p += ntx * 4 + ntx + ntyp * 6 + nchar + leap * 8 + isstd + isut
            isut, isstd, leap, ntx, ntyp, nchar = counts(p)
            p, tsize = p + 44, 8
        fmt = ">%d%s" % (ntx, "q" if tsize == 8 else "i")
        self.tx = list(struct.unpack(fmt, data[p:p + ntx * tsize]))
        p += ntx * tsize
        self.idx = list(data[p:p + ntx])
        p += ntx
        self.zones = []
        for i in range(ntyp):
            off, isdst, _ = struct.unpack(">iBB", data[p + 6 * i:p + 6 * i + 6])
            self.zones.append((off, bool(isdst)))
        p += ntyp * 6 + nchar + leap * (tsize + 4) + isstd + isut
        if not self.tx:
            self.tx, self.idx = [ALPHA], [0]
        self.extend = ""
        if v2 and p < len(data) and data[p:p + 1] == b"\n":
            e = data.find(b"\n", p + 1)
            if e > 0:
                self.extend = data[p + 1:e].decode()
        self.first = 0
        if 0 in self.idx:
            fz = None
            if self.zones[self.idx[0]][1]:
                for zi in range(self.idx[0] - 1, -1, -1):
                    if not self.zones[zi][1]:
                        fz = zi
                        break
            if fz is None:
                fz = next((zi for zi, z in enumerate(self.zones) if not z[1]), 0)
            self.first = fz

    def lookup(self, sec):
        if not self.zones:
            return 0, ALPHA, OMEGA
        if not self.tx or sec < self.tx[0]:
            return self.zones[self.first][0], ALPHA, (self.tx[0] if self.tx else OMEGA)
        end, lo, hi = OMEGA, 0, len(self.tx)
        while hi - lo > 1:
            m = lo + (hi - lo) // 2
            if sec < self.tx[m]:
                end, hi = self.tx[m], m
            else:
                lo = m
        off, start = self.zones[self.idx[lo]][0], self.tx[lo]
        if lo == len(self.tx) - 1 and self.extend:
            r = tzset(self.extend, end, sec)
            if r is not None:
                return r
        return off, start, end

    def date(self, local):
        """time.Date's instant (Unix seconds) of wall clock `local` (seconds, as if UTC):
        go1.17 time.go Date re-looks the zone up at start-1 when utc < start, at end when
        utc >= end (not at utc itself)."""
        off, start, end = self.lookup(local)
        if off != 0:
            utc = local - off
            if utc < start:
                off = self.lookup(start - 1)[0]
            elif utc >= end:
                off = self.lookup(end)[0]
            local -= off
        return local


def wall_seconds(y, mo, d, h, mi, s):
    return _days_from_civil(y, mo, d) * DAY + h * 3600 + mi * 60 + s
