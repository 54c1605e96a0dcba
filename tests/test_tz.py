"""IANA zones for the annotation timestamps (crane-scheduler_amd/csrc/tz.cpp) against
oracle/tz.py, a Python restatement of go1.17's LoadLocationFromTZData, lookup,
tzset and time.Date (utils.GetLocation, pkg/utils/utils.go:35-45), and — for the
offsets and unambiguous wall times — against Python's own zoneinfo on the same
TZif files (the tzdata package's).  Parity with Go itself is unpinned (no Go
toolchain, no reference vectors)."""
import datetime as dt
import os
import zoneinfo

import numpy as np
import pytest

cd = pytest.importorskip("crane_dyn")
tzdata = pytest.importorskip("tzdata")
from oracle import tz as OT  # noqa: E402

ZI = os.path.join(os.path.dirname(tzdata.__file__), "zoneinfo")
ZONES = ["America/New_York", "America/Los_Angeles", "Europe/London", "Europe/Berlin", "Australia/Sydney",
         "Australia/Lord_Howe", "Asia/Shanghai", "Asia/Kolkata", "Asia/Tokyo", "America/Sao_Paulo",
         "Africa/Casablanca", "Pacific/Chatham", "America/St_Johns", "Asia/Tehran", "Europe/Dublin",
         "America/Santiago", "Pacific/Apia", "Etc/GMT-8", "Etc/UTC", "Antarctica/Troll"]


def _zone(name):
    return cd.Zone(name, ZI), OT.Location(open(os.path.join(ZI, name), "rb").read())


@pytest.mark.parametrize("name", ZONES)
def test_lookup_matches_go_restatement_and_zoneinfo(name):
    z, o = _zone(name)
    py = zoneinfo.ZoneInfo.from_file(open(os.path.join(ZI, name), "rb"))
    rng = np.random.default_rng(hash(name) & 0xFFFF)
    secs = list(rng.integers(-2_000_000_000, 5_000_000_000, 400)) + [0, 1_700_000_000]
    # around every transition of the file, and the footer rule's years
    secs += [t + d for t in o.tx[-40:] if t > -(1 << 40) for d in (-1, 0, 1)]
    for s in secs:
        s = int(s)
        assert z.lookup(s) == o.lookup(s), (name, s)
        inst = dt.datetime.fromtimestamp(s, tz=dt.timezone.utc).astimezone(py)
        if 1900 <= inst.year <= 2200:
            assert int(inst.utcoffset().total_seconds()) == z.lookup(s)[0], (name, s)


@pytest.mark.parametrize("name", ZONES)
def test_date_matches_go_restatement(name):
    """time.Date's instant for random wall clocks; unambiguous ones also equal zoneinfo's."""
    z, o = _zone(name)
    py = zoneinfo.ZoneInfo.from_file(open(os.path.join(ZI, name), "rb"))
    rng = np.random.default_rng(7 + (hash(name) & 0xFFF))
    for _ in range(400):
        y, mo, d = int(rng.integers(1971, 2100)), int(rng.integers(1, 13)), int(rng.integers(1, 29))
        h, mi, s = int(rng.integers(0, 24)), int(rng.integers(0, 60)), int(rng.integers(0, 60))
        local = OT.wall_seconds(y, mo, d, h, mi, s)
        got = z.date(local)
        assert got == o.date(local), (name, y, mo, d, h, mi, s)
        w0 = dt.datetime(y, mo, d, h, mi, s, tzinfo=py)
        w1 = w0.replace(fold=1)
        if w0.utcoffset() == w1.utcoffset():  # neither skipped nor repeated
            back = dt.datetime.fromtimestamp(int(w0.timestamp()), tz=py).replace(tzinfo=None)
            if back == w0.replace(tzinfo=None):
                assert got == int(w0.timestamp()), (name, y, mo, d, h, mi, s)


def test_transition_wall_times_as_go_chooses():
    """America/New_York: 2021-03-14 02:30 does not exist, 2021-11-07 01:30 happens twice.
    time.Date looks the zone up at the wall time taken as UTC and again at the result."""
    z, o = _zone("America/New_York")
    skipped = OT.wall_seconds(2021, 3, 14, 2, 30, 0)
    # lookup(02:30 UTC) -> EST (-5h); 07:30 UTC is past that period's end (07:00 UTC) -> EDT (-4h)
    assert z.date(skipped) == o.date(skipped) == skipped + 4 * 3600
    repeated = OT.wall_seconds(2021, 11, 7, 1, 30, 0)
    # lookup(01:30 UTC) -> EDT; 05:30 UTC lies inside EDT's period: the first 01:30 (EDT)
    assert z.date(repeated) == o.date(repeated) == repeated + 4 * 3600
    v, ts = z.parse_annotation("0.25,2021-11-07T01:30:00Z")
    assert v == 0.25 and ts == (repeated + 4 * 3600) * 10**9
    # southern hemisphere (the footer's DST rule wraps the year end), half-hour DST shift
    for name in ("Australia/Sydney", "Australia/Lord_Howe"):
        z, o = _zone(name)
        for (y, mo, d, h, mi) in ((2030, 4, 7, 2, 30), (2030, 10, 6, 2, 15), (2031, 1, 1, 0, 0)):
            local = OT.wall_seconds(y, mo, d, h, mi, 0)
            assert z.date(local) == o.date(local)


def _tzif(tx, idx, offs):
    """A minimal version-2 TZif file (both data blocks, empty footer), abbreviation "ZZZ"."""
    import struct

    def block(tsize):
        hdr = b"TZif2" + b"\0" * 15 + struct.pack(">6I", 0, 0, 0, len(tx), len(offs), 4)
        body = b"".join(struct.pack(">q" if tsize == 8 else ">i", t) for t in tx) + bytes(idx)
        body += b"".join(struct.pack(">iBB", o, 0, 0) for o in offs) + b"ZZZ\0"
        return hdr + body
    return block(4) + block(8) + b"\n\n"


def test_date_close_transitions_looks_up_period_edge():
    """go1.17 time.Date: when the wall time taken as UTC lands in a period whose offset puts
    the instant before that period's start, the zone is looked up at start-1 (the period just
    before), not at the instant itself.  Two transitions one hour apart make the two differ:
    zones +0 (before 0), +1h on [0, 3600), +2h from 3600; wall 01:01:40 (3700 as UTC) ->
    lookup(3700) = +2h, 3700 - 7200 < 3600 -> lookup(3599) = +1h -> 100 (lookup(-3500) would
    give +0 -> 3700)."""
    data = _tzif([0, 3600], [1, 2], [0, 3600, 7200])
    z, o = cd.Zone(tzif=data), OT.Location(data)
    assert o.date(3700) == z.date(3700) == 100
    # and the symmetric edge: utc >= end -> lookup(end)
    data = _tzif([0, 3600], [1, 2], [-7200, -3600, 0])
    z, o = cd.Zone(tzif=data), OT.Location(data)
    # lookup(-100) = -7200 (before 0), utc = 7100 >= end 0 -> lookup(0) = -3600 -> 3500
    assert o.date(-100) == z.date(-100) == 3500


def test_load_rules():
    """time.LoadLocation: "" and "UTC" are UTC, ".." and absolute names invalid, unknown
    names fail (the reference would then panic in ParseInLocation with a nil Location)."""
    assert cd.Zone("", ZI).lookup(123) == (0, OT.ALPHA, OT.OMEGA)
    assert cd.Zone("UTC", ZI).date(1000) == 1000
    for bad in ("../etc/passwd", "/usr/share/zoneinfo/UTC", "No/Such_Zone"):
        with pytest.raises(cd.CraneError):
            cd.Zone(bad, ZI)
    with pytest.raises(cd.CraneError):
        cd.Zone(tzif=b"TZif4" + b"\0" * 60)  # version 4: not readable by go1.17


def test_shanghai_zone_equals_fixed_offset_since_1991():
    """The fixed-offset path (UTC+8) and the tzdata zone agree on every stamp a live
    controller writes; bulk parses through both agree."""
    z, _ = _zone("Asia/Shanghai")
    rng = np.random.default_rng(3)
    strs = []
    for _ in range(2000):
        y = int(rng.integers(1992, 2090))
        s = "%04d-%02d-%02dT%02d:%02d:%02dZ" % (y, rng.integers(1, 13), rng.integers(1, 29), rng.integers(0, 24),
                                             rng.integers(0, 60), rng.integers(0, 60))
        strs.append("0.%d,%s" % (rng.integers(0, 1000), s))
    for s in strs[:200]:
        assert z.parse_annotation(s) == cd.parse_annotation(s, 8 * 3600), s
    nodes = [{"m": s} for s in strs]
    snap = cd.SnapshotStrings(["m"], nodes)
    snap.parse(z, 4)
    a = snap.ts.copy()
    snap.parse(8 * 3600, 4)
    assert np.array_equal(a, snap.ts)
