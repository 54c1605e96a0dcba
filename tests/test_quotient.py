"""CPU check of the division-free quotient used by K3 variant 4 (kernels.hip eval_pair).

trunc(RN(s/W)) for W > 0 is recovered from q0 = RN(s * RN(1/W)) and the host
thresholds T[k] = min{s : RN(s/W) >= k}.  This restates the device arithmetic
in Python floats (IEEE binary64, correctly rounded) and checks it exhaustively
around every threshold for several weight sums.
"""
import math
import struct

import numpy as np
import pytest

KQMAX, KQFAST = 127, 125.0


def bits(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def frombits(b):
    return struct.unpack("<d", struct.pack("<Q", b))[0]


def thresholds(W):
    T = [-math.inf]
    for k in range(1, KQMAX + 1):
        lo, hi = 0, bits(math.inf)
        while hi - lo > 1:
            mid = (lo + hi) // 2
            if frombits(mid) / W >= k:
                hi = mid
            else:
                lo = mid
        T.append(frombits(hi))
    return T


def device_base(s, W, T):
    q0 = s * (1.0 / W)
    if not q0 < KQFAST:
        return None  # exact path
    k0 = int(q0) if abs(q0) < 2**31 else (2**31 - 1 if q0 > 0 else -(2**31))
    k0 = min(max(k0, 0), KQMAX - 1)
    return k0 + (1 if s >= T[k0 + 1] else 0) - (1 if s < T[k0] else 0)


def ref_final(s, W, pen):
    q = s / W
    base = int(q)  # trunc; |q| small here
    return min(max(base - pen, 0), 100)


@pytest.mark.parametrize("W", [2.0, 0.3, 1.7, 0.1, 3.0, 1e-3, 7.25])
def test_threshold_quotient(W):
    T = thresholds(W)
    rng = np.random.default_rng(int(W * 1000))
    cands = []
    for k in range(1, KQMAX + 1):
        t = T[k]
        for d in range(-3, 4):
            cands.append(frombits(bits(t) + d) if t > 0 else t)
    cands += list(rng.uniform(-50 * W, 130 * W, 20000))
    for s in cands:
        if not math.isfinite(s):
            continue
        b = device_base(s, W, T)
        if b is None:
            continue
        for pen in (0, 1, 10, 30):
            assert min(max(b - pen, 0), 100) == ref_final(s, W, pen), (W, s, pen)
