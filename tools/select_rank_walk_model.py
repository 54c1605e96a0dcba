"""Lane-level model of k_sel_chain_rs's rank-space walk (select.hip), checked against a
brute-force window walk on random queues (tests/test_select_model.py).  Test
infrastructure: it mirrors the kernel's wave logic (64 lanes as numpy vectors: ballots,
the cached list entries, the rotation shifts) so the chain's bookkeeping can be checked
on the CPU; the GPU tests check the kernel itself against the streaming kernel and the
oracle.  use_cache=True models a variant that keeps 64 list entries in registers across
pods (measured slower, profiles/ab/r03_select_rank_walk.txt; not in the kernel).  brute(): per pod, walk positions from the start until K nodes are feasible
(generic_scheduler.go's findNodesThatPassFilters with numFeasibleNodesToFind)."""
import sys

import numpy as np
INF = np.iinfo(np.int64).max

def brute(fth, now, ds_f, dfeas, K, start):
    N = len(fth); s = start; out = []
    for t, d in zip(now, ds_f):
        feas = dfeas if d else (fth <= t)
        cnt = 0; end = None
        for k in range(N):
            n = (s + k) % N
            if feas[n]:
                cnt += 1
                if cnt == K: end = s + k; break
        if end is None: end = s + N - 1
        out.append((s, end - s + 1)); s = (end + 1) % N
    return out, s

def emu(fth, now, ds_f, dfeas, K, start, use_cache=True):
    N = len(fth)
    tmin = min([t for t, d in zip(now, ds_f) if not d], default=INF)
    tmax = max([t for t, d in zip(now, ds_f) if not d], default=-INF)
    A = fth <= tmin; I = (fth > tmin) & (fth <= tmax); D = dfeas
    TA, TI, TD = A.sum(), I.sum(), D.sum()
    posA = np.flatnonzero(A); posI = np.flatnonzero(I); posD = np.flatnonzero(D)
    iRA = np.searchsorted(posA, posI)  # A nodes before each I node
    iFth = fth[posI]
    assert TA >= K
    rank = lambda pos, s: np.searchsorted(pos, s)
    lanes = np.arange(64)
    lt = lambda l: l  # popc(m & lt) = number of set lanes below
    rA, rI = rank(posA, start), rank(posI, start)
    s = start; spos = True; dsc = None; descs = []
    cb = -10**9; cra = np.zeros(64, np.int64); cft = np.zeros(64, np.int64)
    def endpos(dsc):
        k, v = dsc
        if k == 0: return posA[v - TA if v >= TA else v]
        if k == 1: return posI[v - TI if v >= TI else v]
        return v
    for t, d in zip(now, ds_f):
        if d:
            if not spos:
                e = endpos(dsc); s = e + 1 - N if e + 1 >= N else e + 1
            if TD < K: end = s + N - 1
            else:
                r = rank(posD, s) + K - 1
                end = posD[r] if r < TD else N + posD[r - TD]
            en = end - N if end >= N else end
            dsc = (2, en); s = en + 1 - N if en + 1 >= N else en + 1; spos = True
            rA, rI = rank(posA, s), rank(posI, s)
        else:
            rT = rA + K - 1
            c_lt = cbase = nin = 0; hit = -1; hra = 0
            off = rI - cb
            if not use_cache or off < 0 or off > 32:
                cb = rI; off = 0
                h = cb + lanes
                rot = h // TI if TI else np.zeros(64, np.int64)
                ic = h - rot * TI if TI else np.zeros(64, np.int64)
                cra = (iRA[ic] if TI else np.zeros(64, np.int64)) + rot * TA
                cft = iFth[ic] if TI else np.zeros(64, np.int64)
            cval = (lanes >= off) & (lanes - off < TI)
            inr = cval & (cra <= rT)
            cand = inr & (cft <= t)
            pre = np.cumsum(cand) - cand
            mr = cra - rA + pre
            c_lt = int((cand & (mr < K - 1)).sum())
            eq = cand & (mr == K - 1)
            if eq.any():
                l = int(np.flatnonzero(eq)[0]); hit = cb + l; hra = int(cra[l])
            cbase = int(cand.sum()); nin = int(inr.sum())
            one = eq.any() or not inr[off:].all() or 64 - off >= TI
            if not one:
                q0 = 64 - off
                while q0 < TI:
                    q = q0 + lanes; h = rI + q; wrap = h >= TI
                    ic = np.minimum(h - np.where(wrap, TI, 0), TI - 1)
                    ra = iRA[ic] + np.where(wrap, TA, 0)
                    inr = (q < TI) & (ra <= rT)
                    if not inr.any(): break
                    cand = inr & (iFth[ic] <= t)
                    mr = ra - rA + cbase + (np.cumsum(cand) - cand)
                    c_lt += int((cand & (mr < K - 1)).sum())
                    eq = cand & (mr == K - 1)
                    if eq.any():
                        l = int(np.flatnonzero(eq)[0]); hit = rI + q0 + l; hra = int(ra[l]); break
                    cbase += int(cand.sum()); nin += int(inr.sum())
                    if not inr.all(): break
                    q0 += 64
            if hit >= 0:
                dsc = (1, hit); rA = hra; rI = hit + 1
            else:
                e = rT - c_lt; dsc = (0, e); rA = e + 1
                if c_lt == 0: rI += nin
                elif one: rI += int((cval & (cra <= e)).sum())
                else:
                    cnt = 0; q0 = 0
                    while q0 < TI:
                        q = q0 + lanes; h = rI + q; wrap = h >= TI
                        ic = np.minimum(h - np.where(wrap, TI, 0), TI - 1)
                        ra = iRA[ic] + np.where(wrap, TA, 0)
                        bm = (q < TI) & (ra <= e)
                        cnt += int(bm.sum())
                        if not bm.all(): break
                        q0 += 64
                    rI += cnt
            if rA >= TA and rI >= TI:
                rA -= TA; rI -= TI; cb -= TI; cra = cra - TA
            spos = False
        descs.append(dsc)
    ends = [endpos(x) for x in descs]
    out = []; prev = start - 1
    for e in ends:
        s0 = prev + 1 - N if prev + 1 >= N else prev + 1
        dl = e - s0
        if dl < 0: dl += N
        out.append((s0, dl + 1)); prev = e
    return out

def random_case(rng):
    N = int(rng.integers(50, 3000)); P = int(rng.integers(1, 300))
    t0 = 1000
    now = np.sort(rng.integers(t0, t0 + 1000, P)) if rng.random() < 0.7 else rng.integers(t0, t0 + 1000, P)
    ds = rng.random(P) < rng.choice([0.0, 0.1, 0.5])
    fth = np.where(rng.random(N) < rng.random(), rng.integers(0, t0, N), rng.integers(t0, t0 + 1200, N))
    fth = np.where(rng.random(N) < 0.1, INF, fth)
    dfeas = rng.random(N) < 0.8
    tmin = now[~ds].min() if (~ds).any() else INF
    TA = int((fth <= tmin).sum())
    if TA < 1:
        return None
    K = int(rng.integers(1, TA + 1))
    start = int(rng.integers(0, N))
    return fth, now, ds, dfeas, K, start


def main(seed, trials=300):
    rng = np.random.default_rng(seed)
    bad = 0
    for trial in range(trials):
        case = random_case(rng)
        if case is None:
            continue
        want, _ = brute(*case)
        want = [tuple(map(int, w)) for w in want]
        for uc in (False, True):
            got = [tuple(map(int, g)) for g in emu(*case, uc)]
            if got != want:
                print("mismatch: trial", trial, "cache", uc)
                bad += 1
    return bad


if __name__ == "__main__":
    print("bad", main(int(sys.argv[1]) if len(sys.argv) > 1 else 0))

