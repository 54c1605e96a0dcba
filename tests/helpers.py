"""Shared test helpers: run the HIP engine and the CPU oracle on the same inputs."""
import numpy as np

import crane_dyn as cd
from crane_dyn import synth
from oracle import oracle as O

SH = 8 * 3600


def engine_for(spec, cluster=None, device=0, opts=None):
    eng = cd.Engine(cd.Policy(spec), device)
    for k, v in (opts or {}).items():
        eng.set_option(k, v)
    if cluster is not None:
        val, ts, _ = cluster.rows(eng.metric_names)
        eng.upload_nodes(val, ts, cluster.hv, cluster.hv_ts)
    return eng


def oracle_soa(spec, c, now=None, ds=None, want_matrix=True, threads=8, hv_override=None):
    hv_ok = (c.hv_ts != synth.TS_INVALID).astype(np.uint8)
    hv, hv_ts = c.hv, c.hv_ts
    if hv_override is not None:
        hv, hv_ts = hv_override
        hv_ok = np.ones(len(hv), np.uint8)
    return O.eval_soa(spec, c.metric_names, c.ok, c.val, np.where(c.ok == 1, c.ts, 0), hv_ok, hv, hv_ts,
                      c.now if now is None else now, c.ds if ds is None else ds, threads=threads,
                      want_matrix=want_matrix)
