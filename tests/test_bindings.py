"""BindingRecords (pkg/controller/annotator/binding.go:50-123) and
translateEventToBinding (event.go:118-145): the controller-side feed of K2.

CPU: the C oracle's heap restatement against an independent pure-Python
restatement of go1.17 container/heap (identical slice order after every op
sequence, ties included); the host event-message scanner.
GPU: the engine's heap mode (crane_dyn_binding_records / add / gc) against the
oracle heap: same Len() and the same per-node hot values after refreshes.
"""
import numpy as np
import pytest

cd = pytest.importorskip("crane_dyn")
from crane_dyn import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

M_NS = 60 * 10**9


class GoHeap:
    """container/heap over BindingHeap (Less = Timestamp <), written from heap.go."""

    def __init__(self, size, gc_tr_ns):
        self.h, self.size, self.gc = [], size, gc_tr_ns

    def _less(self, i, j):
        return self.h[i][1] < self.h[j][1]

    def _up(self, j):
        while True:
            i = int((j - 1) / 2)  # Go truncates toward zero
            if i == j or not self._less(j, i):
                break
            self.h[i], self.h[j] = self.h[j], self.h[i]
            j = i

    def _down(self, i, n):
        while True:
            j1 = 2 * i + 1
            if j1 >= n:
                break
            j = j1
            if j1 + 1 < n and self._less(j1 + 1, j1):
                j = j1 + 1
            if not self._less(j, i):
                break
            self.h[i], self.h[j] = self.h[j], self.h[i]
            i = j

    def push(self, b):
        self.h.append(b)
        self._up(len(self.h) - 1)

    def pop(self):
        n = len(self.h) - 1
        self.h[0], self.h[n] = self.h[n], self.h[0]
        self._down(0, n)
        return self.h.pop()

    def add(self, node, ts):  # AddBinding
        if len(self.h) == self.size:
            self.pop()
        self.push((node, ts))

    def gc_at(self, now_unix):  # BindingsGC
        if self.gc == 0:
            return
        timeline = now_unix - int(self.gc // 10**9)
        while self.h:
            b = self.pop()
            if b[1] > timeline:
                self.push(b)
                return


def _ops(rng, n, n_nodes, t0, tie_span):
    ops = (rng.random(n) < 0.03).astype(np.uint8)
    node = rng.integers(0, n_nodes, n).astype(np.int32)
    # mostly rising timestamps with many ties and some out-of-order inserts
    ts = t0 + np.cumsum(rng.integers(0, 2, n)) // tie_span + rng.integers(-3, 1, n) * (rng.random(n) < 0.1)
    arg = np.where(ops == 1, ts + rng.integers(30, 400, n), ts).astype(np.int64)
    return ops, node, arg


@pytest.mark.parametrize("size,seed", [(1, 1), (2, 2), (7, 3), (64, 4), (1000, 5)])
def test_oracle_heap_matches_go_restatement(size, seed):
    rng = np.random.default_rng(seed)
    ops, node, arg = _ops(rng, 5000, 50, 1_000_000, 3)
    g = GoHeap(size, 5 * M_NS)
    for o, n, a in zip(ops, node, arg):
        if o == 0:
            g.add(int(n), int(a))
        else:
            g.gc_at(int(a))
    on, ot = O.binding_heap(size, 5 * M_NS, ops, node, arg)
    assert list(zip(on.tolist(), ot.tolist())) == g.h


def test_oracle_heap_rejects_zero_size():
    with pytest.raises(ValueError):
        O.binding_heap(0, 0, [0], [1], [5])


@pytest.mark.parametrize("msg,count,expect", [
    ("Successfully assigned default/nginx-6799fc88d8-5wbx5 to node-1", 0, ("default", "nginx-6799fc88d8-5wbx5",
                                                                          "node-1", "ev")),
    ("Successfully assigned default/p to n1", 3, ("default", "p", "n1", "last")),
    ("Successfully assigned p to n1", 1, ("", "p", "n1", "last")),                  # SplitMetaNamespaceKey: 1 part
    ("Successfully   assigned \t ns/p    to  n1 and more", 0, ("ns", "p", "n1", "ev")),  # spaces: one or more
    ("Successfully assigned ns/p to n1\n", 0, ("ns", "p", "n1", "ev")),
    ("Successfully assigned\u00a0ns/p to n1", 0, ("ns", "p", "n1", "ev")),     # U+00A0 is a space to fmt
    ("Successfully assigned a/b/c to n1", 0, None),                                 # too many '/'
    ("Successfully assigned ns/p", 0, None),                                        # EOF before "to"
    ("Successfully assigned ns/p to ", 0, None),                                    # empty %s at EOF
    ("Successfully assigned ns/p to\n n1", 0, None),                                # newline before the token
    (" Successfully assigned ns/p to n1", 0, None),                                 # literal must match first
    ("Successfullyassigned ns/p to n1", 0, None),                                   # format space needs >= 1
    ("Successfully assigned ns/p tonode", 0, None),
    ("Bound ns/p to n1", 0, None),
])
def test_translate_event(msg, count, expect):
    ev_ns, last_ns = 1792065600_987654321, 1792065599_000000001
    got = cd.translate_event(msg, count, ev_ns, last_ns)
    if expect is None:
        assert got is None
    else:
        ns, pod, node, which = expect
        assert got == (ns, pod, node, (ev_ns if which == "ev" else last_ns) // 10**9)


def test_translate_event_negative_time_floors():
    # metav1.Time.Unix() floors: -1 ns -> -1 s
    assert cd.translate_event("Successfully assigned a/b to c", 0, -1, 0)[3] == -1


def _engine_heap_case(eng, spec, size, gc, ops, node, arg, n_nodes, checks):
    """Replays ops through the engine in batches split at GC ops and checks hot values
    at the given times against the oracle heap."""
    i = 0
    while i < len(ops):
        if ops[i] == 1:
            eng.gc_bindings(int(arg[i]) * 10**9 + 5)
            i += 1
            continue
        j = i
        while j < len(ops) and ops[j] == 0:
            j += 1
        eng.add_bindings(node[i:j], arg[i:j])
        i = j
    on, ot = O.binding_heap(size, gc, ops, node, arg)
    assert eng.binding_count() == len(on)
    for now_unix in checks:
        now_ns = now_unix * 10**9 + 7
        eng.refresh_hot_values(now_ns, now_ns)
        _, hv = O.hot_values(spec, on, ot, n_nodes, now_unix)
        assert np.array_equal(eng.hot_values(), hv.astype(np.float64)), now_unix


@pytest.mark.gpu
@pytest.mark.parametrize("size,n_ops,n_nodes,seed", [(1, 300, 5, 1), (16, 3000, 40, 2), (1000, 20000, 300, 3),
                                                     (4096, 50000, 3000, 4)])
def test_engine_heap_matches_oracle(size, n_ops, n_nodes, seed):
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, n_nodes, 1, seed=seed)
    from helpers import engine_for
    eng = engine_for(spec, c)
    gc = max(tr for tr, _ in spec["hotValue"])  # controller.go:57 (getMaxHotVauleTimeRange)
    eng.binding_records(size, gc)
    rng = np.random.default_rng(seed)
    ops, node, arg = _ops(rng, n_ops, n_nodes + 3, synth.NOW0 - 700, 40)  # + nodes past the shard
    node[::53] = -1
    last = int(arg[ops == 0].max())
    _engine_heap_case(eng, spec, size, gc, ops, node, arg, n_nodes, [last, last - 100, last + 250])


@pytest.mark.gpu
def test_engine_heap_config3_syncs():
    """A 1M-entry heap (config 3's log) filled once, then controller syncs that append one
    second of bindings and GC: hot values equal the oracle heap's after every sync."""
    spec = cd.default_policy_spec()
    N, B = 100_000, 1_000_000
    c = synth.make_cluster(spec, N, 1, n_bindings=B, seed=41)
    from helpers import engine_for
    eng = engine_for(spec, c)
    gc = 5 * M_NS
    eng.binding_records(B, gc)
    eng.add_bindings(c.b_node, c.b_ts)
    rng = np.random.default_rng(41)
    ops = [np.zeros(B, np.uint8)]
    nodes, args = [c.b_node], [c.b_ts]
    for s in range(1, 4):
        nb = rng.integers(1000, 2500)
        bn = rng.integers(0, N, nb).astype(np.int32)
        bt = np.full(nb, synth.NOW0 + s, np.int64)
        eng.add_bindings(bn, bt)
        eng.gc_bindings((synth.NOW0 + s) * 10**9)
        ops += [np.zeros(nb, np.uint8), np.ones(1, np.uint8)]
        nodes += [bn, np.zeros(1, np.int32)]
        args += [bt, np.array([synth.NOW0 + s], np.int64)]
        on, ot = O.binding_heap(B, gc, np.concatenate(ops), np.concatenate(nodes), np.concatenate(args))
        assert eng.binding_count() == len(on)
        now_ns = (synth.NOW0 + s) * 10**9
        eng.refresh_hot_values(now_ns, now_ns)
        _, hv = O.hot_values(spec, on, ot, N, synth.NOW0 + s)
        assert np.array_equal(eng.hot_values(), hv.astype(np.float64)), s


@pytest.mark.gpu
def test_heap_change_waits_for_async_step():
    """A step enqueued on a caller stream reads the binding log; add_bindings / gc_bindings
    issued right after (no host sync) must not change the slots under it: each step's keys
    equal a fresh engine's keys for the log as it stood when the step was enqueued."""
    import torch
    spec = cd.default_policy_spec()
    N, P = 20_000, 2_000
    c = synth.make_cluster(spec, N, P, n_bindings=200_000, seed=31)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    d_now = torch.from_numpy(c.now).to(dev)
    d_flags = torch.from_numpy(c.ds).to(dev)
    eng = cd.Engine(cd.Policy(spec), 0)
    val, ts, _ = c.rows(eng.metric_names)
    eng.upload_nodes(val, ts, c.hv, c.hv_ts)
    gc = 5 * M_NS
    eng.binding_records(150_000, gc)
    eng.add_bindings(c.b_node, c.b_ts)  # the heap evicts the oldest 50k
    now = int(synth.NOW0_NS)
    rng = np.random.default_rng(3)
    keys = []
    for rep in range(4):
        k = torch.empty(P, dtype=torch.int64, device=dev)
        eng.step_keys_async(now, now, d_now, d_flags, k, st.cuda_stream)
        keys.append(k)
        hot = rng.integers(0, 50, 40_000).astype(np.int32)  # hammer the hottest nodes' slots
        eng.add_bindings(hot, np.full(len(hot), synth.NOW0 - rep, np.int64))
        eng.gc_bindings(now + rep * 10**9)
    st.synchronize()
    # replay the same history through the oracle heap and a fresh engine per step
    ops, nodes, args = [np.zeros(len(c.b_node), np.uint8)], [c.b_node], [c.b_ts]
    rng = np.random.default_rng(3)
    for rep in range(4):
        on, ot = O.binding_heap(150_000, gc, np.concatenate(ops), np.concatenate(nodes), np.concatenate(args))
        ref = cd.Engine(cd.Policy(spec), 0)
        ref.upload_nodes(val, ts, c.hv, c.hv_ts)
        ref.upload_bindings(on, ot)
        rk = torch.empty(P, dtype=torch.int64, device=dev)
        ref.step_keys_async(now, now, d_now, d_flags, rk, st.cuda_stream)
        st.synchronize()
        ref.close()
        assert torch.equal(keys[rep], rk), rep
        hot = rng.integers(0, 50, 40_000).astype(np.int32)
        ops += [np.zeros(len(hot), np.uint8), np.ones(1, np.uint8)]
        nodes += [hot, np.zeros(1, np.int32)]
        args += [np.full(len(hot), synth.NOW0 - rep, np.int64), np.array([(now + rep * 10**9) // 10**9], np.int64)]
    eng.close()
