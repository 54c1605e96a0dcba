# GPU capacity for the config-3 step beyond one process's launch rate: two processes on the one GPU,
# each with its own engines and streams (2 batches in flight each), timed loops started together,
# against one process with 4 in flight (same box, two rounds).  Each process's HIP launches go
# through its own runtime, so the pair's combined batches/s is bounded by the GPU, not by one
# thread's launch cost.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05procs}
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 200 python tools/inflight_probe.py --bound --inflight 4 --steps 4000 > $O/one_$rep.json 2>&1 || { tail $O/one_$rep.json; exit 1; }
  T=$(python3 -c "import time; print(time.time() + 75)")
  timeout -k 10 200 python tools/inflight_probe.py --bound --inflight 2 --steps 4000 --start-at $T > $O/a_$rep.json 2>&1 &
  pa=$!
  timeout -k 10 200 python tools/inflight_probe.py --bound --inflight 2 --steps 4000 --start-at $T > $O/b_$rep.json 2>&1 &
  pb=$!
  wait $pa || { tail $O/a_$rep.json; exit 1; }
  wait $pb || { tail $O/b_$rep.json; exit 1; }
  python3 - $O $rep <<'PY'
import json, sys
o, r = sys.argv[1:3]
ld = lambda f: json.loads(open(f).read().strip().splitlines()[-1])
one, a, b = ld(f"{o}/one_{r}.json")["inflight4"], ld(f"{o}/a_{r}.json")["inflight2"], ld(f"{o}/b_{r}.json")["inflight2"]
ov = min(a["wall"][1], b["wall"][1]) - max(a["wall"][0], b["wall"][0])
span = max(a["wall"][1], b["wall"][1]) - min(a["wall"][0], b["wall"][0])
print(f"rep {r}: one process x4 {one['ms_per_step']} ms/batch (enqueue {one['host_enqueue_ms_per_step']}); "
      f"two processes x2: {a['ms_per_step']} / {b['ms_per_step']} ms/batch each, overlap {ov*1e3:.1f} of {span*1e3:.1f} ms, "
      f"combined {2 * 4000 / span / 1e3:.1f} batches/ms = {span * 1e3 / 8000:.4f} ms/batch")
PY
done
