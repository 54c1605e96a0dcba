# Host-enqueue variants of the in-flight step at config 3 (tools/inflight_probe.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/host; mkdir -p $O
timeout -k 10 200 python tools/inflight_probe.py --inflight 1,4 > $O/plain.json 2>&1 || { tail $O/plain.json; exit 1; }
timeout -k 10 200 python tools/inflight_probe.py --inflight 1,4 --bound > $O/bound.json 2>&1 || { tail $O/bound.json; exit 1; }
timeout -k 10 200 python tools/inflight_probe.py --inflight 4 --bound --threads > $O/threads.json 2>&1 || { tail $O/threads.json; exit 1; }
tail -qn1 $O/plain.json $O/bound.json $O/threads.json
