set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/t4m; mkdir -p $O
timeout -k 10 200 python tools/trace_step.py --config 3 --nodes 4000000 --bindings 16000000 > $O/trace4m.json 2> $O/trace4m.err || { tail $O/trace4m.err; exit 1; }
timeout -k 10 200 python tools/stream_bench.py --k2 auto --flush read --opt k1_threads=128 > $O/s128.json 2> $O/s128.err || { tail $O/s128.err; exit 1; }
timeout -k 10 200 python tools/trace_step.py --config 3 > $O/trace3.json 2> $O/trace3.err || { tail $O/trace3.err; exit 1; }
cat $O/s128.json
