# The drop-in harness's first engine-changing cycle: plain, with the update
# trace on stderr (CRANE_DYN_TRACE_UPD=1), under rocprofv3's kernel + HIP runtime trace, with 15
# fan-out threads, and with HIP limited to one hardware queue.   Usage: bash tools/gpu_dropin_probe.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp TZ=Asia/Shanghai
D=/tmp/crane_dd
python3 tools/dropin_files.py $D > $O/files.txt || exit 1
read PP SP PD < <(python3 -c "import ast; print(*ast.literal_eval(open('$O/files.txt').read().strip().splitlines()[-1]))")
H=crane-scheduler_amd/lib/dropin_bench
run() {  # label, env, args
  env $2 CRANE_DYN_TRACE_UPD=1 timeout -k 10 300 $H $PP $SP $PD --churn 10 $3 > $O/$1.json 2> $O/$1.err || { tail $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', 'median', d['cycle_ms_median'], 'max', d['cycle_ms_max'], 'max_after_first', d['cycle_ms_max_after_first_change'])"
  head -3 $O/$1.err
}
for spec in "plain||--threads 16" "threads8||--threads 8" "threads4||--threads 4" "nointr|HSA_ENABLE_INTERRUPT=0|--threads 16" "plain2||--threads 16" $PROBE_EXTRA; do
  IFS='|' read -r lab ev ar <<< "$spec"
  run "$lab" "$ev" "$ar"
done
[ -n "$NO_TRACE" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o tr \
  -- $GRAFT_REPO_ROOT/$H $PP $SP $PD --churn 10 --threads 16 > $O/traced.json 2> $O/traced.err || { tail $O/traced.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/traced.json').read().strip().splitlines()[-1]); print('traced max', d['cycle_ms_max'])"
ls $O/trace
