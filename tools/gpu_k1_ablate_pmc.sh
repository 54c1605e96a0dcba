# VALU / SALU / LDS instructions per wave of the cold K1 for ablation builds (tools/k1_ablate_build.sh)
# swapped in as the engine library: one rocprofv3 --pmc pass per build (counters only).
# Usage: bash tools/gpu_k1_ablate_pmc.sh <tag> <name> ...
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/$1; shift; mkdir -p $O
L=crane-scheduler_amd/lib/libcrane_dyn.so
cp $L $O/orig.so
trap 'cp $O/orig.so $L' EXIT
for m in "$@"; do
  cp crane-scheduler_amd/lib_ab/lib_$m.so $L || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      --output-format csv -d $O/$m -o p -- python3 $GRAFT_REPO_ROOT/bench.py --leg cold --steps 2 > $O/$m.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$m rc=$rc"; tail -5 $O/$m.log; exit $rc; }
  python3 - $O/$m/p_counter_collection.csv $m <<'PY'
import csv, sys, collections
tot = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"]
    if "k1_stream_steps" not in k: continue
    tot[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
def avg(c):
    d = tot[c]; return sum(d.values()) / max(1, len(d))
w = avg("SQ_WAVES")
print(sys.argv[2], "waves", round(w), "valu/wave", round(avg("SQ_INSTS_VALU") / w, 1), "salu/wave",
      round(avg("SQ_INSTS_SALU") / w, 1), "lds/wave", round(avg("SQ_INSTS_LDS") / w, 1),
      "valu/block", round(avg("SQ_INSTS_VALU") / w * 4, 1), "wave_cycles/wave", round(avg("SQ_WAVE_CYCLES") / w, 1))
PY
done
