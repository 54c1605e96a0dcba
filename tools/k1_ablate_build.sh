# Builds variants of the streamed K1 (k1stream.hip with extra -D flags; K1S_SKIP masks give wrong
# tables, timing only) as crane-scheduler_amd/lib_ab/lib_<name>.so, the product objects
# otherwise.  Usage: bash tools/k1_ablate_build.sh name=-DFLAG=V,-DFLAG2=V ...  (name alone: no flags)
set -e
cd "$(dirname "$0")/../crane-scheduler_amd/csrc"
make -j8 >/dev/null
mkdir -p ../lib_ab _obj_ab
for spec in "$@"; do
  name=${spec%%=*}; flags=""; [ "$spec" != "$name" ] && flags=$(echo "${spec#*=}" | tr ',' ' ')
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall --offload-arch=gfx950 \
      $flags -c k1stream.hip -o _obj_ab/k1stream_$name.o
  objs=$(ls _obj/*.o | grep -v k1stream.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib_ab/lib_$name.so $objs _obj_ab/k1stream_$name.o \
      -L/opt/rocm/lib -lrccl
done
