# Builds cost-ablation variants of the streamed K1 (k1stream.hip with -DK1S_SKIP=<mask>: wrong
# tables, timing only) as crane-scheduler_amd/lib_ab/lib_s<mask>.so, the product objects
# otherwise.  Usage: bash tools/k1_ablate_build.sh 0 1 2 3 ...
set -e
cd "$(dirname "$0")/../crane-scheduler_amd/csrc"
make -j8 >/dev/null
mkdir -p ../lib_ab _obj_ab
# a mask may carry a wave count: 0w8 = K1S_SKIP 0 built for 8 waves per SIMD
for m in "$@"; do
  sk=${m%%w*}; wv=7; [ "$m" != "$sk" ] && wv=${m##*w}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall --offload-arch=gfx950 \
      -DK1S_SKIP=$sk -DK1S_WAVES=$wv -c k1stream.hip -o _obj_ab/k1stream_$m.o
  objs=$(ls _obj/*.o | grep -v k1stream.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib_ab/lib_s$m.so $objs _obj_ab/k1stream_$m.o \
      -L/opt/rocm/lib -lrccl
done
