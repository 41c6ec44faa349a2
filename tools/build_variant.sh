# build a variant of libvlp_hip.so with extra -D flags into build_exp/<name>/libvlp_hip.so
#   tools/build_variant.sh NAME "-DVLP_BIG_SCHED=1 ..." [object ...]
# with object names given (e.g. conv_ops), only those are recompiled with the
# flags; the others are linked from the product build (csrc/build/*.o)
set -e
NAME=$1; FLAGS=$2; shift 2
ONLY="$*"
ROOT=$(cd $(dirname $0)/.. && pwd)
CSRC=$ROOT/vision-language-pretraining-for-bone-tumor-detection_amd/csrc
OUT=$ROOT/build_exp/$NAME
mkdir -p $OUT/obj
ALL="conv_ops stem_ops bn_ops bert_ops head_ops optim_ops probe_ops retrieval_ops nest_ops prep_ops"
for f in $ALL; do
  if [ -n "$ONLY" ] && ! echo " $ONLY " | grep -q " $f "; then
    cp $CSRC/build/$f.o $OUT/obj/$f.o
    continue
  fi
  EXTRA=""
  [ $f = nest_ops ] && EXTRA="-mllvm -amdgpu-mfma-vgpr-form=1"
  [ $f = prep_ops ] && EXTRA="-ffp-contract=off"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -fvisibility=hidden \
    -Wno-unused-result -Wno-c++20-extensions $EXTRA $FLAGS -c $CSRC/$f.hip -o $OUT/obj/$f.o &
  PIDS="$PIDS $!"
done
for p in $PIDS; do wait $p || { echo "variant $NAME: compile failed"; exit 1; }; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT/libvlp_hip.so $OUT/obj/*.o
rm -rf $OUT/obj
echo built $OUT/libvlp_hip.so
