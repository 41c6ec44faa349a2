# A/B of (library variant, env) arms on the conv micro-benchmark, interleaved:
#   ARMS="default| split| split|VLP_MN256=1"   (variant|env ; arms separated by spaces)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-libab2}
n=0
for rep in 1 2; do
for A in ${ARMS}; do
  V=${A%%|*}; E=${A#*|}
  if [ "$V" = default ]; then L=$PWD/vision-language-pretraining-for-bone-tumor-detection_amd/vlp_amd/libvlp_hip.so; else L=$PWD/build_exp/$V/libvlp_hip.so; fi
  echo "== $V [$E]"
  env $E VLP_HIP_LIB=$L timeout -k 10 200 python tools/conv_bench.py ${CB_ARGS:---layers l2,l3,l4} > gpurun_out/${T}_$n.log 2>&1 || { echo CB FAILED; tail -20 gpurun_out/${T}_$n.log; exit 1; }
  grep -v "^{" gpurun_out/${T}_$n.log | grep -v amdgpu.ids
  n=$((n+1))
done
done
