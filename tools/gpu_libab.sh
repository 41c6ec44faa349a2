# A/B of library variants (build_exp/<name>/libvlp_hip.so) on the conv micro-benchmark
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-libab}
for V in ${VARIANTS:-default}; do
  if [ "$V" = default ]; then L=$PWD/vision-language-pretraining-for-bone-tumor-detection_amd/vlp_amd/libvlp_hip.so; else L=$PWD/build_exp/$V/libvlp_hip.so; fi
  echo "== $V"
  VLP_HIP_LIB=$L timeout -k 10 200 python tools/conv_bench.py ${CB_ARGS:---layers l2,l3,l4} > gpurun_out/${T}_$V.log 2>&1 || { echo CB FAILED; tail -20 gpurun_out/${T}_$V.log; exit 1; }
  grep -v "^{" gpurun_out/${T}_$V.log | grep -v amdgpu.ids
done
