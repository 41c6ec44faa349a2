# weight-gradient split count sized for 1/DIV of the chip (side-stream contention A/B)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-r3o}
VARIANTS=${VARIANTS:-"default wg_div2 wg_div4"}
VLP_HIP_LIB=$PWD/build_exp/wg_div4/libvlp_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q -k "wgrad" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for R in 1 2; do
for V in $VARIANTS; do
  if [ "$V" = default ]; then L=$PWD/vision-language-pretraining-for-bone-tumor-detection_amd/vlp_amd/libvlp_hip.so; else L=$PWD/build_exp/$V/libvlp_hip.so; fi
  VLP_HIP_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-loss-check --pcie-steps 0 > gpurun_out/${T}_bench_${V}_$R.log 2>&1 || { echo BENCH FAILED; tail -10 gpurun_out/${T}_bench_${V}_$R.log; exit 1; }
  echo "$V $(tail -1 gpurun_out/${T}_bench_${V}_$R.log | cut -c1-160)"
done
done
