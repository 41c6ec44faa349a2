# streaming BN passes: pipelined (default) vs not (ew_nopipe), then the bench line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-r3l}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q -k "bn or relu or maxpool" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for V in default ew_nopipe; do
  if [ "$V" = default ]; then L=$PWD/vision-language-pretraining-for-bone-tumor-detection_amd/vlp_amd/libvlp_hip.so; else L=$PWD/build_exp/$V/libvlp_hip.so; fi
  echo "== $V"
  VLP_HIP_LIB=$L timeout -k 10 200 python tools/ew_bench.py > gpurun_out/${T}_ew_$V.log 2>&1 || { echo EW FAILED; tail -5 gpurun_out/${T}_ew_$V.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/${T}_ew_$V.log
done
for V in default ew_nopipe default ew_nopipe; do
  if [ "$V" = default ]; then L=$PWD/vision-language-pretraining-for-bone-tumor-detection_amd/vlp_amd/libvlp_hip.so; else L=$PWD/build_exp/$V/libvlp_hip.so; fi
  VLP_HIP_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-loss-check --pcie-steps 0 > gpurun_out/${T}_bench_$V.log 2>&1 || { echo BENCH FAILED; tail -10 gpurun_out/${T}_bench_$V.log; exit 1; }
  echo "$V $(tail -1 gpurun_out/${T}_bench_$V.log | cut -c1-160)"
done
