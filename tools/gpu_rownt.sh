# row-chunk epilogue stores: plain (default) vs non-temporal (row_nt); conv bench + interleaved bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-r3x}
PKG=$PWD/vision-language-pretraining-for-bone-tumor-detection_amd
VLP_HIP_LIB=$PWD/build_exp/row_nt/libvlp_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q -k "dgrad" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for V in default row_nt; do
  if [ "$V" = default ]; then L=$PKG/vlp_amd/libvlp_hip.so; else L=$PWD/build_exp/$V/libvlp_hip.so; fi
  VLP_HIP_LIB=$L timeout -k 10 200 python tools/conv_bench.py --ops dgrad_bn,dgrad_relu > gpurun_out/${T}_cb_$V.log 2>&1 || { echo CB FAILED; tail -5 gpurun_out/${T}_cb_$V.log; exit 1; }
  echo "== $V"; grep -v amdgpu.ids gpurun_out/${T}_cb_$V.log | head -8
done
for V in default row_nt default row_nt; do
  if [ "$V" = default ]; then L=$PKG/vlp_amd/libvlp_hip.so; else L=$PWD/build_exp/$V/libvlp_hip.so; fi
  VLP_HIP_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-loss-check --pcie-steps 0 > gpurun_out/${T}_bench_$V.log 2>&1 || { echo BENCH FAILED; tail -10 gpurun_out/${T}_bench_$V.log; exit 1; }
  echo "$V $(tail -1 gpurun_out/${T}_bench_$V.log | cut -c1-140)"
done
