# BN-apply + ReLU on the ping-pong kernel's A fragments:
# conv forward with in_scale/in_shift, fragment transform (default) vs the
# register-staged BN-on-load engine (fwdbn_reg), against the plain forward
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-r3p}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q -k "conv_fwd" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for V in default fwdbn_reg default; do
  if [ "$V" = default ]; then L=$PWD/vision-language-pretraining-for-bone-tumor-detection_amd/vlp_amd/libvlp_hip.so; else L=$PWD/build_exp/$V/libvlp_hip.so; fi
  echo "== $V"
  VLP_HIP_LIB=$L timeout -k 10 200 python tools/conv_bench.py --ops fwd,fwd_bn --layers l2,l3,l4 > gpurun_out/${T}_cb_$V.log 2>&1 || { echo CB FAILED; tail -5 gpurun_out/${T}_cb_$V.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/${T}_cb_$V.log
done
timeout -k 10 200 python tools/ew_bench.py > gpurun_out/${T}_ew.log 2>&1 || { echo EW FAILED; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_ew.log
