# layer-1 conv2 with bn1 + ReLU in the rows kernel's ring (vlp_conv_fwd_act):
# op parity, model tests, conv bench (fused vs pass + conv), interleaved bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-r3q}
PKG=$PWD/vision-language-pretraining-for-bone-tumor-detection_amd
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fullres.py tests/test_gpu_model.py tests/test_gpu_streams.py -m gpu -x -q -k "conv_fwd_act or fullres or model or stream or bf16" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 gpurun_out/${T}_tests.log
for L in $PKG/vlp_amd/libvlp_hip.so $PWD/build_exp/act_nt/libvlp_hip.so; do
  VLP_HIP_LIB=$L timeout -k 10 200 python tools/conv_bench.py --ops fwd,fwd_act,pass_fwd --layers l1 > gpurun_out/${T}_cb.log 2>&1 || { echo CB FAILED; tail -5 gpurun_out/${T}_cb.log; exit 1; }
  echo "== $L"; grep -v amdgpu.ids gpurun_out/${T}_cb.log | head -3
done
for V in fused pass fused pass; do
  if [ "$V" = fused ]; then F=True; else F=False; fi
  timeout -k 10 200 python -c "import sys; sys.path.insert(0, '$PKG'); sys.argv = ['bench.py', '--no-cpu-baseline', '--no-loss-check', '--pcie-steps', '0']; import vlp_amd.resnet34 as r; r._USE_ACT_FUSED = $F; import runpy; runpy.run_path('bench.py', run_name='__main__')" > gpurun_out/${T}_bench_$V.log 2>&1 || { echo BENCH FAILED; tail -10 gpurun_out/${T}_bench_$V.log; exit 1; }
  echo "$V $(tail -1 gpurun_out/${T}_bench_$V.log | cut -c1-160)"
done
