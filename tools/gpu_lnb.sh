# TinyBERT LayerNorm backward: 8-wave blocks at text-sized M (default) vs 4 (lnb4)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-r3u}
PKG=$PWD/vision-language-pretraining-for-bone-tumor-detection_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_bert_ops.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for V in default lnb4 default lnb4; do
  if [ "$V" = default ]; then L=$PKG/vlp_amd/libvlp_hip.so; else L=$PWD/build_exp/$V/libvlp_hip.so; fi
  VLP_HIP_LIB=$L timeout -k 10 200 python tools/text_tower_bench.py > gpurun_out/${T}_tt_$V.log 2>&1 || { echo TT FAILED; tail -5 gpurun_out/${T}_tt_$V.log; exit 1; }
  echo "== $V"; grep -v amdgpu.ids gpurun_out/${T}_tt_$V.log | tail -4
done
for V in default lnb4 default lnb4; do
  if [ "$V" = default ]; then L=$PKG/vlp_amd/libvlp_hip.so; else L=$PWD/build_exp/$V/libvlp_hip.so; fi
  VLP_HIP_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-loss-check --pcie-steps 0 > gpurun_out/${T}_bench_$V.log 2>&1 || { echo BENCH FAILED; tail -10 gpurun_out/${T}_bench_$V.log; exit 1; }
  echo "$V $(tail -1 gpurun_out/${T}_bench_$V.log | cut -c1-140)"
done
