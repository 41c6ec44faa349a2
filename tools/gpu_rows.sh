# layer-1 rows-kernel A/B (conv_bench fwd / dgrad variants) + text tower alone
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-r3i}
for V in default ${VARIANTS:-}; do
  if [ "$V" = default ]; then L=$PWD/vision-language-pretraining-for-bone-tumor-detection_amd/vlp_amd/libvlp_hip.so; else L=$PWD/build_exp/$V/libvlp_hip.so; fi
  echo "== $V"
  VLP_HIP_LIB=$L timeout -k 10 200 python tools/conv_bench.py --layers l1 --ops fwd,dgrad,dgrad_bn,dgrad_relu > gpurun_out/${T}_conv_$V.log 2>&1 || { echo CB FAILED; tail -5 gpurun_out/${T}_conv_$V.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/${T}_conv_$V.log | tail -6
done
timeout -k 10 200 python tools/text_tower_bench.py > gpurun_out/${T}_text.json 2>&1 || { echo TEXT FAILED; tail -5 gpurun_out/${T}_text.json; exit 1; }
tail -1 gpurun_out/${T}_text.json | cut -c1-1500
