# A/B of library variants (build_exp/<name>/libvlp_hip.so) on the NesT per-kernel bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-nestab}
for V in ${VARIANTS:-default}; do
  if [ "$V" = default ]; then L=$PWD/vision-language-pretraining-for-bone-tumor-detection_amd/vlp_amd/libvlp_hip.so; else L=$PWD/build_exp/$V/libvlp_hip.so; fi
  echo "== $V"
  VLP_HIP_LIB=$L timeout -k 10 300 python tools/nest_gemm_bench.py ${NB_ARGS} --out gpurun_out/${T}_$V.json > gpurun_out/${T}_$V.log 2>&1 || { echo NB FAILED; tail -20 gpurun_out/${T}_$V.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/${T}_$V.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print(d['level'], f\"{d['kernel']:20s} {d['us']:8.1f} us {d['TF/s']:7.1f} TF/s {d['GB/s']:7.1f} GB/s\")"
done
