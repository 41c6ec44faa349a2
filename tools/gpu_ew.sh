# A/B of the BN streaming-pass variants (VLP_EW) on tools/ew_bench.py
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for arm in ${ARMS:-0 1 2 3 4}; do
  VLP_EW=$arm timeout -k 10 200 python tools/ew_bench.py > gpurun_out/ew_$arm.log 2>&1 || { echo EW FAILED; tail -20 gpurun_out/ew_$arm.log; exit 1; }
  echo "arm $arm"; grep -v amdgpu.ids gpurun_out/ew_$arm.log
done
