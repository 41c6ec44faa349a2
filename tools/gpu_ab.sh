# A/B: GPU tests, then conv/GEMM micro-benchmarks under two GEMM variants
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-ab}
VLP_GEMM_VARIANT=${TEST_VARIANT:-4} timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for V in ${VARIANTS:-3 4}; do
echo "== variant $V"
VLP_GEMM_VARIANT=$V timeout -k 10 200 python tools/conv_bench.py ${CB_ARGS:---gemm} > gpurun_out/${T}_v$V.log 2>&1 || { echo CB FAILED; tail -20 gpurun_out/${T}_v$V.log; exit 1; }
grep -v "^{" gpurun_out/${T}_v$V.log | grep -v amdgpu.ids
done
