# Round-6 GPU step: a pytest selection (TESTS) then the bench (BENCH=0 skips it).
#   TAG=r6a TESTS="tests/test_gpu_dp.py tests/test_fusion.py" tools/gpu_r6.sh
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r6}
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -3 gpurun_out/${TAG}_tests.log
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python bench.py $BENCH_ARGS --kernel-report gpurun_out/${TAG}_kreport.json > gpurun_out/${TAG}_bench.log 2>&1 || { echo BENCH FAILED; tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
  tail -1 gpurun_out/${TAG}_bench.log
fi
