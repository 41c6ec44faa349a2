# GPU parity tests (all, no -x: every failure is reported) then a bench line.
# A crash/timeout of the test step (exit >= 2 other than test failures) stops the call.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r2}
SEL=${SEL:-tests}
timeout -k 10 ${TT:-900} python -u -m pytest $SEL -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED" gpurun_out/${TAG}_tests.log | tail -60
tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TEST STEP rc=$rc: stopping"; exit $rc; fi
if [ -n "$NOBENCH" ]; then exit $rc; fi
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/${TAG}_bench.log; exit 3; }
tail -1 gpurun_out/${TAG}_bench.log
