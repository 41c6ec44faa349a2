# final-tree check: the new streams test, then the whole GPU suite and smoke
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-r3y}
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py -m gpu -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_streams.log 2>&1 || { echo STREAMS FAILED; tail -30 gpurun_out/${T}_streams.log; exit 1; }
tail -1 gpurun_out/${T}_streams.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 250 python bench.py > gpurun_out/${T}_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/${T}_bench.log; exit 1; }
tail -1 gpurun_out/${T}_bench.log | cut -c1-200
