# round-3 check on the committed tree: all GPU tests, smoke, bench with kernel report
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r3b}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 250 python bench.py --kernel-report gpurun_out/${TAG}_kreport.json > gpurun_out/${TAG}_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
