# targeted re-check: stream/stem/only-imaging tests, then the full GPU suite, smoke, bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r3c}
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_stem.py tests/test_only_imaging.py -m gpu -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_t1.log 2>&1 || { echo T1 FAILED; grep -E "PASSED|FAILED|Error|worst" gpurun_out/${TAG}_t1.log | cut -c1-400 | tail -30; exit 1; }
grep -E "worst|passed|failed" gpurun_out/${TAG}_t1.log | cut -c1-400 | tail -8
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 250 python bench.py --kernel-report gpurun_out/${TAG}_kreport.json > gpurun_out/${TAG}_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
timeout -k 10 200 python bench.py --split-fwd 0 --no-cpu-baseline --no-loss-check --pcie-steps 0 > gpurun_out/${TAG}_bench_nosplit.log 2>&1 || { echo BENCH2 FAILED; tail -20 gpurun_out/${TAG}_bench_nosplit.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench_nosplit.log | cut -c1-200
timeout -k 10 200 python bench.py --split-bwd 1 --no-cpu-baseline --no-loss-check --pcie-steps 0 > gpurun_out/${TAG}_bench_splitbwd.log 2>&1 || { echo BENCH3 FAILED; tail -20 gpurun_out/${TAG}_bench_splitbwd.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench_splitbwd.log | cut -c1-200
