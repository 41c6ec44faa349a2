# round-3 artefacts on one MI355X: GPU tests, smoke, bench (kernel report), rocprofv3 kernel
# stats of the bench command, separate FETCH_SIZE / WRITE_SIZE PMC passes
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r3f}
if [ -z "$NOTESTS" ]; then
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
fi
timeout -k 10 250 python bench.py --kernel-report gpurun_out/${TAG}_kreport.json > gpurun_out/${TAG}_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-900
B="python bench.py --no-cpu-baseline --no-loss-check --pcie-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o stats -- $B > gpurun_out/${TAG}_prof.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
tail -1 gpurun_out/${TAG}_prof.log | cut -c1-300
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc -o fetch -- $B --steps 2 --warmup 1 --roofline-steps 1 > gpurun_out/${TAG}_pmcf.log 2>&1 || { echo PMC1 FAILED; tail -20 gpurun_out/${TAG}_pmcf.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc -o write -- $B --steps 2 --warmup 1 --roofline-steps 1 > gpurun_out/${TAG}_pmcw.log 2>&1 || { echo PMC2 FAILED; tail -20 gpurun_out/${TAG}_pmcw.log; exit 1; }
find gpurun_out/${TAG}_prof gpurun_out/${TAG}_pmc -name "*.csv" | head -20
