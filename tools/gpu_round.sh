# Round artefacts on one MI355X: GPU parity tests, smoke, bench (with CPU
# baseline), rocprofv3 kernel stats of the bench command, PMC HBM traffic passes.
# BENCH_ARGS="--image-model nest_small" gives the NesT (configs[3]) artefacts.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r1}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python bench.py $BENCH_ARGS --kernel-report gpurun_out/${TAG}_kreport.json > gpurun_out/${TAG}_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o stats -- python bench.py $BENCH_ARGS --no-cpu-baseline --no-loss-check --pcie-steps 0 > gpurun_out/${TAG}_prof.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
tail -1 gpurun_out/${TAG}_prof.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc -o fetch -- python bench.py $BENCH_ARGS --steps 2 --warmup 1 --no-cpu-baseline --no-loss-check --pcie-steps 0 > gpurun_out/${TAG}_pmcf.log 2>&1 || { echo PMC1 FAILED; tail -20 gpurun_out/${TAG}_pmcf.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc -o write -- python bench.py $BENCH_ARGS --steps 2 --warmup 1 --no-cpu-baseline --no-loss-check --pcie-steps 0 > gpurun_out/${TAG}_pmcw.log 2>&1 || { echo PMC2 FAILED; tail -20 gpurun_out/${TAG}_pmcw.log; exit 1; }
find gpurun_out/${TAG}_prof gpurun_out/${TAG}_pmc -name "*.csv" | head -20
