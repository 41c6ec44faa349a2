# NesT (BASELINE configs[3]) artefacts on one MI355X: bench line with kernel report,
# rocprofv3 kernel stats of the same command, and the two PMC traffic passes
# (FETCH_SIZE, WRITE_SIZE in separate runs).  Every step has its own time limit.
#   TAG=r6n bash tools/gpu_nest_round.sh
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-nest}
BA="--image-model nest_small"
timeout -k 10 600 python bench.py $BA --kernel-report gpurun_out/${TAG}_kreport.json > gpurun_out/${TAG}_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o stats -- python bench.py $BA --no-cpu-baseline --no-loss-check --pcie-steps 0 --dp-rehearsal 0 > gpurun_out/${TAG}_prof.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc -o fetch -- python bench.py $BA --steps 2 --warmup 1 --no-cpu-baseline --no-loss-check --pcie-steps 0 --dp-rehearsal 0 > gpurun_out/${TAG}_pmcf.log 2>&1 || { echo PMC1 FAILED; tail -20 gpurun_out/${TAG}_pmcf.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc -o write -- python bench.py $BA --steps 2 --warmup 1 --no-cpu-baseline --no-loss-check --pcie-steps 0 --dp-rehearsal 0 > gpurun_out/${TAG}_pmcw.log 2>&1 || { echo PMC2 FAILED; tail -20 gpurun_out/${TAG}_pmcw.log; exit 1; }
find gpurun_out/${TAG}_prof gpurun_out/${TAG}_pmc -name "*.csv" | head -20
