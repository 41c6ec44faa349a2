# NesT-Small (BASELINE configs[3]) round artefacts: bench line, rocprofv3 kernel
# stats, separate FETCH_SIZE / WRITE_SIZE PMC passes for the roofline family
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r3n}
B="python bench.py --image-model nest_small --no-cpu-baseline --no-loss-check --pcie-steps 0"
timeout -k 10 400 python bench.py --image-model nest_small --steps 10 --warmup 3 --kernel-report gpurun_out/${TAG}_kreport.json > gpurun_out/${TAG}_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o stats -- $B --steps 5 --warmup 2 > gpurun_out/${TAG}_prof.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
tail -1 gpurun_out/${TAG}_prof.log | cut -c1-300
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc -o fetch -- $B --steps 1 --warmup 1 --roofline-steps 1 > gpurun_out/${TAG}_pmcf.log 2>&1 || { echo PMC1 FAILED; tail -20 gpurun_out/${TAG}_pmcf.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc -o write -- $B --steps 1 --warmup 1 --roofline-steps 1 > gpurun_out/${TAG}_pmcw.log 2>&1 || { echo PMC2 FAILED; tail -20 gpurun_out/${TAG}_pmcw.log; exit 1; }
find gpurun_out/${TAG}_prof gpurun_out/${TAG}_pmc -name "*.csv" | head -20
