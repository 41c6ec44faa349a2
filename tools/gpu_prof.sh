# rocprofv3 kernel stats of the bench command (no CPU baseline / loss check), TAG-named
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r2}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o stats -- python bench.py --no-cpu-baseline --no-loss-check --pcie-steps 0 --steps ${STEPS:-20} --kernel-report gpurun_out/${TAG}_kreport.json > gpurun_out/${TAG}_prof.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
tail -1 gpurun_out/${TAG}_prof.log | cut -c1-400
find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -3
