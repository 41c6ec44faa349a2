# full artifact round: bench with CPU baseline, then rocprofv3 kernel stats of the same command
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
#timeout -k 10 600 python bench.py --kernel-report gpurun_out/kreport_full.json > gpurun_out/bench_full.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o r1 -- python bench.py --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof.log; exit 1; }
find gpurun_out/prof -name "*stats*" | head
