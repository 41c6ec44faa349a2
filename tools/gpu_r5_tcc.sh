cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r5t_counters.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/r5t_tcc -o p -- python tools/conv_bench.py --ops fwd --layers l2,l3,l4 --iters 3 > gpurun_out/r5t_tcc.log 2>&1 || { echo TCC FAILED; tail -3 gpurun_out/r5t_tcc.log; }
PMC_FILTER=. python tools/pmc_summary.py $(find gpurun_out/r5t_tcc -name "*counter_collection.csv") | grep -A3 gemm
