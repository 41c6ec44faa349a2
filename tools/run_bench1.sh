set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --kernel-report gpurun_out/kreport1.json > gpurun_out/bench1.log 2>&1
