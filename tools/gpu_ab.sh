cd $GRAFT_REPO_ROOT
for e in "VLP_WGRAD_DYT=1" "VLP_WGRAD_DYT=0"; do
  env $e timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --kernel-report gpurun_out/kr_ab.json > gpurun_out/ab.log 2>&1 || { echo FAIL $e; tail -5 gpurun_out/ab.log; exit 1; }
  echo "$e $(tail -1 gpurun_out/ab.log | cut -c1-200)"
  python tools/kreport.py gpurun_out/kr_ab.json 8
done
