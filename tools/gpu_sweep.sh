# GPU round: parity tests, then one short bench per GEMM pipeline variant
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q -m gpu > gpurun_out/check.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/check.log; exit 1; }
tail -2 gpurun_out/check.log
for v in ${VARIANTS:-4 1 2 3 0}; do
  VLP_GEMM_VARIANT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --kernel-report gpurun_out/kreport_v$v.json > gpurun_out/bench_v$v.log 2>&1 || { echo "variant $v failed"; tail -20 gpurun_out/bench_v$v.log; exit 1; }
  echo "v$v: $(tail -1 gpurun_out/bench_v$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
