# quick GPU round: parity tests + bench with kernel report
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q -m gpu > gpurun_out/check.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/check.log; exit 1; }
tail -2 gpurun_out/check.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --kernel-report gpurun_out/kreport.json > gpurun_out/bench.log 2>&1
tail -1 gpurun_out/bench.log
timeout -k 10 200 python tools/conv_bench.py > gpurun_out/conv_bench.log 2>&1 && grep -v "^{" gpurun_out/conv_bench.log | grep -v amdgpu.ids
