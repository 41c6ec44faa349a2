# quick A/B loop: conv op tests, conv micro-bench, then the bench with a kernel report
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-q}
timeout -k 10 300 python -u -m pytest ${SEL:-tests/test_gpu_ops.py} -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python tools/conv_bench.py > gpurun_out/${TAG}_cb.log 2>&1 || { echo CB FAILED; tail -20 gpurun_out/${TAG}_cb.log; exit 1; }
grep TF gpurun_out/${TAG}_cb.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-loss-check --pcie-steps 0 --steps 20 --kernel-report gpurun_out/${TAG}_kreport.json ${BENCH_ARGS} > gpurun_out/${TAG}_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-300
python tools/kreport.py gpurun_out/${TAG}_kreport.json 2>/dev/null | head -30 || true
