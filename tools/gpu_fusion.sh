# Late-fusion finetune on one MI355X: parity tests, bs=512 512^2 bench, rocprofv3 kernel stats.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r1f}
timeout -k 10 300 python -u -m pytest tests/test_fusion.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python tools/fusion_bench.py --out gpurun_out/${TAG}_bench.json > gpurun_out/${TAG}_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o stats -- python tools/fusion_bench.py --steps 5 --warmup 2 > gpurun_out/${TAG}_prof.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
tail -1 gpurun_out/${TAG}_prof.log
