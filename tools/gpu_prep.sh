# stem1 u8 prep with 32-bit index math: stem tests + kernel report of one bench run
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-r3v}
timeout -k 10 400 python -u -m pytest tests/test_gpu_stem.py tests/test_gpu_ops.py -m gpu -x -q -k "stem" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 250 python bench.py --no-cpu-baseline --no-loss-check --pcie-steps 0 --kernel-report gpurun_out/${T}_kreport.json > gpurun_out/${T}_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/${T}_bench.log; exit 1; }
tail -1 gpurun_out/${T}_bench.log | cut -c1-150
python -c "import json; r=json.load(open('gpurun_out/${T}_kreport.json')); print({k: r[k] for k in r if 'stem' in k or 'prep' in k})"
