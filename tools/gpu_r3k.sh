# conv op tests + layer-1 conv bench + bench line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-r3k}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fullsize_ops.py tests/test_gpu_model.py tests/test_gpu_stem.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 200 python tools/conv_bench.py --layers l1 --ops fwd,dgrad,dgrad_bn,dgrad_relu > gpurun_out/${T}_conv.log 2>&1 || { echo CB FAILED; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_conv.log | tail -1
timeout -k 10 200 python tools/stem_bench.py > gpurun_out/${T}_stem_bench.json 2>&1 || { echo STEM BENCH FAILED; exit 1; }
tail -1 gpurun_out/${T}_stem_bench.json
timeout -k 10 250 python bench.py --no-cpu-baseline --no-loss-check --kernel-report gpurun_out/${T}_kreport.json > gpurun_out/${T}_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/${T}_bench.log; exit 1; }
tail -1 gpurun_out/${T}_bench.log | cut -c1-400
