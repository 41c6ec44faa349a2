# fused layer-1 forward: op parity + conv bench (fwd / fused / pass + fwd)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-r3r}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q -k "conv_fwd_act" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for R in 1 2; do
timeout -k 10 200 python tools/conv_bench.py --ops fwd,fwd_act,pass_fwd --layers l1 > gpurun_out/${T}_cb.log 2>&1 || { echo CB FAILED; tail -5 gpurun_out/${T}_cb.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_cb.log | head -3
done
