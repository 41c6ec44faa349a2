# A/B of the 1-wave-per-SIMD 256x256 GEMM tiles (VLP_BIG_W1) on the conv micro-bench + op tests under the variant
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-w1}
for arm in 0 1 2; do
  VLP_BIG_W1=$arm timeout -k 10 200 python tools/conv_bench.py --layers l2,l3,l4 --ops ${OPS:-fwd,dgrad,dgrad_bn,wgrad} > gpurun_out/${T}_cb$arm.log 2>&1 || { echo CB FAILED; tail -20 gpurun_out/${T}_cb$arm.log; exit 1; }
  echo "arm $arm"; grep -v '^{' gpurun_out/${T}_cb$arm.log | grep -v amdgpu.ids
done
VLP_BIG_W1=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_ops.log 2>&1; tail -3 gpurun_out/${T}_ops.log
