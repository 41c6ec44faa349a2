# ping-pong GEMM kernel: op tests under a variant (VLP_PP=$TV) + conv micro-bench arms
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-pp}
VLP_PP=${TV:-4} timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_ops.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_ops.log; [ $rc = 0 ] || exit 1
for arm in ${ARMS:-VLP_PP=0 VLP_PP=1 VLP_PP=4}; do
  env $arm timeout -k 10 200 python tools/conv_bench.py --layers ${LAYERS:-l2,l3,l4} --ops ${OPS:-fwd,dgrad,dgrad_bn,wgrad} > gpurun_out/${T}_cb_$arm.log 2>&1 || { echo CB FAILED; tail -20 gpurun_out/${T}_cb_$arm.log; exit 1; }
  echo "arm $arm"; grep -v '^{' gpurun_out/${T}_cb_$arm.log | grep -v amdgpu.ids
done
