# layer-1 rows kernels with the planar ring: op parity, block parity, interleaved timings vs -DVLP_RC_PLANAR=0
cd $GRAFT_REPO_ROOT
T=${T:-r5r2}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "conv" > gpurun_out/${T}_ops.log 2>&1 || { echo OPS FAILED; tail -30 gpurun_out/${T}_ops.log; exit 1; }
tail -1 gpurun_out/${T}_ops.log
for r in 1 2; do
timeout -k 10 200 python tools/conv_bench.py --ops fwd,fwd_act,dgrad_bn_act,dgrad_relu_act,dgrad,dgrad_bn,dgrad_relu --layers l1 --iters 10 > gpurun_out/${T}_cb_planar_$r.log 2>&1 || exit 1
VLP_HIP_LIB=build_exp/rcold/libvlp_hip.so timeout -k 10 200 python tools/conv_bench.py --ops fwd,fwd_act,dgrad_bn_act,dgrad_relu_act,dgrad,dgrad_bn,dgrad_relu --layers l1 --iters 10 > gpurun_out/${T}_cb_old_$r.log 2>&1 || exit 1
done
for f in gpurun_out/${T}_cb_*.log; do echo "== $f"; grep TF/s $f; done
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_blocks.py > gpurun_out/${T}_blocks.log 2>&1 || { echo BLOCKS FAILED; tail -30 gpurun_out/${T}_blocks.log; exit 1; }
tail -1 gpurun_out/${T}_blocks.log
