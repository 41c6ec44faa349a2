# ping-pong window kernel: EpiDgradRelu's y staged in LDS (default library now) vs not (build_exp/norelu)
cd $GRAFT_REPO_ROOT
T=${T:-r5u}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "dgrad_relu" > gpurun_out/${T}_ops.log 2>&1 || { echo OPS FAILED; tail -30 gpurun_out/${T}_ops.log; exit 1; }
tail -1 gpurun_out/${T}_ops.log
for r in 1 2; do
timeout -k 10 200 python tools/conv_bench.py --ops dgrad_relu,dgrad_bn --layers l2,l4 --iters 10 > gpurun_out/${T}_cb_lds_$r.log 2>&1 || exit 1
VLP_HIP_LIB=build_exp/norelu/libvlp_hip.so timeout -k 10 200 python tools/conv_bench.py --ops dgrad_relu,dgrad_bn --layers l2,l4 --iters 10 > gpurun_out/${T}_cb_nolds_$r.log 2>&1 || exit 1
done
for f in gpurun_out/${T}_cb_*.log; do echo "== $f"; grep TF/s $f; done
