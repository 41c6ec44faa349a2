cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "conv_fwd_act or conv_fwd" > gpurun_out/r5y_ops.log 2>&1 || { echo OPS FAILED; tail -30 gpurun_out/r5y_ops.log; exit 1; }
tail -1 gpurun_out/r5y_ops.log
timeout -k 10 300 python tools/conv_bench.py --ops fwd,fwd_act,pass_fwd --layers l2,l3,l4 --iters 10 > gpurun_out/r5y_cb.log 2>&1 || exit 1
grep TF/s gpurun_out/r5y_cb.log
