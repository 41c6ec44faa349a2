# window kernel with the epilogue operand staged in LDS: op parity, block parity, timings
# (default library: layers 2 and 4 on the window kernel; build_exp/allw: layer 3 too)
cd $GRAFT_REPO_ROOT
T=${T:-r5l}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "conv" > gpurun_out/${T}_ops.log 2>&1 || { echo OPS FAILED; tail -30 gpurun_out/${T}_ops.log; exit 1; }
tail -1 gpurun_out/${T}_ops.log
timeout -k 10 200 python tools/conv_bench.py --ops fwd,dgrad,dgrad_bn,dgrad_relu --layers l2,l3,l4 --iters 10 > gpurun_out/${T}_cb.log 2>&1 || exit 1
VLP_HIP_LIB=build_exp/allw/libvlp_hip.so timeout -k 10 200 python tools/conv_bench.py --ops fwd,dgrad,dgrad_bn,dgrad_relu --layers l3 --iters 10 > gpurun_out/${T}_cb_allw.log 2>&1 || exit 1
grep TF/s gpurun_out/${T}_cb.log; echo "== all widths (l3 on the window kernel)"; grep TF/s gpurun_out/${T}_cb_allw.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_blocks.py > gpurun_out/${T}_blocks.log 2>&1 || { echo BLOCKS FAILED; tail -30 gpurun_out/${T}_blocks.log; exit 1; }
tail -1 gpurun_out/${T}_blocks.log
