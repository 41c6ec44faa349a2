# epilogue timing experiments (VLP_EPI_EXP variants of conv_ops.o; wrong results by design):
# 1 = staged epilogues skip global stores, 2 = skip stats, 3 = row epilogues skip operand loads
cd $GRAFT_REPO_ROOT
T=${T:-r5f}
timeout -k 10 200 python tools/conv_bench.py --ops fwd,dgrad,dgrad_bn,dgrad_relu --layers l2,l3,l4 --iters 10 > gpurun_out/${T}_default.log 2>&1 || exit 1
for i in 1 2 3; do
  VLP_HIP_LIB=build_exp/epi$i/libvlp_hip.so timeout -k 10 200 python tools/conv_bench.py --ops fwd,dgrad,dgrad_bn,dgrad_relu --layers l2,l3,l4 --iters 10 > gpurun_out/${T}_exp$i.log 2>&1 || { echo EXP $i FAILED; tail -3 gpurun_out/${T}_exp$i.log; exit 1; }
done
for f in gpurun_out/${T}_default.log gpurun_out/${T}_exp*.log; do echo "== $f"; grep "TF/s" $f; done
