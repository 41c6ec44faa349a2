# window kernel: 8-wave (default library; layer 3 on the ping-pong GEMM) vs 4-wave variant (all widths)
cd $GRAFT_REPO_ROOT
T=${T:-r5n}
timeout -k 10 200 python tools/conv_bench.py --ops fwd,dgrad,dgrad_bn,dgrad_relu --layers l2,l3,l4 --iters 10 > gpurun_out/${T}_nw8.log 2>&1 || { echo NW8 FAILED; tail -3 gpurun_out/${T}_nw8.log; exit 1; }
VLP_HIP_LIB=build_exp/nw4/libvlp_hip.so timeout -k 10 200 python tools/conv_bench.py --ops fwd,dgrad,dgrad_bn,dgrad_relu --layers l2,l3,l4 --iters 10 > gpurun_out/${T}_nw4.log 2>&1 || { echo NW4 FAILED; tail -3 gpurun_out/${T}_nw4.log; exit 1; }
VLP_HIP_LIB=build_exp/stamp/libvlp_hip.so timeout -k 10 120 python tools/conv_bench.py --ops fwd,dgrad_bn --layers l2,l4 --iters 2 > gpurun_out/${T}_stamp.log 2>&1 || { echo STAMP FAILED; tail -3 gpurun_out/${T}_stamp.log; exit 1; }
for f in gpurun_out/${T}_nw8.log gpurun_out/${T}_nw4.log; do echo "== $f"; grep "TF/s" $f; done
grep "win TW" gpurun_out/${T}_stamp.log | sort | uniq -c | sort -rn | head -8
