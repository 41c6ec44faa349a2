# r5: conv_bench timings of every GEMM family at the bench shapes, SQ counters of the
# forward ping-pong / 128x128 kernels (layers 3 / 2) and HBM bytes + SQ counters of the
# layer-1 backward kernels (rows kernels, the folded stride-2 entry, the 64x192 wgrad).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-r5p}
timeout -k 10 240 python tools/conv_bench.py --ops fwd,dgrad,dgrad_bn,dgrad_relu,wgrad --layers l2,l3,l4 --iters 10 > gpurun_out/${T}_cb_wide.log 2>&1 || { echo CB1 FAILED; tail -5 gpurun_out/${T}_cb_wide.log; exit 1; }
timeout -k 10 240 python tools/conv_bench.py --ops fwd,fwd_act,dgrad_bn_act,dgrad_relu_act,wgrad --layers l1 --iters 10 > gpurun_out/${T}_cb_l1.log 2>&1 || { echo CB2 FAILED; tail -5 gpurun_out/${T}_cb_l1.log; exit 1; }
timeout -k 10 240 python tools/conv_bench.py --ops dgrad_relu_ds,wgrad --layers l2s,l3s,l4s --iters 10 > gpurun_out/${T}_cb_s2.log 2>&1 || { echo CB3 FAILED; tail -5 gpurun_out/${T}_cb_s2.log; exit 1; }
grep -h "TF/s" gpurun_out/${T}_cb_*.log
SQ1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU"
SQ2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM"
run_pmc() {  # name, counters, conv_bench args
  timeout -s KILL 120 rocprofv3 --pmc $2 --output-format csv -d gpurun_out/${T}_pmc_$1 -o p -- python tools/conv_bench.py $3 --iters 3 > gpurun_out/${T}_pmc_$1.log 2>&1 || { echo PMC $1 FAILED; tail -5 gpurun_out/${T}_pmc_$1.log; return 1; }
}
run_pmc fwd_sq1 "$SQ1" "--ops fwd,dgrad_bn --layers l2,l3" && \
run_pmc fwd_sq2 "$SQ2" "--ops fwd,dgrad_bn --layers l2,l3" && \
run_pmc l1_sq1 "$SQ1" "--ops dgrad_bn_act,dgrad_relu_act,wgrad --layers l1" && \
run_pmc l1_sq2 "$SQ2" "--ops dgrad_bn_act,dgrad_relu_act,wgrad --layers l1" && \
run_pmc l1_fetch "FETCH_SIZE" "--ops dgrad_bn_act,dgrad_relu_act,wgrad --layers l1" && \
run_pmc l1_write "WRITE_SIZE" "--ops dgrad_bn_act,dgrad_relu_act,wgrad --layers l1" && \
run_pmc s2_fetch "FETCH_SIZE" "--ops dgrad_relu_ds --layers l2s" && \
run_pmc s2_write "WRITE_SIZE" "--ops dgrad_relu_ds --layers l2s" && \
run_pmc s2_sq1 "$SQ1" "--ops dgrad_relu_ds --layers l2s" || exit 1
for f in gpurun_out/${T}_pmc_*/; do echo "== $f"; PMC_FILTER=. python tools/pmc_summary.py $(find $f -name "*counter_collection.csv") | grep -v "^ *$" | head -60; done > gpurun_out/${T}_pmc_summary.txt
echo done
