# r5: LDS-window kernel (layers 2-4, 3x3 stride 1): op parity, block-range parity,
# conv_bench timings against the im2col GEMMs (build_exp/nowin = -DVLP_WIN=0)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-r5w}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "conv" > gpurun_out/${T}_ops.log 2>&1 || { echo OPS FAILED; tail -30 gpurun_out/${T}_ops.log; exit 1; }
tail -2 gpurun_out/${T}_ops.log
timeout -k 10 300 python tools/conv_bench.py --ops fwd,fwd_act,pass_fwd,dgrad,dgrad_bn,dgrad_relu --layers l2,l3,l4 --iters 10 > gpurun_out/${T}_cb_win.log 2>&1 || { echo CB FAILED; tail -5 gpurun_out/${T}_cb_win.log; exit 1; }
VLP_HIP_LIB=build_exp/nowin/libvlp_hip.so timeout -k 10 300 python tools/conv_bench.py --ops fwd,pass_fwd,dgrad,dgrad_bn,dgrad_relu --layers l2,l3,l4 --iters 10 > gpurun_out/${T}_cb_nowin.log 2>&1 || { echo CB0 FAILED; tail -5 gpurun_out/${T}_cb_nowin.log; exit 1; }
echo "== window"; grep -h "TF/s" gpurun_out/${T}_cb_win.log
echo "== im2col"; grep -h "TF/s" gpurun_out/${T}_cb_nowin.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_blocks.py > gpurun_out/${T}_blocks.log 2>&1 || { echo BLOCKS FAILED; tail -30 gpurun_out/${T}_blocks.log; exit 1; }
tail -2 gpurun_out/${T}_blocks.log
echo done
SQ1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU"
SQ2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM"
run_pmc() {  # name, counters, conv_bench args
  timeout -s KILL 120 rocprofv3 --pmc $2 --output-format csv -d gpurun_out/${T}_pmc_$1 -o p -- python tools/conv_bench.py $3 --iters 3 > gpurun_out/${T}_pmc_$1.log 2>&1 || { echo PMC $1 FAILED; tail -5 gpurun_out/${T}_pmc_$1.log; return 1; }
}
if [ -n "$PMC" ]; then
run_pmc win_sq1 "$SQ1" "--ops fwd,dgrad_bn --layers l2,l3" && \
run_pmc win_sq2 "$SQ2" "--ops fwd,dgrad_bn --layers l2,l3" || exit 1
for f in gpurun_out/${T}_pmc_*/; do echo "== $f"; PMC_FILTER=. python tools/pmc_summary.py $(find $f -name "*counter_collection.csv") | grep -v "^ *$" | head -40; done > gpurun_out/${T}_pmc_summary.txt
cat gpurun_out/${T}_pmc_summary.txt
fi
echo done2
