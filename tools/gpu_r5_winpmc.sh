# SQ counters of the ping-pong window kernel (layers 2 / 4, forward and BN data gradient)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-r5w2}
SQ1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU"
SQ2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM"
run_pmc() {
  timeout -s KILL 120 rocprofv3 --pmc $2 --output-format csv -d gpurun_out/${T}_pmc_$1 -o p -- python tools/conv_bench.py $3 --iters 3 > gpurun_out/${T}_pmc_$1.log 2>&1 || { echo PMC $1 FAILED; tail -5 gpurun_out/${T}_pmc_$1.log; return 1; }
}
run_pmc sq1 "$SQ1" "--ops fwd,dgrad_bn --layers l2,l4" && run_pmc sq2 "$SQ2" "--ops fwd,dgrad_bn --layers l2,l4" || exit 1
for f in gpurun_out/${T}_pmc_*/; do echo "== $f"; PMC_FILTER=winpp python tools/pmc_summary.py $(find $f -name "*counter_collection.csv") | grep -v "^ *$" | head -80; done > gpurun_out/${T}_pmc_summary.txt
cat gpurun_out/${T}_pmc_summary.txt | head -100
