# PMC passes on the weight-gradient GEMM (layer-3 shape) and the forward (reference)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-pw}
OPS=${OPS:-wgrad,fwd}
L=${L:-l3}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU --output-format csv -d gpurun_out/${T}_pmc -o p1 -- python tools/conv_bench.py --ops $OPS --layers $L --iters 3 > gpurun_out/${T}_p1.log 2>&1 || { echo PMC1 FAILED; tail -5 gpurun_out/${T}_p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM --output-format csv -d gpurun_out/${T}_pmc -o p2 -- python tools/conv_bench.py --ops $OPS --layers $L --iters 3 > gpurun_out/${T}_p2.log 2>&1 || { echo PMC2 FAILED; tail -5 gpurun_out/${T}_p2.log; exit 1; }
python tools/pmc_summary.py $(find gpurun_out/${T}_pmc -name "*counter_collection.csv")
