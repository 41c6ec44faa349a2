# conv micro-benchmarks (all layers) + focused PMC passes on layer1 / layer3 shapes
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-cv}
timeout -k 10 200 python tools/conv_bench.py > gpurun_out/${T}_bench.log 2>&1 || { echo CB FAILED; tail -20 gpurun_out/${T}_bench.log; exit 1; }
cat gpurun_out/${T}_bench.log | tail -14
for L in l1 l3; do
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU --output-format csv -d gpurun_out/${T}_pmc -o ${L}_p1 -- python tools/conv_bench.py --layers $L --iters 3 > gpurun_out/${T}_p1.log 2>&1 || { echo PMC1 FAILED; tail -20 gpurun_out/${T}_p1.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/${T}_pmc -o ${L}_p2 -- python tools/conv_bench.py --layers $L --iters 3 > gpurun_out/${T}_p2.log 2>&1 || { echo PMC2 FAILED; tail -20 gpurun_out/${T}_p2.log; exit 1; }
done
echo done
