# PMC passes over the plain GEMM micro-benchmarks (kk / kmn / mnmn) under one GEMM variant
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-pg}
export VLP_GEMM_VARIANT=${V:-5}
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VMEM --output-format csv -d gpurun_out/${T} -o p1 -- python tools/conv_bench.py --layers "" --gemm --iters 3 > gpurun_out/${T}_p1.log 2>&1 || { echo P1 FAILED; tail -5 gpurun_out/${T}_p1.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/${T} -o p2 -- python tools/conv_bench.py --layers "" --gemm --iters 3 > gpurun_out/${T}_p2.log 2>&1 || { echo P2 FAILED; tail -5 gpurun_out/${T}_p2.log; exit 1; }
echo done
