# conv micro-benchmarks + focused PMC passes on one wgrad shape
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python tools/conv_bench.py > gpurun_out/conv_bench.log 2>&1 || { echo CB FAILED; tail -20 gpurun_out/conv_bench.log; exit 1; }
cat gpurun_out/conv_bench.log | head -20
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU --output-format csv -d gpurun_out/cpmc -o p1 -- python tools/conv_bench.py --layers l3 --iters 3 > gpurun_out/cpmc1.log 2>&1 || { echo PMC1 FAILED; tail -20 gpurun_out/cpmc1.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/cpmc -o p2 -- python tools/conv_bench.py --layers l3 --iters 3 > gpurun_out/cpmc2.log 2>&1 || { echo PMC2 FAILED; tail -20 gpurun_out/cpmc2.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr --output-format csv -d gpurun_out/cpmc -o p3 -- python tools/conv_bench.py --layers l3 --iters 3 > gpurun_out/cpmc3.log 2>&1 || { echo PMC3 FAILED; tail -20 gpurun_out/cpmc3.log; exit 1; }
echo done
