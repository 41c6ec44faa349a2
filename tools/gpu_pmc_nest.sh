cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python tools/nest_attn_bench.py --levels 2 --iters 3 > gpurun_out/r4x_nab.log 2>&1 || { echo NAB FAILED; tail -5 gpurun_out/r4x_nab.log; exit 1; }
cat gpurun_out/r4x_nab.log | grep -v amdgpu
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU --output-format csv -d gpurun_out/r4x_pmc -o p1 -- python tools/nest_attn_bench.py --levels 2 --iters 1 > gpurun_out/r4x_p1.log 2>&1 || { echo PMC1 FAILED; tail -5 gpurun_out/r4x_p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_VALU_TRANS_F32 --output-format csv -d gpurun_out/r4x_pmc -o p2 -- python tools/nest_attn_bench.py --levels 2 --iters 1 > gpurun_out/r4x_p2.log 2>&1 || { echo PMC2 FAILED; tail -5 gpurun_out/r4x_p2.log; exit 1; }
echo done
