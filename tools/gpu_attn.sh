# NesT attention micro-bench + PMC passes on the level-2 shape
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-at}
timeout -k 10 200 python tools/nest_attn_bench.py > gpurun_out/${T}_bench.log 2>&1 || { echo AB FAILED; tail -20 gpurun_out/${T}_bench.log; exit 1; }
grep level gpurun_out/${T}_bench.log
if [ -n "$PMC" ]; then
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU --output-format csv -d gpurun_out/${T}_pmc -o p1 -- python tools/nest_attn_bench.py --levels 2 --iters 1 > gpurun_out/${T}_p1.log 2>&1 || { echo PMC1 FAILED; tail -5 gpurun_out/${T}_p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM --output-format csv -d gpurun_out/${T}_pmc -o p2 -- python tools/nest_attn_bench.py --levels 2 --iters 1 > gpurun_out/${T}_p2.log 2>&1 || { echo PMC2 FAILED; tail -5 gpurun_out/${T}_p2.log; exit 1; }
python - <<'PY'
import csv, glob, collections, os
T = os.environ.get("T", "at")
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob(f"gpurun_out/{T}_pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        vals[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    if "nest" in k:
        print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
fi
