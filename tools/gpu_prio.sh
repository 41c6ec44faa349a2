# main-stream priority A/B (interleaved), bench only
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-r3m}
for P in 0 -1 0 -1; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-loss-check --pcie-steps 0 --main-priority $P > gpurun_out/${T}_bench_p$P.log 2>&1 || { echo BENCH FAILED; tail -10 gpurun_out/${T}_bench_p$P.log; exit 1; }
  echo "prio $P $(tail -1 gpurun_out/${T}_bench_p$P.log | cut -c80-200)"
done
