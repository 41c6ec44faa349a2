# Interleaved bench A/B over host-side schedule switches (environment variables read
# by vlp_amd at import): ARMS="A:VAR=0,VAR2=0 B:" (name:comma-separated assignments)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-envab}
for r in $(seq 1 ${BENCH_REPS:-2}); do
  for arm in $ARMS; do
    name=${arm%%:*}; vars=${arm#*:}
    env $(echo $vars | tr ',' ' ') timeout -k 10 300 python bench.py --no-cpu-baseline --no-loss-check --pcie-steps 0 $BENCH_ARGS \
      > gpurun_out/${TAG}_${name}_$r.log 2>&1 || { echo BENCH FAILED $name; tail -5 gpurun_out/${TAG}_${name}_$r.log; exit 1; }
    echo "$name#$r $(tail -1 gpurun_out/${TAG}_${name}_$r.log | cut -c1-140)"
  done
done
