# A/B of environment switches on the bench (interleaved, same box): ENVS="A=1 B=0;C=1" (';'-separated arms)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-ab}
IFS=';' read -ra ARMS <<< "${ENVS}"
for rep in 1 2; do
  i=0
  for arm in "" "${ARMS[@]}"; do
    env $arm timeout -k 10 200 python bench.py --no-cpu-baseline --no-loss-check --pcie-steps 0 --steps ${STEPS:-20} > gpurun_out/${TAG}_${rep}_${i}.log 2>&1 || { echo "ARM [$arm] FAILED"; tail -20 gpurun_out/${TAG}_${rep}_${i}.log; exit 1; }
    echo "rep $rep arm [$arm]: $(tail -1 gpurun_out/${TAG}_${rep}_${i}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    i=$((i+1))
  done
done
