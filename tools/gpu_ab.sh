cd $GRAFT_REPO_ROOT
for d in 0 1 6 7; do
  echo "dbg=$d $(VLP_GEMM_DBG=$d timeout -k 10 120 python tools/conv_bench.py --ops fwd,dgrad --layers l1,l3 2>&1 | grep -E '^(fwd|dgrad)' | tr '\n' ' ')"
done
