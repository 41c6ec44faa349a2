cd $GRAFT_REPO_ROOT
for v in 3 1 2; do
  echo "v=$v: $(VLP_GEMM_VARIANT=$v timeout -k 10 120 python tools/conv_bench.py --ops fwd,wgrad --layers l3,l4 --gemm 2>&1 | grep -E '^(wgrad|fwd|gemm)' | tr '\n' ' ')"
done
