# One parameterised GPU A/B driver (replaces the per-experiment gpu_*.sh scripts).
# Every step runs under its own time limit; the first failure ends the script.
#
#   TAG=r4a                        prefix of every log under gpurun_out/
#   TESTS="tests/test_gpu_ops.py"  optional pytest selection (run once, default library)
#   TESTK="dgrad or stem"          optional -k expression for TESTS
#   VARIANTS="default row_nt"      libraries: default = the in-tree libvlp_hip.so,
#                                  NAME = build_exp/NAME/libvlp_hip.so (tools/build_variant.sh NAME "-D...")
#   CB_ARGS="--ops dgrad_bn,dgrad_relu"      optional tools/conv_bench.py run per variant
#   BENCH_REPS=2                   interleaved bench.py rounds over the variants (0: none)
#   BENCH_ARGS="--steps 20"        extra bench.py arguments
#   KREPORT=1                      also write a --kernel-report per bench run
#   EXTRA="python tools/x.py"      optional extra command per variant (VLP_HIP_LIB set)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-ab}
PKG=$PWD/vision-language-pretraining-for-bone-tumor-detection_amd
VARIANTS=${VARIANTS:-default}
lib_of() { if [ "$1" = default ]; then echo $PKG/vlp_amd/libvlp_hip.so; else echo $PWD/build_exp/$1/libvlp_hip.so; fi; }

if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS ${TESTK:+-k "$TESTK"} -m gpu -x -v -s --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
if [ -n "$CB_ARGS" ]; then
  for V in $VARIANTS; do
    VLP_HIP_LIB=$(lib_of $V) timeout -k 10 300 python tools/conv_bench.py $CB_ARGS > gpurun_out/${TAG}_cb_$V.log 2>&1 \
      || { echo CB FAILED $V; tail -10 gpurun_out/${TAG}_cb_$V.log; exit 1; }
    echo "== conv_bench $V"; grep -v amdgpu.ids gpurun_out/${TAG}_cb_$V.log | grep -v "^{" | head -20
  done
fi
if [ -n "$EXTRA" ]; then
  for V in $VARIANTS; do
    VLP_HIP_LIB=$(lib_of $V) timeout -k 10 300 $EXTRA > gpurun_out/${TAG}_extra_$V.log 2>&1 \
      || { echo EXTRA FAILED $V; tail -10 gpurun_out/${TAG}_extra_$V.log; exit 1; }
    echo "== extra $V"; grep -v amdgpu.ids gpurun_out/${TAG}_extra_$V.log | tail -${EXTRA_LINES:-12}
  done
fi
for r in $(seq 1 ${BENCH_REPS:-0}); do
  for V in $VARIANTS; do
    KR=""
    [ -n "$KREPORT" ] && KR="--kernel-report gpurun_out/${TAG}_kreport_${V}_$r.json"
    VLP_HIP_LIB=$(lib_of $V) timeout -k 10 300 python bench.py --no-cpu-baseline --no-loss-check --pcie-steps 0 $KR $BENCH_ARGS \
      > gpurun_out/${TAG}_bench_${V}_$r.log 2>&1 || { echo BENCH FAILED $V; tail -10 gpurun_out/${TAG}_bench_${V}_$r.log; exit 1; }
    echo "$V#$r $(tail -1 gpurun_out/${TAG}_bench_${V}_$r.log | cut -c1-160)"
  done
done
