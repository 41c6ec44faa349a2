# stem kernel tests + micro-bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-r3e}
timeout -k 10 300 python -u -m pytest tests/test_gpu_stem.py -m gpu -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_stem.log 2>&1
rc=$?; grep -E "PASSED|FAILED|stem fused|passed|failed" gpurun_out/${T}_stem.log | cut -c1-300 | tail -30
if [ $rc -gt 1 ]; then echo "STEM TESTS rc=$rc"; exit $rc; fi
timeout -k 10 200 python tools/stem_bench.py > gpurun_out/${T}_stem_bench.json 2>&1 || { echo STEM BENCH FAILED; tail -5 gpurun_out/${T}_stem_bench.json; exit 3; }
tail -1 gpurun_out/${T}_stem_bench.json
for V in ${VARIANTS:-}; do
  VLP_HIP_LIB=$PWD/build_exp/$V/libvlp_hip.so timeout -k 10 200 python tools/stem_bench.py > gpurun_out/${T}_stem_bench_$V.json 2>&1 || { echo STEM BENCH $V FAILED; tail -5 gpurun_out/${T}_stem_bench_$V.json; exit 3; }
  echo "== $V"; tail -1 gpurun_out/${T}_stem_bench_$V.json
done
