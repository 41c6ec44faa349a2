# Fused-stem / loss check: op tests, then the stem micro-benchmark at the bench shape.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r3}
SEL=${SEL:-tests/test_gpu_stem.py tests/test_gpu_streams.py tests/test_gpu_head.py}
timeout -k 10 600 python -u -m pytest $SEL -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_stem_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|per rank|worst" gpurun_out/${TAG}_stem_tests.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TEST STEP rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python tools/stem_bench.py > gpurun_out/${TAG}_stem_bench.json 2>&1 || { echo STEM BENCH FAILED; tail -20 gpurun_out/${TAG}_stem_bench.json; exit 3; }
cat gpurun_out/${TAG}_stem_bench.json
