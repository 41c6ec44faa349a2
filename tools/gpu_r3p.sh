# round-3 check: stem kernels (tests + bench), NesT per-kernel bench, text/NesT/fullres GPU tests
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${T:-r3p}
timeout -k 10 300 python -u -m pytest tests/test_gpu_stem.py -m gpu -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_stem.log 2>&1
rc=$?; grep -E "PASSED|FAILED|stem fused|passed|failed" gpurun_out/${T}_stem.log | cut -c1-300 | tail -30
if [ $rc -gt 1 ]; then echo "STEM TESTS rc=$rc"; exit $rc; fi
timeout -k 10 200 python tools/stem_bench.py > gpurun_out/${T}_stem_bench.json 2>&1 || { echo STEM BENCH FAILED; tail -5 gpurun_out/${T}_stem_bench.json; exit 3; }
tail -1 gpurun_out/${T}_stem_bench.json
timeout -k 10 300 python tools/nest_gemm_bench.py --out gpurun_out/${T}_gemm.json > gpurun_out/${T}_gemm.log 2>&1 || { echo NEST BENCH FAILED; exit 3; }
timeout -k 10 900 python -u -m pytest ${SEL:-tests/test_gpu_bert_ops.py tests/test_gpu_nest.py tests/test_gpu_streams.py tests/test_gpu_fullres.py} -m gpu -v -s --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|NesT bf16|bs=16|passed|failed" gpurun_out/${T}_tests.log | cut -c1-500 | tail -60
exit $rc
