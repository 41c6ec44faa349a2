cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py::test_conv_dgrad_relu_ds_fold tests/test_gpu_ops.py::test_conv_dgrad_relu2_three_sums tests/test_gpu_streams.py::test_ds_fold_matches_separate_downsample_bf16 tests/test_gpu_model.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4f_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r4f_tests.log; exit 1; }
tail -1 gpurun_out/r4f_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-loss-check --pcie-steps 0 --kernel-report gpurun_out/r4f_kreport.json > gpurun_out/r4f_bench.log 2>&1 || { echo BENCH FAILED; tail -5 gpurun_out/r4f_bench.log; exit 1; }
tail -1 gpurun_out/r4f_bench.log | cut -c1-200
timeout -k 10 400 python tools/fusion_bench.py --out gpurun_out/r4f_fusion_bench.json > gpurun_out/r4f_fusion.log 2>&1 || { echo FUSION FAILED; tail -5 gpurun_out/r4f_fusion.log; exit 1; }
tail -1 gpurun_out/r4f_fusion.log | cut -c1-300
timeout -k 10 500 python bench.py --image-model nest_small --steps 10 --warmup 3 --no-cpu-baseline --no-loss-check --pcie-steps 0 --kernel-report gpurun_out/r4f_nest_kreport.json > gpurun_out/r4f_nest_bench.log 2>&1 || { echo NEST FAILED; tail -5 gpurun_out/r4f_nest_bench.log; exit 1; }
tail -1 gpurun_out/r4f_nest_bench.log | cut -c1-300
