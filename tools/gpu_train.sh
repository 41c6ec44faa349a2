# src/train.py + data-module GPU checks: the new GPU tests, a bench line with the
# prefetched PCIe-inclusive rates, and a 10-step src/train.py run at configs[1].
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r1t}
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_model.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
timeout -k 10 400 python vision-language-pretraining-for-bone-tumor-detection_amd/src/train.py experiment=pretrain/pretrain_resnet34_tinybert_mi355x > gpurun_out/${TAG}_train.log 2>&1 || { echo TRAIN FAILED; tail -20 gpurun_out/${TAG}_train.log; exit 1; }
tail -4 gpurun_out/${TAG}_train.log
