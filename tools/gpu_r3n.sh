# stem forward packed-stats A/B, then NesT-Small profile (bench, rocprofv3 stats, PMC traffic)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python tools/stem_bench.py > gpurun_out/r3h_stem_bench.json 2>&1 || { echo STEM BENCH FAILED; tail -5 gpurun_out/r3h_stem_bench.json; exit 3; }
tail -1 gpurun_out/r3h_stem_bench.json
VLP_HIP_LIB=$PWD/build_exp/stem_pk0/libvlp_hip.so timeout -k 10 200 python tools/stem_bench.py > gpurun_out/r3h_stem_bench_pk0.json 2>&1 || { echo STEM BENCH2 FAILED; exit 3; }
tail -1 gpurun_out/r3h_stem_bench_pk0.json
TAG=r3n bash tools/gpu_nest_prof.sh
