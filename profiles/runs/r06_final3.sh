set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_f3_tests.log 2>&1 || exit 4
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_f3_bench.json 2> gpurun_out/r06_f3_bench.err || exit 6
PHASE=inbatch_cold bash profiles/gpu_only_timeline.sh r06_i_cold || exit 5
PHASE=inbatch bash profiles/gpu_only_timeline.sh r06_i_warm || exit 6
bash profiles/phase_prof.sh r06_i inbatch 20 --modes inbatch --no-f32-probe > /dev/null || exit 7
bash profiles/phase_prof.sh r06_i text 20 --modes text --no-f32-probe > /dev/null || exit 8
find $GRAFT_REPO_ROOT/gpurun_out/prof_r06_i -name "*kernel_trace.csv" -delete
