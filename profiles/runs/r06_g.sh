set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_text.py > gpurun_out/r06_g_tests.log 2>&1 || exit 1
bash profiles/pmc_traffic.sh r06_g inbatch || exit 2
bash profiles/pmc_traffic.sh r06_g text || exit 3
PHASE=inbatch_cold bash profiles/gpu_only_timeline.sh r06_g_cold || exit 4
