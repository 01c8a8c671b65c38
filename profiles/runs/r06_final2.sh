set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
bash profiles/pmc_traffic.sh r06_h inbatch || exit 2
bash profiles/pmc_traffic.sh r06_h text || exit 3
DCUE_W1K=1 bash profiles/pmc_traffic.sh r06_h_w1k inbatch || exit 4
PHASE=inbatch_cold bash profiles/gpu_only_timeline.sh r06_h_cold || exit 5
PHASE=inbatch bash profiles/gpu_only_timeline.sh r06_h_warm || exit 6
bash profiles/phase_prof.sh r06_h inbatch 20 --modes inbatch --no-f32-probe > /dev/null || exit 7
bash profiles/phase_prof.sh r06_h text 20 --modes text --no-f32-probe > /dev/null || exit 8
find $R/gpurun_out/prof_r06_h -name "*kernel_trace.csv" -delete
