set -o pipefail
cd $GRAFT_REPO_ROOT
B="python bench.py --steps 20 --warmup 5 --modes inbatch --no-eval --no-cpu-baseline --no-f32-probe --host-trace"
timeout -k 10 200 env DCUE_SIDE_THREAD=0 $B > gpurun_out/r06_q_st0.json 2> gpurun_out/r06_q_st0.err || exit 3
timeout -k 10 200 env DCUE_FROZEN_ROWS=0 $B > gpurun_out/r06_q_fr0.json 2> gpurun_out/r06_q_fr0.err || exit 4
timeout -k 10 200 env DCUE_XQ_WAIT=event $B > gpurun_out/r06_q_xq.json 2> gpurun_out/r06_q_xq.err || exit 5
timeout -k 10 200 $B > gpurun_out/r06_q_base.json 2> gpurun_out/r06_q_base.err || exit 6
