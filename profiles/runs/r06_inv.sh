set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
W="python -u tests/race_worker.py bn conv2 0"
timeout -k 10 150 $W > gpurun_out/r06_inv_def.txt 2>&1 || exit 2
timeout -k 10 150 env DCUE_LEGACY_ORDERS=1 $W > gpurun_out/r06_inv_leg_cur.txt 2>&1 || exit 3
timeout -k 10 150 env DCUE_LEGACY_ORDERS=1 DCUE_HIP_LIB=$R/alt_lib/libdcue_hip.so $W > gpurun_out/r06_inv_leg_prev.txt 2>&1 || exit 4
timeout -k 10 150 env DCUE_LEGACY_ORDERS=1 $W > gpurun_out/r06_inv_leg_cur2.txt 2>&1 || exit 5
timeout -k 10 150 env DCUE_LEGACY_ORDERS=1 DCUE_HIP_LIB=$R/alt_lib/libdcue_hip.so python -u tests/race_worker.py bn wgrad_2,dgrad_2 5000 > gpurun_out/r06_inv_leg_prev_test.txt 2>&1 || exit 6
