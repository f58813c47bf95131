# c4 at the wide batches: per-launch grids (FSM_TSR_GRID = expand blocks per slot, reduce blocks, k_dl blocks)
set -o pipefail
mkdir -p gpurun_out
C4_ENVS="- FSM_TSR_GRID=4096,8,1024 FSM_TSR_GRID=4096,8,2048 FSM_TSR_GRID=4096,4,1024 FSM_TSR_GRID=4096,8,256 -" REPS=3 bash tools/c4_ab.sh > gpurun_out/c4grid.txt || exit 1
cat gpurun_out/c4grid.txt
