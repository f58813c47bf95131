#!/bin/bash
# TSR per-launch grid sweep (GPU box): one Kosarak-shaped prefix, each grid
# setting under its own time limit; stops at the first failure.
D=${1:-30000}
set -e -o pipefail
mkdir -p gpurun_out
for g in 128,8,512 64,8,512 256,8,512 128,4,512 128,16,512 128,32,512 128,8,128 128,8,1024; do
  echo "=== grid $g" | tee -a gpurun_out/sweep.log
  FSM_TSR_GRID=$g timeout -k 10 120 python tools/run_one.py tsr kosarak --D $D --verbose 2>&1 | grep -E "fsm tsr\] exp|wall_ms" | cut -c1-200 | tee -a gpurun_out/sweep.log
done
