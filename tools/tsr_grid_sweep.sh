#!/bin/bash
# TSR per-launch grid sweep (GPU box): FSM_TSR_GRID="expand,collect,dl" settings
# on one Kosarak-shaped DB size, each run under its own time limit.
#   tools/tsr_grid_sweep.sh <D> <grid> [<grid> ...]
D=${1:-30000}
shift
set -e -o pipefail
mkdir -p gpurun_out
for g in "$@"; do
  echo "=== D=$D grid $g" | tee -a gpurun_out/sweep.log
  FSM_TSR_GRID=$g timeout -k 10 120 python tools/run_one.py tsr kosarak --D $D --verbose 2>&1 | grep -E "fsm tsr\] exp|wall_ms" | cut -c1-200 | tee -a gpurun_out/sweep.log
done
