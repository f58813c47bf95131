#!/bin/bash
# TSR child-speculation sweep (GPU box): FSM_TSR_SPEC="depth,max" settings on
# one Kosarak-shaped prefix, each under its own time limit.
D=${1:-100000}
set -e -o pipefail
mkdir -p gpurun_out
for sp in 3,128 6,128 3,512 8,512 16,1024 32,2048; do
  echo "=== spec $sp" | tee -a gpurun_out/spec_sweep.log
  FSM_TSR_SPEC=$sp timeout -k 10 120 python tools/run_one.py tsr kosarak --D $D --verbose 2>&1 | grep -E "fsm tsr\] (exp|child)|wall_ms" | cut -c1-230 | tee -a gpurun_out/spec_sweep.log
done
