#!/bin/bash
# TSR speculation-threshold sweep (GPU box): FSM_TSR_SPEC_FRAC values on one
# Kosarak-shaped DB size, each run under its own time limit.
#   tools/tsr_frac_sweep.sh <D> <frac> [<frac> ...]
D=${1:-100000}
shift
set -e -o pipefail
mkdir -p gpurun_out
for f in "$@"; do
  echo "=== D=$D frac $f" | tee -a gpurun_out/frac_sweep.log
  FSM_TSR_SPEC_FRAC=$f timeout -k 10 150 python tools/run_one.py tsr kosarak --D $D --verbose 2>&1 | grep -E "fsm tsr\] (exp|child)|wall_ms" | cut -c1-200 | tee -a gpurun_out/frac_sweep.log
done
