#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first step
# that times out, aborts or crashes (exit codes other than 0/1).
# usage: tools/gpu_steps.sh "<seconds>|<name>|<command>" ...
mkdir -p gpurun_out
for step in "$@"; do
  secs="${step%%|*}"; rest="${step#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $name (limit ${secs}s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc elapsed=$(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/steps.log; exit $rc; fi
done
exit 0
