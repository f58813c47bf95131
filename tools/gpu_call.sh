#!/bin/bash
# tools/gpu_call.sh OUT TIMEOUT CMD: one gpurun call, re-queued only while no GPU slot is free
# (exit 3: nothing ran, nothing charged); any other outcome ends it.  Output in OUT.
out=$1; lim=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$@" > "$out" 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  sleep 120
done
echo "EXIT $rc" >> "$out"
