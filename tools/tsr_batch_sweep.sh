#!/bin/bash
# TSR c4 (Kosarak-shaped 990,002 sequences, k = 1000, minconf 0.5) at several
# rules-per-launch batch sizes; one JSON line per run in gpurun_out/tsr_batch.jsonl
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
for b in ${*:-32 64 128}; do
    FSM_TSR_BATCH=$b timeout -k 10 150 python3 "$R/tools/run_one.py" tsr kosarak --D 990002 --k 1000 --minconf 0.5 \
        | sed "s/^/{\"batch\": $b, \"run\": /; s/\$/}/" >> "$R/gpurun_out/tsr_batch.jsonl"
done
