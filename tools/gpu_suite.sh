#!/bin/bash
# The whole GPU test suite under gpurun, one process, with a heartbeat file so that a long
# (not hung) test is not taken for a silent run; each test has its own time limit.
#   bash tools/gpu_suite.sh [pytest -k expr]
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
( while true; do sleep 50; date +%s >> "$R/gpurun_out/heartbeat.txt"; done ) &
HB=$!
K=()
[ -n "$1" ] && K=(-k "$1")
timeout -k 10 1000 python -u -m pytest -v -m gpu --timeout 240 --timeout-method thread --durations=40 "${K[@]}" tests \
    > "$R/gpurun_out/suite.log" 2>&1
rc=$?
kill $HB
tail -3 "$R/gpurun_out/suite.log"
exit $rc
