#!/bin/bash
# GPU-box profiling recipe for bench.py (run from the repo root under gpurun):
#   1. rocprofv3 --kernel-trace --stats of a 3-step bench   -> gpurun_out/prof/
#   2. one --pmc pass per counter group (FETCH_SIZE, WRITE_SIZE) over ONE step
#   3. tools/pmc_summary.py folds the passes into gpurun_out/pmc_latest.json
# Each GPU step has its own time limit; the script stops at the first failure.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="$R/bench.py --no-cpu-baseline"
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 $BENCH --steps 3 --warmup 1 > "$OUT/prof_bench.json"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 $BENCH --steps 1 --warmup 0 > /dev/null
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 $BENCH --steps 1 --warmup 0 > /dev/null
cd "$R"
python3 tools/pmc_summary.py "$OUT/pmc_latest.json" "$OUT/pmc_fetch" "$OUT/pmc_write"
