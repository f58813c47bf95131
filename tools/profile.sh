#!/bin/bash
# GPU-box profiling recipe for bench.py (run from the repo root under gpurun):
#   1. rocprofv3 --kernel-trace --stats of a 3-step SPADE bench  -> gpurun_out/prof/ (stats + trace)
#   2. the same for one c4 TSR mine (tools/run_one.py)            -> gpurun_out/prof_tsr/ (stats only)
#   3. one --pmc pass per counter group (FETCH_SIZE, WRITE_SIZE) over ONE SPADE step
#   4. tools/pmc_summary.py folds the passes into gpurun_out/pmc_latest.json
# Raw rocprof output goes to /tmp (TSR traces are large); only summaries come back.
# Each GPU step has its own time limit; the script stops at the first failure.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT/prof" "$OUT/prof_tsr"
export TMPDIR=/tmp
BENCH="$R/bench.py --no-cpu-baseline --no-tsr"
cd /tmp
rm -rf /tmp/p_spade /tmp/p_tsr /tmp/p_fetch /tmp/p_write
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_spade -o run -- \
    python3 $BENCH --steps 3 --warmup 1 > "$OUT/prof_bench.json"
find /tmp/p_spade -name "*.csv" -exec cp {} "$OUT/prof/" \;
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_tsr -o run -- \
    python3 "$R/tools/run_one.py" tsr kosarak --D 990002 --k 1000 --minconf 0.5 > "$OUT/prof_tsr/run.json"
find /tmp/p_tsr -name "*kernel_stats.csv" -exec cp {} "$OUT/prof_tsr/" \;
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/p_fetch -o run -- \
    python3 $BENCH --steps 1 --warmup 0 > /dev/null
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/p_write -o run -- \
    python3 $BENCH --steps 1 --warmup 0 > /dev/null
cd "$R"
python3 tools/pmc_summary.py "$OUT/pmc_latest.json" /tmp/p_fetch /tmp/p_write
echo "profile done"
