#!/bin/bash
# The round's GPU evidence (profiles/rN): under gpurun, from the repo root:
#   1. rocprofv3 --kernel-trace --stats over a 4-step SPADE D1M bench -> stats CSV + the bench line
#   2. the same for one c4 TSR mine (tools/run_one.py)             -> stats CSV
#   3. one --pmc pass per counter (FETCH_SIZE, WRITE_SIZE) over a bench run of a warmup step and
#      one step, summarised over the last mine (the steady state: no DB build) -> pmc.json
# Each GPU step has its own time limit; the script stops at the first failure.
#   OUT=gpurun_out/ev bash tools/round_evidence.sh
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${OUT:-gpurun_out/ev}
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="$R/bench.py --no-cpu-baseline --no-tsr --no-c2"
cd /tmp
rm -rf /tmp/e_spade /tmp/e_tsr /tmp/e_fetch /tmp/e_write
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/e_spade -o run -- \
    python3 $BENCH --steps 4 --warmup 2 > "$OUT/bench_prof.json"
cp "$(find /tmp/e_spade -name '*kernel_stats.csv' | head -1)" "$OUT/spade_d1m_kernel_stats.csv"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/e_tsr -o run -- \
    python3 "$R/tools/run_one.py" tsr kosarak --D 990002 --k 1000 --minconf 0.5 > "$OUT/tsr_c4_run.json"
cp "$(find /tmp/e_tsr -name '*kernel_stats.csv' | head -1)" "$OUT/tsr_c4_kernel_stats.csv"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/e_fetch -o run -- \
    python3 $BENCH --steps 1 --warmup 1 > /dev/null
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/e_write -o run -- \
    python3 $BENCH --steps 1 --warmup 1 > /dev/null
cd "$R"
python3 tools/pmc_summary.py --last-mine "$OUT/pmc.json" /tmp/e_fetch /tmp/e_write > /dev/null
echo "evidence done"
