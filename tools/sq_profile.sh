#!/bin/bash
# SQ / LDS / TCC counter passes over D1M mines (tools/run_one.py, the last of 2 summarised), one
# rocprofv3 --pmc run per counter group (gfx950 slot limits: 8 SQ, 4 TCC per
# pass), each under its own time limit.  Output: gpurun_out/sq/<pass>/ and
# gpurun_out/sq/summary.json (tools/pmc_summary.py).
#   bash tools/sq_profile.sh [extra run_one.py args...]
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sq
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${*:-"spade quest --D 1000000 --support 0.001 --reps 2"}
cd /tmp
pass() {
    local name=$1; shift
    timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
        python3 "$R/tools/run_one.py" $ARGS > "$OUT/$name.log" 2>&1
}
pass issue SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
pass mix SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS
pass fetch FETCH_SIZE
pass write WRITE_SIZE
cd "$R"
python3 tools/pmc_summary.py --last-mine "$OUT/summary.json" "$OUT/issue" "$OUT/mix" "$OUT/fetch" "$OUT/write" > /dev/null
echo "sq profile done"
