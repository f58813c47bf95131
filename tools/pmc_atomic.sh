#!/bin/bash
# Atomic-path and issue counters over ONE mine (tools/run_one.py), one rocprofv3
# --pmc run per pass (gfx950 slot limits), each under its own time limit.
# Output: gpurun_out/atom/<pass>/ and gpurun_out/atom/summary.json.
#   bash tools/pmc_atomic.sh [run_one.py args...]
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/atom
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${*:-"spade quest --D 1000000 --support 0.001"}
cd /tmp
pass() {
    local name=$1; shift
    timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "/tmp/atom_$name" -o run -- \
        python3 "$R/tools/run_one.py" $ARGS > "$OUT/$name.log" 2>&1
}
pass atomics TCC_EA0_ATOMIC_sum TCC_ATOMIC_sum
pass issue SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD
cd "$R"
python3 tools/pmc_summary.py "$OUT/summary.json" /tmp/atom_atomics /tmp/atom_issue > /dev/null
echo "atomic profile done"
