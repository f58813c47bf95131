#!/bin/bash
# PMC passes over one TSR mine (tools/run_one.py tsr ...), one rocprofv3 --pmc
# run per counter group; output gpurun_out/tsr_pmc/<pass>/ + the counter list.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/tsr_pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${*:-"tsr kosarak --D 200000 --k 1000 --minconf 0.5"}
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
pass() {
    local name=$1; shift
    timeout -s KILL ${PMC_LIMIT:-120} rocprofv3 --pmc "$@" --output-format csv -d "/tmp/tp_$name" -o run -- \
        python3 "$R/tools/run_one.py" $ARGS > "$OUT/$name.log" 2>&1
    python3 - "/tmp/tp_$name" "$OUT/$name.json" <<'PY'
import csv, glob, json, sys, collections
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    agg[k]["_dispatches_x_counters"] += 1
json.dump(agg, open(sys.argv[2], "w"), indent=1)
PY
}
PASSES=${TSR_PMC_PASSES:-"issue mem atom"}
for p in $PASSES; do
  case $p in
    issue) pass issue SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU ;;
    mem) pass mem SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_FLAT TCC_HIT_sum TCC_MISS_sum ;;
    atom) pass atom TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum ;;
    lds) pass lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM ;;
    fetch) pass fetch FETCH_SIZE ;;
    write) pass write WRITE_SIZE ;;
  esac
done
echo "tsr pmc done"
