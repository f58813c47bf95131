#!/bin/bash
# c4 TSR timing over libfsm variants (build/variants/*/libfsm.so, default lib if none)
# and environment settings: one JSON line each in gpurun_out/tsr_sweep.jsonl
#   bash tools/tsr_sweep.sh "FSM_TSR_GRID=128,8,512 FSM_TSR_SPB=48;FSM_TSR_GRID=64,8,512 ..."
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
OUT=$R/gpurun_out/tsr_sweep.jsonl
: > "$OUT"
IFS=';' read -r -a SETS <<< "${1:-FSM_TSR_GRID=128,8,512}"
LIBS=$(ls "$R"/build/variants/*/libfsm.so 2>/dev/null || echo "$R/spark-fsm_amd/spark_fsm_amd/libfsm.so")
for so in $LIBS; do
  for g in "${SETS[@]}"; do
    v=$(basename "$(dirname "$so")")
    env FSM_LIB_PATH=$so $g timeout -k 10 100 python3 "$R/tools/run_one.py" tsr kosarak --D 990002 \
        --k 1000 --minconf 0.5 > /tmp/tsr_sweep.log 2>&1
    python3 - "$v" "$g" >> "$OUT" <<'PY'
import json, sys
l = [x for x in open("/tmp/tsr_sweep.log") if x.startswith("{")][-1]
d = json.loads(l)
print(json.dumps({"variant": sys.argv[1], "grid": sys.argv[2], "wall_ms": round(d["wall_ms"]),
                  "final_minsup": d["meta"]["final_minsup"],
                  "kernels": {k["name"]: k["ms"] for k in d["kernels"][:3]}}))
PY
    tail -1 "$OUT"
  done
done
