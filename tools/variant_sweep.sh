#!/bin/bash
# bench.py (no CPU baseline) against every build/variants/*/libfsm.so:
# one JSON summary line per variant in gpurun_out/variants.jsonl
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
: > "$R/gpurun_out/variants.jsonl"
for so in "$R"/build/variants/*/libfsm.so; do
    v=$(basename "$(dirname "$so")")
    FSM_LIB_PATH=$so timeout -k 10 120 python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline "$@" \
        > "$R/gpurun_out/variant_$v.json" 2> "$R/gpurun_out/variant_$v.err"
    python3 - "$v" "$R/gpurun_out/variant_$v.json" >> "$R/gpurun_out/variants.jsonl" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ks = {k["name"]: k["ms"] for k in d["extra"]["kernels"]}
print(json.dumps({"variant": sys.argv[1], "ms": round(d["ms_per_step"], 3), "k_emit": ks.get("k_emit"),
                  "lattice": round(d["extra"]["ms_lattice"], 3)}))
PY
done
cat "$R/gpurun_out/variants.jsonl"
