#!/bin/bash
# A/B of the in-tree libfsm.so against variant builds on the D1M bench (no CPU legs),
# alternating, 3 rounds: bash tools/ab_d1m.sh VARIANT_SO [VARIANT_SO ...]
for rep in 1 2 3; do
  for lib in "" "$@"; do
    FSM_LIB_PATH=$lib timeout -k 10 100 python bench.py --no-cpu-baseline --no-tsr --no-c2 --steps 20 --warmup 5 \
        > gpurun_out/ab.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('${lib:-in-tree}', round(d['ms_per_step'],3))"
  done
done
