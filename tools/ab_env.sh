#!/bin/bash
# A/B of one environment knob on the D1M bench (no CPU legs): bash tools/ab_env.sh VAR v1 v2 [...]
VAR=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    env "$VAR=$v" timeout -k 10 100 python bench.py --no-cpu-baseline --no-tsr --no-c2 --steps 20 --warmup 5 \
        > gpurun_out/ab.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$VAR=$v', round(d['ms_per_step'],3))"
  done
done
