#!/bin/bash
# A/B of D1M bench variants (no CPU legs), alternating, 3 rounds.  Each argument is
#   LIB            a variant libfsm.so ("" or "-": the in-tree one), or
#   LIB@VAR=VALUE  the same with one environment variable set
#   bash tools/ab_d1m.sh - spark-fsm_amd/build/var/prev/libfsm.so -@FSM_KCLOCK=0
for rep in 1 2 3; do
  for arg in "$@"; do
    lib=${arg%%@*}; [ "$lib" = "-" ] && lib=""
    ev=""; [[ "$arg" == *@* ]] && ev=${arg#*@}
    env $ev FSM_LIB_PATH=$lib timeout -k 10 100 python bench.py --no-cpu-baseline --no-tsr --no-c2 --steps 20 --warmup 5 \
        > gpurun_out/ab.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$arg', round(d['ms_per_step'],3))"
  done
done
