#!/bin/bash
# A/B of any tools/run_one.py run (its args in RUN), alternating libs (tools/ab_d1m.sh argument forms),
# 2 rounds; prints the wall ms of every mine after the first of each process
#   RUN="spade sign --support 0.015 --reps 4" bash tools/ab_run.sh - spark-fsm_amd/build/var/prev/libfsm.so
for rep in 1 2; do
  for arg in "$@"; do
    lib=${arg%%@*}; [ "$lib" = "-" ] && lib=""
    ev=""; [[ "$arg" == *@* ]] && ev=${arg#*@}
    env $ev FSM_KCLOCK=0 FSM_LIB_PATH=$lib timeout -k 10 200 python tools/run_one.py $RUN 2>/dev/null | python3 -c "
import json,sys
ws=[json.loads(l)['wall_ms'] for l in sys.stdin if l.startswith('{')]
print('$arg', [round(w,1) for w in ws[1:]])" || exit 1
  done
done
