#!/bin/bash
# A/B of TSR c4 mine time (990,002 Kosarak-shaped sequences, k = 1000, minconf 0.5), alternating libs
# (same argument forms as tools/ab_d1m.sh), 2 rounds of 2 mines each
for rep in 1 2; do
  for arg in "$@"; do
    lib=${arg%%@*}; [ "$lib" = "-" ] && lib=""
    ev=""; [[ "$arg" == *@* ]] && ev=${arg#*@}
    env $ev FSM_LIB_PATH=$lib timeout -k 10 200 python tools/run_one.py tsr kosarak --D 990002 --k 1000 --minconf 0.5 --reps 2 \
        2>/dev/null | python3 -c "
import json,sys
ws=[json.loads(l)['wall_ms'] for l in sys.stdin if l.startswith('{')]
print('$arg', [round(w,1) for w in ws])" || exit 1
  done
done
