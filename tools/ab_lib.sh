#!/bin/bash
# A/B of the in-tree libfsm.so against a variant build (tools/build_variant.sh) on one config:
#   bash tools/ab_lib.sh VARIANT_SO run_one.py args...
V=$1; shift
for rep in 1 2; do
  for lib in "" "$V"; do
    FSM_LIB_PATH=$lib timeout -k 10 120 python tools/run_one.py "$@" 2>/dev/null | python3 -c "
import json,sys
ws=[json.loads(l)['wall_ms'] for l in sys.stdin if l.startswith('{')]
print('${lib:-in-tree}', sorted(round(w,2) for w in ws))" || exit 1
  done
done
