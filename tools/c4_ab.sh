#!/bin/bash
# c4 TSR mine under env variants, same box: C4_ENVS = space-separated variants, each "-"
# (defaults) or '+'-separated VAR=value settings; one summary line per variant.  C4_ARGS:
# extra run_one.py arguments (--head 5000: the bench's CPU-baseline prefix).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for V in ${C4_ENVS:--}; do
  E=""; [ "$V" != "-" ] && E=$(echo "$V" | tr '+' ' ')
  env $E timeout -k 10 200 python tools/run_one.py tsr kosarak --D 990002 --k 1000 --minconf 0.5 --reps ${REPS:-3} $C4_ARGS > gpurun_out/c4_ab.log 2>&1 || exit 1
  python - "$V" gpurun_out/c4_ab.log <<'PY'
import json, statistics, sys
rows = [json.loads(l) for l in open(sys.argv[2]) if l.startswith('{')]
rows = rows[1:] if len(rows) > 1 else rows
st = rows[-1]['stats']
print(sys.argv[1], 'wall %.1f' % statistics.median(r['wall_ms'] for r in rows), 'rules %d exp %d launches %d'
      % (st['rules'], st['expansions'], st['count_launches']),
      [(k['name'], round(k['ms'], 1)) for k in rows[-1]['kernels']][:5])
PY
done
