#!/bin/bash
# One GPU session of the build loop: a parity subset (TESTS, pytest -k), D1M mines and
# the c4 TSR mine (tools/run_one.py), each step under its own time limit; stops at
# the first failure.  SQ=1 adds the SQ / LDS / FETCH / WRITE counter passes over one
# D1M mine (tools/sq_profile.sh).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_parity_gpu.py \
    tests/test_fullsize_gpu.py -k "$TESTS" > gpurun_out/c_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/c_tests.log; exit 1; }
  tail -2 gpurun_out/c_tests.log
fi
summ() { python - "$1" <<'PY'
import json,sys,statistics
rows=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')]
rows=rows[1:] if len(rows) > 1 else rows
st=rows[-1]['stats']
print(' wall %.3f f1 %.3f f2 %.3f lat %.3f pat %d joins %d rules %d' % (statistics.median(r['wall_ms'] for r in rows),
  statistics.median(r['stats']['ms_f1'] for r in rows), statistics.median(r['stats']['ms_f2'] for r in rows),
  statistics.median(r['stats']['ms_lattice'] for r in rows), st['patterns'], st['joins'], st['rules']))
print('  ', [(k['name'],k['ms']) for k in rows[-1]['kernels']])
PY
}
# D1M_ENVS: space-separated variants, each "-" (defaults) or comma-separated VAR=value settings
for V in ${D1M_ENVS:--}; do
  E=""; [ "$V" != "-" ] && E=$(echo "$V" | tr ',' ' ')
  env $E timeout -k 10 120 python tools/run_one.py spade quest --D 1000000 --support 0.001 --reps 8 > gpurun_out/c_d1m.log 2>&1 || exit 1
  echo "D1M [$V]"; summ gpurun_out/c_d1m.log
done
if [ "${C4:-1}" = 1 ]; then
  timeout -k 10 180 python tools/run_one.py tsr kosarak --D 990002 --k 1000 --minconf 0.5 --reps 2 > gpurun_out/c_c4.log 2>&1 || exit 1
  echo "C4"; summ gpurun_out/c_c4.log
fi
if [ "${SQ:-0}" = 1 ]; then
  timeout -k 10 500 bash tools/sq_profile.sh > gpurun_out/c_sq.log 2>&1 || exit 1
  echo "SQ profile"; tail -2 gpurun_out/c_sq.log
fi
exit 0
