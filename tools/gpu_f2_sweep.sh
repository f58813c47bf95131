#!/bin/bash
# Root F2 / DB-direct root sweep on one MI355X: the SPADE parity subset first, then
# D1M mines (tools/run_one.py) over FSM_ROOT_DB x FSM_F2_PASSES x FSM_F2_BLOCKS.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_parity_gpu.py \
  -k "${TESTS:-root_f2 or spade_quest_vs_oracle or sharded_spade_two_ranks or emit_paths or spade_golden or spade_random or long_sequence}" \
  > gpurun_out/t1.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
for RD in ${ROOTDB:-1 0}; do
for P in ${PASSES:-1 3}; do
  for B in ${BLOCKS:-1024}; do
    FSM_ROOT_DB=$RD FSM_F2_PASSES=$P FSM_F2_BLOCKS=$B timeout -k 10 120 python tools/run_one.py spade quest --D 1000000 --support 0.001 --reps 8 > gpurun_out/r$RD.p$P.b$B.log 2>&1 || exit 1
    echo "ROOTDB=$RD P=$P B=$B"; python - gpurun_out/r$RD.p$P.b$B.log <<'PY'
import json,sys,statistics
rows=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][2:]
st=rows[-1]['stats']
print(' wall %.3f f1 %.3f f2 %.3f lat %.3f pat %d joins %d' % (statistics.median(r['wall_ms'] for r in rows),
  statistics.median(r['stats']['ms_f1'] for r in rows), statistics.median(r['stats']['ms_f2'] for r in rows),
  statistics.median(r['stats']['ms_lattice'] for r in rows), st['patterns'], st['joins']))
print('  ', [(k['name'],k['ms']) for k in rows[-1]['kernels']])
PY
  done
done
done
