#!/bin/bash
# One GPU call that gathers a round's evidence, each step under its own limit, stopping
# at the first failure: the full GPU test suite, D1M variants + c4 (tools/gpu_check.sh),
# the SQ / LDS / FETCH / WRITE passes (SQ=1), the rocprof stats + PMC evidence
# (tools/round_evidence.sh) and the driver's bench command.
#   bash tools/gpu_round.sh            (SKIP_TESTS=1, SKIP_BENCH=1, SKIP_EV=1 to skip steps)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/round_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/round_tests.log; exit 1; }
  tail -2 gpurun_out/round_tests.log
fi
TESTS="" D1M_ENVS="${D1M_ENVS:--}" SQ=${SQ:-1} bash tools/gpu_check.sh || exit 1
if [ "${SKIP_EV:-0}" != 1 ]; then
  OUT=gpurun_out/ev timeout -k 10 900 bash tools/round_evidence.sh > gpurun_out/ev.log 2>&1 || { echo EVFAIL; tail -20 gpurun_out/ev.log; exit 1; }
  tail -1 gpurun_out/ev.log
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCHFAIL; tail -20 gpurun_out/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print('bench', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'])"
fi
exit 0
