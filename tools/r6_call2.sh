#!/bin/bash
# round-6 probe: new in-process tests, then the W=1 lohi A/B, host-phase traces and a kernel trace of D1M
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r6
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fullsize_gpu.py \
    -k "inproc or stalled or first_claim" > $O/inproc.log 2>&1 || { tail -40 $O/inproc.log; exit 1; }
tail -3 $O/inproc.log
timeout -k 10 300 bash tools/ab_d1m.sh spark-fsm_amd/build/var/w1lohi/libfsm.so > $O/ab_lohi.txt 2>&1 || { cat $O/ab_lohi.txt; exit 1; }
cat $O/ab_lohi.txt
FSM_HOST_TRACE=2 timeout -k 10 120 python tools/run_one.py spade quest --D 1000000 --support 0.001 --reps 3 > $O/trace2.log 2>&1 || exit 1
FSM_HOST_TRACE=1 timeout -k 10 120 python tools/run_one.py spade quest --D 1000000 --support 0.001 --reps 3 > $O/trace1.log 2>&1 || exit 1
grep "fsm host" $O/trace1.log | tail -2
bash tools/ktrace.sh d1m_r6 > /dev/null 2>&1 || exit 1
cp -r gpurun_out/ktrace/d1m_r6 $O/ 2>/dev/null
echo done
