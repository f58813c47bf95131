# D1M per-batch host phases (FSM_HOST_TRACE=2)
set -o pipefail
mkdir -p gpurun_out
FSM_HOST_TRACE=2 timeout -k 10 200 python tools/run_one.py spade quest --D 1000000 --support 0.001 --reps 4 > gpurun_out/d1m_batches.log 2>&1 || exit 1
grep "fsm batch" gpurun_out/d1m_batches.log | tail -5
