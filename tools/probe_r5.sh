set -o pipefail
mkdir -p gpurun_out
FSM_HOST_TRACE=1 timeout -k 10 200 python tools/run_one.py spade quest --D 1000000 --support 0.001 --reps 5 > gpurun_out/d1m_host.log 2>&1 || exit 1
C4_ENVS="- FSM_TSR_BATCH=512+FSM_TSR_SPEC=6,1024 FSM_TSR_BATCH=448+FSM_TSR_SPEC=6,896 FSM_TSR_BATCH=512+FSM_TSR_SPEC=8,1024" REPS=3 bash tools/c4_ab.sh > gpurun_out/c4ab.txt || exit 1
C4_ARGS="--head 5000" C4_ENVS="- FSM_TSR_BATCH=512+FSM_TSR_SPEC=6,1024 FSM_TSR_BATCH=448+FSM_TSR_SPEC=6,896 FSM_TSR_BATCH=512+FSM_TSR_SPEC=8,1024" REPS=3 bash tools/c4_ab.sh >> gpurun_out/c4ab.txt || exit 1
cat gpurun_out/c4ab.txt
