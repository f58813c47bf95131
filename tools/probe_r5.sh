# host sampling profile of SIGN-shaped mines (line-table build of libfsm.so); THP state of the box
set -o pipefail
mkdir -p gpurun_out
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag > gpurun_out/thp.txt 2>&1 || true
FSM_LIB_PATH=spark-fsm_amd/build/var/lines/libfsm.so FSM_HOST_PROF=gpurun_out/sign.prof FSM_HOST_TRACE=1 timeout -k 10 120 python tools/run_one.py spade sign --support 0.015 --reps 4 > gpurun_out/signprof.log 2>&1 || exit 1
grep -c . gpurun_out/sign.prof
