# c4: in-tree libfsm.so (result intake on the host pool) against the serial-intake build; TSR parity subset
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "tsr_c4 or tsr_expansion or batch_sizes" > gpurun_out/tsrtests.log 2>&1 || { tail -20 gpurun_out/tsrtests.log; exit 1; }
tail -1 gpurun_out/tsrtests.log
bash tools/ab_lib.sh spark-fsm_amd/build/var/serintake/libfsm.so tsr kosarak --D 990002 --k 1000 --minconf 0.5 --reps 3 > gpurun_out/ab_intake.txt || exit 1
bash tools/ab_lib.sh spark-fsm_amd/build/var/serintake/libfsm.so tsr kosarak --D 990002 --k 1000 --minconf 0.5 --reps 3 >> gpurun_out/ab_intake.txt || exit 1
cat gpurun_out/ab_intake.txt
