# D1M: in-tree libfsm.so against the previous build (root F2 records through mapped memory)
set -o pipefail
mkdir -p gpurun_out
bash tools/ab_lib.sh spark-fsm_amd/build/var/prev/libfsm.so spade quest --D 1000000 --support 0.001 --reps 12 > gpurun_out/ab_d1m.txt || exit 1
bash tools/ab_lib.sh spark-fsm_amd/build/var/prev/libfsm.so spade quest --D 1000000 --support 0.001 --reps 12 >> gpurun_out/ab_d1m.txt || exit 1
cat gpurun_out/ab_d1m.txt
