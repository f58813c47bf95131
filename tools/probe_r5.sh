# c4: in-tree libfsm.so (candidate buckets sorted on the host pool) against the serial-sort build
set -o pipefail
mkdir -p gpurun_out
bash tools/ab_lib.sh spark-fsm_amd/build/var/noparsort/libfsm.so tsr kosarak --D 990002 --k 1000 --minconf 0.5 --reps 3 > gpurun_out/ab_sort.txt || exit 1
bash tools/ab_lib.sh spark-fsm_amd/build/var/noparsort/libfsm.so tsr kosarak --D 990002 --k 1000 --minconf 0.5 --reps 3 --head 5000 >> gpurun_out/ab_sort.txt || exit 1
cat gpurun_out/ab_sort.txt
