# D1M: k_emit2 wave range / record capacity (build variants) against the in-tree build
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_e2.txt
for v in r64 r256 cap128; do
  echo "== $v" >> gpurun_out/ab_e2.txt
  bash tools/ab_lib.sh spark-fsm_amd/build/var/$v/libfsm.so spade quest --D 1000000 --support 0.001 --reps 10 >> gpurun_out/ab_e2.txt || exit 1
done
cat gpurun_out/ab_e2.txt
