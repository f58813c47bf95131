# D1M: k_emit2 wave range (build variants) and emit grid cap (FSM_EMIT_GRID) sweeps
set -o pipefail
mkdir -p gpurun_out
bash tools/ab_lib.sh spark-fsm_amd/build/var/r64/libfsm.so spade quest --D 1000000 --support 0.001 --reps 10 > gpurun_out/ab_e2.txt || exit 1
bash tools/ab_lib.sh spark-fsm_amd/build/var/r256/libfsm.so spade quest --D 1000000 --support 0.001 --reps 10 >> gpurun_out/ab_e2.txt || exit 1
for g in 16384 32768 131072 262144; do
  FSM_EMIT_GRID=$g timeout -k 10 120 python tools/run_one.py spade quest --D 1000000 --support 0.001 --reps 10 2>/dev/null | python3 -c "
import json,sys
ws=sorted(round(json.loads(l)['wall_ms'],2) for l in sys.stdin if l.startswith('{'))
print('grid $g', ws)" >> gpurun_out/ab_e2.txt || exit 1
done
cat gpurun_out/ab_e2.txt
