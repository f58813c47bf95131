# D1M: root F2 row blocks (FSM_F2_BLOCKS) for the unordered-pair kernel
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/f2blocks.txt
for b in 256 512 1024 2048 512 1024; do
  FSM_F2_BLOCKS=$b timeout -k 10 120 python tools/run_one.py spade quest --D 1000000 --support 0.001 --reps 10 2>/dev/null | python3 -c "
import json,sys
rows=[json.loads(l) for l in sys.stdin if l.startswith('{')]
ws=sorted(round(r['wall_ms'],2) for r in rows)
k=[(q['name'],q['ms']) for q in rows[-1]['kernels'] if q['name'] in ('k_f2_keys','k_f2_count','k_f2_plan')]
print('blocks $b', ws[:9], k)" >> gpurun_out/f2blocks.txt || exit 1
done
cat gpurun_out/f2blocks.txt
