# D1M A/B: k_emit1's long-run launch skipped when no class exceeds 64 members; emit / count parity subset
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "emit_paths or count_paths or fullsize_digest or wide or quest_vs_oracle" > gpurun_out/t.log 2>&1 || { tail -20 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
bash tools/ab_lib.sh spark-fsm_amd/build/var/prev/libfsm.so spade quest --D 1000000 --support 0.001 --reps 12 > gpurun_out/ab_d1m.txt || exit 1
bash tools/ab_lib.sh spark-fsm_amd/build/var/prev/libfsm.so spade quest --D 1000000 --support 0.001 --reps 12 >> gpurun_out/ab_d1m.txt || exit 1
bash tools/ab_lib.sh spark-fsm_amd/build/var/prev/libfsm.so spade sign --support 0.015 --reps 5 >> gpurun_out/ab_d1m.txt || exit 1
cat gpurun_out/ab_d1m.txt
