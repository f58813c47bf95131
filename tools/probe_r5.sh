# TSR defaults (rules per launch by the pair-phase minsup) on c4 and its 5K / 50K / 250K prefixes
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/c4ab.txt
for H in 5000 50000 250000; do
  C4_ARGS="--head $H" REPS=3 bash tools/c4_ab.sh >> gpurun_out/c4ab.txt || exit 1
done
REPS=3 bash tools/c4_ab.sh >> gpurun_out/c4ab.txt || exit 1
for H in 5000 50000 990002; do
  timeout -k 10 100 python tools/run_one.py tsr kosarak --D 990002 --k 1000 --minconf 0.5 --head $H --reps 1 --verbose 2>&1 | grep -E "pair phase|child spec" | cut -c1-200 >> gpurun_out/c4ab.txt || exit 1
done
cat gpurun_out/c4ab.txt
