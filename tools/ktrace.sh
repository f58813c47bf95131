#!/bin/bash
# rocprofv3 kernel trace + stats (CSV) of tools/run_one.py, copied to
# gpurun_out/ktrace/<name>/ (trace kept only when small).
#   bash tools/ktrace.sh <name> [run_one.py args...]
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
NAME=$1; shift
ARGS=${*:-"spade quest --D 1000000 --support 0.001 --reps 3"}
OUT=$R/gpurun_out/ktrace/$NAME
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
rm -rf /tmp/kt_$NAME
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$NAME -o run -- \
    python3 "$R/tools/run_one.py" $ARGS > "$OUT/run.log" 2>&1
for f in $(find /tmp/kt_$NAME -name "*.csv"); do
    sz=$(stat -c %s "$f")
    if [ "$sz" -lt 20000000 ]; then cp "$f" "$OUT/"; fi
done
ls "$OUT"
