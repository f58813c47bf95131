# bench TSR leg (every launch of the warmup mine timed) beside rocprof's kernel stats of one c4 mine
set -o pipefail
mkdir -p gpurun_out/ev2
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline --no-c2 --steps 5 --warmup 2 > gpurun_out/ev2/bench_nocpu.json || exit 1
cd /tmp && rm -rf /tmp/e_tsr
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/e_tsr -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/run_one.py" tsr kosarak --D 990002 --k 1000 --minconf 0.5 > "$GRAFT_REPO_ROOT/gpurun_out/ev2/tsr_c4_run.json" || exit 1
cp "$(find /tmp/e_tsr -name '*kernel_stats.csv' | head -1)" "$GRAFT_REPO_ROOT/gpurun_out/ev2/tsr_c4_kernel_stats.csv"
