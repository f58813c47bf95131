#!/bin/bash
# verbose sharded SPADE run (N ranks sharing this GPU over gloo): the per-rank
# first-level plan lines ("[fsm] rank r: ... heavy (split)") into gpurun_out/shard_trace.log
#   bash tools/shard_trace.sh N shape D support
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=$1; shift
cd "$R" && mkdir -p gpurun_out
export FSM_WORKER_VERBOSE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 WORLD_SIZE=$N
pids=()
for r in $(seq 0 $((N - 1))); do
    RANK=$r LOCAL_RANK=$r timeout -k 5 110 python tests/dist_worker.py spade_digest gpurun_out/trace_r$r.json "$@" \
        > gpurun_out/trace_r$r.log 2>&1 &
    pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
grep -h "\[fsm\] rank" gpurun_out/trace_r*.log > gpurun_out/shard_trace.log || true
cat gpurun_out/shard_trace.log
exit $rc
