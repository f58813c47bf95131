cd $GRAFT_REPO_ROOT
run() { echo "=== $*"; env "$@" timeout -k 10 120 python -u tools/run_one.py tsr kosarak --D 990002 --verbose > gpurun_out/t27_run.log 2>&1; echo "rc=$?"; grep -E "expansions [0-9]+ in" gpurun_out/t27_run.log | cut -c1-240; tail -1 gpurun_out/t27_run.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('wall', round(d['wall_ms']), 'minsup', d['meta']['final_minsup'], 'rules', d['stats']['rules'])"; }
run FSM_X=1
run FSM_TSR_BATCH=128
run FSM_TSR_BATCH=192
run FSM_TSR_SPEC=4,128
run FSM_TSR_SPEC=3,256
run FSM_X=1
