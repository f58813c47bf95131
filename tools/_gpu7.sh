cd $GRAFT_REPO_ROOT
run() { echo "=== $*"; env "$@" timeout -k 10 120 python -u tools/run_one.py tsr kosarak --D 990002 --verbose > gpurun_out/t7_run.log 2>&1; echo "rc=$?"; grep -E "expansions [0-9]+ in" gpurun_out/t7_run.log | cut -c1-200; tail -1 gpurun_out/t7_run.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('wall', round(d['wall_ms']), 'minsup', d['meta']['final_minsup'], 'rules', d['stats']['rules'], [(k['name'],round(k['ms'])) for k in d['kernels'][:4]])"; }
run FSM_TSR_SPB=128
run FSM_TSR_SPB=256
run FSM_TSR_PART_MB=64
run FSM_TSR_PART_MB=16
run FSM_TSR_SPB=256 FSM_TSR_PART_MB=16
run FSM_TSR_BATCH=128
TSR_PMC_PASSES="issue lds" bash tools/tsr_pmc.sh tsr kosarak --D 400000 --k 1000 --minconf 0.5
