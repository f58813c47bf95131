cd $GRAFT_REPO_ROOT
run() { echo "=== $*"; env "$@" timeout -k 10 120 python -u tools/run_one.py tsr kosarak --D 990002 --verbose 2>&1 | grep -E "expansions|wall_ms" | sed -e 's/"stats".*"kernels"/"kernels"/' | cut -c1-600; }
run FSM_TSR_SPB=64
run FSM_TSR_SPB=16 FSM_TSR_GRID=256,8,512 FSM_TSR_PART_MB=256
run FSM_TSR_SPB=32 FSM_TSR_GRID=128,8,512 FSM_TSR_PART_MB=128
run FSM_TSR_SPB=8 FSM_TSR_GRID=1024,8,512 FSM_TSR_PART_MB=1024
