cd $GRAFT_REPO_ROOT
for cfg in "FSM_K0_THREADS=1" "FSM_K0_THREADS=4" "FSM_K0_THREADS=16" "FSM_K0_CHUNK=4194304" "FSM_K0_CHUNK=262144" "FSM_K0_THREADS=8 FSM_K0_CHUNK=4194304"; do
echo "== $cfg"
env $cfg FSM_HOST_TRACE=1 timeout -k 10 100 python -u tools/run_one.py spade quest --D 1000000 --support 0.001 2>&1 | grep "fsm k0"
done
