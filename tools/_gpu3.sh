cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_parity_gpu.py -k "tsr and not sharded" > gpurun_out/t3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t3_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run() { echo "=== $*"; env "$@" timeout -k 10 120 python -u tools/run_one.py tsr kosarak --D 990002 --verbose 2>&1 | grep -E "expansions|wall_ms" | sed -e 's/"stats".*"kernels"/"kernels"/' | cut -c1-600; }
run FSM_TSR_SPB=64
run FSM_TSR_SPB=64 FSM_TSR_PART_MB=64
run FSM_TSR_SPB=64 FSM_TSR_PART_MB=128
run FSM_TSR_SPB=256 FSM_TSR_PART_MB=32
