cd $GRAFT_REPO_ROOT
run() { echo "=== $*"; env "$@" timeout -k 10 120 python -u tools/run_one.py tsr kosarak --D 990002 --verbose > gpurun_out/t20_run.log 2>&1; echo "rc=$?"; grep -E "expansions [0-9]+ in" gpurun_out/t20_run.log | cut -c1-300; tail -1 gpurun_out/t20_run.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('wall', round(d['wall_ms']), 'minsup', d['meta']['final_minsup'], 'rules', d['stats']['rules'], 'exp', d['stats']['expansions'], d['kernels'][:4])"; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_parity_gpu.py -k "tsr" > gpurun_out/t20_tests.log 2>&1
rc=$?; echo "tsr tests rc=$rc"; tail -3 gpurun_out/t20_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_fullsize_gpu.py -k "tsr" > gpurun_out/t20_full.log 2>&1
rc=$?; echo "fullsize tsr rc=$rc"; tail -3 gpurun_out/t20_full.log
if [ $rc -ne 0 ]; then exit $rc; fi
run FSM_X=1
run FSM_TSR_STREAMS=1
run FSM_X=2
