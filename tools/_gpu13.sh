cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_parity_gpu.py -k "count or emit or spade_quest or golden" > gpurun_out/t13_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t13_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
b() { echo "== $*"; env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-tsr --steps 20 --warmup 5 > gpurun_out/t13_bench.log 2>&1; echo "rc=$?"; tail -1 gpurun_out/t13_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print(round(d['ms_per_step'],3), 'up', round(e['ms_upload'],2), 'fl', round(e['ms_flatten'],2), [(k['name'],round(k['ms'],3)) for k in e['kernels'][:5]])"; }
b FSM_NONE=1
b FSM_COUNT_KERNEL=thread
b FSM_NONE=1
