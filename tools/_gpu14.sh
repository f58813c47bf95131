cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_k0_gpu.py > gpurun_out/t14_k0.log 2>&1
rc=$?; echo "k0 tests rc=$rc"; tail -2 gpurun_out/t14_k0.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
FSM_HOST_TRACE=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-tsr --steps 20 --warmup 5 > gpurun_out/t14_bench.log 2>&1
echo "bench rc=$?"; grep "fsm k0" gpurun_out/t14_bench.log; tail -1 gpurun_out/t14_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print(round(d['ms_per_step'],3), 'up', round(e['ms_upload'],2), 'fl', round(e['ms_flatten'],2))"
done
