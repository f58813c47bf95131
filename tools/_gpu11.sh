cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/micro/np_read.py > gpurun_out/t11_np.log 2>&1; echo "np rc=$?"; tail -7 gpurun_out/t11_np.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_k0_gpu.py tests/test_parity_gpu.py -k "k0 or emit or spade or root or count" > gpurun_out/t11_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t11_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-tsr --steps 20 --warmup 5 > gpurun_out/t11_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/t11_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print(d['ms_per_step'], e['ms_flatten'], e['ms_upload'], [(k['name'],k['ms']) for k in e['kernels'][:8]])"
FSM_EMIT_PATH=chunk timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-tsr --steps 20 --warmup 5 > gpurun_out/t11_bench2.log 2>&1
rc=$?; echo "bench chunk rc=$rc"; tail -1 gpurun_out/t11_bench2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print(d['ms_per_step'], [(k['name'],k['ms']) for k in e['kernels'][:8]])"
