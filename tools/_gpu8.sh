cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_k0_gpu.py > gpurun_out/t8_k0.log 2>&1
rc=$?; echo "k0 tests rc=$rc"; tail -2 gpurun_out/t8_k0.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-tsr --steps 10 --warmup 3 > gpurun_out/t8_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/t8_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print(d['ms_per_step'], e['ms_flatten'], e['ms_upload'])"
VARIANTS="head" bash tools/_gpu6.sh
