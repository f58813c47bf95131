set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_parity_gpu.py -k "tsr" > gpurun_out/t1_tsr.log 2>&1
rc=$?; echo "tsr tests rc=$rc"; tail -5 gpurun_out/t1_tsr.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/run_one.py tsr kosarak --D 990002 --verbose > gpurun_out/t1_c4.log 2>&1
rc=$?; echo "c4 rc=$rc"; tail -12 gpurun_out/t1_c4.log | cut -c1-1500
