cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_parity_gpu.py -k "count or emit or wide or long or golden or timestamp or random" > gpurun_out/t23_par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/t23_par.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_fullsize_gpu.py -k "spade_fullsize" > gpurun_out/t23_full.log 2>&1
rc=$?; echo "fullsize rc=$rc"; tail -2 gpurun_out/t23_full.log
if [ $rc -ne 0 ]; then exit $rc; fi
r() { echo "== $*"; env "$@" timeout -k 10 120 python -u tools/run_one.py spade $SHAPE --support $SUP --reps 4 > gpurun_out/t23.log 2>&1; echo "rc=$?"; python3 -c "
import json
for l in open('gpurun_out/t23.log'):
    if l.startswith('{'):
        d=json.loads(l); s=d['stats']; print(round(d['wall_ms'],1), 'mine', round(s['ms_mine'],1), 'lat', round(s['ms_lattice'],1), 'out', round(s['ms_output'],1), 'wait', round(s['ms_gpu_wait'],1), [(k['name'],k['ms']) for k in d['kernels'][:4]])
"; }
SHAPE=bible SUP=0.004 r FSM_X=1
SHAPE=bible SUP=0.004 r FSM_COUNT_PATH=atomic
SHAPE=bible SUP=0.004 r FSM_LIB_PATH=spark-fsm_amd/build/var/prev/libfsm.so
SHAPE=sign SUP=0.015 r FSM_X=1
SHAPE=sign SUP=0.015 r FSM_COUNT_PATH=atomic
SHAPE=sign SUP=0.015 r FSM_LIB_PATH=spark-fsm_amd/build/var/prev/libfsm.so
