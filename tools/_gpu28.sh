cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_fullsize_gpu.py -k "spade_fullsize" > gpurun_out/t28_full.log 2>&1
rc=$?; echo "fullsize rc=$rc"; tail -2 gpurun_out/t28_full.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_parity_gpu.py -k "emit or count or golden or keyed or sharded" > gpurun_out/t28_par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/t28_par.log
if [ $rc -ne 0 ]; then exit $rc; fi
r() { echo "== $*"; env "$@" timeout -k 10 120 python -u tools/run_one.py spade $SHAPE --support $SUP --reps 4 > gpurun_out/t28.log 2>&1; echo "rc=$?"; python3 -c "
import json
for l in open('gpurun_out/t28.log'):
    if l.startswith('{'):
        d=json.loads(l); s=d['stats']; print(round(d['wall_ms'],1), 'mine', round(s['ms_mine'],1), 'lat', round(s['ms_lattice'],1), 'out', round(s['ms_output'],1), 'wait', round(s['ms_gpu_wait'],1))
"; grep "fsm host" gpurun_out/t28.log | tail -2; }
SHAPE=sign SUP=0.015 r FSM_HOST_TRACE=1
bash tools/_gpu27.sh
