cd $GRAFT_REPO_ROOT
r() { echo "== $*"; env "$@" timeout -k 10 120 python -u tools/run_one.py spade $SHAPE --support $SUP --reps 3 > gpurun_out/t18.log 2>&1; echo "rc=$?"; python3 -c "
import json
for l in open('gpurun_out/t18.log'):
    if l.startswith('{'):
        d=json.loads(l); s=d['stats']; print(round(d['wall_ms'],1), 'mine', round(s['ms_mine'],1), 'lat', round(s['ms_lattice'],1), 'out', round(s['ms_output'],1), 'wait', round(s['ms_gpu_wait'],1), [(k['name'],k['ms']) for k in d['kernels'][:3]])
"; grep "fsm host" gpurun_out/t18.log | tail -2; }
SHAPE=sign SUP=0.015 r FSM_HOST_TRACE=1
SHAPE=bible SUP=0.004 r FSM_HOST_TRACE=1
