cd $GRAFT_REPO_ROOT
r() { echo "== $*"; env "$@" timeout -k 10 120 python -u tools/run_one.py spade $SHAPE --support $SUP --reps 3 > gpurun_out/t15.log 2>&1; echo "rc=$?"; python3 -c "
import json
for l in open('gpurun_out/t15.log'):
    if l.startswith('{'):
        d=json.loads(l); print(round(d['wall_ms'],1), [(k['name'],k['ms']) for k in d['kernels'][:4]])
"; }
SHAPE=sign SUP=0.015 r FSM_X=1
SHAPE=sign SUP=0.015 r FSM_LIB_PATH=spark-fsm_amd/build/var/base/libfsm.so
SHAPE=bible SUP=0.004 r FSM_X=1
SHAPE=bible SUP=0.004 r FSM_LIB_PATH=spark-fsm_amd/build/var/base/libfsm.so
SHAPE=sign SUP=0.015 r FSM_HOST_TRACE=1
grep "fsm host" gpurun_out/t15.log | tail -1
