cd $GRAFT_REPO_ROOT
timeout -k 10 60 tools/micro/first_touch
b() { echo "== $*"; env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-tsr --steps 20 --warmup 5 > gpurun_out/t12_bench.log 2>&1; echo "rc=$?"; tail -1 gpurun_out/t12_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print(round(d['ms_per_step'],3), 'up', round(e['ms_upload'],2), 'fl', round(e['ms_flatten'],2), [(k['name'],round(k['ms'],3)) for k in e['kernels'][:4]])"; }
for v in r64c128 r128c128 r128c192; do b FSM_LIB_PATH=spark-fsm_amd/build/var/$v/libfsm.so; done
