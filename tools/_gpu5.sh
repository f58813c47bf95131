cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/run_one.py tsr kosarak --D 990002 --verbose > gpurun_out/t5_c4.log 2>&1
echo "c4 rc=$?"
grep -E "fsm tsr" gpurun_out/t5_c4.log | cut -c1-400
tail -1 gpurun_out/t5_c4.log | cut -c1-3000
