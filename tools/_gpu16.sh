cd $GRAFT_REPO_ROOT
FULL=1 bash tools/_gpu6.sh
FSM_LIB_PATH=spark-fsm_amd/build/var/hostdbg/libfsm.so FSM_HOST_PROF=gpurun_out/sign.prof timeout -k 10 120 python -u tools/run_one.py spade sign --support 0.015 --reps 2 > gpurun_out/t16_sign.log 2>&1
echo "sign prof rc=$?"
python3 tools/host_prof_report.py gpurun_out/sign.prof spark-fsm_amd/build/var/hostdbg/libfsm.so --lines > gpurun_out/sign_prof_lines.txt 2>&1
python3 tools/host_prof_report.py gpurun_out/sign.prof spark-fsm_amd/build/var/hostdbg/libfsm.so > gpurun_out/sign_prof.txt 2>&1
head -30 gpurun_out/sign_prof.txt
