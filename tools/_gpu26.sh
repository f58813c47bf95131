cd $GRAFT_REPO_ROOT
rm -f gpurun_out/steps.log
bash tools/gpu_steps.sh "600|gputests|python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread" "240|bench|python -u bench.py > gpurun_out/bench.json" "400|profile|bash tools/profile.sh" "400|configs|python -u tools/bench_configs.py --gpu-only > gpurun_out/configs_gpu.jsonl"
