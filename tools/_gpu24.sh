cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c5prof
for shp in "bible 0.004" "sign 0.015"; do
  set -- $shp
  rm -rf /tmp/p_$1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_$1 -o run -- python3 $R/tools/run_one.py spade $1 --support $2 --reps 2 > $R/gpurun_out/c5prof/$1.json || exit 1
  find /tmp/p_$1 -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/c5prof/$1_kernel_stats.csv \;
done
echo done
