# kernel trace of one c4 TSR mine (per-dispatch durations and grids of the expansion kernels)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt -o run -- python3 $R/tools/run_one.py tsr kosarak --D 990002 > $R/gpurun_out/t4_run.log 2>&1
echo "rocprof rc=$?"
f=$(find /tmp/kt -name "*kernel_trace.csv" | head -1)
python3 - "$f" > $R/gpurun_out/t4_trace.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
by = collections.defaultdict(list)
for r in rows:
    import re
    m = re.search(r"\b(k0?_\w+)", r["Kernel_Name"])
    name = m.group(1) if m else r["Kernel_Name"][:30]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    g = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
    gy = int(r.get("Grid_Size_Y", 1) or 1)
    by[name].append((d, g, gy, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for name, v in sorted(by.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
    ds = sorted(x[0] for x in v)
    n = len(ds)
    print("%-22s n=%6d tot=%9.1f ms avg=%7.1f us p10=%6.1f p50=%6.1f p90=%6.1f p99=%7.1f max=%8.1f" % (
        name, n, sum(ds) / 1000, sum(ds) / n, ds[n // 10], ds[n // 2], ds[9 * n // 10], ds[99 * n // 100], ds[-1]))
ex = by.get("k_expand_bm", [])
if ex:
    # duration vs grid (blocks = Grid_Size_X / block threads)
    bins = collections.defaultdict(list)
    for d, g, gy, s, e in ex:
        b = g // 512
        k = 1 if b <= 64 else (2 if b <= 256 else (3 if b <= 1024 else 4))
        bins[k].append(d)
    for k in sorted(bins):
        ds = sorted(bins[k]); n = len(ds)
        print("  blocks bin %d: n=%d avg %.1f us p50 %.1f p90 %.1f tot %.1f ms" % (k, n, sum(ds)/n, ds[n//2], ds[9*n//10], sum(ds)/1000))
    # gaps between consecutive expansion kernels (host time per launch)
    ex.sort(key=lambda x: x[3])
    gaps = sorted((ex[i+1][3] - ex[i][4]) / 1000.0 for i in range(len(ex) - 1))
    n = len(gaps)
    print("  gap between k_expand_bm launches: avg %.1f us p50 %.1f p90 %.1f" % (sum(gaps)/n, gaps[n//2], gaps[9*n//10]))
    print("  first start -> last end: %.1f ms" % ((ex[-1][4] - ex[0][3]) / 1e6))
print(list(rows[0].keys()))
PY
cat $R/gpurun_out/t4_trace.txt
gzip -c "$f" > $R/gpurun_out/t4_kernel_trace.csv.gz
