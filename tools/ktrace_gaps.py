"""Idle gaps between kernels in a rocprofv3 kernel trace (tools/ktrace.sh output).

    python tools/ktrace_gaps.py gpurun_out/ktrace/d1m/run_kernel_trace.csv [--mine N]

Splits the trace into mines at each launch of the kernel named by --start (default
k_f1, the first kernel of a SPADE mine), takes mine N (default: the last one), and prints every kernel in order with the
idle time before it, then the busy / idle totals: the host's share of a mine.
"""
import csv
import re
import sys


def short(name):
    name = re.sub(r"fsm::\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:40]


def main():
    path = sys.argv[1]
    pick = int(sys.argv[sys.argv.index("--mine") + 1]) if "--mine" in sys.argv else -1
    start = sys.argv[sys.argv.index("--start") + 1] if "--start" in sys.argv else "k_f1"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    mines, cur = [], []
    for r in rows:
        if cur and r[2] == start:
            mines.append(cur)
            cur = []
        cur.append(r)
    if cur:
        mines.append(cur)
    m = mines[pick]
    t0, busy, idle, prev = m[0][0], 0, 0, m[0][0]
    for s, e, n in m:
        gap = max(0, s - prev)
        idle += gap
        busy += e - s
        print("%9.3f  +%7.3f  %7.3f  %s" % ((s - t0) / 1e6, gap / 1e6, (e - s) / 1e6, n))
        prev = max(prev, e)
    print("mine %d of %d: span %.3f ms, kernels %.3f ms, idle %.3f ms, %d launches"
          % (pick if pick >= 0 else len(mines) + pick, len(mines), (prev - t0) / 1e6, busy / 1e6, idle / 1e6, len(m)))


if __name__ == "__main__":
    main()
