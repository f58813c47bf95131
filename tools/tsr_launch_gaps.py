"""Per-launch timing of the TSR expansion launches in a rocprofv3 kernel trace
(tools/ktrace.sh output of a `run_one.py tsr ...` run):

    python tools/tsr_launch_gaps.py <run_kernel_trace.csv> [--rep N]

A launch is k_exp_domain -> k_exp_rows -> k_expand_reduce -> k_dl on one queue.
Prints, over the launches of the last mine (split at k_pairs): the launch count,
the summed kernel time, the summed in-launch gaps (kernel to kernel on the
queue), the launch span distribution, and the GPU's busy time (the union of all
kernel intervals) against the mine's span: the idle share is the host's.
"""
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            short = name.replace("(anonymous namespace)", "").split("(")[0].split("::")[-1].replace("void ", "")
            q = r.get("Queue_Id") or r.get("Stream_Id") or "0"
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short, q))
    rows.sort()
    mines, cur = [], []
    for r in rows:
        if r[2] == "k_pairs" and cur and any(x[2] == "k_exp_rows" for x in cur):
            mines.append(cur)
            cur = []
        cur.append(r)
    if cur:
        mines.append(cur)
    m = mines[-1]
    order = ["k_exp_domain", "k_exp_rows", "k_expand_reduce", "k_dl"]
    open_l = {}  # queue -> kernels of its current launch
    launches = []
    for s, e, n, q in m:
        if n not in order:
            continue
        if n == "k_exp_domain":
            open_l[q] = [(s, e, n)]
        elif q in open_l:
            open_l[q].append((s, e, n))
            if n == "k_dl":
                launches.append(open_l.pop(q))
    busy, last_end = 0, 0
    for s, e, n, q in m:
        if e <= last_end:
            continue
        busy += e - max(s, last_end)
        last_end = e
    span = (m[-1][1] - m[0][0]) / 1e6
    spans = [(l[-1][1] - l[0][0]) / 1e3 for l in launches]
    kern = [sum(e - s for s, e, _ in l) / 1e3 for l in launches]
    gaps = [sum(max(0, l[i][0] - l[i - 1][1]) for i in range(1, len(l))) / 1e3 for l in launches]
    per = {n: [] for n in order}
    for l in launches:
        for s, e, n in l:
            per[n].append((e - s) / 1e3)
    print("mine span %.1f ms, GPU busy (union) %.1f ms (%.0f %%), %d launches" % (span, busy / 1e6, 100 * busy / 1e6 / span,
                                                                                 len(launches)))
    if not launches:
        return
    q = lambda v, p: sorted(v)[int(p * (len(v) - 1))]
    print("launch span us: median %.1f p10 %.1f p90 %.1f p99 %.1f sum %.1f ms" % (
        statistics.median(spans), q(spans, 0.1), q(spans, 0.9), q(spans, 0.99), sum(spans) / 1e3))
    print("kernels per launch us: median %.1f sum %.1f ms; in-launch gaps: median %.1f sum %.1f ms" % (
        statistics.median(kern), sum(kern) / 1e3, statistics.median(gaps), sum(gaps) / 1e3))
    for n in order:
        v = per[n]
        print("  %-16s median %6.1f us  p90 %6.1f  sum %7.1f ms" % (n, statistics.median(v), q(v, 0.9), sum(v) / 1e3))
    small = [sp for sp, l in zip(spans, launches)]
    print("launches with span < 50 us: %d, 50-200: %d, > 200: %d" % (
        sum(1 for x in small if x < 50), sum(1 for x in small if 50 <= x < 200), sum(1 for x in small if x >= 200)))


if __name__ == "__main__":
    main()
