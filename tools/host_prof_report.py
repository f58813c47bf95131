"""Symbolize a FSM_HOST_PROF sample file (csrc/host_prof.cpp) against libfsm.so.

    python tools/host_prof_report.py gpurun_out/sign.prof [path/to/libfsm.so] [--lines]

Prints the share of samples per object, then per libfsm function (or source
line with --lines).  The library must be the one the samples came from, built
with host line tables (make HOSTDBG="-Xarch_host -gline-tables-only").
"""
import collections
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    lines = "--lines" in sys.argv
    prof = args[0]
    lib = args[1] if len(args) > 1 else os.path.join(ROOT, "spark-fsm_amd", "spark_fsm_amd", "libfsm.so")
    per_obj = collections.Counter()
    fsm_off = collections.Counter()
    other = collections.defaultdict(collections.Counter)
    total = 0
    for ln in open(prof):
        if ln.startswith("#"):
            continue
        n, obj, off = ln.split()
        n = int(n)
        total += n
        per_obj[os.path.basename(obj)] += n
        if obj.endswith("libfsm.so"):
            fsm_off[off] += n
        elif os.path.exists(obj):
            other[obj][off] += n
    print(f"samples {total}")
    for o, n in per_obj.most_common(12):
        print(f"{100.0 * n / total:6.1f}%  {o}")
    offs = list(fsm_off)
    sym = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-symbolizer", f"--obj={lib}", "--inlining=false",
                          "--demangle"] + offs, capture_output=True, text=True).stdout.strip().split("\n\n")
    agg = collections.Counter()
    for off, s in zip(offs, sym):
        parts = s.strip().split("\n")
        fn = parts[0][:110]
        key = (fn + "  " + os.path.basename(parts[1])) if lines and len(parts) > 1 else fn
        agg[key] += fsm_off[off]
    print("--- libfsm")
    for k, n in agg.most_common(40):
        print(f"{100.0 * n / total:6.1f}%  {k}")
    for obj, cnt in other.items():
        offs = list(cnt)
        out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-symbolizer", f"--obj={obj}", "--inlining=false",
                              "--demangle"] + offs, capture_output=True, text=True).stdout.strip().split("\n\n")
        a2 = collections.Counter()
        for off, s in zip(offs, out):
            a2[s.strip().split("\n")[0][:90]] += cnt[off]
        print("---", os.path.basename(obj))
        for k, n in a2.most_common(8):
            print(f"{100.0 * n / total:6.1f}%  {k}")


if __name__ == "__main__":
    main()
