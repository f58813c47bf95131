"""Fold rocprofv3 --pmc CSV passes into profiles/pmc_latest.json.

Usage (each pass is its own rocprofv3 run of a bench command, see tools/round_evidence.sh):
    python tools/pmc_summary.py [--last-mine] OUT.json DIR_FETCH DIR_WRITE [more dirs...]

--last-mine keeps only the dispatches from the last k_f1 on (the last SPADE mine of
the run: a bench run of a warmup step and one step then reports the steady state,
without the DB build's one-time kernels and fills).

For every kernel (named as libfsm's fsm_get_kernel_stats names it) the JSON has
the counter totals over the step's dispatches, in bytes (rocprofv3 reports
FETCH_SIZE / WRITE_SIZE in KiB), plus the dispatch count.  bench.py reads it
for `roofline.traffic` = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md,
HBM [CDNA4]: gfx950 FETCH_SIZE counts half of the bytes of wide reads).
"""
import csv
import glob
import json
import os
import re
import sys


def kernel_name(demangled):
    m = re.search(r"\b(k0?_\w+)(<([^>]*)>)?", demangled)
    if not m:
        return demangled.split("(")[0][:40]
    base, targs = m.group(1), m.group(3) or ""
    if base == "k_emit":
        return "k_emit<write>" if "true" in targs else "k_emit<count>"
    if base in ("k_emit1", "k_emit2"):  # the emit kernels: fsm_get_kernel_stats times them as "k_emit"
        return "k_emit"
    if base in ("k_count2", "k_sparse_keys"):  # the window / sparse counts: timed as "k_count"
        return "k_count"
    if base == "k_f2_plan_db":  # the DB-direct root's F2 plan: timed as "k_f2_plan"
        return "k_f2_plan"
    if base == "k_f2_tri":  # the unordered-pair F2 key enumeration: timed as "k_f2_keys"
        return "k_f2_keys"
    return base


def read_dir(d):
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(path) as f:
            rows.extend(csv.DictReader(f))
    return rows


def last_mine(rows):
    """the rows of the dispatches from the last k_f1 on (Dispatch_Id order)"""
    ids = [int(r.get("Dispatch_Id", 0) or 0) for r in rows if kernel_name(r.get("Kernel_Name", "")) == "k_f1"]
    if not ids:
        return rows
    first = max(ids)
    return [r for r in rows if int(r.get("Dispatch_Id", 0) or 0) >= first]


def main():
    args = sys.argv[1:]
    only_last = "--last-mine" in args
    args = [a for a in args if a != "--last-mine"]
    out, dirs = args[0], args[1:]
    kernels = {}
    for d in dirs:
        rows = read_dir(d)
        if only_last:
            rows = last_mine(rows)
        for r in rows:
            name = kernel_name(r.get("Kernel_Name", ""))
            ctr = r.get("Counter_Name", "")
            val = float(r.get("Counter_Value", 0) or 0)
            k = kernels.setdefault(name, {"dispatches": {}})
            if ctr in ("FETCH_SIZE", "WRITE_SIZE"):
                k[ctr + "_bytes_per_step"] = k.get(ctr + "_bytes_per_step", 0) + int(val * 1024)
            else:
                k[ctr] = k.get(ctr, 0) + val
            k["dispatches"][r.get("Dispatch_Id", "")] = 1
    for k in kernels.values():
        k["dispatches"] = len(k["dispatches"])
    with open(out, "w") as f:
        json.dump({"source": "rocprofv3 --pmc, one pass per counter" + (", the last mine of the run" if only_last
                                                                             else "") + ": " + " ".join(dirs),
                   "note": "bytes summed over the step's dispatches; FETCH_SIZE uncorrected here",
                   "kernels": kernels}, f, indent=1, sort_keys=True)
    print(json.dumps({n: {c: v for c, v in k.items() if c != "dispatches"} for n, k in kernels.items()})[:2000])


if __name__ == "__main__":
    main()
