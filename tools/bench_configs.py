"""Every BASELINE.json config on one GPU, next to the CPU restatement on the
same host (the BASELINE.md table).  bench.py is the driver's one-line contract
(config 3); this is the per-config sweep, run on the GPU box:

    python tools/bench_configs.py [--only c2,c4] [--cpu-reps 3] > gpurun_out/configs.jsonl

One JSON line per config.  GPU: median of 3 timed fsm_*_mine calls after one
warmup, DB resident in HBM.  CPU: oracle/fsm_oracle.c on the same DB and
parameters, 1 thread and every CPU of this process's share:
  SPADE c1, c2, c5: complete mines (median of --cpu-reps), lattice seconds
                    (F1 vertical build excluded, as the GPU's flatten + upload)
  SPADE c3:         a class-stride sample (every 128th first-level class mined
                    completely, 1 thread; every 8th on all CPUs): joins/s
  TSR c4:           a full run on the largest sequence prefix that completes
                    in --cpu-seconds, the GPU timed on that same prefix too.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "spark-fsm_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

CONFIGS = {
    "c1": ("spade", "quest", dict(D=10000), 0.005),
    "c2": ("spade", "quest", dict(D=100000), 0.005),
    "c3": ("spade", "quest", dict(D=1000000), 0.001),
    "c4": ("tsr", "kosarak", dict(D=990002), (1000, 0.5)),
    "c5-bible": ("spade", "bible", dict(), 0.004),
    "c5-sign": ("spade", "sign", dict(), 0.015),
}
# CPU prefix search for TSR starts here (the restatement needs minutes beyond ~20K sequences at k = 1000)
TSR_CPU_PREFIX = 40000


def dataset(shape, kw):
    from tools import gen
    if shape == "quest":
        return gen.quest(kw["D"], seed=1)
    if shape == "kosarak":
        return gen.kosarak(D=kw["D"], seed=1)
    return getattr(gen, shape)(seed=1)


def log(msg):
    print("[configs %s] %s" % (time.strftime("%H:%M:%S"), msg), file=sys.stderr, flush=True)


def time_gpu(fn, reps=3, warmup=True):
    if warmup:
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append((time.perf_counter() - t0) * 1000.0)
    return statistics.median(ts), out


def cpu_share():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                n = min(n, max(1, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def cpu_spade(ds, sup, reps, threads, stride):
    from oracle import oracle
    runs = [oracle.spade_tokens(ds.seq_off, ds.tokens, sup, want_patterns=False, threads=threads, stride=stride)
            for _ in range(reps)]
    lat = [r["seconds"] - r["seconds_f1"] for r in runs]
    return {"threads": threads, "class_stride": stride, "reps": reps, "complete": all(r["complete"] for r in runs),
            "joins": runs[0]["joins"], "seconds_total": [round(r["seconds"], 3) for r in runs],
            "seconds_lattice": [round(v, 3) for v in lat], "seconds_lattice_median": statistics.median(lat),
            "joins_per_s": statistics.median(r["joins"] / max(v, 1e-9) for r, v in zip(runs, lat))}


def run_spade(eng, fsm, name, ds, sup, cpu_reps, gpu_only=False):
    db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_SPADE)
    prep = eng.stats()
    # the warmup mine is instrumented (HIP events around every launch: kernel times); the timed
    # mines run without the events (FSM_KCLOCK=0), as in bench.py
    eng.spade_csr(db, sup)
    ks = sorted(eng.kernel_stats(), key=lambda k: -k["ms"])[:4]
    os.environ["FSM_KCLOCK"] = "0"
    try:
        ms, (csr, meta) = time_gpu(lambda: eng.spade_csr(db, sup), warmup=False)
    finally:
        del os.environ["FSM_KCLOCK"]
    st = eng.stats()
    db.free()
    out = {"config": name, "algo": "SPADE", "dataset": ds.name, "sequences": len(ds), "minsup": sup,
           "minsup_abs": meta["minsup"], "gpu_mine_ms": ms, "patterns": meta["n"], "joins": st["joins"],
           "gpu_joins_per_s": st["joins"] / (ms / 1000.0), "mask_words": st["mask_words"],
           "ms_flatten": prep["ms_flatten"], "ms_upload": prep["ms_upload"],
           "top_kernels": [{"name": k["name"], "ms": round(k["ms"], 3),
                            "GBps": round(k["alg_bytes"] / 1e9 / (k["ms"] / 1e3), 1) if k["ms"] else 0}
                           for k in ks]}
    if gpu_only:
        return out
    nt = cpu_share()
    sampled = name == "c3"  # the complete single-thread mine takes most of an hour
    log("%s: GPU %.2f ms; CPU restatement (%s)" % (name, ms, "class-stride sample" if sampled else "complete"))
    c1 = cpu_spade(ds, sup, 1 if sampled else cpu_reps, 1, 128 if sampled else 1)
    ca = cpu_spade(ds, sup, 1 if sampled else cpu_reps, nt, 8 if sampled else 1) if nt > 1 else None
    out.update({"cpu_1thr": c1, "cpu_all_cores": ca, "cpu_share": nt})
    out["speedup_vs_cpu_1thr_joins_per_s"] = out["gpu_joins_per_s"] / c1["joins_per_s"]
    if not sampled:
        out["speedup_vs_cpu_1thr_time"] = c1["seconds_lattice_median"] * 1000.0 / ms
        if ca:
            out["speedup_vs_cpu_all_cores_time"] = ca["seconds_lattice_median"] * 1000.0 / ms
    return out


def run_tsr(eng, fsm, name, ds, params, cpu_s, gpu_only=False):
    from oracle import oracle
    k, mc = params
    db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_TSR)
    prep = eng.stats()
    # (a full run is seconds: median of 3 after a warmup when the CPU legs are skipped)
    ms, (rules, meta) = time_gpu(lambda: eng.tsr(db, k, mc), reps=3 if gpu_only else 1, warmup=gpu_only)
    st = eng.stats()
    ks = sorted(eng.kernel_stats(), key=lambda q: -q["ms"])[:4]
    db.free()
    # CPU: the largest prefix (halving from TSR_CPU_PREFIX) whose full run fits the bound
    n = 0 if gpu_only else min(len(ds), TSR_CPU_PREFIX)
    cpu = None
    log("%s: GPU %.2f ms; CPU restatement on prefixes (bound %.0f s each)" % (name, ms, cpu_s))
    while n >= 1000:
        log("%s: CPU prefix %d" % (name, n))
        sub = ds.head(n)
        r = oracle.tsr(sub.records(), k, mc, time_limit_s=cpu_s)
        if r["complete"]:
            dbs = eng.db_from_tokens(sub.sids, sub.seq_off, sub.tokens, fsm.MODE_TSR)
            gms, (grules, _) = time_gpu(lambda: eng.tsr(dbs, k, mc), reps=3)
            dbs.free()
            grules.sort(key=lambda t: (-t[2], t[0], t[1]))
            cpu = {"cpu_prefix_sequences": n, "cpu_seconds": r["seconds"], "cpu_expansions": r["expansions"],
                   "gpu_ms_on_prefix": gms, "prefix_rules_identical": grules == r["rules"],
                   "speedup_on_prefix": r["seconds"] * 1000.0 / gms}
            break
        n //= 2
    out = {"config": name, "algo": "TSR", "dataset": ds.name, "sequences": len(ds), "k": k, "minconf": mc,
           "gpu_mine_ms": ms, "rules": len(rules), "final_minsup": meta["final_minsup"],
           "expansions": st["expansions"], "ms_pair_phase": st["ms_f2"], "ms_expansions": st["ms_lattice"],
           "ms_flatten": prep["ms_flatten"], "ms_upload": prep["ms_upload"],
           "top_kernels": [{"name": q["name"], "ms": round(q["ms"], 3)} for q in ks]}
    if not gpu_only:
        out.update(cpu or {"cpu": "no prefix >= 1000 sequences completed within the bound"})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="bound of the TSR prefix runs")
    ap.add_argument("--cpu-reps", type=int, default=1, help="complete SPADE CPU mines per config (median)")
    ap.add_argument("--verbose", action="store_true", help="engine progress on stderr (long TSR runs)")
    ap.add_argument("--gpu-only", action="store_true", help="GPU legs only (the CPU columns from an earlier sweep)")
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime per process, see _lib.py)
    import spark_fsm_amd as fsm
    want = [c for c in args.only.split(",") if c] or list(CONFIGS)
    with fsm.Engine(0, verbose=args.verbose) as eng:
        for name in want:
            algo, shape, kw, par = CONFIGS[name]
            log("%s: generating %s" % (name, shape))
            ds = dataset(shape, kw)
            if algo == "spade":
                res = run_spade(eng, fsm, name, ds, par, args.cpu_reps, args.gpu_only)
            else:
                res = run_tsr(eng, fsm, name, ds, par, args.cpu_seconds, args.gpu_only)
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
