"""One timed mine of one synthetic config on cuda:0, with the engine's stats
(for profiling under rocprofv3 and for host/GPU time splits):

    python tools/run_one.py spade sign --support 0.015 [--reps 3]
    python tools/run_one.py tsr kosarak --D 100000 --k 1000 --minconf 0.5

Prints one JSON line per rep: wall ms, the fsm_stats dict and the top kernels.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "spark-fsm_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("algo", choices=["spade", "tsr"])
    ap.add_argument("shape", choices=["quest", "kosarak", "bible", "sign"])
    ap.add_argument("--D", type=int, default=0)
    ap.add_argument("--support", type=float, default=0.001)
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--minconf", type=float, default=0.5)
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--head", type=int, default=0, help="mine only the first HEAD sequences")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime per process, see _lib.py)
    import spark_fsm_amd as fsm
    from tools import gen
    kw = {"D": a.D} if a.D else {}
    if a.shape == "quest":
        ds = gen.quest(a.D or 100000, seed=1)
    else:
        ds = getattr(gen, a.shape)(seed=1, **kw)
    if a.head:
        ds = ds.head(a.head)
    mode = fsm.MODE_SPADE if a.algo == "spade" else fsm.MODE_TSR
    with fsm.Engine(0, verbose=a.verbose) as eng:
        db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, mode)
        for _ in range(a.reps):
            t0 = time.perf_counter()
            if a.algo == "spade":
                _, meta = eng.spade_csr(db, a.support)
            else:
                _, meta = eng.tsr(db, a.k, a.minconf)
            ms = (time.perf_counter() - t0) * 1000.0
            ks = sorted(eng.kernel_stats(), key=lambda q: -q["ms"])[:8]
            print(json.dumps({"dataset": ds.name, "wall_ms": ms, "meta": {k: v for k, v in meta.items()
                                                                          if isinstance(v, (int, float))},
                              "stats": eng.stats(),
                              "kernels": [{"name": q["name"], "launches": q["launches"], "ms": round(q["ms"], 3)}
                                          for q in ks]}), flush=True)
        db.free()


if __name__ == "__main__":
    main()
