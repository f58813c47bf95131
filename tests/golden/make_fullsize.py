"""Full-size parity fixtures for the BASELINE configs (run once in the build
container; the GPU tests compare libfsm's output against the committed JSON).

For every SPADE config the CPU restatement (oracle/fsm_oracle.c, first-level
classes on OpenMP threads: same pattern set and join count as one thread,
tests/test_oracle.py) mines the complete pattern set; the fixture keeps the
pattern count, the join count, the absolute minsup and the canonical digest of
tests/digest.py.  For TSR (config 4) the restatement cannot finish at 990K
sequences, so the fixture holds the exact rule digest of the largest prefix it
finishes here, and the full-size test checks definitional properties instead.

    python tests/golden/make_fullsize.py [--only c2,c3] [--threads 8]

Writes tests/golden/fullsize.json (merging with what is already there).
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

OUT = os.path.join(HERE, "fullsize.json")

# name -> (algo, generator, kwargs, parameters); datasets are tools/gen.py seed 1
CONFIGS = {
    "c1": ("spade", "quest", {"D": 10000}, 0.005),
    "c2": ("spade", "quest", {"D": 100000}, 0.005),
    "c3": ("spade", "quest", {"D": 1000000}, 0.001),
    "c5-bible": ("spade", "bible", {}, 0.004),
    "c5-sign": ("spade", "sign", {}, 0.015),
    "c4-prefix": ("tsr", "kosarak", {"D": 990002, "prefix": 20000}, (1000, 0.5)),
    "c4-prefix100k": ("tsr", "kosarak", {"D": 990002, "prefix": 100000}, (1000, 0.5)),
}


def dataset(shape, kw):
    from tools import gen
    if shape == "quest":
        return gen.quest(kw["D"], seed=1)
    if shape == "kosarak":
        ds = gen.kosarak(D=kw["D"], seed=1)
        return ds.head(kw["prefix"]) if "prefix" in kw else ds
    return getattr(gen, shape)(seed=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    args = ap.parse_args()
    from digest import pattern_digest, rule_digest
    from oracle import oracle
    have = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            have = json.load(f)
    want = [c for c in args.only.split(",") if c] or list(CONFIGS)
    for name in want:
        algo, shape, kw, par = CONFIGS[name]
        t0 = time.time()
        ds = dataset(shape, kw)
        if algo == "spade":
            csr, meta = oracle.spade_tokens_csr(ds.seq_off, ds.tokens, par, threads=args.threads)
            rec = {"algo": "SPADE", "dataset": ds.name, "sequences": len(ds), "support": par,
                   "minsup": meta["minsup"], "joins": meta["joins"], "digest": pattern_digest(*csr)}
        else:
            k, mc = par
            r = oracle.tsr(ds.records(), k, mc)
            rec = {"algo": "TSR", "dataset": ds.name, "sequences": len(ds), "k": k, "minconf": mc,
                   "final_minsup": r["final_minsup"], "expansions": r["expansions"],
                   "digest": rule_digest(r["rules"])}
        rec["oracle_seconds"] = round(time.time() - t0, 1)
        have[name] = rec
        print(name, json.dumps(rec), flush=True)
        with open(OUT, "w") as f:
            json.dump(have, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
