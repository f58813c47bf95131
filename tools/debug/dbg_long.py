import random, sys, os
sys.path.insert(0, '.'); sys.path.insert(0, 'spark-fsm_amd')
import spark_fsm_amd as fsm
from oracle import oracle
rng = random.Random(3)
eng = fsm.Engine(0, verbose=True)
for nsets in (70, 150, 250):
    recs = []
    for s in range(14):
        toks = [[1000 + s * 1000 + k] for k in range(nsets)]
        pos = sorted(rng.sample(range(nsets), 6))
        for p, it in zip(pos, (1, 2, 3, 1, 4, 2)):
            toks[p] = [it] + ([5] if rng.random() < 0.5 else [])
        recs.append((s, " ".join(" ".join(map(str, t)) + " -1" for t in toks) + " -2"))
    for sup in (0.5, 0.8):
        print("case", nsets, sup, flush=True)
        o = oracle.spade(recs, sup)
        db = eng.db_from_spmf(recs, fsm.MODE_SPADE)
        try:
            pats, meta = eng.spade(db, sup)
            print("  ok", sorted(pats) == o["patterns"], eng.stats()["mask_words"], flush=True)
        except Exception as e:
            print("  EXC", e, flush=True)
        db.free()
