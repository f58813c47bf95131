import sys
sys.path.insert(0, '.'); sys.path.insert(0, 'spark-fsm_amd')
import spark_fsm_amd as fsm
eng = fsm.Engine(0)
def run(n, positions, extra=None):
    recs = []
    for s in range(3):
        toks = []
        for k in range(n):
            it = 1 if k in positions else (2 if extra and k in extra else 1000 + 100000 * s + k)
            toks.append("%d -1" % it)
        recs.append((s, " ".join(toks)))
    db = eng.db_from_spmf(recs, fsm.MODE_SPADE)
    try:
        pats, _ = eng.spade(db, 1.0)
        out = sorted(p for p, _ in pats if len(p) <= 4)
        print(n, positions, extra, "W=%d" % eng.stats()["mask_words"], "npat=%d" % len(pats), out[:8], flush=True)
    except Exception as e:
        print(n, positions, "EXC", e, flush=True)
    db.free()
for n, pos in [(70, (10, 65)), (150, (10, 140)), (250, (10, 200)), (250, (100, 200)), (250, (195, 200)),
               (250, (10, 190)), (250, (130, 140)), (250, (64, 128)), (250, (5, 6)), (200, (5, 195)), (256, (5, 255))]:
    run(n, pos)
run(250, (10, 200), extra=(220,))
run(250, (10, 100), extra=(150,))
