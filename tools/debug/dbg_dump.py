import sys
sys.path.insert(0, '.'); sys.path.insert(0, 'spark-fsm_amd')
import spark_fsm_amd as fsm
eng = fsm.Engine(0, verbose=True)
def run(n, positions, extra):
    recs = []
    for s in range(3):
        toks = []
        for k in range(n):
            it = 1 if k in positions else (2 if k in extra else 1000 + 100000 * s + k)
            toks.append("%d -1" % it)
        recs.append((s, " ".join(toks)))
    db = eng.db_from_spmf(recs, fsm.MODE_SPADE)
    try:
        pats, _ = eng.spade(db, 1.0)
        print("npat", len(pats), sorted(pats)[:10], flush=True)
    except Exception as e:
        print("EXC", e, flush=True)
    db.free()
run(int(sys.argv[1]), tuple(map(int, sys.argv[2].split(","))), tuple(map(int, sys.argv[3].split(","))))
