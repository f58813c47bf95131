"""Which ring settings make TSR's in-flight ring guard fire (fsm_stats.tsr_ring_waits) on
the test DB of test_tsr_expansion_domains_agree, with the rules checked against the oracle."""
import itertools
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "spark-fsm_amd")]
import torch  # noqa: F401,E402
import spark_fsm_amd as fsm  # noqa: E402
from oracle import oracle  # noqa: E402
from tools import gen  # noqa: E402

ds = gen.kosarak(D=6000, seed=3)
o = oracle.tsr(ds.records(), 300, 0.4)
for mb, win, sets, batch in itertools.product(["1", "0.25", "0.0625"], ["16"], ["2", "4"], ["default", "16"]):
    os.environ.update({"FSM_TSR_ARENA_MB": mb, "FSM_TSR_PLIST_WINDOW": win, "FSM_TSR_SETS": sets})
    if batch == "default":
        os.environ.pop("FSM_TSR_BATCH", None)
    else:
        os.environ["FSM_TSR_BATCH"] = batch
    with fsm.Engine(0) as e:
        db = e.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_TSR)
        rules, meta = e.tsr(db, 300, 0.4)
        db.free()
        st = e.stats()
    rules.sort(key=lambda t: (-t[2], t[0], t[1]))
    ok = rules == o["rules"] and meta["final_minsup"] == o["final_minsup"]
    print(mb, win, sets, batch, "waits", st["tsr_ring_waits"], "ok", ok, flush=True)
