"""Host read rate of the generator's token array, before and after the HIP runtime is up."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "spark-fsm_amd"))
import numpy as np
from tools import gen
ds = gen.quest(1000000, seed=1)
def t(label, f):
    t0 = time.perf_counter(); f(); print("%-40s %.2f ms" % (label, (time.perf_counter() - t0) * 1e3), flush=True)
t("astype int32 (fresh)", lambda: ds.tokens.astype(np.int32))
t("astype int32 (again)", lambda: ds.tokens.astype(np.int32))
t("sum", lambda: ds.tokens.sum())
import torch  # noqa
import spark_fsm_amd as fsm
eng = fsm.Engine(0)
t("astype int32 (after engine)", lambda: ds.tokens.astype(np.int32))
os.environ["FSM_HOST_TRACE"] = "1"
db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_SPADE)
t("astype int32 (after K0)", lambda: ds.tokens.astype(np.int32))
db.free()
tok2 = ds.tokens.copy()
so2 = ds.seq_off.copy()
t0 = time.perf_counter()
db = eng.db_from_tokens(ds.sids, so2, tok2, fsm.MODE_SPADE)
print("second K0 on fresh copies %.2f ms" % ((time.perf_counter() - t0) * 1e3))
db.free()
t0 = time.perf_counter()
db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_SPADE)
print("third K0 on the first arrays %.2f ms" % ((time.perf_counter() - t0) * 1e3))
