"""K0 on the GPU: fsm_db_from_tokens builds the vertical
DB on the device (spark-fsm_amd/csrc/k0_build.hip).  The DB it leaves in HBM
must equal the host flatten's (flatten.cpp, FSM_K0=host) byte for byte: row
offsets, dense item ids, eid masks (SPADE) or first / last itemset indexes
(TSR), the item dictionary and the longest-row occurrence count.

Reference rules restated by both builders: SPADE.scala:53-106, :151-210
(implicit timestamps, -1 closes an itemset, -2 ignored, items after the last
-1 dropped; eids rank-compressed) and TSR.scala:52-94, :109-143 (0-based
itemset index counting every -1)."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import spark_fsm_amd as fsm
    e = fsm.Engine(0)
    yield e
    e.close()


def images(eng, ds, mode, monkeypatch):
    """(device image, host image, device stats flag, host stats flag)."""
    out = []
    for k0 in ("device", "host"):
        if k0 == "host":
            monkeypatch.setenv("FSM_K0", "host")
        else:
            monkeypatch.delenv("FSM_K0", raising=False)
        db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, mode)
        try:
            out.append((eng.db_export(db), eng.stats()["k0_device"]))
        finally:
            db.free()
    monkeypatch.delenv("FSM_K0", raising=False)
    return out


def assert_same(a, b):
    assert set(a) == set(b)
    for k in a:
        if isinstance(a[k], np.ndarray):
            assert a[k].dtype == b[k].dtype or a[k].size == 0, k
            assert np.array_equal(a[k], b[k]), k
        else:
            assert a[k] == b[k], k


class Tok:
    def __init__(self, rows):
        lens = [len(r) for r in rows]
        self.seq_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        self.tokens = np.array([t for r in rows for t in r], dtype=np.int64)
        self.sids = np.arange(len(rows), dtype=np.int32)


def random_rows(rng, n, lo_item, hi_item, long_frac):
    rows = []
    for _ in range(n):
        L = rng.randint(65, 400) if rng.random() < long_frac else rng.randint(0, 64)
        rows.append([rng.choice((-1, -1, -2)) if rng.random() < 0.35 else rng.randint(lo_item, hi_item)
                     for _ in range(L)])
    return Tok(rows)


@pytest.mark.parametrize("shape", ["quest20k", "quest1m", "bible", "sign", "random"])
def test_k0_spade_matches_host_flatten(eng, shape, monkeypatch):
    import spark_fsm_amd as fsm
    from tools import gen
    if shape == "quest20k":
        ds = gen.quest(20000, seed=1)
    elif shape == "quest1m":
        ds = gen.quest(1000000, seed=1)
    elif shape == "bible":
        ds = gen.bible(seed=1).head(3000)
    elif shape == "sign":
        ds = gen.sign(seed=1)
    else:  # separators anywhere, empty itemsets, negative items (legal SPADE items), long rows
        ds = random_rows(random.Random(4), 3000, -6, 40, 0.05)
    (dev, kd), (host, kh) = images(eng, ds, fsm.MODE_SPADE, monkeypatch)
    assert kd == 1 and kh == 0
    assert_same(dev, host)


@pytest.mark.parametrize("shape", ["kosarak20k", "random"])
def test_k0_tsr_matches_host_flatten(eng, shape, monkeypatch):
    import spark_fsm_amd as fsm
    from tools import gen
    if shape == "kosarak20k":
        ds = gen.kosarak(D=20000, seed=1)
    else:  # negative tokens only after the last -1 (the reference drops them)
        rng = random.Random(9)
        rows = []
        for _ in range(2000):
            r = [rng.choice((-1, -2)) if rng.random() < 0.4 else rng.randint(0, 30)
                 for _ in range(rng.randint(65, 200) if rng.random() < 0.05 else rng.randint(0, 64))]
            rows.append(r + [-1, rng.randint(-9, -3)])
        ds = Tok(rows)
    (dev, kd), (host, kh) = images(eng, ds, fsm.MODE_TSR, monkeypatch)
    assert kd == 1 and kh == 0
    assert_same(dev, host)


def test_k0_declines_to_host_for_merged_sids_and_errors(eng, monkeypatch):
    """Inputs the device builder does not take (equal sids, tokens outside
    int32, a negative TSR item in a closed itemset) go through the host
    flatten, which merges rows or reports the reference's error."""
    import spark_fsm_amd as fsm
    ds = Tok([[1, 2, -1, 3, -1], [2, -1, 1, -1]])
    ds.sids = np.array([5, 5], dtype=np.int32)
    db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_SPADE)
    img = eng.db_export(db)
    db.free()
    assert eng.stats()["k0_device"] == 0 and img["rows"] == 1
    bad = Tok([[1, 2 ** 40, -1]])
    with pytest.raises(fsm.FsmParseError):
        eng.db_from_tokens(bad.sids, bad.seq_off, bad.tokens, fsm.MODE_SPADE)
    neg = Tok([[1, -1, -5, -1]])
    with pytest.raises(fsm.FsmParseError):
        eng.db_from_tokens(neg.sids, neg.seq_off, neg.tokens, fsm.MODE_TSR)


def test_k0_d1m_build_time(eng):
    """ms_flatten + ms_upload at D1M (under 50 ms on the device)."""
    import spark_fsm_amd as fsm
    from tools import gen
    ds = gen.quest(1000000, seed=1)
    db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_SPADE)  # warm
    db.free()
    db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_SPADE)
    st = eng.stats()
    db.free()
    print("K0 D1M: upload %.1f ms, build %.1f ms" % (st["ms_upload"], st["ms_flatten"]))
    assert st["k0_device"] == 1
    assert st["ms_flatten"] + st["ms_upload"] < 50.0
