"""GPU parity: libfsm (HIP, gfx950) vs the CPU restatement / golden fixtures.

Bit-exact for everything (integer supports, pattern sets, rule sets and the
double confidences, which are the same IEEE division on both sides).  Small
and medium cases compare full outputs with the oracle; full-size configs use
size-independent properties (definitional re-count of sampled outputs,
threshold / top-k invariants)."""
import json
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def fsm():
    import spark_fsm_amd
    return spark_fsm_amd


@pytest.fixture(scope="module")
def eng(fsm):
    e = fsm.Engine(0)
    yield e
    e.close()


def gpu_spade(eng, recs, support, tokens=None):
    from spark_fsm_amd import MODE_SPADE
    if tokens is not None:
        db = eng.db_from_tokens(tokens.sids, tokens.seq_off, tokens.tokens, MODE_SPADE)
    else:
        db = eng.db_from_spmf(recs, MODE_SPADE)
    try:
        pats, meta = eng.spade(db, support)
    finally:
        db.free()
    return sorted(pats), meta, eng.stats()


def gpu_tsr(eng, recs, k, minconf, tokens=None):
    from spark_fsm_amd import MODE_TSR
    if tokens is not None:
        db = eng.db_from_tokens(tokens.sids, tokens.seq_off, tokens.tokens, MODE_TSR)
    else:
        db = eng.db_from_spmf(recs, MODE_TSR)
    try:
        rules, meta = eng.tsr(db, k, minconf)
    finally:
        db.free()
    rules.sort(key=lambda t: (-t[2], t[0], t[1]))
    return rules, meta, eng.stats()


def canon(pats):
    return [(tuple(tuple(s) for s in p), sup) for p, sup in pats]


# ------------------------------------------------------------------ golden
@pytest.mark.parametrize("case", load("spade_cases.json"), ids=lambda c: c["name"])
def test_spade_golden(eng, case):
    recs = [tuple(r) for r in case["records"]]
    pats, meta, st = gpu_spade(eng, recs, case["support"])
    assert pats == canon(case["patterns"])
    assert meta["minsup"] == case["minsup"] or not case["patterns"]
    assert st["joins"] == case["joins"]


@pytest.mark.parametrize("case", load("tsr_cases.json"), ids=lambda c: c["name"])
def test_tsr_golden(eng, case):
    recs = [tuple(r) for r in case["records"]]
    rules, meta, _ = gpu_tsr(eng, recs, case["k"], case["minconf"])
    assert rules == [(tuple(x), tuple(y), s, c) for x, y, s, c in case["rules"]]
    assert meta["final_minsup"] == case["final_minsup"]


ERR = load("error_cases.json")


@pytest.mark.parametrize("case", ERR["spade"], ids=lambda c: c["name"])
def test_spade_errors(eng, fsm, case):
    with pytest.raises(fsm.FsmParseError):
        gpu_spade(eng, [tuple(r) for r in case["records"]], 0.5)


@pytest.mark.parametrize("case", ERR["tsr"], ids=lambda c: c["name"])
def test_tsr_errors(eng, fsm, case):
    with pytest.raises(fsm.FsmParseError):
        gpu_tsr(eng, [tuple(r) for r in case["records"]], 3, 0.5)


def test_tsr_negative_item_in_dropped_trailing_itemset(eng):
    """TSR.newSequence drops the unclosed trailing itemset, so a negative item
    there never indexes the Vertical arrays: the reference succeeds.
    In a closed itemset it still fails (error_cases.json)."""
    from oracle import oracle
    recs = [(0, "1 -1 2 -1 -5 -2"), (1, "1 -1 2 -1 3"), (2, "1 2 -1 -7")]
    o = oracle.tsr(recs, 3, 0.5)
    rules, meta, _ = gpu_tsr(eng, recs, 3, 0.5)
    assert rules == o["rules"] and rules and meta["final_minsup"] == o["final_minsup"]


def test_tsr_k_zero_rejected(eng, fsm):
    with pytest.raises(fsm.FsmError):
        gpu_tsr(eng, [(0, "1 -1 2 -1")], 0, 0.5)


# ------------------------------------------------------- random vs oracle
def rand_records(rng, nseq, nitems, maxsets, maxset, ts):
    recs = []
    for s in range(nseq):
        toks = []
        for _ in range(rng.randint(0, maxsets)):
            if ts and rng.random() < 0.3:
                toks.append("<%d>" % rng.randint(0, 9))
            toks += [str(rng.randint(1, nitems)) for _ in range(rng.randint(1, maxset))]
            toks.append("-1")
        recs.append((s, " ".join(toks + ["-2"])))
    return recs


def test_spade_random_vs_oracle(eng):
    from oracle import oracle
    rng = random.Random(11)
    for it in range(60):
        recs = rand_records(rng, rng.randint(8, 60), rng.randint(2, 12), 6, 3, ts=it % 2 == 0)
        sup = rng.choice([0.15, 0.2, 0.3, 0.5])
        o = oracle.spade(recs, sup)
        pats, _, st = gpu_spade(eng, recs, sup)
        assert pats == o["patterns"], (it, recs, sup)
        assert st["joins"] == o["joins"]


def test_tsr_random_vs_oracle(eng):
    from oracle import oracle
    rng = random.Random(12)
    for it in range(60):
        recs = rand_records(rng, rng.randint(2, 60), rng.randint(2, 12), 6, 3, ts=False)
        if not any(t not in ("-1", "-2") for _, l in recs for t in l.split(" ")):
            continue
        k, mc = rng.randint(1, 40), rng.choice([0.0, 0.2, 0.5, 0.9])
        o = oracle.tsr(recs, k, mc)
        rules, meta, _ = gpu_tsr(eng, recs, k, mc)
        assert rules == o["rules"], (it, recs, k, mc)
        assert meta["final_minsup"] == o["final_minsup"]


def test_long_sequences_multiword_masks(eng):
    """> 64 distinct timestamps per sequence (W = 2 and W = 4 masks): planted
    patterns at positions that straddle 64-bit word boundaries, unique noise
    items elsewhere (so the pattern set stays small enough for the oracle)."""
    from oracle import oracle
    rng = random.Random(3)
    for nsets in (70, 150, 250):
        recs = []
        for s in range(14):
            toks = [[1000 + s * 1000 + k] for k in range(nsets)]
            pos = sorted(rng.sample(range(nsets), 6))
            for p, it in zip(pos, (1, 2, 3, 1, 4, 2)):
                toks[p] = [it] + ([5] if rng.random() < 0.5 else [])
            recs.append((s, " ".join(" ".join(map(str, t)) + " -1" for t in toks) + " -2"))
        for sup in (0.5, 0.8):
            o = oracle.spade(recs, sup)
            pats, _, st = gpu_spade(eng, recs, sup)
            assert pats == o["patterns"] and st["joins"] == o["joins"]
            assert st["mask_words"] >= 2 and len(pats) > 5


@pytest.mark.parametrize("nsets,W", [(1000, 16), (4000, 64), (5000, 128), (30000, 512)])
@pytest.mark.parametrize("count_path", ["default", "keys"])
def test_very_long_sequences_wide_masks(eng, nsets, W, count_path, monkeypatch):
    """~1,000 to 30,000 distinct timestamps per sequence: W = 16 and W = 64
    mask words (the widest register-held width) and W = 128 / 512 (the
    runtime-width kernels, masks read word by word; up to 65,536 distinct
    timestamps, SPADE.scala:74,90 registers any timestamp).  Planted patterns
    across the whole eid range, unique noise items elsewhere; the text path
    (host flatten) and the token path (K0 on the device, or the host flatten
    for more than 4,096 timestamps) against the oracle."""
    import numpy as np
    from oracle import oracle
    rng = random.Random(nsets)
    sets_all = []
    for s in range(12):
        sets = [[100000 + s * 10000 + k] for k in range(nsets)]
        pos = sorted(rng.sample(range(nsets), 6))
        for p, it in zip(pos, (1, 2, 3, 1, 4, 2)):
            sets[p] = [it] + ([5] if rng.random() < 0.5 else [])
        sets_all.append(sets)
    recs = [(s, " ".join(" ".join(map(str, t)) + " -1" for t in sets) + " -2") for s, sets in enumerate(sets_all)]
    toks = [[x for t in sets for x in t + [-1]] + [-2] for sets in sets_all]

    class Tok:
        seq_off = np.concatenate([[0], np.cumsum([len(t) for t in toks])]).astype(np.int64)
        tokens = np.array([x for t in toks for x in t], dtype=np.int64)
        sids = np.arange(len(toks), dtype=np.int32)

    if count_path != "default":
        monkeypatch.setenv("FSM_COUNT_PATH", count_path)
    for sup in (0.5, 0.75):
        o = oracle.spade(recs, sup)
        pats, _, st = gpu_spade(eng, recs, sup)
        assert pats == o["patterns"] and st["joins"] == o["joins"] and st["mask_words"] == W
        pats2, _, st2 = gpu_spade(eng, None, sup, tokens=Tok)
        assert pats2 == o["patterns"] and st2["mask_words"] == W and len(pats) > 5


def test_small_memory_budget_splits_groups(fsm):
    """Force the frontier into many small class groups: same answer."""
    from oracle import oracle
    from tools import gen
    ds = gen.quest(3000, seed=2)
    recs = ds.records()
    o = oracle.spade(recs, 0.008)
    with fsm.Engine(0, mem_budget=1) as e:  # every child class is its own group
        pats, _, st = gpu_spade(e, recs, 0.008)
    assert pats == o["patterns"] and st["joins"] == o["joins"]
    assert st["batches"] > 3


def test_two_contexts_on_two_threads(fsm):
    """Two contexts mining at the same time on two threads (the reference runs
    concurrent requests on one SparkContext, RequestContext.scala:30): each
    context draws device blocks from its own pool, so the results
    are exactly the single-context ones; a DB may outlive its context."""
    import threading
    from oracle import oracle
    from tools import gen
    ds = gen.quest(20000, seed=7)
    exp_s = oracle.spade_tokens(ds.seq_off, ds.tokens, 0.004)["patterns"]
    kds = gen.kosarak(D=4000, seed=2)
    exp_t = oracle.tsr(kds.records(), 100, 0.5)["rules"]
    ok, errs = [], []

    def spade_worker():
        try:
            with fsm.Engine(0) as e:
                for _ in range(3):
                    pats, _, _ = gpu_spade(e, None, 0.004, tokens=ds)
                    ok.append(pats == exp_s)
        except Exception as x:  # noqa: BLE001
            errs.append(repr(x))

    def tsr_worker():
        try:
            with fsm.Engine(0) as e:
                for _ in range(3):
                    rules, _, _ = gpu_tsr(e, None, 100, 0.5, tokens=kds)
                    ok.append(rules == exp_t)
        except Exception as x:  # noqa: BLE001
            errs.append(repr(x))

    th = [threading.Thread(target=f) for f in (spade_worker, spade_worker, tsr_worker)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=110)
    assert not errs and len(ok) == 9 and all(ok), (errs, ok)
    # a DB freed after its context was destroyed returns its blocks to that context's pool
    e = fsm.Engine(0)
    db = e.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_SPADE)
    e.close()
    db.free()


# ------------------------------------------------------ dataset shapes
@pytest.mark.parametrize("D,sup", [(10000, 0.005), (10000, 0.01), (20000, 0.004)])
def test_spade_quest_vs_oracle(eng, D, sup):
    from oracle import oracle
    from tools import gen
    ds = gen.quest(D, seed=1)
    o = oracle.spade_tokens(ds.seq_off, ds.tokens, sup)
    pats, meta, st = gpu_spade(eng, None, sup, tokens=ds)
    assert meta["minsup"] == o["minsup"]
    assert pats == o["patterns"]
    assert st["joins"] == o["joins"]


def test_spade_text_and_token_paths_agree(eng):
    from tools import gen
    ds = gen.quest(3000, seed=5)
    a, _, _ = gpu_spade(eng, ds.records(), 0.01)
    b, _, _ = gpu_spade(eng, None, 0.01, tokens=ds)
    assert a == b and len(a) > 10


@pytest.mark.parametrize("shape,n,sup", [("bible", 2000, 0.03), ("sign", 730, 0.35)])
def test_spade_long_sequence_shapes_vs_oracle(eng, shape, n, sup):
    from oracle import oracle
    from tools import gen
    ds = getattr(gen, shape)(seed=1).head(n)
    o = oracle.spade_tokens(ds.seq_off, ds.tokens, sup)
    pats, _, st = gpu_spade(eng, None, sup, tokens=ds)
    assert pats == o["patterns"] and st["joins"] == o["joins"]
    assert len(pats) > 20


@pytest.mark.parametrize("n,k,mc", [(5000, 50, 0.5), (20000, 200, 0.5), (3000, 100, 0.1)])
def test_tsr_kosarak_shape_vs_oracle(eng, n, k, mc):
    from oracle import oracle
    from tools import gen
    ds = gen.kosarak(D=n, seed=1)
    recs = ds.records()
    o = oracle.tsr(recs, k, mc)
    rules, meta, _ = gpu_tsr(eng, None, k, mc, tokens=ds)
    assert rules == o["rules"]
    assert meta["final_minsup"] == o["final_minsup"]


def test_tsr_bible_shape_vs_oracle(eng):
    from oracle import oracle
    from tools import gen
    ds = gen.bible(seed=2).head(1500)
    o = oracle.tsr(ds.records(), 100, 0.3)
    rules, meta, _ = gpu_tsr(eng, None, 100, 0.3, tokens=ds)
    assert rules == o["rules"] and meta["final_minsup"] == o["final_minsup"]


# ---------------------------------------------- full-size properties
def test_spade_quest_d1m_properties(eng):
    """BASELINE config 3 size (D1M, minsup 0.1%): definitional re-count of a
    sample of the output, exact F1, threshold, prefix anti-monotonicity."""
    from oracle import oracle
    from tools import gen
    ds = gen.quest(1000000, seed=1)
    pats, meta, st = gpu_spade(eng, None, 0.001, tokens=ds)
    assert meta["minsup"] == 1000 and meta["total"] == 1000000
    sup = dict(pats)
    assert min(sup.values()) >= 1000
    # F1: exact distinct-sid supports
    tk, so = ds.tokens, ds.seq_off
    sid = np.repeat(np.arange(len(ds)), np.diff(so))
    m = tk >= 0
    u = np.unique(sid[m].astype(np.int64) * (1 << 32) + tk[m])
    items, counts = np.unique(u & 0xFFFFFFFF, return_counts=True)
    f1 = {((int(i),),): int(c) for i, c in zip(items, counts) if c >= 1000}
    assert {p: s for p, s in sup.items() if len(p) == 1 and len(p[0]) == 1} == f1
    # every pattern's prefix (drop last item) is frequent with >= support
    for p, s in pats:
        if sum(len(x) for x in p) == 1:
            continue
        last = p[-1]
        par = p[:-1] + ((last[:-1],) if len(last) > 1 else ())
        assert sup[par] >= s
    # definitional re-count of a random sample of multi-item patterns
    rng = random.Random(0)
    multi = [x for x in pats if sum(len(s) for s in x[0]) >= 2]
    assert len(multi) > 100
    for p, s in rng.sample(multi, 25):
        assert oracle.pattern_support(so, tk, p) == s, p
    assert st["joins"] > 4.0e7


_CASES = {}


def shape_case(shape):
    """(dataset, support, oracle result) of a path-agreement shape, computed once per test session:
    the path variants of one shape share the dataset and the oracle's answer."""
    if shape not in _CASES:
        from oracle import oracle
        from tools import gen
        if shape == "quest":
            ds, sup = gen.quest(20000, seed=9), 0.003
        elif shape == "quest4":
            ds, sup = gen.quest(20000, seed=4), 0.003
        elif shape == "sign":
            ds, sup = gen.sign(seed=2).head(400), 0.3
        elif shape == "bible":
            ds, sup = gen.bible(seed=2).head(1500), 0.03
        elif shape == "wide":  # runs of more than 64 entries at W = 1
            ds, sup = _wide_runs_db(), 0.05
        else:  # sign-low: first-level classes whose counter matrix spans several groups
            ds, sup = gen.sign(seed=3).head(60), 0.08
        _CASES[shape] = (ds, sup, oracle.spade_tokens(ds.seq_off, ds.tokens, sup))
    return _CASES[shape]


@pytest.mark.parametrize("path", ["group", "group-few-blocks", "atomic", "slab-root", "ordered"])
def test_root_f2_paths_agree(eng, path, monkeypatch):
    """The root F2 implementations (key runs counted per rank group, at the
    default and at a small block chunk; global atomics; from the DB rows (DB-direct root, default) or from the root
    slab) give the oracle's patterns and joins."""
    from oracle import oracle
    from tools import gen
    if path == "atomic":
        monkeypatch.setenv("FSM_ROOT_PATH", "atomic")
    if path == "slab-root":
        monkeypatch.setenv("FSM_ROOT_DB", "0")
    if path == "group-few-blocks":
        monkeypatch.setenv("FSM_F2_BLOCKS", "3")
    if path == "ordered":  # the ordered-pair enumeration (k_f2_keys) instead of the unordered one (k_f2_tri)
        monkeypatch.setenv("FSM_F2_TRI", "0")
    ds, sup, o = shape_case("quest4")
    pats, meta, st = gpu_spade(eng, None, sup, tokens=ds)
    assert pats == o["patterns"] and st["joins"] == o["joins"]


def _wide_runs_db(seed=5, n=600):
    """W = 1 sequences (at most 60 itemsets) holding up to 240 distinct items,
    so root and first-level runs exceed 64 entries (k_emit2's long-run list)."""
    import numpy as np
    from tools import gen
    rng = np.random.default_rng(seed)
    so, tk = [0], []
    for _ in range(n):
        nsets = int(rng.integers(1, 61))
        wide = rng.random() < 0.3
        for _ in range(nsets):
            k = int(rng.integers(2, 9)) if wide else int(rng.integers(1, 3))
            tk.extend(sorted(int(x) for x in rng.choice(300, size=k, replace=False)))
            tk.append(-1)
        tk.append(-2)
        so.append(len(tk))
    return gen.DataSet(np.array(so, dtype=np.int64), np.array(tk, dtype=np.int64), "wide-runs")


@pytest.mark.parametrize("path", ["onepass", "overflow-all", "overflow-some", "chunk", "host-child-of", "device-child-of", "host-kids",
                                  "host-order", "no-defer"])
@pytest.mark.parametrize("shape", ["quest", "sign", "bible", "wide"])
def test_emit_paths_agree(eng, path, shape, monkeypatch):
    """Child-run emission: the window kernel k_emit2 (W = 1: runs of <= 64
    entries in registers, longer runs through k_emit1's run list), the chunk
    kernel k_emit1 (FSM_EMIT_PATH=chunk; every W), and their overflow paths
    (records capped at 0 / 17 per wave, so waves join again while writing)
    give the oracle's patterns and joins; so do both builds of the child class
    table (FSM_CHILD_OF=host, or device: k_child_flag / scan / k_child_of), and
    both orderings of a one-group batch's records (default: on the device, k_rk_*;
    FSM_DEVORDER=0: on the host) with the children built after the emit launch or,
    FSM_EMIT_DEFER=0, before it."""
    from oracle import oracle
    from tools import gen
    if path == "overflow-all":
        monkeypatch.setenv("FSM_EMIT_CAP", "0")
    elif path == "overflow-some":
        monkeypatch.setenv("FSM_EMIT_CAP", "17")
    elif path == "chunk":
        monkeypatch.setenv("FSM_EMIT_PATH", "chunk")
    elif path == "host-child-of":
        monkeypatch.setenv("FSM_CHILD_OF", "host")
    elif path == "device-child-of":
        monkeypatch.setenv("FSM_CHILD_OF", "device")
    elif path == "host-kids":  # the kid table from the host records (default: k_freq_write + k_kid_off)
        monkeypatch.setenv("FSM_KIDS", "host")
    elif path == "host-order":
        monkeypatch.setenv("FSM_DEVORDER", "0")
    elif path == "no-defer":
        monkeypatch.setenv("FSM_EMIT_DEFER", "0")
    ds, sup, o = shape_case(shape)
    pats, meta, st = gpu_spade(eng, None, sup, tokens=ds)
    assert pats == o["patterns"] and st["joins"] == o["joins"]


def test_timestamp_limit(eng, fsm):
    """More than 65,536 distinct timestamps in one sequence (the 16-bit eid
    fields of the slab) is FSM_ELIMIT with a message, never a wrong answer."""
    recs = [(0, " ".join("%d -1" % (10 + k) for k in range(65537)) + " -2"), (1, "1 -1 2 -1 -2")]
    with pytest.raises(fsm.FsmError) as ei:
        gpu_spade(eng, recs, 0.5)
    assert ei.value.code == fsm.FSM_ELIMIT and "65536" in str(ei.value)


@pytest.mark.parametrize("path", ["keys", "atomic", "atomic-thread", "default", "sparse", "sparse-root"])
@pytest.mark.parametrize("shape", ["quest", "sign", "bible", "sign-low", "wide"])
def test_count_paths_agree(eng, path, shape, monkeypatch):
    """Class counting: the keyed count (group-aligned counter layout, u16 keys
    in (group, block) regions, LDS counting, counters written out) forced on
    every batch, the global-atomic count (k_count2's run windows at W = 1, runs
    over 64 entries thread-per-entry; or k_count thread-per-entry throughout,
    FSM_COUNT_KERNEL=thread), the sparse count (joins as u64 keys, radix sort +
    run-length encode; sparse-root: the root class too, through its slab) and the
    default size switch give the oracle's patterns and joins, and the same
    executed pair tests."""
    from oracle import oracle
    from tools import gen
    if path == "atomic-thread":
        monkeypatch.setenv("FSM_COUNT_PATH", "atomic")
        monkeypatch.setenv("FSM_COUNT_KERNEL", "thread")
    elif path == "sparse-root":
        monkeypatch.setenv("FSM_COUNT_PATH", "sparse")
        monkeypatch.setenv("FSM_ROOT_PATH", "atomic")
    elif path != "default":
        monkeypatch.setenv("FSM_COUNT_PATH", path)
    ds, sup, o = shape_case(shape)
    pats, meta, st = gpu_spade(eng, None, sup, tokens=ds)
    assert pats == o["patterns"] and st["joins"] == o["joins"]
    if path in ("keys", "sparse"):
        monkeypatch.setenv("FSM_COUNT_PATH", "atomic")
        _, _, st2 = gpu_spade(eng, None, sup, tokens=ds)
        assert st2["pair_tests"] == st["pair_tests"]


def test_class_with_70k_frequent_children(eng):
    """A prefix class with more than 65,535 frequent children (round 3 returned
    FSM_ELIMIT): 70,000 sequences <a, b_k> at support 1 make 70,001 frequent items
    (too many for the root's rank-group F2: the root is counted sparse) and a
    first-level class [a] of 70,000 members whose dense 140,000 x 140,000 counter
    matrix (78 GB) would not fit: it is counted sparse too.  Known answer: the
    1-patterns and the 70,000 patterns a -> b_k, every support by definition."""
    import numpy as np
    from spark_fsm_amd import MODE_SPADE
    from tools import gen
    n = 70000
    so = np.arange(0, 5 * (n + 1), 5, dtype=np.int64)
    tk = np.empty(5 * n, dtype=np.int64)
    tk[0::5], tk[1::5], tk[2::5], tk[3::5], tk[4::5] = 1, -1, np.arange(2, n + 2), -1, -2
    ds = gen.DataSet(so, tk, "70k-children")
    db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, MODE_SPADE)
    try:
        pats, meta = eng.spade(db, 1.0 / n)
    finally:
        db.free()
    exp = sorted([(((1,),), n)] + [(((b,),), 1) for b in range(2, n + 2)] +
                 [(((1,), (b,)), 1) for b in range(2, n + 2)])
    assert meta["minsup"] == 1 and sorted(pats) == exp
    st = eng.stats()
    F = n + 1  # SURVEY A.2 joins: root F^2 + F(F-1)/2, class [a]: S^2 + S(S-1)/2 with S = n
    assert st["joins"] == F * F + F * (F - 1) // 2 + n * n + n * (n - 1) // 2


# ------------------------------------------------------ sharded (N > 1)
@pytest.mark.parametrize("frac", ["0.1", "0"])
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_heavy_class_split(eng, world, frac, tmp_path, monkeypatch):
    """Heavy first-level classes (volume > FSM_SPLIT_FRAC of a rank's share;
    0.1 splits the largest SIGN-shaped classes, 0 disables splitting) are counted
    by every rank and their sub-classes planned over the ranks.  Every rank
    returns the complete pattern set (no pattern twice) and the single-rank
    join count."""
    from digest import pattern_digest
    from oracle import oracle
    from test_dist import run_ranks
    from tools import gen
    monkeypatch.setenv("FSM_SPLIT_FRAC", frac)
    res = run_ranks(world, ["spade_digest", "sign", "0", "0.07"], tmp_path, timeout=110)
    ds = gen.sign(seed=1)
    csr, meta = oracle.spade_tokens_csr(ds.seq_off, ds.tokens, 0.07, threads=4)
    exp = pattern_digest(*csr)
    for r in res:
        assert r["digest"] == exp and r["joins"] == meta["joins"] and r["minsup"] == meta["minsup"]

@pytest.mark.parametrize("world,recs", [(2, "default"), (3, "default"), (2, "64")])
def test_sharded_tsr_pair_phase(eng, world, recs, tmp_path, monkeypatch):
    """TSR with `world` ranks on this GPU over gloo: each rank counts the pairs of
    its own sequence range, the candidate keys (partial >= ceil(t / world)) are
    exchanged and every rank's partials of their union summed.  Every rank must
    return exactly the oracle's rules and final minsup.  recs = 64 lowers the
    batch-size thresholds (FSM_TSR_PAIR_RECS) so the item batches grow and
    shrink during the phase: every rank must size them alike."""
    from oracle import oracle
    from test_dist import run_ranks
    from tools import gen
    if recs != "default":
        monkeypatch.setenv("FSM_TSR_PAIR_RECS", recs)
    res = run_ranks(world, ["tsr", "8000", "120", "0.4"], tmp_path, timeout=110)
    ds = gen.kosarak(D=8000, seed=3)
    o = oracle.tsr(ds.records(), 120, 0.4)
    exp = sorted([list(x), list(y), s, c] for x, y, s, c in o["rules"])
    for r in res:
        assert r["rules"] == exp and r["final_minsup"] == o["final_minsup"]


@pytest.mark.parametrize("world,D,sup,ref", [(2, 20000, 0.003, "oracle"), (3, 20000, 0.003, "oracle"),
                                             (2, 200000, 0.002, "gpu1")])
def test_sharded_spade_two_ranks(eng, world, D, sup, ref, tmp_path):
    """The sharded SPADE path (F1 all-reduce, root rows split over ranks,
    frequent pairs all-gathered, first-level classes by shard plan, patterns
    all-gathered) with `world` ranks on this one GPU over gloo host
    collectives: every rank returns the complete, single-rank result."""
    from test_dist import run_ranks
    from tools import gen
    res = run_ranks(world, ["spade", str(D), str(sup), "1"], tmp_path, timeout=110)
    ds = gen.quest(D, seed=1)
    if ref == "oracle":
        from oracle import oracle
        o = oracle.spade_tokens(ds.seq_off, ds.tokens, sup)
        exp, joins = o["patterns"], o["joins"]
    else:
        pats, _, st = gpu_spade(eng, None, sup, tokens=ds)
        exp, joins = pats, st["joins"]
    for r in res:
        assert canon(r["patterns"]) == exp
        assert r["joins"] == joins
    assert sum(1 for _ in exp) > 100


@pytest.mark.parametrize("phase", ["root", "lattice"])
def test_sharded_spade_failure_reaches_every_rank(phase, tmp_path, monkeypatch):
    """A failure on one rank of a sharded mine (injected FSM_ELIMIT on rank 1)
    comes back as the same FSM_E* code on every rank instead of leaving the
    peers blocked in a collective."""
    from test_dist import run_ranks
    from spark_fsm_amd import FSM_ELIMIT
    monkeypatch.setenv("FSM_INJECT_FAIL", "1,%s" % phase)
    res = run_ranks(2, ["spade_fail", "20000", "0.003"], tmp_path, timeout=100)
    assert [r["code"] for r in res] == [FSM_ELIMIT, FSM_ELIMIT]
    assert "injected" in res[1]["msg"] and "peer rank failed" in res[0]["msg"]


def test_sharded_tsr_failure_reaches_every_rank(tmp_path, monkeypatch):
    """A failure on one rank of the sharded TSR pair phase (injected FSM_ELIMIT
    on rank 1) comes back as the same FSM_E* code on every rank instead of
    leaving the peer blocked in the key exchange."""
    from test_dist import run_ranks
    from spark_fsm_amd import FSM_ELIMIT
    monkeypatch.setenv("FSM_INJECT_FAIL", "1,pairs")
    res = run_ranks(2, ["tsr_fail", "6000", "100", "0.4"], tmp_path, timeout=100)
    assert [r["code"] for r in res] == [FSM_ELIMIT, FSM_ELIMIT]
    assert "injected" in res[1]["msg"] and "peer rank failed" in res[0]["msg"]


@pytest.mark.parametrize("bitmap", ["1", "0", "passes", "domain-bitmap", "domain-list", "max-kids", "max-pos",
                                    "plist-off", "dlmemo-off", "dlmemo-tiny", "ring-wrap",
                                    "ring-wrap-2sets", "ring-guard", "ring-guard-2sets"])
def test_tsr_expansion_domains_agree(eng, bitmap, monkeypatch):
    """TSR expansions over sid bitmaps (default: each slot's domain from the
    whole-bitmap AND or, for a rare item, from its sid list probed in the other
    bitmaps; domain-bitmap / domain-list force either for every slot; "passes":
    the LDS histograms cover 37 kids per pass, so every expansion runs several kid
    passes) and over the driver item's sid list (FSM_TSR_BITMAP=0, the over-budget
    fallback; max-kids: taken up front because the kept items exceed the cap;
    max-pos: taken after the rows were packed because an itemset index exceeds the
    cap) give the oracle's rules."""
    from oracle import oracle
    from tools import gen
    from spark_fsm_amd import MODE_TSR
    monkeypatch.setenv("FSM_TSR_BITMAP", "0" if bitmap == "0" else "1")
    if bitmap == "passes":
        monkeypatch.setenv("FSM_TSR_PASS_KIDS", "37")
    if bitmap.startswith("domain-"):
        monkeypatch.setenv("FSM_TSR_DOMAIN", bitmap.split("-")[1])
    if bitmap == "max-kids":
        monkeypatch.setenv("FSM_TSR_MAX_KIDS", "10")
    if bitmap == "max-pos":
        monkeypatch.setenv("FSM_TSR_MAX_POS", "3")
    # the replay's default-on features against the oracle, each off or at its edge: the kept-row
    # lists off; the |sids(X u {c})| memo off, or 16 entries (full after a few counts: probes run
    # out, most lookups miss); a 1 MiB kept-row ring
    # (65,536 entries) with 4 (or 2) launch sets in flight, so the head wraps the ring many times
    # and launches still in flight hold ring positions (finished early before an overwrite)
    if bitmap == "plist-off":
        monkeypatch.setenv("FSM_TSR_PLIST", "0")
    if bitmap == "dlmemo-off":
        monkeypatch.setenv("FSM_TSR_DLMEMO", "0")
    if bitmap == "dlmemo-tiny":
        monkeypatch.setenv("FSM_TSR_DLMEMO_LOG2", "4")
    # ring-guard: children read parent lists anywhere in the ring not yet overwritten (window
    # 16/16 instead of the default half), so a launch in flight can hold a position that a later
    # launch is about to overwrite: the guard must finish it first (fsm_stats.tsr_ring_waits > 0;
    # these two settings were found to fire it, tools/ring_probe.py) and the rules stay the oracle's
    if bitmap.startswith("ring-"):
        monkeypatch.setenv("FSM_TSR_ARENA_MB", "0.25" if bitmap == "ring-guard-2sets" else "1")
        monkeypatch.setenv("FSM_TSR_SETS", "2" if bitmap.endswith("2sets") else "4")
    if bitmap.startswith("ring-guard"):
        monkeypatch.setenv("FSM_TSR_PLIST_WINDOW", "16")
    ds = gen.kosarak(D=6000, seed=3)
    o = oracle.tsr(ds.records(), 300, 0.4)
    db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, MODE_TSR)  # bitmaps are built at upload
    try:
        rules, meta = eng.tsr(db, 300, 0.4)
    finally:
        db.free()
    rules.sort(key=lambda t: (-t[2], t[0], t[1]))
    assert rules == o["rules"] and meta["final_minsup"] == o["final_minsup"]
    if bitmap.startswith("ring-guard"):
        assert eng.stats()["tsr_ring_waits"] > 0


@pytest.mark.parametrize("batch", ["1", "7", "128", "768"])
@pytest.mark.parametrize("spb", ["default", "4", "100000"])
def test_tsr_batch_sizes_agree(eng, batch, spb, monkeypatch):
    """Rules expanded per launch (FSM_TSR_BATCH; 768: the wide batches c4-like
    DBs take, here on a DB whose pair phase ends at a low minsup) and the domain
    sids per expansion block (FSM_TSR_SPB: many small blocks, each slot in one
    block) change only how much runs ahead speculatively and how the partial
    histograms are split: the rules and final minsup stay the oracle's."""
    from oracle import oracle
    from tools import gen
    from spark_fsm_amd import MODE_TSR
    monkeypatch.setenv("FSM_TSR_BATCH", batch)
    if spb != "default":
        monkeypatch.setenv("FSM_TSR_SPB", spb)
    ds = gen.kosarak(D=5000, seed=6)
    o = oracle.tsr(ds.records(), 150, 0.5)
    db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, MODE_TSR)
    try:
        rules, meta = eng.tsr(db, 150, 0.5)
    finally:
        db.free()
    rules.sort(key=lambda t: (-t[2], t[0], t[1]))
    assert rules == o["rules"] and meta["final_minsup"] == o["final_minsup"]


@pytest.mark.parametrize("spec", ["0", "3,128", "8,16"])
@pytest.mark.parametrize("grid", ["128,8,512", "16,2,64"])
def test_tsr_speculation_and_grids_agree(eng, spec, grid, monkeypatch):
    """Child speculation (FSM_TSR_SPEC: off / default / deep-narrow) and the
    per-launch grids (FSM_TSR_GRID) change only which expansions run ahead and
    how they are split over blocks: the rules and final minsup stay the oracle's."""
    from oracle import oracle
    from tools import gen
    from spark_fsm_amd import MODE_TSR
    monkeypatch.setenv("FSM_TSR_SPEC", spec)
    monkeypatch.setenv("FSM_TSR_GRID", grid)
    ds = gen.kosarak(D=5000, seed=5)
    o = oracle.tsr(ds.records(), 200, 0.5)
    db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, MODE_TSR)
    try:
        rules, meta = eng.tsr(db, 200, 0.5)
    finally:
        db.free()
    rules.sort(key=lambda t: (-t[2], t[0], t[1]))
    assert rules == o["rules"] and meta["final_minsup"] == o["final_minsup"]


def test_ingested_files_mine_like_their_lines(eng):
    """§8f rows 2-4 end to end: a KOSARAK file converted by fsm_ingest goes
    straight to fsm_db_from_tokens (K0) and mines to the oracle's patterns /
    rules on the builder's "idx|seq" lines; the persisted documents of the
    engine's results equal the restatement's renderings of the oracle's."""
    import random
    from oracle import oracle, spmf_builder as ref
    from spark_fsm_amd import MODE_SPADE, MODE_TSR, PatternSet, RuleSet, ingest
    rng = random.Random(12)
    text = "".join(" ".join(str(rng.randint(1, 40)) for _ in range(rng.randint(1, 12))) + "\n" for _ in range(3000))
    t = ingest(text.encode(), "KOSARAK")
    recs = [(int(l.split("|")[0]), l.split("|", 1)[1]) for l in ref.build(text, "KOSARAK", 10 ** 9)]
    db = eng.db_from_tokens(t.sids, t.seq_off, t.tokens, MODE_SPADE)
    try:
        csr, meta = eng.spade_csr(db, 0.02)
    finally:
        db.free()
    o = oracle.spade(recs, 0.02)
    ps = PatternSet.from_csr(csr, meta)
    got = sorted(ps.serialize().splitlines())
    exp = sorted(ref.patterns_serialize([(s, [list(x) for x in sets]) for sets, s in o["patterns"]]).splitlines())
    assert got == exp and meta["minsup"] == o["minsup"]
    db = eng.db_from_tokens(t.sids, t.seq_off, t.tokens, MODE_TSR)
    try:
        rules, rmeta = eng.tsr(db, 60, 0.3)
    finally:
        db.free()
    rules.sort(key=lambda r: (-r[2], r[0], r[1]))
    ot = oracle.tsr(recs, 60, 0.3)
    assert rules == ot["rules"]
    assert RuleSet(rules, rmeta["total"]).to_json() == ref.rules_json(ot["rules"], ot["total"])


def test_rule_queries_on_gpu_mined_rules(eng):
    """§8f row 4 (FSMQuestor.scala:46-98, get:antecedent / get:consequent) on rules the
    GPU mined: a Kosarak-shaped prefix mined by fsm_tsr_mine (rules identical to the
    oracle's), then fsm_rules_query on the library's own fsm_rules (no copy) for random
    item sets of both sides, against the restatement (oracle/spmf_builder.rules_query)
    over the same rules in the same order; the json4s document as well."""
    import random
    from oracle import oracle, spmf_builder as ref
    from spark_fsm_amd import MODE_TSR
    from tools import gen
    ds = gen.kosarak(D=5000, seed=1)
    recs = ds.records()
    db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, MODE_TSR)
    try:
        mr = eng.tsr_mined(db, 300, 0.5)
    finally:
        db.free()
    rules = mr.rules()
    o = oracle.tsr(recs, 300, 0.5)
    assert sorted(rules, key=lambda t: (-t[2], t[0], t[1])) == o["rules"]
    assert mr.final_minsup == o["final_minsup"] and mr.total == 5000 and len(rules) >= 300
    rng = random.Random(8)
    items = sorted({i for x, y, _, _ in rules for i in x + y})
    hits = 0
    for _ in range(80):
        q = rng.sample(items, rng.randint(0, min(len(items), 25))) + [rng.randint(1, 41270) for _ in range(3)]
        for side in (0, 1):
            got = mr.query(side, q)
            assert got == ref.rules_query(rules, side, q)
            hits += len(got)
    assert hits > 0  # the queries do select rules
    assert mr.query(0, []) == [] and mr.query(1, items) == list(range(len(rules)))
    assert mr.to_json() == ref.rules_json(rules, mr.total)


@pytest.mark.parametrize("devices", [(0, 0), (0, 0, 0)])
def test_inproc_ranks_random_vs_oracle(fsm, devices):
    """In-process ranks (fsm_opts.ndevices: one context, rank r on devices[r] as a thread of
    this process, the drop-in's way to shard) on random SPMF-text DBs and Quest tokens:
    the patterns / rules and thresholds of the oracle, and the join count."""
    from oracle import oracle
    from tools import gen
    rng = random.Random(31 + len(devices))
    with fsm.Engine(devices=list(devices)) as e:
        for it in range(20):
            recs = rand_records(rng, rng.randint(8, 60), rng.randint(2, 12), 6, 3, ts=it % 2 == 0)
            sup = rng.choice([0.15, 0.2, 0.3, 0.5])
            o = oracle.spade(recs, sup)
            pats, _, st = gpu_spade(e, recs, sup)
            assert pats == o["patterns"], (it, recs, sup)
            assert st["joins"] == o["joins"]
        for it in range(10):
            recs = rand_records(rng, rng.randint(2, 60), rng.randint(2, 12), 6, 3, ts=False)
            if not any(t not in ("-1", "-2") for _, l in recs for t in l.split(" ")):
                continue
            k, mc = rng.randint(1, 40), rng.choice([0.0, 0.2, 0.5, 0.9])
            o = oracle.tsr(recs, k, mc)
            rules, meta, _ = gpu_tsr(e, recs, k, mc)
            assert rules == o["rules"], (it, recs, k, mc)
            assert meta["final_minsup"] == o["final_minsup"]
        ds = gen.quest(20000, seed=2)
        o = oracle.spade_tokens(ds.seq_off, ds.tokens, 0.003)
        pats, meta, st = gpu_spade(e, None, 0.003, tokens=ds)
        assert meta["minsup"] == o["minsup"] and pats == o["patterns"] and st["joins"] == o["joins"]
