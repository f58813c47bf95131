"""CPU tests: the CPU restatement (oracle/) against the committed golden
fixtures and against the independent brute-force enumerator.  No GPU."""
import json
import os
import random

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from oracle import brute, oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def canon_patterns(pats):
    return [(tuple(tuple(s) for s in p), sup) for p, sup in pats]


@pytest.mark.parametrize("case", load("spade_cases.json"), ids=lambda c: c["name"])
def test_oracle_spade_golden(case):
    recs = [tuple(r) for r in case["records"]]
    o = oracle.spade(recs, case["support"])
    assert o["patterns"] == canon_patterns(case["patterns"])
    assert o["minsup"] == case["minsup"]
    assert o["joins"] == case["joins"]


@pytest.mark.parametrize("case", load("tsr_cases.json"), ids=lambda c: c["name"])
def test_oracle_tsr_golden(case):
    recs = [tuple(r) for r in case["records"]]
    o = oracle.tsr(recs, case["k"], case["minconf"])
    exp = [(tuple(x), tuple(y), s, c) for x, y, s, c in case["rules"]]
    assert o["rules"] == exp
    assert o["final_minsup"] == case["final_minsup"]
    brute.check_tsr(o["rules"], brute.brute_tsr_valid(recs, case["minconf"]), case["k"])


ERR = load("error_cases.json")


@pytest.mark.parametrize("case", ERR["spade"], ids=lambda c: c["name"])
def test_oracle_spade_errors(case):
    with pytest.raises(oracle.OracleError):
        oracle.spade([tuple(r) for r in case["records"]], 0.5)


@pytest.mark.parametrize("case", ERR["tsr"], ids=lambda c: c["name"])
def test_oracle_tsr_errors(case):
    with pytest.raises(oracle.OracleError):
        oracle.tsr([tuple(r) for r in case["records"]], 3, 0.5)


def test_java_split_semantics():
    assert brute.java_split_space("") == [""]
    assert brute.java_split_space(" ") == []
    assert brute.java_split_space("1 -1  ") == ["1", "-1"]
    assert brute.java_split_space(" 1") == ["", "1"]
    # trailing spaces are legal for the reference, a leading one is not
    assert oracle.spade([(0, "1 -1 2 -1   ")], 1.0)["patterns"] == [(((1,),), 1), (((1,), (2,)), 1), (((2,),), 1)]


def test_threshold_is_ceil_of_support_times_total():
    recs = [(i, "1 -1") for i in range(3)] + [(3, "2 -1")]
    # ceil(0.5 * 4) = 2 ; ceil(0.26 * 4) = ceil(1.04) = 2 ; ceil(0.25*4) = 1
    assert oracle.spade(recs, 0.26)["minsup"] == 2
    assert oracle.spade(recs, 0.25)["minsup"] == 1
    assert [p for p, _ in oracle.spade(recs, 0.26)["patterns"]] == [((1,),)]


records_st = st.lists(
    st.lists(st.lists(st.integers(1, 4), min_size=1, max_size=3), min_size=0, max_size=4),
    min_size=1, max_size=7)


def _render(db, ts_every=0):
    out = []
    for s, seq in enumerate(db):
        toks = []
        for k, iset in enumerate(seq):
            if ts_every and k % ts_every == 1:
                toks.append("<%d>" % (k * 2 % 5))
            toks += [str(i) for i in iset] + ["-1"]
        out.append((s, " ".join(toks + ["-2"])))
    return out


@settings(max_examples=60, deadline=None)
@given(records_st, st.sampled_from([0.0, 0.2, 0.34, 0.5, 0.75, 1.0]), st.integers(0, 3))
def test_oracle_spade_matches_brute(db, support, ts_every):
    recs = _render(db, ts_every)
    assert oracle.spade(recs, support)["patterns"] == brute.brute_spade(recs, support)


@settings(max_examples=60, deadline=None)
@given(records_st, st.integers(1, 6), st.sampled_from([0.0, 0.25, 0.5, 0.9]))
def test_oracle_tsr_invariants(db, k, minconf):
    recs = _render(db)
    if not any(db):
        with pytest.raises(oracle.OracleError):
            oracle.tsr(recs, k, minconf)
        return
    o = oracle.tsr(recs, k, minconf)
    brute.check_tsr(o["rules"], brute.brute_tsr_valid(recs, minconf), k)


def test_oracle_deterministic_on_quest_sample():
    from tools import gen
    ds = gen.quest(2000, seed=3)
    recs = ds.records()
    a = oracle.spade(recs, 0.01)
    b = oracle.spade(list(reversed(recs)), 0.01)  # record order must not matter
    assert a["patterns"] == b["patterns"] and a["joins"] == b["joins"]
    assert len(a["patterns"]) > 50


def test_tsr_random_orders_are_definitional():
    rng = random.Random(5)
    for _ in range(20):
        db = [[[rng.randint(1, 5)] for _ in range(rng.randint(1, 6))] for _ in range(rng.randint(2, 8))]
        recs = _render(db)
        k = rng.randint(1, 10)
        mc = rng.choice([0.0, 0.5])
        brute.check_tsr(oracle.tsr(recs, k, mc)["rules"], brute.brute_tsr_valid(recs, mc), k)


def test_oracle_all_cores_mode_matches_single_thread():
    """CPU baseline mode ii: first-level classes on OpenMP threads
    must give the single-thread result (patterns, supports, join count)."""
    from tools import gen
    ds = gen.quest(3000, seed=4)
    a = oracle.spade_tokens(ds.seq_off, ds.tokens, 0.01)
    b = oracle.spade_tokens(ds.seq_off, ds.tokens, 0.01, threads=4)
    assert a["complete"] and b["complete"]
    assert a["joins"] == b["joins"] and a["patterns"] == b["patterns"]
    assert a["n_patterns"] > 50


def test_tsr_negative_item_only_fails_in_closed_itemsets():
    """TSR.scala:63-75 index the Vertical arrays with the items of closed
    itemsets only; the unclosed trailing itemset is dropped by newSequence."""
    from oracle import oracle
    r = oracle.tsr([(0, "1 -1 2 -1 -5 -2"), (1, "1 -1 2 -1 3"), (2, "1 2 -1 -7")], 3, 0.5)
    assert r["rules"] == [((1,), (2,), 2, 2 / 3)]
    with pytest.raises(oracle.OracleError):
        oracle.tsr([(0, "1 -1 -5 -1")], 3, 0.5)



def _tokens(db):
    so, tk = [0], []
    for seq in db:
        for iset in seq:
            tk += list(iset) + [-1]
        tk.append(-2)
        so.append(len(tk))
    return np.array(so, dtype=np.int64), np.array(tk, dtype=np.int64)


@settings(max_examples=80, deadline=None)
@given(records_st, st.integers(1, 3), st.sampled_from([0.0, 0.3, 0.5, 1.0]))
def test_tsr_exhaustive_matches_brute(db, t, minconf):
    """oracle/tsr_exhaustive.c (the c4 completeness pin) is the definitional
    set: every valid rule with sup >= t, exactly as brute force enumerates it."""
    if not any(db):
        return
    so, tk = _tokens(db)
    got = oracle.tsr_all(so, tk, t, minconf, threads=2)["rules"]
    valid = brute.brute_tsr_valid(_render(db), minconf)
    exp = sorted([(x, y, s, c) for (x, y), (s, c) in valid.items() if s >= t], key=lambda r: (-r[2], r[0], r[1]))
    assert got == exp


def test_tsr_exhaustive_pins_the_topk_result_on_a_prefix():
    """On the 5,000-sequence Kosarak prefix the top-k restatement's result R and
    the fixed-threshold enumeration at R's final minsup m agree as SURVEY
    §8(c)(ii) requires: the valid rules with sup > m are exactly R's, and every
    rule of R is valid with the definitional sup / conf."""
    from tools import gen
    ds = gen.kosarak(D=990002, seed=1).head(5000)
    r = oracle.tsr(ds.records(), 1000, 0.5)
    m = r["final_minsup"]
    a = oracle.tsr_all(ds.seq_off, ds.tokens, m, 0.5, threads=4)
    R = {(x, y): (s, c) for x, y, s, c in r["rules"]}
    A = {(x, y): (s, c) for x, y, s, c in a["rules"]}
    assert {k: v for k, v in A.items() if v[0] > m} == {k: v for k, v in R.items() if v[0] > m}
    assert all(A.get(k) == v for k, v in R.items())
    assert len(R) >= 1000
