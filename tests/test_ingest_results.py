"""SURVEY §8f rows 2-4 on the CPU: libfsm's native SPMFBuilder conversion
(fsm_ingest), result persistence (fsm_patterns_serialize / _json,
fsm_rules_json) and rule queries (fsm_rules_query) against the pure-Python
restatement in oracle/spmf_builder.py ("parity unpinned": the reference holds
no fixtures for these paths, see that file's header).  No GPU is needed: these
entry points never touch the device.  The GPU side (ingested tokens mined
through the engine equal the SPMF-line path) is in tests/test_parity_gpu.py.
"""
import json
import random

import pytest

from oracle import spmf_builder as ref


@pytest.fixture(scope="module")
def fsm():
    import spark_fsm_amd
    return spark_fsm_amd


def native_build(fsm, text, fmt, limit):
    try:
        return fsm.spmf_build(text.encode(), fmt, limit)
    except fsm.FsmParseError:
        return "error"


def oracle_build(text, fmt, limit):
    try:
        return ref.build(text, fmt, limit)
    except ref.BuilderError:
        return "error"


HAND = {
    "CSV": ["1,2,3\n4,5\n", "1,2,3", "7\r\n8,9\r\n", "1\r2\r", "", "\n", "1,,2\n", "1,2,\n", ",1\n",
            "+5,-3\n", "2147483647\n", "2147483648\n", "-2147483648\n", " 1\n", "1\n\n2\n", "a\n", "1,2\n3,x\n"],
    "KOSARAK": ["1 2 3\n4 5\n", "1  2\n", "1 2 \n", " 1\n", "10\n20 30 40\n", "1\t2\n", "007 -0\n"],
    "BMS": ["1\t10\n2\t20\n1\t11\n", " 3 \t 5 \n3\t6\n", "1\t\n", "1\n", "1\t2\t3\n", "x\t1\n", "1\t2\n\n",
            "5\t1\n4\t2\n5\t3\n4\t4\n"],
    "SNAKE": ["ABCDEFGHIJK\nAB\nABCDEFGHIJKLMNOP\n", "short\n", "abcdefghijkl\n", "ZZZZZZZZZZZ\r\n", "           \n"],
    "SPMF": ["1 -1 2 -1 -2\n3 -1 -2\n", "<1> 1 -1 -2\n", "", "x y\n"],
}


@pytest.mark.parametrize("fmt", sorted(HAND))
def test_builder_hand_cases(fsm, fmt):
    for text in HAND[fmt]:
        for limit in (0, 1, 2, 1000):
            assert native_build(fsm, text, fmt, limit) == oracle_build(text, fmt, limit), (fmt, text, limit)


def test_builder_unknown_format_is_none(fsm):
    assert fsm.spmf_build(b"1,2\n", "PARQUET") is None and ref.build("1,2\n", "PARQUET") is None


def _random_text(rng, fmt):
    n = rng.randint(0, 40)
    rows = []
    for _ in range(n):
        if fmt == "BMS":
            rows.append("%d\t%d" % (rng.randint(0, 8), rng.randint(-3, 500)))
        elif fmt == "SNAKE":
            rows.append("".join(chr(rng.randint(65, 90)) for _ in range(rng.randint(5, 20))))
        else:
            sep = "," if fmt == "CSV" else " "
            rows.append(sep.join(str(rng.randint(-5, 2000)) for _ in range(rng.randint(1, 12))))
    if rows and rng.random() < 0.2:  # one malformed line somewhere
        i = rng.randrange(len(rows))
        rows[i] = rows[i] + rng.choice([",", ",,1", " x", "\t", "99999999999"])
    eol = rng.choice(["\n", "\r\n", "\r"])
    return eol.join(rows) + (eol if rng.random() < 0.7 else "")


@pytest.mark.parametrize("fmt", ["BMS", "CSV", "KOSARAK", "SNAKE", "SPMF"])
def test_builder_random_files(fsm, fmt):
    rng = random.Random(sum(map(ord, fmt)))
    for _ in range(150):
        text = _random_text(rng, "KOSARAK" if fmt == "SPMF" else fmt)
        if fmt == "SPMF":
            text = text.replace(" ", " -1 ")
        limit = rng.choice([0, 1, 3, 10, 1000])
        assert native_build(fsm, text, fmt, limit) == oracle_build(text, fmt, limit), (fmt, text, limit)


def test_error_past_the_limit_still_fails(fsm):
    """file.count (SPMFBuilder.scala:192) converts every line: a bad line after
    the kept ones fails the build (except SPMF, whose lines stay unparsed)."""
    with pytest.raises(fsm.FsmParseError, match="line 3"):
        fsm.ingest(b"1,2\n3\n4,x\n", "CSV", limit=1)
    assert len(fsm.ingest(b"1 -1 -2\nx y\n", "SPMF", limit=1)) == 1


def test_ingest_tokens_mine_like_the_lines(fsm):
    """ingest() tokens (the engine-facing form) and the builder's strings are the
    same DB: the oracle mines them to the same patterns."""
    from oracle import oracle
    rng = random.Random(7)
    rows = [" ".join(str(rng.randint(1, 30)) for _ in range(rng.randint(1, 10))) for _ in range(300)]
    text = "\n".join(rows) + "\n"
    t = fsm.ingest(text.encode(), "KOSARAK")
    lines = ref.build(text, "KOSARAK", 10 ** 9)
    recs = [(int(l.split("|")[0]), l.split("|", 1)[1]) for l in lines]
    assert t.records() == recs
    a = oracle.spade(recs, 0.05)
    b = oracle.spade_tokens(t.seq_off, t.tokens, 0.05)
    assert a["patterns"] == b["patterns"] and a["minsup"] == b["minsup"]


def test_indexed_reads_the_builder_output(fsm, tmp_path):
    out = tmp_path / "spmf"
    lines = fsm.spmf_build(b"5,6\n7\n8,9,10\n", "CSV", output=str(out))
    assert (out / "part-00000").read_text() == "".join(l + "\n" for l in lines)
    t = fsm.ingest(str(out), "INDEXED")
    assert t.lines() == lines
    with pytest.raises(fsm.FsmParseError):
        fsm.ingest(b"no bar here\n", "INDEXED")
    with pytest.raises(fsm.FsmParseError, match="fsm_db_from_spmf"):
        fsm.ingest(b"1 -01 -2\n", "SPMF")  # "-01" is an item to the miners' text parsers


# ------------------------------------------------------------- persistence


def _random_patterns(rng, n):
    pats = []
    for _ in range(n):
        sets = [sorted(rng.sample(range(0, 60), rng.randint(1, 4))) for _ in range(rng.randint(1, 5))]
        pats.append((rng.randint(1, 10 ** 6), sets))
    return pats


def test_patterns_documents(fsm):
    rng = random.Random(3)
    for n in (0, 1, 17, 400):
        pats = _random_patterns(rng, n)
        ps = fsm.PatternSet.from_list([(tuple(map(tuple, sets)), s) for s, sets in pats], total=1000, minsup=3)
        assert ps.serialize() == ref.patterns_serialize(pats)
        js = ps.to_json()
        assert js == ref.patterns_json(pats)
        assert json.loads(js) == {"items": [{"support": s, "itemsets": sets} for s, sets in pats]}
        # SPADEActor's own parse of serialize() (SPADEActor.scala:47-58) gives the document back
        objs = [fsm.Pattern(tuple(map(tuple, sets)), s) for s, sets in pats]
        assert fsm.spade_actor_patterns(objs) == [(s, sets) for s, sets in pats]
    neg = [(4, [[-7, 3], [2]])]  # TSR / SPADE items may be negative: rendered as ints
    assert fsm.PatternSet.from_list([(((-7, 3), (2,)), 4)]).to_json() == ref.patterns_json(neg)


JAVA_DOUBLES = [(0.5, "0.5"), (2 / 3, "0.6666666666666666"), (1.0, "1.0"), (1e-4, "1.0E-4"), (0.001, "0.001"),
                (1e7, "1.0E7"), (1234567.0, "1234567.0"), (0.1 + 0.2, "0.30000000000000004"),
                (123456789.0, "1.23456789E8"), (100.0, "100.0"), (0.000123, "1.23E-4"), (1 / 3, "0.3333333333333333"),
                (0.0, "0.0"), (9999999.999, "9999999.999"), (1.7976931348623157e308, "1.7976931348623157E308")]


def test_rules_document_and_java_doubles(fsm):
    for d, s in JAVA_DOUBLES:
        assert ref.java_double(d) == s, d
        rs = fsm.RuleSet([((1,), (2,), 1, d)], total=5)
        assert json.loads(rs.to_json())["items"][0]["confidence"] == d
        assert rs.to_json().endswith('"confidence":%s}]}' % s), (d, rs.to_json())
    rng = random.Random(11)
    for n in (0, 1, 50, 500):
        rules = []
        for _ in range(n):
            x = tuple(sorted(rng.sample(range(100), rng.randint(1, 3))))
            y = tuple(sorted(rng.sample(range(100, 200), rng.randint(1, 3))))
            sup = rng.randint(1, 1000)
            rules.append((x, y, sup, sup / rng.randint(sup, 3000)))
        rs = fsm.RuleSet(rules, total=3000, final_minsup=1)
        assert rs.to_json() == ref.rules_json(rules, 3000)
        got = json.loads(rs.to_json())["items"]
        assert [(tuple(g["antecedent"]), tuple(g["consequent"]), g["support"], g["confidence"]) for g in got] == rules
        assert all(g["total"] == 3000 for g in got)


def test_rule_queries(fsm):
    rng = random.Random(5)
    rules = []
    for _ in range(300):
        x = tuple(sorted(rng.sample(range(12), rng.randint(1, 3))))
        y = tuple(sorted(rng.sample(range(12, 24), rng.randint(1, 3))))
        rules.append((x, y, rng.randint(1, 50), 0.5))
    rs = fsm.RuleSet(rules, total=100)
    for _ in range(60):
        q = rng.sample(range(24), rng.randint(0, 10))
        assert rs.by_antecedent(q) == [rules[i] for i in ref.rules_query(rules, 0, q)]
        assert rs.by_consequent(q) == [rules[i] for i in ref.rules_query(rules, 1, q)]
    assert fsm.RuleSet([], total=0).by_antecedent([1]) == []
