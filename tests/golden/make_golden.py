"""Regenerate the committed golden fixtures in tests/golden/.

The reference ships no tests, fixtures or known-answer vectors (SURVEY.md §4,
§8c) and cannot be run here (no JVM; its miners are unvendored), so these
fixtures are produced from the published definitions:

  spade_cases.json  expected patterns = oracle/brute.py's definitional
                    enumeration (independent of the C restatement); the C
                    restatement must agree (asserted here); "joins" = SURVEY
                    A.2 candidate count from the restatement.
  tsr_cases.json    expected rules = the C restatement's exact top-k (its tie
                    boundary follows the restated SPMF control flow); asserted
                    here against brute.py's definitional invariants.
  error_cases.json  inputs on which the reference throws (parse rules of
                    SPADE.scala:145-212, TSR.scala:41,109-143).

Run:  python tests/golden/make_golden.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import brute, oracle  # noqa: E402


def rand_db(rng, nseq, nitems, maxsets, maxset, ts=False, dup_sids=False, trailing=True):
    recs = []
    for s in range(nseq):
        toks = []
        for _ in range(rng.randint(0, maxsets)):
            if ts and rng.random() < 0.3:
                toks.append("<%d>" % rng.randint(0, 6))
            for _ in range(rng.randint(1, maxset)):
                toks.append(str(rng.randint(1, nitems)))
            toks.append("-1")
        if trailing and rng.random() < 0.2:
            toks.append(str(rng.randint(1, nitems)))
        toks.append("-2")
        sid = rng.randint(0, max(0, nseq - 2)) if dup_sids and rng.random() < 0.3 else s
        recs.append((sid, " ".join(toks)))
    return recs


SPMF_EXAMPLE = [
    (0, "1 -1 1 2 3 -1 1 3 -1 4 -1 3 6 -1 -2"),
    (1, "1 4 -1 3 -1 2 3 -1 1 5 -1 -2"),
    (2, "5 6 -1 1 2 -1 4 6 -1 3 -1 2 -1 -2"),
    (3, "5 -1 7 -1 1 6 -1 3 -1 2 -1 3 -1 -2"),
]

LONG = [(0, " ".join(["1 -1"] * 40 + ["2 -1"] * 30 + ["-2"])),
        (1, " ".join(["1 -1"] * 40 + ["2 -1"] * 30 + ["-2"])),
        (2, "1 -1 2 -1 -2")]


def spade_cases():
    cases = [
        ("spmf_example_s50", SPMF_EXAMPLE, 0.5),
        ("spmf_example_s25", SPMF_EXAMPLE, 0.25),
        ("spmf_example_s100", SPMF_EXAMPLE, 1.0),
        ("timestamps", [(0, "<1> 1 -1 <3> 2 -1 -2"), (1, "<0> 2 -1 <5> 1 2 -1 -2"),
                        (2, "1 -1 <0> 2 -1 -2"), (3, "<2> 1 -1 <2> 3 -1 2 -1 -2")], 0.25),
        ("duplicate_sids", [(0, "1 -1 2 -1"), (0, "3 -1"), (1, "1 -1 2 -1"), (1, "1 3 -1"), (5, "3 -1 1 -1")], 0.3),
        ("trailing_and_empty", [(0, "1 -1 2"), (1, " "), (2, "1 -1 2 -1 3"), (3, "2 -1 1 -1 -2"),
                                (4, "1 2 -1 1 -1 -2 "), (5, "-2")], 0.2),
        ("signed_items", [(0, "+1 -1 -5 -1 -2"), (1, "-5 -1 1 -1 -2"), (2, "-5 1 -1 -2"), (3, "007 -1 -5 -1")], 0.5),
        ("repeated_items", [(0, "1 1 -1 1 -1 -2"), (1, "1 -1 1 -1 1 -1 -2"), (2, "1 2 -1 2 1 -1 -2")], 0.6),
        ("empty_itemsets", [(0, "-1 5 -1 -1 6 -1 -2"), (1, "5 -1 6 -1"), (2, "-1 -1 -2")], 0.5),
        ("support_zero", [(0, "1 -1 2 -1"), (1, "2 -1 1 -1")], 0.0),
        ("support_above_one", [(0, "1 -1 2 -1"), (1, "2 -1 1 -1")], 1.5),
        ("long_sequences_W2", LONG, 0.6),
    ]
    rng = random.Random(20260101)
    for k in range(24):
        recs = rand_db(rng, rng.randint(2, 12), rng.randint(2, 6), 5, 3, ts=(k % 3 == 0), dup_sids=(k % 4 == 1))
        cases.append(("random_%02d" % k, recs, rng.choice([0.1, 0.2, 0.3, 0.5, 0.7])))
    out = []
    for name, recs, sup in cases:
        b = brute.brute_spade(recs, sup)
        o = oracle.spade(recs, sup)
        assert o["patterns"] == b, name
        out.append({"name": name, "records": recs, "support": sup, "minsup": o["minsup"],
                    "joins": o["joins"], "patterns": [[list(map(list, p)), s] for p, s in b]})
    return out


TSR_EXAMPLE = [
    (0, "1 -1 2 -1 3 -1 4 -1 6 -1 -2"),
    (1, "1 -1 4 -1 3 -1 5 -1 6 -1 -2"),
    (2, "1 -1 2 -1 3 -1 5 -1 6 -1 -2"),
    (3, "2 -1 3 -1 4 -1 7 -1 -2"),
    (4, "1 -1 3 -1 4 -1 5 -1 6 -1 -2"),
    (5, "2 -1 1 -1 3 -1 6 -1 -2"),
]


def tsr_cases():
    cases = [
        ("example_k5_c50", TSR_EXAMPLE, 5, 0.5),
        ("example_k1_c0", TSR_EXAMPLE, 1, 0.0),
        ("example_k20_c80", TSR_EXAMPLE, 20, 0.8),
        ("example_k1000_c50", TSR_EXAMPLE, 1000, 0.5),
        ("multi_item_itemsets", [(0, "1 2 -1 3 -1 -2"), (1, "1 -1 2 3 -1 -2"), (2, "2 -1 1 3 -1 4 -1 -2"),
                                 (3, "1 2 3 -1 -2")], 4, 0.3),
        ("trailing_and_empty", [(0, "1 -1 2 -1 9"), (1, " "), (2, "1 -1 -1 2 -1 -2"), (3, "-2")], 3, 0.1),
        ("ties", [(0, "1 -1 2 -1"), (1, "3 -1 4 -1"), (2, "5 -1 6 -1"), (3, "1 -1 2 -1 3 -1 4 -1")], 2, 0.5),
    ]
    rng = random.Random(7)
    for k in range(20):
        recs = rand_db(rng, rng.randint(2, 9), rng.randint(2, 5), 5, 2)
        if not any(int(t) > -1 for _, l in recs for t in l.split(" ") if t):
            continue
        cases.append(("random_%02d" % k, recs, rng.randint(1, 8), rng.choice([0.0, 0.3, 0.5, 0.8])))
    out = []
    for name, recs, k, mc in cases:
        o = oracle.tsr(recs, k, mc)
        brute.check_tsr(o["rules"], brute.brute_tsr_valid(recs, mc), k)
        out.append({"name": name, "records": recs, "k": k, "minconf": mc, "final_minsup": o["final_minsup"],
                    "rules": [[list(x), list(y), s, c] for x, y, s, c in o["rules"]]})
    return out


def error_cases():
    spade = [
        ("empty_line", [(0, "1 -1"), (1, "")]),
        ("double_space", [(0, "1  -1")]),
        ("leading_space", [(0, " 1 -1")]),
        ("bad_item", [(0, "1 -1 x -1")]),
        ("item_overflow", [(0, "2147483648 -1")]),
        ("bad_timestamp", [(0, "<x> 1 -1")]),
        ("lone_lt", [(0, "< 1 -1")]),
        ("negative_timestamp", [(0, "1 <-3> -1 2 -1")]),
        ("negative_sid", [(-1, "1 -1")]),
    ]
    tsr = [
        ("empty_line", [(0, "")]),
        ("timestamp_token", [(0, "<1> 1 -1")]),
        ("not_dense_sids", [(1, "1 -1"), (2, "2 -1")]),
        ("negative_item", [(0, "-5 -1")]),
        ("minus_zero_one", [(0, "-01 -1")]),
        ("no_items", [(0, "-2"), (1, "-1 -2")]),
        ("double_space", [(0, "1  -1")]),
    ]
    for name, recs in spade:
        try:
            oracle.spade(recs, 0.5)
            raise AssertionError("expected error " + name)
        except oracle.OracleError:
            pass
    for name, recs in tsr:
        try:
            oracle.tsr(recs, 3, 0.5)
            raise AssertionError("expected error " + name)
        except oracle.OracleError:
            pass
    return {"spade": [{"name": n, "records": r} for n, r in spade],
            "tsr": [{"name": n, "records": r} for n, r in tsr]}


def main():
    for fname, data in (("spade_cases.json", spade_cases()), ("tsr_cases.json", tsr_cases()),
                        ("error_cases.json", error_cases())):
        with open(os.path.join(HERE, fname), "w") as f:
            json.dump(data, f, indent=0, sort_keys=True)
        print("wrote", fname)


if __name__ == "__main__":
    main()
