"""ctypes wrapper for the CPU restatement in oracle/fsm_oracle.c.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.  Parity status:
"parity unpinned" against the reference (its mining modules are unvendored and
it has no tests); pinned to the published definitions by
oracle/brute.py on the fixtures in tests/golden/.

Outputs are canonical:
  spade() -> patterns sorted by their itemsets (tuple of ascending tuples)
  tsr()   -> rules sorted by (-support, antecedent, consequent)
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")


class OracleError(RuntimeError):
    """The restated reference raised (parse error, invalid parameter, ...)."""


class _Patterns(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int64),
        ("support", ctypes.POINTER(ctypes.c_int32)),
        ("pat_off", ctypes.POINTER(ctypes.c_int64)),
        ("set_off", ctypes.POINTER(ctypes.c_int64)),
        ("items", ctypes.POINTER(ctypes.c_int32)),
        ("n_sets", ctypes.c_int64),
        ("n_items", ctypes.c_int64),
        ("joins", ctypes.c_int64),
        ("minsup", ctypes.c_int32),
        ("complete", ctypes.c_int32),
        ("seconds", ctypes.c_double),
        ("seconds_f1", ctypes.c_double),
    ]


class _Rules(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int64),
        ("support", ctypes.POINTER(ctypes.c_int32)),
        ("confidence", ctypes.POINTER(ctypes.c_double)),
        ("ante_off", ctypes.POINTER(ctypes.c_int64)),
        ("ante", ctypes.POINTER(ctypes.c_int32)),
        ("cons_off", ctypes.POINTER(ctypes.c_int64)),
        ("cons", ctypes.POINTER(ctypes.c_int32)),
        ("total", ctypes.c_int64),
        ("expansions", ctypes.c_int64),
        ("final_minsup", ctypes.c_int32),
        ("complete", ctypes.c_int32),
        ("seconds", ctypes.c_double),
        ("pairs", ctypes.c_int64),
    ]


_lib = None


def build():
    """Compile liboracle.so (gcc) if it is missing or stale."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_spade.argtypes = [
            ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_char_p),
            ctypes.POINTER(ctypes.c_int64), ctypes.c_int64, ctypes.c_double,
            ctypes.POINTER(ctypes.POINTER(_Patterns)), ctypes.c_char_p, ctypes.c_int]
        L.oracle_spade.restype = ctypes.c_int
        L.oracle_patterns_free.argtypes = [ctypes.POINTER(_Patterns)]
        I64P = ctypes.POINTER(ctypes.c_int64)
        L.oracle_spade_tokens.argtypes = [I64P, I64P, ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                                          ctypes.POINTER(ctypes.POINTER(_Patterns)), ctypes.c_char_p, ctypes.c_int]
        L.oracle_spade_tokens.restype = ctypes.c_int
        L.oracle_spade_tokens_mt.argtypes = [I64P, I64P, ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                                             ctypes.c_int, ctypes.POINTER(ctypes.POINTER(_Patterns)),
                                             ctypes.c_char_p, ctypes.c_int]
        L.oracle_spade_tokens_mt.restype = ctypes.c_int
        L.oracle_spade_tokens_sample.argtypes = [I64P, I64P, ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                                                 ctypes.c_int, ctypes.c_int64, ctypes.POINTER(ctypes.POINTER(_Patterns)),
                                                 ctypes.c_char_p, ctypes.c_int]
        L.oracle_spade_tokens_sample.restype = ctypes.c_int
        L.oracle_pattern_support.argtypes = [I64P, I64P, ctypes.c_int64, ctypes.POINTER(ctypes.c_int32),
                                             I64P, ctypes.c_int64]
        L.oracle_pattern_support.restype = ctypes.c_int64
        L.oracle_rule_support.argtypes = [I64P, I64P, ctypes.c_int64, ctypes.POINTER(ctypes.c_int32),
                                          ctypes.c_int64, ctypes.POINTER(ctypes.c_int32), ctypes.c_int64, I64P, I64P]
        L.oracle_rule_support.restype = None
        L.oracle_tsr.argtypes = [
            ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_char_p),
            ctypes.POINTER(ctypes.c_int64), ctypes.c_int64, ctypes.c_int32, ctypes.c_double,
            ctypes.POINTER(ctypes.POINTER(_Rules)), ctypes.c_char_p, ctypes.c_int]
        L.oracle_tsr.restype = ctypes.c_int
        L.oracle_tsr_timed.argtypes = [
            ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_char_p),
            ctypes.POINTER(ctypes.c_int64), ctypes.c_int64, ctypes.c_int32, ctypes.c_double, ctypes.c_double,
            ctypes.POINTER(ctypes.POINTER(_Rules)), ctypes.c_char_p, ctypes.c_int]
        L.oracle_tsr_timed.restype = ctypes.c_int
        L.oracle_rules_free.argtypes = [ctypes.POINTER(_Rules)]
        L.oracle_tsr_all.argtypes = [I64P, I64P, ctypes.c_int64, ctypes.c_int32, ctypes.c_double, ctypes.c_int,
                                     ctypes.POINTER(ctypes.POINTER(_Rules)), ctypes.c_char_p, ctypes.c_int]
        L.oracle_tsr_all.restype = ctypes.c_int
        _lib = L
    return _lib


def _marshal(records):
    n = len(records)
    sids = (ctypes.c_int32 * max(n, 1))(*[int(s) for s, _ in records])
    enc = [line.encode("utf-8") if isinstance(line, str) else bytes(line) for _, line in records]
    lines = (ctypes.c_char_p * max(n, 1))(*enc)
    lens = (ctypes.c_int64 * max(n, 1))(*[len(b) for b in enc])
    return n, sids, lines, lens, enc


def _patterns_out(p):
    pats = []
    for i in range(p.n):
        sets = []
        for s in range(p.pat_off[i], p.pat_off[i + 1]):
            sets.append(tuple(p.items[q] for q in range(p.set_off[s], p.set_off[s + 1])))
        pats.append((tuple(sets), p.support[i]))
    return pats


def _np64(a):
    import numpy as np
    a = np.ascontiguousarray(a, dtype=np.int64)
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))


def spade_tokens(seq_off, tokens, support, time_limit_s=0.0, want_patterns=True, threads=1, stride=1):
    """Token-stream SPADE (sid = record index).  With time_limit_s > 0 the
    lattice stops after that long: returns joins done and seconds.  threads > 1
    mines the first-level classes on that many OpenMP threads (SURVEY §8d mode
    ii).  stride > 1 mines only the first-level classes of rank % stride == 0
    (a class-stride sample of the whole lattice: bench.py's CPU baseline)."""
    L = lib()
    so, so_p = _np64(seq_off)
    tk, tk_p = _np64(tokens)
    out = ctypes.POINTER(_Patterns)()
    err = ctypes.create_string_buffer(512)
    rc = L.oracle_spade_tokens_sample(so_p, tk_p, len(so) - 1, float(support), float(time_limit_s), int(threads),
                                      int(stride), ctypes.byref(out), err, 512)
    if rc != 0:
        raise OracleError(err.value.decode())
    p = out.contents
    res = {"joins": p.joins, "minsup": p.minsup, "complete": bool(p.complete), "seconds": p.seconds, "seconds_f1": p.seconds_f1,
           "n_patterns": p.n}
    if want_patterns:
        res["patterns"] = sorted(_patterns_out(p))
    L.oracle_patterns_free(out)
    return res


def spade_tokens_csr(seq_off, tokens, support, threads=1):
    """Token-stream SPADE returning the pattern CSR as numpy arrays
    (support, pat_off, set_off, items) plus meta: the form the full-size
    digests (tests/digest.py) are computed from without building millions of
    Python tuples."""
    import numpy as np
    L = lib()
    so, so_p = _np64(seq_off)
    tk, tk_p = _np64(tokens)
    out = ctypes.POINTER(_Patterns)()
    err = ctypes.create_string_buffer(512)
    rc = L.oracle_spade_tokens_mt(so_p, tk_p, len(so) - 1, float(support), 0.0, int(threads),
                                  ctypes.byref(out), err, 512)
    if rc != 0:
        raise OracleError(err.value.decode())
    p = out.contents
    try:
        n = p.n
        sup = np.ctypeslib.as_array(p.support, shape=(max(n, 1),))[:n].copy()
        po = np.ctypeslib.as_array(p.pat_off, shape=(n + 1,)).copy()
        st = np.ctypeslib.as_array(p.set_off, shape=(p.n_sets + 1,)).copy()
        it = np.ctypeslib.as_array(p.items, shape=(max(p.n_items, 1),))[:p.n_items].copy()
        meta = {"joins": p.joins, "minsup": p.minsup, "complete": bool(p.complete), "seconds": p.seconds,
                "seconds_f1": p.seconds_f1, "n": n}
    finally:
        L.oracle_patterns_free(out)
    return (sup, po, st, it), meta


def pattern_support(seq_off, tokens, itemsets):
    """Definitional support of one pattern over a token stream."""
    L = lib()
    so, so_p = _np64(seq_off)
    tk, tk_p = _np64(tokens)
    flat = [i for s in itemsets for i in s]
    offs = [0]
    for s in itemsets:
        offs.append(offs[-1] + len(s))
    it = (ctypes.c_int32 * max(len(flat), 1))(*flat)
    of, of_p = _np64(offs)
    return L.oracle_pattern_support(so_p, tk_p, len(so) - 1, it, of_p, len(itemsets))


def rule_support(seq_off, tokens, X, Y):
    """Definitional (support, |sids(X)|) of one rule over a token stream."""
    L = lib()
    so, so_p = _np64(seq_off)
    tk, tk_p = _np64(tokens)
    xa = (ctypes.c_int32 * len(X))(*X)
    ya = (ctypes.c_int32 * len(Y))(*Y)
    sup, nx = ctypes.c_int64(), ctypes.c_int64()
    L.oracle_rule_support(so_p, tk_p, len(so) - 1, xa, len(X), ya, len(Y), ctypes.byref(sup), ctypes.byref(nx))
    return sup.value, nx.value


def spade(records, support):
    """SPADE.extractRDDPatterns restated: records = [(sid, spmf_line)]."""
    L = lib()
    n, sids, lines, lens, _keep = _marshal(records)
    out = ctypes.POINTER(_Patterns)()
    err = ctypes.create_string_buffer(512)
    rc = L.oracle_spade(sids, lines, lens, n, float(support), ctypes.byref(out), err, 512)
    if rc != 0:
        raise OracleError(err.value.decode())
    p = out.contents
    res = {"patterns": sorted(_patterns_out(p)), "joins": p.joins, "minsup": p.minsup}
    L.oracle_patterns_free(out)
    return res


def tsr(records, k, minconf, time_limit_s=0.0):
    """TSR.extractRDDRules restated: records = [(sid, spmf_line)], sids = 0..N-1.
    time_limit_s > 0 bounds the mining time (CPU baseline): complete = False then."""
    L = lib()
    n, sids, lines, lens, _keep = _marshal(records)
    out = ctypes.POINTER(_Rules)()
    err = ctypes.create_string_buffer(512)
    rc = L.oracle_tsr_timed(sids, lines, lens, n, int(k), float(minconf), float(time_limit_s), ctypes.byref(out),
                            err, 512)
    if rc != 0:
        raise OracleError(err.value.decode())
    r = out.contents
    rules = []
    for i in range(r.n):
        x = tuple(r.ante[q] for q in range(r.ante_off[i], r.ante_off[i + 1]))
        y = tuple(r.cons[q] for q in range(r.cons_off[i], r.cons_off[i + 1]))
        rules.append((x, y, r.support[i], r.confidence[i]))
    rules.sort(key=lambda t: (-t[2], t[0], t[1]))
    res = {"rules": rules, "total": r.total, "expansions": r.expansions,
           "final_minsup": r.final_minsup, "complete": bool(r.complete), "seconds": r.seconds, "pairs": r.pairs}
    L.oracle_rules_free(out)
    return res


def _rules_out(r):
    rules = []
    for i in range(r.n):
        x = tuple(r.ante[q] for q in range(r.ante_off[i], r.ante_off[i + 1]))
        y = tuple(r.cons[q] for q in range(r.cons_off[i], r.cons_off[i + 1]))
        rules.append((x, y, r.support[i], r.confidence[i]))
    rules.sort(key=lambda t: (-t[2], t[0], t[1]))
    return rules


def tsr_all(seq_off, tokens, t, minconf, threads=1):
    """Every valid rule with support >= t, by definition at a fixed threshold
    (oracle/tsr_exhaustive.c): the completeness pin of SURVEY §8(c)(ii).
    Token stream: -1 closes an itemset, -2 is ignored, sid = record index."""
    L = lib()
    so, so_p = _np64(seq_off)
    tk, tk_p = _np64(tokens)
    out = ctypes.POINTER(_Rules)()
    err = ctypes.create_string_buffer(512)
    rc = L.oracle_tsr_all(so_p, tk_p, len(so) - 1, int(t), float(minconf), int(threads), ctypes.byref(out), err, 512)
    if rc != 0:
        raise OracleError(err.value.decode())
    r = out.contents
    res = {"rules": _rules_out(r), "total": r.total, "explored": r.expansions, "seeds": r.pairs,
           "t": r.final_minsup, "seconds": r.seconds}
    L.oracle_rules_free(out)
    return res
