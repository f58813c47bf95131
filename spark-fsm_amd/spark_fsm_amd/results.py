"""Mined results as the actors persist and the questor queries them, rendered in
bulk by libfsm (spark-fsm_amd/csrc/results.cpp) straight from the CSR.

  SPADEActor.train -> Patterns(List[Pattern(support, itemsets)])   SPADEActor.scala:47-68
  TSRActor.train   -> Rules(List[Rule(antecedent, consequent, support, total, confidence)])
                                                                   TSRActor.scala:52-71
  FSMQuestor get:antecedent / get:consequent                       FSMQuestor.scala:46-98

PatternSet / RuleSet hold numpy CSR arrays and hand libfsm a view of them
(no copies); the documents come back as str.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check

_P = ctypes.POINTER


def _ptr(a, ct):
    return a.ctypes.data_as(_P(ct))


def _buffer(fn, struct):
    L = _lib.load()
    out = ctypes.c_void_p()
    n = ctypes.c_int64()
    check(getattr(L, fn)(ctypes.byref(struct), ctypes.byref(out), ctypes.byref(n)))
    try:
        return ctypes.string_at(out, n.value).decode("utf-8")
    finally:
        L.fsm_buffer_free(out)


class PatternSet:
    """fsm_patterns over numpy arrays (Engine.spade_csr's output)."""

    def __init__(self, support, pat_off, set_off, items, total=0, minsup=0):
        self.support = np.ascontiguousarray(support, np.int32)
        self.pat_off = np.ascontiguousarray(pat_off, np.int64)
        self.set_off = np.ascontiguousarray(set_off, np.int64)
        self.items = np.ascontiguousarray(items, np.int32)
        self.total, self.minsup = int(total), int(minsup)

    @classmethod
    def from_csr(cls, csr, meta):
        return cls(*csr, total=meta.get("total", 0), minsup=meta.get("minsup", 0))

    @classmethod
    def from_list(cls, patterns, total=0, minsup=0):
        """[(itemsets, support)] (Engine.spade's output)."""
        sup, po, so, it = [], [0], [0], []
        for sets, s in patterns:
            sup.append(s)
            for st in sets:
                it.extend(st)
                so.append(len(it))
            po.append(len(so) - 1)
        return cls(sup, po, so, it, total, minsup)

    def __len__(self):
        return len(self.support)

    def _struct(self):
        return _lib.Patterns(len(self.support), _ptr(self.support, ctypes.c_int32), _ptr(self.pat_off, ctypes.c_int64),
                             _ptr(self.set_off, ctypes.c_int64), _ptr(self.items, ctypes.c_int32),
                             len(self.set_off) - 1, len(self.items), self.total, self.minsup)

    def serialize(self):
        """Every pattern's serialize() line, "\\n"-terminated (SPADEActor.scala:47-50)."""
        return _buffer("fsm_patterns_serialize", self._struct())

    def to_json(self):
        """json4s write(Patterns(...)) as SPADEActor stores it (SPADEActor.scala:58-60)."""
        return _buffer("fsm_patterns_json", self._struct())


class RuleSet:
    """fsm_rules over numpy arrays."""

    def __init__(self, rules, total, final_minsup=0):
        """rules: [(antecedent, consequent, support, confidence)] (Engine.tsr's output)."""
        ao, co, a, c = [0], [0], [], []
        for x, y, _s, _c in rules:
            a.extend(x)
            ao.append(len(a))
            c.extend(y)
            co.append(len(c))
        self.rules = list(rules)
        self.support = np.array([r[2] for r in rules], np.int32)
        self.confidence = np.array([r[3] for r in rules], np.float64)
        self.ante_off, self.cons_off = np.array(ao, np.int64), np.array(co, np.int64)
        self.ante, self.cons = np.array(a, np.int32), np.array(c, np.int32)
        self.total, self.final_minsup = int(total), int(final_minsup)

    def __len__(self):
        return len(self.rules)

    def _struct(self):
        return _lib.Rules(len(self.rules), _ptr(self.support, ctypes.c_int32), _ptr(self.confidence, ctypes.c_double),
                          _ptr(self.ante_off, ctypes.c_int64), _ptr(self.ante, ctypes.c_int32),
                          _ptr(self.cons_off, ctypes.c_int64), _ptr(self.cons, ctypes.c_int32), self.total,
                          self.final_minsup)

    def to_json(self):
        """json4s write(Rules(...)) as TSRActor stores it (TSRActor.scala:52-66)."""
        return _buffer("fsm_rules_json", self._struct())

    def _query(self, side, items):
        L = _lib.load()
        q = np.ascontiguousarray(list(items), np.int32)
        idx = np.zeros(max(len(self.rules), 1), np.int64)
        n = ctypes.c_int64()
        st = self._struct()
        check(L.fsm_rules_query(ctypes.byref(st), side, _ptr(q, ctypes.c_int32), len(q), _ptr(idx, ctypes.c_int64),
                                ctypes.byref(n)))
        return [self.rules[i] for i in idx[:n.value].tolist()]

    def by_antecedent(self, items):
        """Rules whose antecedent items all occur in `items` (get:antecedent)."""
        return self._query(0, items)

    def by_consequent(self, items):
        """Rules whose consequent items all occur in `items` (get:consequent)."""
        return self._query(1, items)
