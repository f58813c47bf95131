"""Host-side mirror of the reference's hot-path API (same names, argument
meaning and error behaviour), backed by libfsm on the GPU.

  SPADE.extractRDDPatterns(dataset, support, dfs=true, stats=true)  SPADE.scala:36
  TSR.extractRDDRules(dataset, k, minconf)                          TSR.scala:31
plus the boundary callers' result mappings:
  SPADEActor.train  pattern.serialize() -> Pattern(support, itemsets)  SPADEActor.scala:47-58
  TSRActor.train    Rule(antecedent, consequent, support, total, conf) TSRActor.scala:52-62

`dataset` is any sequence of (sid, spmf_line) pairs (the RDD[(Int,String)]).
Errors the reference throws surface as FsmParseError (an Exception), which the
actor maps to FAILURE (TrainActor.scala:65-67).
"""
from .engine import default_engine, MODE_SPADE, MODE_TSR


class Pattern:
    """de.kp.core.spade.Pattern as used by the caller: serialize() only."""

    __slots__ = ("itemsets", "support")

    def __init__(self, itemsets, support):
        self.itemsets = itemsets
        self.support = support

    def serialize(self):
        # "1 -1 3 -1 3 -1 | 3"  (format shown at SPADEActor.scala:50)
        body = "".join(" ".join(str(i) for i in s) + " -1 " for s in self.itemsets)
        return body + "| " + str(self.support)

    def __repr__(self):
        return "Pattern(%r, %d)" % (self.itemsets, self.support)


class Rule:
    """de.kp.core.tsr.Rule accessors used by TSRActor.scala:55-59."""

    __slots__ = ("_x", "_y", "_sup", "_conf")

    def __init__(self, x, y, sup, conf):
        self._x, self._y, self._sup, self._conf = list(x), list(y), sup, conf

    def getItemset1(self):
        return list(self._x)

    def getItemset2(self):
        return list(self._y)

    def getAbsoluteSupport(self):
        return self._sup

    def getConfidence(self):
        return self._conf

    def __repr__(self):
        return "Rule(%r => %r, sup=%d, conf=%r)" % (self._x, self._y, self._sup, self._conf)


def extract_rdd_patterns(dataset, support, dfs=True, stats=True, engine=None):
    """SPADE.extractRDDPatterns (SPADE.scala:36-140) on the GPU engine."""
    eng = engine or default_engine()
    db = eng.db_from_spmf(list(dataset), MODE_SPADE)
    try:
        pats, _meta = eng.spade(db, support, dfs)
    finally:
        db.free()
    if stats:  # algorithm.printStatistics() (SPADE.scala:136)
        st = eng.stats()
        print("SPADE[MI355X]: patterns=%d joins=%d classes=%d mine=%.3f ms (flatten %.3f ms, upload %.3f ms)"
              % (st["patterns"], st["joins"], st["classes"], st["ms_mine"], st["ms_flatten"], st["ms_upload"]))
    return [Pattern(s, sup) for s, sup in pats]


def extract_rdd_rules(dataset, k, minconf, engine=None):
    """TSR.extractRDDRules (TSR.scala:31-107) on the GPU engine."""
    eng = engine or default_engine()
    db = eng.db_from_spmf(list(dataset), MODE_TSR)
    try:
        rules, _meta = eng.tsr(db, k, minconf)
    finally:
        db.free()
    return [Rule(x, y, s, c) for x, y, s, c in rules]


def spade_actor_patterns(patterns):
    """SPADEActor.train's mapping (SPADEActor.scala:47-58): serialize(), split on
    '|', support = trim.toInt, itemsets = split("-1") -> trim -> split(" ") -> toInt.
    Returns [(support, [[items]...])]; raises ValueError where Scala would throw."""
    out = []
    for p in patterns:
        line = p.serialize()
        parts = line.split("|")
        if len(parts) != 2:
            raise ValueError("MatchError on %r" % line)
        sequence, cardinality = parts
        support = _java_int(cardinality.strip())
        itemsets = [[_java_int(t) for t in _java_split(s.strip(), " ")]
                    for s in _java_split(sequence.strip(), "-1")]
        out.append((support, itemsets))
    return out


def tsr_actor_rules(rules, total):
    """TSRActor.train's mapping (TSRActor.scala:53-62)."""
    return [(r.getItemset1(), r.getItemset2(), r.getAbsoluteSupport(), int(total), r.getConfidence())
            for r in rules]


def _java_split(s, sep):
    if s == "":
        return [""]
    parts = s.split(sep)
    while parts and parts[-1] == "":
        parts.pop()
    return parts


def _java_int(tok):
    t = tok[1:] if tok[:1] in "+-" and len(tok) > 1 else tok
    if not t or not all("0" <= c <= "9" for c in t):
        raise ValueError("NumberFormatException: %r" % tok)
    v = int(tok)
    if not -(1 << 31) <= v < (1 << 31):
        raise ValueError("NumberFormatException: %r" % tok)
    return v
