"""Definitional brute-force miners for tiny sequence databases.

TEST INFRASTRUCTURE ONLY.  Written from the published definitions (SURVEY.md
Appendix A.1-A.3), independently of oracle/fsm_oracle.c and of the engine: it
enumerates patterns / rules and counts containment by definition.  It pins the
C restatement (which has no reference fixtures to be checked against).

Parsing follows SPADE.scala:145-212 / TSR.scala:41,109-143 (A.1).  Pure Python
loops: use only on databases of a few dozen short sequences.
"""
import math
from itertools import combinations


class BruteError(ValueError):
    pass


def java_split_space(s):
    """java.lang.String.split(" ") (limit 0)."""
    if s == "":
        return [""]
    parts = s.split(" ")
    while parts and parts[-1] == "":
        parts.pop()
    return parts


def _jint(tok, bits=32):
    t = tok[1:] if tok[:1] in "+-" and len(tok) > 1 else tok
    if not t or not all("0" <= c <= "9" for c in t):
        raise BruteError("bad integer %r" % tok)
    v = int(tok)
    lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
    if not lo <= v <= hi:
        raise BruteError("out of range %r" % tok)
    return v


def spade_eid_view(records):
    """sid -> list of itemsets ordered by timestamp (same-timestamp itemsets and
    same-sid records merged, as registerBit(sid, ts) merges them)."""
    bysid = {}
    for sid, line in records:
        if sid < 0:
            raise BruteError("negative sid")
        ts_state, cur, cur_ts = -1, [], 0
        for tok in java_split_space(line):
            if tok == "":
                raise BruteError("empty token")
            if tok[0] == "<":
                if len(tok) < 2:
                    raise BruteError("bad timestamp")
                v = _jint(tok[1:-1], 64)
                ts_state, cur_ts = v, v
            elif tok == "-1":
                ts32 = ((cur_ts & 0xFFFFFFFF) ^ 0x80000000) - 0x80000000
                if cur and ts32 < 0:
                    raise BruteError("negative timestamp")
                d = bysid.setdefault(sid, {})
                for it in cur:
                    d.setdefault(ts32, set()).add(it)
                cur = []
                cur_ts = ((cur_ts + 1 + (1 << 63)) % (1 << 64)) - (1 << 63)
                ts_state = ((ts_state + 1 + (1 << 63)) % (1 << 64)) - (1 << 63)
            elif tok == "-2":
                pass
            else:
                cur.append(_jint(tok))
                if ts_state < 0:
                    ts_state, cur_ts = 1, 1
    return {sid: [frozenset(d[t]) for t in sorted(d)] for sid, d in bysid.items()}


def _contains(seq, pattern):
    pos = 0
    for X in pattern:
        while pos < len(seq) and not X <= seq[pos]:
            pos += 1
        if pos == len(seq):
            return False
        pos += 1
    return True


def brute_spade(records, support):
    """All patterns with support >= max(1, ceil(support * total))."""
    view = spade_eid_view(records)
    total = len(records)
    ms = math.ceil(support * total) if support == support else float("inf")
    minsup = max(1, ms)
    seqs = list(view.values())
    items = sorted({i for s in seqs for X in s for i in X})

    def sup(p):
        sp = [frozenset(X) for X in p]
        return sum(1 for s in seqs if _contains(s, sp))

    out = {}
    frontier = []
    for x in items:
        p = ((x,),)
        c = sup(p)
        if c >= minsup:
            out[p] = c
            frontier.append(p)
    while frontier:
        nxt = []
        for p in frontier:
            for y in items:
                cands = [p + ((y,),)]
                if y > p[-1][-1]:
                    cands.append(p[:-1] + (p[-1] + (y,),))
                for q in cands:
                    c = sup(q)
                    if c >= minsup:
                        out[q] = c
                        nxt.append(q)
        frontier = nxt
    return sorted(out.items())


def tsr_view(records):
    """sid -> list of itemsets (lists), TSR parse rules."""
    seqs = []
    for p, (sid, line) in enumerate(records):
        if sid != p:
            raise BruteError("TSR needs dense sids")
        toks = java_split_space(line)
        vals = [_jint(t) for t in toks]
        cur, sets = [], []
        for t, v in zip(toks, vals):
            if t == "-1":
                sets.append(cur)
                cur = []
            elif t == "-2":
                pass
            else:
                if v < 0:
                    raise BruteError("negative item")
                cur.append(v)
        seqs.append(sets)
    return seqs


def brute_tsr_valid(records, minconf):
    """Every valid rule X => Y (X, Y disjoint non-empty, sup >= 1,
    conf >= minconf) as {(X, Y): (sup, conf)} by definition (A.3)."""
    seqs = tsr_view(records)
    first, last = [], []
    for s in seqs:
        f, l = {}, {}
        for j, X in enumerate(s):
            for it in X:
                f.setdefault(it, j)
                l[it] = j
        first.append(f)
        last.append(l)
    items = sorted({i for f in first for i in f})
    out = {}
    subsets = [c for r in range(1, len(items) + 1) for c in combinations(items, r)]
    for X in subsets:
        sx = [i for i, f in enumerate(first) if all(x in f for x in X)]
        if not sx:
            continue
        for Y in subsets:
            if set(X) & set(Y):
                continue
            sup = 0
            for i in sx:
                f, l = first[i], last[i]
                if all(y in l for y in Y) and max(f[x] for x in X) < min(l[y] for y in Y):
                    sup += 1
            if sup >= 1:
                conf = sup / len(sx)
                if conf >= minconf:
                    out[(X, Y)] = (sup, conf)
    return out


def check_tsr(rules, valid, k):
    """Invariants of SURVEY §8c(2): (i) every returned rule is valid with the
    definitional sup/conf; (ii) every valid rule with sup > min returned sup is
    returned; (iii) |R| >= min(k, |valid|)."""
    got = {(x, y): (s, c) for x, y, s, c in rules}
    assert len(got) == len(rules), "duplicate rules"
    for key, (s, c) in got.items():
        assert key in valid, "rule %r not valid by definition" % (key,)
        vs, vc = valid[key]
        assert s == vs and c == vc, "rule %r: got %r expected %r" % (key, (s, c), (vs, vc))
    if rules:
        m = min(s for _, _, s, _ in rules)
        for key, (s, c) in valid.items():
            if s > m:
                assert key in got, "missing valid rule %r sup=%d > %d" % (key, s, m)
    assert len(rules) >= min(k, len(valid))
