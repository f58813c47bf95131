"""Pure-Python restatement of SPMFBuilder and of the result documents the
actors persist — TEST INFRASTRUCTURE ONLY (the checker for libfsm's
fsm_ingest / fsm_*_json / fsm_rules_query; never imported by the product).

Parity status: "parity unpinned" against a run of the reference — it holds no
fixtures for these paths and Spark / json4s / RedisDB are absent here — so this
restates the Scala source line by line:

  build / index        SPMFBuilder.scala:27-64, 185-198  (count -> zip -> take(limit))
  fromBMS              SPMFBuilder.scala:66-93   (groupBy: groups in order of first
                                                  appearance, items in line order [EXT])
  fromCSV              SPMFBuilder.scala:95-116
  fromKosarak          SPMFBuilder.scala:118-139
  fromSnake            SPMFBuilder.scala:141-176
  fromSPMF             SPMFBuilder.scala:178-183
  patterns document    SPADEActor.scala:47-60  Patterns(List[Pattern(support, itemsets)])
  rules document       TSRActor.scala:52-66    Rules(List[Rule(antecedent, consequent,
                                               support, total, confidence)])
  json4s rendering     compact, fields in constructor order, Double via
                       java.lang.Double.toString [EXT, json4s-native]
  rule queries         FSMQuestor.scala:46-98 -> RedisDB.rulesByAntecedent /
                       rulesByConsequent [EXT, unvendored: subset semantics assumed]
"""
import re
from decimal import Decimal


class BuilderError(Exception):
    """The Spark job would fail (NumberFormatException, ArrayIndexOutOfBounds)."""


def hadoop_lines(text):
    lines = re.split(r"\r\n|\r|\n", text)
    if lines and lines[-1] == "":
        lines.pop()
    return lines


def java_split(s, sep):
    """String.split(sep) for a one-char literal separator, limit 0."""
    if s == "":
        return [""]
    parts = s.split(sep)
    while parts and parts[-1] == "":
        parts.pop()
    return parts


def java_parse_int(tok):
    t = tok[1:] if tok[:1] in ("+", "-") and len(tok) > 1 else tok
    if not t or not all("0" <= c <= "9" for c in t):
        raise BuilderError("NumberFormatException: For input string: %r" % tok)
    v = int(tok)
    if not -(1 << 31) <= v < (1 << 31):
        raise BuilderError("NumberFormatException: For input string: %r" % tok)
    return v


def java_trim(s):
    i, j = 0, len(s)
    while i < j and ord(s[i]) <= 32:
        i += 1
    while j > i and ord(s[j - 1]) <= 32:
        j -= 1
    return s[i:j]


def _from_bms(lines):
    groups = {}
    for line in lines:
        parts = java_split(line, "\t")
        if len(parts) < 2:
            raise BuilderError("ArrayIndexOutOfBoundsException: 1")
        uid = java_parse_int(java_trim(parts[0]))
        pid = java_parse_int(java_trim(parts[1]))
        groups.setdefault(uid, []).append(pid)
    return ["".join("%d -1 " % i for i in items) + "-2" for items in groups.values()]


def _from_sep(lines, sep):
    return ["".join("%d -1 " % java_parse_int(p) for p in java_split(line, sep)) + "-2" for line in lines]


def _from_snake(lines):
    out = []
    for line in lines:
        if len(line) >= 11:
            out.append("".join("%d -1 " % (ord(c) - 65) for c in line) + "-2")
    return out


def build(text, fmt, limit=1000):
    """-> ["idx|sequence"] (SPMFBuilder.build's RDD contents), None for an unknown format."""
    lines = hadoop_lines(text)
    if fmt == "BMS":
        seqs = _from_bms(lines)
    elif fmt == "CSV":
        seqs = _from_sep(lines, ",")
    elif fmt == "KOSARAK":
        seqs = _from_sep(lines, " ")
    elif fmt == "SNAKE":
        seqs = _from_snake(lines)
    elif fmt == "SPMF":
        seqs = lines
    else:
        return None
    return ["%d|%s" % (i, s) for i, s in enumerate(seqs)][:max(limit, 0)]


def java_double(d):
    """java.lang.Double.toString (shortest round-trip digits)."""
    if d != d:
        return "NaN"
    if d in (float("inf"), float("-inf")):
        return "Infinity" if d > 0 else "-Infinity"
    if d == 0.0:
        return "-0.0" if str(d).startswith("-") else "0.0"
    sign = "-" if d < 0 else ""
    a = abs(d)
    t = Decimal(repr(a)).as_tuple()  # repr: the shortest digits that round trip
    e10 = len(t.digits) - 1 + t.exponent
    digits = "".join(map(str, t.digits)).rstrip("0") or "0"
    if 1e-3 <= a < 1e7:
        if e10 >= 0:
            ipart = (digits[:e10 + 1]).ljust(e10 + 1, "0")
            fpart = digits[e10 + 1:] or "0"
        else:
            ipart, fpart = "0", "0" * (-e10 - 1) + digits
        return sign + ipart + "." + fpart
    return sign + digits[0] + "." + (digits[1:] or "0") + "E" + str(e10)


def patterns_json(patterns):
    """patterns: [(support, [[items]...])] in result order."""
    return '{"items":[' + ",".join(
        '{"support":%d,"itemsets":[%s]}' % (s, ",".join("[" + ",".join(map(str, st)) + "]" for st in sets))
        for s, sets in patterns) + "]}"


def patterns_serialize(patterns):
    return "".join("".join(" ".join(map(str, st)) + " -1 " for st in sets) + "| %d\n" % s for s, sets in patterns)


def rules_json(rules, total):
    """rules: [(antecedent, consequent, support, confidence)]."""
    return '{"items":[' + ",".join(
        '{"antecedent":[%s],"consequent":[%s],"support":%d,"total":%d,"confidence":%s}' % (
            ",".join(map(str, x)), ",".join(map(str, y)), s, total, java_double(c)) for x, y, s, c in rules) + "]}"


def rules_query(rules, side, items):
    q = set(items)
    return [i for i, r in enumerate(rules) if set(r[side]) <= q]
