"""Canonical, order-independent digests of SPADE pattern sets and TSR rule sets.

Used by the full-size parity tests: the oracle's output at a BASELINE config is
reduced to (count, support sum, SHA-256) once in the build container
(tests/golden/make_fullsize.py) and the GPU output is reduced the same way on
the box.  The digest does not depend on output order (the reference's order is
discovery order), only on the set of (pattern, support) pairs:

  key(p) = mix(sum over the pattern's items q of mix(itemset# << 40 | pos << 32 | item))
           + support * C
  digest = sha256 of the sorted uint64 keys

Every item carries its itemset index and its position inside the pattern, so
two different patterns collide only through a 64-bit hash collision.
"""
import hashlib

import numpy as np

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_C = np.uint64(0x9E3779B97F4A7C15)


def _mix(x):
    """splitmix64 finalizer over a uint64 array (wrapping arithmetic)."""
    x = np.asarray(x, dtype=np.uint64).copy()
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(30)
        x *= _M1
        x ^= x >> np.uint64(27)
        x *= _M2
        x ^= x >> np.uint64(31)
    return x


def pattern_keys(sup, pat_off, set_off, items):
    """uint64 key per pattern of a CSR pattern set (fsm_patterns layout)."""
    sup = np.asarray(sup, dtype=np.int64)
    pat_off = np.asarray(pat_off, dtype=np.int64)
    set_off = np.asarray(set_off, dtype=np.int64)
    items = np.asarray(items, dtype=np.int64)
    n = len(sup)
    if n == 0:
        return np.zeros(0, np.uint64)
    nsets = len(set_off) - 1
    set_len = np.diff(set_off)
    pat_nsets = np.diff(pat_off)
    set_pat = np.repeat(np.arange(n, dtype=np.int64), pat_nsets)            # pattern of every itemset
    set_idx = np.arange(nsets, dtype=np.int64) - pat_off[set_pat]             # itemset index inside it
    item_set = np.repeat(np.arange(nsets, dtype=np.int64), set_len)          # itemset of every item
    item_pat = set_pat[item_set]
    pos = np.arange(len(items), dtype=np.int64) - set_off[pat_off[item_pat]]  # position inside the pattern
    v = (set_idx[item_set].astype(np.uint64) << np.uint64(40)) ^ (pos.astype(np.uint64) << np.uint64(32)) ^ \
        (items.astype(np.uint64) & np.uint64(0xFFFFFFFF))
    mv = _mix(v)
    first_item = set_off[pat_off[:-1]]
    with np.errstate(over="ignore"):
        h = np.add.reduceat(mv, first_item) if len(items) else np.zeros(n, np.uint64)
        return _mix(h) + sup.astype(np.uint64) * _C


def pattern_digest(sup, pat_off, set_off, items):
    keys = np.sort(pattern_keys(sup, pat_off, set_off, items))
    return {"n": int(len(sup)), "support_sum": int(np.asarray(sup, dtype=np.int64).sum()),
            "sha256": hashlib.sha256(keys.tobytes()).hexdigest()}


def pattern_digest_list(pats):
    """Same digest from a list of (itemsets tuple-of-tuples, support)."""
    sup, po, so, it = [], [0], [0], []
    for sets, s in pats:
        sup.append(s)
        for x in sets:
            it.extend(x)
            so.append(len(it))
        po.append(len(so) - 1)
    return pattern_digest(np.array(sup, np.int64), np.array(po, np.int64), np.array(so, np.int64),
                          np.array(it, np.int64))


def rule_digest(rules):
    """Digest of a rule list [(antecedent, consequent, support, confidence)]:
    SHA-256 over the canonically sorted rules, confidence as its IEEE bits."""
    h = hashlib.sha256()
    for x, y, s, c in sorted(rules, key=lambda t: (-t[2], tuple(t[0]), tuple(t[1]))):
        h.update(repr((tuple(x), tuple(y), int(s), float(c).hex())).encode())
    return {"n": len(rules), "support_sum": int(sum(r[2] for r in rules)), "sha256": h.hexdigest()}
