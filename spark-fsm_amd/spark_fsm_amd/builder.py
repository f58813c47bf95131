"""SPMFBuilder mirror (util/SPMFBuilder.scala:25-204) over libfsm's native
converter (fsm_ingest, spark-fsm_amd/csrc/ingest.cpp).

  SPMFBuilder.build(sc, input, format, limit = 1000, output = None)
      : Option[RDD[String]]                                  SPMFBuilder.scala:27
  -> build(input, fmt, limit=1000, output=None) -> list of "idx|sequence" or None

ingest() is the engine-facing form of the same conversion: token arrays
(sids, seq_off, tokens) for Engine.db_from_tokens, with no strings in between.
"""
import ctypes
import os
import re

import numpy as np

from . import _lib
from ._lib import check

FORMATS = {"SPMF": _lib.FMT_SPMF, "INDEXED": _lib.FMT_INDEXED, "BMS": _lib.FMT_BMS, "CSV": _lib.FMT_CSV,
           "KOSARAK": _lib.FMT_KOSARAK, "SNAKE": _lib.FMT_SNAKE}


class TokenDB:
    """Sequences as fsm_db_from_tokens takes them."""

    __slots__ = ("sids", "seq_off", "tokens")

    def __init__(self, sids, seq_off, tokens):
        self.sids, self.seq_off, self.tokens = sids, seq_off, tokens

    def __len__(self):
        return len(self.sids)

    def lines(self):
        """The builder's "idx|sequence" strings (SPMFBuilder.scala:195)."""
        so, tk = self.seq_off.tolist(), self.tokens.tolist()
        return ["%d|%s" % (s, " ".join(map(str, tk[so[r]:so[r + 1]]))) for r, s in enumerate(self.sids.tolist())]

    def records(self):
        """(sid, spmf_line) pairs: the RDD[(Int, String)] the miners take."""
        so, tk = self.seq_off.tolist(), self.tokens.tolist()
        return [(s, " ".join(map(str, tk[so[r]:so[r + 1]]))) for r, s in enumerate(self.sids.tolist())]


def text_lines(text):
    """Hadoop LineRecordReader records: lines end at \n, \r\n or \r; no empty
    record after a final terminator."""
    lines = re.split(r"\r\n|\r|\n", text)
    if lines and lines[-1] == "":
        lines.pop()
    return lines


def _read(data):
    if isinstance(data, (bytes, bytearray, memoryview)):
        return bytes(data)
    if isinstance(data, str) and os.path.exists(data):
        if os.path.isdir(data):  # a saveAsTextFile directory: its part files in name order
            parts = sorted(f for f in os.listdir(data) if f.startswith("part-"))
            return b"".join(open(os.path.join(data, f), "rb").read() for f in parts)
        with open(data, "rb") as f:
            return f.read()
    raise FileNotFoundError(data)


def ingest(data, fmt, limit=-1):
    """Native conversion of a file (path or bytes) in format `fmt` ("BMS", "CSV",
    "KOSARAK", "SNAKE", "SPMF" or "INDEXED") -> TokenDB.  limit < 0 keeps all."""
    raw = _read(data)
    L = _lib.load()
    out = ctypes.POINTER(_lib.TokenDb)()
    check(L.fsm_ingest(FORMATS[fmt], raw, len(raw), int(limit), ctypes.byref(out)))
    try:
        t = out.contents
        n, nt = t.n, t.n_tokens
        sids = np.ctypeslib.as_array(t.sids, shape=(max(n, 1),))[:n].copy()
        seq_off = np.ctypeslib.as_array(t.seq_off, shape=(n + 1,)).copy()
        tokens = np.ctypeslib.as_array(t.tokens, shape=(max(nt, 1),))[:nt].copy()
    finally:
        L.fsm_token_db_free(out)
    return TokenDB(sids, seq_off, tokens)


def build(data, fmt, limit=1000, output=None):
    """SPMFBuilder.build: "idx|sequence" strings of the first `limit` sequences,
    None for an unknown format (SPMFBuilder.scala:41); `output` writes them as
    saveAsTextFile does (a directory holding part-00000)."""
    if fmt not in ("BMS", "CSV", "KOSARAK", "SNAKE", "SPMF"):
        return None
    if limit <= 0:  # RDD.take(n <= 0) is empty (after file.count ran the conversion)
        ingest(data, fmt, 0)
        out = []
    elif fmt == "SPMF":  # fromSPMF indexes the raw lines (SPMFBuilder.scala:178-183)
        out = ["%d|%s" % (i, l) for i, l in enumerate(text_lines(_read(data).decode("utf-8"))[:limit])]
    else:
        out = ingest(data, fmt, limit).lines()
    if output is not None:
        os.makedirs(output, exist_ok=False)  # saveAsTextFile refuses an existing path
        with open(os.path.join(output, "part-00000"), "w") as f:
            f.writelines(l + "\n" for l in out)
        open(os.path.join(output, "_SUCCESS"), "w").close()
    return out
