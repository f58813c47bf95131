"""Python wrapper for tools/fsmgen.c (seeded synthetic sequence databases).

Configs (BASELINE.json / SURVEY §8d; seeds 1, 2, 3):
  quest(D)        Quest C10 T2.5 S4 I1.25, N_S 5000, N_I 25000, N 10000 items
  kosarak()       990,002 seqs, 41,270 items, Zipf, mean ~8.1, max 2,500, single-item itemsets
  bible() / sign()  word-stream shapes (36,369 x ~21.6 / 730 x ~52)
Each returns a DataSet with (sids, seq_off, tokens) numpy arrays, the input of
fsm_db_from_tokens; .lines() renders SPMF text for the record-based APIs.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libfsmgen.so")
_lib = None


def build():
    os.makedirs(os.path.join(HERE, "build"), exist_ok=True)
    src = os.path.join(HERE, "fsmgen.c")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-o", LIB, src, "-lm"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        P = ctypes.POINTER
        pp = P(P(ctypes.c_int64))
        L.gen_quest.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                                ctypes.c_double, ctypes.c_double, ctypes.c_int32, ctypes.c_int32,
                                ctypes.c_int32, pp, pp, P(ctypes.c_int64)]
        L.gen_zipf.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, ctypes.c_double,
                               ctypes.c_double, ctypes.c_double, ctypes.c_int64, ctypes.c_double,
                               ctypes.c_int32, pp, pp, P(ctypes.c_int64)]
        L.gen_free.argtypes = [ctypes.c_void_p]
        _lib = L
    return _lib


class DataSet:
    def __init__(self, seq_off, tokens, name):
        self.seq_off = seq_off
        self.tokens = tokens
        self.sids = np.arange(len(seq_off) - 1, dtype=np.int32)
        self.name = name

    def __len__(self):
        return len(self.sids)

    def lines(self, a=0, b=None):
        b = len(self) if b is None else b
        toks = self.tokens
        out = []
        for r in range(a, b):
            out.append(" ".join(map(str, toks[self.seq_off[r]:self.seq_off[r + 1]].tolist())))
        return out

    def records(self, a=0, b=None):
        b = len(self) if b is None else b
        return list(zip(range(0, b - a), self.lines(a, b)))

    def head(self, n):
        so = self.seq_off[:n + 1].copy()
        return DataSet(so, self.tokens[:so[-1]].copy(), "%s[:%d]" % (self.name, n))


def _take(so_p, tk_p, n, D, name):
    L = lib()
    so = np.ctypeslib.as_array(so_p, shape=(D + 1,)).copy()
    tk = np.ctypeslib.as_array(tk_p, shape=(max(n.value, 1),))[:n.value].copy()
    L.gen_free(ctypes.cast(so_p, ctypes.c_void_p))
    L.gen_free(ctypes.cast(tk_p, ctypes.c_void_p))
    return DataSet(so, tk, name)


def quest(D, seed=1, C=10.0, T=2.5, S=4.0, I=1.25, NS=5000, NI=25000, N=10000):
    L = lib()
    so, tk, n = ctypes.POINTER(ctypes.c_int64)(), ctypes.POINTER(ctypes.c_int64)(), ctypes.c_int64()
    L.gen_quest(seed, D, C, T, S, I, NS, NI, N, ctypes.byref(so), ctypes.byref(tk), ctypes.byref(n))
    return _take(so, tk, n, D, "quest-C%gT%gS%gI%g-D%d-N%d-seed%d" % (C, T, S, I, D, N, seed))


def zipf(D, nitems, zipf_s, mean_len, sigma, max_len, p_succ, distinct, seed, name):
    L = lib()
    so, tk, n = ctypes.POINTER(ctypes.c_int64)(), ctypes.POINTER(ctypes.c_int64)(), ctypes.c_int64()
    L.gen_zipf(seed, D, nitems, zipf_s, mean_len, sigma, max_len, p_succ, 1 if distinct else 0,
               ctypes.byref(so), ctypes.byref(tk), ctypes.byref(n))
    return _take(so, tk, n, D, "%s-seed%d" % (name, seed))


def kosarak(D=990002, seed=1):
    return zipf(D, 41270, 1.0, 8.1, 1.1, 2500, 0.6, True, seed, "kosarak-shaped-D%d" % D)


def bible(D=36369, seed=1):
    return zipf(D, 13905, 1.05, 21.6, 0.7, 400, 0.25, False, seed, "bible-shaped-D%d" % D)


def sign(D=730, seed=1):
    return zipf(D, 267, 0.8, 52.0, 0.35, 200, 0.3, False, seed, "sign-shaped-D%d" % D)
