"""Engine: one fsm_ctx (HIP stream + device buffers) and its flattened DBs."""
import ctypes
import weakref

import numpy as np

from . import _lib
from ._lib import MODE_SPADE, MODE_TSR, check


class _ResultOwner:
    """Keeps a libfsm result struct alive while numpy views of its arrays exist:
    every view's buffer holds a reference to this object, whose finalizer calls
    the library's free function once the last view is gone."""

    def __init__(self, free_fn, ptr):
        weakref.finalize(self, free_fn, ptr)

    def view(self, ptr, n, dtype):
        dt = np.dtype(dtype)
        if n <= 0 or not ptr:
            return np.zeros(0, dtype=dt)
        buf = (np.ctypeslib.as_ctypes_type(dt) * int(n)).from_address(ctypes.addressof(ptr.contents))
        buf._owner = self
        arr = np.frombuffer(buf, dtype=dt)
        arr.flags.writeable = False  # library memory: read-only views
        return arr


class Engine:
    """Owns a libfsm context on one gfx950 device."""

    def __init__(self, device=0, verbose=False, mem_budget=0, nranks=1, rank=0, unique_id=None, host_comm=None,
                 devices=None):
        """nranks > 1: sharded SPADE, one Engine per rank, collectives over RCCL
        (unique_id from dist.comm_unique_id() on rank 0) or over host_comm
        (a dist.TorchHostComm; kept alive by this Engine).
        devices=[d0, d1, ...] (more than one): ONE Engine whose calls shard over
        in-process ranks, rank r on HIP device d_r (a device may repeat), the way the
        JVM drop-in shards (fsm_opts.ndevices); every call returns the whole result."""
        L = _lib.load()
        opts = _lib.Opts()
        opts.device = device
        if devices is not None and len(devices) > 1:
            if len(devices) > _lib.MAX_DEVICES:
                raise ValueError("at most %d in-process ranks" % _lib.MAX_DEVICES)
            opts.ndevices = len(devices)
            for r, d in enumerate(devices):
                opts.devices[r] = int(d)
        elif devices is not None and len(devices) == 1:
            opts.device = int(devices[0])
        opts.nranks = int(nranks)
        opts.rank = int(rank)
        opts.verbose = 1 if verbose else 0
        opts.mem_budget = int(mem_budget)
        if unique_id is not None:
            ctypes.memmove(opts.unique_id, bytes(unique_id), 128)
        self._host_comm = host_comm
        if host_comm is not None:
            opts.host_comm = ctypes.pointer(host_comm.struct)
        self._ctx = ctypes.c_void_p()
        check(L.fsm_ctx_create(ctypes.byref(opts), ctypes.byref(self._ctx)), None)
        self._L = L

    def close(self):
        if getattr(self, "_ctx", None):
            self._L.fsm_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ------------------------------------------------------------ DBs
    def db_from_spmf(self, records, mode):
        """records: sequence of (sid, spmf_line) — the RDD[(Int,String)]."""
        n = len(records)
        sids = (ctypes.c_int32 * max(n, 1))(*[int(s) for s, _ in records])
        enc = [l.encode("utf-8") if isinstance(l, str) else bytes(l) for _, l in records]
        lines = (ctypes.c_char_p * max(n, 1))(*enc)
        lens = (ctypes.c_int64 * max(n, 1))(*[len(b) for b in enc])
        db = ctypes.c_void_p()
        check(self._L.fsm_db_from_spmf(self._ctx, mode, sids, lines, lens, n, ctypes.byref(db)), self._ctx)
        return DB(self, db, mode)

    def db_from_tokens(self, sids, seq_off, tokens, mode):
        sids = np.ascontiguousarray(sids, dtype=np.int32)
        seq_off = np.ascontiguousarray(seq_off, dtype=np.int64)
        tokens = np.ascontiguousarray(tokens, dtype=np.int64)
        n = len(sids)
        db = ctypes.c_void_p()
        P = ctypes.POINTER
        check(self._L.fsm_db_from_tokens(
            self._ctx, mode, sids.ctypes.data_as(P(ctypes.c_int32)), seq_off.ctypes.data_as(P(ctypes.c_int64)),
            tokens.ctypes.data_as(P(ctypes.c_int64)), n, ctypes.byref(db)), self._ctx)
        return DB(self, db, mode)

    def db_export(self, db):
        """fsm_db_export: the flattened DB as it sits in HBM, as numpy arrays."""
        out = ctypes.POINTER(_lib.DbImage)()
        check(self._L.fsm_db_export(self._ctx, db.handle, ctypes.byref(out)), self._ctx)
        try:
            m = out.contents

            def arr(ptr, n):
                # an empty field keeps its ctypes element type (uint32 / uint64 / int32)
                dt = np.dtype(ptr._type_)
                return np.ctypeslib.as_array(ptr, shape=(max(n, 1),))[:n].copy() if n else np.zeros(0, dtype=dt)

            img = {"mode": m.mode, "mask_words": m.mask_words, "rows": m.rows, "entries": m.entries,
                   "items": m.items, "max_occ": m.max_occ, "row_off": arr(m.row_off, m.rows + 1),
                   "item": arr(m.item, m.entries), "item_val": arr(m.item_val, m.items)}
            if m.mode == MODE_SPADE:
                img["mask"] = arr(m.mask, m.entries * m.mask_words)
            else:
                img["first"] = arr(m.first, m.entries)
                img["last"] = arr(m.last, m.entries)
        finally:
            self._L.fsm_db_image_free(out)
        return img

    # ------------------------------------------------------------ mining
    def spade_csr(self, db, support, dfs=True, copy=False):
        """fsm_spade_mine -> CSR numpy arrays (support, pat_off, set_off, items), meta.

        By default the arrays are read-only views of the library's result
        buffers (no copy of the hundreds of MB a dense mine returns).  The four
        views share ONE lifetime: fsm_patterns_free runs when the last of them
        is garbage-collected, so keeping any one of them (say only `support`)
        keeps every result buffer of the mine alive.  copy=True returns
        independent, writable copies and frees the library's buffers at once."""
        out = ctypes.POINTER(_lib.Patterns)()
        check(self._L.fsm_spade_mine(self._ctx, db.handle, float(support), 1 if dfs else 0,
                                     ctypes.byref(out)), self._ctx)
        owner = _ResultOwner(self._L.fsm_patterns_free, out)
        p = out.contents
        n = p.n
        sup = owner.view(p.support, n, np.int32)
        po = owner.view(p.pat_off, n + 1, np.int64)
        so = owner.view(p.set_off, p.n_sets + 1, np.int64)
        it = owner.view(p.items, p.n_items, np.int32)
        meta = {"total": p.total, "minsup": p.minsup, "n": n}
        if copy:
            sup, po, so, it = sup.copy(), po.copy(), so.copy(), it.copy()
        return (sup, po, so, it), meta

    def spade(self, db, support, dfs=True):
        """-> (patterns: list[(itemsets tuple-of-tuples, support)], meta dict)."""
        (sup, po, so, it), meta = self.spade_csr(db, support, dfs)
        n = meta["n"]
        itl = it.tolist()
        sol = so.tolist()
        pats = []
        for i in range(n):
            sets = tuple(tuple(itl[sol[s]:sol[s + 1]]) for s in range(po[i], po[i + 1]))
            pats.append((sets, int(sup[i])))
        return pats, meta

    def tsr(self, db, k, minconf):
        """-> (rules: list[(antecedent, consequent, support, confidence)], meta)."""
        out = ctypes.POINTER(_lib.Rules)()
        check(self._L.fsm_tsr_mine(self._ctx, db.handle, int(k), float(minconf), ctypes.byref(out)), self._ctx)
        try:
            r = out.contents
            rules = []
            for i in range(r.n):
                x = tuple(r.ante[q] for q in range(r.ante_off[i], r.ante_off[i + 1]))
                y = tuple(r.cons[q] for q in range(r.cons_off[i], r.cons_off[i + 1]))
                rules.append((x, y, r.support[i], r.confidence[i]))
            meta = {"total": r.total, "final_minsup": r.final_minsup}
        finally:
            self._L.fsm_rules_free(out)
        return rules, meta

    def tsr_mined(self, db, k, minconf):
        """fsm_tsr_mine -> MinedRules: the library's rule set kept as mined (no copy), for
        the rule queries and documents that run on it through the C ABI."""
        out = ctypes.POINTER(_lib.Rules)()
        check(self._L.fsm_tsr_mine(self._ctx, db.handle, int(k), float(minconf), ctypes.byref(out)), self._ctx)
        return MinedRules(self._L, out)

    def kernel_stats(self):
        """[{name, launches, alg_bytes, survey_bytes, ms}] of the last mine call (device time, HIP
        events; alg_bytes: the kernel's own layout, survey_bytes: SURVEY §8(d) units)."""
        n = ctypes.c_int32()
        check(self._L.fsm_get_kernel_stats(self._ctx, None, 0, ctypes.byref(n)), self._ctx)
        arr = (_lib.KernelStat * max(n.value, 1))()
        check(self._L.fsm_get_kernel_stats(self._ctx, arr, n.value, ctypes.byref(n)), self._ctx)
        return [{"name": k.name.decode(), "launches": k.launches, "alg_bytes": k.alg_bytes,
                 "survey_bytes": k.survey_bytes, "ms": k.ms} for k in arr[:n.value]]

    def stats(self):
        st = _lib.Stats()
        check(self._L.fsm_get_stats(self._ctx, ctypes.byref(st)), self._ctx)
        return st.as_dict()


class MinedRules:
    """A mined fsm_rules (library-owned, freed with the object): its rules, and the
    rule queries (fsm_rules_query, FSMQuestor.scala:46-98) and json4s document
    (fsm_rules_json) computed on it by the library."""

    def __init__(self, L, ptr):
        self._L, self._p = L, ptr
        weakref.finalize(self, L.fsm_rules_free, ptr)
        r = ptr.contents
        self.total, self.final_minsup, self.n = r.total, r.final_minsup, r.n

    def rules(self):
        """[(antecedent, consequent, support, confidence)] in the library's order."""
        r = self._p.contents
        out = []
        for i in range(r.n):
            x = tuple(r.ante[q] for q in range(r.ante_off[i], r.ante_off[i + 1]))
            y = tuple(r.cons[q] for q in range(r.cons_off[i], r.cons_off[i + 1]))
            out.append((x, y, r.support[i], r.confidence[i]))
        return out

    def query(self, side, items):
        """Indexes (ascending) of the rules whose antecedent (side 0) / consequent (side 1)
        items all occur in `items`."""
        q = np.ascontiguousarray(list(items), np.int32)
        idx = np.zeros(max(self.n, 1), np.int64)
        n = ctypes.c_int64()
        check(self._L.fsm_rules_query(self._p, int(side), q.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(q),
                                      idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), ctypes.byref(n)))
        return idx[:n.value].tolist()

    def to_json(self):
        out, n = ctypes.c_void_p(), ctypes.c_int64()
        check(self._L.fsm_rules_json(self._p, ctypes.byref(out), ctypes.byref(n)))
        try:
            return ctypes.string_at(out, n.value).decode("utf-8")
        finally:
            self._L.fsm_buffer_free(out)


class DB:
    def __init__(self, engine, handle, mode):
        self.engine = engine
        self.handle = handle
        self.mode = mode

    def free(self):
        if self.handle:
            self.engine._L.fsm_db_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


_default = None


def default_engine():
    global _default
    if _default is None:
        _default = Engine(0)
    return _default
