"""ctypes binding of libfsm.so (include/fsm.h).

The library is the product: there is no CPU fallback.  If libfsm.so is missing
or no gfx950 device is present, the calls fail loudly (FsmError).

HIP runtime note: PyTorch wheels bundle their own libamdhip64.so.  To keep a
single HIP runtime per process, torch (when installed) is imported before the
library is loaded, so libfsm binds to the runtime torch already brought in.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FSM_LIB_PATH") or os.path.join(HERE, "libfsm.so")  # override: tuning variants

FSM_OK, FSM_EINVAL, FSM_EPARSE, FSM_EDEVICE, FSM_ENOMEM, FSM_ECOMM, FSM_ELIMIT = range(7)
MODE_SPADE, MODE_TSR = 0, 1
MAX_DEVICES = 16  # FSM_MAX_DEVICES


class FsmError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("[fsm error %d] %s" % (code, msg))
        self.code = code
        self.msg = msg


class FsmParseError(FsmError):
    """Input the reference itself would throw on (-> TrainActor FAILURE)."""


ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int64)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64)
FETCH_ADD_FN = ctypes.CFUNCTYPE(ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64)


class HostComm(ctypes.Structure):
    _fields_ = [
        ("user", ctypes.c_void_p),
        ("allreduce_u32", ALLREDUCE_FN),
        ("allgather", ALLGATHER_FN),
        ("fetch_add", FETCH_ADD_FN),
    ]


class Opts(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int32),
        ("nranks", ctypes.c_int32),
        ("rank", ctypes.c_int32),
        ("verbose", ctypes.c_int32),
        ("unique_id", ctypes.c_uint8 * 128),
        ("mem_budget", ctypes.c_int64),
        ("host_comm", ctypes.POINTER(HostComm)),
        ("ndevices", ctypes.c_int32),
        ("devices", ctypes.c_int32 * MAX_DEVICES),
    ]


class Patterns(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int64),
        ("support", ctypes.POINTER(ctypes.c_int32)),
        ("pat_off", ctypes.POINTER(ctypes.c_int64)),
        ("set_off", ctypes.POINTER(ctypes.c_int64)),
        ("items", ctypes.POINTER(ctypes.c_int32)),
        ("n_sets", ctypes.c_int64),
        ("n_items", ctypes.c_int64),
        ("total", ctypes.c_int64),
        ("minsup", ctypes.c_int32),
    ]


class Rules(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int64),
        ("support", ctypes.POINTER(ctypes.c_int32)),
        ("confidence", ctypes.POINTER(ctypes.c_double)),
        ("ante_off", ctypes.POINTER(ctypes.c_int64)),
        ("ante", ctypes.POINTER(ctypes.c_int32)),
        ("cons_off", ctypes.POINTER(ctypes.c_int64)),
        ("cons", ctypes.POINTER(ctypes.c_int32)),
        ("total", ctypes.c_int64),
        ("final_minsup", ctypes.c_int32),
    ]


class DbImage(ctypes.Structure):
    _fields_ = [
        ("mode", ctypes.c_int32),
        ("mask_words", ctypes.c_int32),
        ("rows", ctypes.c_int64),
        ("entries", ctypes.c_int64),
        ("items", ctypes.c_int64),
        ("max_occ", ctypes.c_int64),
        ("row_off", ctypes.POINTER(ctypes.c_uint32)),
        ("item", ctypes.POINTER(ctypes.c_uint32)),
        ("mask", ctypes.POINTER(ctypes.c_uint64)),
        ("first", ctypes.POINTER(ctypes.c_uint32)),
        ("last", ctypes.POINTER(ctypes.c_uint32)),
        ("item_val", ctypes.POINTER(ctypes.c_int32)),
    ]


class TokenDb(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int64),
        ("sids", ctypes.POINTER(ctypes.c_int32)),
        ("seq_off", ctypes.POINTER(ctypes.c_int64)),
        ("tokens", ctypes.POINTER(ctypes.c_int64)),
        ("n_tokens", ctypes.c_int64),
    ]


FMT_SPMF, FMT_INDEXED, FMT_BMS, FMT_CSV, FMT_KOSARAK, FMT_SNAKE = range(6)


class KernelStat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 40), ("launches", ctypes.c_int64), ("alg_bytes", ctypes.c_int64),
                ("ms", ctypes.c_double), ("survey_bytes", ctypes.c_int64)]


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in (
        "joins", "patterns", "classes", "batches", "entries", "bytes_join_equiv",
        "bytes_streamed", "expansions", "rules")] + [(n, ctypes.c_double) for n in (
        "ms_flatten", "ms_upload", "ms_f1", "ms_f2", "ms_lattice", "ms_mine",
        "ms_count_kernel", "ms_emit_kernel")] + [(n, ctypes.c_int64) for n in (
        "count_launches", "mask_words", "bytes_count_alg")] + [(n, ctypes.c_double) for n in (
        "ms_gpu_wait", "ms_output")] + [(n, ctypes.c_int64) for n in (
        "joins_root", "root_keys", "pair_tests", "root_entries", "k0_device", "exp_domain", "exp_entries",
        "exp_bitmap_bytes", "rank_claims", "rank_root_owned", "rank_root_slab", "rank_units",
        "db_parses", "db_replicas", "tsr_ring_waits")]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


# Every symbol declared in include/fsm.h (checked by tests/test_abi.py).
EXPORTS = [
    "fsm_abi_version", "fsm_comm_unique_id", "fsm_shard_plan", "fsm_comm_selftest", "fsm_ctx_create", "fsm_ctx_destroy",
    "fsm_last_error", "fsm_get_stats", "fsm_get_kernel_stats", "fsm_db_from_spmf", "fsm_db_from_tokens",
    "fsm_db_free", "fsm_spade_mine", "fsm_patterns_free", "fsm_tsr_mine", "fsm_rules_free",
    "fsm_db_export", "fsm_db_image_free", "fsm_ingest", "fsm_token_db_free", "fsm_patterns_serialize",
    "fsm_patterns_json", "fsm_rules_json", "fsm_buffer_free", "fsm_rules_query",
]

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    try:  # one HIP runtime per process: bind to torch's if torch is present
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise FsmError(FSM_EDEVICE, "libfsm.so not built (%s); run __graft_entry__.build()" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER
    vp = ctypes.c_void_p
    L.fsm_abi_version.restype = ctypes.c_int
    L.fsm_comm_unique_id.argtypes = [P(ctypes.c_uint8)]
    L.fsm_shard_plan.argtypes = [P(ctypes.c_uint64), ctypes.c_int64, ctypes.c_int32, P(ctypes.c_int32)]
    L.fsm_comm_selftest.argtypes = [P(Opts)]
    L.fsm_ctx_create.argtypes = [P(Opts), P(vp)]
    L.fsm_ctx_destroy.argtypes = [vp]
    L.fsm_ctx_destroy.restype = None
    L.fsm_last_error.argtypes = [vp]
    L.fsm_last_error.restype = ctypes.c_char_p
    L.fsm_get_stats.argtypes = [vp, P(Stats)]
    L.fsm_get_kernel_stats.argtypes = [vp, P(KernelStat), ctypes.c_int32, P(ctypes.c_int32)]
    L.fsm_db_from_spmf.argtypes = [vp, ctypes.c_int32, P(ctypes.c_int32), P(ctypes.c_char_p),
                                   P(ctypes.c_int64), ctypes.c_int64, P(vp)]
    L.fsm_db_from_tokens.argtypes = [vp, ctypes.c_int32, P(ctypes.c_int32), P(ctypes.c_int64),
                                     P(ctypes.c_int64), ctypes.c_int64, P(vp)]
    L.fsm_db_export.argtypes = [vp, vp, P(P(DbImage))]
    L.fsm_db_image_free.argtypes = [P(DbImage)]
    L.fsm_db_image_free.restype = None
    L.fsm_db_free.argtypes = [vp]
    L.fsm_db_free.restype = None
    L.fsm_spade_mine.argtypes = [vp, vp, ctypes.c_double, ctypes.c_int32, P(P(Patterns))]
    L.fsm_patterns_free.argtypes = [P(Patterns)]
    L.fsm_patterns_free.restype = None
    L.fsm_tsr_mine.argtypes = [vp, vp, ctypes.c_int32, ctypes.c_double, P(P(Rules))]
    L.fsm_rules_free.argtypes = [P(Rules)]
    L.fsm_rules_free.restype = None
    if hasattr(L, "fsm_ingest"):  # (absent only from older builds loaded through FSM_LIB_PATH for A/B runs)
        L.fsm_ingest.argtypes = [ctypes.c_int32, ctypes.c_char_p, ctypes.c_int64, ctypes.c_int64, P(P(TokenDb))]
        L.fsm_token_db_free.argtypes = [P(TokenDb)]
        L.fsm_token_db_free.restype = None
        for fn, st in (("fsm_patterns_serialize", Patterns), ("fsm_patterns_json", Patterns), ("fsm_rules_json", Rules)):
            getattr(L, fn).argtypes = [P(st), P(vp), P(ctypes.c_int64)]
        L.fsm_buffer_free.argtypes = [vp]
        L.fsm_buffer_free.restype = None
        L.fsm_rules_query.argtypes = [P(Rules), ctypes.c_int32, P(ctypes.c_int32), ctypes.c_int64,
                                      P(ctypes.c_int64), P(ctypes.c_int64)]
    _lib = L
    return L


def check(rc, ctx=None):
    if rc == FSM_OK:
        return
    msg = load().fsm_last_error(ctx)
    msg = msg.decode("utf-8", "replace") if msg else ""
    if rc == FSM_EPARSE:
        raise FsmParseError(rc, msg)
    raise FsmError(rc, msg)
