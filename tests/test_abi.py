"""CPU tests of the drop-in boundary: libfsm.so loads, exports every function
include/fsm.h declares, its structs match the ctypes mirror, and it fails
loudly (no CPU fallback) when no gfx950 device is present.  Also the host-side
result mappings of SPADEActor / TSRActor.  No GPU compute calls."""
import ctypes
import os
import re
import subprocess

import pytest

import spark_fsm_amd as fsm
from spark_fsm_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fsm.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fsm_[a-z_0-9]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert header_functions() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    assert os.path.exists(_lib.LIB_PATH), "libfsm.so not built"
    L = ctypes.CDLL(_lib.LIB_PATH)
    for name in header_functions():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (fsm_\w+)", out))
    assert set(header_functions()) <= exported


def test_abi_version_and_struct_sizes():
    L = _lib.load()
    assert L.fsm_abi_version() == 7
    assert ctypes.sizeof(_lib.Opts) == 4 * 4 + 128 + 8 + 8 + 4 + 16 * 4 + 4  # (+4: tail padding)
    assert ctypes.sizeof(_lib.Patterns) == 9 * 8  # 8 x 8-byte fields + int32 padded
    assert ctypes.sizeof(_lib.Stats) == 9 * 8 + 8 * 8 + 3 * 8 + 2 * 8 + 8 * 8 + 4 * 8 + 3 * 8
    assert ctypes.sizeof(_lib.KernelStat) == 40 + 4 * 8
    assert ctypes.sizeof(_lib.HostComm) == 4 * 8
    assert ctypes.sizeof(_lib.DbImage) == 8 + 4 * 8 + 6 * 8


def test_no_cpu_fallback_without_gpu():
    """On a machine without a gfx950 GPU, context creation must fail loudly."""
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present")
    with pytest.raises(fsm.FsmError) as ei:
        fsm.Engine(0)
    assert ei.value.code in (_lib.FSM_EDEVICE, _lib.FSM_EINVAL)


def test_invalid_arguments_are_rejected_before_device_use():
    L = _lib.load()
    out = ctypes.c_void_p()
    assert L.fsm_db_from_spmf(None, 0, None, None, None, 0, ctypes.byref(out)) == _lib.FSM_EINVAL
    assert L.fsm_spade_mine(None, None, 0.5, 1, None) == _lib.FSM_EINVAL
    assert L.fsm_tsr_mine(None, None, 10, 0.5, None) == _lib.FSM_EINVAL
    L.fsm_patterns_free(None)
    L.fsm_rules_free(None)
    L.fsm_db_free(None)
    L.fsm_ctx_destroy(None)


def test_pattern_serialize_and_actor_mapping():
    p = fsm.Pattern(((1,), (3, 4), (3,)), 7)
    assert p.serialize() == "1 -1 3 4 -1 3 -1 | 7"
    assert fsm.spade_actor_patterns([p]) == [(7, [[1], [3, 4], [3]])]


def test_actor_mapping_fails_like_scala_on_minus_one_prefix_items():
    # SPADEActor splits serialize() on "-1": an item -12 serializes to "-12",
    # which the Scala mapping mangles and then fails to parse (SPADEActor.scala:198)
    with pytest.raises(ValueError):
        fsm.spade_actor_patterns([fsm.Pattern(((-12,),), 3)])
    assert fsm.spade_actor_patterns([fsm.Pattern(((-5,), (2,)), 3)]) == [(3, [[-5], [2]])]


def test_tsr_actor_mapping():
    r = fsm.Rule([1, 2], [5], 10, 0.5)
    assert fsm.tsr_actor_rules([r], 99) == [([1, 2], [5], 10, 99, 0.5)]


def test_struct_layout_matches_c_compiler(tmp_path):
    """sizeof / offsetof of every ABI struct as gcc sees include/fsm.h == the ctypes mirror."""
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "fsm.h"\nint main(void){\n'
                   'printf("%zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(fsm_opts), sizeof(fsm_patterns),'
                   ' sizeof(fsm_rules), sizeof(fsm_stats), sizeof(fsm_host_comm), sizeof(fsm_kernel_stat),'
                   ' offsetof(fsm_opts, host_comm), offsetof(fsm_stats, bytes_count_alg));\n'
                   'printf("%zu %zu\\n", offsetof(fsm_opts, ndevices), offsetof(fsm_opts, devices));\nreturn 0;}\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    exp = [ctypes.sizeof(_lib.Opts), ctypes.sizeof(_lib.Patterns), ctypes.sizeof(_lib.Rules),
           ctypes.sizeof(_lib.Stats), ctypes.sizeof(_lib.HostComm), ctypes.sizeof(_lib.KernelStat),
           _lib.Opts.host_comm.offset,
           _lib.Stats.bytes_count_alg.offset, _lib.Opts.ndevices.offset, _lib.Opts.devices.offset]
    assert got == exp
