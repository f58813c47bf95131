"""The JVM drop-in: jvm/native/fsm_jni.c is compiled here
against tests/jni/jni.h (the JNI subset it uses; the image has no JDK) and
driven through tests/jni/jni_harness.c, an in-process JNIEnv that renders the
results exactly as the Scala bodies (jvm/scala/.../GpuSPADE.scala, GpuTSR.scala)
map them: GpuPattern.serialize() lines, GpuRule lines.

CPU: the shim builds, exports the two JNI symbols FsmNativeJNI.java binds, and
turns a failure (no GPU here) into a java.lang.Exception, never a crash or an
Error (TrainActor.scala:66 only catches Exception).
GPU: the shim's results equal the engine's through the Python mirror
(spark_fsm_amd.extract_rdd_patterns / extract_rdd_rules) on the golden records.
"""
import ctypes
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "spark-fsm_amd", "spark_fsm_amd")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("jni") / "libjniharness.so")
    subprocess.run(["gcc", "-O1", "-fPIC", "-shared", "-Wall", "-Wextra", "-Werror",
                    "-I" + os.path.join(ROOT, "tests", "jni"), "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "jvm", "native", "fsm_jni.c"), os.path.join(ROOT, "tests", "jni", "jni_harness.c"),
                    "-L" + LIBDIR, "-lfsm", "-Wl,-rpath," + LIBDIR, "-o", out], check=True)
    import spark_fsm_amd  # noqa: F401  (torch first: one HIP runtime per process)
    L = ctypes.CDLL(out)
    for name in ("harness_spade", "harness_tsr"):
        getattr(L, name).restype = ctypes.c_void_p
    IP = ctypes.POINTER(ctypes.c_int)
    L.harness_spade.argtypes = [ctypes.c_int, IP, ctypes.POINTER(ctypes.c_char_p), ctypes.c_double, ctypes.c_int, IP]
    L.harness_tsr.argtypes = [ctypes.c_int, IP, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.c_double,
                              ctypes.c_int, IP]
    L.harness_free.argtypes = [ctypes.c_void_p]
    L.path = out
    return L


def call(L, fn, records, *args, devices=(0,)):
    """devices: FsmNative.devices as the Scala side passes it (-Dfsm.devices)."""
    n = len(records)
    sids = (ctypes.c_int * max(n, 1))(*[s for s, _ in records])
    lines = (ctypes.c_char_p * max(n, 1))(*[l.encode() for _, l in records])
    devs = (ctypes.c_int * max(len(devices), 1))(*devices)
    p = getattr(L, fn)(n, sids, lines, *args, len(devices), devs)
    try:
        return ctypes.string_at(p).decode()
    finally:
        L.harness_free(p)


def gpu_present():
    try:
        import torch
        return torch.cuda.is_available()
    except ImportError:
        return False


def test_shim_exports_the_bound_symbols(harness):
    out = subprocess.run(["nm", "-D", "--defined-only", harness.path], capture_output=True, text=True).stdout
    assert "Java_de_kp_spark_fsm_gpu_FsmNativeJNI_spade" in out
    assert "Java_de_kp_spark_fsm_gpu_FsmNativeJNI_tsr" in out
    assert "Java_de_kp_spark_fsm_gpu_FsmNativeJNI_release" in out
    java = open(os.path.join(ROOT, "jvm", "java", "de", "kp", "spark", "fsm", "gpu", "FsmNativeJNI.java")).read()
    assert "static native Object[] spade(" in java and "static native Object[] tsr(" in java
    assert "static native void release()" in java


@pytest.mark.skipif(gpu_present(), reason="the no-device failure path needs a machine without a GPU")
def test_shim_turns_failures_into_exceptions(harness):
    s = call(harness, "harness_spade", [(0, "1 -1 2 -1")], 0.5)
    assert s.startswith("EXCEPTION java/lang/Exception: libfsm fsm_ctx_create failed (FSM error 3)")
    t = call(harness, "harness_tsr", [(0, "1 -1 2 -1")], 3, 0.5)
    assert t.startswith("EXCEPTION java/lang/Exception: libfsm fsm_ctx_create failed")
    # a multi-device request fails the same way (every rank context needs a GPU)
    s = call(harness, "harness_spade", [(0, "1 -1 2 -1")], 0.5, devices=(0, 1))
    assert s.startswith("EXCEPTION java/lang/Exception: libfsm fsm_ctx_create failed (FSM error 3)")


def test_shim_rejects_too_many_devices(harness):
    s = call(harness, "harness_spade", [(0, "1 -1 2 -1")], 0.5, devices=tuple(range(17)))
    assert s.startswith("EXCEPTION java/lang/Exception: libfsm fsm_ctx_create failed (FSM error 1)")


GOLD = os.path.join(ROOT, "tests", "golden")


# FsmNative.devices of the cases: one GPU, and in-process ranks on the one GPU of the box
# (-Dfsm.devices=0,0 / 0,0,0: the sharded engine reached from the drop-in)
DEVICE_LISTS = [(0,), (0, 0), (0, 0, 0)]


@pytest.mark.gpu
@pytest.mark.parametrize("devices", DEVICE_LISTS)
def test_shim_spade_matches_golden(harness, devices):
    """The JNI shim's Pattern.serialize() lines (SPADEActor.scala:49-50) equal
    the committed fixtures' patterns rendered the same way: every golden case,
    not a comparison with the engine's own Python path."""
    from spark_fsm_amd.api import Pattern
    for case in json.load(open(os.path.join(GOLD, "spade_cases.json"))):
        recs = [tuple(r) for r in case["records"]]
        got = call(harness, "harness_spade", recs, case["support"], devices=devices)
        exp = [Pattern([list(x) for x in sets], sup).serialize() for sets, sup in case["patterns"]]
        assert sorted(got.splitlines()) == sorted(exp), case["name"]
    err = json.load(open(os.path.join(GOLD, "error_cases.json")))["spade"][0]
    assert call(harness, "harness_spade", [tuple(r) for r in err["records"]], 0.5, devices=devices).startswith(
        "EXCEPTION java/lang/Exception: libfsm fsm_db_from_spmf failed (FSM error 2)")
    # every request above after the first reused the context (and rank group) the shim kept
    # idle; FsmNative's shutdown hook destroys them
    harness.Java_de_kp_spark_fsm_gpu_FsmNativeJNI_release(None, None)


@pytest.mark.gpu
@pytest.mark.parametrize("devices", DEVICE_LISTS)
def test_shim_tsr_matches_golden(harness, devices):
    """The JNI shim's Rule accessors (TSRActor.scala:55-59) equal the committed
    fixtures' rules: antecedent, consequent, support and the confidence as the
    same IEEE double (the shim prints Double.toString's shortest form)."""
    for case in json.load(open(os.path.join(GOLD, "tsr_cases.json"))):
        recs = [tuple(r) for r in case["records"]]
        got = call(harness, "harness_tsr", recs, case["k"], case["minconf"], devices=devices)
        exp = ["%s ==> %s #SUP: %d #CONF: %s" % (",".join(map(str, x)), ",".join(map(str, y)), sup, repr(float(c)))
               for x, y, sup, c in case["rules"]]
        norm = lambda lines: sorted((l.rsplit(" ", 1)[0], float(l.rsplit(" ", 1)[1])) for l in lines)
        assert norm(got.splitlines()) == norm(exp), case["name"]
    for err in json.load(open(os.path.join(GOLD, "error_cases.json")))["tsr"]:
        out = call(harness, "harness_tsr", [tuple(r) for r in err["records"]], 3, 0.5, devices=devices)
        assert out.startswith("EXCEPTION java/lang/Exception: libfsm ") and "(FSM error 2)" in out, err["name"]
    harness.Java_de_kp_spark_fsm_gpu_FsmNativeJNI_release(None, None)
