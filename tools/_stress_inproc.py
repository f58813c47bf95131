import ctypes, json, os, sys, subprocess, time
ROOT = "/root/repo"
sys.path[:0] = [ROOT, ROOT + "/spark-fsm_amd", ROOT + "/tests"]
import spark_fsm_amd  # noqa
out = "/tmp/libjniharness.so"
LIBDIR = ROOT + "/spark-fsm_amd/spark_fsm_amd"
subprocess.run(["gcc", "-O1", "-fPIC", "-shared", "-I" + ROOT + "/tests/jni", "-I" + ROOT + "/include",
                ROOT + "/jvm/native/fsm_jni.c", ROOT + "/tests/jni/jni_harness.c", "-L" + LIBDIR, "-lfsm",
                "-Wl,-rpath," + LIBDIR, "-o", out], check=True)
L = ctypes.CDLL(out)
L.harness_spade.restype = ctypes.c_void_p
IP = ctypes.POINTER(ctypes.c_int)
L.harness_spade.argtypes = [ctypes.c_int, IP, ctypes.POINTER(ctypes.c_char_p), ctypes.c_double, ctypes.c_int, IP]
L.harness_free.argtypes = [ctypes.c_void_p]
cases = json.load(open(ROOT + "/tests/golden/spade_cases.json"))
devs = (ctypes.c_int * 3)(0, 0, 0)
t0 = time.time()
for it in range(int(sys.argv[1])):
    for ci, case in enumerate(cases):
        recs = [tuple(r) for r in case["records"]]
        n = len(recs)
        sids = (ctypes.c_int * max(n, 1))(*[s for s, _ in recs])
        lines = (ctypes.c_char_p * max(n, 1))(*[l.encode() for _, l in recs])
        print("it", it, "case", ci, case["name"], round(time.time() - t0, 1), flush=True)
        p = L.harness_spade(n, sids, lines, case["support"], 3, devs)
        L.harness_free(p)
print("done", flush=True)
