"""N > 1 plumbing on the CPU: the shard plan the engine uses for first-level
prefix classes, and the host-callback collectives (all-reduce, ragged
all-gather) between world_size-2 gloo processes through libfsm's own
fsm_comm_selftest.  The sharded mining itself runs on the GPU in
tests/test_parity_gpu.py::test_sharded_spade_two_ranks."""
import ctypes
import json
import os
import random
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "dist_worker.py")


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(world, args, tmp_path, timeout=300):
    """Start `world` worker processes (gloo rendezvous on 127.0.0.1); return their JSON results."""
    port = free_port()
    procs, outs = [], []
    for r in range(world):
        out = str(tmp_path / ("rank%d.json" % r))
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, WORKER] + [args[0], out] + list(args[1:]), env=env))
        outs.append(out)
    try:
        codes = [p.wait(timeout=timeout) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert codes == [0] * world, codes
    res = []
    for o in outs:
        with open(o) as f:
            res.append(json.load(f))
    return res


def test_shard_plan_is_a_balanced_partition():
    from spark_fsm_amd import shard_plan
    rng = random.Random(5)
    for _ in range(50):
        n = rng.randint(0, 300)
        vol = [rng.choice([1, 10, 100, 5000]) * rng.randint(1, 9) for _ in range(n)]
        for N in (1, 2, 3, 8):
            own = shard_plan(vol, N)
            assert len(own) == n and all(0 <= o < N for o in own)
            assert (own == shard_plan(vol, N)).all()  # deterministic: every rank computes the same plan
            load = np.bincount(own, weights=np.array(vol, dtype=float), minlength=N) if n else np.zeros(N)
            if n:
                # LPT: the heaviest rank carries at most the mean plus one unit
                assert load.max() <= sum(vol) / N + max(vol) + 1e-9


def test_shard_plan_largest_first():
    from spark_fsm_amd import shard_plan
    assert list(shard_plan([5, 3, 9, 1, 1, 7], 3)) == [2, 2, 0, 1, 1, 1]


@pytest.mark.parametrize("claims", ["1", "0", "rank0", "shm"])
@pytest.mark.parametrize("world", [2, 3])
def test_host_comm_collectives_gloo(world, claims, tmp_path, monkeypatch):
    """fsm_comm_selftest over gloo: all-reduce, ragged all-gather and the work-stealing
    counter: ranks claiming ranges of r + 1 units until it runs out take every unit
    exactly once (checked inside the self-test).  claims=1: the store's counter through
    fsm_host_comm.fetch_add; shm: the node's shared-memory counters the RCCL
    communicator uses (a unique id, no callback); 0 / rank0: no common counter, the
    ranks agree on the static plan."""
    monkeypatch.setenv("FSM_TEST_CLAIMS", claims)
    if claims in ("1", "shm"):
        monkeypatch.setenv("FSM_SELFTEST_REQUIRE_CLAIMS", "1")
    res = run_ranks(world, ["selftest"], tmp_path, timeout=180)
    assert [r["rank"] for r in res] == list(range(world)) and all(r["ok"] for r in res)
    assert [r["claims"] for r in res] == [claims == "1" or (claims == "rank0" and r == 0) for r in range(world)]


def test_selftest_rejects_single_rank():
    import ctypes
    from spark_fsm_amd import _lib
    L = _lib.load()
    o = _lib.Opts()
    o.nranks = 1
    assert L.fsm_comm_selftest(ctypes.byref(o)) == _lib.FSM_EINVAL


def test_rccl_unique_id():
    """librccl is dlopen'ed lazily; ncclGetUniqueId needs no GPU."""
    from spark_fsm_amd import FsmError, comm_unique_id
    try:
        uid = comm_unique_id()
    except FsmError as e:  # pragma: no cover - image without librccl
        pytest.skip(str(e))
    assert isinstance(uid, bytes) and len(uid) == 128 and any(uid)


@pytest.mark.parametrize("n", [2, 3, 8, 16])
def test_inproc_comm_selftest(n):
    """The in-process transport of a multi-device context (fsm_opts.ndevices): n host
    threads run the collectives and the claim counter (every unit claimed once)."""
    from spark_fsm_amd import dist as fdist
    for _ in range(5):  # the hub is re-armed between calls
        fdist.selftest_inproc(n)


def test_inproc_comm_failure_releases_peers(monkeypatch):
    """A rank that fails before its first collective aborts the hub: the peers leave their
    barrier with FSM_ECOMM instead of blocking, the caller sees the failing rank's own
    error, and the next call on a fresh group works."""
    from spark_fsm_amd import FsmError, _lib
    from spark_fsm_amd import dist as fdist
    for r in (0, 2):
        monkeypatch.setenv("FSM_INJECT_FAIL", "%d,selftest" % r)
        with pytest.raises(FsmError) as ei:
            fdist.selftest_inproc(4)
        assert ei.value.code == _lib.FSM_ELIMIT and "injected" in ei.value.msg
    monkeypatch.delenv("FSM_INJECT_FAIL")
    fdist.selftest_inproc(4)


def test_inproc_rejects_bad_device_lists():
    from spark_fsm_amd import FsmError, _lib
    L = _lib.load()
    o = _lib.Opts()
    o.ndevices = _lib.MAX_DEVICES + 1
    assert L.fsm_comm_selftest(ctypes.byref(o)) == _lib.FSM_EINVAL
    o.ndevices, o.nranks = 2, 2
    ctx = ctypes.c_void_p()
    assert L.fsm_ctx_create(ctypes.byref(o), ctypes.byref(ctx)) == _lib.FSM_EINVAL


@pytest.mark.parametrize("stall_s", ["1", "6"])
def test_inproc_stalled_rank_returns_ecomm(monkeypatch, stall_s):
    """A rank that stalls (FSM_INJECT_STALL: it sleeps before its first collective) never
    leaves the call hanging: its peers' barriers wait FSM_COMM_TIMEOUT_S, abort the hub and
    the call returns FSM_ECOMM, within the limit plus the group's 2 s grace even while the
    stalled rank is still asleep (6 s: the group is then reported stalled and leaked, so the
    JVM actor records FAILURE instead of staying at MINING_STARTED, TrainActor.scala:56-67).
    A new group works afterwards."""
    import time
    from spark_fsm_amd import FsmError, _lib
    from spark_fsm_amd import dist as fdist
    monkeypatch.setenv("FSM_COMM_TIMEOUT_S", "0.5")
    monkeypatch.setenv("FSM_INJECT_STALL", "2,selftest,%s" % stall_s)
    t0 = time.monotonic()
    with pytest.raises(FsmError) as ei:
        fdist.selftest_inproc(4)
    dt = time.monotonic() - t0
    assert ei.value.code == _lib.FSM_ECOMM, ei.value.msg
    assert dt < 4.5, dt
    if stall_s == "6":
        assert "did not return" in ei.value.msg and "2" in ei.value.msg
    else:
        assert "timed out" in ei.value.msg or "peer rank failed" in ei.value.msg
    monkeypatch.delenv("FSM_INJECT_STALL")
    fdist.selftest_inproc(4)
