"""Full-size parity at the BASELINE configs (VERDICT r1 "next round" item 1).

SPADE (configs 1, 2, 3, 5): libfsm's complete pattern set at the BASELINE
size and minsup must equal the CPU restatement's, compared through the
canonical digest of tests/digest.py (count, support sum, SHA-256 over the
sorted per-pattern keys) plus the join count and the absolute minsup.  The
expected values were computed in the build container by
tests/golden/make_fullsize.py (oracle/fsm_oracle.c, complete runs) and are
committed in tests/golden/fullsize.json.

TSR (config 4, 990,002 Kosarak-shaped sequences, k = 1000, minconf 0.5): the
top-k restatement cannot finish at full size, so (a) the 20,000- and
100,000-sequence prefixes are compared exactly (rule digest, final minsup), and
(b) the full-size result is checked against EVERY valid rule with sup >= 575,
enumerated by definition at that fixed threshold (c4_complete.json): each
returned rule has the definitional support and IEEE confidence, and every valid
rule with sup > the final minsup is returned.
"""
import json
import os

import pytest

from digest import pattern_digest, rule_digest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "fullsize.json")
with open(GOLD) as f:
    FULL = json.load(f)

SPADE_CFG = {"c1": ("quest", 10000), "c2": ("quest", 100000), "c3": ("quest", 1000000),
             "c5-bible": ("bible", None), "c5-sign": ("sign", None)}


def dataset(shape, D):
    from tools import gen
    if shape == "quest":
        return gen.quest(D, seed=1)
    return getattr(gen, shape)(seed=1)


@pytest.fixture(scope="module")
def eng():
    import spark_fsm_amd as fsm
    e = fsm.Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("name", [n for n in SPADE_CFG if n in FULL])
def test_spade_fullsize_digest(eng, name):
    import spark_fsm_amd as fsm
    exp = FULL[name]
    ds = dataset(*SPADE_CFG[name])
    assert ds.name == exp["dataset"] and len(ds) == exp["sequences"]
    db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_SPADE)
    try:
        csr, meta = eng.spade_csr(db, exp["support"])
    finally:
        db.free()
    st = eng.stats()
    assert meta["minsup"] == exp["minsup"]
    assert st["joins"] == exp["joins"]
    assert pattern_digest(*csr) == exp["digest"]


@pytest.mark.parametrize("name", ["c4-prefix", "c4-prefix100k"])
def test_tsr_c4_prefix_exact(eng, name):
    import spark_fsm_amd as fsm
    from tools import gen
    if name not in FULL:
        pytest.skip("fixture not generated")
    exp = FULL[name]
    ds = gen.kosarak(D=990002, seed=1).head(exp["sequences"])
    assert ds.name == exp["dataset"]
    db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_TSR)
    try:
        rules, meta = eng.tsr(db, exp["k"], exp["minconf"])
    finally:
        db.free()
    assert meta["final_minsup"] == exp["final_minsup"]
    assert rule_digest(rules) == exp["digest"]


COMPLETE = os.path.join(os.path.dirname(__file__), "golden", "c4_complete.json")


@pytest.mark.skipif(not os.path.exists(COMPLETE), reason="fixture not generated")
def test_tsr_c4_fullsize_complete(eng):
    """SURVEY §8(c)(i)+(ii) at full size (990,002 sequences, k = 1000, minconf
    0.5; TSR.scala:102-105).  tests/golden/c4_complete.json holds EVERY valid
    rule with sup >= T (oracle/tsr_exhaustive.c: definitional, fixed threshold,
    make_c4_complete.py), so with the GPU's final minsup m >= T:
      (i)  every returned rule is in that set with the identical support and
           the identical IEEE confidence;
      (ii) every valid rule with sup > m is returned (completeness);
    plus |R| >= k and m = min sup(R)."""
    import spark_fsm_amd as fsm
    from tools import gen
    with open(COMPLETE) as f:
        exp = json.load(f)
    ds = gen.kosarak(D=990002, seed=1)
    assert ds.name == exp["dataset"] and len(ds) == exp["sequences"]
    db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_TSR)
    try:
        rules, meta = eng.tsr(db, exp["k"], exp["minconf"])
    finally:
        db.free()
    m = meta["final_minsup"]
    assert meta["total"] == exp["sequences"] and m >= exp["t"]
    assert len(rules) >= exp["k"] and m == min(r[2] for r in rules)
    valid = {(tuple(x), tuple(y)): (s, float.fromhex(c)) for x, y, s, c in exp["rules"]}
    got = {(tuple(x), tuple(y)): (s, c) for x, y, s, c in rules}
    assert len(got) == len(rules)
    for key, v in got.items():
        assert valid.get(key) == v, (key, v, valid.get(key))
    missing = [k for k, v in valid.items() if v[0] > m and k not in got]
    assert not missing, missing[:5]


@pytest.mark.parametrize("shard_min", ["0", "default"])
@pytest.mark.parametrize("world", [2, 3])
def test_tsr_c4_prefix_sharded(world, shard_min, tmp_path, monkeypatch):
    """Sharded TSR at the c4 20,000-sequence prefix over `world` gloo ranks on this
    GPU: the pair phase by sequence range and the expansion launches' rule slots
    split over the ranks (results all-gathered per launch, replay replicated; every
    launch with FSM_TSR_SHARD_MIN=0, by default only those whose expected domain pays
    for the gather, the rest replicated) give the exact prefix digest and final minsup
    on every rank."""
    from test_dist import run_ranks
    if "c4-prefix" not in FULL:
        pytest.skip("fixture not generated")
    if shard_min != "default":
        monkeypatch.setenv("FSM_TSR_SHARD_MIN", shard_min)
    exp = FULL["c4-prefix"]
    res = run_ranks(world, ["tsr_digest", str(exp["sequences"]), str(exp["k"]), str(exp["minconf"])], tmp_path,
                    timeout=110)
    for r in res:
        assert r["digest"] == exp["digest"] and r["final_minsup"] == exp["final_minsup"]
    tot = sum(r["units"] for r in res)
    assert all(0 < r["units"] < tot for r in res)  # every rank expanded a share of the slots


@pytest.mark.parametrize("claims", ["auto", "forced"])
@pytest.mark.parametrize("name,world", [("c3", 2), ("c5-bible", 3)])
def test_spade_fullsize_sharded(name, world, claims, tmp_path, monkeypatch):
    """The sharded path (F1 all-reduce, DB-direct root with the counter rows by rank
    slice, frequent pairs all-gathered, first-level classes by the static largest-first
    plan or, forced here, claimed from the shared work-stealing counter, patterns
    all-gathered) at full BASELINE size, `world` ranks on this GPU over gloo host
    collectives: every rank returns the complete pattern set, and no rank joins root
    entries of classes it did not own."""
    from test_dist import run_ranks
    if claims == "forced":
        monkeypatch.setenv("FSM_SPADE_CLAIMS", "1")
    exp = FULL[name]
    shape, D = SPADE_CFG[name]
    res = run_ranks(world, ["spade_digest", shape, str(D or 0), str(exp["support"])], tmp_path, timeout=110)
    for r in res:
        assert r["digest"] == exp["digest"] and r["joins"] == exp["joins"] and r["minsup"] == exp["minsup"]
        assert r["rank_root_slab"] == 0  # DB-direct root: no rank writes root entries
    # the ranks' owned root entries partition the root (F2 slices + claimed classes: each
    # root entry joined as the owner at most twice, once per phase, by exactly one rank)
    assert sum(r["rank_root_owned"] for r in res) <= 2 * res[0]["root_entries"]
    if claims == "forced":
        assert sum(r["rank_claims"] for r in res) >= 1


def test_bench_two_ranks_dry_run(tmp_path):
    """bench.py's N > 1 code path (torch.distributed.run, barrier + max over
    ranks, sharded engine, one JSON line from rank 0), with two ranks sharing
    this GPU over gloo; the driver runs the same path over RCCL on 8 GPUs."""
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--dist-backend", "gloo", "--no-cpu-baseline"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=str(tmp_path))
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["value"] > 0
    assert d["extra"]["patterns"] == FULL["c3"]["digest"]["n"] and d["extra"]["joins"] == FULL["c3"]["joins"]
    pr = d["extra"]["per_rank"]  # the per-rank trace: each rank mined its share of the classes
    assert [r["rank"] for r in pr] == [0, 1] and all(r["classes"] > 0 for r in pr)
    assert sum(r["classes"] for r in pr) > max(r["classes"] for r in pr)


# ---------------------------------------------------------------- in-process ranks
# The drop-in's way to shard (fsm_opts.ndevices; the JVM caller is one driver thread,
# SPADE.scala:132-133 / TSR.scala:102-103): ONE context whose calls run rank r on
# devices[r] as threads of this process.  On the one-GPU box every rank is device 0.

@pytest.mark.parametrize("name,devices,claims", [("c3", (0, 0), "auto"), ("c3", (0, 0, 0), "forced"),
                                                 ("c5-bible", (0, 0), "forced"), ("c5-bible", (0, 0, 0), "auto"),
                                                 ("c3", (0,) * 4, "auto"), ("c3", (0,) * 8, "auto"),
                                                 ("c3", (0,) * 8, "forced"), ("c5-bible", (0,) * 4, "auto"),
                                                 ("c5-bible", (0,) * 8, "auto")])
def test_spade_fullsize_inproc(name, devices, claims, monkeypatch):
    """Config 3 (and BIBLE) at the rank counts config 3 names (2, 3, 4 and 8; here all on
    device 0): the F2 slices weighted by pair work, the 4- and 8-way static largest-first
    plan or the claims, the heavy-class split, to the full-size digests.  The ranks share
    the device's default memory budget (fsm_ctx::dev_share), and the DB is parsed once:
    rank 0 builds it, the others copy its resident arrays device to device."""
    import spark_fsm_amd as fsm
    if claims == "forced":
        monkeypatch.setenv("FSM_SPADE_CLAIMS", "1")
    exp = FULL[name]
    ds = dataset(*SPADE_CFG[name])
    with fsm.Engine(devices=list(devices)) as e:
        db = e.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_SPADE)
        st = e.stats()
        assert st["db_parses"] == 1 and st["db_replicas"] == len(devices) - 1
        try:
            for _ in range(2):  # the group is re-armed between calls (counters, hub)
                csr, meta = e.spade_csr(db, exp["support"])
                st = e.stats()
                assert meta["minsup"] == exp["minsup"]
                assert st["joins"] == exp["joins"]
                assert pattern_digest(*csr) == exp["digest"]
                assert st["rank_root_slab"] == 0
                if claims == "forced":
                    assert st["rank_claims"] >= 1
                # rank 0 owned only part of the root (the rest went to its peers)
                assert 0 < st["rank_root_owned"] < 2 * st["root_entries"]
        finally:
            db.free()


@pytest.mark.parametrize("devices,shard_min", [((0, 0), "0"), ((0, 0, 0), "0"), ((0, 0, 0), "default"),
                                                ((0,) * 4, "0"), ((0,) * 8, "0"), ((0,) * 8, "default")])
def test_tsr_c4_prefix_inproc(devices, shard_min, monkeypatch):
    """The c4 20K prefix over 2-8 in-process ranks: the pair phase by sequence range and the
    launches' rule slots split over the ranks (every launch with FSM_TSR_SHARD_MIN=0), to the
    exact prefix digest; the DB is parsed once and replicated device to device."""
    import spark_fsm_amd as fsm
    from tools import gen
    if shard_min != "default":
        monkeypatch.setenv("FSM_TSR_SHARD_MIN", shard_min)
    exp = FULL["c4-prefix"]
    ds = gen.kosarak(D=990002, seed=1).head(exp["sequences"])
    with fsm.Engine(devices=list(devices)) as e:
        db = e.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_TSR)
        bst = e.stats()
        assert bst["db_parses"] == 1 and bst["db_replicas"] == len(devices) - 1
        try:
            rules, meta = e.tsr(db, exp["k"], exp["minconf"])
        finally:
            db.free()
        st = e.stats()
    assert meta["final_minsup"] == exp["final_minsup"]
    assert rule_digest(rules) == exp["digest"]
    if shard_min == "0":
        assert 0 < st["rank_units"] < st["expansions"]  # rank 0 counted a share of the rule slots


def test_inproc_failure_agreement():
    """A failure injected on one in-process rank comes back as that rank's error from the one
    call (no rank left blocked), and the same context mines correctly afterwards."""
    import spark_fsm_amd as fsm
    exp = FULL["c1"]
    ds = dataset(*SPADE_CFG["c1"])
    with fsm.Engine(devices=[0, 0, 0]) as e:
        db = e.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_SPADE)
        try:
            for phase in ("root", "lattice"):
                os.environ["FSM_INJECT_FAIL"] = "1," + phase
                try:
                    with pytest.raises(fsm.FsmError) as ei:
                        e.spade_csr(db, exp["support"])
                finally:
                    del os.environ["FSM_INJECT_FAIL"]
                assert ei.value.code == 6 and "injected" in ei.value.msg, ei.value.msg
            csr, meta = e.spade_csr(db, exp["support"])
            assert pattern_digest(*csr) == exp["digest"]
        finally:
            db.free()


def test_inproc_stalled_rank_returns_ecomm(monkeypatch):
    """A rank that stalls inside a mine (FSM_INJECT_STALL: rank 2 sleeps 8 s at the root
    phase) does not hang the caller: its peers' barriers time out (FSM_COMM_TIMEOUT_S = 1 s),
    the call returns FSM_ECOMM within the limit and the 2 s grace, later calls return
    FSM_ECOMM while the rank is still asleep, and once it has returned the same context
    mines correctly again (the JNI shim throws, TrainActor records FAILURE, :65-67)."""
    import time
    import spark_fsm_amd as fsm
    exp = FULL["c1"]
    ds = dataset(*SPADE_CFG["c1"])
    with fsm.Engine(devices=[0, 0, 0]) as e:
        db = e.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_SPADE)
        try:
            monkeypatch.setenv("FSM_COMM_TIMEOUT_S", "1")
            monkeypatch.setenv("FSM_INJECT_STALL", "2,root,8")
            t0 = time.monotonic()
            with pytest.raises(fsm.FsmError) as ei:
                e.spade_csr(db, exp["support"])
            dt = time.monotonic() - t0
            monkeypatch.delenv("FSM_INJECT_STALL")
            assert ei.value.code == 5 and dt < 6.0, (dt, ei.value.msg)
            with pytest.raises(fsm.FsmError) as ei2:  # the rank is still asleep
                e.spade_csr(db, exp["support"])
            assert ei2.value.code == 5
            time.sleep(max(0.0, 9.0 - (time.monotonic() - t0)))
            monkeypatch.setenv("FSM_COMM_TIMEOUT_S", "60")
            csr, meta = e.spade_csr(db, exp["support"])
            assert pattern_digest(*csr) == exp["digest"]
        finally:
            db.free()


@pytest.mark.parametrize("first", ["64", "0.01"])
def test_inproc_whole_list_first_claim(first, monkeypatch):
    """Regression for the claiming root (a first claim that covered every first-level class
    handed the root's children over whole, so the rank's next claim read another batch's
    children: gpurun_out/inproc2.log of round 5): FSM_CLAIM_FIRST=64 makes one rank's first
    claim take every class and the others claim nothing; 0.01 makes many small claims.  Both
    give the full-size digest, twice per context."""
    import spark_fsm_amd as fsm
    monkeypatch.setenv("FSM_SPADE_CLAIMS", "1")
    monkeypatch.setenv("FSM_CLAIM_FIRST", first)
    for name in ("c2", "c5-bible"):
        exp = FULL[name]
        ds = dataset(*SPADE_CFG[name])
        with fsm.Engine(devices=[0, 0]) as e:
            db = e.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_SPADE)
            try:
                for _ in range(2):
                    csr, meta = e.spade_csr(db, exp["support"])
                    assert pattern_digest(*csr) == exp["digest"] and e.stats()["joins"] == exp["joins"]
            finally:
                db.free()
