"""bench.py — SPADE id-list joins/sec + mine time on Quest D1M, minsup 0.1 %.

BASELINE.json metric: "id-list joins/sec + end-to-end SPADE mine time, Quest
D1M minsup 0.1%".  One step = one complete fsm_spade_mine (F1, root F2, the
whole lattice, pattern CSR back on the host) over the flattened DB, which is
resident in HBM before the timed region (flatten + upload are timed
separately and reported in `extra`).  value = SURVEY A.2 candidate joins
(including infrequent ones) / mine time.  Because most A.2 candidates at D1M
are the F x F root pairs, `extra` also reports the work actually executed:
the non-empty root pair joins the F2 counted, the A.2 joins of the classes
below the root, and the lattice-only rate.

CPU baseline: the CPU restatement (oracle/fsm_oracle.c) on the
same DB and minsup, median of 3 bounded samples, in the same scope as `value`
(DB build excluded on both sides: the GPU's flatten + upload, the CPU's F1
vertical build), 1 thread (the reference's one driver thread) and all cores
of this process's CPU share.

The config-4 TSR leg (`tsr_c4`: expansions/s, its own roofline and CPU
baseline) runs after the SPADE steps at N = 1 (--no-tsr skips it).

  python bench.py [--gpus N --steps K --warmup W]   (N > 1 via torch.distributed.run)

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import platform
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "spark-fsm_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec (6.29 TB/s measured copy)
PMC_FILE = "profiles/pmc_latest.json"  # tools/pmc_summary.py output of the committed rocprofv3 --pmc passes
ROOT_F2_KERNELS = ("k_f2_plan", "k_f2_keys", "k_f2_count", "k_f2_vert")


def pmc_traffic(kernel):
    """HBM bytes per step of `kernel` from the committed PMC summary:
    2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md: on gfx950 FETCH_SIZE counts
    half the bytes of wide reads), summed over the kernel's launches in one step."""
    try:
        with open(os.path.join(ROOT, PMC_FILE)) as f:
            d = json.load(f)
        k = d["kernels"][kernel]
        return 2 * k["FETCH_SIZE_bytes_per_step"] + k["WRITE_SIZE_bytes_per_step"]
    except (OSError, KeyError, ValueError):
        return None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def cgroup_cpu_quota():
    """CPUs granted by a cgroup CPU quota (v2 cpu.max, v1 cfs quota/period), or None."""
    import math
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                return max(1, math.ceil(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        if q > 0 and per > 0:
            return max(1, math.ceil(q / per))
    except (OSError, ValueError):
        pass
    return None


def cpu_share():
    """CPUs this process may run on (the GPU box gives each GPU a share of the host):
    the affinity mask, capped by a cgroup CPU quota when one is set."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    q = cgroup_cpu_quota()
    return min(n, q) if q else n


def cpu_baseline(ds, support, seconds, threads, reps, stride):
    """The CPU restatement on a class-stride sample of the same mine: only the
    first-level classes of rank % stride == 0, each mined completely (its root
    joins and its whole subtree), so the sample covers every depth of the
    lattice in proportion (a time-bounded prefix would see only the first
    classes' long root joins).  joins/s over the lattice (F1 vertical build
    excluded, as the GPU's flatten + upload are), median of `reps` runs;
    `seconds` bounds each run (complete = the sample finished)."""
    from oracle import oracle
    runs = [oracle.spade_tokens(ds.seq_off, ds.tokens, support, time_limit_s=seconds, want_patterns=False,
                                threads=threads, stride=stride) for _ in range(reps)]
    lat = [r["joins"] / max(r["seconds"] - r["seconds_f1"], 1e-9) for r in runs]
    return {"value": statistics.median(lat), "unit": "joins/s", "cores": threads, "kind": "port",
            "samples": [round(v, 1) for v in lat], "class_stride": stride,
            "seconds_lattice": [round(r["seconds"] - r["seconds_f1"], 2) for r in runs],
            "seconds_f1": statistics.median(r["seconds_f1"] for r in runs),
            "complete": all(r["complete"] for r in runs), "joins_per_sample": [r["joins"] for r in runs]}


def c2_leg(fsm, gen, cpu_reps, steps=20):
    """BASELINE config 2 (Quest C10 T2.5 S4 I1.25 D100K, minsup 0.5 %): the GPU mine
    (median of `steps` after warmup) beside the COMPLETE single-thread CPU restatement of
    the same mine (every class; SURVEY §8d: wall time from the flattened DB to the
    results, the CPU's F1 vertical build included, median of `cpu_reps`)."""
    from oracle import oracle
    support = 0.005
    ds = gen.quest(100000, seed=1)
    with fsm.Engine(0) as eng:
        db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_SPADE)
        for _ in range(3):
            eng.spade_csr(db, support)
        t = []
        for _ in range(steps):
            t0 = time.perf_counter()
            _, meta = eng.spade_csr(db, support)
            t.append((time.perf_counter() - t0) * 1000.0)
        st = eng.stats()
        db.free()
    runs = [oracle.spade_tokens(ds.seq_off, ds.tokens, support, want_patterns=False, threads=1)
            for _ in range(max(1, cpu_reps))]
    if any(r["joins"] != st["joins"] for r in runs):
        raise SystemExit("c2 leg: CPU restatement and GPU disagree on the join count")
    cpu_s = statistics.median(r["seconds"] for r in runs)
    gpu_ms = statistics.median(t)
    return {"workload": "quest-C10-T2.5-S4-I1.25-D100000-N10000-seed1, minsup 0.005",
            "gpu_mine_ms": gpu_ms, "gpu_joins_per_s": st["joins"] / (gpu_ms / 1000.0),
            "patterns": meta["n"], "joins": st["joins"],
            "cpu_baseline": {"value": st["joins"] / cpu_s, "unit": "joins/s", "cores": 1, "kind": "port",
                             "seconds": [round(r["seconds"], 2) for r in runs], "median_s": cpu_s,
                             "complete": all(r["complete"] for r in runs),
                             "sample": "the complete mine (every class, F1 vertical build included) by the "
                                       "single-thread CPU restatement (oracle/fsm_oracle.c), median of %d"
                                       % max(1, cpu_reps)},
            "gpu_vs_cpu_1thread": (cpu_s * 1000.0) / gpu_ms}


def tsr_leg(fsm, gen, cpu_seconds, cpu_reps, cpu):
    """BASELINE config 4 (TSR, 990,002 Kosarak-shaped sequences, k = 1000,
    minconf 0.5): one mine after a warmup mine, expansions/s, the roofline of
    its dominant kernel (SURVEY §8(d) TSR unit: 8 B per position of every
    sequence where the expanded rule holds, whole rows, summed over the
    kernel's timed launches) and the CPU restatement
    on a bounded sample of the same DB (expansions/s)."""
    k, minconf = 1000, 0.5
    ds = gen.kosarak(D=990002, seed=1)
    with fsm.Engine(0) as eng:
        db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_TSR)
        # warmup (allocations, code objects) with every launch's kernels timed by HIP events: the
        # roofline's kernel time (the timed mine samples every 16th launch, events cost host time)
        os.environ["FSM_TSR_TIME_EVERY"] = "1"
        try:
            eng.tsr(db, k, minconf)
        finally:
            del os.environ["FSM_TSR_TIME_EVERY"]
        ks = eng.kernel_stats()
        t0 = time.perf_counter()
        rules, meta = eng.tsr(db, k, minconf)
        ms = (time.perf_counter() - t0) * 1000.0
        st = eng.stats()
        db.free()
    dom = max(ks, key=lambda q: q["ms"])
    ach = (dom["survey_bytes"] / 1e9) / (dom["ms"] / 1000.0) if dom["ms"] else 0.0
    ach_own = (dom["alg_bytes"] / 1e9) / (dom["ms"] / 1000.0) if dom["ms"] else 0.0
    leg = {"metric": "TSR expansions/s, Kosarak-shaped 990,002 sequences, k = 1000, minconf 0.5",
           "value": st["expansions"] / (ms / 1000.0), "unit": "expansions/s", "mine_ms": ms,
           "rules": len(rules), "final_minsup": meta["final_minsup"], "expansions": st["expansions"],
           "ms_pair_phase": st["ms_f2"], "ms_expansions": st["ms_lattice"], "launches": st["count_launches"],
           "ms_gpu_wait": st["ms_count_kernel"],
           # summed device time of the expansion kernels (every launch of the WARMUP mine timed with
           # HIP events) over the TIMED mine's wall time.  Two runs, and the two launch sets' streams
           # overlap, so this is not a busy fraction: it can exceed 1
           "gpu_kernel_ms": sum(q["ms"] for q in ks),
           "kernel_ms_over_wall": sum(q["ms"] for q in ks) / ms if ms else 0.0,
           "roofline": {"bound": "hbm", "kernel": dom["name"], "achieved": ach, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "kernel_ms": dom["ms"],
                        "alg_bytes": dom["survey_bytes"], "launches": dom["launches"],
                        "bytes_basis": "SURVEY §8(d) TSR unit for the row kernel: 4 B token + 4 B first/last "
                                       "per position of every sequence where the expanded rule holds, whole rows (the "
                                       "reference scans each such sequence); the sid-bitmap operands (N/8 B each) are "
                                       "k_exp_domain's; kernel time: HIP events around every launch of the "
                                       "warmup mine (the same expansions)",
                        "own_bytes": dom["alg_bytes"], "own_frac": ach_own / HBM_PEAK_GBS,
                        "own_bytes_basis": "tsr_engine.hip k_exp_rows: 8 B per row entry walked (the suffix past "
                                           "min(max X, max Y) of the rows where the rule holds) + per domain sid 12 B "
                                           "and 28 B per item of X u Y probed (rank directory, bitmap words, vertical "
                                           "entry), or 44 B per parent kept row (one probe) + 16 B per kept row "
                                           "written + the partial histogram rows written"},
           "kernels": [{"name": q["name"], "launches": q["launches"], "ms": round(q["ms"], 1)} for q in ks]}
    if cpu:
        # the restatement needs hours at 990K sequences, so both sides run the same
        # 5,000-sequence prefix completely (like for like, complete: true)
        from oracle import oracle
        pre = ds.head(5000)
        with fsm.Engine(0) as eng:
            db = eng.db_from_tokens(pre.sids, pre.seq_off, pre.tokens, fsm.MODE_TSR)
            eng.tsr(db, k, minconf)
            t0 = time.perf_counter()
            eng.tsr(db, k, minconf)
            gms = (time.perf_counter() - t0) * 1000.0
            gexp = eng.stats()["expansions"]
            db.free()
        recs = pre.records()
        runs = [oracle.tsr(recs, k, minconf, time_limit_s=cpu_seconds) for _ in range(cpu_reps)]
        rates = [r["expansions"] / max(r["seconds"], 1e-9) for r in runs]
        leg["cpu_baseline"] = {
            "value": statistics.median(rates), "unit": "expansions/s", "cores": 1, "kind": "port",
            "sample": "the 5,000-sequence prefix of the same DB, same k and minconf, mined completely by the "
                      "single-thread CPU restatement (oracle/fsm_oracle.c), median of %d; expansions/s" % cpu_reps,
            "complete": all(r["complete"] for r in runs), "samples": [round(v, 1) for v in rates],
            "seconds": [round(r["seconds"], 2) for r in runs],
            "gpu_same_prefix": {"value": gexp / (gms / 1000.0), "unit": "expansions/s", "mine_ms": gms,
                                "expansions": gexp}}
    return leg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--sequences", type=int, default=1000000)
    ap.add_argument("--support", type=float, default=0.001)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=60.0, help="bound of one CPU sample")
    ap.add_argument("--cpu-reps", type=int, default=3, help="CPU samples per leg (median; SURVEY §8d: 3)")
    ap.add_argument("--cpu-stride", type=int, default=128, help="class stride of the 1-thread CPU sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # all-cores CPU mode (SURVEY §8d ii); 0 = every CPU of this process's share (0 skips: -1)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--dist-backend", default="nccl", help="torch.distributed backend for N > 1 (gloo: CPU dry run)")
    ap.add_argument("--no-tsr", action="store_true", help="skip the config-4 TSR leg (N = 1 only)")
    ap.add_argument("--no-c2", action="store_true", help="skip the config-2 complete-CPU leg (N = 1 only)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist
    import spark_fsm_amd as fsm
    from tools import gen

    if world > 1:
        if args.dist_backend == "nccl":
            torch.cuda.set_device(local_rank)
        dist.init_process_group(args.dist_backend)

    def barrier():
        if world > 1:
            dist.barrier()

    def sync_device():
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    ds = gen.quest(args.sequences, seed=args.seed)
    eng, comm_kind = None, "none"
    if world > 1 and args.dist_backend == "nccl" and os.environ.get("FSM_BENCH_COMM", "rccl") == "rccl":
        # libfsm's own RCCL communicator (its collectives stay on the device): rank 0
        # makes the unique id, torch broadcasts it; if any rank cannot create it, every
        # rank falls back to the host-staged torch collectives below.  The communicator
        # init is non-blocking and bounded (FSM_COMM_INIT_TIMEOUT_S, comm.cpp), so a peer
        # that fails before its own init makes the others fail over, not hang.
        uid = torch.zeros(129, dtype=torch.uint8, device="cuda")
        if rank == 0:
            try:
                uid[:128].copy_(torch.frombuffer(bytearray(fsm.comm_unique_id()), dtype=torch.uint8))
                uid[128] = 1
            except fsm.FsmError:
                uid[128] = 0
        dist.broadcast(uid, 0)
        h = uid.cpu().tolist()
        if h[128]:
            try:
                eng = fsm.Engine(device=local_rank, nranks=world, rank=rank, unique_id=bytes(h[:128]))
            except fsm.FsmError as e:
                print("rank %d: libfsm RCCL communicator failed (%s); host-staged collectives" % (rank, e),
                      file=sys.stderr)
                eng = None
        ok = torch.tensor([1 if eng is not None else 0], dtype=torch.int32, device="cuda")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 1:
            comm_kind = "libfsm RCCL communicator (device buffers)"
        elif eng is not None:
            eng.close()
            eng = None
    if eng is not None:
        pass
    elif world > 1:
        # libfsm's collectives over torch's process group: RCCL (staged through a
        # device tensor) for nccl, CPU tensors for gloo (several ranks may share a GPU)
        from spark_fsm_amd.dist import TorchHostComm
        dev = "cuda:%d" % local_rank if args.dist_backend == "nccl" else None
        hc = TorchHostComm(dist.group.WORLD, device=dev)
        eng = fsm.Engine(device=local_rank % max(torch.cuda.device_count(), 1), nranks=world, rank=rank,
                         host_comm=hc)
        comm_kind = "torch.distributed %s, host-staged" % args.dist_backend
    else:
        eng = fsm.Engine(device=local_rank)
    db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_SPADE)
    prep = eng.stats()

    for _ in range(args.warmup):
        eng.spade_csr(db, args.support)
    # per-kernel device times (HIP events around every launch) of the last warmup mine: the
    # timed steps run without those events (FSM_KCLOCK=0: two event records per launch cost
    # about 0.15 ms of a D1M mine), the same mine's kernels otherwise (--warmup 0: one
    # instrumented mine after the timed steps)
    ks = eng.kernel_stats() if args.warmup > 0 else None

    os.environ["FSM_KCLOCK"] = "0"
    barrier()
    sync_device()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        csr, meta = eng.spade_csr(db, args.support)
    sync_device()
    barrier()
    t1 = time.perf_counter()
    del os.environ["FSM_KCLOCK"]
    st = eng.stats()  # stats of the last timed step
    if ks is None:
        eng.spade_csr(db, args.support)
        ks = eng.kernel_stats()

    ms_local = (t1 - t0) * 1000.0 / max(args.steps, 1)
    ms = ms_local
    joins_all = st["joins"]
    per_rank = None
    if world > 1:
        t = torch.tensor([ms_local], dtype=torch.float64)
        if args.dist_backend == "nccl":
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
        # per-rank trace of the last step: which work each rank did (replicated vs its share)
        mine = {"rank": rank, "ms_per_step": round(ms_local, 4),
                "ms_f1": round(st["ms_f1"], 4), "ms_f2_root": round(st["ms_f2"], 4),
                "ms_lattice": round(st["ms_lattice"], 4), "classes": st["classes"], "entries": st["entries"],
                "kernels": {k["name"]: round(k["ms"], 4) for k in ks}}
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)

    if rank != 0:
        db.free()
        eng.close()
        if world > 1:
            dist.destroy_process_group()
        return

    value = joins_all / (ms / 1000.0)  # joins of all ranks (libfsm sums them) / slowest rank
    # roofline of the dominant kernel: its work priced in SURVEY §8(d) units (12-B (sid, mask)
    # id-list entries read + written) / its device time (HIP events on libfsm's stream, summed
    # over the launches of the last step); the same time over the kernel's own slab bytes
    # (24-B entries: cid, mem, lohi, pos + mask) is `roofline_slab`
    dom = max(ks, key=lambda k: k["ms"])
    # (the dominant kernel is k_emit or the root F2's k_f2_tri, named k_f2_keys in the table: their
    # times are within a few percent since round 6, so the line also carries k_emit's own object)
    dom_basis = ("SURVEY §8(d) F2 unit: 8 B per root (item, sid) entry read per F2 pass"
                 if dom["name"] in ROOT_F2_KERNELS else
                 "SURVEY §8(d): one 12-B (sid u32, eid mask u64) id-list entry per parent entry "
                 "read and per child entry written (4 + 8W B for W mask words)")
    emit = next((k for k in ks if k["name"] == "k_emit"), None)
    achieved = (dom["survey_bytes"] / 1e9) / (dom["ms"] / 1000.0) if dom["ms"] > 0 else 0.0
    achieved_slab = (dom["alg_bytes"] / 1e9) / (dom["ms"] / 1000.0) if dom["ms"] > 0 else 0.0
    traffic = pmc_traffic(dom["name"])  # per step
    traffic_launch = traffic / dom["launches"] if traffic is not None and dom["launches"] else None
    # SURVEY §8(d) unit for the F2: 8 B per (item, sid) first/last pair read per pass,
    # over the device time of the root F2 kernels
    f2_ms = sum(k["ms"] for k in ks if k["name"] in ROOT_F2_KERNELS)
    f2_bytes = 8 * st["root_entries"]
    joins_lattice = st["joins"] - st["joins_root"]
    line = {
        "metric": "id-list joins/sec + end-to-end SPADE mine time, Quest D1M minsup 0.1%",
        "value": value,
        "unit": "joins/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "strong",  # fixed D1M problem: prefix classes sharded over the ranks
        "vs_baseline": None,
        "dtype": "u32/u64 (integer id-list joins)",
        "data": "synthetic (seeded Quest-shaped generator, tools/fsmgen.c)",
        "config": {"workload": "quest-C10-T2.5-S4-I1.25-D%d-N10000-seed%d, minsup %g" % (
            args.sequences, args.seed, args.support), "parallelism": "single GPU" if world == 1 else
            "prefix classes sharded over %d ranks (%s)" % (world, comm_kind)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic_launch,
                     "kernel": dom["name"], "launches_per_step": dom["launches"],
                     "kernel_ms_per_step": dom["ms"], "alg_bytes_per_step": dom["survey_bytes"],
                     "alg_bytes_per_launch": dom["survey_bytes"] / max(dom["launches"], 1),
                     "traffic_per_step": traffic,
                     "traffic_basis": "HBM bytes per launch (average over the step's launches) = "
                                      "(2 x FETCH_SIZE + WRITE_SIZE) / launches from the committed PMC passes",
                     "bytes_basis": dom_basis,
                     "traffic_source": PMC_FILE if traffic is not None else None},
        "roofline_k_emit": None if emit is None or emit["ms"] <= 0 else {
            "bound": "hbm", "kernel": "k_emit", "unit": "GB/s", "peak": HBM_PEAK_GBS,
            "kernel_ms_per_step": emit["ms"], "launches_per_step": emit["launches"],
            "alg_bytes_per_step": emit["survey_bytes"],
            "achieved": (emit["survey_bytes"] / 1e9) / (emit["ms"] / 1000.0),
            "frac": ((emit["survey_bytes"] / 1e9) / (emit["ms"] / 1000.0)) / HBM_PEAK_GBS,
            "traffic_per_step": pmc_traffic("k_emit"),
            "bytes_basis": "SURVEY §8(d): one 12-B (sid u32, eid mask u64) id-list entry per parent entry "
                           "read and per child entry written (4 + 8W B for W mask words)"},
        "roofline_slab": {"bound": "hbm", "achieved": achieved_slab, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": achieved_slab / HBM_PEAK_GBS, "kernel": dom["name"],
                          "alg_bytes_per_step": dom["alg_bytes"],
                          "bytes_basis": "the kernel's own slab layout: 16 + 8W B per entry (cid, mem, lohi, pos, "
                                         "mask) read and written (DESIGN.md §4)"},
        "roofline_survey_f2": {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                               "bytes_basis": "SURVEY §8(d): 8 B per root (item, sid) entry per F2 pass",
                               "alg_bytes": f2_bytes, "kernels_ms": f2_ms,
                               "achieved": (f2_bytes / 1e9) / (f2_ms / 1000.0) if f2_ms else 0.0,
                               "frac": ((f2_bytes / 1e9) / (f2_ms / 1000.0)) / HBM_PEAK_GBS if f2_ms else 0.0},
        "extra": {"mine_ms": ms, "joins": joins_all, "patterns": meta["n"], "minsup": meta["minsup"],
                  "joins_root": st["joins_root"], "joins_lattice": joins_lattice,
                  "root_pair_joins_executed": st["root_keys"], "lattice_pair_tests": st["pair_tests"],
                  "executed_joins": st["root_keys"] + joins_lattice,
                  "lattice_joins_per_s": joins_lattice / (st["ms_lattice"] / 1000.0) if st["ms_lattice"] else 0.0,
                  "classes": st["classes"], "batches": st["batches"], "entries": st["entries"],
                  "root_entries": st["root_entries"],
                  "ms_f1": st["ms_f1"], "ms_f2_root": st["ms_f2"], "ms_lattice": st["ms_lattice"],
                  "ms_gpu_wait": st["ms_gpu_wait"], "ms_output": st["ms_output"],
                  "ms_flatten": prep["ms_flatten"], "ms_upload": prep["ms_upload"],
                  "e2e_joins_per_s": joins_all / ((ms + prep["ms_flatten"] + prep["ms_upload"]) / 1000.0),
                  "join_equiv_GBps": (st["bytes_join_equiv"] / 1e9) / (ms / 1000.0),
                  "kernels": sorted(({"name": k["name"], "launches": k["launches"], "ms": round(k["ms"], 4),
                                      "GBps": round((k["alg_bytes"] / 1e9) / (k["ms"] / 1000.0), 1) if k["ms"] else 0}
                                     for k in ks), key=lambda k: -k["ms"])},
    }
    if per_rank is not None:
        line["extra"]["per_rank"] = per_rank
    if not args.no_cpu_baseline and world == 1:
        host = "%s; nproc %d, this process's CPU share %d" % (cpu_model(), os.cpu_count() or 0, cpu_share())
        cb = cpu_baseline(ds, args.support, args.cpu_seconds, 1, args.cpu_reps, args.cpu_stride)
        cb["sample"] = ("same DB and minsup; the single-thread CPU restatement (oracle/fsm_oracle.c) mining every "
                        "%d-th first-level class completely (class-stride sample of the whole lattice), median of %d; "
                        "joins/s over its lattice (F1 vertical build excluded, as the GPU's flatten + upload are); "
                        "host %s" % (args.cpu_stride, args.cpu_reps, host))
        line["cpu_baseline"] = cb
        nt = cpu_share() if args.cpu_threads == 0 else args.cpu_threads
        if nt > 1:
            st = max(1, args.cpu_stride // nt)
            ca = cpu_baseline(ds, args.support, args.cpu_seconds, nt, args.cpu_reps, st)
            ca["sample"] = ("same DB, minsup and scope; every %d-th first-level class on %d OpenMP threads "
                            "(all CPUs of this process's share; F1 build single-threaded)" % (st, nt))
            line["extra"]["cpu_baseline_all_cores"] = ca
    db.free()
    eng.close()
    if not args.no_tsr and world == 1:
        line["tsr_c4"] = tsr_leg(fsm, gen, args.cpu_seconds, args.cpu_reps, not args.no_cpu_baseline)
    if not args.no_c2 and not args.no_cpu_baseline and world == 1:
        line["c2_complete"] = c2_leg(fsm, gen, args.cpu_reps)
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
