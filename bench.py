"""bench.py — SPADE id-list joins/sec + mine time on Quest D1M, minsup 0.1 %.

BASELINE.json metric: "id-list joins/sec + end-to-end SPADE mine time, Quest
D1M minsup 0.1%".  One step = one complete fsm_spade_mine (F1, root F2 pair
matrix, whole lattice, pattern CSR back on the host) over the flattened DB,
which is resident in HBM before the timed region (flatten + upload are timed
separately and reported in `extra`).  value = SURVEY A.2 candidate joins
(including infrequent ones) / mine time.

  python bench.py [--gpus N --steps K --warmup W]   (N > 1 via torch.distributed.run)

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "spark-fsm_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec (6.29 TB/s measured copy)
PMC_FILE = "profiles/pmc_latest.json"  # tools/pmc_summary.py output of the committed rocprofv3 --pmc passes


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--sequences", type=int, default=1000000)
    ap.add_argument("--support", type=float, default=0.001)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # all-cores CPU mode (SURVEY §8d ii); 16 = the box's CPU share per GPU (0 = skip)
    ap.add_argument("--cpu-threads", type=int, default=16)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist
    import spark_fsm_amd as fsm
    from tools import gen

    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")

    def barrier():
        if world > 1:
            dist.barrier()

    ds = gen.quest(args.sequences, seed=args.seed)
    if world > 1:
        # sharded SPADE over RCCL: rank 0 makes the unique id, torch broadcasts it
        uid = torch.zeros(128, dtype=torch.uint8, device="cuda")
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(fsm.comm_unique_id()), dtype=torch.uint8))
        dist.broadcast(uid, 0)
        eng = fsm.Engine(device=local_rank, nranks=world, rank=rank, unique_id=bytes(uid.cpu().tolist()))
    else:
        eng = fsm.Engine(device=local_rank)
    db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_SPADE)
    prep = eng.stats()

    for _ in range(args.warmup):
        eng.spade_csr(db, args.support)

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        csr, meta = eng.spade_csr(db, args.support)
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    st = eng.stats()  # stats of the last timed step

    ms_local = (t1 - t0) * 1000.0 / max(args.steps, 1)
    ms = ms_local
    joins_all = st["joins"]
    if world > 1:
        t = torch.tensor([ms_local], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())

    if rank != 0:
        db.free()
        eng.close()
        if world > 1:
            dist.destroy_process_group()
        return

    value = joins_all / (ms / 1000.0)  # joins of all ranks (libfsm sums them) / slowest rank
    # roofline of the dominant kernel: algorithmic bytes / its device time (HIP
    # events on libfsm's stream, summed over the launches of the last step)
    ks = eng.kernel_stats()
    dom = max(ks, key=lambda k: k["ms"])
    achieved = (dom["alg_bytes"] / 1e9) / (dom["ms"] / 1000.0) if dom["ms"] > 0 else 0.0
    traffic = pmc_traffic(dom["name"])
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
            "prefix classes sharded over %d GPUs" % world},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": dom["name"], "launches_per_step": dom["launches"],
                     "kernel_ms_per_step": dom["ms"], "alg_bytes_per_step": dom["alg_bytes"],
                     "traffic_source": PMC_FILE if traffic is not None else None},
        "extra": {"mine_ms": ms, "joins": joins_all, "patterns": meta["n"], "minsup": meta["minsup"],
                  "classes": st["classes"], "batches": st["batches"], "entries": st["entries"],
                  "ms_f1": st["ms_f1"], "ms_f2_root": st["ms_f2"], "ms_lattice": st["ms_lattice"],
                  "ms_flatten": prep["ms_flatten"], "ms_upload": prep["ms_upload"],
                  "join_equiv_GBps": (st["bytes_join_equiv"] / 1e9) / (ms / 1000.0),
                  "kernels": sorted(({"name": k["name"], "launches": k["launches"], "ms": round(k["ms"], 4),
                                      "GBps": round((k["alg_bytes"] / 1e9) / (k["ms"] / 1000.0), 1) if k["ms"] else 0}
                                     for k in ks), key=lambda k: -k["ms"])},
    }
    if not args.no_cpu_baseline and world == 1:
        from oracle import oracle
        r = oracle.spade_tokens(ds.seq_off, ds.tokens, args.support, time_limit_s=args.cpu_seconds,
                                want_patterns=False)
        line["cpu_baseline"] = {
            "value": r["joins"] / r["seconds"], "unit": "joins/s", "cores": 1, "kind": "port",
            "lattice_value": r["joins"] / max(r["seconds"] - r["seconds_f1"], 1e-9), "seconds_f1": r["seconds_f1"],
            "sample": "same DB and minsup; first %.0f s of the single-thread vertical SPADE DFS "
                      "(oracle/fsm_oracle.c, F1 build included): %d joins%s; host %s" % (
                          args.cpu_seconds, r["joins"], "" if not r["complete"] else " (complete)",
                          cpu_model())}
        if args.cpu_threads > 1:
            r2 = oracle.spade_tokens(ds.seq_off, ds.tokens, args.support, time_limit_s=args.cpu_seconds,
                                     want_patterns=False, threads=args.cpu_threads)
            line["extra"]["cpu_baseline_all_cores"] = {
                "value": r2["joins"] / r2["seconds"], "unit": "joins/s", "cores": args.cpu_threads,
                "kind": "port", "complete": r2["complete"], "seconds": r2["seconds"], "joins": r2["joins"],
                "lattice_value": r2["joins"] / max(r2["seconds"] - r2["seconds_f1"], 1e-9),
                "seconds_f1": r2["seconds_f1"],
                "sample": "same DB and minsup, same time bound; first-level classes on %d OpenMP threads "
                          "(F1 build single-threaded)" % args.cpu_threads}
    print(json.dumps(line), flush=True)
    db.free()
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
