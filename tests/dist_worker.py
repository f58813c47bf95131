"""One rank of a multi-process libfsm run (launched by tests/test_dist.py and
tests/test_parity_gpu.py as a plain child process).

  python tests/dist_worker.py <mode> <out.json> [args...]
  mode selftest       : fsm_comm_selftest over a gloo TorchHostComm (no GPU)
  mode spade D sup    : sharded SPADE on cuda:0 over a gloo TorchHostComm
  mode spade_fail D sup : the same with a failure injected on one rank (FSM_INJECT_FAIL)
  mode spade_digest shape D sup : sharded SPADE, digest of the result (full-size configs)
  mode tsr D k minconf : TSR with the pair phase sharded by sequence range
  mode tsr_fail D k minconf : the same with a failure injected on one rank (FSM_INJECT_FAIL)
Env: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT (torch.distributed, gloo).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "spark-fsm_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def main():
    mode, out = sys.argv[1], sys.argv[2]
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import spark_fsm_amd as fsm
    from spark_fsm_amd import dist as fdist
    # FSM_TEST_CLAIMS=0: no work-stealing counter (the static class plan); "rank0": only rank 0
    # offers one (the ranks must agree on the static plan)
    # "shm": no callback, but a unique id: the node's shared-memory counters (the RCCL
    # communicator's) under the host collectives
    cl = os.environ.get("FSM_TEST_CLAIMS", "1")
    hc = fdist.TorchHostComm(claims=cl == "1" or (cl == "rank0" and rank == 0))
    res = {"rank": rank, "world": world, "claims": hc._store is not None}
    uid = None
    if cl == "shm":
        obj = [os.urandom(128) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        uid = obj[0]
    if mode == "selftest":
        fdist.selftest(world, rank, host_comm=hc, unique_id=uid)
        res["ok"] = True
    elif mode == "spade":
        from tools import gen
        D, sup = int(sys.argv[3]), float(sys.argv[4])
        ds = gen.quest(D, seed=int(sys.argv[5]) if len(sys.argv) > 5 else 1)
        with fsm.Engine(0, nranks=world, rank=rank, host_comm=hc) as eng:
            db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_SPADE)
            pats, meta = eng.spade(db, sup)
            st = eng.stats()
            db.free()
        res.update(patterns=sorted(pats), minsup=meta["minsup"], joins=st["joins"], classes=st["classes"])
    elif mode == "spade_digest":
        # sharded SPADE at a BASELINE config: the digest of the gathered pattern set
        from digest import pattern_digest
        from tools import gen
        shape, D, sup = sys.argv[3], int(sys.argv[4]), float(sys.argv[5])
        ds = gen.quest(D, seed=1) if shape == "quest" else getattr(gen, shape)(seed=1)
        with fsm.Engine(0, nranks=world, rank=rank, host_comm=hc,
                        verbose=os.environ.get("FSM_WORKER_VERBOSE") == "1") as eng:
            db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_SPADE)
            csr, meta = eng.spade_csr(db, sup)
            st = eng.stats()
            db.free()
        res.update(digest=pattern_digest(*csr), minsup=meta["minsup"], joins=st["joins"],
                   rank_root_slab=st["rank_root_slab"], rank_root_owned=st["rank_root_owned"],
                   rank_claims=st["rank_claims"], root_entries=st["root_entries"])
    elif mode == "tsr_digest":
        # sharded TSR at the c4 prefix: digest of the rule set, slots expanded here
        from digest import rule_digest
        from tools import gen
        D, k, mc = int(sys.argv[3]), int(sys.argv[4]), float(sys.argv[5])
        ds = gen.kosarak(D=990002, seed=1).head(D)
        with fsm.Engine(0, nranks=world, rank=rank, host_comm=hc) as eng:
            db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_TSR)
            rules, meta = eng.tsr(db, k, mc)
            st = eng.stats()
            db.free()
        res.update(digest=rule_digest(rules), final_minsup=meta["final_minsup"], units=st["rank_units"],
                   units_total=st["expansions"])
    elif mode == "tsr":
        # TSR on a Kosarak-shaped DB: pair phase sharded by sequence range (candidate keys
        # exchanged, partial counts summed), expansions on every rank alike
        from tools import gen
        D, k, mc = int(sys.argv[3]), int(sys.argv[4]), float(sys.argv[5])
        ds = gen.kosarak(D=D, seed=3)
        with fsm.Engine(0, nranks=world, rank=rank, host_comm=hc,
                        verbose=os.environ.get("FSM_WORKER_VERBOSE") == "1") as eng:
            db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_TSR)
            rules, meta = eng.tsr(db, k, mc)
            db.free()
        res.update(rules=sorted([list(x), list(y), s, c] for x, y, s, c in rules),
                   final_minsup=meta["final_minsup"])
    elif mode == "tsr_fail":
        # sharded TSR pair phase with FSM_INJECT_FAIL set for one rank: every rank fails, none hangs
        from tools import gen
        D, k, mc = int(sys.argv[3]), int(sys.argv[4]), float(sys.argv[5])
        ds = gen.kosarak(D=D, seed=3)
        with fsm.Engine(0, nranks=world, rank=rank, host_comm=hc) as eng:
            db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_TSR)
            try:
                eng.tsr(db, k, mc)
                res.update(code=0, msg="")
            except fsm.FsmError as e:
                res.update(code=e.code, msg=e.msg)
            db.free()
    elif mode == "spade_fail":
        # sharded SPADE with FSM_INJECT_FAIL set for one rank: every rank must fail, none may hang
        from tools import gen
        D, sup = int(sys.argv[3]), float(sys.argv[4])
        ds = gen.quest(D, seed=1)
        with fsm.Engine(0, nranks=world, rank=rank, host_comm=hc) as eng:
            db = eng.db_from_tokens(ds.sids, ds.seq_off, ds.tokens, fsm.MODE_SPADE)
            try:
                eng.spade(db, sup)
                res.update(code=0, msg="")
            except fsm.FsmError as e:
                res.update(code=e.code, msg=e.msg)
            db.free()
    with open(out, "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
