"""The N>1 decomposition with libmpx engines on the GPU: world_size-2 gloo,
one process per instance shard, each holding a libmpx engine on device 0 (the one-GPU box: two
processes share the card; an 8-GPU node gives each rank its own).  Each rank submits the whole
host trace (the engine keeps every header and its shard's entries), runs it, and the
64-word summaries are all-gathered over gloo and combined with the code bench.py uses (mpx.dist);
the phase-2 decisions go through mdist.gather_decisions (bounds MAX-reduced, parts gathered in rank
order).  Both must equal one engine over the whole trace and the C oracle.  (RCCL itself needs one
GPU per rank: on one card the exchange runs over gloo.)"""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _GlooExchange:
    def __init__(self, world):
        self.world = world

    def allreduce_max(self, vals):
        import torch.distributed as dist
        got = [None] * self.world
        dist.all_gather_object(got, list(vals))
        return [max(col) for col in zip(*got)] if vals else []

    def allgather(self, data):
        import torch.distributed as dist
        got = [None] * self.world
        dist.all_gather_object(got, bytes(data))
        return got


def _rank(rank, world, port, kind, params, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    import mpx
    from mpx import dist as mdist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = mpx.generate_trace(kind, **params)
        hd = mpx.trace_header(t)
        m = max(hd["num_instances"], 1)
        sb, se = mdist.shard_bounds(m, world, rank)
        with mpx.Engine(hd["num_nodes"], sb, se, semantics=hd["semantics"]) as e:
            e.submit_trace(t)
            e.run()
            mine = e.allgather_summary(1)[0]
            allsum = [None] * world
            dist.all_gather_object(allsum, list(mine))
            dec = mdist.gather_decisions(e, _GlooExchange(world), rank) if hd["semantics"] == 0 else None
        if rank == 0:
            q.put((mdist.combine(allsum), dec))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,params", [
    ("clean", dict(num_nodes=9, num_instances=256 * 40 + 17, batch=256)),
    ("faulty", dict(num_nodes=7, num_instances=1 << 14, seed=3, batch=256, proposers=3, drop_rate=500,
                    dup_rate=1000, max_delay=500)),
])
def test_two_shard_engines_combine_to_whole(kind, params):
    import torch.multiprocessing as mp
    import mpx
    from oracles import oracle_run
    k = mpx.GEN_CLEAN if kind == "clean" else mpx.GEN_FAULTY
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, k, params, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, dec = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    t = mpx.generate_trace(k, **params)
    _, whole, _ = oracle_run(t)
    assert [got[x] for x in ("chosen", "promise_entries", "accept_apps", "commit_apps", "violations",
                             "chosen_digest", "state_digest", "scalar_digest")] == whole
    with mpx.Engine.for_trace(t) as e:
        e.run()
        assert dec == e.decisions()
