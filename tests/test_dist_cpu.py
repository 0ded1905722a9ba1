"""The N>1 decomposition on CPU: world_size-2 gloo, one process per shard.

Each rank generates its shard's trace (headers replicated, entries of its
instances only — what every GPU rank holds), runs the CPU oracle on it, and the
64-word summaries are all-gathered over gloo and combined with the same code
bench.py uses.  The combination must equal the oracle over the whole trace:
counters add, digests add mod 2^64, per-acceptor scalars agree on every rank.
"""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import mpx
import mpxd
from mpx import dist as mdist
from oracles import oracle_run


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, n, m, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sb, se = mdist.shard_bounds(m, world, rank)
        t = mpx.generate_trace(mpx.GEN_CLEAN, num_nodes=n, num_instances=m, batch=256,
                               shard_begin=sb, shard_end=se)
        _, stats, _ = oracle_run(t)
        mine = mdist.summary_from_oracle(stats)
        allsum = [None] * world
        dist.all_gather_object(allsum, mine)
        if rank == 0:
            q.put(mdist.combine(allsum))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,m", [(2, 9, 256 * 40), (2, 5, 1000), (3, 3, 256 * 7 + 5)])
def test_sharded_oracle_combines_to_whole(world, n, m):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, n, m, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, whole, _ = oracle_run(mpx.generate_trace(mpx.GEN_CLEAN, num_nodes=n, num_instances=m, batch=256))
    assert [got["chosen"], got["promise_entries"], got["accept_apps"], got["commit_apps"], got["violations"],
            got["chosen_digest"], got["state_digest"], got["scalar_digest"]] == whole
    assert got["chosen"] == m


def test_shard_bounds_cover_and_align():
    for m in (1, 255, 256, 1000, 1 << 20, (1 << 27) + 3):
        for w in (1, 2, 3, 4, 8):
            b = [mdist.shard_bounds(m, w, r) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == m
            for (a0, a1), (c0, c1) in zip(b, b[1:]):
                assert a1 == c0
            for a0, a1 in b:
                assert a0 <= a1 and (a0 % 256 == 0 or a0 == a1 == m)   # trailing ranks may be empty


def test_combine_rejects_disagreeing_scalars():
    a = [0] * 64
    b = [0] * 64
    b[mdist.SW_DSCAL] = 1
    with pytest.raises(AssertionError):
        mdist.combine([a, b])


class _FixtureShard:
    """Stands in for one shard engine (no GPU here): its bounds and its part cut
    from the reference's decision fixture (test_decisions_combine._parts)."""

    def __init__(self, bounds, part, want_global):
        self.bounds, self.part, self.want_global = bounds, part, want_global

    def decision_bounds(self):
        return list(self.bounds)

    def decisions_part(self, gx):
        assert gx == self.want_global                 # the element-wise maximum over ranks
        return self.part


class _GlooExchange:
    """The exchange gather_decisions needs, over torch.distributed gloo (test transport;
    on GPUs the engine's RCCL communicator does it: mdist.EngineExchange)."""

    def __init__(self, world):
        self.world = world

    def allreduce_max(self, vals):
        got = [None] * self.world
        dist.all_gather_object(got, list(vals))
        return [max(col) for col in zip(*got)] if vals else []

    def allgather(self, data):
        got = [None] * self.world
        dist.all_gather_object(got, bytes(data))
        return got


def _dec_rank(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import test_decisions_combine as tdc
        want = open(os.path.join(tdc.GOLD, "fuzz_big_1.mpxd"), "rb").read()
        parts = tdc._parts(want, [60, 130][:world - 1])
        nq = sum(len(ds) for ds in mpxd.parse(want))
        bounds = [[(7 * k + r) % 200 for k in range(nq)] for r in range(world)]
        gx = [max(col) for col in zip(*bounds)]
        got = mdist.gather_decisions(_FixtureShard(bounds[rank], parts[rank], gx), _GlooExchange(world), rank)
        q.put((rank, got == want if rank == 0 else got is None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_decisions_over_gloo(world):
    """mdist.gather_decisions: MAX-reduced bounds reach every rank, the parts come
    back in rank order and rank 0's merge equals the reference's decisions."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dec_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [(r, True) for r in range(world)]


def test_bench_filegroup_rendezvous():
    """bench.py's N>1 rendezvous (no PyTorch): broadcast, barrier and max-reduce over 3 processes."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = str(40000 + os.getpid() % 10000)
    import _filegroup_child                         # a module without torch: the spawned children start fast
    procs = [ctx.Process(target=_filegroup_child.rank_main, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert [r[1] for r in res] == [b"uid-from-rank-0"] * 3
    assert [r[2] for r in res] == [3.0] * 3
