"""Instance sharding and the cross-rank summary.

Paxos instances are independent, so the instance space is split into
contiguous, bucket-aligned shards, one per GPU; per-acceptor scalars depend
only on replicated headers.  The one exchange is an all-gather of each rank's
64-word summary (layout = SW_* in multi-paxos_amd/csrc/mpx_internal.hpp).
Phase-2 decisions (f2) add one more: an all-reduce MAX of the per-quorum fill
bounds, then a gather of the per-shard parts (gather_decisions).
"""
MASK64 = (1 << 64) - 1
SW_C, SW_P, SW_A, SW_L, SW_MSGS, SW_V, SW_DCHOSEN, SW_DSTATE, SW_DSCAL, SW_Q = range(10)
SUMMARY_WORDS = 64
BUCKET = 256


def shard_bounds(num_instances, world, rank, align=BUCKET):
    """[begin, end) of `rank`'s contiguous shard (strong scaling: the whole M at every world size)."""
    per = ((num_instances + world - 1) // world + align - 1) // align * align
    return min(num_instances, rank * per), min(num_instances, (rank + 1) * per)


def summary_from_oracle(stats, num_msgs=0):
    """64-word summary from the CPU oracle's [C,P,A,L,V,chosen_digest,state_digest,scalar_digest]."""
    s = [0] * SUMMARY_WORDS
    s[SW_C], s[SW_P], s[SW_A], s[SW_L], s[SW_V] = stats[0], stats[1], stats[2], stats[3], stats[4]
    s[SW_DCHOSEN], s[SW_DSTATE], s[SW_DSCAL] = stats[5], stats[6], stats[7]
    s[SW_MSGS] = num_msgs
    return s


def combine(summaries):
    """Whole-job totals from every rank's summary.  Counters add, digests add
    mod 2^64 (they are sums of per-entry hashes), per-acceptor scalars must be
    identical on every shard (replicated headers)."""
    if not summaries:
        raise ValueError("no summaries")
    scal = {s[SW_DSCAL] for s in summaries}
    if len(scal) != 1:
        raise AssertionError("per-acceptor scalars differ across shards: %r" % sorted(scal))
    out = {
        "chosen": sum(s[SW_C] for s in summaries),
        "promise_entries": sum(s[SW_P] for s in summaries),
        "accept_apps": sum(s[SW_A] for s in summaries),
        "commit_apps": sum(s[SW_L] for s in summaries),
        "violations": sum(s[SW_V] for s in summaries),
        "chosen_digest": sum(s[SW_DCHOSEN] for s in summaries) & MASK64,
        "state_digest": sum(s[SW_DSTATE] for s in summaries) & MASK64,
        "scalar_digest": summaries[0][SW_DSCAL],
    }
    out["bytes_alg"] = 16 * out["promise_entries"] + 24 * out["accept_apps"] + 16 * out["commit_apps"]
    return out


class EngineExchange:
    """The two collectives of the sharded decisions over the engine's own RCCL
    communicator (libmpx: mpx_comm_allreduce_max, mpx_comm_allgather_bytes)."""

    def __init__(self, engine, nranks):
        self.engine, self.nranks = engine, nranks

    def allreduce_max(self, vals):
        return self.engine.allreduce_max(vals)

    def allgather(self, data):
        return self.engine.allgather_bytes(data, self.nranks)


def gather_decisions(engine, exchange, rank=0):
    """Phase-2 decisions of a sharded run (include/mpx.h mpx_decisions_bounds /
    mpx_read_decisions_part / mpx_decisions_combine): every rank's per-quorum fill
    bounds are max-reduced (the noop fill of a quorum reaches the highest
    committed-or-adopted instance over all shards), each rank writes its part, and
    the parts are merged in rank (= shard) order.  `exchange` provides
    allreduce_max(list of u64) and allgather(bytes) -> [bytes per rank]:
    EngineExchange (RCCL inside libmpx; mpx_read_decisions_sharded is the same flow in
    one native call) or any other transport.  Returns the whole run's MPXD on rank 0,
    None elsewhere."""
    from . import decisions_combine
    mine = engine.decision_bounds()
    n = len(mine)
    # the quorum count must agree: MAX of (n, ~n) yields the max and the complemented min
    chk = exchange.allreduce_max([n, MASK64 ^ n])
    if chk[0] != n or (MASK64 ^ chk[1]) != n:
        raise RuntimeError("ranks disagree on the promise quorums: %d .. %d" % (MASK64 ^ chk[1], chk[0]))
    bounds = exchange.allreduce_max(mine) if mine else []
    parts = exchange.allgather(engine.decisions_part(bounds))
    return decisions_combine(parts) if rank == 0 else None


def gather_proposal_decisions(engine, exchange, rank=0):
    """Phase-2 decisions of a sharded run whose trace has client values (include/mpx.h
    mpx_proposal_part / mpx_proposal_combine): every rank's events of the proposer
    bookkeeping are gathered and walked once in rank (= shard) order.  Returns the whole
    run's MPXD on rank 0, None elsewhere."""
    from . import proposal_combine
    parts = exchange.allgather(bytes(engine.proposal_part()))
    return proposal_combine(parts) if rank == 0 else None
