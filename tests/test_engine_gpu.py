"""Parity of the HIP engine (through the C ABI) with the reference.

* every golden fixture: engine dump == the reference's result, byte for byte
  (the .mpxr files were written by the reference's own handlers);
* generated traces (C2 shape, scaled down and full size): engine == CPU
  oracle (oracle/mpx_oracle.c), dumps and counters/digests;
* the scalar / state / chosen readbacks agree with the dump.
All integer work: the bar is bit-exact.
"""
import json
import os

import pytest

import mpx
import mpxr
import mpxwire
from oracles import oracle_run

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
INDEX = json.load(open(os.path.join(GOLD, "index.json")))


def _read(name, ext):
    with open(os.path.join(GOLD, name + ext), "rb") as f:
        return f.read()


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if mpx.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")


COUNTERS = ("chosen", "promise_entries", "accept_apps", "commit_apps", "violations")


def _step_path(e, want, st_run):
    """The timed path (mpx_step: k_plan + k_store + k_apply_fast's remaining
    pairs, no digest code) gives the same result bytes and counters as the
    digested mpx_run (one-kernel k_apply_fast)."""
    e.step()
    e.sync()
    st = e.stats()
    # what the step's kernels left in HBM, digested by a separate pass
    assert e.state_digest() == (st_run["state_digest"], st_run["chosen_digest"])
    got = e.dump()
    assert got == want, mpxr.diff(got, want)
    assert [st[k] for k in COUNTERS] == [st_run[k] for k in COUNTERS]


def _executed_ok(e, want):
    """mpx_read_executed (device frontier + compaction) against the executed
    payloads of the expected MPXR (reference / oracle), node by node."""
    parsed = mpxr.parse(want)
    for n, nd in enumerate(parsed["nodes"]):
        committed = {iid: h for iid, kind, _b, h in nd["state"] if kind == 2}
        front = 0
        while front in committed:
            front += 1
        below = [committed[i] for i in range(front) if not (committed[i] >> 47) & 1]
        fr, handles = e.read_executed(n)
        assert fr == front, (n, fr, front)
        # membership Values are not executed: a subsequence of `below`, as many as the expected payloads
        it = iter(below)
        assert all(h in it for h in handles), n
        assert len(handles) == len(nd["executed"]), n


@pytest.mark.parametrize("name", sorted(INDEX))
def test_engine_matches_reference_golden(name):
    trace, want = _read(name, ".mpxt"), _read(name, ".mpxr")
    with mpx.Engine.for_trace(trace) as e:
        st = e.run()
        got = e.dump()
        assert got == want, mpxr.diff(got, want)
        _executed_ok(e, want)
        _step_path(e, want, st)
    meta = INDEX[name]
    assert (st["chosen"], st["promise_entries"], st["accept_apps"], st["commit_apps"]) == \
        (meta["C"], meta["P"], meta["A"], meta["L"])


# (9, 256 * 70 + 100): k_store's full 32-bucket chunks, its tail buckets and a partial last bucket
@pytest.mark.parametrize("name", ["fuzz_big_0", "fuzz_big_1", "hm_commit_tags", "hm_promise_merge", "c2_clean_n9_b100", "c5_member_0", "demo5_s3",
                                  "c3_faulty_0", "mm_aggregate"])
def test_two_byte_slots_match(name, monkeypatch):
    """Traces whose pairs all fit 1-byte slots run with 2-byte slots too when
    forced (MPX_SLOT_BYTES=2): the same result bytes on both apply paths."""
    if name not in INDEX:
        pytest.skip("no golden " + name)
    monkeypatch.setenv("MPX_SLOT_BYTES", "2")
    trace, want = _read(name, ".mpxt"), _read(name, ".mpxr")
    with mpx.Engine.for_trace(trace) as e:
        st = e.run()
        got = e.dump()
        assert got == want, mpxr.diff(got, want)
        _step_path(e, want, st)


def test_wide_pairs_take_two_byte_slots():
    """Batch 1: a pair holds up to 512 runs (> 254), so the engine switches to
    2-byte slots by itself; result bytes still equal the oracle's."""
    t = mpx.generate_trace(mpx.GEN_CLEAN, num_nodes=3, num_instances=700, batch=1)
    want, ostats, _ = oracle_run(t)
    with mpx.Engine.for_trace(t) as e:
        st = e.run()
        assert e.dump() == want
        _step_path(e, want, st)


@pytest.mark.parametrize("n,m,b", [(5, 4096, 256), (3, 1000, 100), (7, 5000, 37), (1, 10, 256), (64, 300, 256),
                                   (9, 256 * 70 + 100, 256)])
def test_engine_matches_oracle_clean(n, m, b):
    t = mpx.generate_trace(mpx.GEN_CLEAN, num_nodes=n, num_instances=m, batch=b)
    want, ostats, _ = oracle_run(t)
    with mpx.Engine.for_trace(t) as e:
        st = e.run()
        got = e.dump()
        assert got == want, mpxr.diff(got, want)
        assert [st["chosen"], st["promise_entries"], st["accept_apps"], st["commit_apps"], st["violations"],
                st["chosen_digest"], st["state_digest"], st["scalar_digest"]] == ostats
        # readbacks
        ch = e.read_chosen(0, m)
        assert all(c == mpx.PRESENT | (i + 1) for i, c in enumerate(ch))
        for node in (0, n - 1):
            ab, av, cb, cv = e.read_node_state(node, 0, m)
            assert not any(av) and not any(ab)
            assert all(x == 1 << 16 for x in cb)
            assert e.read_node_scalars(node) == (1 << 16, 1 << 16)
            fr, hs = e.read_executed(node)                  # every instance committed, none a noop
            assert fr == m and hs == [c & ~mpx.PRESENT for c in ch]
        _step_path(e, want, st)


def test_engine_c2_full_size_digests():
    """C2: 2^20 instances x 5 acceptors, clean, batch 256 — counters and
    order-independent digests equal the CPU oracle's."""
    n, m = 5, 1 << 20
    t = mpx.generate_trace(mpx.GEN_CLEAN, num_nodes=n, num_instances=m, batch=256)
    _, ostats, _ = oracle_run(t)
    with mpx.Engine.for_trace(t) as e:
        st = e.run()
        d_run = e.dump()
        _step_path(e, d_run, st)
    assert [st["chosen"], st["promise_entries"], st["accept_apps"], st["commit_apps"], st["violations"],
            st["chosen_digest"], st["state_digest"], st["scalar_digest"]] == ostats
    assert st["chosen"] == m and st["bytes_alg"] == 40 * n * m
    import xxhash                                            # and == the reference's own handlers (full_size.json)
    assert (len(t), "%016x" % xxhash.xxh3_64_intdigest(t)) == (FULL_SIZE["c2"]["trace_bytes"], FULL_SIZE["c2"]["trace_xxh3"])
    assert {k: st[k] for k in STATS_ORDER} == FULL_SIZE["c2"]["stats"]


def test_sends_match_dump():
    name = "fuzz_big_0"
    trace = _read(name, ".mpxt")
    with mpx.Engine.for_trace(trace) as e:
        e.run()
        sends = e.drain_sends()
        parsed = mpxr.parse(e.dump())
    flat = [(i, d, b) for i, nd in enumerate(parsed["nodes"]) for d, b in nd["sends"]]
    assert sends == flat


def test_repeated_runs_are_identical():
    t = mpx.generate_trace(mpx.GEN_CLEAN, num_nodes=5, num_instances=3000, batch=256)
    with mpx.Engine.for_trace(t) as e:
        a = e.run()
        d1 = e.dump()
        for _ in range(3):
            e.step()
        e.sync()
        b = e.run()
        assert e.dump() == d1
    for k in ("chosen", "state_digest", "chosen_digest", "accept_apps"):
        assert a[k] == b[k]


# batch != 256: a bucket meets 2-4 batches (partial runs, segmented plan
# words); batch 7: 38-run pairs; batch 3: 172-run pairs go to k_apply's work list
@pytest.mark.parametrize("n,m,b", [(5, 4096, 256), (9, 256 * 37, 256), (2, 256, 256), (5, 4096 + 77, 100),
                                   (9, 256 * 37 + 5, 255), (9, 256 * 40, 100), (3, 1000, 37), (4, 3000, 7),
                                   (2, 700, 3)])
def test_device_generator_matches_host(n, m, b):
    """The HBM-materialised clean trace (mpx_load_clean_device) gives the same
    result bytes as the host trace through mpx_submit, and the oracle's."""
    t = mpx.generate_trace(mpx.GEN_CLEAN, num_nodes=n, num_instances=m, batch=b)
    want, ostats, _ = oracle_run(t)
    with mpx.Engine(n, 0, m) as e:
        e.load_clean_device(num_instances=m, batch=b)
        st = e.run()
        got = e.dump()
        _step_path(e, want, st)
    assert got == want, mpxr.diff(got, want)
    assert [st["chosen"], st["promise_entries"], st["accept_apps"], st["commit_apps"], st["violations"],
            st["chosen_digest"], st["state_digest"], st["scalar_digest"]] == ostats


@pytest.mark.parametrize("n,m,b,sb", [(9, 1 << 23, 256, 0), (9, (1 << 23) + 256 * 7 + 13, 100, 0), (10, 1 << 22, 255, 0), (11, 1 << 21, 256, 0),
                                      (5, 1 << 23, 256, 256 * 1000), (9, 1 << 20, 256, 0), (2, 256 * 33, 256, 0)])
def test_plan_store_matches_plan_then_store(n, m, b, sb, monkeypatch):
    """k_plan_store8 (the C4 shape's one-launch plan + store: workgroups looping over
    32-bucket groups, a partial last group, shard offsets) leaves the same state and chosen
    log as k_plan + k_store8 (MPX_PLAN_STORE=0) and as the digested run, with the same
    counters."""
    res = []
    for ps in ("1", "0"):
        monkeypatch.setenv("MPX_PLAN_STORE", ps)
        with mpx.Engine(n, sb, m) as e:
            e.load_clean_device(num_instances=m, batch=b)
            st = e.run()
            e.step()
            e.sync()
            got = e.stats()
            assert e.state_digest() == (st["state_digest"], st["chosen_digest"])
            assert [got[k] for k in COUNTERS] == [st[k] for k in COUNTERS]
            assert got["chosen"] == m - sb
            res.append((e.state_digest(), e.read_chosen(m - 300, 300)))
    assert res[0] == res[1]


@pytest.mark.parametrize("shards,b", [(2, 256), (3, 256), (8, 256), (3, 100), (8, 255)])
def test_sharded_device_generator_sums_to_whole(shards, b):
    """Instance sharding: per-shard counters and digests add
    up to the single-engine run; per-acceptor scalars agree on every shard
    (batch 100 / 255: batches straddle the shard boundaries)."""
    n, m = 9, 256 * 64
    with mpx.Engine(n, 0, m) as e:
        e.load_clean_device(num_instances=m, batch=b)
        whole = e.run()
    per = m // shards // 256 * 256
    bounds = [(i * per, m if i == shards - 1 else (i + 1) * per) for i in range(shards)]
    tot = {k: 0 for k in ("chosen", "accept_apps", "commit_apps", "chosen_digest", "state_digest")}
    for sb, se in bounds:
        with mpx.Engine(n, sb, se) as e:
            e.load_clean_device(num_instances=m, batch=b)
            st = e.run()
            assert st["scalar_digest"] == whole["scalar_digest"]
            for k in tot:
                tot[k] = (tot[k] + st[k]) % (1 << 64)
            ch = e.read_chosen(sb, se - sb)
            assert ch == [mpx.PRESENT | (i + 1) for i in range(sb, se)]
            _step_path(e, e.dump(), st)
            assert e.read_chosen(sb, se - sb) == ch
    for k in tot:
        assert tot[k] == whole[k] % (1 << 64), k


@pytest.mark.parametrize("shards", [2, 4])
def test_c3_header_sharding(shards):
    """Header sharding of host-ingested traces: a shard engine leaves out the
    ACCEPT / COMMIT / P_BATCH records with no entry in its shard (and their
    replies), keeping only their ballots for the max_seen scan.  State, scalars,
    promise-quorum events (entries restricted) and chosen batches still equal the
    oracle's whole run, and each rank processes about total / shards + the
    replicated headers."""
    m = 1 << 12
    t = mpx.generate_trace(mpx.GEN_FAULTY, num_nodes=7, num_instances=m, seed=5, batch=64, proposers=3,
                           drop_rate=500, dup_rate=1000, max_delay=500)
    full = mpxr.parse(oracle_run(t)[0])
    with mpx.Engine.for_trace(t) as e:
        st = e.run()
    records = st["messages"] + st["skipped"]
    from mpx import dist as mdist
    kept = []
    for r in range(shards):
        sb, se = mdist.shard_bounds(m, shards, r)
        with mpx.Engine(7, sb, se) as e:
            e.submit_trace(t)
            st = e.run()
            part = mpxr.parse(e.dump())
        assert st["messages"] + st["skipped"] == records
        kept.append(st["messages"])
        for a, b in zip(part["nodes"], full["nodes"]):
            assert a["state"] == [x for x in b["state"] if sb <= x[0] < se]
            assert (a["promised"], a["max_seen"]) == (b["promised"], b["max_seen"])
            assert a["quorums"] == [(q, bal, [x for x in ents if sb <= x[0] < se]) for q, bal, ents in b["quorums"]]
            assert set(a["chosen_batches"]) <= set(b["chosen_batches"])
        assert part["chosen"] == [c for c in full["chosen"] if sb <= c[0] < se]
    print("records %d, kept per rank %s" % (records, kept))
    assert max(kept) < records * (0.75 if shards == 2 else 0.5)


def test_host_sharded_ingest_matches_oracle_restricted():
    """Host ingest with a shard: state / chosen entries equal the oracle's, restricted to the shard."""
    name = "fuzz_big_1"
    trace = _read(name, ".mpxt")
    full = mpxr.parse(_read(name, ".mpxr"))
    n = len(full["nodes"])
    sb, se = 64, 150
    with mpx.Engine(n, sb, se) as e:
        e.submit_trace(trace)
        e.run()
        part = mpxr.parse(e.dump())
    for a, b in zip(part["nodes"], full["nodes"]):
        assert a["state"] == [s for s in b["state"] if sb <= s[0] < se]
        assert (a["promised"], a["max_seen"]) == (b["promised"], b["max_seen"])
    assert part["chosen"] == [c for c in full["chosen"] if sb <= c[0] < se]


@pytest.mark.parametrize("seed,m,p,b", [(11, 1 << 12, 3, 64), (12, 3000, 2, 256), (13, 1 << 13, 3, 17)])
def test_engine_matches_oracle_c3_faulty(seed, m, p, b):
    """C3 shape: 7 acceptors, competing proposers, drop 5 % / dup 10 % (<=3) /
    delay U[0,500) (multi/debug.conf.sample:1) — multi-ballot promise phases,
    promise replies with entries, rejects, duplicates, reordering."""
    t = mpx.generate_trace(mpx.GEN_FAULTY, num_nodes=7, num_instances=m, seed=seed, batch=b, proposers=p,
                           drop_rate=500, dup_rate=1000, max_delay=500)
    want, ostats, _ = oracle_run(t)
    with mpx.Engine.for_trace(t) as e:
        st = e.run()
        got = e.dump()
        _step_path(e, want, st)
    assert got == want, mpxr.diff(got, want)
    assert [st["chosen"], st["promise_entries"], st["accept_apps"], st["commit_apps"], st["violations"],
            st["chosen_digest"], st["state_digest"], st["scalar_digest"]] == ostats
    assert st["promise_entries"] > 0 and st["violations"] == 0


def test_rccl_single_rank_allgather():
    """The RCCL path of a step (communicator + summary all-gather on the comm stream, overlapped
    with the next launch: two summary slots), one rank: after one step, several queued steps
    (each slot reused while the other's all-gather may still run) and a digested run, the
    gathered summary is the last launch's."""
    n, m = 9, 256 * 64
    from mpx import dist as mdist
    with mpx.Engine(n, 0, m) as e:
        e.comm_init(mpx.Engine.comm_unique_id(), 0, 1)
        e.load_clean_device(num_instances=m)
        for steps in (1, 5):
            for _ in range(steps):
                e.step()
            e.sync()
            st = e.stats()
            tot = mdist.combine(e.allgather_summary(1))
            assert tot["chosen"] == m == st["chosen"]
            assert tot["state_digest"] == st["state_digest"]
        chk = e.run()
        tot = mdist.combine(e.allgather_summary(1))
        assert tot["chosen"] == m == chk["chosen"] and tot["state_digest"] == chk["state_digest"]


# ---- member semantics (member/paxos.cpp) ----
@pytest.mark.parametrize("seed,u,m,b,drop,dup", [(21, 8, 1 << 12, 64, 500, 100), (22, 5, 3000, 17, 1000, 300),
                                                  (23, 8, 1 << 14, 256, 0, 100), (24, 3, 500, 1, 0, 0)])
def test_engine_matches_oracle_c5_member(seed, u, m, b, drop, dup):
    """C5 shape: AddAcceptor(1..U-1) then DelAcceptor(1..U-1) (member/main.cpp:119-141),
    version filter, insert semantics, per-epoch quorums, catch-up learns, stale in-flight ACCEPTs."""
    t = mpx.generate_trace(mpx.GEN_MEMBER, num_nodes=u, num_instances=m, seed=seed, batch=b,
                           drop_rate=drop, dup_rate=dup, max_delay=64, noop_permille=15)
    want, ostats, _ = oracle_run(t)
    with mpx.Engine.for_trace(t) as e:
        st = e.run()
        got = e.dump()
        assert got == want, mpxr.diff(got, want)
        _step_path(e, want, st)                 # k_plan_member + store + the pairs it listed
    assert [st["chosen"], st["promise_entries"], st["accept_apps"], st["commit_apps"], st["violations"],
            st["chosen_digest"], st["state_digest"], st["scalar_digest"]] == ostats
    assert st["chosen"] == m and st["violations"] == 0


@pytest.mark.parametrize("seed,u,m,b,drop,dup,props", [(61, 8, 1 << 14, 64, 100, 100, 3), (62, 6, 20000, 200, 300, 300, 2),
                                                        (63, 5, 9000, 33, 0, 0, 3)])
def test_engine_matches_oracle_c5_contended(seed, u, m, b, drop, dup, props):
    """Contended C5 (gen_member proposers > 1): in every epoch from 2 on a rival member proposer
    prepares above the leader over its own unlearned ids — promise replies carrying most of the
    history, merged pre-accepted maps (member/paxos.cpp:1158-1182,1614-1629), rejected ACCEPTs
    and the leader's re-prepare; the engine == the oracle through the run and the step."""
    t = mpx.generate_trace(mpx.GEN_MEMBER, num_nodes=u, num_instances=m, seed=seed, batch=b,
                           drop_rate=drop, dup_rate=dup, max_delay=64, noop_permille=15, proposers=props)
    want, ostats, _ = oracle_run(t)
    with mpx.Engine.for_trace(t) as e:
        st = e.run()
        got = e.dump()
        assert got == want, mpxr.diff(got, want)
        _step_path(e, want, st)
    assert [st[k] for k in STATS_ORDER] == ostats
    assert st["promise_entries"] > m and st["violations"] == 0


def test_c5_contended_2_20_matches_oracle():
    """Contended C5 at 2^20 instances (acceptor universe 8, 3 proposers, 1 % loss / dup):
    several million promise entries; counters and digests == the CPU oracle's."""
    st = _full_size_vs_oracle(mpx.GEN_MEMBER, num_nodes=8, num_instances=1 << 20, seed=0, batch=256,
                              drop_rate=100, dup_rate=100, max_delay=64, noop_permille=15, proposers=3)
    assert st["promise_entries"] >= 10 ** 6 and st["violations"] == 0


@pytest.mark.parametrize("seed,u,m,b,drop,dup", [(41, 8, 1 << 15, 256, 100, 100), (42, 6, 20000, 200, 300, 300),
                                                  (43, 8, 1 << 14, 90, 0, 0), (44, 4, 9000, 33, 500, 500),
                                                  (45, 8, (1 << 15) + 77, 256, 1000, 1000)])
def test_member_plan_path(seed, u, m, b, drop, dup):
    """The member step's plan path (k_plan_member: one plan word per (node, bucket) pair,
    member/paxos.cpp:1744-1793 insert-first accept / learn, Acceptor deletion at E_EPOCH
    markers) equals the oracle through the step, and plans most pairs: the general walk
    takes only what it lists (snapshots to emit, Value checks, > 4 segments or > 16 runs)."""
    t = mpx.generate_trace(mpx.GEN_MEMBER, num_nodes=u, num_instances=m, seed=seed, batch=b,
                           drop_rate=drop, dup_rate=dup, max_delay=64, noop_permille=15)
    want, ostats, _ = oracle_run(t)
    with mpx.Engine.for_trace(t) as e:
        st = e.run()
        assert e.dump() == want
        walked = st["general_pairs"]
        e.step()
        e.sync()
        step = e.stats()
        assert [step[k] for k in STATS_ORDER[:5]] == ostats[:5]
        assert e.state_digest() == (ostats[6], ostats[5])
        assert e.dump() == want
        if b >= 200:
            assert step["general_pairs"] * 4 < walked, (step["general_pairs"], walked)
        # the walk of every pair in the step (MPX_STEP_WALK=1) agrees too
        os.environ["MPX_STEP_WALK"] = "1"
        try:
            e.step()
            e.sync()
            assert e.stats()["general_pairs"] == walked
            assert e.dump() == want
        finally:
            del os.environ["MPX_STEP_WALK"]


def test_engine_member_violations():
    from handmade_member import member_violation_traces
    t = member_violation_traces()["mm_violations"]
    want, ostats, oviol = oracle_run(t)
    with mpx.Engine.for_trace(t) as e:
        st = e.run()
        got = e.dump()
        v = e.violation()
    assert got == want, mpxr.diff(got, want)
    assert st["violations"] == ostats[4] == 3
    assert v["code"] in (3, 6)
    with mpx.Engine.for_trace(t) as e:              # the step: the plan lists the pairs with Value checks
        e.step()
        e.sync()
        assert e.stats()["violations"] == 3
        assert e.dump() == want


def test_engine_commit_value_check_on_planned_pairs():
    """Re-commits through other messages' entries on a whole bucket (the plan path keeps the
    pair and k_commit_check compares the Values): an equal re-commit is silent, a different
    Value is MPX_V_COMMIT_VALUE once per slot (multi/paxos.cpp:1508), as in the oracle."""
    from handmade import B1, B2, B3, v
    w = mpxwire
    ent = [(i, v(i)) for i in range(4)]
    t = w.container([[
        w.prepare(0, B1),
        w.accept(0, 1, B1, ent),
        w.commit(0, 1, B1, ent),
        w.commit(1, 9, B2, ent[1:3]),                                 # equal Values, other entries
        w.commit(2, 4, B3, [(2, v(2, 2, 77)), (3, v(3, 2, 78))]),     # two slots differ
        w.accept(1, 2, B2, [(1, v(1, 1, 90)), (2, v(2, 1, 91))]),     # over committed: skipped
        w.commit(1, 10, B2, ent[:2]),
    ], [w.prepare(0, B1), w.accept(0, 1, B1, ent)], []], 256)
    want, ostats, _ = oracle_run(t)
    assert ostats[4] == 2
    with mpx.Engine.for_trace(t) as e:
        st = e.run()
        assert e.dump() == want
    assert st["violations"] == 2
    with mpx.Engine.for_trace(t) as e:
        e.step()
        e.sync()
        st = e.stats()
        assert st["violations"] == 2 and e.violation()["code"] == 1   # MPX_V_COMMIT_VALUE
        assert e.dump() == want


@pytest.mark.parametrize("shards", [2, 3])
def test_engine_member_sharded_matches_oracle_restricted(shards):
    """Instance shards of a member trace: headers (and so roles, versions, scalars,
    quorums) are replicated, entries split; per-shard state == the oracle's, restricted."""
    m = 2000
    t = mpx.generate_trace(mpx.GEN_MEMBER, num_nodes=6, num_instances=m, seed=31, batch=40,
                           drop_rate=300, dup_rate=200, max_delay=32)
    full = mpxr.parse(oracle_run(t)[0])
    from mpx import dist as mdist
    for r in range(shards):
        sb, se = mdist.shard_bounds(m, shards, r)
        if sb == se:
            continue
        with mpx.Engine(6, sb, se, semantics=mpx.SEM_MEMBER) as e:
            e.submit_trace(t)
            e.run()
            part = mpxr.parse(e.dump())
        for a, b in zip(part["nodes"], full["nodes"]):
            assert a["state"] == [s for s in b["state"] if sb <= s[0] < se]
            assert (a["promised"], a["max_seen"]) == (b["promised"], b["max_seen"])
        assert part["chosen"] == [c for c in full["chosen"] if sb <= c[0] < se]


def _clean_with_extra_runs(n, m, extra):
    """A clean batch-256 trace (gen_clean's shape) where node 1 also receives, for
    each bucket k in `extra`, a partial ACCEPT from proposer 2 at the leader's
    ballot before the bucket's own ACCEPT (granted, then overwritten) and a partial
    ACCEPT after its COMMIT (skipped: committed, multi/paxos.cpp:1380) — pairs
    with more than two runs inside the store chunks, next to uniform ones."""
    from mpxwire import accept, accept_reply, commit, commit_reply, container, p_batch, p_start, prepare, \
        prepare_reply, value
    b0 = 1 << 16
    s0 = [p_start(b0), prepare(0, b0)] + [prepare_reply(i, b0) for i in range(n)]
    si = [[prepare(0, b0)] for _ in range(1, n)]
    for k in range((m + 255) // 256):
        ent = [(i, value(0, i + 1, str(i))) for i in range(256 * k, min(m, 256 * k + 256))]
        acc, com = accept(0, k + 1, b0, ent), commit(0, k + 1, b0, ent)
        s0 += [p_batch(k + 1, ent), acc] + [accept_reply(i, b0, k + 1) for i in range(n)] + [com] + \
            [commit_reply(i, k + 1) for i in range(n)]
        for j in range(1, n):
            if j == 1 and k in extra:
                part = [(i, value(2, 10 ** 6 + i, "x%d" % i)) for i in range(256 * k + 10, 256 * k + 50)]
                si[j - 1] += [accept(2, 7000 + k, b0, part), acc, com, accept(2, 8000 + k, b0, part)]
            else:
                si[j - 1] += [acc, com]
    return container([s0] + si, m)


@pytest.mark.parametrize("extra", [(), (3, 70, 100, 127, 200, 300)])
def test_store_chunks_tails_and_partial_pairs(extra):
    """1-byte slots with two whole 128-bucket store chunks per row, 70 tail buckets and a
    partial last bucket; optionally pairs of 4 runs inside the chunks (plan word
    PLAN_SKIP in both of a lane's plan words) left to the per-slot path."""
    n, m = 3, 256 * (2 * 128 + 70) + 100
    t = _clean_with_extra_runs(n, m, set(extra))
    want, ostats, _ = oracle_run(t)
    with mpx.Engine.for_trace(t) as e:
        st = e.run()
        assert e.dump() == want
        _step_path(e, want, st)
    assert [st["chosen"], st["promise_entries"], st["accept_apps"], st["commit_apps"], st["violations"],
            st["chosen_digest"], st["state_digest"], st["scalar_digest"]] == ostats


@pytest.mark.parametrize("env", [("MPX_PROP_CHUNK", "64"), ("MPX_PROP_CHUNK", "5"), ("MPX_STEP_WALK", "1"),
                                 ("MPX_SCAN_SMALL", "0"), ("MPX_SCAN_SMALL", "1"), ("MPX_PLAN_STORE", "0")])
@pytest.mark.parametrize("name", ["fuzz_big_0", "c3_faulty_1", "c2_clean_n9_b100", "c5_member_1", "c5_member_3",
                                  "demo_s0", "demo5_s3", "hm_promise_merge"])
def test_kept_alternative_paths(name, env, monkeypatch):
    """The supported alternatives stay correct: promise-quorum chunks small
    enough that rounds span chunks (k_prop_chunk's deferred prefixes, k_prop_node's carry),
    either header-scan chunk size whatever the stream length (MPX_SCAN_SMALL: the size
    scan_chunk_for picks by length),
    and a step that walks every pair as the digested run does (MPX_STEP_WALK; the path of
    multi traces with more than FAST_MAX_NODES nodes).  The measured-and-rejected variants
    of earlier rounds are no longer compiled (their A/B records stay in profiles/)."""
    if name not in INDEX:
        pytest.skip("no golden " + name)
    monkeypatch.setenv(*env)
    trace, want = _read(name, ".mpxt"), _read(name, ".mpxr")
    with mpx.Engine.for_trace(trace) as e:
        st = e.run()
        assert e.dump() == want
        _step_path(e, want, st)


def test_clean_long_node_stream_scan_lookback():
    """A node stream of hundreds of header-scan chunks: the single-pass scan's chunk look-back
    walks back over more than 64 predecessors (wave-wide sweeps); the result equals the
    oracle's."""
    n, m = 2, 320000                         # batch 1: node 0 gets 7 records per instance -> 547 chunks of 4096
    t = mpx.generate_trace(mpx.GEN_CLEAN, num_nodes=n, num_instances=m, batch=1)
    _, ostats, _ = oracle_run(t)
    with mpx.Engine.for_trace(t) as e:
        st = e.run()
    assert [st["chosen"], st["promise_entries"], st["accept_apps"], st["commit_apps"], st["violations"],
            st["chosen_digest"], st["state_digest"], st["scalar_digest"]] == ostats


# ---- the stated configs at full size (BASELINE.json configs[2], configs[4]) ----
STATS_ORDER = ("chosen", "promise_entries", "accept_apps", "commit_apps", "violations",
               "chosen_digest", "state_digest", "scalar_digest")


# the same configs judged by the REFERENCE's own handlers, per instance shard (oracle/ref_full_size.py,
# VERDICT r04 item 3): counters + digests, with the size and xxh3 of the trace they judged
FULL_SIZE = json.load(open(os.path.join(GOLD, "full_size.json")))


def _full_size_vs_oracle(kind, oracle_threads=1, ref=None, **kw):
    import time
    from oracles import oracle_run_sharded
    t0 = time.time()
    log = lambda m: print("[full-size] %s: %s (%.0f s)" % (kw.get("num_instances"), m, time.time() - t0), flush=True)
    t = mpx.generate_trace(kind, copy=False, **kw)           # the generator's buffer, no bytes copy
    log("generated %.1f GB" % (len(t) / 1e9))
    if ref is not None:
        import xxhash
        r = FULL_SIZE[ref]
        # the reference judged these very bytes (the generator is deterministic)
        assert (len(t), "%016x" % xxhash.xxh3_64_intdigest(memoryview(t))) == (r["trace_bytes"], r["trace_xxh3"])
    want = oracle_run_sharded(t, shards=oracle_threads, threads=oracle_threads)   # CPU oracle, digests only
    log("oracle")
    if ref is not None:                                      # restatement == reference at full size
        assert want[:4] + want[5:] == [FULL_SIZE[ref]["stats"][k] for k in STATS_ORDER if k != "violations"]
    e = mpx.Engine.for_trace(t)
    del t
    log("ingested")
    with e:
        st = e.run()
        log("run")
        e.step()                                             # the timed path, digested by a separate pass
        e.sync()
        step = e.stats()
        sd = e.state_digest()
    assert [st[k] for k in STATS_ORDER] == want
    assert sd == (st["state_digest"], st["chosen_digest"])
    assert [step[k] for k in STATS_ORDER[:5]] == want[:5]
    return st


def test_c3_full_size_matches_oracle():
    """C3 at its stated size: 2^24 instances x 7 acceptors, 3 competing proposers,
    drop 5 % / dup 10 % (<=3) / delay U[0,500) (multi/debug.conf.sample:1), batch U[1,256];
    every counter and order-independent digest equals the CPU oracle's."""
    st = _full_size_vs_oracle(mpx.GEN_FAULTY, num_nodes=7, num_instances=1 << 24, seed=0, batch=256,
                              proposers=3, drop_rate=500, dup_rate=1000, max_delay=500, ref="c3")
    assert st["chosen"] >= 1 << 24 and st["promise_entries"] > 0 and st["violations"] == 0


@pytest.mark.timeout(900)
def test_c5_contended_full_size_matches_oracle():
    """Contended C5 at its stated size: 2^25 instances, 3 member proposers (a rival round per
    epoch from epoch 2, member/paxos.cpp:1158-1182,1504-1549,1614-1629); >= 10^6 promise
    entries; every counter and digest == the CPU oracle's (node-parallel, 8 threads)."""
    st = _full_size_vs_oracle(mpx.GEN_MEMBER, num_nodes=8, num_instances=1 << 25, seed=0, batch=256,
                              drop_rate=100, dup_rate=100, max_delay=64, noop_permille=15, proposers=3,
                              oracle_threads=8, ref="c5c" if "c5c" in FULL_SIZE else None)
    assert st["promise_entries"] >= 10 ** 6 and st["violations"] == 0


def test_c5_full_size_matches_oracle():
    """C5 at its stated size: 2^25 instances, member semantics, acceptor universe 8 —
    AddAcceptor(1..7) then DelAcceptor(1..7), 15 epochs (member/main.cpp:119-141), 1 % loss,
    1 % duplicates, stale in-flight ACCEPTs across version changes."""
    st = _full_size_vs_oracle(mpx.GEN_MEMBER, num_nodes=8, num_instances=1 << 25, seed=0, batch=256,
                              drop_rate=100, dup_rate=100, max_delay=64, noop_permille=15,
                              ref="c5" if "c5" in FULL_SIZE else None)
    assert st["chosen"] == 1 << 25 and st["violations"] == 0


# ---- phase-2 decisions at promise quorums (multi/paxos.cpp:1056-1130) ----
DECISIONS = json.load(open(os.path.join(GOLD, "decisions.json")))
LEARNS = json.load(open(os.path.join(GOLD, "learns.json")))


@pytest.mark.parametrize("name", sorted(DECISIONS))
def test_engine_decisions_match_reference(name):
    """The device's phase-2 batch at every promise quorum (adopt the merged
    pre-accepted values of instances the node has not committed, noop-fill the
    other uncommitted instances below the highest committed-or-adopted one) ==
    the batch the reference's own OnPrepareReply built (fixture), on both apply paths."""
    trace, want = _read(name, ".mpxt"), _read(name, ".mpxd")
    with mpx.Engine.for_trace(trace) as e:
        e.run()
        assert e.decisions() == want
        e.step()
        e.sync()
        assert e.decisions() == want


PROPOSAL_TRACES = ["demo5_s3", "demo5_s4", "demo_s0", "demo_s1", "demo_s2", "hm_propose"]   # P_PROPOSE records


@pytest.mark.parametrize("name", sorted(set(DECISIONS) - set(PROPOSAL_TRACES)))
def test_proposer_host_sim_matches_device_decisions(name, monkeypatch):
    """The proposer's sequential bookkeeping on the host (MPX_DECIDE_HOST=1; what a trace with
    client values takes) == the device decision kernels on traces without client values."""
    trace, want = _read(name, ".mpxt"), _read(name, ".mpxd")
    with mpx.Engine.for_trace(trace) as e:
        e.run()
        assert e.decisions() == want
        monkeypatch.setenv("MPX_DECIDE_HOST", "1")
        assert e.decisions() == want


@pytest.mark.parametrize("name", ["demo_s1", "hm_propose"])
def test_proposal_traces_refuse_sharded_decisions(name):
    """Client values make the batch depend on the whole node's stream (value ids shared with
    the noop fill): decisions are read from a whole engine; the shard protocol refuses."""
    trace, want = _read(name, ".mpxt"), _read(name, ".mpxd")
    with mpx.Engine.for_trace(trace) as e:
        e.run()
        assert e.decisions() == want
        with pytest.raises(mpx.MpxError):
            e.decision_bounds()


MEMBER_DECISIONS = sorted(k for k in DECISIONS if k.startswith(("c5_", "mm_")))


@pytest.mark.parametrize("shards", [2, 3])
@pytest.mark.parametrize("name", MEMBER_DECISIONS)
def test_member_sharded_decisions(name, shards):
    """Member decisions over instance shards (unaligned): each shard's events — Propose,
    StartPrepare, E_EPOCH, its instances' entries of each LEARN and promise quorum
    (mpx_proposal_part, MPXE version 2 with the epoch table) — merged by record in shard
    order, the member Proposer's walk once over the union (mpx_proposal_combine) == the
    reference's own decisions (fixture, real Proposer::Propose calls)."""
    from mpx import dist as mdist
    trace, want = _read(name, ".mpxt"), _read(name, ".mpxd")
    hd = mpx.trace_header(trace)
    m = max(hd["num_instances"], 1)
    parts = []
    for r in range(shards):
        sb, se = mdist.shard_bounds(m, shards, r, align=1)
        with mpx.Engine(hd["num_nodes"], sb, se, semantics=hd["semantics"]) as e:
            e.submit_trace(trace)
            e.run()
            if sb > 0:
                with pytest.raises(mpx.MpxError):
                    e.decisions()                     # a shard past instance 0 cannot decide alone
            parts.append(e.proposal_part())
    assert mpx.proposal_combine(parts) == want


@pytest.mark.parametrize("shards", [2, 3])
@pytest.mark.parametrize("name", ["demo_s1", "demo5_s3", "hm_propose"])
def test_proposal_traces_sharded_decisions(name, shards):
    """Decisions with client values over instance shards (unaligned): each shard's events
    (mpx_proposal_part) merged by record in shard order, the proposer's walk once over the
    union (mpx_proposal_combine) == the reference's own decisions (fixture)."""
    from mpx import dist as mdist
    trace, want = _read(name, ".mpxt"), _read(name, ".mpxd")
    hd = mpx.trace_header(trace)
    m = max(hd["num_instances"], 1)
    parts = []
    for r in range(shards):
        sb, se = mdist.shard_bounds(m, shards, r, align=1)
        with mpx.Engine(hd["num_nodes"], sb, se) as e:
            e.submit_trace(trace)
            e.run()
            parts.append(e.proposal_part())
    assert mpx.proposal_combine(parts) == want
    with pytest.raises(mpx.MpxError):
        mpx.proposal_combine(parts[::-1])                 # not in shard order


@pytest.mark.parametrize("seed,m", [(81, 1 << 12), (82, 3000), (83, 1 << 14)])
def test_engine_decisions_match_oracle_c3(seed, m):
    from oracles import oracle_decisions
    t = mpx.generate_trace(mpx.GEN_FAULTY, num_nodes=7, num_instances=m, seed=seed, batch=64, proposers=3,
                           drop_rate=500, dup_rate=1000, max_delay=500)
    want = oracle_decisions(t)
    with mpx.Engine.for_trace(t) as e:
        e.run()
        got = e.decisions()
    import mpxd
    assert sum(len(x) for x in mpxd.parse(want)) > 0
    assert got == want


def _sharded_decisions(trace, shards, align=256):
    """The sharded protocol of include/mpx.h: bounds per shard -> max -> parts -> combine."""
    from mpx import dist as mdist
    hd = mpx.trace_header(trace)
    m = max(hd["num_instances"], 1)
    engines = []
    try:
        for r in range(shards):
            sb, se = mdist.shard_bounds(m, shards, r, align=align)
            e = mpx.Engine(hd["num_nodes"], sb, se, semantics=hd["semantics"])
            engines.append(e)
            e.submit_trace(trace)
            e.run()
        bounds = [e.decision_bounds() for e in engines]
        assert len({len(b) for b in bounds}) == 1            # the same promise quorums on every shard
        gx = [max(col) for col in zip(*bounds)]
        parts = [e.decisions_part(gx) for e in engines]
    finally:
        for e in engines:
            e.close()
    return mpx.decisions_combine(parts)


@pytest.mark.parametrize("shards", [2, 3])
@pytest.mark.parametrize("name", ["fuzz_big_1", "fuzz_big_2", "c3_faulty_0", "c3_faulty_1", "hm_promise_merge", "fuzz_007"])
def test_sharded_decisions_match_reference(name, shards):
    """Phase-2 decisions over instance shards (one engine per range; one
    all-reduce-MAX of the per-quorum fill bounds, then the parts merged in shard
    order) == the batch the reference's own OnPrepareReply built (fixture)."""
    trace, want = _read(name, ".mpxt"), _read(name, ".mpxd")
    assert _sharded_decisions(trace, shards, align=1) == want     # unaligned, non-empty shards of small runs


@pytest.mark.parametrize("name", ["fuzz_big_1", "c3_faulty_0", "c3_faulty_1", "hm_promise_merge"])
def test_committed_before_host_prefix_matches_device_pass(name, monkeypatch):
    """'Highest instance committed before the quorum' from the node's COMMIT messages in
    order (host prefix max, the default) == k_decide pass 0's scan of every slot."""
    trace = _read(name, ".mpxt")
    with mpx.Engine.for_trace(trace) as e:
        e.run()
        d_host, c_host, b_host = e.decisions(), e.commits(), e.decision_bounds()
        monkeypatch.setenv("MPX_DECIDE_DEVICE", "1")
        assert (e.decisions(), e.commits(), e.decision_bounds()) == (d_host, c_host, b_host)


@pytest.mark.parametrize("shards", [2, 4])
def test_sharded_decisions_match_oracle_c3(shards):
    from oracles import oracle_decisions
    t = mpx.generate_trace(mpx.GEN_FAULTY, num_nodes=7, num_instances=1 << 13, seed=84, batch=64, proposers=3,
                           drop_rate=500, dup_rate=1000, max_delay=500)
    want = oracle_decisions(t)
    with mpx.Engine.for_trace(t) as e:
        e.run()
        assert e.decisions() == want
    assert _sharded_decisions(t, shards) == want


def test_decisions_refused_for_shards():
    t = mpx.generate_trace(mpx.GEN_CLEAN, num_nodes=3, num_instances=1024, batch=256)
    with mpx.Engine(3, 256, 1024) as e:
        e.submit_trace(t)
        e.run()
        with pytest.raises(mpx.MpxError):
            e.decisions()


# ---- incremental submission (multi/paxos.cpp:1714-1717) ----
def _node_streams(trace):
    """MPXT -> (header, epochs [(version, amask, pmask, lmask)], per-node lists of record bytes)."""
    import struct
    hd = mpx.trace_header(trace)
    epochs = mpx.trace_epochs(trace)
    pos = 40 + (24 if hd["version"] == 1 else 32) * len(epochs)
    streams = []
    for _ in range(hd["num_nodes"]):
        cnt, nb = struct.unpack_from("<QQ", trace, pos)
        offs = struct.unpack_from("<%dQ" % (cnt + 1), trace, pos + 16)
        body = pos + 16 + 8 * (cnt + 1)
        streams.append([bytes(trace[body + offs[k]: body + offs[k + 1]]) for k in range(cnt)])
        pos = (body + nb + 7) & ~7
    return hd, epochs, streams


@pytest.mark.parametrize("name", sorted(INDEX))
def test_incremental_submit_matches_whole(name):
    """Every golden split at 3 points: submit each node's first part, run, submit
    the rest, run again — the result equals the whole trace's (the reference's)."""
    trace, want = _read(name, ".mpxt"), _read(name, ".mpxr")
    hd, epochs, streams = _node_streams(trace)
    for frac in (0.25, 0.5, 0.75):
        with mpx.Engine(hd["num_nodes"], 0, max(hd["num_instances"], 1), semantics=hd["semantics"],
                        epochs=epochs) as e:
            cut = [int(len(s) * frac) for s in streams]
            for n, s in enumerate(streams):
                if cut[n]:
                    e.submit(n, s[:cut[n]])
            e.run()
            for n, s in enumerate(streams):
                if cut[n] < len(s):
                    e.submit(n, s[cut[n]:])
            e.run()
            got = e.dump()
        assert got == want, (frac, mpxr.diff(got, want))


# ---- SoA submission (mpx_submit_soa) ----
def _soa_records(stream):
    """Decode one node's multi wire records (multi/paxos.cpp:741-755,830-856,1282-1297,1345-1357,
    1429-1444,1481-1492; P_START / P_BATCH) into mpx_submit_soa tuples: Values become handles."""
    import struct

    def value(b, o):
        prop, vid, noop = struct.unpack_from("<IQ?", b, o)
        o += 13
        if not noop:
            mem, ln = struct.unpack_from("<?I", b, o)
            assert not mem
            o += 5 + ln
        return mpxwire.handle(prop, vid, noop), o

    out = []
    for m in stream:
        t = struct.unpack_from("<I", m)[0]
        ents = []
        src = ballot = aux = 0
        if t == 0:
            src, ballot, rl = struct.unpack_from("<IQI", m, 4)
            ents = [struct.unpack_from("<QQ", m, 20 + 16 * k) for k in range(rl // 16)]
        elif t == 1:
            src, ballot, vl = struct.unpack_from("<IQI", m, 4)
            o = 20
            while o < 20 + vl:
                iid, pid = struct.unpack_from("<QQ", m, o)
                h, o = value(m, o + 16)
                ents.append((iid, h, pid))
        elif t == 2:
            ballot = struct.unpack_from("<Q", m, 4)[0]
        elif t in (3, 5):
            src, aux, ballot, vl = struct.unpack_from("<IQQI", m, 4)
            o = 28
            while o < 28 + vl:
                iid = struct.unpack_from("<Q", m, o)[0]
                h, o = value(m, o + 8)
                ents.append((iid, h))
        elif t == 4:
            src, ballot, aux = struct.unpack_from("<IQQ", m, 4)
        elif t == 6:
            src, aux = struct.unpack_from("<IQ", m, 4)
        elif t == 16:
            ballot = struct.unpack_from("<Q", m, 4)[0]
        elif t == 17:
            aux, vl = struct.unpack_from("<QI", m, 4)
            o = 16
            while o < 16 + vl:
                iid = struct.unpack_from("<Q", m, o)[0]
                h, o = value(m, o + 8)
                ents.append((iid, h))
        out.append((t, src, ballot, aux, ents))
    return out


@pytest.mark.parametrize("name", ["fuzz_big_0", "hm_commit_tags", "hm_promise_merge", "c3_faulty_0"])
def test_submit_soa_matches_wire(name):
    """The same records through the SoA fast path (no wire codec, payload-free Values) and
    through mpx_submit: identical state, scalars, counters and digests (both name Values
    by handle), and the same replies apart from the Value bytes in PREPARE_REPLYs."""
    trace = _read(name, ".mpxt")
    hd, _ep, streams = _node_streams(trace)
    n, m = hd["num_nodes"], max(hd["num_instances"], 1)
    if hd["semantics"] != mpx.SEM_MULTI:
        pytest.skip("member trace")
    want = _whole(trace)
    with mpx.Engine(n, 0, m) as e:
        for node, s in enumerate(streams):
            e.submit_soa(node, _soa_records(s))
        st = e.run()
        assert {k: st[k] for k in COUNTERS} == want[1]
        assert _observe(e, n, m) == want[2]
        got = [[] for _ in range(n)]
        for src, dst, b in e.drain_sends():
            got[src].append((dst, b))
    for a, b in zip(got, want[0]):
        assert len(a) == len(b)
        assert [x for x in a if x[1][:4] != b"\x01\x00\x00\x00"] == [x for x in b if x[1][:4] != b"\x01\x00\x00\x00"]


# ---- incremental windows (MPX_FLAG_INCREMENTAL; multi/paxos.cpp:1714-1717) ----
def _observe(e, n_nodes, m):
    """Everything a caller can read back after a run: per-node state / scalars / executed
    stream, the chosen log, the device digests."""
    return {"state": [e.read_node_state(n, 0, m) for n in range(n_nodes)],
            "scalars": [e.read_node_scalars(n) for n in range(n_nodes)],
            "executed": [e.read_executed(n) for n in range(n_nodes)],
            "chosen": e.read_chosen(0, m), "digests": e.state_digest()}


def _whole(trace):
    hd = mpx.trace_header(trace)
    n, m = hd["num_nodes"], max(hd["num_instances"], 1)
    with mpx.Engine.for_trace(trace) as e:
        st = e.run()
        sends = [[] for _ in range(n)]
        for src, dst, b in e.drain_sends():
            sends[src].append((dst, b))
        return sends, {k: st[k] for k in COUNTERS}, _observe(e, n, m)


def _windows(trace, fracs, times=None):
    """The trace's node streams cut at `fracs` of each node's records: one mpx_submit per
    node and window, one incremental mpx_run per window."""
    import time
    hd, epochs, streams = _node_streams(trace)
    n, m = hd["num_nodes"], max(hd["num_instances"], 1)
    sends = [[] for _ in range(n)]
    tot = {k: 0 for k in COUNTERS}
    with mpx.Engine(n, 0, m, semantics=hd["semantics"], epochs=epochs, flags=mpx.FLAG_INCREMENTAL) as e:
        prev = [0] * n
        for f in list(fracs) + [1.0]:
            cut = [len(s) if f >= 1.0 else int(len(s) * f) for s in streams]
            t0 = time.perf_counter()
            for node, s in enumerate(streams):
                if cut[node] > prev[node]:
                    e.submit(node, s[prev[node]:cut[node]])
            st = e.run()
            if times is not None:
                times.append(time.perf_counter() - t0)
            prev = cut
            for k in COUNTERS:
                tot[k] += st[k]
            for src, dst, b in e.drain_sends():
                sends[src].append((dst, b))
        with pytest.raises(mpx.MpxError):          # windows are applied once: no replay, no history readback
            e.step()
        with pytest.raises(mpx.MpxError):
            e.dump()
        return sends, tot, _observe(e, n, m)


def test_incremental_member_marker_limit_covers_the_stream():
    """The member incarnation counter (G_SEG: at most 254 E_EPOCH records per node) counts over
    the whole live stream, not per window (include/mpx.h MPX_FLAG_INCREMENTAL, DESIGN.md §9;
    ADVICE r04).  Windows of 127 markers on node 0: two are applied (254 so far), the third
    window's one more marker is refused with MPX_E_RANGE, stays queued (refused again on the
    next run) and leaves the engine readable (not poisoned)."""
    epochs = [(k, 1, 1, 1) for k in range(300)]
    with mpx.Engine(2, 0, 64, semantics=mpx.SEM_MEMBER, epochs=epochs, flags=mpx.FLAG_INCREMENTAL) as e:
        for k0 in (1, 128):
            e.submit(0, [mpxwire.e_epoch(k) for k in range(k0, k0 + 127)])
            e.run()
        d = e.state_digest()
        e.submit(0, [mpxwire.e_epoch(255)])
        for _ in range(2):
            with pytest.raises(mpx.MpxError) as ex:
                e.run()
            assert ex.value.rc == -5
        assert e.state_digest() == d


MULTI_GOLDENS = sorted(k for k in INDEX if not k.startswith(("c5_", "mm_")) and "member" not in k)


@pytest.mark.parametrize("name", sorted(set(DECISIONS) | set(LEARNS)))
def test_incremental_windows_carry_decisions(name):
    """MPX_FLAG_DECISIONS: every golden with a promise quorum (client values included; member:
    also every one with learns) cut into 1, 2 and 4 windows — the proposers' bookkeeping
    advanced window by window over the device's quorums and merged maps gives the reference's
    decisions (fixture); member windows also carry the learn bookkeeping (LearningValues,
    member/paxos.cpp:1345-1381,1472-1549) and give the reference's learns; without the flag a
    window engine keeps neither."""
    trace = _read(name, ".mpxt")
    want = _read(name, ".mpxd") if name in DECISIONS else None
    want_l = _read(name, ".mpxl") if name in LEARNS else None
    hd, epochs, streams = _node_streams(trace)
    n, m = hd["num_nodes"], max(hd["num_instances"], 1)
    kw = dict(semantics=hd["semantics"], epochs=epochs) if hd["semantics"] == mpx.SEM_MEMBER else {}
    for fracs in ((), (0.5,), (0.2, 0.45, 0.8)):
        with mpx.Engine(n, 0, m, flags=mpx.FLAG_INCREMENTAL | mpx.FLAG_DECISIONS, **kw) as e:
            prev = [0] * n
            for f in list(fracs) + [1.0]:
                cut = [len(s) if f >= 1.0 else int(len(s) * f) for s in streams]
                for node, st in enumerate(streams):
                    if cut[node] > prev[node]:
                        e.submit(node, st[prev[node]:cut[node]])
                e.run()
                prev = cut
            if want is not None:
                assert e.decisions() == want, fracs
            if want_l is not None:
                assert e.learns() == want_l, fracs
    with mpx.Engine(n, 0, m, flags=mpx.FLAG_INCREMENTAL, **kw) as e:
        for node, st in enumerate(streams):
            e.submit(node, st)
        e.run()
        with pytest.raises(mpx.MpxError):
            e.decisions()
        with pytest.raises(mpx.MpxError):
            e.learns()


@pytest.mark.parametrize("name", sorted(INDEX))
def test_incremental_windows_match_whole(name):
    """Every golden, multi and member, cut into 1, 2 and 4 windows: the replies of the
    windows, node by node, are the whole run's (the reference's: test_engine_goldens), and so
    are the counters summed over the windows and the final state, scalars, executed streams,
    chosen log and digests.  Member windows carry each node's roles (epoch, Acceptor
    incarnation, Proposer), its scan keys with the incarnation and the batches a marker
    cleared (member/paxos.cpp:841-844 OnReceive per message, :1864-1964)."""
    trace = _read(name, ".mpxt")
    want = _whole(trace)
    for fracs in ((), (0.5,), (0.2, 0.45, 0.8)):
        got = _windows(trace, fracs)
        assert got[0] == want[0], ("sends", fracs)
        assert got[1] == want[1], ("counters", fracs)
        assert got[2] == want[2], ("state", fracs)


@pytest.mark.parametrize("seed", [5, 6])
def test_incremental_windows_c3(seed):
    """A C3-shaped trace (3 competing proposers, drops, duplicates, reordering: promise
    rounds and batches that span windows) in 7 windows == the whole run."""
    t = mpx.generate_trace(mpx.GEN_FAULTY, num_nodes=7, num_instances=1 << 15, seed=seed, batch=64, proposers=3,
                           drop_rate=500, dup_rate=1000, max_delay=500)
    want = _whole(t)
    got = _windows(t, [k / 7 for k in range(1, 7)])
    assert got[0] == want[0]
    assert got[1] == want[1]
    assert got[2] == want[2]


@pytest.mark.parametrize("seed,W,drain", [(5, 7, False), (6, 5, True), (7, 16, False)])
def test_incremental_async_submit_equals_whole(seed, W, drain):
    """The pipelined live loop (mpx_submit_trace_range_async: window k + 1 decoded on a host thread
    while window k is built and run; mpx_run joins it when nothing else is queued, a Value readback
    joins it first) == the whole run: counters summed over the windows, replies (drained per window,
    which joins the decode in flight) and the final state, scalars, executed streams, chosen log and
    digests, and the decisions of MPX_FLAG_DECISIONS."""
    t = mpx.generate_trace(mpx.GEN_FAULTY, num_nodes=7, num_instances=1 << 15, seed=seed, batch=64, proposers=3,
                           drop_rate=500, dup_rate=1000, max_delay=500)
    want = _whole(t)
    with mpx.Engine.for_trace(t) as e:
        e.run()
        want_dec = e.decisions()
    hd = mpx.trace_header(t)
    idx = mpx.trace_index(t)
    n, m = hd["num_nodes"], max(hd["num_instances"], 1)
    cuts = [[c * w // W for (c, _, _) in idx] for w in range(W + 1)]
    tot = {k: 0 for k in COUNTERS}
    sends = [[] for _ in range(n)]
    with mpx.Engine(n, 0, m, flags=mpx.FLAG_INCREMENTAL | mpx.FLAG_DECISIONS) as e:
        e.submit_window(t, cuts[0], cuts[1])
        for w in range(1, W + 1):
            if w < W:
                e.submit_window_async(t, cuts[w], cuts[w + 1])
            st = e.run()
            for k in COUNTERS:
                tot[k] += st[k]
            if drain:
                for src, dst, b in e.drain_sends():
                    sends[src].append((dst, b))
        assert tot == want[1]
        if drain:
            assert sends == want[0]
        assert _observe(e, n, m) == want[2]
        assert e.decisions() == want_dec


def test_incremental_async_submit_refused_without_incremental():
    """mpx_submit_trace_range_async needs an incremental multi-semantics engine (MPX_E_STATE)."""
    t = mpx.generate_trace(mpx.GEN_CLEAN, num_nodes=3, num_instances=512, batch=256)
    idx = mpx.trace_index(t)
    with mpx.Engine(3, 0, 512) as e:
        with pytest.raises(mpx.MpxError) as ex:
            e.submit_window_async(t, [0] * 3, [c for (c, _, _) in idx])
        assert ex.value.rc == -6


@pytest.mark.parametrize("seed,u,m,b,drop,dup", [(51, 8, 1 << 15, 256, 100, 100), (52, 6, 20000, 90, 500, 500),
                                                  (53, 5, 9000, 33, 1000, 1000)])
def test_incremental_windows_member(seed, u, m, b, drop, dup):
    """C5-shaped member traces (AddAcceptor / DelAcceptor epochs, stale versions, loss and
    duplicates: markers, Acceptor deletions and Proposer resets in every window) in 7 windows
    == the whole run."""
    t = mpx.generate_trace(mpx.GEN_MEMBER, num_nodes=u, num_instances=m, seed=seed, batch=b,
                           drop_rate=drop, dup_rate=dup, max_delay=64, noop_permille=15)
    want = _whole(t)
    got = _windows(t, [k / 7 for k in range(1, 7)])
    assert got[0] == want[0]
    assert got[1] == want[1]
    assert got[2] == want[2]


@pytest.mark.parametrize("seed,props", [(71, 1), (72, 3)])
def test_incremental_windows_member_decisions_and_learns_c5(seed, props):
    """C5-shaped member traces beyond fixture size (contended too) in 7 windows with
    MPX_FLAG_DECISIONS: decisions and learns == one engine over the whole trace."""
    t = mpx.generate_trace(mpx.GEN_MEMBER, num_nodes=8, num_instances=1 << 14, seed=seed, batch=64,
                           drop_rate=300, dup_rate=300, max_delay=64, noop_permille=15, proposers=props)
    with mpx.Engine.for_trace(t) as e:
        e.run()
        want, want_l = e.decisions(), e.learns()
    hd, epochs, streams = _node_streams(t)
    n, m = hd["num_nodes"], hd["num_instances"]
    with mpx.Engine(n, 0, m, semantics=hd["semantics"], epochs=epochs,
                    flags=mpx.FLAG_INCREMENTAL | mpx.FLAG_DECISIONS) as e:
        prev = [0] * n
        for f in [k / 7 for k in range(1, 7)] + [1.0]:
            cut = [len(s) if f >= 1.0 else int(len(s) * f) for s in streams]
            for node, st in enumerate(streams):
                if cut[node] > prev[node]:
                    e.submit(node, st[prev[node]:cut[node]])
            e.run()
            prev = cut
        assert e.decisions() == want
        assert e.learns() == want_l


def test_incremental_window_cost_is_per_window_member():
    """C5 at 2^20 instances (acceptor universe 8, 15 epochs, loss / dup) in 16 equal windows:
    each window's host + device time stays within 2x of the second window's as the history
    grows — O(window), not O(history) — and the windows together give the whole run's digests."""
    t = mpx.generate_trace(mpx.GEN_MEMBER, num_instances=1 << 20, copy=False, num_nodes=8, seed=0, batch=256,
                           drop_rate=100, dup_rate=100, max_delay=64, noop_permille=15)
    with mpx.Engine.for_trace(t) as e:
        st = e.run()
        want = (st["state_digest"], st["chosen_digest"])
        want_c = {k: st[k] for k in COUNTERS}
    times = []
    _sends, tot, obs = _windows(bytes(t), [k / 16 for k in range(1, 16)], times)
    assert obs["digests"] == want and tot == want_c
    print("window times (s):", ["%.3f" % x for x in times])
    assert max(times[2:]) <= 2.0 * times[1], times


def test_incremental_window_range_error_keeps_state():
    """A window the engine cannot encode (MPX_E_RANGE: a member node past 254 E_EPOCH markers,
    the device incarnation counter) is refused before it touches the carry: the state read back
    is the earlier windows', and the same records are refused again."""
    import struct
    t = mpx.generate_trace(mpx.GEN_MEMBER, num_nodes=4, num_instances=4096, seed=7, batch=64,
                           drop_rate=100, dup_rate=100, max_delay=32)
    hd, epochs, streams = _node_streams(t)
    n, m = hd["num_nodes"], hd["num_instances"]
    with mpx.Engine(n, 0, m, semantics=hd["semantics"], epochs=epochs, flags=mpx.FLAG_INCREMENTAL) as e:
        for node, s in enumerate(streams):
            e.submit(node, s[:len(s) // 2])
        e.run()
        before = _observe(e, n, m)
        e.submit(0, [struct.pack("<II", 18, 0)] * 300)      # E_EPOCH{epoch 0} x 300
        for _ in range(2):
            with pytest.raises(mpx.MpxError) as ex:
                e.run()
            assert ex.value.rc == -5                         # MPX_E_RANGE
        assert _observe(e, n, m) == before


def test_incremental_window_cost_is_per_window():
    """C3 at 2^20 instances in 16 equal windows: each window's host + device time (submit +
    run) stays within 2x of the second window's as the history grows — O(window), not
    O(history) — and the windows together give the whole run's digests."""
    t = mpx.generate_trace(mpx.GEN_FAULTY, num_instances=1 << 20, copy=False, num_nodes=7, seed=0, batch=256,
                           proposers=3, drop_rate=500, dup_rate=1000, max_delay=500)
    hd = mpx.trace_header(t)
    with mpx.Engine.for_trace(t) as e:
        st = e.run()
        want = (st["state_digest"], st["chosen_digest"])
        want_c = {k: st[k] for k in COUNTERS}
    times = []
    _sends, tot, obs = _windows(bytes(t), [k / 16 for k in range(1, 16)], times)
    assert obs["digests"] == want and tot == want_c
    print("window times (s):", ["%.3f" % x for x in times])
    assert max(times[2:]) <= 2.0 * times[1], times
    assert hd["num_instances"] >= 1 << 20


# ---- commit reliability (multi/paxos.cpp:1184-1197,1416-1421,1625-1641) ----
COMMITS = json.load(open(os.path.join(GOLD, "commits.json")))


# ---- member learn reliability (member/paxos.cpp:1345-1381,1472-1549) ----
@pytest.mark.parametrize("name", sorted(LEARNS))
def test_engine_learns_match_reference(name):
    """Every LearningValues the member proposers create (accept quorums from k_votes,
    promise quorums from k_prop_*, LearnersChanged at the epoch markers) and what k_learns
    makes of their LEARN_REPLYs and AcceptorsChanged calls == the reference's own
    bookkeeping (fixture, oracle/ref_member_driver.cpp), after run and after a timed step."""
    trace, want = _read(name, ".mpxt"), _read(name, ".mpxl")
    with mpx.Engine.for_trace(trace) as e:
        e.run()
        assert e.learns() == want
        e.step()
        e.sync()
        assert e.learns() == want


@pytest.mark.parametrize("seed,m,batch", [(7, 1 << 16, 64), (8, 50000, 256)])
def test_engine_learns_match_model_c5(seed, m, batch):
    """C5-shaped traces beyond fixture size: the engine's learn bookkeeping == the Python
    restatement (oracle/learns_model.py, pinned to the reference's fixtures on CPU) fed by
    the C oracle's promise quorums and chosen batches."""
    from oracles import oracle_run
    import learns_model
    import mpxl
    t = mpx.generate_trace(mpx.GEN_MEMBER, num_nodes=8, num_instances=m, seed=seed, batch=batch,
                           drop_rate=300, dup_rate=300, max_delay=64, noop_permille=15)
    want = learns_model.learns(t, oracle_run(t)[0])
    assert sum(len(x) for x in mpxl.parse(want)) > 100
    with mpx.Engine.for_trace(t) as e:
        e.run()
        assert e.learns() == want


@pytest.mark.parametrize("seed,m,batch", [(9, 1 << 16, 64), (10, 40000, 200)])
def test_engine_member_decisions_match_model_c5(seed, m, batch):
    """Member phase-2 decisions beyond fixture size: the engine == the Python restatement
    (oracle/member_decisions_model.py, pinned to the reference's fixtures on CPU) fed by the
    C oracle's promise quorums and merged maps."""
    from oracles import oracle_run
    import member_decisions_model
    import mpxd
    t = mpx.generate_trace(mpx.GEN_MEMBER, num_nodes=8, num_instances=m, seed=seed, batch=batch,
                           drop_rate=300, dup_rate=300, max_delay=64, noop_permille=15)
    want = member_decisions_model.decisions(t, oracle_run(t)[0])
    assert sum(len(x) for x in mpxd.parse(want)) >= 15
    with mpx.Engine.for_trace(t) as e:
        e.run()
        assert e.decisions() == want


def test_learns_refused_off_member_and_on_shards():
    """mpx_read_learns is member bookkeeping of an engine that kept every record: multi
    semantics and a shard that left records out for another shard are refused; a shard at
    instance 0 that kept every record (its LEARNs / batches meet it) answers as the whole."""
    with mpx.Engine.for_trace(_read("hm_clean3", ".mpxt")) as e:
        e.run()
        with pytest.raises(mpx.MpxError):
            e.learns()
    trace = _read("mm_clean3", ".mpxt")
    hd = mpx.trace_header(trace)
    with mpx.Engine(hd["num_nodes"], 0, 8, semantics=hd["semantics"]) as e:
        e.submit_trace(trace)
        e.run()
        assert e.learns() == _read("mm_clean3", ".mpxl")
    with mpx.Engine(hd["num_nodes"], 3, 64, semantics=hd["semantics"]) as e:
        e.submit_trace(trace)
        e.run()
        with pytest.raises(mpx.MpxError):
            e.learns()


@pytest.mark.parametrize("name", sorted(COMMITS))
def test_engine_commits_match_reference(name):
    """Every CommittingValues the device finds (accept quorums from k_votes,
    promise quorums with committed values from k_decide) and what k_commits makes
    of its COMMIT_REPLYs == the reference's own bookkeeping (fixture)."""
    trace, want = _read(name, ".mpxt"), _read(name, ".mpxc")
    with mpx.Engine.for_trace(trace) as e:
        e.run()
        assert e.commits() == want
        e.step()
        e.sync()
        assert e.commits() == want


@pytest.mark.parametrize("seed,m", [(91, 1 << 12), (92, 1 << 14)])
def test_engine_commits_match_oracle_c3(seed, m):
    from oracles import oracle_commits
    import mpxc
    t = mpx.generate_trace(mpx.GEN_FAULTY, num_nodes=7, num_instances=m, seed=seed, batch=64, proposers=3,
                           drop_rate=500, dup_rate=1000, max_delay=500)
    want = oracle_commits(t)
    with mpx.Engine.for_trace(t) as e:
        e.run()
        got = e.commits()
    p = mpxc.parse(want)
    assert sum(1 for x in p for r in x if r[4] != mpxc.OPEN) > 0
    assert got == want


def _sharded_commits(trace, shards, align=256):
    """The sharded protocol of include/mpx.h: points per shard -> union -> OnCommitReply
    on the shard at instance 0."""
    from mpx import dist as mdist
    hd = mpx.trace_header(trace)
    m = max(hd["num_instances"], 1)
    engines = []
    try:
        for r in range(shards):
            sb, se = mdist.shard_bounds(m, shards, r, align=align)
            e = mpx.Engine(hd["num_nodes"], sb, se)
            engines.append(e)
            e.submit_trace(trace)
            e.run()
        pts = mpx.commit_points_combine([e.commit_points() for e in engines])
        return engines[0].commits_at(pts)
    finally:
        for e in engines:
            e.close()


@pytest.mark.parametrize("shards", [2, 3])
@pytest.mark.parametrize("name", ["fuzz_big_1", "fuzz_big_2", "c3_faulty_0", "demo_s1", "fuzz_007"])
def test_sharded_commits_match_reference(name, shards):
    """Commit reliability over instance shards (each shard's creation points: the batches
    it kept, the promise quorums where the node held a committed instance of it; their
    union; OnCommitReply on the shard holding instance 0) == the reference's own
    committing_values_ bookkeeping (fixture)."""
    if name not in COMMITS:
        pytest.skip("no commits fixture " + name)
    trace, want = _read(name, ".mpxt"), _read(name, ".mpxc")
    assert _sharded_commits(trace, shards, align=1) == want


@pytest.mark.parametrize("shards", [2, 4])
def test_sharded_commits_match_oracle_c3(shards):
    from oracles import oracle_commits
    t = mpx.generate_trace(mpx.GEN_FAULTY, num_nodes=7, num_instances=1 << 13, seed=93, batch=64, proposers=3,
                           drop_rate=500, dup_rate=1000, max_delay=500)
    want = oracle_commits(t)
    with mpx.Engine.for_trace(t) as e:
        e.run()
        assert e.commit_points() == mpx.commit_points_combine([e.commit_points()])
        assert e.commits_at(e.commit_points()) == want
    assert _sharded_commits(t, shards) == want


def test_engine_commits_clean_device_trace():
    """Device-generated clean trace: every batch is chosen and every COMMIT is
    answered by all N learners, so every commit retires with the full mask."""
    import mpxc
    N, M = 5, 1 << 14
    with mpx.Engine(N, 0, M) as e:
        e.load_clean_device(num_instances=M, batch=256)
        e.run()
        p = mpxc.parse(e.commits())
    assert len(p[0]) == M // 256 and all(len(x) == 0 for x in p[1:])
    assert all(r[2] == 0 and r[4] != mpxc.OPEN and r[5] == (1 << N) - 1 for r in p[0])
    with mpx.Engine(N, 0, M // 2) as e:     # a device-generated shard keeps only its own batches'
        e.load_clean_device(num_instances=M, batch=256)   # messages: no stream positions to merge on
        e.run()
        with pytest.raises(mpx.MpxError):
            e.commits()
        with pytest.raises(mpx.MpxError):
            e.commit_points()
    with mpx.Engine(N, 0, M) as e:
        e.load_clean_device(num_instances=M, batch=256)
        e.run()
        assert e.commits_at(e.commit_points()) == e.commits()


# ---- closed loop (the engine's decisions drive the next messages) ----
def test_closed_loop_contending_proposers_match_reference():
    """mpx.loop.ClosedLoop: node 0 prepares with four client values queued, its phase-2 batch
    (the engine's decision) reaches only 2 of 5 acceptors; node 1 prepares higher with two
    values of its own — its quorum adopts node 0's half-accepted values (the engine's merge)
    and queues its own after them; the batch is chosen and committed.  Every node executes
    a0..a3, b0, b1 in order; the recorded streams, replayed through the reference's own
    handlers, give the engine's result and the reference's decisions equal the engine's."""
    from mpx.loop import ClosedLoop
    import mpxd
    L = ClosedLoop(5, 64)
    try:
        L.prepare(0, range(5))
        for i in range(4):
            L.propose(0, "a%d" % i)
        L.run(); L.run()                               # promises -> node 0's quorum
        assert L.accept_decided(0, [0, 1]) == 1        # reaches 2 of 5: no quorum
        L.run(); L.run()
        assert not L.commit_chosen(0, range(5))
        L.prepare(1, range(5))
        L.propose(1, "b0"); L.propose(1, "b1")
        L.run(); L.run()                               # node 1's quorum merges node 0's values
        d1 = mpxd.parse(L.engine.decisions())[1][-1][1]
        assert [iid for iid, _ in d1] == list(range(6))
        assert [h >> 48 for _, h in d1] == [0, 0, 0, 0, 1, 1]
        assert L.accept_decided(1, range(5)) == 1
        L.run(); L.run()
        assert L.commit_chosen(1, range(5)) == [1]
        L.run(); L.run()
        want = [b"a0", b"a1", b"a2", b"a3", b"b0", b"b1"]
        for n in range(5):
            fr, handles = L.engine.read_executed(n)
            assert fr == 6 and [L.payload[(h >> 48, h & ((1 << 47) - 1))] for h in handles] == want
        trace = L.trace()
        from oracles import oracle_run, ref_available
        assert L.engine.dump() == oracle_run(trace)[0]
        if ref_available():
            from oracles import ref_decisions, ref_run
            assert L.engine.dump() == ref_run(trace)[0]
            assert L.engine.decisions() == ref_decisions(trace)
    finally:
        L.close()


@pytest.mark.parametrize("seed", [3, 5, 7])
def test_closed_loop_random_schedule_matches_oracle(seed):
    """Random closed-loop schedules: three proposers prepare, propose client values, send the
    engine's decided batches and commit what the engine found chosen, each to a random subset
    of the five acceptors.  The streams replayed through the C oracle give the engine's result,
    decisions and commits; the executed streams are prefixes of one another (safety); with the
    reference built, its own handlers agree too (these seeds: no ASSERT case, checked on CPU)."""
    import random
    from mpx.loop import ClosedLoop
    from oracles import oracle_commits, oracle_decisions, oracle_run, ref_available
    rng = random.Random(seed)
    L = ClosedLoop(5, 256)
    try:
        vals = 0
        for _ in range(40):
            p = rng.randrange(3)
            to = sorted(rng.sample(range(5), rng.randint(2, 5)))
            op = rng.random()
            if op < 0.2:
                L.prepare(p, to)
                for _ in range(rng.randint(0, 3)):
                    L.propose(p, "v%d" % vals)
                    vals += 1
            elif op < 0.65 and L.engine is not None:
                L.accept_decided(p, to)
            elif L.engine is not None:
                L.commit_chosen(p, to)
            L.run(); L.run()
        trace = L.trace()
        want, _st, viol = oracle_run(trace)
        assert L.engine.dump() == want and viol[0] == 0
        assert L.engine.decisions() == oracle_decisions(trace)
        assert L.engine.commits() == oracle_commits(trace)
        ex = [L.engine.read_executed(n)[1] for n in range(5)]
        longest = max(ex, key=len)
        assert all(e == longest[:len(e)] for e in ex)
        assert len(L.batches) >= 2
        if ref_available():
            from oracles import ref_decisions, ref_run
            assert L.engine.dump() == ref_run(trace)[0]
            assert L.engine.decisions() == ref_decisions(trace)
    finally:
        L.close()


@pytest.mark.timeout(300)
def test_member_learns_and_decisions_at_2_18_match_restatements():
    """The member proposer bookkeeping at 2^18 instances (C5's schedule and fault rates, 8 nodes,
    15 epochs): the engine's learns and phase-2 decisions == the oracle/ restatements (pinned to
    the reference's fixtures) over the C oracle's quorums — about 2 M decided entries."""
    from oracles import oracle_run
    import learns_model
    import member_decisions_model
    t = mpx.generate_trace(mpx.GEN_MEMBER, num_nodes=8, num_instances=1 << 18, seed=0, batch=256,
                           drop_rate=100, dup_rate=100, max_delay=64, noop_permille=15)
    r = oracle_run(t)[0]
    with mpx.Engine.for_trace(t) as e:
        e.run()
        assert e.dump() == r
        assert e.learns() == learns_model.learns(t, r)
        assert e.decisions() == member_decisions_model.decisions(t, r)


def test_closed_loop_incremental_equals_replay():
    """The closed loop on one incremental engine (MPX_FLAG_INCREMENTAL | MPX_FLAG_DECISIONS:
    each step submits only the new records) makes the same moves as the replaying loop: the
    same streams and decisions, and the streams replayed whole give the C oracle's result."""
    import random
    from mpx.loop import ClosedLoop
    from oracles import oracle_decisions, oracle_run

    def play(incremental):
        rng = random.Random(5)
        L = ClosedLoop(5, 256, incremental=incremental)
        vals = 0
        for _ in range(40):
            p = rng.randrange(3)
            to = sorted(rng.sample(range(5), rng.randint(2, 5)))
            op = rng.random()
            if op < 0.2:
                L.prepare(p, to)
                for _ in range(rng.randint(0, 3)):
                    L.propose(p, "v%d" % vals)
                    vals += 1
            elif op < 0.65 and L.engine is not None:
                L.accept_decided(p, to)
            elif L.engine is not None:
                L.commit_chosen(p, to)
            L.run(); L.run()
        out = (L.trace(), L.engine.decisions(), len(L.batches), len(L.committed))
        L.close()
        return out

    a, b = play(False), play(True)
    assert a == b
    assert a[2] >= 2
    assert oracle_decisions(a[0]) == b[1]
    with mpx.Engine.for_trace(a[0]) as e:
        e.run()
        assert e.dump() == oracle_run(a[0])[0]


def _loop_schedule(L, seed, steps=40):
    import random
    rng = random.Random(seed)
    vals = 0
    started = False
    for _ in range(steps):
        p = rng.randrange(3)
        to = sorted(rng.sample(range(5), rng.randint(2, 5)))
        op = rng.random()
        if op < 0.2:
            L.prepare(p, to)
            for _ in range(rng.randint(0, 3)):
                L.propose(p, "v%d" % vals)
                vals += 1
        elif op < 0.65 and started:
            L.accept_decided(p, to)
        elif started:
            L.commit_chosen(p, to)
        L.run(); L.run()
        started = True


@pytest.mark.parametrize("seed", [5, 11])
def test_native_loop_equals_python_loop(seed):
    """The closed loop inside libmpx (mpx_loop_*) makes the Python driver's moves
    (mpx.loop.ClosedLoop on one incremental engine) for the same schedule: identical recorded streams
    and decisions; replayed through the C oracle and, built, the reference's own handlers, the
    streams give the native loop's engine result and decisions."""
    from mpx.loop import ClosedLoop, NativeLoop
    from oracles import oracle_decisions, oracle_run, ref_available
    py, nat = ClosedLoop(5, 256, incremental=True), NativeLoop(5, 256)
    try:
        _loop_schedule(py, seed)
        _loop_schedule(nat, seed)
        t = nat.trace()
        assert t == py.trace()
        assert nat.engine.decisions() == py.engine.decisions() == oracle_decisions(t)
        assert nat.stats()["batches"] == len(py.batches) >= 1
        with mpx.Engine.for_trace(t) as e:
            e.run()
            assert e.dump() == oracle_run(t)[0]
            if ref_available():
                from oracles import ref_decisions, ref_run
                assert e.dump() == ref_run(t)[0] and e.decisions() == ref_decisions(t)
    finally:
        py.close()
        nat.close()


def test_native_loop_leader_rounds_match_reference():
    """mpx_loop_leader_rounds: a leader's rounds (StartPrepare with client values queued, the engine's
    decided batch accepted, chosen and committed to every node) entirely in libmpx; every value is
    chosen and executed in order on every node, and the recorded streams replayed through the
    reference's own handlers give the engine's result and decisions."""
    from mpx.loop import NativeLoop
    from oracles import oracle_run, ref_available
    L = NativeLoop(5, 4096)
    try:
        L.leader_rounds(0, range(5), 4, 300)
        st = L.stats()
        assert st["committed_instances"] == 1200 and st["windows"] == 20
        chosen = L.engine.read_chosen(0, 1200)
        assert all(c >> 63 for c in chosen)
        ex = [L.engine.read_executed(n)[1] for n in range(5)]
        assert all(len(x) == 1200 and x == ex[0] for x in ex)
        t = L.trace()
        with mpx.Engine.for_trace(t) as e:
            e.run()
            assert e.dump() == oracle_run(t)[0]
            if ref_available():
                from oracles import ref_decisions, ref_run
                assert e.dump() == ref_run(t)[0] and e.decisions() == ref_decisions(t)
    finally:
        L.close()


# ---- membership learned at run time (MPX_FLAG_LEARN_EPOCHS; member/paxos.cpp:1040-1073,1864-1964) ----
MEMBER_GOLDENS = sorted(k for k in INDEX if k.startswith(("c5_", "mm_")))


def _strip_markers(streams):
    """What NetWork::OnReceive hands a live node: the trace's records without the E_EPOCH markers."""
    return [[r for r in s if r[:4] != b"\x12\x00\x00\x00"] for s in streams]


@pytest.mark.parametrize("name", MEMBER_GOLDENS)
def test_learned_epochs_match_reference(name):
    """Every member golden on an engine created with the genesis epoch only: the engine applies the
    membership Values its nodes' Learners apply (ingest EpochLearn) and places its own E_EPOCH
    records — the result is the reference's byte for byte (its roles come from the reference's
    own ChangeMemberships), the learned epoch table is the trace's, and the decisions and learns
    are the reference's fixtures."""
    trace, want = _read(name, ".mpxt"), _read(name, ".mpxr")
    table = mpx.trace_epochs(trace)
    with mpx.Engine.for_trace(trace, flags=mpx.FLAG_LEARN_EPOCHS) as e:
        e.run()
        assert e.dump() == want
        got = e.epochs()
        assert got == table[:len(got)] and len(got) > 1
        if name in DECISIONS:
            assert e.decisions() == _read(name, ".mpxd")
        if name in LEARNS:
            assert e.learns() == _read(name, ".mpxl")


@pytest.mark.parametrize("name", ["c5_member_2", "c5_member_3", "c5_contended_2", "mm_learners", "mm_acceptor_reset"])
def test_learned_epochs_in_windows_marker_free(name):
    """A live member host: every node's stream WITHOUT its E_EPOCH markers, in 4 and 7 incremental
    windows, on an engine that knows only the genesis epoch (MPX_FLAG_LEARN_EPOCHS): the epoch
    table grows window by window as the nodes apply membership Values, and the windows give the
    whole run's replies, counters, state, executed streams and chosen log, and the reference's
    decisions and learns (MPXD / MPXL fixtures)."""
    trace = _read(name, ".mpxt")
    want = _whole(trace)
    hd, epochs, streams = _node_streams(trace)
    live = _strip_markers(streams)
    n, m = hd["num_nodes"], max(hd["num_instances"], 1)
    for W in (4, 7):
        sends = [[] for _ in range(n)]
        tot = {k: 0 for k in COUNTERS}
        sizes = []
        with mpx.Engine(n, 0, m, semantics=mpx.SEM_MEMBER, epochs=epochs[:1],
                        flags=mpx.FLAG_INCREMENTAL | mpx.FLAG_DECISIONS | mpx.FLAG_LEARN_EPOCHS) as e:
            prev = [0] * n
            for w in range(1, W + 1):
                cut = [len(s) * w // W for s in live]
                for node, s in enumerate(live):
                    if cut[node] > prev[node]:
                        e.submit(node, s[prev[node]:cut[node]])
                st = e.run()
                prev = cut
                for k in COUNTERS:
                    tot[k] += st[k]
                for src, dst, b in e.drain_sends():
                    sends[src].append((dst, b))
                sizes.append(len(e.epochs()))
            assert e.epochs() == epochs[:sizes[-1]] and sizes[-1] > 1
            assert sizes == sorted(sizes), sizes
            if name.startswith("c5_"):
                assert len(set(sizes)) >= 3, sizes                  # the table grows window by window
            assert sends == want[0] and tot == want[1]
            assert _observe(e, n, m) == want[2]
            if name in DECISIONS:
                assert e.decisions() == _read(name, ".mpxd")
            if name in LEARNS:
                assert e.learns() == _read(name, ".mpxl")


# ---- the member host's Callback calls (member/paxos.h:142-164) ----
CALLBACKS = json.load(open(os.path.join(GOLD, "callbacks.json")))


def _cb_of(vb):
    """The cb string of a member Value_m (FillValue, member/paxos.cpp:330-363); b"" for a noop."""
    import struct
    if vb[12]:
        return b""
    mem, n = vb[13] != 0, struct.unpack_from("<I", vb, 14)[0]
    p = 18 + (8 * n if mem else n)
    cl = struct.unpack_from("<I", vb, p)[0]
    return bytes(vb[p + 4:p + 4 + cl])


def _engine_callbacks(e, streams):
    """Every Callback call a member host makes from the engine's readbacks, per node sorted
    (record, kind, cb): Accepted for a kind-0 learn's values at its creation, Applied for a
    kind-1 / kind-2 learn's values at its applied record (MPXL + MPXV), Unproposable for the
    P_PROPOSE records MPXV names (the cb of the host's own record)."""
    import mpxl
    import mpxv
    learns, vals = mpxl.parse(e.learns()), mpxv.parse(e.learn_values())
    cache = {}

    def cb(h):
        if h not in cache:
            cache[h] = _cb_of(e.value_bytes(h))
        return cache[h]
    out = []
    for n, (rows, (vs, unprop)) in enumerate(zip(learns, vals)):
        assert len(rows) == len(vs)
        calls = []
        for row, v in zip(rows, vs):
            kind, created, applied = row[2], row[1], row[4]
            if kind == 0:
                calls += [(created, 0, cb(h)) for _i, h in v]
            elif applied != mpxl.NONE:
                calls += [(applied, 1, cb(h)) for _i, h in v]
        calls += [(k, 2, _cb_of(streams[n][k][8:])) for k in unprop]
        out.append(sorted(calls))
    return out


def _reference_callbacks(name):
    import mpxb
    return [sorted(x) for x in mpxb.parse(_read(name, ".mpxb"))]


@pytest.mark.parametrize("name", sorted(CALLBACKS))
def test_member_callbacks_match_reference(name):
    """Every paxos::Callback call the reference's nodes made (Accepted at an accept quorum,
    member/paxos.cpp:1327-1332; Applied for the values of a learn created at a promise quorum or a
    learner change once an acceptor quorum learned it, :1360-1368,1523-1526 — the whole learned map
    for those; Unproposable, :784-787), by record and cb string, equals what the engine's learns
    and their Values (mpx_read_learns + mpx_read_learn_values) make a host call: whole run, and
    marker-free in 4 incremental windows on a genesis-only engine (MPX_FLAG_LEARN_EPOCHS)."""
    trace = _read(name, ".mpxt")
    want = _reference_callbacks(name)
    _hd, epochs, streams = _node_streams(trace)
    with mpx.Engine.for_trace(trace) as e:
        e.run()
        assert _engine_callbacks(e, streams) == want
    live = _strip_markers(streams)
    hd = mpx.trace_header(trace)
    n, m = hd["num_nodes"], max(hd["num_instances"], 1)
    with mpx.Engine(n, 0, m, semantics=mpx.SEM_MEMBER, epochs=epochs[:1],
                    flags=mpx.FLAG_INCREMENTAL | mpx.FLAG_DECISIONS | mpx.FLAG_LEARN_EPOCHS) as e:
        prev = [0] * n
        for w in range(1, 5):
            cut = [len(s) * w // 4 for s in live]
            for node, s in enumerate(live):
                if cut[node] > prev[node]:
                    e.submit(node, s[prev[node]:cut[node]])
            e.run()
            prev = cut
        assert _engine_callbacks(e, streams) == want


def test_member_unproposable_reported():
    """Node::Propose on a node without a Proposer calls Callback::Unproposable (NodeImpl::Loop,
    member/paxos.cpp:784-787): a P_PROPOSE at node 1 (no Proposer in the genesis epoch) is named by
    MPXV, one at node 0 (the genesis Proposer) is not — as the reference's own nodes do (MPXB)."""
    from mpxwire import container, m_p_propose, mvalue
    import mpxb
    import mpxv
    from oracles import ref_available, ref_callbacks
    streams = [[m_p_propose(mvalue(0, 1, "a", cb="c0"))], [m_p_propose(mvalue(1, 1, "b", cb="c1"))]]
    trace = container(streams, 16, semantics=1, epochs=[(0, 1, 1)])
    with mpx.Engine.for_trace(trace) as e:
        e.run()
        v = mpxv.parse(e.learn_values())
    assert [x[1] for x in v] == [[], [0]]
    if ref_available():
        assert [[(k, kind, cb) for k, kind, cb in x] for x in mpxb.parse(ref_callbacks(trace))] == [[], [(0, 2, b"c1")]]


def test_learned_epochs_refused_change_poisons_engine():
    """A membership Value the reference ASSERTs on (AddAcceptor of a node that already is one,
    NodeImpl::ChangeMemberships, member/paxos.cpp:1864-1964) fails the submit with MPX_E_STATE, and
    the engine — whose Learner frontier and view may have moved past that record — refuses every
    later call: no run or read on half-learned epochs; the epoch table is unchanged."""
    from handmade_member import B0, add_acceptor
    from mpxwire import m_learn, mvalue
    ok = [(0, B0, mvalue(0, 1, cb="m1", changes=add_acceptor(1)))]
    twice = [(1, B0, mvalue(0, 2, cb="m2", changes=add_acceptor(1)))]    # node 1 is an acceptor already
    with mpx.Engine(2, 0, 64, semantics=mpx.SEM_MEMBER, epochs=[(0, 1, 1)], flags=mpx.FLAG_LEARN_EPOCHS) as e:
        e.submit(0, [m_learn(0, 1, ok)])
        assert len(e.epochs()) == 2
        with pytest.raises(mpx.MpxError) as ex:
            e.submit(0, [m_learn(0, 2, twice)])
        assert ex.value.rc == -6                            # MPX_E_STATE
        assert len(e.epochs()) == 2
        for call in (e.run, lambda: e.submit(1, [m_learn(0, 1, ok)])):
            with pytest.raises(mpx.MpxError) as ex:
                call()
            assert ex.value.rc == -6


@pytest.mark.parametrize("seed,props", [(81, 1), (82, 3)])
def test_learned_epochs_c5_generated(seed, props):
    """C5-shaped traces beyond fixture size (2^16 instances, contended too): the marker-free streams
    on a genesis-only engine == the whole run with the generator's markers (state, digests,
    decisions, learns), and every one of the schedule's 15 epochs is learned."""
    t = mpx.generate_trace(mpx.GEN_MEMBER, num_nodes=8, num_instances=1 << 16, seed=seed, batch=128,
                           drop_rate=200, dup_rate=200, max_delay=64, noop_permille=15, proposers=props)
    with mpx.Engine.for_trace(t) as e:
        st = e.run()
        want = ({k: st[k] for k in COUNTERS}, e.state_digest(), e.decisions(), e.learns())
    hd, epochs, streams = _node_streams(t)
    live = _strip_markers(streams)
    with mpx.Engine(8, 0, hd["num_instances"], semantics=mpx.SEM_MEMBER, epochs=epochs[:1],
                    flags=mpx.FLAG_LEARN_EPOCHS) as e:
        for node, s in enumerate(live):
            e.submit(node, s)
        st = e.run()
        assert ({k: st[k] for k in COUNTERS}, e.state_digest(), e.decisions(), e.learns()) == want
        assert e.epochs() == epochs and len(epochs) == 15
