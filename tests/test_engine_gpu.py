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


@pytest.mark.parametrize("name", sorted(INDEX))
def test_engine_matches_reference_golden(name):
    trace, want = _read(name, ".mpxt"), _read(name, ".mpxr")
    with mpx.Engine.for_trace(trace) as e:
        st = e.run()
        got = e.dump()
    assert got == want, mpxr.diff(got, want)
    meta = INDEX[name]
    assert (st["chosen"], st["promise_entries"], st["accept_apps"], st["commit_apps"]) == \
        (meta["C"], meta["P"], meta["A"], meta["L"])


@pytest.mark.parametrize("n,m,b", [(5, 4096, 256), (3, 1000, 100), (7, 5000, 37), (1, 10, 256), (64, 300, 256)])
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


def test_engine_c2_full_size_digests():
    """C2: 2^20 instances x 5 acceptors, clean, batch 256 — counters and
    order-independent digests equal the CPU oracle's."""
    n, m = 5, 1 << 20
    t = mpx.generate_trace(mpx.GEN_CLEAN, num_nodes=n, num_instances=m, batch=256)
    _, ostats, _ = oracle_run(t)
    with mpx.Engine.for_trace(t) as e:
        st = e.run()
    assert [st["chosen"], st["promise_entries"], st["accept_apps"], st["commit_apps"], st["violations"],
            st["chosen_digest"], st["state_digest"], st["scalar_digest"]] == ostats
    assert st["chosen"] == m and st["bytes_alg"] == 40 * n * m


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


@pytest.mark.parametrize("n,m", [(5, 4096), (9, 256 * 37), (2, 256)])
def test_device_generator_matches_host(n, m):
    """The HBM-materialised clean trace (mpx_load_clean_device) gives the same
    result bytes as the host trace through mpx_submit, and the oracle's."""
    t = mpx.generate_trace(mpx.GEN_CLEAN, num_nodes=n, num_instances=m, batch=256)
    want, ostats, _ = oracle_run(t)
    with mpx.Engine(n, 0, m) as e:
        e.load_clean_device(num_instances=m)
        st = e.run()
        got = e.dump()
    assert got == want, mpxr.diff(got, want)
    assert [st["chosen"], st["promise_entries"], st["accept_apps"], st["commit_apps"], st["violations"],
            st["chosen_digest"], st["state_digest"], st["scalar_digest"]] == ostats


@pytest.mark.parametrize("shards", [2, 3, 8])
def test_sharded_device_generator_sums_to_whole(shards):
    """Instance sharding: per-shard counters and digests add
    up to the single-engine run; per-acceptor scalars agree on every shard."""
    n, m = 9, 256 * 64
    with mpx.Engine(n, 0, m) as e:
        e.load_clean_device(num_instances=m)
        whole = e.run()
    per = m // shards // 256 * 256
    bounds = [(i * per, m if i == shards - 1 else (i + 1) * per) for i in range(shards)]
    tot = {k: 0 for k in ("chosen", "accept_apps", "commit_apps", "chosen_digest", "state_digest")}
    for sb, se in bounds:
        with mpx.Engine(n, sb, se) as e:
            e.load_clean_device(num_instances=m)
            st = e.run()
            assert st["scalar_digest"] == whole["scalar_digest"]
            for k in tot:
                tot[k] = (tot[k] + st[k]) % (1 << 64)
            ch = e.read_chosen(sb, se - sb)
            assert ch == [mpx.PRESENT | (i + 1) for i in range(sb, se)]
    for k in tot:
        assert tot[k] == whole[k] % (1 << 64), k


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
    assert got == want, mpxr.diff(got, want)
    assert [st["chosen"], st["promise_entries"], st["accept_apps"], st["commit_apps"], st["violations"],
            st["chosen_digest"], st["state_digest"], st["scalar_digest"]] == ostats
    assert st["promise_entries"] > 0 and st["violations"] == 0


def test_rccl_single_rank_allgather():
    """The RCCL path of a step (communicator + summary all-gather on the engine stream), one rank."""
    n, m = 9, 256 * 64
    with mpx.Engine(n, 0, m) as e:
        e.comm_init(mpx.Engine.comm_unique_id(), 0, 1)
        e.load_clean_device(num_instances=m)
        e.step()
        e.sync()
        st = e.stats()
        summ = e.allgather_summary(1)
    from mpx import dist as mdist
    tot = mdist.combine(summ)
    assert tot["chosen"] == m == st["chosen"]
    assert tot["state_digest"] == st["state_digest"]
