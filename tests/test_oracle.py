"""The CPU restatement (oracle/mpx_oracle.c) against the reference.

* every committed golden fixture: oracle(trace) == reference(trace) byte for byte
  (the .mpxr files were written by the reference's own handlers, make_golden.py);
* where oracle/_ref exists (this container): fresh random traces, oracle vs the
  reference driven live;
* the reference's own UNITTEST codec vectors (multi/paxos.cpp:1753-1777).
"""
import json
import os
import struct

import pytest

import mpxr
from fuzztrace import fuzz_trace
from mpxwire import container, value
from oracles import oracle_run, ref_available, ref_run, ref_run_shards

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
INDEX = json.load(open(os.path.join(GOLD, "index.json")))


def _read(name, ext):
    with open(os.path.join(GOLD, name + ext), "rb") as f:
        return f.read()


@pytest.mark.parametrize("name", sorted(INDEX))
def test_oracle_matches_reference_golden(name):
    trace, want = _read(name, ".mpxt"), _read(name, ".mpxr")
    got, stats, viol = oracle_run(trace)
    assert got == want, mpxr.diff(got, want)
    meta = INDEX[name]
    assert stats[:4] == [meta["C"], meta["P"], meta["A"], meta["L"]]


@pytest.mark.ref
@pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("name", sorted(INDEX))
def test_ref_shard_mode_matches_whole(name):
    """The reference's instance-shard mode (oracle/ref_full_size.py: the full-size values in
    tests/golden/full_size.json) sums to the whole-trace result over 1, 3 and 7 unaligned shards:
    each shard's entries cut with the reference's own codec; member shards apply the marker's
    membership step with the reference's own ChangeMemberships (a shard never learns the
    instances below it, so Learner::Apply cannot); proposer-only bookkeeping (Propose, the id sets
    below the shard) differs and stays out of the digests.  Whole == oracle stats here, and the
    oracle == the reference's bytes on this golden (test_oracle_matches_reference_golden)."""
    trace = _read(name, ".mpxt")
    _, want, _ = oracle_run(trace)
    want[4] = 0                                    # (violations: the reference would have crashed)
    for shards in (1, 3, 7):
        assert ref_run_shards(trace, shards) == want, shards


@pytest.mark.ref
@pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("n,m,shards", [(9, 1 << 16, 4), (5, 40000, 3)])
def test_ref_c4_shard_generation_matches_whole_trace_shard(n, m, shards):
    """oracle/ref_full_size.py's C4 entry (the whole 2^27 x 9 trace is ~85 GB): each shard process
    generates only its shard of the clean trace (every record, entries outside the shard left out).
    The reference's shard mode over those bytes must equal its shard mode over the WHOLE trace, shard
    by shard — so the sum over generated shards is the reference's verdict on the whole C4 trace."""
    import ctypes
    from oracles import REF_SO
    f = ctypes.CDLL(REF_SO).mpxref_run_shard
    f.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    whole = _mpx.generate_trace(_mpx.GEN_CLEAN, num_nodes=n, num_instances=m, batch=256)
    per = -(-m // shards)
    per = -(-per // 256) * 256
    for k in range(shards):
        sb, se = k * per, min(m, (k + 1) * per)
        part = _mpx.generate_trace(_mpx.GEN_CLEAN, num_nodes=n, num_instances=m, batch=256, shard_begin=sb,
                                   shard_end=se)
        a, b = (ctypes.c_uint64 * 8)(), (ctypes.c_uint64 * 8)()
        assert f(whole, len(whole), sb, se, a) == 0 and f(part, len(part), sb, se, b) == 0
        assert list(a) == list(b), (sb, se)
        assert a[0] == se - sb


def test_codec_unittest_vectors():
    # multi/paxos.cpp:1753-1777: Value(1,2) encodes to 13 bytes, Value(1,2,"123") to 21
    assert len(value(1, 2, noop=True)) == 13
    assert len(value(1, 2, "123")) == 21
    assert value(1, 2, "123") == struct.pack("<IQ??I", 1, 2, False, False, 3) + b"123"


@pytest.mark.ref
@pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("seed", range(100, 160))
def test_oracle_matches_reference_live(seed):
    trace = fuzz_trace(seed)
    got, stats, _ = oracle_run(trace)
    want, rstats = ref_run(trace)
    assert got == want, mpxr.diff(got, want)
    assert stats[:4] == rstats


def test_oracle_rejects_unknown_type():
    with pytest.raises(RuntimeError):
        oracle_run(container([[struct.pack("<I", 9)]], 1))


# ---- member semantics (member/paxos.cpp) -----------------------------------------
import sys as _sys  # noqa: E402
_sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multi-paxos_amd"))
import mpx as _mpx  # noqa: E402  (host generator only)
from handmade_member import member_violation_traces, Member  # noqa: E402
from mpxwire import e_epoch, m_learn, m_prepare  # noqa: E402


@pytest.mark.ref
@pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("seed", range(200, 216))
def test_member_oracle_matches_reference_live(seed):
    U = 3 + seed % 6
    trace = _mpx.generate_trace(_mpx.GEN_MEMBER, num_nodes=U, num_instances=300 + 37 * seed % 500, seed=seed,
                                batch=1 + seed % 40, drop_rate=(seed % 3) * 700, dup_rate=(seed % 4) * 150,
                                max_delay=32, noop_permille=seed % 30)
    got, stats, viol = oracle_run(trace)
    want, rstats = ref_run(trace)
    assert got == want, mpxr.diff(got, want)
    assert stats[:4] == rstats and stats[4] == 0


def test_member_violations_recorded():
    got, stats, viol = oracle_run(member_violation_traces()["mm_violations"])
    # learned-value mismatch (Proposer::OnLearn :1398), accept of a learned instance
    # with another Value (:1767), PREPARE_REPLY from a non-acceptor (:1163)
    assert stats[4] == 3
    assert viol[:2] == [6, 0]


@pytest.mark.ref
@pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built (needs /root/reference)")
def test_member_reference_checks_epoch_markers():
    # node 1 learns AddAcceptor(1) but the trace omits its E_EPOCH marker: the
    # reference driver refuses the trace (the epoch table would be a lie)
    m = Member(2, 2)
    m.bootstrap([0])
    m.streams[1] += [m_learn(0, 1, m.boot), m_prepare(1, 0, 5 << 16)]
    with pytest.raises(RuntimeError, match="-11"):
        ref_run(m.trace())


def test_member_epoch_gates_roles():
    # a node outside epoch 0's acceptor set ignores PREPARE; after E_EPOCH it answers
    m = Member(2, 2)
    m.streams[1] += [m_prepare(1, 0, 7 << 16), m_learn(0, 1, m.boot), e_epoch(1), m_prepare(1, 0, 7 << 16)]
    got, stats, _ = oracle_run(m.trace())
    res = mpxr.parse(got)
    node1 = res["nodes"][1]
    assert node1["promised"] == 7 << 16
    assert [s[1][:4] for s in node1["sends"]][-1] == struct.pack("<I", 1)


@pytest.mark.parametrize("n,m,sb,se", [(5, 3000, 0, 3000), (9, 256 * 40, 0, 256 * 40), (9, 256 * 40, 256 * 8, 256 * 24),
                                       (3, 777, 0, 777)])
def test_clean_closed_form_matches_oracle(n, m, sb, se):
    """bench.py verifies its full-size run against mpxo_clean_expect: pin that closed form to the oracle's
    replay of the same clean trace (digests restricted to the shard via the state entries)."""
    import ctypes
    import mpxr
    from oracles import ORACLE_SO
    t = _mpx.generate_trace(_mpx.GEN_CLEAN, num_nodes=n, num_instances=m, batch=256)
    res, st, _ = oracle_run(t)
    lib = ctypes.CDLL(ORACLE_SO)
    f = lib.mpxo_clean_expect
    f.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                  ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    a, b = ctypes.c_uint64(), ctypes.c_uint64()
    assert f(n, sb, se, 1 << 16, 3, ctypes.byref(a), ctypes.byref(b)) == 0
    if (sb, se) == (0, m):
        assert (a.value, b.value) == (st[6], st[5])
    # shard: every node's state in [sb, se) is (ballot 1<<16, committed, handle iid+1)
    R = mpxr.parse(res)
    for nd in R["nodes"]:
        assert [s for s in nd["state"] if sb <= s[0] < se] == [(i, 2, 1 << 16, i + 1) for i in range(sb, se)]


# ---- phase-2 decisions at promise quorums (multi/paxos.cpp:1056-1130) ----
DECISIONS = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "decisions.json")))


@pytest.mark.parametrize("name", sorted(n for n in DECISIONS if not n.startswith(("mm_", "c5_"))))
def test_oracle_decisions_match_reference_golden(name):
    """The oracle's restatement of OnPrepareReply's batch == what the reference's
    own code built (fixture written by oracle/ref_multi_driver.cpp)."""
    from oracles import oracle_decisions
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    trace = open(os.path.join(gold, name + ".mpxt"), "rb").read()
    want = open(os.path.join(gold, name + ".mpxd"), "rb").read()
    assert oracle_decisions(trace) == want


@pytest.mark.parametrize("seed", range(12))
def test_oracle_decisions_match_reference_live(seed):
    if not ref_available():
        pytest.skip("reference driver not built (needs /root/reference)")
    from oracles import oracle_decisions, ref_decisions
    t = fuzz_trace(50_000 + seed, n_nodes=5, n_inst=120, n_msgs=400)
    assert oracle_decisions(t) == ref_decisions(t)
    t = _mpx.generate_trace(_mpx.GEN_FAULTY, num_nodes=7, num_instances=400, seed=70 + seed, batch=32, proposers=3,
                            drop_rate=500, dup_rate=1000, max_delay=500)
    assert oracle_decisions(t) == ref_decisions(t)


# ---- commit reliability (multi/paxos.cpp:1184-1197,1416-1421,1625-1641) ----
COMMITS = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "commits.json")))


@pytest.mark.parametrize("name", sorted(COMMITS))
def test_oracle_commits_match_reference_golden(name):
    """The oracle's CommittingValues bookkeeping (creation at accept / promise
    quorums, OnCommitReply retirement, replied_ masks) == the reference's own
    (fixture written by oracle/ref_multi_driver.cpp)."""
    from oracles import oracle_commits
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    trace = open(os.path.join(gold, name + ".mpxt"), "rb").read()
    want = open(os.path.join(gold, name + ".mpxc"), "rb").read()
    assert oracle_commits(trace) == want


def test_commit_fixtures_cover_both_kinds_and_retirement():
    kinds = sum(v["promise_quorum"] for v in COMMITS.values())
    total = sum(v["commits"] for v in COMMITS.values())
    retired = sum(v["retired"] for v in COMMITS.values())
    assert 0 < kinds < total and 0 < retired < total


@pytest.mark.parametrize("seed", range(12))
def test_oracle_commits_match_reference_live(seed):
    if not ref_available():
        pytest.skip("reference driver not built (needs /root/reference)")
    from oracles import oracle_commits, ref_commits
    t = fuzz_trace(60_000 + seed, n_nodes=5, n_inst=120, n_msgs=400)
    assert oracle_commits(t) == ref_commits(t)
    t = _mpx.generate_trace(_mpx.GEN_FAULTY, num_nodes=7, num_instances=400, seed=90 + seed, batch=32, proposers=3,
                            drop_rate=500, dup_rate=1000, max_delay=500)
    assert oracle_commits(t) == ref_commits(t)
