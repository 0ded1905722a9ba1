"""C1 — the reference's own multi/ demo, replayed (BASELINE configs[0]).

tests/golden/demo/*.log.gz are TRACE logs of the reference demo (multi/main.cpp,
run with the shipped debug.conf.sample arguments at --log-level=0, captured by
tests/golden/capture_demo.py).  tests/demotrace.py rebuilds each node's
processing-order stream from the log; the result is the golden demo_*.mpxt, and
demo_*.mpxr is what the reference's handlers (oracle/_ref) produce for it.

Checked here on the CPU, per node, against what the demo itself printed:
  * every acceptor / learner reply it sent (PREPARE_REPLY, REJECT, ACCEPT_REPLY,
    COMMIT_REPLY: multi/paxos.cpp:888-899,1391-1403,1577-1582), bytes and
    destinations, in order;
  * the executed stream (StateMachine::Execute via OnCommit, :1584-1622);
  * the batches chosen by an accept quorum (OnAcceptReply, :1416-1421), in order;
  * the "final committed values" line (:1694-1703) — ballot tag, proposer,
    value id, noop, payload, in instance order — and no accepted-but-uncommitted
    entry left (the ASSERT at :1685);
  * the chosen log == every node's final committed values (main.cpp:567-573).
The same fixtures run through the HIP engine in test_engine_gpu.py (index.json).
"""
import glob
import os

import pytest

import demotrace as D
import mpxr
from oracles import oracle_run

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
LOGS = sorted(glob.glob(os.path.join(GOLD, "demo", "*.log.gz")))
NAMES = [os.path.basename(p)[:-len(".log.gz")] for p in LOGS]


def _load(name):
    text = D.read_log(os.path.join(GOLD, "demo", name + ".log.gz"))
    with open(os.path.join(GOLD, name + ".mpxt"), "rb") as f:
        trace = f.read()
    with open(os.path.join(GOLD, name + ".mpxr"), "rb") as f:
        result = f.read()
    return text, trace, result


def test_demo_logs_present():
    assert len(NAMES) >= 3


@pytest.mark.parametrize("name", NAMES)
def test_demo_log_converts_to_golden_trace(name):
    text, trace, _ = _load(name)
    assert D.to_trace(text) == trace


@pytest.mark.parametrize("name", NAMES)
def test_demo_replay_reproduces_the_log(name):
    text, trace, result = _load(name)
    R = mpxr.parse(result)
    facts = D.log_facts(text)
    batches = {}                      # (node, accept_id) -> values, from the P_BATCH records
    for n, nd in sorted(D.parse_log(text).items()):
        for m in D.node_stream(n, nd, len(facts)):
            if D._u32(m, 0) == 17:
                batches[(n, D._u64(m, 4))] = frozenset(D._entries_multi(m[16:]))
    every_final = None
    for n, f in sorted(facts.items()):
        nd = R["nodes"][n]
        assert nd["sends"] == f["sends"], "node %d replies differ" % n
        assert nd["executed"] == f["executed"], "node %d executed stream differs" % n
        chosen = [batches[(n, aid)] for _, aid in nd["chosen_batches"]]
        assert chosen == [vals for _, vals in f["commits"]], "node %d chosen batches differ" % n
        committed = [(s[2], s[3]) for s in nd["state"] if s[1] == 2]
        assert not [s for s in nd["state"] if s[1] == 1], "node %d has accepted-only entries" % n
        final = [(b, (p << 48) | (int(noop) << 47) | v) for b, p, v, noop, _ in f["final"]]
        assert committed == final, "node %d final committed values differ" % n
        iids = [s[0] for s in nd["state"] if s[1] == 2]
        if every_final is None:
            every_final = [(i, h) for i, (_, h) in zip(iids, committed)]
        assert [(i, h) for i, (_, h) in zip(iids, committed)] == every_final
    assert R["chosen"] == every_final


@pytest.mark.parametrize("name", NAMES)
def test_oracle_replays_demo(name):
    _, trace, result = _load(name)
    got, stats, viol = oracle_run(trace)
    assert got == result, mpxr.diff(got, result)
    assert viol[0] == 0
