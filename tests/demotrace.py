"""C1: turn a captured TRACE log of the reference's multi/ demo into an MPXT trace (test helper).

The demo (multi/main.cpp) runs one server thread and one paxos thread per node.
At --log-level=0 the server thread logs every message it hands to
NetWork::OnReceiveMessage (multi/main.cpp:351, then :352 -> multi/paxos.cpp:1714),
in the order it enqueues them, and the paxos thread drains that queue FIFO
(multi/paxos.cpp:1654-1673).  So each node's receive stream — the engine's
input — is exactly the server thread's "receive from srv[j]" lines.

What the log does not give directly is where, between two received messages,
the node's proposer control plane (out of scope) acted.
Those actions are the engine-local P_START / P_BATCH / P_PROPOSE records
(include/mpx.h), and the paxos thread logs every one of them:
  * Propose             "propose: V"                 (multi/paxos.cpp:1253)     -> P_PROPOSE(V);
  * StartPrepare        "add restart prepare timer"  (multi/paxos.cpp:1246) -> P_START,
                        ballot = the next PREPARE this node broadcasts (:814-825);
  * a new AcceptingValues "broadcast accept" (:1310) with an accept id not seen
                        before (retries resend the same id, :975-977)       -> P_BATCH.
They are placed right after the last received message whose handler has
already logged (an "anchor"), i.e. as early as the log allows:
  * PREPARE    -> OnPrepare "proposal id: ..."           (:860, always)
  * ACCEPT     -> OnAccept  "proposal id: ..."           (:1361, always)
  * COMMIT     -> OnCommit  "reply commit to C for K"    (:1575, always)
  * COMMIT_REPLY -> "commit replied from L for K"        (:1629, known commit only)
  * PREPARE_REPLY -> "update by pre-accepted values"     (:1211, id == proposal_id_ while preparing)
  * ACCEPT_REPLY that completes a quorum -> "broadcast commit" (:1464) of that
                        batch's values, right after `new CommitRetryTimeout` (:1419-1421)
Messages that do not log (REJECT, stale replies, accept votes short of a quorum)
are placed after the proposer action.  That choice is invisible to the
handlers: such a vote either completes no quorum before the action or is
ignored after it (stale ballot / unknown batch, :1038,1408-1410).  The placement
is then CHECKED, not assumed: log_facts() extracts what the reference printed
(every acceptor/learner reply, the executed stream, the quorum commits, the
final committed values) and tests/test_demo.py requires the replay of the
reconstructed streams to reproduce all of it.
"""
import gzip
import re
import struct

import mpxwire as W

RX = re.compile(r"srv\[(\d+)\] receive from srv\[(\d+)\]: ?(.*)$")
TX = re.compile(r"srv\[(\d+)\] send to srv\[(-?\d+)\] by (tcp|udp): ?(.*)$")
THREAD = re.compile(r"\[srv-(\d+)(-paxos)?:\d+\]")


def read_log(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rb") as f:
        return f.read().decode("latin-1")


def _hex(s):
    s = s.strip()
    return bytes.fromhex(s) if s else b""


def parse_log(text):
    """-> {node: {"fifo": [(src, bytes)], "px": [(func, msg)]}} (paxos-thread lines in order)."""
    nodes = {}
    for line in text.split("\n"):
        f = line.split("\t")
        if len(f) < 6:
            continue
        m = THREAD.fullmatch(f[2])
        if not m:
            continue
        n = int(m.group(1))
        nd = nodes.setdefault(n, {"fifo": [], "px": []})
        func = f[4][1:-1]
        msg = "\t".join(f[5:])
        if m.group(2) is None:
            r = RX.match(msg)
            if r:
                assert int(r.group(1)) == n, line
                nd["fifo"].append((int(r.group(2)), _hex(r.group(3))))
        else:
            nd["px"].append((func, msg))
    return nodes


def _sent(msg):
    t = TX.match(msg)
    return int(t.group(2)), _hex(t.group(4))


def _entries_multi(body):
    """{u64 iid, Value}* (ExtractInstanceValues, multi/paxos.cpp:644-662) -> [(iid, value_bytes)]."""
    out, pos = [], 0
    while pos < len(body):
        iid = struct.unpack_from("<Q", body, pos)[0]
        pos += 8
        start = pos
        pos += 13                                   # u32 proposer, u64 value_id, u8 noop
        if not body[start + 12]:
            member = body[pos]
            pos += 1
            if member:                              # membership change (never proposed by the demo)
                pos += 4
                has_node = body[pos]
                pos += 1
                if has_node:
                    ln = struct.unpack_from("<I", body, pos)[0]
                    pos += 4 + ln + 2
            else:
                ln = struct.unpack_from("<I", body, pos)[0]
                pos += 4 + ln
        out.append((iid, bytes(body[start:pos])))
    assert pos == len(body)
    return out


def _u32(b, o):
    return struct.unpack_from("<I", b, o)[0]


def _u64(b, o):
    return struct.unpack_from("<Q", b, o)[0]


def node_stream(n, nd, n_nodes):
    """Rebuild node n's processing-order stream (received messages + P_START / P_BATCH)."""
    fifo, px = nd["fifo"], nd["px"]
    quorum = n_nodes // 2 + 1
    out = []
    p = 0
    cur = None                    # current proposal ballot (after the last P_START)
    live = {}                     # accept_id -> frozenset(entries)      (accepting_values_)
    votes = {}                    # accept_id -> set(acceptor)
    seen_batch = set()

    def take(k):
        """Hand fifo[p..k] to the stream, tracking accept votes of the current ballot."""
        nonlocal p
        for j in range(p, k + 1):
            src, m = fifo[j]
            if _u32(m, 0) == 4 and _u64(m, 8) == cur and _u64(m, 16) in live:
                votes.setdefault(_u64(m, 16), set()).add(_u32(m, 4))
            out.append(m)
        p = k + 1

    def find(pred, what):
        for j in range(p, len(fifo)):
            if pred(fifo[j][1]):
                return j
        raise ValueError("node %d: no received message for anchor %s" % (n, what))

    def next_send(i, typ):
        for func, msg in px[i + 1:]:
            if func in ("SendMessageUDP", "SendMessageTCP"):
                dst, b = _sent(msg)
                if _u32(b, 0) == typ:
                    return b
        return None

    for i, (func, msg) in enumerate(px):
        if func == "OnPrepare" and msg.startswith("proposal id:"):
            take(find(lambda m: _u32(m, 0) == 0, "OnPrepare"))
        elif func == "OnAccept" and msg.startswith("proposal id:"):
            take(find(lambda m: _u32(m, 0) == 3, "OnAccept"))
        elif func == "OnCommit" and msg.startswith("reply commit to"):
            c, k = map(int, re.match(r"reply commit to (\d+) for (\d+)", msg).groups())
            take(find(lambda m: _u32(m, 0) == 5 and _u32(m, 4) == c and _u64(m, 8) == k, "OnCommit"))
        elif func == "OnCommitReply":
            lr, k = map(int, re.match(r"commit replied from (\d+) for (\d+)", msg).groups())
            take(find(lambda m: _u32(m, 0) == 6 and _u32(m, 4) == lr and _u64(m, 8) == k, "OnCommitReply"))
        elif func == "UpdateByPreAcceptedValues":
            take(find(lambda m: _u32(m, 0) == 1 and _u64(m, 8) == cur, "OnPrepareReply"))
        elif func == "Propose" and msg.startswith("propose: "):
            # a client value reaches PaxosImpl::Propose (:1250-1253; the demo proposes
            # id2str(id), main.cpp:298-301, and Debug prints it back, :214-219)
            out.append(W.p_propose(msg[len("propose: "):]))
        elif func == "StartPrepare" and msg.startswith("add restart prepare timer"):
            b = next_send(i, 0)
            if b is None:             # the run ended before this prepare went out:
                ballot = ((cur >> 16) + 1) << 16 | n if cur else (1 << 16) | n   # no reply can match
            else:
                ballot = _u64(b, 8)
            out.append(W.p_start(ballot))
            cur = ballot
            live.clear()
            votes.clear()
        elif func == "Accept" and msg.startswith("broadcast accept"):
            b = next_send(i, 3)
            aid = _u64(b, 8)
            assert _u64(b, 16) == cur, "node %d: accept with ballot %d, proposal %r" % (n, _u64(b, 16), cur)
            if aid not in seen_batch:
                seen_batch.add(aid)
                ents = _entries_multi(b[28:])
                out.append(W.p_batch(aid, ents))
                live[aid] = frozenset(ents)
        elif func == "Commit" and msg.startswith("broadcast commit"):
            prev = px[i - 1] if i else ("", "")
            if not (prev[0] == "SystemInc" and "CommitRetryTimeout" in prev[1]):
                continue              # a commit retry (:1009-1031): no handler state changes
            b = next_send(i, 5)
            if b is None:
                raise ValueError("node %d: commit without its COMMIT bytes" % n)
            ents = frozenset(_entries_multi(b[28:]))
            batch = [a for a, e in live.items() if e == ents]
            if not batch:
                continue              # the re-commit after a promise quorum (:1184-1197)
            aid = batch[0]
            have = votes.setdefault(aid, set())
            j = p
            while len(have) < quorum:
                if j >= len(fifo):
                    raise ValueError("node %d: quorum of batch %d not found" % (n, aid))
                m = fifo[j][1]
                if _u32(m, 0) == 4 and _u64(m, 8) == cur and _u64(m, 16) == aid:
                    have.add(_u32(m, 4))
                j += 1
            take(j - 1)
            del live[aid]
            votes.pop(aid, None)
    take(len(fifo) - 1)
    return out


def _max_iid(m):
    t = _u32(m, 0)
    if t in (3, 5):
        ents = _entries_multi(m[28:])
    elif t == 17:
        ents = _entries_multi(m[16:])
    elif t == 1:                  # {u64 iid, u64 pid, Value}*
        body, ents, pos = m[20:], [], 0
        while pos < len(body):
            ents.append((_u64(body, pos), b""))
            pos = _skip_accepted(body, pos)
    else:
        return -1
    return max((i for i, _ in ents), default=-1)


def _skip_accepted(body, pos):
    """One {u64 iid, u64 pid, Value} of a PREPARE_REPLY (FillAcceptedValues, multi/paxos.cpp:664-711)."""
    pos += 16
    noop = body[pos + 12]
    pos += 13
    if not noop:
        member = body[pos]
        pos += 1
        if member:
            pos += 4
            has_node = body[pos]
            pos += 1
            if has_node:
                pos += 4 + _u32(body, pos) + 2
        else:
            pos += 4 + _u32(body, pos)
    return pos


def to_trace(text):
    """MPXT container of the demo run's per-node streams; M = largest instance id + 1."""
    nodes = parse_log(text)
    n_nodes = max(nodes) + 1
    assert sorted(nodes) == list(range(n_nodes))
    streams = [node_stream(n, nodes[n], n_nodes) for n in range(n_nodes)]
    m = max(_max_iid(x) for st in streams for x in st) + 1
    return W.container(streams, num_instances=max(m, 1))


# ---- what the reference printed (checked against the replay) ---------------------
VAL = re.compile(r"<(\d+)>\((\d+):(\d+)\)([+-m])([^,]*)")


def log_facts(text):
    """Per node: acceptor/learner replies (types 1,2,4,6) with destinations, in order;
    executed payloads (Execute, multi/paxos.cpp:1584-1622); the batches chosen by an
    accept quorum, as value sets, in order (:1416-1421); the final committed values
    (:1694-1703) as (ballot, proposer, value_id, noop, payload).
    A "broadcast commit" right after `new CommitRetryTimeout` is either an accept
    quorum (OnAcceptReply, :1416-1421) or, inside the OnPrepareReply that reached
    the promise quorum, the re-commit of everything committed (:1184-1197); the
    latter is told apart by having no other handler's line in between."""
    nodes = parse_log(text)
    facts = {}
    for n, nd in sorted(nodes.items()):
        px = nd["px"]
        sends, executed, commits, final = [], [], [], None
        in_quorum = False     # inside the OnPrepareReply that reached the promise quorum
        for i, (func, msg) in enumerate(px):
            if func == "UpdateByPreAcceptedValues":
                in_quorum = True
            elif func not in ("SendMessageUDP", "SendMessageTCP", "SystemInc", "SystemDec",
                              "Accept", "Commit"):
                in_quorum = False
            if func in ("SendMessageUDP", "SendMessageTCP"):
                dst, b = _sent(msg)
                if _u32(b, 0) in (1, 2, 4, 6):
                    sends.append((dst, b))
            elif func == "OnCommit" and msg.startswith("execute: "):
                for item in msg[len("execute: "):].split(", ["):
                    v = VAL.search(item)
                    if v.group(4) == "+":
                        executed.append(v.group(5).encode())
            elif func == "Commit" and msg.startswith("broadcast commit") and i and \
                    px[i - 1][0] == "SystemInc" and "CommitRetryTimeout" in px[i - 1][1]:
                if in_quorum:         # the re-commit of everything committed (:1184-1197)
                    in_quorum = False
                    continue
                for func2, msg2 in px[i + 1:]:
                    if func2 in ("SendMessageUDP", "SendMessageTCP"):
                        b = _sent(msg2)[1]
                        if _u32(b, 0) == 5:
                            commits.append((_u64(b, 16), frozenset(_entries_multi(b[28:]))))
                            break
            elif func == "Loop" and msg.startswith("final committed values: "):
                body = msg[len("final committed values: "):]
                body = body[:body.rindex(" (")]
                final = [(int(v.group(1)), int(v.group(2)), int(v.group(3)), v.group(4) == "-",
                          v.group(5).encode() if v.group(4) == "+" else b"")
                         for v in VAL.finditer(body)]
        facts[n] = {"sends": sends, "executed": executed, "commits": commits, "final": final}
    return facts
