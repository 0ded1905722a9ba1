"""Wire encoder for hand-made traces (test helper).

Encodes the reference's packed little-endian messages (SURVEY.md Appendix A;
multi/paxos.cpp:741-755,830-856,1282-1297,1345-1357,1429-1444,1481-1492) and
the Value codec (FillValue, multi/paxos.cpp:556-598), plus the engine-local
proposer markers P_START / P_BATCH (include/mpx.h), and packs per-node
receive streams into an MPXT trace container (DESIGN.md §Trace container).
"""
import struct

U64_MAX_EXCL = (1 << 64) - 1   # AvailableInstanceIDs starts as [0, 2^64-1), multi/paxos.cpp:259


def value(proposer, value_id, payload=None, noop=False):
    """FillValue: u32 proposer, u64 value_id, bool noop, [bool member=0, u32 len, bytes]."""
    b = struct.pack("<IQ?", proposer, value_id, noop)
    if noop:
        return b
    if isinstance(payload, str):
        payload = payload.encode()
    return b + struct.pack("<?I", False, len(payload)) + payload


def value_member(proposer, value_id, node_id, ip=None, port=0):
    """Membership-change Value (multi codec keeps it even though proposing is #if 0)."""
    b = struct.pack("<IQ??I", proposer, value_id, False, True, node_id)
    if ip is None:
        return b + struct.pack("<?", False)
    ip = ip.encode()
    return b + struct.pack("<?I", True, len(ip)) + ip + struct.pack("<H", port)


def handle(proposer, value_id, noop=False):
    return (proposer << 48) | (int(bool(noop)) << 47) | value_id


def prepare(proposer, ballot, ranges=((0, U64_MAX_EXCL),)):
    body = b"".join(struct.pack("<QQ", a, b) for a, b in ranges)
    return struct.pack("<IIQI", 0, proposer, ballot, len(body)) + body


def prepare_reply(acceptor, ballot, entries=()):
    """entries: (iid, pid, value_bytes)"""
    body = b"".join(struct.pack("<QQ", i, p) + v for i, p, v in entries)
    return struct.pack("<IIQI", 1, acceptor, ballot, len(body)) + body


def reject(max_id):
    return struct.pack("<IQ", 2, max_id)


def accept(proposer, accept_id, ballot, entries):
    """entries: (iid, value_bytes)"""
    body = b"".join(struct.pack("<Q", i) + v for i, v in entries)
    return struct.pack("<IIQQI", 3, proposer, accept_id, ballot, len(body)) + body


def accept_reply(acceptor, ballot, accept_id):
    return struct.pack("<IIQQ", 4, acceptor, ballot, accept_id)


def commit(committer, commit_id, ballot, entries):
    body = b"".join(struct.pack("<Q", i) + v for i, v in entries)
    return struct.pack("<IIQQI", 5, committer, commit_id, ballot, len(body)) + body


def commit_reply(learner, commit_id):
    return struct.pack("<IIQ", 6, learner, commit_id)


def p_start(ballot):
    return struct.pack("<IQ", 16, ballot)


def p_batch(batch_id, entries):
    body = b"".join(struct.pack("<Q", i) + v for i, v in entries)
    return struct.pack("<IQI", 17, batch_id, len(body)) + body


def p_propose(payload):
    """PaxosImpl::Propose(value) of a client value (multi/paxos.cpp:1250-1280)."""
    if isinstance(payload, str):
        payload = payload.encode()
    return struct.pack("<II", 19, len(payload)) + payload


def container(streams, num_instances=0, semantics=0, epochs=()):
    """streams: list (per node) of lists of message bytes, in processing order.
    epochs (member): (version, acceptor_mask, proposer_mask[, learner_mask]) per epoch; a
    member container is version 2 (32-byte entries, learner_mask defaults to proposer_mask)."""
    out = bytearray(b"MPXT")
    out += struct.pack("<III", 2 if epochs else 1, len(streams), semantics)
    out += struct.pack("<QII", num_instances, len(epochs), 0)
    out += struct.pack("<Q", 0)
    assert len(out) == 40
    for e in epochs:
        ver, amask, pmask = e[:3]
        out += struct.pack("<IIQQQ", ver, 0, amask, pmask, e[3] if len(e) > 3 else pmask)
    for msgs in streams:
        offs = [0]
        for m in msgs:
            offs.append(offs[-1] + len(m))
        out += struct.pack("<QQ", len(msgs), offs[-1])
        out += struct.pack("<%dQ" % len(offs), *offs)
        for m in msgs:
            out += m
        while len(out) % 8:
            out += b"\0"
    return bytes(out)


# ---- member semantics (member/paxos.cpp:321-440,846-932) ----------------------
ADD_LEARNER, LEARNER_TO_PROPOSER, PROPOSER_TO_ACCEPTOR = 0, 1, 2
DEL_LEARNER, PROPOSER_TO_LEARNER, ACCEPTOR_TO_PROPOSER = 3, 4, 5


def mvalue(proposer, value_id, payload=None, cb=b"", noop=False, changes=None):
    """FillValue (member): u32 proposer, u64 value_id, bool noop; unless noop:
    bool membership, then u32 count + {u32 node, u32 type}* or u32 len + bytes;
    then u32 cblen + cb."""
    b = struct.pack("<IQ?", proposer, value_id, noop)
    if noop:
        return b
    if isinstance(payload, str):
        payload = payload.encode()
    if isinstance(cb, str):
        cb = cb.encode()
    if changes is not None:
        b += struct.pack("<?I", True, len(changes)) + b"".join(struct.pack("<II", n, t) for n, t in changes)
    else:
        b += struct.pack("<?I", False, len(payload)) + payload
    return b + struct.pack("<I", len(cb)) + cb


def m_entries(entries):
    """(iid, pid, value_bytes) -> {u64 iid, u64 pid, Value_m}*"""
    return b"".join(struct.pack("<QQ", i, p) + v for i, p, v in entries)


def m_prepare(version, proposer, ballot, ranges=((0, U64_MAX_EXCL),)):
    body = b"".join(struct.pack("<QQ", a, b) for a, b in ranges)
    return struct.pack("<IIIQI", 0, version, proposer, ballot, len(body)) + body


def m_prepare_reply(acceptor, ballot, entries=()):
    body = m_entries(entries)
    return struct.pack("<IIQI", 1, acceptor, ballot, len(body)) + body


def m_accept(version, proposer, accept_id, ballot, entries):
    body = m_entries(entries)
    return struct.pack("<IIIQQI", 3, version, proposer, accept_id, ballot, len(body)) + body


def m_accept_reply(acceptor, accept_id):
    return struct.pack("<IIQ", 4, acceptor, accept_id)


def m_learn(proposer, learn_id, entries):
    body = m_entries(entries)
    return struct.pack("<IIQI", 5, proposer, learn_id, len(body)) + body


def m_learn_reply(learner, learn_id):
    return struct.pack("<IIQ", 6, learner, learn_id)


def m_p_batch(batch_id, entries):
    body = m_entries(entries)
    return struct.pack("<IQI", 17, batch_id, len(body)) + body


def m_p_propose(value):
    """Node::Propose / AddAcceptor / ... reaching the member Proposer (member/paxos.cpp:630-733,
    1122-1156): the Value_m bytes after proposer / value id / noop (membership flag, payload or
    change list, cb), as {u32 type=19, u32 len, body}.  `value`: an mvalue (not a noop)."""
    body = value[13:]
    return struct.pack("<II", 19, len(body)) + body


def e_epoch(epoch):
    return struct.pack("<II", 18, epoch)
