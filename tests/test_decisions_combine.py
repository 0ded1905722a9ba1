"""CPU checks of mpx_decisions_combine (include/mpx.h): the
host-only merge of per-shard decision parts (MPXP) into MPXD.  Parts are cut
from the reference's own decision fixtures (tests/golden/*.mpxd) at instance
boundaries, with the fill noops' handles blanked to ~0 as a shard writes them;
merging them must give the fixture back byte for byte."""
import json
import os
import struct

import pytest

import mpx
import mpxd

GOLD = os.path.join(os.path.dirname(__file__), "golden")
DECISIONS = sorted(json.load(open(os.path.join(GOLD, "decisions.json"))))
NOOP_SLOT = (1 << 64) - 1


def _handle(node, noop, vid):
    return (node << 48) | ((1 if noop else 0) << 47) | vid


def _parts(buf, cuts):
    """Split MPXD into MPXP parts at the instance boundaries `cuts` (ascending)."""
    nodes = mpxd.parse(buf)
    begins = [0] + list(cuts)
    out = []
    for k, sb in enumerate(begins):
        se = begins[k + 1] if k + 1 < len(begins) else 1 << 63
        b = bytearray(b"MPXP" + struct.pack("<IIQ", 1, len(nodes), sb))
        for node, ds in enumerate(nodes):
            b += struct.pack("<Q", len(ds))
            vid = 0
            for seq, ents in ds:
                mine = []
                for iid, h in ents:
                    fill = h == _handle(node, True, vid + 1)      # the next number of the node's fill noops
                    if fill:
                        vid += 1
                    if sb <= iid < se:
                        mine.append((iid, NOOP_SLOT if fill else h))
                b += struct.pack("<QQ", seq, len(mine))
                for iid, h in mine:
                    b += struct.pack("<QQ", iid, h)
        out.append(bytes(b))
    return out


@pytest.mark.parametrize("name", DECISIONS)
def test_combine_restores_reference_decisions(name):
    want = open(os.path.join(GOLD, name + ".mpxd"), "rb").read()
    iids = sorted({i for ds in mpxd.parse(want) for _, ents in ds for i, _ in ents})
    assert mpx.decisions_combine(_parts(want, [])) == want
    if iids:
        mid = iids[len(iids) // 2]
        assert mpx.decisions_combine(_parts(want, [mid])) == want
        q = [iids[len(iids) * j // 4] for j in (1, 2, 3)]
        assert mpx.decisions_combine(_parts(want, sorted(set(x for x in q if x > 0)))) == want


def test_combine_rejects_mismatched_parts():
    want = open(os.path.join(GOLD, "fuzz_big_1.mpxd"), "rb").read()
    a, b = _parts(want, [100])
    with pytest.raises(mpx.MpxError):
        mpx.decisions_combine([b, a])                           # not in shard order
    with pytest.raises(mpx.MpxError):
        mpx.decisions_combine([a, b[:-8]])                      # truncated
    with pytest.raises(mpx.MpxError):
        mpx.decisions_combine([a, b"MPXD" + b[4:]])             # not a part
    with pytest.raises(mpx.MpxError):
        mpx.decisions_combine([a, b + b"\0" * 16])              # trailing bytes
    with pytest.raises(mpx.MpxError):
        mpx.decisions_combine([a, b[:4] + struct.pack("<I", 2) + b[8:]])   # another layout version


def test_combine_rejects_entries_outside_their_shard():
    """A part may only hold instances of its own shard: [its shard_begin, the next part's)."""
    want = open(os.path.join(GOLD, "fuzz_big_1.mpxd"), "rb").read()
    iids = sorted({i for ds in mpxd.parse(want) for _, ents in ds for i, _ in ents})
    mid = iids[len(iids) // 2]
    a, b = _parts(want, [mid])
    # re-label part b as beginning one past its first instance: its entries now start below it
    b2 = b[:12] + struct.pack("<Q", mid + 1) + b[20:]
    with pytest.raises(mpx.MpxError):
        mpx.decisions_combine([a, b2])
    # and part a claiming an instance of b's range
    a2 = _parts(want, [mid + 1])[0]
    with pytest.raises(mpx.MpxError):
        mpx.decisions_combine([a2, b])


# ---- mpx_commit_points_combine (include/mpx.h: sharded commit reliability) ----
def _mpxq(nodes):
    import struct
    b = b"MPXQ" + struct.pack("<II", 1, len(nodes))
    for pts in nodes:
        b += struct.pack("<Q", len(pts))
        for seq, aid in pts:
            b += struct.pack("<QQ", seq, aid)
    return b


def test_commit_points_union():
    """The union of per-shard creation points: a batch kept by two shards is one point,
    promise-quorum points (~0) merge with accept-quorum points in stream order."""
    P = (1 << 64) - 1
    a = _mpxq([[(3, 1), (9, P)], [], [(5, 2)]])
    b = _mpxq([[(3, 1), (7, 4)], [(2, P)], []])
    assert mpx.commit_points_combine([a, b]) == _mpxq([[(3, 1), (7, 4), (9, P)], [(2, P)], [(5, 2)]])
    assert mpx.commit_points_combine([a]) == a


def test_commit_points_reject_bad_parts():
    P = (1 << 64) - 1
    a = _mpxq([[(3, 1)], []])
    with pytest.raises(mpx.MpxError):
        mpx.commit_points_combine([a, _mpxq([[(3, 1)]])])          # node counts differ
    with pytest.raises(mpx.MpxError):
        mpx.commit_points_combine([a, _mpxq([[(3, 2)], []])])      # two creations at one record
    with pytest.raises(mpx.MpxError):
        mpx.commit_points_combine([a + b"\0" * 8])                 # trailing bytes
    with pytest.raises(mpx.MpxError):
        mpx.commit_points_combine([_mpxq([[(4, P), (3, 1)], []])])  # not ascending


def _mpxe(parts_events, n_nodes, sb, se):
    b = bytearray(b"MPXE") + struct.pack("<IIQQ", 1, n_nodes, sb, se)
    for evs in parts_events:
        b += struct.pack("<Q", len(evs))
        for seq, t, ents in evs:
            b += struct.pack("<QII", seq, t, len(ents))
            for iid, h in ents:
                b += struct.pack("<QQ", iid, h)
    return bytes(b)


def test_proposal_combine_walks_client_values():
    """mpx_proposal_combine (host only): a client value proposed while idle takes the next
    unproposed id (Propose, multi/paxos.cpp:1250-1280); a COMMIT of another value there
    re-proposes it (:1519-1570); after StartPrepare a quorum adopts the other shard's
    pre-accepted value and noop-fills the gap (:1056-1175)."""
    other = (1 << 48) | 7
    a = _mpxe([[(0, 19, []), (1, 5, [(0, other)]), (2, 16, []), (3, 1, [])]], 1, 0, 4)
    b = _mpxe([[(0, 19, []), (2, 16, []), (3, 1, [(5, (1 << 48) | 9)])]], 1, 4, 16)
    got = mpx.proposal_combine([a, b])
    # value 1 at instance 0, committed there as another value -> re-proposed at 1 (idle);
    # the quorum: unproposed = [1, inf) minus adopted 5 -> the noop fill comes first and takes
    # 1..4 (value ids 2..5), so the own value finds its id gone (it waits for that commit)
    want = bytearray(b"MPXD") + struct.pack("<IIQ", 1, 1, 1) + struct.pack("<QQ", 3, 5)
    for iid, h in [(1, (1 << 47) | 2), (2, (1 << 47) | 3), (3, (1 << 47) | 4), (4, (1 << 47) | 5),
                   (5, (1 << 48) | 9)]:
        want += struct.pack("<QQ", iid, h)
    assert got == bytes(want), mpxd.parse(got)
    with pytest.raises(mpx.MpxError):
        mpx.proposal_combine([b, a])                       # not in shard order
    with pytest.raises(mpx.MpxError):
        mpx.proposal_combine([a, _mpxe([[(3, 5, [])]], 1, 4, 16)])   # record types disagree
    with pytest.raises(mpx.MpxError):
        mpx.proposal_combine([a[:-4]])                     # truncated


MEMBER_DECISIONS = [k for k in DECISIONS if k.startswith(("c5_", "mm_"))]


def _member_mpxe(trace, result, cuts):
    """Member MPXE parts (version 2, include/mpx.h) of a trace cut at instance boundaries:
    every shard lists each node's Propose / StartPrepare / E_EPOCH records, its quorums and
    LEARNs with the entries of its own instances — the quorums' merged maps from the oracle's
    MPXR result (what the device computes)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "oracle"))
    import mpxr
    from learns_model import _streams
    from member_decisions_model import _learn_entries
    epochs, streams = _streams(trace)
    res = mpxr.parse(result)
    bounds = [0] + list(cuts) + [1 << 62]
    parts = []
    for s in range(len(bounds) - 1):
        sb, se = bounds[s], bounds[s + 1]
        b = bytearray(b"MPXE") + struct.pack("<IIQQ", 2, len(streams), sb, se)
        b += struct.pack("<I", len(epochs))
        for _v, am, pm, _lm in epochs:
            b += struct.pack("<QQ", am, pm)
        for n, msgs in enumerate(streams):
            quorums = {q[0]: q[2] for q in res["nodes"][n]["quorums"]}
            evs = []
            for k, m in enumerate(msgs):
                t = struct.unpack_from("<I", m)[0]
                if t in (16, 19):
                    evs.append((k, t, 0, []))
                elif t == 18:
                    evs.append((k, t, struct.unpack_from("<I", m, 4)[0], []))
                elif t == 5:
                    evs.append((k, t, 0, [e for e in _learn_entries(m) if sb <= e[0] < se]))
                elif t == 1 and k in quorums:
                    evs.append((k, t, 0, sorted((i, h) for i, _p, h in quorums[k] if sb <= i < se)))
            b += struct.pack("<Q", len(evs))
            for k, t, aux, ents in evs:
                b += struct.pack("<QIIQ", k, t, len(ents), aux)
                for iid, h in ents:
                    b += struct.pack("<QQ", iid, h)
        parts.append(bytes(b))
    return parts


@pytest.mark.parametrize("name", MEMBER_DECISIONS)
def test_member_proposal_combine_restores_reference_decisions(name):
    """The engine's member Proposer walk (engine.cpp mprop_advance, host only) over the union
    of member MPXE parts — whole, and cut into 2 and 3 instance shards — gives the reference's
    own decisions (fixture: real Proposer::Propose calls, member/paxos.cpp:1122-1297,1383-1470)."""
    from oracles import oracle_run
    trace = open(os.path.join(GOLD, name + ".mpxt"), "rb").read()
    want = open(os.path.join(GOLD, name + ".mpxd"), "rb").read()
    result = oracle_run(trace)[0]
    m = struct.unpack_from("<Q", trace, 16)[0]
    for cuts in ([], [m // 2], [m // 3, 2 * m // 3]):
        assert mpx.proposal_combine(_member_mpxe(trace, result, [c for c in cuts if c > 0])) == want, cuts


def test_member_proposal_combine_rejects_mixed_parts():
    from oracles import oracle_run
    trace = open(os.path.join(GOLD, "mm_propose.mpxt"), "rb").read()
    parts = _member_mpxe(trace, oracle_run(trace)[0], [3])
    multi = _mpxe([[(0, 19, [])]], 1, 3, 16)
    with pytest.raises(mpx.MpxError):
        mpx.proposal_combine([parts[0], multi])                   # member and multi parts
    bad = bytearray(parts[1])
    bad[36] ^= 1                                                   # another epoch table
    with pytest.raises(mpx.MpxError):
        mpx.proposal_combine([parts[0], bytes(bad)])
