"""Member phase-2 decisions restated in Python — TEST INFRASTRUCTURE (oracle/: only tests use it, as the checker).

The batch member Proposer::OnPrepareReply builds at a promise quorum
(member/paxos.cpp:1183-1297): unproposed = the proposer's unlearned ids; adopt the merged
pre-accepted value of every unproposed id, noop-fill every unproposed range but the last,
then its initial proposals still unproposed and its queued values at the next free ids.
Proposer::OnLearn (:1383-1470) keeps the sets: a learned id leaves unlearned / unproposed,
an initial proposal that lost its id is proposed again (now, or queued while preparing).
A P_PROPOSE record is Node::Propose -> Proposer::Propose (:1122-1156): value_id_ + 1, the
next unproposed id at once, or queued while preparing (no Proposer: Unproposable).  A
Proposer starts with every id unlearned (:1074-1082); the engine model and the reference
driver idle it at each E_EPOCH step that creates it or changes its acceptors until its next
P_START.
The promise quorums and merged maps come from an MPXR result (what the device computes).
Checked against the reference's own decisions (tests/golden/*.mpxd) on CPU; the engine's
host walk (engine.cpp member_decisions) is the same algorithm.
"""
import bisect
import struct

import mpxr
from learns_model import _streams

INF = (1 << 64) - 1


class IdSet:
    """AvailableInstanceIDs (multi/paxos.cpp:253-318): disjoint [a, b) ranges, kept as sorted
    start / end lists (binary search)."""

    def __init__(self):
        self.a, self.b = [0], [INF]

    def copy(self):
        c = IdSet()
        c.a, c.b = list(self.a), list(self.b)
        return c

    @property
    def r(self):
        return list(zip(self.a, self.b))

    def _find(self, i):
        k = bisect.bisect_right(self.a, i) - 1
        return k if k >= 0 and i < self.b[k] else -1

    def contains(self, i):
        return self._find(i) >= 0

    def remove(self, i):
        k = self._find(i)
        if k < 0:
            return
        a, b = self.a[k], self.b[k]
        if a != i and i + 1 != b:
            self.b[k] = i
            self.a.insert(k + 1, i + 1)
            self.b.insert(k + 1, b)
        elif a != i:
            self.b[k] = i
        elif i + 1 != b:
            self.a[k] = i + 1
        else:
            del self.a[k], self.b[k]

    def next(self):
        a = self.a[0]
        self.remove(a)
        return a

    def pop_first(self):
        a, b = self.a.pop(0), self.b.pop(0)
        return a, b


def _value(m, pos):
    """member Value_m at pos -> (handle, end)"""
    p, vid, noop = struct.unpack_from("<IQ?", m, pos)
    pos += 13
    h = (p << 48) | (int(noop) << 47) | vid
    if noop:
        return h, pos
    mem, ln = struct.unpack_from("<?I", m, pos)
    pos += 5
    pos += 8 * ln if mem else ln
    (cl,) = struct.unpack_from("<I", m, pos)
    return h, pos + 4 + cl


def _learn_entries(m):
    (ln,) = struct.unpack_from("<I", m, 16)
    pos, end, out = 20, 20 + ln, []
    while pos < end:
        iid = struct.unpack_from("<Q", m, pos)[0]
        h, pos = _value(m, pos + 16)
        out.append((iid, h))
    return sorted(out)


def decisions(trace, result):
    epochs, streams = _streams(trace)
    res = mpxr.parse(result)
    b = bytearray(b"MPXD") + struct.pack("<II", 1, len(streams))
    for n, msgs in enumerate(streams):
        quorums = {q[0]: q[2] for q in res["nodes"][n]["quorums"]}
        learned = {}
        st = None                                   # the Proposer, if any

        def new_proposer():
            return {"unlearned": IdSet(), "unproposed": IdSet(), "initial": {}, "newly": set(), "vid": 0,
                    "prep": True}

        if (epochs[0][2] >> n) & 1:
            st = new_proposer()
            st["prep"] = False
        out, ei, idle = [], 0, False
        for k, m in enumerate(msgs):
            t = struct.unpack_from("<I", m)[0]
            if t != 18 and idle:
                if st:
                    st["prep"] = False
                idle = False
            if t == 16 and st:
                st["prep"] = True
            elif t == 19 and st:                    # Proposer::Propose (:1122-1156)
                st["vid"] += 1
                if not st["prep"]:
                    st["initial"][st["unproposed"].next()] = st["vid"]
                else:
                    st["newly"].add(st["vid"])
            elif t == 1 and k in quorums and st:
                un = st["unlearned"].copy()
                batch = []
                for iid, _pid, h in quorums[k]:
                    if un.contains(iid):
                        un.remove(iid)
                        batch.append((iid, h))
                while len(un.a) != 1:
                    a, e = un.pop_first()
                    for i in range(a, e):
                        st["vid"] += 1
                        batch.append((i, (n << 48) | (1 << 47) | st["vid"]))
                for iid in sorted(st["initial"]):
                    if un.contains(iid):
                        un.remove(iid)
                        batch.append((iid, (n << 48) | st["initial"][iid]))
                for vid in sorted(st["newly"]):
                    iid = un.next()
                    st["initial"][iid] = vid
                    batch.append((iid, (n << 48) | vid))
                st["newly"].clear()
                st["unproposed"] = un
                st["prep"] = False
                out.append((k, sorted(batch)))
            elif t == 5:
                ents = _learn_entries(m)
                if st:                              # Proposer::OnLearn (:1383-1470)
                    conflicts = set()
                    for iid, h in ents:
                        if iid not in learned and st["unlearned"].contains(iid):
                            st["unlearned"].remove(iid)
                        if st["unproposed"].contains(iid):
                            st["unproposed"].remove(iid)
                        if iid in st["initial"]:
                            v0 = st["initial"].pop(iid)
                            if (h >> 48) != n or (h & ((1 << 47) - 1)) != v0:
                                conflicts.add(v0)
                    if conflicts:
                        if not st["prep"]:
                            for vid in sorted(conflicts):
                                st["initial"][st["unproposed"].next()] = vid
                        else:
                            st["newly"] |= conflicts
                for iid, h in ents:
                    learned.setdefault(iid, h)
            elif t == 18:
                ej = struct.unpack_from("<I", m, 4)[0]
                o, x = epochs[ei], epochs[ej]
                was, now = bool((o[2] >> n) & 1), bool((x[2] >> n) & 1)
                if now and not was:
                    st = new_proposer()             # the constructor's StartPrepare: preparing
                if was and not now:
                    st = None
                if st and (x[1] != o[1]):
                    st["prep"] = True               # AcceptorsChanged -> RestartPrepare / AcceptRejected
                if now and (not was or o[1] != x[1]):
                    idle = True                     # the driver idles it once the LEARN's changes ran
                ei = ej
        b += struct.pack("<Q", len(out))
        for k, batch in out:
            b += struct.pack("<QQ", k, len(batch))
            for iid, h in batch:
                b += struct.pack("<QQ", iid, h)
    return bytes(b)
