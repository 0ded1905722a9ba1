"""Closed loop: the engine's own results drive the protocol's next messages.

The recorded-trace path replays streams a reference run produced.  Here the proposer's control
plane (out of scope for the device) is a small host driver over the engine:
every message it sends is made from what the engine computed —

  * StartPrepare: P_START at the proposer, PREPARE over [0, 2^64-1) to the acceptors it picks
    (multi/paxos.cpp:1233-1248);
  * the acceptors' replies are the engine's drained sends (OnPrepare / OnAccept / OnCommit on the
    device), delivered to the node they are addressed to;
  * at the promise quorum the phase-2 batch is the engine's decision (mpx_read_decisions:
    adopted pre-accepted values, noop fill, the proposer's queued client values;
    :1056-1175), sent as P_BATCH + ACCEPT with accepting_id_ + 1 (:1299-1326);
  * a batch whose instances the engine's chosen log holds is committed (Commit, :1429-1444)
    to the nodes picked, with committing_id_ + 1.

Deliveries may reach only some acceptors, so rounds of different proposers contend and the next
quorum adopts what the last one left half-accepted.  The loop only moves bytes: promises,
quorums, merges, decisions, votes and the chosen log all come from the device.  Each step
re-runs the engine over the streams so far (an MPXT trace, `trace()`), or with
`incremental=True` submits only the records added since the last step to one engine
(MPX_FLAG_INCREMENTAL | MPX_FLAG_DECISIONS: state, promise rounds and the decisions'
bookkeeping carried across windows, O(window) per step).  Replayed through the reference's
own handlers the recorded trace gives the engine's result byte for byte (tests).
"""
import ctypes
import struct

from . import FLAG_DECISIONS, FLAG_INCREMENTAL, Engine, lib, _ck

INF = (1 << 64) - 1


def _hdr_prepare(proposer, ballot):
    body = struct.pack("<QQ", 0, INF)                 # AvailableInstanceIDs [0, 2^64-1), :741-755
    return struct.pack("<IIQI", 0, proposer, ballot, len(body)) + body


def _parse_mpxd(b):
    """MPXD -> per node [(seq, [(iid, handle)])] (include/mpx.h mpx_read_decisions)."""
    _ver, n = struct.unpack_from("<II", b, 4)
    pos, out = 12, []
    for _ in range(n):
        (c,) = struct.unpack_from("<Q", b, pos)
        pos += 8
        qs = []
        for _ in range(c):
            seq, k = struct.unpack_from("<QQ", b, pos)
            pos += 16
            qs.append((seq, [struct.unpack_from("<QQ", b, pos + 16 * i) for i in range(k)]))
            pos += 16 * k
        out.append(qs)
    return out


class ClosedLoop:
    """N nodes (multi semantics; every node an acceptor and learner), instances [0, M)."""

    def __init__(self, num_nodes, num_instances, incremental=False):
        self.N, self.M = num_nodes, num_instances
        self.incremental = incremental
        self.submitted = [0] * num_nodes              # incremental: records of each stream already submitted
        self.streams = [[] for _ in range(num_nodes)]
        self.delivered = {}                           # src -> replies of src already routed
        self.ballot_count = [0] * num_nodes
        self.ballot = [0] * num_nodes
        self.accepting_id = [0] * num_nodes
        self.committing_id = [0] * num_nodes
        self.value_id = [0] * num_nodes               # value_id_: Propose's and the noop fill's (:335)
        self.payload = {}                             # (node, value id) -> client payload
        self.batches = {}                             # (node, accept id) -> (ballot, [(iid, handle)])
        self.decided = [0] * num_nodes                # quorum decisions of each node already sent
        self.committed = set()                        # (node, accept id) already committed
        self.engine = None

    # ---- the trace and the engine over it ------------------------------------------------
    def trace(self):
        out = bytearray(b"MPXT") + struct.pack("<III", 1, self.N, 0) + struct.pack("<QII", self.M, 0, 0)
        out += struct.pack("<Q", 0)
        for msgs in self.streams:
            offs = [0]
            for m in msgs:
                offs.append(offs[-1] + len(m))
            out += struct.pack("<QQ", len(msgs), offs[-1]) + struct.pack("<%dQ" % len(offs), *offs)
            for m in msgs:
                out += m
            while len(out) % 8:
                out += b"\0"
        return bytes(out)

    def run(self):
        """Re-run the engine over every stream so far (or, incremental, one window of the records
        added since the last step); route the new replies to their nodes."""
        if self.incremental:
            if self.engine is None:
                self.engine = Engine(self.N, 0, self.M, flags=FLAG_INCREMENTAL | FLAG_DECISIONS)
            for n, msgs in enumerate(self.streams):
                if len(msgs) > self.submitted[n]:
                    self.engine.submit(n, msgs[self.submitted[n]:])
                    self.submitted[n] = len(msgs)
            st = self.engine.run()
            for _src, dst, b in self.engine.drain_sends():   # a window's replies are all new
                self.streams[dst].append(b)
            return st
        if self.engine is not None:
            self.engine.close()
        self.engine = Engine.for_trace(self.trace())
        st = self.engine.run()
        fresh = {}
        for src, dst, b in self.engine.drain_sends():
            fresh.setdefault(src, []).append((dst, b))
        for src, lst in fresh.items():                # a node's replies grow at the end of its list
            for dst, b in lst[self.delivered.get(src, 0):]:
                self.streams[dst].append(b)
            self.delivered[src] = len(lst)
        return st

    def value_bytes(self, handle):
        node, vid, noop = (handle >> 48) & 0x3FFF, handle & ((1 << 47) - 1), (handle >> 47) & 1
        if noop:
            return struct.pack("<IQ?", node, vid, True)
        if (node, vid) in self.payload:               # a client value of this loop
            p = self.payload[(node, vid)]
            return struct.pack("<IQ??I", node, vid, False, False, len(p)) + p
        buf = (ctypes.c_uint8 * 65536)()
        n = ctypes.c_uint32()
        _ck("mpx_value_bytes", lib().mpx_value_bytes(self.engine.h, handle, buf, len(buf), ctypes.byref(n)))
        return bytes(buf[: n.value])

    # ---- the proposer's moves --------------------------------------------------------------
    def prepare(self, node, to):
        """StartPrepare at `node`: a higher ballot (:1233-1248), PREPARE to the acceptors `to`."""
        self.ballot_count[node] += 1
        b = (self.ballot_count[node] << 16) | node
        self.ballot[node] = b
        self.streams[node].append(struct.pack("<IQ", 16, b))          # P_START (include/mpx.h)
        for a in to:
            self.streams[a].append(_hdr_prepare(node, b))

    def propose(self, node, payload):
        """A client value reaches Propose at `node` (queued while preparing, :1250-1280)."""
        if isinstance(payload, str):
            payload = payload.encode()
        self.value_id[node] += 1
        self.payload[(node, self.value_id[node])] = payload
        self.streams[node].append(struct.pack("<II", 19, len(payload)) + payload)   # P_PROPOSE

    def accept_decided(self, node, to):
        """Send the phase-2 batch the engine decided at `node`'s latest unsent promise quorum."""
        qs = _parse_mpxd(self.engine.decisions())[node]
        if self.decided[node] >= len(qs):
            return None
        for _s, es in qs[self.decided[node]:]:       # value_id_ also counts the noops (:1117-1130)
            self.value_id[node] += sum(1 for _i, h in es if (h >> 47) & 1 and (h >> 48) == node)
        _seq, ents = qs[-1]
        self.decided[node] = len(qs)
        if not ents:
            return None
        self.accepting_id[node] += 1
        aid, b = self.accepting_id[node], self.ballot[node]
        body = b"".join(struct.pack("<Q", iid) + self.value_bytes(h) for iid, h in ents)
        self.streams[node].append(struct.pack("<IQI", 17, aid, len(body)) + body)          # P_BATCH
        acc = struct.pack("<IIQQI", 3, node, aid, b, len(body)) + body                     # ACCEPT
        for a in to:
            self.streams[a].append(acc)
        self.batches[(node, aid)] = (b, ents)
        return aid

    def commit_chosen(self, node, to):
        """COMMIT every batch of `node` whose instances are all in the engine's chosen log."""
        done = []
        chosen = None                                 # the chosen log, read once per call
        for (n, aid), (b, ents) in sorted(self.batches.items()):
            if n != node or (n, aid) in self.committed:
                continue
            if chosen is None:
                chosen = self.engine.read_chosen(0, self.M)
            if not all(chosen[iid] >> 63 for iid, _h in ents):
                continue
            self.committed.add((n, aid))
            self.committing_id[node] += 1
            body = b"".join(struct.pack("<Q", iid) + self.value_bytes(h) for iid, h in ents)
            com = struct.pack("<IIQQI", 5, node, self.committing_id[node], b, len(body)) + body
            for a in to:
                self.streams[a].append(com)
            done.append(aid)
        return done

    def close(self):
        if self.engine is not None:
            self.engine.close()
            self.engine = None


def _mask(to):
    m = 0
    for a in to:
        m |= 1 << a
    return m


class NativeLoop:
    """The same driver inside libmpx (mpx_loop_*, csrc/loop.cpp): ClosedLoop's moves in C++ on one
    incremental engine, no Python between a window's decisions / chosen log and the next window's
    P_BATCH / ACCEPT / COMMIT records.  Same method names and arguments as ClosedLoop(...,
    incremental=True); for one schedule both record identical streams."""

    def __init__(self, num_nodes, num_instances, device=0):
        from . import LoopStats  # noqa: F401
        self.N, self.M = num_nodes, num_instances
        h = ctypes.c_void_p()
        _ck("mpx_loop_create", lib().mpx_loop_create(num_nodes, num_instances, device, ctypes.byref(h)))
        self.h = h
        self.engine = Engine.__new__(Engine)              # a view of the loop's engine (the loop owns it)
        self.engine.h = ctypes.c_void_p(lib().mpx_loop_engine(h))
        self.engine.num_nodes = num_nodes
        self.engine.shard_begin, self.engine.shard_end = 0, num_instances
        self.engine.close = lambda: None

    def prepare(self, node, to):
        _ck("mpx_loop_prepare", lib().mpx_loop_prepare(self.h, node, _mask(to)))

    def propose(self, node, payload):
        if isinstance(payload, str):
            payload = payload.encode()
        _ck("mpx_loop_propose", lib().mpx_loop_propose(self.h, node, payload, len(payload)))

    def run(self):
        _ck("mpx_loop_step", lib().mpx_loop_step(self.h))

    def accept_decided(self, node, to):
        aid = ctypes.c_uint64()
        _ck("mpx_loop_accept_decided", lib().mpx_loop_accept_decided(self.h, node, _mask(to), ctypes.byref(aid)))
        return aid.value or None

    def commit_chosen(self, node, to):
        c = ctypes.c_uint32()
        _ck("mpx_loop_commit_chosen", lib().mpx_loop_commit_chosen(self.h, node, _mask(to), ctypes.byref(c)))
        return c.value

    def leader_rounds(self, leader, to, rounds, values):
        _ck("mpx_loop_leader_rounds", lib().mpx_loop_leader_rounds(self.h, leader, _mask(to), rounds, values))

    def stats(self):
        from . import LoopStats
        st = LoopStats()
        _ck("mpx_loop_stats_get", lib().mpx_loop_stats_get(self.h, ctypes.byref(st)))
        return {k: getattr(st, k) for k, _ in LoopStats._fields_}

    def trace(self):
        from . import _take
        out = ctypes.POINTER(ctypes.c_uint8)()
        size = ctypes.c_uint64()
        _ck("mpx_loop_trace", lib().mpx_loop_trace(self.h, ctypes.byref(out), ctypes.byref(size)))
        return _take(out, size.value)

    def close(self):
        if self.h:
            lib().mpx_loop_destroy(self.h)
            self.h = None
