"""MPXL: member learn-reliability bookkeeping (include/mpx.h mpx_read_learns).

    "MPXL" u32 version u32 nodes; per node: u64 count, then per LearningValues in creation
    order: u64 id, u64 created_seq, u64 kind (0 accept quorum, 1 promise quorum, 2 learners
    changed), u64 accept_id (kind 0), u64 applied_seq, u64 retired_seq, u64 dropped_seq
    (~0: did not happen), u64 learned mask (learner bits)
"""
import struct

NONE = (1 << 64) - 1


def parse(buf):
    assert buf[:4] == b"MPXL", buf[:4]
    _ver, n = struct.unpack_from("<II", buf, 4)
    pos = 12
    nodes = []
    for _ in range(n):
        (k,) = struct.unpack_from("<Q", buf, pos)
        pos += 8
        nodes.append([struct.unpack_from("<8Q", buf, pos + 64 * i) for i in range(k)])
        pos += 64 * k
    assert pos == len(buf), (pos, len(buf))
    return nodes
