"""MPXC: commit-reliability bookkeeping (include/mpx.h mpx_read_commits).

    "MPXC" u32 version u32 nodes; per node: u64 count, then per CommittingValues
    (id 1, 2, ...): u64 id, u64 created_seq, u64 kind (0 accept quorum, 1 promise
    quorum re-commit), u64 accept_id (kind 0), u64 retired_seq (~0: open),
    u64 replied mask (learner bits)
"""
import struct

OPEN = (1 << 64) - 1


def parse(buf):
    assert buf[:4] == b"MPXC", buf[:4]
    _ver, n = struct.unpack_from("<II", buf, 4)
    pos = 12
    nodes = []
    for _ in range(n):
        (k,) = struct.unpack_from("<Q", buf, pos)
        pos += 8
        nodes.append([struct.unpack_from("<6Q", buf, pos + 48 * i) for i in range(k)])
        pos += 48 * k
    assert pos == len(buf), (pos, len(buf))
    return nodes
