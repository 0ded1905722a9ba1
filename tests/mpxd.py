"""MPXD: phase-2 decisions at promise quorums.

    "MPXD" u32 version u32 nodes; per node: u64 count, then per decision
    u64 seq (record index in the node's stream), u64 n, {u64 iid, u64 handle} * n
"""
import struct


def parse(buf):
    assert buf[:4] == b"MPXD", buf[:4]
    _ver, n = struct.unpack_from("<II", buf, 4)
    pos = 12
    nodes = []
    for _ in range(n):
        (k,) = struct.unpack_from("<Q", buf, pos)
        pos += 8
        ds = []
        for _ in range(k):
            seq, m = struct.unpack_from("<QQ", buf, pos)
            pos += 16
            ents = [struct.unpack_from("<QQ", buf, pos + 16 * i) for i in range(m)]
            pos += 16 * m
            ds.append((seq, ents))
        nodes.append(ds)
    assert pos == len(buf), (pos, len(buf))
    return nodes
