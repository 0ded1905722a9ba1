"""MPXB: the Callback calls of the reference's member nodes (oracle/ref_member_driver.cpp
mpxref_member_callbacks): "MPXB" u32 1, u32 nodes; per node u64 count, then per call {u64 record,
u64 kind (0 Accepted, 1 Applied, 2 Unproposable), u32 len, cb bytes} in call order."""
import struct

KINDS = ("accepted", "applied", "unproposable")


def parse(b):
    assert b[:4] == b"MPXB"
    ver, n = struct.unpack_from("<II", b, 4)
    assert ver == 1
    p, out = 12, []
    for _ in range(n):
        (c,) = struct.unpack_from("<Q", b, p)
        p += 8
        calls = []
        for _ in range(c):
            seq, kind, ln = struct.unpack_from("<QQI", b, p)
            p += 20
            calls.append((seq, kind, bytes(b[p:p + ln])))
            p += ln
        out.append(calls)
    assert p == len(b)
    return out
