"""MPXV (include/mpx.h mpx_read_learn_values): "MPXV" u32 1, u32 nodes; per node u64 count, per
learn {u64 n, n x {u64 iid, u64 handle}}, then u64 u, u x u64 unproposable record."""
import struct


def parse(b):
    assert b[:4] == b"MPXV"
    ver, n = struct.unpack_from("<II", b, 4)
    assert ver == 1
    p, out = 12, []
    for _ in range(n):
        (c,) = struct.unpack_from("<Q", b, p)
        p += 8
        learns = []
        for _ in range(c):
            (k,) = struct.unpack_from("<Q", b, p)
            p += 8
            learns.append([struct.unpack_from("<QQ", b, p + 16 * i) for i in range(k)])
            p += 16 * k
        (u,) = struct.unpack_from("<Q", b, p)
        p += 8
        unprop = list(struct.unpack_from("<%dQ" % u, b, p))
        p += 8 * u
        out.append((learns, unprop))
    assert p == len(b)
    return out
