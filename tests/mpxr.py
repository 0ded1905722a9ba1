"""Parser for the canonical MPXR result — for readable diffs."""
import struct


def parse(buf):
    assert buf[:4] == b"MPXR", buf[:4]
    ver, n_nodes, sem = struct.unpack_from("<III", buf, 4)
    pos = 16
    nodes = []

    def u64():
        nonlocal pos
        v = struct.unpack_from("<Q", buf, pos)[0]
        pos += 8
        return v

    for _ in range(n_nodes):
        nd = {"promised": u64(), "max_seen": u64()}
        nd["state"] = [tuple(u64() for _ in range(4)) for _ in range(u64())]  # iid, kind, ballot, handle
        sends = []
        for _ in range(u64()):
            dst, ln = struct.unpack_from("<II", buf, pos)
            pos += 8
            sends.append((dst, bytes(buf[pos:pos + ln])))
            pos += ln
        nd["sends"] = sends
        qs = []
        for _ in range(u64()):
            seq, ballot, n = u64(), u64(), u64()
            qs.append((seq, ballot, [tuple(u64() for _ in range(3)) for _ in range(n)]))
        nd["quorums"] = qs
        nd["chosen_batches"] = [(u64(), u64()) for _ in range(u64())]
        ex = []
        for _ in range(u64()):
            ln = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
            ex.append(bytes(buf[pos:pos + ln]))
            pos += ln
        nd["executed"] = ex
        nodes.append(nd)
    chosen = [(u64(), u64()) for _ in range(u64())]
    assert pos == len(buf), (pos, len(buf))
    return {"nodes": nodes, "chosen": chosen, "semantics": sem}


def diff(a, b, limit=5):
    """Human-readable first differences between two MPXR blobs."""
    pa, pb = parse(a), parse(b)
    out = []
    if len(pa["nodes"]) != len(pb["nodes"]):
        return ["node count %d != %d" % (len(pa["nodes"]), len(pb["nodes"]))]
    for i, (x, y) in enumerate(zip(pa["nodes"], pb["nodes"])):
        for k in x:
            if x[k] != y[k]:
                if isinstance(x[k], list):
                    for j, (u, w) in enumerate(zip(x[k], y[k])):
                        if u != w:
                            out.append("node %d %s[%d]: %r != %r" % (i, k, j, u, w))
                            break
                    if len(x[k]) != len(y[k]):
                        out.append("node %d %s: len %d != %d" % (i, k, len(x[k]), len(y[k])))
                else:
                    out.append("node %d %s: %r != %r" % (i, k, x[k], y[k]))
            if len(out) >= limit:
                return out
    if pa["chosen"] != pb["chosen"]:
        out.append("chosen log differs (%d vs %d entries)" % (len(pa["chosen"]), len(pb["chosen"])))
    return out
