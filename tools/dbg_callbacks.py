"""Debug: engine vs reference Callback calls for one member golden in 4 marker-free windows."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "multi-paxos_amd")]
import mpx
import test_engine_gpu as T
name = sys.argv[1]
W = int(sys.argv[2]) if len(sys.argv) > 2 else 4
trace = T._read(name, ".mpxt")
want = T._reference_callbacks(name)
_hd, epochs, streams = T._node_streams(trace)
live = T._strip_markers(streams)
hd = mpx.trace_header(trace)
n, m = hd["num_nodes"], max(hd["num_instances"], 1)
with mpx.Engine(n, 0, m, semantics=mpx.SEM_MEMBER, epochs=epochs[:1],
                flags=mpx.FLAG_INCREMENTAL | mpx.FLAG_DECISIONS | mpx.FLAG_LEARN_EPOCHS) as e:
    prev = [0] * n
    for w in range(1, W + 1):
        cut = [len(s) * w // W for s in live]
        for node, s in enumerate(live):
            if cut[node] > prev[node]:
                e.submit(node, s[prev[node]:cut[node]])
        e.run()
        prev = cut
    got = T._engine_callbacks(e, streams)
    import mpxl
    L = mpxl.parse(e.learns())
for k in range(n):
    a, b = got[k], want[k]
    if a != b:
        from collections import Counter
        ca, cb = Counter(a), Counter(b)
        print("node", k, "engine-only", sorted((ca - cb).elements())[:40])
        print("node", k, "ref-only", sorted((cb - ca).elements())[:40])
        print("node", k, "learns", L[k][:40])
import mpxv
for WW in (1, 2, 3, 4):
    with mpx.Engine(n, 0, m, semantics=mpx.SEM_MEMBER, epochs=epochs[:1],
                    flags=mpx.FLAG_INCREMENTAL | mpx.FLAG_DECISIONS | mpx.FLAG_LEARN_EPOCHS) as e:
        prev = [0] * n
        for w in range(1, WW + 1):
            cut = [len(s) * w // WW for s in live]
            for node, s in enumerate(live):
                if cut[node] > prev[node]:
                    e.submit(node, s[prev[node]:cut[node]])
            e.run()
            prev = cut
            print("W", WW, "window", w, "cut node0", cut[0])
        V = mpxv.parse(e.learn_values())
        L = mpxl.parse(e.learns())
        print("W", WW, [(row[0], row[1], row[2], row[3], len(vs)) for row, vs in zip(L[0], V[0][0])][:14])
