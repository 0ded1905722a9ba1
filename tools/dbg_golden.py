import sys, struct
sys.path[:0] = ["tests", "multi-paxos_amd"]
import mpx, mpxr
name = sys.argv[1]
t = open("tests/golden/%s.mpxt" % name, "rb").read()
want = open("tests/golden/%s.mpxr" % name, "rb").read()
with mpx.Engine.for_trace(t) as e:
    e.run()
    got = e.dump()
open("gpurun_out/got_%s.mpxr" % name, "wb").write(got)
g, w = mpxr.parse(got), mpxr.parse(want)
def ents(body):
    L = struct.unpack_from("<I", body, 16)[0]; cur = 20; out = []
    while cur < 20 + L:
        iid, pid = struct.unpack_from("<QQ", body, cur); cur += 16
        if body[cur + 12]: cur += 13
        else: cur += 18 + struct.unpack_from("<I", body, cur + 14)[0]
        out.append((iid, pid))
    return out
for n in range(len(w["nodes"])):
    for i, (a, b) in enumerate(zip(g["nodes"][n]["sends"], w["nodes"][n]["sends"])):
        if a != b:
            print("node", n, "send", i, "dst", a[0], b[0], "types", a[1][:4], b[1][:4])
            if a[1][0] == 1:
                ea, eb = ents(a[1]), ents(b[1])
                print(" got", len(ea), "want", len(eb))
                print(" extra", sorted(set(ea) - set(eb))[:20]); print(" missing", sorted(set(eb) - set(ea))[:20])
            break
