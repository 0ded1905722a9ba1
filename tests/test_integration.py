"""The integration example (examples/engine_host.cpp): the reference's own
paxos::NetWork / paxos::StateMachine classes (multi/paxos.h:193-222) bound to
libmpx.so.  On the GPU its transport and state machines must see exactly what
the Python binding reports for the same trace."""
import os
import subprocess

import pytest

import mpx
import mpxr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "examples", "_build", "engine_host")
GOLD = os.path.join(ROOT, "tests", "golden")


def _fnv(h, b):
    for x in b:
        h = ((h ^ x) * 1099511628211) & ((1 << 64) - 1)
    return h


def test_example_links_libmpx():
    """Built here against the reference header (build()); it loads libmpx.so and checks its arguments."""
    if not os.path.exists(BIN):
        pytest.skip("examples/_build/engine_host not built (needs /root/reference at build time)")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("windows", [0, 3])
@pytest.mark.parametrize("name", ["fuzz_big_0", "hm_commit_tags", "c3_faulty_0", "demo_s0"])
def test_example_host_matches_binding(name, windows):
    """The demo's own NodeInfoMap addresses every reply (port = node index,
    multi/main.cpp:265-268); whole run (windows 0) and three incremental windows
    (MPX_FLAG_INCREMENTAL: receive a slice, apply it, send its replies) alike."""
    if not os.path.exists(BIN):
        pytest.fail("examples/_build/engine_host missing: build() builds it where /root/reference exists")
    path = os.path.join(GOLD, name + ".mpxt")
    if not os.path.exists(path):
        pytest.skip("no golden " + name)
    out = subprocess.run([BIN, path, str(windows)], capture_output=True, text=True, timeout=120,
                         check=True).stdout.split("\n")
    trace = open(path, "rb").read()
    with mpx.Engine.for_trace(trace) as e:
        e.run()
        sends = e.drain_sends()
        parsed = mpxr.parse(e.dump())
        fronts = [e.read_executed(n)[0] for n in range(e.num_nodes)]
    h = 0
    for src, dst, b in sends:
        h = (h + _fnv(1469598103934665603, src.to_bytes(4, "little") + dst.to_bytes(4, "little") + b)) % (1 << 64)
    assert out[0] == "sends %d %016x" % (len(sends), h)
    for n, nd in enumerate(parsed["nodes"]):
        hx = 1469598103934665603
        for p in nd["executed"]:
            hx = _fnv(hx, p)
        assert out[1 + n] == "executed %d %d %d %016x" % (n, fronts[n], len(nd["executed"]), hx)


# ---- the member host hooks (examples/member_host.cpp; member/paxos.h:142-191) ----
MBIN = os.path.join(ROOT, "examples", "_build", "member_host")
NONE = (1 << 64) - 1


def test_member_example_links_libmpx():
    if not os.path.exists(MBIN):
        pytest.skip("examples/_build/member_host not built (needs /root/reference at build time)")
    r = subprocess.run([MBIN], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage" in r.stderr


def _member_expect(name):
    """What the reference's own node showed its host, from its fixtures: the replies it sent and
    the values StateMachine::Apply received (.mpxr), and every Callback call its nodes made —
    Accepted, Applied, Unproposable, each learn kind counted (.mpxb: a recording Callback in
    oracle/ref_member_driver.cpp, member/paxos.cpp:784-787,1327-1332,1360-1368,1523-1526)."""
    import mpxb
    from test_engine_gpu import _node_streams
    trace = open(os.path.join(GOLD, name + ".mpxt"), "rb").read()
    ref = mpxr.parse(open(os.path.join(GOLD, name + ".mpxr"), "rb").read())
    calls = mpxb.parse(open(os.path.join(GOLD, name + ".mpxb"), "rb").read())
    _hd, epochs, _streams = _node_streams(trace)
    h = 0
    count = 0
    for src, nd in enumerate(ref["nodes"]):
        for dst, b in nd["sends"]:
            h = (h + _fnv(1469598103934665603, src.to_bytes(4, "little") + dst.to_bytes(4, "little") + b)) % (1 << 64)
            count += 1
    lines = ["sends %d %016x" % (count, h)]
    for n, nd in enumerate(ref["nodes"]):
        hx = 1469598103934665603
        for p in nd["executed"]:
            hx = _fnv(hx, p)
        tally = [[0, 0] for _ in range(3)]                # Accepted, Applied, Unproposable
        for _seq, kind, cb in calls[n]:
            t = tally[kind]
            t[0] += 1
            t[1] = (t[1] + _fnv(1469598103934665603, cb)) % (1 << 64)
        lines.append(("applied", n, len(nd["executed"]), hx))
        lines.append("callbacks %d %s" % (n, " ".join("%d %016x" % (c, x) for c, x in tally)))
    return lines, epochs


@pytest.mark.gpu
@pytest.mark.parametrize("windows", [1, 4])
@pytest.mark.parametrize("name", ["mm_clean3", "mm_learners", "mm_acceptor_reset", "c5_member_2", "c5_member_4",
                                  "c5_contended_1", "c5_contended_2"])
def test_member_host_matches_reference(name, windows):
    """The reference's member/paxos.h NetWork / StateMachine / Callback classes on libmpx: a live
    host submits only what NetWork::OnReceive receives (no markers; the engine learns the
    membership from the Values its Learners apply, MPX_FLAG_LEARN_EPOCHS), whole and in 4
    incremental windows; its transport, state machines and callbacks see what the reference's own
    node showed its host (fixtures: every Accepted / Applied / Unproposable call, all learn kinds),
    and the epochs the engine learned are the trace's."""
    if not os.path.exists(MBIN):
        pytest.fail("examples/_build/member_host missing: build() builds it where /root/reference exists")
    path = os.path.join(GOLD, name + ".mpxt")
    out = subprocess.run([MBIN, path, str(windows)], capture_output=True, text=True, timeout=120,
                         check=True).stdout.strip().split("\n")
    want, epochs = _member_expect(name)
    assert out[0] == want[0]
    body = [x for x in out if x.startswith(("applied", "callbacks"))]
    for k, w in enumerate(want[1:]):
        if isinstance(w, tuple):                            # applied <node> <frontier> <count> <hash>
            f = body[k].split()
            assert (f[0], int(f[1]), int(f[3]), int(f[4], 16)) == w, body[k]
        else:
            assert body[k] == w
    ep = [x for x in out if x.startswith("epochs ")][0].split()[1:]
    got = [tuple(int(v, 16) if i else int(v) for i, v in enumerate(s.split(":"))) for s in ep]
    assert got == [tuple(e) for e in epochs[:len(got)]] and len(got) > 1
    per = [int(x) for x in [x for x in out if x.startswith("epochs_per_window")][0].split()[1:]]
    assert per == sorted(per) and per[-1] == len(got) and len(per) == windows
