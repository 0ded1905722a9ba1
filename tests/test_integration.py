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
