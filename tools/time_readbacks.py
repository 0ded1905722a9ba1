#!/usr/bin/env python3
"""Cost of the history readbacks at C3's stated size: one 2^24 x 7 faulty
trace, one digested run, then mpx_read_decisions and mpx_read_commits timed.
    python tools/time_readbacks.py [log2 instances]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-paxos_amd"))
import mpx  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 24
t = mpx.generate_trace(mpx.GEN_FAULTY, num_nodes=7, num_instances=1 << lg, seed=0, batch=256, proposers=3,
                       drop_rate=500, dup_rate=1000, max_delay=500, copy=False)
out = {"instances": 1 << lg}
with mpx.Engine.for_trace(t) as e:
    del t
    e.run()
    got = {}
    for name, fn in (("decisions", e.decisions), ("commits", e.commits)):
        t0 = time.perf_counter()
        got[name] = fn()
        out[name + "_s"] = time.perf_counter() - t0
        out[name + "_bytes"] = len(got[name])
    os.environ["MPX_DECIDE_DEVICE"] = "1"           # k_decide pass 0 over every slot per quorum (A/B)
    t0 = time.perf_counter()
    same = e.decisions() == got["decisions"]
    out["decisions_device_pass0_s"] = time.perf_counter() - t0
    out["device_pass0_same"] = same
print(json.dumps(out), flush=True)
