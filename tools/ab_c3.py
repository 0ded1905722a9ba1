#!/usr/bin/env python3
"""Interleaved A/B on the C3 general path in ONE process: MPX_KNOBS values and
k_apply grid sizes, per-phase device times (mpx_timings_detail).

    python tools/ab_c3.py --log2 22 --knobs 0,4096 --wgs 8,16 --rounds 3
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-paxos_amd"))
import mpx  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2", type=int, default=22)
    ap.add_argument("--knobs", default="0")
    ap.add_argument("--wgs", default="8")
    ap.add_argument("--variants", default="0", help="MPX_APPLY_VARIANT values (1: the general k_apply unconstrained, 3 waves/SIMD)")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    t = mpx.generate_trace(mpx.GEN_FAULTY, num_nodes=7, num_instances=1 << a.log2, seed=0, batch=256, proposers=3,
                           drop_rate=500, dup_rate=1000, max_delay=500, copy=False)
    e = mpx.Engine.for_trace(t)
    del t
    base = e.run()
    e.timings()
    arms = [(k, w, x) for k in a.knobs.split(",") for w in a.wgs.split(",") for x in a.variants.split(",")]
    res = {arm: [] for arm in arms}
    for _ in range(a.rounds):
        for k, w, x in arms:
            os.environ["MPX_KNOBS"] = k
            os.environ["MPX_APPLY_WGS_PER_CU"] = w
            os.environ["MPX_APPLY_VARIANT"] = x
            for _ in range(a.steps):
                e.step()
            e.sync()
            res[(k, w, x)].extend(e.timings_detail())
    os.environ["MPX_KNOBS"] = "0"
    os.environ["MPX_APPLY_VARIANT"] = "0"
    chk = e.run()
    assert chk["state_digest"] == base["state_digest"]
    for arm in arms:
        ph = res[arm]
        med = {p: statistics.median(x[p] for x in ph) for p in mpx.Engine.PHASES}
        print("knobs %s wgs/cu %s variant %s: " % arm + " ".join("%s %.3f" % (p, med[p]) for p in mpx.Engine.PHASES), flush=True)


if __name__ == "__main__":
    main()
