#!/usr/bin/env python3
"""Interleaved A/B on the clean C4 step (device-generated trace) in ONE
process: MPX_KNOBS values, per-phase device times (mpx_timings_detail).

    python tools/ab_c4.py --log2 27 --batch 100 --knobs 0,8192 --rounds 5
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
    ap.add_argument("--log2", type=int, default=27)
    ap.add_argument("--nodes", type=int, default=9)
    ap.add_argument("--batch", default="256", help="comma list")
    ap.add_argument("--knobs", default="0")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    m = 1 << a.log2
    for b in (int(x) for x in a.batch.split(",")):
        e = mpx.Engine(a.nodes, 0, m)
        e.load_clean_device(num_instances=m, batch=b)
        base = e.run()
        e.timings()
        arms = a.knobs.split(",")
        res = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k in arms:
                os.environ["MPX_KNOBS"] = k
                for _ in range(a.steps):
                    e.step()
                e.sync()
                res[k].extend(e.timings_detail())
                assert e.state_digest() == (base["state_digest"], base["chosen_digest"]), k
        os.environ["MPX_KNOBS"] = "0"
        for k in arms:
            med = {p: statistics.median(x[p] for x in res[k]) for p in mpx.Engine.PHASES}
            print("batch %d knobs %s: " % (b, k) + " ".join("%s %.3f" % (p, med[p]) for p in mpx.Engine.PHASES),
                  flush=True)
        e.close()


if __name__ == "__main__":
    main()
