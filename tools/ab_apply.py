#!/usr/bin/env python3
"""Interleaved A/B of k_apply variants / grid sizes in ONE process (rule: perf
deltas come from interleaved rounds in one process).  C4 workload by default.

    python tools/ab_apply.py --variants 0,1,3 --wgs 8 --rounds 5
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
    ap.add_argument("--instances", type=int, default=1 << 27)
    ap.add_argument("--nodes", type=int, default=9)
    ap.add_argument("--variants", default="0")
    ap.add_argument("--wgs", default="8", help="workgroups per CU, comma list")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=4)
    a = ap.parse_args()
    e = mpx.Engine(a.nodes, 0, a.instances)
    e.load_clean_device(num_instances=a.instances)
    base = e.run()
    arms = [(v, w) for v in a.variants.split(",") for w in a.wgs.split(",")]
    res = {arm: [] for arm in arms}
    for r in range(a.rounds):
        for v, w in arms:
            os.environ["MPX_APPLY_VARIANT"] = v
            os.environ["MPX_APPLY_WGS_PER_CU"] = w
            for _ in range(a.steps):
                e.step()
            e.sync()
            st = e.stats()
            assert st["state_digest"] == base["state_digest"] and st["chosen"] == base["chosen"]
            ap_ms, run_ms = e.timings()
            res[(v, w)].extend(ap_ms)
    alg = base["bytes_alg"]
    for arm in arms:
        xs = res[arm]
        med = statistics.median(xs)
        print("variant %s wgs/cu %s: k_apply median %.3f ms min %.3f ms -> %.0f GB/s alg (%.1f%% of 8 TB/s)" % (
            arm[0], arm[1], med, min(xs), alg / med / 1e6, 100 * alg / med / 1e6 / 8000))


if __name__ == "__main__":
    main()
