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
    ap.add_argument("--knobs", default="0", help="MPX_KNOBS values, comma list (kernel experiment switches)")
    ap.add_argument("--wgs", default="8", help="workgroups per CU, comma list")
    ap.add_argument("--store-wgs", default="8", help="k_store workgroups per CU, comma list")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=4)
    a = ap.parse_args()
    e = mpx.Engine(a.nodes, 0, a.instances)
    e.load_clean_device(num_instances=a.instances)
    base = e.run()
    arms = [(v, w, k, sw) for v in a.variants.split(",") for w in a.wgs.split(",") for k in a.knobs.split(",")
            for sw in a.store_wgs.split(",")]
    res = {arm: [] for arm in arms}
    runs = {arm: [] for arm in arms}
    for r in range(a.rounds):
        for v, w, k, sw in arms:
            os.environ["MPX_STORE_WGS_PER_CU"] = sw
            os.environ["MPX_APPLY_VARIANT"] = v
            os.environ["MPX_APPLY_WGS_PER_CU"] = w
            os.environ["MPX_KNOBS"] = k
            for _ in range(a.steps):
                e.step()
            e.sync()
            st = e.stats()
            for key in ("chosen", "accept_apps", "commit_apps", "promise_entries", "violations"):
                assert st[key] == base[key], (key, v, w, k)   # steps leave the digests 0 (mpx_step)
            ap_ms, run_ms = e.timings()
            res[(v, w, k, sw)].extend(ap_ms)
            runs[(v, w, k, sw)].extend(run_ms)
    if int(a.knobs.split(",")[0]) & 16 == 0:
        chk = e.run()                       # a digested run after the timed steps
        assert chk["state_digest"] == base["state_digest"] and chk["chosen_digest"] == base["chosen_digest"]
    alg = base["bytes_alg"]
    for arm in arms:
        xs = res[arm]
        med = statistics.median(xs)
        print("variant %s wgs/cu %s knobs %s store wgs/cu %s: apply median %.3f ms min %.3f ms -> %.0f GB/s alg (%.1f%% of 8 TB/s); "
              "run median %.3f ms" % (arm[0], arm[1], arm[2], arm[3], med, min(xs), alg / med / 1e6, 100 * alg / med / 1e6 / 8000,
                                      statistics.median(runs[arm])))


if __name__ == "__main__":
    main()
