#!/usr/bin/env python3
"""Reference CPU rate of one bench leg's workload (TEST / BASELINE INFRASTRUCTURE: run only by
bench.py's cpu_baseline legs, as a child process; VERDICT r05 item 1, SURVEY.md §8(d) "CPU side").

The reference's own handlers (oracle/_ref: multi/paxos.cpp or member/paxos.cpp compiled in place,
-O2) replay a trace of the leg's own generator configuration (the same parameters and seed the
bench leg uses, at a sampled instance count) on P host cores: P forked processes each run
mpxref_run_shard / mpxref_member_run_shard over the whole sampled trace (one process per core:
the reference's objects are not made for concurrent use in one process).  decisions/s = P x the
trace's chosen instances / the wall time of the slowest process.

Why a smaller trace of the same configuration and not an instance shard of the full-size trace:
the shard mode replays EVERY record's header on every shard (multi/paxos.cpp's handlers run for
each message; only the entries are cut), so a 2^16-instance shard of the 2^24 C3 trace walks all
of its ~5 M headers (≈ 19 s here) for 3 s of entry work and would understate the reference's rate
several times; a whole trace of the same generator at 2^17 instances has the full size's mix of
headers and entries per decision.  tests/golden/full_size.json's cpu_s (the reference over the
full-size traces, 16 shards) is reported beside it as a cross-check.

    python oracle/ref_leg_rate.py c3 --instances 131072 --procs 16      (c3 | c5 | c5c)
    python oracle/ref_leg_rate.py loop --trace loop.mpxt --procs 16      (the closed loop's streams)
prints one JSON object.
"""
import argparse
import ctypes
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-paxos_amd"))

# bench.py's C3 / C5 / C5C generator parameters (BASELINE.json configs[2], configs[4])
LEGS = {
    "c3": dict(kind="GEN_FAULTY", num_nodes=7, seed=0, batch=256, proposers=3, drop_rate=500, dup_rate=1000,
               max_delay=500),
    "c5": dict(kind="GEN_MEMBER", num_nodes=8, seed=0, batch=256, drop_rate=100, dup_rate=100, max_delay=64,
               noop_permille=15),
    "c5c": dict(kind="GEN_MEMBER", num_nodes=8, seed=0, batch=256, drop_rate=100, dup_rate=100, max_delay=64,
                noop_permille=15, proposers=3),
}

_TRACE = None          # the sampled trace, inherited by the forked workers


def _worker(member):
    so = os.path.join(ROOT, "oracle", "_ref", "libmpx_ref_member.so" if member else "libmpx_ref.so")
    f = getattr(ctypes.CDLL(so), "mpxref_member_run_shard" if member else "mpxref_run_shard")
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    f.restype = ctypes.c_int
    st = (ctypes.c_uint64 * 8)()
    t0 = time.perf_counter()
    rc = f(ctypes.addressof(_TRACE), len(_TRACE), 0, (1 << 64) - 1, st)
    return rc, list(st), time.perf_counter() - t0


def main():
    global _TRACE
    ap = argparse.ArgumentParser()
    ap.add_argument("leg", choices=sorted(LEGS) + ["loop"])
    ap.add_argument("--instances", type=int, default=1 << 17)
    ap.add_argument("--procs", type=int, default=16)
    ap.add_argument("--trace", help="leg 'loop': the closed loop's recorded streams (an MPXT file) instead of "
                                    "a generated trace")
    a = ap.parse_args()
    t0 = time.perf_counter()
    if a.leg == "loop":
        data = open(a.trace, "rb").read()
        _TRACE = (ctypes.c_char * len(data)).from_buffer_copy(data)
        a.instances = int.from_bytes(data[16:24], "little")
    else:
        import mpx
        p = dict(LEGS[a.leg])
        kind = getattr(mpx, p.pop("kind"))
        _TRACE = mpx.generate_trace(kind, num_instances=a.instances, copy=False, **p)
    t_gen = time.perf_counter() - t0
    member = a.leg not in ("c3", "loop")
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(a.procs) as pool:
        res = pool.map(_worker, [member] * a.procs, chunksize=1)
    wall = time.perf_counter() - t0
    if any(rc for rc, _, _ in res):
        raise SystemExit("reference driver failed: %r" % [rc for rc, _, _ in res])
    chosen = res[0][1][0]
    if any(st != res[0][1] for _, st, _ in res):
        raise SystemExit("the processes disagree on the trace's result")
    per = [dt for _, _, dt in res]
    out = {"leg": a.leg, "instances_sampled": a.instances, "trace_bytes": len(_TRACE), "procs": a.procs,
           "chosen": chosen, "wall_s": wall, "slowest_s": max(per), "fastest_s": min(per),
           "value": a.procs * chosen / max(per), "generate_s": t_gen,
           "stats": dict(zip(("chosen", "promise_entries", "accept_apps", "commit_apps"), res[0][1][:4]))}
    full = os.path.join(ROOT, "tests", "golden", "full_size.json")
    if os.path.exists(full):
        fs = json.load(open(full)).get(a.leg)
        if fs:
            out["full_size_check"] = {
                "decisions": fs["stats"]["chosen"], "cpu_s": fs["cpu_s"], "shards": fs["shards"],
                "per_core": fs["stats"]["chosen"] / fs["cpu_s"],
                "note": "the reference over the full-size trace in %d instance shards (each replays every "
                        "header), tests/golden/full_size.json" % fs["shards"]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
