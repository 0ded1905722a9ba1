"""Regenerate the golden fixtures under tests/golden/ (run in the build container).

Each fixture is a trace (.mpxt: MPXT container of per-node receive streams)
and the result the REFERENCE's own handlers produce for it (.mpxr: canonical
MPXR dump), computed by oracle/_ref/libmpx_ref.so — multi/paxos.cpp compiled
in place from /root/reference (oracle/Makefile, oracle/ref_multi_driver.cpp) —
or, for member-semantics traces (mm_*, c5_*), by oracle/_ref/libmpx_ref_member.so
(member/paxos.cpp, oracle/ref_member_driver.cpp).
The reference itself cannot travel; these vectors are what the oracle and the
engine are pinned against (tests/test_oracle.py, tests/test_engine_gpu.py).

    python tests/golden/make_golden.py
"""
import glob
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from fuzztrace import fuzz_trace  # noqa: E402
from handmade import handmade_traces  # noqa: E402
from handmade_member import member_traces  # noqa: E402
from oracles import ref_available, ref_run  # noqa: E402
import demotrace  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "multi-paxos_amd"))
import mpx  # noqa: E402  (host generators only: no GPU needed)


def main():
    if not ref_available():
        sys.exit("oracle/_ref/libmpx_ref.so missing: run `make -C oracle` where /root/reference exists")
    cases = {}
    for name, trace in handmade_traces().items():
        cases[name] = trace
    for seed in range(48):
        cases["fuzz_%03d" % seed] = fuzz_trace(seed)
    for seed in range(4):
        cases["fuzz_big_%d" % seed] = fuzz_trace(10_000 + seed, n_nodes=5, n_inst=200, n_msgs=600)
    # C2-shaped clean traces and C3-shaped contended, lossy traces at fixture size
    cases["c2_clean_n5"] = mpx.generate_trace(mpx.GEN_CLEAN, num_nodes=5, num_instances=1000, batch=256)
    cases["c2_clean_n9_b100"] = mpx.generate_trace(mpx.GEN_CLEAN, num_nodes=9, num_instances=777, batch=100)
    for seed in range(4):
        cases["c3_faulty_%d" % seed] = mpx.generate_trace(
            mpx.GEN_FAULTY, num_nodes=7, num_instances=300, seed=seed, batch=32, proposers=3,
            drop_rate=500, dup_rate=1000, max_delay=500)
    # member semantics (reference: member/paxos.cpp via oracle/_ref/libmpx_ref_member.so)
    for name, trace in member_traces().items():
        cases[name] = trace
    for seed, (U, M, B, drop, dup, noop) in enumerate([(3, 64, 4, 0, 0, 0), (4, 200, 8, 0, 0, 0),
                                                       (8, 1000, 16, 500, 100, 15), (8, 2000, 64, 1000, 300, 50),
                                                       (6, 1500, 32, 0, 200, 0)]):
        cases["c5_member_%d" % seed] = mpx.generate_trace(
            mpx.GEN_MEMBER, num_nodes=U, num_instances=M, seed=seed, batch=B, drop_rate=drop,
            dup_rate=dup, max_delay=64, noop_permille=noop)
    # C5 contended: rival proposers' rounds (proposers > 1: multi-ballot promise phases, adopted
    # values, rejected ACCEPTs, own values proposed again)
    for seed, (U, M, B, drop, dup, P) in enumerate([(4, 400, 8, 0, 0, 2), (5, 2000, 16, 0, 0, 3),
                                                    (6, 3000, 32, 500, 200, 3)]):
        cases["c5_contended_%d" % seed] = mpx.generate_trace(
            mpx.GEN_MEMBER, num_nodes=U, num_instances=M, seed=seed, batch=B, drop_rate=drop, dup_rate=dup,
            max_delay=64, proposers=P)
    # C1: the reference's own demo, captured by capture_demo.py (tests/demotrace.py, test_demo.py)
    for path in sorted(glob.glob(os.path.join(HERE, "demo", "*.log.gz"))):
        cases[os.path.basename(path)[:-len(".log.gz")]] = demotrace.to_trace(demotrace.read_log(path))
    extra = os.path.join(HERE, "extra_traces")
    if os.path.isdir(extra):
        for fn in sorted(os.listdir(extra)):
            if fn.endswith(".mpxt"):
                with open(os.path.join(extra, fn), "rb") as f:
                    cases[fn[:-5]] = f.read()
    index = {}
    for name, trace in sorted(cases.items()):
        result, stats = ref_run(trace)
        with open(os.path.join(HERE, name + ".mpxt"), "wb") as f:
            f.write(trace)
        with open(os.path.join(HERE, name + ".mpxr"), "wb") as f:
            f.write(result)
        index[name] = {"C": stats[0], "P": stats[1], "A": stats[2], "L": stats[3],
                       "trace_sha1": hashlib.sha1(trace).hexdigest(),
                       "result_sha1": hashlib.sha1(result).hexdigest()}
    with open(os.path.join(HERE, "index.json"), "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)
    print("wrote %d fixtures" % len(index))


if __name__ == "__main__":
    main()
