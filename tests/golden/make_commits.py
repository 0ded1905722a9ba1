"""Write the commit-reliability fixtures (tests/golden/<name>.mpxc, format tests/mpxc.py):
for every multi-semantics golden trace in which a proposer created a
CommittingValues, the bookkeeping the REFERENCE's own handlers kept — creation at
accept quorums (multi/paxos.cpp:1416-1421) and promise quorums (:1184-1197),
OnCommitReply retirement and replied_ sets (:1625-1641) — recorded by
oracle/ref_multi_driver.cpp (mpxref_commits).  Run in the build container.

    python tests/golden/make_commits.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import mpxc  # noqa: E402
from oracles import ref_available, ref_commits  # noqa: E402


def main():
    if not ref_available():
        sys.exit("oracle/_ref/libmpx_ref.so missing: run `make -C oracle` where /root/reference exists")
    index = json.load(open(os.path.join(HERE, "index.json")))
    out = {}
    for name in sorted(index):
        trace = open(os.path.join(HERE, name + ".mpxt"), "rb").read()
        if trace[12:16] != b"\x00\x00\x00\x00":
            continue
        d = ref_commits(trace)
        parsed = mpxc.parse(d)
        nc = sum(len(x) for x in parsed)
        if not nc:
            continue
        with open(os.path.join(HERE, name + ".mpxc"), "wb") as f:
            f.write(d)
        out[name] = {"commits": nc,
                     "retired": sum(1 for x in parsed for r in x if r[4] != mpxc.OPEN),
                     "promise_quorum": sum(1 for x in parsed for r in x if r[2] == 1)}
    with open(os.path.join(HERE, "commits.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("%d commit fixtures" % len(out))


if __name__ == "__main__":
    main()
