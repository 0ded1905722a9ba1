"""Write the learn-reliability fixtures (tests/golden/<name>.mpxl, format tests/mpxl.py):
for every member-semantics golden trace, the LearningValues bookkeeping the REFERENCE's
own Proposer kept — creation at accept quorums (member/paxos.cpp:1334-1337), promise
quorums (:1299-1307) and LearnersChanged (:1472-1491), Applied (:1355-1370,1504-1533),
OnLearnReply retirement (:1373-1380) and drops — recorded by
oracle/ref_member_driver.cpp (mpxref_member_learns).  Run in the build container.

    python tests/golden/make_learns.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import mpxl  # noqa: E402
from oracles import ref_available, ref_learns  # noqa: E402


def main():
    if not ref_available():
        sys.exit("oracle/_ref/libmpx_ref_member.so missing: run `make -C oracle` where /root/reference exists")
    index = json.load(open(os.path.join(HERE, "index.json")))
    out = {}
    for name in sorted(index):
        trace = open(os.path.join(HERE, name + ".mpxt"), "rb").read()
        if trace[12:16] != b"\x01\x00\x00\x00":
            continue
        d = ref_learns(trace)
        parsed = mpxl.parse(d)
        with open(os.path.join(HERE, name + ".mpxl"), "wb") as f:
            f.write(d)
        rows = [r for x in parsed for r in x]
        out[name] = {"learns": len(rows),
                     "by_kind": [sum(1 for r in rows if r[2] == k) for k in range(3)],
                     "applied": sum(1 for r in rows if r[4] != mpxl.NONE),
                     "retired": sum(1 for r in rows if r[5] != mpxl.NONE),
                     "dropped": sum(1 for r in rows if r[6] != mpxl.NONE)}
    with open(os.path.join(HERE, "learns.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("%d learn fixtures" % len(out))


if __name__ == "__main__":
    main()
