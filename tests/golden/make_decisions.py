"""Write the phase-2 decision fixtures (tests/golden/<name>.mpxd, format tests/mpxd.py):
for every golden trace with a promise quorum, the batch the REFERENCE's own
OnPrepareReply built there (multi/paxos.cpp:1056-1182, member/paxos.cpp:1183-1297),
recorded by oracle/ref_multi_driver.cpp (mpxref_decisions) or
oracle/ref_member_driver.cpp (mpxref_member_decisions).  Run in the build container.

    python tests/golden/make_decisions.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import mpxd  # noqa: E402
from oracles import ref_available, ref_decisions, ref_member_decisions  # noqa: E402


def main():
    if not ref_available():
        sys.exit("oracle/_ref/libmpx_ref.so missing: run `make -C oracle` where /root/reference exists")
    index = json.load(open(os.path.join(HERE, "index.json")))
    out = {}
    for name in sorted(index):
        trace = open(os.path.join(HERE, name + ".mpxt"), "rb").read()
        d = ref_decisions(trace) if trace[12:16] == b"\x00\x00\x00\x00" else ref_member_decisions(trace)
        parsed = mpxd.parse(d)
        nq = sum(len(x) for x in parsed)
        if not nq:
            continue
        with open(os.path.join(HERE, name + ".mpxd"), "wb") as f:
            f.write(d)
        out[name] = {"quorums": nq, "entries": sum(len(e) for x in parsed for _, e in x)}
    with open(os.path.join(HERE, "decisions.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("%d decision fixtures" % len(out))


if __name__ == "__main__":
    main()
