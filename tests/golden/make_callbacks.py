"""Write the Callback fixtures (tests/golden/<name>.mpxb, format tests/mpxb.py): for every
member-semantics golden trace, every Callback::Accepted (member/paxos.cpp:1332), Applied
(:1368,1526) and Unproposable (:787) call the REFERENCE's own nodes made, with its record and cb
string, recorded by oracle/ref_member_driver.cpp (mpxref_member_callbacks).  Run in the build
container.

    python tests/golden/make_callbacks.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import mpxb  # noqa: E402
from oracles import ref_available, ref_callbacks  # noqa: E402


def main():
    if not ref_available():
        sys.exit("oracle/_ref/libmpx_ref_member.so missing: run `make -C oracle` where /root/reference exists")
    index = json.load(open(os.path.join(HERE, "index.json")))
    out = {}
    for name in sorted(index):
        trace = open(os.path.join(HERE, name + ".mpxt"), "rb").read()
        if trace[12:16] != b"\x01\x00\x00\x00":
            continue
        d = ref_callbacks(trace)
        calls = [c for node in mpxb.parse(d) for c in node]
        with open(os.path.join(HERE, name + ".mpxb"), "wb") as f:
            f.write(d)
        out[name] = {k: sum(1 for c in calls if c[1] == i) for i, k in enumerate(mpxb.KINDS)}
    with open(os.path.join(HERE, "callbacks.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("%d callback fixtures" % len(out))


if __name__ == "__main__":
    main()
