#!/usr/bin/env python3
"""Kernel timeline of the last timed step of a leg from a rocprofv3 results database: every
dispatch (all queues) from the step's first header-scan kernel to its summary, with start /
duration / end relative to the step start.

    python tools/c3_timeline.py gpurun_out/x/prof_results.db [marker-kernel-substring] [out.txt]
"""
import re
import sqlite3
import sys


def main():
    db = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "k_plan_list"
    con = sqlite3.connect(db)
    names = dict(con.execute("select id, kernel_name from rocpd_info_kernel_symbol").fetchall())
    rows = con.execute("select kernel_id, start, end, queue_id from rocpd_kernel_dispatch order by start").fetchall()

    def nm(k):
        n = re.sub(r"\(.*", "", names[k])
        return n.replace("_ZN3mpx", "").replace("ENS_7DevView", "").replace(".kd", "")[:56]

    marks = [i for i, r in enumerate(rows) if marker in names[r[0]]]
    idx = marks[-1]
    j = idx
    while j > 0 and "k_scan_chunk" not in names[rows[j][0]]:
        j -= 1
    base = rows[j][1]
    out = []
    for r in rows[j:]:
        out.append("%-56s q%-3s start %9.1f dur %8.1f end %9.1f" % (nm(r[0]), r[3], (r[1] - base) / 1e3, (r[2] - r[1]) / 1e3,
                                                               (r[2] - base) / 1e3))
        if "k_reduce" in names[r[0]] or "k_store8ILb1ELj128ELb1" in names[r[0]]:
            break
    txt = "\n".join(out)
    print(txt)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(txt + "\n")


if __name__ == "__main__":
    main()
