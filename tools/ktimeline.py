#!/usr/bin/env python3
"""Per-step kernel timeline from a rocprofv3 results database: the dispatches of one queue in
start order, cut into steps at each launch of the first kernel named, then per position the
median kernel duration and the median gap since the previous kernel ended (the dependent-launch
cost the chain pays).

    python tools/ktimeline.py gpurun_out/prof/x_results.db k_scan_chunk [out.csv]
"""
import csv
import re
import sqlite3
import statistics
import sys


def timeline(db, first):
    con = sqlite3.connect(db)
    names = dict(con.execute("select id, kernel_name from rocpd_info_kernel_symbol").fetchall())
    rows = con.execute("select kernel_id, start, end from rocpd_kernel_dispatch order by start").fetchall()
    steps, cur = [], None
    for kid, s, e in rows:
        n = re.sub(r"\(.*", "", names.get(kid, str(kid)))
        if first in n:
            cur = []
            steps.append(cur)
        if cur is not None:
            cur.append((n, s, e))
    # the common shape: the most frequent kernel sequence
    shapes = {}
    for st in steps:
        shapes.setdefault(tuple(k[0] for k in st), []).append(st)
    shape, runs = max(shapes.items(), key=lambda kv: (len(kv[1]), len(kv[0])))
    out = []
    for i, n in enumerate(shape):
        dur = statistics.median(r[i][2] - r[i][1] for r in runs)
        gap = statistics.median(r[i][1] - r[i - 1][2] for r in runs) if i else 0
        out.append((n, dur, gap))
    span = statistics.median(r[-1][2] - r[0][1] for r in runs)
    return out, span, len(runs), len(steps)


if __name__ == "__main__":
    out, span, nrun, nstep = timeline(sys.argv[1], sys.argv[2])
    w = csv.writer(open(sys.argv[3], "w") if len(sys.argv) > 3 else sys.stdout)
    w.writerow(["Position", "Name", "MedianDurationNs", "MedianGapBeforeNs"])
    for i, (n, d, g) in enumerate(out):
        w.writerow([i, n, int(d), int(g)])
    w.writerow(["span", "first start -> last end (median)", int(span), "steps %d of %d" % (nrun, nstep)])
