#!/usr/bin/env python3
"""Per-kernel duration summary from a rocprofv3 results database (rocpd SQLite):
kernel name, calls, total / average / min / max ns — the --stats table, written
as CSV so it can be committed under profiles/.

    python tools/kstats.py gpurun_out/prof/x_results.db [out.csv]
"""
import csv
import re
import sqlite3
import sys


def stats(db):
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("pragma table_info(rocpd_kernel_dispatch)")]
    name_col = "kernel_id"
    rows = con.execute("select d.%s, d.start, d.end from rocpd_kernel_dispatch d" % name_col).fetchall()
    names = dict(con.execute("select id, kernel_name from rocpd_info_kernel_symbol").fetchall())
    agg = {}
    for kid, s, e in rows:
        n = names.get(kid, str(kid))
        n = re.sub(r"\(.*", "", n)
        a = agg.setdefault(n, [0, 0, 1 << 62, 0])
        d = e - s
        a[0] += 1; a[1] += d; a[2] = min(a[2], d); a[3] = max(a[3], d)
    out = sorted(((n, c, t, t / c, mn, mx) for n, (c, t, mn, mx) in agg.items()), key=lambda x: -x[2])
    return cols, out


if __name__ == "__main__":
    _, out = stats(sys.argv[1])
    tot = sum(x[2] for x in out)
    w = csv.writer(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
    for n, c, t, avg, mn, mx in out:
        w.writerow([n, c, t, "%.1f" % avg, mn, mx, "%.2f" % (100.0 * t / tot)])
