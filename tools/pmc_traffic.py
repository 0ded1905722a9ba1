#!/usr/bin/env python3
"""HBM traffic per apply phase (k_plan + k_store + k_apply_fast) from rocprofv3 PMC counters (run on the GPU box).

Follows MI355X_MICROARCH.md §HBM / §rocprofv3 PMC slots:
  * FETCH_SIZE (3 TCC slots) and WRITE_SIZE (2) do not fit one pass together:
    one --pmc pass each, kernel-trace only (no sys/runtime trace with --pmc);
  * both are in KiB; on gfx950 FETCH_SIZE counts half the bytes of a wide
    coalesced streaming read (128-B requests tallied at 64 B): x2;
  * WRITE_SIZE is exact for 16-B-per-lane stores (k_apply's state stores).
The result goes to gpurun_out/pmc/<tag>_pmc.json; committed copies live in
profiles/, where bench.py picks them up as roofline.traffic.

    python tools/pmc_traffic.py --tag r01 [bench args...]
    python tools/pmc_traffic.py --tag r02_c3 --c3 --sq     (C3 general path, + SQ wave-state pass)
    python tools/pmc_traffic.py --tag r02_c5 --c5          (C5 member path)
    python tools/pmc_traffic.py --tag r04_c3w --c3w        (C3 as 16 incremental windows: k_apply_win)
    python tools/pmc_traffic.py --tag r04_c5c --c5c        (contended C5: 3 member proposers)
"""
import argparse
import csv
import glob
import re
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-paxos_amd"))
import mpx  # noqa: E402  (source_digest only: no GPU call)
# one pass: at most 8 SQ counters (MI355X_MICROARCH.md §rocprofv3 PMC slots); WAIT_ANY +
# WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES (quad-cycles)
SQ_COUNTERS = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
               "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU", "SQ_INSTS_SALU"]


def run_pass(counters, outdir, bench_args, tag, limit=400):
    """One rocprofv3 --pmc pass (kernel trace only); {counter: {kernel: [values per dispatch]}}."""
    d = os.path.join(outdir, "%s_pmc_%s" % (tag, "_".join(c.lower() for c in counters)))
    cmd = ["timeout", "-s", "KILL", str(limit), "rocprofv3", "--pmc"] + counters + ["-d", d, "-o", "pmc",
           "--output-format", "csv", "--", sys.executable, os.path.join(ROOT, "bench.py"),
           "--no-cpu-baseline"] + bench_args
    subprocess.check_call(cmd, cwd=ROOT)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection.csv under " + d)
    vals = {c: {} for c in counters}
    with open(files[0]) as f:
        for row in csv.DictReader(f):
            c = row.get("Counter_Name")
            if c not in vals:
                continue
            vals[c].setdefault(row.get("Kernel_Name", ""), []).append(float(row["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--outdir", default=os.path.join(ROOT, "gpurun_out", "pmc"))
    ap.add_argument("--instances", type=int, default=1 << 27)
    ap.add_argument("--nodes", type=int, default=9)
    ap.add_argument("--c3", action="store_true", help="the C3 general-path leg (bench.py --c3-only)")
    ap.add_argument("--c5", action="store_true", help="the C5 member leg (bench.py --c5-only)")
    ap.add_argument("--c3w", action="store_true", help="the C3 windows leg (bench.py --c3-windows-only)")
    ap.add_argument("--c5c", action="store_true", help="the contended C5 leg (bench.py --c5c-only)")
    ap.add_argument("--sq", action="store_true", help="also one pass of SQ wave-state counters")
    a, rest = ap.parse_known_args()
    # the workload's true size, recorded with the profile (bench.py matches it exactly)
    if a.c3w:
        a.instances, a.nodes = 1 << 24, 7
        bench_args = ["--c3-windows-only", "--c3-instances", str(a.instances)] + rest
    elif a.c5:
        a.instances, a.nodes = 1 << 25, 8
        bench_args = ["--c5-only", "--c5-steps", "3", "--c5-instances", str(a.instances)] + rest
    elif a.c5c:
        a.instances, a.nodes = 1 << 25, 8
        bench_args = ["--c5c-only", "--c5-steps", "3", "--c5c-instances", str(a.instances)] + rest
    elif a.c3:
        a.instances, a.nodes = 1 << 24, 7
        bench_args = ["--c3-only", "--c3-steps", "3", "--c3-instances", str(a.instances)] + rest
    else:
        bench_args = ["--steps", "3", "--warmup", "0", "--instances", str(a.instances), "--nodes", str(a.nodes),
                      "--c3-instances", "0", "--c5-instances", "0", "--c5c-instances", "0", "--shard-of", "0",
                      "--loop-values", "0"] + rest
    lim = 480 if a.c5c else 400                     # (the contended trace takes ~2.5 min to generate and ingest)
    fetch = run_pass(["FETCH_SIZE"], a.outdir, bench_args, a.tag, lim)["FETCH_SIZE"]
    write = run_pass(["WRITE_SIZE"], a.outdir, bench_args, a.tag, lim)["WRITE_SIZE"]
    sq = run_pass(SQ_COUNTERS, a.outdir, bench_args, a.tag, lim) if a.sq else {}
    out = {"tag": a.tag, "workload": "C3W 2^%d x 7 in 16 windows (bench.py --c3-windows-only)" % (a.instances.bit_length() - 1)
           if a.c3w else "C5 2^%d member (bench.py --c5-only)" % (a.instances.bit_length() - 1) if a.c5 else
           "C5C 2^%d member, 3 proposers (bench.py --c5c-only)" % (a.instances.bit_length() - 1) if a.c5c else
           "C3 2^%d x 7 (bench.py --c3-only)" % (a.instances.bit_length() - 1) if a.c3 else "C4",
           "instances": a.instances, "nodes": a.nodes, "gpus": 1, "source_digest": mpx.source_digest(),
           "kernels": {}}
    mean = lambda xs: sum(xs) / len(xs) if xs else 0.0
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, [0.0])
        w = write.get(name, [0.0])
        fk, wk = mean(f), mean(w)
        out["kernels"][name] = {"dispatches": len(f), "FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk,
                                "hbm_bytes_per_launch": 2 * fk * 1024 + wk * 1024}
        for c, per in sq.items():
            if name in per:
                out["kernels"][name][c] = mean(per[name])
    # the timed apply phase: k_plan + k_store + k_apply_fast<1, false, true>
    # (digest runs use the one-kernel k_apply_fast<..., true, false>)
    # C3 adds the general k_apply of the timed steps
    if a.c3w:                                       # the window apply (one launch per window)
        phase = [v for k, v in out["kernels"].items() if "k_apply_win" in k]
    else:
        phase = [v for k, v in out["kernels"].items()
                 if "k_plan" in k or "k_store" in k or "k_commit_check" in k   # (the Value check: timed steps only)
                 or ((a.c3 or a.c5 or a.c5c) and re.search(r"k_apply<\d+, false", k))]   # k_apply<waves, DIGEST, ...>: not the digested run's
    out["apply_phase_kernels"] = [k for k, v in out["kernels"].items() if v in phase]
    out["hbm_bytes_per_launch"] = sum(v["hbm_bytes_per_launch"] for v in phase) if phase else None
    out["correction"] = "FETCH_SIZE x2 (gfx950 half-count of wide streaming reads), KiB -> bytes"
    # written under gpurun_out/ (merged back from the GPU box); copy into profiles/ to commit
    path = os.path.join(a.outdir, "%s_pmc.json" % a.tag)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
