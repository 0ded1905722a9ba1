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
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_pass(counter, outdir, bench_args):
    d = os.path.join(outdir, "pmc_" + counter.lower())
    cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc", counter, "-d", d, "-o", "pmc",
           "--output-format", "csv", "--", sys.executable, os.path.join(ROOT, "bench.py"),
           "--no-cpu-baseline"] + bench_args
    subprocess.check_call(cmd, cwd=ROOT)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection.csv under " + d)
    vals = {}
    with open(files[0]) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            name = row.get("Kernel_Name", "")
            vals.setdefault(name, []).append(float(row["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--outdir", default=os.path.join(ROOT, "gpurun_out", "pmc"))
    ap.add_argument("--instances", type=int, default=1 << 27)
    ap.add_argument("--nodes", type=int, default=9)
    a, rest = ap.parse_known_args()
    bench_args = ["--steps", "3", "--warmup", "0", "--instances", str(a.instances), "--nodes", str(a.nodes)] + rest
    fetch = run_pass("FETCH_SIZE", a.outdir, bench_args)
    write = run_pass("WRITE_SIZE", a.outdir, bench_args)
    out = {"tag": a.tag, "instances": a.instances, "nodes": a.nodes, "gpus": 1, "kernels": {}}
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, [0.0])
        w = write.get(name, [0.0])
        fk, wk = sum(f) / len(f), sum(w) / len(w)
        out["kernels"][name] = {"dispatches": len(f), "FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk,
                                "hbm_bytes_per_launch": 2 * fk * 1024 + wk * 1024}
    # the timed apply phase: k_plan + k_store + k_apply_fast<1, false, true>
    # (digest runs use the one-kernel k_apply_fast<..., true, false>)
    phase = [v for k, v in out["kernels"].items()
             if "k_plan" in k or "k_store" in k or ("k_apply_fast" in k and "true>" in k and "false" in k)]
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
