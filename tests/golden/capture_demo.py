"""Capture C1 demo traces: run the REFERENCE's own multi/ demo and keep its TRACE log.

C1 (BASELINE.json configs[0]) is "multi/ demo as shipped via run.sh on CPU".
run.sh runs `./main $(cat debug.conf)` (multi/run.sh:5); this script runs the
same program — oracle/_ref/multi_demo, built by `make -C oracle ref` from
/root/reference/multi/{main,paxos}.cpp exactly as multi/Makefile builds it —
with the shipped debug.conf.sample arguments, except:
  * --log-level=0 (TRACE): every received and sent message is logged as hex
    (multi/main.cpp:146,351), which is what the replay needs;
  * --seed=K, so the captured runs differ.
The demo is multi-threaded and wall-clock driven, so each run is a different
trace; the captured log IS the fixture (tests/golden/demo/*.log.gz, data
written by the reference).  tests/demotrace.py turns a log into per-node
receive streams; make_golden.py pins them with oracle/_ref.

Runs only in the build container (needs /root/reference).

    python tests/golden/capture_demo.py [--seeds 0 1 2] [--args "4 4 10 100"]
"""
import argparse
import gzip
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
DEMO = os.path.join(ROOT, "oracle", "_ref", "multi_demo")
CONF = "/root/reference/multi/debug.conf.sample"


def demo_args(seed, positional=None):
    args = open(CONF).read().split()
    out = []
    for a in args:
        if a.startswith("--log-level="):
            a = "--log-level=0"
        elif a.startswith("--seed="):
            a = "--seed=%d" % seed
        out.append(a)
    if positional:
        pos = positional.split()
        out = pos + [a for a in out if a.startswith("--")]
    return out


def capture(seed, name, positional=None, timeout=600):
    argv = [DEMO] + demo_args(seed, positional)
    with tempfile.TemporaryFile() as f:
        rc = subprocess.call(argv, stdout=f, stderr=subprocess.STDOUT, timeout=timeout)
        f.seek(0)
        data = f.read()
    if rc != 0 or b"All done" not in data:
        raise RuntimeError("demo run %s failed (rc=%d)" % (name, rc))
    os.makedirs(os.path.join(HERE, "demo"), exist_ok=True)
    path = os.path.join(HERE, "demo", name + ".log.gz")
    with gzip.GzipFile(path, "wb", mtime=0) as g:
        g.write(data)
    print("%s: %d lines -> %s" % (name, data.count(b"\n"), path))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="*", default=[0, 1, 2])
    ap.add_argument("--args", default=None, help="positional srvcnt cltcnt idcnt interval")
    ap.add_argument("--prefix", default="demo")
    a = ap.parse_args()
    if not os.path.exists(DEMO):
        sys.exit("oracle/_ref/multi_demo missing: run `make -C oracle ref` where /root/reference exists")
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(len(a.seeds)) as ex:
        futs = [ex.submit(capture, s, "%s_s%d" % (a.prefix, s), a.args) for s in a.seeds]
        for f in futs:
            f.result()


if __name__ == "__main__":
    main()
