"""Host ingest invariants (no GPU): build_trace's bucket-run aliasing keeps every run's entries
its message's own, and FR_VCHK marks exactly the runs whose re-commits the device's Value check
(k_commit_check) must compare (tests/ingest_invariants.cpp, built here from the engine's own
ingest and generator sources)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "multi-paxos_amd", "csrc")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("ingest") / "ingest_invariants")
    src = [os.path.join(ROOT, "tests", "ingest_invariants.cpp")] + \
          [os.path.join(CSRC, f) for f in ("ingest.cpp", "gen.cpp", "gen_faulty.cpp", "gen_member.cpp")]
    subprocess.run(["g++", "-O2", "-std=c++17", "-I" + CSRC, "-I" + os.path.join(ROOT, "include")] + src +
                   ["-o", exe], check=True, timeout=600)
    return exe


@pytest.mark.parametrize("kind,lg,proposers", [("faulty", 16, 3), ("faulty", 15, 2), ("member", 15, 0), ("member", 15, 3)])
def test_run_aliasing_and_value_check_marks(checker, kind, lg, proposers):
    r = subprocess.run([checker, kind, str(lg), str(proposers)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
    runs, aliased, marked, veq, upid = map(int, r.stdout.split()[1:6])
    assert runs > 0 and veq > 0
    if kind == "faulty":
        assert aliased > 0          # competing proposers' re-commits of equal Values share entries
        assert upid > 0             # promise replies to a contending proposer's prepare


# ---- membership learned at run time (MPX_FLAG_LEARN_EPOCHS, ingest.cpp EpochLearn) ----
GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def epoch_checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("elearn") / "epoch_learn_check")
    src = [os.path.join(ROOT, "tests", "epoch_learn_check.cpp")] + \
          [os.path.join(CSRC, f) for f in ("ingest.cpp", "gen.cpp", "gen_faulty.cpp", "gen_member.cpp")]
    subprocess.run(["g++", "-O2", "-std=c++17", "-I" + CSRC, "-I" + os.path.join(ROOT, "include")] + src +
                   ["-o", exe], check=True, timeout=600)
    return exe


MEMBER_GOLDENS = sorted(f[:-5] for f in os.listdir(GOLD) if f.endswith(".mpxt") and f.startswith(("mm_", "c5_")))


@pytest.mark.parametrize("name", MEMBER_GOLDENS)
@pytest.mark.parametrize("windows", [1, 3])
def test_learned_epochs_match_reference_markers(epoch_checker, name, windows):
    """The engine's own E_EPOCH records (a node's Learner applying a membership Value in instance
    order, member/paxos.cpp:1040-1073,1864-1964) land where the trace's markers are — which the
    reference driver checks against the reference's own ChangeMemberships — with the same epochs,
    whole and with the learner state carried over windows; the learned table is the container's."""
    r = subprocess.run([epoch_checker, os.path.join(GOLD, name + ".mpxt"), str(windows)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
    assert int(r.stdout.split()[2]) > 0


@pytest.mark.parametrize("lg,proposers,windows", [(16, 0, 4), (15, 3, 5)])
def test_learned_epochs_on_generated_c5(epoch_checker, lg, proposers, windows):
    r = subprocess.run([epoch_checker, "gen", str(lg), str(proposers), str(windows)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
    assert int(r.stdout.split()[3]) == 15          # every step of the C5 schedule learned


# ---- chunked multi-threaded decode (ingest.cpp decode_parallel, submit_container) ----
@pytest.fixture(scope="module")
def par_checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("pdec") / "parallel_decode_check")
    src = [os.path.join(ROOT, "tests", "parallel_decode_check.cpp")] + \
          [os.path.join(CSRC, f) for f in ("ingest.cpp", "gen.cpp", "gen_faulty.cpp", "gen_member.cpp")]
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I" + CSRC, "-I" + os.path.join(ROOT, "include")] + src +
                   ["-o", exe], check=True, timeout=600)
    return exe


@pytest.mark.parametrize("kind,lg,proposers,chunk,threads", [("faulty", 15, 3, 4096, 5), ("faulty", 14, 0, 1 << 16, 8),
                                                             ("member", 14, 3, 2048, 6), ("member", 13, 0, 512, 3)])
def test_parallel_decode_equals_serial_generated(par_checker, kind, lg, proposers, chunk, threads):
    """decode_parallel (a node's stream in chunks on a thread pool, later chunks appended with their
    entry offsets rebased) gives the serial decode array for array, after records already queued."""
    r = subprocess.run([par_checker, kind, str(lg), str(proposers), str(chunk), str(threads)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok "), r.stdout + r.stderr
    assert int(r.stdout.split()[2]) > 1          # several chunks per node


def test_parallel_decode_equals_serial_goldens(par_checker):
    for f in sorted(os.listdir(GOLD)):
        if f.endswith(".mpxt"):
            r = subprocess.run([par_checker, os.path.join(GOLD, f), "0", "0", "64", "4"], capture_output=True,
                               text=True, timeout=120)
            assert r.returncode == 0 and r.stdout.startswith("ok"), f + ": " + r.stdout + r.stderr


def test_parallel_decode_violations_in_record_order(par_checker, tmp_path):
    """Duplicate iids (MPX_V_DUP_IID, the reference ASSERTs) in later chunks of several nodes: the
    first violation (node, record index) and the count are the serial decode's."""
    import mpxwire as w
    streams = []
    for n in range(3):
        s = [w.accept(0, k, 5, [(2 * k, w.value(0, 2 * k + 1, "x" * 40)), (2 * k + 1, w.value(0, 2 * k + 2, "y"))])
             for k in range(60)]
        if n:
            s[40 + n] = w.accept(0, 99, 5, [(7, w.value(0, 500, "a")), (7, w.value(0, 501, "b"))])
            s[50] = w.prepare(1, 9, ((0, 10), (0, 10)))
        streams.append(s)
    p = tmp_path / "dup.mpxt"
    p.write_bytes(w.container(streams, 256))
    r = subprocess.run([par_checker, str(p), "0", "0", "256", "4"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.startswith("ok "), r.stdout + r.stderr
    assert int(r.stdout.split()[3]) == 4


# ---- node-parallel build (ingest.cpp build_trace vs build_trace_serial) ----
@pytest.fixture(scope="module")
def build_checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("bchk") / "build_check")
    src = [os.path.join(ROOT, "tests", "build_check.cpp")] + \
          [os.path.join(CSRC, f) for f in ("ingest.cpp", "gen.cpp", "gen_faulty.cpp", "gen_member.cpp")]
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I" + CSRC, "-I" + os.path.join(ROOT, "include")] + src +
                   ["-o", exe], check=True, timeout=600)
    return exe


@pytest.mark.parametrize("kind,lg,proposers,windows,threads,shard", [
    ("faulty", 15, 3, 1, 4, 0), ("faulty", 15, 3, 6, 8, 0), ("faulty", 14, 2, 3, 3, 1), ("faulty", 14, 0, 2, 2, 0),
    ("member", 14, 3, 1, 4, 0), ("member", 14, 3, 5, 6, 1), ("member", 13, 0, 3, 3, 0)])
def test_parallel_build_equals_serial_generated(build_checker, kind, lg, proposers, windows, threads, shard):
    """build_trace's node-parallel walk (per-node parts rebased, the entry pool's first occurrences
    found per hash shard) gives build_trace_serial's HostTrace field for field — whole, window by
    window with the carry, and on a shard of the instances."""
    r = subprocess.run([build_checker, kind, str(lg), str(proposers), str(windows), str(threads), str(shard)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok "), r.stdout + r.stderr


def test_parallel_build_equals_serial_goldens(build_checker):
    for f in sorted(os.listdir(GOLD)):
        if not f.endswith(".mpxt"):
            continue
        for args in (("0", "0", "1", "3", "0"), ("0", "0", "3", "3", "0"), ("0", "0", "2", "2", "1")):
            r = subprocess.run([build_checker, os.path.join(GOLD, f)] + list(args), capture_output=True, text=True,
                               timeout=120)
            assert r.returncode == 0 and r.stdout.startswith("ok"), f + " %r: " % (args,) + r.stdout + r.stderr
