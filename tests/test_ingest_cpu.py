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
    runs, aliased, marked = map(int, r.stdout.split()[1:4])
    assert runs > 0
    if kind == "faulty":
        assert aliased > 0          # competing proposers' re-commits of equal Values share entries


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
