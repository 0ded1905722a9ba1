"""Member proposer bookkeeping — learn reliability and phase-2 decisions
(f2): the Python restatements of the engine's algorithms (oracle/learns_model.py,
oracle/member_decisions_model.py) against the reference's own bookkeeping — CPU only."""
import json
import os
import struct

import pytest

import learns_model
import member_decisions_model
import mpxl

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
LEARNS = json.load(open(os.path.join(GOLD, "learns.json")))


def _read(name, ext):
    with open(os.path.join(GOLD, name + ext), "rb") as f:
        return f.read()


@pytest.mark.parametrize("name", sorted(LEARNS))
def test_learns_model_matches_reference_golden(name):
    """learns_model over the trace and its reference MPXR (promise quorums, chosen batches)
    == the reference Proposer's learning_values_ bookkeeping (.mpxl fixture)."""
    assert learns_model.learns(_read(name, ".mpxt"), _read(name, ".mpxr")) == _read(name, ".mpxl")


def test_learn_fixtures_cover_every_outcome():
    """Across the fixtures: all three creation kinds, Applied, retirement, drops, a learn
    retired by a non-learner's reply (|learned_| == |learners_|, :1373) and a learner-only
    epoch change (learner_mask != proposer_mask)."""
    rows = [r for n in sorted(LEARNS) for x in mpxl.parse(_read(n, ".mpxl")) for r in x]
    assert {r[2] for r in rows} == {0, 1, 2}
    assert any(r[4] != mpxl.NONE for r in rows) and any(r[5] != mpxl.NONE for r in rows)
    assert any(r[6] != mpxl.NONE for r in rows)
    lm = [r for r in mpxl.parse(_read("mm_learners", ".mpxl"))[0]]
    assert any(r[5] != mpxl.NONE and bin(r[7]).count("1") == 3 and not (r[7] >> 3) & 1 for r in lm)
    t = _read("mm_learners", ".mpxt")
    ne = struct.unpack_from("<I", t, 24)[0]
    assert struct.unpack_from("<I", t, 4)[0] == 2
    assert any(struct.unpack_from("<Q", t, 40 + 32 * i + 16) != struct.unpack_from("<Q", t, 40 + 32 * i + 24)
               for i in range(ne))


DECISIONS = json.load(open(os.path.join(GOLD, "decisions.json")))


@pytest.mark.parametrize("name", sorted(n for n in DECISIONS if n.startswith(("mm_", "c5_"))))
def test_member_decisions_model_matches_reference_golden(name):
    """member_decisions_model over the trace and its reference MPXR (promise quorums and their
    merged maps) == the batch the reference's member OnPrepareReply built (.mpxd fixture)."""
    assert member_decisions_model.decisions(_read(name, ".mpxt"), _read(name, ".mpxr")) == _read(name, ".mpxd")
