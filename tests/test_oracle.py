"""The CPU restatement (oracle/mpx_oracle.c) against the reference.

* every committed golden fixture: oracle(trace) == reference(trace) byte for byte
  (the .mpxr files were written by the reference's own handlers, make_golden.py);
* where oracle/_ref exists (this container): fresh random traces, oracle vs the
  reference driven live;
* the reference's own UNITTEST codec vectors (multi/paxos.cpp:1753-1777).
"""
import json
import os
import struct

import pytest

import mpxr
from fuzztrace import fuzz_trace
from mpxwire import container, value
from oracles import oracle_run, ref_available, ref_run

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
INDEX = json.load(open(os.path.join(GOLD, "index.json")))


def _read(name, ext):
    with open(os.path.join(GOLD, name + ext), "rb") as f:
        return f.read()


@pytest.mark.parametrize("name", sorted(INDEX))
def test_oracle_matches_reference_golden(name):
    trace, want = _read(name, ".mpxt"), _read(name, ".mpxr")
    got, stats, viol = oracle_run(trace)
    assert got == want, mpxr.diff(got, want)
    meta = INDEX[name]
    assert stats[:4] == [meta["C"], meta["P"], meta["A"], meta["L"]]


def test_codec_unittest_vectors():
    # multi/paxos.cpp:1753-1777: Value(1,2) encodes to 13 bytes, Value(1,2,"123") to 21
    assert len(value(1, 2, noop=True)) == 13
    assert len(value(1, 2, "123")) == 21
    assert value(1, 2, "123") == struct.pack("<IQ??I", 1, 2, False, False, 3) + b"123"


@pytest.mark.ref
@pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("seed", range(100, 160))
def test_oracle_matches_reference_live(seed):
    trace = fuzz_trace(seed)
    got, stats, _ = oracle_run(trace)
    want, rstats = ref_run(trace)
    assert got == want, mpxr.diff(got, want)
    assert stats[:4] == rstats


def test_oracle_rejects_unknown_type():
    with pytest.raises(RuntimeError):
        oracle_run(container([[struct.pack("<I", 9)]], 1))
