"""CPU-side checks of the C ABI library (no compute calls without a GPU)."""
import ctypes

import pytest

import mpx
from oracles import oracle_run, ref_available, ref_run
import mpxr


def test_library_exports_every_declared_symbol():
    L = mpx.lib()
    declared = mpx.declared_symbols()
    assert len(declared) >= 25
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing


def test_abi_version():
    assert mpx.lib().mpx_version() == mpx.ABI_VERSION


def test_create_rejects_bad_config():
    L = mpx.lib()
    h = ctypes.c_void_p()
    cfg = mpx.Config(999, 5, 0, 0, 0, 10, 0, 0, None)
    assert L.mpx_create(ctypes.byref(cfg), ctypes.byref(h)) == -1
    cfg = mpx.Config(mpx.ABI_VERSION, 0, 0, 0, 0, 10, 0, 0, None)
    assert L.mpx_create(ctypes.byref(cfg), ctypes.byref(h)) == -1
    cfg = mpx.Config(mpx.ABI_VERSION, 65, 0, 0, 0, 10, 0, 0, None)
    assert L.mpx_create(ctypes.byref(cfg), ctypes.byref(h)) == -1


def test_no_cpu_fallback_without_gpu():
    if mpx.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(mpx.MpxError) as ei:
        mpx.Engine(5, 0, 1024)
    assert ei.value.rc == -7          # MPX_E_NODEVICE: the engine never runs on the CPU


@pytest.mark.parametrize("n,m,b", [(1, 1, 256), (3, 300, 256), (5, 1000, 64), (9, 777, 100)])
def test_clean_generator_is_valid_for_the_oracle(n, m, b):
    t = mpx.generate_trace(mpx.GEN_CLEAN, num_nodes=n, num_instances=m, batch=b)
    res, stats, viol = oracle_run(t)
    C, P, A, L_, V = stats[:5]
    assert (C, P, A, L_, V) == (m, 0, n * m, n * m, 0)
    parsed = mpxr.parse(res)
    assert parsed["chosen"][0] == (0, mpx.lib() and (1 << 48) * 0 + 1)
    for nd in parsed["nodes"]:
        assert nd["promised"] == 1 << 16 and nd["max_seen"] == 1 << 16
        assert len(nd["state"]) == m and all(s[1] == 2 and s[2] == 1 << 16 for s in nd["state"])
        assert nd["executed"] == [str(i).encode() for i in range(m)]


@pytest.mark.ref
@pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built (needs /root/reference)")
def test_clean_generator_matches_reference():
    t = mpx.generate_trace(mpx.GEN_CLEAN, num_nodes=5, num_instances=2000, batch=256)
    a, sa, _ = oracle_run(t)
    b, sb = ref_run(t)
    assert a == b, mpxr.diff(a, b)
    assert sa[:4] == sb
