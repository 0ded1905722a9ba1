"""ctypes loaders for the parity checkers (TEST INFRASTRUCTURE).

  oracle/_build/libmpx_oracle.so : C restatement (oracle/mpx_oracle.c)
  oracle/_ref/libmpx_ref.so      : the reference's own handlers (oracle/ref_multi_driver.cpp)
  oracle/_ref/libmpx_ref_member.so : the same for member/paxos.cpp (oracle/ref_member_driver.cpp)

Both take an MPXT trace and return the canonical MPXR result bytes.
"""
import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "libmpx_oracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libmpx_ref.so")
REF_MEMBER_SO = os.path.join(ROOT, "oracle", "_ref", "libmpx_ref_member.so")

_u8p = ctypes.POINTER(ctypes.c_uint8)


def _load(path, fn):
    lib = ctypes.CDLL(path)
    f = getattr(lib, fn)
    return lib, f


class _Runner:
    def __init__(self, path, fn, nstats, has_viol):
        self.lib = ctypes.CDLL(path)
        self.fn = getattr(self.lib, fn)
        self.nstats = nstats
        self.has_viol = has_viol
        argt = [ctypes.c_char_p, ctypes.c_uint64, ctypes.POINTER(_u8p),
                ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        if has_viol:
            argt.append(ctypes.POINTER(ctypes.c_uint64))
        self.fn.argtypes = argt
        self.fn.restype = ctypes.c_int
        self.libc = ctypes.CDLL(None)
        self.libc.free.argtypes = [ctypes.c_void_p]

    def __call__(self, trace):
        out = _u8p()
        size = ctypes.c_uint64()
        stats = (ctypes.c_uint64 * 8)()
        args = [trace, len(trace), ctypes.byref(out), ctypes.byref(size), stats]
        viol = (ctypes.c_uint64 * 4)()
        if self.has_viol:
            args.append(viol)
        rc = self.fn(*args)
        if rc != 0:
            raise RuntimeError("%s failed: %d" % (self.fn.__name__, rc))
        addr = ctypes.cast(out, ctypes.c_void_p).value
        data = bytes(memoryview((ctypes.c_char * size.value).from_address(addr))) if size.value else b""
        self.libc.free(out)
        return data, list(stats)[: self.nstats], list(viol)


_oracle = None
_ref = None
_ref_member = None


def oracle_run(trace):
    """-> (mpxr bytes, [C,P,A,L,V,chosen_digest,state_digest,scalar_digest], violation[4])"""
    global _oracle
    if _oracle is None:
        _oracle = _Runner(ORACLE_SO, "mpxo_run", 8, True)
    return _oracle(trace)


def ref_available():
    return os.path.exists(REF_SO) and os.path.exists(REF_MEMBER_SO)


def ref_run(trace):
    """-> (mpxr bytes, [C,P,A,L]); multi or member driver by the trace's semantics"""
    global _ref, _ref_member
    if trace[12:16] == b"\x01\x00\x00\x00":
        if _ref_member is None:
            _ref_member = _Runner(REF_MEMBER_SO, "mpxref_member_run", 4, False)
        data, stats, _ = _ref_member(trace)
        return data, stats
    if _ref is None:
        _ref = _Runner(REF_SO, "mpxref_run", 4, False)
    data, stats, _ = _ref(trace)
    return data, stats


_sharded = None


def oracle_run_sharded(trace, shards=16, threads=None):
    """Counters + digests of the whole trace from `shards` instance shards of
    the CPU oracle on host threads (oracle mpxo_run_sharded: instances are
    independent given the replicated headers, so counters / digests add and
    per-node scalars agree) -> [C,P,A,L,V,chosen_digest,state_digest,scalar_digest]."""
    global _sharded
    if _sharded is None:
        lib = ctypes.CDLL(ORACLE_SO)
        f = lib.mpxo_run_sharded
        f.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                      ctypes.POINTER(ctypes.c_uint64)]
        f.restype = ctypes.c_int
        _sharded = (lib, f)
    threads = threads or max(1, min(16, os.cpu_count() or 1))
    stats = (ctypes.c_uint64 * 8)()
    rc = _sharded[1](trace, len(trace), shards, threads, stats)
    if rc != 0:
        raise RuntimeError("mpxo_run_sharded failed: %d" % rc)
    return list(stats)


def _blob_call(so, fn, trace):
    lib = ctypes.CDLL(so)
    f = getattr(lib, fn)
    f.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)),
                  ctypes.POINTER(ctypes.c_uint64)]
    f.restype = ctypes.c_int
    out = ctypes.POINTER(ctypes.c_uint8)()
    size = ctypes.c_uint64()
    rc = f(bytes(trace), len(trace), ctypes.byref(out), ctypes.byref(size))
    if rc != 0:
        raise RuntimeError("%s failed: %d" % (fn, rc))
    data = ctypes.string_at(out, size.value)
    ctypes.CDLL(None).free(out)
    return data


def ref_decisions(trace):
    """The reference's own phase-2 batch at every promise quorum (MPXD; multi semantics),
    recorded by oracle/ref_multi_driver.cpp (mpxref_decisions)."""
    return _blob_call(REF_SO, "mpxref_decisions", trace)


def oracle_decisions(trace):
    """The oracle's restatement of the same decisions (mpxo_decisions)."""
    return _blob_call(ORACLE_SO, "mpxo_decisions", trace)


def ref_commits(trace):
    """The reference's own CommittingValues bookkeeping (MPXC; multi semantics):
    creation at accept / promise quorums, OnCommitReply retirement, replied masks
    (oracle/ref_multi_driver.cpp mpxref_commits)."""
    return _blob_call(REF_SO, "mpxref_commits", trace)


def ref_member_decisions(trace):
    """The reference's own member phase-2 batch at every promise quorum (MPXD),
    recorded by oracle/ref_member_driver.cpp (mpxref_member_decisions)."""
    return _blob_call(REF_MEMBER_SO, "mpxref_member_decisions", trace)


def ref_learns(trace):
    """The reference's own member LearningValues bookkeeping (MPXL): creation at accept /
    promise quorums and LearnersChanged, Applied, OnLearnReply retirement, drops
    (oracle/ref_member_driver.cpp mpxref_member_learns)."""
    return _blob_call(REF_MEMBER_SO, "mpxref_member_learns", trace)


def ref_callbacks(trace):
    """Every Callback call the REFERENCE's member nodes made — Accepted, Applied, Unproposable — as
    MPXB (oracle/ref_member_driver.cpp mpxref_member_callbacks; parse: tests/mpxb.py)."""
    return _blob_call(REF_MEMBER_SO, "mpxref_member_callbacks", trace)


def oracle_commits(trace):
    """The oracle's restatement of the same bookkeeping (mpxo_commits)."""
    return _blob_call(ORACLE_SO, "mpxo_commits", trace)


_ref_shard = {}


def ref_run_shards(trace, shards):
    """Counters + digests of a trace from the REFERENCE's own handlers, summed over `shards`
    instance shards (oracle/_ref mpxref_run_shard / mpxref_member_run_shard: each shard's entries
    only, every record's header; oracle/ref_full_size.py runs them at full size) ->
    [C,P,A,L,0,chosen_digest,state_digest,scalar_digest] (the reference counts no violations)."""
    member = trace[12:16] == b"\x01\x00\x00\x00"
    name = "mpxref_member_run_shard" if member else "mpxref_run_shard"
    if name not in _ref_shard:
        f = getattr(ctypes.CDLL(REF_MEMBER_SO if member else REF_SO), name)
        f.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                      ctypes.POINTER(ctypes.c_uint64)]
        f.restype = ctypes.c_int
        _ref_shard[name] = f
    m = int.from_bytes(bytes(trace[16:24]), "little")
    per = -(-m // shards)
    tot, scal = [0] * 8, None
    for k in range(shards):
        st = (ctypes.c_uint64 * 8)()
        se = (k + 1) * per if k + 1 < shards else (1 << 64) - 1
        rc = _ref_shard[name](trace, len(trace), k * per, se, st)
        if rc != 0:
            raise RuntimeError("%s failed: %d" % (name, rc))
        for w in range(7):
            tot[w] = (tot[w] + st[w]) % (1 << 64)
        if scal is not None and scal != st[7]:
            raise RuntimeError("per-node scalars differ between shards")
        scal = st[7]
    tot[7] = scal
    return tot
