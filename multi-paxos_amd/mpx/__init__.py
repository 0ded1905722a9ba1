"""ctypes binding of libmpx.so (include/mpx.h) — the host mirror used by the
tests, bench.py and __graft_entry__.

The reference's host drives its protocol core through NetWork::OnReceiveMessage
/ SendMessage* / StateMachine::Execute (multi/paxos.h:193-222); `Engine`
exposes the batched equivalents: submit (OnReceiveMessage), run, drain_sends
(SendMessage*), dump (canonical result) and the state readbacks.

There is no Python or CPU fallback: without the built library or without a
GPU every compute call raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(HERE), "lib", "libmpx.so")
if os.environ.get("MPX_LIB_VARIANT"):         # A/B builds of the same sources (tools/ab_*.sh)
    LIB_PATH = os.path.join(os.path.dirname(HERE), "lib_" + os.environ["MPX_LIB_VARIANT"], "libmpx.so")
INCLUDE_H = os.path.join(os.path.dirname(os.path.dirname(HERE)), "include", "mpx.h")

ABI_VERSION = 2
SEM_MULTI, SEM_MEMBER = 0, 1
FLAG_INCREMENTAL = 1            # mpx_config.flags: each mpx_run applies one window (include/mpx.h)
FLAG_DECISIONS = 2              # with FLAG_INCREMENTAL: decisions carried across windows
FLAG_LEARN_EPOCHS = 4           # member: roles from the applied membership Values (include/mpx.h)
GEN_CLEAN, GEN_FAULTY, GEN_MEMBER = 0, 1, 2
PRESENT = 1 << 63
UID_BYTES = 128

ERRORS = {0: "OK", -1: "E_INVAL", -2: "E_NOMEM", -3: "E_HIP", -4: "E_DECODE", -5: "E_RANGE",
          -6: "E_STATE", -7: "E_NODEVICE", -8: "E_COMM", -9: "E_VALUE"}


class MpxError(RuntimeError):
    def __init__(self, fn, rc):
        super().__init__("%s failed: %s (%d)" % (fn, ERRORS.get(rc, "?"), rc))
        self.rc = rc


class LoopStats(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint64) for k in ("windows", "records", "batches", "committed_batches",
                                               "committed_instances", "proposed", "submit_ns", "run_ns",
                                               "drain_ns")]


class Epoch(ctypes.Structure):
    _fields_ = [("version", ctypes.c_uint32), ("flags", ctypes.c_uint32), ("acceptor_mask", ctypes.c_uint64),
                ("proposer_mask", ctypes.c_uint64), ("learner_mask", ctypes.c_uint64)]


class Config(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_uint32), ("num_nodes", ctypes.c_uint32),
                ("semantics", ctypes.c_uint32), ("device", ctypes.c_int32),
                ("shard_begin", ctypes.c_uint64), ("shard_end", ctypes.c_uint64),
                ("num_epochs", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("epochs", ctypes.POINTER(Epoch))]


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "chosen", "promise_entries", "accept_apps", "commit_apps", "messages", "violations",
        "chosen_digest", "state_digest", "scalar_digest", "device_ns", "apply_ns", "ingest_ns",
        "bytes_alg", "skipped", "general_pairs", "num_runs", "slot_bytes", "r2")]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_ if not f.startswith("r")}


class SoaRecords(ctypes.Structure):
    _fields_ = [("count", ctypes.c_uint64), ("type", ctypes.POINTER(ctypes.c_uint8)),
                ("src", ctypes.POINTER(ctypes.c_uint32)), ("ballot", ctypes.POINTER(ctypes.c_uint64)),
                ("aux", ctypes.POINTER(ctypes.c_uint64)), ("ent_off", ctypes.POINTER(ctypes.c_uint64)),
                ("ent_a", ctypes.POINTER(ctypes.c_uint64)), ("ent_b", ctypes.POINTER(ctypes.c_uint64)),
                ("ent_pid", ctypes.POINTER(ctypes.c_uint64))]


class Violation(ctypes.Structure):
    _fields_ = [("code", ctypes.c_uint64), ("node", ctypes.c_uint32), ("pad", ctypes.c_uint32),
                ("seq", ctypes.c_uint64), ("iid", ctypes.c_uint64)]


class GenParams(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint32), ("num_nodes", ctypes.c_uint32),
                ("num_instances", ctypes.c_uint64), ("seed", ctypes.c_uint64),
                ("batch", ctypes.c_uint32), ("proposers", ctypes.c_uint32),
                ("drop_rate", ctypes.c_uint32), ("dup_rate", ctypes.c_uint32),
                ("max_delay", ctypes.c_uint32), ("noop_permille", ctypes.c_uint32),
                ("shard_begin", ctypes.c_uint64), ("shard_end", ctypes.c_uint64)]


SEND_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                           ctypes.POINTER(ctypes.c_uint8), ctypes.c_uint32)

_lib = None


def lib():
    """Load libmpx.so (raises if it was not built: no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError("libmpx.so not built: run `make -C multi-paxos_amd` (%s)" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        P = ctypes.POINTER
        u8p, u64p = P(ctypes.c_uint8), P(ctypes.c_uint64)
        vp = ctypes.c_void_p
        sig = {
            "mpx_version": [],
            "mpx_device_count": [P(ctypes.c_int)],
            "mpx_create": [P(Config), P(vp)],
            "mpx_destroy": [vp],
            "mpx_submit": [vp, ctypes.c_uint32, ctypes.c_char_p, u64p, ctypes.c_uint64],
            "mpx_submit_trace": [vp, ctypes.c_char_p, ctypes.c_uint64],
            "mpx_submit_trace_range": [vp, ctypes.c_char_p, ctypes.c_uint64, u64p, u64p],
            "mpx_submit_trace_range_async": [vp, ctypes.c_char_p, ctypes.c_uint64, u64p, u64p],
            "mpx_submit_soa": [vp, ctypes.c_uint32, P(SoaRecords)],
            "mpx_run": [vp], "mpx_reset_state": [vp], "mpx_step": [vp], "mpx_sync": [vp],
            "mpx_timings": [vp, ctypes.c_uint32, P(ctypes.c_double), P(ctypes.c_double), P(ctypes.c_uint32)],
            "mpx_timings_detail": [vp, ctypes.c_uint32, P(ctypes.c_double), P(ctypes.c_uint32)],
            "mpx_timing_every": [vp, ctypes.c_uint32],
            "mpx_drain_sends": [vp, SEND_FN, vp],
            "mpx_read_chosen": [vp, ctypes.c_uint64, ctypes.c_uint64, u64p],
            "mpx_read_epochs": [vp, P(Epoch), ctypes.c_uint32, P(ctypes.c_uint32)],
            "mpx_read_node_scalars": [vp, ctypes.c_uint32, u64p, u64p],
            "mpx_read_executed": [vp, ctypes.c_uint32, u64p, u64p, u64p, ctypes.c_uint64],
            "mpx_read_node_state": [vp, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, u64p, u64p, u64p, u64p],
            "mpx_stats_get": [vp, P(Stats)],
            "mpx_state_digest": [vp, u64p, u64p],
            "mpx_last_violation": [vp, P(Violation)],
            "mpx_dump_result": [vp, P(u8p), u64p],
            "mpx_read_decisions": [vp, P(u8p), u64p],
            "mpx_read_commits": [vp, P(u8p), u64p],
            "mpx_read_learns": [vp, P(u8p), u64p],
            "mpx_read_learn_values": [vp, P(u8p), u64p],
            "mpx_proposal_part": [vp, P(u8p), u64p],
            "mpx_proposal_combine": [P(u8p), u64p, ctypes.c_uint32, P(u8p), u64p],
            "mpx_decisions_bounds": [vp, u64p, ctypes.c_uint64, u64p],
            "mpx_read_decisions_part": [vp, u64p, ctypes.c_uint64, P(u8p), u64p],
            "mpx_decisions_combine": [P(u8p), u64p, ctypes.c_uint32, P(u8p), u64p],
            "mpx_value_bytes": [vp, ctypes.c_uint64, u8p, ctypes.c_uint32, P(ctypes.c_uint32)],
            "mpx_trace_generate": [P(GenParams), P(u8p), u64p],
            "mpx_load_clean_device": [vp, P(GenParams)],
            "mpx_comm_unique_id": [u8p],
            "mpx_comm_init": [vp, u8p, ctypes.c_int, ctypes.c_int],
            "mpx_allgather_summary": [vp, u64p],
            "mpx_comm_allreduce_max": [vp, u64p, ctypes.c_uint64],
            "mpx_comm_allgather_bytes": [vp, ctypes.c_char_p, ctypes.c_uint64, P(u8p), u64p],
            "mpx_read_decisions_sharded": [vp, P(u8p), u64p],
            "mpx_commit_points": [vp, P(u8p), u64p],
            "mpx_commit_points_combine": [P(u8p), u64p, ctypes.c_uint32, P(u8p), u64p],
            "mpx_read_commits_at": [vp, ctypes.c_char_p, ctypes.c_uint64, P(u8p), u64p],
            "mpx_read_commits_sharded": [vp, P(u8p), u64p],
            "mpx_loop_create": [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, P(vp)],
            "mpx_loop_destroy": [vp],
            "mpx_loop_prepare": [vp, ctypes.c_uint32, ctypes.c_uint64],
            "mpx_loop_propose": [vp, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32],
            "mpx_loop_step": [vp],
            "mpx_loop_accept_decided": [vp, ctypes.c_uint32, ctypes.c_uint64, u64p],
            "mpx_loop_commit_chosen": [vp, ctypes.c_uint32, ctypes.c_uint64, P(ctypes.c_uint32)],
            "mpx_loop_leader_rounds": [vp, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32],
            "mpx_loop_stats_get": [vp, P(LoopStats)],
            "mpx_loop_trace": [vp, P(u8p), u64p],
        }
        for name, args in sig.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = ctypes.c_int
        L.mpx_loop_engine.argtypes = [vp]
        L.mpx_loop_engine.restype = vp
        L.mpx_free.argtypes = [vp]
        L.mpx_free.restype = None
        _lib = L
    return _lib


def _ck(name, rc):
    if rc != 0:
        raise MpxError(name, rc)


def device_count():
    n = ctypes.c_int(0)
    _ck("mpx_device_count", lib().mpx_device_count(ctypes.byref(n)))
    return n.value


def _take(ptr, size):
    # (ctypes.string_at takes a C int size: traces of C3 / C5 at full size exceed 2^31 bytes)
    addr = ctypes.cast(ptr, ctypes.c_void_p).value
    data = bytes(memoryview((ctypes.c_char * size).from_address(addr))) if size else b""
    lib().mpx_free(ptr)
    return data


def generate_trace(kind=GEN_CLEAN, num_nodes=5, num_instances=1 << 10, seed=0, batch=256,
                   proposers=1, drop_rate=0, dup_rate=0, max_delay=0, noop_permille=0,
                   shard_begin=0, shard_end=0, copy=True):
    """Deterministic synthetic MPXT trace (host generator in libmpx).  copy=False
    returns the generator's own buffer as a ctypes char array (len, slicing, the
    buffer protocol and every c_char_p argument accept it; freed when collected):
    C3 / C5 at full size are 15-20 GB, and a bytes copy would double that."""
    p = GenParams(kind, num_nodes, num_instances, seed, batch, proposers, drop_rate, dup_rate,
                  max_delay, noop_permille, shard_begin, shard_end)
    out = ctypes.POINTER(ctypes.c_uint8)()
    size = ctypes.c_uint64()
    _ck("mpx_trace_generate", lib().mpx_trace_generate(ctypes.byref(p), ctypes.byref(out), ctypes.byref(size)))
    if copy:
        return _take(out, size.value)
    import weakref
    addr = ctypes.cast(out, ctypes.c_void_p).value
    arr = (ctypes.c_char * size.value).from_address(addr)
    weakref.finalize(arr, lib().mpx_free, addr)
    return arr


def trace_header(trace):
    import struct
    assert trace[:4] == b"MPXT"
    ver, n, sem, m = struct.unpack_from("<IIIQ", trace, 4)
    return {"num_nodes": n, "semantics": sem, "num_instances": m, "version": ver}


def trace_epochs(trace):
    """The container's epoch table: [(version, acceptor_mask, proposer_mask, learner_mask)]
    (version-1 containers: 24-byte entries, learner_mask = proposer_mask)."""
    import struct
    ver, ne = struct.unpack_from("<I", trace, 4)[0], struct.unpack_from("<I", trace, 24)[0]
    esz = 24 if ver == 1 else 32
    out = []
    for i in range(ne):
        v, a, p = struct.unpack_from("<IxxxxQQ", trace, 40 + esz * i)
        out.append((v, a, p, struct.unpack_from("<Q", trace, 40 + esz * i + 24)[0] if esz == 32 else p))
    return out


def _addr(buf):
    """Address of a bytes object's or ctypes array's data (valid while `buf` lives)."""
    if isinstance(buf, bytes):
        return ctypes.cast(ctypes.c_char_p(buf), ctypes.c_void_p).value
    return ctypes.addressof(buf)


def trace_index(trace):
    """Per node of an MPXT container: (record count, byte offset of its offsets array, byte
    offset of its record bytes) — what Engine.submit_range needs."""
    import struct
    hd = trace_header(trace)
    ne = struct.unpack_from("<I", trace, 24)[0]
    pos = 40 + (24 if hd["version"] == 1 else 32) * ne
    out = []
    for _ in range(hd["num_nodes"]):
        cnt, nb = struct.unpack_from("<QQ", trace, pos)
        out.append((cnt, pos + 16, pos + 16 + 8 * (cnt + 1)))
        pos = (pos + 16 + 8 * (cnt + 1) + nb + 7) & ~7
    return out


class Engine:
    """One engine = one GPU, one instance shard [shard_begin, shard_end)."""

    def __init__(self, num_nodes, shard_begin=0, shard_end=None, device=0, semantics=SEM_MULTI, epochs=(), flags=0):
        L = lib()
        if shard_end is None:
            raise ValueError("shard_end required")
        # epochs: (version, acceptor_mask, proposer_mask[, learner_mask = proposer_mask])
        self._epochs = (Epoch * max(len(epochs), 1))(*[Epoch(x[0], 0, x[1], x[2], x[3] if len(x) > 3 else x[2])
                                                        for x in epochs])
        cfg = Config(ABI_VERSION, num_nodes, semantics, device, shard_begin, shard_end,
                     len(epochs), flags, self._epochs if epochs else None)
        h = ctypes.c_void_p()
        _ck("mpx_create", L.mpx_create(ctypes.byref(cfg), ctypes.byref(h)))
        self.h = h
        self.num_nodes = num_nodes
        self.shard_begin, self.shard_end = shard_begin, shard_end

    @classmethod
    def for_trace(cls, trace, device=0, flags=0):
        """An engine for a whole MPXT trace.  flags FLAG_LEARN_EPOCHS (member): created with the
        container's genesis epoch only; the engine learns the rest and ignores the container's
        E_EPOCH records."""
        hd = trace_header(trace)
        epochs = trace_epochs(trace)[:1] if flags & FLAG_LEARN_EPOCHS else ()
        e = cls(hd["num_nodes"], 0, max(hd["num_instances"], 1), device=device, semantics=hd["semantics"],
                epochs=epochs, flags=flags)
        e.submit_trace(trace)
        return e

    def epochs(self):
        """The member epoch table [(version, acceptor_mask, proposer_mask, learner_mask)] (mpx_read_epochs)."""
        n = ctypes.c_uint32()
        _ck("mpx_read_epochs", lib().mpx_read_epochs(self.h, None, 0, ctypes.byref(n)))
        arr = (Epoch * max(n.value, 1))()
        _ck("mpx_read_epochs", lib().mpx_read_epochs(self.h, arr, n.value, ctypes.byref(n)))
        return [(x.version, x.acceptor_mask, x.proposer_mask, x.learner_mask) for x in arr[: n.value]]

    def close(self):
        if self.h:
            lib().mpx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # inbound
    def submit(self, node, messages):
        blob = b"".join(messages)
        offs = [0]
        for m in messages:
            offs.append(offs[-1] + len(m))
        arr = (ctypes.c_uint64 * len(offs))(*offs)
        _ck("mpx_submit", lib().mpx_submit(self.h, node, blob, arr, len(messages)))

    def submit_soa(self, node, records):
        """mpx_submit_soa: records as (type, src, ballot, aux, entries), entries (a, b[, pid])
        — {iid, handle} / {iid, handle, pid} / PREPARE ranges {start, end}."""
        n = len(records)
        offs, ea, eb, ep = [0], [], [], []
        for r in records:
            for x in r[4]:
                ea.append(x[0]); eb.append(x[1]); ep.append(x[2] if len(x) > 2 else 0)
            offs.append(len(ea))
        arr = lambda t, v: (t * max(len(v), 1))(*v)
        keep = [arr(ctypes.c_uint8, [r[0] for r in records]), arr(ctypes.c_uint32, [r[1] for r in records]),
                arr(ctypes.c_uint64, [r[2] for r in records]), arr(ctypes.c_uint64, [r[3] for r in records]),
                arr(ctypes.c_uint64, offs), arr(ctypes.c_uint64, ea), arr(ctypes.c_uint64, eb),
                arr(ctypes.c_uint64, ep)]
        rec = SoaRecords(n, *[ctypes.cast(k, ctypes.POINTER(k._type_)) for k in keep])   # keep: alive for the call
        _ck("mpx_submit_soa", lib().mpx_submit_soa(self.h, node, ctypes.byref(rec)))

    def submit_trace(self, trace):
        _ck("mpx_submit_trace", lib().mpx_submit_trace(self.h, trace, len(trace)))

    def submit_window(self, trace, begin, end):
        """mpx_submit_trace_range: records [begin[n], end[n]) of every node's stream."""
        n = len(begin)
        b = (ctypes.c_uint64 * n)(*begin)
        e = (ctypes.c_uint64 * n)(*end)
        _ck("mpx_submit_trace_range", lib().mpx_submit_trace_range(self.h, trace, len(trace), b, e))

    def submit_window_async(self, trace, begin, end):
        """mpx_submit_trace_range_async: the same window decoded on a background host thread (joined by
        the next submit, a Value read, or mpx_run when nothing else is queued); `trace` must outlive it."""
        n = len(begin)
        b = (ctypes.c_uint64 * n)(*begin)
        e = (ctypes.c_uint64 * n)(*end)
        _ck("mpx_submit_trace_range_async", lib().mpx_submit_trace_range_async(self.h, trace, len(trace), b, e))

    def submit_range(self, trace, node, k0, k1, index=None):
        """mpx_submit of records [k0, k1) of `node`'s stream in an MPXT container, in place (no
        copy: the bytes and offsets are the container's own; a window of a live stream)."""
        if k1 <= k0:
            return
        idx = index if index is not None else trace_index(trace)
        base = _addr(trace)
        cnt, offs_at, body_at = idx[node]
        if k1 > cnt:
            raise ValueError("records [%d, %d) of a %d-record stream" % (k0, k1, cnt))
        f = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_uint64)(("mpx_submit", lib()))
        _ck("mpx_submit", f(self.h, node, base + body_at, base + offs_at + 8 * k0, k1 - k0))

    def load_clean_device(self, **kw):
        p = GenParams(GEN_CLEAN, kw.get("num_nodes", self.num_nodes), kw["num_instances"], kw.get("seed", 0),
                      kw.get("batch", 256), 1, 0, 0, 0, 0, self.shard_begin, self.shard_end)
        _ck("mpx_load_clean_device", lib().mpx_load_clean_device(self.h, ctypes.byref(p)))

    # execution
    def run(self):
        _ck("mpx_run", lib().mpx_run(self.h))
        return self.stats()

    def step(self):
        _ck("mpx_step", lib().mpx_step(self.h))

    def sync(self):
        _ck("mpx_sync", lib().mpx_sync(self.h))

    def reset_state(self):
        _ck("mpx_reset_state", lib().mpx_reset_state(self.h))

    def timings(self, max_n=4096):
        a = (ctypes.c_double * max_n)()
        r = (ctypes.c_double * max_n)()
        n = ctypes.c_uint32()
        _ck("mpx_timings", lib().mpx_timings(self.h, max_n, a, r, ctypes.byref(n)))
        return list(a[: n.value]), list(r[: n.value])

    def timing_every(self, every):
        """Phase events on every `every`-th run / step only (mpx_timing_every)."""
        _ck("mpx_timing_every", lib().mpx_timing_every(self.h, every))

    PHASES = ("run", "scan", "fast_apply", "general_apply", "tail")

    def timings_detail(self, max_n=4096):
        """Per run/step since the last timings call: dict of phase -> ms (mpx_timings_detail)."""
        a = (ctypes.c_double * (5 * max_n))()
        n = ctypes.c_uint32()
        _ck("mpx_timings_detail", lib().mpx_timings_detail(self.h, max_n, a, ctypes.byref(n)))
        return [dict(zip(self.PHASES, a[5 * i: 5 * i + 5])) for i in range(n.value)]

    # results
    def stats(self):
        s = Stats()
        _ck("mpx_stats_get", lib().mpx_stats_get(self.h, ctypes.byref(s)))
        return s.as_dict()

    def state_digest(self):
        """(state_digest, chosen_digest) of what the last run/step left in HBM (separate device pass)."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        _ck("mpx_state_digest", lib().mpx_state_digest(self.h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def violation(self):
        v = Violation()
        _ck("mpx_last_violation", lib().mpx_last_violation(self.h, ctypes.byref(v)))
        return {"code": v.code, "node": v.node, "seq": v.seq, "iid": v.iid}

    def dump(self):
        out = ctypes.POINTER(ctypes.c_uint8)()
        size = ctypes.c_uint64()
        _ck("mpx_dump_result", lib().mpx_dump_result(self.h, ctypes.byref(out), ctypes.byref(size)))
        return _take(out, size.value)

    def decisions(self):
        """MPXD bytes: the phase-2 batch at every promise quorum (mpx_read_decisions)."""
        out = ctypes.POINTER(ctypes.c_uint8)()
        size = ctypes.c_uint64()
        _ck("mpx_read_decisions", lib().mpx_read_decisions(self.h, ctypes.byref(out), ctypes.byref(size)))
        return _take(out, size.value)

    def decision_bounds(self):
        """Per promise quorum, this shard's absolute fill bound (mpx_decisions_bounds)."""
        cnt = ctypes.c_uint64()
        _ck("mpx_decisions_bounds", lib().mpx_decisions_bounds(self.h, None, 0, ctypes.byref(cnt)))
        buf = (ctypes.c_uint64 * max(cnt.value, 1))()
        _ck("mpx_decisions_bounds", lib().mpx_decisions_bounds(self.h, buf, cnt.value, ctypes.byref(cnt)))
        return list(buf[:cnt.value])

    def decisions_part(self, global_bounds):
        """MPXP bytes: this shard's part of the decisions, fills cut at the global bounds."""
        n = len(global_bounds)
        buf = (ctypes.c_uint64 * max(n, 1))(*global_bounds)
        out = ctypes.POINTER(ctypes.c_uint8)()
        size = ctypes.c_uint64()
        _ck("mpx_read_decisions_part",
            lib().mpx_read_decisions_part(self.h, buf, n, ctypes.byref(out), ctypes.byref(size)))
        return _take(out, size.value)

    def commits(self):
        """MPXC bytes: every CommittingValues with its OnCommitReply retirement (mpx_read_commits)."""
        out = ctypes.POINTER(ctypes.c_uint8)()
        size = ctypes.c_uint64()
        _ck("mpx_read_commits", lib().mpx_read_commits(self.h, ctypes.byref(out), ctypes.byref(size)))
        return _take(out, size.value)

    def proposal_part(self):
        """MPXE bytes: this shard's events of the proposer bookkeeping (mpx_proposal_part)."""
        out = ctypes.POINTER(ctypes.c_uint8)()
        size = ctypes.c_uint64()
        _ck("mpx_proposal_part", lib().mpx_proposal_part(self.h, ctypes.byref(out), ctypes.byref(size)))
        return _take(out, size.value)

    def learns(self):
        """MPXL bytes: every member LearningValues and what became of it (mpx_read_learns)."""
        out = ctypes.POINTER(ctypes.c_uint8)()
        size = ctypes.c_uint64()
        _ck("mpx_read_learns", lib().mpx_read_learns(self.h, ctypes.byref(out), ctypes.byref(size)))
        return _take(out, size.value)

    def value_bytes(self, handle):
        """The canonical wire bytes of the Value a handle names (mpx_value_bytes)."""
        cap = 1 << 12
        while True:
            buf = (ctypes.c_uint8 * cap)()
            n = ctypes.c_uint32()
            rc = lib().mpx_value_bytes(self.h, handle, buf, cap, ctypes.byref(n))
            if rc == 0 and n.value <= cap:
                return bytes(buf[:n.value])
            if rc != 0 and n.value <= cap:
                _ck("mpx_value_bytes", rc)
            cap = n.value

    def learn_values(self):
        """MPXV bytes: every learn's Values and the Unproposable records (mpx_read_learn_values)."""
        out = ctypes.POINTER(ctypes.c_uint8)()
        size = ctypes.c_uint64()
        _ck("mpx_read_learn_values", lib().mpx_read_learn_values(self.h, ctypes.byref(out), ctypes.byref(size)))
        return _take(out, size.value)

    def commit_points(self):
        """MPXQ bytes: this engine's commit creation points (mpx_commit_points)."""
        out = ctypes.POINTER(ctypes.c_uint8)()
        size = ctypes.c_uint64()
        _ck("mpx_commit_points", lib().mpx_commit_points(self.h, ctypes.byref(out), ctypes.byref(size)))
        return _take(out, size.value)

    def commits_at(self, points):
        """MPXC bytes from the union of every shard's creation points (mpx_read_commits_at;
        the engine whose shard starts at instance 0)."""
        out = ctypes.POINTER(ctypes.c_uint8)()
        size = ctypes.c_uint64()
        _ck("mpx_read_commits_at", lib().mpx_read_commits_at(self.h, bytes(points), len(points), ctypes.byref(out),
                                                             ctypes.byref(size)))
        return _take(out, size.value)

    def commits_sharded(self):
        """The whole run's MPXC from this rank's shard over the engine's communicator
        (mpx_read_commits_sharded: points all-gather, union, OnCommitReply on the shard at 0)."""
        out = ctypes.POINTER(ctypes.c_uint8)()
        size = ctypes.c_uint64()
        _ck("mpx_read_commits_sharded", lib().mpx_read_commits_sharded(self.h, ctypes.byref(out), ctypes.byref(size)))
        return _take(out, size.value)

    def drain_sends(self):
        sends = []

        def cb(_u, src, dst, p, n):
            sends.append((src, dst, ctypes.string_at(p, n)))

        f = SEND_FN(cb)
        _ck("mpx_drain_sends", lib().mpx_drain_sends(self.h, f, None))
        return sends

    def read_chosen(self, first, count):
        out = (ctypes.c_uint64 * count)()
        _ck("mpx_read_chosen", lib().mpx_read_chosen(self.h, first, count, out))
        return list(out)

    def read_node_scalars(self, node):
        p, m = ctypes.c_uint64(), ctypes.c_uint64()
        _ck("mpx_read_node_scalars", lib().mpx_read_node_scalars(self.h, node, ctypes.byref(p), ctypes.byref(m)))
        return p.value, m.value

    def read_executed(self, node):
        """(next_id_to_apply_, [handles executed in instance order]) of one node,
        computed on the device (mpx_read_executed; multi/paxos.cpp:1584-1622)."""
        fr, cnt = ctypes.c_uint64(), ctypes.c_uint64()
        _ck("mpx_read_executed", lib().mpx_read_executed(self.h, node, ctypes.byref(fr), ctypes.byref(cnt), None, 0))
        out = (ctypes.c_uint64 * max(cnt.value, 1))()
        _ck("mpx_read_executed", lib().mpx_read_executed(self.h, node, ctypes.byref(fr), ctypes.byref(cnt), out,
                                                         cnt.value))
        return fr.value, list(out[: cnt.value])

    def read_node_state(self, node, first, count):
        arrs = [(ctypes.c_uint64 * count)() for _ in range(4)]
        _ck("mpx_read_node_state", lib().mpx_read_node_state(self.h, node, first, count, *arrs))
        return [list(a) for a in arrs]

    # multi-GPU
    @staticmethod
    def comm_unique_id():
        buf = (ctypes.c_uint8 * UID_BYTES)()
        _ck("mpx_comm_unique_id", lib().mpx_comm_unique_id(buf))
        return bytes(buf)

    def comm_init(self, uid, rank, nranks):
        buf = (ctypes.c_uint8 * UID_BYTES).from_buffer_copy(uid)
        _ck("mpx_comm_init", lib().mpx_comm_init(self.h, buf, rank, nranks))
        self.nranks = nranks

    def allreduce_max(self, vals):
        """Element-wise MAX over the ranks (RCCL, mpx_comm_allreduce_max); identity without a communicator."""
        buf = (ctypes.c_uint64 * max(len(vals), 1))(*vals)
        _ck("mpx_comm_allreduce_max", lib().mpx_comm_allreduce_max(self.h, buf, len(vals)))
        return list(buf[:len(vals)])

    def allgather_bytes(self, data, nranks=1):
        """Every rank's byte string, in rank order (RCCL, mpx_comm_allgather_bytes)."""
        out = ctypes.POINTER(ctypes.c_uint8)()
        lens = (ctypes.c_uint64 * max(nranks, 1))()
        _ck("mpx_comm_allgather_bytes", lib().mpx_comm_allgather_bytes(self.h, bytes(data), len(data),
                                                                        ctypes.byref(out), lens))
        blob = _take(out, sum(lens))
        parts, at = [], 0
        for n in lens:
            parts.append(blob[at:at + n])
            at += n
        return parts

    def decisions_sharded(self):
        """The whole run's MPXD from this rank's shard over the engine's communicator
        (mpx_read_decisions_sharded: bounds all-reduce MAX, parts all-gather, combine)."""
        out = ctypes.POINTER(ctypes.c_uint8)()
        size = ctypes.c_uint64()
        _ck("mpx_read_decisions_sharded",
            lib().mpx_read_decisions_sharded(self.h, ctypes.byref(out), ctypes.byref(size)))
        return _take(out, size.value)

    def allgather_summary(self, nranks=1):
        out = (ctypes.c_uint64 * (64 * nranks))()
        _ck("mpx_allgather_summary", lib().mpx_allgather_summary(self.h, out))
        return [list(out[64 * r: 64 * (r + 1)]) for r in range(nranks)]


def source_digest():
    """16 hex digits of SHA-256 over the sources that decide the device traffic — the kernels,
    the device generator, the shared layout header, the launch code (engine.cpp: grids, which
    kernels run) and ingest (which runs share entries, which pairs go to which kernel): what a
    committed PMC profile was measured with (tools/pmc_traffic.py), so bench.py can refuse a
    profile of other kernels or another trace layout."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(os.path.dirname(HERE), "csrc")
    for name in ("gen_device.hip", "kernels.hip", "mpx_internal.hpp", "engine.cpp", "ingest.cpp", "ingest.hpp"):
        full = os.path.join(csrc, name)
        h.update(name.encode() + b"\0")
        with open(full, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def declared_symbols(header=INCLUDE_H):
    """Function names declared in include/mpx.h."""
    import re
    txt = open(header).read()
    return sorted(set(re.findall(r"^\s*(?:int|void)\s+(mpx_\w+)\s*\(", txt, re.M)))


def decisions_combine(parts):
    """Merge MPXP parts (shard order) into the whole run's MPXD (mpx_decisions_combine)."""
    n = len(parts)
    raw = [ctypes.create_string_buffer(bytes(p), max(len(p), 1)) for p in parts]   # kept alive for the call
    arr = (ctypes.POINTER(ctypes.c_uint8) * n)(*[ctypes.cast(b, ctypes.POINTER(ctypes.c_uint8)) for b in raw])
    sizes = (ctypes.c_uint64 * n)(*[len(p) for p in parts])
    out = ctypes.POINTER(ctypes.c_uint8)()
    size = ctypes.c_uint64()
    _ck("mpx_decisions_combine", lib().mpx_decisions_combine(arr, sizes, n, ctypes.byref(out), ctypes.byref(size)))
    return _take(out, size.value)


def _combine(fn, parts):
    n = len(parts)
    raw = [ctypes.create_string_buffer(bytes(p), max(len(p), 1)) for p in parts]   # kept alive for the call
    arr = (ctypes.POINTER(ctypes.c_uint8) * n)(*[ctypes.cast(b, ctypes.POINTER(ctypes.c_uint8)) for b in raw])
    sizes = (ctypes.c_uint64 * n)(*[len(p) for p in parts])
    out = ctypes.POINTER(ctypes.c_uint8)()
    size = ctypes.c_uint64()
    _ck(fn, getattr(lib(), fn)(arr, sizes, n, ctypes.byref(out), ctypes.byref(size)))
    return _take(out, size.value)


def commit_points_combine(parts):
    """Union of MPXQ commit creation points of every shard (mpx_commit_points_combine)."""
    return _combine("mpx_commit_points_combine", parts)


def proposal_combine(parts):
    """Merge MPXE parts (shard order) into the whole run's MPXD with client values (mpx_proposal_combine)."""
    return _combine("mpx_proposal_combine", parts)
