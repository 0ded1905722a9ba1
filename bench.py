#!/usr/bin/env python3
"""Benchmark: quorum decisions/s of the MI355X Multi-Paxos engine (BASELINE.json metric).

Workload (config.workload): C4 — 2^27 instances x 9 acceptors, clean single
round (one proposer, ballot 1<<16, 256 instances per ACCEPT/COMMIT), the trace
materialised in HBM by the device generator before timing.  The instance space
is sharded contiguously over the ranks (strong scaling: the whole C4 trace at
every N); each rank owns one GPU.

One step = one pass of the hot path over the resident trace from genesis
state: header scan, promise quorum, accept-vote quorum, acceptor/learner apply
(k_apply), chosen log, counters, and — for N > 1 — the RCCL all-gather of the
64-word per-shard summary.  decisions/s = chosen instances per step (summed
over ranks) / max-over-ranks step time.

roofline: the dominant unit is the apply phase — k_plan_store8, one launch:
per 32-bucket group, one thread per (acceptor, bucket) pair decides which
message run fixes it into LDS while other waves of the workgroup stream the
previous group's slots and chosen log (before round 6: k_plan + k_store8,
the plan words through HBM) — bracketed by HIP events on the engine's
stream.  frac is the hardware
fraction: traffic (HBM bytes per launch of those kernels from rocprofv3 PMC,
FETCH_SIZE x2 + WRITE_SIZE, committed under profiles/ and matched to these
sources by digest, tools/pmc_traffic.py) / the phase's mean duration in this
run / 8 TB/s.  Beside it: the engine's own byte model (1-byte
slot per (acceptor, instance), 1-byte chosen log, 16-byte descriptors per run;
frac_engine_model) and SURVEY.md §8(d)'s 16 P + 24 A + 16 L
(frac_survey_model, > 1 on the clean trace: a measure of the representation,
not a bandwidth).  Without a matching profile frac falls back to the engine
model and roofline.basis says so.

Verification: steps leave the order-independent digests off (mpx_step); after
the timed region one digested run (mpx_run) is checked against the closed-form
final state of the clean trace (oracle mpxo_clean_expect), per rank.

cpu_baseline: the reference's own handlers (multi/paxos.cpp compiled -O2 in
oracle/_ref, kind "reference") on a bounded sample of the same clean stream,
rank 0 at N=1 only.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
(the launcher only starts the ranks; rendezvous, barriers and the max-reduce of
the step time go through FileGroup, the RCCL communicator through mpx_comm_*)
"""
import argparse
import ctypes
import glob
import json
import os
import re
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "multi-paxos_amd"))

import mpx  # noqa: E402
from mpx import dist as mdist  # noqa: E402

METRIC = "quorum decisions/sec (instances chosen/s) + achieved HBM GB/s, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E, MI355X_MICROARCH.md chip-level table


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--instances", type=int, default=1 << 27, help="M (C4: 2^27)")
    ap.add_argument("--nodes", type=int, default=9, help="acceptors N (C4: 9)")
    ap.add_argument("--batch", type=int, default=256, help="instances per ACCEPT / COMMIT batch (C4: 256)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the cpu_baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--c3-instances", type=int, default=1 << 24, help="C3 general-path leg: M (2^24); 0 = skip")
    ap.add_argument("--c3-steps", type=int, default=5)
    ap.add_argument("--c3-only", action="store_true", help="only the C3 leg (profiling)")
    ap.add_argument("--c3-windows", type=int, default=16,
                    help="the C3 trace again as this many incremental windows (the live OnReceiveMessage path, "
                         "k_apply_win); 0 = skip")
    ap.add_argument("--c3-windows-only", action="store_true", help="only the C3 windows leg (profiling)")
    ap.add_argument("--c5-instances", type=int, default=1 << 25, help="C5 member-path leg: M (2^25); 0 = skip")
    ap.add_argument("--c5-steps", type=int, default=5)
    ap.add_argument("--c5-only", action="store_true", help="only the C5 leg (profiling)")
    ap.add_argument("--c5c-instances", type=int, default=1 << 25,
                    help="contended C5 leg (3 member proposers, a rival round per epoch): M (2^25); 0 = skip")
    ap.add_argument("--c5c-only", action="store_true", help="only the contended C5 leg (profiling)")
    ap.add_argument("--loop-values", type=int, default=1 << 16,
                    help="closed-loop leg (libmpx's own proposer loop, mpx_loop_leader_rounds): client values per "
                         "round; 0 = skip")
    ap.add_argument("--loop-rounds", type=int, default=4)
    ap.add_argument("--loop-only", action="store_true", help="only the closed-loop leg")
    ap.add_argument("--shard-of", type=int, default=8,
                    help="also time rank 0's shard of the same trace at world G on this GPU (a 1-GPU scaling "
                         "projection, no RCCL); 0 / 1 = skip")
    ap.add_argument("--shard-only", action="store_true", help="only the shard projection (profiling)")
    ap.add_argument("--detail", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="the full result (every leg's notes, per-window times) is written here; the JSON line on "
                         "stdout carries the headline figures of every leg")
    ap.add_argument("--leg-cpu-instances", type=int, default=1 << 17,
                    help="instances of the sampled trace each leg's reference cpu_baseline replays")
    ap.add_argument("--events-every", type=int, default=8,
                    help="phase events (HIP start / stop timestamps on the kernels) on every k-th timed step of "
                         "the C4 and shard loops: each costs the step ~1.5-2 us (mpx_timing_every)")
    return ap.parse_args()


# C3 (BASELINE.json configs[2]): 7 acceptors, 3 competing proposers, the
# HijackSend fault model of multi/debug.conf.sample:1 (drop 500, dup 1000 per 10^4, delay U[0,500)),
# batches of U[1,256] instances
C3 = dict(num_nodes=7, seed=0, batch=256, proposers=3, drop_rate=500, dup_rate=1000, max_delay=500)
# C5: member semantics, acceptor universe 8, AddAcceptor(1..7) then DelAcceptor(1..7)
# (member/main.cpp:119-141), 1 % loss / duplicates, stale in-flight ACCEPTs across version changes
C5 = dict(num_nodes=8, seed=0, batch=256, drop_rate=100, dup_rate=100, max_delay=64, noop_permille=15)
# contended C5: the same schedule with 3 member proposers — from epoch 2 a
# rival prepares above the leader over its own unlearned ids (member/paxos.cpp:1158-1182,
# 1504-1549,1614-1629): promise replies carrying most of the history, merged maps, rejects
C5C = dict(C5, proposers=3)


def log(msg):
    print("[bench] " + msg, file=sys.stderr, flush=True)


def c3_leg(args, kind="c3"):
    """The general path on C3: every pair goes through k_apply (multi-ballot promise phases,
    promise replies with entries, rejects, duplicates, reordering).  The trace is generated
    and ingested through mpx_submit_trace before timing (host work, reported apart); a step
    is the same mpx_step the C4 line times.  roofline on SURVEY §8(d)'s bytes
    (16 P + 24 A + 16 L from the engine's counters) over the apply phase.
    kind "c5": the same over the C5 member trace (member role gates, insert-first apply,
    per-epoch quorums: the member instantiation of k_apply); "c5c": contended C5."""
    member = kind in ("c5", "c5c")
    m = args.c5c_instances if kind == "c5c" else args.c5_instances if member else args.c3_instances
    steps = args.c5_steps if member else args.c3_steps
    t0 = time.perf_counter()
    if member:
        trace = mpx.generate_trace(mpx.GEN_MEMBER, num_instances=m, copy=False, **(C5C if kind == "c5c" else C5))
    else:
        trace = mpx.generate_trace(mpx.GEN_FAULTY, num_instances=m, copy=False, **C3)
    t_gen = time.perf_counter() - t0
    log("%s: generated %.1f MB in %.1f s" % (kind, len(trace) / 1e6, t_gen))
    hd = mpx.trace_header(trace)
    trace_bytes = len(trace)
    eng = mpx.Engine(hd["num_nodes"], 0, max(hd["num_instances"], 1), semantics=hd["semantics"])
    t0 = time.perf_counter()
    eng.submit_trace(trace)                         # (member: the trace's epoch table comes with it)
    t_ingest = time.perf_counter() - t0
    log("%s: ingested in %.1f s" % (kind, t_ingest))
    windows_trace = trace if (not member and args.c3_windows and not args.c3_only) else None
    del trace
    t0 = time.perf_counter()
    chk = eng.run()                                 # upload + one digested run (verification)
    t_first = time.perf_counter() - t0
    log("%s: upload + first run %.1f s" % (kind, t_first))
    eng.timings()
    for _ in range(2):
        eng.step()
    eng.sync()
    eng.timings()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.step()
    eng.sync()
    dt = time.perf_counter() - t0
    st = eng.stats()
    ph = eng.timings_detail()
    step_digests = eng.state_digest()
    step_ok = step_digests == (chk["state_digest"], chk["chosen_digest"]) and \
        all(st[k] == chk[k] for k in ("chosen", "promise_entries", "accept_apps", "commit_apps", "violations"))
    assert step_ok, "%s: the timed step's state differs from the digested run's" % kind.upper()
    assert st["violations"] == 0
    mean = lambda k: sum(p[k] for p in ph) / max(len(ph), 1)
    general_ms, fast_ms = mean("general_apply"), mean("fast_apply")
    apply_ms = general_ms + fast_ms
    b_alg = 16 * st["promise_entries"] + 24 * st["accept_apps"] + 16 * st["commit_apps"]
    achieved = b_alg / (apply_ms * 1e-3) / 1e9 if apply_ms else 0.0
    # the engine's own compulsory bytes (as the C4 line): one state slot per
    # (acceptor, instance) and one chosen-log slot written, every message run's 16-byte
    # descriptor read, one 8-byte plan word per (row, bucket) written and read back
    nb_l = (hd["num_instances"] + 255) // 256
    b_eng = st["slot_bytes"] * (hd["num_nodes"] + 1) * nb_l * 256 + 16 * st["num_runs"] + \
        16 * (hd["num_nodes"] + 1) * nb_l
    achieved_eng = b_eng / (apply_ms * 1e-3) / 1e9 if apply_ms else 0.0
    pmc = latest_pmc(8 if member else 7, m, 1, workload=kind.upper())
    hw = hw_roofline(pmc, apply_ms)
    ms_step = dt / steps * 1e3
    eng.close()
    win = None
    if windows_trace is not None:
        win = c3_windows_leg(args, windows_trace, (chk["state_digest"], chk["chosen_digest"]),
                             {k: chk[k] for k in ("chosen", "promise_entries", "accept_apps", "commit_apps")})
        del windows_trace
    if member:
        workload = ("C5: 2^%d instances, member semantics, acceptor universe 8, AddAcceptor(1..7) then "
                    "DelAcceptor(1..7) = 15 epochs (member/main.cpp:119-141), 1%% loss / 1%% duplicates, "
                    "batch U[1,256]" % (m.bit_length() - 1))
        if kind == "c5c":
            workload += (", contended: 3 member proposers (a rival round above the leader in every epoch from "
                         "2, over its own unlearned ids; the leader re-prepares)")
    else:
        workload = ("C3: 2^%d instances x 7 acceptors, 3 competing proposers, drop 5%% / dup 10%% (<=3) / "
                    "delay U[0,500) (multi/debug.conf.sample:1), batch U[1,256]" % (m.bit_length() - 1))
    return {
        "workload": workload,
        "instances_proposed": m, "instances": hd["num_instances"], "acceptors": hd["num_nodes"],
        "decisions_per_step": st["chosen"], "ms_per_step": ms_step,
        "value": st["chosen"] / (ms_step * 1e-3), "unit": "decisions/s",
        "counters": {k: st[k] for k in ("chosen", "promise_entries", "accept_apps", "commit_apps", "messages")},
        "phases_ms": {k: mean(k) for k in mpx.Engine.PHASES},
        "roofline": {"bound": "hbm", "kernel": "apply phase: k_plan_list<member> + k_store (planned pairs), "
                     "k_apply<member> (the pairs it lists, promise rounds)" if member else
                     "apply phase: k_plan (lean pairs) + k_plan_list (work-list pairs without promise rounds) + "
                     "k_store, k_apply (the pairs k_plan_list lists, promise rounds)",
                     "bytes_alg_per_launch": b_alg, "bytes_model": "SURVEY §8(d): 16 P + 24 A + 16 L",
                     "kernel_ms": apply_ms, "general_ms": general_ms, "fast_ms": fast_ms,
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     # the hardware fraction: PMC HBM bytes of the same kernels / the same mean duration
                     "frac_hw": hw["frac"] if hw else None, "achieved_hw": hw["achieved"] if hw else None,
                     "bytes_engine_model_per_launch": b_eng,
                     "frac_engine_model": achieved_eng / HBM_PEAK_GBS,
                     "note": "frac_hw is what the HBM moved (PMC traffic / kernel_ms / 8 TB/s); "
                             "frac is on SURVEY §8(d)'s bytes (every acceptor's own 16-24 B copy per entry); the "
                             "engine stores a broadcast once and its slots name the run that fixed them, so it "
                             "moves far fewer bytes: frac > 1 (C5) measures that representation, and "
                             "frac_engine_model (the slots, chosen log, run descriptors and plan words it must "
                             "move) is far below 1 because the per-pair walk is latency-bound, not HBM-bound",
                     "counters_engine": {"runs": st["num_runs"], "slot_bytes": st["slot_bytes"],
                                         "general_pairs": st["general_pairs"]},
                     "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
                     "traffic_source": ("profiles/%s_pmc.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE of the apply "
                                        "phase, bench.py --%s-only; not measured inside this process)"
                                        % (pmc["tag"], kind))
                     if pmc else None},
        "verified": {"step_state_digest_vs_run": step_ok, "state_digest": chk["state_digest"],
                     "chosen_digest": chk["chosen_digest"]},
        "host": {"generate_s": t_gen, "ingest_s": t_ingest, "upload_and_first_run_s": t_first,
                 "trace_bytes": trace_bytes},
        **({"windows": win} if win else {}),
    }


def c3_windows_leg(args, trace, want_digests, want_counters):
    """The live path: the C3 trace as args.c3_windows incremental windows
    (MPX_FLAG_INCREMENTAL: the drop-in for NetWork::OnReceiveMessage, multi/paxos.cpp:1714-1717).
    Each window = mpx_submit_trace_range of 1/W of every node's records (host decode) + one
    mpx_run (k_apply_win over the pairs the window touches, on the value state the earlier
    windows left).  The windows together must give the batch run's digests and counters."""
    W = args.c3_windows
    hd = mpx.trace_header(trace)
    idx = mpx.trace_index(trace)
    n, m = hd["num_nodes"], hd["num_instances"]
    eng = mpx.Engine(n, 0, m, flags=mpx.FLAG_INCREMENTAL)
    eng.timing_every(1)
    host_ms, sub_ms, dev, gp = [], [], [], []
    tot = {k: 0 for k in want_counters}
    prev = [0] * n
    for w in range(1, W + 1):
        cut = [c * w // W for (c, _, _) in idx]
        t0 = time.perf_counter()
        eng.submit_window(trace, prev, cut)
        sub_ms.append((time.perf_counter() - t0) * 1e3)
        st = eng.run()
        host_ms.append((time.perf_counter() - t0) * 1e3)
        ph = eng.timings_detail()
        dev.append(ph[-1])
        gp.append(st["general_pairs"])
        for k in tot:
            tot[k] += st[k]
        prev = cut
    digests = eng.state_digest()
    eng.close()
    ok = digests == tuple(want_digests) and tot == want_counters
    assert ok, "C3 windows: the windows' state differs from the batch run's (%r vs %r, %r vs %r)" % (
        digests, want_digests, tot, want_counters)
    # the pipelined live loop: window k + 1 decoded on a host thread (mpx_submit_trace_range_async)
    # while window k is built and run — wall time of the whole loop
    eng = mpx.Engine(n, 0, m, flags=mpx.FLAG_INCREMENTAL)
    cuts = [[c * w // W for (c, _, _) in idx] for w in range(W + 1)]
    ptot = {k: 0 for k in want_counters}
    t0 = time.perf_counter()
    eng.submit_window(trace, cuts[0], cuts[1])
    for w in range(1, W + 1):
        if w < W:
            eng.submit_window_async(trace, cuts[w], cuts[w + 1])
        st = eng.run()
        for k in ptot:
            ptot[k] += st[k]
    pipe_s = time.perf_counter() - t0
    pdig = eng.state_digest()
    eng.close()
    pok = pdig == tuple(want_digests) and ptot == want_counters
    assert pok, "C3 windows (pipelined): the state differs from the batch run's"
    log("c3 windows pipelined: %.1f ms / window, %.3g decisions/s end to end" % (pipe_s / W * 1e3,
                                                                                  ptot["chosen"] / pipe_s))
    run_ms = [p["run"] for p in dev]
    apply_ms = [p["fast_apply"] + p["general_apply"] for p in dev]   # k_apply_win's start / stop events
    mean = lambda xs: sum(xs) / max(len(xs), 1)
    # profiles record the proposed instance count (2^24), not the trace header's (every
    # instance a proposer ever touched): look up by the same key as the C3 leg
    pmc = latest_pmc(7, args.c3_instances, 1, workload="C3W")
    hw = hw_roofline(pmc, mean(apply_ms))
    # engine model of a window's apply: each pair it touches reads and writes 256 slots of
    # 16-B value state (s_bal, s_val) and its runs' 16-B descriptors
    b_eng = sum(32 * 256 * x for x in gp) / W
    log("c3 windows: %d windows, host %.1f ms / window (submit %.1f; device %.2f), k_apply_win %.3f ms" %
        (W, mean(host_ms), mean(sub_ms), mean(run_ms), mean(apply_ms)))
    return {"windows": W, "chosen": tot["chosen"],
            "value": ptot["chosen"] / pipe_s, "unit": "decisions/s",
            "value_sequential": tot["chosen"] / (sum(host_ms) * 1e-3),
            "value_device": tot["chosen"] / (sum(run_ms) * 1e-3),
            "note": "value: chosen instances / the wall time of the pipelined window loop (window k + 1 decoded "
                    "on a host thread while window k is built, uploaded and run: mpx_submit_trace_range_async); "
                    "value_sequential: the same with each window's decode, build, upload and run in turn; "
                    "value_device: / the device run time alone",
            "host_ms_per_window": pipe_s / W * 1e3, "host_ms_per_window_sequential": mean(host_ms),
            "submit_ms_per_window": mean(sub_ms),
            "device_ms_per_window": mean(run_ms),
            "host_ms": host_ms, "device_ms": run_ms, "apply_ms": apply_ms, "pairs_per_window": gp,
            "roofline": {"bound": "hbm", "kernel": "k_apply_win", "kernel_ms": mean(apply_ms),
                         "frac_hw": hw["frac"] if hw else None, "achieved_hw": hw["achieved"] if hw else None,
                         "traffic": hw["traffic"] if hw else None, "traffic_source": hw["source"] if hw else None,
                         "bytes_engine_model_per_launch": b_eng,
                         "frac_engine_model": b_eng / (mean(apply_ms) * 1e-3) / 1e9 / HBM_PEAK_GBS if mean(apply_ms) else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s"},
            "verified": {"digests_vs_batch_run": ok and pok}}


def secondary_loop(args):
    try:
        return closed_loop_leg(args)
    except mpx.MpxError as ex:
        if ex.rc != -2:
            raise
        return {"error": repr(ex)}


def closed_loop_leg(args):
    """The closed loop: libmpx's own proposer loop over one
    incremental engine (csrc/loop.cpp) — node 0 leads 7 acceptors/learners; per round it starts a
    prepare with --loop-values client values queued (Propose while preparing, multi/paxos.cpp:
    1250-1280), and the engine's promise quorum decision becomes the ACCEPT, its chosen log the COMMIT,
    with no Python between windows (5 windows per round).  decisions/s = values chosen, committed and
    executed on every node / wall time of the rounds (host encode + decode + build, device run)."""
    from mpx.loop import NativeLoop
    N, V, R = 7, args.loop_values, args.loop_rounds
    L = NativeLoop(N, (R + 1) * V)
    try:
        L.leader_rounds(0, range(N), 1, V)                  # warm-up round (allocations, first window)
        s0 = L.stats()
        t0 = time.perf_counter()
        L.leader_rounds(0, range(N), R, V)
        dt = time.perf_counter() - t0
        s1 = L.stats()
        ex = [L.engine.read_executed(n) for n in range(N)]
        ok = all(fr == (R + 1) * V and len(h) == (R + 1) * V for fr, h in ex) and all(h == ex[0][1] for _, h in ex)
        assert ok, "closed loop: not every value was executed in order on every node"
        d = {k: s1[k] - s0[k] for k in s1}
        trace_file = None
        if not args.no_cpu_baseline:                         # the streams the loop sent, for the reference
            import tempfile
            trace_file = os.path.join(tempfile.gettempdir(), "mpx_loop_%d.mpxt" % os.getpid())
            with open(trace_file, "wb") as fh:
                fh.write(L.trace())
    finally:
        L.close()
    w = max(d["windows"], 1)
    out = {"workload": "closed loop: 7 nodes, leader 0, %d rounds x %d client values (prepare with values "
                       "queued -> the engine's decided batch -> ACCEPT -> chosen -> COMMIT), libmpx mpx_loop_*" % (R, V),
           "value": d["committed_instances"] / dt, "unit": "decisions/s", "rounds": R, "values_per_round": V,
           "windows": d["windows"], "ms_per_window": dt / w * 1e3,
           "host_split_ms_per_window": {"submit": d["submit_ns"] / w / 1e6, "run": d["run_ns"] / w / 1e6,
                                        "drain": d["drain_ns"] / w / 1e6},
           "verified": {"executed_in_order_on_every_node": ok}}
    if trace_file:
        cb = leg_cpu_baseline("loop", trace_file=trace_file)
        os.remove(trace_file)
        if cb and cb.get("value"):
            # the reference replays all R + 1 rounds' streams (the warm-up round too): rate per chosen instance
            out["cpu_baseline"] = cb
            out["vs_cpu"] = out["value"] / cb["value"]
    log("closed loop: %d rounds x %d values in %.3f s: %.3g decisions/s (%.2f ms / window: submit %.2f, run %.2f, "
        "drain %.2f)" % (R, V, dt, out["value"], out["ms_per_window"], out["host_split_ms_per_window"]["submit"],
                         out["host_split_ms_per_window"]["run"], out["host_split_ms_per_window"]["drain"]))
    return out


class FileGroup:
    """Rendezvous, barrier, max-reduce and broadcast between the ranks of one node
    through files (the contract launches every rank on one node; no PyTorch): a
    directory keyed by the launcher's MASTER_PORT and PID, one file per rank and
    round, written atomically (write + rename) and polled."""

    def __init__(self, rank, world):
        self.rank, self.world, self.k = rank, world, 0
        # torchrun gives every rank of one launch the same TORCHELASTIC_RUN_ID: a crashed
        # earlier launch on the same port never shares its directory; without it the ranks'
        # common parent (one launcher process) keys it
        rid = os.environ.get("TORCHELASTIC_RUN_ID")
        key = "%s_%s" % (os.environ.get("MASTER_PORT", "0"), rid if rid else "p%d" % os.getppid())
        self.dir = os.path.join("/tmp", "mpx_bench_" + re.sub(r"[^A-Za-z0-9_.-]", "_", key))
        os.makedirs(self.dir, exist_ok=True)
        if os.path.exists(os.path.join(self.dir, "r1_%d" % rank)):
            raise RuntimeError("rendezvous directory %s holds an earlier run's files" % self.dir)

    def _put(self, name, data):
        tmp = os.path.join(self.dir, ".%s.%d" % (name, self.rank))
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, os.path.join(self.dir, name))

    def _get(self, name, timeout=600.0):
        path = os.path.join(self.dir, name)
        t0 = time.monotonic()
        while not os.path.exists(path):
            if time.monotonic() - t0 > timeout:
                raise TimeoutError("rendezvous: %s missing after %.0f s" % (path, timeout))
            time.sleep(0.001)
        with open(path, "rb") as f:
            return f.read()

    def exchange(self, data):
        """All-gather of one bytes object per rank (also the barrier)."""
        self.k += 1
        self._put("r%d_%d" % (self.k, self.rank), data)
        return [self._get("r%d_%d" % (self.k, r)) for r in range(self.world)]

    def close(self):
        self.exchange(b"")
        self._put("done_%d" % self.rank, b"")       # this rank reads no file of the directory any more
        if self.rank == 0:
            for r in range(self.world):
                self._get("done_%d" % r)
            import shutil
            shutil.rmtree(self.dir, ignore_errors=True)


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    pg = None
    # under torchrun (WORLD_SIZE set) the distributed path runs even at N=1, so
    # the rendezvous / RCCL communicator / all-gather code is exercised
    if world > 1 or "TORCHELASTIC_RUN_ID" in os.environ:
        pg = FileGroup(rank, world)
    return world, rank, local, pg


def barrier(pg):
    if pg is not None:
        pg.exchange(b"")


def allreduce_max(pg, x):
    if pg is None:
        return x
    import struct
    return max(struct.unpack("<d", b)[0] for b in pg.exchange(struct.pack("<d", x)))


def broadcast_bytes(pg, data, rank):
    if pg is None:
        return data
    return pg.exchange(data if rank == 0 else b"")[0]


def latest_pmc(n_nodes, instances, world, workload="C4"):
    """HBM bytes per apply-phase launch from the newest profiles/*pmc*.json measured on this
    workload (nodes, instances, GPUs) AND with these kernels (the engine's source digest, as
    tools/pmc_traffic.py records it); None — reported as traffic null — when no profile matches."""
    best = None
    digest = mpx.source_digest()

    def natural(path):                              # r01_v10 after r01_v9
        return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(path))]

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), key=natural):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if d.get("workload", "C4").split()[0] != workload or d.get("source_digest") != digest:
            continue
        if d.get("nodes") == n_nodes and d.get("instances") == instances and d.get("gpus", 1) == world:
            best = d
    return best


def reference_c4(M, N, batch):
    """The reference's own verdict on the clean trace (tests/golden/full_size.json "c4": multi/paxos.cpp's
    handlers over 128 instance shards, oracle/ref_full_size.py) when this run is that configuration."""
    path = os.path.join(ROOT, "tests", "golden", "full_size.json")
    try:
        c4 = json.load(open(path)).get("c4")
    except (OSError, ValueError):
        return None
    if not c4:
        return None
    p = c4["params"]
    if (p["num_instances"], p["num_nodes"], p["batch"]) != (M, N, batch):
        return None
    return c4["stats"]


def clean_expect(n_nodes, sb, se, ballot=1 << 16):
    """(state_digest, chosen_digest) of the clean trace's final state over [sb, se) — closed form, oracle C."""
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libmpx_oracle.so"))
    f = lib.mpxo_clean_expect
    f.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                  ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    a, b = ctypes.c_uint64(), ctypes.c_uint64()
    threads = max(1, min(16, os.cpu_count() or 1))
    if f(n_nodes, sb, se, ballot, threads, ctypes.byref(a), ctypes.byref(b)) != 0:
        raise RuntimeError("mpxo_clean_expect failed")
    return a.value, b.value


def host_cpus():
    """(cores this process may run on, nproc, the cgroup CPU quota in cores or None)."""
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    return usable, os.cpu_count() or usable, quota


def cpu_note():
    usable, nproc, quota = host_cpus()
    return "nproc %d, usable %d%s" % (nproc, usable, ", cgroup quota %.1f cores" % quota if quota else "")


def cpu_threads():
    """Threads the CPU baselines run: every usable core, but no more than the cgroup CPU quota
    allows (on the GPU box: 256 usable cores under a 16-core quota -> 16 threads; more would only
    time-slice the same 16 cores and understate the baseline)."""
    usable, _, quota = host_cpus()
    if quota:
        import math
        return max(1, min(usable, int(math.ceil(quota))))
    return max(1, usable)


def hw_roofline(pmc, kernel_ms):
    """The hardware fraction: PMC HBM bytes of the timed apply-phase kernels (one launch each,
    rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md gfx950 correction) over the
    phase's mean duration from the HIP events of this run, against the 8 TB/s peak.  None when
    no committed profile matches this workload and these kernels (source digest)."""
    if not pmc or not kernel_ms or not pmc.get("hbm_bytes_per_launch"):
        return None
    gbps = pmc["hbm_bytes_per_launch"] / (kernel_ms * 1e-3) / 1e9
    return {"achieved": gbps, "frac": gbps / HBM_PEAK_GBS, "traffic": pmc["hbm_bytes_per_launch"],
            "source": "profiles/%s_pmc.json" % pmc["tag"]}


def cpu_baseline(args, budget_s):
    """Reference handlers (oracle/_ref) on the host cores this process may use (cpu_threads: the
    usable cores, capped at the cgroup CPU quota): node 1's accept+commit stream of a clean trace,
    one independent replay per thread."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libmpx_ref.so")
    kind = "reference"
    if not os.path.exists(ref_so):
        return None
    lib = ctypes.CDLL(ref_so)
    fn = lib.mpxref_time_node
    fn.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]
    fn.restype = ctypes.c_int64
    sample_m = 1 << 16
    trace = mpx.generate_trace(mpx.GEN_CLEAN, num_nodes=args.nodes, num_instances=sample_m, batch=256)
    threads = cpu_threads()
    done = [0] * threads

    def parallel(reps):
        def work(i):
            done[i] = fn(trace, len(trace), 1, reps)
        ts = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        return time.perf_counter() - t0

    # calibrate one pass on every thread at once (the box's CPU quota may be far below
    # its core count, so a single-thread pass would size the sample many times too long),
    # then size the sample to the budget
    one = parallel(1)
    reps = max(1, int(budget_s / max(one, 1e-6)))
    log("cpu_baseline: %d threads, one pass %.2f s, %d passes" % (threads, one, reps))
    dt = parallel(reps)
    apps = threads * reps * sample_m            # (acceptor, instance) accept+commit applications
    # one decision needs every acceptor's accept + commit application: N of them
    decisions = apps / args.nodes
    return {"value": decisions / dt, "unit": "decisions/s", "cores": threads, "kind": kind,
            "sample": "reference multi/paxos.cpp handlers (-O2) on node 1's stream of a clean C4-shaped trace: "
                      "%d instances x %d passes x %d threads, accept+commit (OnAccept/OnCommit), %.1f s wall; "
                      "decisions/s = acceptor-instance applications/s / N=%d (%s)"
                      % (sample_m, reps, threads, dt, args.nodes, cpu_note()),
            "node_instance_apps_per_s": apps / dt}


def leg_cpu_baseline(leg, instances=1 << 17, trace_file=None):
    """The reference's own handlers (oracle/_ref, -O2) on the leg's own generator configuration
    (bench's C3 / C5 / C5C parameters and seed, sampled at `instances`), one forked process per
    core the quota gives, each replaying the whole sampled trace (oracle/ref_leg_rate.py, run as a
    child process: the reference's objects are not made for concurrent use in one process, and this
    process holds the GPU).  Rank 0, N = 1, the default run only (not the --*-only profiling modes)."""
    import subprocess
    so = os.path.join(ROOT, "oracle", "_ref", "libmpx_ref.so" if leg == "c3" else "libmpx_ref_member.so")
    if not os.path.exists(so):
        return None
    procs = cpu_threads()
    cmd = [sys.executable, os.path.join(ROOT, "oracle", "ref_leg_rate.py"), leg, "--instances", str(instances),
           "--procs", str(procs)] + (["--trace", trace_file] if trace_file else [])
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    except subprocess.TimeoutExpired:
        return {"error": "timeout"}
    if r.returncode:
        log("%s cpu_baseline failed: %s" % (leg, r.stderr.strip()[-300:]))
        return {"error": "rc %d" % r.returncode}
    d = json.loads(r.stdout.strip().splitlines()[-1])
    fs = d.get("full_size_check")
    return {"value": d["value"], "unit": "decisions/s", "cores": procs, "kind": "reference",
            "sample": ("reference %s handlers (-O2, oracle/_ref) over %s (%d chosen, %.0f MB), %d processes each "
                       "replaying the whole trace, slowest %.1f s (%s)"
                       % ("member/paxos.cpp" if leg in ("c5", "c5c") else "multi/paxos.cpp",
                          "the closed loop's own recorded streams" if leg == "loop" else
                          "the leg's own generator configuration at %d instances" % instances,
                          d["chosen"], d["trace_bytes"] / 1e6, procs, d["slowest_s"], cpu_note())),
            "full_size_ref_per_core": fs["per_core"] if fs else None}


def compact_leg(d):
    """The leg's headline figures for the JSON line (the full leg goes to --detail)."""
    if not d or "error" in d:
        return d
    r = d["roofline"]
    out = {"ms_per_step": round(d["ms_per_step"], 4), "value": d["value"], "decisions_per_step": d["decisions_per_step"],
           "kernel_ms": round(r["kernel_ms"], 4), "frac_hw": r["frac_hw"] and round(r["frac_hw"], 4),
           "traffic": r["traffic"], "frac_survey_model": round(r["frac"], 3),
           "frac_engine_model": round(r["frac_engine_model"], 4),
           "verified": d["verified"]["step_state_digest_vs_run"]}
    cb = d.get("cpu_baseline")
    if cb:
        out["cpu_baseline"] = {k: cb.get(k) for k in ("value", "unit", "cores", "kind", "error") if k in cb}
        if cb.get("value"):
            out["vs_cpu"] = round(d["value"] / cb["value"], 1)
    w = d.get("windows")
    if w:
        out["windows"] = {"windows": w["windows"], "host_ms_per_window": round(w["host_ms_per_window"], 2),
                          "host_ms_per_window_sequential": round(w["host_ms_per_window_sequential"], 2),
                          "value_sequential": w["value_sequential"],
                          "submit_ms_per_window": round(w["submit_ms_per_window"], 2),
                          "device_ms_per_window": round(w["device_ms_per_window"], 4), "value": w["value"],
                          "value_device": w["value_device"], "kernel_ms": round(w["roofline"]["kernel_ms"], 4),
                          "frac_hw": w["roofline"]["frac_hw"] and round(w["roofline"]["frac_hw"], 4),
                          "verified": w["verified"]["digests_vs_batch_run"]}
        if cb:                                   # (the same C3 workload, fed window by window)
            out["windows"]["cpu_baseline"] = out["cpu_baseline"]
            if cb.get("value"):
                out["windows"]["vs_cpu"] = round(w["value"] / cb["value"], 2)
    return out


def log_leg(name, d):
    if not d or "error" in d:
        log("leg %s: %r" % (name, d))
        return
    r = d["roofline"]
    cb = d.get("cpu_baseline") or {}
    log("leg %s: ms_per_step %.4f, %.3f G decisions/s, apply kernel_ms %.4f, frac_hw %s, cpu_baseline %s" % (
        name, d["ms_per_step"], d["value"] / 1e9, r["kernel_ms"],
        "%.3f" % r["frac_hw"] if r["frac_hw"] else "null",
        "%.3g decisions/s on %s cores (%s)" % (cb["value"], cb["cores"], cb["kind"]) if cb.get("value") else "none"))
    w = d.get("windows")
    if w:
        log("leg %s.windows: host %.2f ms / window pipelined (%.2f sequential, submit %.2f), device %.4f ms, "
            "%.3g decisions/s end to end, %.3g on the device, k_apply_win %.4f ms, frac_hw %s" % (
                name, w["host_ms_per_window"], w["host_ms_per_window_sequential"], w["submit_ms_per_window"],
                w["device_ms_per_window"], w["value"],
                w["value_device"], w["roofline"]["kernel_ms"],
                "%.3f" % w["roofline"]["frac_hw"] if w["roofline"]["frac_hw"] else "null"))


def native_oracle():
    """oracle/mpx_oracle.c compiled here with -O2 -march=native (the CPU
    restatement built for this host's CPU); the prebuilt generic one when gcc is missing."""
    import subprocess
    import tempfile
    out = os.path.join(tempfile.gettempdir(), "mpx_oracle_native_%d.so" % os.getpid())
    try:
        subprocess.check_call(["gcc", "-O2", "-march=native", "-std=gnu99", "-fPIC", "-shared", "-o", out,
                               os.path.join(ROOT, "oracle", "mpx_oracle.c"), "-lpthread"],
                              stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        return out, "-O2 -march=native (built on this host)"
    except (OSError, subprocess.CalledProcessError):
        return os.path.join(ROOT, "oracle", "_build", "libmpx_oracle.so"), "-O2 generic (gcc unavailable here)"


def cpu_port_baseline(args, budget_s):
    """The build's own CPU restatement (oracle/mpx_oracle.c, SURVEY §8(d)(ii): -O2 -march=native,
    the host cores cpu_threads allows) over a clean C4-shaped trace: instance shards in parallel
    (mpxo_run_sharded), each shard every node's stream on its own thread; counters + digests only."""
    so, flags = native_oracle()
    lib = ctypes.CDLL(so)
    f = lib.mpxo_run_sharded
    f.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]
    f.restype = ctypes.c_int
    cores = cpu_threads()
    shards = max(1, cores // args.nodes)              # shards x N node threads ~ the cores the quota gives
    sample_m = max(1 << 18, shards << 15)
    trace = mpx.generate_trace(mpx.GEN_CLEAN, num_nodes=args.nodes, num_instances=sample_m, batch=256, copy=False)
    stats = (ctypes.c_uint64 * 8)()

    def once():
        if f(trace, len(trace), shards, shards, stats) != 0:
            raise RuntimeError("mpxo_run_sharded failed")

    t0 = time.perf_counter()
    once()
    one = time.perf_counter() - t0
    assert stats[0] == sample_m
    reps = max(1, int(budget_s / max(one, 1e-6)))
    log("cpu_baseline_port: %d shards x %d node threads, one pass %.2f s, %d passes" % (shards, args.nodes, one, reps))
    t0 = time.perf_counter()
    for _ in range(reps):
        once()
    dt = time.perf_counter() - t0
    if so.startswith("/tmp") or "mpx_oracle_native" in so:
        try:
            os.remove(so)
        except OSError:
            pass
    return {"value": reps * sample_m / dt, "unit": "decisions/s", "cores": shards * args.nodes, "kind": "port",
            "sample": "oracle/mpx_oracle.c (the build's C restatement, %s) over a clean C4-shaped trace of %d "
                      "instances x %d acceptors: %d instance shards x %d node threads, %d passes in %.1f s (%s)"
                      % (flags, sample_m, args.nodes, shards, args.nodes, reps, dt, cpu_note())}


def shard_projection(args, t1_ms):
    """Rank 0's instance shard of the headline trace at world G, run alone on this GPU: the
    per-rank work of a G-GPU strong-scaling run without its RCCL all-gather.  eff = T1 / (G * T_shard)
    is a projection, not a scaling measurement (instance shards are independent)."""
    G, M, N = args.shard_of, args.instances, args.nodes
    sb, se = mdist.shard_bounds(M, G, 0)
    eng = mpx.Engine(N, sb, se)
    eng.load_clean_device(num_instances=M, batch=args.batch)
    for _ in range(max(args.warmup, 3)):
        eng.step()
    eng.sync()
    eng.timings()
    eng.timing_every(max(args.events_every, 1) * 2)
    steps = max(args.steps, 50)
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.step()
    eng.sync()
    dt = time.perf_counter() - t0
    ph = eng.timings_detail()
    st = eng.stats()
    want = clean_expect(N, sb, se)
    ok = eng.state_digest() == want and st["chosen"] == se - sb
    eng.close()
    assert ok, "shard projection: the step's state differs from the closed form"
    t_shard = dt / steps * 1e3
    out = {"G": G, "shard": [sb, se], "steps": steps, "T1_ms": t1_ms, "T_shard_ms": t_shard,
           "phase_events_every": max(args.events_every, 1) * 2,
           "eff": t1_ms / (G * t_shard) if t1_ms else None,
           "phases_ms": {k: sum(p[k] for p in ph) / max(len(ph), 1) for k in mpx.Engine.PHASES},
           "verified": ok,
           "note": "projection, no RCCL: rank 0's shard of the same trace timed alone on one GPU"}
    log("shard-of-%d: %.4f ms per step (T1 %.4f ms): projected efficiency %.3f" %
        (G, t_shard, t1_ms or 0.0, out["eff"] or 0.0))
    return out


def main():
    args = parse()
    if args.shard_only:
        print(json.dumps({"scaling_projection": shard_projection(args, None)}), flush=True)
        return
    if args.c3_only:
        print(json.dumps({"c3": c3_leg(args)}), flush=True)
        return
    if args.c3_windows_only:
        trace = mpx.generate_trace(mpx.GEN_FAULTY, num_instances=args.c3_instances, copy=False, **C3)
        with mpx.Engine.for_trace(trace) as e:
            chk = e.run()
        print(json.dumps({"c3_windows": c3_windows_leg(args, trace, (chk["state_digest"], chk["chosen_digest"]),
                                                       {k: chk[k] for k in ("chosen", "promise_entries",
                                                                            "accept_apps", "commit_apps")})}),
              flush=True)
        return
    if args.c5_only:
        print(json.dumps({"c5": c3_leg(args, "c5")}), flush=True)
        return
    if args.loop_only:
        print(json.dumps({"closed_loop": closed_loop_leg(args)}), flush=True)
        return
    if args.c5c_only:
        print(json.dumps({"c5_contended": c3_leg(args, "c5c")}), flush=True)
        return
    world, rank, local, pg = dist_setup(args)
    if args.gpus != world and world > 1:
        print("warning: --gpus %d but WORLD_SIZE %d" % (args.gpus, world), file=sys.stderr)
    M, N = args.instances, args.nodes
    sb, se = mdist.shard_bounds(M, world, rank)       # contiguous, bucket-aligned instance shard
    eng = mpx.Engine(N, sb, se, device=local)
    if pg is not None:
        uid = broadcast_bytes(pg, mpx.Engine.comm_unique_id() if rank == 0 else None, rank)
        eng.comm_init(uid, rank, world)
    t_gen = time.perf_counter()
    eng.load_clean_device(num_instances=M, batch=args.batch)
    t_gen = time.perf_counter() - t_gen

    for _ in range(args.warmup):
        eng.step()
    eng.sync()
    eng.timings()                                   # drop warmup timings
    eng.timing_every(max(args.events_every, 1))     # phase events on a sample of the timed steps

    barrier(pg)
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.step()
    eng.sync()
    dt = time.perf_counter() - t0
    barrier(pg)
    dt_max = allreduce_max(pg, dt)

    st = eng.stats()
    ph = eng.timings_detail()                       # per timed step: phase -> ms (HIP events)
    apply_ms = [p["fast_apply"] + p["general_apply"] for p in ph]
    run_ms = [p["run"] for p in ph]
    phases = {k: sum(p[k] for p in ph) / max(len(ph), 1) for k in mpx.Engine.PHASES}
    tot = mdist.combine(eng.allgather_summary(world))   # also checks per-acceptor scalars agree
    chosen_total = tot["chosen"]
    assert chosen_total == M, "chosen %d != %d instances" % (chosen_total, M)
    assert tot["violations"] == 0
    # verification, outside the timed region: (1) the state the last TIMED step's kernel
    # (k_plan_store8) wrote, digested by a separate device pass; (2) one digested run
    want_state, want_chosen = clean_expect(N, sb, se)
    step_state, step_chosen = eng.state_digest()
    step_ok = (step_state, step_chosen) == (want_state, want_chosen) and \
        st["accept_apps"] == N * (se - sb) == st["commit_apps"]
    assert step_ok, "the timed step's final state differs from the clean trace's closed form"
    # (3) the reference's own handlers on the same C4 trace (oracle/ref_full_size.py: 128 instance
    # shards of multi/paxos.cpp compiled in place, tests/golden/full_size.json["c4"]) — the shards'
    # digests add up to the whole trace's (sums of per-entry hashes mod 2^64)
    import struct
    parts = pg.exchange(struct.pack("<QQ", step_state, step_chosen)) if pg is not None else \
        [struct.pack("<QQ", step_state, step_chosen)]
    tot_state = sum(struct.unpack("<QQ", b)[0] for b in parts) & ((1 << 64) - 1)
    tot_chosen = sum(struct.unpack("<QQ", b)[1] for b in parts) & ((1 << 64) - 1)
    ref_c4 = reference_c4(M, N, args.batch)
    step_vs_ref = None if ref_c4 is None else \
        (tot_state, tot_chosen) == (ref_c4["state_digest"], ref_c4["chosen_digest"])
    assert step_vs_ref is not False, "the timed step's digests differ from the reference's own handlers"
    chk = eng.run()
    eng.timings()
    verified = (chk["state_digest"] == want_state and chk["chosen_digest"] == want_chosen and
                chk["accept_apps"] == N * (se - sb) == chk["commit_apps"] and chk["chosen"] == se - sb)
    assert verified, "digests / counters differ from the clean trace's closed form"

    value = chosen_total * args.steps / dt_max
    ms_per_step = dt_max / args.steps * 1e3
    apply_mean = sum(apply_ms) / max(len(apply_ms), 1)
    bytes_survey = st["bytes_alg"]                  # this rank's 16P + 24A + 16L per launch
    L = se - sb
    # 1-B state slots + 1-B chosen log (the device-generated clean trace has 2 runs per pair, so
    # mpx_load_clean_device picks 1-byte slots) + the ACCEPT and COMMIT descriptors of every (node, bucket)
    # (k_plan_store8 keeps the plan words in LDS; before round 6, k_plan wrote them and k_store8 read them back:
    # + 16 B per (row, bucket))
    nb = (L + 255) // 256
    runs = sum(((min(b0 + 256, se) - 1) // args.batch - b0 // args.batch + 1)
               for b0 in range(sb, se, 256)) if args.batch != 256 else nb   # batch runs meeting each bucket
    bytes_min = 1 * N * L + 1 * L + 2 * 16 * N * runs
    achieved_eng = bytes_min / (apply_mean * 1e-3) / 1e9 if apply_mean else 0.0
    pmc = latest_pmc(N, M, world)
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    traffic_src = ("profiles/%s_pmc.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE passes of this command, "
                   "committed; not measured inside this process)" % pmc["tag"]) if pmc else None
    # roofline.frac is the hardware fraction: the PMC bytes the timed
    # apply-phase kernels move per launch / the phase's mean duration of THIS run / 8 TB/s.
    # Without a profile at these sources it falls back to the engine's byte model (basis says so).
    hw = hw_roofline(pmc, apply_mean)
    achieved = hw["achieved"] if hw else achieved_eng
    basis = ("pmc: %s traffic / this run's kernel_ms" % hw["source"]) if hw else \
        "engine_model (no PMC profile at this source digest): DESIGN.md §4 bytes / kernel_ms"

    log("C4: %.4f ms per step over %d steps, verified %s (closed form), step digests vs the reference's own "
        "handlers %s" % (dt_max / args.steps * 1e3, args.steps, verified, step_vs_ref))
    out = None
    if rank == 0:
        cpu = cpu_port = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args, args.cpu_seconds)
            cpu_port = cpu_port_baseline(args, args.cpu_seconds / 2)
        proj = shard_projection(args, ms_per_step) if world == 1 and args.shard_of > 1 else None
        c3 = c3_leg(args) if world == 1 and args.c3_instances else None
        def secondary(kind):
            try:                                    # a secondary leg: out of memory is reported, not fatal;
                return c3_leg(args, kind)           # a wrong result (AssertionError) or any other error is
            except MemoryError as ex:               # fatal
                return {"error": repr(ex)}
            except mpx.MpxError as ex:
                if ex.rc != -2:                     # MPX_E_NOMEM
                    raise
                return {"error": repr(ex)}
        c5 = secondary("c5") if world == 1 and args.c5_instances else None
        c5c = secondary("c5c") if world == 1 and args.c5c_instances else None
        loop = secondary_loop(args) if world == 1 and args.loop_values else None
        # every leg's same-workload reference CPU rate
        for name, leg in (("c3", c3), ("c5", c5), ("c5c", c5c)):
            if leg and "error" not in leg and world == 1 and not args.no_cpu_baseline:
                leg["cpu_baseline"] = leg_cpu_baseline(name, args.leg_cpu_instances)
                if leg["cpu_baseline"] and leg["cpu_baseline"].get("value"):
                    leg["vs_cpu"] = leg["value"] / leg["cpu_baseline"]["value"]
            log_leg(name, leg)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "decisions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (device-generated clean trace, decoded+bucketed in HBM before timing)",
            "config": {"workload": "C4: 2^27 instances x 9 acceptors, clean single round, batch 256, "
                                   "instance-sharded over the GPUs" if (M, N, args.batch) == (1 << 27, 9, 256) else
                                   "clean: %d instances x %d acceptors, batch %d" % (M, N, args.batch),
                       "instances": M, "acceptors": N, "batch": args.batch, "shard_per_gpu": se - sb,
                       "parallelism": "instance-shard x%d (RCCL all-gather of 64-word summaries)" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "basis": basis,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "apply phase: k_plan_store8 (plan in LDS + store, one launch)",
                         "kernel_ms": apply_mean, "bytes_alg_per_launch": bytes_min,
                         "achieved_engine_model": achieved_eng,
                         "frac_engine_model": achieved_eng / HBM_PEAK_GBS,
                         "bytes_model": "engine model, DESIGN.md §4: 1-B slot per (acceptor, instance) + 1-B chosen "
                                        "log + 16-B ACCEPT / COMMIT descriptors per run (plan words stay in LDS)",
                         "bytes_survey_model_per_launch": bytes_survey,
                         "survey_model_gbps": bytes_survey / (apply_mean * 1e-3) / 1e9 if apply_mean else 0.0,
                         "frac_survey_model": bytes_survey / (apply_mean * 1e-3) / 1e9 / HBM_PEAK_GBS
                         if apply_mean else 0.0,
                         "note": "frac = PMC traffic / kernel_ms / 8 TB/s (what the HBM moved); frac_survey_model is "
                                 "NOT a fraction when > 1. "
                                 "The clean trace fixes every (acceptor, bucket) pair with one full run, so its apply "
                                 "phase reduces to one plan word per pair and a byte stream of slots (k_plan_store8): the "
                                 "survey model's 360 B/instance (16-B slot writes + per-acceptor Value reads) are "
                                 "never moved, and frac_survey_model > 1 measures representation, not bandwidth; "
                                 "c3.roofline is the per-slot general path on the survey's bytes"},
            "cpu_baseline": cpu,
            "cpu_baseline_port": cpu_port,
            **({"scaling_projection": proj} if proj else {}),
            "c3": c3,
            **({"c5": c5} if c5 else {}),
            **({"c5_contended": c5c} if c5c else {}),
            **({"closed_loop": loop} if loop else {}),
            "verified": {"step_state_digest_vs_closed_form": step_ok, "step_digests_vs_reference": step_vs_ref,
                         "step_state_digest": step_state,
                         "step_chosen_digest": step_chosen, "run_digests_vs_closed_form": verified,
                         "state_digest": chk["state_digest"], "chosen_digest": chk["chosen_digest"]},
            "hbm_gbps_alg_step": bytes_min * world / (dt_max / args.steps) / 1e9,
            "decisions_per_step": chosen_total,
            "run_ms_device": sum(run_ms) / max(len(run_ms), 1),
            "phases_ms": phases,
            "phase_events_every": max(args.events_every, 1),
            "trace_materialise_s": t_gen,
        }
        if args.detail:
            try:
                os.makedirs(os.path.dirname(os.path.abspath(args.detail)), exist_ok=True)
                with open(args.detail, "w") as fh:
                    json.dump(out, fh, indent=1)
            except OSError as ex:
                log("detail not written: %r" % ex)
        # the JSON line: the contract's keys, the headline roofline and CPU baseline, then every
        # leg's headline figures — short enough that a driver's tail of stdout holds all of it
        keep_roof = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "kernel_ms",
                     "bytes_alg_per_launch", "frac_engine_model", "frac_survey_model")
        line = {k: out[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                    "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")}
        line["roofline"] = dict({k: out["roofline"][k] for k in keep_roof},
                                basis=out["roofline"]["basis"].split(" traffic")[0])
        line["cpu_baseline"] = cpu
        line["legs"] = {"c3": compact_leg(c3), "c5": compact_leg(c5), "c5_contended": compact_leg(c5c)}
        if loop:
            line["legs"]["closed_loop"] = {k: loop[k] for k in ("value", "unit", "windows", "ms_per_window",
                                                                "verified", "vs_cpu") if k in loop} \
                if "error" not in loop else loop
            if loop.get("cpu_baseline"):
                line["legs"]["closed_loop"]["cpu_baseline"] = {k: loop["cpu_baseline"].get(k) for k in
                                                              ("value", "unit", "cores", "kind")}
        if proj:
            line["scaling_projection"] = {k: proj[k] for k in ("G", "T1_ms", "T_shard_ms", "eff", "verified")}
        line["cpu_baseline_port"] = {k: cpu_port[k] for k in ("value", "unit", "cores", "kind")} if cpu_port else None
        line["verified"] = {k: out["verified"][k] for k in ("step_state_digest_vs_closed_form",
                                                            "run_digests_vs_closed_form")}
        for k in ("step_digests_vs_reference",):
            if k in out["verified"]:
                line["verified"][k] = out["verified"][k]
        line["phases_ms"] = {k: round(v, 4) for k, v in phases.items()}
        line["detail"] = args.detail
        print(json.dumps(line), flush=True)
    eng.close()
    if pg is not None:
        pg.close()


if __name__ == "__main__":
    main()
