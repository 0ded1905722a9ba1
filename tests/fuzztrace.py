"""Random, reference-valid traces for parity testing (test helper).

Every trace exercises the quirks listed in SURVEY.md Appendix B — prepare with
an equal ballot is silent, accept does not raise the promise and overwrites
even with a lower ballot, the first commit wins the ballot tag, promise
replies carry accepted and committed entries, the pre-accepted merge keeps the
first arrival on ties, stale / unknown-batch replies are ignored — while never
tripping one of the reference's ASSERTs (so the reference driver can run it):
  * an instance is always committed with the same Value (paxos.cpp:1508);
  * iids are unique inside a message, prepare ranges are disjoint;
  * replies name real nodes; P_BATCH only when the proposer is not preparing
    (paxos.cpp:1054);
  * every Value belongs to one instance (OnCommit's proposer bookkeeping,
    paxos.cpp:1512-1537).
"""
import random

from mpxwire import (U64_MAX_EXCL, accept, accept_reply, commit, commit_reply,
                     container, p_batch, p_start, prepare, prepare_reply,
                     reject, value, value_member)


def fuzz_trace(seed, n_nodes=None, n_inst=None, n_msgs=None, member_values=False):
    rng = random.Random(seed)
    N = n_nodes or rng.randint(1, 6)
    M = n_inst or rng.randint(1, 48)
    K = n_msgs if n_msgs is not None else rng.randint(10, 120)
    ballots = sorted({(rng.randint(1, 6) << 16) | rng.randrange(max(N, 1)) for _ in range(6)})

    # candidate Values per instance; value ids globally unique per proposer
    vid = [0] * 8
    cands = []
    for i in range(M):
        row = []
        for _ in range(rng.randint(1, 3)):
            p = rng.randrange(min(N + 1, 8))          # sometimes a proposer that is no node
            vid[p] += 1
            kind = rng.random()
            if kind < 0.15:
                v = value(p, vid[p], noop=True)
            elif member_values and kind < 0.25:
                v = value_member(p, vid[p], rng.randrange(9))   # delete form: the add form double-frees in the reference (implicit MembershipChange copy, paxos.cpp:112-123)
            else:
                v = value(p, vid[p], "v%d-%d" % (i, len(row)) * rng.randint(0, 2))
            row.append(v)
        cands.append(row)
    chosen = [rng.choice(r) for r in cands]

    def iids(lo=1, hi=8):
        k = min(M, rng.randint(lo, hi))
        return sorted(rng.sample(range(M), k))

    streams = []
    for node in range(N):
        msgs = []
        ballot = 0
        preparing = False
        mask = 0
        batches = []
        for _ in range(K):
            r = rng.random()
            if r < 0.12:
                ranges = []
                cuts = sorted(rng.sample(range(M + 1), min(M + 1, 2 * rng.randint(1, 2))))
                for a, b in zip(cuts[0::2], cuts[1::2]):
                    ranges.append((a, b))
                if rng.random() < 0.5:
                    lo = (ranges[-1][1] if ranges else 0) + rng.randint(0, 3)
                    ranges.append((lo, U64_MAX_EXCL))
                msgs.append(prepare(rng.randrange(N), rng.choice(ballots), ranges))
            elif r < 0.34:
                ent = [(i, rng.choice(cands[i])) for i in iids()]
                msgs.append(accept(rng.randrange(N), rng.randint(1, 9), rng.choice(ballots), ent))
            elif r < 0.48:
                ent = [(i, chosen[i]) for i in iids()]
                msgs.append(commit(rng.randrange(N), rng.randint(1, 50), rng.choice(ballots), ent))
            elif r < 0.53:
                msgs.append(reject(rng.choice(ballots + [0, 1 << 40])))
            elif r < 0.58:
                ballot = rng.choice(ballots)
                msgs.append(p_start(ballot))
                preparing, mask, batches = True, 0, []
            elif r < 0.72:
                # promise reply, mostly for the current ballot
                b = ballot if rng.random() < 0.75 else rng.choice(ballots)
                acc = rng.randrange(N)
                ent = [(i, rng.choice(ballots), rng.choice(cands[i])) for i in iids(0, 6)]
                msgs.append(prepare_reply(acc, b, ent))
                if preparing and b == ballot:
                    mask |= 1 << acc
                    if bin(mask).count("1") >= N // 2 + 1:
                        preparing, mask = False, 0
            elif r < 0.80:
                if not preparing and ballot:
                    bid = rng.randint(1, 1 << 20)
                    while bid in batches:
                        bid += 1
                    batches.append(bid)
                    ent = [(i, rng.choice(cands[i])) for i in iids()]
                    msgs.append(p_batch(bid, ent))
            elif r < 0.95:
                b = ballot if rng.random() < 0.8 else rng.choice(ballots)
                bid = rng.choice(batches) if batches and rng.random() < 0.85 else rng.randint(1, 9)
                msgs.append(accept_reply(rng.randrange(N), b, bid))
            else:
                msgs.append(commit_reply(rng.randrange(N), rng.randint(1, 50)))
        streams.append(msgs)
    return container(streams, M)
