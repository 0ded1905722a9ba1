"""Hand-written traces, one per reference quirk."""
from mpxwire import (U64_MAX_EXCL, accept, accept_reply, commit, commit_reply,
                     container, p_batch, p_propose, p_start, prepare, prepare_reply,
                     reject, value)

B1 = (1 << 16) | 0
B2 = (2 << 16) | 1
B3 = (3 << 16) | 2


def v(i, p=0, vid=None):
    return value(p, (vid if vid is not None else i + 1), str(i))


def handmade_traces():
    t = {}
    # 1. clean single round, 3 nodes
    ent = [(0, v(0)), (1, v(1)), (2, v(2))]
    s0 = [p_start(B1), prepare(0, B1)] + [prepare_reply(i, B1) for i in range(3)] + \
         [p_batch(1, ent), accept(0, 1, B1, ent)] + [accept_reply(i, B1, 1) for i in range(3)] + \
         [commit(0, 1, B1, ent)] + [commit_reply(i, 1) for i in range(3)]
    si = [prepare(0, B1), accept(0, 1, B1, ent), commit(0, 1, B1, ent)]
    t["hm_clean3"] = container([s0, si, si], 3)

    # 2. Appendix B.1-3: equal-ballot prepare silent, lower rejected, promise is one scalar
    t["hm_prepare_ballots"] = container([[
        prepare(1, B2), prepare(1, B2), prepare(0, B1), prepare(2, B3), prepare(1, B2)], [], []], 1)

    # 3. B.2: accept does not raise promise; lower (>= promised) accept overwrites higher
    t["hm_accept_overwrite"] = container([[
        prepare(0, B1),
        accept(1, 7, B2, [(5, v(5, 1, 50))]),
        accept(0, 3, B1, [(5, v(5, 0, 51))]),          # B1 >= promised(B1): overwrites B2's value
        prepare(2, B2),                                 # granted (B2 > B1): replies with iid 5 @B1
        accept(0, 4, B1, [(6, v(6))]),                  # B1 < promised(B2): REJECT(max_seen=B2)
        reject(B3),
        accept(1, 8, B2, [(6, v(6, 1, 60))]),
        prepare(0, B1, [(0, 6)]),                       # rejected with max_seen = B3
    ], [], []], 10)

    # 4. B.5-7: commit first wins the tag, accept skips committed, replies mix tags
    t["hm_commit_tags"] = container([[
        accept(0, 1, B1, [(1, v(1)), (2, v(2)), (3, v(3))]),
        commit(0, 1, B1, [(2, v(2))]),
        commit(1, 9, B2, [(2, v(2)), (3, v(3))]),      # iid 2 keeps B1, iid 3 gets B2
        accept(2, 1, B3, [(2, v(2, 2, 99)), (4, v(4))]),   # iid 2 committed: skipped
        prepare(2, B3, [(0, 3), (4, U64_MAX_EXCL)]),    # ranges: iid 1,2 and 4
        commit(0, 2, B1, [(0, v(0)), (1, v(1))]),       # executes 0,1,2,3 in order
    ], [], []], 8)

    # 5. B.8-9: promise merge strict >, ties keep first arrival; stale / late replies ignored
    e_a = [(4, B1, v(4, 1, 40)), (5, B2, v(5, 1, 50))]
    e_b = [(4, B1, v(4, 2, 41)), (5, B3, v(5, 2, 52)), (6, B1, v(6))]
    t["hm_promise_merge"] = container([[
        prepare_reply(0, B2, e_a),                      # not preparing: ignored
        p_start(B2),
        prepare_reply(0, B1, e_b),                      # stale ballot: ignored
        prepare_reply(1, B2, e_a),
        prepare_reply(1, B2, e_b),                      # same acceptor again: merges, no new vote
        prepare_reply(3, B2, e_b),                      # quorum (3 of 4)
        prepare_reply(2, B2, e_a),                      # after quorum: ignored
        reject(B3),
    ], [], [], []], 8)

    # 6. accept votes: unknown batch, stale ballot, duplicate acceptor, after-quorum
    ent = [(0, v(0)), (1, v(1))]
    t["hm_votes"] = container([[
        p_start(B1), prepare_reply(0, B1), prepare_reply(1, B1), prepare_reply(2, B1),
        p_batch(11, ent), p_batch(12, [(2, v(2))]),
        accept_reply(0, B1, 11), accept_reply(0, B1, 11), accept_reply(1, B2, 11),
        accept_reply(3, B1, 99), accept_reply(2, B1, 12), accept_reply(4, B1, 11),
        accept_reply(1, B1, 11),                        # quorum for 11 (0,4,1)
        accept_reply(2, B1, 11),                        # retired: ignored
        p_start(B2),                                    # AcceptRejected: batch 12 dropped
        accept_reply(3, B1, 12), accept_reply(0, B1, 12), accept_reply(1, B1, 12),
        commit_reply(2, 1),
    ], [], [], [], []], 4)

    # 7. client proposals (Propose, OnPrepareReply's own / new values, OnCommit re-propose;
    # multi/paxos.cpp:1132-1175,1250-1280,1524-1570): node 0 of 3
    a, b, c = value(0, 1, "a"), value(0, 2, "b"), value(0, 6, "c")
    other = value(1, 7, "x")
    t["hm_propose"] = container([[
        p_propose("a"),                                 # not preparing: instance 0 at once (value id 1)
        p_batch(1, [(0, a)]),
        p_start(B1),                                    # AcceptRejected -> preparing
        p_propose("b"),                                 # queued (value id 2)
        prepare_reply(1, B1, [(3, B1 - 1, other)]),
        prepare_reply(2, B1),                           # quorum: adopt 3, noops 0..2 (ids 3..5), b at 4
        commit(1, 5, B1, [(0, value(0, 3, noop=True))]),   # 0 committed as a noop: "a" re-proposed at 5
        p_batch(3, [(5, a)]),
        p_propose("c"),                                 # not preparing: instance 6 (value id 6)
        p_batch(4, [(6, c)]),
        p_start(B3),
        prepare_reply(1, B3, [(2, B1, value(1, 8, "y"))]),
        commit(2, 6, B3, [(1, value(0, 4, noop=True)), (6, other)]),   # 6 lost: "c" queued again
        prepare_reply(2, B3),                           # quorum: adopt 2, noops 3..5 (own 4, 5 among
                                                        # them: the fill comes first), c at 7
    ], [prepare(0, B1), accept(0, 1, B1, [(0, a)])], []], 16)
    return t
