"""Hand-written member-semantics traces.

Every node starts in epoch 0 = {node 0} (NodeImpl::Loop, member/paxos.cpp:738-747);
larger acceptor sets are reached the way the reference reaches them: membership
Values learned in instance order and applied by ChangeMemberships (:1864-1964),
each version step marked by an E_EPOCH record in the node's stream.  Node 0's own
Values reach its Proposer as P_PROPOSE records (Node::Propose -> Proposer::Propose,
:1122-1156) before they are sent, and carry the value ids Propose gives them
(value_id_ + 1 per Propose and per noop of its own batches).
"""
from mpxwire import (U64_MAX_EXCL, ADD_LEARNER, LEARNER_TO_PROPOSER, PROPOSER_TO_ACCEPTOR,
                     ACCEPTOR_TO_PROPOSER, PROPOSER_TO_LEARNER, DEL_LEARNER,
                     container, e_epoch, m_accept, m_accept_reply, m_learn, m_learn_reply,
                     m_p_batch, m_p_propose, m_prepare, m_prepare_reply, mvalue, p_start, reject)

B0 = (1 << 16) | 0
B1 = (2 << 16) | 0
B2 = (3 << 16) | 1
B3 = (4 << 16) | 2


def add_acceptor(i):
    return [(i, ADD_LEARNER), (i, LEARNER_TO_PROPOSER), (i, PROPOSER_TO_ACCEPTOR)]


def del_acceptor(i):
    return [(i, ACCEPTOR_TO_PROPOSER), (i, PROPOSER_TO_LEARNER), (i, DEL_LEARNER)]


def mask(*nodes):
    m = 0
    for n in nodes:
        m |= 1 << n
    return m


def v(i, p=0, vid=None, cb="cb"):
    """normal Value: payload = decimal instance id, cb as the demo's (member/main.cpp)"""
    return mvalue(p, vid if vid is not None else 100 + i, str(i), cb)


class Member:
    """Bootstrap: instances 0..k-1 hold AddAcceptor(1..k) proposed by node 0 (value ids 1..k,
    its first Proposes, taken at once: its Proposer is idle, member/paxos.cpp:1131-1150)."""

    def __init__(self, n_nodes, n_acceptors, extra_epochs=()):
        self.N = n_nodes
        self.k = n_acceptors - 1
        self.epochs = [(0, 1, 1)]
        for j in range(1, n_acceptors):
            m = mask(*range(j + 1))
            self.epochs.append((j, m, m))
        self.epochs += list(extra_epochs)
        self.boot = [(j - 1, B0, mvalue(0, j, cb="m%d" % j, changes=add_acceptor(j))) for j in range(1, n_acceptors)]
        self.vid = self.k                         # node 0's value_id_ after the bootstrap proposals
        self.streams = [[] for _ in range(n_nodes)]

    def bootstrap(self, nodes=None):
        """every listed node learns the bootstrap values and steps its epochs; node 0 proposed them"""
        for i in (range(self.N) if nodes is None else nodes):
            pre = [m_p_propose(v) for _i, _p, v in self.boot] if i == 0 else []
            self.streams[i] += pre + [m_learn(0, 1, self.boot)] + [e_epoch(j) for j in range(1, self.k + 1)]

    def own(self, i, cb="cb", changes=None):
        """node 0's next own Value (the next value id its Proposer gives) and its P_PROPOSE record"""
        self.vid += 1
        val = mvalue(0, self.vid, cb=cb, changes=changes) if changes else mvalue(0, self.vid, str(i), cb)
        return val, m_p_propose(val)

    def trace(self, M=64):
        return container(self.streams, M, semantics=1, epochs=self.epochs)


def member_traces():
    t = {}
    ver = 2                                               # after AddAcceptor(1), AddAcceptor(2)

    # 1. clean round with 3 acceptors of 3 nodes
    m = Member(3, 3)
    m.bootstrap()
    own = [m.own(i) for i in (2, 3, 4)]
    ent = [(i, B1, own[i - 2][0]) for i in (2, 3, 4)]
    s0 = m.streams[0]
    s0 += [p_start(B1)] + [x[1] for x in own] + [m_prepare(ver, 0, B1, [(2, U64_MAX_EXCL)])]
    s0 += [m_prepare_reply(i, B1) for i in range(3)]
    s0 += [m_p_batch(1, ent), m_accept(ver, 0, 1, B1, ent)] + [m_accept_reply(i, 1) for i in range(3)]
    s0 += [m_learn(0, 2, ent)] + [m_learn_reply(i, 2) for i in range(3)]
    for i in (1, 2):
        m.streams[i] += [m_prepare(ver, 0, B1, [(2, U64_MAX_EXCL)]), m_accept(ver, 0, 1, B1, ent), m_learn(0, 2, ent)]
    t["mm_clean3"] = m.trace()

    # 2. version filter: other versions are dropped silently (:1702,1744), before max_seen
    m = Member(3, 3)
    m.bootstrap()
    m.streams[1] += [
        m_prepare(1, 0, B3),                              # stale version: dropped
        m_prepare(ver, 0, B1),                            # granted
        m_accept(ver + 1, 0, 5, B3, [(7, B3, v(7))]),     # future version: dropped
        m_accept(1, 0, 5, B3, [(7, B3, v(7))]),           # stale: dropped
        m_accept(ver, 0, 6, B1, [(7, B1, v(7))]),         # granted
        m_prepare(ver, 0, B0),                            # lower: REJECT(max_seen = B1)
    ]
    t["mm_version_drop"] = m.trace()

    # 3. accept = insert: the first accepted value sticks, even under a higher ballot (:1765)
    m = Member(3, 3)
    m.bootstrap()
    m.streams[2] += [
        m_prepare(ver, 0, B1),
        m_accept(ver, 0, 1, B1, [(5, B1, v(5, 0, 50)), (6, B1, v(6))]),
        m_accept(ver, 1, 2, B2, [(5, B2, v(5, 1, 51)), (7, B2, v(7, 1))]),
        m_prepare(ver, 1, B2, [(5, 8)]),                  # B2 > promised(B1): reply 5@B1, 6@B1, 7@B2
        m_accept(ver, 0, 3, B1, [(8, B1, v(8))]),         # B1 < promised(B2): REJECT(max B2)
        m_prepare(ver, 2, B3, [(0, 6), (7, U64_MAX_EXCL)]),   # learned 0,1 + accepted 5, 7
    ]
    t["mm_insert_first"] = m.trace()

    # 4. learn = insert (:1040); Acceptor::OnLearn erases accepted (:1786-1793);
    #    accept of a learned instance is skipped (:1763-1769); apply in order
    m = Member(3, 3)
    m.bootstrap()
    m.streams[1] += [
        m_prepare(ver, 0, B1),
        m_accept(ver, 0, 1, B1, [(3, B1, v(3)), (4, B1, v(4)), (5, B1, v(5))]),
        m_learn(0, 7, [(4, B1, v(4)), (2, B0, v(2))]),    # 4 leaves accepted; executes 2
        m_accept(ver, 0, 2, B1, [(4, B1, v(4)), (6, B1, v(6))]),   # 4 learned: skipped
        m_learn(2, 8, [(3, B2, v(3)), (4, B3, v(4))]),    # 4 already learned: keeps B1
        m_prepare(ver, 2, B3, [(2, U64_MAX_EXCL)]),       # learned 2,3,4 + accepted 5,6
    ]
    t["mm_learn_first"] = m.trace()

    # 5. acceptor reset: AcceptorToProposer(2) then ProposerToAcceptor(2) — the new
    #    Acceptor starts with promised = max = 0 and nothing accepted (:1897-1901,1952-1957)
    m = Member(3, 3, extra_epochs=[(3, mask(0, 1), mask(0, 1, 2)), (4, mask(0, 1, 2), mask(0, 1, 2))])
    m.bootstrap()
    a2p, pa2p = m.own(2, cb="a2p", changes=[(2, ACCEPTOR_TO_PROPOSER)])
    p2a, pp2a = m.own(3, cb="p2a", changes=[(2, PROPOSER_TO_ACCEPTOR)])
    m.streams[2] += [
        m_prepare(ver, 0, B2),
        m_accept(ver, 0, 1, B2, [(5, B2, v(5)), (6, B2, v(6))]),
        m_learn(0, 3, [(2, B2, a2p)]), e_epoch(3),        # acceptor deleted
        m_prepare(3, 0, B3),                              # not an acceptor: not dispatched (Loop)
        m_learn(0, 4, [(3, B2, p2a)]), e_epoch(4),        # fresh acceptor, version 4
        m_accept(4, 0, 2, B0, [(5, B0, v(5, 0, 55))]),    # B0 >= promised(0): accepted
        m_prepare(4, 0, B1),
    ]
    m.streams[0] += [pa2p, pp2a, m_learn(0, 3, [(2, B2, a2p)]), e_epoch(3), m_learn(0, 4, [(3, B2, p2a)]), e_epoch(4)]
    m.streams[1] += [m_learn(0, 3, [(2, B2, a2p)]), e_epoch(3), m_learn(0, 4, [(3, B2, p2a)]), e_epoch(4)]
    t["mm_acceptor_reset"] = m.trace()

    # 6. proposer aggregation: quorum |acceptors|/2+1 of the node's epoch, accept
    #    replies matched by batch id only (:1317-1343), promise merge strict >
    m = Member(4, 4)
    m.bootstrap()
    ver4 = 3
    e_a = [(8, B0, v(8, 1, 80)), (9, B1, v(9, 1, 90))]
    e_b = [(8, B0, v(8, 2, 81)), (9, B2, v(9, 2, 92)), (10, B0, v(10))]
    s0 = m.streams[0]
    s0 += [
        m_prepare_reply(0, B2, e_a),                      # not preparing: ignored
        p_start(B2),
        m_prepare_reply(0, B1, e_b),                      # stale ballot: ignored
        m_prepare_reply(1, B2, e_a),
        m_prepare_reply(1, B2, e_b),                      # same acceptor: merges, no vote
        m_prepare_reply(3, B2, e_b),
        m_prepare_reply(2, B2, e_a),                      # 3 of 4: quorum
        m_prepare_reply(0, B2, e_b),                      # after quorum: ignored
        reject(B3),                                       # proposer-side max only
        m_p_batch(21, [(8, B2, v(8, 2, 81)), (9, B2, v(9, 2, 92))]),
        m_p_batch(22, [(10, B2, v(10))]),
        m_accept_reply(0, 21), m_accept_reply(0, 21), m_accept_reply(1, 99),
        m_accept_reply(2, 22), m_accept_reply(3, 21),
        m_accept_reply(1, 21),                            # quorum 3 of 4 for batch 21
        m_accept_reply(2, 21),                            # retired: ignored
        m_accept_reply(0, 22), m_accept_reply(3, 22),     # quorum for 22
        m_learn_reply(2, 1),
    ]
    for i in range(1, 4):
        m.streams[i] += [m_prepare_reply(0, B2, e_a), m_accept_reply(0, 5)]   # no proposer... node i has one
    t["mm_aggregate"] = m.trace()

    # 7. late joiner: node 3 learns every membership Value in one LEARN and steps
    #    through all epochs in a row; before that it is no acceptor (drops PREPARE)
    m = Member(4, 4)
    m.bootstrap([0, 1, 2])
    m.streams[3] += [
        m_prepare(0, 0, B1),                              # node 3 has no Acceptor yet
        m_learn(0, 1, m.boot + [(3, B1, v(3))]), e_epoch(1), e_epoch(2), e_epoch(3),
        m_prepare(3, 0, B1),
        m_accept(3, 0, 4, B1, [(4, B1, v(4)), (5, B1, mvalue(0, 0, noop=True))]),
        m_learn(0, 2, [(5, B1, mvalue(0, 0, noop=True)), (4, B1, v(4))]),   # noop is not executed
    ]
    t["mm_catchup"] = m.trace()

    # 8. learn reliability (f4): a promise quorum re-learns what was learned (:1299-1307), an
    #    accept quorum learns its batch (:1334-1337); Applied at |acceptors|/2+1 replies and
    #    retirement at |learners_| (:1345-1381); AddLearner / DelLearner alone change learners_
    #    only (LearnersChanged, :1472-1502: drop every open learn, re-learn all)
    m = Member(4, 2, extra_epochs=[(1, mask(0, 1), mask(0, 1), mask(0, 1, 3)), (1, mask(0, 1), mask(0, 1), mask(0, 1))])
    m.bootstrap([0])
    o1, o2 = m.own(1), m.own(2)
    ents = [(1, B1, o1[0]), (2, B1, o2[0])]
    al3, pal3 = m.own(3, cb="al3", changes=[(3, ADD_LEARNER)])
    dl3, pdl3 = m.own(4, cb="dl3", changes=[(3, DEL_LEARNER)])
    m.streams[0] += [
        # (learn 1: AddAcceptor(1)'s ADD_LEARNER while the bootstrap LEARN applies)
        p_start(B1), o1[1], o2[1],                                    # queued while preparing
        m_prepare_reply(0, B1), m_prepare_reply(1, B1),               # quorum: learn 2 (learned boot value)
        m_p_batch(5, ents), m_accept_reply(0, 5), m_accept_reply(1, 5),   # chosen: learn 3
        m_learn_reply(0, 2), m_learn_reply(1, 2),                     # learn 2 applied, retired (2 learners)
        m_learn(0, 2, ents), m_learn_reply(0, 3),
        pal3, pdl3,                                                   # proposed at once: 3, 4
        m_learn(0, 3, [(3, B1, al3)]), e_epoch(2),                    # learners {0,1,3}: drops 3, learn 4
        m_learn_reply(0, 4), m_learn_reply(1, 4), m_learn_reply(2, 4), m_learn_reply(3, 4),   # 2: not a learner
        m_learn(0, 4, [(4, B1, dl3)]), e_epoch(3),                    # learners {0,1}: learn 5
        m_learn_reply(1, 5), m_learn_reply(3, 1), m_learn_reply(0, 5),
    ]
    t["mm_learners"] = m.trace()

    # 9. Propose (f2; member/paxos.cpp:1122-1156, OnPrepareReply :1183-1297, OnLearn :1383-1470):
    #    values proposed at once and queued while preparing; a quorum adopts another proposer's
    #    value at an instance node 0 had proposed, so its LEARN is a conflict: the lost value is
    #    proposed again at once (not preparing), and a second conflict while preparing is queued
    #    for the next quorum's batch
    m = Member(3, 3)
    m.bootstrap()
    a, b, c, d = m.own(2), m.own(3), m.own(4), m.own(5)
    x3 = mvalue(1, 7, "x3", "cb")                         # node 1's value at instance 3
    x5 = mvalue(2, 9, "x5", "cb")                         # node 2's value at instance 5
    s0 = m.streams[0]
    s0 += [
        a[1], b[1],                                       # at once: instances 2, 3
        m_p_batch(1, [(2, B0, a[0]), (3, B0, b[0])]),
        p_start(B1), c[1],                                # queued while preparing
        m_prepare_reply(1, B1, [(2, B0, a[0]), (3, B2, x3)]),
        m_prepare_reply(2, B1, [(3, B1, b[0])]),          # quorum: adopt 2 = a, 3 = x3 (B2 > B1); c at 4
        m_p_batch(2, [(2, B1, a[0]), (3, B1, x3), (4, B1, c[0])]),
        m_learn(1, 3, [(3, B2, x3)]),                     # conflict: b proposed again at once (5)
        d[1],                                             # at once: 6
        p_start(B3),
        m_learn(2, 4, [(5, B2, x5)]),                     # conflict while preparing: b queued
        m_prepare_reply(0, B3, [(4, B1, c[0]), (6, B1, d[0])]),
        m_prepare_reply(1, B3),                           # quorum: adopt 4 = c, 6 = d; 2 (unlearned,
                                                          # no reply holds it): noop; b queued -> 7
    ]
    t["mm_propose"] = m.trace()
    return t


def member_violation_traces():
    """ASSERT cases (the reference crashes; oracle and engine record them)."""
    t = {}
    ver = 2
    m = Member(3, 3)
    m.bootstrap()
    m.streams[0] += [
        m_learn(1, 5, [(6, B1, v(6))]),
        m_learn(1, 6, [(6, B2, v(6, 1, 66))]),           # proposer exists: learned value differs
        m_accept(ver, 0, 3, B1, [(6, B1, v(6, 2, 67))]),  # accept of a learned instance, other value
        p_start(B1),
        m_prepare_reply(5, B1),                           # not an acceptor of the epoch
    ]
    m.streams[1] += [m_learn(1, 5, [(6, B1, v(6))])]
    t["mm_violations"] = m.trace()
    return t
