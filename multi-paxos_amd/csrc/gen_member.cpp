// gen_member.cpp — C5 member-semantics traces, host.
//
// One leader (node 0, the demo's `first`, member/main.cpp:187-195) drives the
// demo's membership schedule (member/main.cpp:119-141): AddAcceptor(1..U-1),
// then DelAcceptor(1..U-1), one membership Value per change, so the acceptor
// set grows 1,2,..,U and shrinks back (2U-1 epochs, version = epoch).  The
// instance space is split about evenly over the epochs.
//
// The leader's Proposer is the reference's (member/paxos.cpp:1074-1470) held in
// a model that the trace's P_PROPOSE / P_START records drive, so every Value it
// sends is one the reference Proposer would have sent:
//   * client values and membership changes reach it as P_PROPOSE records
//     (Node::Propose -> Proposer::Propose, :1122-1156): value_id_ + 1; while not
//     preparing the next unproposed instance, else queued;
//   * every epoch change (AcceptorsChanged, :1504-1549) starts a new round:
//     P_START, PREPARE over the unlearned ids, the promise quorum's merged map
//     (:1158-1182), and the phase-2 batch OnPrepareReply builds (:1183-1297):
//     adopted values, noop gap fill, its initial proposals, its queued values;
//   * Proposer::OnLearn (:1383-1470): a learned id leaves the unlearned /
//     unproposed sets; an own value that lost its instance is proposed again.
// Every node's acceptor / learner is simulated with the reference's rules
// (:1029-1060,1700-1793) while its receive stream is written, so each reply a
// proposer receives carries what that node would send:
//   * batches of U[1,B] instances (one P_BATCH per batch), ACCEPT to the
//     acceptors, LEARN to the learners once a quorum replied (:1317-1343),
//     LEARN_REPLY back;
//   * batches the leader sent after a membership Value and before applying it
//     are in flight across the change: acceptors that switched version drop
//     them (:1744), the others accept them under the old ballot, and the new
//     round adopts or re-proposes them (insert keeps the first pid, :1765);
//   * a new learner receives one catch-up LEARN with every learned Value
//     (LearnersChanged, :1265-1289) and walks through all epochs at once;
//   * drop_rate: a PREPARE/ACCEPT/LEARN delivery is lost and re-sent at the
//     next retry point; dup_rate: a delivery is duplicated, the copy arriving up
//     to max_delay deliveries later (stale versions get dropped).
// Contention (proposers > 1, the c5_contended workload): in epochs 2.. a rival
// proposer (nodes 1 .. proposers-1 in turn, each once it is an acceptor and a
// proposer) runs a round of its own after the leader's last batch of the epoch
// was learned: P_START with a ballot above the leader's, PREPARE over ITS
// unlearned ids — a Proposer created by a membership step has missed every
// earlier learn, so that is most of the history (:1074-1082,1559) — the
// acceptors' promise replies with their accepted and learned values, its
// quorum's batch (the adopted values), ACCEPT / LEARN of it; the leader's next
// ACCEPTs meet the higher promise, are rejected, and it re-prepares above it.
// Epoch changes are marked with E_EPOCH records right after the LEARN whose
// apply performed them (include/mpx.h).
#include <algorithm>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "gen.hpp"
#include "mpx.h"

namespace mpx {

namespace {

template <typename T> inline void app(std::string &s, T v) { s.append((const char *)&v, sizeof v); }

enum { ADD_LEARNER = 0, LEARNER_TO_PROPOSER = 1, PROPOSER_TO_ACCEPTOR = 2,
       DEL_LEARNER = 3, PROPOSER_TO_LEARNER = 4, ACCEPTOR_TO_PROPOSER = 5 };

struct Rng {
    uint64_t s;
    uint64_t next()
    {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};

// AvailableInstanceIDs (member/paxos.cpp, as multi/paxos.cpp:253-318): disjoint [a, b)
struct IdSet {
    std::map<uint64_t, uint64_t> r;
    IdSet() { r[0] = ~0ull; }
    bool contains(uint64_t id) const
    {
        auto it = r.upper_bound(id);
        if (it == r.begin()) return false;
        --it;
        return id < it->second;
    }
    void remove(uint64_t id)
    {
        auto it = r.upper_bound(id);
        if (it == r.begin()) return;
        --it;
        if (id >= it->second) return;
        const uint64_t a = it->first, b = it->second;
        r.erase(it);
        if (a != id) r[a] = id;
        if (id + 1 != b) r[id + 1] = b;
    }
    uint64_t next() { const uint64_t a = r.begin()->first; remove(a); return a; }
};

constexpr uint64_t VID_MASK = (1ull << 47) - 1;
inline uint64_t handle(uint32_t p, bool noop, uint64_t vid) { return ((uint64_t)p << 48) | ((uint64_t)noop << 47) | vid; }

// one member Proposer (member/paxos.cpp:1074-1470), the bookkeeping its decisions read
struct Prop {
    uint32_t self = 0;
    IdSet unlearned, unproposed;
    std::map<uint64_t, uint64_t> initial;          // initial_proposals_: instance -> value id
    std::set<uint64_t> newly;                      // newly_proposed_values_
    uint64_t vid = 0;                              // value_id_
    bool preparing = false;
    uint64_t ballot = 0, count = 0;                // proposal_id_, proposal_count_
    // Propose (:1122-1156): the instance it takes now, or ~0 (queued)
    uint64_t propose()
    {
        ++vid;
        if (preparing) { newly.insert(vid); return ~0ull; }
        const uint64_t iid = unproposed.next();
        initial[iid] = vid;
        return iid;
    }
    // OnLearn (:1383-1470) before the learner inserts; returns the values proposed again at once
    std::vector<std::pair<uint64_t, uint64_t>> on_learn(const std::vector<std::pair<uint64_t, uint64_t>> &vals,
                                                        const std::vector<uint64_t> &learned_pid)
    {
        std::set<uint64_t> conflicts;
        for (auto &x : vals) {
            const uint64_t iid = x.first, h = x.second;
            if (!learned_pid[iid]) unlearned.remove(iid);
            unproposed.remove(iid);
            auto it = initial.find(iid);
            if (it != initial.end()) {
                if ((uint32_t)(h >> 48) != self || (h & VID_MASK) != it->second) conflicts.insert(it->second);
                initial.erase(it);
            }
        }
        std::vector<std::pair<uint64_t, uint64_t>> again;
        if (!preparing)
            for (uint64_t v : conflicts) { const uint64_t iid = unproposed.next(); initial[iid] = v; again.push_back({iid, v}); }
        else
            newly.insert(conflicts.begin(), conflicts.end());
        return again;
    }
    // OnPrepareReply's batch at the quorum (:1183-1297): {iid, handle}, iid ascending; the
    // adopted values come from the merged map (iid -> handle)
    std::vector<std::pair<uint64_t, uint64_t>> decide(const std::map<uint64_t, std::pair<uint64_t, uint64_t>> &merged)
    {
        IdSet un = unlearned;
        std::vector<std::pair<uint64_t, uint64_t>> b;
        for (auto &x : merged)
            if (un.contains(x.first)) { un.remove(x.first); b.push_back({x.first, x.second.second}); }
        while (un.r.size() > 1) {
            const auto first = *un.r.begin();
            un.r.erase(un.r.begin());
            for (uint64_t id = first.first; id != first.second; ++id) b.push_back({id, handle(self, true, ++vid)});
        }
        for (auto &x : initial)
            if (un.contains(x.first)) { un.remove(x.first); b.push_back({x.first, handle(self, false, x.second)}); }
        for (uint64_t v : newly) { const uint64_t iid = un.next(); initial[iid] = v; b.push_back({iid, handle(self, false, v)}); }
        newly.clear();
        unproposed = un;
        preparing = false;
        std::sort(b.begin(), b.end());
        return b;
    }
};

enum Kind { D_PREPARE, D_ACCEPT, D_LEARN };

struct Delivery {
    Kind kind;
    uint32_t version, from;       // from: the proposer (replies go to its stream)
    uint64_t ballot, id;          // ballot; batch or learn id
    std::vector<std::pair<uint64_t, uint64_t>> ranges;   // PREPARE
    std::vector<uint64_t> iids, pids, hs;                 // ACCEPT / LEARN entries
    // entry bytes, encoded once and shared by every copy of the delivery
    mutable std::shared_ptr<const std::string> body;
};

struct Pending { uint64_t due; Delivery d; };

struct SimNode {
    uint32_t epoch = 0;
    bool acc = false;
    uint64_t promised = 0, maxs = 0;
    std::map<uint64_t, std::pair<uint64_t, uint64_t>> accepted;   // iid -> {pid, handle}
    std::vector<uint64_t> learned_pid;                            // per instance (0: not learned)
    uint64_t next_apply = 0, max_learned = 0;
    uint64_t appended = 0;
    std::string bytes;                        // receive stream: concatenated records
    std::vector<uint64_t> offs{0};
    std::deque<Pending> later;
    // proposer side
    std::unique_ptr<Prop> prop;
    uint64_t learners = 0;                    // learners_ (bit mask)
    // the current round's promise replies: merged map (iid -> {pid, handle}), repliers
    std::map<uint64_t, std::pair<uint64_t, uint64_t>> merged;
    uint64_t promise_mask = 0;
    bool quorum = false;
};

struct Gen {
    uint32_t U;
    uint64_t M, cap = 0;                  // instances; arrays sized cap (M + margin)
    bool over = false;                    // an instance id reached M
    uint32_t E;                               // epochs
    std::vector<mpx_epoch> ep;
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> changes;   // per change c >= 1
    std::vector<uint64_t> chosen_h;           // per instance: the learned Value (unique: safety)
    std::vector<SimNode> nd;
    Rng rng;
    uint32_t drop, dup, max_delay;
    uint64_t learn_id = 0;

    // Value_m bytes (member/paxos.cpp:321-408): proposer, value id, noop; a client value's
    // payload and cb are the decimal of its value id (Propose(ToStr(i), ToStr(i)),
    // member/main.cpp:208); a membership change c: its change list, cb "member c"
    std::unordered_map<uint64_t, uint32_t> change_of;   // membership handle -> change
    std::string value(uint64_t h) const
    {
        std::string s;
        const uint32_t p = (uint32_t)(h >> 48);
        const bool noop = (h >> 47) & 1;
        app<uint32_t>(s, p); app<uint64_t>(s, h & VID_MASK); app<uint8_t>(s, noop);
        if (noop) return s;
        s += value_body(h);
        return s;
    }
    std::string value_body(uint64_t h) const
    {
        std::string s;
        auto it = change_of.find(h);
        if (it != change_of.end()) {
            app<uint8_t>(s, 1);
            app<uint32_t>(s, (uint32_t)changes[it->second].size());
            for (auto &c : changes[it->second]) { app<uint32_t>(s, c.first); app<uint32_t>(s, c.second); }
            const std::string cb = "member " + std::to_string(it->second);
            app<uint32_t>(s, (uint32_t)cb.size()); s += cb;
        } else {
            const std::string p = std::to_string(h & VID_MASK);
            app<uint8_t>(s, 0); app<uint32_t>(s, (uint32_t)p.size()); s += p;
            app<uint32_t>(s, (uint32_t)p.size()); s += p;
        }
        return s;
    }
    std::string entries(const std::vector<uint64_t> &iids, const std::vector<uint64_t> &pids,
                        const std::vector<uint64_t> &hs) const
    {
        std::string s;
        s.reserve(iids.size() * 48);
        for (size_t i = 0; i < iids.size(); ++i) { app<uint64_t>(s, iids[i]); app<uint64_t>(s, pids[i]); s += value(hs[i]); }
        return s;
    }
    const std::string &body_of(const Delivery &d) const
    {
        if (!d.body) d.body = std::make_shared<const std::string>(entries(d.iids, d.pids, d.hs));
        return *d.body;
    }

    void append(uint32_t n, const std::string &m)
    {
        SimNode &x = nd[n];
        x.bytes += m;
        x.offs.push_back(x.bytes.size());
        x.appended++;
    }

    // ---- acceptor / learner simulation while writing node n's stream --------
    // returns 1 granted, 0 otherwise
    int process(uint32_t n, const Delivery &d)
    {
        SimNode &x = nd[n];
        std::string m;
        if (d.kind == D_PREPARE) {
            std::string rg;
            for (auto &r : d.ranges) { app<uint64_t>(rg, r.first); app<uint64_t>(rg, r.second); }
            app<uint32_t>(m, MPX_MSG_PREPARE); app<uint32_t>(m, d.version); app<uint32_t>(m, d.from);
            app<uint64_t>(m, d.ballot); app<uint32_t>(m, (uint32_t)rg.size()); m += rg;
            append(n, m);
            if (!x.acc || d.version != ep[x.epoch].version) return 0;
            x.maxs = std::max(x.maxs, d.ballot);
            if (d.ballot > x.promised) {
                x.promised = d.ballot;
                // FilterAcceptedValues: accepted and learned entries in the ranges (:1806-1818)
                std::map<uint64_t, std::pair<uint64_t, uint64_t>> all;
                for (auto &r : d.ranges) {
                    for (auto it = x.accepted.lower_bound(r.first); it != x.accepted.end() && it->first < r.second; ++it)
                        all[it->first] = it->second;
                    for (uint64_t i = r.first; i <= x.max_learned && i < M && i < r.second; ++i)
                        if (x.learned_pid[i]) all[i] = {x.learned_pid[i], chosen_h[i]};
                }
                std::vector<uint64_t> ii, pp, hh;
                for (auto &e : all) { ii.push_back(e.first); pp.push_back(e.second.first); hh.push_back(e.second.second); }
                std::string body = entries(ii, pp, hh), r;
                app<uint32_t>(r, MPX_MSG_PREPARE_REPLY); app<uint32_t>(r, n); app<uint64_t>(r, d.ballot);
                app<uint32_t>(r, (uint32_t)body.size()); r += body;
                to_proposer(d.from, r, n, d.ballot, &all);
                return 1;
            }
            if (d.ballot < x.promised) { std::string r; app<uint32_t>(r, MPX_MSG_REJECT); app<uint64_t>(r, x.maxs); to_proposer(d.from, r); }
            return 0;
        }
        if (d.kind == D_ACCEPT) {
            const std::string &body = body_of(d);
            app<uint32_t>(m, MPX_MSG_ACCEPT); app<uint32_t>(m, d.version); app<uint32_t>(m, d.from);
            app<uint64_t>(m, d.id); app<uint64_t>(m, d.ballot); app<uint32_t>(m, (uint32_t)body.size()); m += body;
            append(n, m);
            if (!x.acc || d.version != ep[x.epoch].version) return 0;
            x.maxs = std::max(x.maxs, d.ballot);
            if (d.ballot >= x.promised) {
                for (size_t i = 0; i < d.iids.size(); ++i)
                    if (!x.learned_pid[d.iids[i]]) x.accepted.insert({d.iids[i], {d.pids[i], d.hs[i]}});
                std::string r;
                app<uint32_t>(r, MPX_MSG_ACCEPT_REPLY); app<uint32_t>(r, n); app<uint64_t>(r, d.id);
                to_proposer(d.from, r);
                return 1;
            }
            std::string r; app<uint32_t>(r, MPX_MSG_REJECT); app<uint64_t>(r, x.maxs); to_proposer(d.from, r);
            return 0;
        }
        // LEARN: Learner::OnLearn (:1029-1060) — the Proposer first (:1034-1038), then insert
        const std::string &body = body_of(d);
        app<uint32_t>(m, MPX_MSG_COMMIT); app<uint32_t>(m, d.from); app<uint64_t>(m, d.id);
        app<uint32_t>(m, (uint32_t)body.size()); m += body;
        append(n, m);
        if (x.prop) {
            std::vector<std::pair<uint64_t, uint64_t>> vals;
            for (size_t i = 0; i < d.iids.size(); ++i) vals.push_back({d.iids[i], d.hs[i]});
            std::sort(vals.begin(), vals.end());
            auto again = x.prop->on_learn(vals, x.learned_pid);
            for (auto &a : again) reproposed.push_back({n, a});
        }
        for (size_t i = 0; i < d.iids.size(); ++i) {
            const uint64_t iid = d.iids[i];
            x.accepted.erase(iid);
            if (!x.learned_pid[iid]) {
                x.learned_pid[iid] = d.pids[i];
                x.max_learned = std::max(x.max_learned, iid);
                chosen_h[iid] = d.hs[i];
            }
        }
        std::vector<uint32_t> steps;
        while (x.next_apply < M && x.learned_pid[x.next_apply]) {
            auto it = change_of.find(chosen_h[x.next_apply++]);
            if (it != change_of.end()) steps.push_back(it->second);
        }
        for (uint32_t c : steps) {
            std::string e; app<uint32_t>(e, MPX_MSG_E_EPOCH); app<uint32_t>(e, c);
            append(n, e);
            const mpx_epoch &o = ep[x.epoch], &w = ep[c];
            const bool acc = (w.acceptor_mask >> n) & 1, was_p = (o.proposer_mask >> n) & 1, now_p = (w.proposer_mask >> n) & 1;
            if (acc != x.acc) { x.accepted.clear(); x.promised = x.maxs = 0; x.acc = acc; }
            if (now_p && !was_p) { x.prop.reset(new Prop); x.prop->self = n; x.prop->preparing = true; }   // ctor: StartPrepare
            if (!now_p && was_p) x.prop.reset();
            // AcceptorsChanged (RestartPrepare) / the new Proposer: the engine model idles it at the
            // marker until its next P_START (include/mpx.h); its accepting_values_ go
            if (x.prop && (!was_p || o.acceptor_mask != w.acceptor_mask)) {
                x.prop->preparing = false;
                x.merged.clear(); x.promise_mask = 0; x.quorum = true;
            }
            x.learners = w.learner_mask;
            x.epoch = c;
        }
        std::string r; app<uint32_t>(r, MPX_MSG_COMMIT_REPLY); app<uint32_t>(r, n); app<uint64_t>(r, d.id);
        to_proposer(d.from, r);
        return 1;
    }
    // values proposed again at once by a Proposer::OnLearn (node, {iid, value id})
    std::vector<std::pair<uint32_t, std::pair<uint64_t, uint64_t>>> reproposed;

    // a reply to proposer p's stream; a PREPARE_REPLY is merged into its round
    // (UpdateByPreAcceptedValues, :1158-1182,1614-1629: strict >, first arrival on ties)
    void to_proposer(uint32_t p, const std::string &r, uint32_t from = 0, uint64_t ballot = 0,
                     const std::map<uint64_t, std::pair<uint64_t, uint64_t>> *vals = nullptr)
    {
        append(p, r);
        if (!vals) return;
        SimNode &x = nd[p];
        if (!x.prop || !x.prop->preparing || ballot != x.prop->ballot || x.quorum) return;
        for (auto &e : *vals) {
            auto it = x.merged.find(e.first);
            if (it == x.merged.end() || e.second.first > it->second.first) x.merged[e.first] = e.second;
        }
        x.promise_mask |= 1ull << from;
        const uint32_t Q = (uint32_t)__builtin_popcountll(ep[x.epoch].acceptor_mask) / 2 + 1;
        if ((uint32_t)__builtin_popcountll(x.promise_mask) >= Q) x.quorum = true;
    }

    // deliver due delayed copies, then this one (unless lost)
    void flush_due(uint32_t n)
    {
        SimNode &x = nd[n];
        while (!x.later.empty() && x.later.front().due <= x.appended) {
            Delivery d = x.later.front().d;
            x.later.pop_front();
            process(n, d);
        }
    }
    void flush_all(uint32_t n)
    {
        SimNode &x = nd[n];
        while (!x.later.empty()) { Delivery d = x.later.front().d; x.later.pop_front(); process(n, d); }
    }
    // -1 lost (re-sent at the retry point), else granted
    int send(uint32_t n, const Delivery &d, bool may_lose)
    {
        flush_due(n);
        if (may_lose && drop && rng.below(10000) < drop) return -1;
        int g = process(n, d);
        if (dup && rng.below(10000) < dup) {
            Pending p{nd[n].appended + 1 + rng.below(max_delay ? max_delay : 1), d};
            auto &q = nd[n].later;
            q.insert(std::upper_bound(q.begin(), q.end(), p, [](const Pending &a, const Pending &b) { return a.due < b.due; }), p);
        }
        return g;
    }
};

// one proposer's moves, written into the streams
struct Driver {
    Gen &g;
    uint32_t B;
    std::vector<uint64_t> batch_id;           // per proposer: its batch ids (P_BATCH / ACCEPT accept id)

    std::vector<uint32_t> acceptors(uint32_t e) const
    {
        std::vector<uint32_t> a;
        for (uint32_t n = 0; n < g.U; ++n) if ((g.ep[e].acceptor_mask >> n) & 1) a.push_back(n);
        return a;
    }
    uint32_t quorum(uint32_t e) const { return (uint32_t)__builtin_popcountll(g.ep[e].acceptor_mask) / 2 + 1; }
    void shuffle(std::vector<uint32_t> &v)
    {
        for (size_t i = v.size(); i > 1; --i) std::swap(v[i - 1], v[g.rng.below(i)]);
    }
    // Node::Propose -> Proposer::Propose of a client value or membership change c (0: client)
    void p_propose(uint32_t n, uint64_t h)
    {
        std::string s, b = g.value_body(h);
        app<uint32_t>(s, MPX_MSG_P_PROPOSE); app<uint32_t>(s, (uint32_t)b.size()); s += b;
        g.append(n, s);
    }
    // a new round of proposer n (StartPrepare, :1551-1571): P_START, PREPARE over its unlearned ids
    // to the acceptors (lost ones re-sent until a quorum granted, PrepareRetryTimeout); false when
    // no quorum can grant (a higher promise)
    bool prepare(uint32_t n, uint64_t ballot, bool lossy)
    {
        SimNode &x = g.nd[n];
        Prop &P = *x.prop;
        P.ballot = ballot;
        P.preparing = true;
        x.merged.clear(); x.promise_mask = 0; x.quorum = false;
        { std::string s; app<uint32_t>(s, MPX_MSG_P_START); app<uint64_t>(s, ballot); g.append(n, s); }
        const uint32_t e = x.epoch;
        Delivery pd{D_PREPARE, g.ep[e].version, n, ballot, 0, {}, {}, {}, {}, nullptr};
        for (auto &r : P.unlearned.r) pd.ranges.push_back(r);
        std::vector<uint32_t> order = acceptors(e), missing;
        shuffle(order);
        for (uint32_t a : order) if (g.send(a, pd, lossy && a != n) <= 0) missing.push_back(a);
        for (size_t k = 0; !x.quorum && k < missing.size(); ++k) {
            g.flush_all(missing[k]);
            g.process(missing[k], pd);
        }
        return x.quorum;
    }
    // one batch of proposer n: P_BATCH, ACCEPT to the acceptors (AcceptRetryTimeout re-sends the
    // lost ones), LEARN to its learners once chosen; `fly_d`: the batch is left in flight (its
    // ACCEPTs delivered by the caller), returned there; `defer`: the LEARN is left to the caller
    // (returned there).  false: rejected.
    bool batch(uint32_t n, const std::vector<std::pair<uint64_t, uint64_t>> &ents, bool lossy, Delivery *fly_d = nullptr,
               Delivery *defer = nullptr)
    {
        SimNode &x = g.nd[n];
        const uint32_t e = x.epoch;
        for (auto &v : ents)
            if (v.first >= g.M) { g.over = true; if (v.first >= g.cap) return true; }   // (reported at the end)
        const uint64_t bid = ++batch_id[n];
        std::vector<uint64_t> ii, pp, hh;
        for (auto &v : ents) { ii.push_back(v.first); pp.push_back(x.prop->ballot); hh.push_back(v.second); }
        {
            std::string s, body = g.entries(ii, pp, hh);
            app<uint32_t>(s, MPX_MSG_P_BATCH); app<uint64_t>(s, bid); app<uint32_t>(s, (uint32_t)body.size());
            s += body; g.append(n, s);
        }
        Delivery ad{D_ACCEPT, g.ep[e].version, n, x.prop->ballot, bid, {}, ii, pp, hh, nullptr};
        if (fly_d) { *fly_d = ad; return true; }
        std::vector<uint32_t> order = acceptors(e), missing;
        shuffle(order);
        uint32_t votes = 0;
        for (uint32_t a : order) { const int r = g.send(a, ad, lossy && a != n); if (r > 0) ++votes; else if (r < 0) missing.push_back(a); }
        for (size_t k = 0; votes < quorum(e) && k < missing.size(); ++k) {
            g.flush_all(missing[k]);
            if (g.process(missing[k], ad) > 0) ++votes;
        }
        if (votes < quorum(e)) return false;
        if (defer) { *defer = Delivery{D_LEARN, 0, n, 0, 0, {}, ii, pp, hh, nullptr}; return true; }
        learn(n, ii, pp, hh, lossy);
        return true;
    }
    // OnAcceptReply at the quorum (:1317-1343): LEARN to the node's learners_, itself first
    // (others = false: only itself; the caller sends the rest with learn_others)
    Delivery learn(uint32_t n, const std::vector<uint64_t> &ii, const std::vector<uint64_t> &pp,
                   const std::vector<uint64_t> &hh, bool lossy, bool others = true)
    {
        Delivery ld{D_LEARN, 0, n, 0, ++g.learn_id, {}, ii, pp, hh, nullptr};
        const uint64_t learners = g.nd[n].learners;        // (before the LEARN changes them)
        if ((learners >> n) & 1) g.send(n, ld, false);
        if (others) learn_others(n, ld, learners, lossy);
        return ld;
    }
    void learn_others(uint32_t n, const Delivery &ld, uint64_t learners, bool lossy)
    {
        for (uint32_t m = 0; m < g.U; ++m) {
            if (m == n || !((learners >> m) & 1)) continue;
            if (g.send(m, ld, lossy) < 0) {                               // LearnRetryTimeout
                Pending pe{g.nd[m].appended + 1 + g.rng.below(g.max_delay), ld};
                auto &q = g.nd[m].later;
                q.insert(std::upper_bound(q.begin(), q.end(), pe, [](const Pending &a, const Pending &b) { return a.due < b.due; }), pe);
            }
        }
    }
    // the values a Proposer::OnLearn proposed again at once: one batch each
    bool flush_reproposed(bool lossy)
    {
        while (!g.reproposed.empty()) {
            auto r = g.reproposed.front();
            g.reproposed.erase(g.reproposed.begin());
            SimNode &x = g.nd[r.first];
            if (!x.prop) continue;
            if (!batch(r.first, {{r.second.first, handle(r.first, false, r.second.second)}}, lossy)) return false;
        }
        return true;
    }
    // the phase-2 batch of a round that reached its quorum, in batches of U[1, B]
    bool phase2(uint32_t n, bool lossy)
    {
        SimNode &x = g.nd[n];
        auto b = x.prop->decide(x.merged);
        for (size_t pos = 0; pos < b.size();) {
            const size_t take = std::min<size_t>(b.size() - pos, 1 + g.rng.below(B));
            std::vector<std::pair<uint64_t, uint64_t>> part(b.begin() + pos, b.begin() + pos + take);
            if (!batch(n, part, lossy)) return false;
            pos += take;
        }
        return true;
    }
};

}  // namespace

int gen_member(const mpx_gen_params &p, std::string &out)
{
    const uint32_t U = p.num_nodes;
    if (U < 2 || U > 64) return MPX_E_INVAL;
    Gen g;
    g.U = U;
    g.M = p.num_instances;
    g.E = 2 * (U - 1) + 1;
    const uint32_t B = p.batch ? p.batch : 64;
    const uint32_t rivals = p.proposers > 1 ? std::min<uint32_t>(p.proposers - 1, U - 1) : 0;
    // room above the last epoch for the values proposed again after a rival round took their
    // instances (or lost across a change); a trace that still runs past M is refused
    const uint64_t slack = rivals ? 8ull * B + 64 : 2ull * B + 8;
    if (g.M < 4ull * g.E + slack || g.M >= (1ull << 40)) return MPX_E_INVAL;
    g.rng.s = p.seed * 0x2545F4914F6CDD1Dull + 7;
    g.cap = g.M + 64ull * B + 4096;
    g.drop = p.drop_rate; g.dup = p.dup_rate; g.max_delay = p.max_delay ? p.max_delay : 64;

    // epochs and membership changes (member/paxos.cpp:646-733 change lists)
    g.ep.resize(g.E);
    g.changes.resize(g.E);
    uint64_t set = 1;
    g.ep[0] = mpx_epoch{0, 0, 1, 1, 1};
    for (uint32_t c = 1; c < g.E; ++c) {
        if (c < U) {
            g.changes[c] = {{c, ADD_LEARNER}, {c, LEARNER_TO_PROPOSER}, {c, PROPOSER_TO_ACCEPTOR}};
            set |= 1ull << c;
        } else {
            const uint32_t j = c - (U - 1);
            g.changes[c] = {{j, ACCEPTOR_TO_PROPOSER}, {j, PROPOSER_TO_LEARNER}, {j, DEL_LEARNER}};
            set &= ~(1ull << j);
        }
        g.ep[c] = mpx_epoch{c, 0, set, set, set};   // (the change lists move all three roles at once)
    }
    const uint64_t Meff = g.M - slack;
    std::vector<uint64_t> target(g.E + 1);
    for (uint32_t e = 0; e <= g.E; ++e) target[e] = Meff * e / g.E;

    g.chosen_h.assign(g.cap, 0);
    g.nd.resize(U);
    for (uint32_t n = 0; n < U; ++n) g.nd[n].learned_pid.assign(g.cap, 0);
    // address space for each node's stream up front, somewhat above its mean size (C5: 82 B per
    // instance, contended 152 B; pages are only touched as they are written): a stream that grew by
    // doubling copied itself and held both copies at once — 2^25 contended traces (41 GB) peaked
    // past 60 GB of resident memory that way
    // a first guess at each node's stream (it grows past it as needed), capped at 8 GB per node: an
    // up-front reservation of M x 224 B is hundreds of GB at large M
    for (uint32_t n = 0; n < U; ++n)
        g.nd[n].bytes.reserve((size_t)std::min<uint64_t>(std::min<uint64_t>(g.M, 1ull << 30) * (p.proposers > 1 ? 224 : 128),
                                                         8ull << 30));
    SimNode &L = g.nd[0];
    L.acc = true;
    L.learners = 1;
    L.prop.reset(new Prop);                   // node 0's Proposer (Loop :738-747), idle until P_START
    Driver d{g, B, std::vector<uint64_t>(U, 0)};

    uint64_t top = 0;                         // the highest ballot count any proposer used
    auto new_ballot = [&](uint32_t n) { Prop &P = *g.nd[n].prop; P.count = std::max(P.count, top) + 1; top = P.count; return (P.count << 16) | n; };
    auto lead_round = [&]() -> bool {         // the leader's round, to its phase-2 batch
        for (int tries = 0; tries < 8; ++tries) {
            if (!d.prepare(0, new_ballot(0), true)) continue;
            if (d.phase2(0, true) && d.flush_reproposed(true)) return true;
        }
        return false;
    };
    uint32_t rival_k = 0;
    for (uint32_t e = 0; e < g.E; ++e) {
        if (!lead_round()) return MPX_E_INVAL;
        const uint64_t end = e + 1 < g.E ? target[e + 1] - 1 : g.M;     // the membership Value's instance
        const uint64_t mid = (target[e] + end) / 2;
        bool contended = false, changed = false;
        while (!changed) {
            if (rivals && e >= 2 && !contended && L.prop->unproposed.r.begin()->first >= mid) {
                // a rival round (see the head of the file): every delivery settled first
                contended = true;
                const uint32_t c = 1 + (rival_k++ % rivals);
                SimNode &R = g.nd[c];
                if (R.prop && R.acc) {
                    for (uint32_t n = 0; n < U; ++n) g.flush_all(n);   // (may apply a change to c)
                    if (R.prop && R.acc && (!d.prepare(c, new_ballot(c), false) || !d.phase2(c, false)))
                        return MPX_E_INVAL;
                }
            }
            // the next batch of new values: each one a P_PROPOSE at the next unproposed instance;
            // the membership Value of the next epoch closes its batch
            std::vector<std::pair<uint64_t, uint64_t>> ents;
            const size_t take = 1 + g.rng.below(B);
            bool has_mem = false;
            while (ents.size() < take) {
                const uint64_t nxt = L.prop->unproposed.r.begin()->first;
                if (nxt >= end && e + 1 < g.E) {
                    const uint64_t h = handle(0, false, L.prop->vid + 1);
                    g.change_of[h] = e + 1;
                    d.p_propose(0, h);
                    const uint64_t iid = L.prop->propose();
                    ents.push_back({iid, h});
                    has_mem = true;
                    break;
                }
                if (nxt >= end) break;                            // the last epoch is full
                const uint64_t h = handle(0, false, L.prop->vid + 1);
                d.p_propose(0, h);
                ents.push_back({L.prop->propose(), h});
            }
            if (ents.empty()) break;
            Delivery mem_learn;
            if (!d.batch(0, ents, true, nullptr, has_mem ? &mem_learn : nullptr)) {   // rejected (a rival's promise)
                if (!lead_round()) return MPX_E_INVAL;
                continue;
            }
            if (!d.flush_reproposed(true)) { if (!lead_round()) return MPX_E_INVAL; }
            if (!has_mem) continue;
            changed = true;
            // batches the leader created after the membership Value and before its own LEARN
            // applied it: in flight across the change (AcceptorsChanged clears them, :1322)
            const uint64_t lim = e + 2 < g.E ? target[e + 2] - 1 : g.M;
            std::vector<Delivery> fly;
            const size_t extra = g.rng.below(3);
            for (size_t x = 0; x < extra; ++x) {
                std::vector<std::pair<uint64_t, uint64_t>> fe;
                const size_t t2 = 1 + g.rng.below(B);
                while (fe.size() < t2 && L.prop->unproposed.r.begin()->first < lim) {
                    const uint64_t h = handle(0, false, L.prop->vid + 1);
                    d.p_propose(0, h);
                    fe.push_back({L.prop->propose(), h});
                }
                if (fe.empty()) break;
                Delivery fd;
                d.batch(0, fe, true, &fd);
                fly.push_back(fd);
            }
            // chosen: LEARN to the learners, the leader first (it applies the change there); then
            // the in-flight ACCEPTs — an acceptor gets them before its own LEARN of the change,
            // accepted under the old ballot, or after it, dropped by version
            const uint64_t learners = L.learners;
            const Delivery ld = d.learn(0, mem_learn.iids, mem_learn.pids, mem_learn.hs, true, false);
            const uint32_t c = e + 1;
            for (const Delivery &fd : fly)
                for (uint32_t a : d.acceptors(e)) {
                    if (a == 0 || g.rng.below(2)) g.send(a, fd, false);
                    else g.nd[a].later.push_front(Pending{g.nd[a].appended + 1, fd});
                }
            d.learn_others(0, ld, learners, true);
            if (c < U) {
                // LearnersChanged: the new learner gets every learned Value in one LEARN
                std::vector<uint64_t> ci, cp, ch;
                for (uint64_t i = 0; i < L.next_apply; ++i) { ci.push_back(i); cp.push_back(L.learned_pid[i]); ch.push_back(g.chosen_h[i]); }
                Delivery cd{D_LEARN, 0, 0, 0, ++g.learn_id, {}, ci, cp, ch, nullptr};
                g.send(c, cd, false);
            }
            // every acceptor of the next epoch has switched before the new PREPARE
            for (uint32_t n = 0; n < U; ++n)
                if ((g.ep[c].acceptor_mask >> n) & 1) g.flush_all(n);
        }
    }
    for (uint32_t n = 0; n < U; ++n) g.flush_all(n);
    if (g.over) return MPX_E_INVAL;           // num_instances too small for this schedule

    TraceWriter w;
    w.begin(U, MPX_SEM_MEMBER, g.M, g.ep);
    uint64_t total = w.out.size();
    for (auto &x : g.nd) total += 24 + 8 * x.offs.size() + x.bytes.size();
    w.out.reserve(total);
    for (uint32_t n = 0; n < U; ++n) {
        w.node_raw(g.nd[n].bytes, g.nd[n].offs);
        std::string().swap(g.nd[n].bytes);
        std::vector<uint64_t>().swap(g.nd[n].offs);
    }
    out.swap(w.out);
    return MPX_OK;
}

}  // namespace mpx
