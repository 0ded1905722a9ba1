// gen_faulty.cpp — C3 traces: competing proposers over a lossy network.
//
// A deterministic discrete-event simulation (integer ticks, counter-based RNG)
// of Multi-Paxos with P competing proposers and N acceptors/learners.  The
// network is the demo's HijackSend model (multi/main.cpp:116-132): an original
// send is dropped with p = drop/10^4, each send first spawns a duplicate with
// p = dup/10^4 (recursively, at most 3 deep), and every copy is delayed
// U[0, max_delay) ticks, which reorders.  Proposers follow the reference's
// shape (multi/paxos.cpp): StartPrepare with a ballot (++count << 16 | node)
// above max_seen (:792-799), a delayed PREPARE over the uncommitted ranges
// (:757-790), retries then a higher ballot (:770-784), at the promise quorum
// adopt the highest pre-accepted value per instance, re-propose their own
// values, fill holes with noops and assign new values (:1058-1182), accept in
// batches with retries then AcceptRejected (:969-983,1328-1343), commit on
// the accept quorum and resend the commit until every learner replied
// (:1406-1479,1625-1641).  Acceptors and learners in the simulation follow the
// reference's semantics, so the replies each proposer receives are the ones
// the handlers produce.
//
// The output is each node's receive stream in delivery order plus the
// P_START / P_BATCH proposer markers, in the MPXT container.  The trace is
// what the engine, the CPU oracle and the reference driver all replay.
//
// Scale (C3 is 2^24 instances x 7 nodes): every step costs
// O(entries touched), never O(instances so far):
//   * a node's accepted / committed maps are dense per-instance arrays with
//     present / committed bitmaps, so a PREPARE's FilterAcceptedValues, the
//     proposer's uncommitted ranges and its noop gap fill walk bitmap words
//     over the instance window only;
//   * a message carries its entry list by reference (one shared Body per
//     batch: the P_BATCH marker, every ACCEPT copy and the COMMIT have the same
//     body bytes), and its wire bytes are appended to the receiving node's
//     stream at delivery;
//   * Values are 64-bit keys (MPX_HANDLE); a client Value's payload is the
//     decimal of its global client id, a closed form of the key.
//
// Safety guard: the reference's acceptor does not raise its promise on accept
// and lets a lower (>= promised) ballot overwrite (:1366,1387), so a delayed
// stale ACCEPT can in rare schedules let two values be chosen for one
// instance; a learner receiving both would ASSERT (:1508).  The simulator
// registers the first committed value per instance and never sends a COMMIT
// that contradicts it (counted in the trace header's reserved word).
#include <algorithm>
#include <charconv>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "gen.hpp"
#include "mpx.h"

namespace mpx {

namespace {

template <typename T> inline void app(std::string &s, T v) { s.append((const char *)&v, sizeof v); }

struct Rng {
    uint64_t s;
    uint64_t next()
    {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    uint64_t range(uint64_t lo, uint64_t hi) { return hi <= lo ? lo : lo + next() % (hi - lo); }   // [lo, hi)
};

typedef std::pair<uint64_t, uint64_t> IV;       // (iid, Value key)

// shared entry list of one message body, with its wire bytes
struct Body {
    std::vector<IV> ent;                         // ACCEPT / COMMIT / P_BATCH: (iid, key), iid ascending
    std::vector<uint64_t> pid;                   // PREPARE_REPLY: the tag of ent[i]
    std::vector<std::pair<uint64_t, uint64_t>> ranges;   // PREPARE
    std::string wire;
};
typedef std::shared_ptr<const Body> BodyP;

struct Msg {
    uint32_t type = 0, from = 0;                 // sender field of the header (proposer / acceptor / ...)
    uint64_t x = 0, y = 0;                       // type-dependent header words (ballot, accept / commit id)
    BodyP body;
};

struct Ev {
    uint64_t t, seq;
    int kind;                    // 0 deliver, 1 timer
    uint32_t dst, src;
    Msg msg;
    uint32_t tkind;              // timer kind
    uint64_t token, aux;
};
struct EvLater {
    bool operator()(const Ev &a, const Ev &b) const { return a.t != b.t ? a.t > b.t : a.seq > b.seq; }
};

enum { T_PREPARE_SEND = 1, T_PREPARE_RETRY, T_ACCEPT_RETRY, T_COMMIT_RETRY, T_PROPOSE };

struct Batch {
    BodyP body;
    uint64_t mask = 0;
    uint32_t retries = 0;
    bool live = true;
};

struct Commit {
    BodyP body;
    uint64_t ballot;
    uint64_t replied = 0;
    uint32_t retries = 0;
};

// growable bitmap over instance ids
struct Bits {
    std::vector<uint64_t> w;
    bool get(uint64_t i) const { return (i >> 6) < w.size() && ((w[i >> 6] >> (i & 63)) & 1); }
    void set(uint64_t i)
    {
        if ((i >> 6) >= w.size()) w.resize(std::max<size_t>((i >> 6) + 1, 2 * w.size()), 0);
        w[i >> 6] |= 1ull << (i & 63);
    }
    // first set (want=1) or clear (want=0) bit in [i, end), or end
    uint64_t next(uint64_t i, uint64_t end, bool want) const
    {
        while (i < end) {
            const uint64_t k = i >> 6;
            uint64_t word = k < w.size() ? w[k] : 0;
            if (!want) word = ~word;
            word &= ~0ull << (i & 63);
            if (word) {
                const uint64_t r = (k << 6) + (uint64_t)__builtin_ctzll(word);
                return r < end ? r : end;
            }
            i = (k + 1) << 6;
        }
        return end;
    }
};

struct Node {
    // acceptor / learner (reference semantics): accepted_values_ and
    // committed_values_ (multi/paxos.cpp:492-495) as dense arrays, disjoint
    uint64_t promised = 0, max_seen = 0;
    std::vector<uint8_t> kind;                   // 0 none, 1 accepted, 2 committed
    std::vector<uint64_t> bal, key;
    Bits pres, comb;                             // present (either), committed
    uint64_t hi = 0;                             // max present iid + 1
    uint64_t com_hi = 0, com_lo = 0;             // max committed + 1; every iid < com_lo committed
    // proposer
    bool proposer = false;
    uint64_t count = 0, ballot = 0, epoch = 0;
    bool preparing = false, prepare_sent = false;
    uint32_t prepare_retries = 0;
    uint64_t promises = 0;
    std::map<uint64_t, std::pair<uint64_t, uint64_t>> pre;   // iid -> (pid, key)
    std::map<uint64_t, Batch> batches;
    uint64_t next_batch = 0, next_commit = 0, next_vid = 0;
    std::map<uint64_t, Commit> commits;
    std::deque<uint64_t> pending;        // own values not assigned to an instance
    std::map<uint64_t, uint64_t> assigned;   // own values at an instance, not yet known committed
    std::shared_ptr<const Body> prep;    // the PREPARE of the current round (uncommitted ranges)
    // output: receive stream
    std::string bytes;
    std::vector<uint64_t> offs{0};

    void ensure(uint64_t iid)
    {
        if (iid < kind.size()) return;
        const size_t n = std::max<size_t>(iid + 1, kind.size() * 3 / 2 + 1024);
        kind.resize(n, 0); bal.resize(n, 0); key.resize(n, 0);
    }
    bool committed(uint64_t iid) const { return comb.get(iid); }
    void commit_at(uint64_t iid, uint64_t b, uint64_t k)
    {
        ensure(iid);
        kind[iid] = 2; bal[iid] = b; key[iid] = k;
        pres.set(iid); comb.set(iid);
        hi = std::max(hi, iid + 1);
        com_hi = std::max(com_hi, iid + 1);
        if (iid == com_lo) com_lo = comb.next(com_lo, com_hi, false);
    }
};

struct Sim {
    const mpx_gen_params &p;
    uint32_t N, P, B;
    Rng rng;
    uint64_t now = 0, seq = 0;
    std::vector<Ev> q;                                // binary heap (EvLater)
    std::vector<Node> nodes;
    std::vector<uint64_t> chosen;                     // iid -> first committed value key (0: none)
    uint64_t suppressed = 0;
    uint64_t delay_min = 100, delay_max;              // PrepareDelay ticks
    uint64_t retry_timeout;
    explicit Sim(const mpx_gen_params &pp) : p(pp) {}

    uint32_t quorum() const { return N / 2 + 1; }

    // ---- Values: key = MPX_HANDLE(proposer, noop, value_id); client value k
    // of proposer p carries the decimal of global client id (k-1)*P + p ----
    void enc(std::string &s, uint64_t k) const
    {
        const uint32_t pr = MPX_HANDLE_PROPOSER(k);
        const uint64_t id = MPX_HANDLE_VALUE_ID(k);
        const bool noop = MPX_HANDLE_NOOP(k);
        app<uint32_t>(s, pr); app<uint64_t>(s, id); app<uint8_t>(s, noop ? 1 : 0);
        if (noop) return;
        char d[24];
        const auto r = std::to_chars(d, d + sizeof d, (id - 1) * P + pr);
        app<uint8_t>(s, 0); app<uint32_t>(s, (uint32_t)(r.ptr - d));
        s.append(d, (size_t)(r.ptr - d));
    }
    BodyP entry_body(std::vector<IV> &&ent) const
    {
        auto b = std::make_shared<Body>();
        b->ent = std::move(ent);
        b->wire.reserve(b->ent.size() * 34);
        for (auto &e : b->ent) { app<uint64_t>(b->wire, e.first); enc(b->wire, e.second); }
        return b;
    }

    // the reference's packed wire bytes of a message, appended to a node's stream
    static void wire(std::string &s, const Msg &m)
    {
        app<uint32_t>(s, m.type);
        const uint32_t bl = m.body ? (uint32_t)m.body->wire.size() : 0;
        switch (m.type) {
        case MPX_MSG_PREPARE:
        case MPX_MSG_PREPARE_REPLY:
            app<uint32_t>(s, m.from); app<uint64_t>(s, m.x); app<uint32_t>(s, bl); break;
        case MPX_MSG_REJECT: app<uint64_t>(s, m.x); break;
        case MPX_MSG_ACCEPT:
        case MPX_MSG_COMMIT:
            app<uint32_t>(s, m.from); app<uint64_t>(s, m.y); app<uint64_t>(s, m.x); app<uint32_t>(s, bl); break;
        case MPX_MSG_ACCEPT_REPLY: app<uint32_t>(s, m.from); app<uint64_t>(s, m.x); app<uint64_t>(s, m.y); break;
        case MPX_MSG_COMMIT_REPLY: app<uint32_t>(s, m.from); app<uint64_t>(s, m.y); break;
        case MPX_MSG_P_START: app<uint64_t>(s, m.x); break;
        case MPX_MSG_P_BATCH: app<uint64_t>(s, m.y); app<uint32_t>(s, bl); break;
        }
        if (bl) s += m.body->wire;
    }
    static void record(Node &n, const Msg &m)
    {
        wire(n.bytes, m);
        n.offs.push_back(n.bytes.size());
    }
    static Msg mk(uint32_t type, uint32_t from, uint64_t x, uint64_t y = 0, BodyP body = BodyP())
    {
        Msg m; m.type = type; m.from = from; m.x = x; m.y = y; m.body = std::move(body);
        return m;
    }

    void push(Ev &&e) { q.push_back(std::move(e)); std::push_heap(q.begin(), q.end(), EvLater()); }
    void push_deliver(uint64_t at, uint32_t src, uint32_t dst, const Msg &m)
    {
        Ev e{at, seq++, 0, dst, src, m, 0, 0, 0};
        push(std::move(e));
    }
    void timer(uint64_t at, uint32_t node, uint32_t kind, uint64_t token, uint64_t aux = 0)
    {
        Ev e{at, seq++, 1, node, node, Msg(), kind, token, aux};
        push(std::move(e));
    }
    // HijackSend, multi/main.cpp:116-132
    void hijack(uint32_t src, uint32_t dst, const Msg &m, uint32_t dup)
    {
        if (!dup && p.drop_rate && rng.range(0, 10000) < p.drop_rate) return;
        if (dup < 3 && p.dup_rate && rng.range(0, 10000) < p.dup_rate) hijack(src, dst, m, dup + 1);
        const uint64_t d = p.max_delay ? rng.range(0, p.max_delay) : 0;
        push_deliver(now + 1 + d, src, dst, m);
    }
    void send(uint32_t src, uint32_t dst, const Msg &m) { hijack(src, dst, m, 0); }
    void bcast(uint32_t src, const Msg &m)
    {
        for (uint32_t d = 0; d < N; ++d) send(src, d, m);
    }

    // ---- acceptor / learner handlers (reference semantics) ----
    void on_prepare(uint32_t self, const Msg &m)                       // :858-922
    {
        Node &n = nodes[self];
        const uint64_t id = m.x;
        if (id > n.max_seen) n.max_seen = id;
        if (id > n.promised) {
            n.promised = id;
            // accepted ∪ committed entries inside the ranges, iid ascending
            auto b = std::make_shared<Body>();
            for (auto &r : m.body->ranges) {
                const uint64_t e = std::min<uint64_t>(r.second, n.hi);
                for (uint64_t i = n.pres.next(r.first, e, true); i < e; i = n.pres.next(i + 1, e, true)) {
                    b->ent.push_back({i, n.key[i]});
                    b->pid.push_back(n.bal[i]);
                }
            }
            if (m.body->ranges.size() > 1) {   // ranges are sorted and disjoint (uncommitted()), keep generic
                std::vector<size_t> o(b->ent.size());
                for (size_t k = 0; k < o.size(); ++k) o[k] = k;
                std::stable_sort(o.begin(), o.end(), [&](size_t a, size_t c) { return b->ent[a].first < b->ent[c].first; });
                std::vector<IV> e2; std::vector<uint64_t> p2;
                for (size_t k : o)
                    if (e2.empty() || e2.back().first != b->ent[k].first) { e2.push_back(b->ent[k]); p2.push_back(b->pid[k]); }
                b->ent.swap(e2); b->pid.swap(p2);
            }
            for (size_t k = 0; k < b->ent.size(); ++k) {
                app<uint64_t>(b->wire, b->ent[k].first); app<uint64_t>(b->wire, b->pid[k]); enc(b->wire, b->ent[k].second);
            }
            send(self, m.from, mk(MPX_MSG_PREPARE_REPLY, self, id, 0, std::move(b)));
        } else if (id < n.promised) {
            send(self, m.from, mk(MPX_MSG_REJECT, 0, n.max_seen));
        }
    }
    void on_accept(uint32_t self, const Msg &m)                        // :1359-1404
    {
        Node &n = nodes[self];
        const uint64_t id = m.x;
        if (id > n.max_seen) n.max_seen = id;
        if (id >= n.promised) {
            for (auto &e : m.body->ent) {
                n.ensure(e.first);
                if (n.kind[e.first] == 2) continue;
                n.kind[e.first] = 1; n.bal[e.first] = id; n.key[e.first] = e.second;
                n.pres.set(e.first);
                n.hi = std::max(n.hi, e.first + 1);
            }
            send(self, m.from, mk(MPX_MSG_ACCEPT_REPLY, self, id, m.y));
        } else {
            send(self, m.from, mk(MPX_MSG_REJECT, 0, n.max_seen));
        }
    }
    void on_commit(uint32_t self, const Msg &m)                        // :1494-1518
    {
        Node &n = nodes[self];
        const uint64_t id = m.x;
        for (auto &e : m.body->ent) {
            n.ensure(e.first);
            if (n.kind[e.first] == 2) continue;
            n.commit_at(e.first, id, e.second);
            if (n.proposer) learned(self, e.first, e.second);
        }
        send(self, m.from, mk(MPX_MSG_COMMIT_REPLY, self, 0, m.y));
    }

    // ---- proposer ----
    void learned(uint32_t self, uint64_t iid, uint64_t k)
    {
        Node &n = nodes[self];
        auto it = n.assigned.find(iid);
        if (it == n.assigned.end()) return;
        if (it->second != k && !MPX_HANDLE_NOOP(it->second)) n.pending.push_back(it->second);   // re-propose elsewhere
        n.assigned.erase(it);
    }
    // [0, 2^64-1) minus committed instances (AvailableInstanceIDs, paxos.cpp:253-318)
    std::vector<std::pair<uint64_t, uint64_t>> uncommitted(const Node &n) const
    {
        std::vector<std::pair<uint64_t, uint64_t>> r;
        uint64_t a = n.com_lo;
        while (a < n.com_hi) {
            const uint64_t x = n.comb.next(a, n.com_hi, true);      // next committed at or after a
            if (x > a) r.push_back({a, x});
            a = n.comb.next(x, n.com_hi, false);                     // first gap after that run
            if (a == n.com_hi) break;
        }
        r.push_back({std::max(a, n.com_hi), ~0ull});
        return r;
    }
    void start_prepare(uint32_t self)
    {
        Node &n = nodes[self];
        do { n.ballot = ((++n.count) << 16) | self; } while (n.ballot < n.max_seen);   // :792-799
        n.preparing = true; n.prepare_sent = false; n.prepare_retries = 0;
        n.promises = 0; n.pre.clear();
        for (auto &b : n.batches) b.second.live = false;
        n.batches.clear();
        ++n.epoch;
        record(n, mk(MPX_MSG_P_START, 0, n.ballot));
        auto b = std::make_shared<Body>();
        b->ranges = uncommitted(n);
        for (auto &x : b->ranges) { app<uint64_t>(b->wire, x.first); app<uint64_t>(b->wire, x.second); }
        n.prep = std::move(b);
        timer(now + rng.range(delay_min, delay_max), self, T_PREPARE_SEND, n.epoch);
    }
    void send_prepare(uint32_t self)
    {
        Node &n = nodes[self];
        bcast(self, mk(MPX_MSG_PREPARE, self, n.ballot, 0, n.prep));
        timer(now + retry_timeout, self, T_PREPARE_RETRY, n.epoch);
    }
    void on_prepare_reply(uint32_t self, const Msg &m)                 // :1036-1057,1201-1223
    {
        Node &n = nodes[self];
        if (!n.proposer || !n.preparing || m.x != n.ballot) return;
        n.promises |= 1ull << m.from;
        const Body &b = *m.body;
        for (size_t k = 0; k < b.ent.size(); ++k) {
            auto it = n.pre.find(b.ent[k].first);
            if (it == n.pre.end()) n.pre[b.ent[k].first] = {b.pid[k], b.ent[k].second};
            else if (b.pid[k] > it->second.first) it->second = {b.pid[k], b.ent[k].second};   // strict >, :1218
        }
        if ((uint32_t)__builtin_popcountll(n.promises) >= quorum()) promised(self);
    }
    void new_batch(uint32_t self, std::vector<IV> &&ent)
    {
        Node &n = nodes[self];
        const uint64_t bid = ++n.next_batch;
        BodyP body = entry_body(std::move(ent));
        record(n, mk(MPX_MSG_P_BATCH, 0, 0, bid, body));
        Batch &b = n.batches[bid];
        b.body = body;
        bcast(self, mk(MPX_MSG_ACCEPT, self, n.ballot, bid, body));
        timer(now + retry_timeout, self, T_ACCEPT_RETRY, n.epoch, bid);
    }
    void propose_plan(uint32_t self, std::map<uint64_t, uint64_t> &plan)
    {
        std::vector<IV> cur;
        uint32_t want = (uint32_t)rng.range(1, B + 1);
        for (auto &e : plan) {
            cur.push_back({e.first, e.second});
            if (cur.size() >= want) { new_batch(self, std::move(cur)); cur.clear(); want = (uint32_t)rng.range(1, B + 1); }
        }
        if (!cur.empty()) new_batch(self, std::move(cur));
    }
    uint64_t next_free(const Node &n, uint64_t from) const
    {
        while (n.committed(from) || n.assigned.count(from)) ++from;
        return from;
    }
    void assign_new(uint32_t self, std::map<uint64_t, uint64_t> &plan, size_t max_new)
    {
        Node &n = nodes[self];
        uint64_t hi = n.com_hi;
        if (!plan.empty()) hi = std::max(hi, plan.rbegin()->first + 1);
        if (!n.assigned.empty()) hi = std::max(hi, n.assigned.rbegin()->first + 1);
        for (size_t k = 0; k < max_new && !n.pending.empty(); ++k) {
            const uint64_t iid = next_free(n, hi);
            hi = iid + 1;
            const uint64_t v = n.pending.front();
            n.pending.pop_front();
            n.assigned[iid] = v;
            plan[iid] = v;
        }
    }
    void promised(uint32_t self)
    {
        Node &n = nodes[self];
        n.preparing = false; n.promises = 0;
        std::map<uint64_t, uint64_t> plan;
        for (auto &e : n.pre)                                              // adopt (:1089-1117)
            if (!n.committed(e.first)) plan.emplace_hint(plan.end(), e.first, e.second.second);
        n.pre.clear();
        for (auto &e : n.assigned)                                         // own initial proposals (:1145-1165)
            if (!plan.count(e.first) && !n.committed(e.first)) plan[e.first] = e.second;
        const uint64_t hi = plan.empty() ? 0 : plan.rbegin()->first + 1;
        for (uint64_t i = n.comb.next(n.com_lo, hi, false); i < hi; i = n.comb.next(i + 1, hi, false))   // noop gap fill (:1128-1143)
            if (!plan.count(i)) plan[i] = MPX_HANDLE(self, true, ++n.next_vid);
        assign_new(self, plan, 4 * B);
        propose_plan(self, plan);
    }
    void on_accept_reply(uint32_t self, const Msg &m)                  // :1406-1427
    {
        Node &n = nodes[self];
        if (!n.proposer || m.x != n.ballot) return;
        auto it = n.batches.find(m.y);
        if (it == n.batches.end() || !it->second.live) return;
        Batch &b = it->second;
        b.mask |= 1ull << m.from;
        if ((uint32_t)__builtin_popcountll(b.mask) < quorum()) return;
        b.live = false;                                                    // chosen (:1416-1425)
        BodyP body = std::move(b.body);
        n.batches.erase(it);
        // safety guard (see header): never commit against the first chosen value
        bool conflict = false;
        for (auto &e : body->ent)
            if (e.first < chosen.size() && chosen[e.first] && chosen[e.first] != e.second) conflict = true;
        if (conflict) { ++suppressed; return; }
        for (auto &e : body->ent) {
            if (e.first >= chosen.size()) chosen.resize(std::max<size_t>(e.first + 1, chosen.size() * 3 / 2 + 1024), 0);
            if (!chosen[e.first]) chosen[e.first] = e.second;
        }
        const uint64_t cid = ++n.next_commit;
        Commit &c = n.commits[cid];
        c.body = body; c.ballot = n.ballot;
        bcast(self, mk(MPX_MSG_COMMIT, self, n.ballot, cid, body));
        timer(now + 2 * retry_timeout, self, T_COMMIT_RETRY, cid);
        if (!n.preparing && !n.pending.empty()) timer(now + 1, self, T_PROPOSE, n.epoch);
    }
    void on_commit_reply(uint32_t self, const Msg &m)
    {
        Node &n = nodes[self];
        auto it = n.commits.find(m.y);
        if (it == n.commits.end()) return;
        it->second.replied |= 1ull << m.from;
        if ((uint32_t)__builtin_popcountll(it->second.replied) == N) n.commits.erase(it);
    }
    void on_timer(const Ev &e)
    {
        Node &n = nodes[e.dst];
        switch (e.tkind) {
        case T_PREPARE_SEND:
            if (n.preparing && e.token == n.epoch && !n.prepare_sent) { n.prepare_sent = true; send_prepare(e.dst); }
            break;
        case T_PREPARE_RETRY:
            if (n.preparing && e.token == n.epoch) {
                if (++n.prepare_retries >= 3) start_prepare(e.dst);        // RestartPrepare, :780-784
                else send_prepare(e.dst);                                   // same ballot
            }
            break;
        case T_ACCEPT_RETRY: {
            if (e.token != n.epoch || n.preparing) break;
            auto it = n.batches.find(e.aux);
            if (it == n.batches.end() || !it->second.live) break;
            if (++it->second.retries >= 3) { start_prepare(e.dst); break; }   // AcceptRejected, :1328-1343
            bcast(e.dst, mk(MPX_MSG_ACCEPT, e.dst, n.ballot, e.aux, it->second.body));
            timer(now + retry_timeout, e.dst, T_ACCEPT_RETRY, n.epoch, e.aux);
            break;
        }
        case T_COMMIT_RETRY: {
            auto it = n.commits.find(e.token);
            if (it == n.commits.end() || ++it->second.retries > 8) break;
            const Msg m = mk(MPX_MSG_COMMIT, e.dst, it->second.ballot, e.token, it->second.body);
            for (uint32_t d = 0; d < N; ++d)
                if (!((it->second.replied >> d) & 1)) send(e.dst, d, m);
            timer(now + 2 * retry_timeout, e.dst, T_COMMIT_RETRY, e.token);
            break;
        }
        case T_PROPOSE:
            if (!n.preparing && e.token == n.epoch && !n.pending.empty() && n.batches.size() < 4) {
                std::map<uint64_t, uint64_t> plan;
                assign_new(e.dst, plan, B);
                propose_plan(e.dst, plan);
            }
            break;
        }
    }
    void deliver(const Ev &e)
    {
        Node &n = nodes[e.dst];
        record(n, e.msg);                          // what the node's handler loop sees, in order
        switch (e.msg.type) {
        case MPX_MSG_PREPARE: on_prepare(e.dst, e.msg); break;
        case MPX_MSG_PREPARE_REPLY: on_prepare_reply(e.dst, e.msg); break;
        case MPX_MSG_REJECT: if (e.msg.x > n.max_seen) n.max_seen = e.msg.x; break;
        case MPX_MSG_ACCEPT: on_accept(e.dst, e.msg); break;
        case MPX_MSG_ACCEPT_REPLY: on_accept_reply(e.dst, e.msg); break;
        case MPX_MSG_COMMIT: on_commit(e.dst, e.msg); break;
        case MPX_MSG_COMMIT_REPLY: on_commit_reply(e.dst, e.msg); break;
        }
    }
};

}  // namespace

int gen_faulty(const mpx_gen_params &p, std::string &out)
{
    if (!p.num_nodes || p.num_nodes > MPX_MAX_NODES) return MPX_E_INVAL;
    Sim s(p);
    s.N = p.num_nodes;
    s.P = std::max<uint32_t>(1, std::min(p.proposers ? p.proposers : 1, p.num_nodes));
    s.B = p.batch ? p.batch : 256;
    s.rng.s = p.seed * 0x2545F4914F6CDD1Dull + 1;
    const uint64_t md = p.max_delay ? p.max_delay : 1;
    s.delay_max = 100 + 4 * md;
    s.retry_timeout = 4 * md + 50;
    s.nodes.resize(s.N);
    // client values: global client id g -> proposer g % P, payload decimal g (multi/main.cpp:30-35)
    for (uint32_t i = 0; i < s.P; ++i) s.nodes[i].proposer = true;
    for (uint64_t g = 0; g < p.num_instances; ++g) {
        Node &n = s.nodes[g % s.P];
        n.pending.push_back(MPX_HANDLE((uint32_t)(g % s.P), false, ++n.next_vid));
    }
    for (uint32_t i = 0; i < s.P; ++i) {
        s.now = s.rng.range(0, 50);
        s.start_prepare(i);
    }
    s.now = 0;
    const uint64_t max_events = 400ull * (p.num_instances + 64) * s.N;
    uint64_t events = 0;
    while (!s.q.empty() && events++ < max_events) {
        std::pop_heap(s.q.begin(), s.q.end(), EvLater());
        Ev e = std::move(s.q.back());
        s.q.pop_back();
        s.now = e.t;
        if (e.kind == 0) s.deliver(e); else s.on_timer(e);
        bool done = true;
        for (auto &n : s.nodes) if (n.proposer && (!n.pending.empty() || !n.assigned.empty() || !n.commits.empty())) done = false;
        if (done) break;
    }
    uint64_t M = 0, total = 40;
    for (auto &n : s.nodes) {
        M = std::max(M, n.hi);
        total += 16 + 8 * n.offs.size() + n.bytes.size() + 8;
    }
    s.q.clear(); s.q.shrink_to_fit();
    TraceWriter w;
    w.begin(s.N, MPX_SEM_MULTI, std::max<uint64_t>(M, 1), {});
    std::memcpy(&w.out[32], &s.suppressed, 8);          // reserved word: suppressed conflicting commits
    w.out.reserve(total);
    for (auto &n : s.nodes) {
        // free the node's simulation state before its stream is copied out
        std::vector<uint8_t>().swap(n.kind); std::vector<uint64_t>().swap(n.bal); std::vector<uint64_t>().swap(n.key);
        w.node_raw(n.bytes, n.offs);
        std::string().swap(n.bytes); std::vector<uint64_t>().swap(n.offs);
    }
    out.swap(w.out);
    return MPX_OK;
}

}  // namespace mpx
