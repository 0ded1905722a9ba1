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
// Safety guard: the reference's acceptor does not raise its promise on accept
// and lets a lower (>= promised) ballot overwrite (:1366,1387), so a delayed
// stale ACCEPT can in rare schedules let two values be chosen for one
// instance; a learner receiving both would ASSERT (:1508).  The simulator
// registers the first committed value per instance and never sends a COMMIT
// that contradicts it (counted in the trace header's reserved word).
#include <algorithm>
#include <cstring>
#include <deque>
#include <map>
#include <queue>
#include <set>
#include <string>
#include <unordered_map>
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

struct Val {                     // a reference Value: (proposer, value_id, noop, payload)
    uint32_t proposer = 0;
    uint64_t id = 0;
    bool noop = false;
    std::string payload;
    uint64_t key() const { return MPX_HANDLE(proposer, noop, id); }
};

void enc(std::string &s, const Val &v) { enc_value(s, v.proposer, v.id, v.noop, v.payload); }

struct Ev {
    uint64_t t, seq;
    int kind;                    // 0 deliver, 1 timer
    uint32_t dst, src;
    std::string msg;
    uint32_t tkind;              // timer kind
    uint64_t token, aux;
    bool operator<(const Ev &o) const { return t != o.t ? t > o.t : seq > o.seq; }
};

enum { T_PREPARE_SEND = 1, T_PREPARE_RETRY, T_ACCEPT_RETRY, T_COMMIT_RETRY, T_PROPOSE };

struct Batch {
    std::vector<std::pair<uint64_t, Val>> ent;
    uint64_t mask = 0;
    uint32_t retries = 0;
    bool live = true;
};

struct Commit {
    std::string body;
    uint64_t ballot;
    uint64_t replied = 0;
    uint32_t retries = 0;
};

struct Node {
    // acceptor / learner (reference semantics)
    uint64_t promised = 0, max_seen = 0;
    std::unordered_map<uint64_t, std::pair<uint64_t, Val>> acc, com;
    // proposer
    bool proposer = false;
    uint64_t count = 0, ballot = 0, epoch = 0;
    bool preparing = false, prepare_sent = false;
    uint32_t prepare_retries = 0;
    uint64_t promises = 0;
    std::map<uint64_t, std::pair<uint64_t, Val>> pre;
    std::map<uint64_t, Batch> batches;
    uint64_t next_batch = 0, next_commit = 0, next_vid = 0;
    std::map<uint64_t, Commit> commits;
    std::deque<Val> pending;             // own values not assigned to an instance
    std::map<uint64_t, Val> assigned;    // own values at an instance, not yet known committed
    std::vector<std::pair<uint64_t, uint64_t>> prep_ranges;
    // output
    std::vector<std::string> stream;
};

struct Sim {
    const mpx_gen_params &p;
    uint32_t N, P, B;
    Rng rng;
    uint64_t now = 0, seq = 0;
    std::priority_queue<Ev> q;
    std::vector<Node> nodes;
    std::unordered_map<uint64_t, uint64_t> chosen;   // iid -> first committed value key
    uint64_t suppressed = 0;
    uint64_t delay_min = 100, delay_max;              // PrepareDelay ticks
    uint64_t retry_timeout;
    explicit Sim(const mpx_gen_params &pp) : p(pp) {}

    uint32_t quorum() const { return N / 2 + 1; }

    void push_deliver(uint64_t at, uint32_t src, uint32_t dst, const std::string &m)
    {
        Ev e{at, seq++, 0, dst, src, m, 0, 0, 0};
        q.push(std::move(e));
    }
    void timer(uint64_t at, uint32_t node, uint32_t kind, uint64_t token, uint64_t aux = 0)
    {
        Ev e{at, seq++, 1, node, node, std::string(), kind, token, aux};
        q.push(std::move(e));
    }
    // HijackSend, multi/main.cpp:116-132
    void hijack(uint32_t src, uint32_t dst, const std::string &m, uint32_t dup)
    {
        if (!dup && p.drop_rate && rng.range(0, 10000) < p.drop_rate) return;
        if (dup < 3 && p.dup_rate && rng.range(0, 10000) < p.dup_rate) hijack(src, dst, m, dup + 1);
        const uint64_t d = p.max_delay ? rng.range(0, p.max_delay) : 0;
        push_deliver(now + 1 + d, src, dst, m);
    }
    void send(uint32_t src, uint32_t dst, const std::string &m) { hijack(src, dst, m, 0); }
    void bcast(uint32_t src, const std::string &m)
    {
        for (uint32_t d = 0; d < N; ++d) send(src, d, m);
    }

    // ---- acceptor / learner handlers (reference semantics) ----
    void on_prepare(uint32_t self, const std::string &m)
    {
        Node &n = nodes[self];
        uint32_t proposer; uint64_t id; uint32_t len;
        std::memcpy(&proposer, m.data() + 4, 4); std::memcpy(&id, m.data() + 8, 8); std::memcpy(&len, m.data() + 16, 4);
        if (id > n.max_seen) n.max_seen = id;
        if (id > n.promised) {
            n.promised = id;
            std::map<uint64_t, std::pair<uint64_t, Val>> out;
            for (uint32_t r = 0; r < len / 16; ++r) {
                uint64_t a, b;
                std::memcpy(&a, m.data() + 20 + 16 * r, 8); std::memcpy(&b, m.data() + 28 + 16 * r, 8);
                for (auto &e : n.acc) if (e.first >= a && e.first < b) out[e.first] = e.second;
                for (auto &e : n.com) if (e.first >= a && e.first < b) out[e.first] = e.second;
            }
            std::string body;
            for (auto &e : out) { app<uint64_t>(body, e.first); app<uint64_t>(body, e.second.first); enc(body, e.second.second); }
            send(self, proposer, msg_prepare_reply(self, id, body));
        } else if (id < n.promised) {
            send(self, proposer, msg_reject(n.max_seen));
        }
    }
    static std::vector<std::pair<uint64_t, Val>> decode_entries(const std::string &m, size_t at, uint32_t len)
    {
        std::vector<std::pair<uint64_t, Val>> v;
        size_t cur = at, end = at + len;
        while (cur < end) {
            uint64_t iid; std::memcpy(&iid, m.data() + cur, 8); cur += 8;
            Val x;
            std::memcpy(&x.proposer, m.data() + cur, 4); std::memcpy(&x.id, m.data() + cur + 4, 8);
            x.noop = m[cur + 12] != 0;
            if (x.noop) cur += 13;
            else {
                uint32_t l; std::memcpy(&l, m.data() + cur + 14, 4);
                x.payload.assign(m.data() + cur + 18, l);
                cur += 18 + l;
            }
            v.push_back({iid, std::move(x)});
        }
        return v;
    }
    void on_accept(uint32_t self, const std::string &m)
    {
        Node &n = nodes[self];
        uint32_t proposer, len; uint64_t aid, id;
        std::memcpy(&proposer, m.data() + 4, 4); std::memcpy(&aid, m.data() + 8, 8);
        std::memcpy(&id, m.data() + 16, 8); std::memcpy(&len, m.data() + 24, 4);
        if (id > n.max_seen) n.max_seen = id;
        if (id >= n.promised) {
            for (auto &e : decode_entries(m, 28, len))
                if (!n.com.count(e.first)) n.acc[e.first] = {id, e.second};
            send(self, proposer, msg_accept_reply(self, id, aid));
        } else {
            send(self, proposer, msg_reject(n.max_seen));
        }
    }
    void on_commit(uint32_t self, const std::string &m)
    {
        Node &n = nodes[self];
        uint32_t committer, len; uint64_t cid, id;
        std::memcpy(&committer, m.data() + 4, 4); std::memcpy(&cid, m.data() + 8, 8);
        std::memcpy(&id, m.data() + 16, 8); std::memcpy(&len, m.data() + 24, 4);
        for (auto &e : decode_entries(m, 28, len)) {
            n.acc.erase(e.first);
            if (!n.com.count(e.first)) {
                n.com[e.first] = {id, e.second};
                if (n.proposer) learned(self, e.first, e.second);
            }
        }
        send(self, committer, msg_commit_reply(self, cid));
    }

    // ---- proposer ----
    void learned(uint32_t self, uint64_t iid, const Val &v)
    {
        Node &n = nodes[self];
        auto it = n.assigned.find(iid);
        if (it == n.assigned.end()) return;
        if (it->second.key() != v.key() && !it->second.noop) n.pending.push_back(it->second);   // re-propose elsewhere
        n.assigned.erase(it);
    }
    std::vector<std::pair<uint64_t, uint64_t>> uncommitted(const Node &n) const
    {
        // [0, 2^64-1) minus committed instances (AvailableInstanceIDs, paxos.cpp:253-318)
        std::vector<uint64_t> c;
        c.reserve(n.com.size());
        for (auto &e : n.com) c.push_back(e.first);
        std::sort(c.begin(), c.end());
        std::vector<std::pair<uint64_t, uint64_t>> r;
        uint64_t a = 0;
        for (uint64_t x : c) { if (x > a) r.push_back({a, x}); a = x + 1; }
        r.push_back({a, ~0ull});
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
        n.stream.push_back(msg_p_start(n.ballot));
        n.prep_ranges = uncommitted(n);
        timer(now + rng.range(delay_min, delay_max), self, T_PREPARE_SEND, n.epoch);
    }
    void send_prepare(uint32_t self)
    {
        Node &n = nodes[self];
        bcast(self, msg_prepare(self, n.ballot, n.prep_ranges));
        timer(now + retry_timeout, self, T_PREPARE_RETRY, n.epoch);
    }
    void on_prepare_reply(uint32_t self, const std::string &m)
    {
        Node &n = nodes[self];
        uint32_t acceptor, len; uint64_t id;
        std::memcpy(&acceptor, m.data() + 4, 4); std::memcpy(&id, m.data() + 8, 8); std::memcpy(&len, m.data() + 16, 4);
        if (!n.proposer || !n.preparing || id != n.ballot) return;
        n.promises |= 1ull << acceptor;
        size_t cur = 20, end = 20 + len;
        while (cur < end) {
            uint64_t iid, pid; std::memcpy(&iid, m.data() + cur, 8); std::memcpy(&pid, m.data() + cur + 8, 8); cur += 16;
            Val x;
            std::memcpy(&x.proposer, m.data() + cur, 4); std::memcpy(&x.id, m.data() + cur + 4, 8);
            x.noop = m[cur + 12] != 0;
            if (x.noop) cur += 13;
            else { uint32_t l; std::memcpy(&l, m.data() + cur + 14, 4); x.payload.assign(m.data() + cur + 18, l); cur += 18 + l; }
            auto it = n.pre.find(iid);
            if (it == n.pre.end()) n.pre[iid] = {pid, x};
            else if (pid > it->second.first) it->second = {pid, x};         // strict >, :1218
        }
        if ((uint32_t)__builtin_popcountll(n.promises) >= quorum()) promised(self);
    }
    void new_batch(uint32_t self, std::vector<std::pair<uint64_t, Val>> &&ent)
    {
        Node &n = nodes[self];
        const uint64_t bid = ++n.next_batch;
        std::string body;
        for (auto &e : ent) { app<uint64_t>(body, e.first); enc(body, e.second); }
        n.stream.push_back(msg_p_batch(bid, body));
        Batch &b = n.batches[bid];
        b.ent = std::move(ent);
        bcast(self, msg_accept(self, bid, n.ballot, body));
        timer(now + retry_timeout, self, T_ACCEPT_RETRY, n.epoch, bid);
    }
    void propose_plan(uint32_t self, std::map<uint64_t, Val> &plan)
    {
        std::vector<std::pair<uint64_t, Val>> cur;
        uint32_t want = (uint32_t)rng.range(1, B + 1);
        for (auto &e : plan) {
            cur.push_back({e.first, e.second});
            if (cur.size() >= want) { new_batch(self, std::move(cur)); cur.clear(); want = (uint32_t)rng.range(1, B + 1); }
        }
        if (!cur.empty()) new_batch(self, std::move(cur));
    }
    uint64_t next_free(const Node &n, uint64_t from) const
    {
        while (n.com.count(from) || n.assigned.count(from)) ++from;
        return from;
    }
    void assign_new(uint32_t self, std::map<uint64_t, Val> &plan, size_t max_new)
    {
        Node &n = nodes[self];
        uint64_t hi = 0;
        for (auto &e : n.com) hi = std::max(hi, e.first + 1);
        for (auto &e : plan) hi = std::max(hi, e.first + 1);
        for (auto &e : n.assigned) hi = std::max(hi, e.first + 1);
        for (size_t k = 0; k < max_new && !n.pending.empty(); ++k) {
            const uint64_t iid = next_free(n, hi);
            hi = iid + 1;
            Val v = n.pending.front();
            n.pending.pop_front();
            n.assigned[iid] = v;
            plan[iid] = v;
        }
    }
    void promised(uint32_t self)
    {
        Node &n = nodes[self];
        n.preparing = false; n.promises = 0;
        std::map<uint64_t, Val> plan;
        for (auto &e : n.pre)                                              // adopt (:1089-1117)
            if (!n.com.count(e.first)) plan[e.first] = e.second.second;
        n.pre.clear();
        for (auto &e : n.assigned)                                         // own initial proposals (:1145-1165)
            if (!plan.count(e.first) && !n.com.count(e.first)) plan[e.first] = e.second;
        uint64_t hi = 0;
        for (auto &e : plan) hi = std::max(hi, e.first + 1);
        for (uint64_t i = 0; i < hi; ++i)                                  // noop gap fill (:1128-1143)
            if (!plan.count(i) && !n.com.count(i)) {
                Val z; z.proposer = self; z.id = ++n.next_vid; z.noop = true;
                plan[i] = z;
            }
        assign_new(self, plan, 4 * B);
        propose_plan(self, plan);
    }
    void on_accept_reply(uint32_t self, const std::string &m)
    {
        Node &n = nodes[self];
        uint32_t acceptor; uint64_t id, aid;
        std::memcpy(&acceptor, m.data() + 4, 4); std::memcpy(&id, m.data() + 8, 8); std::memcpy(&aid, m.data() + 16, 8);
        if (!n.proposer || id != n.ballot) return;
        auto it = n.batches.find(aid);
        if (it == n.batches.end() || !it->second.live) return;
        Batch &b = it->second;
        b.mask |= 1ull << acceptor;
        if ((uint32_t)__builtin_popcountll(b.mask) < quorum()) return;
        b.live = false;                                                    // chosen (:1416-1425)
        std::vector<std::pair<uint64_t, Val>> ent = std::move(b.ent);
        n.batches.erase(it);
        // safety guard (see header): never commit against the first chosen value
        bool conflict = false;
        for (auto &e : ent) {
            auto c = chosen.find(e.first);
            if (c != chosen.end() && c->second != e.second.key()) conflict = true;
        }
        if (conflict) { ++suppressed; return; }
        for (auto &e : ent) chosen.emplace(e.first, e.second.key());
        std::string body;
        for (auto &e : ent) { app<uint64_t>(body, e.first); enc(body, e.second); }
        const uint64_t cid = ++n.next_commit;
        Commit &c = n.commits[cid];
        c.body = body; c.ballot = n.ballot;
        bcast(self, msg_commit(self, cid, n.ballot, body));
        timer(now + 2 * retry_timeout, self, T_COMMIT_RETRY, cid);
        if (!n.preparing && !n.pending.empty()) timer(now + 1, self, T_PROPOSE, n.epoch);
    }
    void on_commit_reply(uint32_t self, const std::string &m)
    {
        Node &n = nodes[self];
        uint32_t learner; uint64_t cid;
        std::memcpy(&learner, m.data() + 4, 4); std::memcpy(&cid, m.data() + 8, 8);
        auto it = n.commits.find(cid);
        if (it == n.commits.end()) return;
        it->second.replied |= 1ull << learner;
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
            std::string body;
            for (auto &x : it->second.ent) { app<uint64_t>(body, x.first); enc(body, x.second); }
            bcast(e.dst, msg_accept(e.dst, e.aux, n.ballot, body));
            timer(now + retry_timeout, e.dst, T_ACCEPT_RETRY, n.epoch, e.aux);
            break;
        }
        case T_COMMIT_RETRY: {
            auto it = n.commits.find(e.token);
            if (it == n.commits.end() || ++it->second.retries > 8) break;
            const std::string m = msg_commit(e.dst, e.token, it->second.ballot, it->second.body);
            for (uint32_t d = 0; d < N; ++d)
                if (!((it->second.replied >> d) & 1)) send(e.dst, d, m);
            timer(now + 2 * retry_timeout, e.dst, T_COMMIT_RETRY, e.token);
            break;
        }
        case T_PROPOSE:
            if (!n.preparing && e.token == n.epoch && !n.pending.empty() && n.batches.size() < 4) {
                std::map<uint64_t, Val> plan;
                assign_new(e.dst, plan, B);
                propose_plan(e.dst, plan);
            }
            break;
        }
    }
    void deliver(const Ev &e)
    {
        Node &n = nodes[e.dst];
        n.stream.push_back(e.msg);                     // what the node's handler loop sees, in order
        uint32_t t; std::memcpy(&t, e.msg.data(), 4);
        switch (t) {
        case MPX_MSG_PREPARE: on_prepare(e.dst, e.msg); break;
        case MPX_MSG_PREPARE_REPLY: on_prepare_reply(e.dst, e.msg); break;
        case MPX_MSG_REJECT: { uint64_t x; std::memcpy(&x, e.msg.data() + 4, 8); if (x > n.max_seen) n.max_seen = x; break; }
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
        Val v; v.proposer = (uint32_t)(g % s.P); v.id = ++n.next_vid; v.payload = std::to_string(g);
        n.pending.push_back(v);
    }
    for (uint32_t i = 0; i < s.P; ++i) {
        s.now = s.rng.range(0, 50);
        s.start_prepare(i);
    }
    s.now = 0;
    const uint64_t max_events = 400ull * (p.num_instances + 64) * s.N;
    uint64_t events = 0;
    while (!s.q.empty() && events++ < max_events) {
        Ev e = s.q.top();
        s.q.pop();
        s.now = e.t;
        if (e.kind == 0) s.deliver(e); else s.on_timer(e);
        bool done = true;
        for (auto &n : s.nodes) if (n.proposer && (!n.pending.empty() || !n.assigned.empty() || !n.commits.empty())) done = false;
        if (done) break;
    }
    uint64_t M = 0;
    for (auto &n : s.nodes) for (auto &c : n.com) M = std::max(M, c.first + 1);
    for (auto &n : s.nodes) for (auto &c : n.acc) M = std::max(M, c.first + 1);
    TraceWriter w;
    w.begin(s.N, MPX_SEM_MULTI, std::max<uint64_t>(M, 1), {});
    std::memcpy(&w.out[32], &s.suppressed, 8);          // reserved word: suppressed conflicting commits
    for (auto &n : s.nodes) w.node(n.stream);
    out.swap(w.out);
    return MPX_OK;
}

}  // namespace mpx
