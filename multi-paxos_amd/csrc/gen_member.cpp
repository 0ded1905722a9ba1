// gen_member.cpp — C5 member-semantics traces, host.
//
// One leader (node 0, the demo's `first`, member/main.cpp:187-195) drives the
// demo's membership schedule (member/main.cpp:119-141): AddAcceptor(1..U-1),
// then DelAcceptor(1..U-1), one membership Value per change, so the acceptor
// set grows 1,2,..,U and shrinks back (2U-1 epochs, version = epoch).  The
// instance space is split evenly over the epochs; the last instance of each
// epoch's range holds the membership Value of the next change.
//
// Every node's acceptor / learner is simulated with the reference's rules
// (member/paxos.cpp:1029-1060,1700-1793) while its receive stream is written,
// so each reply the leader receives carries what that node would send:
//   * PREPARE over [first unlearned, 2^64-1) after every epoch change
//     (AcceptorsChanged -> StartPrepare, :1291-1322); the promise quorum is
//     |acceptors|/2+1 of the epoch;
//   * batches of U[1,B] instances, ACCEPT to the acceptors, LEARN to the
//     learners once a quorum replied (:1317-1343), LEARN_REPLY back;
//   * batches the leader sent after the membership Value and before applying
//     it are in flight across the change: acceptors that switched version drop
//     them (:1744), the others accept them under the old ballot, and the new
//     leader round re-proposes them (insert keeps the first pid, :1765);
//   * a new learner receives one catch-up LEARN with every learned Value
//     (LearnersChanged, :1265-1289) and walks through all epochs at once;
//   * drop_rate: a PREPARE/ACCEPT/LEARN delivery is lost and re-sent at the
//     next retry point (PrepareRetryTimeout / AcceptRetryTimeout /
//     LearnRetryTimeout); dup_rate: a delivery is duplicated, the copy arriving
//     up to max_delay deliveries later (stale versions get dropped).
// Epoch changes are marked with E_EPOCH records right after the LEARN whose
// apply performed them (include/mpx.h); the leader's new rounds with P_START.
#include <algorithm>
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

// instance Values: kind 0 normal, 1 noop, 2 membership change c
struct Inst { uint64_t vid; uint32_t kind; uint32_t change; };

enum Kind { D_PREPARE, D_ACCEPT, D_LEARN };

struct Delivery {
    Kind kind;
    uint32_t version;
    uint64_t ballot, id;          // ballot; batch or learn id
    uint64_t lo;                  // PREPARE range start
    std::vector<uint64_t> iids;   // ACCEPT / LEARN entries
    std::vector<uint64_t> pids;
    // entry bytes, encoded once and shared by every copy of the delivery
    mutable std::shared_ptr<const std::string> body;
};

struct Pending { uint64_t due; Delivery d; };

struct SimNode {
    uint32_t epoch = 0;
    bool acc = false;
    uint64_t promised = 0, maxs = 0;
    std::map<uint64_t, uint64_t> accepted;    // iid -> pid (Value = the instance's)
    std::vector<uint8_t> learned;             // per instance
    std::vector<uint64_t> learned_pid;
    uint64_t next_apply = 0, max_learned = 0;
    uint64_t appended = 0;
    std::string bytes;                        // receive stream: concatenated records
    std::vector<uint64_t> offs{0};
    std::deque<Pending> later;
};

struct Gen {
    uint32_t U;
    uint64_t M;
    uint32_t E;                               // epochs
    std::vector<mpx_epoch> ep;
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> changes;   // per change c >= 1
    std::vector<Inst> inst;
    std::vector<SimNode> nd;
    Rng rng;
    uint32_t drop, dup, max_delay;

    std::string value(uint64_t iid) const
    {
        const Inst &x = inst[iid];
        std::string s;
        app<uint32_t>(s, 0); app<uint64_t>(s, x.vid); app<uint8_t>(s, x.kind == 1);
        if (x.kind == 1) return s;
        if (x.kind == 2) {
            app<uint8_t>(s, 1);
            app<uint32_t>(s, (uint32_t)changes[x.change].size());
            for (auto &c : changes[x.change]) { app<uint32_t>(s, c.first); app<uint32_t>(s, c.second); }
            const std::string cb = "member " + std::to_string(x.change);
            app<uint32_t>(s, (uint32_t)cb.size()); s += cb;
        } else {
            const std::string p = std::to_string(x.vid - 1);        // Propose(ToStr(i), ToStr(i)), main.cpp:208
            app<uint8_t>(s, 0); app<uint32_t>(s, (uint32_t)p.size()); s += p;
            app<uint32_t>(s, (uint32_t)p.size()); s += p;
        }
        return s;
    }
    std::string entries(const std::vector<uint64_t> &iids, const std::vector<uint64_t> &pids) const
    {
        std::string s;
        s.reserve(iids.size() * 48);
        for (size_t i = 0; i < iids.size(); ++i) { app<uint64_t>(s, iids[i]); app<uint64_t>(s, pids[i]); s += value(iids[i]); }
        return s;
    }
    const std::string &body_of(const Delivery &d) const
    {
        if (!d.body) d.body = std::make_shared<const std::string>(entries(d.iids, d.pids));
        return *d.body;
    }

    void append(uint32_t n, const std::string &m)
    {
        SimNode &x = nd[n];
        x.bytes += m;
        x.offs.push_back(x.bytes.size());
        x.appended++;
    }
    // the leader's receive stream gets replies at once
    void to_leader(const std::string &m) { append(0, m); }

    // ---- acceptor / learner simulation while writing node n's stream --------
    // returns 1 granted, 0 otherwise
    int process(uint32_t n, const Delivery &d)
    {
        SimNode &x = nd[n];
        std::string m;
        if (d.kind == D_PREPARE) {
            app<uint32_t>(m, MPX_MSG_PREPARE); app<uint32_t>(m, d.version); app<uint32_t>(m, 0);
            app<uint64_t>(m, d.ballot); app<uint32_t>(m, 16); app<uint64_t>(m, d.lo); app<uint64_t>(m, ~0ull);
            append(n, m);
            if (!x.acc || d.version != ep[x.epoch].version) return 0;
            x.maxs = std::max(x.maxs, d.ballot);
            if (d.ballot > x.promised) {
                x.promised = d.ballot;
                std::vector<uint64_t> ii, pp;
                std::map<uint64_t, uint64_t> all;
                for (auto it = x.accepted.lower_bound(d.lo); it != x.accepted.end(); ++it) all[it->first] = it->second;
                for (uint64_t i = d.lo; i <= x.max_learned && i < M; ++i)
                    if (x.learned[i]) all[i] = x.learned_pid[i];
                for (auto &e : all) { ii.push_back(e.first); pp.push_back(e.second); }
                std::string body = entries(ii, pp), r;
                app<uint32_t>(r, MPX_MSG_PREPARE_REPLY); app<uint32_t>(r, n); app<uint64_t>(r, d.ballot);
                app<uint32_t>(r, (uint32_t)body.size()); r += body;
                to_leader(r);
                return 1;
            }
            if (d.ballot < x.promised) { std::string r; app<uint32_t>(r, MPX_MSG_REJECT); app<uint64_t>(r, x.maxs); to_leader(r); }
            return 0;
        }
        if (d.kind == D_ACCEPT) {
            const std::string &body = body_of(d);
            app<uint32_t>(m, MPX_MSG_ACCEPT); app<uint32_t>(m, d.version); app<uint32_t>(m, 0);
            app<uint64_t>(m, d.id); app<uint64_t>(m, d.ballot); app<uint32_t>(m, (uint32_t)body.size()); m += body;
            append(n, m);
            if (!x.acc || d.version != ep[x.epoch].version) return 0;
            x.maxs = std::max(x.maxs, d.ballot);
            if (d.ballot >= x.promised) {
                for (size_t i = 0; i < d.iids.size(); ++i)
                    if (!x.learned[d.iids[i]]) x.accepted.insert(std::make_pair(d.iids[i], d.pids[i]));
                std::string r;
                app<uint32_t>(r, MPX_MSG_ACCEPT_REPLY); app<uint32_t>(r, n); app<uint64_t>(r, d.id);
                to_leader(r);
                return 1;
            }
            std::string r; app<uint32_t>(r, MPX_MSG_REJECT); app<uint64_t>(r, x.maxs); to_leader(r);
            return 0;
        }
        // LEARN
        const std::string &body = body_of(d);
        app<uint32_t>(m, MPX_MSG_COMMIT); app<uint32_t>(m, 0); app<uint64_t>(m, d.id);
        app<uint32_t>(m, (uint32_t)body.size()); m += body;
        append(n, m);
        for (size_t i = 0; i < d.iids.size(); ++i) {
            const uint64_t iid = d.iids[i];
            x.accepted.erase(iid);
            if (!x.learned[iid]) { x.learned[iid] = 1; x.learned_pid[iid] = d.pids[i]; x.max_learned = std::max(x.max_learned, iid); }
        }
        std::vector<uint32_t> steps;
        while (x.next_apply < M && x.learned[x.next_apply]) {
            const Inst &v = inst[x.next_apply++];
            if (v.kind == 2) steps.push_back(v.change);
        }
        for (uint32_t c : steps) {
            std::string e; app<uint32_t>(e, MPX_MSG_E_EPOCH); app<uint32_t>(e, c);
            append(n, e);
            const bool acc = (ep[c].acceptor_mask >> n) & 1;
            if (acc != x.acc) { x.accepted.clear(); x.promised = x.maxs = 0; x.acc = acc; }
            x.epoch = c;
        }
        std::string r; app<uint32_t>(r, MPX_MSG_COMMIT_REPLY); app<uint32_t>(r, n); app<uint64_t>(r, d.id);
        to_leader(r);
        return 1;
    }

    // deliver due delayed copies, then this one (unless lost); returns granted
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

}  // namespace

int gen_member(const mpx_gen_params &p, std::string &out)
{
    const uint32_t U = p.num_nodes;
    if (U < 2 || U > 64) return MPX_E_INVAL;
    Gen g;
    g.U = U;
    g.M = p.num_instances;
    g.E = 2 * (U - 1) + 1;
    if (g.M < 4ull * g.E || g.M >= (1ull << 40)) return MPX_E_INVAL;
    g.rng.s = p.seed * 0x2545F4914F6CDD1Dull + 7;
    g.drop = p.drop_rate; g.dup = p.dup_rate; g.max_delay = p.max_delay ? p.max_delay : 64;
    const uint32_t B = p.batch ? p.batch : 64;

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
    // instance Values: the epoch ranges, membership Value last in each range
    std::vector<uint64_t> start(g.E + 1);
    for (uint32_t e = 0; e <= g.E; ++e) start[e] = g.M * e / g.E;
    g.inst.resize(g.M);
    uint64_t vid = 0;
    for (uint64_t i = 0; i < g.M; ++i) {
        g.inst[i].vid = ++vid;
        g.inst[i].kind = (p.noop_permille && g.rng.below(1000) < p.noop_permille) ? 1 : 0;
        g.inst[i].change = 0;
    }
    for (uint32_t c = 1; c < g.E; ++c) { g.inst[start[c] - 1].kind = 2; g.inst[start[c] - 1].change = c; }

    g.nd.resize(U);
    for (uint32_t n = 0; n < U; ++n) {
        g.nd[n].learned.assign(g.M, 0);
        g.nd[n].learned_pid.assign(g.M, 0);
    }
    g.nd[0].acc = true;

    uint64_t bcount = 0, batch_id = 0, learn_id = 0;
    std::deque<uint64_t> inflight;            // proposed, not chosen (instance order)
    uint64_t next_new = 0;
    uint64_t learners = 1;                    // learners_ of the leader
    for (uint32_t e = 0; e < g.E; ++e) {
        const uint64_t S = g.ep[e].acceptor_mask;
        const uint32_t Q = (uint32_t)__builtin_popcountll(S) / 2 + 1;
        std::vector<uint32_t> acc;
        for (uint32_t n = 0; n < U; ++n) if ((S >> n) & 1) acc.push_back(n);
        // ---- new leader round: P_START, PREPARE over the unlearned tail ----
        const uint64_t ballot = (++bcount << 16) | 0;
        { std::string s; app<uint32_t>(s, MPX_MSG_P_START); app<uint64_t>(s, ballot); g.to_leader(s); }
        Delivery pd{D_PREPARE, g.ep[e].version, ballot, 0, g.nd[0].next_apply, {}, {}};
        std::vector<uint32_t> order = acc;
        for (size_t i = order.size(); i > 1; --i) std::swap(order[i - 1], order[g.rng.below(i)]);
        uint32_t granted = 0;
        std::vector<uint32_t> missing;
        for (uint32_t n : order) { int r = g.send(n, pd, n != 0); if (r > 0) ++granted; else missing.push_back(n); }
        for (size_t k = 0; granted < Q && k < missing.size(); ++k) {     // PrepareRetryTimeout: re-send
            g.flush_all(missing[k]);
            if (g.process(missing[k], pd) > 0) ++granted;
        }
        if (granted < Q) return MPX_E_INVAL;    // cannot happen: every acceptor is in epoch e by now
        // ---- accept phase: in-flight instances first (same Values), then new ones
        const uint64_t end = start[e + 1];
        std::vector<uint64_t> todo(inflight.begin(), inflight.end());
        inflight.clear();
        while (next_new < end) todo.push_back(next_new++);
        const uint64_t mem_iid = e + 1 < g.E ? end - 1 : ~0ull;
        size_t pos = 0;
        bool changed = false;
        while (pos < todo.size() && !changed) {
            size_t take = 1 + g.rng.below(B);
            std::vector<uint64_t> ii, pp;
            for (size_t k = 0; k < take && pos < todo.size(); ++k) {
                ii.push_back(todo[pos++]);
                pp.push_back(ballot);
                if (ii.back() == mem_iid) break;   // the membership Value closes its batch
            }
            const uint64_t bid = ++batch_id;
            { std::string s, body = g.entries(ii, pp); app<uint32_t>(s, MPX_MSG_P_BATCH); app<uint64_t>(s, bid);
              app<uint32_t>(s, (uint32_t)body.size()); s += body; g.to_leader(s); }
            Delivery ad{D_ACCEPT, g.ep[e].version, ballot, bid, 0, ii, pp};
            for (size_t i = order.size(); i > 1; --i) std::swap(order[i - 1], order[g.rng.below(i)]);
            uint32_t votes = 0;
            missing.clear();
            for (uint32_t n : order) { int r = g.send(n, ad, n != 0); if (r > 0) ++votes; else missing.push_back(n); }
            for (size_t k = 0; votes < Q && k < missing.size(); ++k) {   // AcceptRetryTimeout
                g.flush_all(missing[k]);
                if (g.process(missing[k], ad) > 0) ++votes;
            }
            if (votes < Q) return MPX_E_INVAL;
            // chosen: LEARN to the learners, the leader first
            const bool has_mem = ii.back() == mem_iid;
            std::vector<Delivery> fly;
            if (has_mem) {
                // batches the leader created after the membership Value, before
                // applying it (AcceptRejected drops them at the change, :1322)
                // (instances of the next epoch's range, short of its membership Value)
                const uint64_t lim = e + 2 < g.E ? start[e + 2] - 1 : g.M;
                const size_t extra = g.rng.below(3);
                for (size_t x = 0; x < extra && next_new < lim; ++x) {
                    std::vector<uint64_t> fi, fp;
                    size_t t2 = 1 + g.rng.below(B);
                    for (size_t k = 0; k < t2 && next_new < lim; ++k) { fi.push_back(next_new++); fp.push_back(ballot); }
                    const uint64_t fb = ++batch_id;
                    std::string s, body = g.entries(fi, fp);
                    app<uint32_t>(s, MPX_MSG_P_BATCH); app<uint64_t>(s, fb); app<uint32_t>(s, (uint32_t)body.size());
                    s += body; g.to_leader(s);
                    fly.push_back(Delivery{D_ACCEPT, g.ep[e].version, ballot, fb, 0, fi, fp});
                    for (uint64_t i : fi) inflight.push_back(i);
                }
            }
            Delivery ld{D_LEARN, 0, 0, ++learn_id, 0, ii, pp};
            g.send(0, ld, false);
            // in-flight ACCEPTs: an acceptor gets them before its own LEARN of the
            // change (accepted under the old ballot) or after it (version dropped)
            for (const Delivery &fd : fly)
                for (uint32_t n : acc) {
                    if (n == 0 || g.rng.below(2)) g.send(n, fd, false);
                    else g.nd[n].later.push_front(Pending{g.nd[n].appended + 1, fd});
                }
            for (uint32_t n = 1; n < U; ++n) {
                if (!((learners >> n) & 1)) continue;
                if (g.send(n, ld, true) < 0) {                             // LearnRetryTimeout
                    Pending pe{g.nd[n].appended + 1 + g.rng.below(g.max_delay), ld};
                    auto &q = g.nd[n].later;
                    q.insert(std::upper_bound(q.begin(), q.end(), pe, [](const Pending &a, const Pending &b) { return a.due < b.due; }), pe);
                }
            }
            if (has_mem) {
                changed = true;
                const uint32_t c = e + 1;
                if (c < U) {
                    // LearnersChanged: the new learner gets every learned Value
                    learners |= 1ull << c;
                    std::vector<uint64_t> ci, cp;
                    for (uint64_t i = 0; i < g.nd[0].next_apply; ++i) { ci.push_back(i); cp.push_back(g.nd[0].learned_pid[i]); }
                    Delivery cd{D_LEARN, 0, 0, ++learn_id, 0, ci, cp};
                    g.send(c, cd, false);
                } else {
                    learners &= ~(1ull << (c - (U - 1)));
                }
                // every acceptor of the next epoch must have switched before the
                // new PREPARE: deliver what is still pending for them
                for (uint32_t n = 0; n < U; ++n)
                    if ((g.ep[c].acceptor_mask >> n) & 1) g.flush_all(n);
                for (size_t k = pos; k < todo.size(); ++k) inflight.push_back(todo[k]);
                std::sort(inflight.begin(), inflight.end());
            }
        }
    }
    for (uint32_t n = 0; n < U; ++n) g.flush_all(n);

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
