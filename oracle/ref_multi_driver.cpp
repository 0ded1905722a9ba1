// ref_multi_driver.cpp — drives the REFERENCE's own handlers.  TEST INFRASTRUCTURE ONLY.
//
// Built by oracle/Makefile into oracle/_ref/libmpx_ref.so, only where
// /root/reference exists (never on the GPU box; the built .so travels).
// The reference source is compiled where it lies: this translation unit
// #includes /root/reference/multi/paxos.cpp; nothing of it is copied here.
//
// Technique (SURVEY.md §4 "Driving the handlers single-threaded"):
//   * `private` is widened so the handlers (PaxosImpl::OnPrepare, OnAccept,
//     OnCommit, OnPrepareReply, OnAcceptReply, OnReject) can be called directly;
//   * pthread_create / pthread_join are wrapped (-Wl,--wrap) so PaxosImpl's
//     ctor does not start its event loop thread (multi/paxos.cpp:345);
//   * a frozen Clock, a capturing NetWork and a recording StateMachine
//     (the reference's own abstract interfaces, multi/paxos.h:193-222).
// The proposer control plane (out of scope) is held still: P_START / P_BATCH
// trace markers set the fields StartPrepare / Accept would set, and batches
// the reference's own decision code creates after a promise quorum are
// discarded (their sends are not in-scope replies either).  A P_PROPOSE marker
// calls the reference's own Propose, so its bookkeeping (value_id_,
// initial_proposals_, newly_proposed_values_) is the real one; the batch it may
// create is replaced by the trace's P_BATCH with the same accept id.
//
// Output: the canonical MPXR result, byte-comparable with
// oracle/mpx_oracle.c and the engine's mpx_dump_result.

#include <string.h>
#include <stdarg.h>
#include <time.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <stdlib.h>
#include <stdio.h>
#include <stdint.h>
#include <pthread.h>
#include <assert.h>
#include <set>
#include <map>
#include <list>
#include <deque>
#include <vector>
#include <string>
#include <algorithm>
#include <sstream>

#define private public
#define protected public
#include "/root/reference/multi/paxos.cpp"
#undef private
#undef protected

extern "C" {
int __wrap_pthread_create(pthread_t *t, const pthread_attr_t *, void *(*)(void *), void *)
{
    memset(t, 0, sizeof *t);   // the paxos thread never runs: handlers are driven directly
    return 0;
}
int __wrap_pthread_join(pthread_t, void **) { return 0; }
}

namespace {

typedef unsigned long long u64;

struct FrozenClock : public Clock {
    TimeStamp Now() { return 1000; }
};

struct Send { uint32_t dst; std::string bytes; };

struct CapNet : public paxos::NetWork {
    std::vector<Send> *out;
    void SendMessageTCP(const std::string &, unsigned short port, const std::string &msg) { out->push_back(Send{port, msg}); }
    void SendMessageUDP(const std::string &, unsigned short port, const std::string &msg) { out->push_back(Send{port, msg}); }
};

struct RecSM : public paxos::StateMachine {
    std::vector<std::string> executed;
    bool keep = true;                        // (digest runs only count: mpxref_run_shard)
    u64 n_exec = 0;
    void Execute(const std::string &v) { ++n_exec; if (keep) executed.push_back(v); }
};

struct NopCallback : public paxos::Callback { void Run() {} };
NopCallback g_nop;

u64 handle_of(const paxos::Value &v) { return ((u64)v.proposer_ << 48) | ((u64)(v.noop_ ? 1 : 0) << 47) | v.value_id_; }

template <typename T> void put(std::string &b, T v) { b.append((const char *)&v, sizeof v); }

uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
u64 rd64(const uint8_t *p) { u64 v; memcpy(&v, p, 8); return v; }

struct Node {
    paxos::PaxosImpl *impl;
    CapNet net;
    RecSM sm;
    std::vector<Send> sends;
    std::string events_q; u64 n_q = 0;
    std::string events_c; u64 n_c = 0;
    std::string events_d; u64 n_d = 0;                  // the reference's own phase-2 batch per promise quorum
    std::set<paxos::AcceptingID> marker_batches;       // created by P_BATCH markers
    std::map<paxos::AcceptingID, std::map<paxos::InstanceID, paxos::Value> > batch_values;
    u64 P = 0, A = 0, L = 0;
    // the reference's own CommittingValues bookkeeping (MPXC): per commit id
    // {created seq, kind (0 accept quorum, 1 promise quorum), accept id, retired seq, replied mask}
    std::vector<std::vector<u64> > commits;
};

}  // namespace

// Collect every Value of the trace whose initial proposer is `index`, so the
// proposer bookkeeping OnCommit asserts on (multi/paxos.cpp:1512-1513,1526-1537)
// holds: uncommitted_proposed_values_ is what Propose() would have filled.
static void scan_values(const uint8_t *m, size_t len, std::map<u64, paxos::Value> &vals, Logger *lg)
{
    uint32_t t = rd32(m);
    std::map<paxos::InstanceID, paxos::Value> iv;
    std::map<paxos::InstanceID, paxos::AcceptedValue> av;
    if ((t == 3 || t == 5) && len >= 28) paxos::ExtractInstanceValues(lg, (const char *)m + 28, rd32(m + 24), &iv);
    else if (t == 17 && len >= 16) paxos::ExtractInstanceValues(lg, (const char *)m + 16, rd32(m + 12), &iv);
    else if (t == 1 && len >= 20) paxos::ExtractAcceptedValues(lg, (const char *)m + 20, rd32(m + 16), &av);
    for (auto &e : iv) vals.insert(std::make_pair(handle_of(e.second), e.second));
    for (auto &e : av) vals.insert(std::make_pair(handle_of(e.second.value_), e.second.value_));
}


// mix64 / the digests of oracle/mpx_oracle.c dump() (counters + order-independent digests of a
// result, the engine's mpx_stats): shard runs sum them over instance shards
static u64 mix64(u64 x)
{
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    x ^= x >> 31; return x;
}

// One record with its entries outside [sb, se) removed (shard runs).  Entries are walked with the
// reference's own ExtractValue; the wire lists them iid-sorted (Fill* walks a std::map), so the
// shard's entries are one byte range and keeping that range is what Extract* -> erase -> Fill*
// would write; an unsorted list takes exactly that path.
static const uint8_t *shard_cut(const uint8_t *m, size_t len, u64 sb, u64 se, std::string &buf, Logger *lg)
{
    size_t lo = 0, vo = 0;
    bool pid = false;                            // AcceptedValues (iid, proposal id, Value)
    switch (rd32(m)) {
    case 1: lo = offsetof(paxos::PrepareReplyMsg, len_); vo = offsetof(paxos::PrepareReplyMsg, values_); pid = true; break;
    case 3: lo = offsetof(paxos::AcceptMsg, len_); vo = offsetof(paxos::AcceptMsg, values_); break;
    case 5: lo = offsetof(paxos::CommitMsg, len_); vo = offsetof(paxos::CommitMsg, values_); break;
    case 17: lo = 12; vo = 16; break;            // P_BATCH {u32 type, u64 accept id, u32 len, values}
    default: return m;
    }
    if (len < vo) return m;
    const char *v = (const char *)m + vo;
    const unsigned int vl = rd32(m + lo);
    unsigned int cur = 0, a = vl, b = vl;
    u64 prev = 0;
    bool sorted = true;
    while (cur != vl) {
        const unsigned int at = cur;
        const u64 iid = rd64((const uint8_t *)v + cur);
        if (at && iid <= prev) sorted = false;
        prev = iid;
        cur += pid ? 16 : 8;
        paxos::ExtractValue(v, cur);
        if (iid >= sb && a == vl) a = at;
        if (iid >= se && b == vl) b = at;
    }
    if (a > b) a = b;
    if (sorted && a == 0 && b == vl) return m;   // every entry in the shard
    buf.assign((const char *)m, vo);
    unsigned int nl = 0;
    if (sorted) {
        nl = b - a;
        buf.append(v + a, nl);
    } else if (pid) {
        std::map<paxos::InstanceID, paxos::AcceptedValue> x, keep;
        paxos::ExtractAcceptedValues(lg, v, vl, &x);
        keep.insert(x.lower_bound(sb), x.lower_bound(se));
        nl = paxos::CalcAcceptedValuesLength(&keep);
        buf.resize(vo + nl);
        paxos::FillAcceptedValues(&buf[vo], &keep);
    } else {
        std::map<paxos::InstanceID, paxos::Value> x, keep;
        paxos::ExtractInstanceValues(lg, v, vl, &x);
        keep.insert(x.lower_bound(sb), x.lower_bound(se));
        nl = paxos::CalcInstanceValuesLength(&keep);
        buf.resize(vo + nl);
        paxos::FillInstanceValues(&buf[vo], &keep);
    }
    memcpy(&buf[lo], &nl, 4);
    return (const uint8_t *)buf.data();
}

static int run_impl(const uint8_t *trace, uint64_t size, uint8_t **out, uint64_t *out_size, uint64_t *stats,
                    std::string *decisions, std::string *commits = NULL, u64 sb = 0, u64 se = ~0ull);

extern "C" int mpxref_run(const uint8_t *trace, uint64_t size, uint8_t **out, uint64_t *out_size, uint64_t *stats)
{
    return run_impl(trace, size, out, out_size, stats, NULL);
}

// The reference's own commit-reliability bookkeeping (MPXC):
// every CommittingValues each node created (multi/paxos.cpp:1184-1197,1416-1421),
// in id order, with the COMMIT_REPLY that retired it (OnCommitReply, :1625-1641)
// and its replied_ set as a mask (at retirement, or at the end of the trace).
extern "C" int mpxref_commits(const uint8_t *trace, uint64_t size, uint8_t **out, uint64_t *out_size)
{
    uint8_t *r = NULL;
    uint64_t rs = 0;
    std::string d;
    int rc = run_impl(trace, size, &r, &rs, NULL, NULL, &d);
    free(r);
    if (rc) return rc;
    *out = (uint8_t *)malloc(d.size() ? d.size() : 1);
    if (!*out) return -2;
    memcpy(*out, d.data(), d.size());
    *out_size = d.size();
    return 0;
}

// The reference's own phase-2 decisions (MPXD): per node, per
// promise quorum {u64 seq, u64 count, {u64 iid, u64 handle} * count}, the batch
// OnPrepareReply built with this driver's proposer bookkeeping (client proposals
// from P_PROPOSE markers: initial_proposals_ / newly_proposed_values_).
extern "C" int mpxref_decisions(const uint8_t *trace, uint64_t size, uint8_t **out, uint64_t *out_size)
{
    uint8_t *r = NULL;
    uint64_t rs = 0;
    std::string d;
    int rc = run_impl(trace, size, &r, &rs, NULL, &d);
    free(r);
    if (rc) return rc;
    *out = (uint8_t *)malloc(d.size() ? d.size() : 1);
    if (!*out) return -2;
    memcpy(*out, d.data(), d.size());
    *out_size = d.size();
    return 0;
}

static int run_impl(const uint8_t *trace, uint64_t size, uint8_t **out, uint64_t *out_size, uint64_t *stats,
                    std::string *decisions, std::string *commits, u64 sb, u64 se)
{
    // Instance shard [sb, se) (mpxref_run_shard, out == NULL): what one GPU rank ingests
    //  — every record's header is processed, the entries of
    // PREPARE_REPLY / ACCEPT / COMMIT / P_BATCH outside the shard are cut with the reference's
    // own codec (Extract* -> erase -> Calc* / Fill*); only counters and digests are kept.
    const bool shard = sb != 0 || se != ~0ull;
    const bool digest = out == NULL;
    if (size < 40 || memcmp(trace, "MPXT", 4)) return -4;
    uint32_t N = rd32(trace + 8), sem = rd32(trace + 12), ne = rd32(trace + 24);
    if (sem != 0 || N == 0 || N > 64) return -1;
    // Clock, Logger and Timer outlive this call on purpose: the leaked
    // PaxosImpl objects and the queued (never processed) retry timeouts point
    // into them, and ~Timer would ASSERT on the uncancelled commit retries.
    FrozenClock &clock = *new FrozenClock;
    Logger &logger = *new Logger(&clock, 7);   // above CRITICAL: silent (ASSERT still crashes)
    Timer &timer = *new Timer(&logger);
    Rand &rand = *new Rand(0);
    paxos::Paxos::Config cfg;
    paxos::NodeInfoMap nodes;
    for (uint32_t i = 0; i < N; ++i) nodes.insert(std::make_pair(i, paxos::NodeInfo("0.0.0.0", (unsigned short)i)));

    // locate node sections
    std::vector<const uint8_t *> offs(N), bytes(N);
    std::vector<u64> cnt(N);
    size_t pos = 40 + (size_t)ne * 24;
    for (uint32_t i = 0; i < N; ++i) {
        if (pos + 16 > size) return -4;
        cnt[i] = rd64(trace + pos);
        u64 nb = rd64(trace + pos + 8);
        pos += 16;
        offs[i] = trace + pos;
        bytes[i] = trace + pos + 8 * (cnt[i] + 1);
        pos += 8 * (cnt[i] + 1) + nb;
        pos = (pos + 7) & ~(size_t)7;
        if (pos > size + 7) return -4;
    }
    std::map<u64, paxos::Value> allvals;
    if (!shard)
        for (uint32_t i = 0; i < N; ++i)
            for (u64 k = 0; k < cnt[i]; ++k) {
                u64 a = rd64(offs[i] + 8 * k), b = rd64(offs[i] + 8 * k + 8);
                scan_values(bytes[i] + a, b - a, allvals, &logger);
            }

    std::vector<Node> ns(N);
    for (uint32_t i = 0; i < N; ++i) {
        Node &n = ns[i];
        n.net.out = &n.sends;
        n.sm.keep = !digest;
        n.impl = new paxos::PaxosImpl(&logger, "ref", &clock, &timer, &rand, nodes, i,
                                      &n.net, &n.sm, cfg, NULL);
        if (shard) {
            // the proposer's id sets start at the shard: instances below it are never committed
            // here, and a noop fill of [0, sb) at every promise quorum (:1117-1130) would only
            // build batches the driver discards (proposer-side, out of the digested state)
            n.impl->uncommitted_instance_ids_.ids_.clear();
            n.impl->uncommitted_instance_ids_.ids_.insert(std::make_pair((paxos::InstanceID)sb, (paxos::InstanceID)-1));
        }
        for (auto &v : allvals)
            if (v.second.proposer_ == i && !v.second.noop_)
                n.impl->uncommitted_proposed_values_.insert(
                    std::make_pair(v.second.value_id_, paxos::ProposedValue(v.second.value_, &g_nop)));
    }

    static paxos::PrepareRetryTimeout *dummy_prt = NULL;
    std::string cutbuf;
    for (uint32_t i = 0; i < N; ++i) {
        Node &n = ns[i];
        paxos::PaxosImpl *p = n.impl;
        if (!dummy_prt) dummy_prt = new paxos::PrepareRetryTimeout(p, 1000000);
        std::set<paxos::ValueID> registered;            // (shard runs: own Values seen at a COMMIT)
        for (u64 k = 0; k < cnt[i]; ++k) {
            u64 a = rd64(offs[i] + 8 * k), b = rd64(offs[i] + 8 * k + 8);
            const uint8_t *m = bytes[i] + a;
            if (shard) m = shard_cut(m, b - a, sb, se, cutbuf, &logger);
            uint32_t type = rd32(m);
            size_t before = n.sends.size();
            const paxos::CommittingID cid0 = p->committing_id_;
            u64 retire_id = 0, retire_mask = 0;
            if (type == 6) {               // OnCommitReply below: the commit it may retire
                const paxos::CommitReplyMsg *msg = (const paxos::CommitReplyMsg *)m;
                auto it = p->committing_values_.find(msg->commit_);
                if (it != p->committing_values_.end()) {
                    retire_id = msg->commit_;
                    for (unsigned int x : it->second->replied_) if (x < 64) retire_mask |= 1ull << x;
                    if (msg->learner_ < 64) retire_mask |= 1ull << msg->learner_;
                }
            }
            switch (type) {
            case 0: {
                // P: entries in a granted reply are counted from the reply itself below
                p->OnPrepare((const paxos::PrepareMsg *)m);
                break;
            }
            case 1: {
                const paxos::PrepareReplyMsg *msg = (const paxos::PrepareReplyMsg *)m;
                bool quorum_next = p->prepare_retry_timeout_ && msg->id_ == p->proposal_id_ &&
                    nodes.find(msg->acceptor_) != nodes.end() && [&] {
                        std::set<unsigned int> s = p->prepare_promised_;
                        s.insert(msg->acceptor_);
                        return s.size() >= nodes.size() / 2 + 1;
                    }();
                if (quorum_next && digest) {
                    // (digest runs: no snapshot or decision record; the re-commit of every committed
                    // value a promise quorum creates, :1184-1197, is proposer-side and would copy the
                    // whole committed map per quorum: it sees an empty map here)
                    std::map<paxos::InstanceID, paxos::AcceptedValue> held;
                    held.swap(p->committed_values_);
                    std::set<paxos::AcceptingID> before_b;
                    for (auto &e : p->accepting_values_) before_b.insert(e.first);
                    p->OnPrepareReply(msg);
                    held.swap(p->committed_values_);
                    for (auto it = p->accepting_values_.begin(); it != p->accepting_values_.end();) {
                        if (!before_b.count(it->first)) {
                            it->second->retry_timeout_->Cancel();
                            it = p->accepting_values_.erase(it);
                        } else ++it;
                    }
                } else if (quorum_next) {
                    // snapshot the merged map with the reference's own merge
                    std::map<paxos::InstanceID, paxos::AcceptedValue> saved = p->pre_accepted_values_;
                    std::map<paxos::InstanceID, paxos::AcceptedValue> vals;
                    paxos::ExtractAcceptedValues(&logger, msg->values_, msg->len_, &vals);
                    p->UpdateByPreAcceptedValues(&vals);
                    std::map<paxos::InstanceID, paxos::AcceptedValue> merged = p->pre_accepted_values_;
                    p->pre_accepted_values_ = saved;
                    put<u64>(n.events_q, k); put<u64>(n.events_q, p->proposal_id_);
                    put<u64>(n.events_q, merged.size());
                    for (auto &e : merged) {
                        put<u64>(n.events_q, e.first);
                        put<u64>(n.events_q, e.second.proposal_id_);
                        put<u64>(n.events_q, handle_of(e.second.value_));
                    }
                    n.n_q++;
                    std::set<paxos::AcceptingID> before_b;
                    for (auto &e : p->accepting_values_) before_b.insert(e.first);
                    p->OnPrepareReply(msg);
                    // record, then discard, what the reference's decision logic created
                    // (multi/paxos.cpp:1056-1182: adopt pre-accepted, noop gap fill, ...)
                    {
                        std::string d;
                        u64 cnt_d = 0;
                        for (auto &e : p->accepting_values_)
                            if (!before_b.count(e.first))
                                for (auto &v : e.second->values_) {
                                    put<u64>(d, v.first); put<u64>(d, handle_of(v.second)); ++cnt_d;
                                }
                        put<u64>(n.events_d, k); put<u64>(n.events_d, cnt_d); n.events_d += d;
                        n.n_d++;
                    }
                    for (auto it = p->accepting_values_.begin(); it != p->accepting_values_.end();) {
                        if (!before_b.count(it->first)) {
                            it->second->retry_timeout_->Cancel();
                            it = p->accepting_values_.erase(it);
                        } else ++it;
                    }
                } else {
                    p->OnPrepareReply(msg);
                }
                break;
            }
            case 2: p->OnReject((const paxos::RejectMsg *)m); break;
            case 3: {
                const paxos::AcceptMsg *msg = (const paxos::AcceptMsg *)m;
                if (msg->id_ >= p->promised_proposal_id_) {
                    std::map<paxos::InstanceID, paxos::Value> vals;
                    paxos::ExtractInstanceValues(&logger, msg->values_, msg->len_, &vals);
                    for (auto &e : vals) if (!p->committed_values_.count(e.first)) n.A++;
                }
                p->OnAccept(msg);
                break;
            }
            case 4: {
                const paxos::AcceptReplyMsg *msg = (const paxos::AcceptReplyMsg *)m;
                bool live = msg->id_ == p->proposal_id_ && p->accepting_values_.count(msg->accept_);
                p->OnAcceptReply(msg);
                if (live && !p->accepting_values_.count(msg->accept_)) {
                    put<u64>(n.events_c, k); put<u64>(n.events_c, msg->accept_);
                    n.n_c++;
                }
                break;
            }
            case 5: {
                const paxos::CommitMsg *msg = (const paxos::CommitMsg *)m;
                std::map<paxos::InstanceID, paxos::Value> vals;
                paxos::ExtractInstanceValues(&logger, msg->values_, msg->len_, &vals);
                n.L += vals.size();
                if (shard)   // the prefill, per shard: a node's own Value exists before its first COMMIT
                    for (auto &e : vals)
                        if (e.second.proposer_ == i && !e.second.noop_ && registered.insert(e.second.value_id_).second)
                            p->uncommitted_proposed_values_.insert(
                                std::make_pair(e.second.value_id_, paxos::ProposedValue(e.second.value_, &g_nop)));
                p->OnCommit(msg);
                break;
            }
            case 6: p->OnCommitReply((const paxos::CommitReplyMsg *)m); break;
            case 16: {         // P_START
                p->proposal_id_ = rd64(m + 4);
                p->prepare_promised_.clear();
                p->pre_accepted_values_.clear();
                for (auto &e : p->accepting_values_) e.second->retry_timeout_->Cancel();
                p->accepting_values_.clear();
                p->prepare_retry_timeout_ = dummy_prt;
                break;
            }
            case 19: {         // P_PROPOSE: the reference's own Propose (multi/paxos.cpp:1250-1280)
                // (shard runs skip it: Propose only moves the proposer's id bookkeeping, which
                // numbers instances across shards; the digested acceptor / learner state and the
                // chosen log come from the trace's P_BATCH / ACCEPT / COMMIT records)
                if (shard) break;
                const uint32_t pl = rd32(m + 4);
                p->Propose(paxos::ProposedValue(std::string((const char *)m + 8, pl), &g_nop));
                break;
            }
            case 17: {         // P_BATCH
                u64 bid = rd64(m + 4);
                paxos::AcceptingValues *acc = new paxos::AcceptingValues(&logger, bid);
                std::map<paxos::InstanceID, paxos::Value> vals;
                paxos::ExtractInstanceValues(&logger, (const char *)m + 16, rd32(m + 12), &vals);
                for (auto &e : vals) acc->AddValue(e.first, e.second);
                acc->retry_timeout_ = new paxos::AcceptRetryTimeout(p, acc, 1000000);
                p->accepting_values_[bid] = acc;
                n.marker_batches.insert(bid);
                n.batch_values[bid] = vals;
                break;
            }
            default: return -4;
            }
            if (digest) {                      // counters only: P from this record's PREPARE_REPLYs
                for (size_t j = before; j < n.sends.size(); ++j)
                    if (rd32((const uint8_t *)n.sends[j].bytes.data()) == 1) {
                        const paxos::PrepareReplyMsg *r = (const paxos::PrepareReplyMsg *)n.sends[j].bytes.data();
                        std::map<paxos::InstanceID, paxos::AcceptedValue> vals;
                        paxos::ExtractAcceptedValues(&logger, r->values_, r->len_, &vals);
                        n.P += vals.size();
                    }
                n.sends.clear();
                continue;
            }
            for (paxos::CommittingID id = cid0 + 1; id <= p->committing_id_; ++id) {
                const u64 acc = type == 4 ? ((const paxos::AcceptReplyMsg *)m)->accept_ : 0;
                n.commits.push_back(std::vector<u64>{k, type == 4 ? 0ull : 1ull, acc, ~0ull, 0});
            }
            if (retire_id && !p->committing_values_.count(retire_id) && retire_id <= n.commits.size()) {
                n.commits[retire_id - 1][3] = k;
                n.commits[retire_id - 1][4] = retire_mask;
            }
            // keep only the acceptor / learner replies (types 1,2,4,6)
            std::vector<Send> keep(n.sends.begin(), n.sends.begin() + before);
            for (size_t j = before; j < n.sends.size(); ++j) {
                uint32_t t = rd32((const uint8_t *)n.sends[j].bytes.data());
                if (t == 1 || t == 2 || t == 4 || t == 6) keep.push_back(n.sends[j]);
                if (t == 1) {
                    const paxos::PrepareReplyMsg *r = (const paxos::PrepareReplyMsg *)n.sends[j].bytes.data();
                    std::map<paxos::InstanceID, paxos::AcceptedValue> vals;
                    paxos::ExtractAcceptedValues(&logger, r->values_, r->len_, &vals);
                    n.P += vals.size();
                }
            }
            n.sends.swap(keep);
        }
    }

    if (digest) {
        // [C, P, A, L, V, chosen digest, state digest, scalar digest] as oracle/mpx_oracle.c dump()
        u64 P = 0, A = 0, L = 0, ds = 0, dsc = 0, dc = 0;
        std::map<u64, u64> chosen;
        for (uint32_t i = 0; i < N; ++i) {
            Node &n = ns[i];
            paxos::PaxosImpl *p = n.impl;
            dsc += mix64(mix64((u64)i * 0x9E3779B97F4A7C15ull ^ p->promised_proposal_id_) ^ p->max_proposal_id_);
            for (int pass = 0; pass < 2; ++pass)
                for (auto &e : pass ? p->committed_values_ : p->accepted_values_)
                    ds += mix64(mix64(mix64(e.first + (u64)i * 0x9E3779B97F4A7C15ull) ^ e.second.proposal_id_)
                                ^ (handle_of(e.second.value_) + (pass ? 2 : 1) * 0xD6E8FEB86659FD93ull));
            P += n.P; A += n.A; L += n.L;
            for (u64 k = 0; k < n.n_c; ++k) {
                u64 bid = rd64((const uint8_t *)n.events_c.data() + 16 * k + 8);
                for (auto &e : n.batch_values[bid])
                    if (chosen.insert(std::make_pair(e.first, handle_of(e.second))).second)
                        dc += mix64(mix64(e.first) ^ handle_of(e.second));
            }
        }
        stats[0] = chosen.size(); stats[1] = P; stats[2] = A; stats[3] = L; stats[4] = 0;
        stats[5] = dc; stats[6] = ds; stats[7] = dsc;
        return 0;
    }
    // canonical MPXR dump
    std::string r;
    r.append("MPXR", 4);
    put<uint32_t>(r, 1); put<uint32_t>(r, N); put<uint32_t>(r, 0);
    u64 P = 0, A = 0, L = 0;
    std::map<u64, u64> chosen;
    for (uint32_t i = 0; i < N; ++i) {
        Node &n = ns[i];
        paxos::PaxosImpl *p = n.impl;
        put<u64>(r, p->promised_proposal_id_);
        put<u64>(r, p->max_proposal_id_);
        std::map<u64, std::pair<u64, const paxos::AcceptedValue *> > st;
        for (auto &e : p->accepted_values_) st[e.first] = std::make_pair(1ull, &e.second);
        for (auto &e : p->committed_values_) st[e.first] = std::make_pair(2ull, &e.second);
        put<u64>(r, st.size());
        for (auto &e : st) {
            put<u64>(r, e.first); put<u64>(r, e.second.first);
            put<u64>(r, e.second.second->proposal_id_); put<u64>(r, handle_of(e.second.second->value_));
        }
        put<u64>(r, n.sends.size());
        for (auto &s : n.sends) { put<uint32_t>(r, s.dst); put<uint32_t>(r, (uint32_t)s.bytes.size()); r += s.bytes; }
        put<u64>(r, n.n_q); r += n.events_q;
        put<u64>(r, n.n_c); r += n.events_c;
        put<u64>(r, n.sm.executed.size());
        for (auto &s : n.sm.executed) { put<uint32_t>(r, (uint32_t)s.size()); r += s; }
        P += n.P; A += n.A; L += n.L;
        for (u64 k = 0; k < n.n_c; ++k) {
            u64 bid = rd64((const uint8_t *)n.events_c.data() + 16 * k + 8);
            for (auto &e : n.batch_values[bid]) chosen.insert(std::make_pair(e.first, handle_of(e.second)));
        }
    }
    put<u64>(r, chosen.size());
    for (auto &e : chosen) { put<u64>(r, e.first); put<u64>(r, e.second); }
    if (decisions) {
        decisions->append("MPXD", 4);
        put<uint32_t>(*decisions, 1); put<uint32_t>(*decisions, N);
        for (uint32_t i = 0; i < N; ++i) { put<u64>(*decisions, ns[i].n_d); *decisions += ns[i].events_d; }
    }
    if (commits) {
        commits->append("MPXC", 4);
        put<uint32_t>(*commits, 1); put<uint32_t>(*commits, N);
        for (uint32_t i = 0; i < N; ++i) {
            Node &n = ns[i];
            put<u64>(*commits, n.commits.size());
            for (size_t c = 0; c < n.commits.size(); ++c) {
                std::vector<u64> &x = n.commits[c];
                auto it = n.impl->committing_values_.find(c + 1);
                if (it != n.impl->committing_values_.end())
                    for (unsigned int y : it->second->replied_) if (y < 64) x[4] |= 1ull << y;
                put<u64>(*commits, c + 1);
                for (u64 w : x) put<u64>(*commits, w);
            }
        }
    }
    if (stats) { stats[0] = chosen.size(); stats[1] = P; stats[2] = A; stats[3] = L; }
    *out = (uint8_t *)malloc(r.size());
    if (!*out) return -2;
    memcpy(*out, r.data(), r.size());
    *out_size = r.size();
    // PaxosImpl objects are leaked on purpose: their dtor joins the (never
    // started) paxos thread and the timers hold raw pointers into them.
    return 0;
}

// Counters and digests of the instance shard [sb, se) of a trace, from the reference's own
// handlers (full-size parity per (node, instance shard)); stats = the 8
// words of oracle/mpx_oracle.c mpxo_run: C, P, A, L, violations (0: the reference would have
// crashed), chosen / state / scalar digests.  Counters and digests of disjoint shards add up;
// the scalar digest is the same on every shard.  oracle/ref_full_size.py runs the shards.
extern "C" int mpxref_run_shard(const uint8_t *trace, uint64_t size, uint64_t sb, uint64_t se, uint64_t *stats)
{
    if (!stats || se <= sb) return -3;
    return run_impl(trace, size, NULL, NULL, stats, NULL, NULL, sb, se);
}

// Timing entry for bench.py's cpu_baseline leg: apply `reps` passes of one
// node's stream through the reference handlers (fresh PaxosImpl per pass).
// Returns the number of records processed.
extern "C" int64_t mpxref_time_node(const uint8_t *trace, uint64_t size, uint32_t node, uint32_t reps)
{
    if (size < 40 || memcmp(trace, "MPXT", 4)) return -4;
    uint32_t N = rd32(trace + 8), ne = rd32(trace + 24);
    FrozenClock &clock = *new FrozenClock;
    Logger &logger = *new Logger(&clock, 7);
    Timer &timer = *new Timer(&logger);
    Rand &rand = *new Rand(0);
    paxos::Paxos::Config cfg;
    paxos::NodeInfoMap nodes;
    for (uint32_t i = 0; i < N; ++i) nodes.insert(std::make_pair(i, paxos::NodeInfo("0.0.0.0", (unsigned short)i)));
    size_t pos = 40 + (size_t)ne * 24;
    const uint8_t *offs = NULL, *bytes = NULL;
    u64 cnt = 0;
    for (uint32_t i = 0; i <= node && i < N; ++i) {
        cnt = rd64(trace + pos);
        u64 nb = rd64(trace + pos + 8);
        pos += 16;
        offs = trace + pos;
        bytes = trace + pos + 8 * (cnt + 1);
        pos += 8 * (cnt + 1) + nb;
        pos = (pos + 7) & ~(size_t)7;
    }
    int64_t done = 0;
    for (uint32_t r = 0; r < reps; ++r) {
        CapNet net;
        std::vector<Send> sends;
        sends.reserve(cnt);
        net.out = &sends;
        RecSM sm;
        paxos::PaxosImpl *p = new paxos::PaxosImpl(&logger, "ref", &clock, &timer, &rand, nodes, node, &net, &sm, cfg, NULL);
        for (u64 k = 0; k < cnt; ++k) {
            u64 a = rd64(offs + 8 * k);
            const uint8_t *m = bytes + a;
            switch (rd32(m)) {
            case 0: p->OnPrepare((const paxos::PrepareMsg *)m); break;
            case 2: p->OnReject((const paxos::RejectMsg *)m); break;
            case 3: p->OnAccept((const paxos::AcceptMsg *)m); break;
            case 5: p->OnCommit((const paxos::CommitMsg *)m); break;
            default: break;   // proposer-side records: this leg times the acceptor/learner path
            }
            ++done;
        }
        // the instance is dropped without its dtor (see mpxref_run)
        p->accepted_values_.clear();
        p->committed_values_.clear();
    }
    return done;
}
