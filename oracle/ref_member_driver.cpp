// ref_member_driver.cpp — drives the REFERENCE's own member handlers.  TEST INFRASTRUCTURE ONLY.
//
// Built by oracle/Makefile into oracle/_ref/libmpx_ref_member.so, only where
// /root/reference exists.  The reference source is compiled where it lies:
// this translation unit #includes /root/reference/member/paxos.cpp; nothing of
// it is copied here.
//
// Technique: `private` is widened; every node is a real
// NodeImpl whose Acceptor / Learner / Proposer objects are the reference's, and
// each record of the node's stream is dispatched exactly as NodeImpl::Loop does
// (member/paxos.cpp:749-790), single-threaded: NodeImpl::Init (which starts the
// paxos thread) is never called.  The abstract platform interfaces of indet.h
// (Thread, SpinLock, AtomicBool, Clock) get trivial single-thread
// implementations; NetWork::Send is captured, StateMachine::Apply recorded.
//
// Membership: the reference applies learned membership Values itself
// (Learner::Apply -> NodeImpl::ChangeMemberships, :1062-1073,1864-1964).  The
// trace's E_EPOCH markers are CHECKED against what it did: before every
// non-marker record the node's version_, acceptors_, proposer_ and acceptor_
// must equal the marker-driven epoch (else mpxref_member_run returns -11).
// Proposer control plane (out of scope) is held still as in the multi driver:
// P_START / P_BATCH set what StartPrepare / Accept would, a proposer that was
// created or saw its acceptor set change is made idle at the marker (the engine
// model, include/mpx.h), and batches / learns its own decision code creates are
// discarded (their sends are proposer broadcasts, not in-scope replies).
//
// Output: the canonical MPXR result; mpxref_member_decisions: the
// ACCEPT batch each promise quorum's OnPrepareReply built (MPXD, :1183-1297); mpxref_member_learns: the
// proposers' learn reliability bookkeeping as MPXL (include/mpx.h
// mpx_read_learns): every LearningValues a Proposer created (learning_id_, :1334-1337,
// 1299-1307, 1487-1491), the record where Applied ran for it (learning_values_for_
// acceptors_ reached |acceptors|/2+1, :1355-1370,1507-1533), where it retired (every
// learner replied, :1373-1380) or was dropped (LearnersChanged, :1472-1502, or the
// Proposer deleted, :1916-1942), and its learned_ set.  The reference's own objects are
// read after every record; Applied is attributed to its learn by tagging the cb_ of the
// values of every learn in learning_values_for_acceptors_ around the record.

#include <string.h>
#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <stdint.h>
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
#include "/root/reference/member/paxos.cpp"
#undef private
#undef protected

namespace {

typedef unsigned long long u64;

struct DLock : public SpinLock {
    void Lock(const Thread *) {}
    void Unlock() {}
};
struct DBool : public AtomicBool {
    explicit DBool(bool b) : AtomicBool(b) {}
    void Set(bool b, const Thread *) { b_ = b; }
    bool Get(const Thread *) { return b_; }
};
struct DThread : public Thread {
    DThread() : Thread(std::vector<ThreadID>(1, 0), "ref", "/tmp", Rand(0), 0) {}
    void USleep(unsigned long long) {}
    void Sleep(unsigned long long) {}
    SpinLock *NewSpinLock(const std::string &) { return new DLock; }
    AtomicBool *NewAtomicBool(bool b, const std::string &) { return new DBool(b); }
    Thread *NewThread(const std::vector<ThreadID> &, const std::string &, const std::string &, const Rand &,
                      unsigned long long) { return new DThread; }
    FILE *OpenClockLog(const std::string &) { return NULL; }
};
struct FrozenClock : public Clock {
    TimeStamp Now(const Thread *) { return 1000; }
};

struct Sent { uint32_t dst; std::string bytes; };

// Callback capture: Applied (the tags name the learn, see above) and, for the callback
// fixture (mpxref_member_callbacks), every Accepted / Applied / Unproposable call in order
struct CapCb : public paxos::Callback {
    std::vector<std::string> applied;
    std::vector<std::pair<int, std::string> > calls;     // {0 Accepted | 1 Applied | 2 Unproposable, cb}
    void Accepted(Thread *, const std::string &cb) { calls.push_back(std::make_pair(0, cb)); }
    void Applied(Thread *, const std::string &cb, const std::string *)
    {
        applied.push_back(cb);
        calls.push_back(std::make_pair(1, cb));
    }
    void Unproposable(Thread *, const std::string &cb) { calls.push_back(std::make_pair(2, cb)); }
};

struct LearnRec { u64 id, created, kind, src, applied, retired, ended, learned; };

struct CapNet : public paxos::NetWork {
    std::vector<Sent> *out;
    void Send(Thread *, paxos::NodeID node, const std::string &msg) { out->push_back(Sent{node, msg}); }
};
struct RecSM : public paxos::StateMachine {
    std::vector<std::string> executed;
    bool Apply(Thread *, const std::string &v, std::string *) { executed.push_back(v); return true; }
};

u64 handle_of(const paxos::Value &v) { return ((u64)v.proposer_ << 48) | ((u64)(v.noop_ ? 1 : 0) << 47) | v.value_id_; }

template <typename T> void put(std::string &b, T v) { b.append((const char *)&v, sizeof v); }
uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
u64 rd64(const uint8_t *p) { u64 v; memcpy(&v, p, 8); return v; }

struct Epoch { uint32_t version; u64 amask, pmask, lmask; };

typedef std::map<paxos::InstanceID, paxos::ProposalValue> PVMap;

struct Node {
    paxos::NodeImpl *impl;
    CapNet net;
    RecSM sm;
    std::vector<Sent> sends;
    std::string events_q; u64 n_q = 0;
    std::string events_c; u64 n_c = 0;
    std::map<paxos::AcceptingID, std::map<paxos::InstanceID, u64> > batch_values;
    uint32_t epoch = 0;
    u64 P = 0, A = 0, L = 0;
    std::string events_d; u64 n_d = 0;               // phase-2 decisions (MPXD)
    std::vector<LearnRec> lrec;                      // learn reliability (MPXL), creation order
    std::string events_b; u64 n_b = 0;               // the Callback calls (MPXB): {seq, kind, cb}
    std::map<paxos::LearningID, size_t> llive;       // the current Proposer's open learns
};

DThread *g_thread;
paxos::PrepareRetryTimeout *g_dummy_prt;

u64 set_mask(const std::set<paxos::NodeID> &s)
{
    u64 m = 0;
    for (paxos::NodeID x : s) if (x < 64) m |= 1ull << x;
    return m;
}

// reference node == marker-driven epoch?
bool consistent(const Node &n, uint32_t id, const Epoch &e)
{
    const paxos::NodeImpl *p = n.impl;
    return p->version_ == e.version && set_mask(p->acceptors_) == e.amask && set_mask(p->learners_) == e.lmask &&
           (p->acceptor_ != NULL) == (bool)((e.amask >> id) & 1) &&
           (p->proposer_ != NULL) == (bool)((e.pmask >> id) & 1);
}

// P_PROPOSE body -> the ProposedValue Node::Propose / AddAcceptor / ... hand to the Proposer
// (member/paxos.cpp:630-733): {u8 membership, u32 n, payload | n x {u32 node, u32 type},
// u32 cblen, cb}, the Value_m layout after proposer / value id / noop (:330-408)
bool proposed_value(const uint8_t *b, uint32_t len, paxos::ProposedValue &pv)
{
    if (len < 5) return false;
    const bool mem = b[0] != 0;
    const uint32_t n = rd32(b + 1);
    size_t pos = 5;
    if (mem) {
        if ((len - pos) / 8 < n) return false;
        pv.membership_changes_ = new std::vector<paxos::MembershipChange>();
        for (uint32_t k = 0; k < n; ++k)
            pv.membership_changes_->push_back(paxos::MembershipChange(rd32(b + pos + 8 * k),
                                                                      (paxos::MembershipChangeType)rd32(b + pos + 8 * k + 4)));
        pos += 8 * (size_t)n;
    } else {
        if (len - pos < n) return false;
        pv.membership_changes_ = NULL;
        pv.value_.assign((const char *)b + pos, n);
        pos += n;
    }
    if (len - pos < 4) return false;
    const uint32_t cl = rd32(b + pos);
    pos += 4;
    if (len - pos < cl) return false;
    pv.cb_.assign((const char *)b + pos, cl);
    return true;
}

void make_idle(paxos::Proposer *p)
{
    if (p->prepare_delay_) { p->prepare_delay_->Cancel(); p->prepare_delay_ = NULL; }
    if (p->prepare_retry_timeout_) { p->prepare_retry_timeout_->Cancel(); p->prepare_retry_timeout_ = NULL; }
    p->prepare_promised_.clear();
    p->pre_accepted_values_.clear();
    for (auto &e : p->accepting_values_) e.second->retry_timeout_->Cancel();
    p->accepting_values_.clear();
}

void discard_new_batches(paxos::Proposer *p, const std::set<paxos::AcceptingID> &before)
{
    if (!p) return;
    for (auto it = p->accepting_values_.begin(); it != p->accepting_values_.end();) {
        if (!before.count(it->first)) {
            it->second->retry_timeout_->Cancel();
            it = p->accepting_values_.erase(it);
        } else ++it;
    }
}

int parse_pvalues(Logger *lg, const uint8_t *buf, uint32_t len, PVMap *out)
{
    paxos::ExtractProposalValues(lg, g_thread, (const char *)buf, len, out);
    return 0;
}


// mix64 / the digests of oracle/mpx_oracle.c dump() (shard runs sum them)
u64 mix64(u64 x)
{
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    x ^= x >> 31; return x;
}

// One record with its entries outside [sb, se) removed (shard runs), walked with the reference's
// own ExtractValue; iid-sorted lists (FillProposalValues walks a std::map) keep one byte range,
// which is what ExtractProposalValues -> erase -> FillProposalValues writes; others take that path.
const uint8_t *shard_cut(const uint8_t *m, size_t len, u64 sb, u64 se, std::string &buf, Logger *lg)
{
    size_t lo = 0, vo = 0;
    switch (rd32(m)) {
    case 1: lo = offsetof(paxos::PrepareReplyMsg, len_); vo = offsetof(paxos::PrepareReplyMsg, values_); break;
    case 3: lo = offsetof(paxos::AcceptMsg, len_); vo = offsetof(paxos::AcceptMsg, values_); break;
    case 5: lo = offsetof(paxos::LearnMsg, len_); vo = offsetof(paxos::LearnMsg, values_); break;
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
        cur += 16;
        paxos::ExtractValue(v, cur);
        if (iid >= sb && a == vl) a = at;
        if (iid >= se && b == vl) b = at;
    }
    if (a > b) a = b;
    if (sorted && a == 0 && b == vl) return m;
    buf.assign((const char *)m, vo);
    unsigned int nl = 0;
    if (sorted) {
        nl = b - a;
        buf.append(v + a, nl);
    } else {
        PVMap x, keep;
        paxos::ExtractProposalValues(lg, g_thread, v, vl, &x);
        keep.insert(x.lower_bound(sb), x.lower_bound(se));
        nl = paxos::CalcProposalValuesLength(keep);
        buf.resize(vo + nl);
        paxos::FillProposalValues(&buf[vo], keep);
    }
    memcpy(&buf[lo], &nl, 4);
    return (const uint8_t *)buf.data();
}

// The change list of a membership step from one epoch to the next (shard runs: the learned
// membership Values are applied by the marker, see member_run), in the order the reference's own
// lists use (Node::AddAcceptor / DelAcceptor ..., member/paxos.cpp:635-721): gains, then losses
std::vector<paxos::MembershipChange> epoch_changes(const Epoch &o, const Epoch &x)
{
    std::vector<paxos::MembershipChange> ch;
    for (uint32_t j = 0; j < 64; ++j) {
        const u64 b = 1ull << j;
        if ((x.lmask & b) && !(o.lmask & b)) ch.push_back(paxos::MembershipChange(j, paxos::ADD_LEARNER));
        if ((x.pmask & b) && !(o.pmask & b)) ch.push_back(paxos::MembershipChange(j, paxos::LEARNER_TO_PROPOSER));
        if ((x.amask & b) && !(o.amask & b)) ch.push_back(paxos::MembershipChange(j, paxos::PROPOSER_TO_ACCEPTOR));
    }
    for (uint32_t j = 0; j < 64; ++j) {
        const u64 b = 1ull << j;
        if ((o.amask & b) && !(x.amask & b)) ch.push_back(paxos::MembershipChange(j, paxos::ACCEPTOR_TO_PROPOSER));
        if ((o.pmask & b) && !(x.pmask & b)) ch.push_back(paxos::MembershipChange(j, paxos::PROPOSER_TO_LEARNER));
        if ((o.lmask & b) && !(x.lmask & b)) ch.push_back(paxos::MembershipChange(j, paxos::DEL_LEARNER));
    }
    return ch;
}

}  // namespace

static int member_run(const uint8_t *trace, uint64_t size, uint8_t **out, uint64_t *out_size,
                      uint64_t *stats, uint8_t **lout, uint64_t *lsize, uint8_t **dout = NULL, uint64_t *dsize = NULL,
                      u64 sb = 0, u64 se = ~0ull, bool digest = false, uint8_t **bout = NULL, uint64_t *bsize = NULL)
{
    // digest (mpxref_member_run_shard): counters and digests of the instance shard [sb, se) only
    // (SURVEY.md §8(c)(ii)).  Every record's header is processed; entries outside the shard are cut
    // with the reference's own codec.  A shard never learns the instances below it, so its Learner
    // would never apply a membership Value (Learner::Apply runs in instance order, :1042-1053): here
    // nothing is applied (next_id_to_apply_ parked) and each E_EPOCH marker — which whole runs
    // CHECK against what Apply did, at the record after the LEARN that applied it — calls the
    // reference's own NodeImpl::ChangeMemberships with that step's change list.  The consistency
    // check below still holds the node to the marker's epoch before every record.
    if (size < 40 || memcmp(trace, "MPXT", 4)) return -4;
    uint32_t N = rd32(trace + 8), sem = rd32(trace + 12), ne = rd32(trace + 24);
    if (sem != 1 || N == 0 || N > 64 || ne == 0) return -1;
    std::vector<Epoch> ep(ne);
    const size_t esz = rd32(trace + 4) == 1 ? 24 : 32;    // container version 2: + learner_mask
    for (uint32_t e = 0; e < ne; ++e) {
        ep[e].version = rd32(trace + 40 + esz * e);
        ep[e].amask = rd64(trace + 48 + esz * e);
        ep[e].pmask = rd64(trace + 56 + esz * e);
        ep[e].lmask = esz == 32 ? rd64(trace + 64 + esz * e) : ep[e].pmask;
    }
    // the reference starts every node in {first} (NodeImpl::Loop, :738-747)
    if (ep[0].amask == 0 || (ep[0].amask & (ep[0].amask - 1)) || ep[0].pmask != ep[0].amask || ep[0].version != 0)
        return -1;
    const uint32_t first = (uint32_t)__builtin_ctzll(ep[0].amask);

    // Platform objects outlive the call on purpose (the leaked NodeImpls and
    // their queued timeouts point into them), like the multi driver.
    if (!g_thread) g_thread = new DThread;
    FrozenClock &clock = *new FrozenClock;
    Logger &logger = *new Logger(new DLock, &clock, 7);   // above CRITICAL: silent (ASSERT still crashes)
    Timer &timer = *new Timer(&logger);
    Rand &rand = *new Rand(0);
    CapCb &cb = *new CapCb;
    paxos::Config cfg;

    std::vector<const uint8_t *> offs(N), bytes(N);
    std::vector<u64> cnt(N);
    size_t pos = 40 + (size_t)ne * esz;
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

    std::vector<Node> ns(N);
    for (uint32_t i = 0; i < N; ++i) {
        Node &n = ns[i];
        n.net.out = &n.sends;
        n.impl = new paxos::NodeImpl(g_thread, i, first, &logger, &clock, &timer, &rand, &cb, &n.net, &n.sm, cfg);
        n.impl->thread_ = g_thread;
        n.net.node_ = n.impl;
        // NodeImpl::Loop prologue (:738-747)
        paxos::NodeImpl *p = n.impl;
        p->learners_.insert(first);
        p->proposers_.insert(first);
        p->acceptors_.insert(first);
        if (first == i) {
            p->proposer_ = new paxos::Proposer(p);
            p->acceptor_ = new paxos::Acceptor(p);
            make_idle(p->proposer_);     // the engine model: idle until P_START
        }
        if (digest) p->learner_.next_id_to_apply_ = ~0ull;
    }
    if (!g_dummy_prt) g_dummy_prt = new paxos::PrepareRetryTimeout(NULL, 1000000);

    std::string cutbuf;
    for (uint32_t i = 0; i < N; ++i) {
        Node &n = ns[i];
        paxos::NodeImpl *ni = n.impl;
        paxos::Proposer *shard_prop = NULL;              // (digest: the Proposer whose id sets start at sb)
        for (u64 k = 0; k < cnt[i]; ++k) {
            u64 a = rd64(offs[i] + 8 * k), b = rd64(offs[i] + 8 * k + 8);
            const uint8_t *m = bytes[i] + a;
            if (b - a < 4) return -4;
            if (digest) {
                m = shard_cut(m, b - a, sb, se, cutbuf, &logger);
                if (ni->proposer_ && ni->proposer_ != shard_prop) {
                    // a new Proposer's unlearned ids (:552, [0, 2^64-1)) start at the shard: ids
                    // below it are never learned here, and a noop fill of [0, sb) at every promise
                    // quorum would only build batches the driver discards (proposer-side)
                    shard_prop = ni->proposer_;
                    shard_prop->unlearned_instance_ids_.ids_.clear();
                    shard_prop->unlearned_instance_ids_.ids_.insert(std::make_pair((paxos::InstanceID)sb, (paxos::InstanceID)-1));
                }
            }
            uint32_t type = rd32(m);
            if (type != 18 && !consistent(n, i, ep[n.epoch])) return -11;   // an E_EPOCH marker is missing
            size_t before = n.sends.size();
            paxos::Proposer *pr = ni->proposer_;
            // learn bookkeeping: tag the learns Applied may run for, note the id counter
            const paxos::LearningID lid0 = pr ? pr->learning_id_ : 0;
            std::map<std::string, std::string> orig_cb;      // tag -> the value's own cb
            std::map<paxos::LearningID, u64> prev_mask;
            if (pr && !digest) {
                for (auto &f : pr->learning_values_for_acceptors_) {
                    auto it = pr->learning_values_.find(f.first);
                    if (it == pr->learning_values_.end()) continue;
                    for (auto &v : it->second->values_) {
                        const std::string tag = "\x01" + std::to_string(f.first) + "." + std::to_string(v.first);
                        orig_cb[tag] = v.second.value_.cb_;
                        v.second.value_.cb_ = tag;
                    }
                }
                for (auto &l : pr->learning_values_) prev_mask[l.first] = set_mask(l.second->learned_);
            }
            cb.applied.clear();
            cb.calls.clear();
            std::set<paxos::AcceptingID> before_b;
            if (pr) for (auto &e : pr->accepting_values_) before_b.insert(e.first);
            switch (type) {
            case 0:
                if (ni->acceptor_) ni->acceptor_->OnPrepare((const paxos::PrepareMsg *)m);
                break;
            case 1: {
                if (!pr) break;
                const paxos::PrepareReplyMsg *msg = (const paxos::PrepareReplyMsg *)m;
                bool live = pr->prepare_retry_timeout_ && msg->id_ == pr->proposal_id_;
                bool quorum_next = !digest && live && [&] {
                    std::set<paxos::NodeID> s = pr->prepare_promised_;
                    s.insert(msg->acceptor_);
                    return s.size() >= ni->acceptors_.size() / 2 + 1;
                }();
                if (quorum_next) {
                    // snapshot the merged map with the reference's own merge
                    PVMap saved(pr->pre_accepted_values_);
                    PVMap vals;
                    parse_pvalues(&logger, (const uint8_t *)msg->values_, msg->len_, &vals);
                    pr->UpdateByPreAcceptedValues(vals);
                    put<u64>(n.events_q, k); put<u64>(n.events_q, pr->proposal_id_);
                    put<u64>(n.events_q, pr->pre_accepted_values_.size());
                    for (auto &e : pr->pre_accepted_values_) {
                        put<u64>(n.events_q, e.first);
                        put<u64>(n.events_q, e.second.proposal_id_);
                        put<u64>(n.events_q, handle_of(e.second.value_));
                    }
                    n.n_q++;
                    pr->pre_accepted_values_.swap(saved);
                }
                pr->OnPrepareReply(msg);
                if (quorum_next) {
                    // the phase-2 batch the reference's decision logic built (:1183-1297:
                    // adopt pre-accepted, noop gap fill, own initial / queued values)
                    std::string d;
                    u64 cnt_d = 0;
                    for (auto &e : pr->accepting_values_)
                        if (!before_b.count(e.first))
                            for (auto &v : e.second->values_) {
                                put<u64>(d, v.first); put<u64>(d, handle_of(v.second.value_)); ++cnt_d;
                            }
                    put<u64>(n.events_d, k); put<u64>(n.events_d, cnt_d); n.events_d += d;
                    n.n_d++;
                }
                discard_new_batches(pr, before_b);
                break;
            }
            case 2:
                if (pr) pr->OnReject((const paxos::RejectMsg *)m);
                break;
            case 3: {
                paxos::Acceptor *ac = ni->acceptor_;
                if (!ac) break;
                const paxos::AcceptMsg *msg = (const paxos::AcceptMsg *)m;
                if (msg->version_ == ni->version_ && msg->id_ >= ac->promised_proposal_id_) {
                    PVMap vals;
                    parse_pvalues(&logger, (const uint8_t *)msg->values_, msg->len_, &vals);
                    const PVMap &learned = ni->learner_.learned_values_;
                    for (auto &e : vals)
                        if (!learned.count(e.first) && !ac->accepted_values_.count(e.first)) n.A++;
                }
                ac->OnAccept(msg);
                break;
            }
            case 4: {
                if (!pr) break;
                const paxos::AcceptReplyMsg *msg = (const paxos::AcceptReplyMsg *)m;
                bool live = pr->accepting_values_.count(msg->accept_) != 0;
                pr->OnAcceptReply(msg);
                if (live && !pr->accepting_values_.count(msg->accept_)) {
                    put<u64>(n.events_c, k); put<u64>(n.events_c, msg->accept_);
                    n.n_c++;
                }
                break;
            }
            case 5: {
                const paxos::LearnMsg *msg = (const paxos::LearnMsg *)m;
                PVMap lv;
                parse_pvalues(&logger, (const uint8_t *)msg->values_, msg->len_, &lv);
                n.L += lv.size();
                if (digest && pr) {
                    // (digest runs do not replay Propose: a node's own Value is registered as
                    // proposed at the instance it is first learned at, which is all Proposer::OnLearn
                    // asks of it, :1398-1425 — proposer-side bookkeeping, out of the digested state)
                    const PVMap &learned = ni->learner_.learned_values_;
                    for (auto &e : lv) {
                        const paxos::Value &x = e.second.value_;
                        if (x.proposer_ != i || x.noop_ || learned.count(e.first) ||
                            pr->unlearned_proposed_values_.count(x.value_id_))
                            continue;
                        paxos::ProposedValue pv;
                        if (x.membership_changes_) pv.membership_changes_ = new std::vector<paxos::MembershipChange>(*x.membership_changes_);
                        pv.value_ = x.value_;
                        pv.cb_ = x.cb_;
                        pr->unlearned_proposed_values_.insert(std::make_pair(x.value_id_, pv));
                        pr->initial_proposals_.insert(std::make_pair(e.first, x.value_id_));
                    }
                }
                ni->learner_.OnLearn(msg);
                discard_new_batches(ni->proposer_ == pr ? pr : NULL, before_b);
                break;
            }
            case 6:
                if (pr) pr->OnLearnReply((const paxos::LearnReplyMsg *)m);
                break;
            case 16:       // P_START
                if (pr) {
                    make_idle(pr);
                    pr->proposal_id_ = rd64(m + 4);
                    pr->prepare_retry_timeout_ = g_dummy_prt;
                }
                break;
            case 17: {     // P_BATCH
                if (!pr) break;
                u64 bid = rd64(m + 4);
                PVMap vals;
                parse_pvalues(&logger, m + 16, rd32(m + 12), &vals);
                paxos::AcceptingValues *acc = new paxos::AcceptingValues(bid, vals);
                acc->retry_timeout_ = new paxos::AcceptRetryTimeout(pr, acc, 1000000);
                pr->accepting_values_[bid] = acc;
                for (auto &e : vals) n.batch_values[bid][e.first] = handle_of(e.second.value_);
                break;
            }
            case 18: {     // E_EPOCH
                uint32_t e = rd32(m + 4);
                if (e >= ne) return -4;
                const Epoch &o = ep[n.epoch], &x = ep[e];
                if (digest) ni->ChangeMemberships(epoch_changes(o, x));
                bool was = (o.pmask >> i) & 1, now = (x.pmask >> i) & 1;
                n.epoch = e;
                if (now && ni->proposer_ && (!was || o.amask != x.amask)) make_idle(ni->proposer_);
                break;
            }
            case 19: {     // P_PROPOSE: the reference's own Propose (Node::Propose -> :1122-1156)
                const uint32_t pl = rd32(m + 4);
                if (b - a < 8 + (u64)pl) return -4;
                paxos::ProposedValue pv;
                if (!proposed_value(m + 8, pl, pv)) return -4;
                // (digest runs skip it: Propose only moves the proposer's id bookkeeping, which
                // numbers instances across shards; the digested state and the chosen log come from
                // the trace's P_BATCH / ACCEPT / LEARN records)
                if (pr && !digest) pr->Propose(pv);
                else if (!pr && !digest) cb.Unproposable(g_thread, pv.cb_);    // NodeImpl::Loop, :784-787
                discard_new_batches(pr, before_b);       // the trace's P_BATCH is the batch
                break;
            }
            default: return -4;
            }
            if (digest) {                      // counters only: P from this record's PREPARE_REPLYs
                for (size_t j = before; j < n.sends.size(); ++j)
                    if (rd32((const uint8_t *)n.sends[j].bytes.data()) == 1) {
                        const paxos::PrepareReplyMsg *r = (const paxos::PrepareReplyMsg *)n.sends[j].bytes.data();
                        PVMap vals;
                        parse_pvalues(&logger, (const uint8_t *)r->values_, r->len_, &vals);
                        n.P += vals.size();
                    }
                n.sends.clear();
                continue;
            }
            {
                paxos::Proposer *p1 = ni->proposer_;
                if (pr && p1 == pr)                    // untag (learns built from tagged copies too)
                    for (auto &l : pr->learning_values_)
                        for (auto &v : l.second->values_)
                            if (!v.second.value_.cb_.empty() && v.second.value_.cb_[0] == '\x01')
                                v.second.value_.cb_ = orig_cb[v.second.value_.cb_];
                for (auto &c : cb.calls) {             // the fixture: every call, Applied untagged
                    std::string x = c.second;
                    if (c.first == 1 && !x.empty() && x[0] == '\x01') {
                        auto o = orig_cb.find(x);
                        if (o == orig_cb.end()) return -12;
                        x = o->second;
                    }
                    put<u64>(n.events_b, k); put<u64>(n.events_b, (u64)c.first);
                    put<uint32_t>(n.events_b, (uint32_t)x.size()); n.events_b += x;
                    n.n_b++;
                }
                for (auto &a : cb.applied) {
                    if (a.empty() || a[0] != '\x01') continue;
                    auto it = n.llive.find(std::stoull(a.substr(1)));
                    if (it != n.llive.end() && n.lrec[it->second].applied == ~0ull) n.lrec[it->second].applied = k;
                }
                if (pr && p1 != pr) {                  // the Proposer was deleted: its open learns end
                    for (auto &l : n.llive) n.lrec[l.second].ended = k;
                    n.llive.clear();
                }
                if (p1) {
                    const paxos::LearningID base = p1 == pr ? lid0 : 0;
                    const u64 kind = type == 4 ? 0 : type == 1 ? 1 : 2;
                    const u64 src = type == 4 ? ((const paxos::AcceptReplyMsg *)m)->accept_ : 0;
                    for (paxos::LearningID id = base + 1; id <= p1->learning_id_; ++id) {
                        n.llive[id] = n.lrec.size();
                        n.lrec.push_back(LearnRec{id, k, kind, src, ~0ull, ~0ull, ~0ull, 0});
                    }
                    for (auto it = n.llive.begin(); it != n.llive.end();) {
                        LearnRec &r = n.lrec[it->second];
                        auto lv = p1->learning_values_.find(it->first);
                        if (lv != p1->learning_values_.end()) {
                            r.learned = set_mask(lv->second->learned_);
                            ++it;
                            continue;
                        }
                        if (type == 6) {                   // OnLearnReply: every learner replied
                            r.retired = k;
                            r.learned = prev_mask[it->first] | (1ull << ((const paxos::LearnReplyMsg *)m)->learner_);
                        } else r.ended = k;                // LearnersChanged dropped it
                        it = n.llive.erase(it);
                    }
                }
            }
            // keep only the acceptor / learner replies (types 1,2,4,6)
            std::vector<Sent> keep(n.sends.begin(), n.sends.begin() + before);
            for (size_t j = before; j < n.sends.size(); ++j) {
                uint32_t t = rd32((const uint8_t *)n.sends[j].bytes.data());
                if (t == 1 || t == 2 || t == 4 || t == 6) keep.push_back(n.sends[j]);
                if (t == 1) {
                    const paxos::PrepareReplyMsg *r = (const paxos::PrepareReplyMsg *)n.sends[j].bytes.data();
                    PVMap vals;
                    parse_pvalues(&logger, (const uint8_t *)r->values_, r->len_, &vals);
                    n.P += vals.size();
                }
            }
            n.sends.swap(keep);
        }
        if (!consistent(n, i, ep[n.epoch])) return -11;
    }

    if (digest) {
        // [C, P, A, L, V, chosen digest, state digest, scalar digest] as oracle/mpx_oracle.c dump()
        u64 P = 0, A = 0, L = 0, ds = 0, dsc = 0, dc = 0;
        std::map<u64, u64> chosen;
        for (uint32_t i = 0; i < N; ++i) {
            Node &n = ns[i];
            paxos::NodeImpl *ni = n.impl;
            paxos::Acceptor *ac = ni->acceptor_;
            dsc += mix64(mix64((u64)i * 0x9E3779B97F4A7C15ull ^ (ac ? ac->promised_proposal_id_ : 0)) ^
                         (ac ? ac->max_proposal_id_ : 0));
            for (int pass = 0; pass < 2; ++pass) {
                if (!pass && !ac) continue;
                for (auto &e : pass ? ni->learner_.learned_values_ : ac->accepted_values_)
                    ds += mix64(mix64(mix64(e.first + (u64)i * 0x9E3779B97F4A7C15ull) ^ e.second.proposal_id_)
                                ^ (handle_of(e.second.value_) + (pass ? 2 : 1) * 0xD6E8FEB86659FD93ull));
            }
            P += n.P; A += n.A; L += n.L;
            for (u64 k = 0; k < n.n_c; ++k) {
                u64 bid = rd64((const uint8_t *)n.events_c.data() + 16 * k + 8);
                for (auto &e : n.batch_values[bid])
                    if (chosen.insert(e).second) dc += mix64(mix64(e.first) ^ e.second);
            }
        }
        stats[0] = chosen.size(); stats[1] = P; stats[2] = A; stats[3] = L; stats[4] = 0;
        stats[5] = dc; stats[6] = ds; stats[7] = dsc;
        return 0;
    }
    // canonical MPXR dump
    std::string r;
    r.append("MPXR", 4);
    put<uint32_t>(r, 1); put<uint32_t>(r, N); put<uint32_t>(r, 1);
    u64 P = 0, A = 0, L = 0;
    std::map<u64, u64> chosen;
    for (uint32_t i = 0; i < N; ++i) {
        Node &n = ns[i];
        paxos::NodeImpl *ni = n.impl;
        paxos::Acceptor *ac = ni->acceptor_;
        put<u64>(r, ac ? ac->promised_proposal_id_ : 0);
        put<u64>(r, ac ? ac->max_proposal_id_ : 0);
        std::map<u64, std::pair<u64, const paxos::ProposalValue *> > st;
        if (ac) for (auto &e : ac->accepted_values_) st[e.first] = std::make_pair(1ull, &e.second);
        for (auto &e : ni->learner_.learned_values_) st[e.first] = std::make_pair(2ull, &e.second);
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
            for (auto &e : n.batch_values[bid]) chosen.insert(e);
        }
    }
    put<u64>(r, chosen.size());
    for (auto &e : chosen) { put<u64>(r, e.first); put<u64>(r, e.second); }
    if (stats) { stats[0] = chosen.size(); stats[1] = P; stats[2] = A; stats[3] = L; }
    if (out) {
        *out = (uint8_t *)malloc(r.size());
        if (!*out) return -2;
        memcpy(*out, r.data(), r.size());
        *out_size = r.size();
    }
    if (dout) {
        std::string d;
        d.append("MPXD", 4);
        put<uint32_t>(d, 1); put<uint32_t>(d, N);
        for (uint32_t i = 0; i < N; ++i) { put<u64>(d, ns[i].n_d); d += ns[i].events_d; }
        *dout = (uint8_t *)malloc(d.size());
        if (!*dout) return -2;
        memcpy(*dout, d.data(), d.size());
        *dsize = d.size();
    }
    if (bout) {
        std::string b;
        b.append("MPXB", 4);
        put<uint32_t>(b, 1); put<uint32_t>(b, N);
        for (uint32_t i = 0; i < N; ++i) { put<u64>(b, ns[i].n_b); b += ns[i].events_b; }
        *bout = (uint8_t *)malloc(b.size());
        if (!*bout) return -2;
        memcpy(*bout, b.data(), b.size());
        *bsize = b.size();
    }
    if (lout) {
        std::string l;
        l.append("MPXL", 4);
        put<uint32_t>(l, 1); put<uint32_t>(l, N);
        for (uint32_t i = 0; i < N; ++i) {
            put<u64>(l, ns[i].lrec.size());
            for (auto &x : ns[i].lrec) {
                put<u64>(l, x.id); put<u64>(l, x.created); put<u64>(l, x.kind); put<u64>(l, x.src);
                put<u64>(l, x.applied); put<u64>(l, x.retired); put<u64>(l, x.ended); put<u64>(l, x.learned);
            }
        }
        *lout = (uint8_t *)malloc(l.size());
        if (!*lout) return -2;
        memcpy(*lout, l.data(), l.size());
        *lsize = l.size();
    }
    // NodeImpl objects are leaked on purpose (their dtors expect a joined thread).
    return 0;
}

extern "C" int mpxref_member_run(const uint8_t *trace, uint64_t size, uint8_t **out, uint64_t *out_size,
                                 uint64_t *stats)
{
    return member_run(trace, size, out, out_size, stats, NULL, NULL);
}

// Counters and digests of the instance shard [sb, se) of a member trace (the 8 words of
// mpxo_run; see member_run), for full-size parity per instance shard (oracle/ref_full_size.py).
extern "C" int mpxref_member_run_shard(const uint8_t *trace, uint64_t size, uint64_t sb, uint64_t se, uint64_t *stats)
{
    if (!stats || se <= sb) return -3;
    return member_run(trace, size, NULL, NULL, stats, NULL, NULL, NULL, NULL, sb, se, true);
}

extern "C" int mpxref_member_learns(const uint8_t *trace, uint64_t size, uint8_t **out, uint64_t *out_size)
{
    return member_run(trace, size, NULL, NULL, NULL, out, out_size);
}

// Every Callback call the reference's nodes made (MPXB): per node u64 count, {u64 record, u64 kind
// (0 Accepted :1332, 1 Applied :1368,1526, 2 Unproposable :787), u32 len, cb bytes} in call order
extern "C" int mpxref_member_callbacks(const uint8_t *trace, uint64_t size, uint8_t **out, uint64_t *out_size)
{
    return member_run(trace, size, NULL, NULL, NULL, NULL, NULL, NULL, NULL, 0, ~0ull, false, out, out_size);
}

extern "C" int mpxref_member_decisions(const uint8_t *trace, uint64_t size, uint8_t **out, uint64_t *out_size)
{
    return member_run(trace, size, NULL, NULL, NULL, NULL, NULL, out, out_size);
}
