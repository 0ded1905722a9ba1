// member_host.cpp — the reference's own member host hooks bound to libmpx.so.
//
// A member host talks to its node through paxos::NetWork (member/paxos.h:173-190: Send out,
// OnReceive in), paxos::StateMachine (:166-171: Apply in instance order) and paxos::Callback
// (:142-164: Accepted when a batch reaches its accept quorum, Applied when an acceptor quorum
// learned it, Unproposable).  Here those classes come from the reference's own header, and the
// node core behind them is the engine:
//   * EngineNetWork::Receive batches what NetWork::OnReceive would hand to the node
//     (member/paxos.cpp:841-844) and gives it to mpx_submit — the messages only: no E_EPOCH
//     markers, no epoch table beyond the genesis one.  The engine is created with
//     MPX_FLAG_LEARN_EPOCHS and applies the membership Values its Learners apply itself
//     (Learner::Apply -> NodeImpl::ChangeMemberships, :1062-1073,1864-1964), so the roles, the
//     version gates and the quorums follow the membership the node discovers at run time;
//   * mpx_drain_sends calls back into EngineNetWork::Send with the destination node (the
//     acceptors' / learners' replies, :1700-1793,1029-1060);
//   * the executed Values (mpx_read_executed + mpx_value_bytes) go to StateMachine::Apply in
//     instance order as each window makes them applicable — membership and noop Values are
//     not passed, as Learner::Apply does not (:1062-1073);
//   * Callback::Accepted / Applied / Unproposable from the learn bookkeeping (mpx_read_learns
//     + mpx_read_learn_values with MPX_FLAG_DECISIONS): a learn created at an accept quorum (kind
//     0) is the batch whose values Proposer::OnAcceptReply passes to Accepted (:1327-1332); a
//     learn created at a promise quorum or a learner change (kinds 1, 2: the whole learned map,
//     plus the open learns' values) passes its values to Applied at its applied record — an
//     acceptor quorum of repliers, OnLearnReply or AcceptorsChanged (:1360-1368,1523-1526); a
//     P_PROPOSE the node received without a Proposer is Unproposable (:784-787).  The cb strings
//     come from the Values' own bytes (mpx_value_bytes).
// It replays a member MPXT trace, dropping its E_EPOCH markers, in W windows (an incremental
// engine: the OnReceive loop of a live host), and prints what the transport, the state machines
// and the callbacks saw, plus the epochs the engine learned, so a test can compare them with the
// Python binding and the reference's fixtures.
//
//   member_host <trace.mpxt> [windows]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <map>
#include <string>
#include <vector>

#include "paxos.h"     // the reference's member/paxos.h (include path from examples/Makefile)
#include "mpx.h"

namespace {

uint64_t fnv(uint64_t h, const void *p, size_t n)
{
    const uint8_t *b = (const uint8_t *)p;
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

template <typename T> T rd(const uint8_t *p)
{
    T v;
    std::memcpy(&v, p, sizeof v);
    return v;
}

struct Tally {                         // count + order-independent sum of per-event hashes
    uint64_t count = 0, hash = 0;
    void add(uint64_t h) { ++count; hash += h; }
};

class EngineNetWork : public paxos::NetWork {
public:
    EngineNetWork(mpx_engine *eng, uint32_t node, Tally *wire) : eng_(eng), node_(node), wire_(wire) { offs_.push_back(0); }

    void Receive(const std::string &msg)                   // where NetWork::OnReceive hands msg to the node
    {
        buf_ += msg;
        offs_.push_back(buf_.size());
    }
    int Flush()
    {
        int rc = mpx_submit(eng_, node_, (const uint8_t *)buf_.data(), offs_.data(), offs_.size() - 1);
        buf_.clear();
        offs_.assign(1, 0);
        return rc;
    }
    void Send(Thread *, paxos::NodeID node, const std::string &msg)
    {
        const uint32_t src = node_, dst = node;
        uint64_t h = 1469598103934665603ull;
        h = fnv(h, &src, 4);
        h = fnv(h, &dst, 4);
        wire_->add(fnv(h, msg.data(), msg.size()));
    }

private:
    mpx_engine *eng_;
    uint32_t node_;
    Tally *wire_;
    std::string buf_;
    std::vector<uint64_t> offs_;
};

class CountingStateMachine : public paxos::StateMachine {
public:
    bool Apply(Thread *, const std::string &value, std::string *)
    {
        ++count;
        hash = fnv(hash, value.data(), value.size());
        return true;
    }
    uint64_t count = 0, hash = 1469598103934665603ull;
};

class CountingCallback : public paxos::Callback {
public:
    void Accepted(Thread *, const std::string &cb) { accepted.add(fnv(1469598103934665603ull, cb.data(), cb.size())); }
    void Applied(Thread *, const std::string &cb, const std::string *) { applied.add(fnv(1469598103934665603ull, cb.data(), cb.size())); }
    void Unproposable(Thread *, const std::string &cb) { unproposable.add(fnv(1469598103934665603ull, cb.data(), cb.size())); }
    Tally accepted, applied, unproposable;
};

struct DrainCtx { std::vector<EngineNetWork *> *nets; };

void on_send(void *user, uint32_t src, uint32_t dst, const uint8_t *bytes, uint32_t len)
{
    DrainCtx *c = (DrainCtx *)user;
    (*c->nets)[src]->Send(nullptr, dst, std::string((const char *)bytes, len));
}

// the cb string of a member Value_m: u32 proposer, u64 value_id, u8 noop [, u8 membership, u32 n,
// payload or n changes, u32 cb length, cb] (FillValue, member/paxos.cpp:330-363); "" for a noop
bool value_cb(const uint8_t *v, size_t len, std::string &cb)
{
    cb.clear();
    if (len < 13) return false;
    if (v[12]) return true;
    if (len < 18) return false;
    const bool mem = v[13] != 0;
    const uint32_t n = rd<uint32_t>(v + 14);
    const size_t p = 18 + (mem ? 8 * (size_t)n : (size_t)n);
    if (p + 4 > len) return false;
    const uint32_t cl = rd<uint32_t>(v + p);
    if (p + 4 + cl > len) return false;
    cb.assign((const char *)v + p + 4, cl);
    return true;
}

bool handle_cb(mpx_engine *eng, uint64_t h, std::string &cb)
{
    std::vector<uint8_t> buf(256);
    uint32_t len = 0;
    if (mpx_value_bytes(eng, h, buf.data(), (uint32_t)buf.size(), &len)) return false;
    if (len > buf.size()) {
        buf.resize(len);
        if (mpx_value_bytes(eng, h, buf.data(), (uint32_t)buf.size(), &len)) return false;
    }
    return value_cb(buf.data(), len, cb);
}

}  // namespace

int main(int argc, char **argv)
{
    if (argc < 2) { std::fprintf(stderr, "usage: %s trace.mpxt [windows]\n", argv[0]); return 2; }
    const uint32_t W = argc > 2 ? (uint32_t)std::max(1, std::atoi(argv[2])) : 1;
    std::ifstream f(argv[1], std::ios::binary);
    std::string t((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    const uint8_t *tb = (const uint8_t *)t.data();
    if (t.size() < 40 || t.compare(0, 4, "MPXT") != 0) { std::fprintf(stderr, "not an MPXT trace\n"); return 2; }
    const uint32_t ver = rd<uint32_t>(tb + 4), N = rd<uint32_t>(tb + 8), sem = rd<uint32_t>(tb + 12), ne = rd<uint32_t>(tb + 24);
    const uint64_t M = rd<uint64_t>(tb + 16);
    if (sem != MPX_SEM_MEMBER || !ne) { std::fprintf(stderr, "member semantics only\n"); return 2; }
    const size_t esz = ver == 1 ? 24 : 32;
    // the genesis epoch only: {first} learner, proposer and acceptor (NodeImpl::Loop, :738-747)
    mpx_epoch genesis{rd<uint32_t>(tb + 40), 0, rd<uint64_t>(tb + 48), rd<uint64_t>(tb + 56),
                      esz == 32 ? rd<uint64_t>(tb + 64) : rd<uint64_t>(tb + 56)};
    mpx_config cfg;
    std::memset(&cfg, 0, sizeof cfg);
    cfg.abi_version = MPX_ABI_VERSION; cfg.num_nodes = N; cfg.semantics = MPX_SEM_MEMBER; cfg.device = 0;
    cfg.shard_begin = 0; cfg.shard_end = M ? M : 1;
    cfg.num_epochs = 1; cfg.epochs = &genesis;
    cfg.flags = MPX_FLAG_INCREMENTAL | MPX_FLAG_DECISIONS | MPX_FLAG_LEARN_EPOCHS;
    mpx_engine *eng = nullptr;
    int rc = mpx_create(&cfg, &eng);
    if (rc) { std::fprintf(stderr, "mpx_create: %d\n", rc); return 1; }
    Tally wire;
    std::vector<EngineNetWork *> nets;
    std::vector<CountingStateMachine> sms(N);
    std::vector<CountingCallback> cbs(N);
    for (uint32_t n = 0; n < N; ++n) nets.push_back(new EngineNetWork(eng, n, &wire));
    // MPXT body: per node {u64 count, u64 nbytes, u64 offsets[count + 1], bytes, pad to 8}
    std::vector<size_t> offs(N), body(N);
    std::vector<uint64_t> cnt(N);
    size_t pos = 40 + (size_t)ne * esz;
    for (uint32_t n = 0; n < N; ++n) {
        cnt[n] = rd<uint64_t>(tb + pos);
        const uint64_t nb = rd<uint64_t>(tb + pos + 8);
        offs[n] = pos + 16; body[n] = offs[n] + 8 * (cnt[n] + 1);
        pos = body[n] + ((nb + 7) & ~7ull);
    }
    DrainCtx ctx{&nets};
    // The engine's record indices count its own E_EPOCH records, which it places where the reference
    // applies a membership Value — here, where the trace's markers were: positions count them too
    std::vector<uint64_t> applied_sm(N, 0);          // executed values handed to Apply so far
    std::vector<std::map<uint64_t, std::pair<bool, bool>>> seen(N);   // learn -> (accepted, applied) reported
    std::vector<uint64_t> unprop_seen(N, 0);         // Unproposable records reported
    std::vector<uint32_t> epochs_after;              // the learned table's size after each window
    for (uint32_t w = 0; w < W; ++w) {
        for (uint32_t n = 0; n < N; ++n) {
            const uint64_t k0 = cnt[n] * w / W, k1 = cnt[n] * (w + 1) / W;
            for (uint64_t k = k0; k < k1; ++k) {
                const uint64_t a = rd<uint64_t>(tb + offs[n] + 8 * k), b = rd<uint64_t>(tb + offs[n] + 8 * (k + 1));
                const uint8_t *m = tb + body[n] + a;
                const uint32_t type = rd<uint32_t>(m);
                if (type == MPX_MSG_E_EPOCH) continue;            // the engine learns the membership itself
                nets[n]->Receive(std::string((const char *)m, b - a));
            }
            if ((rc = nets[n]->Flush())) { std::fprintf(stderr, "mpx_submit: %d\n", rc); return 1; }
        }
        if ((rc = mpx_run(eng))) { std::fprintf(stderr, "mpx_run: %d\n", rc); return 1; }
        if ((rc = mpx_drain_sends(eng, on_send, &ctx))) { std::fprintf(stderr, "mpx_drain_sends: %d\n", rc); return 1; }
        // StateMachine::Apply for what became applicable in this window, in instance order
        for (uint32_t n = 0; n < N; ++n) {
            uint64_t frontier = 0, c = 0;
            if ((rc = mpx_read_executed(eng, n, &frontier, &c, nullptr, 0))) return 1;
            std::vector<uint64_t> h(c ? c : 1);
            if ((rc = mpx_read_executed(eng, n, &frontier, &c, h.data(), c))) return 1;
            for (uint64_t i = applied_sm[n]; i < c; ++i) {
                uint8_t buf[1 << 12];
                uint32_t len = 0;
                if ((rc = mpx_value_bytes(eng, h[i], buf, sizeof buf, &len)) || len < 13) return 1;
                if (buf[12] || len < 18 || buf[13]) continue;     // noop / membership: not the state machine's
                const uint32_t sz = rd<uint32_t>(buf + 14);
                sms[n].Apply(nullptr, std::string((const char *)buf + 18, sz), nullptr);
            }
            applied_sm[n] = c;
        }
        // Callback::Accepted / Applied / Unproposable from the learns (MPXL) and their Values (MPXV)
        // this window created or applied
        uint8_t *ml = nullptr, *mv = nullptr;
        uint64_t ms = 0, mvs = 0;
        if ((rc = mpx_read_learns(eng, &ml, &ms))) { std::fprintf(stderr, "mpx_read_learns: %d\n", rc); return 1; }
        if ((rc = mpx_read_learn_values(eng, &mv, &mvs))) { std::fprintf(stderr, "mpx_read_learn_values: %d\n", rc); return 1; }
        size_t p = 12, q = 12;
        std::string cb;
        for (uint32_t n = 0; n < N; ++n) {
            const uint64_t nl = rd<uint64_t>(ml + p);
            if (rd<uint64_t>(mv + q) != nl) { std::fprintf(stderr, "MPXV / MPXL differ\n"); return 1; }
            p += 8; q += 8;
            for (uint64_t k = 0; k < nl; ++k, p += 64) {
                const uint64_t kind = rd<uint64_t>(ml + p + 16), applied = rd<uint64_t>(ml + p + 32);
                const uint64_t nv = rd<uint64_t>(mv + q);
                const uint8_t *vals = mv + q + 8;                    // {u64 iid, u64 handle}*
                q += 8 + 16 * nv;
                auto &s = seen[n][k];                                // (MPXL: every learn so far, in creation order)
                const bool acc = kind == 0 && !s.first, app = kind != 0 && !s.second && applied != ~0ull;
                if (!acc && !app) continue;
                for (uint64_t j = 0; j < nv; ++j) {
                    if (!handle_cb(eng, rd<uint64_t>(vals + 16 * j + 8), cb)) { std::fprintf(stderr, "bad Value\n"); return 1; }
                    if (acc) cbs[n].Accepted(nullptr, cb);
                    else cbs[n].Applied(nullptr, cb, nullptr);
                }
                (acc ? s.first : s.second) = true;
            }
            const uint64_t nu = rd<uint64_t>(mv + q);
            q += 8;
            for (uint64_t j = unprop_seen[n]; j < nu; ++j) {          // the host's own P_PROPOSE record
                const uint64_t k = rd<uint64_t>(mv + q + 8 * j);
                if (k >= cnt[n]) { std::fprintf(stderr, "bad Unproposable record\n"); return 1; }
                const uint64_t a = rd<uint64_t>(tb + offs[n] + 8 * k), b = rd<uint64_t>(tb + offs[n] + 8 * (k + 1));
                if (b - a < 8 || !value_cb(tb + body[n] + a + 8, b - a - 8, cb)) { std::fprintf(stderr, "bad P_PROPOSE\n"); return 1; }
                cbs[n].Unproposable(nullptr, cb);
            }
            unprop_seen[n] = nu;
            q += 8 * nu;
        }
        mpx_free(ml);
        mpx_free(mv);
        uint32_t ec = 0;
        if ((rc = mpx_read_epochs(eng, nullptr, 0, &ec))) return 1;
        epochs_after.push_back(ec);
    }
    std::printf("sends %llu %016llx\n", (unsigned long long)wire.count, (unsigned long long)wire.hash);
    for (uint32_t n = 0; n < N; ++n) {
        uint64_t frontier = 0, c = 0;
        if ((rc = mpx_read_executed(eng, n, &frontier, &c, nullptr, 0))) return 1;
        std::printf("applied %u %llu %llu %016llx\n", n, (unsigned long long)frontier, (unsigned long long)sms[n].count,
                    (unsigned long long)sms[n].hash);
        std::printf("callbacks %u %llu %016llx %llu %016llx %llu %016llx\n", n, (unsigned long long)cbs[n].accepted.count,
                    (unsigned long long)cbs[n].accepted.hash, (unsigned long long)cbs[n].applied.count,
                    (unsigned long long)cbs[n].applied.hash, (unsigned long long)cbs[n].unproposable.count,
                    (unsigned long long)cbs[n].unproposable.hash);
    }
    uint32_t ec = 0;
    mpx_read_epochs(eng, nullptr, 0, &ec);
    std::vector<mpx_epoch> ep(ec ? ec : 1);
    mpx_read_epochs(eng, ep.data(), ec, &ec);
    std::printf("epochs");
    for (uint32_t k = 0; k < ec; ++k)
        std::printf(" %u:%llx:%llx:%llx", ep[k].version, (unsigned long long)ep[k].acceptor_mask,
                    (unsigned long long)ep[k].proposer_mask, (unsigned long long)ep[k].learner_mask);
    std::printf("\nepochs_per_window");
    for (uint32_t x : epochs_after) std::printf(" %u", x);
    std::printf("\n");
    for (auto *x : nets) delete x;
    mpx_destroy(eng);
    return 0;
}
