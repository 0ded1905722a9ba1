// engine_host.cpp — the reference's own host hooks bound to libmpx.so.
//
// The reference host talks to its protocol core through paxos::NetWork
// (multi/paxos.h:193-212: SendMessageTCP/UDP out, OnReceiveMessage in) and
// paxos::StateMachine (multi/paxos.h:214-222: Execute in instance order).
// Here those classes come from the reference's own header, and the core
// behind them is the engine:
//   * EngineNetWork::Receive batches a node's received bytes and hands them
//     to mpx_submit (where the reference calls OnReceiveMessage, :1714-1717);
//   * mpx_drain_sends calls back into EngineNetWork::SendMessageUDP with the
//     destination's address, as the handlers' replies do (:888-899,1391-1403);
//   * the in-order executed Values (mpx_read_executed + mpx_value_bytes) go to
//     StateMachine::Execute (:1584-1622).
// The nodes' addresses are the demo's own paxos::NodeInfoMap (multi/main.cpp:265-268:
// node i at "0.0.0.0", port i): a reply leaves through SendMessageUDP(ip, port) of the
// destination's NodeInfo, and the transport maps (ip, port) back to the node by that map.
// It replays an MPXT trace (multi semantics) and prints what the transport and the state
// machines saw, so a test can compare it with the Python binding.  With a window count W
// the engine runs incrementally (MPX_FLAG_INCREMENTAL): each node's stream is received in
// W slices, and after each slice the engine applies just that window and the replies it
// produced are sent — the OnReceiveMessage loop of a live host.
//
//   engine_host <trace.mpxt> [windows]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <map>
#include <string>
#include <vector>

#include "paxos.h"     // the reference's multi/paxos.h (include path from examples/Makefile)
#include "mpx.h"

namespace {

uint64_t fnv(uint64_t h, const void *p, size_t n)
{
    const uint8_t *b = (const uint8_t *)p;
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

struct Wire {                         // what the host's transport saw: count, and a sum of
    uint64_t count = 0, hash = 0;     // per-send hashes (windows interleave the nodes' sends)
};

class EngineNetWork : public paxos::NetWork {
public:
    EngineNetWork(mpx_engine *eng, uint32_t node, Wire *wire, const paxos::NodeInfoMap *nodes)
        : eng_(eng), node_(node), wire_(wire), nodes_(nodes) { offs_.push_back(0); }

    void Receive(const char *msg, unsigned len)
    {
        buf_.append(msg, len);
        offs_.push_back(buf_.size());
    }
    int Flush()
    {
        int rc = mpx_submit(eng_, node_, (const uint8_t *)buf_.data(), offs_.data(), offs_.size() - 1);
        buf_.clear();
        offs_.assign(1, 0);
        return rc;
    }
    void SendMessageTCP(const std::string &ip, unsigned short port, const std::string &msg) { Send(ip, port, msg); }
    void SendMessageUDP(const std::string &ip, unsigned short port, const std::string &msg) { Send(ip, port, msg); }

private:
    void Send(const std::string &ip, unsigned short port, const std::string &msg)
    {
        uint32_t dst = ~0u;                                        // the node at (ip, port)
        for (paxos::NodeInfoMap::const_iterator it = nodes_->begin(); it != nodes_->end(); ++it)
            if (it->second.ip_ == ip && it->second.port_ == port) dst = it->first;
        const uint32_t src = node_;
        uint64_t h = 1469598103934665603ull;
        h = fnv(h, &src, 4);
        h = fnv(h, &dst, 4);
        h = fnv(h, msg.data(), msg.size());
        wire_->count++;
        wire_->hash += h;
    }
    mpx_engine *eng_;
    uint32_t node_;
    Wire *wire_;
    const paxos::NodeInfoMap *nodes_;
    std::string buf_;
    std::vector<uint64_t> offs_;
};

class CountingStateMachine : public paxos::StateMachine {
public:
    void Execute(const std::string &value)
    {
        ++count;
        hash = fnv(hash, value.data(), value.size());
    }
    uint64_t count = 0, hash = 1469598103934665603ull;
};

struct DrainCtx { std::vector<EngineNetWork *> *nets; const paxos::NodeInfoMap *nodes; };

// a reply of node src to node dst: out through src's NetWork to dst's address
void on_send(void *user, uint32_t src, uint32_t dst, const uint8_t *bytes, uint32_t len)
{
    DrainCtx *c = (DrainCtx *)user;
    const paxos::NodeInfo &to = c->nodes->find(dst)->second;
    (*c->nets)[src]->SendMessageUDP(to.ip_, to.port_, std::string((const char *)bytes, len));
}

template <typename T> T rd(const std::string &s, size_t o)
{
    T v;
    std::memcpy(&v, s.data() + o, sizeof v);
    return v;
}

}  // namespace

int main(int argc, char **argv)
{
    if (argc < 2) { std::fprintf(stderr, "usage: %s trace.mpxt [windows]\n", argv[0]); return 2; }
    const uint32_t W = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 0;     // 0: one batch run
    std::ifstream f(argv[1], std::ios::binary);
    std::string t((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (t.size() < 40 || t.compare(0, 4, "MPXT") != 0) { std::fprintf(stderr, "not an MPXT trace\n"); return 2; }
    const uint32_t N = rd<uint32_t>(t, 8), sem = rd<uint32_t>(t, 12);
    const uint64_t M = rd<uint64_t>(t, 16);
    if (sem != MPX_SEM_MULTI) { std::fprintf(stderr, "multi semantics only\n"); return 2; }
    mpx_config cfg;
    std::memset(&cfg, 0, sizeof cfg);
    cfg.abi_version = MPX_ABI_VERSION; cfg.num_nodes = N; cfg.semantics = sem; cfg.device = 0;
    cfg.shard_begin = 0; cfg.shard_end = M ? M : 1;
    cfg.flags = W ? MPX_FLAG_INCREMENTAL : 0;
    mpx_engine *eng = nullptr;
    int rc = mpx_create(&cfg, &eng);
    if (rc) { std::fprintf(stderr, "mpx_create: %d\n", rc); return 1; }
    // the demo's addresses (multi/main.cpp:265-268)
    paxos::NodeInfoMap nodes;
    for (uint32_t i = 0; i < N; ++i) nodes.insert(std::make_pair(i, paxos::NodeInfo("0.0.0.0", (unsigned short)i)));
    Wire wire;
    std::vector<EngineNetWork *> nets;
    for (uint32_t n = 0; n < N; ++n) nets.push_back(new EngineNetWork(eng, n, &wire, &nodes));
    // MPXT body: per node {u64 count, u64 nbytes, u64 offsets[count + 1], bytes, pad to 8}
    std::vector<size_t> offs(N), body(N);
    std::vector<uint64_t> cnt(N);
    size_t pos = 40;
    for (uint32_t n = 0; n < N; ++n) {
        cnt[n] = rd<uint64_t>(t, pos);
        const uint64_t nb = rd<uint64_t>(t, pos + 8);
        offs[n] = pos + 16; body[n] = offs[n] + 8 * (cnt[n] + 1);
        pos = body[n] + ((nb + 7) & ~7ull);
    }
    DrainCtx ctx{&nets, &nodes};
    const uint32_t windows = W ? W : 1;
    for (uint32_t w = 0; w < windows; ++w) {
        for (uint32_t n = 0; n < N; ++n) {
            const uint64_t k0 = cnt[n] * w / windows, k1 = cnt[n] * (w + 1) / windows;
            for (uint64_t k = k0; k < k1; ++k) {
                const uint64_t a = rd<uint64_t>(t, offs[n] + 8 * k), b = rd<uint64_t>(t, offs[n] + 8 * (k + 1));
                nets[n]->Receive(t.data() + body[n] + a, (unsigned)(b - a));   // = NetWork::OnReceiveMessage
            }
            if ((rc = nets[n]->Flush())) { std::fprintf(stderr, "mpx_submit: %d\n", rc); return 1; }
        }
        if ((rc = mpx_run(eng))) { std::fprintf(stderr, "mpx_run: %d\n", rc); return 1; }
        if ((rc = mpx_drain_sends(eng, on_send, &ctx))) { std::fprintf(stderr, "mpx_drain_sends: %d\n", rc); return 1; }
    }
    std::printf("sends %llu %016llx\n", (unsigned long long)wire.count, (unsigned long long)wire.hash);
    for (uint32_t n = 0; n < N; ++n) {
        uint64_t frontier = 0, cnt = 0;
        if ((rc = mpx_read_executed(eng, n, &frontier, &cnt, nullptr, 0))) return 1;
        std::vector<uint64_t> h(cnt ? cnt : 1);
        if ((rc = mpx_read_executed(eng, n, &frontier, &cnt, h.data(), cnt))) return 1;
        CountingStateMachine sm;
        for (uint64_t i = 0; i < cnt; ++i) {
            uint8_t buf[1 << 12];
            uint32_t len = 0;
            if ((rc = mpx_value_bytes(eng, h[i], buf, sizeof buf, &len)) || len < 18) return 1;
            // FillValue layout (multi/paxos.cpp:567-599): u32 proposer, u64 value_id, bool noop,
            // bool membership, u32 size, payload
            uint32_t sz;
            std::memcpy(&sz, buf + 14, 4);
            sm.Execute(std::string((const char *)buf + 18, sz));
        }
        std::printf("executed %u %llu %llu %016llx\n", n, (unsigned long long)frontier, (unsigned long long)sm.count,
                    (unsigned long long)sm.hash);
    }
    for (auto *p : nets) delete p;
    mpx_destroy(eng);
    return 0;
}
