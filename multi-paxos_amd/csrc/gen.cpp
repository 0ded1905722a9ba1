// gen.cpp — deterministic synthetic traces (host), MPXT containers.
//
// Traces are per-node receive streams in the reference's wire vocabulary plus
// the P_START / P_BATCH proposer markers (include/mpx.h).  Config names follow
// C2/C4 are MPX_GEN_CLEAN, C3 is MPX_GEN_FAULTY.
#include <cstring>
#include <string>
#include <vector>

#include "gen.hpp"
#include "mpx.h"

namespace mpx {

template <typename T> static inline void app(std::string &s, T v) { s.append((const char *)&v, sizeof v); }

void TraceWriter::begin(uint32_t N, uint32_t semantics, uint64_t M, const std::vector<mpx_epoch> &epochs)
{
    out.clear();
    out.append("MPXT", 4);
    app<uint32_t>(out, epochs.empty() ? 1 : 2);     // version 2: 32-byte epoch entries (learner_mask)
    app<uint32_t>(out, N);
    app<uint32_t>(out, semantics);
    app<uint64_t>(out, M);
    app<uint32_t>(out, (uint32_t)epochs.size());
    app<uint32_t>(out, 0);
    app<uint64_t>(out, 0);
    for (auto &e : epochs) {
        app<uint32_t>(out, e.version); app<uint32_t>(out, e.flags);
        app<uint64_t>(out, e.acceptor_mask); app<uint64_t>(out, e.proposer_mask); app<uint64_t>(out, e.learner_mask);
    }
}

void TraceWriter::node(const std::vector<std::string> &msgs)
{
    uint64_t total = 0;
    for (auto &m : msgs) total += m.size();
    app<uint64_t>(out, msgs.size());
    app<uint64_t>(out, total);
    uint64_t off = 0;
    app<uint64_t>(out, 0);
    for (auto &m : msgs) { off += m.size(); app<uint64_t>(out, off); }
    for (auto &m : msgs) out += m;
    while (out.size() % 8) out.push_back('\0');
}

void TraceWriter::node_raw(const std::string &bytes, const std::vector<uint64_t> &offs)
{
    app<uint64_t>(out, offs.size() - 1);
    app<uint64_t>(out, bytes.size());
    out.append((const char *)offs.data(), 8 * offs.size());
    out += bytes;
    while (out.size() % 8) out.push_back('\0');
}

// ---- wire encoders ----
void enc_value(std::string &s, uint32_t proposer, uint64_t value_id, bool noop, const std::string &payload)
{
    app<uint32_t>(s, proposer); app<uint64_t>(s, value_id); app<uint8_t>(s, noop ? 1 : 0);
    if (!noop) { app<uint8_t>(s, 0); app<uint32_t>(s, (uint32_t)payload.size()); s += payload; }
}
std::string msg_prepare(uint32_t proposer, uint64_t ballot, const std::vector<std::pair<uint64_t, uint64_t>> &ranges)
{
    std::string s;
    app<uint32_t>(s, MPX_MSG_PREPARE); app<uint32_t>(s, proposer); app<uint64_t>(s, ballot);
    app<uint32_t>(s, (uint32_t)(16 * ranges.size()));
    for (auto &r : ranges) { app<uint64_t>(s, r.first); app<uint64_t>(s, r.second); }
    return s;
}
std::string msg_prepare_reply(uint32_t acceptor, uint64_t ballot, const std::string &body)
{
    std::string s;
    app<uint32_t>(s, MPX_MSG_PREPARE_REPLY); app<uint32_t>(s, acceptor); app<uint64_t>(s, ballot);
    app<uint32_t>(s, (uint32_t)body.size());
    return s + body;
}
std::string msg_reject(uint64_t max_id)
{
    std::string s;
    app<uint32_t>(s, MPX_MSG_REJECT); app<uint64_t>(s, max_id);
    return s;
}
std::string msg_accept(uint32_t proposer, uint64_t accept, uint64_t ballot, const std::string &body)
{
    std::string s;
    app<uint32_t>(s, MPX_MSG_ACCEPT); app<uint32_t>(s, proposer); app<uint64_t>(s, accept);
    app<uint64_t>(s, ballot); app<uint32_t>(s, (uint32_t)body.size());
    return s + body;
}
std::string msg_accept_reply(uint32_t acceptor, uint64_t ballot, uint64_t accept)
{
    std::string s;
    app<uint32_t>(s, MPX_MSG_ACCEPT_REPLY); app<uint32_t>(s, acceptor); app<uint64_t>(s, ballot); app<uint64_t>(s, accept);
    return s;
}
std::string msg_commit(uint32_t committer, uint64_t commit, uint64_t ballot, const std::string &body)
{
    std::string s;
    app<uint32_t>(s, MPX_MSG_COMMIT); app<uint32_t>(s, committer); app<uint64_t>(s, commit);
    app<uint64_t>(s, ballot); app<uint32_t>(s, (uint32_t)body.size());
    return s + body;
}
std::string msg_commit_reply(uint32_t learner, uint64_t commit)
{
    std::string s;
    app<uint32_t>(s, MPX_MSG_COMMIT_REPLY); app<uint32_t>(s, learner); app<uint64_t>(s, commit);
    return s;
}
std::string msg_p_start(uint64_t ballot)
{
    std::string s;
    app<uint32_t>(s, MPX_MSG_P_START); app<uint64_t>(s, ballot);
    return s;
}
std::string msg_p_batch(uint64_t batch, const std::string &body)
{
    std::string s;
    app<uint32_t>(s, MPX_MSG_P_BATCH); app<uint64_t>(s, batch); app<uint32_t>(s, (uint32_t)body.size());
    return s + body;
}

// ---- C2 / C4: one proposer (node 0, ballot 1<<16), no faults ----------------
// The order is what a fault-free run of the reference produces for one
// leader: StartPrepare (paxos.cpp:1233) -> PREPARE to all -> N promises ->
// per batch: new AcceptingValues, ACCEPT to all, N accept replies, COMMIT to
// all, N commit replies.  Values are (0, iid+1, decimal iid): the demo's
// client ids as payload (multi/main.cpp:30-35,414-423).
int gen_clean(const mpx_gen_params &p, std::string &out)
{
    const uint32_t N = p.num_nodes;
    const uint64_t M = p.num_instances, B = p.batch ? p.batch : 256;
    const uint64_t sb = p.shard_end > p.shard_begin ? p.shard_begin : 0;
    const uint64_t se = p.shard_end > p.shard_begin ? p.shard_end : ~0ull;
    if (!N || N > MPX_MAX_NODES) return MPX_E_INVAL;
    const uint64_t b0 = (1ull << 16) | 0;
    const uint64_t K = (M + B - 1) / B;
    std::vector<std::string> s0, si;
    s0.push_back(msg_p_start(b0));
    const std::string prep = msg_prepare(0, b0, {{0, ~0ull}});
    s0.push_back(prep);
    si.push_back(prep);
    for (uint32_t i = 0; i < N; ++i) s0.push_back(msg_prepare_reply(i, b0, std::string()));
    std::string body;
    for (uint64_t k = 0; k < K; ++k) {
        body.clear();
        for (uint64_t iid = k * B; iid < std::min(M, (k + 1) * B); ++iid) {
            if (iid < sb || iid >= se) continue;
            app<uint64_t>(body, iid);
            enc_value(body, 0, iid + 1, false, std::to_string(iid));
        }
        s0.push_back(msg_p_batch(k + 1, body));
        const std::string acc = msg_accept(0, k + 1, b0, body);
        const std::string com = msg_commit(0, k + 1, b0, body);
        s0.push_back(acc);
        for (uint32_t i = 0; i < N; ++i) s0.push_back(msg_accept_reply(i, b0, k + 1));
        s0.push_back(com);
        for (uint32_t i = 0; i < N; ++i) s0.push_back(msg_commit_reply(i, k + 1));
        si.push_back(acc);
        si.push_back(com);
    }
    TraceWriter w;
    w.begin(N, MPX_SEM_MULTI, M, {});
    w.node(s0);
    for (uint32_t i = 1; i < N; ++i) w.node(si);
    out.swap(w.out);
    return MPX_OK;
}

}  // namespace mpx
