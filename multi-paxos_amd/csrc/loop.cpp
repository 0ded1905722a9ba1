// loop.cpp — the closed loop in libmpx: the engine's own
// results drive the proposers' next messages with no host-language round trip.
//
// The proposer's control plane (out of scope for the device) is a small host
// driver over one incremental engine (MPX_FLAG_INCREMENTAL | MPX_FLAG_DECISIONS); every message it
// sends is made from what the engine computed:
//   * StartPrepare (multi/paxos.cpp:1233-1248): P_START at the proposer, PREPARE over [0, 2^64-1)
//     to the acceptors picked;
//   * the acceptors' replies are the engine's drained sends (OnPrepare / OnAccept / OnCommit on the
//     device), appended to the stream of the node they are addressed to;
//   * at a promise quorum the phase-2 batch is the engine's decision (mpx_read_decisions: adopted
//     pre-accepted values, noop fill, the proposer's queued client values, :1056-1175), sent as
//     P_BATCH + ACCEPT with accepting_id_ + 1 (:1299-1326);
//   * a batch whose instances the engine's chosen log holds is committed (Commit, :1429-1444)
//     with committing_id_ + 1.
// A step submits only the records added since the last one and runs them as one window.  The
// recorded streams (mpx_loop_trace) replayed through the reference's own handlers give the
// engine's result and decisions byte for byte (tests/test_engine_gpu.py).  mpx/loop.py is the
// same driver in Python; both make identical streams for identical schedules.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "mpx.h"

namespace {

template <typename T> inline void put(std::string &s, T v) { s.append((const char *)&v, sizeof v); }
template <typename T> inline T get(const uint8_t *p) { T v; std::memcpy(&v, p, sizeof v); return v; }

}  // namespace

struct mpx_loop {
    uint32_t N = 0;
    uint64_t M = 0;
    mpx_engine *eng = nullptr;
    std::vector<std::vector<std::string>> streams;
    std::vector<uint64_t> submitted, ballot_count, ballot, accepting_id, committing_id, value_id, decided;
    std::map<std::pair<uint32_t, uint64_t>, std::string> payload;              // (node, value id) -> client payload
    struct Batch { uint64_t ballot; std::vector<std::pair<uint64_t, uint64_t>> ents; };
    std::map<std::pair<uint32_t, uint64_t>, Batch> batches;                     // (node, accept id) -> batch
    std::set<std::pair<uint32_t, uint64_t>> committed;
    std::vector<uint64_t> chosen;                                               // scratch: the chosen log
    mpx_loop_stats st{};
};

namespace {

// FillValue (multi/paxos.cpp:556-598) of a handle: a noop, this loop's own client value, or the
// engine's value table (a value some node adopted)
int value_bytes(mpx_loop *L, uint64_t h, std::string &out)
{
    const uint32_t node = MPX_HANDLE_PROPOSER(h);
    const uint64_t vid = MPX_HANDLE_VALUE_ID(h);
    out.clear();
    if (MPX_HANDLE_NOOP(h)) {
        put<uint32_t>(out, node); put<uint64_t>(out, vid); put<uint8_t>(out, 1);
        return MPX_OK;
    }
    auto it = L->payload.find({node, vid});
    if (it != L->payload.end()) {
        put<uint32_t>(out, node); put<uint64_t>(out, vid); put<uint8_t>(out, 0); put<uint8_t>(out, 0);
        put<uint32_t>(out, (uint32_t)it->second.size());
        out += it->second;
        return MPX_OK;
    }
    uint32_t len = 0;
    out.resize(64);
    if (int rc = mpx_value_bytes(L->eng, h, (uint8_t *)&out[0], (uint32_t)out.size(), &len)) return rc;
    if (len > out.size()) {
        out.resize(len);
        if (int rc = mpx_value_bytes(L->eng, h, (uint8_t *)&out[0], (uint32_t)out.size(), &len)) return rc;
    }
    out.resize(len);
    return MPX_OK;
}

void on_send(void *user, uint32_t, uint32_t dst, const uint8_t *bytes, uint32_t len)
{
    mpx_loop *L = (mpx_loop *)user;
    if (dst < L->N) L->streams[dst].emplace_back((const char *)bytes, len);
}

void to_nodes(mpx_loop *L, uint64_t mask, const std::string &m)
{
    for (uint32_t a = 0; a < L->N; ++a)
        if ((mask >> a) & 1) L->streams[a].push_back(m);
}

uint64_t now_ns()
{
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

extern "C" int mpx_loop_create(uint32_t num_nodes, uint64_t num_instances, int device, mpx_loop **out)
{
    if (!out || !num_nodes || num_nodes > MPX_MAX_NODES || !num_instances) return MPX_E_INVAL;
    mpx_config cfg;
    std::memset(&cfg, 0, sizeof cfg);
    cfg.abi_version = MPX_ABI_VERSION; cfg.num_nodes = num_nodes; cfg.semantics = MPX_SEM_MULTI; cfg.device = device;
    cfg.shard_begin = 0; cfg.shard_end = num_instances;
    cfg.flags = MPX_FLAG_INCREMENTAL | MPX_FLAG_DECISIONS;
    mpx_engine *e = nullptr;
    if (int rc = mpx_create(&cfg, &e)) return rc;
    mpx_loop *L = new mpx_loop;
    L->N = num_nodes; L->M = num_instances; L->eng = e;
    L->streams.assign(num_nodes, {});
    for (auto *v : {&L->submitted, &L->ballot_count, &L->ballot, &L->accepting_id, &L->committing_id, &L->value_id,
                    &L->decided})
        v->assign(num_nodes, 0);
    *out = L;
    return MPX_OK;
}

extern "C" int mpx_loop_destroy(mpx_loop *L)
{
    if (!L) return MPX_E_INVAL;
    mpx_destroy(L->eng);
    delete L;
    return MPX_OK;
}

extern "C" mpx_engine *mpx_loop_engine(mpx_loop *L) { return L ? L->eng : nullptr; }

// StartPrepare at `node` (:1233-1248): a higher ballot (count << 16 | node), P_START at the
// proposer, PREPARE over AvailableInstanceIDs [0, 2^64-1) (:741-755) to the acceptors in `to`
extern "C" int mpx_loop_prepare(mpx_loop *L, uint32_t node, uint64_t to)
{
    if (!L || node >= L->N) return MPX_E_INVAL;
    const uint64_t b = (++L->ballot_count[node] << 16) | node;
    L->ballot[node] = b;
    std::string ps;
    put<uint32_t>(ps, MPX_MSG_P_START); put<uint64_t>(ps, b);
    L->streams[node].push_back(ps);
    std::string p;
    put<uint32_t>(p, MPX_MSG_PREPARE); put<uint32_t>(p, node); put<uint64_t>(p, b); put<uint32_t>(p, 16);
    put<uint64_t>(p, 0); put<uint64_t>(p, ~0ull);
    to_nodes(L, to, p);
    return MPX_OK;
}

// a client value reaches Propose at `node` (:1250-1280): value_id_ + 1, a P_PROPOSE record
extern "C" int mpx_loop_propose(mpx_loop *L, uint32_t node, const uint8_t *bytes, uint32_t len)
{
    if (!L || node >= L->N || (len && !bytes)) return MPX_E_INVAL;
    const uint64_t vid = ++L->value_id[node];
    std::string pl((const char *)bytes, len);
    std::string r;
    put<uint32_t>(r, MPX_MSG_P_PROPOSE); put<uint32_t>(r, len); r += pl;
    L->payload[{node, vid}] = std::move(pl);
    L->streams[node].push_back(r);
    return MPX_OK;
}

// one window: every stream's records since the last step, run on the carried state; the
// replies go to the streams of the nodes they are addressed to
extern "C" int mpx_loop_step(mpx_loop *L)
{
    if (!L) return MPX_E_INVAL;
    const uint64_t t0 = now_ns();
    std::string buf;
    std::vector<uint64_t> offs;
    for (uint32_t n = 0; n < L->N; ++n) {
        auto &s = L->streams[n];
        if (s.size() <= L->submitted[n]) continue;
        buf.clear(); offs.assign(1, 0);
        for (size_t k = L->submitted[n]; k < s.size(); ++k) { buf += s[k]; offs.push_back(buf.size()); }
        if (int rc = mpx_submit(L->eng, n, (const uint8_t *)buf.data(), offs.data(), offs.size() - 1)) return rc;
        L->st.records += offs.size() - 1;
        L->submitted[n] = s.size();
    }
    const uint64_t t1 = now_ns();
    if (int rc = mpx_run(L->eng)) return rc;
    const uint64_t t2 = now_ns();
    if (int rc = mpx_drain_sends(L->eng, on_send, L)) return rc;
    L->st.windows++;
    L->st.submit_ns += t1 - t0;
    L->st.run_ns += t2 - t1;
    L->st.drain_ns += now_ns() - t2;
    return MPX_OK;
}

// the phase-2 batch the engine decided at `node`'s latest promise quorum not sent yet (MPXD):
// P_BATCH at the proposer, ACCEPT to `to`; value_id_ also counts the node's own noops
// (:1117-1130).  *accept_id: the batch's id, 0 when there was none to send.
extern "C" int mpx_loop_accept_decided(mpx_loop *L, uint32_t node, uint64_t to, uint64_t *accept_id)
{
    if (!L || node >= L->N) return MPX_E_INVAL;
    if (accept_id) *accept_id = 0;
    uint8_t *d = nullptr;
    uint64_t ds = 0;
    if (int rc = mpx_read_decisions(L->eng, &d, &ds)) return rc;
    // MPXD: "MPXD" u32 1, u32 nodes; per node u64 count, {u64 seq, u64 k, k x {u64 iid, u64 handle}}
    std::vector<std::pair<uint64_t, uint64_t>> last;
    uint64_t nq = 0;
    size_t p = 12;
    for (uint32_t n = 0; n < L->N && p + 8 <= ds; ++n) {
        const uint64_t c = get<uint64_t>(d + p);
        p += 8;
        for (uint64_t q = 0; q < c; ++q) {
            const uint64_t k = get<uint64_t>(d + p + 8);
            const uint8_t *e = d + p + 16;
            if (n == node && q >= L->decided[node]) {
                for (uint64_t j = 0; j < k; ++j) {
                    const uint64_t h = get<uint64_t>(e + 16 * j + 8);
                    if (MPX_HANDLE_NOOP(h) && MPX_HANDLE_PROPOSER(h) == node) ++L->value_id[node];
                }
                if (q + 1 == c) {
                    last.resize(k);
                    for (uint64_t j = 0; j < k; ++j) last[j] = {get<uint64_t>(e + 16 * j), get<uint64_t>(e + 16 * j + 8)};
                }
            }
            p += 16 + 16 * k;
        }
        if (n == node) nq = c;
    }
    mpx_free(d);
    if (L->decided[node] >= nq) return MPX_OK;
    L->decided[node] = nq;
    if (last.empty()) return MPX_OK;
    const uint64_t aid = ++L->accepting_id[node], b = L->ballot[node];
    std::string body, vb;
    for (auto &x : last) {
        if (int rc = value_bytes(L, x.second, vb)) return rc;
        put<uint64_t>(body, x.first);
        body += vb;
    }
    std::string pb, acc;
    put<uint32_t>(pb, MPX_MSG_P_BATCH); put<uint64_t>(pb, aid); put<uint32_t>(pb, (uint32_t)body.size()); pb += body;
    L->streams[node].push_back(pb);
    put<uint32_t>(acc, MPX_MSG_ACCEPT); put<uint32_t>(acc, node); put<uint64_t>(acc, aid); put<uint64_t>(acc, b);
    put<uint32_t>(acc, (uint32_t)body.size()); acc += body;
    to_nodes(L, to, acc);
    L->batches[{node, aid}] = mpx_loop::Batch{b, std::move(last)};
    L->st.batches++;
    if (accept_id) *accept_id = aid;
    return MPX_OK;
}

// COMMIT (:1429-1444) every batch of `node` whose instances are all in the engine's chosen log
extern "C" int mpx_loop_commit_chosen(mpx_loop *L, uint32_t node, uint64_t to, uint32_t *count)
{
    if (!L || node >= L->N) return MPX_E_INVAL;
    uint32_t done = 0;
    bool have = false;
    std::string body, vb;
    for (auto &x : L->batches) {
        if (x.first.first != node || L->committed.count(x.first)) continue;
        if (!have) {
            L->chosen.resize(L->M);
            if (int rc = mpx_read_chosen(L->eng, 0, L->M, L->chosen.data())) return rc;
            have = true;
        }
        bool all = true;
        for (auto &e : x.second.ents) all = all && e.first < L->M && (L->chosen[e.first] & MPX_PRESENT);
        if (!all) continue;
        L->committed.insert(x.first);
        body.clear();
        for (auto &e : x.second.ents) {
            if (int rc = value_bytes(L, e.second, vb)) return rc;
            put<uint64_t>(body, e.first);
            body += vb;
        }
        std::string com;
        put<uint32_t>(com, MPX_MSG_COMMIT); put<uint32_t>(com, node); put<uint64_t>(com, ++L->committing_id[node]);
        put<uint64_t>(com, x.second.ballot); put<uint32_t>(com, (uint32_t)body.size()); com += body;
        to_nodes(L, to, com);
        L->st.committed_batches++;
        L->st.committed_instances += x.second.ents.size();
        ++done;
    }
    if (count) *count = done;
    return MPX_OK;
}

// A leader's rounds (the closed-loop bench leg): per round, node `leader` starts a new round
// (StartPrepare to `to`) with `values` client values queued (Propose while preparing), and the
// loop steps until the round's batch is decided (promise quorum), chosen (accept quorum) and
// committed to every node in `to` — 5 windows per round: PREPARE + queued Propose, promises ->
// decision -> ACCEPT, accept replies -> chosen -> COMMIT, commits, commit replies.  Payloads are
// the decimal client id (multi/main.cpp:30-35).
extern "C" int mpx_loop_leader_rounds(mpx_loop *L, uint32_t leader, uint64_t to, uint32_t rounds, uint32_t values)
{
    if (!L || leader >= L->N || !rounds) return MPX_E_INVAL;
    for (uint32_t r = 0; r < rounds; ++r) {
        if (int rc = mpx_loop_prepare(L, leader, to)) return rc;
        for (uint32_t k = 0; k < values; ++k) {
            const std::string p = std::to_string(L->st.proposed++);
            if (int rc = mpx_loop_propose(L, leader, (const uint8_t *)p.data(), (uint32_t)p.size())) return rc;
        }
        if (int rc = mpx_loop_step(L)) return rc;                 // acceptors promise
        if (int rc = mpx_loop_step(L)) return rc;                 // the leader's quorum: the decision
        uint64_t aid = 0;
        if (int rc = mpx_loop_accept_decided(L, leader, to, &aid)) return rc;
        if (!aid) return MPX_E_STATE;                             // (a round without a quorum batch)
        if (int rc = mpx_loop_step(L)) return rc;                 // acceptors accept
        if (int rc = mpx_loop_step(L)) return rc;                 // accept quorum: chosen
        uint32_t c = 0;
        if (int rc = mpx_loop_commit_chosen(L, leader, to, &c)) return rc;
        if (!c) return MPX_E_STATE;
        if (int rc = mpx_loop_step(L)) return rc;                 // learners commit, reply
    }
    return MPX_OK;
}

extern "C" int mpx_loop_stats_get(mpx_loop *L, mpx_loop_stats *out)
{
    if (!L || !out) return MPX_E_INVAL;
    *out = L->st;
    return MPX_OK;
}

// the recorded streams as an MPXT container (version 1, multi semantics): what the loop sent
// every node, replayable through the reference's own handlers
extern "C" int mpx_loop_trace(mpx_loop *L, uint8_t **out, uint64_t *size)
{
    if (!L || !out || !size) return MPX_E_INVAL;
    std::string t;
    t.append("MPXT", 4);
    put<uint32_t>(t, 1); put<uint32_t>(t, L->N); put<uint32_t>(t, MPX_SEM_MULTI); put<uint64_t>(t, L->M);
    put<uint32_t>(t, 0); put<uint32_t>(t, 0); put<uint64_t>(t, 0);
    for (auto &s : L->streams) {
        uint64_t tot = 0;
        for (auto &m : s) tot += m.size();
        put<uint64_t>(t, s.size()); put<uint64_t>(t, tot);
        uint64_t o = 0;
        put<uint64_t>(t, 0);
        for (auto &m : s) { o += m.size(); put<uint64_t>(t, o); }
        for (auto &m : s) t += m;
        while (t.size() % 8) t.push_back('\0');
    }
    *out = (uint8_t *)std::malloc(t.size());
    if (!*out) return MPX_E_NOMEM;
    std::memcpy(*out, t.data(), t.size());
    *size = t.size();
    return MPX_OK;
}
