// ingest.cpp — wire decode and instance bucketing (host, C++17).
//
// The reference decodes inside each handler (ExtractAvailableInstanceIDs,
// ExtractInstanceValues, ExtractAcceptedValues; multi/paxos.cpp:523-711) into
// std::map/std::set.  Here every record is decoded once into flat SoA arrays;
// entry-carrying records are then cut into per-(node, 256-instance bucket)
// fragments so one GPU workgroup sees all events of its instances, in order,
// with coalesced entry reads.
#include "ingest.hpp"

#include <algorithm>
#include <cstring>

#include "mpx.h"

namespace mpx {

static inline uint32_t rd32(const uint8_t *p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
static inline uint64_t rd64(const uint8_t *p) { uint64_t v; std::memcpy(&v, p, 8); return v; }
template <typename T> static inline void app(std::string &s, T v) { s.append((const char *)&v, sizeof v); }

long ValueTable::parse(const uint8_t *p, size_t avail, uint64_t *handle)
{
    // FillValue / ExtractValue layout, multi/paxos.cpp:556-644
    if (avail < 13) return MPX_E_DECODE;
    const uint32_t proposer = rd32(p);
    const uint64_t value_id = rd64(p + 4);
    const bool noop = p[12] != 0;
    if (proposer >= (1u << 14) || value_id >= (1ull << 47)) return MPX_E_RANGE;
    std::string enc;
    enc.reserve(32);
    app<uint32_t>(enc, proposer);
    app<uint64_t>(enc, value_id);
    app<uint8_t>(enc, noop ? 1 : 0);
    size_t used;
    uint32_t exec_off = 0, exec_len = 0;
    if (noop) {
        used = 13;
    } else {
        if (avail < 14) return MPX_E_DECODE;
        const bool member = p[13] != 0;
        app<uint8_t>(enc, member ? 1 : 0);
        if (member) {
            if (avail < 19) return MPX_E_DECODE;
            app<uint32_t>(enc, rd32(p + 14));
            const bool add = p[18] != 0;
            app<uint8_t>(enc, add ? 1 : 0);
            if (add) {
                if (avail < 23) return MPX_E_DECODE;
                const uint32_t iplen = rd32(p + 19);
                if (avail < 25 + (size_t)iplen) return MPX_E_DECODE;
                app<uint32_t>(enc, iplen);
                enc.append((const char *)p + 23, iplen);
                enc.append((const char *)p + 23 + iplen, 2);
                used = 25 + iplen;
            } else {
                used = 19;
            }
        } else {
            if (avail < 18) return MPX_E_DECODE;
            const uint32_t len = rd32(p + 14);
            if (avail < 18 + (size_t)len) return MPX_E_DECODE;
            app<uint32_t>(enc, len);
            exec_off = (uint32_t)enc.size();
            exec_len = len;
            enc.append((const char *)p + 18, len);
            used = 18 + len;
        }
    }
    const uint64_t h = MPX_HANDLE(proposer, noop, value_id);
    auto it = idx.find(h);
    if (it != idx.end()) {
        const Rec &r = it->second;
        if (r.len != enc.size() || std::memcmp(bytes.data() + r.off, enc.data(), enc.size()) != 0)
            return MPX_E_VALUE;
    } else {
        Rec r{bytes.size(), (uint32_t)enc.size(), exec_off, exec_len};
        bytes += enc;
        idx.emplace(h, r);
    }
    *handle = h;
    return (long)used;
}

bool ValueTable::encode(uint64_t h, std::string &out) const
{
    auto it = idx.find(h);
    if (it != idx.end()) {
        out.append(bytes.data() + it->second.off, it->second.len);
        return true;
    }
    if (synthetic_clean && MPX_HANDLE_PROPOSER(h) == 0 && !MPX_HANDLE_NOOP(h)) {
        const std::string s = std::to_string(MPX_HANDLE_VALUE_ID(h) - 1);
        app<uint32_t>(out, 0); app<uint64_t>(out, MPX_HANDLE_VALUE_ID(h));
        app<uint8_t>(out, 0); app<uint8_t>(out, 0);
        app<uint32_t>(out, (uint32_t)s.size());
        out += s;
        return true;
    }
    return false;
}

bool ValueTable::exec_payload(uint64_t h, std::string &out) const
{
    auto it = idx.find(h);
    if (it != idx.end()) {
        out.assign(bytes.data() + it->second.off + it->second.exec_off, it->second.exec_len);
        return true;
    }
    if (synthetic_clean && MPX_HANDLE_PROPOSER(h) == 0 && !MPX_HANDLE_NOOP(h)) {
        out = std::to_string(MPX_HANDLE_VALUE_ID(h) - 1);
        return true;
    }
    return false;
}

static void flag(IngestViolation &v, uint64_t code, uint64_t node, uint64_t seq, uint64_t iid)
{
    v.count++;
    if (!v.code) { v.code = code; v.node = node; v.seq = seq; v.iid = iid; }
}

// entries {u64 iid, [u64 pid,] Value}* of an ACCEPT / COMMIT / P_BATCH /
// PREPARE_REPLY body, sorted by iid (the reference's std::map order)
static int decode_entries(ValueTable &vt, const uint8_t *b, size_t len, bool with_pid,
                          std::vector<uint64_t> &iid, std::vector<uint64_t> &pid,
                          std::vector<uint64_t> &val, size_t &n_all, bool &dup)
{
    size_t cur = 0;
    const size_t first = iid.size();
    n_all = 0;
    while (cur < len) {
        const size_t need = with_pid ? 16 : 8;
        if (len - cur < need) return MPX_E_DECODE;
        const uint64_t i = rd64(b + cur);
        const uint64_t pd = with_pid ? rd64(b + cur + 8) : 0;
        cur += need;
        uint64_t h;
        const long u = vt.parse(b + cur, len - cur, &h);
        if (u < 0) return (int)u;
        cur += (size_t)u;
        iid.push_back(i);
        if (with_pid) pid.push_back(pd);
        val.push_back(h);
        ++n_all;
    }
    // sort this message's entries by iid (stable permutation)
    const size_t n = iid.size() - first;
    bool sorted = true;
    for (size_t k = first + 1; k < iid.size(); ++k)
        if (iid[k - 1] >= iid[k]) { sorted = false; break; }
    dup = false;
    if (!sorted) {
        std::vector<size_t> perm(n);
        for (size_t k = 0; k < n; ++k) perm[k] = first + k;
        std::stable_sort(perm.begin(), perm.end(), [&](size_t a, size_t c) { return iid[a] < iid[c]; });
        std::vector<uint64_t> ti(n), tp(with_pid ? n : 0), tv(n);
        for (size_t k = 0; k < n; ++k) {
            ti[k] = iid[perm[k]]; tv[k] = val[perm[k]];
            if (with_pid) tp[k] = pid[perm[k]];
        }
        for (size_t k = 0; k < n; ++k) {
            iid[first + k] = ti[k]; val[first + k] = tv[k];
            if (with_pid) pid[first + k] = tp[k];
        }
        for (size_t k = first + 1; k < iid.size(); ++k)
            if (iid[k - 1] == iid[k]) dup = true;
    }
    return MPX_OK;
}

int decode_record(ValueTable &vt, NodeStream &ns, uint32_t node, uint32_t N, const uint8_t *m, size_t len,
                  uint64_t sb, uint64_t se, IngestViolation &viol)
{
    if (len < 4) return MPX_E_DECODE;
    const uint32_t t = rd32(m);
    const uint64_t seq = ns.type.size();
    uint32_t src = 0;
    uint64_t ballot = 0, aux = 0, ent = 0;
    uint32_t cnt = 0;
    (void)N;
    auto keep_shard = [&](std::vector<uint64_t> &iid, std::vector<uint64_t> *pid, std::vector<uint64_t> &val,
                          size_t first) {
        // drop entries outside this engine's shard (headers stay: SURVEY §8(e))
        size_t w = first;
        for (size_t k = first; k < iid.size(); ++k) {
            if (iid[k] >= sb && iid[k] < se) {
                iid[w] = iid[k]; val[w] = val[k];
                if (pid) (*pid)[w] = (*pid)[k];
                ++w;
            }
        }
        iid.resize(w); val.resize(w);
        if (pid) pid->resize(w);
        return w - first;
    };
    switch (t) {
    case MPX_MSG_PREPARE: {                       // multi/paxos.cpp:741-755
        if (len < 20) return MPX_E_DECODE;
        src = rd32(m + 4); ballot = rd64(m + 8);
        const uint32_t rl = rd32(m + 16);
        if (rl % 16 || 20 + (size_t)rl > len) return MPX_E_DECODE;
        ent = ns.g_a.size();
        const uint32_t nr = rl / 16;
        std::vector<std::pair<uint64_t, uint64_t>> r(nr);
        for (uint32_t k = 0; k < nr; ++k) r[k] = {rd64(m + 20 + 16 * k), rd64(m + 28 + 16 * k)};
        std::sort(r.begin(), r.end());            // std::set order (:533-537)
        // The kernel binary-searches disjoint ranges: drop empty ones and
        // merge overlaps (the reference returns an entry once per covering
        // range and ASSERTs on the duplicate, :909; a repeated pair is an
        // ASSERT in ExtractAvailableInstanceIDs, :536).
        cnt = 0;
        for (uint32_t k = 0; k < nr; ++k) {
            if (k && r[k] == r[k - 1]) flag(viol, MPX_V_DUP_IID, node, seq, r[k].first);
            if (r[k].first >= r[k].second) continue;
            if (cnt && r[k].first < ns.g_b.back()) {
                ns.g_b.back() = std::max(ns.g_b.back(), r[k].second);
                continue;
            }
            ns.g_a.push_back(r[k].first);
            ns.g_b.push_back(r[k].second);
            ++cnt;
        }
        break;
    }
    case MPX_MSG_PREPARE_REPLY: {                 // :830-844
        if (len < 20) return MPX_E_DECODE;
        src = rd32(m + 4); ballot = rd64(m + 8);
        const uint32_t vl = rd32(m + 16);
        if (20 + (size_t)vl > len) return MPX_E_DECODE;
        const size_t first = ns.r_iid.size();
        size_t n_all; bool dup;
        int rc = decode_entries(vt, m + 20, vl, true, ns.r_iid, ns.r_pid, ns.r_val, n_all, dup);
        if (rc) return rc;
        if (dup) flag(viol, MPX_V_DUP_IID, node, seq, 0);
        ent = first;
        cnt = (uint32_t)keep_shard(ns.r_iid, &ns.r_pid, ns.r_val, first);
        break;
    }
    case MPX_MSG_REJECT:                          // :846-856
        if (len < 12) return MPX_E_DECODE;
        ballot = rd64(m + 4);
        break;
    case MPX_MSG_ACCEPT:                          // :1282-1297
    case MPX_MSG_COMMIT: {                        // :1429-1444
        if (len < 28) return MPX_E_DECODE;
        src = rd32(m + 4); aux = rd64(m + 8); ballot = rd64(m + 16);
        const uint32_t vl = rd32(m + 24);
        if (28 + (size_t)vl > len) return MPX_E_DECODE;
        const size_t first = ns.e_iid.size();
        size_t n_all; bool dup;
        std::vector<uint64_t> nopid;
        int rc = decode_entries(vt, m + 28, vl, false, ns.e_iid, nopid, ns.e_val, n_all, dup);
        if (rc) return rc;
        if (dup) flag(viol, MPX_V_DUP_IID, node, seq, 0);
        ent = first;
        cnt = (uint32_t)keep_shard(ns.e_iid, nullptr, ns.e_val, first);
        break;
    }
    case MPX_MSG_ACCEPT_REPLY:                    // :1345-1357
        if (len < 24) return MPX_E_DECODE;
        src = rd32(m + 4); ballot = rd64(m + 8); aux = rd64(m + 16);
        break;
    case MPX_MSG_COMMIT_REPLY:                    // :1481-1492
        if (len < 16) return MPX_E_DECODE;
        src = rd32(m + 4); aux = rd64(m + 8);
        break;
    case MPX_MSG_P_START:
        if (len < 12) return MPX_E_DECODE;
        ballot = rd64(m + 4);
        break;
    case MPX_MSG_P_BATCH: {
        if (len < 16) return MPX_E_DECODE;
        aux = rd64(m + 4);
        const uint32_t vl = rd32(m + 12);
        if (16 + (size_t)vl > len) return MPX_E_DECODE;
        const size_t first = ns.e_iid.size();
        size_t n_all; bool dup;
        std::vector<uint64_t> nopid;
        int rc = decode_entries(vt, m + 16, vl, false, ns.e_iid, nopid, ns.e_val, n_all, dup);
        if (rc) return rc;
        if (dup) flag(viol, MPX_V_DUP_IID, node, seq, 0);
        ent = first;
        cnt = (uint32_t)keep_shard(ns.e_iid, nullptr, ns.e_val, first);
        break;
    }
    default:
        return MPX_E_DECODE;                      // ASSERT(false), :1671-1672
    }
    ns.type.push_back((uint8_t)t);
    ns.src.push_back(src);
    ns.ballot.push_back(ballot);
    ns.aux.push_back(aux);
    ns.ent.push_back(ent);
    ns.cnt.push_back(cnt);
    return MPX_OK;
}

// Cut entries [first, first+count) of one message (sorted by iid, inside the
// shard) into per-bucket runs.
template <typename F>
static void cut_runs(const uint64_t *iid, uint64_t first, uint32_t count, uint64_t sb, F &&emit)
{
    uint32_t k = 0;
    while (k < count) {
        const uint64_t b = (iid[first + k] - sb) >> BSH;
        uint32_t e = k + 1;
        while (e < count && ((iid[first + e] - sb) >> BSH) == b) ++e;
        bool dense = true;
        for (uint32_t j = k + 1; j < e; ++j)
            if (iid[first + j] != iid[first + j - 1] + 1) { dense = false; break; }
        emit(b, first + k, e - k, (uint8_t)((iid[first + k] - sb) & (BS - 1)), dense);
        k = e;
    }
}

int build_trace(const std::vector<NodeStream> &nodes, uint64_t sb, uint64_t slen, HostTrace &ht)
{
    ht = HostTrace();
    const uint32_t N = (uint32_t)nodes.size();
    ht.N = N;
    ht.shard_begin = sb;
    ht.shard_len = slen;
    ht.NB = (uint32_t)((slen + BS - 1) >> BSH);
    const uint64_t NB = ht.NB;
    uint64_t G = 0, E = 0, R = 0, GR = 0;
    for (auto &ns : nodes) { G += ns.type.size(); E += ns.e_iid.size(); R += ns.r_iid.size(); GR += ns.g_a.size(); }
    if (G >= NONE32) return MPX_E_RANGE;
    ht.m_type.reserve(G); ht.m_src.reserve(G); ht.m_cnt.reserve(G); ht.m_node.reserve(G);
    ht.m_ballot.reserve(G); ht.m_aux.reserve(G); ht.m_ent.reserve(G);
    ht.e_val.reserve(E); ht.e_iid.reserve(E); ht.r_pid.reserve(R); ht.r_val.reserve(R); ht.r_iid.reserve(R);
    ht.g_a.reserve(GR); ht.g_b.reserve(GR);
    ht.node_off.assign(N + 1, 0);
    ht.n_after_prepare.assign(N, 0);

    struct FragKey { uint64_t key; Frag f; };
    std::vector<uint64_t> fcount(N * NB + 1, 0), cfcount(NB + 1, 0);
    std::vector<FragKey> fr, cfr;
    std::vector<uint32_t> ev, pl;
    std::vector<uint64_t> ev_cnt(N, 0), pl_cnt(N, 0);

    for (uint32_t n = 0; n < N; ++n) {
        const NodeStream &ns = nodes[n];
        ht.node_off[n] = ht.m_type.size();
        const uint64_t ebase = ht.e_val.size(), rbase = ht.r_val.size(), gbase = ht.g_a.size();
        ht.e_val.insert(ht.e_val.end(), ns.e_val.begin(), ns.e_val.end());
        ht.e_iid.insert(ht.e_iid.end(), ns.e_iid.begin(), ns.e_iid.end());
        ht.r_pid.insert(ht.r_pid.end(), ns.r_pid.begin(), ns.r_pid.end());
        ht.r_val.insert(ht.r_val.end(), ns.r_val.begin(), ns.r_val.end());
        ht.r_iid.insert(ht.r_iid.end(), ns.r_iid.begin(), ns.r_iid.end());
        ht.g_a.insert(ht.g_a.end(), ns.g_a.begin(), ns.g_a.end());
        ht.g_b.insert(ht.g_b.end(), ns.g_b.begin(), ns.g_b.end());
        uint32_t pstart = NONE32;                       // epoch of the batches that follow
        for (size_t k = 0; k < ns.type.size(); ++k) {
            const uint32_t g = (uint32_t)ht.m_type.size();
            const uint8_t t = ns.type[k];
            uint64_t ent = ns.ent[k];
            if (t == MPX_MSG_PREPARE) ent += gbase;
            else if (t == MPX_MSG_PREPARE_REPLY) ent += rbase;
            else if (t == MPX_MSG_ACCEPT || t == MPX_MSG_COMMIT || t == MPX_MSG_P_BATCH) ent += ebase;
            ht.m_type.push_back(t);
            ht.m_src.push_back(ns.src[k]);
            ht.m_ballot.push_back(ns.ballot[k]);
            ht.m_aux.push_back(ns.aux[k]);
            ht.m_ent.push_back(ent);
            ht.m_cnt.push_back(ns.cnt[k]);
            ht.m_node.push_back(n);
            if (t == MPX_MSG_PREPARE || t == MPX_MSG_PREPARE_REPLY || t == MPX_MSG_P_START) { ev.push_back(g); ev_cnt[n]++; }
            if (t == MPX_MSG_PREPARE) ht.n_after_prepare[n] = g + 1;
            if (t == MPX_MSG_PREPARE_REPLY || t == MPX_MSG_P_START) { pl.push_back(g); pl_cnt[n]++; }
            if (t == MPX_MSG_P_START) pstart = g;
            if (t == MPX_MSG_P_BATCH) {
                ht.b_msg.push_back(g);
                ht.b_pstart.push_back(pstart);
            }
            if (t == MPX_MSG_ACCEPT || t == MPX_MSG_COMMIT || t == MPX_MSG_PREPARE_REPLY) {
                const uint8_t kind = t == MPX_MSG_ACCEPT ? K_ACCEPT : t == MPX_MSG_COMMIT ? K_COMMIT : K_PREPLY;
                const uint64_t *iid = t == MPX_MSG_PREPARE_REPLY ? ht.r_iid.data() : ht.e_iid.data();
                cut_runs(iid, ent, ns.cnt[k], sb, [&](uint64_t b, uint64_t e0, uint32_t c, uint8_t st, bool dense) {
                    Frag f{e0, g, (uint16_t)c, st, (uint8_t)((dense ? FR_DENSE : 0) | (kind << 4))};
                    if (!dense) ht.any_sparse = true;
                    fr.push_back({(uint64_t)n * NB + b, f});
                    fcount[(uint64_t)n * NB + b]++;
                });
            }
            if (t == MPX_MSG_P_BATCH) {
                const uint32_t j = (uint32_t)ht.b_msg.size() - 1;
                cut_runs(ht.e_iid.data(), ent, ns.cnt[k], sb, [&](uint64_t b, uint64_t e0, uint32_t c, uint8_t st, bool dense) {
                    Frag f{e0, j, (uint16_t)c, st, (uint8_t)((dense ? FR_DENSE : 0) | (K_BATCH << 4))};
                    if (!dense) ht.any_sparse = true;
                    cfr.push_back({b, f});
                    cfcount[b]++;
                });
            }
        }
    }
    ht.node_off[N] = ht.m_type.size();

    // vote lists: replies attributed to the live batch of the same id, same epoch
    {
        std::vector<std::vector<uint32_t>> reps(ht.b_msg.size());
        for (uint32_t n = 0; n < N; ++n) {
            std::unordered_map<uint64_t, uint32_t> live;
            uint32_t j = 0;
            // batches of node n are contiguous in b_msg, in message order
            while (j < ht.b_msg.size() && ht.m_node[ht.b_msg[j]] < n) ++j;
            uint32_t jn = j;
            for (uint64_t g = ht.node_off[n]; g < ht.node_off[n + 1]; ++g) {
                const uint8_t t = ht.m_type[g];
                if (t == MPX_MSG_P_START) live.clear();
                else if (t == MPX_MSG_P_BATCH) live[ht.m_aux[g]] = jn++;
                else if (t == MPX_MSG_ACCEPT_REPLY) {
                    auto it = live.find(ht.m_aux[g]);
                    if (it != live.end()) reps[it->second].push_back((uint32_t)g);
                }
            }
        }
        ht.b_rep_off.assign(ht.b_msg.size() + 1, 0);
        for (size_t j = 0; j < reps.size(); ++j) ht.b_rep_off[j + 1] = ht.b_rep_off[j] + reps[j].size();
        ht.b_rep.reserve(ht.b_rep_off.back());
        for (auto &r : reps) ht.b_rep.insert(ht.b_rep.end(), r.begin(), r.end());
    }

    // fragment CSR per (node, bucket), stable (keeps message order)
    ht.f_off.assign(N * NB + 1, 0);
    for (uint64_t i = 0; i < N * NB; ++i) ht.f_off[i + 1] = ht.f_off[i] + fcount[i];
    ht.frags.resize(fr.size());
    {
        std::vector<uint64_t> pos(ht.f_off.begin(), ht.f_off.end() - 1);
        for (auto &x : fr) ht.frags[pos[x.key]++] = x.f;
    }
    ht.cf_off.assign(NB + 1, 0);
    for (uint64_t i = 0; i < NB; ++i) ht.cf_off[i + 1] = ht.cf_off[i] + cfcount[i];
    ht.cfrags.resize(cfr.size());
    {
        std::vector<uint64_t> pos(ht.cf_off.begin(), ht.cf_off.end() - 1);
        for (auto &x : cfr) ht.cfrags[pos[x.key]++] = x.f;
    }
    // pairs the lean dense kernel cannot take (same predicate as pair_is_fast
    // in kernels.hip): they go to the general kernel's work list
    for (uint32_t n = 0; n < N; ++n)
        for (uint64_t b = 0; b < NB; ++b) {
            const uint64_t p = (uint64_t)n * NB + b, f0 = ht.f_off[p], nf = ht.f_off[p + 1] - f0;
            if (!nf) continue;
            bool fast = nf <= 64 && ht.frags[f0].msg >= ht.n_after_prepare[n];
            for (uint64_t f = f0; fast && f < f0 + nf; ++f) {
                const uint8_t fl = ht.frags[f].flags;
                fast = (fl & FR_DENSE) && ((fl >> 4) == K_ACCEPT || (fl >> 4) == K_COMMIT);
            }
            if (!fast) ht.gp_list.push_back(p);
        }
    // slots for sparse fragments
    if (ht.any_sparse) {
        ht.e_slot.resize(ht.e_iid.size());
        for (size_t k = 0; k < ht.e_iid.size(); ++k) ht.e_slot[k] = (uint8_t)((ht.e_iid[k] - sb) & (BS - 1));
        ht.r_slot.resize(ht.r_iid.size());
        for (size_t k = 0; k < ht.r_iid.size(); ++k) ht.r_slot[k] = (uint8_t)((ht.r_iid[k] - sb) & (BS - 1));
    }
    // event / proposer lists
    ht.ev_off.assign(N + 1, 0);
    ht.pl_off.assign(N + 1, 0);
    for (uint32_t n = 0; n < N; ++n) { ht.ev_off[n + 1] = ht.ev_off[n] + ev_cnt[n]; ht.pl_off[n + 1] = ht.pl_off[n] + pl_cnt[n]; }
    ht.ev_msg = std::move(ev);
    ht.pl_msg = std::move(pl);
    // header-scan chunks
    ht.node_chunk_off.assign(N + 1, 0);
    for (uint32_t n = 0; n < N; ++n) {
        ht.node_chunk_off[n] = (uint32_t)ht.chunk_node.size();
        for (uint64_t g = ht.node_off[n]; g < ht.node_off[n + 1]; g += SCAN_CHUNK) {
            ht.chunk_node.push_back(n);
            ht.chunk_beg.push_back(g);
            ht.chunk_end.push_back(std::min<uint64_t>(g + SCAN_CHUNK, ht.node_off[n + 1]));
        }
    }
    ht.node_chunk_off[N] = (uint32_t)ht.chunk_node.size();
    return MPX_OK;
}

}  // namespace mpx
