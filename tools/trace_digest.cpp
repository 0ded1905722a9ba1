// trace_digest.cpp — a digest of every HostTrace array build_trace produces for a generated trace
// (host only): two builds of ingest.cpp that must lay out the same trace print the same line.
//   trace_digest <faulty|member> <log2 instances> [proposers]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gen.hpp"
#include "ingest.hpp"

using namespace mpx;

static uint32_t rd32(const uint8_t *p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
static uint64_t rd64(const uint8_t *p) { uint64_t v; std::memcpy(&v, p, 8); return v; }

template <class T> static void dg(uint64_t &d, const std::vector<T> &v)
{
    const unsigned char *p = reinterpret_cast<const unsigned char *>(v.data());
    uint64_t h = 0xcbf29ce484222325ull ^ v.size();
    for (size_t i = 0; i < v.size() * sizeof(T); ++i) h = (h ^ p[i]) * 0x100000001b3ull;
    d = (d ^ h) * 0x9E3779B97F4A7C15ull + 1;
}

int main(int argc, char **argv)
{
    const bool member = argc > 1 && !std::strcmp(argv[1], "member");
    const uint32_t lg = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 16;
    mpx_gen_params p{};
    p.num_instances = 1ull << lg;
    if (member) {
        p.kind = MPX_GEN_MEMBER; p.num_nodes = 8; p.batch = 256; p.drop_rate = 100; p.dup_rate = 100;
        p.max_delay = 64; p.noop_permille = 15;
    } else {
        p.kind = MPX_GEN_FAULTY; p.num_nodes = 7; p.batch = 256; p.drop_rate = 500; p.dup_rate = 1000;
        p.max_delay = 500;
    }
    p.proposers = argc > 3 ? (uint32_t)std::atoi(argv[3]) : (member ? 0 : 3);
    std::string t;
    int rc = member ? gen_member(p, t) : gen_faulty(p, t);
    if (rc) { std::printf("FAIL gen rc %d\n", rc); return 1; }
    const uint8_t *b = (const uint8_t *)t.data();
    const uint32_t N = rd32(b + 8), ne = rd32(b + 24);
    const uint64_t M = rd64(b + 16);
    const size_t esz = rd32(b + 4) == 1 ? 24 : 32;
    std::vector<mpx_epoch> ep(ne);
    for (uint32_t k = 0; k < ne; ++k) {
        std::memcpy(&ep[k], b + 40 + k * esz, 24);
        ep[k].learner_mask = esz == 32 ? rd64(b + 40 + k * esz + 24) : ep[k].proposer_mask;
    }
    size_t pos = 40 + (size_t)ne * esz;
    std::vector<NodeStream> nodes(N);
    ValueTable vt;
    vt.member = member;
    IngestViolation iv;
    for (uint32_t n = 0; n < N; ++n) {
        const uint64_t cnt = rd64(b + pos), nb = rd64(b + pos + 8);
        const uint64_t *offs = reinterpret_cast<const uint64_t *>(b + pos + 16);
        const uint8_t *bytes = b + pos + 16 + 8 * (cnt + 1);
        for (uint64_t i = 0; i < cnt; ++i) {
            rc = member ? decode_record_member(vt, nodes[n], n, bytes + offs[i], offs[i + 1] - offs[i], 0, M, iv)
                        : decode_record(vt, nodes[n], n, N, bytes + offs[i], offs[i + 1] - offs[i], 0, M, iv);
            if (rc) { std::printf("FAIL decode rc %d\n", rc); return 1; }
        }
        pos += 16 + 8 * (cnt + 1) + nb;
        pos = (pos + 7) & ~(size_t)7;
    }
    HostTrace h;
    rc = build_trace(nodes, 0, M, member ? ep : std::vector<mpx_epoch>(), h);
    if (rc) { std::printf("FAIL build rc %d\n", rc); return 1; }
    uint64_t d = 0;
    dg(d, h.m_type); dg(d, h.m_src); dg(d, h.m_cnt); dg(d, h.m_node); dg(d, h.m_ballot); dg(d, h.m_aux); dg(d, h.m_ent);
    dg(d, h.node_off); dg(d, h.m_seq); dg(d, h.prop_off); dg(d, h.prop_seq); dg(d, h.chunk_node); dg(d, h.node_chunk_off);
    dg(d, h.chunk_beg); dg(d, h.chunk_end); dg(d, h.sc_type); dg(d, h.sc_key); dg(d, h.sc_idx); dg(d, h.m_flags0);
    dg(d, h.m_ver); dg(d, h.ee_msg); dg(d, h.sc_ver); dg(d, h.ee_off); dg(d, h.sc_off); dg(d, h.e_val); dg(d, h.e_iid);
    dg(d, h.e_pid); dg(d, h.r_pid); dg(d, h.r_val); dg(d, h.r_iid); dg(d, h.g_a); dg(d, h.g_b); dg(d, h.e_slot);
    dg(d, h.r_slot); dg(d, h.f_off); dg(d, h.frags); dg(d, h.gp_list); dg(d, h.ev_off); dg(d, h.pl_off); dg(d, h.ev_msg);
    dg(d, h.pl_msg); dg(d, h.ev_aux); dg(d, h.pair_ev); dg(d, h.pair_gp); dg(d, h.b_msg); dg(d, h.b_pstart); dg(d, h.b_rep);
    dg(d, h.b_rsrc); dg(d, h.b_rbal); dg(d, h.b_bal); dg(d, h.b_aid); dg(d, h.b_rep_off); dg(d, h.cf_off); dg(d, h.cfrags);
    std::printf("digest %016llx simple %llu snap %llu gp %zu e %zu\n", (unsigned long long)d,
                (unsigned long long)h.num_gp_simple, (unsigned long long)h.num_gp_snap, h.gp_list.size(), h.e_iid.size());
    return 0;
}
