// build_check.cpp — host-only check that build_trace (the node-parallel walk) gives
// build_trace_serial's HostTrace field for field, whole and window by window (the WindowCarry too),
// built by tests/test_ingest_cpu.py against the engine's own ingest and generator sources (no GPU).
//   build_check <trace.mpxt | faulty | member> [log2 instances] [proposers] [windows] [threads] [shard 0|1]
// shard 1: the engine's shard is the middle half of the instances (header sharding: left-out
// records, partial entry lists).  Prints "ok <windows> <messages> <runs>" or the first difference.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "gen.hpp"
#include "ingest.hpp"

using namespace mpx;

static uint32_t rd32(const uint8_t *p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
static uint64_t rd64(const uint8_t *p) { uint64_t v; std::memcpy(&v, p, 8); return v; }

static bool bad = false;
template <typename V> static void cmp(const char *what, const V &a, const V &b)
{
    if (bad || a == b) return;
    bad = true;
    size_t k = 0;
    while (k < a.size() && k < b.size() && a[k] == b[k]) ++k;
    std::printf("FAIL %s: sizes %zu / %zu, first difference at %zu\n", what, a.size(), b.size(), k);
}
static void cmpf(const char *what, const std::vector<Frag> &a, const std::vector<Frag> &b)
{
    if (bad) return;
    if (a.size() != b.size() || (a.size() && std::memcmp(a.data(), b.data(), a.size() * sizeof(Frag)))) {
        bad = true;
        size_t k = 0;
        while (k < a.size() && k < b.size() && !std::memcmp(&a[k], &b[k], sizeof(Frag))) ++k;
        std::printf("FAIL %s: sizes %zu / %zu, first difference at %zu\n", what, a.size(), b.size(), k);
    }
}
template <typename T> static void cmps(const char *what, T a, T b)
{
    if (bad || a == b) return;
    bad = true;
    std::printf("FAIL %s: %llu / %llu\n", what, (unsigned long long)a, (unsigned long long)b);
}

static void compare(const HostTrace &a, const HostTrace &b)
{
#define C(x) cmp(#x, a.x, b.x)
    cmps("N", a.N, b.N); cmps("NB", a.NB, b.NB); cmps("dropped", a.dropped, b.dropped);
    cmps("part_dropped", a.part_dropped, b.part_dropped); cmps("scan_chunk", a.scan_chunk, b.scan_chunk);
    cmps("any_sparse", a.any_sparse, b.any_sparse); cmps("num_gp_simple", a.num_gp_simple, b.num_gp_simple);
    cmps("num_gp_snap", a.num_gp_snap, b.num_gp_snap);
    C(m_type); C(m_src); C(m_cnt); C(m_node); C(m_ballot); C(m_aux); C(m_ent); C(node_off); C(m_seq);
    C(prop_off); C(prop_seq); C(chunk_node); C(node_chunk_off); C(chunk_beg); C(chunk_end);
    C(sc_type); C(sc_key); C(sc_idx); C(m_flags0); C(m_ver); C(ee_msg); C(sc_ver); C(ee_off); C(sc_off);
    C(e_val); C(e_iid); C(e_pid); C(r_pid); C(r_val); C(r_iid); C(g_a); C(g_b); C(e_slot); C(r_slot);
    C(f_off); C(gp_list); C(ev_off); C(pl_off); C(ev_msg); C(pl_msg); C(ev_aux); C(pair_ev); C(pair_gp);
    C(b_msg); C(b_pstart); C(b_rep); C(b_rsrc); C(b_rbal); C(b_bal); C(b_aid); C(b_rep_off); C(cf_off);
    C(b_gid); C(b_node); C(gp_base); C(cb_list); C(f_pid);
    cmpf("frags", a.frags, b.frags); cmpf("cfrags", a.cfrags, b.cfrags);
#undef C
}

static void compare(const WindowCarry &a, const WindowCarry &b)
{
    cmps("wc.batches", a.batches, b.batches);
    if (!bad && a.live != b.live) { bad = true; std::printf("FAIL wc.live\n"); }
    cmp("wc.round_ballot", a.round_ballot, b.round_ballot);
    if (!bad && a.state_b != b.state_b) { bad = true; std::printf("FAIL wc.state_b\n"); }
    cmp("wc.maxb", a.maxb, b.maxb);
    if (!bad && a.round_b != b.round_b) { bad = true; std::printf("FAIL wc.round_b\n"); }
    cmp("wc.b_bal", a.b_bal, b.b_bal); cmp("wc.b_aid", a.b_aid, b.b_aid); cmp("wc.markers", a.markers, b.markers);
    if (!bad && a.b_ents != b.b_ents) { bad = true; std::printf("FAIL wc.b_ents\n"); }
}

int main(int argc, char **argv)
{
    if (argc < 2) { std::printf("usage\n"); return 2; }
    std::string t;
    const uint32_t lg = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 14;
    const uint32_t props = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 0;
    const uint32_t W = argc > 4 ? (uint32_t)std::max(1, std::atoi(argv[4])) : 1;
    const uint32_t threads = argc > 5 ? (uint32_t)std::atoi(argv[5]) : 4;
    const bool shard = argc > 6 && std::atoi(argv[6]) != 0;
    mpx_gen_params p{};
    p.num_instances = 1ull << lg; p.batch = 256; p.proposers = props;
    if (!std::strcmp(argv[1], "faulty")) {
        p.kind = MPX_GEN_FAULTY; p.num_nodes = 7; p.drop_rate = 500; p.dup_rate = 1000; p.max_delay = 500;
        if (gen_faulty(p, t)) { std::printf("FAIL gen\n"); return 1; }
    } else if (!std::strcmp(argv[1], "member")) {
        p.kind = MPX_GEN_MEMBER; p.num_nodes = 8; p.drop_rate = 100; p.dup_rate = 100; p.max_delay = 64; p.noop_permille = 15;
        if (gen_member(p, t)) { std::printf("FAIL gen\n"); return 1; }
    } else {
        std::ifstream f(argv[1], std::ios::binary);
        t.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    }
    const uint8_t *b = (const uint8_t *)t.data();
    if (t.size() < 40) { std::printf("FAIL short trace\n"); return 1; }
    const uint32_t N = rd32(b + 8), ne = rd32(b + 24);
    const bool member = rd32(b + 12) == MPX_SEM_MEMBER;
    const uint64_t M = std::max<uint64_t>(rd64(b + 16), 1);
    const size_t esz = rd32(b + 4) == 1 ? 24 : 32;
    std::vector<mpx_epoch> ep(ne);
    for (uint32_t k = 0; k < ne; ++k) {
        std::memcpy(&ep[k], b + 40 + k * esz, 24);
        ep[k].learner_mask = esz == 32 ? rd64(b + 40 + k * esz + 24) : ep[k].proposer_mask;
    }
    if (member && ep.empty()) { std::printf("ok-skip no epochs\n"); return 0; }
    const uint64_t sb = shard ? M / 4 : 0, se = shard ? M - M / 4 : M;
    size_t pos = 40 + (size_t)ne * esz;
    std::vector<StreamSlice> all(N);
    for (uint32_t n = 0; n < N; ++n) {
        const uint64_t cnt = rd64(b + pos), nb = rd64(b + pos + 8);
        all[n] = StreamSlice{reinterpret_cast<const uint64_t *>(b + pos + 16), b + pos + 16 + 8 * (cnt + 1), cnt};
        pos = (pos + 16 + 8 * (cnt + 1) + nb + 7) & ~(size_t)7;
    }
    ValueTable vt;
    vt.member = member;
    IngestViolation iv;
    WindowCarry wa, wb;
    const uint64_t NB = (se - sb + BS - 1) / BS;
    if (W > 1) { wa.init(N, NB); wb.init(N, NB); }
    uint64_t msgs = 0, runs = 0;
    for (uint32_t w = 0; w < W; ++w) {
        // (decode_parallel: the records carry their value sections' ids, which the parallel build's
        // entry pool takes as equality; the serial build compares every list)
        std::vector<NodeStream> nodes(N), parts;
        std::vector<StreamSlice> sl(N);
        for (uint32_t n = 0; n < N; ++n) {
            const uint64_t k0 = all[n].cnt * w / W, k1 = all[n].cnt * (w + 1) / W;
            sl[n] = StreamSlice{all[n].offs + k0, all[n].bytes, k1 - k0};
        }
        if (int rc = decode_parallel(vt, nodes, parts, sl, member, nullptr, sb, se, iv, 3, 4096)) {
            std::printf("ok-decode-error %d\n", rc);
            return 0;
        }
        HostTrace ha, hb;
        const std::vector<mpx_epoch> e = member ? ep : std::vector<mpx_epoch>();
        const int ra = build_trace_serial(nodes, sb, se - sb, e, ha, W > 1 ? &wa : nullptr);
        const int rb = build_trace(nodes, sb, se - sb, e, hb, W > 1 ? &wb : nullptr, threads);
        if (ra != rb) { std::printf("FAIL window %u: rc %d serial, %d parallel\n", w, ra, rb); return 1; }
        if (ra) { std::printf("ok-error %d\n", ra); return 0; }
        compare(ha, hb);
        if (W > 1) compare(wa, wb);
        if (bad) { std::printf("  (window %u)\n", w); return 1; }
        msgs += ha.m_type.size();
        runs += ha.frags.size();
    }
    std::printf("ok %u %llu %llu\n", W, (unsigned long long)msgs, (unsigned long long)runs);
    return 0;
}
