// epoch_learn_check.cpp — host-only check of MPX_FLAG_LEARN_EPOCHS (ingest.cpp EpochLearn), built by
// tests/test_ingest_cpu.py with g++ against the engine's own ingest and generator sources (no GPU).
//   epoch_learn_check <trace.mpxt> [windows]
//   epoch_learn_check gen <log2 instances> <proposers> [windows]
// Each node's stream is decoded twice: as submitted (the trace's E_EPOCH markers, which the
// reference driver checks against the reference's own ChangeMemberships, oracle/ref_member_driver.cpp)
// and with an EpochLearn from the genesis epoch, fed in `windows` slices (the learner state carries
// over, as across MPX_FLAG_INCREMENTAL windows).  The learned run must place the same E_EPOCH
// records at the same stream positions with the same epochs, and the epochs it learned must be the
// container's table.  The learned pass runs skimming every value section and copying every
// section's decode (SectionCache).
// Prints "ok <records> <markers> <epochs>" or the first difference.
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

static bool same(const mpx_epoch &a, const mpx_epoch &b)
{
    return a.version == b.version && a.acceptor_mask == b.acceptor_mask && a.proposer_mask == b.proposer_mask &&
           a.learner_mask == b.learner_mask;
}

int main(int argc, char **argv)
{
    if (argc < 2) { std::printf("usage\n"); return 2; }
    std::string t;
    uint32_t W = 1;
    if (!std::strcmp(argv[1], "gen")) {
        mpx_gen_params p{};
        p.kind = MPX_GEN_MEMBER; p.num_nodes = 8; p.batch = 256; p.drop_rate = 100; p.dup_rate = 100;
        p.max_delay = 64; p.noop_permille = 15;
        p.num_instances = 1ull << (argc > 2 ? std::atoi(argv[2]) : 14);
        p.proposers = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 0;
        W = argc > 4 ? (uint32_t)std::atoi(argv[4]) : 1;
        if (gen_member(p, t)) { std::printf("FAIL gen\n"); return 1; }
    } else {
        std::ifstream f(argv[1], std::ios::binary);
        t.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
        W = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 1;
    }
    const uint8_t *b = (const uint8_t *)t.data();
    if (t.size() < 40 || rd32(b + 12) != MPX_SEM_MEMBER) { std::printf("FAIL not a member trace\n"); return 1; }
    const uint32_t N = rd32(b + 8), ne = rd32(b + 24);
    const uint64_t M = rd64(b + 16);
    const size_t esz = rd32(b + 4) == 1 ? 24 : 32;
    std::vector<mpx_epoch> ep(ne);
    for (uint32_t k = 0; k < ne; ++k) {
        const uint8_t *x = b + 40 + k * esz;
        ep[k] = mpx_epoch{rd32(x), 0, rd64(x + 8), rd64(x + 16), esz == 32 ? rd64(x + 24) : rd64(x + 16)};
    }
    size_t pos = 40 + (size_t)ne * esz;
    uint64_t records = 0, markers = 0;
    std::vector<mpx_epoch> learned(1, ep[0]);
    for (uint32_t n = 0; n < N; ++n) {
        const uint64_t cnt = rd64(b + pos), nb = rd64(b + pos + 8);
        const uint64_t *offs = reinterpret_cast<const uint64_t *>(b + pos + 16);
        const uint8_t *bytes = b + pos + 16 + 8 * (cnt + 1);
        NodeStream as_is;
        ValueTable v1;
        v1.member = true;
        IngestViolation iv;
        for (uint64_t i = 0; i < cnt; ++i)
            if (int rc = decode_record_member(v1, as_is, n, bytes + offs[i], offs[i + 1] - offs[i], 0, M, iv)) {
                std::printf("FAIL decode rc %d\n", rc); return 1;
            }
        // the learned pass twice: once skimming every value section (as a decode thread does when
        // another thread claimed the section and has not decoded it yet: its table stays empty, so
        // the learner must read membership changes off the wire), once copying every section from
        // another decode's Result (SectionCache, the membership Values' wire offsets with it)
        for (int share = 0; share < 2; ++share) {
        NodeStream got;
        ValueTable v2;
        v2.member = true;
        EpochLearn el;
        el.view = ep[0];
        SectionCache sc;
        sc.share = share != 0;
        {
            NodeStream sink;
            ValueTable v3;
            v3.member = true;
            for (uint64_t i = 0; i < cnt; ++i)
                decode_record_member(v3, sink, n, bytes + offs[i], offs[i + 1] - offs[i], 0, M, iv, nullptr, &sc);
        }
        for (uint32_t w = 0; w < W; ++w) {                   // windows: the learner state carries over
            NodeStream part;
            for (uint64_t i = cnt * w / W; i < cnt * (w + 1) / W; ++i)
                if (int rc = decode_record_member(v2, part, n, bytes + offs[i], offs[i + 1] - offs[i], 0, M, iv, &el, &sc)) {
                    std::printf("FAIL learned decode rc %d node %u record %llu\n", rc, n, (unsigned long long)i);
                    return 1;
                }
            got.type.insert(got.type.end(), part.type.begin(), part.type.end());
            got.ver.insert(got.ver.end(), part.ver.begin(), part.ver.end());
        }
        if (got.type.size() != as_is.type.size()) {
            std::printf("FAIL node %u: %zu records learned, %zu submitted\n", n, got.type.size(), as_is.type.size());
            for (size_t k = 0, j = 0; k < as_is.type.size() && j < got.type.size(); ++k, ++j)
                if (as_is.type[k] != got.type[j]) { std::printf("  first difference at record %zu\n", k); break; }
            return 1;
        }
        for (size_t k = 0; k < got.type.size(); ++k) {
            if (got.type[k] != as_is.type[k] || (got.type[k] == MPX_MSG_E_EPOCH && got.ver[k] != as_is.ver[k])) {
                std::printf("FAIL node %u record %zu: type %u epoch %u learned, type %u epoch %u submitted\n", n, k,
                            got.type[k], got.ver[k], as_is.type[k], as_is.ver[k]);
                return 1;
            }
            markers += share && got.type[k] == MPX_MSG_E_EPOCH;
        }
        for (size_t k = 0; k < el.steps.size(); ++k) {
            if (k + 1 < learned.size()) {
                if (!same(learned[k + 1], el.steps[k])) { std::printf("FAIL node %u step %zu disagrees\n", n, k); return 1; }
            } else learned.push_back(el.steps[k]);
        }
        }
        records += cnt;
        pos += 16 + 8 * (cnt + 1) + nb;
        pos = (pos + 7) & ~(size_t)7;
    }
    // the container's table may hold epochs no node reached; every learned one must be in it, in order
    if (learned.size() > ep.size()) { std::printf("FAIL %zu epochs learned, %u in the table\n", learned.size(), ne); return 1; }
    for (size_t k = 0; k < learned.size(); ++k)
        if (!same(learned[k], ep[k])) { std::printf("FAIL epoch %zu differs from the table\n", k); return 1; }
    std::printf("ok %llu %llu %zu\n", (unsigned long long)records, (unsigned long long)markers, learned.size());
    return 0;
}
