// parallel_decode_check.cpp — host-only check of ingest.cpp decode_parallel (submit_container's
// chunked, thread-pooled decode), built by tests/test_ingest_cpu.py against the engine's own ingest
// and generator sources (no GPU).
//   parallel_decode_check <trace.mpxt | faulty | member> [log2 instances] [proposers] [chunk bytes] [threads]
// Every node's stream is decoded twice: serially, record by record (decode_record /
// decode_record_member, one value table, no section claims), and — after the same first third of
// every stream decoded serially, so chunks append to streams that already hold records — by
// decode_parallel with small chunks on several threads.  The two must agree array for array
// (records, their entry offsets, entries, ranges) and on the violations (first code, node, record
// index, count).  Prints "ok <records> <chunks-per-node>" or the first difference.
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

template <typename V> static bool same(const char *what, uint32_t n, const V &a, const V &b)
{
    if (a == b) return true;
    size_t k = 0;
    while (k < a.size() && k < b.size() && a[k] == b[k]) ++k;
    std::printf("FAIL node %u %s: sizes %zu / %zu, first difference at %zu\n", n, what, a.size(), b.size(), k);
    return false;
}

int main(int argc, char **argv)
{
    if (argc < 2) { std::printf("usage\n"); return 2; }
    std::string t;
    const uint32_t lg = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 14;
    const uint32_t props = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 0;
    const uint64_t chunk = argc > 4 ? std::strtoull(argv[4], nullptr, 10) : 4096;
    const uint32_t threads = argc > 5 ? (uint32_t)std::atoi(argv[5]) : 5;
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
    const uint64_t M = rd64(b + 16);
    size_t pos = 40 + (size_t)ne * (rd32(b + 4) == 1 ? 24 : 32);
    std::vector<StreamSlice> all(N), rest(N);
    std::vector<NodeStream> serial(N), par(N), parts;
    ValueTable v1, v2;
    v1.member = v2.member = member;
    IngestViolation iv1, iv2;
    uint64_t records = 0;
    for (uint32_t n = 0; n < N; ++n) {
        const uint64_t cnt = rd64(b + pos), nb = rd64(b + pos + 8);
        all[n].offs = reinterpret_cast<const uint64_t *>(b + pos + 16);
        all[n].bytes = b + pos + 16 + 8 * (cnt + 1);
        all[n].cnt = cnt;
        records += cnt;
        pos = (pos + 16 + 8 * (cnt + 1) + nb + 7) & ~(size_t)7;
    }
    auto dec = [&](ValueTable &vt, NodeStream &ns, uint32_t n, uint64_t k, IngestViolation &iv) {
        const StreamSlice &x = all[n];
        const uint8_t *m = x.bytes + x.offs[k];
        const size_t len = x.offs[k + 1] - x.offs[k];
        return member ? decode_record_member(vt, ns, n, m, len, 0, M, iv) : decode_record(vt, ns, n, N, m, len, 0, M, iv);
    };
    int rc1 = 0;
    for (uint32_t n = 0; n < N && !rc1; ++n)
        for (uint64_t k = 0; k < all[n].cnt && !rc1; ++k) rc1 = dec(v1, serial[n], n, k, iv1);
    int rc2 = 0;
    for (uint32_t n = 0; n < N && !rc2; ++n) {
        const uint64_t head = all[n].cnt / 3;
        for (uint64_t k = 0; k < head && !rc2; ++k) rc2 = dec(v2, par[n], n, k, iv2);
        rest[n] = StreamSlice{all[n].offs + head, all[n].bytes, all[n].cnt - head};
    }
    if (!rc2) rc2 = decode_parallel(v2, par, parts, rest, member, nullptr, 0, M, iv2, threads, chunk);
    if (rc1 != rc2) { std::printf("FAIL rc %d serial, %d parallel\n", rc1, rc2); return 1; }
    if (rc1) { std::printf("ok-error %d\n", rc1); return 0; }
    for (uint32_t n = 0; n < N; ++n) {
        const NodeStream &a = serial[n], &c = par[n];
        if (!(same("type", n, a.type, c.type) && same("src", n, a.src, c.src) && same("ballot", n, a.ballot, c.ballot) &&
              same("aux", n, a.aux, c.aux) && same("ent", n, a.ent, c.ent) && same("cnt", n, a.cnt, c.cnt) &&
              same("ver", n, a.ver, c.ver) && same("part", n, a.part, c.part) && same("e_iid", n, a.e_iid, c.e_iid) &&
              same("e_val", n, a.e_val, c.e_val) && same("e_pid", n, a.e_pid, c.e_pid) && same("r_iid", n, a.r_iid, c.r_iid) &&
              same("r_pid", n, a.r_pid, c.r_pid) && same("r_val", n, a.r_val, c.r_val) && same("g_a", n, a.g_a, c.g_a) &&
              same("g_b", n, a.g_b, c.g_b)))
            return 1;
    }
    if (iv1.code != iv2.code || iv1.node != iv2.node || iv1.seq != iv2.seq || iv1.iid != iv2.iid || iv1.count != iv2.count) {
        std::printf("FAIL violations: serial %llu@%llu/%llu x%llu, parallel %llu@%llu/%llu x%llu\n",
                    (unsigned long long)iv1.code, (unsigned long long)iv1.node, (unsigned long long)iv1.seq,
                    (unsigned long long)iv1.count, (unsigned long long)iv2.code, (unsigned long long)iv2.node,
                    (unsigned long long)iv2.seq, (unsigned long long)iv2.count);
        return 1;
    }
    std::printf("ok %llu %zu %llu\n", (unsigned long long)records, parts.size() / std::max(1u, N), (unsigned long long)iv1.count);
    return 0;
}
