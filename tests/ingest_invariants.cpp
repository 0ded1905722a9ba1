// ingest_invariants.cpp — host-only checks of build_trace's bucket-run aliasing and FR_VCHK marks
// (ingest.cpp mark_value_checks), built by tests/test_ingest_cpu.py with g++ against the engine's own
// ingest and generator sources (no GPU).
//   ingest_invariants <faulty|member> <log2 instances> [proposers]
// Checks, for every dense ACCEPT / COMMIT run of every (node, bucket) pair:
//   1. the entries the run names are its message's own (iid, Value, member: proposal id) on every
//      slot it covers — aliasing onto another run's entries never changes what the run says;
//   2. FR_VCHK is set exactly when a commit / learn (member: also an accept) covers a slot an
//      earlier commit / learn of the pair fixed through another entry index holding another Value
//      (the re-commits the device's Value check could find different), on the pairs k_plan_list
//      can plan;
//   3. aliasing took effect: no unmarked run names other entries than its slot's fixing run;
//   4. FR_VEQ is set exactly on the runs whose every earlier-committed slot holds an equal Value;
//   5. FR_UPID is set exactly on the promise-reply runs whose entries share one proposal id (f_pid).
// Prints "ok <runs> <aliased> <marked>" or the first failure.
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
    const uint64_t NP = (uint64_t)N * h.NB;
    uint64_t runs = 0, aliased = 0, marked = 0, veq = 0, upid = 0;
    std::vector<int64_t> fix(BS);
    for (uint64_t q = 0; q < NP; ++q) {
        const uint64_t f0 = h.f_off[q], f1 = h.f_off[q + 1], bk = q / N;
        bool plain = true;
        for (uint64_t f = f0; f < f1; ++f) {
            const uint32_t kind = h.frags[f].flags >> 4;
            plain = plain && (h.frags[f].flags & FR_DENSE) && (kind == K_ACCEPT || kind == K_COMMIT);
        }
        for (uint32_t s = 0; s < BS; ++s) fix[s] = -1;
        for (uint64_t f = f0; f < f1; ++f) {
            const Frag &fr = h.frags[f];
            const uint32_t kind = fr.flags >> 4;
            if (!(fr.flags & FR_DENSE) || (kind != K_ACCEPT && kind != K_COMMIT)) continue;
            ++runs;
            // 1. the run's entries are its message's own
            const uint64_t me = h.m_ent[fr.msg], mc = h.m_cnt[fr.msg];
            const uint64_t iid0 = (bk << BSH) + fr.start;
            uint64_t lo = me, hi = me + mc;                       // the message's entries are iid-sorted
            while (lo < hi) {
                const uint64_t mid = (lo + hi) / 2;
                if (h.e_iid[mid] < iid0) lo = mid + 1; else hi = mid;
            }
            if (lo != fr.entry) ++aliased;
            for (uint32_t d = 0; d < fr.count; ++d) {
                const uint64_t x = fr.entry + d, y = lo + d;
                if (y >= me + mc || h.e_iid[x] != iid0 + d || h.e_iid[y] != iid0 + d || h.e_val[x] != h.e_val[y] ||
                    (member && h.e_pid[x] != h.e_pid[y])) {
                    std::printf("FAIL entries pair %llu run %llu slot %u\n", (unsigned long long)q,
                                (unsigned long long)(f - f0), fr.start + d);
                    return 1;
                }
            }
            // 2. / 3. the Value-check mark on plannable pairs
            const bool learn = kind == K_COMMIT;
            bool want = false;
            if (learn || member)
                for (uint32_t d = 0; d < fr.count; ++d) {
                    const int64_t j = fix[fr.start + d];
                    want = want || (j >= 0 && (uint64_t)j != fr.entry + d && h.e_val[j] != h.e_val[fr.entry + d]);
                }
            const bool got = (fr.flags & FR_VCHK) != 0;
            marked += got;
            if (plain && got != want) {
                std::printf("FAIL mark pair %llu run %llu: FR_VCHK %d, want %d\n", (unsigned long long)q,
                            (unsigned long long)(f - f0), (int)got, (int)want);
                return 1;
            }
            if (learn)
                for (uint32_t d = 0; d < fr.count; ++d)
                    if (fix[fr.start + d] < 0) fix[fr.start + d] = (int64_t)(fr.entry + d);
        }
        // 4. FR_VEQ on every accept / commit run (dense or sparse): set exactly when each slot it
        //    covers that an earlier commit of the pair fixed holds the same Value through its entry
        std::vector<int64_t> fx(BS, -1);
        for (uint64_t f = f0; f < f1; ++f) {
            const Frag &fr = h.frags[f];
            const uint32_t kind = fr.flags >> 4;
            if (kind != K_ACCEPT && kind != K_COMMIT) continue;
            bool eq = true;
            for (uint32_t d = 0; d < fr.count; ++d) {
                const uint64_t x = fr.entry + d;
                const uint32_t sl = (fr.flags & FR_DENSE) ? fr.start + d : (uint32_t)(h.e_iid[x] & (BS - 1));
                if (fx[sl] >= 0 && (uint64_t)fx[sl] != x && h.e_val[fx[sl]] != h.e_val[x]) eq = false;
                if (kind == K_COMMIT && fx[sl] < 0) fx[sl] = (int64_t)x;
            }
            veq += eq;
            if (eq != ((fr.flags & FR_VEQ) != 0)) {
                std::printf("FAIL equal-Value mark pair %llu run %llu: FR_VEQ %d, want %d\n", (unsigned long long)q,
                            (unsigned long long)(f - f0), (int)((fr.flags & FR_VEQ) != 0), (int)eq);
                return 1;
            }
        }
        // 5. FR_UPID on every promise-reply run: set exactly when its entries share one proposal id,
        //    which f_pid holds for the run
        for (uint64_t f = f0; f < f1; ++f) {
            const Frag &fr = h.frags[f];
            if ((fr.flags >> 4) != K_PREPLY || !fr.count) continue;
            bool u = true;
            for (uint32_t d = 1; d < fr.count; ++d) u = u && h.r_pid[fr.entry + d] == h.r_pid[fr.entry];
            upid += u;
            if (u != ((fr.flags & FR_UPID) != 0) || (u && h.f_pid[f] != h.r_pid[fr.entry])) {
                std::printf("FAIL uniform-id mark pair %llu run %llu: FR_UPID %d, want %d\n", (unsigned long long)q,
                            (unsigned long long)(f - f0), (int)((fr.flags & FR_UPID) != 0), (int)u);
                return 1;
            }
        }
    }
    std::printf("ok %llu %llu %llu %llu %llu\n", (unsigned long long)runs, (unsigned long long)aliased,
                (unsigned long long)marked, (unsigned long long)veq, (unsigned long long)upid);
    return 0;
}
