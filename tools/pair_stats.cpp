// pair_stats.cpp — shape of a generated trace's (node, bucket) pairs after ingest
// (host only: the generators + ingest.cpp, no GPU).  Used to size the member
// plan path (how many pairs one plan word can describe, events per pair).
//   tools/pair_stats <member|faulty> <log2 instances>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
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
    const uint32_t lg = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 20;
    mpx_gen_params p{};
    p.num_instances = 1ull << lg;
    if (member) {
        p.kind = MPX_GEN_MEMBER; p.num_nodes = 8; p.batch = 256; p.drop_rate = 100; p.dup_rate = 100;
        p.proposers = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 0;
        p.max_delay = 64; p.noop_permille = 15;
    } else {
        p.kind = MPX_GEN_FAULTY; p.num_nodes = 7; p.batch = 256; p.proposers = 3; p.drop_rate = 500;
        p.dup_rate = 1000; p.max_delay = 500;
    }
    std::string t;
    int rc = member ? gen_member(p, t) : gen_faulty(p, t);
    if (rc) { std::fprintf(stderr, "gen rc %d\n", rc); return 1; }
    const uint8_t *b = (const uint8_t *)t.data();
    const uint32_t N = rd32(b + 8), ne = rd32(b + 24);
    const uint64_t M = rd64(b + 16);
    const size_t esz = rd32(b + 4) == 1 ? 24 : 32;      // container version 2: learner_mask
    std::vector<mpx_epoch> ep(ne);
    for (uint32_t k = 0; k < ne; ++k) {
        std::memcpy(&ep[k], b + 40 + k * esz, 24);
        ep[k].learner_mask = esz == 32 ? rd64(b + 40 + k * esz + 24) : ep[k].proposer_mask;
    }
    size_t pos = 40 + (size_t)ne * esz;
    std::vector<NodeStream> nodes(N);
    const auto t_d0 = std::chrono::steady_clock::now();
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
            if (rc) { std::fprintf(stderr, "decode rc %d\n", rc); return 1; }
        }
        pos += 16 + 8 * (cnt + 1) + nb;
        pos = (pos + 7) & ~(size_t)7;
    }
    std::printf("decode %.3f s (one thread)\n", std::chrono::duration<double>(std::chrono::steady_clock::now() - t_d0).count());
    HostTrace h;
    const auto t_b0 = std::chrono::steady_clock::now();
    rc = build_trace(nodes, 0, M, member ? ep : std::vector<mpx_epoch>(), h);
    if (rc) { std::fprintf(stderr, "build rc %d\n", rc); return 1; }
    std::printf("build_trace %.3f s\n", std::chrono::duration<double>(std::chrono::steady_clock::now() - t_b0).count());
    const uint64_t NP = (uint64_t)N * h.NB;
    uint64_t with = 0, gp = 0, preply = 0, sparse = 0, shape_ok = 0, ev_tot = 0, ev_prep = 0, ev_epoch = 0, ev_other = 0;
    std::map<uint64_t, uint64_t> runs_h, splits_h, ev_h;
    for (uint64_t q = 0; q < NP; ++q) {
        const uint64_t f0 = h.f_off[q], nf = h.f_off[q + 1] - f0;
        if (!nf) continue;
        ++with;
        gp += h.pair_gp[q];
        bool pr = false, sp = false, lean = true;
        uint32_t s[3] = {BS, BS, BS};
        uint32_t nsplit_ok = 1;
        std::vector<uint32_t> bnd;
        for (uint64_t f = f0; f < f0 + nf; ++f) {
            const Frag &fr = h.frags[f];
            const uint32_t kind = fr.flags >> 4;
            if (kind == K_PREPLY) pr = true;
            if (!(fr.flags & FR_DENSE)) sp = true;
            if (kind != K_ACCEPT && kind != K_COMMIT) lean = false;
            if (fr.start) bnd.push_back(fr.start);
            if (fr.start + fr.count < BS) bnd.push_back(fr.start + fr.count);
            if (!plan_add_split(fr.start, s) || !plan_add_split(fr.start + fr.count, s)) nsplit_ok = 0;
        }
        std::sort(bnd.begin(), bnd.end());
        bnd.erase(std::unique(bnd.begin(), bnd.end()), bnd.end());
        preply += pr; sparse += sp;
        shape_ok += lean && !sp && nsplit_ok && nf <= 16;
        runs_h[nf < 16 ? nf : 16]++;
        splits_h[bnd.size() < 8 ? bnd.size() : 8]++;
        const uint64_t e0 = h.ev_off[q], e1 = h.ev_off[q + 1];
        ev_tot += e1 - e0;
        ev_h[(e1 - e0) < 64 ? (e1 - e0) / 4 * 4 : 64]++;
        for (uint64_t e = e0; e < e1; ++e) {
            const uint8_t ty = h.m_type[h.ev_msg[e]];
            if (ty == MPX_MSG_PREPARE) ++ev_prep;
            else if (ty == MPX_MSG_E_EPOCH) ++ev_epoch;
            else ++ev_other;
        }
    }
    std::printf("N %u NB %u pairs %llu with runs %llu gp %llu (simple %llu snap %llu) preply %llu sparse %llu "
                "shape_ok(dense acc/commit, <=3 splits, <=16 runs) %llu\n",
                N, h.NB, (unsigned long long)NP, (unsigned long long)with, (unsigned long long)gp,
                (unsigned long long)h.num_gp_simple, (unsigned long long)h.num_gp_snap, (unsigned long long)preply,
                (unsigned long long)sparse, (unsigned long long)shape_ok);
    std::printf("events %llu (prepare %llu, epoch %llu, other %llu), runs %zu, messages %zu, markers %zu\n",
                (unsigned long long)ev_tot, (unsigned long long)ev_prep, (unsigned long long)ev_epoch,
                (unsigned long long)ev_other, h.frags.size(), h.m_type.size(), h.ee_msg.size());
    // the AM_SNAP range of the general work list: PREPARE events after the pair's first run
    // (a snapshot can only be non-empty then), runs per pair
    {
        uint64_t snap_pairs = 0, snap_late = 0, snap_late_ev = 0, snap_runs = 0, snap_ev = 0, snap_lean = 0;
        for (uint64_t it = h.num_gp_simple; it < h.num_gp_snap; ++it) {
            const uint64_t q = h.gp_list[it];                // host form: the pair itself
            const uint64_t f0 = h.f_off[q], f1 = h.f_off[q + 1], e0 = h.ev_off[q], e1 = h.ev_off[q + 1];
            ++snap_pairs; snap_runs += f1 - f0; snap_ev += e1 - e0;
            bool lean = f1 - f0 <= 16;
            uint32_t s[3] = {BS, BS, BS};
            for (uint64_t f = f0; f < f1; ++f) {
                const Frag &fr = h.frags[f];
                const uint32_t kind = fr.flags >> 4;
                if (!(fr.flags & FR_DENSE) || (kind != K_ACCEPT && kind != K_COMMIT)) lean = false;
                if (!plan_add_split(fr.start, s) || !plan_add_split(fr.start + fr.count, s)) lean = false;
            }
            snap_lean += lean;
            const uint32_t first = f1 > f0 ? h.frags[f0].msg : NONE32;
            uint64_t late = 0;
            for (uint64_t e = e0; e < e1; ++e) late += h.ev_msg[e] > first;
            snap_late += late > 0; snap_late_ev += late;
        }
        std::printf("AM_SNAP pairs %llu: runs %llu events %llu, lean-shaped %llu, with a PREPARE after the first run %llu "
                    "(%llu such events)\n", (unsigned long long)snap_pairs, (unsigned long long)snap_runs,
                    (unsigned long long)snap_ev, (unsigned long long)snap_lean, (unsigned long long)snap_late,
                    (unsigned long long)snap_late_ev);
    }
    // the work list's pairs without promise rounds that a plan walk with up to S segments and
    // R runs would take (dense accept / commit runs only)
    {
        const uint32_t RS[4][2] = {{16, 4}, {32, 8}, {32, 16}, {64, 32}};
        uint64_t lst = 0, cov[4] = {0, 0, 0, 0};
        for (uint64_t it = 0; it < h.num_gp_snap; ++it) {
            const uint64_t q = h.gp_list[it];
            const uint64_t f0 = h.f_off[q], f1 = h.f_off[q + 1];
            ++lst;
            bool dense = true;
            std::vector<uint32_t> bnd;
            for (uint64_t f = f0; f < f1; ++f) {
                const Frag &fr = h.frags[f];
                const uint32_t kind = fr.flags >> 4;
                if (!(fr.flags & FR_DENSE) || (kind != K_ACCEPT && kind != K_COMMIT)) dense = false;
                if (fr.start) bnd.push_back(fr.start);
                if (fr.start + fr.count < BS) bnd.push_back(fr.start + fr.count);
            }
            std::sort(bnd.begin(), bnd.end());
            bnd.erase(std::unique(bnd.begin(), bnd.end()), bnd.end());
            for (int k = 0; k < 4; ++k)
                cov[k] += dense && f1 - f0 <= RS[k][0] && bnd.size() + 1 <= RS[k][1];
        }
        std::printf("list pairs %llu; plannable with (runs, segments) <= (16,4) %llu, (32,8) %llu, (32,16) %llu, (64,32) %llu\n",
                    (unsigned long long)lst, (unsigned long long)cov[0], (unsigned long long)cov[1],
                    (unsigned long long)cov[2], (unsigned long long)cov[3]);
    }
    // walk lengths (runs + events) of the pairs left on k_apply: the listed pairs a (32, 8) plan
    // cannot describe (AM_SNAP) and the promise-round pairs (AM_FULL) — tail versus throughput
    {
        std::vector<uint64_t> snapw, fullw;
        for (uint64_t it = 0; it < h.gp_list.size(); ++it) {
            const uint64_t q = h.gp_list[it];
            const uint64_t f0 = h.f_off[q], f1 = h.f_off[q + 1], e0 = h.ev_off[q], e1 = h.ev_off[q + 1];
            if (it >= h.num_gp_snap) { fullw.push_back(f1 - f0 + e1 - e0); continue; }
            bool dense = true;
            std::vector<uint32_t> bnd;
            for (uint64_t f = f0; f < f1; ++f) {
                const Frag &fr = h.frags[f];
                const uint32_t kind = fr.flags >> 4;
                if (!(fr.flags & FR_DENSE) || (kind != K_ACCEPT && kind != K_COMMIT)) dense = false;
                if (fr.start) bnd.push_back(fr.start);
                if (fr.start + fr.count < BS) bnd.push_back(fr.start + fr.count);
            }
            std::sort(bnd.begin(), bnd.end());
            bnd.erase(std::unique(bnd.begin(), bnd.end()), bnd.end());
            if (!(dense && f1 - f0 <= 32 && bnd.size() + 1 <= 8)) snapw.push_back(f1 - f0 + e1 - e0);
        }
        for (int k = 0; k < 2; ++k) {
            std::vector<uint64_t> &w = k ? fullw : snapw;
            std::sort(w.begin(), w.end());
            uint64_t sum = 0;
            for (uint64_t x : w) sum += x;
            auto pc = [&](double f) { return w.empty() ? 0ull : (unsigned long long)w[(size_t)(f * (w.size() - 1))]; };
            std::printf("%s pairs %zu: steps (runs + events) sum %llu, p50 %llu p90 %llu p99 %llu p99.9 %llu max %llu\n",
                        k ? "AM_FULL" : "AM_SNAP (not (32, 8)-plannable)", w.size(), (unsigned long long)sum, pc(0.5),
                        pc(0.9), pc(0.99), pc(0.999), pc(1.0));
        }
    }
    // the promise-round pairs' runs by kind and density, and their events by type
    {
        uint64_t k_n[4] = {0, 0, 0, 0}, k_sp[4] = {0, 0, 0, 0}, k_ent[4] = {0, 0, 0, 0}, evq = 0;
        for (uint64_t it = h.num_gp_snap; it < h.gp_list.size(); ++it) {
            const uint64_t q = h.gp_list[it];
            for (uint64_t f = h.f_off[q]; f < h.f_off[q + 1]; ++f) {
                const Frag &fr = h.frags[f];
                const uint32_t kind = (fr.flags >> 4) & 3;
                k_n[kind]++; k_sp[kind] += !(fr.flags & FR_DENSE); k_ent[kind] += fr.count;
            }
            evq += h.ev_off[q + 1] - h.ev_off[q];
        }
        for (uint32_t k = 0; k < 4; ++k)
            std::printf("AM_FULL runs of kind %u: %llu (sparse %llu, entries %llu)\n", k, (unsigned long long)k_n[k],
                        (unsigned long long)k_sp[k], (unsigned long long)k_ent[k]);
        std::printf("AM_FULL events %llu\n", (unsigned long long)evq);
    }
    // k_plan_list stages a wave's (64 consecutive pairs') descriptor words in LDS, MPLAN_LDS per
    // wave: the GP_LIST pairs a (32, 8) plan could take that the staging window leaves out
    {
        uint64_t over = 0, wmax = 0;
        for (uint64_t w0 = 0; w0 < NP; w0 += 64) {
            const uint64_t wb = h.f_off[w0], we = h.f_off[std::min<uint64_t>(w0 + 64, NP)];
            wmax = std::max<uint64_t>(wmax, we - wb);
            for (uint64_t q = w0; q < std::min<uint64_t>(w0 + 64, NP); ++q)
                if (h.pair_gp[q] == GP_LIST && h.f_off[q + 1] - h.f_off[q] <= 32 &&
                    h.f_off[q + 1] - wb > MPLAN_LDS) ++over;
        }
        std::printf("GP_LIST pairs (<= 32 runs) past a wave's %u-word LDS window: %llu (max runs per wave %llu)\n",
                    MPLAN_LDS, (unsigned long long)over, (unsigned long long)wmax);
    }
    // k_plan_list's Value check: a COMMIT over a committed segment whose entry index differs
    // lists the pair for k_apply; how many (32, 8)-shaped pairs that is, and how many of them
    // carry equal Values (handles) on every such slot
    {
        uint64_t shaped = 0, recommit = 0, equal = 0, vchk = 0;
        for (uint64_t it = 0; it < h.num_gp_snap; ++it) {
            const uint64_t q = h.gp_list[it];
            const uint64_t f0 = h.f_off[q], f1 = h.f_off[q + 1];
            bool dense = f1 - f0 <= 32;
            std::vector<uint32_t> bnd;
            for (uint64_t f = f0; f < f1; ++f) {
                const Frag &fr = h.frags[f];
                const uint32_t kind = fr.flags >> 4;
                if (!(fr.flags & FR_DENSE) || (kind != K_ACCEPT && kind != K_COMMIT)) dense = false;
                if (fr.start) bnd.push_back(fr.start);
                if (fr.start + fr.count < BS) bnd.push_back(fr.start + fr.count);
            }
            std::sort(bnd.begin(), bnd.end());
            bnd.erase(std::unique(bnd.begin(), bnd.end()), bnd.end());
            if (!dense || bnd.size() + 1 > 8) continue;
            ++shaped;
            int64_t fix[BS];
            for (uint32_t s = 0; s < BS; ++s) fix[s] = -1;
            bool rc = false, eq = true;
            for (uint64_t f = f0; f < f1; ++f) {
                const Frag &fr = h.frags[f];
                if ((fr.flags >> 4) != K_COMMIT) continue;
                for (uint32_t s = fr.start; s < (uint32_t)fr.start + fr.count; ++s) {
                    const uint64_t x = fr.entry + (s - fr.start);
                    if (fix[s] < 0) { fix[s] = (int64_t)x; continue; }
                    if ((uint64_t)fix[s] != x) { rc = true; eq = eq && h.e_val[fix[s]] == h.e_val[x]; }
                }
            }
            recommit += rc; equal += rc && eq;
            bool vb = false;
            for (uint64_t f = f0; f < f1; ++f) vb = vb || (h.frags[f].flags & FR_VCHK);
            vchk += vb;
        }
        std::printf("(32, 8)-shaped list pairs %llu: re-committed with another entry %llu, all such slots equal Values %llu; "
                    "with an FR_VCHK run (after ingest's aliasing) %llu\n",
                    (unsigned long long)shaped, (unsigned long long)recommit, (unsigned long long)equal, (unsigned long long)vchk);
    }
    std::printf("runs/pair:");
    for (auto &x : runs_h) std::printf(" %llu:%llu", (unsigned long long)x.first, (unsigned long long)x.second);
    std::printf("\ninterior boundaries/pair:");
    for (auto &x : splits_h) std::printf(" %llu:%llu", (unsigned long long)x.first, (unsigned long long)x.second);
    std::printf("\nevents/pair (bins of 4):");
    for (auto &x : ev_h) std::printf(" %llu:%llu", (unsigned long long)x.first, (unsigned long long)x.second);
    std::printf("\n");
    return 0;
}
