// ingest_bench.cpp — host cost of a live window: the C3 trace cut into W
// windows, each decoded (decode_parallel, as submit_container does) and built
// (build_trace with the window carry), timed per phase.  No GPU.  Measurement tool.
//
//   g++ -O3 -std=c++17 -pthread -Imulti-paxos_amd/csrc -Iinclude tools/ingest_bench.cpp \
//       multi-paxos_amd/csrc/{ingest,gen,gen_faulty,gen_member}.cpp -o tools/ingest_bench
//   tools/ingest_bench <log2 instances> [windows] [chunked 0|1] [serial 0|1]
#include <chrono>
#include <ctime>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "gen.hpp"
#include "ingest.hpp"

using namespace mpx;

static uint64_t rd64(const uint8_t *p) { uint64_t v; std::memcpy(&v, p, 8); return v; }
static double cpu() { timespec ts; clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &ts); return ts.tv_sec + ts.tv_nsec * 1e-9; }
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char **argv)
{
    const uint32_t lg = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 22;
    const uint32_t W = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 16;
    const bool use_cache = argc > 3 ? std::atoi(argv[3]) != 0 : true;      // (0: one chunk per node)
    const bool serial = argc > 4 && std::atoi(argv[4]) != 0;     // (profiling: one thread)
    mpx_gen_params p{};
    p.kind = MPX_GEN_FAULTY; p.num_nodes = 7; p.num_instances = 1ull << lg; p.batch = 256; p.proposers = 3;
    p.drop_rate = 500; p.dup_rate = 1000; p.max_delay = 500;
    std::string t;
    double t0 = now();
    if (gen_faulty(p, t)) { std::printf("gen failed\n"); return 1; }
    std::printf("generated %.2f GB in %.1f s\n", t.size() / 1e9, now() - t0);
    const uint8_t *b = (const uint8_t *)t.data();
    const uint32_t N = 7;
    const uint64_t M = rd64(b + 16);
    size_t pos = 40;
    std::vector<uint64_t> cnt(N);
    std::vector<const uint64_t *> offs(N);
    std::vector<const uint8_t *> body(N);
    for (uint32_t n = 0; n < N; ++n) {
        cnt[n] = rd64(b + pos);
        const uint64_t nb = rd64(b + pos + 8);
        offs[n] = reinterpret_cast<const uint64_t *>(b + pos + 16);
        body[n] = b + pos + 16 + 8 * (cnt[n] + 1);
        pos = (pos + 16 + 8 * (cnt[n] + 1) + nb + 7) & ~(size_t)7;
    }
    WindowCarry wc;
    const uint64_t NB = (M + BS - 1) / BS;
    wc.init(N, NB);
    std::vector<NodeStream> nodes(N);
    ValueTable vt;
    double t_dec = 0, t_merge = 0, t_build = 0, c_dec = 0;
    std::vector<NodeStream> parts;
    const uint32_t threads = serial ? 1 : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    for (uint32_t w = 0; w < W; ++w) {
        double a = now(), ca = cpu();
        IngestViolation iv;
        std::vector<StreamSlice> sl(N);
        for (uint32_t n = 0; n < N; ++n) {
            const uint64_t k0 = cnt[n] * w / W, k1 = cnt[n] * (w + 1) / W;
            sl[n] = StreamSlice{offs[n] + k0, body[n], k1 - k0};
        }
        if (int rc = decode_parallel(vt, nodes, parts, sl, false, nullptr, 0, M, iv, threads, use_cache ? 0 : ~0ull)) {
            std::printf("decode rc %d\n", rc); return 1;
        }
        double m = now();
        c_dec += cpu() - ca;
        double c = now();
        HostTrace ht;
        int rc = build_trace(nodes, 0, M, std::vector<mpx_epoch>(), ht, &wc);
        if (rc) { std::printf("build rc %d\n", rc); return 1; }
        for (auto &ns : nodes) ns.clear();
        double d = now();
        t_dec += m - a; t_merge += c - m; t_build += d - c;
        if (w < 3 || w == W - 1)
            std::printf("window %u: decode %.1f ms, value-table merge %.1f ms, build_trace %.1f ms (%zu messages, %zu runs)\n", w,
                        (m - a) * 1e3, (c - m) * 1e3, (d - c) * 1e3, ht.m_type.size(), ht.frags.size());
    }
    std::printf("per window: decode %.1f ms (cpu %.1f ms), merge %.1f ms, build %.1f ms\n", t_dec / W * 1e3, c_dec / W * 1e3,
                t_merge / W * 1e3, t_build / W * 1e3);
    return 0;
}
