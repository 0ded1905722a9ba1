// gen_device.hip — materialise the clean trace (MPX_GEN_CLEAN, C2/C4) directly
// in HBM, already decoded and bucketed: the exact arrays that mpx_submit +
// build_trace produce for gen_clean()'s wire trace restricted to the engine's
// shard (tests/test_engine_gpu.py::test_device_generator_matches_host).
//
// Shard pruning: a shard engine keeps the replicated headers (P_START,
// PREPARE, promises) and the batches that overlap its shard.  Out-of-shard
// ACCEPT/COMMIT/P_BATCH records and their replies belong to the rank owning
// those instances; in the clean trace they cannot change this shard's state
// or scalars (every ACCEPT carries the PREPARE's ballot, already seen).
//
// Layout (batch size B, shard aligned to 256; B = 256 puts one batch per bucket):
//   node 0 : P_START, PREPARE, N x PREPARE_REPLY, then per kept batch
//            P_BATCH, ACCEPT, N x ACCEPT_REPLY, COMMIT, N x COMMIT_REPLY
//   node i : PREPARE, then per kept batch ACCEPT, COMMIT
//   entries: one run per batch, shared by its P_BATCH, ACCEPT and COMMIT at
//            every node (the content-addressed pool of ingest.cpp: a
//            broadcast is stored once), so e_val[i - sb] = handle of i
//   pairs:   f_off / frags indexed bucket-major, q = bucket * N + node; a pair
//            holds an ACCEPT and a COMMIT run for every batch meeting its
//            bucket (f_off / cf_off: prefix counts computed on the host)
#include <hip/hip_runtime.h>
#include "mpx_internal.hpp"

namespace mpx {

struct CleanGeo {
    uint32_t N;
    uint64_t K;          // kept batches (= buckets of the shard)
    uint64_t k0;         // first kept batch
    uint64_t sb, se;     // shard, se clamped to M
    uint64_t G0;         // messages of node 0
    uint64_t G1;         // messages of node i > 0
    uint64_t ballot;
    uint64_t B;          // instances per batch
};

__device__ inline uint64_t batch_cnt(const CleanGeo &c, uint64_t j)
{
    const uint64_t lo = (c.k0 + j) * c.B, hi = lo + c.B;
    const uint64_t a = lo > c.sb ? lo : c.sb, b = hi < c.se ? hi : c.se;
    return b > a ? b - a : 0;
}
__device__ inline uint64_t batch_pre(const CleanGeo &c, uint64_t j)   // in-shard entries before batch j
{
    const uint64_t x = (c.k0 + j) * c.B;
    const uint64_t m = x < c.se ? x : c.se;
    return m > c.sb ? m - c.sb : 0;
}
__device__ inline uint64_t node_msg0(const CleanGeo &c, uint32_t n) { return n == 0 ? 0 : c.G0 + (uint64_t)(n - 1) * c.G1; }

// one thread per message
__global__ void k_gen_msgs(CleanGeo c, uint8_t *type, uint32_t *src, uint64_t *ballot, uint64_t *aux,
                           uint64_t *ent, uint32_t *cnt, uint32_t *node)
{
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t total = c.G0 + (uint64_t)(c.N - 1) * c.G1;
    if (g >= total) return;
    uint32_t n;
    uint64_t k;
    if (g < c.G0) { n = 0; k = g; } else { n = 1 + (uint32_t)((g - c.G0) / c.G1); k = (g - c.G0) % c.G1; }
    uint8_t t = 0; uint32_t s = 0; uint64_t b = 0, a = 0, e = 0; uint32_t ct = 0;
    const uint32_t N = c.N;
    if (n == 0) {
        if (k == 0) { t = MPX_MSG_P_START; b = c.ballot; }
        else if (k == 1) { t = MPX_MSG_PREPARE; b = c.ballot; e = 0; ct = 1; }
        else if (k < 2 + N) { t = MPX_MSG_PREPARE_REPLY; s = (uint32_t)(k - 2); b = c.ballot; }
        else {
            const uint64_t r = k - 2 - N, j = r / (3 + 2 * N), o = r % (3 + 2 * N);
            const uint64_t bc = batch_cnt(c, j), be = batch_pre(c, j);
            a = c.k0 + j + 1;
            if (o == 0) { t = MPX_MSG_P_BATCH; e = be; ct = (uint32_t)bc; }
            else if (o == 1) { t = MPX_MSG_ACCEPT; b = c.ballot; e = be; ct = (uint32_t)bc; }
            else if (o < 2 + N) { t = MPX_MSG_ACCEPT_REPLY; s = (uint32_t)(o - 2); b = c.ballot; }
            else if (o == 2 + N) { t = MPX_MSG_COMMIT; b = c.ballot; e = be; ct = (uint32_t)bc; }
            else { t = MPX_MSG_COMMIT_REPLY; s = (uint32_t)(o - 3 - N); }
        }
    } else {
        if (k == 0) { t = MPX_MSG_PREPARE; b = c.ballot; e = n; ct = 1; }
        else {
            const uint64_t j = (k - 1) / 2;
            const uint64_t bc = batch_cnt(c, j), be = batch_pre(c, j);
            a = c.k0 + j + 1;
            b = c.ballot;
            t = (k - 1) % 2 == 0 ? MPX_MSG_ACCEPT : MPX_MSG_COMMIT;
            e = be;
            ct = (uint32_t)bc;
        }
    }
    type[g] = t; src[g] = s; ballot[g] = b; aux[g] = a; ent[g] = e; cnt[g] = ct; node[g] = n;
}

// one thread per in-shard instance: the shared entry pool (batch runs are
// contiguous and in instance order, so entry li holds instance sb + li)
__global__ void k_gen_entries(CleanGeo c, uint64_t *e_val)
{
    const uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= c.se - c.sb) return;
    e_val[li] = MPX_HANDLE(0, 0, c.sb + li + 1);
}

// one thread per (bucket, node) pair q = bucket * N + node: for every batch
// meeting the bucket, in message order, its ACCEPT run then its COMMIT run
// (f_off from the host); the (bucket, 0) thread also writes the bucket's
// chosen-log runs (cf_off)
__global__ void k_gen_frags(CleanGeo c, uint32_t NB, Frag *frags, const uint64_t *f_off, Frag *cfrags,
                            const uint64_t *cf_off)
{
    const uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t np = (uint64_t)c.N * NB;
    if (x >= np) return;
    const uint32_t N = c.N;
    const uint32_t n = (uint32_t)(x % N);
    const uint64_t b = x / N;
    const uint64_t lo = c.sb + (b << 8), hi = lo + 256 < c.se ? lo + 256 : c.se;
    const uint64_t j0 = lo / c.B - c.k0, j1 = (hi - 1) / c.B - c.k0;
    uint64_t at = f_off[x];
    for (uint64_t j = j0; j <= j1; ++j) {
        const uint64_t blo = (c.k0 + j) * c.B, bhi = blo + c.B;
        const uint64_t a = blo > lo ? blo : lo, e = bhi < hi ? bhi : hi;     // the batch's run in this bucket
        uint64_t acc_msg, com_msg;
        if (n == 0) {
            const uint64_t base = 2 + N + j * (3 + 2 * N);
            acc_msg = base + 1; com_msg = base + 2 + N;
        } else {
            const uint64_t base = node_msg0(c, n) + 1 + 2 * j;
            acc_msg = base; com_msg = base + 1;
        }
        const uint8_t start = (uint8_t)((a - c.sb) & 255);
        const Frag fa{a - c.sb, (uint32_t)acc_msg, (uint16_t)(e - a), start, (uint8_t)(FR_DENSE | (K_ACCEPT << 4))};
        const Frag fc{a - c.sb, (uint32_t)com_msg, (uint16_t)(e - a), start, (uint8_t)(FR_DENSE | (K_COMMIT << 4))};
        frags[at++] = fa;
        frags[at++] = fc;
        if (n == 0) {
            const Frag fb{a - c.sb, (uint32_t)j, (uint16_t)(e - a), start, (uint8_t)(FR_DENSE | (K_BATCH << 4))};
            cfrags[cf_off[b] + (j - j0)] = fb;
        }
    }
}

// one thread per header-scan record: node n's PREPARE, then its K ACCEPTs
// (index n * (K + 1) + r; mpx_internal.hpp SC_*)
__global__ void k_gen_scan(CleanGeo c, uint8_t *sc_type, uint64_t *sc_key, uint32_t *sc_idx)
{
    const uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= (uint64_t)c.N * (c.K + 1)) return;
    const uint32_t n = (uint32_t)(x / (c.K + 1));
    const uint64_t r = x - (uint64_t)n * (c.K + 1);
    uint64_t g;
    if (r == 0) g = n == 0 ? 1 : node_msg0(c, n);
    else if (n == 0) g = 2 + c.N + (r - 1) * (3 + 2 * c.N) + 1;
    else g = node_msg0(c, n) + 1 + 2 * (r - 1);
    sc_type[x] = r == 0 ? SC_PREP : SC_ACC;
    sc_key[x] = c.ballot;
    sc_idx[x] = (uint32_t)g;
}

// one thread per batch: proposer marker, vote list (+ the replies' headers)
__global__ void k_gen_batches(CleanGeo c, uint32_t *b_msg, uint32_t *b_pstart, uint64_t *b_rep_off, uint32_t *b_rep,
                              uint64_t *b_rbal, uint32_t *b_rsrc, uint64_t *b_bal)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j > c.K) return;
    const uint32_t N = c.N;
    b_rep_off[j] = (uint64_t)N * j;
    if (j == c.K) return;
    const uint64_t base = 2 + N + j * (3 + 2 * N);
    b_msg[j] = (uint32_t)base;
    b_pstart[j] = 0;
    b_bal[j] = c.ballot;
    for (uint32_t i = 0; i < N; ++i) {
        b_rep[(uint64_t)N * j + i] = (uint32_t)(base + 2 + i);
        b_rbal[(uint64_t)N * j + i] = c.ballot;
        b_rsrc[(uint64_t)N * j + i] = i;
    }
}

static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

int launch_gen_clean(void *stream_, uint32_t N, uint64_t K, uint64_t k0, uint64_t sb, uint64_t se,
                        uint64_t G0, uint64_t G1, uint64_t ballot, uint64_t B, uint32_t NB,
                        uint8_t *type, uint32_t *src, uint64_t *bal, uint64_t *aux, uint64_t *ent, uint32_t *cnt,
                        uint32_t *node, uint64_t *e_val, Frag *frags, uint64_t *f_off, uint32_t *b_msg,
                        uint32_t *b_pstart, uint64_t *b_rep_off, uint32_t *b_rep, uint64_t *cf_off, Frag *cfrags,
                        uint8_t *sc_type, uint64_t *sc_key, uint32_t *sc_idx, uint64_t *b_rbal, uint32_t *b_rsrc,
                        uint64_t *b_bal)
{
    hipStream_t s = (hipStream_t)stream_;
    CleanGeo c{N, K, k0, sb, se, G0, G1, ballot, B};
    const uint64_t G = G0 + (uint64_t)(N - 1) * G1;
    hipLaunchKernelGGL(k_gen_msgs, dim3(cdiv(G, 256)), dim3(256), 0, s, c, type, src, bal, aux, ent, cnt, node);
    hipLaunchKernelGGL(k_gen_entries, dim3(cdiv(se - sb, 256)), dim3(256), 0, s, c, e_val);
    hipLaunchKernelGGL(k_gen_frags, dim3(cdiv((uint64_t)N * NB, 256)), dim3(256), 0, s, c, NB, frags, f_off, cfrags,
                       cf_off);
    hipLaunchKernelGGL(k_gen_batches, dim3(cdiv(K + 1, 256)), dim3(256), 0, s, c, b_msg, b_pstart, b_rep_off, b_rep,
                       b_rbal, b_rsrc, b_bal);
    hipLaunchKernelGGL(k_gen_scan, dim3(cdiv((uint64_t)N * (K + 1), 256)), dim3(256), 0, s, c, sc_type, sc_key, sc_idx);
    return (int)hipGetLastError();
}

}  // namespace mpx
