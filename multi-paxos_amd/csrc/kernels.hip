// kernels.hip — CDNA4 (gfx950) kernels of the batched Multi-Paxos engine.
//
// One run = the whole resident trace applied from genesis state:
//   k_scan_chunk / k_scan_node / k_scan_apply
//       per-message header scan: promised = running max of PREPARE ids,
//       max_seen = running max of PREPARE/ACCEPT ids and REJECT max_ids
//       (multi/paxos.cpp:862-865,1363-1366,1229-1230) -> granted / reject flags
//   k_proposer   promise quorum per proposer epoch (OnPrepareReply, :1036-1057)
//   k_votes      accept-vote quorum per batch: 64-bit acceptor mask, popcount
//                against N/2+1 (OnAcceptReply, :1406-1427)
//   k_apply      the acceptor / learner / pre-accepted merge state machines of
//                one (node, 256-instance bucket) per workgroup iteration
//                (OnAccept :1359-1404, OnCommit :1494-1518, FilterAcceptedValues
//                :902-922, UpdateByPreAcceptedValues :1213-1222)
//   k_chosen     chosen log: instances of batches whose votes reached quorum
//   k_reduce     counters, digests -> 64-word summary
// Everything is integer, HBM-bound; no MFMA.
#include <hip/hip_runtime.h>
#include "mpx_internal.hpp"

namespace mpx {

__device__ inline void record_violation(const DevView &v, uint64_t code, uint64_t node, uint64_t seq, uint64_t iid)
{
    atomicAdd(&v.viol->count, 1ull);
    if (atomicCAS(&v.viol->code, 0ull, (unsigned long long)code) == 0ull) {
        v.viol->node = node;
        v.viol->seq = seq;
        v.viol->iid = iid;
    }
}

// ---------------------------------------------------------------- scans --
// wave64 inclusive max scan
__device__ inline uint64_t wave_scan_max(uint64_t x)
{
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x = x > y ? x : y;
    }
    return x;
}

// block (256 threads) exclusive max scan of one value per thread; returns the
// exclusive prefix and writes the block total to *total
__device__ inline uint64_t block_excl_max(uint64_t x, uint64_t *lds4, uint64_t *total)
{
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t inc = wave_scan_max(x);
    if (lane == 63) lds4[w] = inc;
    __syncthreads();
    uint64_t pre = 0;
    for (uint32_t i = 0; i < w; ++i) pre = pre > lds4[i] ? pre : lds4[i];
    uint64_t t = 0;
    for (uint32_t i = 0; i < 4; ++i) t = t > lds4[i] ? t : lds4[i];
    *total = t;
    uint64_t excl = __shfl_up(inc, 1, 64);
    if (lane == 0) excl = 0;
    excl = excl > pre ? excl : pre;
    __syncthreads();
    return excl;
}

// contribution of one message to promised (p) and max_seen (s)
__device__ inline void msg_contrib(const DevView &v, uint64_t g, uint64_t &p, uint64_t &s)
{
    uint8_t t = v.m_type[g];
    uint64_t b = v.m_ballot[g];
    p = t == MPX_MSG_PREPARE ? b : 0;
    s = (t == MPX_MSG_PREPARE || t == MPX_MSG_ACCEPT || t == MPX_MSG_REJECT) ? b : 0;
}

__global__ __launch_bounds__(256) void k_scan_chunk(DevView v)
{
    __shared__ uint64_t l[8];
    const uint32_t c = blockIdx.x;
    const uint64_t beg = v.chunk_beg[c], end = v.chunk_end[c];
    uint64_t pm = 0, sm = 0;
    for (uint64_t g = beg + threadIdx.x; g < end; g += 256) {
        uint64_t p, s;
        msg_contrib(v, g, p, s);
        pm = pm > p ? pm : p;
        sm = sm > s ? sm : s;
    }
    uint64_t tp, ts;
    block_excl_max(pm, l, &tp);
    block_excl_max(sm, l + 4, &ts);
    if (threadIdx.x == 0) { v.chunk_agg[2 * c] = tp; v.chunk_agg[2 * c + 1] = ts; }
}

__global__ __launch_bounds__(256) void k_scan_node(DevView v)
{
    __shared__ uint64_t l[8];
    const uint32_t n = blockIdx.x;
    const uint32_t c0 = v.node_chunk_off[n], c1 = v.node_chunk_off[n + 1];
    uint64_t carry_p = 0, carry_s = 0;
    for (uint32_t base = c0; base < c1; base += 256) {
        uint32_t c = base + threadIdx.x;
        uint64_t p = c < c1 ? v.chunk_agg[2 * c] : 0, s = c < c1 ? v.chunk_agg[2 * c + 1] : 0;
        uint64_t tp, ts;
        uint64_t ep = block_excl_max(p, l, &tp);
        uint64_t es = block_excl_max(s, l + 4, &ts);
        if (c < c1) {
            v.chunk_carry[2 * c] = ep > carry_p ? ep : carry_p;
            v.chunk_carry[2 * c + 1] = es > carry_s ? es : carry_s;
        }
        carry_p = carry_p > tp ? carry_p : tp;
        carry_s = carry_s > ts ? carry_s : ts;
    }
    if (threadIdx.x == 0) { v.node_scal[2 * n] = carry_p; v.node_scal[2 * n + 1] = carry_s; }
}

// per message: granted / reject flags, max_seen carried by REJECTs.
// Chunk = 1024 messages, 4 consecutive per thread.
__global__ __launch_bounds__(256) void k_scan_apply(DevView v)
{
    __shared__ uint64_t l[8];
    const uint32_t c = blockIdx.x;
    const uint64_t beg = v.chunk_beg[c], end = v.chunk_end[c];
    const uint64_t g0 = beg + 4ull * threadIdx.x;
    uint64_t p[4], s[4];
    uint64_t tp = 0, ts = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        p[i] = s[i] = 0;
        if (g0 + i < end) msg_contrib(v, g0 + i, p[i], s[i]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) { tp = tp > p[i] ? tp : p[i]; ts = ts > s[i] ? ts : s[i]; }
    uint64_t bt;
    uint64_t ep = block_excl_max(tp, l, &bt);
    uint64_t es = block_excl_max(ts, l + 4, &bt);
    uint64_t cp = v.chunk_carry[2 * c], cs = v.chunk_carry[2 * c + 1];
    uint64_t run_p = ep > cp ? ep : cp;      // promised before message g0
    uint64_t run_s = es > cs ? es : cs;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint64_t g = g0 + i;
        if (g >= end) break;
        const uint8_t t = v.m_type[g];
        const uint64_t id = v.m_ballot[g];
        run_s = run_s > s[i] ? run_s : s[i];   // max_seen after this message
        uint8_t f = 0;
        if (t == MPX_MSG_PREPARE) {
            if (id > run_p) f = F_GRANTED;                        // :865
            else if (id < run_p) f = F_REJECT;                    // :894
        } else if (t == MPX_MSG_ACCEPT) {
            f = id >= run_p ? F_GRANTED : F_REJECT;               // :1366
        }
        if ((t == MPX_MSG_PREPARE || t == MPX_MSG_ACCEPT || t == MPX_MSG_COMMIT) && v.m_src[g] >= v.N)
            f |= F_BADNODE;
        v.m_flags[g] = f;
        if (f & F_REJECT) v.m_maxseen[g] = run_s;
        if (f & F_BADNODE) record_violation(v, MPX_V_BAD_NODE, v.m_node[g], g - v.node_off[v.m_node[g]], 0);
        run_p = run_p > p[i] ? run_p : p[i];
    }
}

// --------------------------------------------------------- proposer side --
// Promise quorum per node: serial over the node's (few) P_START and
// PREPARE_REPLY records.  One lane per node.
__global__ void k_proposer(DevView v)
{
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= v.N) return;
    uint64_t ballot = 0, mask = 0;         // proposal_id_ = 0 at genesis (:338)
    bool preparing = false;                // prepare_retry_timeout_ = NULL
    for (uint64_t i = v.pl_off[n]; i < v.pl_off[n + 1]; ++i) {
        const uint32_t g = v.pl_msg[i];
        const uint8_t t = v.m_type[g];
        if (t == MPX_MSG_P_START) {
            ballot = v.m_ballot[g]; preparing = true; mask = 0;
        } else if (preparing && v.m_ballot[g] == ballot) {      // :1038
            const uint32_t a = v.m_src[g];
            if (a >= v.N) { record_violation(v, MPX_V_BAD_NODE, n, g - v.node_off[n], 0); continue; }
            uint8_t f = F_COUNTED;
            mask |= 1ull << a;
            if ((uint32_t)__popcll(mask) >= v.quorum) {          // :1047
                f |= F_QUORUM; preparing = false; mask = 0;
            }
            v.m_flags[g] |= f;
        }
    }
}

// Accept-vote quorum, one lane per batch (AcceptingValues::accepted_ as a mask).
__global__ void k_votes(DevView v)
{
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= v.num_batches) return;
    const uint32_t ps = v.b_pstart[j];
    const uint64_t ballot = ps == NONE32 ? 0 : v.m_ballot[ps];
    uint64_t mask = 0;
    uint32_t chosen = NONE32;
    for (uint64_t r = v.b_rep_off[j]; r < v.b_rep_off[j + 1]; ++r) {
        const uint32_t g = v.b_rep[r];
        if (v.m_ballot[g] != ballot) continue;                  // :1408
        const uint32_t a = v.m_src[g];
        if (a >= v.N) {
            const uint32_t n = v.m_node[g];
            record_violation(v, MPX_V_BAD_NODE, n, g - v.node_off[n], 0);
            continue;
        }
        mask |= 1ull << a;
        if ((uint32_t)__popcll(mask) >= v.quorum) { chosen = g; break; }   // :1416
    }
    v.b_chosen[j] = chosen;
}

// ------------------------------------------------------------- apply ----
__device__ inline void emit(const DevView &v, bool want, uint32_t msg, uint32_t kind, uint64_t iid,
                            uint64_t ballot, uint64_t handle)
{
    const uint64_t m = __ballot(want);
    if (!m) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t rank = __popcll(m & ((1ull << lane) - 1));
    unsigned long long base = 0;
    if (lane == (uint32_t)(__ffsll((long long)m) - 1)) base = atomicAdd(v.out_cursor, (unsigned long long)__popcll(m));
    base = __shfl(base, __ffsll((long long)m) - 1, 64);
    if (want && base + rank < v.out_cap) {
        OutRec r;
        r.msg = msg; r.kind = kind; r.iid = iid; r.ballot = ballot; r.handle = handle;
        v.out[base + rank] = r;
    }
}

// A workgroup owns one (node, bucket) pair at a time, one thread per instance
// slot; the pair's fragments and the node's snapshot events are walked in
// message order, so every instance sees its events in the reference's order.
__global__ __launch_bounds__(256) void k_apply(DevView v)
{
    __shared__ uint16_t lidx[256];
    __shared__ unsigned long long red[4][8];
    const uint32_t t = threadIdx.x;
    lidx[t] = 0xFFFF;
    __syncthreads();
    unsigned long long cA = 0, cL = 0, cP = 0, cQ = 0, dig = 0;
    const uint64_t npairs = (uint64_t)v.N * v.NB;
    for (uint64_t p = blockIdx.x; p < npairs; p += gridDim.x) {
        const uint32_t n = (uint32_t)(p / v.NB);
        const uint32_t b = (uint32_t)(p - (uint64_t)n * v.NB);
        const uint64_t li = ((uint64_t)b << BSH) + t;
        const bool in = li < v.shard_len;
        const uint64_t iid = v.shard_begin + li;
        uint64_t sb = 0, sw = 0, pb = 0, pw = 0;
        uint64_t fi = v.f_off[p];
        const uint64_t fe = v.f_off[p + 1];
        uint64_t ei = v.ev_off[n];
        const uint64_t ee = v.ev_off[n + 1];
        while (fi < fe || ei < ee) {
            const uint32_t fm = fi < fe ? v.frags[fi].msg : NONE32;
            const uint32_t em = ei < ee ? v.ev_msg[ei] : NONE32;
            if (fm <= em) {
                const Frag F = v.frags[fi++];
                const uint32_t kind = F.flags >> 4;
                const uint8_t fl = v.m_flags[F.msg];
                int k = -1;
                if (F.flags & FR_DENSE) {
                    const int d = (int)t - (int)F.start;
                    if (d >= 0 && d < (int)F.count) k = d;
                } else {
                    const uint8_t *slots = kind == K_PREPLY ? v.r_slot : v.e_slot;
                    if (t < F.count) lidx[slots[F.entry + t]] = (uint16_t)t;
                    __syncthreads();
                    k = lidx[t] == 0xFFFF ? -1 : (int)lidx[t];
                    __syncthreads();
                    lidx[t] = 0xFFFF;
                    __syncthreads();
                }
                if (kind == K_ACCEPT) {
                    if ((fl & F_GRANTED) && k >= 0) {
                        const uint64_t val = v.e_val[F.entry + k];
                        if (!(sw & W_COMMITTED)) {                          // :1380
                            sb = v.m_ballot[F.msg];                        // :1387
                            sw = W_PRESENT | val;
                            ++cA;
                        }
                    }
                } else if (kind == K_COMMIT) {
                    if (k >= 0) {
                        const uint64_t val = v.e_val[F.entry + k];
                        if (sw & W_COMMITTED) {                             // :1508
                            if ((sw & W_HANDLE) != val) {
                                const uint32_t g = F.msg;
                                record_violation(v, MPX_V_COMMIT_VALUE, n, g - v.node_off[n], iid);
                            }
                        } else {
                            sb = v.m_ballot[F.msg];                        // :1515
                            sw = W_PRESENT | W_COMMITTED | val;
                        }
                        ++cL;
                    }
                } else if (kind == K_PREPLY) {
                    if ((fl & F_COUNTED) && k >= 0) {
                        const uint64_t pid = v.r_pid[F.entry + k];
                        const uint64_t val = v.r_val[F.entry + k];
                        if (!pw || pid > pb) { pb = pid; pw = W_PRESENT | val; }   // :1216-1221
                    }
                }
            } else {
                const uint32_t g = em;
                ++ei;
                const uint8_t t8 = v.m_type[g];
                const uint8_t fl = v.m_flags[g];
                if (t8 == MPX_MSG_PREPARE) {
                    if (fl & F_GRANTED) {
                        // FilterAcceptedValues over the prepare's ranges (:902-922);
                        // ranges are sorted by start and disjoint (ingest)
                        const uint64_t r0 = v.m_ent[g];
                        const uint32_t nr = v.m_cnt[g];
                        bool hit = false;
                        if (nr && in && (sw & W_PRESENT)) {
                            uint32_t lo = 0, hi = nr;          // last range with a <= iid
                            while (lo < hi) {
                                const uint32_t mid = (lo + hi) >> 1;
                                if (v.g_a[r0 + mid] <= iid) lo = mid + 1; else hi = mid;
                            }
                            hit = lo > 0 && iid < v.g_b[r0 + lo - 1];
                        }
                        emit(v, hit, g, 0, iid, sb, sw & W_HANDLE);
                        cP += hit;
                    }
                } else if (t8 == MPX_MSG_P_START) {
                    pb = pw = 0;
                } else if (t8 == MPX_MSG_PREPARE_REPLY) {
                    if (fl & F_QUORUM) {
                        const bool hit = in && pw;
                        emit(v, hit, g, 1, iid, pb, pw & W_HANDLE);
                        cQ += hit;
                        pb = pw = 0;                                  // :1105
                    }
                }
            }
        }
        const int any = __syncthreads_or(sw != 0);
        if (any) {
            if (in) {
                uint64_t *s = v.st + 2 * ((uint64_t)n * v.shard_len + li);
                *reinterpret_cast<ulonglong2 *>(s) = make_ulonglong2(sb, sw);
            }
            if (t == 0) v.st_valid[p] = 1;
            if (sw) dig += state_digest(n, iid, (sw & W_COMMITTED) ? 2 : 1, sb, sw & W_HANDLE);
        }
    }
    // workgroup reduction of the counters
    unsigned long long c[5] = {cA, cL, cP, cQ, dig};
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        unsigned long long x = c[i];
        for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
        c[i] = x;
    }
    if ((t & 63) == 0) {
#pragma unroll
        for (int i = 0; i < 5; ++i) red[t >> 6][i] = c[i];
    }
    __syncthreads();
    if (t < 5) {
        unsigned long long s = red[0][t] + red[1][t] + red[2][t] + red[3][t];
        const int slot = t == 0 ? PC_A : t == 1 ? PC_L : t == 2 ? PC_P : t == 3 ? PC_Q : PC_DSTATE;
        v.partials[8 * blockIdx.x + slot] = s;
    }
}

// Chosen log per bucket: every batch whose votes reached quorum contributes
// its instances; the first one wins, later ones must agree (safety).
__global__ __launch_bounds__(256) void k_chosen(DevView v, uint32_t partial_base)
{
    __shared__ uint16_t lidx[256];
    __shared__ unsigned long long red[4][2];
    const uint32_t t = threadIdx.x;
    lidx[t] = 0xFFFF;
    __syncthreads();
    unsigned long long cC = 0, dig = 0;
    for (uint64_t b = blockIdx.x; b < v.NB; b += gridDim.x) {
        const uint64_t li = (b << BSH) + t;
        const uint64_t iid = v.shard_begin + li;
        uint64_t cv = 0;
        for (uint64_t f = v.cf_off[b]; f < v.cf_off[b + 1]; ++f) {
            const Frag F = v.cfrags[f];
            const bool live = v.b_chosen[F.msg] != NONE32;
            int k = -1;
            if (F.flags & FR_DENSE) {
                const int d = (int)t - (int)F.start;
                if (d >= 0 && d < (int)F.count) k = d;
            } else {
                if (t < F.count) lidx[v.e_slot[F.entry + t]] = (uint16_t)t;
                __syncthreads();
                k = lidx[t] == 0xFFFF ? -1 : (int)lidx[t];
                __syncthreads();
                lidx[t] = 0xFFFF;
                __syncthreads();
            }
            if (live && k >= 0) {
                const uint64_t val = v.e_val[F.entry + k];
                if (!cv) { cv = W_PRESENT | val; ++cC; dig += chosen_digest(iid, val); }
                else if ((cv & W_HANDLE) != val) record_violation(v, MPX_V_CHOSEN_VALUE, 0, 0, iid);
            }
        }
        const int any = __syncthreads_or(cv != 0);
        if (any) {
            if (li < v.shard_len) v.chosen[li] = cv;
            if (t == 0) v.chosen_valid[b] = 1;
        }
    }
    unsigned long long c[2] = {cC, dig};
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        unsigned long long x = c[i];
        for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
        c[i] = x;
    }
    if ((t & 63) == 0) { red[t >> 6][0] = c[0]; red[t >> 6][1] = c[1]; }
    __syncthreads();
    if (t < 2) {
        unsigned long long s = red[0][t] + red[1][t] + red[2][t] + red[3][t];
        v.partials[8 * (partial_base + blockIdx.x) + (t == 0 ? PC_C : PC_DCHOSEN)] = s;
    }
}

__global__ __launch_bounds__(256) void k_reduce(DevView v, uint32_t n_partials)
{
    __shared__ unsigned long long red[4][8];
    const uint32_t t = threadIdx.x;
    unsigned long long s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t w = t; w < n_partials; w += 256)
#pragma unroll
        for (int i = 0; i < 8; ++i) s[i] += v.partials[8 * w + i];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        unsigned long long x = s[i];
        for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
        s[i] = x;
    }
    if ((t & 63) == 0)
        for (int i = 0; i < 8; ++i) red[t >> 6][i] = s[i];
    __syncthreads();
    if (t == 0) {
        unsigned long long r[8];
        for (int i = 0; i < 8; ++i) r[i] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
        unsigned long long ds = 0;
        for (uint32_t n = 0; n < v.N; ++n) ds += scalar_digest(n, v.node_scal[2 * n], v.node_scal[2 * n + 1]);
        unsigned long long *o = v.summary;
        o[SW_C] = r[PC_C]; o[SW_P] = r[PC_P]; o[SW_A] = r[PC_A]; o[SW_L] = r[PC_L];
        o[SW_MSGS] = v.num_msgs; o[SW_V] = v.viol->count;
        o[SW_DCHOSEN] = r[PC_DCHOSEN]; o[SW_DSTATE] = r[PC_DSTATE]; o[SW_DSCAL] = ds; o[SW_Q] = r[PC_Q];
        for (uint32_t n = 0; n < v.N && n < 24; ++n) {
            o[SW_NODE_SCAL + 2 * n] = v.node_scal[2 * n];
            o[SW_NODE_SCAL + 2 * n + 1] = v.node_scal[2 * n + 1];
        }
    }
}

__global__ void k_reset(DevView v, uint32_t n_partials)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t np = (uint64_t)v.N * v.NB;
    if (i < np) v.st_valid[i] = 0;
    if (i < v.NB) v.chosen_valid[i] = 0;
    if (i < 8ull * n_partials) v.partials[i] = 0;
    if (i == 0) {
        *v.out_cursor = 0;
        v.viol->code = v.viol->node = v.viol->seq = v.viol->iid = v.viol->count = 0;
    }
}

static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

int launch_run(const DevView &v, void *stream_, LaunchGeom g, void *ev_begin, void *ev_apply0,
               void *ev_apply1, void *ev_end)
{
    hipStream_t s = (hipStream_t)stream_;
    const uint32_t n_partials = g.apply_wgs + g.chosen_wgs;
    uint64_t reset_n = (uint64_t)v.N * v.NB;
    if (v.NB > reset_n) reset_n = v.NB;
    if (8ull * n_partials > reset_n) reset_n = 8ull * n_partials;
    if (ev_begin) (void)hipEventRecord((hipEvent_t)ev_begin, s);
    hipLaunchKernelGGL(k_reset, dim3(cdiv(reset_n ? reset_n : 1, 256)), dim3(256), 0, s, v, n_partials);
    if (v.num_chunks) {
        hipLaunchKernelGGL(k_scan_chunk, dim3(v.num_chunks), dim3(256), 0, s, v);
        hipLaunchKernelGGL(k_scan_node, dim3(v.N), dim3(256), 0, s, v);
        hipLaunchKernelGGL(k_scan_apply, dim3(v.num_chunks), dim3(256), 0, s, v);
    }
    hipLaunchKernelGGL(k_proposer, dim3(cdiv(v.N, 64)), dim3(64), 0, s, v);
    if (v.num_batches) hipLaunchKernelGGL(k_votes, dim3(cdiv(v.num_batches, 256)), dim3(256), 0, s, v);
    if (ev_apply0) (void)hipEventRecord((hipEvent_t)ev_apply0, s);
    hipLaunchKernelGGL(k_apply, dim3(g.apply_wgs), dim3(256), 0, s, v);
    if (ev_apply1) (void)hipEventRecord((hipEvent_t)ev_apply1, s);
    hipLaunchKernelGGL(k_chosen, dim3(g.chosen_wgs), dim3(256), 0, s, v, g.apply_wgs);
    hipLaunchKernelGGL(k_reduce, dim3(1), dim3(256), 0, s, v, n_partials);
    if (ev_end) (void)hipEventRecord((hipEvent_t)ev_end, s);
    return (int)hipGetLastError();
}

}  // namespace mpx
