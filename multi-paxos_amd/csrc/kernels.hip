// kernels.hip — CDNA4 (gfx950) kernels of the batched Multi-Paxos engine.
//
// One run = the whole resident trace applied from genesis state:
//   k_scan_chunk / k_headers
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
#include <hip/hip_ext.h>
#include "mpx_internal.hpp"

namespace mpx {

typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
// slot array access, slot_w bytes per slot (element index i = row * shard_len + li)
typedef unsigned char u8x4 __attribute__((ext_vector_type(4)));
__device__ inline uint32_t st_get(const DevView &v, uint64_t i)
{
    return v.slot_w == 1 ? (uint32_t)static_cast<const uint8_t *>(v.st)[i] : (uint32_t)static_cast<const uint16_t *>(v.st)[i];
}
__device__ inline void st_put(const DevView &v, uint64_t i, uint32_t x)
{
    if (v.slot_w == 1) static_cast<uint8_t *>(v.st)[i] = (uint8_t)x;
    else static_cast<uint16_t *>(v.st)[i] = (uint16_t)x;
}
// four consecutive slots i..i+3 (i a multiple of 4), non-temporal
__device__ inline void st_put4(const DevView &v, uint64_t i, uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
    if (v.slot_w == 1)
        __builtin_nontemporal_store(u8x4{(uint8_t)a, (uint8_t)b, (uint8_t)c, (uint8_t)d},
                                    reinterpret_cast<u8x4 *>(static_cast<uint8_t *>(v.st) + i));
    else
        __builtin_nontemporal_store(u16x4{(uint16_t)a, (uint16_t)b, (uint16_t)c, (uint16_t)d},
                                    reinterpret_cast<u16x4 *>(static_cast<uint16_t *>(v.st) + i));
}


__device__ inline void record_violation(const DevView &v, uint64_t code, uint64_t node, uint64_t seq, uint64_t iid)
{
    atomicAdd(&v.viol->count, 1ull);
    if (atomicCAS(&v.viol->code, 0ull, (unsigned long long)code) == 0ull) {
        v.viol->node = node;
        v.viol->seq = seq;
        v.viol->iid = iid;
    }
}

// wave-uniform read of lane i
__device__ inline uint64_t rl64(uint64_t x, uint32_t i)
{
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)x, i);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(x >> 32), i);
    return ((uint64_t)hi << 32) | lo;
}
__device__ inline uint32_t rl32(uint32_t x, uint32_t i) { return __builtin_amdgcn_readlane(x, i); }

// per-pair arrays (st_valid, the state rows' plan words) are pair-major like
// the fragment CSR, q = bucket * N + node, so the pair-per-lane kernels write
// them coalesced; the chosen log's plan words follow at N * NB + bucket
__device__ inline uint64_t sv_idx(const DevView &v, uint32_t n, uint64_t b) { return b * v.N + n; }
__device__ inline uint64_t plan_idx(const DevView &v, uint32_t row, uint64_t b)
{
    return row < v.N ? b * v.N + row : (uint64_t)v.N * v.NB + b;
}

__device__ inline void wave_lds_fence()
{
    // LDS instructions of one wave execute in order; keep the compiler from
    // reordering the scatter / gather around this point
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
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

// contribution of one scan record (SC_* type t, key) to promised (p) and
// max_seen (s): PREPARE ids feed both, ACCEPT ids and REJECT max_ids max_seen
// (multi/paxos.cpp:862-863,1363-1364,1229-1230); member keys carry the Acceptor
// incarnation in their top byte, so both restart with each new Acceptor
// (member/paxos.cpp:1700-1760) and an E_EPOCH record starts the incarnation
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ inline void contrib(uint8_t t, uint64_t key, uint64_t &p, uint64_t &s)
{
    const uint32_t k = t & SC_KIND;
    p = (k == SC_PREP || k == SC_PS) ? key : 0;
    s = k <= SC_PS ? key : 0;
}

__device__ inline uint64_t wave_max(uint64_t x)
{
#pragma unroll
    for (uint32_t d = 32; d >= 1; d >>= 1) {
        const uint64_t y = __shfl_xor(x, d, 64);
        x = x > y ? x : y;
    }
    return x;
}

// ------------------------------------------------- member role gates ----
// NodeImpl::ChangeMemberships (member/paxos.cpp:1864-1964) as it reaches each
// node's stream: an E_EPOCH marker moves the node to epochs[x].  The gate of a
// record follows from the node's roles after the last marker before it —
//   PREPARE / ACCEPT: the acceptor incarnation when the node has an Acceptor and
//     the message carries its version (Loop :749-756, :1702,1744), else 0 (dropped);
//   LEARN: G_PROP when it has a Proposer (Proposer::OnLearn's check, :1398);
//   replies / P_START / P_BATCH: (epoch + 1) << 16 when it has a Proposer;
// a marker itself: the new incarnation (bumped when the acceptor role flips:
// the Acceptor is deleted, :1952-1957, or created, :1897-1901) | G_ACCCLR on that
// flip | G_PRECLR when the Proposer is deleted, created or sees a new acceptor
// set (AcceptorsChanged, :1504-1549).  Four passes at the head of every member run.
// (an incremental window starts from the roles the windows before left, ee_init)
__device__ inline uint32_t ee_genesis(const DevView &v, uint32_t n)
{
    if (v.window) return v.ee_init[n];
    return (1u << EE_SEG_SHIFT) | (((v.ep_amask[0] >> n) & 1) ? EE_ACC : 0) | (((v.ep_pmask[0] >> n) & 1) ? EE_PROP : 0);
}

// the node's roles before message g (the state after its last marker < g)
__device__ inline uint32_t ee_before(const DevView &v, uint32_t n, uint32_t g)
{
    uint64_t lo = v.ee_off[n], hi = v.ee_off[n + 1];
    while (lo < hi) {                                   // first marker >= g
        const uint64_t mid = (lo + hi) >> 1;
        if (v.ee_msg[mid] < g) lo = mid + 1; else hi = mid;
    }
    return lo > v.ee_off[n] ? v.ee_state[lo - 1] : ee_genesis(v, n);
}

// The passes below look up, per record, the last marker of its node before it.
// The markers are few (one per membership step and node), so each block stages
// them in LDS once and its binary searches run there rather than as chains of
// dependent global loads (a trace with more than GATE_LDS markers searches
// global memory, as ee_before does).
constexpr uint32_t GATE_LDS = 2048;
struct GateLds { uint32_t msg[GATE_LDS], state[GATE_LDS]; uint64_t off[MPX_MAX_NODES + 1]; uint32_t init[MPX_MAX_NODES]; };
__device__ inline bool gate_stage(const DevView &v, GateLds &L)
{
    const uint64_t E = v.ee_off[v.N];
    const bool staged = E <= GATE_LDS;
    if (staged)
        for (uint32_t i = threadIdx.x; i < E; i += blockDim.x) { L.msg[i] = v.ee_msg[i]; L.state[i] = v.ee_state[i]; }
    for (uint32_t i = threadIdx.x; i <= v.N; i += blockDim.x) L.off[i] = v.ee_off[i];
    for (uint32_t i = threadIdx.x; i < v.N; i += blockDim.x) L.init[i] = ee_genesis(v, i);
    __syncthreads();
    return staged;
}
__device__ inline uint32_t ee_before_lds(const DevView &v, const GateLds &L, bool staged, uint32_t n, uint32_t g)
{
    if (!staged) return ee_before(v, n, g);
    uint32_t lo = (uint32_t)L.off[n], hi = (uint32_t)L.off[n + 1];
    const uint32_t first = lo;
    while (lo < hi) {                                   // first marker >= g
        const uint32_t mid = (lo + hi) >> 1;
        if (L.msg[mid] < g) lo = mid + 1; else hi = mid;
    }
    return lo > first ? L.state[lo - 1] : L.init[n];
}

// pass 1: one block per node; its markers' epochs and role sets are loaded in
// parallel into LDS, then one lane walks them in order (the incarnation counter
// and the previous roles are the only chain) and the block writes the results
__global__ __launch_bounds__(256) void k_gate_epochs(DevView v)
{
    __shared__ uint32_t sg[256], sgate[256], sst[256];
    __shared__ uint64_t sa[256], sp[256];
    const uint32_t n = blockIdx.x, j = threadIdx.x;
    const uint64_t k0 = v.ee_off[n], k1 = v.ee_off[n + 1];
    uint32_t st = ee_genesis(v, n);                      // lane 0's walk state
    uint64_t am_prev = v.ep_amask[st & 0xFFFF];         // the acceptor set of st's epoch
    for (uint64_t c = k0; c < k1; c += 256) {
        const uint32_t m = (uint32_t)(k1 - c < 256 ? k1 - c : 256);
        if (j < m) {
            const uint32_t g = v.ee_msg[c + j], x = v.m_ver[g];
            sg[j] = g; sa[j] = v.ep_amask[x]; sp[j] = v.ep_pmask[x];
            sst[j] = x;
        }
        __syncthreads();
        if (j == 0) {
            for (uint32_t i = 0; i < m; ++i) {
                const uint32_t x = sst[i];
                uint32_t seg = (st >> EE_SEG_SHIFT) & G_SEG;
                const bool acc = st & EE_ACC, prop = st & EE_PROP;
                const bool a2 = (sa[i] >> n) & 1, p2 = (sp[i] >> n) & 1;
                uint32_t gate = 0;
                if (a2 != acc) { ++seg; gate |= G_ACCCLR; }
                if (p2 != prop || (p2 && sa[i] != am_prev)) gate |= G_PRECLR;
                sgate[i] = gate | seg;
                st = x | (seg << EE_SEG_SHIFT) | (a2 ? EE_ACC : 0) | (p2 ? EE_PROP : 0);
                sst[i] = st;
                am_prev = sa[i];
            }
        }
        __syncthreads();
        if (j < m) {
            const uint32_t gate = sgate[j];
            v.m_gate[sg[j]] = gate;
            v.m_flags[sg[j]] = (uint8_t)(((gate & G_ACCCLR) ? F_ACCCLR : 0) | ((gate & G_PRECLR) ? F_PRECLR : 0));
            v.ee_state[c + j] = sst[j];
        }
        __syncthreads();
    }
    if (v.window && j == 0) v.ee_out[n] = st;           // the roles the next window starts from
}

// pass 2: every other record of the trace.  GATE_PER records per thread, their loads all issued
// before the block's marker staging (one occupancy round of blocks instead of several, each
// paying the staging and three dependent round trips: C5 45.8 us with one record per thread)
#ifndef MPX_GATE_PER
#define MPX_GATE_PER 4
#endif
constexpr uint32_t GATE_PER = MPX_GATE_PER;
__global__ __launch_bounds__(256) void k_gate_msgs(DevView v)
{
    __shared__ GateLds L;
    const uint64_t g0 = (uint64_t)blockIdx.x * 256 * GATE_PER + threadIdx.x;
    uint8_t t[GATE_PER], f[GATE_PER];
    uint32_t n[GATE_PER], ver[GATE_PER];
#pragma unroll
    for (uint32_t k = 0; k < GATE_PER; ++k) {           // (clamped, no branch: in flight during the staging)
        const uint64_t g = g0 + 256 * k, gc = g < v.num_msgs ? g : 0;
        t[k] = v.m_type[gc]; n[k] = v.m_node[gc]; ver[k] = v.m_ver[gc]; f[k] = v.m_flags[gc];
    }
    const bool staged = gate_stage(v, L);
#pragma unroll
    for (uint32_t k = 0; k < GATE_PER; ++k) {
        const uint64_t g = g0 + 256 * k;
        if (g >= v.num_msgs || t[k] == MPX_MSG_E_EPOCH) continue;
        const uint32_t st = ee_before_lds(v, L, staged, n[k], (uint32_t)g), ep = st & 0xFFFF;
        const bool acc = st & EE_ACC, prop = st & EE_PROP;
        uint32_t gate = 0;
        if (t[k] == MPX_MSG_PREPARE || t[k] == MPX_MSG_ACCEPT) {
            gate = acc && ver[k] == v.ep_ver[ep] ? (st >> EE_SEG_SHIFT) & G_SEG : 0;
        } else if (t[k] == MPX_MSG_COMMIT) {
            gate = prop ? G_PROP : 0;
            if (prop) v.m_flags[g] = f[k] | F_PROP;
        } else if (t[k] == MPX_MSG_PREPARE_REPLY || t[k] == MPX_MSG_ACCEPT_REPLY || t[k] == MPX_MSG_P_START ||
                   t[k] == MPX_MSG_P_BATCH) {
            gate = prop ? (ep + 1) << G_EPOCH_SHIFT : 0;
        }
        v.m_gate[g] = gate;
    }
}

// pass 3: the header-scan stream — a PREPARE / ACCEPT of a node without an
// Acceptor of its version leaves the stream (SC_NONE), the others (and the
// left-out ACCEPTs of header sharding, SC_VIRT) take the incarnation in their key,
// so one prefix max restarts with every new Acceptor; a marker's key is its
// incarnation.  Idempotent (a rerun finds the same keys and types).  GATE_PER records
// per thread as k_gate_msgs.
__global__ __launch_bounds__(256) void k_gate_scan(DevView v, uint64_t num_sc)
{
    __shared__ GateLds L;
    const uint64_t i0 = (uint64_t)blockIdx.x * 256 * GATE_PER + threadIdx.x;
    uint8_t t[GATE_PER];
    uint32_t g[GATE_PER], ver[GATE_PER];
    uint64_t key[GATE_PER];
#pragma unroll
    for (uint32_t k = 0; k < GATE_PER; ++k) {           // (clamped, no branch: in flight during the staging)
        const uint64_t i = i0 + 256 * k, ic = i < num_sc ? i : 0;
        t[k] = v.sc_type[ic]; g[k] = v.sc_idx[ic]; ver[k] = v.sc_ver[ic]; key[k] = v.sc_key[ic];
    }
    uint32_t gate[GATE_PER], nd[GATE_PER];
#pragma unroll
    for (uint32_t k = 0; k < GATE_PER; ++k) {
        const uint32_t gc = g[k] < v.num_msgs ? g[k] : 0;
        gate[k] = v.m_gate[gc]; nd[k] = v.m_node[gc];
    }
    const bool staged = gate_stage(v, L);
#pragma unroll
    for (uint32_t k = 0; k < GATE_PER; ++k) {
        const uint64_t i = i0 + 256 * k;
        if (i >= num_sc) continue;
        const uint32_t kind = t[k] & SC_KIND;
        if (kind == SC_PS) {
            v.sc_key[i] = (uint64_t)(gate[k] & G_SEG) << SEG_SHIFT;
            continue;
        }
        if (!(kind == SC_PREP || kind == SC_ACC || (kind == SC_SONLY && (t[k] & SC_VIRT)))) continue;
        uint32_t n;
        if (t[k] & SC_VIRT) {                           // the node whose scan range holds i
            uint32_t lo = 0, hi = v.N;
            while (hi - lo > 1) { const uint32_t mid = (lo + hi) >> 1; if (v.sc_off[mid] <= i) lo = mid; else hi = mid; }
            n = lo;
        } else {
            n = nd[k];
        }
        const uint32_t st = ee_before_lds(v, L, staged, n, g[k]), ep = st & 0xFFFF;
        if ((st & EE_ACC) && ver[k] == v.ep_ver[ep])
            v.sc_key[i] = (key[k] & LOW56) | ((uint64_t)((st >> EE_SEG_SHIFT) & G_SEG) << SEG_SHIFT);
        else
            v.sc_type[i] = SC_NONE;                     // dropped silently (:1702,1744)
    }
}

// pass 4: vote lists — a reply counts only while its node has a Proposer
// (epoch bits beside the list) and only for a batch made while it had one and
// not reset since (a marker with G_PRECLR clears accepting_values_)
__global__ __launch_bounds__(256) void k_gate_votes(DevView v)
{
    __shared__ GateLds L;                               // msg: the markers, state: their G_PRECLR bit
    const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t g0 = 0, n = 0;
    // (a window: a batch of an earlier window has no message here, b_msg NONE32; its node is b_node)
    if (j < v.num_batches) { g0 = v.b_msg[j]; n = v.window ? v.b_node[j] : v.m_node[g0]; }
    const uint64_t E = v.ee_off[v.N];
    const bool staged = E <= GATE_LDS;
    if (staged)
        for (uint32_t i = threadIdx.x; i < E; i += blockDim.x) {
            const uint32_t g = v.ee_msg[i];
            L.msg[i] = g; L.state[i] = v.m_gate[g] & G_PRECLR;
        }
    for (uint32_t i = threadIdx.x; i <= v.N; i += blockDim.x) L.off[i] = v.ee_off[i];
    __syncthreads();
    if (j >= v.num_batches) return;
    uint32_t kill = NONE32;
    const bool carried = g0 == NONE32;                  // first marker of the window: "after the batch"
    const uint32_t gid = v.window && j < v.num_batches ? v.b_gid[j] : 0;
    const uint32_t gs = carried ? 0 : g0;
    if (carried && (v.g_done[gid] & 2)) {
        kill = 0;                                       // cleared in an earlier window
    } else if (!carried && !(v.m_gate[g0] >> G_EPOCH_SHIFT)) {
        kill = g0;
    } else if (staged) {
        uint32_t lo = (uint32_t)L.off[n], hi = (uint32_t)L.off[n + 1];
        const uint32_t end = hi;
        while (lo < hi) {                               // first marker after the batch
            const uint32_t mid = (lo + hi) >> 1;
            if (L.msg[mid] < gs) lo = mid + 1; else hi = mid;
        }
        for (; lo < end; ++lo)
            if (L.state[lo]) { kill = L.msg[lo]; break; }
    } else {
        uint64_t lo = v.ee_off[n], hi = v.ee_off[n + 1];
        while (lo < hi) {                               // first marker after the batch
            const uint64_t mid = (lo + hi) >> 1;
            if (v.ee_msg[mid] < gs) lo = mid + 1; else hi = mid;
        }
        for (; lo < v.ee_off[n + 1]; ++lo)
            if (v.m_gate[v.ee_msg[lo]] & G_PRECLR) { kill = v.ee_msg[lo]; break; }
    }
    if (v.window && kill != NONE32) v.g_done[gid] |= 2;   // no vote counts in a later window
    // (the replies one per thread, each finding its batch in the block's offsets:
    // 21.8 vs 15.1 us at C5)
    for (uint64_t r = v.b_rep_off[j]; r < v.b_rep_off[j + 1]; ++r) {
        const uint32_t g = v.b_rep[r];
        const uint32_t ep = g < kill ? v.m_gate[g] >> G_EPOCH_SHIFT : 0;
        v.b_rsrc[r] = (v.b_rsrc[r] & 0xFFFF) | (ep << 16);
    }
}


// the summary word a partial-row column adds into (-1: none)
__device__ inline int summary_word(uint32_t pc)
{
    return pc == PC_C ? SW_C : pc == PC_P ? SW_P : pc == PC_A ? SW_A : pc == PC_L ? SW_L :
           pc == PC_DCHOSEN ? SW_DCHOSEN : pc == PC_DSTATE ? SW_DSTATE : pc == PC_Q ? SW_Q : -1;
}

// Per-step reset of what the step accumulates (k_reset, or the head of k_scan_chunk when
// it is the step's first kernel): thread t of T zeroes its share, grid-stride.  The scalars
// of a node with scan records are left to its last scan chunk; the violation record is
// double-buffered (a launch records into v.viol and clears v.viol_next, the one the next
// launch records into), so no kernel of a launch both clears and records.
__device__ inline void reset_state(const DevView &v, uint32_t n_partials, uint64_t t, uint64_t T)
{
    const uint64_t np = (uint64_t)v.N * v.NB;
    const uint64_t n16 = v.window ? 0 : (np + 15) / 16;     // (a window keeps no slot rows)
    for (uint64_t i = t; i < n16; i += T) {          // st_valid: 16 bytes per thread, byte tail
        if (16 * i + 16 <= np) *reinterpret_cast<uint4 *>(v.st_valid + 16 * i) = uint4{0, 0, 0, 0};
        else for (uint64_t k = 16 * i; k < np; ++k) v.st_valid[k] = 0;
    }
    for (uint64_t i = t; i < (v.window ? 0 : v.NB); i += T) v.chosen_valid[i] = 0;
    for (uint64_t i = t; i < 8ull * n_partials; i += T) v.partials[i] = 0;
    // nodes without messages keep promised = max_seen = 0 (a window: what the windows before left;
    // member keys carry the Acceptor's incarnation above LOW56, the readback does not)
    for (uint64_t i = t; i < 2ull * v.N; i += T) {
        const uint32_t n = (uint32_t)(i >> 1);
        if (v.node_chunk_off[n + 1] != v.node_chunk_off[n]) continue;   // the scan writes them
        const uint64_t k = v.window ? v.scal_base[i] : 0;
        v.node_scal[i] = v.semantics == MPX_SEM_MEMBER ? k & LOW56 : k;
        if (v.window) v.scal_key[i] = k;
    }
    for (uint64_t i = t; i < v.out_subs; i += T) v.out_cursor[OUT_STRIDE * i] = 0;
    if (t == 0) {
        v.fast_rest[0] = 0;
        v.fast_rest[1] = 0;                          // k_chosen's last-block ticket
        *v.gp_dyn_n = 0;
        *v.gp_ext_n = 0;
        *v.gp_chk_n = 0;
        *v.gp_rt_n = 0;
        if (v.window) *v.outv_n = 0;
        for (uint32_t pc = 0; pc < 8; ++pc)          // the counter words k_reduce's workgroups add into
            if (summary_word(pc) >= 0) v.summary[summary_word(pc)] = 0;
        v.viol_next->code = v.viol_next->node = v.viol_next->seq = v.viol_next->iid = v.viol_next->count = 0;
    }
}

// Chunk aggregates over the header-scan stream: max of the PREPARE ids and of
// the max_seen contributions of CH records (order-free, coalesced)
// RESET: the step's first kernel also does k_reset's work (one launch less per step)
// Loads: four records per thread per round — their types as one aligned u32 and their keys
// as two 16-byte loads (a wave reads 256 B of types and 4 KiB of keys per round) instead of
// a byte and a u64 per record; the words may start before the chunk and end after it (the
// record index decides), and device buffers are padded to 64 bytes (DevBuf::alloc)
template <bool RESET, uint32_t CH>
__global__ __launch_bounds__(256) void k_scan_chunk(DevView v, uint32_t n_partials)
{
    __shared__ uint64_t l[2][4];
    if (RESET) reset_state(v, n_partials, (uint64_t)blockIdx.x * 256 + threadIdx.x, (uint64_t)gridDim.x * 256);
    const uint32_t c = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t beg = v.chunk_beg[c], end = v.chunk_end[c];
    const uint64_t w0 = beg >> 2, w1 = (end + 3) >> 2;
    constexpr uint32_t WR = (CH / 4 + 256) / 256;             // words of a chunk, one slack word
    const uint32_t *tw = reinterpret_cast<const uint32_t *>(v.sc_type);
    const u64x2 *kw = reinterpret_cast<const u64x2 *>(v.sc_key);
    uint32_t ty[WR];
    u64x2 k0[WR], k1[WR];
#pragma unroll
    for (uint32_t i = 0; i < WR; ++i) {                      // all loads in flight at once
        const uint64_t wd = w0 + threadIdx.x + 256ull * i;
        ty[i] = (uint32_t)SC_NONE * 0x01010101u;
        k0[i] = u64x2{0, 0}; k1[i] = u64x2{0, 0};
        if (wd < w1) { ty[i] = tw[wd]; k0[i] = kw[2 * wd]; k1[i] = kw[2 * wd + 1]; }
    }
    uint64_t lp = 0, ls = 0;
#pragma unroll
    for (uint32_t i = 0; i < WR; ++i) {
        const uint64_t g0 = 4 * (w0 + threadIdx.x + 256ull * i);
        const uint64_t key[4] = {k0[i].x, k0[i].y, k1[i].x, k1[i].y};
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const bool in = g0 + j >= beg && g0 + j < end;
            uint64_t p, s;
            contrib(in ? (uint8_t)(ty[i] >> (8 * j)) : (uint8_t)SC_NONE, key[j], p, s);
            lp = lp > p ? lp : p;
            ls = ls > s ? ls : s;
        }
    }
    lp = wave_max(lp);
    ls = wave_max(ls);
    if (lane == 0) { l[0][w] = lp; l[1][w] = ls; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t tp = 0, ts = 0;
        for (int i = 0; i < 4; ++i) { tp = tp > l[0][i] ? tp : l[0][i]; ts = ts > l[1][i] ? ts : l[1][i]; }
        v.chunk_agg[2 * c] = tp;
        v.chunk_agg[2 * c + 1] = ts;
    }
}

__global__ __launch_bounds__(256) void k_scan_node(DevView v)
{
    __shared__ uint64_t l[8];
    const uint32_t n = blockIdx.x;
    const uint32_t c0 = v.node_chunk_off[n], c1 = v.node_chunk_off[n + 1];
    uint64_t carry_p = v.window ? v.scal_base[2 * n] : 0, carry_s = v.window ? v.scal_base[2 * n + 1] : 0;
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
    if (v.window && threadIdx.x == 0) { v.scal_key[2 * n] = carry_p; v.scal_key[2 * n + 1] = carry_s; }
    if (v.semantics == MPX_SEM_MEMBER) { carry_p &= LOW56; carry_s &= LOW56; }   // current incarnation
    if (threadIdx.x == 0) { v.node_scal[2 * n] = carry_p; v.node_scal[2 * n + 1] = carry_s; }
}

// Per scan record: granted / reject flags and the max_seen a REJECT carries.
// Wave w of the chunk's block owns CH / 4 consecutive records, 64 per
// round (coalesced), staged in LDS between the two phases: (1) wave maxima ->
// the wave's carry-in, (2) per round the promised value before each record
// (an exclusive wave scan, only in rounds that hold a PREPARE) and, in rounds
// with a REJECT, the inclusive max_seen scan.  Flags go to the record's
// message (m_flags[sc_idx]); messages outside the stream keep their static flags.
// (the body of one chunk's workgroup: k_scan_apply, or a scan block of k_headers)
template <bool MEMBER, uint32_t CH>
__device__ inline void scan_apply_chunk(const DevView &v, const uint32_t c, uint64_t (&l)[2][4], uint64_t (&lc)[2][4],
                                        uint64_t *lky, uint8_t *lty, uint32_t *lix)
{
    constexpr uint32_t SCAN_ROUNDS = CH / 256;                // rounds of 64 records per wave
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t beg = v.chunk_beg[c], end = v.chunk_end[c];
    const uint64_t wb = beg + (uint64_t)w * (CH / 4) + lane;
    const uint32_t lb = w * (CH / 4) + lane;
    constexpr bool member = MEMBER;
    // staging: the chunk's records into LDS (record g at g - beg), four per thread per
    // round — their types as one aligned u32, keys and message indices as 16-byte loads
    // (as k_scan_chunk); the words may start before the chunk and end after it
    const uint64_t w0 = beg >> 2, w1 = (end + 3) >> 2;
    constexpr uint32_t WR = (CH / 4 + 256) / 256;
    const uint32_t *tw = reinterpret_cast<const uint32_t *>(v.sc_type);
    const u64x2 *kw = reinterpret_cast<const u64x2 *>(v.sc_key);
    const u32x4 *iw = reinterpret_cast<const u32x4 *>(v.sc_idx);
    uint32_t ty[WR];
    u64x2 k0[WR], k1[WR];
    u32x4 ix[WR];
#pragma unroll
    for (uint32_t i = 0; i < WR; ++i) {                      // all loads in flight at once
        const uint64_t wd = w0 + threadIdx.x + 256ull * i;
        ty[i] = 0; k0[i] = u64x2{0, 0}; k1[i] = u64x2{0, 0}; ix[i] = u32x4{0, 0, 0, 0};
        if (wd < w1) { ty[i] = tw[wd]; k0[i] = kw[2 * wd]; k1[i] = kw[2 * wd + 1]; ix[i] = iw[wd]; }
    }
    // carry-in = max over the node's earlier chunk aggregates (k_scan_chunk),
    // read here from L2 instead of a separate per-node scan kernel (its loads in flight
    // with the staging loads) — O(chunks^2) per node, so a node with more than
    // SCAN_INLINE_CHUNKS chunks reads the carry k_scan_node computed instead (v.scan_node_pass)
    const uint32_t cn = v.chunk_node[c];
    const uint32_t c0 = v.node_chunk_off[cn], c1 = v.node_chunk_off[cn + 1];
    uint64_t xp = 0, xs = 0;
    if (v.scan_node_pass) {
        if (threadIdx.x == 0) { xp = v.chunk_carry[2 * c]; xs = v.chunk_carry[2 * c + 1]; }
    } else {
        if (v.window && threadIdx.x == 0) { xp = v.scal_base[2 * cn]; xs = v.scal_base[2 * cn + 1]; }   // earlier windows
        for (uint32_t k = c0 + threadIdx.x; k < c; k += 256) {
            const uint64_t ap = v.chunk_agg[2 * k], as = v.chunk_agg[2 * k + 1];
            xp = xp > ap ? xp : ap;
            xs = xs > as ? xs : as;
        }
    }
    const uint32_t len = (uint32_t)(end - beg);
#pragma unroll
    for (uint32_t i = 0; i < WR; ++i) {
        const uint64_t g0 = 4 * (w0 + threadIdx.x + 256ull * i);
        const uint64_t key[4] = {k0[i].x, k0[i].y, k1[i].x, k1[i].y};
        const uint32_t idx[4] = {ix[i].x, ix[i].y, ix[i].z, ix[i].w};
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
            if (g0 + j >= beg && g0 + j < end) {
                const uint32_t o = (uint32_t)(g0 + j - beg);
                lty[o] = (uint8_t)(ty[i] >> (8 * j));
                lky[o] = key[j];
                lix[o] = idx[j];
            }
    }
    for (uint32_t o = len + threadIdx.x; o < CH; o += 256) { lty[o] = SC_NONE; lky[o] = 0; }
    __syncthreads();
    // the wave's own records (its CH / 4, 64 per round): its maxima
    uint64_t lp = 0, ls = 0;
#pragma unroll
    for (uint32_t r = 0; r < SCAN_ROUNDS; ++r) {
        uint64_t p, s;
        contrib(lty[lb + 64 * r], lky[lb + 64 * r], p, s);
        lp = lp > p ? lp : p;
        ls = ls > s ? ls : s;
    }
    xp = wave_max(xp);
    xs = wave_max(xs);
    lp = wave_max(lp);
    ls = wave_max(ls);
    if (lane == 0) { l[0][w] = lp; l[1][w] = ls; lc[0][w] = xp; lc[1][w] = xs; }
    __syncthreads();
    uint64_t cp = 0, cs = 0;                   // wave-uniform running maxima
    for (uint32_t i = 0; i < 4; ++i) { cp = cp > lc[0][i] ? cp : lc[0][i]; cs = cs > lc[1][i] ? cs : lc[1][i]; }
    if (c == c1 - 1 && threadIdx.x == 0) {
        // the node's last chunk: its promised / max_seen after the whole stream
        uint64_t tp = cp, ts = cs;
        for (uint32_t i = 0; i < 4; ++i) { tp = tp > l[0][i] ? tp : l[0][i]; ts = ts > l[1][i] ? ts : l[1][i]; }
        if (v.window) { v.scal_key[2 * cn] = tp; v.scal_key[2 * cn + 1] = ts; }   // the next window's carry-in
        if (member) { tp &= LOW56; ts &= LOW56; }   // current incarnation
        v.node_scal[2 * cn] = tp;
        v.node_scal[2 * cn + 1] = ts;
    }
    for (uint32_t i = 0; i < w; ++i) { cp = cp > l[0][i] ? cp : l[0][i]; cs = cs > l[1][i] ? cs : l[1][i]; }
    ls = 0;                                    // this lane's max_seen contributions since cs
#pragma unroll 1
    for (uint32_t r = 0; r < SCAN_ROUNDS; ++r) {
        const uint64_t g = wb + 64 * r;
        if (!__ballot(g < end)) break;
        const uint8_t t = lty[lb + 64 * r];    // staged above, before the barrier
        const uint64_t key = lky[lb + 64 * r];
        const uint32_t kind = t & SC_KIND;
        uint64_t p, s;
        contrib(t, key, p, s);
        // promised before this record
        uint64_t prom = cp;
        if (__ballot(p != 0)) {
            uint64_t x = wave_scan_max(p);
            cp = cp > rl64(x, 63) ? cp : rl64(x, 63);
            x = __shfl_up(x, 1, 64);
            if (lane == 0) x = 0;
            prom = prom > x ? prom : x;
        }
        uint8_t f = 0;
        if (kind == SC_PREP || kind == SC_ACC) {
            uint64_t id = key, pr = prom;
            if (member) {
                // the Acceptor's own promise: zero when prom is an earlier incarnation's
                id = key & LOW56;
                pr = (prom >> SEG_SHIFT) == (key >> SEG_SHIFT) ? (prom & LOW56) : 0;
            }
            if (kind == SC_PREP) {
                if (id > pr) f = F_GRANTED;                             // :865 / member :1711
                else if (id < pr) f = F_REJECT;                         // :894 / :1734
            } else {
                f = id >= pr ? F_GRANTED : F_REJECT;                    // :1366 / :1753
            }
        }
        // max_seen after this record, for the REJECTs it carries (:894,1398)
        if (__ballot(f & F_REJECT)) {
            const uint64_t pre = wave_max(ls);
            cs = cs > pre ? cs : pre;
            ls = 0;
            uint64_t x = wave_scan_max(s);
            x = x > cs ? x : cs;
            if (f & F_REJECT) v.m_maxseen[lix[lb + 64 * r]] = member ? x & LOW56 : x;
        }
        ls = ls > s ? ls : s;
        if (g < end && (kind <= SC_ACC || (t & SC_BAD))) {
            const uint32_t idx = lix[lb + 64 * r];
            if (kind <= SC_ACC) v.m_flags[idx] = f | ((t & SC_BAD) ? F_BADNODE : 0);
            if (t & SC_BAD) {
                const uint32_t n = v.m_node[idx];
                record_violation(v, MPX_V_BAD_NODE, n, idx - v.node_off[n], 0);
            }
        }
    }
}


// --------------------------------------------------------- proposer side --
// Promise quorum per node (OnPrepareReply, multi/paxos.cpp:1036-1057; member
// Proposer::OnPrepareReply, member/paxos.cpp:1158-1182): one wave per node over
// its P_START / PREPARE_REPLY (/ E_EPOCH) records, 64 per window, all lanes at
// once.  A P_START (a gated one in member) starts a round — new ballot,
// preparing, empty promise set — and a member E_EPOCH that resets the proposer
// ends one (idle until the next P_START); each record's round is the last such
// head at or before it in the window, or the state carried in.  A reply
// counts while its round is preparing and its ballot is the round's (:1038);
// the promise set up to it is a segmented OR scan of the counted replies'
// acceptor bits, and the round's quorum reply is its first reply whose set
// reaches |acceptors|/2+1 (:1047) — later replies of the round are not counted.
__device__ inline uint64_t shfl64(uint64_t x, int src)
{
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)x, src, 64), hi = (uint32_t)__shfl((int)(uint32_t)(x >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}
__device__ inline uint64_t shfl64_up(uint64_t x, uint32_t d)
{
    const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)x, d, 64), hi = (uint32_t)__shfl_up((int)(uint32_t)(x >> 32), d, 64);
    return ((uint64_t)hi << 32) | lo;
}

// The window walk over records [i0, i1) of node n's list.  `known`: the state
// carried in (cb, cprep, cmask) is the real one; otherwise records before the
// range's first round head are left alone (their round started in an earlier
// chunk: k_prop_node walks them).  Returns, in `head`, the offset of the first
// head from i0 (~0u: none).
struct PropState { uint64_t cb, cmask; uint32_t cprep, known; };
__device__ inline void prop_range(const DevView &v, uint32_t n, uint64_t i0, uint64_t i1, PropState &st, uint32_t &head)
{
    const uint32_t lane = threadIdx.x & 63;
    const bool member = v.semantics == MPX_SEM_MEMBER;
    const uint64_t le = ~0ull >> (63 - lane);                  // lanes 0..lane
    const uint64_t all_nodes = v.N >= 64 ? ~0ull : ((1ull << v.N) - 1);
    head = ~0u;
    for (uint64_t base = i0; base < i1; base += 64) {
        const uint32_t cnt = (uint32_t)(i1 - base < 64 ? i1 - base : 64);
        const bool valid = lane < cnt;
        uint32_t g = 0, t = 0xFF, src = 0, gt = 0;
        uint64_t b = 0, am = all_nodes;
        if (valid) {
            g = v.pl_msg[base + lane];
            t = v.m_type[g]; b = v.m_ballot[g]; src = v.m_src[g];
            if (member) {
                gt = v.m_gate[g];
                am = (gt >> G_EPOCH_SHIFT) ? v.ep_amask[(gt >> G_EPOCH_SHIFT) - 1] : 0;
            }
        }
        const bool gated = !member || (gt >> G_EPOCH_SHIFT) != 0;
        const bool ps = valid && gated && t == MPX_MSG_P_START;                     // round head: preparing
        const bool ec = valid && member && t == MPX_MSG_E_EPOCH && (gt & G_PRECLR); // round head: idle
        const bool rep = valid && gated && t == MPX_MSG_PREPARE_REPLY;
        const uint64_t heads = __ballot(ps || ec), psm = __ballot(ps);
        if (heads && head == ~0u) head = (uint32_t)(base - i0) + (uint32_t)__builtin_ctzll(heads);
        const uint64_t hm = heads & le;
        const int sh = hm ? 63 - __builtin_clzll(hm) : -1;                         // this record's round head
        const bool mine = sh >= 0 || st.known;                                      // its round's state is known here
        const uint64_t rb = sh >= 0 ? shfl64(b, sh) : st.cb;
        const bool prep0 = sh >= 0 ? ((psm >> sh) & 1) != 0 : st.cprep != 0;
        const uint64_t mask0 = sh >= 0 ? 0 : st.cmask;
        const bool m1 = rep && prep0 && b == rb;                                    // :1038 / :1160
        const bool bad = m1 && (src >= 64 || !((am >> src) & 1));                  // :1040 / :1163
        const bool match = m1 && !bad;
        // segmented inclusive OR scan of the counted replies' acceptor bits
        uint64_t x = match ? 1ull << src : 0;
        bool f = ps || ec;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint64_t y = shfl64_up(x, d);
            const bool fy = __shfl_up((int)f, d, 64) != 0;
            if (lane >= d && !f) { x |= y; f = f || fy; }
        }
        const uint64_t incl = x | mask0;
        const uint32_t Q = member ? (uint32_t)__popcll(am) / 2 + 1 : v.quorum;
        const bool cand = match && (uint32_t)__popcll(incl) >= Q;
        const uint64_t cm = __ballot(cand);
        const uint64_t seg = le & ~((sh > 0 ? (1ull << sh) : 1ull) - 1);           // lanes sh..lane (or 0..lane)
        const uint64_t cseg = cm & seg;
        const uint32_t fc = cseg ? (uint32_t)__builtin_ctzll(cseg) : 64;          // the round's quorum reply
        uint32_t fl = 0;
        if (match && fc >= lane) fl = F_COUNTED | (fc == lane ? F_QUORUM : 0);
        if (mine && bad && fc > lane) record_violation(v, MPX_V_BAD_NODE, n, g - v.node_off[n], 0);
        if (mine && rep) v.m_flags[g] = (uint8_t)fl;    // a reply's flags are this kernel's alone (static ones are 0)
        // carry the last record's round into the next window
        const uint32_t L = cnt - 1;
        if (psm) st.cb = rl64(b, 63 - __builtin_clzll(psm));
        const bool prepL = rl32((uint32_t)prep0, L) && !rl32((uint32_t)(cseg != 0), L);
        st.cprep = prepL;
        st.cmask = prepL ? rl64(incl, L) : 0;
        if (heads) st.known = 1;
    }
}

// Promise quorums, pass 1: one wave per chunk of PROP_CHUNK records of a node's
// list; a node's first chunk starts from the genesis state (proposal_id_ = 0,
// :338; not preparing), later ones from their first round head — the records
// before it wait for k_prop_node.  Writes the chunk's first head and its state
// after the last record (valid when it has a head or is the node's first).
__device__ inline void prop_chunk_wave(const DevView &v, const uint32_t c)
{
    const uint32_t n = v.pc_node[c];
    const uint64_t i0 = v.pc_beg[c], i1 = v.pc_end[c];
    PropState st{0, 0, 0, i0 == v.pl_off[n] ? 1u : 0u};
    if (v.window && st.known)                          // a window's first chunk: the round carried in
        st = PropState{v.prop_in[3 * n], v.prop_in[3 * n + 1], (uint32_t)v.prop_in[3 * n + 2], 1u};
    uint32_t head;
    prop_range(v, n, i0, i1, st, head);
    if ((threadIdx.x & 63) == 0) {
        v.pc_head[c] = head;
        v.pc_state[3 * c] = st.cb; v.pc_state[3 * c + 1] = st.cmask; v.pc_state[3 * c + 2] = st.cprep | (st.known << 1);
    }
}

// pass 2: one wave per node, its chunks in order: the records before each
// chunk's first head under the state carried from the chunk before
__global__ __launch_bounds__(64) void k_prop_node(DevView v)
{
    const uint32_t n = blockIdx.x;
    if (n >= v.N) return;
    const uint32_t c0 = v.pc_node_off[n], c1 = v.pc_node_off[n + 1];
    if (c0 == c1) {
        if (v.window && threadIdx.x < 3) v.prop_out[3 * n + threadIdx.x] = v.prop_in[3 * n + threadIdx.x];
        return;
    }
    PropState st{v.pc_state[3 * c0], v.pc_state[3 * c0 + 1], (uint32_t)(v.pc_state[3 * c0 + 2] & 1), 1};
    for (uint32_t c = c0 + 1; c < c1; ++c) {
        const uint64_t i0 = v.pc_beg[c], i1 = v.pc_end[c];
        const uint32_t h = v.pc_head[c];
        uint32_t dummy;
        prop_range(v, n, i0, h == ~0u ? i1 : i0 + h, st, dummy);
        if (h != ~0u) {
            st.cb = v.pc_state[3 * c]; st.cmask = v.pc_state[3 * c + 1]; st.cprep = (uint32_t)(v.pc_state[3 * c + 2] & 1);
        }
    }
    if (v.window && threadIdx.x == 0) {                // the round the next window starts from
        v.prop_out[3 * n] = st.cb; v.prop_out[3 * n + 1] = st.cmask; v.prop_out[3 * n + 2] = st.cprep;
    }
}

// Accept-vote quorum (OnAcceptReply, multi/paxos.cpp:1406-1427; member
// Proposer::OnAcceptReply, member/paxos.cpp:1317-1343): AcceptingValues::
// accepted_ as a 64-bit acceptor mask per batch, chosen at |mask| >= quorum.
// A wave takes 64 consecutive batches: their vote lists are one contiguous
// range of the CSR, staged through LDS with coalesced loads of the replies'
// headers (ballot, acceptor, epoch: laid out beside the list at ingest), then
// each lane walks its own batch's replies in order from LDS.
constexpr uint32_t VOTE_LDS = 768;             // reply headers staged per wave
__device__ inline void votes_block(const DevView &v, const uint32_t blk, uint64_t (*lbal)[VOTE_LDS],
                                   uint32_t (*lsrc)[VOTE_LDS])
{
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t j0 = ((uint64_t)blk * 4 + wv) * 64;
    if (j0 >= v.num_batches) return;
    const uint64_t j = j0 + lane;
    const bool have = j < v.num_batches;
    const uint64_t jl = j0 + 64 < v.num_batches ? j0 + 64 : v.num_batches;
    const uint64_t r0 = v.b_rep_off[j0], r1 = v.b_rep_off[jl];
    const uint64_t rs = have ? v.b_rep_off[j] : r1, re = have ? v.b_rep_off[j + 1] : r1;
    const uint64_t staged = r1 - r0 < VOTE_LDS ? r1 - r0 : VOTE_LDS;
    {   // every staging load in flight at once, then the LDS writes
        constexpr uint32_t K = VOTE_LDS / 64;
        uint64_t xb[K];
        uint32_t xs[K];
#pragma unroll
        for (uint32_t k = 0; k < K; ++k) {
            const uint64_t x = lane + 64 * k;
            xb[k] = 0; xs[k] = 0;
            if (x < staged) { xb[k] = v.b_rbal[r0 + x]; xs[k] = v.b_rsrc[r0 + x]; }
        }
#pragma unroll
        for (uint32_t k = 0; k < K; ++k)
            if (lane + 64 * k < staged) { lbal[wv][lane + 64 * k] = xb[k]; lsrc[wv][lane + 64 * k] = xs[k]; }
    }
    wave_lds_fence();
    const uint64_t ballot = have ? v.b_bal[j] : 0;
    const bool member = v.semantics == MPX_SEM_MEMBER;
    uint64_t mask = 0;
    uint64_t chosen_r = ~0ull;
    // a window: the batch's accepted_ so far, and no more votes once an earlier window chose it
    // (OnAcceptReply erases the batch at quorum, multi/paxos.cpp:1416-1424)
    const uint32_t gid = v.window && have ? v.b_gid[j] : 0;
    const bool done = v.window && have && (v.g_done[gid] & 1);
    if (v.window && have) mask = v.g_mask[gid];
    for (uint64_t r = done ? re : rs; r < re; ++r) {
        const uint64_t o = r - r0;
        const uint64_t b = o < VOTE_LDS ? lbal[wv][o] : v.b_rbal[r];
        const uint32_t x = o < VOTE_LDS ? lsrc[wv][o] : v.b_rsrc[r];
        const uint32_t a = x & 0xFFFF;
        uint64_t am;
        if (member) {
            if (!(x >> 16)) continue;                    // no Proposer, or its batch was cleared (k_gate_votes)
            am = v.ep_amask[(x >> 16) - 1];              // the node's acceptors at the reply (:1324-1327)
        } else {
            if (b != ballot) continue;                   // :1408
            am = v.N >= 64 ? ~0ull : ((1ull << v.N) - 1);
        }
        if (a >= 64 || !((am >> a) & 1)) {              // :1414 / :1324
            const uint32_t g = v.b_rep[r];
            const uint32_t n = v.m_node[g];
            record_violation(v, MPX_V_BAD_NODE, n, g - v.node_off[n], 0);
            continue;
        }
        mask |= 1ull << a;
        const uint32_t q = member ? (uint32_t)__popcll(am) / 2 + 1 : v.quorum;
        if ((uint32_t)__popcll(mask) >= q) { chosen_r = r; break; }   // :1416
    }
    if (have) v.b_chosen[j] = chosen_r == ~0ull ? NONE32 : v.b_rep[chosen_r];
    if (v.window && have && !done) {
        v.g_mask[gid] = mask;
        if (chosen_r != ~0ull) v.g_done[gid] |= 1;
    }
}

// The header kernels that depend only on the scan chunks' aggregates (or on nothing) in
// one launch — the scan's flag pass (scan_apply_chunk), the promise-quorum chunks (one per
// wave) and the accept votes (votes_block) — by workgroup range: fewer dependent launches
// per step (each costs a dispatch and a floor of a few us).  They touch disjoint outputs: the
// scan's flags on PREPARE / ACCEPT records, the quorum flags on PREPARE_REPLYs, b_chosen.
// LDS: the larger of the scan's chunk staging and the votes' reply staging, shared.
constexpr uint32_t HDR_LDS_WORDS = (VOTE_LDS * 4 * 12 + 7) / 8;   // 4 waves x 768 x (8 + 4) bytes
static_assert(HDR_LDS_WORDS * 8 >= SCAN_CHUNK * 13, "the scan staging fits");
template <bool MEMBER, uint32_t CH>
__global__ __launch_bounds__(256) void k_headers(DevView v, uint32_t nb_scan, uint32_t nb_prop)
{
    __shared__ uint64_t raw[HDR_LDS_WORDS];
    __shared__ uint64_t l[2][4], lc[2][4];
    const uint32_t b = blockIdx.x;
    if (b < nb_scan) {
        scan_apply_chunk<MEMBER, CH>(v, b, l, lc, raw, reinterpret_cast<uint8_t *>(raw + CH),
                                     reinterpret_cast<uint32_t *>(raw + CH + CH / 8));
    } else if (b < nb_scan + nb_prop) {
        const uint32_t c = 4 * (b - nb_scan) + (threadIdx.x >> 6);
        if (c < v.num_pc) prop_chunk_wave(v, c);
    } else {
        votes_block(v, b - nb_scan - nb_prop, reinterpret_cast<uint64_t (*)[VOTE_LDS]>(raw),
                    reinterpret_cast<uint32_t (*)[VOTE_LDS]>(raw + 4 * VOTE_LDS));
    }
}

// ------------------------------------------------------------- apply ----
// Wave-level helpers: descriptors are loaded one per lane and then broadcast
// with v_readlane, so one (node, bucket) pair costs three dependent memory
// round trips — (1) CSR offsets, (2) fragment / event descriptors, (3) the
// scan's per-message flags + the entry values — and (1) of the next pair is
// already in flight while the current one is processed.

// Snapshot records of one event of a pair: lane l's slot j is emitted when
// want[j] (record: ref[j], aux = slot | kind); one append (atomicAdd on the
// wave's sub-buffer cursor) per event.
constexpr uint32_t SPL_ = 4;
__device__ inline void emit_rows(const DevView &v, const bool (&want)[SPL_], uint32_t msg, uint32_t kind_aux,
                                 const uint32_t (&ref)[SPL_], const uint32_t *ext = nullptr)
{
    const uint32_t lane = threadIdx.x & 63;
    uint64_t m[SPL_];
    uint32_t tot = 0;
#pragma unroll
    for (uint32_t j = 0; j < SPL_; ++j) { m[j] = __ballot(want[j]); tot += (uint32_t)__popcll(m[j]); }
    if (!tot) return;
    const uint32_t sub = (blockIdx.x * 4 + (threadIdx.x >> 6)) & (v.out_subs - 1);
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(&v.out_cursor[OUT_STRIDE * sub], (unsigned long long)tot);
    base = __shfl(base, 0, 64);
    const uint64_t below = (1ull << lane) - 1;
    uint32_t off = 0;
#pragma unroll
    for (uint32_t j = 0; j < SPL_; ++j) {
        const uint64_t at = base + off + (uint64_t)__popcll(m[j] & below);
        if (want[j] && at < v.out_cap) {
            OutRec r;
            r.msg = msg; r.ref = ref[j]; r.aux = kind_aux | (lane + 64 * j) | (ext ? ext[j] : 0);
            v.out[(uint64_t)sub * v.out_cap + at] = r;
        }
        off += (uint32_t)__popcll(m[j]);
    }
}

constexpr uint32_t SPL = BS / 64;
static_assert(SPL == SPL_, "4 slots per lane");

// slots of this lane that fragment (start, count, dense) covers: k[j] = entry
// offset within the fragment or -1.  Sparse runs scatter through the wave's
// own LDS row.
__device__ inline void frag_slots(uint16_t *lidx, const uint8_t *slots, uint64_t entry, uint32_t count,
                                  uint32_t start, bool dense, int (&k)[SPL])
{
    const uint32_t lane = threadIdx.x & 63;
    if (dense) {
#pragma unroll
        for (uint32_t j = 0; j < SPL; ++j) {
            const int d = (int)(lane + 64 * j) - (int)start;
            k[j] = (d >= 0 && d < (int)count) ? d : -1;
        }
        return;
    }
    for (uint32_t q = lane; q < count; q += 64) lidx[slots[entry + q]] = (uint16_t)q;
    wave_lds_fence();
#pragma unroll
    for (uint32_t j = 0; j < SPL; ++j) {
        const uint16_t x = lidx[lane + 64 * j];
        k[j] = x == 0xFFFF ? -1 : (int)x;
    }
    wave_lds_fence();
#pragma unroll
    for (uint32_t j = 0; j < SPL; ++j) lidx[lane + 64 * j] = 0xFFFF;
    wave_lds_fence();
}

// Chosen log of one bucket, general walk: every batch whose votes reached
// quorum contributes its instances (OnAcceptReply -> Commit, multi/paxos.cpp:
// 1416-1421); the first one wins, later ones must agree (safety).
__device__ inline void chosen_walk(const DevView &v, uint64_t b, uint16_t *lidx, unsigned long long &cC,
                                   unsigned long long &dig)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t li0 = b << BSH;
    uint64_t off = lane < 2 ? v.cf_off[b + lane] : 0;
    uint64_t fi = rl64(off, 0);
    const uint64_t fe = rl64(off, 1), cbase = fi;
    uint32_t cv[SPL];                          // bucket-local chosen fragment + 1 of the first chosen Value
    uint32_t ce[SPL];                          // its entry index (agreement check: Values compared
                                               // only when two chosen runs name different entries)
#pragma unroll
    for (uint32_t j = 0; j < SPL; ++j) { cv[j] = 0; ce[j] = 0; }
    while (fi < fe) {
        const uint32_t nf = (uint32_t)(fe - fi < 64 ? fe - fi : 64);
        uint64_t fw0 = 0, fw1 = 0;
        if (lane < nf) {
            const ulonglong2 x = *reinterpret_cast<const ulonglong2 *>(v.cfrags + fi + lane);
            fw0 = x.x; fw1 = x.y;
        }
        const uint32_t live = lane < nf ? (v.b_chosen[(uint32_t)fw1] != NONE32) : 0;
        for (uint32_t a = 0; a < nf; ++a) {
            if (!rl32(live, a)) continue;
            const uint64_t ent = rl64(fw0, a), w1 = rl64(fw1, a);
            const uint32_t cnt = (uint32_t)(w1 >> 32) & 0xFFFF, st0 = (uint32_t)(w1 >> 48) & 0xFF;
            const bool dense = (w1 >> 56) & FR_DENSE;
            int k[SPL];
            frag_slots(lidx, v.e_slot, ent, cnt, st0, dense, k);
#pragma unroll
            for (uint32_t j = 0; j < SPL; ++j) {
                if (k[j] < 0) continue;
                const uint64_t iid = v.shard_begin + li0 + lane + 64 * j;
                const uint32_t x = (uint32_t)(ent + k[j]);
                if (!cv[j]) {
                    cv[j] = (uint32_t)(fi + a - cbase + 1); ce[j] = x; ++cC;
                    if (v.digest) dig += chosen_digest(iid, v.e_val[x]);
                } else if (ce[j] != x && v.e_val[ce[j]] != v.e_val[x]) record_violation(v, MPX_V_CHOSEN_VALUE, 0, 0, iid);
            }
        }
        fi += nf;
    }
    bool have = false;
#pragma unroll
    for (uint32_t j = 0; j < SPL; ++j) have |= cv[j] != 0;
    if (__ballot(have)) {
#pragma unroll
        for (uint32_t j = 0; j < SPL; ++j) {
            const uint64_t li = li0 + lane + 64 * j;
            if (li < v.shard_len) st_put(v, (uint64_t)v.N * v.shard_len + li, cv[j]);
        }
        if (lane == 0) v.chosen_valid[b] = 1;
    }
}

// A state slot back to {ballot, PRESENT | COMMITTED? | handle}
// (mpx_internal.hpp): the fixing fragment's message type and header ballot
// (member: the entry's proposal id), the Value handle of its entry at bucket
// position s (sparse runs: found in the run's slot list)
__device__ inline void decode_slot(const DevView &v, uint32_t q, uint32_t s, uint64_t &ballot, uint64_t &word)
{
    ballot = word = 0;
    if (!q) return;
    const Frag f = v.frags[q - 1];
    uint64_t ent = f.entry + (s - f.start);
    if (!(f.flags & FR_DENSE))
        for (uint32_t k = 0; k < f.count; ++k)
            if (v.e_slot[f.entry + k] == s) { ent = f.entry + k; break; }
    ballot = v.semantics == MPX_SEM_MEMBER ? v.e_pid[ent] : v.m_ballot[f.msg];
    word = W_PRESENT | ((f.flags >> 4) == K_COMMIT ? W_COMMITTED : 0) | v.e_val[ent];
}

// the stored slot of (node, shard index li) as a global fragment index + 1
__device__ inline uint32_t slot_global(const DevView &v, uint32_t node, uint64_t li)
{
    const uint32_t s = st_get(v, (uint64_t)node * v.shard_len + li);
    return s ? (uint32_t)(v.f_off[(li >> BSH) * v.N + node] + s) : 0;
}

__device__ inline uint64_t slot_digest(const DevView &v, uint32_t n, uint64_t iid, uint32_t q)
{
    if (!q) return 0;
    uint64_t b, w;
    decode_slot(v, q, (uint32_t)(iid - v.shard_begin) & (BS - 1), b, w);
    return state_digest(n, iid, (w & W_COMMITTED) ? 2 : 1, b, w & W_HANDLE);
}

// Wave id with consecutive ids on one XCD: workgroups are dealt round-robin
// over the 8 XCDs (blockIdx % 8), so id = xcd * (waves per XCD) + local id.
// Neighbouring buckets then share their XCD's L2 (headers, descriptors).
__device__ inline uint64_t xcd_wave_id_g(uint32_t wv, uint32_t grid)
{
    if (grid & 7) return (uint64_t)blockIdx.x * 4 + wv;
    const uint64_t per = (uint64_t)(grid >> 3) * 4;
    return (uint64_t)(blockIdx.x & 7) * per + (uint64_t)(blockIdx.x >> 3) * 4 + wv;
}
__device__ inline uint64_t xcd_wave_id(uint32_t wv) { return xcd_wave_id_g(wv, gridDim.x); }

// Lean acceptor/learner apply plus the chosen log, G consecutive buckets per
// wave step (fast_group: G * N + 1 <= 64, at most 4).
//
// Per slot only the fragment that fixes its final state matters: the first
// COMMIT covering it (first commit wins, multi/paxos.cpp:1515, and later
// accepts skip committed slots, :1380), else the last granted ACCEPT (:1387).
// The slot is written as that fragment's pair-local index + 1 — 2 bytes, no Value load
// (mpx_internal.hpp).
//
// Lane p < G*N owns pair (bucket b0 + p / N, node p % N); pairs are
// bucket-major in the CSR, so a step's offsets are one contiguous load.  Each
// pair lane loads its first FAST_PAIR_FRAGS descriptors and their scan flags
// itself and plans its pair in registers: when all its fragments are full
// runs (the clean case) the fixing fragment is wave-uniform per pair and the
// pair is one 16-byte store per lane — lane l holds slots 4l..4l+3, so a
// node row gets G KiB of contiguous stores per step.  The three dependent
// loads (offsets, descriptors, flags) are issued two / one / zero steps ahead,
// so a step waits once for memory (vmcnt also counts stores on gfx9, so
// every wait drains the step's stores: fewer, larger steps amortise it).
// Pairs with partial runs, a re-commit or more fragments take the per-slot
// path (descriptors loaded for that bucket, lane i = fragment i).  The
// chosen log of a bucket whose one live batch is a full run is written the
// same way (entry + 1 per slot); k_chosen walks every other bucket.  Value
// loads happen only for the re-commit check (:1508, rare) and in digest runs.
//
// State and chosen-log stores are non-temporal (written once per run, read
// back only by k_decode): tools/bw_probe2.hip measures this store pattern with
// one wait per step at 5.3 TB/s cached vs 5.7 TB/s nt on MI355X.
//
// A pair is taken here iff (same predicate as ingest.cpp's work list):
// N <= FAST_MAX_NODES, the pair has at most FAST_MAX_FRAGS fragments, all dense
// ACCEPT / COMMIT runs and its node has no PREPARE after the first of them —
// its snapshot events see empty state, so skipping them changes no output.
constexpr uint32_t FAST_PAIR_FRAGS = 2;      // descriptors a pair lane prefetches
constexpr uint64_t EV_BIT = 1ull << 63;      // k_apply_fast: pair_gp folded into the lane's CSR offset
constexpr uint64_t OFF_FLAGS = EV_BIT;
__host__ __device__ inline uint32_t fast_group(uint32_t N, uint32_t cap = 4)
{
    return N ? (63 / N < cap ? 63 / N : cap) : 1;
}

__device__ inline bool frag_lean(uint64_t w1)
{
    const uint32_t fl = (uint32_t)(w1 >> 56);
    return (fl & FR_DENSE) && ((fl >> 4) == K_ACCEPT || (fl >> 4) == K_COMMIT);
}
__device__ inline bool frag_full(uint64_t w1) { return ((w1 >> 48) & 0xFF) == 0 && ((w1 >> 32) & 0xFFFF) == BS; }

template <int WAVES_PER_EU, bool DIGEST>
__global__ __launch_bounds__(256, WAVES_PER_EU) void k_apply_fast(DevView v)
{
    constexpr uint32_t F = FAST_PAIR_FRAGS;
    __shared__ unsigned long long red[4][5];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned long long cA = 0, cL = 0, dig = 0, cC = 0, cdig = 0;
    const uint32_t N = v.N;
    const uint64_t NB = v.NB;
    if (N > FAST_MAX_NODES) return;
    const uint32_t G = fast_group(N);
    const uint64_t steps = (NB + G - 1) / G;
    const uint64_t nwaves = (uint64_t)gridDim.x * 4;
    const uint64_t *__restrict__ e_val = v.e_val;
    const uint32_t s0 = 4 * lane;                        // the lane's slots s0..s0+3

    // stage 1 (two steps ahead): pair CSR offsets (lanes 0..nb*N), chosen-log
    // CSR offsets (lanes 0..nb)
    auto ld_off = [&](uint64_t st, uint64_t &oa, uint64_t &oc) {
        oa = oc = 0;
        if (st >= steps) return;
        const uint64_t b0 = st * G, nb = NB - b0 < G ? NB - b0 : G;
        if (lane <= nb * N) oa = v.f_off[b0 * N + lane] | (lane < nb * N && v.pair_gp[b0 * N + lane] ? EV_BIT : 0);
        if (lane <= nb) oc = v.cf_off[b0 + lane];
    };
    // stage 2 (one step ahead): each pair's first F descriptors, each
    // bucket's chosen-log descriptor when it is the only one
    auto ld_desc = [&](uint64_t st, uint64_t oa, uint64_t oc, uint64_t (&e)[F], uint64_t (&w)[F], uint64_t &ce,
                       uint64_t &cw) {
        const uint64_t o1 = __shfl(oa, (int)((lane + 1) & 63), 64) & ~OFF_FLAGS;
        const uint64_t c1 = __shfl(oc, (int)((lane + 1) & 63), 64);
        oa &= ~OFF_FLAGS;
#pragma unroll
        for (uint32_t k = 0; k < F; ++k) { e[k] = 0; w[k] = NONE32; }
        ce = 0; cw = NONE32;
        if (st >= steps) return;
        const uint64_t b0 = st * G, nb = NB - b0 < G ? NB - b0 : G;
        if (lane < nb * N) {
            const uint64_t len = o1 - oa;
#pragma unroll
            for (uint32_t k = 0; k < F; ++k)
                if (k < len) {
                    const ulonglong2 x = *reinterpret_cast<const ulonglong2 *>(v.frags + oa + k);
                    e[k] = x.x; w[k] = x.y;
                }
        }
        if (lane < nb && c1 - oc == 1) {
            const ulonglong2 x = *reinterpret_cast<const ulonglong2 *>(v.cfrags + oc);
            ce = x.x; cw = x.y;
        }
    };

    uint64_t st_c = xcd_wave_id(wv);
    uint64_t oa_c, oc_c, oa_n, oc_n;
    ld_off(st_c, oa_c, oc_c);
    ld_off(st_c + nwaves, oa_n, oc_n);
    uint64_t ne[F], nw[F], nce, ncw;
    ld_desc(st_c, oa_c, oc_c, ne, nw, nce, ncw);
    for (; st_c < steps; st_c += nwaves) {
        const uint64_t st = st_c;
        const uint64_t b0 = st * G, nb = NB - b0 < G ? NB - b0 : G;
        const bool pev = (oa_c & EV_BIT) != 0;                 // the pair has snapshot events
        const uint64_t oa = oa_c & ~OFF_FLAGS;
        const uint64_t pev_m = __ballot(pev);
        uint64_t e[F], w[F];
#pragma unroll
        for (uint32_t k = 0; k < F; ++k) { e[k] = ne[k]; w[k] = nw[k]; }
        const uint64_t ce = nce, cw = ncw;
        // the next step's descriptors, the one after's offsets
        ld_desc(st + nwaves, oa_n, oc_n, ne, nw, nce, ncw);
        oa_c = oa_n; oc_c = oc_n;
        ld_off(st + 2 * nwaves, oa_n, oc_n);
        // stage 3: scan flags of this step's fragment messages, quorum of the
        // chosen-log batch
        uint32_t fg[F];
#pragma unroll
        for (uint32_t k = 0; k < F; ++k) fg[k] = (uint32_t)w[k] != NONE32 ? v.m_flags[(uint32_t)w[k]] : 0;
        const uint32_t clive = (uint32_t)cw != NONE32 ? v.b_chosen[(uint32_t)cw] != NONE32 : 0;
        // One wait per step, before its stores (vmcnt(0); expcnt / lgkmcnt free).
        __builtin_amdgcn_s_waitcnt(0x0F70);

        // plan, one pair per lane
        const uint64_t o1 = __shfl(oa, (int)((lane + 1) & 63), 64);
        const bool pair = lane < nb * N;
        const uint32_t len = pair ? (uint32_t)(o1 - oa) : 0;
        const bool in_list = len && len <= FAST_MAX_FRAGS;                  // else: the general work list
        bool elig = in_list && len <= F, full = true, again = false, comm = false;
        uint32_t fix = NONE32, nA = 0, nL = 0;
#pragma unroll
        for (uint32_t k = 0; k < F; ++k) {
            if (k >= len) continue;
            elig = elig && frag_lean(w[k]);
            full = full && frag_full(w[k]);
            if ((w[k] >> 60) == K_COMMIT) { ++nL; if (comm) again = true; else { comm = true; fix = k; } }
            else if (!comm && (fg[k] & F_GRANTED)) { ++nA; fix = k; }
        }
        elig = elig && !pev;
        const bool uni = elig && full && !again;
        const uint64_t uni_m = __ballot(uni);
        const uint64_t slow_m = __ballot((elig && !uni) || (in_list && len > F));
        if (uni) { cA += nA * BS; cL += nL * BS; }
        const uint32_t qv = fix == NONE32 ? 0 : (uint32_t)(oa + fix + 1);   // global fragment + 1
        const uint32_t ql = fix == NONE32 ? 0 : fix + 1;                     // as stored: pair-local
        if (elig) v.st_valid[b0 * N + lane] = 1;

        // uniform pairs, node-major so each row gets its G buckets back to back
        const bool whole = (b0 + nb) * BS <= v.shard_len;
        for (uint32_t n = 0; n < N; ++n) {
            const uint64_t row = (uint64_t)n * v.shard_len + b0 * BS;
            for (uint32_t g = 0; g < nb; ++g) {
                const uint32_t p = g * N + n;
                if (!((uni_m >> p) & 1)) continue;
                const uint32_t q = rl32(qv, p);
                const uint32_t sq = rl32(ql, p);
                if (whole) {
                    st_put4(v, row + g * BS + s0, sq, sq, sq, sq);
                } else {
#pragma unroll
                    for (uint32_t j = 0; j < SPL; ++j)
                        if ((b0 + g) * BS + s0 + j < v.shard_len) st_put(v, row + g * BS + s0 + j, sq);
                }
                if (DIGEST)
#pragma unroll
                    for (uint32_t j = 0; j < SPL; ++j) dig += slot_digest(v, n, v.shard_begin + (b0 + g) * BS + s0 + j, q);
            }
        }

        // per-slot path (rare): the pair's fragments, lane i = fragment i
        for (uint64_t m = slow_m; m; m &= m - 1) {
            const uint32_t p = (uint32_t)__builtin_ctzll(m);
            const uint32_t g = p / N, n = p - g * N;
            const uint64_t b = b0 + g, li0 = b << BSH, ib = v.shard_begin + li0;
            const uint64_t f_base = rl64(oa, p);
            const uint32_t total = (uint32_t)(rl64(oa, p + 1) - f_base);   // <= FAST_MAX_FRAGS
            const uint32_t f0 = 0, f1 = total;
            uint64_t fw0 = 0, fw1 = NONE32;
            uint32_t fflag = 0;
            if (lane < total) {
                const ulonglong2 x = *reinterpret_cast<const ulonglong2 *>(v.frags + f_base + lane);
                fw0 = x.x; fw1 = x.y;
                fflag = v.m_flags[(uint32_t)fw1];
            }
            // eligibility of a pair with more fragments than a lane prefetches
            const uint64_t badm = __ballot(lane < total && !frag_lean(fw1));
            if (badm || ((pev_m >> p) & 1)) continue;
            if (lane == 0) v.st_valid[sv_idx(v, n, b)] = 1;
            uint32_t q0 = 0, q1 = 0, q2 = 0, q3 = 0;   // the lane's four slots
            uint32_t bad = 0;
            // per slot: the fixing fragment (8 bits per slot: its lane, 0xFF
            // none), the committed bit and the counters
            uint32_t src = 0xFFFFFFFFu;
            uint32_t com = 0;
            uint32_t recommit = 0;                     // a later COMMIT covers a committed slot
            for (uint32_t a = f0; a < f1; ++a) {
                const uint64_t w1 = rl64(fw1, a);
                const uint32_t cnt = (uint32_t)(w1 >> 32) & 0xFFFF, st0 = (uint32_t)(w1 >> 48) & 0xFF;
                const bool commit = (w1 >> 60) == K_COMMIT;
                if (!commit && !(rl32(fflag, a) & F_GRANTED)) continue;
#pragma unroll
                for (uint32_t j = 0; j < SPL; ++j) {
                    const uint32_t s = s0 + j;
                    if (s < st0 || s >= st0 + cnt) continue;
                    if (commit) {
                        ++cL;
                        if ((com >> j) & 1) recommit = 1;
                        else { com |= 1u << j; src = (src & ~(0xFFu << (8 * j))) | (a << (8 * j)); }
                    } else if (!((com >> j) & 1)) {
                        ++cA;
                        src = (src & ~(0xFFu << (8 * j))) | (a << (8 * j));
                    }
                }
            }
#define MPX_SLOT(J, Q)                                                                        \
            {                                                                                 \
                const uint32_t fa = (src >> (8 * J)) & 0xFF;                                  \
                if (fa != 0xFF) Q = (uint32_t)(f_base + fa + 1);                              \
            }
            MPX_SLOT(0, q0) MPX_SLOT(1, q1) MPX_SLOT(2, q2) MPX_SLOT(3, q3)
#undef MPX_SLOT
            // re-commit check: every later COMMIT must carry the committed Value (:1508)
            if (__ballot(recommit)) {
                uint64_t cval[SPL];                    // the committed Value of slot j
#pragma unroll
                for (uint32_t j = 0; j < SPL; ++j) {
                    const uint32_t fa = (src >> (8 * j)) & 0xFF;
                    const uint64_t ent = __shfl(fw0, (int)(fa & 63), 64);
                    const uint64_t w1 = __shfl(fw1, (int)(fa & 63), 64);
                    cval[j] = fa != 0xFF ? e_val[ent + (s0 + j - ((uint32_t)(w1 >> 48) & 0xFF))] : 0;
                }
                for (uint32_t a = f0; a < f1; ++a) {
                    const uint64_t w1 = rl64(fw1, a);
                    if ((w1 >> 60) != K_COMMIT) continue;
                    const uint32_t cnt = (uint32_t)(w1 >> 32) & 0xFFFF, st0 = (uint32_t)(w1 >> 48) & 0xFF;
                    const uint64_t ent = rl64(fw0, a);
#pragma unroll
                    for (uint32_t j = 0; j < SPL; ++j) {
                        const uint32_t s = s0 + j;
                        if (s < st0 || s >= st0 + cnt || ((src >> (8 * j)) & 0xFF) == a) continue;
                        if (e_val[ent + (s - st0)] != cval[j]) bad = 1;
                    }
                }
            }
            if (__ballot(bad) && lane == 0) record_violation(v, MPX_V_COMMIT_VALUE, n, 0, ib);
            const uint64_t srow = (uint64_t)n * v.shard_len + li0;
            const uint64_t pbase = f_base;             // the pair's first fragment
            const uint32_t l0 = q0 ? (uint32_t)(q0 - pbase) : 0, l1 = q1 ? (uint32_t)(q1 - pbase) : 0,
                           l2 = q2 ? (uint32_t)(q2 - pbase) : 0, l3 = q3 ? (uint32_t)(q3 - pbase) : 0;
            if (li0 + BS <= v.shard_len) {
                st_put4(v, srow + s0, l0, l1, l2, l3);
            } else {
                if (li0 + s0 < v.shard_len) st_put(v, srow + s0, l0);
                if (li0 + s0 + 1 < v.shard_len) st_put(v, srow + s0 + 1, l1);
                if (li0 + s0 + 2 < v.shard_len) st_put(v, srow + s0 + 2, l2);
                if (li0 + s0 + 3 < v.shard_len) st_put(v, srow + s0 + 3, l3);
            }
            if (DIGEST)
                dig += slot_digest(v, n, ib + s0, q0) + slot_digest(v, n, ib + s0 + 1, q1) +
                       slot_digest(v, n, ib + s0 + 2, q2) + slot_digest(v, n, ib + s0 + 3, q3);
        }

        // chosen log of the buckets whose one live batch is a full run
        const bool cok = clive && frag_full(cw) && (b0 + lane + 1) * BS <= v.shard_len;
        const uint64_t cok_m = __ballot(cok);
        if (cok) v.chosen_valid[b0 + lane] = 1;
        for (uint64_t m = cok_m; m; m &= m - 1) {
            const uint32_t g = (uint32_t)__builtin_ctzll(m);
            const uint64_t li0 = (b0 + g) << BSH;
            // the bucket's only chosen fragment: local index 0, stored + 1
            st_put4(v, (uint64_t)N * v.shard_len + li0 + s0, 1, 1, 1, 1);
            cC += SPL;
            if (DIGEST) {
                const uint64_t c0 = rl64(ce, g), ib = v.shard_begin + li0;
#pragma unroll
                for (uint32_t j = 0; j < SPL; ++j) cdig += chosen_digest(ib + s0 + j, e_val[c0 + s0 + j]);
            }
        }
    }
    unsigned long long cc[5] = {cA, cL, dig, cC, cdig};
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        unsigned long long x = cc[i];
        for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
        cc[i] = x;
    }
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < 5; ++i) red[wv][i] = cc[i];
    }
    __syncthreads();
    if (threadIdx.x < 5) {
        const uint32_t t = threadIdx.x;
        unsigned long long s = red[0][t] + red[1][t] + red[2][t] + red[3][t];
        const int slot = t == 0 ? PC_A : t == 1 ? PC_L : t == 2 ? PC_DSTATE : t == 3 ? PC_C : PC_DCHOSEN;
        v.partials[8 * blockIdx.x + slot] += s;
    }
}

__device__ inline uint64_t frag_w1(const Frag *f) { return reinterpret_cast<const uint64_t *>(f)[1]; }

// Plan words (k_plan -> k_store / k_store8; 64 bits per (row, bucket)): the
// row's 256 slots as at most four segments of equal value —
//   bits  0..31  v0..v3, the slot value of segment k (8 bits each)
//   bits 32..58  s1, s2, s3 (9 bits each): segment k = slots [s_k, s_k+1) with
//                s_0 = 0, s_4 = 256; unused splits are 256 and unused segments
//                repeat the last value, so a one-segment word has v0 = .. = v3
//                and its low half is already four slots' bytes
// PLAN_SKIP: not k_store's row (k_apply_fast / k_chosen write it).
constexpr uint64_t PLAN_SKIP = ~0ull;
constexpr uint32_t PLAN_LDS = 512;                          // descriptor words a k_plan wave stages (4 KiB)
constexpr uint32_t PLAN_UNI = BS | BS << 9 | BS << 18;      // bits 32..58 of a one-segment word

__device__ inline uint32_t plan_split(uint64_t q, uint32_t k) { return (uint32_t)(q >> (32 + 9 * k)) & 511; }
__device__ inline uint32_t plan_slot(uint64_t q, uint32_t s)
{
    const uint32_t k = (s >= plan_split(q, 0)) + (s >= plan_split(q, 1)) + (s >= plan_split(q, 2));
    return (uint32_t)(q >> (8 * k)) & 0xFF;
}
// one-byte slots p..p+15: every byte picks its segment's value out of the low
// word with v_perm (selector byte = segment index 0..3 = splits at or below it)
__device__ inline u32x4 plan_bytes16(uint64_t q, uint32_t p)
{
    constexpr uint64_t ONES = 0x0101010101010101ull;
    const uint32_t V = (uint32_t)q;
    uint64_t lo = 0, hi = 0;
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) {
        const int t = (int)plan_split(q, k) - (int)p;        // window bytes >= t are at or past split k
        lo += t <= 0 ? ONES : t >= 8 ? 0 : ONES << (8 * t);
        hi += t <= 8 ? ONES : t >= 16 ? 0 : ONES << (8 * (t - 8));
    }
    return u32x4{__builtin_amdgcn_perm(V, V, (uint32_t)lo), __builtin_amdgcn_perm(V, V, (uint32_t)(lo >> 32)),
                 __builtin_amdgcn_perm(V, V, (uint32_t)hi), __builtin_amdgcn_perm(V, V, (uint32_t)(hi >> 32))};
}
__device__ inline uint64_t plan_pack(const uint32_t (&val)[4], const uint32_t (&s)[3])
{
    return (uint64_t)(val[0] | val[1] << 8 | val[2] << 16 | val[3] << 24) |
           ((uint64_t)s[0] << 32) | ((uint64_t)s[1] << 41) | ((uint64_t)s[2] << 50);
}

// The chosen-log plan word of bucket i (row N; k_plan, k_plan_member): every live
// batch run of the bucket (its votes reached quorum, k_votes) contributes its
// instances (OnAcceptReply -> Commit, multi/paxos.cpp:1416-1421); when at most
// four segments describe the bucket and no instance lies under two live runs
// (k_chosen compares their Values) the word is written and chosen_valid set,
// else PLAN_SKIP leaves the bucket to k_chosen.
// CLAMPED: the vote loads take clamped indices and no branch, so they are all in flight at once
// (under a lane condition each was issued and waited for in turn); k_plan_store8 keeps the
// conditional loads — one live run per bucket there, and 8 more VGPRs cost it occupancy
template <bool CLAMPED = true>
__device__ inline uint64_t plan_chosen_at(const DevView &v, uint64_t i, uint64_t oc, uint64_t c1, unsigned long long &cC)
{
    constexpr uint32_t F = PLAN_FRAGS;
    const uint32_t len = (uint32_t)(c1 - oc);
    uint64_t q = PLAN_SKIP;
    if (len && len <= F && (i + 1) * BS <= v.shard_len) {
        uint64_t w[F];
        uint32_t live[F];
#pragma unroll
        for (uint32_t k = 0; k < F; ++k) w[k] = k < len ? frag_w1(v.cfrags + oc + k) : 0;
        if (CLAMPED) {
#pragma unroll
            for (uint32_t k = 0; k < F; ++k) live[k] = v.b_chosen[k < len ? (uint32_t)w[k] : 0];
#pragma unroll
            for (uint32_t k = 0; k < F; ++k) live[k] = k < len && live[k] != NONE32;
        } else {
#pragma unroll
            for (uint32_t k = 0; k < F; ++k) live[k] = k < len ? v.b_chosen[(uint32_t)w[k]] != NONE32 : 0;
        }
        bool ok = true;
        uint32_t sp[3] = {BS, BS, BS};
#pragma unroll
        for (uint32_t k = 0; k < F; ++k) {
            if (k >= len) continue;
            const uint32_t cnt = (uint32_t)(w[k] >> 32) & 0xFFFF, st0 = (uint32_t)(w[k] >> 48) & 0xFF;
            ok = ok && ((w[k] >> 56) & FR_DENSE) && plan_add_split(st0, sp) && plan_add_split(st0 + cnt, sp);
        }
        uint32_t val[4];
        unsigned long long c = 0;
#pragma unroll
        for (uint32_t g = 0; g < 4; ++g) {
            const uint32_t lo = g ? sp[g - 1] : 0, hi = g < 3 ? sp[g] : BS;
            if (lo >= BS) { val[g] = val[g - 1]; continue; }
            uint32_t fix = NONE32;
#pragma unroll
            for (uint32_t k = 0; k < F; ++k) {
                if (k >= len || !live[k]) continue;
                const uint32_t cnt = (uint32_t)(w[k] >> 32) & 0xFFFF, st0 = (uint32_t)(w[k] >> 48) & 0xFF;
                if (lo < st0 || lo >= st0 + cnt) continue;
                if (fix != NONE32) ok = false;                    // two chosen runs: k_chosen compares Values
                else fix = k;
            }
            val[g] = fix == NONE32 ? 0 : fix + 1;
            if (fix != NONE32) c += hi - lo;
        }
        if (ok) {
            q = plan_pack(val, sp);
            v.chosen_valid[i] = 1;
            cC = c;
        }
    }
    return q;
}
template <bool CLAMPED = true>
__device__ inline uint64_t plan_chosen_word(const DevView &v, uint64_t i, unsigned long long &cC)
{
    return plan_chosen_at<CLAMPED>(v, i, v.cf_off[i], v.cf_off[i + 1], cC);
}
__device__ inline void plan_chosen(const DevView &v, uint64_t i, unsigned long long &cC)
{
    v.plan[(uint64_t)v.N * v.NB + i] = plan_chosen_word(v, i, cC);
}

// k_plan's reduction of lean multi pair i (bucket b, len runs): its plan word, or PLAN_SKIP
// (rest = 1 when the pair is in the list but no plan word describes it).  ldw(k) loads the
// pair's k-th run descriptor word.  CLAMPED: the scan-flag loads all in flight (plan_chosen_at).
template <bool CLAMPED, typename LoadW>
__device__ inline uint64_t plan_lean(const DevView &v, uint64_t i, uint64_t b, uint32_t len, bool in_list, LoadW ldw,
                                     unsigned long long &cA, unsigned long long &cL, uint32_t &rest)
{
    constexpr uint32_t F = PLAN_FRAGS;
    uint64_t q = PLAN_SKIP;
    if (in_list && len <= F) {
        uint64_t w[F];
        uint32_t fg[F];
#pragma unroll
        for (uint32_t k = 0; k < F; ++k) w[k] = k >= len ? 0 : ldw(k);
        if (CLAMPED) {                     // a COMMIT run's scan flag is never read
#pragma unroll
            for (uint32_t k = 0; k < F; ++k) fg[k] = v.m_flags[k < len && (w[k] >> 60) != K_COMMIT ? (uint32_t)w[k] : 0];
#pragma unroll
            for (uint32_t k = 0; k < F; ++k) fg[k] = k < len && (w[k] >> 60) != K_COMMIT ? fg[k] : 0;
        } else {
#pragma unroll
            for (uint32_t k = 0; k < F; ++k)
                fg[k] = k < len && (w[k] >> 60) != K_COMMIT ? v.m_flags[(uint32_t)w[k]] : 0;
        }
        bool ok = (b + 1) * BS <= v.shard_len;
        uint32_t sp[3] = {BS, BS, BS};
#pragma unroll
        for (uint32_t k = 0; k < F; ++k) {
            if (k >= len) continue;
            const uint32_t cnt = (uint32_t)(w[k] >> 32) & 0xFFFF, st0 = (uint32_t)(w[k] >> 48) & 0xFF;
            ok = ok && frag_lean(w[k]) && plan_add_split(st0, sp) && plan_add_split(st0 + cnt, sp);
        }
        uint32_t val[4];
        unsigned long long a = 0, l = 0;
#pragma unroll
        for (uint32_t g = 0; g < 4; ++g) {
            const uint32_t lo = g ? sp[g - 1] : 0, hi = g < 3 ? sp[g] : BS;
            if (lo >= BS) { val[g] = val[g - 1]; continue; }
            bool comm = false;
            uint32_t fix = NONE32, nA = 0, nL = 0;
#pragma unroll
            for (uint32_t k = 0; k < F; ++k) {
                if (k >= len) continue;
                const uint32_t cnt = (uint32_t)(w[k] >> 32) & 0xFFFF, st0 = (uint32_t)(w[k] >> 48) & 0xFF;
                if (lo < st0 || lo >= st0 + cnt) continue;          // segments lie inside or outside a run
                if ((w[k] >> 60) == K_COMMIT) { ++nL; if (comm) ok = false; else { comm = true; fix = k; } }
                else if (!comm && (fg[k] & F_GRANTED)) { ++nA; fix = k; }
            }
            val[g] = fix == NONE32 ? 0 : fix + 1;               // the slot as stored: pair-local fragment + 1
            a += (unsigned long long)nA * (hi - lo);
            l += (unsigned long long)nL * (hi - lo);
        }
        if (ok) {
            q = plan_pack(val, sp);
            v.st_valid[i] = 1;
            cA += a; cL += l;
        }
    }
    if (q == PLAN_SKIP && in_list) ++rest;
    return q;
}

// Apply split in two (the default for multi runs): k_plan decides every pair
// with one thread per pair — no per-step chain, so its gathers (CSR offsets,
// up to PLAN_FRAGS descriptors and scan flags) all overlap — and k_store
// streams the result.  A (node, bucket) pair whose runs are all dense ACCEPT /
// COMMIT runs cuts its bucket into segments at the runs' boundaries; in each
// segment one run fixes every slot (the first COMMIT over it, else the last
// granted ACCEPT, as in the per-slot path), so up to four segments are one
// plan word of pair-local fragment + 1 values.  Batch 256 gives one segment,
// batch 100 / 255 two to four (a bucket meets two to four batches).  The
// chosen log of a bucket whose live batch runs do not overlap is row N the
// same way (bucket-local chosen run + 1).  Pairs with more runs or segments, a
// re-commit (its Value check) or a partial last bucket are counted in
// fast_rest and left to k_apply_fast<.., AFTER_STORE>.
__global__ __launch_bounds__(256) void k_plan(DevView v, uint32_t apply_wgs)
{
    __shared__ unsigned long long red[4][3];
    __shared__ uint32_t rest_w[4];
    __shared__ uint64_t w_lds[4][PLAN_LDS];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t N = v.N;
    const uint64_t NB = v.NB, np = (uint64_t)N * NB;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    unsigned long long cA = 0, cL = 0, cC = 0;
    uint32_t rest = 0;
    // the wave's 64 pairs own one contiguous descriptor range: stream its
    // second words into LDS with coalesced loads (lane r: words r, r + 64, ..),
    // then every pair lane reads its runs from there
    const uint64_t oa = v.f_off[i < np ? i : np], o1 = v.f_off[i < np ? i + 1 : np];
    const uint8_t gp = i < np ? v.pair_gp[i] : 1;   // issued with the offsets, not after the staging
    const uint64_t wbase = rl64(oa, 0);
    {
        // the staging loads of a wave's runs all in flight, then the LDS writes
        // (C4: two runs per pair, 128 words per wave; longer ranges loop)
        const uint64_t wend = rl64(o1, 63);
        const uint32_t R = (uint32_t)(wend - wbase < PLAN_LDS ? wend - wbase : PLAN_LDS);
        constexpr uint32_t K = 4;
        for (uint32_t r0 = 0; r0 < R; r0 += 64 * K) {
            uint64_t x[K];
#pragma unroll
            for (uint32_t k = 0; k < K; ++k) {
                const uint32_t r = r0 + lane + 64 * k;
                x[k] = r < R ? v.frag_w1[wbase + r] : 0;
            }
#pragma unroll
            for (uint32_t k = 0; k < K; ++k) {
                const uint32_t r = r0 + lane + 64 * k;
                if (r < R) w_lds[wv][r] = x[k];
            }
        }
        wave_lds_fence();
    }
    if (i < np) {
        const uint64_t b = i / N;

        const uint32_t len = (uint32_t)(o1 - oa);
        const bool in_list = len && len <= FAST_MAX_FRAGS && !gp;
        const uint64_t rel = oa - wbase;                     // past the staged words: global loads (rare)
        v.plan[i] = plan_lean<true>(v, i, b, len, in_list,
                              [&](uint32_t k) { return rel + k < PLAN_LDS ? w_lds[wv][rel + k] : v.frag_w1[oa + k]; },
                              cA, cL, rest);
    }
    if (i < NB) plan_chosen(v, i, cC);
    unsigned long long cc[3] = {cA, cL, cC};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        unsigned long long x = cc[k];
        for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
        cc[k] = x;
    }
    const uint64_t rm = __ballot(rest);
    if (lane == 0) {
        red[wv][0] = cc[0]; red[wv][1] = cc[1]; red[wv][2] = cc[2];
        rest_w[wv] = (uint32_t)__builtin_popcountll(rm);
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        const uint32_t t = threadIdx.x;
        const unsigned long long x = red[0][t] + red[1][t] + red[2][t] + red[3][t];
        const int slot = t == 0 ? PC_A : t == 1 ? PC_L : PC_C;
        if (x) atomicAdd(&v.partials[8 * (blockIdx.x % apply_wgs) + slot], x);
    } else if (threadIdx.x == 3) {
        const uint32_t r = rest_w[0] + rest_w[1] + rest_w[2] + rest_w[3];
        if (r) atomicAdd(v.fast_rest, r);
    }
}

// One snapshot run record (OUT_RUN): slots [lo, lo + len) of a planned pair's bucket, all
// fixed by fragment `ref`, go into the PREPARE_REPLY of message `msg`; the host expands it
// slot by slot (engine.cpp fetch_results), so a segment costs one 12-byte record instead
// of one per slot.
__device__ inline void emit_run(const DevView &v, uint32_t msg, uint32_t ref, uint32_t lo, uint32_t len)
{
    const uint32_t sub = (blockIdx.x * 4 + (threadIdx.x >> 6)) & (v.out_subs - 1);
    const unsigned long long at = atomicAdd(&v.out_cursor[OUT_STRIDE * sub], 1ull);
    if (at < v.out_cap) {
        OutRec r;
        r.msg = msg; r.ref = ref; r.aux = OUT_RUN | lo | (len << OUT_RUN_SHIFT);
        v.out[(uint64_t)sub * v.out_cap + at] = r;
    }
}

// List plan path (the timed step for the general work list's pairs without promise
// rounds): k_plan's reduction extended to pairs with snapshot events, one thread per
// (node, bucket) pair whose pair_gp is GP_LIST.  Runs cut the bucket into at most LSEG (4)
// segments (seg_add_split); within a segment every run covers all or none of it, so the
// pair walks its runs and its events in message order with one state per segment instead
// of 256 slot states, and one plan word (k_store / k_store8 stream it) holds the result.
//   multi (multi/paxos.cpp:1359-1404 OnAccept, :1494-1518 OnCommit): a granted ACCEPT
//     overwrites every segment it covers that is not committed, the first COMMIT fixes it;
//   MEMBER (member/paxos.cpp:1744-1793 Acceptor::OnAccept / OnLearn, :1029-1060
//     Learner::OnLearn, :1952-1957 Acceptor deletion): accept and learn are
//     std::map::insert — the FIRST learn covering an instance fixes it, else the first
//     granted accept after the last marker that deleted or recreated the node's Acceptor
//     (F_ACCCLR: its accepted map goes, learned entries stay with the Learner).
// A granted PREPARE while a segment holds an entry is FilterAcceptedValues (multi :902-922,
// member :1700-1727): per segment meeting the prepare's ranges, one run record (emit_run).
// The counters follow the per-slot walk exactly (A = applications, L = every learn /
// commit-covered slot, P = snapshot entries).
//
// The pair is listed for k_apply instead (gp_dyn, one append per wave) when: more than
// F (16) runs, a run that is not a dense accept / commit run, a fifth segment or a
// partial last bucket.  A commit / learn (member: also an accept) over a committed segment
// through another message's entries changes nothing there, but the reference compares the
// Values (multi :1508, member :1765,1040): the pair stays planned and goes to the check list
// (gp_chk, one append per wave), whose slots k_commit_check compares.  Nothing is emitted
// for a listed pair: the walk runs once to decide, and a second time to emit only when it
// emits and the pair is kept.  Promise-round pairs (GP_ROUNDS)
// are never taken: the host range of the full k_apply has them.  MEMBER also plans the
// chosen log (bucket i < NB, plan_chosen); multi's k_plan did.  The staged descriptor
// words carry the accept runs' scan flag (F_GRANTED) in bit 57 after the gather, so the
// walk reads only LDS.
constexpr uint64_t MP_GRANTED = 1ull << 57;
// descriptor-window staging loads in flight per lane, and scan-flag gathers in flight (A/B knobs)
#ifndef MPX_PL_STAGE_K
#define MPX_PL_STAGE_K 4
#endif
#ifndef MPX_PL_FLAG_C
#define MPX_PL_FLAG_C 16
#endif
// the distinct run boundaries of a pair, sorted into s[0 .. LSEG-2] (BS = unused); false once
// an LSEG + 1-th segment appears
template <uint32_t LSEG>
__device__ inline bool seg_add_split(uint32_t x, uint32_t (&s)[LSEG - 1])
{
    if (x == 0 || x >= BS) return true;
    bool have = false;
#pragma unroll
    for (uint32_t k = 0; k < LSEG - 1; ++k) have = have || s[k] == x;
    if (have) return true;
    if (s[LSEG - 2] != BS) return false;                      // an LSEG + 1-th segment
    uint32_t y = x;                                            // insertion: s stays sorted, BS last
#pragma unroll
    for (uint32_t k = 0; k < LSEG - 1; ++k)
        if (y < s[k]) { const uint32_t t = s[k]; s[k] = y; y = t; }
    return true;
}
// LSEG: segments a pair may have — up to 4 fit one plan word (k_store); a pair with 5..8
// (multi: LSEG = PLAN_XSEG, up to F = PLAN_XFRAGS runs) goes to the extension list as its split
// points and segment values, which k_store_ext writes one wave per pair (round 3 measured the
// same walk writing those slots per thread: C3 general apply 1.01 -> 0.80 ms but k_plan_list
// 0.19 -> 0.40 ms).
// RETRY (member): the pairs the (LSEG = 8) plan listed only for having more segments, planned again
// with up to 16 (the retry list gp_rt, one lane per pair, each lane's runs staged in its own LDS
// row); what still does not fit goes to the listed-pair walk as before.  Contended C5: the walk's
// pairs with more than 8 segments (one kernel at 16 segments needs 215
// VGPRs and runs at 2 waves per SIMD over every pair: slower, profiles/r06_ab_member_plan16_2waves.txt).
template <bool MEMBER, uint32_t LSEG = 4, uint32_t F = MPLAN_FRAGS, int WAVES = 4, bool RETRY = false>
__global__ __launch_bounds__(256, WAVES) void k_plan_list(DevView v, uint32_t apply_wgs)
{
    constexpr uint32_t LDSW = RETRY ? 64 * F : MPLAN_LDS;
    __shared__ uint64_t w_lds[4][LDSW];
    __shared__ unsigned long long red[4][4];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t N = v.N;
    const uint64_t NB = v.NB, np = (uint64_t)N * NB;
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (RETRY) {
        const uint64_t nrt = *v.gp_rt_n;
        if ((uint64_t)blockIdx.x * 256 >= nrt) return;      // (the grid covers every list pair: most blocks idle)
        i = i < nrt ? v.gp_rt[i] : np;
    }
    unsigned long long cA = 0, cL = 0, cC = 0, cP = 0;
    const uint64_t ic = i < np ? i : np, in = i < np ? i + 1 : np;
    const uint64_t oa = v.f_off[ic], o1 = v.f_off[in];
    const uint64_t e0 = v.ev_off[ic], e1 = v.ev_off[in];
    const uint8_t gp = i < np ? v.pair_gp[i] : 0;
    // the wave's runs are one contiguous descriptor range, staged MPLAN_LDS words at a time: a
    // pair whose runs end past the staged window waits for the next window, which starts at
    // the first such pair (pairs are in lane order, their runs ascend), until every pair of
    // the wave is decided (each window decides at least its first pair: len <= F)
    const uint64_t wend = rl64(o1, 63);
    const uint32_t len = (uint32_t)(o1 - oa);
    uint64_t sbase = RETRY ? oa - (uint64_t)lane * F : rl64(oa, 0);
    bool todo = i < np;
    bool fb = false;                                   // list the pair for k_apply
    bool rt = false;                                   // ... or for the retry at 16 segments (RETRY: never)
    bool ck = false;                                   // ... planned, its re-commits' Values to check
    bool xt = false;                                   // ... or for k_store_ext (k_store_ext's item formats)
    uint64_t xw0 = 0, xw1 = 0, xw2 = 0, xw3 = 0;
    uint32_t xns = EXT_LEGACY;
    for (;;) {
    if (RETRY) {
        // each lane's own runs into its own LDS row (rel = lane * F), loads all in flight
        const uint32_t L = todo && len <= F ? len : 0;
        constexpr uint32_t K8 = 8;                             // (8 in flight at a time: no private array)
        for (uint32_t k0 = 0; k0 < L; k0 += K8) {
            uint64_t x0 = k0 + 0 < L ? v.frag_w1[oa + k0 + 0] : 0, x1 = k0 + 1 < L ? v.frag_w1[oa + k0 + 1] : 0;
            uint64_t x2 = k0 + 2 < L ? v.frag_w1[oa + k0 + 2] : 0, x3 = k0 + 3 < L ? v.frag_w1[oa + k0 + 3] : 0;
            uint64_t x4 = k0 + 4 < L ? v.frag_w1[oa + k0 + 4] : 0, x5 = k0 + 5 < L ? v.frag_w1[oa + k0 + 5] : 0;
            uint64_t x6 = k0 + 6 < L ? v.frag_w1[oa + k0 + 6] : 0, x7 = k0 + 7 < L ? v.frag_w1[oa + k0 + 7] : 0;
            uint64_t *d = &w_lds[wv][lane * F + k0];
            d[0] = x0; if (k0 + 1 < L) d[1] = x1; if (k0 + 2 < L) d[2] = x2; if (k0 + 3 < L) d[3] = x3;
            if (k0 + 4 < L) d[4] = x4; if (k0 + 5 < L) d[5] = x5; if (k0 + 6 < L) d[6] = x6; if (k0 + 7 < L) d[7] = x7;
        }
        wave_lds_fence();
    } else {
        // the window's second words into LDS with coalesced loads, all in flight before the
        // LDS writes
        const uint32_t R = (uint32_t)(wend - sbase < MPLAN_LDS ? wend - sbase : MPLAN_LDS);
        constexpr uint32_t K = MPX_PL_STAGE_K;
        for (uint32_t r0 = 0; r0 < R; r0 += 64 * K) {
            uint64_t x[K];
#pragma unroll
            for (uint32_t k = 0; k < K; ++k) {
                const uint32_t r = r0 + lane + 64 * k;
                x[k] = r < R ? v.frag_w1[sbase + r] : 0;
            }
#pragma unroll
            for (uint32_t k = 0; k < K; ++k) {
                const uint32_t r = r0 + lane + 64 * k;
                if (r < R) w_lds[wv][r] = x[k];
            }
        }
        wave_lds_fence();
    }
    const bool wait = !RETRY && MEMBER && todo && len && gp == GP_LIST && len <= F && (i / N + 1) * BS <= v.shard_len &&
                      oa - sbase + len > MPLAN_LDS;
    if (todo && !wait) {
        todo = false;
        const uint64_t rel = oa - sbase, b = i / N;
        uint64_t q = PLAN_SKIP;
        if (len && gp == GP_LIST) {
            bool ok = len <= F && rel + len <= LDSW && (b + 1) * BS <= v.shard_len;
            uint64_t *const W = &w_lds[wv][ok ? rel : 0];
            uint32_t sp[LSEG - 1];
#pragma unroll
            for (uint32_t k = 0; k < LSEG - 1; ++k) sp[k] = BS;
            if (ok) {
                bool lean_all = true, fit_all = true;
                for (uint32_t k = 0; k < len; ++k) {
                    const uint64_t w = W[k];
                    const uint32_t cnt = (uint32_t)(w >> 32) & 0xFFFF, st0 = (uint32_t)(w >> 48) & 0xFF;
                    lean_all = lean_all && frag_lean(w);
                    if (lean_all && fit_all) fit_all = seg_add_split<LSEG>(st0, sp) && seg_add_split<LSEG>(st0 + cnt, sp);
                }
                // a pair that failed only on its segment count (every run lean): the retry
                if (MEMBER && !RETRY && PLAN_RETRY) rt = lean_all && !fit_all;
                ok = lean_all && fit_all;
            }
            if (ok) {
                // the accept runs' scan flags, 16 in flight at a time, then folded into bit 57
                // (the loads take clamped indices and no branch: a load under a lane condition
                // was issued and waited for one at a time, a memory round trip per run)
                constexpr uint32_t FC = F < MPX_PL_FLAG_C ? F : MPX_PL_FLAG_C;
                for (uint32_t k0 = 0; k0 < len; k0 += FC) {
                    uint32_t ix[FC], fg[FC];
                    uint32_t acc = 0;
#pragma unroll
                    for (uint32_t k = 0; k < FC; ++k) {
                        const uint64_t w = k0 + k < len ? W[k0 + k] : 0;
                        const bool a = k0 + k < len && (w >> 60) == K_ACCEPT;
                        ix[k] = a ? (uint32_t)w : 0;
                        acc |= (uint32_t)a << k;
                    }
#pragma unroll
                    for (uint32_t k = 0; k < FC; ++k) fg[k] = v.m_flags[ix[k]];
#pragma unroll
                    for (uint32_t k = 0; k < FC; ++k)
                        if (((acc >> k) & 1) && (fg[k] & F_GRANTED)) W[k0 + k] |= MP_GRANTED;
                }
                uint32_t lo[LSEG], sl[LSEG];
#pragma unroll
                for (uint32_t g = 0; g < LSEG; ++g) {
                    lo[g] = g ? sp[g - 1] : 0;
                    sl[g] = lo[g] >= BS ? 0 : (g < LSEG - 1 ? sp[g] : BS) - lo[g];
                }
                const uint64_t blo = v.shard_begin + (b << BSH);
                // one pass over the pair in message order; EMIT: the second pass, which
                // writes the snapshot records (the first one decided the pair is kept)
                // the snapshot run records: counted by the deciding pass, one reservation per pair,
                // written by the emitting pass (no returning atomic per record)
                unsigned long long rbase = 0;
                uint32_t rnext = 0, nrec = 0;
                const uint32_t rsub = (blockIdx.x * 4 + (threadIdx.x >> 6)) & (v.out_subs - 1);
                auto walk = [&](auto emit_tag, uint32_t &pres, uint32_t &comm, uint32_t (&fix)[LSEG],
                                unsigned long long &a, unsigned long long &l, unsigned long long &p,
                                bool &snap) {
                    constexpr bool EMIT = decltype(emit_tag)::value;
                    auto run = [&](uint32_t k) {
                        const uint64_t w = W[k];
                        const uint32_t cnt = (uint32_t)(w >> 32) & 0xFFFF, st0 = (uint32_t)(w >> 48) & 0xFF;
                        const bool learn = (w >> 60) == K_COMMIT;
                        if (!learn && !(w & MP_GRANTED)) return;          // a rejected / dropped accept
#pragma unroll
                        for (uint32_t g = 0; g < LSEG; ++g) {
                            if (!sl[g] || lo[g] < st0 || lo[g] >= st0 + cnt) continue;
                            if (learn) l += sl[g];
                            if ((comm >> g) & 1) {
                                // through another entry (ingest's FR_VCHK): the Value check, k_commit_check
                                if ((MEMBER || learn) && ((w >> 56) & FR_VCHK)) ck = true;
                                // (multi: an ACCEPT over a committed instance is skipped, :1380)
                            } else if (learn) {
                                comm |= 1u << g; pres |= 1u << g; fix[g] = k;
                            } else if (MEMBER) {
                                if (!((pres >> g) & 1)) { pres |= 1u << g; fix[g] = k; a += sl[g]; }   // insert
                            } else {
                                pres |= 1u << g; fix[g] = k; a += sl[g];     // multi: the last granted accept
                            }
                        }
                    };
                    // FilterAcceptedValues over the bucket-local interval [il, ih)
                    auto snap_iv = [&](uint32_t g8, uint32_t il, uint32_t ih) {
#pragma unroll
                        for (uint32_t g = 0; g < LSEG; ++g) {
                            if (!((pres >> g) & 1)) continue;
                            const uint32_t x0 = lo[g] > il ? lo[g] : il, x1 = lo[g] + sl[g] < ih ? lo[g] + sl[g] : ih;
                            if (x0 >= x1) continue;
                            p += x1 - x0;
                            if (EMIT) {                            // at the place reserved after the first pass
                                const unsigned long long at = rbase + rnext++;
                                if (at < v.out_cap) {
                                    OutRec r;
                                    r.msg = g8; r.ref = (uint32_t)(oa + fix[g]); r.aux = OUT_RUN | x0 | ((x1 - x0) << OUT_RUN_SHIFT);
                                    v.out[(uint64_t)rsub * v.out_cap + at] = r;
                                }
                            } else {
                                ++nrec;
                            }
                        }
                    };
                    auto event = [&](uint32_t info, uint32_t g8, uint64_t e) {
                        const uint32_t t8 = info & 0xFF, fl = info >> 8;
                        if (MEMBER && t8 == MPX_MSG_E_EPOCH) {
                            if (fl & F_ACCCLR) pres &= comm;               // the Acceptor's accepted map goes
                        } else if (t8 == MPX_MSG_PREPARE) {
                            if (!(fl & F_GRANTED) || !pres) return;
                            snap = true;
                            const uint64_t ax = v.ev_aux[e];
                            if (ax & EVX_ONE) {
                                snap_iv(g8, (uint32_t)(ax >> 40) & 0x1FF, (uint32_t)(ax >> 49) & 0x1FF);
                            } else {
                                const uint32_t r0 = (uint32_t)ax, nr = (uint32_t)(ax >> 32) & 0xFF;
                                for (uint32_t r = 0; r < nr; ++r) {        // sorted, disjoint ranges
                                    const uint64_t ra = v.g_a[r0 + r], rb = v.g_b[r0 + r];
                                    const uint64_t x0 = ra > blo ? ra - blo : 0, x1 = rb < blo + BS ? rb - blo : BS;
                                    if (rb > blo && ra < blo + BS && x0 < x1) snap_iv(g8, (uint32_t)x0, (uint32_t)x1);
                                }
                            }
                        }
                        // any other event of a pair without promise-reply runs acts on nothing
                        // here (k_apply AM_SNAP: a P_START clears an empty merge, a quorum emits it)
                    };
                    uint32_t k = 0;
                    for (uint64_t e = e0; e < e1 && !fb; e += 8) {
                        const uint32_t m = (uint32_t)(e1 - e < 8 ? e1 - e : 8);
                        uint32_t em[8], ei[8];
#pragma unroll
                        for (uint32_t j = 0; j < 8; ++j) em[j] = j < m ? v.ev_msg[e + j] : NONE32;
                        uint32_t et[8], ef[8];
#pragma unroll
                        for (uint32_t j = 0; j < 8; ++j) {       // (clamped, unconditional: all in flight)
                            const uint32_t x = j < m ? em[j] : 0;
                            et[j] = v.m_type[x];
                            ef[j] = v.m_flags[x];
                        }
#pragma unroll
                        for (uint32_t j = 0; j < 8; ++j) ei[j] = j < m ? et[j] | (ef[j] << 8) : 0;
#pragma unroll
                        for (uint32_t j = 0; j < 8; ++j) {
                            if (j >= m) break;
                            while (k < len && (uint32_t)W[k] <= em[j]) run(k++);   // a message's runs before its event
                            event(ei[j], em[j], e + j);
                        }
                    }
                    while (k < len && !fb) run(k++);
                };
                uint32_t pres = 0, comm = 0, fix[LSEG];
#pragma unroll
                for (uint32_t g = 0; g < LSEG; ++g) fix[g] = 0;
                bool snap = false;
                walk(std::false_type{}, pres, comm, fix, cA, cL, cP, snap);
                if (!fb) {
                    if (snap && nrec) rbase = atomicAdd(&v.out_cursor[OUT_STRIDE * rsub], (unsigned long long)nrec);
                    if (snap) {                                    // kept: the emitting pass
                        uint32_t p2 = 0, c2 = 0, f2[LSEG];
#pragma unroll
                        for (uint32_t g = 0; g < LSEG; ++g) f2[g] = 0;
                        unsigned long long a2 = 0, l2 = 0, pp2 = 0;
                        bool s2 = false;
                        walk(std::true_type{}, p2, c2, f2, a2, l2, pp2, s2);
                    }
                    uint32_t val[LSEG];
#pragma unroll
                    for (uint32_t g = 0; g < LSEG; ++g)
                        val[g] = !sl[g] ? val[g ? g - 1 : 0] : ((pres >> g) & 1) ? fix[g] + 1 : 0;
                    if (LSEG == 4 || sp[LSEG == 4 ? 0 : 3] == BS) {   // <= 4 segments: one plan word for k_store
                        const uint32_t v4[4] = {val[0], val[1], val[2], val[3]}, s3[3] = {sp[0], sp[1], sp[2]};
                        q = plan_pack(v4, s3);
                    } else {
                        // 5..LSEG segments: the split points and segment values to the extension
                        // list (k_store_ext writes the slots; k_store skips the bucket)
                        if constexpr (LSEG <= 8) {
                            // split points as 7 x 9 bits (BS = unused), segment values as bytes
                            xw0 = xw1 = 0;
#pragma unroll
                            for (uint32_t k = 0; k < LSEG - 1 && k < 7; ++k) xw0 |= (uint64_t)(sp[k] & 0x1FF) << (9 * k);
#pragma unroll
                            for (uint32_t k = 0; k < LSEG && k < 8; ++k) xw1 |= (uint64_t)(val[k] & 0xFF) << (8 * k);
                        } else {
                            // up to 15 split points (1..255) as bytes, their count in the item's top byte;
                            // up to 16 segment values as bytes
                            xw0 = xw1 = xw2 = xw3 = 0;
                            uint32_t ns = 0;
#pragma unroll
                            for (uint32_t k = 0; k < LSEG - 1; ++k) {
                                if (sp[k] >= BS) continue;
                                ++ns;
                                if (k < 8) xw0 |= (uint64_t)(sp[k] & 0xFF) << (8 * k);
                                else xw1 |= (uint64_t)(sp[k] & 0xFF) << (8 * (k - 8));
                            }
#pragma unroll
                            for (uint32_t k = 0; k < LSEG; ++k) {
                                if (k < 8) xw2 |= (uint64_t)(val[k] & 0xFF) << (8 * k);
                                else xw3 |= (uint64_t)(val[k] & 0xFF) << (8 * (k - 8));
                            }
                            xns = ns;
                        }
                        xt = true;
                    }
                    v.st_valid[i] = 1;
                }
            } else {
                fb = true;
            }
            if (fb) cA = cL = cP = 0;
        }
        if (!RETRY && (gp == GP_LIST || MEMBER)) v.plan[i] = q;
        else if (RETRY && q != PLAN_SKIP) v.plan[i] = q;       // (the first plan wrote PLAN_SKIP)
    }
    const uint64_t rem = __ballot(todo);
    if (!rem || RETRY) break;
    sbase = rl64(oa, (uint32_t)__builtin_ctzll(rem));
    wave_lds_fence();                                  // the window is read: restage
    }
    if (!RETRY && MEMBER && PLAN_RETRY) {              // the retry list: fb pairs that failed only on segments
        const uint64_t rm = __ballot(rt && fb);
        if (rm) {
            unsigned long long base = 0;
            if (lane == 0) base = atomicAdd(v.gp_rt_n, (unsigned long long)__popcll(rm));
            base = __shfl(base, 0, 64);
            if (rt && fb) v.gp_rt[base + (uint64_t)__popcll(rm & ((1ull << lane) - 1))] = i;
        }
        fb = fb && !rt;
    }
    const uint64_t fm = __ballot(fb);
    if (fm) {
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(v.gp_dyn_n, (unsigned long long)__popcll(fm));
        base = __shfl(base, 0, 64);
        if (fb) {
            uint64_t *w = v.gp_dyn + GP_WORDS * (base + (uint64_t)__popcll(fm & ((1ull << lane) - 1)));
            w[0] = oa; w[1] = o1; w[2] = e0; w[3] = e1; w[4] = i;
        }
    }
    const uint64_t cm = __ballot(ck && !fb);
    if (cm) {
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(v.gp_chk_n, (unsigned long long)__popcll(cm));
        base = __shfl(base, 0, 64);
        if (ck && !fb) {
            uint64_t *w = v.gp_chk + CHK_WORDS * (base + (uint64_t)__popcll(cm & ((1ull << lane) - 1)));
            w[0] = oa; w[1] = o1; w[2] = i;
        }
    }
    const uint64_t xm = __ballot(xt && !fb);
    if (xm) {
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(v.gp_ext_n, (unsigned long long)__popcll(xm));
        base = __shfl(base, 0, 64);
        if (xt && !fb) {
            uint64_t *w = v.gp_ext + EXT_WORDS * (base + (uint64_t)__popcll(xm & ((1ull << lane) - 1)));
            w[0] = i | (uint64_t)xns << 56; w[1] = xw0; w[2] = xw1; w[3] = xw2; w[4] = xw3;
        }
    }
    if (MEMBER && !RETRY && i < NB) plan_chosen(v, i, cC);
    unsigned long long cc[4] = {cA, cL, cC, cP};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        unsigned long long x = cc[k];
        for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
        cc[k] = x;
    }
    if (lane == 0) { red[wv][0] = cc[0]; red[wv][1] = cc[1]; red[wv][2] = cc[2]; red[wv][3] = cc[3]; }
    __syncthreads();
    if (threadIdx.x < 4) {
        const uint32_t t = threadIdx.x;
        const unsigned long long x = red[0][t] + red[1][t] + red[2][t] + red[3][t];
        const int slot = t == 0 ? PC_A : t == 1 ? PC_L : t == 2 ? PC_C : PC_P;
        if (x) atomicAdd(&v.partials[8 * (blockIdx.x % apply_wgs) + slot], x);
    }
}

// The slots of the pairs k_plan_list described by 5..PLAN_XSEG (multi) / PLAN_XSEG_MEMBER (member)
// segments: one wave per pair, 4 slots per lane — the slot's segment is the number of split points
// at or below it, its value that segment's (pair-local run + 1, or 0).  Items (EXT_WORDS words):
// up to 8 segments {pair | EXT_LEGACY << 56, 7 x 9-bit split points (BS = unused), 8 value bytes};
// up to 16 {pair | splits << 56, 15 split-point bytes (ascending) in two words, 16 value bytes in two}.
__global__ __launch_bounds__(256) void k_store_ext(DevView v)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t n_ext = *v.gp_ext_n, nwaves = (uint64_t)gridDim.x * 4;
    for (uint64_t x = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); x < n_ext; x += nwaves) {
        const uint64_t *it = v.gp_ext + EXT_WORDS * x;
        const uint64_t w = it[0], s0 = it[1], s1 = it[2], v0 = it[3], v1 = it[4];
        const uint64_t i = w & ((1ull << 56) - 1);
        const uint32_t ns = (uint32_t)(w >> 56);
        const uint64_t b = i / v.N, n = i - b * v.N;
        uint32_t val[4];
        if (ns == EXT_LEGACY) {
#pragma unroll
            for (uint32_t t = 0; t < 4; ++t) {
                const uint32_t sl = 4 * lane + t;
                uint32_t g = 0;
#pragma unroll
                for (uint32_t k = 0; k < 7; ++k) g += sl >= ((s0 >> (9 * k)) & 0x1FF);
                val[t] = (uint32_t)(s1 >> (8 * g)) & 0xFF;
            }
        } else {
#pragma unroll
            for (uint32_t t = 0; t < 4; ++t) {
                const uint32_t sl = 4 * lane + t;
                uint32_t g = 0;
#pragma unroll
                for (uint32_t k = 0; k < 15; ++k)
                    g += k < ns && sl >= (uint32_t)(((k < 8 ? s0 : s1) >> (8 * (k & 7))) & 0xFF);
                val[t] = (uint32_t)((g < 8 ? v0 : v1) >> (8 * (g & 7))) & 0xFF;
            }
        }
        const uint64_t at = n * v.shard_len + (b << BSH) + 4 * lane;
        if (v.slot_w == 1)
            *reinterpret_cast<u8x4 *>(static_cast<uint8_t *>(v.st) + at) =
                u8x4{(uint8_t)val[0], (uint8_t)val[1], (uint8_t)val[2], (uint8_t)val[3]};
        else
            *reinterpret_cast<u16x4 *>(static_cast<uint16_t *>(v.st) + at) =
                u16x4{(uint16_t)val[0], (uint16_t)val[1], (uint16_t)val[2], (uint16_t)val[3]};
    }
}

// The Value check of the planned pairs k_plan_list put on gp_chk, one wave per pair, 4 slots
// per lane, the pair's runs in message order (k_apply's rules, without its state): the first
// commit / learn of a slot fixes its entry; a later one through another entry (member: also
// a granted accept; a learn only when its message is the proposer's own, F_PROP) whose Value
// differs is the violation k_apply records — MPX_V_COMMIT_VALUE (multi/paxos.cpp:1508),
// MPX_V_LEARN_VALUE (member/paxos.cpp:1765,1040) — once per slot.  Plan-list pairs hold
// dense accept / commit runs only.
template <bool MEMBER>
__global__ __launch_bounds__(256) void k_commit_check(DevView v)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t n_chk = *v.gp_chk_n, nwaves = (uint64_t)gridDim.x * 4;
    // Software pipeline over the wave's pairs (the chain item words -> run descriptors -> member
    // scan flags -> Values is one dependent round trip per link): the next pair's descriptors and
    // the pair after's item words are in flight while a pair is checked, its flags one pair
    // ahead, so a pair waits only for its Values — the first commit's and the checked runs', four
    // runs per round trip, the first group issued with the first commits'.
    // (Since ingest marks only the re-commits whose Values differ, FR_VCHK, valid traces put no pair
    // here and the kernel is not launched, any_vchk; it runs on violation traces, the goldens.)
    auto words = [&](uint64_t x) -> uint64_t { return x < n_chk && lane < CHK_WORDS ? v.gp_chk[CHK_WORDS * x + lane] : 0; };
    struct Desc { uint64_t fw0, fw1; };
    auto descr = [&](uint64_t w) -> Desc {
        Desc d{0, 0};
        const uint64_t f0 = rl64(w, 0), f1 = rl64(w, 1);
        if (lane < f1 - f0 && lane < 64) {
            const ulonglong2 x = *reinterpret_cast<const ulonglong2 *>(v.frags + f0 + lane);
            d.fw0 = x.x; d.fw1 = x.y;
        }
        return d;
    };
    auto flags = [&](const Desc &d) -> uint32_t { return MEMBER && d.fw1 ? v.m_flags[(uint32_t)d.fw1] : 0; };
    uint64_t x = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    uint64_t w0 = words(x), w1 = words(x + nwaves), w2 = words(x + 2 * nwaves);
    Desc d0 = descr(w0), d1 = descr(w1);
    uint32_t m0 = flags(d0);
    for (; x < n_chk; x += nwaves) {
        const uint64_t w = w0;
        const Desc d = d0;
        const uint32_t mf = m0;
        m0 = flags(d1);                                           // pair x + 1
        d0 = d1; d1 = descr(w2);                                  // pair x + 2
        w0 = w1; w1 = w2; w2 = words(x + 3 * nwaves);             // pair x + 3
        const uint64_t f0 = rl64(w, 0), f1 = rl64(w, 1), i = rl64(w, 2);
        const uint64_t fw0 = d.fw0, fw1 = d.fw1;
        const uint32_t b = (uint32_t)(i / v.N), n = (uint32_t)(i - (uint64_t)b * v.N);
        const uint64_t li0 = (uint64_t)b << BSH;
        // plan-list pairs have at most PLAN_XFRAGS (32) runs: one descriptor window
        const uint32_t nf = (uint32_t)(f1 - f0 < 64 ? f1 - f0 : 64);
        // pass 1 (no loads): each slot's first commit / learn — its entry and run
        uint32_t se[SPL], sa[SPL];
#pragma unroll
        for (uint32_t j = 0; j < SPL; ++j) { se[j] = 0; sa[j] = 64; }
        for (uint32_t a = 0; a < nf; ++a) {
            const uint64_t wv1 = rl64(fw1, a);
            if ((uint32_t)(wv1 >> 60) != K_COMMIT) continue;
            const uint32_t ent = (uint32_t)rl64(fw0, a);      // (entries < MAX_ENTRIES < 2^32: ingest refuses more)
            const uint32_t cnt = (uint32_t)(wv1 >> 32) & 0xFFFF, st0 = (uint32_t)(wv1 >> 48) & 0xFF;
#pragma unroll
            for (uint32_t j = 0; j < SPL; ++j) {
                const int dd = (int)(lane + 64 * j) - (int)st0;
                if (dd >= 0 && dd < (int)cnt && sa[j] == 64) { se[j] = ent + dd; sa[j] = a; }
            }
        }
        // pass 2: the later checked runs over committed slots through another entry, four runs'
        // Values in flight at a time (the first group together with the first commits' Values)
        uint64_t sv[SPL];
        bool sv_loaded = false;
        for (uint32_t a0 = 0; a0 < nf; a0 += 4) {
            uint64_t xv[4][SPL];
            uint32_t xm[4];
#pragma unroll
            for (uint32_t r = 0; r < 4; ++r) {
                xm[r] = 0;
                const uint32_t a = a0 + r;
                if (a >= nf) continue;
                const uint64_t wv1 = rl64(fw1, a);
                const bool learn = (uint32_t)(wv1 >> 60) == K_COMMIT;
                const uint32_t f = MEMBER ? rl32(mf, a) : 0;
                if (!(MEMBER ? (learn ? (f & F_PROP) != 0 : (f & F_GRANTED) != 0) : learn)) continue;
                const uint32_t ent = (uint32_t)rl64(fw0, a);
                const uint32_t cnt = (uint32_t)(wv1 >> 32) & 0xFFFF, st0 = (uint32_t)(wv1 >> 48) & 0xFF;
#pragma unroll
                for (uint32_t j = 0; j < SPL; ++j) {
                    const int dd = (int)(lane + 64 * j) - (int)st0;
                    const bool c = dd >= 0 && dd < (int)cnt && sa[j] < a && ent + dd != se[j];
                    xv[r][j] = c ? v.e_val[ent + dd] : 0;
                    xm[r] |= (uint32_t)c << j;
                }
            }
            if (!__ballot(xm[0] | xm[1] | xm[2] | xm[3])) continue;    // nothing to compare in this group
            if (!sv_loaded) {
#pragma unroll
                for (uint32_t j = 0; j < SPL; ++j) sv[j] = sa[j] < 64 ? v.e_val[se[j]] : 0;
                sv_loaded = true;
            }
#pragma unroll
            for (uint32_t r = 0; r < 4; ++r)
#pragma unroll
                for (uint32_t j = 0; j < SPL; ++j)
                    if (((xm[r] >> j) & 1) && xv[r][j] != sv[j])
                        record_violation(v, MEMBER ? MPX_V_LEARN_VALUE : MPX_V_COMMIT_VALUE, n,
                                         (uint32_t)rl64(fw1, a0 + r) - (uint32_t)v.node_off[n], v.shard_begin + li0 + lane + 64 * j);
        }
    }
}

// Streams the plan: a wave takes a chunk of C whole buckets of one row — a
// state row or the chosen log (row N), 2-byte slots, 512 B per bucket — and
// writes it contiguously, one non-temporal
// store per lane per bucket, 4 slots per lane.  The chunk's plan words are
// loaded one chunk ahead and the inner loop has no branch — a PLAN_SKIP
// bucket's store goes to a scratch sink — so the only wait per chunk is for
// that one load, with the previous chunk's C stores still in flight (vmcnt
// counts stores on gfx9: a data-dependent store count would force a full drain
// instead).  A wave walks chunks c = wid, wid + nwaves, ... over the N + 1
// rows; buckets past the last whole chunk of a row take a plain tail loop.
template <uint32_t C, bool NT, typename T, typename V>
__device__ inline uint64_t store_chunks(const DevView &v, uint64_t c, const uint64_t c_base, const uint64_t c_end,
                                        const uint64_t cpr, const uint32_t prow0, T *const base0, const uint64_t stride,
                                        T *const sink, const uint64_t nwaves)
{
    if (c >= c_end) return c;
    const uint32_t lane = threadIdx.x & 63, s0 = 4 * lane;
    const uint64_t rel = c - c_base;
    uint32_t rn = (uint32_t)(rel / cpr), kn = (uint32_t)(rel - (uint64_t)rn * cpr);
    const uint32_t step_r = (uint32_t)(nwaves / cpr), step_k = (uint32_t)(nwaves - (uint64_t)step_r * cpr);
    // unconditional plan load (lanes >= C repeat lanes 0..C-1; past the end:
    // a valid dummy address) so the compiler can count it exactly
    auto ptr = [&](uint64_t cc, uint32_t rr, uint32_t kk) -> const uint64_t * {
        return cc < c_end ? v.plan + plan_idx(v, prow0 + rr, (uint64_t)kk * C + (lane & (C - 1))) : v.plan;
    };
    uint64_t qn = *ptr(c, rn, kn);
    // settled before the loop: the loop-carried plan word then has one pending
    // source, the in-loop load, which waits as vmcnt(C) (its C stores in flight)
    __builtin_amdgcn_s_waitcnt(0x0F70);
    for (; c < c_end; c += nwaves) {
        const uint64_t qw = qn;
        const uint32_t rc = rn, kc = kn;
        rn += step_r; kn += step_k;
        if (kn >= cpr) { kn -= (uint32_t)cpr; ++rn; }
        qn = *ptr(c + nwaves, rn, kn);
        T *const base = base0 + (uint64_t)rc * stride + ((uint64_t)kc * C << BSH) + s0;
#pragma unroll
        for (uint32_t j = 0; j < C; ++j) {
            const uint64_t q = rl64(qw, j);                 // wave-uniform: the segment math is scalar
            T *const dst = q == PLAN_SKIP ? sink : base + j * BS;
            const V val = V{(T)plan_slot(q, s0), (T)plan_slot(q, s0 + 1), (T)plan_slot(q, s0 + 2), (T)plan_slot(q, s0 + 3)};
            if (NT) __builtin_nontemporal_store(val, reinterpret_cast<V *>(dst));
            else *reinterpret_cast<V *>(dst) = val;
        }
    }
    return c;
}

template <uint32_t C, bool NT, typename T, typename V>
__global__ __launch_bounds__(256) void k_store(DevView v)
{
    // wave-uniform chunk walk in scalar registers (readfirstlane): the row
    // address math stays off the VGPRs the plan load writes
    const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t N = v.N;

    const uint64_t whole = v.shard_len >> BSH;            // buckets wholly inside the shard
    const uint64_t cpr = whole / C, S = (uint64_t)(N + 1) * cpr;   // rows 0..N-1 state, row N chosen log
    const uint64_t nwaves = (uint64_t)gridDim.x * 4;
    const uint64_t wid = xcd_wave_id(wv);
    const uint32_t s0 = 4 * lane;
    uint32_t *const sink = v.store_dummy + (wid & 63) * BS;
    T *const st = static_cast<T *>(v.st);
    store_chunks<C, NT, T, V>(v, wid, 0, S, cpr, 0, st, v.shard_len, reinterpret_cast<T *>(sink) + s0, nwaves);
    // tail: the whole buckets after each row's last full chunk
    const uint64_t tpr = whole - cpr * C, tails = (uint64_t)(N + 1) * tpr;
    for (uint64_t t = wid; t < tails; t += nwaves) {
        const uint64_t r = t / tpr, b = cpr * C + (t - r * tpr);
        const uint64_t q = v.plan[plan_idx(v, (uint32_t)r, b)];
        if (q == PLAN_SKIP) continue;
        __builtin_nontemporal_store(V{(T)plan_slot(q, s0), (T)plan_slot(q, s0 + 1), (T)plan_slot(q, s0 + 2),
                                      (T)plan_slot(q, s0 + 3)},
                                    reinterpret_cast<V *>(st + r * v.shard_len + (b << BSH) + s0));
    }
}

// 1-byte slots: a 256-B bucket row is too small a unit for one wave store, so
// a wave takes a chunk of C (default 128) whole buckets (C / 4 KiB of one row)
// and writes it as C / 4 contiguous KiB-stores: lane l of store j covers bytes
// 16l..16l+15 of buckets 4j..4j+3, its plan word fetched with a cross-lane
// shuffle (LDS permute, lgkmcnt) from the chunk's plan words (one or two per
// lane), which are loaded one chunk ahead as in k_store (the loop waits
// vmcnt(C / 4): the previous chunk's stores stay in flight).  When every word
// of a store is one segment (batch 256) its low half is the 16 bytes; else
// plan_bytes16 expands the segments.  Tail buckets of a row go through the
// per-bucket loop.
template <uint32_t W>
__device__ inline void reduce_summary(const DevView &v, uint32_t n_partials, unsigned long long (&red)[W][8],
                                      uint32_t row0, uint32_t stride, bool scal);

// REDUCE: workgroups [store_grid, gridDim.x) fold the partials into the summary (k_reduce's
// work) while the others store — launched when the store is the step's last kernel (the
// partials are all written by the kernels before it), so the summary's dependent launch and
// its ramp leave the step's chain (C4 shard at world 8: 64.1 vs 68.9 us, same-box A/B,
// profiles/r03_v20_fused_reduce_ab.json)
template <bool NT, uint32_t C = 64, bool REDUCE = false>
__global__ __launch_bounds__(256) void k_store8(DevView v, uint32_t store_grid, uint32_t n_partials)
{
    static_assert(C == 64 || C == 128, "one or two plan words per lane");
    if (REDUCE && blockIdx.x >= store_grid) {
        __shared__ unsigned long long red[4][8];
        const uint32_t r = blockIdx.x - store_grid, R = gridDim.x - store_grid;
        reduce_summary<4>(v, n_partials, red, 256 * r, 256 * R, r == 0);
        return;
    }
    const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t N = v.N;

    const uint64_t whole = v.shard_len >> BSH;
    const uint64_t cpr = whole / C, S = (uint64_t)(N + 1) * cpr;
    const uint64_t nwaves = (uint64_t)store_grid * 4;
    const uint64_t wid = xcd_wave_id_g(wv, store_grid);
    uint8_t *const st = static_cast<uint8_t *>(v.st);
    uint8_t *const sink = reinterpret_cast<uint8_t *>(v.store_dummy) + (wid & 63) * 1024 + 16 * lane;
    const uint32_t p16 = 16 * (lane & 15);                 // the lane's first slot in its bucket
    if (wid < S) {
        uint32_t rn = (uint32_t)(wid / cpr), kn = (uint32_t)(wid - (uint64_t)rn * cpr);
        const uint32_t step_r = (uint32_t)(nwaves / cpr), step_k = (uint32_t)(nwaves - (uint64_t)step_r * cpr);
        // plan words of bucket kk * C + lane (and + 64) of row rr; past the end: a valid dummy
        auto ld = [&](uint64_t cc, uint32_t rr, uint32_t kk, uint32_t off) -> uint64_t {
            return v.plan[cc < S ? plan_idx(v, rr, (uint64_t)kk * C + off + lane) : lane];
        };
        uint64_t qn = ld(wid, rn, kn, 0), qn1 = C == 128 ? ld(wid, rn, kn, 64) : 0;
        __builtin_amdgcn_s_waitcnt(0x0F70);
        for (uint64_t c = wid; c < S; c += nwaves) {
            const uint64_t qw = qn, qw1 = qn1;
            const uint32_t rc = rn, kc = kn;
            rn += step_r; kn += step_k;
            if (kn >= cpr) { kn -= (uint32_t)cpr; ++rn; }
            qn = ld(c + nwaves, rn, kn, 0);
            if (C == 128) qn1 = ld(c + nwaves, rn, kn, 64);
            uint8_t *const base = st + (uint64_t)rc * v.shard_len + ((uint64_t)kc * C << BSH) + 16 * lane;
#pragma unroll
            for (uint32_t j = 0; j < C / 4; ++j) {
                const uint64_t q = __shfl(j < 16 ? qw : qw1, (int)((4 * j + (lane >> 4)) & 63), 64);
                uint8_t *const dst = q == PLAN_SKIP ? sink : base + 1024 * j;
                u32x4 x;
                if (__ballot(q != PLAN_SKIP && (uint32_t)(q >> 32) != PLAN_UNI)) x = plan_bytes16(q, p16);
                else x = u32x4{(uint32_t)q, (uint32_t)q, (uint32_t)q, (uint32_t)q};
                if (NT) __builtin_nontemporal_store(x, reinterpret_cast<u32x4 *>(dst));
                else *reinterpret_cast<u32x4 *>(dst) = x;
            }
        }
    }
    const uint32_t s0 = 4 * lane;
    const uint64_t tpr = whole - cpr * C, tails = (uint64_t)(N + 1) * tpr;
    for (uint64_t t = wid; t < tails; t += nwaves) {
        const uint64_t r = t / tpr, b = cpr * C + (t - r * tpr);
        const uint64_t q = v.plan[plan_idx(v, (uint32_t)r, b)];
        if (q == PLAN_SKIP) continue;
        __builtin_nontemporal_store(u8x4{(uint8_t)plan_slot(q, s0), (uint8_t)plan_slot(q, s0 + 1),
                                         (uint8_t)plan_slot(q, s0 + 2), (uint8_t)plan_slot(q, s0 + 3)},
                                    reinterpret_cast<u8x4 *>(st + r * v.shard_len + (b << BSH) + s0));
    }
}

// Plan and store in one launch (the C4 shape only — every pair lean, the chosen log planned
// statically, the store ends the step: run_ends_with_store — with 1-byte slots).  A workgroup
// of 8 waves takes groups of PS_G buckets: waves 0 .. PS_PW-1 plan a group into one LDS buffer
// — lane t < PS_G * N the group's pair t (plan_lean, its descriptors loaded straight from
// frag_w1: the group's pairs are consecutive), the lanes of the last planner wave its buckets'
// chosen-log words (plan_chosen_word, no divergence with the pair lanes) — while the other
// waves store the previous group's rows from the other buffer (1 KiB nontemporal stores of 4
// buckets each); then all cross a barrier that orders LDS only (the stores stay in flight) and
// swap buffers.  No plan words go through HBM, there is no k_plan launch, and a group's
// dependent descriptor / flag loads run under the previous group's stores — so a group's store
// has to outlast a plan's three dependent round trips under that write traffic (PS_G: C4 shard
// 62.1 -> 53.4 us, C4 0.364 -> 0.344 ms at 32 buckets / 6 planner waves; 16 / 24 / 28 / 40
// buckets slower, as is loading the next group's offsets a group ahead (one round trip less
// per plan, 73 VGPRs: shard 54.2 us, C4 0.361 ms), profiles/r06_ab_plan_store.json).  The
// plan counters go straight to the summary words (one atomic per counter and workgroup);
// workgroups [ps_grid, gridDim.x) fold the partial rows of the kernels before (k_store8<..,
// REDUCE>'s split).  
#ifndef MPX_PS_G
#define MPX_PS_G 32
#endif
#ifndef MPX_PS_PW
#define MPX_PS_PW 6
#endif
#ifndef MPX_PS_WG
#define MPX_PS_WG 8
#endif
// PS_WG waves per workgroup, PS_PW of them planners
constexpr uint32_t PS_G = MPX_PS_G, PS_PW = MPX_PS_PW, PS_WG = MPX_PS_WG, PS_CHOSEN = 64 * (PS_PW - 1);
static_assert(PS_G % 4 == 0 && PS_G <= 64 && PS_PW >= 2 && PS_PW < PS_WG && PS_WG <= 16, "k_plan_store8 shape");
__device__ inline void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
// (72 VGPRs: 3 workgroups per CU; MPX_PS_WAVES=8 forces 64 with a 28-B spill, A/B build)
#ifndef MPX_PS_WAVES
#define MPX_PS_WAVES 6
#endif
#ifndef MPX_PS_WPC
#define MPX_PS_WPC (MPX_PS_WAVES * 4 / MPX_PS_WG)
#endif
__global__ __launch_bounds__(64 * PS_WG, MPX_PS_WAVES) void k_plan_store8(DevView v, uint32_t ps_grid, uint32_t n_partials)
{
    constexpr uint32_t S = PS_WG - PS_PW, KPR = PS_G / 4;    // storer waves, KiB stores per row
    __shared__ uint64_t pw[2][64 * PS_PW];
    __shared__ unsigned long long red[PS_WG][8];
    if (blockIdx.x >= ps_grid) {
        const uint32_t r = blockIdx.x - ps_grid, R = gridDim.x - ps_grid;
        reduce_summary<PS_WG>(v, n_partials, red, 64 * PS_WG * r, 64 * PS_WG * R, r == 0);
        return;
    }
    const uint32_t t = threadIdx.x, lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);
    const bool planner = wv < PS_PW;
    const uint32_t N = v.N;
    const uint64_t NB = v.NB, ngroups = (NB + PS_G - 1) / PS_G;
    uint8_t *const st = static_cast<uint8_t *>(v.st);
    unsigned long long cA = 0, cL = 0, cC = 0;
    uint32_t rest = 0;
    auto plan_group = [&](uint64_t g, uint64_t *out) {
        const uint64_t b0 = g * PS_G;
        uint64_t q = PLAN_SKIP;
        if (t < PS_G * N) {
            const uint64_t i = b0 * N + t, b = b0 + t / N;
            if (b < NB) {
                const uint64_t oa = v.f_off[i], o1 = v.f_off[i + 1];
                const uint8_t gp = v.pair_gp[i];
                const uint32_t len = (uint32_t)(o1 - oa);
                const bool in_list = len && len <= FAST_MAX_FRAGS && !gp;
                q = plan_lean<false>(v, i, b, len, in_list, [&](uint32_t k) { return v.frag_w1[oa + k]; }, cA, cL, rest);
            }
        } else if (t >= PS_CHOSEN && t < PS_CHOSEN + PS_G) {
            const uint64_t b = b0 + (t - PS_CHOSEN);
            if (b < NB) {
                unsigned long long c = 0;
                q = plan_chosen_word<false>(v, b, c);
                cC += c;
            }
        }
        out[t] = q;
    };
    auto store_group = [&](uint64_t g, const uint64_t *in) {
        const uint32_t p16 = 16 * (lane & 15);
        uint8_t *const base = st + ((g * PS_G) << BSH) + p16;
        for (uint32_t u = wv - PS_PW; u < (N + 1) * KPR; u += S) {
            const uint32_t r = u / KPR, bl = 4 * (u - r * KPR) + (lane >> 4);
            const uint64_t q = in[r < N ? bl * N + r : PS_CHOSEN + bl];   // (PLAN_SKIP past NB)
            if (q == PLAN_SKIP) continue;
            u32x4 x;
            if (__ballot((uint32_t)(q >> 32) != PLAN_UNI)) x = plan_bytes16(q, p16);
            else x = u32x4{(uint32_t)q, (uint32_t)q, (uint32_t)q, (uint32_t)q};
            __builtin_nontemporal_store(x, reinterpret_cast<u32x4 *>(base + (uint64_t)r * v.shard_len + ((uint64_t)bl << BSH)));
        }
    };
    uint64_t g = blockIdx.x;                                  // (uniform: every wave crosses every barrier)
    uint32_t buf = 0;
    if (planner && g < ngroups) plan_group(g, pw[0]);
    lds_barrier();
    for (; g < ngroups; g += ps_grid) {
        const uint64_t gn = g + ps_grid;
        if (planner) {
            if (gn < ngroups) plan_group(gn, pw[buf ^ 1]);
        } else {
            store_group(g, pw[buf]);
        }
        lds_barrier();
        buf ^= 1;
    }
    if (planner) {
        unsigned long long cc[4] = {cA, cL, cC, rest};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            unsigned long long x = cc[k];
            for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
            if (lane == 0) red[wv][k] = x;
        }
    }
    __syncthreads();
    if (t < 4) {
        unsigned long long x = 0;
        for (uint32_t k = 0; k < PS_PW; ++k) x += red[k][t];
        if (x) {
            if (t == 3) atomicAdd(v.fast_rest, (uint32_t)x);
            else atomicAdd(&v.summary[summary_word(t == 0 ? PC_A : t == 1 ? PC_L : PC_C)], x);
        }
    }
}

// General apply: one wave owns one (node, bucket) pair of the host-built work
// list at a time, its 256 instance slots 4 per lane.  The pair's fragments and
// its snapshot events (ingest.cpp: only the events that can act on this pair)
// are walked in message order, so every instance sees its events in the
// reference's order.
//
// A slot's state is held as the entry index of its Value in the resident pool
// (AcceptedValue by reference, mpx_internal.hpp), never the Value itself: a
// fragment costs no memory access beyond its window's descriptors, scan flags
// and header ballots, loaded lane-parallel 64 fragments at a time.  Values are
// read only where the reference looks at them: the re-commit / learned-Value
// checks when the two entry indices differ (the pool is content-addressed, so a
// duplicate or retried COMMIT carries the same entries), and the snapshots a
// granted PREPARE or a promise quorum emits.
// DIGEST: the digested verification run (mpx_run) — the only user of the slot's ballot
// MEMBER: member semantics (insert-first apply, epoch events) — compiled apart so
// the multi kernel carries none of it
// MODE (multi): which work items [it0, it1) the instantiation takes — ingest.cpp
// orders the list: AM_SIMPLE pairs (no snapshot events, no promise-reply runs:
// ACCEPT / COMMIT runs only), then AM_SNAP pairs (no promise-reply runs, so their
// only events are PREPAREs: snapshots), then AM_FULL (promise rounds: merges, round
// resets, quorum emission).  The narrower ones are compiled without the code they
// never run, so they hold fewer registers and more waves per SIMD hide the
// descriptor latency.
enum { AM_FULL = 0, AM_SIMPLE = 1, AM_SNAP = 2 };
// waves per SIMD the timed instantiations are built for (the register budget: 512 / waves)
#ifndef MPX_APPLY_WAVES_SNAP
#define MPX_APPLY_WAVES_SNAP 4
#endif
#ifndef MPX_APPLY_WAVES_FULL
#define MPX_APPLY_WAVES_FULL 4
#endif
constexpr int APPLY_WAVES_SNAP = MPX_APPLY_WAVES_SNAP, APPLY_WAVES_FULL = MPX_APPLY_WAVES_FULL;
template <int WAVES_PER_EU, bool DIGEST, bool MEMBER, int MODE = AM_FULL>
__global__ __launch_bounds__(256, WAVES_PER_EU) void k_apply(DevView v, uint64_t it0, uint64_t it1)
{
    if (it1 == ~0ull) it1 = *v.gp_dyn_n;          // the device-built list (k_plan_member)
    __shared__ uint16_t lidx_all[4][BS];
    __shared__ u64x2 pre_all[4][BS];           // pre-accepted merge (pid, PRESENT | r-entry): rare, kept in LDS
    __shared__ unsigned long long red[4][8];
// (snapshot records staged in a per-wave LDS queue, one reservation per 128: measured slower,
// C3 step 1.447 vs 1.388 ms, profiles/r04_v9_ab_emit_queue.json)
#define EMIT(...) emit_rows(v, __VA_ARGS__)
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint16_t *lidx = lidx_all[wv];
    u64x2 *pre = pre_all[wv];
    constexpr bool SIMPLE = MODE == AM_SIMPLE;   // no events at all
    constexpr bool ROUNDS = MODE == AM_FULL;     // promise-round runs and events
#pragma unroll
    for (uint32_t j = 0; j < SPL; ++j) lidx[lane + 64 * j] = 0xFFFF;
    wave_lds_fence();
    uint32_t cA = 0, cL = 0, cP = 0, cQ = 0;    // per-lane counts stay far below 2^32
    unsigned long long dig = 0;
    constexpr bool member = MEMBER;
    const uint64_t stride = (uint64_t)gridDim.x * 4;
    const uint64_t *__restrict__ e_val = v.e_val;
    constexpr uint32_t S_PRESENT = 1, S_COMMITTED = 2;

    // work list: the pairs the lean kernel does not take (ingest.cpp), GP_WORDS
    // per item.  Three-stage software pipeline over this wave's items, issued at
    // the top of item i so each stage's loads had a whole item to land: (1) the
    // item's CSR ranges three items ahead, (2) its first descriptor window two
    // ahead, (3) that window's scan flags one ahead — one wait per item.
    auto rt1 = [&](uint64_t i) -> uint64_t {
        if (i >= it1 || lane > 4) return 0;
        return v.gp_list[GP_WORDS * i + lane];          // lanes 0..4: fi, fe, ei, ee, q
    };
    // the event window carries each event's aux word (PREPARE: its ranges in the bucket)
    // (ROUNDS: with each run's uniform proposal id, f_pid, so a promise-reply run whose entries
    // share one — FR_UPID — merges without loading its slots' ids)
    struct Win { uint64_t fw0, fw1; uint32_t evm; uint64_t eax; uint64_t fpid; };
    auto rt2 = [&](uint64_t off) -> Win {
        Win w{0, NONE32, NONE32, 0, 0};
        const uint64_t fi = rl64(off, 0), fe = rl64(off, 1), ei = rl64(off, 2), ee = rl64(off, 3);
        if (lane < fe - fi && lane < 64) {
            const ulonglong2 x = *reinterpret_cast<const ulonglong2 *>(v.frags + fi + lane);
            w.fw0 = x.x; w.fw1 = x.y;
            if (ROUNDS) w.fpid = v.f_pid[fi + lane];
        }
        if (!SIMPLE && lane < ee - ei && lane < 64) { w.evm = v.ev_msg[ei + lane]; w.eax = v.ev_aux[ei + lane]; }
        return w;
    };
    struct Flg { uint32_t fflag, einfo; uint64_t fbal; };
    auto rt3 = [&](const Win &w) -> Flg {
        Flg f{0, 0, 0};
        if ((uint32_t)w.fw1 != NONE32) {
            f.fflag = v.m_flags[(uint32_t)w.fw1];
            if (DIGEST) f.fbal = v.m_ballot[(uint32_t)w.fw1];
        }
        if (!SIMPLE && w.evm != NONE32) f.einfo = (uint32_t)v.m_type[w.evm] | ((uint32_t)v.m_flags[w.evm] << 8);
        return f;
    };
    uint64_t it = it0 + (uint64_t)blockIdx.x * 4 + wv;
    uint64_t off0 = rt1(it), off1 = rt1(it + stride), off2 = rt1(it + 2 * stride);
    Win win0 = rt2(off0), win1 = rt2(off1);
    Flg flg0 = rt3(win0);
    for (; it < it1; it += stride) {
        const uint64_t off_c = off0;
        const Win win = win0;
        const Flg flg = flg0;
        flg0 = rt3(win1);                        // item i + 1
        win0 = win1; win1 = rt2(off2);           // item i + 2
        off0 = off1; off1 = off2; off2 = rt1(it + 3 * stride);   // item i + 3
        const uint64_t q = rl64(off_c, 4);
        const uint32_t b = (uint32_t)(q / v.N);
        const uint32_t n = (uint32_t)(q - (uint64_t)b * v.N);
        uint64_t fi = rl64(off_c, 0), fe = rl64(off_c, 1), ei = rl64(off_c, 2), ee = rl64(off_c, 3);
        const uint64_t pbase = fi;               // the pair's first fragment (slots are pair-local)
        const uint64_t li0 = (uint64_t)b << BSH;
        uint64_t sb[DIGEST ? SPL : 1];           // ballot (multi: accept / commit id; member: proposal id)
        uint32_t sfl = 0;                        // S_* flags of slot j in byte j
        uint32_t se[SPL], sm[SPL];               // Value entry index, fixing fragment + 1
#define SF(j) ((sfl >> (8 * (j))) & 0xFF)
#define SF_SET(j, x) (sfl = (sfl & ~(0xFFu << (8 * (j)))) | ((uint32_t)(x) << (8 * (j))))
#pragma unroll
        for (uint32_t j = 0; j < SPL; ++j) { if (DIGEST) sb[j] = 0; se[j] = sm[j] = 0; if (ROUNDS) pre[lane + 64 * j] = u64x2{0, 0}; }

        bool first = true;
        while (fi < fe || ei < ee) {
            const uint32_t nf = (uint32_t)(fe - fi < 64 ? fe - fi : 64);
            const uint32_t ne = SIMPLE ? 0 : (uint32_t)(ee - ei < 64 ? ee - ei : 64);
            // descriptors (one per lane) and their scan flags: the pipelined
            // first window, then loaded here for the rare longer pairs
            uint64_t fw0 = win.fw0, fw1 = win.fw1, eax = win.eax, fpid = win.fpid;
            uint32_t evm = win.evm;
            uint32_t fflag = flg.fflag, einfo = flg.einfo;
            uint64_t fbal = flg.fbal;
            if (!first) {
                Win w2{0, NONE32, NONE32, 0, 0};
                if (lane < nf) {
                    const ulonglong2 x = *reinterpret_cast<const ulonglong2 *>(v.frags + fi + lane);
                    w2.fw0 = x.x; w2.fw1 = x.y;
                    if (ROUNDS) w2.fpid = v.f_pid[fi + lane];
                }
                if (!SIMPLE && lane < ne) { w2.evm = v.ev_msg[ei + lane]; w2.eax = v.ev_aux[ei + lane]; }
                const Flg f2 = rt3(w2);
                fw0 = w2.fw0; fw1 = w2.fw1; evm = w2.evm; eax = w2.eax; fpid = w2.fpid;
                fflag = f2.fflag; einfo = f2.einfo; fbal = f2.fbal;
            }
            first = false;
            const uint32_t fmsg = (uint32_t)fw1;
            // the window's events that can act:
            // a rejected PREPARE, or a member E_EPOCH that neither deletes nor recreates the
            // node's Acceptor (nor, with rounds, resets its Proposer), changes nothing here
            // — member pairs get every marker of their node, most of them such no-ops
            uint64_t umask = ~0ull;
            if (!SIMPLE) {
                const uint32_t t8l = einfo & 0xFF, fll = einfo >> 8;
                bool u = t8l == MPX_MSG_PREPARE && (fll & F_GRANTED);
                if (MEMBER) u = u || (t8l == MPX_MSG_E_EPOCH && (fll & (ROUNDS ? (F_ACCCLR | F_PRECLR) : F_ACCCLR)));
                if (ROUNDS) u = u || t8l == MPX_MSG_P_START || (t8l == MPX_MSG_PREPARE_REPLY && (fll & F_QUORUM));
                umask = __ballot(lane < ne && u);
            }
            // merge-walk fragments and events by message index
            uint32_t a = 0, c = 0;
            for (;;) {
                if (!SIMPLE) {                            // step over the no-op events
                    const uint64_t r = c < 64 ? umask >> c : 0;
                    c = r ? c + (uint32_t)__builtin_ctzll(r) : ne;
                    if (c > ne) c = ne;
                }
                const bool fmore = a < nf, emore = c < ne;
                if ((!fmore && fi + nf < fe) || (!emore && ei + ne < ee) || (!fmore && !emore)) break;
                const uint32_t fm = fmore ? rl32(fmsg, a) : NONE32;
                const uint32_t em = emore ? rl32(evm, c) : NONE32;
                if (fm <= em) {
                    const uint64_t ent = rl64(fw0, a), w1 = rl64(fw1, a);
                    const uint32_t cnt = (uint32_t)(w1 >> 32) & 0xFFFF, st0 = (uint32_t)(w1 >> 48) & 0xFF;
                    const uint32_t fl = (uint32_t)(w1 >> 56), kind = fl >> 4;
                    const uint32_t mf = rl32(fflag, a);
                    const uint64_t ballot = DIGEST ? rl64(fbal, a) : 0;
                    const bool dense = fl & FR_DENSE;
                    const uint32_t fq = (uint32_t)(fi + a + 1);
                    int k[SPL];
                    frag_slots(lidx, kind == K_PREPLY ? v.r_slot : v.e_slot, ent, cnt, st0, dense, k);
                    if (member && (kind == K_ACCEPT || kind == K_COMMIT)) {
                        // member: accept and learn are std::map::insert — the first
                        // Value and its proposal id stick (member/paxos.cpp:1765,1040);
                        // a learned instance is not accepted (:1763-1769) and a learn
                        // erases the accepted entry (:1786-1793)
                        const bool learn = kind == K_COMMIT;
                        if (learn || (mf & F_GRANTED)) {
                            const uint32_t seq = rl32(fmsg, a) - (uint32_t)v.node_off[n];
                            // the learned-Value check of every slot at once (FR_VEQ: ingest found every
                            // such Value equal — no loads; clamped indices, no branch per slot)
                            uint32_t chk = 0;
                            if (!(fl & FR_VEQ) && (!learn || (mf & F_PROP))) {
#pragma unroll
                                for (uint32_t j = 0; j < SPL; ++j)
                                    chk |= (uint32_t)(k[j] >= 0 && (SF(j) & S_COMMITTED) &&
                                                      se[j] != (uint32_t)(ent + k[j])) << j;
                            }
                            if (__ballot(chk)) {
                                uint64_t va[SPL], vb[SPL];
#pragma unroll
                                for (uint32_t j = 0; j < SPL; ++j) {
                                    const bool c = (chk >> j) & 1;
                                    va[j] = e_val[c ? se[j] : 0];
                                    vb[j] = e_val[c ? (uint32_t)(ent + k[j]) : 0];
                                }
#pragma unroll
                                for (uint32_t j = 0; j < SPL; ++j)
                                    if (((chk >> j) & 1) && va[j] != vb[j])
                                        record_violation(v, MPX_V_LEARN_VALUE, n, seq, v.shard_begin + li0 + lane + 64 * j);
                            }
#pragma unroll
                            for (uint32_t j = 0; j < SPL; ++j) {
                                if (k[j] < 0) continue;
                                const uint32_t x = (uint32_t)(ent + k[j]);
                                if (SF(j) & S_COMMITTED) {
                                    // (checked above)
                                } else if (learn) {
                                    if (DIGEST) sb[j] = v.e_pid[x];
                                    SF_SET(j, S_PRESENT | S_COMMITTED); se[j] = x; sm[j] = fq;
                                } else if (!(SF(j) & S_PRESENT)) {
                                    if (DIGEST) sb[j] = v.e_pid[x];
                                    SF_SET(j, S_PRESENT); se[j] = x; sm[j] = fq;
                                    ++cA;
                                }
                                cL += learn;
                            }
                        }
                    } else if (kind == K_ACCEPT) {
                        if (mf & F_GRANTED) {
#pragma unroll
                            for (uint32_t j = 0; j < SPL; ++j)
                                if (k[j] >= 0 && !(SF(j) & S_COMMITTED)) {           // :1380
                                    if (DIGEST) sb[j] = ballot;                                   // :1387
                                    SF_SET(j, S_PRESENT); se[j] = (uint32_t)(ent + k[j]); sm[j] = fq;
                                    ++cA;
                                }
                        }
                    } else if (kind == K_COMMIT) {
                        // the re-commit Value check (:1508): the slots' two Values loaded together
                        // (clamped indices, no branch per slot: one round trip, not one per slot)
                        uint32_t chk = 0;
#pragma unroll
                        for (uint32_t j = 0; j < SPL; ++j)
                            chk |= (uint32_t)(k[j] >= 0 && (SF(j) & S_COMMITTED) && !(fl & FR_VEQ) &&
                                              se[j] != (uint32_t)(ent + k[j])) << j;
                        if (__ballot(chk)) {
                            uint64_t va[SPL], vb[SPL];
#pragma unroll
                            for (uint32_t j = 0; j < SPL; ++j) {
                                const bool c = (chk >> j) & 1;
                                va[j] = e_val[c ? se[j] : 0];
                                vb[j] = e_val[c ? (uint32_t)(ent + k[j]) : 0];
                            }
#pragma unroll
                            for (uint32_t j = 0; j < SPL; ++j)
                                if (((chk >> j) & 1) && va[j] != vb[j])
                                    record_violation(v, MPX_V_COMMIT_VALUE, n, rl32(fmsg, a) - v.node_off[n],
                                                     v.shard_begin + li0 + lane + 64 * j);
                        }
#pragma unroll
                        for (uint32_t j = 0; j < SPL; ++j)
                            if (k[j] >= 0) {
                                const uint32_t x = (uint32_t)(ent + k[j]);
                                if (SF(j) & S_COMMITTED) {                            // :1508 (checked above)
                                } else {
                                    if (DIGEST) sb[j] = ballot;                                   // :1515
                                    SF_SET(j, S_PRESENT | S_COMMITTED); se[j] = x; sm[j] = fq;
                                }
                                ++cL;
                            }
                    } else if (ROUNDS && kind == K_PREPLY) {
                        if (mf & F_COUNTED) {
                            // the run's proposal ids all in flight, then the merge (loading the next
                            // runs' ids ahead, 1 or 2 deep, measured slower: C3 step 1.366 / 1.452 vs
                            // 1.270 ms — the registers spill; profiles/r04_v12_ab_preply_prefetch.json)
                            uint64_t pid[SPL];
                            if (fl & FR_UPID) {                        // one id for the run, from the window
                                const uint64_t pu = rl64(fpid, a);
#pragma unroll
                                for (uint32_t j = 0; j < SPL; ++j) pid[j] = pu;
                            } else {
#pragma unroll
                                for (uint32_t j = 0; j < SPL; ++j)   // (clamped index, no branch: all in flight)
                                    pid[j] = v.r_pid[ent + (k[j] >= 0 ? k[j] : 0)];
                            }
#pragma unroll
                            for (uint32_t j = 0; j < SPL; ++j)
                                if (k[j] >= 0) {
                                    const u64x2 cur = pre[lane + 64 * j];
                                    if (!cur.y || pid[j] > cur.x) pre[lane + 64 * j] = u64x2{pid[j], W_PRESENT | (ent + k[j])};   // :1216-1221
                                }
                        }
                    }
                    ++a;
                } else if (!SIMPLE) {
                    const uint32_t g = em;
                    const uint32_t info = rl32(einfo, c);
                    const uint32_t t8 = info & 0xFF, fl = info >> 8;
                    if (t8 == MPX_MSG_PREPARE) {
                        bool have = false;
#pragma unroll
                        for (uint32_t j = 0; j < SPL; ++j) have |= (SF(j) & S_PRESENT) != 0;
                        if ((fl & F_GRANTED) && __ballot(have)) {
                            // FilterAcceptedValues over the prepare's ranges (:902-922):
                            // ingest listed which of them meet this bucket (ev_aux, in the
                            // event window: first range | count, or one range's bucket-local
                            // interval inline — then no range loads at all)
                            const uint64_t ax = rl64(eax, c);
                            bool hit[SPL];
                            if (ax & EVX_ONE) {
                                const uint32_t il = (uint32_t)(ax >> 40) & 0x1FF, ih = (uint32_t)(ax >> 49) & 0x1FF;
#pragma unroll
                                for (uint32_t j = 0; j < SPL; ++j) hit[j] = lane + 64 * j >= il && lane + 64 * j < ih;
                            } else {
                                const uint32_t r0 = (uint32_t)ax, nr = (uint32_t)(ax >> 32) & 0xFF;
                                const uint64_t blo = v.shard_begin + li0;
                                uint64_t la = 0, lb = 0;
                                if (lane < nr) { la = v.g_a[r0 + lane]; lb = v.g_b[r0 + lane]; }
#pragma unroll
                                for (uint32_t j = 0; j < SPL; ++j) hit[j] = false;
                                for (uint32_t r = 0; r < nr; ++r) {
                                    const uint64_t ra = rl64(la, r), rb = rl64(lb, r);
#pragma unroll
                                    for (uint32_t j = 0; j < SPL; ++j) {
                                        const uint64_t iid = blo + lane + 64 * j;
                                        hit[j] |= iid >= ra && iid < rb;
                                    }
                                }
                            }
                            uint32_t ref[SPL];
#pragma unroll
                            for (uint32_t j = 0; j < SPL; ++j) {
                                hit[j] = hit[j] && li0 + lane + 64 * j < v.shard_len && (SF(j) & S_PRESENT);
                                ref[j] = sm[j] - 1;                 // the fixing fragment (global)
                                cP += hit[j];
                            }
                            // (one record per slot: run records — OUT_RUN segments — measured slower,
                            // 1.015 vs 0.992 ms C3 general apply, profiles/r04_v5_ab_snap_runs.json)
                            EMIT(hit, g, 0, ref);
                        }
                    } else if (!ROUNDS) {
                        // AM_SNAP: a pair without promise-reply runs gets no round events; member:
                        // an E_EPOCH that deletes / recreates the Acceptor still clears it (below)
                        if (MEMBER && t8 == MPX_MSG_E_EPOCH && (fl & F_ACCCLR)) {
#pragma unroll
                            for (uint32_t j = 0; j < SPL; ++j)
                                if (!(SF(j) & S_COMMITTED)) { if (DIGEST) sb[j] = 0; SF_SET(j, 0); se[j] = sm[j] = 0; }
                        }
                    } else if (t8 == MPX_MSG_P_START || (t8 == MPX_MSG_E_EPOCH && (fl & F_PRECLR))) {
#pragma unroll
                        for (uint32_t j = 0; j < SPL; ++j) pre[lane + 64 * j] = u64x2{0, 0};
                        if (t8 == MPX_MSG_E_EPOCH && (fl & F_ACCCLR)) {
#pragma unroll
                            for (uint32_t j = 0; j < SPL; ++j)
                                if (!(SF(j) & S_COMMITTED)) { if (DIGEST) sb[j] = 0; SF_SET(j, 0); se[j] = sm[j] = 0; }
                        }
                    } else if (t8 == MPX_MSG_E_EPOCH && (fl & F_ACCCLR)) {
                        // the Acceptor is deleted / recreated: its accepted values go
                        // (member/paxos.cpp:1952-1957); learned ones stay with the Learner
#pragma unroll
                        for (uint32_t j = 0; j < SPL; ++j)
                            if (!(SF(j) & S_COMMITTED)) { if (DIGEST) sb[j] = 0; SF_SET(j, 0); se[j] = sm[j] = 0; }
                    } else if (t8 == MPX_MSG_PREPARE_REPLY && (fl & F_QUORUM)) {
                        bool hit[SPL];
                        uint32_t ref[SPL], ext[SPL];
#pragma unroll
                        for (uint32_t j = 0; j < SPL; ++j) {
                            const u64x2 cur = pre[lane + 64 * j];
                            hit[j] = li0 + lane + 64 * j < v.shard_len && cur.y;
                            ref[j] = (uint32_t)(cur.y & ~W_PRESENT);                 // the PREPARE_REPLY entry
                            ext[j] = (SF(j) & S_COMMITTED) ? OUT_CMT : 0;            // not adoptable (:1091)
                            cQ += hit[j];
                            pre[lane + 64 * j] = u64x2{0, 0};                        // :1105
                        }
                        // the merged map leaves as run records: consecutive slots whose entries are
                        // consecutive (one reply run) with the same OUT_CMT bit are one record
                        // (OUT_RUN: slot, length; the host expands entry ref + i to slot + i)
                        bool cont[SPL];
                        uint64_t cm[SPL];
#pragma unroll
                        for (uint32_t j = 0; j < SPL; ++j) {
                            uint32_t pr = __shfl_up(ref[j], 1, 64), pe = __shfl_up(ext[j], 1, 64);
                            int ph = __shfl_up((int)hit[j], 1, 64);
                            if (j) {                                                 // lane 0: the previous strip's lane 63
                                const uint32_t r63 = __shfl(ref[j - 1], 63, 64), e63 = __shfl(ext[j - 1], 63, 64);
                                const int h63 = __shfl((int)hit[j - 1], 63, 64);
                                if (lane == 0) { pr = r63; pe = e63; ph = h63; }
                            } else if (lane == 0) {
                                ph = 0;
                            }
                            cont[j] = hit[j] && ph && pr + 1 == ref[j] && pe == ext[j];
                            cm[j] = __ballot(cont[j]);
                        }
                        bool start[SPL];
                        uint32_t ext2[SPL];
#pragma unroll
                        for (uint32_t j = 0; j < SPL; ++j) {
                            start[j] = hit[j] && !cont[j];
                            uint32_t len = 1;
                            if (start[j]) {
                                uint32_t p = lane + 64 * j + 1;                      // count the continuation bits after it
                                while (p < BS) {
                                    // (the word by an unrolled select, not cm[p >> 6]: a run-time index
                                    // would put cm in scratch)
                                    uint64_t cw = 0;
#pragma unroll
                                    for (uint32_t jj = 0; jj < SPL; ++jj)
                                        if (jj == (p >> 6)) cw = cm[jj];
                                    const uint64_t w = cw >> (p & 63);
                                    const uint32_t room = 64 - (p & 63);
                                    const uint32_t ones = ~w ? (uint32_t)__builtin_ctzll(~w) : 64;
                                    const uint32_t take = ones < room ? ones : room;
                                    len += take;
                                    if (take < room) break;
                                    p += take;
                                }
                            }
                            ext2[j] = ext[j] | OUT_RUN | (len << OUT_RUN_SHIFT);
                        }
                        EMIT(start, g, OUT_K1, ref, ext2);
                    }
                    ++c;
                }
            }
            fi += a;
            ei += c;
        }
        bool have = false;
#pragma unroll
        for (uint32_t j = 0; j < SPL; ++j) have |= SF(j) != 0;
        if (__ballot(have)) {
#pragma unroll
            for (uint32_t j = 0; j < SPL; ++j) {
                const uint64_t li = li0 + lane + 64 * j;
                if (li < v.shard_len) st_put(v, (uint64_t)n * v.shard_len + li, sm[j] ? (uint32_t)(sm[j] - pbase) : 0);
                if (DIGEST && SF(j))
                    dig += state_digest(n, v.shard_begin + li, (SF(j) & S_COMMITTED) ? 2 : 1, sb[DIGEST ? j : 0], e_val[se[j]]);
            }
            if (lane == 0) v.st_valid[sv_idx(v, n, b)] = 1;
        }
    }
#undef EMIT
    // workgroup reduction of the counters
    unsigned long long cc[5] = {cA, cL, cP, cQ, dig};
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        unsigned long long x = cc[i];
        for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
        cc[i] = x;
    }
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < 5; ++i) red[wv][i] = cc[i];
    }
    __syncthreads();
    if (threadIdx.x < 5) {
        const uint32_t t = threadIdx.x;
        unsigned long long s = red[0][t] + red[1][t] + red[2][t] + red[3][t];
        const int slot = t == 0 ? PC_A : t == 1 ? PC_L : t == 2 ? PC_P : t == 3 ? PC_Q : PC_DSTATE;
        if (s) atomicAdd(&v.partials[8 * blockIdx.x + slot], s);   // (the rounds launch may run beside the listed pairs')
    }
#undef SF
#undef SF_SET
}

// ------------------------------------------------------------ windows ----
// Incremental runs (MPX_FLAG_INCREMENTAL).  The trace
// arrays hold one window of records; what the windows before left is carried as values:
// the acceptor / learner state (s_bal, s_val), a promise round's pre-accepted map (p_pid,
// p_val, tagged per pair with its round's ballot), the chosen log (c_val), the scalars and
// rounds (scal_base, prop_in) and the batches' votes (g_mask, g_done).

// Snapshot records with their values (OutEnt): lane l's slot j is emitted when want[j];
// one append per event (a wave-wide atomic on the window cursor).
__device__ inline void emit_vals(const DevView &v, const bool (&want)[SPL_], uint32_t msg, uint32_t kind,
                                 uint64_t iid0, const uint64_t (&bal)[SPL_], const uint64_t (&val)[SPL_],
                                 const uint32_t (&kx)[SPL_])
{
    const uint32_t lane = threadIdx.x & 63;
    uint64_t m[SPL_];
    uint32_t tot = 0;
#pragma unroll
    for (uint32_t j = 0; j < SPL_; ++j) { m[j] = __ballot(want[j]); tot += (uint32_t)__popcll(m[j]); }
    if (!tot) return;
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(v.outv_n, (unsigned long long)tot);
    base = __shfl(base, 0, 64);
    const uint64_t below = (1ull << lane) - 1;
    uint32_t off = 0;
#pragma unroll
    for (uint32_t j = 0; j < SPL_; ++j) {
        const uint64_t at = base + off + (uint64_t)__popcll(m[j] & below);
        if (want[j] && at < v.outv_cap) {
            OutEnt r;
            r.msg = msg; r.kind = kind | kx[j]; r.iid = iid0 + lane + 64 * j; r.ballot = bal[j]; r.handle = val[j] & W_HANDLE;
            v.outv[at] = r;
        }
        off += (uint32_t)__popcll(m[j]);
    }
}

// Window apply: one wave per work-list pair of the window (every pair with runs or events
// in it), 4 slots per lane.  The pair's runs and events are merge-walked in message order
// with k_apply's semantics — OnPrepare's FilterAcceptedValues (multi/paxos.cpp:902-922),
// OnAccept (:1359-1404: a granted ACCEPT overwrites what is not committed), OnCommit
// (:1494-1518: the first COMMIT fixes the slot, a later one must carry its Value),
// UpdateByPreAcceptedValues (:1201-1223: the highest proposal id wins, first arrival on
// ties), the quorum's merged map (:1047-1105) and StartPrepare's clear (:1233-1248) —
// but the slot state is {ballot, handle | flags} itself, started from what earlier
// windows left and written back at the end.  MEMBER: the member Acceptor / Learner
// (member/paxos.cpp:1744-1793, 1029-1060) — accept and learn insert (the first Value and
// its proposal id stick), a learned instance takes no accept (its Value must agree), a
// learn replaces the accepted entry, and an E_EPOCH marker that deletes / recreates the
// node's Acceptor clears what it accepted (:1952-1957) or, resetting its Proposer, the
// pre-accepted map (the flags k_gate_epochs wrote from the carried roles).
template <bool MEMBER>
__global__ __launch_bounds__(256) void k_apply_win(DevView v)
{
    __shared__ uint16_t lidx_all[4][BS];
    __shared__ u64x2 pre_all[4][BS];
    __shared__ unsigned long long red[4][4];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint16_t *lidx = lidx_all[wv];
    u64x2 *pre = pre_all[wv];
#pragma unroll
    for (uint32_t j = 0; j < SPL; ++j) lidx[lane + 64 * j] = 0xFFFF;
    wave_lds_fence();
    uint32_t cA = 0, cL = 0, cP = 0, cQ = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 4;
    for (uint64_t it = (uint64_t)blockIdx.x * 4 + wv; it < v.num_gp; it += stride) {
        const uint64_t w = lane < 5 ? v.gp_list[GP_WORDS * it + lane] : 0;
        uint64_t fi = rl64(w, 0), ei = rl64(w, 2);
        const uint64_t fe = rl64(w, 1), ee = rl64(w, 3), q = rl64(w, 4);
        const uint32_t b = (uint32_t)(q / v.N), n = (uint32_t)(q - (uint64_t)b * v.N);
        const uint64_t li0 = (uint64_t)b << BSH, row = (uint64_t)n * v.shard_len;
        const bool base = v.gp_base[it] != 0;
        // a promise round that spans windows: its pre-accepted map, if this pair's is the round's
        const uint64_t pr = v.p_round[sv_idx(v, n, b)];
        const bool pload = pr && v.prop_in[3 * n + 2] && pr == v.prop_in[3 * n];
        uint64_t sbal[SPL], sval[SPL];
#pragma unroll
        for (uint32_t j = 0; j < SPL; ++j) {
            const uint64_t li = li0 + lane + 64 * j;
            const bool in = li < v.shard_len;
            sbal[j] = base && in ? v.s_bal[row + li] : 0;
            sval[j] = base && in ? v.s_val[row + li] : 0;
            pre[lane + 64 * j] = pload && in ? u64x2{v.p_pid[row + li], v.p_val[row + li]} : u64x2{0, 0};
        }
        while (fi < fe || ei < ee) {
            const uint32_t nf = (uint32_t)(fe - fi < 64 ? fe - fi : 64);
            const uint32_t ne = (uint32_t)(ee - ei < 64 ? ee - ei : 64);
            uint64_t fw0 = 0, fw1 = NONE32, eax = 0, fbal = 0;
            uint32_t evm = NONE32, fflag = 0, einfo = 0;
            if (lane < nf) {
                const ulonglong2 x = *reinterpret_cast<const ulonglong2 *>(v.frags + fi + lane);
                fw0 = x.x; fw1 = x.y;
            }
            if (lane < ne) { evm = v.ev_msg[ei + lane]; eax = v.ev_aux[ei + lane]; }
            if (lane < nf) { fflag = v.m_flags[(uint32_t)fw1]; fbal = v.m_ballot[(uint32_t)fw1]; }
            if (lane < ne) einfo = (uint32_t)v.m_type[evm] | ((uint32_t)v.m_flags[evm] << 8);
            const uint32_t fmsg = (uint32_t)fw1;
            uint32_t a = 0, c = 0;
            for (;;) {
                const bool fmore = a < nf, emore = c < ne;
                if ((!fmore && fi + nf < fe) || (!emore && ei + ne < ee) || (!fmore && !emore)) break;
                const uint32_t fm = fmore ? rl32(fmsg, a) : NONE32;
                const uint32_t em = emore ? rl32(evm, c) : NONE32;
                if (fm <= em) {
                    const uint64_t ent = rl64(fw0, a), w1 = rl64(fw1, a);
                    const uint32_t cnt = (uint32_t)(w1 >> 32) & 0xFFFF, st0 = (uint32_t)(w1 >> 48) & 0xFF;
                    const uint32_t fl = (uint32_t)(w1 >> 56), kind = fl >> 4;
                    const uint32_t mf = rl32(fflag, a);
                    const uint64_t ballot = rl64(fbal, a);
                    int k[SPL];
                    frag_slots(lidx, kind == K_PREPLY ? v.r_slot : v.e_slot, ent, cnt, st0, (fl & FR_DENSE) != 0, k);
                    if (MEMBER && (kind == K_ACCEPT || kind == K_COMMIT)) {
                        const bool learn = kind == K_COMMIT;
                        if (learn || (mf & F_GRANTED)) {
                            uint64_t pid[SPL], hv[SPL];
#pragma unroll
                            for (uint32_t j = 0; j < SPL; ++j) {   // (clamped, no branch: all in flight)
                                pid[j] = v.e_pid[ent + (k[j] >= 0 ? k[j] : 0)];
                                hv[j] = v.e_val[ent + (k[j] >= 0 ? k[j] : 0)];
                            }
#pragma unroll
                            for (uint32_t j = 0; j < SPL; ++j) {
                                if (k[j] < 0) continue;
                                if (sval[j] & W_COMMITTED) {                                  // :1763-1769, :1398
                                    if ((sval[j] & W_HANDLE) != hv[j] && (!learn || (mf & F_PROP)))
                                        record_violation(v, MPX_V_LEARN_VALUE, n, rl32(fmsg, a) - (uint32_t)v.node_off[n],
                                                         v.shard_begin + li0 + lane + 64 * j);
                                } else if (learn) {                                           // :1040, :1786-1793
                                    sbal[j] = pid[j]; sval[j] = W_PRESENT | W_COMMITTED | hv[j];
                                } else if (!(sval[j] & W_PRESENT)) {                          // :1765 insert
                                    sbal[j] = pid[j]; sval[j] = W_PRESENT | hv[j];
                                    ++cA;
                                }
                                cL += learn;
                            }
                        }
                    } else if (kind == K_ACCEPT) {
                        if (mf & F_GRANTED) {
                            uint64_t hv[SPL];
#pragma unroll
                            for (uint32_t j = 0; j < SPL; ++j) hv[j] = v.e_val[ent + (k[j] >= 0 ? k[j] : 0)];
#pragma unroll
                            for (uint32_t j = 0; j < SPL; ++j)
                                if (k[j] >= 0 && !(sval[j] & W_COMMITTED)) {                  // :1380
                                    sbal[j] = ballot; sval[j] = W_PRESENT | hv[j];             // :1387
                                    ++cA;
                                }
                        }
                    } else if (kind == K_COMMIT) {
                        uint64_t hv[SPL];
#pragma unroll
                        for (uint32_t j = 0; j < SPL; ++j) hv[j] = v.e_val[ent + (k[j] >= 0 ? k[j] : 0)];
#pragma unroll
                        for (uint32_t j = 0; j < SPL; ++j)
                            if (k[j] >= 0) {
                                const uint64_t x = hv[j];
                                if (sval[j] & W_COMMITTED) {                                  // :1508
                                    if ((sval[j] & W_HANDLE) != x)
                                        record_violation(v, MPX_V_COMMIT_VALUE, n, rl32(fmsg, a) - v.node_off[n],
                                                         v.shard_begin + li0 + lane + 64 * j);
                                } else {
                                    sbal[j] = ballot; sval[j] = W_PRESENT | W_COMMITTED | x;   // :1515
                                }
                                ++cL;
                            }
                    } else if (kind == K_PREPLY && (mf & F_COUNTED)) {
                        uint64_t pid[SPL], hv[SPL];
#pragma unroll
                        for (uint32_t j = 0; j < SPL; ++j) {
                            pid[j] = v.r_pid[ent + (k[j] >= 0 ? k[j] : 0)];
                            hv[j] = v.r_val[ent + (k[j] >= 0 ? k[j] : 0)];
                        }
#pragma unroll
                        for (uint32_t j = 0; j < SPL; ++j)
                            if (k[j] >= 0) {
                                const u64x2 cur = pre[lane + 64 * j];
                                if (!cur.y || pid[j] > cur.x) pre[lane + 64 * j] = u64x2{pid[j], W_PRESENT | hv[j]};   // :1216-1221
                            }
                    }
                    ++a;
                } else {
                    const uint32_t g = em;
                    const uint32_t info = rl32(einfo, c);
                    const uint32_t t8 = info & 0xFF, fl = info >> 8;
                    bool hit[SPL];
                    uint64_t hb[SPL], hvv[SPL];
                    uint32_t kx[SPL];
                    if (t8 == MPX_MSG_PREPARE) {
                        bool have = false;
#pragma unroll
                        for (uint32_t j = 0; j < SPL; ++j) have |= (sval[j] & W_PRESENT) != 0;
                        if ((fl & F_GRANTED) && __ballot(have)) {
                            const uint64_t ax = rl64(eax, c);
                            if (ax & EVX_ONE) {
                                const uint32_t il = (uint32_t)(ax >> 40) & 0x1FF, ih = (uint32_t)(ax >> 49) & 0x1FF;
#pragma unroll
                                for (uint32_t j = 0; j < SPL; ++j) hit[j] = lane + 64 * j >= il && lane + 64 * j < ih;
                            } else {
                                const uint32_t r0 = (uint32_t)ax, nr = (uint32_t)(ax >> 32) & 0xFF;
                                const uint64_t blo = v.shard_begin + li0;
                                uint64_t la = 0, lb = 0;
                                if (lane < nr) { la = v.g_a[r0 + lane]; lb = v.g_b[r0 + lane]; }
#pragma unroll
                                for (uint32_t j = 0; j < SPL; ++j) hit[j] = false;
                                for (uint32_t r = 0; r < nr; ++r) {
                                    const uint64_t ra = rl64(la, r), rb = rl64(lb, r);
#pragma unroll
                                    for (uint32_t j = 0; j < SPL; ++j) {
                                        const uint64_t iid = blo + lane + 64 * j;
                                        hit[j] |= iid >= ra && iid < rb;
                                    }
                                }
                            }
#pragma unroll
                            for (uint32_t j = 0; j < SPL; ++j) {
                                hit[j] = hit[j] && li0 + lane + 64 * j < v.shard_len && (sval[j] & W_PRESENT);
                                kx[j] = 0;
                                cP += hit[j];
                            }
                            emit_vals(v, hit, g, 0, v.shard_begin + li0, sbal, sval, kx);
                        }
                    } else if (t8 == MPX_MSG_P_START || (MEMBER && t8 == MPX_MSG_E_EPOCH && (fl & F_PRECLR))) {
#pragma unroll
                        for (uint32_t j = 0; j < SPL; ++j) pre[lane + 64 * j] = u64x2{0, 0};
                        if (MEMBER && t8 == MPX_MSG_E_EPOCH && (fl & F_ACCCLR)) {
#pragma unroll
                            for (uint32_t j = 0; j < SPL; ++j)
                                if (!(sval[j] & W_COMMITTED)) { sbal[j] = 0; sval[j] = 0; }
                        }
                    } else if (MEMBER && t8 == MPX_MSG_E_EPOCH && (fl & F_ACCCLR)) {
                        // the Acceptor is deleted / recreated: its accepted values go
                        // (member/paxos.cpp:1952-1957); learned ones stay with the Learner
#pragma unroll
                        for (uint32_t j = 0; j < SPL; ++j)
                            if (!(sval[j] & W_COMMITTED)) { sbal[j] = 0; sval[j] = 0; }
                    } else if (t8 == MPX_MSG_PREPARE_REPLY && (fl & F_QUORUM)) {
#pragma unroll
                        for (uint32_t j = 0; j < SPL; ++j) {
                            const u64x2 cur = pre[lane + 64 * j];
                            hit[j] = li0 + lane + 64 * j < v.shard_len && cur.y;
                            hb[j] = cur.x; hvv[j] = cur.y;
                            kx[j] = (sval[j] & W_COMMITTED) ? 2u : 0u;                         // not adoptable (:1091)
                            cQ += hit[j];
                            pre[lane + 64 * j] = u64x2{0, 0};                                  // :1105
                        }
                        emit_vals(v, hit, g, 1, v.shard_begin + li0, hb, hvv, kx);
                    }
                    ++c;
                }
            }
            fi += a;
            ei += c;
        }
        // what the next window starts from: the slots, and the pre-accepted map of a round
        // still preparing after this window (tagged with its ballot)
        const bool psave = v.prop_out[3 * n + 2] != 0;
#pragma unroll
        for (uint32_t j = 0; j < SPL; ++j) {
            const uint64_t li = li0 + lane + 64 * j;
            if (li >= v.shard_len) continue;
            v.s_bal[row + li] = sbal[j];
            v.s_val[row + li] = sval[j];
            if (psave) {
                const u64x2 cur = pre[lane + 64 * j];
                v.p_pid[row + li] = cur.x;
                v.p_val[row + li] = cur.y;
            }
        }
        if (lane == 0) v.p_round[sv_idx(v, n, b)] = psave ? v.prop_out[3 * n] : 0;
    }
    unsigned long long cc[4] = {cA, cL, cP, cQ};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        unsigned long long x = cc[i];
        for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
        cc[i] = x;
    }
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < 4; ++i) red[wv][i] = cc[i];
    __syncthreads();
    if (threadIdx.x < 4) {
        const uint32_t t = threadIdx.x;
        const int slot = t == 0 ? PC_A : t == 1 ? PC_L : t == 2 ? PC_P : PC_Q;
        v.partials[8 * blockIdx.x + slot] += red[0][t] + red[1][t] + red[2][t] + red[3][t];
    }
}

// Window chosen log: one wave per bucket with chosen-log runs in the window; the runs of
// batches whose votes reached quorum in this window (k_votes) write their Values where the
// log is empty (OnAcceptReply -> Commit, multi/paxos.cpp:1416-1421), and must agree where
// it is not (safety).  C counts the instances first chosen here.
__global__ __launch_bounds__(256) void k_chosen_win(DevView v, uint32_t partial_base)
{
    __shared__ uint16_t lidx_all[4][BS];
    __shared__ unsigned long long red[4];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint16_t *lidx = lidx_all[wv];
#pragma unroll
    for (uint32_t j = 0; j < SPL; ++j) lidx[lane + 64 * j] = 0xFFFF;
    wave_lds_fence();
    unsigned long long cC = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 4;
    for (uint64_t it = (uint64_t)blockIdx.x * 4 + wv; it < v.num_cb; it += stride) {
        const uint64_t b = v.cb_list[it], li0 = b << BSH;
        const uint64_t off = lane < 2 ? v.cf_off[b + lane] : 0;
        uint64_t fi = rl64(off, 0);
        const uint64_t fe = rl64(off, 1);
        uint64_t cv[SPL];
        bool had[SPL];
#pragma unroll
        for (uint32_t j = 0; j < SPL; ++j) {
            const uint64_t li = li0 + lane + 64 * j;
            cv[j] = li < v.shard_len ? v.c_val[li] : 0;
            had[j] = (cv[j] & W_PRESENT) != 0;
        }
        while (fi < fe) {
            const uint32_t nf = (uint32_t)(fe - fi < 64 ? fe - fi : 64);
            uint64_t fw0 = 0, fw1 = 0;
            uint32_t live = 0;
            if (lane < nf) {
                const ulonglong2 x = *reinterpret_cast<const ulonglong2 *>(v.cfrags + fi + lane);
                fw0 = x.x; fw1 = x.y;
                live = v.b_chosen[(uint32_t)fw1] != NONE32;
            }
            uint64_t lm = __ballot(live);
            while (lm) {
                const uint32_t a = (uint32_t)__builtin_ctzll(lm);
                lm &= lm - 1;
                const uint64_t ent = rl64(fw0, a), w1 = rl64(fw1, a);
                const uint32_t cnt = (uint32_t)(w1 >> 32) & 0xFFFF, st0 = (uint32_t)(w1 >> 48) & 0xFF;
                int k[SPL];
                frag_slots(lidx, v.e_slot, ent, cnt, st0, ((w1 >> 56) & FR_DENSE) != 0, k);
#pragma unroll
                for (uint32_t j = 0; j < SPL; ++j) {
                    if (k[j] < 0) continue;
                    const uint64_t x = v.e_val[ent + k[j]];
                    if (!(cv[j] & W_PRESENT)) cv[j] = W_PRESENT | x;
                    else if ((cv[j] & W_HANDLE) != x)
                        record_violation(v, MPX_V_CHOSEN_VALUE, 0, 0, v.shard_begin + li0 + lane + 64 * j);
                }
            }
            fi += nf;
        }
#pragma unroll
        for (uint32_t j = 0; j < SPL; ++j) {
            const uint64_t li = li0 + lane + 64 * j;
            if (li < v.shard_len && !had[j] && (cv[j] & W_PRESENT)) { v.c_val[li] = cv[j]; ++cC; }
        }
    }
    for (int d = 32; d >= 1; d >>= 1) cC += __shfl_xor(cC, d, 64);
    if (lane == 0) red[wv] = cC;
    __syncthreads();
    if (threadIdx.x == 0) v.partials[8 * (partial_base + blockIdx.x) + PC_C] = red[0] + red[1] + red[2] + red[3];
}

// Digests of the carried state (mpx_state_digest in incremental mode): the same
// definitions as the batch engine's (mpx_internal.hpp state_digest / chosen_digest)
__global__ __launch_bounds__(256) void k_state_digest_win(DevView v, unsigned long long *out)
{
    const uint64_t total = (uint64_t)(v.N + 1) * v.shard_len;
    unsigned long long ds = 0, dc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (uint64_t)gridDim.x * 256) {
        const uint32_t row = (uint32_t)(i / v.shard_len);
        const uint64_t li = i - (uint64_t)row * v.shard_len;
        const uint64_t iid = v.shard_begin + li;
        if (row < v.N) {
            const uint64_t x = v.s_val[i];
            if (x & W_PRESENT) ds += state_digest(row, iid, (x & W_COMMITTED) ? 2 : 1, v.s_bal[i], x & W_HANDLE);
        } else {
            const uint64_t x = v.c_val[li];
            if (x & W_PRESENT) dc += chosen_digest(iid, x & W_HANDLE);
        }
    }
    for (int d = 32; d >= 1; d >>= 1) { ds += __shfl_xor(ds, d, 64); dc += __shfl_xor(dc, d, 64); }
    if ((threadIdx.x & 63) == 0) {
        if (ds) atomicAdd(&out[0], ds);
        if (dc) atomicAdd(&out[1], dc);
    }
}

// The step's summary (mpx_allgather_summary's 64 words) from every workgroup's
// partial counters: this workgroup (64 W threads) sums the partial rows row0, row0 + stride,
// ... into the summary's counter words (zeroed by reset_state; integer sums, so the order of
// the workgroups' atomics does not matter); SCAL: it also writes the node scalars' words
template <uint32_t W>
__device__ inline void reduce_summary(const DevView &v, uint32_t n_partials, unsigned long long (&red)[W][8],
                                      uint32_t row0, uint32_t stride, bool scal)
{
    // each partial row is 64 bytes, read as four 16-byte loads
    const uint32_t t = threadIdx.x;
    unsigned long long s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const u64x2 *p2 = reinterpret_cast<const u64x2 *>(v.partials);
#pragma unroll 1
    for (uint32_t w = row0 + t; w < n_partials; w += stride) {
        u64x2 x[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = __builtin_nontemporal_load(&p2[4 * (uint64_t)w + i]);
#pragma unroll
        for (int i = 0; i < 4; ++i) { s[2 * i] += x[i].x; s[2 * i + 1] += x[i].y; }
    }
#pragma unroll 1
    for (int i = 0; i < 8; ++i) {
        unsigned long long x = s[i];
        for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
        if ((t & 63) == 0) red[t >> 6][i] = x;
    }
    // the per-node scalars, one lane per node (N <= 64): their loads all in flight at once
    // (a serial loop over the nodes in one thread waited out N memory latencies)
    unsigned long long *o = v.summary;
    if (scal && t < 64) {
        unsigned long long ds = 0;
        if (t < v.N) {
            const uint64_t p = v.node_scal[2 * t], m = v.node_scal[2 * t + 1];
            ds = scalar_digest(t, p, m);
            if (t < 24) { o[SW_NODE_SCAL + 2 * t] = p; o[SW_NODE_SCAL + 2 * t + 1] = m; }
        }
        for (int d = 32; d >= 1; d >>= 1) ds += __shfl_xor(ds, d, 64);
        if (t == 0) { o[SW_DSCAL] = ds; o[SW_MSGS] = v.num_msgs; o[SW_V] = v.viol->count; }
    }
    __syncthreads();
    if (t < 8) {
        unsigned long long r = 0;
        for (uint32_t k = 0; k < W; ++k) r += red[k][t];
        const int w = summary_word(t);
        if (w >= 0 && r) atomicAdd(&o[w], r);
    }
}

// Chosen log, one wave per bucket, for the buckets k_apply_fast did not
// write from registers (multi) or every bucket (member: chosen_valid is 0).
// (Folding the summary into its last workgroup was measured slower: every workgroup's
// device-scope fence writes back its XCD's L2 before the ticket; C4 tail 75 vs 15 us.)
__global__ __launch_bounds__(256) void k_chosen(DevView v, uint32_t partial_base)
{
    __shared__ uint16_t lidx_all[4][BS];
    __shared__ unsigned long long red[4][8];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint16_t *lidx = lidx_all[wv];
#pragma unroll
    for (uint32_t j = 0; j < SPL; ++j) lidx[lane + 64 * j] = 0xFFFF;
    wave_lds_fence();
    unsigned long long cC = 0, dig = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 4;
    // 64 buckets per wave step, strided by the wave count (b = base + lane *
    // stride) so the walks spread over every wave even when few buckets need
    // one: one lane-parallel load of their chosen_valid bytes, then a walk of
    // only the buckets k_plan / k_apply_fast left
    for (uint64_t base = xcd_wave_id(wv); base < v.NB; base += 64 * stride) {
        const uint64_t bl = base + (uint64_t)lane * stride;
        uint64_t todo = __ballot(bl < v.NB && !v.chosen_valid[bl]);
        while (todo) {
            const uint32_t i = (uint32_t)__builtin_ctzll(todo);
            todo &= todo - 1;
            chosen_walk(v, base + (uint64_t)i * stride, lidx, cC, dig);
        }
    }
    unsigned long long cc[2] = {cC, dig};
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        unsigned long long x = cc[i];
        for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
        cc[i] = x;
    }
    if (lane == 0) { red[wv][0] = cc[0]; red[wv][1] = cc[1]; }
    __syncthreads();
    if (threadIdx.x < 2) {
        const uint32_t t = threadIdx.x;
        unsigned long long s = red[0][t] + red[1][t] + red[2][t] + red[3][t];
        v.partials[8 * (partial_base + blockIdx.x) + (t == 0 ? PC_C : PC_DCHOSEN)] = s;
    }
}

// the summary pass: one partial row per thread, every row's loads in flight at once over cdiv(rows, 256) workgroups
// (one workgroup of 512 threads looping over the rows waited out six memory latencies in turn:
// 10.7 us at the C4 shard)
__global__ __launch_bounds__(256) void k_reduce(DevView v, uint32_t n_partials)
{
    __shared__ unsigned long long red[4][8];
    reduce_summary<4>(v, n_partials, red, 256 * blockIdx.x, 256 * gridDim.x, blockIdx.x == 0);
}

__global__ void k_reset(DevView v, uint32_t n_partials)
{
    reset_state(v, n_partials, (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, (uint64_t)gridDim.x * blockDim.x);
}

static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

// Readback (mpx_read_node_state / mpx_read_chosen / mpx_dump_result): slots of
// one node, or the chosen log (node >= N), to {ballot, word} pairs
__global__ __launch_bounds__(256) void k_decode(DevView v, uint32_t node, uint64_t l0, uint64_t count, uint64_t *out)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    const uint64_t li = l0 + i;
    uint64_t b = 0, w = 0;
    if (node >= v.N) {
        const uint32_t c = v.chosen_valid[li >> BSH] ? st_get(v, (uint64_t)v.N * v.shard_len + li) : 0;
        if (c) {
            // the bucket's chosen fragment c - 1 and its entry at this slot
            const Frag f = v.cfrags[v.cf_off[li >> BSH] + c - 1];
            const uint32_t sl = (uint32_t)li & (BS - 1);
            uint64_t ent = f.entry + (sl - f.start);
            if (!(f.flags & FR_DENSE))
                for (uint32_t k = 0; k < f.count; ++k)
                    if (v.e_slot[f.entry + k] == sl) { ent = f.entry + k; break; }
            w = W_PRESENT | v.e_val[ent];
        }
    } else if (v.st_valid[sv_idx(v, node, li >> BSH)]) {
        decode_slot(v, slot_global(v, node, li), (uint32_t)li & (BS - 1), b, w);
    }
    out[2 * i] = b;
    out[2 * i + 1] = w;
}

// Order-independent digests of the state the last run / step left in HBM
// (mpx_state_digest): every (node, instance) slot decoded as k_decode does,
// plus the chosen log.  The timed step carries no digest code; this pass
// verifies what its kernels (k_plan + k_store8, or k_apply) wrote, at any size.
__global__ __launch_bounds__(256) void k_state_digest(DevView v, unsigned long long *out)
{
    const uint64_t total = (uint64_t)(v.N + 1) * v.shard_len;
    unsigned long long ds = 0, dc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (uint64_t)gridDim.x * 256) {
        const uint32_t row = (uint32_t)(i / v.shard_len);
        const uint64_t li = i - (uint64_t)row * v.shard_len;
        const uint64_t iid = v.shard_begin + li;
        if (row < v.N) {
            if (v.st_valid[sv_idx(v, row, li >> BSH)]) ds += slot_digest(v, row, iid, slot_global(v, row, li));
        } else if (v.chosen_valid[li >> BSH]) {
            const uint32_t c = st_get(v, (uint64_t)v.N * v.shard_len + li);
            if (c) {
                const Frag f = v.cfrags[v.cf_off[li >> BSH] + c - 1];
                const uint32_t sl = (uint32_t)li & (BS - 1);
                uint64_t ent = f.entry + (sl - f.start);
                if (!(f.flags & FR_DENSE))
                    for (uint32_t k = 0; k < f.count; ++k)
                        if (v.e_slot[f.entry + k] == sl) { ent = f.entry + k; break; }
                dc += chosen_digest(iid, v.e_val[ent]);
            }
        }
    }
    for (int d = 32; d >= 1; d >>= 1) { ds += __shfl_xor(ds, d, 64); dc += __shfl_xor(dc, d, 64); }
    if ((threadIdx.x & 63) == 0) {
        if (ds) atomicAdd(&out[0], ds);
        if (dc) atomicAdd(&out[1], dc);
    }
}

int launch_state_digest(const DevView &v, void *stream, unsigned long long *out)
{
    const uint64_t total = (uint64_t)(v.N + 1) * v.shard_len;
    const uint64_t blocks = total / 256 + 1 < 16384 ? total / 256 + 1 : 16384;
    if (hipMemsetAsync(out, 0, 16, (hipStream_t)stream) != hipSuccess) return -1;
    if (v.window) {
        hipLaunchKernelGGL(k_state_digest_win, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, v, out);
        return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(k_state_digest, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, v, out);
    return (int)hipGetLastError();
}

// ---- in-order executor: multi/paxos.cpp:1584-1622 applies
// next_id_to_apply_ forward while the instance is committed, skipping noops
// (:1601-1606); member/paxos.cpp:1042-1053 the same over learned_.  On the GPU
// the frontier is the first shard slot of the node that is not committed (a
// min-reduction), and the executed Values are the non-noop handles below it,
// compacted in instance order by a count / scan / scatter over buckets.
// aux layout: [0] frontier, [1 .. NB] bucket counts, [NB + 1 .. 2 NB + 1] offsets
__device__ inline uint64_t exec_word(const DevView &v, uint32_t node, uint64_t li)
{
    if (!v.st_valid[sv_idx(v, node, li >> BSH)]) return 0;
    uint64_t b, w;
    decode_slot(v, slot_global(v, node, li), (uint32_t)li & (BS - 1), b, w);
    return w;
}

__global__ __launch_bounds__(256) void k_exec_frontier(DevView v, uint32_t node, unsigned long long *aux)
{
    const uint64_t li = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const bool gap = li < v.shard_len && !(exec_word(v, node, li) & W_COMMITTED);
    const uint64_t m = __ballot(gap);
    if (m && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(m)) atomicMin(&aux[0], (unsigned long long)li);
}

// one workgroup per bucket: executed slots (below the frontier, not a noop)
__device__ inline bool exec_take(const DevView &v, uint32_t node, uint64_t li, uint64_t frontier, uint64_t &h)
{
    if (li >= frontier) return false;
    h = exec_word(v, node, li) & W_HANDLE;
    return !((h >> 47) & 1);                   // MPX_HANDLE_NOOP
}

__global__ __launch_bounds__(256) void k_exec_count(DevView v, uint32_t node, unsigned long long *aux)
{
    __shared__ uint32_t wc[4];
    const uint64_t li = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint64_t h;
    const uint64_t m = __ballot(exec_take(v, node, li, aux[0], h));
    if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = (uint32_t)__builtin_popcountll(m);
    __syncthreads();
    if (threadIdx.x == 0) aux[1 + blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
}

// exclusive scan of the NB bucket counts, one workgroup of 1024, carried over chunks
__global__ __launch_bounds__(1024) void k_exec_scan(DevView v, unsigned long long *aux)
{
    __shared__ unsigned long long sh[1024];
    const uint64_t NB = v.NB;
    const uint32_t t = threadIdx.x;
    unsigned long long carry = 0;
    for (uint64_t base = 0; base < NB; base += 1024) {
        const unsigned long long x = base + t < NB ? aux[1 + base + t] : 0;
        sh[t] = x;
        __syncthreads();
        for (uint32_t d = 1; d < 1024; d <<= 1) {
            const unsigned long long y = t >= d ? sh[t - d] : 0;
            __syncthreads();
            sh[t] += y;
            __syncthreads();
        }
        if (base + t < NB) aux[1 + NB + base + t] = carry + sh[t] - x;
        carry += sh[1023];
        __syncthreads();
    }
    if (t == 0) aux[1 + 2 * NB] = carry;
}

__global__ __launch_bounds__(256) void k_exec_scatter(DevView v, uint32_t node, const unsigned long long *aux,
                                                     uint64_t *out)
{
    __shared__ uint32_t wc[4];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t li = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint64_t h = 0;
    const bool take = exec_take(v, node, li, aux[0], h);
    const uint64_t m = __ballot(take);
    if (lane == 0) wc[wv] = (uint32_t)__builtin_popcountll(m);
    __syncthreads();
    uint64_t at = aux[1 + v.NB + blockIdx.x] + __builtin_popcountll(m & ((1ull << lane) - 1));
    for (uint32_t k = 0; k < wv; ++k) at += wc[k];
    if (take) out[at] = h;
}

int launch_exec(const DevView &v, void *stream_, uint32_t node, unsigned long long *aux, uint64_t *out)
{
    hipStream_t s = (hipStream_t)stream_;
    const uint32_t blocks = cdiv(v.shard_len, 256);
    if (!out) {
        const unsigned long long init = v.shard_len;
        if (hipMemcpyAsync(aux, &init, 8, hipMemcpyHostToDevice, s) != hipSuccess) return -1;
        if (!blocks) return 0;
        hipLaunchKernelGGL(k_exec_frontier, dim3(blocks), dim3(256), 0, s, v, node, aux);
        hipLaunchKernelGGL(k_exec_count, dim3(blocks), dim3(256), 0, s, v, node, aux);
        hipLaunchKernelGGL(k_exec_scan, dim3(1), dim3(1024), 0, s, v, aux);
    } else if (blocks) {
        hipLaunchKernelGGL(k_exec_scatter, dim3(blocks), dim3(256), 0, s, v, node, aux, out);
    }
    return (int)hipGetLastError();
}

__global__ void k_frag_w1(const Frag *frags, uint64_t *out, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = frag_w1(frags + i);
}

int launch_frag_w1(const Frag *frags, uint64_t *out, uint64_t n, void *stream)
{
    if (!n) return 0;
    hipLaunchKernelGGL(k_frag_w1, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, frags, out, n);
    return (int)hipGetLastError();
}

// ---------------------------------------------------- phase-2 decisions --
// OnPrepareReply's batch at a promise quorum (multi/paxos.cpp:1056-1130; SURVEY
// §8 f2): adopt every pre-accepted value of an instance the node has not
// committed (the quorum's merged map, k_apply's OUT_K1 records without OUT_CMT),
// then fill every instance of the unproposed set below its last, open range
// with a noop — the instances not committed before the quorum and not adopted,
// below 1 + the highest committed-or-adopted instance.  The per-instance work is
// here; the host only merges the two sorted lists and numbers the noops.
// the message of the first COMMIT that reached (node n, instance li), NONE32 if none
__device__ inline uint32_t commit_msg(const DevView &v, uint32_t n, uint64_t li)
{
    if (!v.st_valid[sv_idx(v, n, li >> BSH)]) return NONE32;
    const uint32_t q = slot_global(v, n, li);
    if (!q) return NONE32;
    const uint64_t w1 = frag_w1(v.frags + q - 1);
    return (w1 >> 60) == K_COMMIT ? (uint32_t)w1 : NONE32;
}

__global__ __launch_bounds__(256) void k_decide(DevView v, uint32_t pass, DecideArgs a)
{
    __shared__ uint32_t wc[4];
    const uint32_t e = blockIdx.y, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t n = a.ev_node[e], g = a.ev_msg[e];
    const uint64_t li = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (pass == 0) {
        uint64_t x = 0;
        if (li < v.shard_len && commit_msg(v, n, li) < g) x = li + 1;
        x = wave_max(x);
        if (lane == 0 && x) atomicMax(&a.xmax[e], (unsigned long long)x);
        return;
    }
    const uint64_t end = a.xend[e];
    if ((uint64_t)blockIdx.x * 256 >= end) return;           // block-uniform
    bool fill = false;
    if (li < end && !(commit_msg(v, n, li) < g)) {
        const uint64_t a0 = a.ad_off[e], a1 = a.ad_off[e + 1];
        uint64_t lo = a0, hi = a1;                          // adopted: binary search
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (a.ad_li[mid] < li) lo = mid + 1; else hi = mid;
        }
        fill = !(lo < a1 && a.ad_li[lo] == li);
    }
    const uint64_t m = __ballot(fill);
    if (lane == 0) wc[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    const uint64_t bi = a.blk_off[e] + blockIdx.x;
    if (pass == 1) {
        if (threadIdx.x == 0) a.blk_cnt[bi] = wc[0] + wc[1] + wc[2] + wc[3];
        return;
    }
    uint32_t before = 0;
    for (uint32_t i = 0; i < wv; ++i) before += wc[i];
    if (fill)
        a.noop_li[a.ev_base[e] + a.blk_cnt[bi] + before + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = (uint32_t)li;
}

// per event: its block counts -> exclusive offsets (in place), total -> ev_total
__global__ __launch_bounds__(256) void k_decide_scan(DecideArgs a)
{
    __shared__ uint32_t ws[4];
    const uint32_t e = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t b0 = a.blk_off[e], b1 = a.blk_off[e + 1];
    uint64_t carry = 0;
    for (uint64_t base = b0; base < b1; base += 256) {
        const uint64_t i = base + threadIdx.x;
        const uint32_t x = i < b1 ? a.blk_cnt[i] : 0;
        uint32_t inc = x;                                    // wave inclusive scan
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(inc, d, 64);
            if (lane >= d) inc += y;
        }
        if (lane == 63) ws[wv] = inc;
        __syncthreads();
        uint32_t pre = 0, tot = 0;
        for (uint32_t k = 0; k < 4; ++k) { if (k < wv) pre += ws[k]; tot += ws[k]; }
        if (i < b1) a.blk_cnt[i] = (uint32_t)(carry + pre + inc - x);
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) a.ev_total[e] = carry;
}

int launch_decide(const DevView &v, void *stream, uint32_t pass, const DecideArgs &a)
{
    hipStream_t s = (hipStream_t)stream;
    if (!a.E) return 0;
    for (uint32_t e0 = 0; e0 < a.E; e0 += 65535) {           // grid.y limit: events in slices
        DecideArgs sl = a;
        sl.E = a.E - e0 < 65535 ? a.E - e0 : 65535;
        sl.ev_node = a.ev_node + e0; sl.ev_msg = a.ev_msg + e0;
        sl.xmax = a.xmax + e0; sl.xend = a.xend + e0; sl.ad_off = a.ad_off + e0;
        sl.blk_off = a.blk_off + e0; sl.ev_base = a.ev_base + e0; sl.ev_total = a.ev_total + e0;
        if (pass == 3) {
            hipLaunchKernelGGL(k_decide_scan, dim3(sl.E), dim3(256), 0, s, sl);
            continue;
        }
        const uint64_t blocks = pass == 0 ? cdiv(v.shard_len, 256) : a.max_blocks;
        if (!blocks) continue;
        hipLaunchKernelGGL(k_decide, dim3((uint32_t)blocks, sl.E), dim3(256), 0, s, v, pass, sl);
    }
    return (int)hipGetLastError();
}

// ------------------------------------------------- commit reliability --
// OnCommitReply (multi/paxos.cpp:1625-1641): a COMMIT_REPLY for a
// CommittingValues that exists (created at an earlier message: the accept
// quorum, :1418, or a promise quorum of a node holding commits, :1184-1197) and
// is not yet retired adds its learner to replied_; the commit retires at the
// reply that makes |replied_| == |nodes_|, and later replies find nothing
// (:1627).  One lane per (node, commit id) list; the replies' learner ids lie
// beside the list (no gathers), so a lane reads 8 B per reply.
__global__ __launch_bounds__(256) void k_commits(DevView v, CommitArgs a)
{
    const uint64_t l = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (l >= a.L) return;
    const uint32_t n = a.cr_node[l];
    const uint64_t c = a.cr_id[l], c0 = a.cm_off[n], c1 = a.cm_off[n + 1];
    uint32_t ret = NONE32;
    unsigned long long mask = 0;
    if (c >= 1 && c <= c1 - c0) {
        const uint32_t created = a.cm_pos[c0 + c - 1];
        for (uint64_t r = a.cr_off[l]; r < a.cr_off[l + 1]; ++r) {
            const uint32_t g = a.cr_msg[r], learner = a.cr_src[r];
            if (g < created) continue;                         // no such commit yet (:1627)
            mask |= 1ull << learner;                           // :1633 (learner < 64: checked by the host)
            if ((uint32_t)__popcll(mask) == v.N) { ret = g; break; }   // :1635-1640
        }
    }
    a.ret[l] = ret;
    a.mask[l] = mask;
}

int launch_commits(const DevView &v, void *stream, const CommitArgs &a)
{
    if (!a.L) return 0;
    hipLaunchKernelGGL(k_commits, dim3(cdiv(a.L, 256)), dim3(256), 0, (hipStream_t)stream, v, a);
    return (int)hipGetLastError();
}

// ------------------------------------------------- learn reliability --
// member Proposer (member/paxos.cpp:1345-1381, 1504-1533), one lane per
// LearningValues, over its events in processing order: a LEARN_REPLY adds its learner to
// learned_ and, while the learn is in learning_values_for_acceptors_, an acceptor of the
// node's epoch to that set; |set| >= |acceptors|/2+1 runs Applied and drops the entry
// (:1363-1370); |learned_| == |learners_| retires the learn (:1373-1380).  An
// AcceptorsChanged call removes a deleted acceptor from the set or adds an added one that
// had replied, then checks the quorum of the new set (:1507-1533).  A learn neither
// retired nor open at the end was dropped at `end` (LearnersChanged / the proposer deleted).
__global__ __launch_bounds__(256) void k_learns(LearnArgs a)
{
    const uint64_t l = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (l >= a.L) return;
    bool facc = a.facc[l] != 0;
    unsigned long long learned = 0, acc = 0;
    uint32_t applied = NONE32, retired = NONE32;
    for (uint64_t k = a.ev_off[l]; k < a.ev_off[l + 1]; ++k) {
        const uint64_t w = a.ev_a[k];
        const uint64_t am = a.ev_m[k];
        const uint32_t pos = (uint32_t)(w >> 32), who = (uint32_t)w & 63;
        const uint32_t quorum = (uint32_t)__popcll(am) / 2 + 1;
        if (((w >> 24) & 0xFF) == LEV_REPLY) {
            learned |= 1ull << who;                                        // :1353
            if (facc && ((am >> who) & 1)) {                               // :1355-1358
                acc |= 1ull << who;
                if ((uint32_t)__popcll(acc) >= quorum) { applied = pos; facc = false; }   // :1363-1370
            }
            if ((uint32_t)__popcll(learned) == ((w >> 8) & 0x7F)) { retired = pos; break; }   // :1373-1380
        } else if (facc) {
            if ((w >> 23) & 1) { if ((learned >> who) & 1) acc |= 1ull << who; }          // :1518-1519
            else acc &= ~(1ull << who);                                                      // :1511-1512
            if ((uint32_t)__popcll(acc) >= quorum) { applied = pos; facc = false; }          // :1521-1528
        }
    }
    a.applied[l] = applied;
    a.retired[l] = retired;
    a.ended[l] = retired == NONE32 ? a.end[l] : NONE32;
    a.mask[l] = learned;
}

int launch_learns(const DevView &, void *stream, const LearnArgs &a)
{
    if (!a.L) return 0;
    hipLaunchKernelGGL(k_learns, dim3(cdiv(a.L, 256)), dim3(256), 0, (hipStream_t)stream, a);
    return (int)hipGetLastError();
}

int launch_decode(const DevView &v, void *stream, uint32_t node, uint64_t l0, uint64_t count, uint64_t *out)
{
    if (!count) return 0;
    hipLaunchKernelGGL(k_decode, dim3(cdiv(count, 256)), dim3(256), 0, (hipStream_t)stream, v, node, l0, count, out);
    return (int)hipGetLastError();
}

LaunchGeom launch_geometry(uint32_t N, uint64_t NB, uint32_t num_cus)
{
    LaunchGeom g{};
    const uint64_t npairs = (uint64_t)N * NB;
    // k_apply_fast holds 5 waves/SIMD (82 VGPRs); 8 workgroups of 4 waves per
    // CU measured best on C4 (2.17 ms vs 2.31 ms at 5)
    g.apply_wgs = (uint32_t)(npairs < 1 ? 1 : npairs < (uint64_t)num_cus * 8 ? npairs : (uint64_t)num_cus * 8);
    g.chosen_wgs = (uint32_t)(NB < 1 ? 1 : NB < (uint64_t)num_cus * 4 ? NB : (uint64_t)num_cus * 4);
    // k_store: 8 workgroups of 4 waves per CU at C4 size; a smaller shard (fewer 128-bucket
    // chunks than 2.5 per wave) takes fewer, so each wave still has a next chunk in flight
    // (C4 shard at world 8: 94 vs 101 us per step, profiles/r03_v7_shard_ab.json)
    const uint64_t chunks = (uint64_t)(N + 1) * (NB / 128 + 1), want = chunks / 10;
    const uint64_t hi = (uint64_t)num_cus * 8;
    g.store_wgs = (uint32_t)(want > hi ? hi : want < num_cus ? num_cus : want);
    // k_plan_store8: MPX_PS_WPC workgroups of 8 waves per CU (all resident), at most one per group
    const uint64_t groups = (NB + PS_G - 1) / PS_G, ps = (uint64_t)num_cus * MPX_PS_WPC;
    g.ps_wgs = (uint32_t)(groups < 1 ? 1 : groups < ps ? groups : ps);
    return g;
}

bool run_ends_with_store(const DevView &v)
{
    const bool member = v.semantics == MPX_SEM_MEMBER;
    const bool plan_path = !v.digest && !v.walk_all && !v.window && (member || v.N <= FAST_MAX_NODES);
    const bool lplan = plan_path && (member || v.num_gp_snap);
    return plan_path && v.chosen_static && !member && !lplan && v.num_gp == 0 && v.slot_w == 1;
}

int launch_run(const DevView &v, void *stream_, LaunchGeom g, void *const ev[5], LaunchSide side)
{
    void *ev_begin = ev[0], *ev_apply0 = ev[1], *ev_apply1 = ev[2], *ev_general = ev[3], *ev_end = ev[4];
    hipStream_t s = (hipStream_t)stream_;
    const uint32_t n_partials = g.apply_wgs + g.chosen_wgs;
    const bool member = v.semantics == MPX_SEM_MEMBER;
    uint64_t reset_n = ((uint64_t)v.N * v.NB + 15) / 16;
    if (v.NB > reset_n) reset_n = v.NB;
    if (8ull * n_partials > reset_n) reset_n = 8ull * n_partials;
    if (2ull * v.N > reset_n) reset_n = 2ull * v.N;
    if (v.out_subs > reset_n) reset_n = v.out_subs;
    // Phase events ride on kernel dispatches (hipExtLaunchKernelGGL start / stop events) where a
    // kernel begins or ends the phase: a separate event record costs a 5-10 us bubble between
    // dependent kernels (rocprof, C4: 16 us of a 395 us step)
    // multi: the reset rides on the first header-scan kernel (one launch less per step)
    // (a single-pass scan — the chunk aggregates found by a decoupled look-back inside
    // k_headers, agent-coherent atomics, no k_scan_chunk launch — was measured slower: C4 shard
    // scan phase 22.0 vs 17.9 us, the look-back's serialized round trips cost more than the
    // launch; profiles/r04_v1_bench.json)
    const bool fold_reset = !member && v.num_chunks;
    if (!fold_reset)
        hipExtLaunchKernelGGL(k_reset, dim3(cdiv(reset_n ? reset_n : 1, 256)), dim3(256), 0, s,
                              (hipEvent_t)ev_begin, (hipEvent_t)nullptr, 0, v, n_partials);
    if (member) {
        // member role / version gates from the E_EPOCH markers (k_gate_*)
        hipLaunchKernelGGL(k_gate_epochs, dim3(v.N), dim3(256), 0, s, v);
        if (v.num_msgs) hipLaunchKernelGGL(k_gate_msgs, dim3(cdiv(v.num_msgs, 256 * GATE_PER)), dim3(256), 0, s, v);
        if (v.num_sc) hipLaunchKernelGGL(k_gate_scan, dim3(cdiv(v.num_sc, 256 * GATE_PER)), dim3(256), 0, s, v, v.num_sc);
        if (v.num_batches) hipLaunchKernelGGL(k_gate_votes, dim3(cdiv(v.num_batches, 256)), dim3(256), 0, s, v);
    }
    const bool small = v.scan_chunk == SCAN_CHUNK_SMALL;      // (the host cut the chunks: scan_chunk_for)
    if (v.num_chunks) {
        if (fold_reset) {
            if (small) hipExtLaunchKernelGGL((k_scan_chunk<true, SCAN_CHUNK_SMALL>), dim3(v.num_chunks), dim3(256), 0, s,
                                             (hipEvent_t)ev_begin, (hipEvent_t)nullptr, 0, v, n_partials);
            else hipExtLaunchKernelGGL((k_scan_chunk<true, SCAN_CHUNK>), dim3(v.num_chunks), dim3(256), 0, s,
                                       (hipEvent_t)ev_begin, (hipEvent_t)nullptr, 0, v, n_partials);
        } else if (small) hipLaunchKernelGGL((k_scan_chunk<false, SCAN_CHUNK_SMALL>), dim3(v.num_chunks), dim3(256), 0, s,
                                             v, n_partials);
        else hipLaunchKernelGGL((k_scan_chunk<false, SCAN_CHUNK>), dim3(v.num_chunks), dim3(256), 0, s, v, n_partials);
        if (v.scan_node_pass) hipLaunchKernelGGL(k_scan_node, dim3(v.N), dim3(256), 0, s, v);   // long node streams
    }
    // the scan's flag pass, the promise-quorum chunks and the accept votes: one launch (k_headers)
    {
        const uint32_t nb_scan = v.num_chunks, nb_prop = cdiv(v.num_pc, 4), nb_votes = cdiv(v.num_batches, 256);
        if (nb_scan + nb_prop + nb_votes) {
            const dim3 grid(nb_scan + nb_prop + nb_votes);
            if (member && small) hipLaunchKernelGGL((k_headers<true, SCAN_CHUNK_SMALL>), grid, dim3(256), 0, s, v, nb_scan, nb_prop);
            else if (member) hipLaunchKernelGGL((k_headers<true, SCAN_CHUNK>), grid, dim3(256), 0, s, v, nb_scan, nb_prop);
            else if (small) hipLaunchKernelGGL((k_headers<false, SCAN_CHUNK_SMALL>), grid, dim3(256), 0, s, v, nb_scan, nb_prop);
            else hipLaunchKernelGGL((k_headers<false, SCAN_CHUNK>), grid, dim3(256), 0, s, v, nb_scan, nb_prop);
        }
    }
    // plan path (the timed step): k_plan (multi: the lean pairs) / k_plan_list (the work
    // list's pairs without promise rounds) + store, then k_apply over the pairs k_plan_list
    // listed and the promise-round pairs.  A digested run (verification) and v.walk_all
    // (MPX_STEP_WALK=1) walk every pair instead, as do multi traces with more than
    // FAST_MAX_NODES nodes.
    const bool plan_path = !v.digest && !v.walk_all && !v.window && (member || v.N <= FAST_MAX_NODES);
    const bool lplan = plan_path && (member || v.num_gp_snap);
    // Three streams on the list plan path (the kernels are latency-bound walks, so running them
    // side by side hides their round trips behind each other's):
    //   s  : k_plan -> k_plan_list -> k_store_ext -> k_commit_check -> store          (planned pairs)
    //   s2 : [k_prop_node ->] k_apply AM_FULL  from the end of the header kernels     (promise rounds)
    //   s3 : k_chosen from the end of the plan of its buckets, k_apply AM_SNAP from the end of
    //        k_plan_list (the pairs it listed)
    // Each writes its own pairs / rows (a listed pair has no plan word; k_chosen walks only the
    // buckets plan_chosen left, whose row-N plan word is PLAN_SKIP) and adds counters with
    // atomics; all joined before the summary.  k_prop_node feeds only the promise-round walk
    // (k_plan / k_plan_list pairs have no promise-reply runs).
    const bool rounds = lplan && v.num_gp > v.num_gp_snap;
    const bool side_rounds = rounds && side.stream2;
    const bool side3 = lplan && side.stream3;
    hipStream_t s2 = side_rounds ? (hipStream_t)side.stream2 : s;
    hipStream_t s3 = side3 ? (hipStream_t)side.stream3 : s;
    const bool prop = (v.num_pc && v.pc_multi) || v.window;
    // (a window: every node's round after the window, prop_out, comes from k_prop_node)
    if (prop && !side_rounds) hipLaunchKernelGGL(k_prop_node, dim3(v.N), dim3(64), 0, s, v);
    if (v.window) {
        // incremental window: every pair of the window on the value-state walk, the chosen log
        // of the batches chosen in it, the summary
        if (member) hipExtLaunchKernelGGL(k_apply_win<true>, dim3(g.apply_wgs), dim3(256), 0, s, (hipEvent_t)ev_apply0,
                                          (hipEvent_t)ev_general, 0, v);
        else hipExtLaunchKernelGGL(k_apply_win<false>, dim3(g.apply_wgs), dim3(256), 0, s, (hipEvent_t)ev_apply0,
                                   (hipEvent_t)ev_general, 0, v);
        if (ev_apply1) (void)hipEventRecord((hipEvent_t)ev_apply1, s);
        hipLaunchKernelGGL(k_chosen_win, dim3(g.chosen_wgs), dim3(256), 0, s, v, g.apply_wgs);
        hipExtLaunchKernelGGL(k_reduce, dim3(cdiv(n_partials ? n_partials : 1, 256)), dim3(256), 0, s, (hipEvent_t)nullptr, (hipEvent_t)ev_end, 0, v, n_partials);
        return (int)hipGetLastError();
    }
    if (side_rounds) {
        (void)hipEventRecord((hipEvent_t)side.fork, s);
        (void)hipStreamWaitEvent(s2, (hipEvent_t)side.fork, 0);
        if (prop) hipLaunchKernelGGL(k_prop_node, dim3(v.N), dim3(64), 0, s2, v);
    }
    auto launch_rounds = [&]() {
        if (member) hipLaunchKernelGGL((k_apply<APPLY_WAVES_FULL, false, true>), dim3(g.apply_wgs), dim3(256), 0, s2, v, v.num_gp_snap, v.num_gp);
        else hipLaunchKernelGGL((k_apply<APPLY_WAVES_FULL, false, false>), dim3(g.apply_wgs), dim3(256), 0, s2, v, v.num_gp_snap, v.num_gp);
        if (side_rounds) (void)hipEventRecord((hipEvent_t)side.join, s2);
    };
    // (A/B: MPX_FULL_LATE starts the promise-round walk at the end of k_plan_list instead, so the
    // plan runs alone)
    const bool full_late = side_rounds && side.stream3 && ab_env("MPX_FULL_LATE") != nullptr;
    if (side_rounds && !full_late) launch_rounds();
    auto launch_rounds_late = [&]() {
        if (!full_late) return;
        (void)hipStreamWaitEvent(s2, (hipEvent_t)side.fork3b, 0);
        launch_rounds();
    };
    if (ev_apply0 && !plan_path) (void)hipEventRecord((hipEvent_t)ev_apply0, s);
    // the chosen log needs no k_chosen launch when the trace's chosen-log runs passed
    // plan_chosen's static test at load; then, with no general pair either (the C4 shape), the
    // store ends the step and the summary rides on its extra workgroups
    const bool skip_chosen = plan_path && v.chosen_static;
    const bool fuse_reduce = run_ends_with_store(v);
    const uint32_t reduce_wgs = cdiv(n_partials ? n_partials : 1, 256);
    auto launch_chosen = [&](hipStream_t cs, hipEvent_t start) {
        hipExtLaunchKernelGGL(k_chosen, dim3(g.chosen_wgs), dim3(256), 0, cs, start, (hipEvent_t)nullptr, 0, v, g.apply_wgs);
    };
    // the pairs k_plan_list listed (their count is on the device)
    auto launch_listed = [&](hipStream_t ls) {
        DevView vd = v;
        vd.gp_list = v.gp_dyn;
        if (member) hipLaunchKernelGGL((k_apply<APPLY_WAVES_SNAP, false, true, AM_SNAP>), dim3(g.apply_wgs), dim3(256), 0, ls, vd, 0ull, ~0ull);
        else hipLaunchKernelGGL((k_apply<APPLY_WAVES_SNAP, false, false, AM_SNAP>), dim3(g.apply_wgs), dim3(256), 0, ls, vd, 0ull, ~0ull);
    };
    // the plan words of every (row, bucket) -> state rows and the chosen log
    // (1-byte slots: 128-bucket chunks, 32 KiB per row and two plan words per lane, 0.295 vs
    // 0.315 ms for 64-bucket chunks at C4)
    auto launch_store = [&](hipEvent_t stop) {
        if (v.slot_w == 1 && fuse_reduce)
            hipExtLaunchKernelGGL((k_store8<true, 128, true>), dim3(g.store_wgs + reduce_wgs), dim3(256), 0, s, nullptr,
                                  stop, 0, v, g.store_wgs, n_partials);
        else if (v.slot_w == 1)
            hipExtLaunchKernelGGL((k_store8<true, 128>), dim3(g.store_wgs), dim3(256), 0, s, nullptr, stop, 0, v,
                                  g.store_wgs, 0u);
        else
            hipExtLaunchKernelGGL((k_store<32, true, uint16_t, u16x4>), dim3(g.store_wgs), dim3(256), 0, s, nullptr, stop, 0, v);
    };
    const uint32_t plan_blocks = cdiv((uint64_t)v.N * v.NB, 256);
    bool chosen_done = false;                            // k_chosen launched on s3 already
    // plan and store in one launch (k_plan_store8) where the store ends the step
    const bool plan_store = PLAN_STORE && fuse_reduce && v.slot_w == 1 && PS_G * v.N <= PS_CHOSEN && g.ps_wgs;
    if (plan_path) {
        if (member) {
            // (8 segments / 32 runs since the Value check left the walk — 128 VGPRs, no spill:
            // C5 0.451 -> 0.384 ms, contended C5 2.745 -> 2.582 ms, profiles/r04_v25_ab_member_plan8.json)
            if constexpr (PLAN_RETRY) {
                // the 9..16-segment pairs planned again (one lane per listed pair, 2 waves per SIMD);
                // the listed-pair walk starts after it
                hipExtLaunchKernelGGL((k_plan_list<true, PLAN_XSEG_MEMBER, PLAN_XFRAGS, PLAN_WAVES_MEMBER>), dim3(plan_blocks),
                                      dim3(256), 0, s, (hipEvent_t)ev_apply0, (hipEvent_t)nullptr, 0, v, g.apply_wgs);
                hipExtLaunchKernelGGL((k_plan_list<true, PLAN_RETRY_SEG, PLAN_XFRAGS, 2, true>), dim3(cdiv(v.num_gp_snap ? v.num_gp_snap : 1, 256)), dim3(256), 0,
                                      s, (hipEvent_t)nullptr, side3 ? (hipEvent_t)side.fork3b : (hipEvent_t)nullptr, 0, v,
                                      g.apply_wgs);
            } else {
                hipExtLaunchKernelGGL((k_plan_list<true, PLAN_XSEG_MEMBER, PLAN_XFRAGS, PLAN_WAVES_MEMBER>), dim3(plan_blocks),
                                      dim3(256), 0, s, (hipEvent_t)ev_apply0,
                                      side3 ? (hipEvent_t)side.fork3b : (hipEvent_t)nullptr, 0, v, g.apply_wgs);
            }
            if (side3) {                                 // (the listed pairs' walk, the step's longest chain)
                (void)hipStreamWaitEvent(s3, (hipEvent_t)side.fork3b, 0);
                launch_listed(s3);
                (void)hipEventRecord((hipEvent_t)side.join3, s3);
                launch_rounds_late();
            }
            hipLaunchKernelGGL(k_store_ext, dim3(g.chosen_wgs), dim3(256), 0, s, v);
            if (v.any_vchk) hipLaunchKernelGGL(k_commit_check<true>, dim3(g.apply_wgs), dim3(256), 0, s, v);
            // member k_plan_list planned the chosen log too: k_chosen walks the rest beside the listed
            // pairs (it reads only the votes and the chosen-log runs)
            if (side3 && !skip_chosen) { launch_chosen(s, nullptr); chosen_done = true; }
        } else if (plan_store) {
            hipExtLaunchKernelGGL(k_plan_store8, dim3(g.ps_wgs + cdiv(n_partials ? n_partials : 1, 64 * PS_WG)), dim3(64 * PS_WG), 0, s,
                                  (hipEvent_t)ev_apply0, (hipEvent_t)ev_apply1, 0, v, g.ps_wgs, n_partials);
        } else {
            // (a fused plan-and-store kernel — four buckets' plan words decided per wave step and
            // written as NN + 1 KiB stores, loads three / two / one step ahead — measured slower:
            // 0.391 vs 0.304 ms apply phase at C4; the compiler drains vmcnt at its loop head)
            hipExtLaunchKernelGGL(k_plan, dim3(plan_blocks), dim3(256), 0, s, (hipEvent_t)ev_apply0,
                                  side3 ? (hipEvent_t)side.fork3a : (hipEvent_t)nullptr, 0, v, g.apply_wgs);
            if (side3 && !skip_chosen) {                 // k_plan decided which buckets' chosen log it plans
                (void)hipStreamWaitEvent(s3, (hipEvent_t)side.fork3a, 0);
                launch_chosen(s3, nullptr);
                chosen_done = true;
            }
            if (lplan) {
#ifdef MPX_PLAN_LSEG4
                hipExtLaunchKernelGGL((k_plan_list<false>), dim3(plan_blocks), dim3(256), 0, s, (hipEvent_t)nullptr,
                                      side3 ? (hipEvent_t)side.fork3b : (hipEvent_t)nullptr, 0, v, g.apply_wgs);   // (A/B build)
#else
                hipExtLaunchKernelGGL((k_plan_list<false, PLAN_XSEG, PLAN_XFRAGS>), dim3(plan_blocks), dim3(256), 0, s,
                                      (hipEvent_t)nullptr, side3 ? (hipEvent_t)side.fork3b : (hipEvent_t)nullptr, 0, v,
                                      g.apply_wgs);
#endif
                if (side3) {
                    (void)hipStreamWaitEvent(s3, (hipEvent_t)side.fork3b, 0);
                    launch_listed(s3);
                    (void)hipEventRecord((hipEvent_t)side.join3, s3);
                    launch_rounds_late();
                }
#ifndef MPX_PLAN_LSEG4
                hipLaunchKernelGGL(k_store_ext, dim3(g.chosen_wgs), dim3(256), 0, s, v);
#endif
                if (v.any_vchk) hipLaunchKernelGGL(k_commit_check<false>, dim3(g.apply_wgs), dim3(256), 0, s, v);
            }
        }
        // every pair the trace marks lean (pair_gp 0) is one k_plan can describe (ingest.cpp /
        // mpx_load_clean_device use its predicate, plan_shape_ok), so nothing is left for the
        // lean per-slot kernel after the store (fast_rest 0, checked when the run is collected)
        if (!plan_store) launch_store((hipEvent_t)ev_apply1);
    } else if (member) {
        if (ev_apply1) (void)hipEventRecord((hipEvent_t)ev_apply1, s);
    } else {
        // digest runs (verification) take their own instantiation, so the timed kernel
        // carries no digest code; the lean kernel also writes the chosen log of clean buckets
        if (v.digest) hipLaunchKernelGGL((k_apply_fast<1, true>), dim3(g.apply_wgs), dim3(256), 0, s, v);
        else hipLaunchKernelGGL((k_apply_fast<1, false>), dim3(g.apply_wgs), dim3(256), 0, s, v);
        if (ev_apply1) (void)hipEventRecord((hipEvent_t)ev_apply1, s);
    }
    if (lplan) {
        if (!side3) launch_listed(s);
        if (rounds && !side_rounds) launch_rounds();
        if (side_rounds) (void)hipStreamWaitEvent(s, (hipEvent_t)side.join, 0);
        if (side3) (void)hipStreamWaitEvent(s, (hipEvent_t)side.join3, 0);
    } else {
        // every pair of the host-built work list on the general kernel, in three ranges
        // (ingest.cpp orders the list): event-free pairs (AM_SIMPLE), pairs without
        // promise-reply runs (PREPARE / member E_EPOCH events, AM_SNAP), the rest (promise rounds).
        // Occupancy (C3 2^24 general apply): AM_SNAP at 4 waves / SIMD 1.324 ms vs 1.469
        // unconstrained (3 waves) and 1.496 at 5 (spills); the full kernel at 4 waves 1.394 vs
        // 1.580 ms unconstrained; one kernel over the whole list 1.351 ms (C5: 2.165 vs 2.544 ms)
        const uint64_t ns = v.num_gp_simple, nq = v.num_gp_snap;
        if (v.digest) {
            if (ns) { if (member) hipLaunchKernelGGL((k_apply<1, true, true, AM_SIMPLE>), dim3(g.apply_wgs), dim3(256), 0, s, v, 0ull, ns);
                      else hipLaunchKernelGGL((k_apply<1, true, false, AM_SIMPLE>), dim3(g.apply_wgs), dim3(256), 0, s, v, 0ull, ns); }
            if (nq > ns) { if (member) hipLaunchKernelGGL((k_apply<1, true, true, AM_SNAP>), dim3(g.apply_wgs), dim3(256), 0, s, v, ns, nq);
                           else hipLaunchKernelGGL((k_apply<1, true, false, AM_SNAP>), dim3(g.apply_wgs), dim3(256), 0, s, v, ns, nq); }
            if (v.num_gp > nq) { if (member) hipLaunchKernelGGL((k_apply<1, true, true>), dim3(g.apply_wgs), dim3(256), 0, s, v, nq, v.num_gp);
                                 else hipLaunchKernelGGL((k_apply<1, true, false>), dim3(g.apply_wgs), dim3(256), 0, s, v, nq, v.num_gp); }
        } else {
            if (ns) { if (member) hipLaunchKernelGGL((k_apply<1, false, true, AM_SIMPLE>), dim3(g.apply_wgs), dim3(256), 0, s, v, 0ull, ns);
                      else hipLaunchKernelGGL((k_apply<1, false, false, AM_SIMPLE>), dim3(g.apply_wgs), dim3(256), 0, s, v, 0ull, ns); }
            if (nq > ns) { if (member) hipLaunchKernelGGL((k_apply<APPLY_WAVES_SNAP, false, true, AM_SNAP>), dim3(g.apply_wgs), dim3(256), 0, s, v, ns, nq);
                           else hipLaunchKernelGGL((k_apply<APPLY_WAVES_SNAP, false, false, AM_SNAP>), dim3(g.apply_wgs), dim3(256), 0, s, v, ns, nq); }
            if (v.num_gp > nq) { if (member) hipLaunchKernelGGL((k_apply<APPLY_WAVES_FULL, false, true>), dim3(g.apply_wgs), dim3(256), 0, s, v, nq, v.num_gp);
                                 else hipLaunchKernelGGL((k_apply<APPLY_WAVES_FULL, false, false>), dim3(g.apply_wgs), dim3(256), 0, s, v, nq, v.num_gp); }
        }
    }
    // the chosen log of the buckets no plan word covered (none when the trace's chosen-log runs
    // passed plan_chosen's static test at load: k_chosen is not launched), then the summary
    if (fuse_reduce) {
        // (the apply phase ends with the store; the general and tail phases are empty: the
        // host reads the store's stop event for them, run_ends_with_store)
    } else if (skip_chosen || chosen_done) {
        hipExtLaunchKernelGGL(k_reduce, dim3(cdiv(n_partials ? n_partials : 1, 256)), dim3(256), 0, s, (hipEvent_t)ev_general,
                              (hipEvent_t)ev_end, 0, v, n_partials);
    } else {
        launch_chosen(s, (hipEvent_t)ev_general);
        hipExtLaunchKernelGGL(k_reduce, dim3(cdiv(n_partials ? n_partials : 1, 256)), dim3(256), 0, s, (hipEvent_t)nullptr, (hipEvent_t)ev_end, 0, v, n_partials);
    }
    return (int)hipGetLastError();
}

}  // namespace mpx
