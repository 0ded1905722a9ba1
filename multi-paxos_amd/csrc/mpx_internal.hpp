// mpx_internal.hpp — shared layout of the engine (host ingest, launch code, kernels).
//
// HBM layout (DESIGN.md §Data layout):
//   * messages, all nodes flattened in processing order: SoA headers
//     m_type u8 | m_src u32 | m_ballot u64 | m_aux u64 | m_ent u64 | m_cnt u32
//   * entry pools: e_val u64 (+ e_slot u8 when a fragment is sparse) for
//     ACCEPT / COMMIT / P_BATCH, content-addressed: an entry list that reaches
//     several nodes (a broadcast, its P_BATCH, duplicates) is stored once;
//     r_pid,r_val u64 (+ r_slot) for PREPARE_REPLY; g_a,g_b u64 prepare ranges
//   * fragments: every entry-carrying message split into runs that fall in one
//     256-instance bucket, listed per pair in processing order (CSR); pairs are
//     bucket-major, q = bucket * N + node, so one wave can walk a bucket's
//     nodes and reuse the shared Values
//   * state: one 1- or 2-byte slot (slot_w) per (node, instance) = fragment + 1 counted from
//       the pair's first fragment (f_off[bucket * N + node]), 0 = empty:
//       the message run (fragment) that fixed the slot.  Its message's type
//       says accepted or committed, its header ballot is the tag (multi;
//       member: the entry's proposal id e_pid) and its entry at the slot's
//       position holds the Value handle — AcceptedValue(id, value) by
//       reference to the resident trace; k_decode turns a slot back into
//       {ballot, word}.  Accepted and committed entries of a node are disjoint
//       (OnCommit erases accepted_values_, multi/paxos.cpp:1501; OnAccept skips
//       committed, :1380), so one slot holds either.
//   * chosen log: one slot per instance = index + 1 of the chosen batch's run
//       among its bucket's chosen fragments (cf_off), 0 = none; stored as
//       row N of the state array so k_store streams both alike
#pragma once
#include <cstdint>
#include <cstdlib>
#include <cstddef>

#include "mpx.h"

#ifdef __HIP__
#define MPX_HD __host__ __device__
#else
#define MPX_HD
#endif

namespace mpx {

// Environment knobs.  std::getenv is read only for the alternative paths the GPU tests compare
// with the default one (MPX_SLOT_BYTES, MPX_PROP_CHUNK, MPX_STEP_WALK, MPX_SCAN_NODE_PASS,
// MPX_SCAN_SMALL, MPX_DECIDE_HOST, MPX_DECIDE_DEVICE).  Launch-tuning knobs kept for same-box
// A/B runs (tools/ab_*.sh) go through ab_env: only a variant built with -DMPX_AB
// (make EXTRA=-DMPX_AB OUT=$PWD/multi-paxos_amd/lib_<v> OBJ=$PWD/multi-paxos_amd/build_<v>) reads them;
// the product library ignores them.
inline const char *ab_env(const char *k)
{
#ifdef MPX_AB
    return std::getenv(k);
#else
    (void)k;
    return nullptr;
#endif
}

constexpr uint32_t BSH = 8;                  // bucket = 256 instances
constexpr uint32_t BS = 1u << BSH;
#ifndef MPX_SCAN_CHUNK
#define MPX_SCAN_CHUNK 2048                     // (a build knob for A/B: make EXTRA=-DMPX_SCAN_CHUNK=1024)
#endif
constexpr uint32_t SCAN_CHUNK = MPX_SCAN_CHUNK;        // header-scan chunk (messages): 8 per thread
// a short scan stream (an instance shard) is cut into half-size chunks: twice the
// workgroups for the two scan launches, which are latency-bound at that size (C4 shard at
// world 8: 1024-record chunks -2.7 us per step; at C4 size +2 %, profiles/r03_v11_scan_chunk_ab.json)
constexpr uint32_t SCAN_CHUNK_SMALL = SCAN_CHUNK / 2;
constexpr uint64_t SCAN_SMALL_RECORDS = 1ull << 21;
inline uint32_t scan_chunk_for(uint64_t records)
{
    if (const char *x = std::getenv("MPX_SCAN_SMALL")) return std::atoi(x) ? SCAN_CHUNK_SMALL : SCAN_CHUNK;   // (A/B)
    return records <= SCAN_SMALL_RECORDS ? SCAN_CHUNK_SMALL : SCAN_CHUNK;
}
constexpr uint32_t PROP_CHUNK = 512;         // promise-quorum chunk (pl records): 8 windows of 64 (C3 2^24 scan
                                             // phase 0.112 ms vs 0.128 at 2048, 0.134 at 256)
// k_headers' scan blocks re-reduce a node's earlier chunk aggregates inline (O(chunks^2)
// per node) up to this many chunks per node; longer streams take k_scan_node
constexpr uint32_t SCAN_INLINE_CHUNKS = 512;
constexpr uint32_t NONE32 = 0xFFFFFFFFu;
constexpr uint64_t EVX_ONE = 1ull << 63;     // ev_aux: the PREPARE has one range in the bucket (interval inline)

constexpr uint64_t W_PRESENT = 1ull << 63;
constexpr uint64_t W_COMMITTED = 1ull << 62;
constexpr uint64_t W_HANDLE = (1ull << 62) - 1;

// state slot / chosen-log encoding (see the layout note above): fragments and
// entries stay below 2^32 - 1
constexpr uint64_t MAX_ENTRIES = 0xFFFFFFFEull;
constexpr uint64_t MAX_FRAGS = 0xFFFFFFFEull;
// 2-byte state slots hold the pair-local fragment index + 1
constexpr uint64_t MAX_PAIR_FRAGS = 0xFFFEull;
constexpr uint64_t MAX_PAIR_FRAGS_1 = 0xFEull;   // 1-byte slots when every pair fits
typedef uint16_t slot_t;

// m_flags bits, written by the header scan / proposer kernels
enum : uint8_t {
    F_GRANTED = 1,    // PREPARE id > promised, ACCEPT id >= promised (paxos.cpp:865,1366)
    F_REJECT = 2,     // reply REJECT(max_seen) (paxos.cpp:894,1398)
    F_COUNTED = 4,    // PREPARE_REPLY merged into pre_accepted (paxos.cpp:1038-1045)
    F_QUORUM = 8,     // PREPARE_REPLY that reached the promise quorum (paxos.cpp:1047)
    F_BADNODE = 16,
    // member semantics (set by k_gate_epochs / k_gate_msgs from the E_EPOCH markers)
    F_ACCCLR = 32,    // E_EPOCH: the node's Acceptor is deleted or recreated (member/paxos.cpp:1897-1901,1952-1957)
    F_PRECLR = 64,    // E_EPOCH: its Proposer is deleted, created or sees new acceptors (idle)
    F_PROP = 128      // LEARN: the node has a Proposer (Proposer::OnLearn's ASSERT, :1398)
};

// member semantics: per-message role / version gate, computed on the device
// (kernels.hip k_gate_*) from the E_EPOCH markers and the epoch table (include/mpx.h):
//   PREPARE / ACCEPT : acceptor incarnation (1..255) when the node has an
//                      Acceptor of the message's version, 0 = dropped
//                      (Loop :749-756, version filter :1702,1744)
//   E_EPOCH          : the node's new incarnation | G_ACCCLR | G_PRECLR
//   LEARN            : G_PROP when the node has a Proposer
//   PREPARE_REPLY / ACCEPT_REPLY / P_START / P_BATCH :
//                      (epoch + 1) << G_EPOCH_SHIFT when the node has a Proposer
// The header scan runs over (incarnation << 56 | ballot), so one prefix max
// restarts at every new Acceptor; member ballots must stay below 2^56.
enum : uint32_t { G_SEG = 0xFF, G_ACCCLR = 1u << 8, G_PRECLR = 1u << 9, G_PROP = 1u << 10, G_EPOCH_SHIFT = 16 };
// ee_state: epoch (low 16 bits) | incarnation << 16 | acceptor << 24 | proposer << 25
enum : uint32_t { EE_SEG_SHIFT = 16, EE_ACC = 1u << 24, EE_PROP = 1u << 25 };
constexpr uint64_t SEG_SHIFT = 56;
constexpr uint64_t LOW56 = (1ull << 56) - 1;

// Header-scan stream (ingest.cpp, gen_device.hip): per node, in processing
// order, only the records that move the acceptor scalars promised / max_seen or
// take a scan flag — PREPARE, ACCEPT, REJECT (multi), E_EPOCH (member), and any
// record with a bad source (violation) — as {type, key, message index}; the
// key is the ballot (member: incarnation << 56 | ballot).  The scan reads 13 B
// per such record instead of every header of the trace.
enum : uint8_t {
    SC_PREP = 0,      // p = s = key; granted if id > promised, reject if <      (multi/paxos.cpp:862-894)
    SC_ACC = 1,       // s = key; granted if id >= promised, else reject        (:1363-1398)
    SC_SONLY = 2,     // s = key (REJECT's max_id, :1229-1230)
    SC_PS = 3,        // p = s = key (member E_EPOCH: a new Acceptor incarnation)
    SC_NONE = 4,      // no contribution (a COMMIT with a bad source)
    SC_KIND = 7,
    SC_BAD = 8,       // the record's source is not a node: F_BADNODE + violation
    SC_VIRT = 16      // member: a left-out ACCEPT (header sharding), sc_idx = the next kept message
};

// fragment kinds (Frag::flags >> 4)
enum : uint8_t { K_ACCEPT = 0, K_COMMIT = 1, K_PREPLY = 2, K_BATCH = 3 };
// FR_VCHK (ingest): a commit / learn (member: also an accept) run that meets a slot committed
// earlier in its pair through another entry holding another Value — the Value check
// (k_commit_check) may find a violation there (equal Values through another entry cannot).
// (flags bit 1 stays free: k_plan_list's staged words carry F_GRANTED in it, MP_GRANTED)
// FR_VEQ (ingest): every slot the run meets that an earlier commit / learn of its pair fixed holds
// an equal Value — the walks (k_apply) skip their Value compare (ingest.cpp mark_equal_values).
// FR_UPID (ingest, on a promise-reply run; the same bit as FR_VEQ, which only accept / commit runs
// carry): every entry of the run has the same proposal id, f_pid[run] (the promise-round walk takes
// it with the run's descriptor instead of loading each slot's id).
enum : uint8_t { FR_DENSE = 1, FR_VCHK = 4, FR_VEQ = 8, FR_UPID = 8 };

struct Frag {
    uint64_t entry;      // first entry in its pool
    uint32_t msg;        // global message index (K_BATCH in chosen lists: batch index)
    uint16_t count;      // entries in this bucket run (<= 256)
    uint8_t start;       // bucket-local slot of the first entry (dense runs)
    uint8_t flags;       // FR_DENSE | kind << 4
};
static_assert(sizeof(Frag) == 16, "Frag is 16 bytes");

// snapshot output record (12 bytes): an entry of a granted PREPARE_REPLY
// (kind 0: FilterAcceptedValues, multi/paxos.cpp:902-922) or of a
// promise-quorum merged map (kind 1: :1047-1105), by reference to the resident
// trace — the host resolves iid, tag and Value (fetch_results):
//   kind 0: ref = global index of the fragment that fixed the slot, aux = slot
//           in its bucket (the entry at that slot: iid, Value; its message's
//           ballot, member: the entry's proposal id)
//   kind 1: ref = PREPARE_REPLY entry index (r_iid, r_pid, r_val), aux = OUT_K1
//           (| OUT_CMT: the node had committed the instance by then — not
//           adoptable by the phase-2 batch, multi/paxos.cpp:1091)
struct OutRec {
    uint32_t msg;
    uint32_t ref;
    uint32_t aux;
};
static_assert(sizeof(OutRec) == 12, "OutRec is 12 bytes");
constexpr uint32_t OUT_K1 = 0x100;
constexpr uint32_t OUT_CMT = 0x200;
// kind 0 run record (k_plan_list): slots aux & 0xFF .. + (aux >> OUT_RUN_SHIFT) of the
// fragment's bucket, all fixed by fragment `ref` (the host expands it); kind 1 run record (a
// quorum's merged map, k_apply): slot aux & 0xFF + i takes PREPARE_REPLY entry ref + i
constexpr uint32_t OUT_RUN = 0x400;
constexpr uint32_t OUT_RUN_SHIFT = 16;
// host form of a snapshot record
struct OutEnt {
    uint32_t msg;
    uint32_t kind;                  // bit 0: kind; bit 1: OUT_CMT
    uint64_t iid;
    uint64_t ballot;
    uint64_t handle;
};

// snapshot output: out_subs (a power of two <= OUT_SUBS, 64 by default; env
// MPX_OUT_SUBS at create) sub-buffers with their own cursors, a wave appends to
// sub (wave id mod out_subs) — the host sorts records by message and iid, so
// their order is free and the append needs no single global atomic
constexpr uint32_t OUT_SUBS = 4096;
constexpr uint32_t GP_WORDS = 8;
constexpr uint32_t OUT_STRIDE = 16;

// violation record written once (first code wins) + count
struct DevViolation {
    unsigned long long code, node, seq, iid, count;
};

// Everything a kernel needs, passed by value (kernarg).
struct DevView {
    uint32_t N, quorum, NB, semantics;
    uint32_t walk_all;              // a step walks every pair like a digested run (MPX_STEP_WALK=1)
    uint32_t digest;                // 1: accumulate the order-independent state / chosen digests
                                    //    (mpx_run; verification only, mpx_step leaves them 0)
    uint64_t shard_begin, shard_len;
    uint64_t num_msgs;
    // messages
    const uint8_t *m_type;
    const uint32_t *m_src;
    const uint64_t *m_ballot;
    const uint64_t *m_aux;
    const uint64_t *m_ent;
    const uint32_t *m_cnt;
    const uint32_t *m_node;         // node of each message
    const uint64_t *node_off;       // N+1
    const uint8_t *pair_gp;         // per (bucket, node) pair: 1 = not lean, on k_apply's work list
    uint8_t *m_flags;
    uint64_t *m_maxseen;
    // member semantics
    uint32_t *m_gate;               // per message, see G_* (written by k_gate_*)
    const uint64_t *e_pid;          // per ACCEPT / LEARN entry: its proposal id
    const uint64_t *ep_amask;       // per epoch: acceptor set
    const uint64_t *ep_pmask;       // per epoch: proposer set
    const uint32_t *ep_ver;         // per epoch: NodeImpl::version_
    uint32_t num_epochs;
    const uint32_t *m_ver;          // per message: PREPARE / ACCEPT version, E_EPOCH epoch
    const uint64_t *ee_off;         // N + 1: each node's E_EPOCH messages in ee_msg
    const uint32_t *ee_msg;
    uint32_t *ee_state;             // per marker: the node's roles after it (k_gate_epochs, EE_*)
    const uint32_t *sc_ver;         // per scan record: its message's version
    const uint64_t *sc_off;         // N + 1: each node's scan-stream range
    uint64_t num_sc;                // scan records
    // header scan over the scan stream (SC_*): chunks of SCAN_CHUNK records per node
    uint8_t *sc_type;               // member: types / keys finished by k_gate_scan
    uint64_t *sc_key;
    const uint32_t *sc_idx;         // global message index of the record
    uint32_t num_chunks;
    const uint32_t *chunk_node;
    const uint64_t *chunk_beg;      // scan-stream index of chunk start
    const uint64_t *chunk_end;
    const uint32_t *node_chunk_off; // N+1
    uint64_t *chunk_agg;            // 2 per chunk: pmax, smax
    uint64_t *chunk_carry;          // 2 per chunk: exclusive prefix (k_scan_node)
    uint32_t scan_node_pass;        // 1: a node has > SCAN_INLINE_CHUNKS chunks, carry-in from k_scan_node
    uint32_t scan_chunk;            // records per header-scan chunk (SCAN_CHUNK or SCAN_CHUNK_SMALL)
    uint32_t seq;                   // this launch's sequence number (from 1)
    uint64_t *node_scal;            // 2 per node: promised, max_seen
    // pools
    const uint64_t *e_val;
    const uint8_t *e_slot;
    const uint64_t *r_pid;
    const uint64_t *r_val;
    const uint8_t *r_slot;
    const uint64_t *g_a;
    const uint64_t *g_b;
    // fragment lists
    const uint64_t *f_off;          // N*NB+1, pair q = bucket * N + node
    const Frag *frags;
    uint64_t num_gp;                // pairs for the general apply kernel
    uint64_t num_gp_simple;         // ... the first of them: no snapshot events, no promise-reply runs (multi)
    uint64_t num_gp_snap;           // ... then up to here: no promise-reply runs (PREPARE events only)
    const uint64_t *gp_list;        // general-apply work items, GP_WORDS each: the pair's fragment CSR
                                    // range, its event CSR range, the pair q (one coalesced load per item)
    // list plan path (k_plan_list): the pairs it cannot describe by one plan word are
    // appended here (GP_WORDS per item, as gp_list) for k_apply; gp_dyn_n counts them
    uint64_t *gp_dyn;
    unsigned long long *gp_dyn_n;
    // ... and the pairs it describes by 5..PLAN_XSEG segments: {pair, split points, values}
    // (EXT_WORDS per item) for k_store_ext; gp_ext_n counts them
    uint64_t *gp_ext;
    unsigned long long *gp_ext_n;
    // ... and the planned pairs where a commit / learn (member: also an accept) meets a committed
    // segment through another message's entries: {first run, end run, pair} (CHK_WORDS per item)
    // for k_commit_check, which compares their Values slot by slot; gp_chk_n counts them
    uint64_t *gp_chk;
    unsigned long long *gp_chk_n;
    // ... and (member) the pairs it listed only for having more than PLAN_XSEG_MEMBER segments: their
    // pair indices, planned again with up to 16 by k_plan_list<..., RETRY>; gp_rt_n counts them
    uint64_t *gp_rt;
    unsigned long long *gp_rt_n;
    const uint64_t *ev_off;         // N * NB + 1: snapshot events per pair (ingest.cpp), message order
    const uint32_t *ev_msg;
    // promise-quorum chunks (k_prop_chunk / k_prop_node): PROP_CHUNK records of one
    // node's pl list each, CSR per node; outputs: first round head, state after
    uint32_t num_pc, pc_multi;      // pc_multi: some node has more than one chunk (k_prop_node runs)
    const uint32_t *pc_node, *pc_node_off;
    const uint64_t *pc_beg, *pc_end;
    uint32_t *pc_head;
    uint64_t *pc_state;             // 3 words per chunk: ballot, promise mask, preparing | known << 1
    const uint64_t *ev_aux;         // per event: PREPARE: first range (g_a index) meeting the bucket | count << 32
                                    // (8 bits) | one range: its bucket-local [lo << 40, hi << 49) | EVX_ONE
    const uint64_t *pl_off;         // N+1
    const uint32_t *pl_msg;
    // batches
    uint32_t num_batches;
    const uint32_t *b_msg;
    const uint32_t *b_pstart;
    const uint64_t *b_rep_off;
    const uint32_t *b_rep;
    const uint64_t *b_rbal;         // per vote-list entry: the reply's ballot
    uint32_t *b_rsrc;               // ... its acceptor (low 16 bits, clamped) | member: (epoch + 1) << 16 (k_gate_votes)
    const uint64_t *b_bal;          // per batch: the ballot of its proposer round (0: none)
    uint32_t *b_chosen;             // global msg index of the quorum reply, NONE32
    const uint64_t *cf_off;         // NB+1
    const Frag *cfrags;
    // state
    void *st;                       // one slot per (node, instance), node-major, slot_w bytes each
    uint32_t slot_w;                // 1 when every pair / bucket has <= MAX_PAIR_FRAGS_1 fragments, else 2
    uint8_t *st_valid;              // per (node, bucket) pair: bucket * N + node (sv_idx)
    // chosen log: row N of st (per instance: the bucket's chosen fragment (cf_off) + 1)
    uint8_t *chosen_valid;          // per bucket
    const uint64_t *f_pid;          // per run: its entries' common proposal id (FR_UPID promise-reply runs), else 0
    const uint64_t *frag_w1;        // frags[i]'s second word (message, count, start, flags): k_plan's
                                    // half of the descriptor, streamed without the entry words
    uint64_t *plan;                 // (N + 1) * NB: the segments k_store writes over a whole (row, bucket) (plan_idx),
                                    // rows 0..N-1 state, row N chosen log; PLAN_SKIP = not by k_store
    uint32_t chosen_static;         // every bucket's chosen-log runs pass plan_chosen's static test (<= 4
                                    // disjoint dense runs, a whole bucket): the plan step needs no k_chosen
    uint32_t any_vchk;              // some run carries FR_VCHK: k_commit_check has pairs (else not launched)
    uint32_t *fast_rest;            // [0]: pairs k_plan leaves to k_apply_fast (0: it exits at once);
                                    // [1]: k_chosen's last-workgroup ticket
    uint32_t *store_dummy;          // 64 KiB sink for k_store's skipped (row, bucket) stores
    // outputs
    OutRec *out;
    unsigned long long *out_cursor;  // OUT_SUBS cursors, one per 128-byte line (stride OUT_STRIDE words)
    uint64_t out_cap;               // records per sub-buffer: sub s owns out[s * out_cap .. (s + 1) * out_cap)
    uint32_t out_subs;              // sub-buffers in use (power of two <= OUT_SUBS)
    unsigned long long *partials;   // 8 words per apply workgroup, then chosen workgroups
    DevViolation *viol;             // this launch's first-violation record (double-buffered: reset_state
    DevViolation *viol_next;        //   clears the next launch's, which nothing writes in this one)
    unsigned long long *summary;    // 64 words
    // incremental windows (MPX_FLAG_INCREMENTAL): the trace arrays above
    // hold one window, the state below carries across windows — as values, not as
    // references to runs of earlier windows (which are gone)
    uint32_t window;                // 1: a window run (k_apply_win, k_chosen_win, carried scan / rounds / votes)
    uint64_t *s_bal, *s_val;        // per (node, instance), node-major: the entry's ballot; handle | W_PRESENT |
                                    //   W_COMMITTED (0: none)
    uint64_t *p_pid, *p_val;        // per (node, instance): the promise round's pre-accepted entry (proposal id;
                                    //   handle | W_PRESENT), valid while p_round of its pair is the node's round
    uint64_t *p_round;              // per pair (sv_idx): ballot of the round p_* belong to (0: none)
    uint64_t *c_val;                // per instance: the chosen log (handle | W_PRESENT)
    uint64_t *scal_base;            // 2 per node: promised / max_seen scan keys before the window (member: with
                                    //   the acceptor incarnation << SEG_SHIFT)
    uint64_t *scal_key;             // ... after it (the scan's unmasked keys; node_scal holds the readback)
    const uint64_t *prop_in;        // 3 per node: the round before the window (ballot, promise mask, preparing)
    uint64_t *prop_out;             // ... after it (k_prop_node)
    const uint32_t *b_gid;          // per batch of the window's list: its global id
    uint64_t *g_mask;               // per global batch: accepted_ (acceptor mask)
    uint8_t *g_done;                // per global batch: bit 0 its votes reached quorum in an earlier window;
                                    //   bit 1 (member) its proposer's batches were cleared (k_gate_votes)
    const uint32_t *b_node;         // per batch of the window's list: its node
    const uint32_t *ee_init;        // member, per node: its roles before the window (EE_* state; genesis
                                    //   from epochs[0] for the first)
    uint32_t *ee_out;               // ... after it (k_gate_epochs)
    const uint8_t *gp_base;         // per work item: earlier windows left state in the pair
    const uint32_t *cb_list;        // buckets with chosen-log runs in the window
    uint32_t num_cb;
    OutEnt *outv;                   // window snapshot records, values inline
    unsigned long long *outv_n;
    uint64_t outv_cap;
};

// k_plan / k_apply_fast take a pair only when its bucket's CSR offsets (N+1,
// plus two chosen-log offsets) fit one wave's lanes and the pair has at most
// FAST_MAX_FRAGS fragments (its per-slot path: lane i = fragment i); the rest
// go to k_apply's work list (kernels.hip, ingest.cpp, engine.cpp)
constexpr uint32_t FAST_MAX_NODES = 61;
constexpr uint32_t FAST_MAX_FRAGS = 63;
// A *lean* pair is one k_plan turns into one plan word (kernels.hip): at most
// PLAN_FRAGS runs, all dense ACCEPT / COMMIT runs, at most three distinct run
// boundaries inside the bucket (four segments of equal slots), no instance under
// two COMMIT runs (a re-commit's Value check), a whole bucket, no snapshot
// events; ingest.cpp / mpx_load_clean_device put every other pair on the work
// list of the general k_apply (pair_gp = 1).  All static: no run-time flag enters.
constexpr uint32_t PLAN_FRAGS = 8;
// pair_gp of the work list's pairs: GP_LIST = no promise-reply runs (k_plan_list plans
// them or lists them for k_apply), GP_ROUNDS = promise rounds (k_apply AM_FULL only);
// member: every pair with runs is on the work list
enum : uint8_t { GP_LIST = 1, GP_ROUNDS = 2 };
// k_plan_list: runs per pair it plans (walked from LDS) and runs a wave stages
constexpr uint32_t MPLAN_FRAGS = 16;
constexpr uint32_t MPLAN_LDS = 1024;
constexpr uint32_t PLAN_XSEG = 8;            // k_plan_list: up to 8 segments, 32 runs per pair
constexpr uint32_t PLAN_XFRAGS = 32;
#ifndef MPX_PLAN_XSEG_MEMBER
#define MPX_PLAN_XSEG_MEMBER 8
#endif
// member k_plan_list: segments and waves per SIMD (A/B knobs: 16 segments need 215 VGPRs, 2 waves —
// contended C5 1.791 vs 1.515 ms at 8 / 4, profiles/r06_ab_member_plan16_2waves.txt)
constexpr uint32_t PLAN_XSEG_MEMBER = MPX_PLAN_XSEG_MEMBER;
#ifndef MPX_PLAN_WAVES_MEMBER
#define MPX_PLAN_WAVES_MEMBER 4
#endif
constexpr int PLAN_WAVES_MEMBER = MPX_PLAN_WAVES_MEMBER;
// member: the 9..16-segment retry of the pairs the plan lists for their segment count (k_plan_list
// RETRY, an A/B build variant: contended C5 2.405 vs 1.515 ms, C5 0.525 vs 0.387 ms without it — the
// retry kernel spills 1.4 KB per lane at 16 segments and its launch sits on the plan -> listed-walk
// chain; profiles/r06_ab_member_retry.txt)
#ifndef MPX_PLAN_RETRY
#define MPX_PLAN_RETRY 0
#endif
constexpr bool PLAN_RETRY = MPX_PLAN_RETRY != 0;
constexpr uint32_t PLAN_RETRY_SEG = 16;
constexpr uint32_t CHK_WORDS = 3;           // gp_chk items
constexpr uint32_t EXT_WORDS = 5;
constexpr uint32_t EXT_LEGACY = 0xFF;       // k_store_ext item of <= 8 segments (9-bit split points)
// the distinct run boundaries inside (0, 256), sorted into s[0..2] (BS = unused);
// false once a fourth one appears
MPX_HD inline bool plan_add_split(uint32_t x, uint32_t (&s)[3])
{
    if (x == 0 || x >= BS || x == s[0] || x == s[1] || x == s[2]) return true;
    if (s[2] != BS) return false;
    if (x < s[0]) { s[2] = s[1]; s[1] = s[0]; s[0] = x; }
    else if (x < s[1]) { s[2] = s[1]; s[1] = x; }
    else s[2] = x;
    return true;
}
// the run shape of a lean pair, from its runs' second descriptor words
MPX_HD inline bool plan_shape_ok(const uint64_t *w1, uint32_t len)
{
    if (!len || len > PLAN_FRAGS) return false;
    uint32_t sp[3] = {BS, BS, BS};
    for (uint32_t k = 0; k < len; ++k) {
        const uint32_t fl = (uint32_t)(w1[k] >> 56), kind = fl >> 4;
        const uint32_t cnt = (uint32_t)(w1[k] >> 32) & 0xFFFF, st0 = (uint32_t)(w1[k] >> 48) & 0xFF;
        if (!(fl & FR_DENSE) || (kind != K_ACCEPT && kind != K_COMMIT)) return false;
        if (!plan_add_split(st0, sp) || !plan_add_split(st0 + cnt, sp)) return false;
        if (kind == K_COMMIT)
            for (uint32_t j = 0; j < k; ++j) {
                const uint32_t c2 = (uint32_t)(w1[j] >> 32) & 0xFFFF, s2 = (uint32_t)(w1[j] >> 48) & 0xFF;
                if ((w1[j] >> 60) == K_COMMIT && st0 < s2 + c2 && s2 < st0 + cnt) return false;
            }
    }
    return true;
}
constexpr uint32_t APPLY_WGS_MAX = 2048;
constexpr uint32_t CHOSEN_WGS_MAX = 1024;
// partial counter slots
enum { PC_A = 0, PC_L, PC_P, PC_Q, PC_C, PC_DSTATE, PC_DCHOSEN, PC_MSGS };
// summary words (mpx_allgather_summary)
enum { SW_C = 0, SW_P, SW_A, SW_L, SW_MSGS, SW_V, SW_DCHOSEN, SW_DSTATE, SW_DSCAL, SW_Q,
       SW_NODE_SCAL = 16 };   // then promised, max_seen per node (up to 24 nodes summarised)

MPX_HD inline uint64_t mix64(uint64_t x)
{
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    x ^= x >> 31; return x;
}
MPX_HD inline uint64_t state_digest(uint32_t node, uint64_t iid, uint64_t kind,
                                                 uint64_t ballot, uint64_t handle)
{
    return mix64(mix64(mix64(iid + (uint64_t)node * 0x9E3779B97F4A7C15ull) ^ ballot) ^
                 (handle + kind * 0xD6E8FEB86659FD93ull));
}
MPX_HD inline uint64_t chosen_digest(uint64_t iid, uint64_t handle)
{
    return mix64(mix64(iid) ^ handle);
}
MPX_HD inline uint64_t scalar_digest(uint32_t node, uint64_t promised, uint64_t max_seen)
{
    return mix64(mix64((uint64_t)node * 0x9E3779B97F4A7C15ull ^ promised) ^ max_seen);
}

// kernels (kernels.hip); every launcher queues on `stream`, returns hipError_t as int
// k_plan_store8 (kernels.hip) in place of k_plan + k_store8 on the C4 shape (A/B build flag)
#ifndef MPX_PLAN_STORE
#define MPX_PLAN_STORE 1
#endif
constexpr bool PLAN_STORE = MPX_PLAN_STORE != 0;
struct LaunchGeom { uint32_t apply_wgs, chosen_wgs, store_wgs, ps_wgs; };
// ev (hipEvent_t, each may be null): begin, apply phase start (after the header
// scan / quorum kernels), after the plan / store / fast-apply kernels, after the
// general k_apply, end
// a second stream and two events (fork / join, timing off) for kernels of a run that may
// overlap others of it; nullptr: everything on `stream`
// side streams of a run (nullptr: one stream): stream2 takes the promise-round pairs (after the
// header kernels), stream3 the chosen log (after the plan of its buckets) and the pairs k_plan_list
// lists (after it); both joined before the summary
struct LaunchSide { void *stream2, *fork, *join, *stream3, *fork3a, *fork3b, *join3; };
int launch_run(const DevView &v, void *stream, LaunchGeom g, void *const ev[5], LaunchSide side);
// the run's last kernel is the store, the step summary folded into it (the clean multi
// plan path, C4): launch_run then records neither the general-apply nor the end event
bool run_ends_with_store(const DevView &v);
// the grids of a trace of N nodes x NB buckets on a device with num_cus CUs
LaunchGeom launch_geometry(uint32_t N, uint64_t NB, uint32_t num_cus);
// readback: count slots of node `node` (node >= N: the chosen log) from shard
// offset l0 -> out, 2 words each {ballot, PRESENT | COMMITTED? | handle}
// (chosen: {0, PRESENT | handle}); unwritten buckets read as empty
int launch_decode(const DevView &v, void *stream, uint32_t node, uint64_t l0, uint64_t count, uint64_t *out);
// in-order executor of one node: out == nullptr queues frontier / count / scan
// into aux (2 NB + 2 words: frontier, counts, offsets, total); then with out
// (total words) the scatter of the executed handles in instance order
int launch_exec(const DevView &v, void *stream, uint32_t node, unsigned long long *aux, uint64_t *out);
// digests of the resident state / chosen log -> out[0], out[1] (16 bytes, device)
int launch_state_digest(const DevView &v, void *stream, unsigned long long *out);
// out[i] = second word of frags[i], i < n (once per trace load)
int launch_frag_w1(const Frag *frags, uint64_t *out, uint64_t n, void *stream);
// Phase-2 decisions (mpx_read_decisions, kernels.hip k_decide*): E promise-quorum
// events (node, message) over the shard, in four launches —
//   pass 0: xmax[e] = 1 + the highest instance the event's node had committed
//           before the event (0: none);
//   pass 1: (xend[e] = where the noop fill ends; the adopted instances of event
//           e sorted in ad_li[ad_off[e] .. ad_off[e + 1])) per 256-instance block
//           below xend the number of instances to fill -> blk_cnt[blk_off[e] + block];
//   scan:   per event, blk_cnt -> exclusive block offsets in place, total -> ev_total[e];
//   pass 2: the instances to fill, in instance order -> noop_li[ev_base[e] + ...].
struct DecideArgs {
    uint32_t E;
    const uint32_t *ev_node, *ev_msg;
    unsigned long long *xmax;
    const uint64_t *xend, *ad_off, *blk_off, *ev_base;
    const uint32_t *ad_li;
    uint32_t *blk_cnt, *noop_li;
    uint64_t *ev_total;
    uint64_t max_blocks;            // blocks of the widest event (pass 1 / 2 grid)
};
int launch_decide(const DevView &v, void *stream, uint32_t pass, const DecideArgs &a);
// Commit reliability (mpx_read_commits, kernels.hip k_commits):
// L reply lists, one per (node, commit id named by its COMMIT_REPLYs), each the
// replies in the node's processing order with their learner ids beside them;
// per node the messages at which its CommittingValues were created (cm_pos,
// CSR cm_off, commit id c = position c - 1).  Per list: the message of the reply
// that completed the replied set (NONE32: open) and the final learner mask.
struct CommitArgs {
    uint32_t L;
    const uint64_t *cr_off, *cr_id, *cm_off;
    const uint32_t *cr_msg, *cr_src, *cr_node, *cm_pos;
    uint32_t *ret;
    unsigned long long *mask;
};
int launch_commits(const DevView &v, void *stream, const CommitArgs &a);
// Learn reliability (member; mpx_read_learns, kernels.hip k_learns): per
// learn its events in processing order — LEARN_REPLYs and the AcceptorsChanged calls of
// its proposer while it is open — as ev_a = pos << 32 | kind << 24 | add << 23 |
// lcount << 8 | node (kind 0 reply: node = learner, lcount = |learners_|; kind 1
// AcceptorsChanged: add, node), ev_m = the node's acceptor mask at the event (after the
// change); facc: the learn has a learning_values_for_acceptors_ entry; end: the record
// that drops it (NONE32: none)
enum : uint32_t { LEV_REPLY = 0, LEV_ACC = 1 };
struct LearnArgs {
    uint32_t L;
    const uint64_t *ev_off, *ev_a, *ev_m;
    const uint8_t *facc;
    const uint32_t *end;
    uint32_t *applied, *retired, *ended;
    unsigned long long *mask;
};
int launch_learns(const DevView &v, void *stream, const LearnArgs &a);
// f_off / cf_off: host-computed prefix counts (per pair, per bucket), read by the generator
int launch_gen_clean(void *stream, uint32_t N, uint64_t K, uint64_t k0, uint64_t sb, uint64_t se,
                     uint64_t G0, uint64_t G1, uint64_t ballot, uint64_t B, uint32_t NB,
                     uint8_t *type, uint32_t *src, uint64_t *bal, uint64_t *aux, uint64_t *ent, uint32_t *cnt,
                     uint32_t *node, uint64_t *e_val, Frag *frags, uint64_t *f_off, uint32_t *b_msg,
                     uint32_t *b_pstart, uint64_t *b_rep_off, uint32_t *b_rep, uint64_t *cf_off, Frag *cfrags,
                     uint8_t *sc_type, uint64_t *sc_key, uint32_t *sc_idx, uint64_t *b_rbal, uint32_t *b_rsrc,
                     uint64_t *b_bal);

}  // namespace mpx
