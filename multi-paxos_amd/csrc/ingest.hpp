// ingest.hpp — host side of mpx_submit: wire decode into SoA, value table,
// instance bucketing into fragments.
#pragma once
#include <atomic>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "mpx.h"

#include "mpx_internal.hpp"

namespace mpx {

// Interned reference Values: handle -> canonical FillValue bytes
// (multi/paxos.cpp:556-598) and what StateMachine::Execute receives.  Sharded by handle, each
// shard behind its own lock, so the node-parallel decode threads intern into one table (no
// per-thread tables merged afterwards); the readers (encode, exec_payload) run when no decode
// is in flight.
struct ValueTable {
    struct Rec { const char *p; uint32_t len; uint32_t exec_off; uint32_t exec_len; };   // p == nullptr: absent
    static constexpr uint32_t SHARDS = 64;
    static constexpr size_t BLOCK = 1 << 20;
    static constexpr uint64_t EMPTY = ~0ull;            // (no group key: proposer < 2^14 keeps bits 62-63 clear)
    // A proposer numbers its Values 1, 2, 3, ... and a batch's instances carry consecutive ids, so
    // the records sit in groups of 16 consecutive handles (h >> 4): a section's lookups walk a
    // group's 384 contiguous bytes instead of one random slot per Value.  Groups are found through
    // an open-addressing table (at most half full) of {group key, group} and allocated in chunks.
    static constexpr uint32_t GSH = 4, GN = 1u << GSH;
    struct Group { Rec r[GN]; };
    struct GSlot { uint64_t key; Group *g; };
    struct Shard {
        std::mutex mu;
        std::vector<GSlot> slot;
        size_t count = 0;                                // groups
        std::vector<std::unique_ptr<Group[]>> gchunks;   // group storage: stable addresses
        size_t gused = 0;                                // groups used in the last chunk
        std::vector<std::unique_ptr<char[]>> blocks;     // canonical bytes: stable addresses, no regrowth copies
        size_t used = BLOCK;                             // bytes used in the last block
        // the slot array's current address and mask, published under mu for prefetch_slot
        std::atomic<const GSlot *> sp{nullptr};
        std::atomic<size_t> smask{0};
        const Rec *find(uint64_t h) const;
        Rec *insert(uint64_t h, bool &fresh);
        void release()
        {
            slot.clear(); slot.shrink_to_fit(); count = 0; gchunks.clear(); gused = 0;
            sp.store(nullptr, std::memory_order_relaxed); smask.store(0, std::memory_order_relaxed);
        }
    };
    static uint32_t shard_of(uint64_t h) { return (uint32_t)(((h >> GSH) * 0x9E3779B97F4A7C15ull) >> 58); }
    std::unique_ptr<Shard[]> sh{new Shard[SHARDS]};
    // synthetic resolver for device-generated clean traces: value_id v of
    // proposer 0 is the decimal string of v-1
    bool synthetic_clean = false;
    // member Value_m codec (member/paxos.cpp:321-408): + cb, membership list
    bool member = false;
    // section id ranges handed to the submit calls' SectionCaches (ids unique over the engine)
    std::atomic<uint64_t> sections{0};
    // parse one Value; returns bytes used (>0) or a negative MPX_E_* code; *mem: a member
    // membership Value (a change list instead of a payload)
    long parse(const uint8_t *p, size_t avail, uint64_t *handle, bool *mem = nullptr);
    bool encode(uint64_t handle, std::string &out) const;    // canonical bytes
    // what StateMachine::Execute / Apply receives; false for unknown handles
    // and for member membership Values (applied by ChangeMemberships instead)
    bool exec_payload(uint64_t handle, std::string &out) const;
    void clear()
    {
        for (uint32_t k = 0; k < SHARDS; ++k) {
            Shard &x = sh[k];
            x.release(); x.blocks.clear(); x.used = BLOCK;
        }
        synthetic_clean = false;
    }
    // a handle with no bytes yet: the payload-free Value it names (mpx_submit_soa)
    int plain(uint64_t handle);
    // the canonical bytes of handle h, interned (thread-safe): MPX_E_VALUE when h already names
    // other bytes (a Value is named by (proposer, value_id), multi/paxos.cpp:439)
    int intern(uint64_t h, const char *b, uint32_t len, uint32_t exec_off, uint32_t exec_len);
    // a run of Values whose canonical bytes are their wire bytes, interned with one lock per run of
    // the same shard (a section's consecutive handles share groups, hence shards)
    struct Pending { uint64_t h; const char *b; uint32_t len, exec_off, exec_len; };
    int intern_batch(const Pending *v, size_t n);
    const Rec *find(uint64_t h) const { return sh[shard_of(h)].find(h); }
    // prefetch h's home slot (key and record): a section's Values are looked up one after another,
    // each a likely cache miss, so the decode touches them all first (no lock: a stale address
    // after a concurrent growth only wastes the prefetch)
    void prefetch_slot(uint64_t h) const;
};

// One submit call's value sections (the entry lists of ACCEPT / COMMIT / P_BATCH bodies): a
// broadcast reaches every node with the same bytes, and a batch's ACCEPT, COMMIT and P_BATCH carry
// the same list.  The first decode thread to claim a section interns its Values (in batches, one
// lock per shard run) and keeps the sorted entries as the section's Result; a thread that meets
// the section later copies them, and one that meets it while it is still being decoded reads its
// entries off the wire (skim: the handle is (proposer, noop, value_id) itself) — no thread waits
// for another.  Every record notes its section's id (NodeStream::sec), which build_trace's entry
// pool takes as list equality.  Sections are compared in full (the key only picks candidates)
// and point into the submitted buffers: the set lives for one submit call.
struct SectionCache {
    struct Result {
        const uint8_t *b; size_t len; bool with_pid;
        uint64_t id;                                      // the section's identity (NodeStream::sec)
        std::atomic<int> ready{0};
        int rc = MPX_OK;                                  // the section's decode error (reported in record order)
        std::vector<uint64_t> iid, pid, val;              // sorted by iid (sort_entries)
        std::vector<std::pair<uint64_t, uint32_t>> memh;  // member: membership Values, offset in the section
        size_t n_all = 0;
        bool dup = false;
    };
    static constexpr uint32_t SHARDS = 64;
    struct Shard { std::mutex mu; std::unordered_multimap<uint64_t, std::unique_ptr<Result>> m; };
    std::unique_ptr<Shard[]> sh{new Shard[SHARDS]};
    bool share = true;                                    // (tests: false = owners keep no Result, others skim)
    uint64_t id_base = 0;                                 // section ids: id_base + k (ValueTable::sections)
    std::atomic<uint64_t> next_id{1};
    // the section's Result; own = the caller is the first with these bytes (it decodes them)
    Result *claim(const uint8_t *b, size_t len, bool with_pid, bool &own);
};

// Membership discovered at run time (MPX_FLAG_LEARN_EPOCHS, member semantics): every node's
// Learner applies learned Values in instance order (Learner::OnLearn, member/paxos.cpp:1040-1053;
// a LEARN is handled whatever the node's roles, Loop :771-772), and applying a membership Value
// runs NodeImpl::ChangeMemberships (Learner::Apply :1062-1073, :1864-1964).  Per node: the apply
// frontier (next_id_to_apply_), the instances learned above it with their first Value (insert:
// the first learned Value sticks, :1040), the node's membership view, and the epochs it stepped
// through.  Epoch k = the view after the k-th membership Value in instance order; every node
// applies the same Values in the same order (one chosen Value per instance), so the per-node
// lists agree on their common prefix (checked when they are merged, mpx_engine::epochs).
struct EpochLearn {
    using Changes = std::vector<std::pair<uint32_t, uint32_t>>;   // {node, MembershipChangeType}*
    struct Learned { bool mem; Changes ch; };
    uint64_t front = 0;
    std::map<uint64_t, Learned> above;            // learned, not yet applied: iid -> (membership?, its changes)
    mpx_epoch view{};                             // NodeImpl's version_ / acceptors_ / proposers_ / learners_
    std::vector<mpx_epoch> steps;                 // epochs 1.. this node reached
};

// One node's decoded receive stream (submission order).
struct NodeStream {
    std::vector<uint8_t> type;
    std::vector<uint32_t> src;
    std::vector<uint64_t> ballot, aux, ent;
    std::vector<uint32_t> cnt;
    std::vector<uint64_t> e_iid, e_val;           // ACCEPT / COMMIT / P_BATCH entries (in shard)
    std::vector<uint64_t> e_pid;                  // member: their proposal ids
    std::vector<uint32_t> ver;                    // member: PREPARE / ACCEPT version, E_EPOCH epoch
    std::vector<uint64_t> r_iid, r_pid, r_val;    // PREPARE_REPLY entries (in shard)
    std::vector<uint64_t> g_a, g_b;               // PREPARE ranges (all), sorted by start
    std::vector<uint8_t> part;                    // 1: the record carried entries, none in the shard
    std::vector<uint64_t> sec;                    // its value section's id (SectionCache; 0: none / unknown):
                                                  //   equal ids = byte-equal sections = equal entry lists
    // (keeps the capacity: a live engine decodes window after window into the same streams)
    void clear()
    {
        type.clear(); src.clear(); ballot.clear(); aux.clear(); ent.clear(); cnt.clear(); e_iid.clear(); e_val.clear();
        e_pid.clear(); ver.clear(); r_iid.clear(); r_pid.clear(); r_val.clear(); g_a.clear(); g_b.clear(); part.clear();
        sec.clear();
    }
};

struct IngestViolation { uint64_t code = 0, node = 0, seq = 0, iid = 0, count = 0; };

// One node's records to decode: offs[0 .. cnt] index bytes (an MPXT stream, or a slice of one).
struct StreamSlice { const uint64_t *offs = nullptr; const uint8_t *bytes = nullptr; uint64_t cnt = 0; };

// Incremental runs (MPX_FLAG_INCREMENTAL): what build_trace needs from
// the windows before the current one to list the current window's snapshot events and
// vote lists without its history.  O(nodes + buckets with state + live batches).
struct WindowCarry {
    bool on = false;
    uint64_t batches = 0;                                        // batches of earlier windows (global ids 0..)
    std::vector<std::unordered_map<uint64_t, uint32_t>> live;    // per node: accept id -> global batch id
    std::vector<uint64_t> round_ballot;                          // per node: its last P_START's ballot (0: none)
    std::vector<std::vector<uint8_t>> state_b;                   // per node, per bucket: a run of the node met it
    std::vector<int64_t> maxb;                                   // per node: the highest such bucket (-1: none)
    std::vector<std::vector<uint64_t>> round_b;                  // per node: buckets with promise-reply runs since
                                                                 //   its last P_START
    std::vector<uint64_t> b_bal;                                 // per global batch: its round's ballot
    std::vector<uint64_t> b_aid;                                 // per global batch: its accept id (P_BATCH aux)
    std::vector<uint32_t> markers;                               // member, per node: E_EPOCH markers so far
    // per global batch still live and not chosen: its entries {iid, handle}, for the
    // chosen log when a later window completes its votes
    std::unordered_map<uint32_t, std::vector<std::pair<uint64_t, uint64_t>>> b_ents;
    void init(uint32_t N, uint64_t NB)
    {
        on = true; batches = 0;
        live.assign(N, {}); round_ballot.assign(N, 0); state_b.assign(N, std::vector<uint8_t>(NB, 0));
        maxb.assign(N, -1); round_b.assign(N, {}); b_bal.clear(); b_aid.clear(); b_ents.clear(); markers.assign(N, 0);
    }
};

// Flattened, bucketed host copy of the trace — mirrors the device arrays.
struct HostTrace {
    uint32_t N = 0, NB = 0;
    uint64_t shard_begin = 0, shard_len = 0;
    std::vector<uint8_t> m_type;
    std::vector<uint32_t> m_src, m_cnt, m_node;
    std::vector<uint64_t> m_ballot, m_aux, m_ent;
    std::vector<uint64_t> node_off;
    std::vector<uint32_t> m_seq;                    // record index in its node's submitted stream
    // P_PROPOSE records (the proposers' client values: host bookkeeping only, no device work):
    // per node [prop_off[n], prop_off[n + 1]) of prop_seq, their record indices; they are not in
    // the device's message arrays
    std::vector<uint64_t> prop_off;
    std::vector<uint32_t> prop_seq;
    uint64_t dropped = 0;                           // records of other shards left out (header sharding)
    uint64_t part_dropped = 0;                      // ... of them, records whose entries all lie in other shards
    std::vector<uint32_t> chunk_node, node_chunk_off;
    uint32_t scan_chunk = SCAN_CHUNK;               // records per header-scan chunk (scan_chunk_for)
    std::vector<uint64_t> chunk_beg, chunk_end;
    std::vector<uint8_t> sc_type;                   // header-scan stream (mpx_internal.hpp SC_*)
    std::vector<uint64_t> sc_key;
    std::vector<uint32_t> sc_idx;
    std::vector<uint8_t> m_flags0;                  // static message flags (bad source)
    // member semantics (gated on the device, kernels.hip k_gate_*): per message its
    // version (PREPARE / ACCEPT) or epoch (E_EPOCH); per node its E_EPOCH messages;
    // per scan record its version; per node its scan-stream range
    std::vector<uint32_t> m_ver, ee_msg, sc_ver;
    std::vector<uint64_t> ee_off, sc_off;
    std::vector<uint64_t> e_val, e_iid, e_pid, r_pid, r_val, r_iid, g_a, g_b;
    std::vector<uint8_t> e_slot, r_slot;
    bool any_sparse = false;
    std::vector<uint64_t> f_off;
    std::vector<Frag> frags;
    std::vector<uint64_t> f_pid;                    // per run: the common proposal id of an FR_UPID promise-reply run
    std::vector<uint64_t> gp_list;                  // (node, bucket) pairs for the general apply kernel
    uint64_t num_gp_simple = 0;                     // ... the first of them: no events, no promise-reply runs
    uint64_t num_gp_snap = 0;                       // ... then up to here: no promise-reply runs
    std::vector<uint64_t> ev_off, pl_off;           // ev_off: per (bucket, node) pair (N * NB + 1); pl_off: per node
    std::vector<uint32_t> ev_msg, pl_msg;
    std::vector<uint64_t> ev_aux;                   // per event: PREPARE's first range meeting the bucket | count << 32
    std::vector<uint8_t> pair_ev;                   // per pair: 1 when it has snapshot events
    std::vector<uint8_t> pair_gp;                   // per pair: 1 when not lean (mpx_internal.hpp plan_shape_ok)
    std::vector<uint32_t> b_msg, b_pstart, b_rep, b_rsrc;
    std::vector<uint64_t> b_rbal, b_bal;
    std::vector<uint64_t> b_aid;                    // per batch: its accept id (the P_BATCH's, or carried)
    std::vector<uint64_t> b_rep_off;
    std::vector<uint64_t> cf_off;
    std::vector<Frag> cfrags;
    // incremental window (build_trace with a WindowCarry): per batch of the window's list
    // its global id (new batches and earlier ones that get votes here; b_msg = NONE32 for
    // an earlier one), per work-list pair whether earlier windows left state in it, and the
    // buckets with chosen-log runs
    std::vector<uint32_t> b_gid, b_node;
    std::vector<uint8_t> gp_base;
    std::vector<uint32_t> cb_list;
};

// Decode one record of `node`'s stream into `ns`.  Entries outside
// [shard_begin, shard_end) are dropped; a record whose entries all lie outside
// is marked (`part`) and left out by build_trace (header sharding).
int decode_record(ValueTable &vt, NodeStream &ns, uint32_t node, uint32_t N, const uint8_t *m, size_t len,
                  uint64_t shard_begin, uint64_t shard_end, IngestViolation &viol, SectionCache *sc = nullptr);
// one record handed over already decoded (mpx_submit_soa, multi semantics): the same
// NodeStream fields decode_record fills from the wire bytes
struct SoaRecord {
    uint32_t type, src;
    uint64_t ballot, aux;
    uint64_t n;                                   // entries (PREPARE: ranges)
    const uint64_t *a, *b, *pid;                  // iid, handle, proposal id (PREPARE: range start, end)
};
int append_record(ValueTable &vt, NodeStream &ns, uint32_t node, const SoaRecord &r, uint64_t shard_begin,
                  uint64_t shard_end, IngestViolation &viol);
// member semantics wire formats (member/paxos.cpp:846-932).  With `el` (MPX_FLAG_LEARN_EPOCHS)
// the record's E_EPOCH markers come from the engine: a submitted E_EPOCH is dropped, and a LEARN
// that makes the node apply membership Values is followed by one E_EPOCH per Value
int decode_record_member(ValueTable &vt, NodeStream &ns, uint32_t node, const uint8_t *m, size_t len,
                         uint64_t shard_begin, uint64_t shard_end, IngestViolation &viol, EpochLearn *el = nullptr,
                         SectionCache *sc = nullptr);

// Decode every node's slice sl[n], appended to nodes[n], on `threads` host threads: each stream is
// cut into chunks of about `chunk_bytes` (0: the total over 4 x threads, at least 1 MiB) decoded
// independently into the one value table — a node's first chunk straight into its stream, the
// later ones into `parts` (scratch, capacity kept), appended in record order with their entry
// offsets rebased — so the result is the serial decode's record for record.  `el` (learned
// epochs): one chunk per node, the Learner's apply frontier walks its records in order.  The
// violations are merged into `iv` in record order; the first failing chunk's code is returned.
int decode_parallel(ValueTable &vt, std::vector<NodeStream> &nodes, std::vector<NodeStream> &parts,
                    const std::vector<StreamSlice> &sl, bool member, std::vector<EpochLearn> *el,
                    uint64_t shard_begin, uint64_t shard_end, IngestViolation &iv, uint32_t threads,
                    uint64_t chunk_bytes);

// Flatten node streams and build every index the kernels walk.  `epochs`
// non-empty selects member semantics (role / version gates, E_EPOCH events).
// With `wc` (incremental runs): `nodes` hold one window's records; the window is built on
// the carried state and, only when the build succeeds, the carry is advanced past it.
// The walk over the nodes' records runs a thread per node (`threads`: at most that many; 0: up
// to 16) and the result is build_trace_serial's, field for field (tests/build_check.cpp).
int build_trace(const std::vector<NodeStream> &nodes, uint64_t shard_begin, uint64_t shard_len,
                const std::vector<mpx_epoch> &epochs, HostTrace &ht, WindowCarry *wc = nullptr, uint32_t threads = 0);
int build_trace_serial(const std::vector<NodeStream> &nodes, uint64_t shard_begin, uint64_t shard_len,
                       const std::vector<mpx_epoch> &epochs, HostTrace &ht, WindowCarry *wc = nullptr);

}  // namespace mpx
