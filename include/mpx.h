/*
 * mpx.h — C ABI of the MI355X batched Multi-Paxos acceptor/learner engine.
 *
 * This header is the drop-in boundary for the hot path of yuchenkan/multi-paxos
 * (SURVEY.md §8(b)).  The reference host talks to its protocol core through
 *
 *   paxos::NetWork::OnReceiveMessage(const char *msg, unsigned len)
 *       multi/paxos.h:202, multi/paxos.cpp:1714-1717     (inbound bytes)
 *   paxos::NetWork::SendMessageTCP / SendMessageUDP(ip, port, msg)
 *       multi/paxos.h:199-200                            (outbound bytes)
 *   paxos::StateMachine::Execute(const std::string &)
 *       multi/paxos.h:219                                (in-order apply)
 *   member: NetWork::OnReceive / Send, StateMachine::Apply
 *       member/paxos.h:169,180-181
 *
 * and the engine replaces the per-message handlers behind them
 * (OnPrepare/OnAccept/OnCommit/OnPrepareReply/OnAcceptReply/OnReject,
 * multi/paxos.cpp:858-1623; member/paxos.cpp:1029-1818) with HIP kernels
 * over structure-of-arrays state in HBM.
 *
 * Conventions
 *   - plain C types only; every function returns int (MPX_OK = 0, <0 error);
 *   - a handle is single-threaded (like the reference's one paxos thread per
 *     node, multi/paxos.cpp:345); one HIP stream per engine;
 *   - the caller keeps ownership of every buffer it passes in (the reference's
 *     OnReceiveMessage copies into a std::string, multi/paxos.cpp:1716);
 *   - where the reference would ASSERT-crash (multi/paxos.h:110) the engine
 *     records the first violation (mpx_last_violation) and keeps going.
 *
 * Wire vocabulary: messages are the reference's packed little-endian structs
 * (SURVEY.md Appendix A).  Two engine-local record types describe what the
 * proposer control plane of the reference did at that point in the node's
 * processing order (it is out of scope):
 *   MPX_MSG_P_START  {u32 type=16, u64 ballot}            StartPrepare, multi/paxos.cpp:1233-1248
 *                                                        (+ AcceptRejected's batch clear, :1328-1343)
 *   MPX_MSG_P_BATCH  {u32 type=17, u64 accept_id, u32 len, {u64 iid, Value}*}
 *                                                        a new AcceptingValues, multi/paxos.cpp:1299-1326
 *   MPX_MSG_P_PROPOSE {u32 type=19, u32 len, payload}     PaxosImpl::Propose(value), :1250-1280: the
 *                    client value gets the node's next value id; it is proposed at once (the P_BATCH that
 *                    follows) or, while preparing, at the next promise quorum (mpx_read_decisions)
 *                    (member: entries are {u64 iid, u64 pid, Value_m}, member/paxos.cpp:1158-1160)
 * and, for member semantics only, where the node applied a learned membership
 * change (NodeImpl::ChangeMemberships, member/paxos.cpp:1864-1964):
 *   MPX_MSG_E_EPOCH  {u32 type=18, u32 epoch}            the node moves to epochs[epoch]
 * Member E_EPOCH semantics:
 *   - the node's version_ becomes epochs[epoch].version; PREPARE / ACCEPT
 *     with another version are dropped silently (member/paxos.cpp:1702,1744);
 *   - acceptor role lost: the Acceptor object and its state are deleted
 *     (:1952-1957); gained: a fresh Acceptor (:1897-1901);
 *   - proposer role lost: the Proposer is deleted (:1927-1930); gained, or
 *     kept while the acceptor set changed (AcceptorsChanged, :1291-1322): the
 *     proposer is idle (no promise round, no batches) until its next P_START;
 *   - quorum for replies is |acceptors of the node's epoch|/2+1 (:1171,1327),
 *     and a reply from a non-acceptor is an ASSERT (:1163,1324).
 */
#ifndef MPX_H
#define MPX_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: mpx_epoch carries learner_mask (32 bytes), and mpx_stats grew from 16 to 18 u64
 *    words (general_pairs, num_runs, slot_bytes; reserved[] is the extension area from
 *    here on: the struct stays 144 bytes within ABI 2) */
#define MPX_ABI_VERSION 2u

/* ---- status codes ------------------------------------------------------ */
enum {
    MPX_OK            = 0,
    MPX_E_INVAL       = -1,   /* bad argument                                   */
    MPX_E_NOMEM       = -2,   /* host or device allocation failed               */
    MPX_E_HIP         = -3,   /* a HIP runtime call failed                      */
    MPX_E_DECODE      = -4,   /* malformed wire message (unknown type, short)   */
    MPX_E_RANGE       = -5,   /* value outside what the engine encodes          */
    MPX_E_STATE       = -6,   /* call not valid in the engine's current state   */
    MPX_E_NODEVICE    = -7,   /* no usable GPU (the engine never falls back)    */
    MPX_E_COMM        = -8,   /* RCCL failure                                   */
    MPX_E_VALUE       = -9    /* two different Values share (proposer,value_id) */
};

/* ---- wire message types (multi/paxos.cpp:742,831,847,1283,1346,1430,1482) */
enum {
    MPX_MSG_PREPARE       = 0,
    MPX_MSG_PREPARE_REPLY = 1,
    MPX_MSG_REJECT        = 2,
    MPX_MSG_ACCEPT        = 3,
    MPX_MSG_ACCEPT_REPLY  = 4,
    MPX_MSG_COMMIT        = 5,   /* member: LEARN       (member/paxos.cpp:611) */
    MPX_MSG_COMMIT_REPLY  = 6,   /* member: LEARN_REPLY (member/paxos.cpp:612) */
    MPX_MSG_P_START       = 16,  /* engine-local proposer marker, see above   */
    MPX_MSG_P_BATCH       = 17,
    MPX_MSG_E_EPOCH       = 18,  /* member only */
    MPX_MSG_P_PROPOSE     = 19   /* multi: a client value reaches Propose, see above */
};

enum { MPX_SEM_MULTI = 0, MPX_SEM_MEMBER = 1 };

/* Largest node count: votes are one 64-bit acceptor mask per batch. */
#define MPX_MAX_NODES 64u

/*
 * Value handles.  A reference Value is (u32 proposer, u64 value_id, bool noop,
 * payload) and (proposer, value_id) names it uniquely (multi/paxos.cpp:439).
 * On the device a Value is the 64-bit handle
 *     proposer << 48 | noop << 47 | value_id
 * (proposer < 2^14, value_id < 2^47, else MPX_E_RANGE); payload bytes stay in
 * a host table and are checked to be unique per handle at ingest (MPX_E_VALUE).
 */
#define MPX_HANDLE(proposer, noop, value_id) \
    (((uint64_t)(proposer) << 48) | ((uint64_t)((noop) ? 1 : 0) << 47) | (uint64_t)(value_id))
#define MPX_HANDLE_PROPOSER(h) ((uint32_t)(((h) >> 48) & 0x3FFFu))
#define MPX_HANDLE_NOOP(h)     ((unsigned)(((h) >> 47) & 1u))
#define MPX_HANDLE_VALUE_ID(h) ((h) & ((1ull << 47) - 1))
/* mpx_read_chosen / mpx_read_node_state mark present entries with this bit */
#define MPX_PRESENT (1ull << 63)

/* member semantics: one entry per membership epoch — the node sets after one
 * step of NodeImpl::ChangeMemberships (member/paxos.cpp:1864-1964).  Every
 * node starts in epoch 0 (Loop: {first} is learner, proposer and acceptor,
 * member/paxos.cpp:738-747).  An acceptor drops PREPARE/ACCEPT whose version
 * differs from its own (:1702,1744); the quorum is |acceptors|/2+1 (:1171,1327).
 * In an MPXT container (version 2) each entry is 32 bytes, in this layout; a
 * version-1 container holds 24-byte entries without learner_mask (read as
 * learner_mask = proposer_mask).  learners_ matter only to learn reliability
 * (mpx_read_learns): a Proposer retires a learn when |learners_| replied, and
 * a learner change re-learns (LearnersChanged, member/paxos.cpp:1345-1381,1472-1502). */
typedef struct mpx_epoch {
    uint32_t version;         /* NodeImpl::version_ in this epoch               */
    uint32_t flags;           /* 0                                              */
    uint64_t acceptor_mask;   /* bit i set: node i is an acceptor (acceptors_)  */
    uint64_t proposer_mask;   /* bit i set: node i runs a Proposer (proposers_) */
    uint64_t learner_mask;    /* bit i set: node i is a learner (learners_)     */
} mpx_epoch;

typedef struct mpx_config {
    uint32_t abi_version;      /* MPX_ABI_VERSION                                  */
    uint32_t num_nodes;        /* node ids 0..num_nodes-1 (multi: all roles)       */
    uint32_t semantics;        /* MPX_SEM_MULTI | MPX_SEM_MEMBER                   */
    int32_t  device;           /* HIP device ordinal                               */
    uint64_t shard_begin;      /* this engine owns instances [shard_begin,         */
    uint64_t shard_end;        /*                              shard_end)          */
    uint32_t num_epochs;       /* member only                                      */
    uint32_t flags;            /* 0, MPX_FLAG_INCREMENTAL [| MPX_FLAG_DECISIONS],  */
                               /* member: [| MPX_FLAG_LEARN_EPOCHS]                */
    const mpx_epoch *epochs;   /* member only, indexed by E_EPOCH's epoch          */
} mpx_config;

/* Incremental runs (the drop-in for NetWork::OnReceiveMessage, multi/paxos.cpp:1714-1717,
 * and member NetWork::OnReceive, member/paxos.cpp:841-844, on a live stream).
 * Each mpx_run applies only the records submitted since the previous one — a window — to
 * the state the earlier windows left, on the device: acceptor / learner entries, the chosen
 * log, promised / max_seen, promise rounds with their pre-accepted maps, and the batches'
 * votes carry over as values; member windows also carry each node's roles (epoch, Acceptor
 * incarnation, Proposer) and which batches a membership step cleared.  A window's host and
 * device work is O(window records + state they touch), not O(history).
 * mpx_drain_sends returns the window's replies; the mpx_read_* state readbacks and
 * mpx_state_digest give the cumulative state; mpx_stats counts the window.  Not
 * available in this mode (MPX_E_STATE): mpx_step / mpx_reset_state (windows are applied
 * once), mpx_dump_result, the commits readback and the sharded decisions (they walk the
 * run's history), and the decisions / learns readbacks unless MPX_FLAG_DECISIONS carries
 * their bookkeeping.
 * Errors: a window refused while it is built (MPX_E_RANGE, MPX_E_DECODE, ...) leaves the
 * engine as it was — its records stay queued and are refused again; a failure after the
 * window was taken (a HIP error) may leave it partly applied, so the engine is poisoned:
 * every later mpx_run, submit and readback returns MPX_E_STATE.
 * Limits that count over the whole live stream, not per window: member semantics allow at
 * most 254 E_EPOCH records per node over the stream (the device's Acceptor incarnation
 * counter, G_SEG); the window that would place a node's 255th is refused with MPX_E_RANGE
 * and, as above, stays queued, so that stream cannot advance (start a new engine).  With
 * MPX_FLAG_DECISIONS a node's record index (sends' and events' seq) is 32-bit over the
 * stream (< 2^32 - 1 records per node, else MPX_E_RANGE). */
#define MPX_FLAG_INCREMENTAL 1u
/* With MPX_FLAG_INCREMENTAL: every mpx_run also advances the proposers' phase-2
 * bookkeeping over the window's events (the quorums' merged maps, COMMIT / LEARN entries,
 * client values; member: E_EPOCH role changes), so mpx_read_decisions returns the
 * decisions of every window so far — the MPXD of one run over the whole stream (host work
 * per window, O(window)).  Member semantics: the learn bookkeeping (LearningValues
 * creation, replies, AcceptorsChanged, drops) advances the same way and mpx_read_learns
 * returns the MPXL of the whole stream (k_learns over every learn at read time). */
#define MPX_FLAG_DECISIONS 2u
/* Member semantics: membership learned at run time, as the reference does it — a node's
 * Learner applies learned Values in instance order and a membership Value (Node::AddAcceptor
 * ... ProposerToLearner, member/paxos.cpp:635-721) changes the node's roles when it is applied
 * (Learner::Apply -> NodeImpl::ChangeMemberships, :1062-1073,1864-1964).  The engine is created
 * with the genesis epoch only (num_epochs = 1: {first} learner, proposer and acceptor, version 0,
 * :738-747); at ingest it tracks every node's apply frontier over its LEARN entries (all of
 * them, whatever the shard), and after a LEARN that makes the node apply membership Values it
 * places one E_EPOCH record per Value, the node's view after that change, in its stream.  The
 * epoch table grows as the nodes apply membership Values (epoch k = the view after the k-th
 * membership Value in instance order; every node reaches the same sequence, MPX_E_STATE if two
 * disagree) and mpx_read_epochs returns it.  Submitted E_EPOCH records are ignored, so a live host
 * submits exactly what NetWork::OnReceive receives (member/paxos.cpp:841-844); combines with
 * MPX_FLAG_INCREMENTAL (the frontier and the views carry over between windows).  Record indices
 * (sends' and events' seq) count the engine's E_EPOCH records.  A change the reference ASSERTs
 * on (a member added twice, an absent one removed, the last acceptor removed) fails the submit
 * with MPX_E_STATE. */
#define MPX_FLAG_LEARN_EPOCHS 4u

typedef struct mpx_engine mpx_engine;

/* Counters of the last run.  B_alg = 16 P + 24 A + 16 L. */
typedef struct mpx_stats {
    uint64_t chosen;           /* C: distinct instances whose accept votes first
                                  reached quorum (multi/paxos.cpp:1416)           */
    uint64_t promise_entries;  /* P: entries in granted PREPARE_REPLYs           */
    uint64_t accept_apps;      /* A: granted (acceptor, instance) applications    */
    uint64_t commit_apps;      /* L: (learner, instance) commit applications     */
    uint64_t messages;         /* records processed                               */
    uint64_t violations;       /* reference ASSERTs that would have fired         */
    uint64_t chosen_digest;    /* order-independent digest of the chosen log      */
    uint64_t state_digest;     /* ... of every node's final acceptor/learner state */
    uint64_t scalar_digest;    /* ... of every node's promised / max_seen         */
    uint64_t device_ns;        /* device time of the last run (first..last kernel) */
    uint64_t apply_ns;         /* device time of the acceptor/learner kernel      */
    uint64_t ingest_ns;        /* host ingest + H2D of the last submit batch       */
    uint64_t bytes_alg;        /* 16 P + 24 A + 16 L                               */
    uint64_t skipped;          /* submitted records left out: all their entries
                                  belong to other shards (header sharding)       */
    uint64_t general_pairs;    /* (node, bucket) pairs the general per-slot walk
                                  (k_apply) took in the last run: its work list, or
                                  in a plan step what k_plan_list left to it       */
    uint64_t num_runs;         /* message runs (fragments) of the resident trace: an
                                  entry-carrying message cut per 256-instance bucket */
    uint64_t slot_bytes;       /* bytes per (node, instance) state slot (1 or 2)   */
    uint64_t reserved[1];
} mpx_stats;

typedef struct mpx_violation {
    uint64_t code;             /* MPX_V_*                                          */
    uint32_t node;
    uint32_t pad;
    uint64_t seq;              /* record index in the node's stream               */
    uint64_t iid;
} mpx_violation;

enum {
    MPX_V_NONE          = 0,
    MPX_V_COMMIT_VALUE  = 1,   /* re-commit with another Value, multi/paxos.cpp:1508-1509 */
    MPX_V_CHOSEN_VALUE  = 2,   /* two chosen batches disagree on an instance (safety)     */
    MPX_V_BAD_NODE      = 3,   /* reply from a node not in the set, multi/paxos.cpp:1040,1414 */
    MPX_V_DUP_IID       = 4,   /* an instance twice in one message / overlapping ranges   */
    MPX_V_BATCH_BEFORE_QUORUM = 5, /* P_BATCH while preparing, multi/paxos.cpp:1054   */
    MPX_V_LEARN_VALUE   = 6    /* member: accept/learn differs from the learned Value,
                                  member/paxos.cpp:1767-1769,1398-1399           */
};

/* ---- lifecycle ----------------------------------------------------------- */
int  mpx_version(void);
int  mpx_device_count(int *count);
int  mpx_create(const mpx_config *cfg, mpx_engine **out);
int  mpx_destroy(mpx_engine *eng);

/* ---- inbound: batched NetWork::OnReceiveMessage -------------------------- *
 * Appends `count` records to node `node`'s receive stream in arrival order.
 * Record i is bytes[offsets[i] .. offsets[i+1]) (offsets has count+1 entries).
 * Decoding and instance bucketing happen here, on the host (the reference
 * decodes in the handlers: ExtractInstanceValues etc., multi/paxos.cpp:523-711).
 */
int  mpx_submit(mpx_engine *eng, uint32_t node, const uint8_t *bytes,
                const uint64_t *offsets, uint64_t count);
/* SoA fast path (multi semantics): `count` records already decoded, as arrays — what
 * mpx_submit decodes from the wire, without the codec.  Per record: its MPX_MSG_* type,
 * source id, ballot (proposal id; REJECT: its max id), aux (accept id: ACCEPT /
 * ACCEPT_REPLY / P_BATCH; commit id: COMMIT / COMMIT_REPLY), and entries
 * [ent_off[i], ent_off[i+1]) of ent_a / ent_b / ent_pid: ACCEPT / COMMIT / P_BATCH
 * {iid, handle}, PREPARE_REPLY {iid, handle, accepted proposal id}, PREPARE its ranges
 * {start, end (exclusive)}.  A handle with no Value bytes yet names the payload-free
 * Value(proposer, value_id, noop) (MPX_HANDLE).  ent_pid may be NULL (ids 0). */
typedef struct mpx_soa_records {
    uint64_t count;
    const uint8_t *type;
    const uint32_t *src;
    const uint64_t *ballot;
    const uint64_t *aux;
    const uint64_t *ent_off;     /* count + 1 */
    const uint64_t *ent_a;
    const uint64_t *ent_b;
    const uint64_t *ent_pid;
} mpx_soa_records;
int  mpx_submit_soa(mpx_engine *eng, uint32_t node, const mpx_soa_records *records);
/* Convenience: submit every node of an MPXT trace container (see mpx_trace_*). */
int  mpx_submit_trace(mpx_engine *eng, const uint8_t *trace, uint64_t size);
/* The same for one slice of every node's stream — records [begin[n], end[n]) of node n
 * (one window of a live stream, MPX_FLAG_INCREMENTAL): = mpx_submit of each node's slice,
 * decoded on one host thread per node for large slices. */
int  mpx_submit_trace_range(mpx_engine *eng, const uint8_t *trace, uint64_t size,
                            const uint64_t *begin, const uint64_t *end);
/* The same slice decoded on a background host thread: the call returns at once and the decode
 * overlaps the build and device run of the window queued before it — the pipelined live loop
 * submit_async(k + 1), mpx_run(k), ... (MPX_FLAG_INCREMENTAL, multi semantics, no
 * MPX_FLAG_LEARN_EPOCHS; MPX_E_STATE otherwise).  mpx_run joins the decode only when nothing else
 * is queued; every submit and every call that reads Values (mpx_drain_sends, mpx_value_bytes,
 * mpx_read_executed, mpx_dump_result) joins it first, so records keep their submission order.  A
 * decode error is returned by the call that joins it (that window is dropped, the engine stays
 * usable).  `trace` must stay valid until then. */
int  mpx_submit_trace_range_async(mpx_engine *eng, const uint8_t *trace, uint64_t size,
                                  const uint64_t *begin, const uint64_t *end);

/* Apply everything submitted since the last run (state carries over). */
int  mpx_run(mpx_engine *eng);
/* Drop all acceptor/learner/proposer state back to genesis (the PaxosImpl
 * ctor state, multi/paxos.cpp:323-346).  The resident trace is kept. */
int  mpx_reset_state(mpx_engine *eng);
/* One bench step: reset_state + replay the whole resident trace, no host
 * synchronisation (kernels queued on the engine's stream). */
int  mpx_step(mpx_engine *eng);
int  mpx_sync(mpx_engine *eng);
/* Device timings (HIP events on the engine's stream) of the runs/steps since
 * the previous call: per run the acceptor/learner kernel (k_apply) and the
 * whole run, in milliseconds.  Writes at most `max` pairs, *n = pairs written. */
int  mpx_timings(mpx_engine *eng, uint32_t max, double *apply_ms, double *run_ms, uint32_t *n);
/* The same runs/steps split into phases, 5 doubles (ms) per run: whole run,
 * header scan + promise / vote quorums, plan + store + fast apply (clean
 * pairs), general apply (k_apply: every other pair), chosen log + counters.
 * apply_ms of mpx_timings = phases 2 + 3.  Consumes the timings like mpx_timings. */
int  mpx_timings_detail(mpx_engine *eng, uint32_t max, double *phases, uint32_t *n);
/* Record those phase events on every `every`-th run / step only (1: all, the default; 0:
 * none).  Each event rides on a kernel dispatch and costs the step ~1.5-2 us; a digested
 * mpx_run is always timed. */
int  mpx_timing_every(mpx_engine *eng, uint32_t every);

/* ---- outbound ------------------------------------------------------------ */
/* Replies generated by the acceptor/learner handlers of the last run, in the
 * reference's generation order per node (types 1,2,4,6; multi/paxos.cpp:
 * 888-899,1391-1403,1577-1582).  The callback gets a pointer valid for the
 * duration of the call (the reference passes a const std::string&). */
typedef void (*mpx_send_fn)(void *user, uint32_t src, uint32_t dst,
                            const uint8_t *bytes, uint32_t len);
int  mpx_drain_sends(mpx_engine *eng, mpx_send_fn fn, void *user);

/* chosen log: out[i] = MPX_PRESENT | handle, or 0 if instance first+i is not
 * chosen yet (instances outside the shard are an error). */
int  mpx_read_chosen(mpx_engine *eng, uint64_t first, uint64_t count, uint64_t *out);
/* The member epoch table: with MPX_FLAG_LEARN_EPOCHS the epochs learned so far (genesis first),
 * else the table the engine was created with or took from a container.  Writes min(cap, total)
 * entries, *count = total. */
int  mpx_read_epochs(mpx_engine *eng, mpx_epoch *out, uint32_t cap, uint32_t *count);
/* per-node scalars: promised_proposal_id_ and max_proposal_id_
 * (multi/paxos.cpp:492,460) */
/* In-order executor of one node, on the device (replaces the
 * apply loop of PaxosImpl::OnCommit, multi/paxos.cpp:1584-1622, and the
 * member Learner's, member/paxos.cpp:1042-1053): *frontier = the node's
 * next_id_to_apply_ (first instance of the shard not committed there),
 * *count = Values executed below it (noops and member membership Values
 * skipped), handles[0 .. min(count, cap)) = their handles in instance order
 * (payload bytes: mpx_value_bytes).  handles may be NULL when cap is 0. */
int  mpx_read_executed(mpx_engine *eng, uint32_t node, uint64_t *frontier,
                       uint64_t *count, uint64_t *handles, uint64_t cap);
int  mpx_read_node_scalars(mpx_engine *eng, uint32_t node,
                           uint64_t *promised, uint64_t *max_seen);
/* per-node per-instance state; any output pointer may be NULL.
 * acc_value / com_value carry MPX_PRESENT when the entry exists. */
int  mpx_read_node_state(mpx_engine *eng, uint32_t node, uint64_t first, uint64_t count,
                         uint64_t *acc_ballot, uint64_t *acc_value,
                         uint64_t *com_ballot, uint64_t *com_value);
int  mpx_stats_get(mpx_engine *eng, mpx_stats *out);
/* Order-independent digests (the mpx_stats.state_digest / chosen_digest
 * definitions) of the acceptor/learner state and chosen log the last run OR
 * step left in HBM, computed by a separate device pass.  mpx_step carries no
 * digest code, so this is how a caller verifies what the timed kernels wrote. */
int  mpx_state_digest(mpx_engine *eng, uint64_t *state_digest, uint64_t *chosen_digest);
int  mpx_last_violation(mpx_engine *eng, mpx_violation *out);
/* Canonical result dump (format "MPXR"): the byte format
 * the CPU oracle and the reference driver also write, so parity is a
 * byte comparison.  *out is malloc'ed; free with mpx_free. */
int  mpx_dump_result(mpx_engine *eng, uint8_t **out, uint64_t *size);
/* Phase-2 decisions (an engine whose shard starts at instance
 * 0): for every promise quorum of the last run, the batch OnPrepareReply builds
 * (multi/paxos.cpp:1056-1175) — every pre-accepted value of an instance the node
 * has not committed (:1071-1102), then a noop Value(node, ++value_id) for every
 * other uncommitted instance below the highest committed-or-adopted one
 * (:1117-1130; value ids count from 1 per node over its quorums), then the node's
 * own client values (P_PROPOSE records: initial proposals still unproposed, the
 * queued ones at the next free ids, :1132-1175, with Propose :1250-1280 and the
 * OnCommit re-propose :1519-1570 kept in order; they share the value ids).
 * Without client values the noop fill is computed on the device from the run's
 * state; with them (and for member) it is the proposer's sequential bookkeeping
 * on the host over the device's quorums and merged maps.  Member semantics
 * (member/paxos.cpp:1183-1297, an engine that kept every record): the same batch
 * over the Proposer's unlearned ids, kept by Proposer::OnLearn (:1383-1470); a
 * Proposer's initial proposals are the node's own Values of the trace not yet
 * learned when it starts (what Propose would have recorded).  Format MPXD: "MPXD"
 * u32 1, u32 nodes; per node u64 count, per quorum {u64 seq (record index in the
 * node's stream), u64 n, {u64 iid, u64 handle} * n, iid ascending}.  *out is
 * malloc'ed; free with mpx_free.  MPX_E_STATE for a shard engine. */
int  mpx_read_decisions(mpx_engine *eng, uint8_t **out, uint64_t *size);
/* Sharded phase-2 decisions (one engine per instance range, shards in rank
 * order).  The fill of each quorum reaches the highest committed-or-adopted
 * instance over ALL shards, so it takes one exchange of per-quorum bounds:
 *  1. mpx_decisions_bounds: per promise quorum of the run (node-major stream
 *     order, the same list on every shard) the shard's own bound, absolute:
 *     shard_begin + 1 + its highest committed-or-adopted instance, 0 if none.
 *     Writes min(cap, count) bounds, *count = the number of quorums.
 *  2. the caller takes the element-wise maximum over shards (an all-reduce MAX
 *     of `count` u64) and passes it to mpx_read_decisions_part, which writes
 *     this shard's adopted entries and noop-fill instances.  Format MPXP:
 *     "MPXP" u32 1, u32 nodes, u64 shard_begin; then MPXD's body with a noop
 *     entry's handle ~0 (numbered only once the parts are merged).
 *  3. mpx_decisions_combine merges the parts (given in shard order) into the
 *     MPXD mpx_read_decisions writes on one engine holding every instance:
 *     each quorum's entries concatenated in shard order, noops numbered
 *     Value(node, ++value_id) per node.  Pure host work.
 * MPX_E_STATE for member semantics; MPX_E_INVAL for a bound count or parts
 * that do not match. */
int  mpx_decisions_bounds(mpx_engine *eng, uint64_t *bounds, uint64_t cap, uint64_t *count);
int  mpx_read_decisions_part(mpx_engine *eng, const uint64_t *global_bounds, uint64_t count,
                             uint8_t **out, uint64_t *size);
int  mpx_decisions_combine(const uint8_t *const *parts, const uint64_t *sizes, uint32_t nparts,
                           uint8_t **out, uint64_t *size);
/* Commit reliability (multi semantics, an engine that kept
 * every record — shard starting at 0, nothing left out for another shard):
 * every CommittingValues each node's proposer created in the last run — at an
 * accept quorum (OnAcceptReply, multi/paxos.cpp:1416-1421) and at a promise
 * quorum while it held committed values (OnPrepareReply re-commits all of them,
 * :1184-1197) — numbered 1, 2, ... per node like committing_id_ (:340), and what
 * OnCommitReply (:1625-1641) made of it: replied_ as a learner mask and the
 * reply at which every node had replied (the commit retires; a retry timer,
 * Commit :1474-1478, resends to the learners not in the mask).  Computed on the
 * device (k_commits) from the run's accept / promise quorums.  Format MPXC:
 * "MPXC" u32 1, u32 nodes; per node u64 count, per commit {u64 id, u64
 * created_seq, u64 kind (0 accept quorum, 1 promise quorum), u64 accept_id
 * (kind 0, else 0), u64 retired_seq (~0: still open), u64 replied_mask}, seqs
 * = record indices in the node's stream.  *out is malloc'ed; free with
 * mpx_free.  MPX_E_STATE for member semantics or a shard engine, MPX_E_RANGE
 * for a COMMIT_REPLY naming a learner >= 64. */
int  mpx_read_commits(mpx_engine *eng, uint8_t **out, uint64_t *size);
/* Sharded commit reliability (one engine per instance range, shards in rank order).
 * A commit is created at an accept quorum of a batch (only the shards holding its
 * instances keep it) or at a promise quorum where the node holds any committed
 * instance (of any shard), so the creation points are a union over shards:
 *  1. mpx_commit_points: this engine's creation points, format MPXQ: "MPXQ" u32 1,
 *     u32 nodes; per node u64 count, {u64 seq, u64 accept_id (~0: promise quorum)}
 *     ascending by seq (record index in the node's stream);
 *  2. mpx_commit_points_combine: their union (pure host work);
 *  3. mpx_read_commits_at, on the engine whose shard starts at instance 0 (header
 *     sharding keeps every COMMIT_REPLY there): OnCommitReply over the union —
 *     the MPXC mpx_read_commits writes on one engine holding every instance.
 * mpx_read_commits_sharded runs 1-3 over the engine's communicator; every rank
 * receives the MPXC.  MPX_E_STATE for member semantics. */
int  mpx_commit_points(mpx_engine *eng, uint8_t **out, uint64_t *size);
int  mpx_commit_points_combine(const uint8_t *const *parts, const uint64_t *sizes, uint32_t nparts,
                               uint8_t **out, uint64_t *size);
int  mpx_read_commits_at(mpx_engine *eng, const uint8_t *points, uint64_t points_size,
                         uint8_t **out, uint64_t *size);
int  mpx_read_commits_sharded(mpx_engine *eng, uint8_t **out, uint64_t *size);
/* Learn reliability (member semantics, an engine holding every
 * instance): every LearningValues each node's Proposer created in the last run — at an
 * accept quorum (OnAcceptReply, member/paxos.cpp:1334-1337), at a promise quorum once its
 * learner learned anything (OnPrepareReply re-learns all of it, :1299-1307), and at
 * LearnersChanged while not preparing (every learned and open learn's Value, :1472-1491)
 * — numbered like learning_id_ (1, 2, ... per Proposer; a node's new Proposer starts
 * again), and what became of it: OnLearnReply's learned_ set, the record where its
 * learning_values_for_acceptors_ entry reached |acceptors|/2+1 and Applied ran (replies,
 * or AcceptorsChanged :1504-1533), the record where every learner had replied (retired),
 * or where LearnersChanged or the Proposer's deletion (:1916-1942) dropped it.  Learner
 * and acceptor sets come from the epoch table (mpx_epoch.learner_mask); a membership step
 * is the E_EPOCH run after the LEARN that applied it.  The replies are walked on the
 * device (k_learns).  Format MPXL: "MPXL" u32 1, u32 nodes; per node u64 count, per learn
 * {u64 id, u64 created_seq, u64 kind (0 accept quorum, 1 promise quorum, 2 learners
 * changed), u64 accept_id (kind 0, else 0), u64 applied_seq, u64 retired_seq, u64
 * dropped_seq, u64 learned_mask} (~0: did not happen), seqs = record indices in the
 * node's stream.  *out is malloc'ed; free with mpx_free.  MPX_E_STATE for multi
 * semantics, a shard engine or an E_EPOCH step that both adds and removes roles. */
int  mpx_read_learns(mpx_engine *eng, uint8_t **out, uint64_t *size);
/* The Values of the same learns, for the host's paxos::Callback (member/paxos.h:142-164):
 * LearningValues::values_ in instance order — kind 0: the chosen batch (the cb strings
 * Callback::Accepted receives at creation, :1327-1332); kinds 1 and 2: the node's Learner's
 * learned values at creation (:1299-1301, :1476), kind 2 with every open learn's values
 * added (std::map::insert, id order, :1477-1482) — what Applied receives at applied_seq
 * (:1360-1368, :1523-1526); and the records where a P_PROPOSE found the node without a
 * Proposer (Node::Propose -> Callback::Unproposable, NodeImpl::Loop :784-787).  Format MPXV:
 * "MPXV" u32 1, u32 nodes; per node u64 count (= MPXL's), per learn {u64 n, n x {u64 iid,
 * u64 handle}}, then u64 u, u x u64 unproposable_seq.  Replaces the reference's
 * Callback calls from Proposer::OnAcceptReply / OnLearnReply / AcceptorsChanged (member/
 * paxos.cpp:1317-1381,1504-1533).  Same state requirements as mpx_read_learns. */
int  mpx_read_learn_values(mpx_engine *eng, uint8_t **out, uint64_t *size);
/* Encoded reference Value bytes (multi/paxos.cpp:556-598) for a handle. */
int  mpx_value_bytes(mpx_engine *eng, uint64_t handle, uint8_t *buf,
                     uint32_t cap, uint32_t *len);
void mpx_free(void *p);

/* ---- synthetic traces (host generator, deterministic) --------------------- */
typedef struct mpx_gen_params {
    uint32_t kind;             /* MPX_GEN_CLEAN | MPX_GEN_FAULTY | MPX_GEN_MEMBER  */
    uint32_t num_nodes;
    uint64_t num_instances;    /* M                                                */
    uint64_t seed;
    uint32_t batch;            /* instances per ACCEPT/COMMIT (clean: fixed)       */
    uint32_t proposers;        /* competing proposers (faulty)                     */
    uint32_t drop_rate;        /* per 10000, HijackSend model multi/main.cpp:116-132 */
    uint32_t dup_rate;         /* per 10000, duplicates up to depth 3              */
    uint32_t max_delay;        /* delay U[0,max_delay) ticks: reordering           */
    uint32_t noop_permille;    /* faulty: share of noop gap-fill values            */
    uint64_t shard_begin;      /* emit only instance entries in [begin,end);       */
    uint64_t shard_end;        /*   headers are replicated       */
} mpx_gen_params;

enum { MPX_GEN_CLEAN = 0, MPX_GEN_FAULTY = 1, MPX_GEN_MEMBER = 2 };

/* Build an MPXT trace container in host memory (free with mpx_free). */
int  mpx_trace_generate(const mpx_gen_params *p, uint8_t **out, uint64_t *size);
/* Materialise the clean trace of `p` directly in HBM (GPU generator kernel;
 * same content as mpx_trace_generate for MPX_GEN_CLEAN, restricted to the
 * engine's shard).  Replaces the resident trace. */
int  mpx_load_clean_device(mpx_engine *eng, const mpx_gen_params *p);

/* ---- multi-GPU: RCCL over xGMI, summary all-gather only -- */
#define MPX_UID_BYTES 128
int  mpx_comm_unique_id(uint8_t out[MPX_UID_BYTES]);
int  mpx_comm_init(mpx_engine *eng, const uint8_t uid[MPX_UID_BYTES],
                   int rank, int nranks);
/* All-gather every rank's 64-word run summary (mpx_stats words + per-node
 * scalars) over RCCL on the engine's stream; out holds nranks*64 words. */
int  mpx_allgather_summary(mpx_engine *eng, uint64_t *out);
/* Element-wise MAX of `n` u64 over every rank of the engine's communicator
 * (ncclAllReduce over xGMI on the engine's stream), in place in a host buffer.
 * Without a communicator (or one rank) the values stay as they are. */
int  mpx_comm_allreduce_max(mpx_engine *eng, uint64_t *vals, uint64_t n);
/* All-gather of one byte string per rank: *out (malloc'ed; free with mpx_free)
 * = every rank's string in rank order, lens[r] = rank r's length (nranks
 * entries).  Lengths go first (one u64 all-gather), then the strings padded to
 * the longest. */
int  mpx_comm_allgather_bytes(mpx_engine *eng, const uint8_t *mine, uint64_t len,
                              uint8_t **out, uint64_t *lens);
/* Sharded phase-2 decisions over the engine's own communicator (ranks = shards
 * in instance order): mpx_decisions_bounds, mpx_comm_allreduce_max (also of the
 * quorum count, which must agree), mpx_read_decisions_part, the parts gathered
 * with mpx_comm_allgather_bytes and merged with mpx_decisions_combine.  Every
 * rank receives the whole run's MPXD.  One rank: mpx_read_decisions' bytes.  A
 * trace with client values (P_PROPOSE) takes the proposal parts instead
 * (mpx_proposal_part gathered, mpx_proposal_combine). */
int  mpx_read_decisions_sharded(mpx_engine *eng, uint8_t **out, uint64_t *size);
/* Decisions with client values over instance shards (multi semantics, host traces):
 * the proposer's bookkeeping reads events of its own stream — Propose, StartPrepare,
 * each COMMIT's entries, each promise quorum's merged map — and a shard holds its own
 * instances' entries of them.  mpx_proposal_part writes this shard's events, format
 * MPXE: "MPXE" u32 1, u32 nodes, u64 shard_begin, u64 shard_end; per node u64 count,
 * per event {u64 seq, u32 type (19 P_PROPOSE, 16 P_START, 5 COMMIT, 1 promise
 * quorum), u32 n, {u64 iid, u64 handle} * n}.  Member semantics (every member decision
 * walk, client values or not): "MPXE" u32 2, the same header, then u32 E and E x {u64
 * acceptor_mask, u64 proposer_mask} (the epoch table), and per event {u64 seq, u32 type
 * (as above, 5 = LEARN, plus 18 E_EPOCH), u32 n, u64 aux (E_EPOCH: the epoch), entries}.
 * mpx_proposal_combine takes every
 * shard's part in shard order (contiguous ranges from 0), merges each node's events
 * by record (entries concatenated in shard order) and writes the MPXD
 * mpx_read_decisions writes on one engine holding every instance.  Pure host work. */
int  mpx_proposal_part(mpx_engine *eng, uint8_t **out, uint64_t *size);
int  mpx_proposal_combine(const uint8_t *const *parts, const uint64_t *sizes, uint32_t nparts,
                          uint8_t **out, uint64_t *size);

/* ---- the closed loop (the engine generates its own accepts and commits) ----
 * A proposer control plane over one incremental engine (MPX_FLAG_INCREMENTAL |
 * MPX_FLAG_DECISIONS, multi semantics, every node an acceptor and learner): each message it
 * sends is made from the engine's results — StartPrepare (P_START + PREPARE over [0, 2^64-1),
 * multi/paxos.cpp:1233-1248), Propose (P_PROPOSE, :1250-1280), the phase-2 batch the engine
 * decided at the proposer's promise quorum (mpx_read_decisions -> P_BATCH + ACCEPT,
 * :1056-1175,1299-1326), COMMIT of a batch the chosen log holds (:1429-1444); the acceptors'
 * replies are the engine's drained sends, appended to their destinations' streams.  `to`:
 * a bit mask of the nodes a message is delivered to.  mpx_loop_step submits every stream's new
 * records as one window and runs it.  mpx_loop_trace: the recorded streams as MPXT (replayable
 * through the reference's handlers).  mpx_loop_leader_rounds: `rounds` rounds of node `leader`
 * with `values` client values queued each (5 windows per round).  Replaces what the reference's
 * Proposer does between its receive and send calls (multi/paxos.cpp:1036-1343,1406-1444) for
 * the decisions the engine computes; the timers stay the caller's. */
typedef struct mpx_loop mpx_loop;
typedef struct mpx_loop_stats {
    uint64_t windows, records, batches, committed_batches, committed_instances, proposed;
    uint64_t submit_ns, run_ns, drain_ns;
} mpx_loop_stats;
int  mpx_loop_create(uint32_t num_nodes, uint64_t num_instances, int device, mpx_loop **out);
int  mpx_loop_destroy(mpx_loop *loop);
mpx_engine *mpx_loop_engine(mpx_loop *loop);
int  mpx_loop_prepare(mpx_loop *loop, uint32_t node, uint64_t to);
int  mpx_loop_propose(mpx_loop *loop, uint32_t node, const uint8_t *payload, uint32_t len);
int  mpx_loop_step(mpx_loop *loop);
int  mpx_loop_accept_decided(mpx_loop *loop, uint32_t node, uint64_t to, uint64_t *accept_id);
int  mpx_loop_commit_chosen(mpx_loop *loop, uint32_t node, uint64_t to, uint32_t *count);
int  mpx_loop_leader_rounds(mpx_loop *loop, uint32_t leader, uint64_t to, uint32_t rounds, uint32_t values);
int  mpx_loop_stats_get(mpx_loop *loop, mpx_loop_stats *out);
int  mpx_loop_trace(mpx_loop *loop, uint8_t **out, uint64_t *size);

#ifdef __cplusplus
}
#endif
#endif /* MPX_H */
