// engine.cpp — the C ABI (include/mpx.h) over the HIP kernels.
//
// Host responsibilities: decode + bucket submitted records (ingest.cpp), keep
// the trace resident in HBM, queue a run (kernels.hip) on the engine's stream,
// and turn device results back into the reference's vocabulary (sends,
// canonical MPXR dump).  There is no CPU execution path: without a GPU every
// compute entry point returns MPX_E_NODEVICE.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <functional>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <unordered_map>
#include <set>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "gen.hpp"
#include "ingest.hpp"
#include "mpx.h"
#include "mpx_internal.hpp"

using namespace mpx;

static_assert(sizeof(mpx_stats) == 144, "mpx_stats is 18 u64 words within ABI 2 (include/mpx.h)");

namespace {

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    ~DevBuf() { if (p) (void)hipFree(p); }
    int alloc(size_t n)
    {
        if (n <= bytes && p) return MPX_OK;
        if (p) { (void)hipFree(p); p = nullptr; bytes = 0; }
        if (!n) return MPX_OK;
        n = (n + 63) & ~(size_t)63;     // padded: vector loads may read a tail word past the last element
        if (hipMalloc(&p, n) != hipSuccess) { p = nullptr; return MPX_E_NOMEM; }
#ifdef MPX_AB
        if (ab_env("MPX_POISON")) {                     // (A/B builds: find reads of unwritten memory; the
            (void)hipMemset(p, 0xA5, n);                // null stream does not order the non-blocking
            (void)hipDeviceSynchronize();               // engine streams, so wait here)
        }
#endif
        bytes = n;
        return MPX_OK;
    }
    template <typename T> T *as() const { return (T *)p; }
};

template <typename T> int upload(DevBuf &b, const std::vector<T> &v, hipStream_t s)
{
    int rc = b.alloc(std::max<size_t>(v.size() * sizeof(T), 8));
    if (rc) return rc;
    if (!v.empty() && hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s) != hipSuccess)
        return MPX_E_HIP;
    return MPX_OK;
}

struct StepEvents { hipEvent_t e[5]; bool store_last; };   // launch_run's event points (store_last: e[3], e[4]
                                                          // not recorded, run_ends_with_store)

}  // namespace

struct PropNode;
struct MPropNode;
static std::vector<PropNode> *prop_new(uint32_t nodes);
static void prop_free(std::vector<PropNode> *p);
static std::vector<MPropNode> *mprop_new(uint32_t nodes);
static void mprop_free(std::vector<MPropNode> *p);
struct LearnCarry;
static LearnCarry *learn_new(uint32_t nodes);
static void learn_free(LearnCarry *c);
struct mpx_engine;
static int prop_window(mpx_engine *e);

struct mpx_engine {
    mpx_config cfg{};
    uint64_t ab_build_ns = 0;                  // (MPX_HOST_TIMES, A/B builds: build_trace's share of upload_trace)
    std::vector<mpx_epoch> epochs;
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t num_cus = 256;
    ValueTable vt;
    std::vector<NodeStream> nodes;
    std::vector<NodeStream> parts;             // submit_container's record chunks past each node's first (capacity kept)
    std::vector<EpochLearn> elearn;                  // MPX_FLAG_LEARN_EPOCHS: per node (ingest.hpp)
    IngestViolation iv;
    // mpx_submit_trace_range_async: the next window's records decoded on a host thread while the
    // current one is built and run (pf_join moves them into `nodes`)
    std::thread pf_thread;
    bool pf_pending = false;
    int pf_rc = MPX_OK;
    std::vector<NodeStream> pf_nodes, pf_parts;
    IngestViolation pf_iv;
    uint64_t pf_ns = 0;
    HostTrace ht;
    bool dirty = true;
    bool device_trace = false;       // trace materialised by a device generator
    bool whole = true;               // no record left out for another shard (mpx_read_commits)
    uint64_t shard_len = 0;
    uint32_t NB = 0;
    // device buffers
    DevBuf m_type, m_src, m_ballot, m_aux, m_ent, m_cnt, m_node, node_off, pair_gp, m_flags, m_maxseen;
    DevBuf m_gate, e_pid, ep_amask, ep_pmask, ep_ver, m_ver, ee_off, ee_msg, ee_state, sc_ver, sc_off;
    DevBuf chunk_node, chunk_beg, chunk_end, node_chunk_off, chunk_agg, chunk_carry, node_scal;
    DevBuf sc_type, sc_key, sc_idx, b_rbal, b_rsrc, b_bal;
    DevBuf e_val, e_slot, r_pid, r_val, r_slot, g_a, g_b;
    DevBuf f_off, frags, frag_w1, gp_list, ev_off, ev_msg, ev_aux, pl_off, pl_msg;
    DevBuf pc_node, pc_node_off, pc_beg, pc_end, pc_head, pc_state;
    uint64_t num_frags = 0;
    DevBuf b_msg, b_pstart, b_rep_off, b_rep, b_chosen, cf_off, cfrags;
    DevBuf st, st_valid, chosen, chosen_valid, plan, fast_rest, store_dummy, exec_aux, exec_out;
    DevBuf f_pid;                           // per run: an FR_UPID promise-reply run's proposal id
    DevBuf gp_dyn, gp_dyn_n;                // list plan path: the pairs k_plan_list lists for k_apply
    DevBuf gp_ext, gp_ext_n;                //   ... and those it describes by 5..8 segments (k_store_ext)
    DevBuf gp_chk, gp_chk_n;                //   ... and its planned pairs whose re-commits need the Value check
    DevBuf gp_rt, gp_rt_n;                  //   ... and (member) its 9..16-segment pairs, planned again
    DevBuf decode_buf;                      // readback scratch (k_decode)
    DevBuf out, out_cursor, partials, viol, summary;
    uint64_t out_cap = 0;
    uint32_t out_subs = 64;
    DevView view{};
    LaunchGeom geom{};
    uint64_t num_msgs = 0;
    // results of the last synchronised run
    std::vector<uint64_t> last_summary;
    mpx_stats stats{};
    // timing
    std::vector<StepEvents> ev_pool;
    size_t ev_used = 0;
    // comm
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1;
    DevBuf gather_buf;
    // the per-launch summary all-gather runs on its own stream, overlapped with the next
    // launch's kernels: summaries and gather buffers alternate between two slots, and a launch
    // waits only for the all-gather that last read its slot (two launches back)
    hipStream_t comm_stream = nullptr;
    hipStream_t stream2 = nullptr;                  // a run's promise-round pairs beside its plan path
    hipEvent_t fork_ev = nullptr, join_ev = nullptr;
    hipStream_t stream3 = nullptr;                  // the listed pairs and the chosen log beside the store chain
    hipEvent_t fork3a = nullptr, fork3b = nullptr, join3 = nullptr;
    hipEvent_t sum_ev[2] = {nullptr, nullptr}, ag_ev[2] = {nullptr, nullptr};
    bool ag_pending[2] = {false, false};
    uint32_t sum_idx = 0;
    DevBuf comm_buf, comm_buf2;             // mpx_comm_allreduce_max / mpx_comm_allgather_bytes
    // incremental runs (MPX_FLAG_INCREMENTAL): the host carry between windows,
    // the device state carried as values, and each node's records in earlier windows
    bool incremental = false;
    WindowCarry wc;
    DevBuf s_bal, s_val, p_pid, p_val, p_round, c_val, scal_base, scal_key, prop_in, prop_out;
    DevBuf b_gid, b_node, g_mask, g_done, gp_base, cb_list, outv, outv_n, ee_init, ee_out;
    bool ee_ready = false;                  // member: ee_init holds the roles the next window starts from
    uint64_t consumed = 0;                  // windows whose records build_trace took (the carry moved past them)
    bool poisoned = false;                  // a window failed after it was consumed, or a LEARN_EPOCHS submit
                                            // failed mid-stream: state undefined, every later call MPX_E_STATE
    uint64_t g_cap = 0;                     // global batches g_mask / g_done hold
    std::vector<uint64_t> seq_base, win_seq_base;
    std::vector<PropNode> *prop = nullptr;           // MPX_FLAG_DECISIONS: the bookkeeping carried across windows
    std::vector<MPropNode> *mprop = nullptr;         //   (member semantics: + the learn bookkeeping)
    LearnCarry *lrn = nullptr;
    uint64_t windows = 0;
    uint64_t events_every = 1, step_no = 0;   // mpx_timing_every
    uint32_t seq = 0;                         // launches so far (DevView::seq, the violation record's buffer)
};

static int hip_ok(hipError_t e) { return e == hipSuccess ? MPX_OK : MPX_E_HIP; }
// event k of a run (a run that ends with the store recorded no e[3], e[4]: they are e[2])
static hipEvent_t evk(const StepEvents &x, int k) { return x.store_last && k > 2 ? x.e[2] : x.e[k]; }
template <typename T> static int d2h(std::vector<T> &v, const DevBuf &b, size_t n, size_t off = 0)
{
    v.resize(n);
    if (!n) return MPX_OK;
    return hip_ok(hipMemcpy(v.data(), (const char *)b.p + off * sizeof(T), n * sizeof(T), hipMemcpyDeviceToHost));
}
#define TRY(x) do { int _rc = (x); if (_rc) return _rc; } while (0)
#define HTRY(x) do { if ((x) != hipSuccess) return MPX_E_HIP; } while (0)

static uint64_t now_ns()
{
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
        std::chrono::steady_clock::now().time_since_epoch()).count();
}

extern "C" int mpx_version(void) { return (int)MPX_ABI_VERSION; }

extern "C" int mpx_device_count(int *count)
{
    if (!count) return MPX_E_INVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return MPX_OK;
}

extern "C" int mpx_create(const mpx_config *cfg, mpx_engine **out)
{
    if (!cfg || !out) return MPX_E_INVAL;
    if (cfg->abi_version != MPX_ABI_VERSION) return MPX_E_INVAL;
    if (!cfg->num_nodes || cfg->num_nodes > MPX_MAX_NODES) return MPX_E_INVAL;
    if (cfg->shard_end <= cfg->shard_begin) return MPX_E_INVAL;
    if (cfg->semantics != MPX_SEM_MULTI && cfg->semantics != MPX_SEM_MEMBER) return MPX_E_INVAL;
    if (cfg->semantics == MPX_SEM_MULTI && cfg->num_epochs) return MPX_E_INVAL;
    if (cfg->flags & ~(uint32_t)(MPX_FLAG_INCREMENTAL | MPX_FLAG_DECISIONS | MPX_FLAG_LEARN_EPOCHS)) return MPX_E_INVAL;
    if ((cfg->flags & MPX_FLAG_LEARN_EPOCHS) &&
        (cfg->semantics != MPX_SEM_MEMBER || cfg->num_epochs != 1 || !cfg->epochs)) return MPX_E_INVAL;
    if ((cfg->flags & MPX_FLAG_DECISIONS) && !(cfg->flags & MPX_FLAG_INCREMENTAL)) return MPX_E_INVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return MPX_E_NODEVICE;
    if (cfg->device < 0 || cfg->device >= n) return MPX_E_NODEVICE;
    std::unique_ptr<mpx_engine> e(new mpx_engine);
    e->cfg = *cfg;
    if (cfg->epochs && cfg->num_epochs) e->epochs.assign(cfg->epochs, cfg->epochs + cfg->num_epochs);
    e->cfg.epochs = nullptr;
    e->device = cfg->device;
    HTRY(hipSetDevice(e->device));
    HTRY(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, e->device) == hipSuccess && prop.multiProcessorCount > 0)
        e->num_cus = (uint32_t)prop.multiProcessorCount;
    e->nodes.resize(cfg->num_nodes);
    if (cfg->flags & MPX_FLAG_LEARN_EPOCHS) {        // every node starts in the genesis epoch
        e->elearn.resize(cfg->num_nodes);
        for (auto &l : e->elearn) l.view = e->epochs[0];
    }
    e->vt.member = cfg->semantics == MPX_SEM_MEMBER;
    e->shard_len = cfg->shard_end - cfg->shard_begin;
    e->NB = (uint32_t)((e->shard_len + BS - 1) >> BSH);
    if ((uint64_t)e->NB * cfg->num_nodes > (1ull << 40)) return MPX_E_RANGE;
    if (cfg->flags & MPX_FLAG_INCREMENTAL) {
        // the carried state, as values: 16 B per (node, instance) for the acceptor / learner
        // entries and 16 B for a promise round's pre-accepted map, 8 B per instance of
        // chosen log (all zero: the PaxosImpl ctor state, multi/paxos.cpp:323-346)
        e->incremental = true;
        if ((cfg->flags & MPX_FLAG_DECISIONS) && cfg->semantics == MPX_SEM_MULTI) e->prop = prop_new(cfg->num_nodes);
        if ((cfg->flags & MPX_FLAG_DECISIONS) && cfg->semantics == MPX_SEM_MEMBER) {
            e->mprop = mprop_new(cfg->num_nodes);
            e->lrn = learn_new(cfg->num_nodes);
        }
        e->wc.init(cfg->num_nodes, e->NB);
        e->seq_base.assign(cfg->num_nodes, 0);
        const uint64_t NL = (uint64_t)cfg->num_nodes * e->shard_len;
        DevBuf *bufs[] = {&e->s_bal, &e->s_val, &e->p_pid, &e->p_val};
        for (DevBuf *b : bufs) TRY(b->alloc(8 * NL));
        TRY(e->p_round.alloc(8ull * cfg->num_nodes * e->NB)); TRY(e->c_val.alloc(8 * e->shard_len));
        TRY(e->scal_base.alloc(16ull * cfg->num_nodes)); TRY(e->scal_key.alloc(16ull * cfg->num_nodes));
        TRY(e->ee_init.alloc(4ull * cfg->num_nodes)); TRY(e->ee_out.alloc(4ull * cfg->num_nodes));
        TRY(e->prop_in.alloc(24ull * cfg->num_nodes)); TRY(e->prop_out.alloc(24ull * cfg->num_nodes));
        TRY(e->outv_n.alloc(8));
        DevBuf *z[] = {&e->s_bal, &e->s_val, &e->p_pid, &e->p_val, &e->p_round, &e->c_val, &e->scal_base, &e->prop_in,
                       &e->prop_out};
        for (DevBuf *b : z) HTRY(hipMemsetAsync(b->p, 0, b->bytes, e->stream));
        HTRY(hipStreamSynchronize(e->stream));
    }
    *out = e.release();
    return MPX_OK;
}

extern "C" int mpx_destroy(mpx_engine *e)
{
    if (!e) return MPX_E_INVAL;
    if (e->pf_pending) { e->pf_thread.join(); e->pf_pending = false; }
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    for (auto &s : e->ev_pool) for (auto ev : s.e) (void)hipEventDestroy(ev);
    if (e->comm_stream) (void)hipStreamSynchronize(e->comm_stream);
    if (e->comm) ncclCommDestroy(e->comm);
    for (int k = 0; k < 2; ++k) {
        if (e->sum_ev[k]) (void)hipEventDestroy(e->sum_ev[k]);
        if (e->ag_ev[k]) (void)hipEventDestroy(e->ag_ev[k]);
    }
    if (e->comm_stream) (void)hipStreamDestroy(e->comm_stream);
    if (e->stream2) (void)hipStreamSynchronize(e->stream2);
    if (e->fork_ev) (void)hipEventDestroy(e->fork_ev);
    if (e->join_ev) (void)hipEventDestroy(e->join_ev);
    if (e->stream2) (void)hipStreamDestroy(e->stream2);
    if (e->stream3) (void)hipStreamSynchronize(e->stream3);
    for (hipEvent_t x : {e->fork3a, e->fork3b, e->join3}) if (x) (void)hipEventDestroy(x);
    if (e->stream3) (void)hipStreamDestroy(e->stream3);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    prop_free(e->prop);
    mprop_free(e->mprop);
    learn_free(e->lrn);
    delete e;
    return MPX_OK;
}

// MPX_FLAG_LEARN_EPOCHS: the epochs each node reached (EpochLearn::steps) extend the table;
// nodes apply the same membership Values in the same instance order, so a node's k-th step
// must equal every other node's (the reference's safety: one chosen Value per instance)
// (every node is checked against the table and against the longest node before anything is
// appended, so a disagreement leaves the table as it was)
static int merge_epochs(mpx_engine *e)
{
    auto same = [](const mpx_epoch &a, const mpx_epoch &b) {
        return a.version == b.version && a.acceptor_mask == b.acceptor_mask && a.proposer_mask == b.proposer_mask &&
               a.learner_mask == b.learner_mask;
    };
    const EpochLearn *longest = nullptr;
    for (const EpochLearn &l : e->elearn)
        if (!longest || l.steps.size() > longest->steps.size()) longest = &l;
    if (!longest) return MPX_OK;
    for (const EpochLearn &l : e->elearn)
        for (size_t k = 0; k < l.steps.size(); ++k) {
            if (k + 1 < e->epochs.size() && !same(e->epochs[k + 1], l.steps[k])) return MPX_E_STATE;
            if (!same(longest->steps[k], l.steps[k])) return MPX_E_STATE;
        }
    for (size_t k = e->epochs.size() ? e->epochs.size() - 1 : 0; k < longest->steps.size(); ++k)
        e->epochs.push_back(longest->steps[k]);
    return MPX_OK;
}

// the pending background decode (mpx_submit_trace_range_async): joined, and its records queued
// behind any already queued (a node's queue is empty whenever a window was run in between, the
// pipelined use; otherwise the records are appended with their entry offsets rebased)
static int pf_join(mpx_engine *e)
{
    if (!e->pf_pending) return MPX_OK;
    e->pf_thread.join();
    e->pf_pending = false;
    e->stats.ingest_ns += e->pf_ns;
    if (e->pf_rc) return e->pf_rc;                  // (nothing consumed: the window is dropped, the engine stays)
    for (uint32_t n = 0; n < e->cfg.num_nodes; ++n) {
        NodeStream &ns = e->nodes[n], &p = e->pf_nodes[n];
        if (ns.type.empty()) { std::swap(ns, p); p.clear(); continue; }
        const uint64_t eb = ns.e_iid.size(), qb = ns.r_iid.size(), gb = ns.g_a.size();
        auto cat = [](auto &dst, const auto &src) { dst.insert(dst.end(), src.begin(), src.end()); };
        cat(ns.type, p.type); cat(ns.src, p.src); cat(ns.ballot, p.ballot); cat(ns.aux, p.aux);
        cat(ns.cnt, p.cnt); cat(ns.ver, p.ver); cat(ns.part, p.part); cat(ns.sec, p.sec);
        cat(ns.e_iid, p.e_iid); cat(ns.e_val, p.e_val); cat(ns.e_pid, p.e_pid);
        cat(ns.r_iid, p.r_iid); cat(ns.r_pid, p.r_pid); cat(ns.r_val, p.r_val);
        cat(ns.g_a, p.g_a); cat(ns.g_b, p.g_b);
        for (size_t k = 0; k < p.ent.size(); ++k) {
            const uint8_t t = p.type[k];
            const uint64_t base = t == MPX_MSG_PREPARE ? gb : t == MPX_MSG_PREPARE_REPLY ? qb :
                                  (t == MPX_MSG_ACCEPT || t == MPX_MSG_COMMIT || t == MPX_MSG_P_BATCH) ? eb : 0;
            ns.ent.push_back(p.ent[k] + base);
        }
        p.clear();
    }
    if (e->pf_iv.count) {
        if (!e->iv.code) e->iv = e->pf_iv;
        else e->iv.count += e->pf_iv.count;
    }
    e->pf_iv = IngestViolation();
    e->dirty = true;
    return MPX_OK;
}

extern "C" int mpx_read_epochs(mpx_engine *e, mpx_epoch *out, uint32_t cap, uint32_t *count)
{
    if (!e || !count || (cap && !out)) return MPX_E_INVAL;
    *count = (uint32_t)e->epochs.size();
    for (uint32_t k = 0; k < cap && k < e->epochs.size(); ++k) out[k] = e->epochs[k];
    return MPX_OK;
}

extern "C" int mpx_submit(mpx_engine *e, uint32_t node, const uint8_t *bytes, const uint64_t *offsets, uint64_t count)
{
    if (!e || node >= e->cfg.num_nodes || (count && (!bytes || !offsets))) return MPX_E_INVAL;
    if (e->poisoned) return MPX_E_STATE;            // (MPX_FLAG_INCREMENTAL: a failed window)
    if (e->device_trace) return MPX_E_STATE;
    TRY(pf_join(e));                                // (records queue in submission order)
    const uint64_t t0 = now_ns();
    NodeStream &ns = e->nodes[node];
    const bool member = e->cfg.semantics == MPX_SEM_MEMBER;
    for (uint64_t i = 0; i < count; ++i) {
        if (offsets[i + 1] < offsets[i]) return MPX_E_INVAL;
        const uint8_t *m = bytes + offsets[i];
        const size_t len = (size_t)(offsets[i + 1] - offsets[i]);
        int rc = member ? decode_record_member(e->vt, ns, node, m, len, e->cfg.shard_begin, e->cfg.shard_end, e->iv,
                                               e->elearn.empty() ? nullptr : &e->elearn[node])
                        : decode_record(e->vt, ns, node, e->cfg.num_nodes, m, len, e->cfg.shard_begin, e->cfg.shard_end, e->iv);
        if (rc) {
            // MPX_FLAG_LEARN_EPOCHS: the Learner's apply frontier, the node's view and its placed
            // E_EPOCH records may already have moved past the failing record: no
            // later call may run on that half-learned state
            if (!e->elearn.empty()) e->poisoned = true;
            return rc;
        }
    }
    if (int rc = merge_epochs(e)) { e->poisoned = true; return rc; }
    e->dirty = true;
    e->stats.ingest_ns += now_ns() - t0;
    return MPX_OK;
}

// SoA fast path: records the caller already holds decoded — a synthetic
// trace generator, or a host that keeps its messages as arrays — skip the wire codec.
extern "C" int mpx_submit_soa(mpx_engine *e, uint32_t node, const mpx_soa_records *r)
{
    if (!e || !r || node >= e->cfg.num_nodes) return MPX_E_INVAL;
    if (e->poisoned) return MPX_E_STATE;            // (MPX_FLAG_INCREMENTAL: a failed window)
    if (e->device_trace || e->cfg.semantics != MPX_SEM_MULTI) return MPX_E_STATE;
    TRY(pf_join(e));
    if (r->count && (!r->type || !r->src || !r->ballot || !r->aux || !r->ent_off)) return MPX_E_INVAL;
    const uint64_t t0 = now_ns();
    NodeStream &ns = e->nodes[node];
    for (uint64_t i = 0; i < r->count; ++i) {
        SoaRecord x{r->type[i], r->src[i], r->ballot[i], r->aux[i], 0, nullptr, nullptr, nullptr};
        if (r->ent_off[i + 1] < r->ent_off[i]) return MPX_E_INVAL;
        x.n = r->ent_off[i + 1] - r->ent_off[i];
        if (x.n) {
            if (!r->ent_a || !r->ent_b) return MPX_E_INVAL;
            x.a = r->ent_a + r->ent_off[i]; x.b = r->ent_b + r->ent_off[i];
            x.pid = r->ent_pid ? r->ent_pid + r->ent_off[i] : nullptr;
        }
        TRY(append_record(e->vt, ns, node, x, e->cfg.shard_begin, e->cfg.shard_end, e->iv));
    }
    e->dirty = true;
    e->stats.ingest_ns += now_ns() - t0;
    return MPX_OK;
}

static inline uint32_t rd32(const uint8_t *p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
static inline uint64_t rd64(const uint8_t *p) { uint64_t v; std::memcpy(&v, p, 8); return v; }

// the records [begin[n], end[n]) of every node's stream of an MPXT container (nullptr: all of them)
static int submit_container(mpx_engine *e, const uint8_t *t, uint64_t size, const uint64_t *begin, const uint64_t *end,
                            bool async = false)
{
    if (!e || !t || size < 40 || std::memcmp(t, "MPXT", 4)) return MPX_E_INVAL;
    if (e->poisoned) return MPX_E_STATE;            // (MPX_FLAG_INCREMENTAL: a failed window)
    TRY(pf_join(e));                                // (records queue in submission order)
    const uint32_t N = rd32(t + 8), sem = rd32(t + 12), ne = rd32(t + 24), ver = rd32(t + 4);
    if (N != e->cfg.num_nodes || sem != e->cfg.semantics || ver < 1 || ver > 2) return MPX_E_INVAL;
    const uint32_t esz = ver == 1 ? 24 : 32;         // version 1: no learner_mask (= proposer_mask)
    if (size < 40 + (uint64_t)ne * esz) return MPX_E_DECODE;
    if (ne && e->elearn.empty()) {
        // the container's epoch table: adopted by an engine created without
        // one, else it must be the same table (MPX_FLAG_LEARN_EPOCHS: the engine learns its own)
        std::vector<mpx_epoch> ep(ne);
        for (uint32_t k = 0; k < ne; ++k) {
            const uint8_t *x = t + 40 + (size_t)k * esz;
            ep[k] = mpx_epoch{rd32(x), rd32(x + 4), rd64(x + 8), rd64(x + 16), esz == 32 ? rd64(x + 24) : rd64(x + 16)};
        }
        if (e->epochs.empty()) e->epochs = ep;
        else if (e->epochs.size() != ep.size() || std::memcmp(e->epochs.data(), ep.data(), (size_t)ne * sizeof(mpx_epoch)))
            return MPX_E_INVAL;
    }
    size_t pos = 40 + (size_t)ne * esz;
    std::vector<size_t> at(N);                      // each node's stream: count word
    for (uint32_t n = 0; n < N; ++n) {
        if (pos + 16 > size) return MPX_E_DECODE;
        const uint64_t cnt = rd64(t + pos), nb = rd64(t + pos + 8);
        at[n] = pos;
        pos += 16;
        if (pos + 8 * (cnt + 1) + nb > size) return MPX_E_DECODE;
        pos += 8 * (cnt + 1) + nb;
        pos = (pos + 7) & ~(size_t)7;
    }
    if (begin && end)
        for (uint32_t n = 0; n < N; ++n)
            if (begin[n] > end[n] || end[n] > rd64(t + at[n])) return MPX_E_INVAL;
    // node n's records [k0, k1): offs[k0 .. k1] index the container's record bytes
    auto stream = [&](uint32_t n, const uint64_t *&offs, const uint8_t *&bytes) {
        const uint64_t cnt = rd64(t + at[n]);
        const uint64_t k0 = begin ? begin[n] : 0, k1 = end ? end[n] : cnt;
        offs = reinterpret_cast<const uint64_t *>(t + at[n] + 16) + k0;    // 8-aligned in the container
        bytes = t + at[n] + 16 + 8 * (cnt + 1);
        return k1 - k0;
    };
    uint64_t total = 0;
    for (uint32_t n = 0; n < N; ++n) { const uint64_t *o; const uint8_t *b; const uint64_t c = stream(n, o, b); if (c) total += o[c] - o[0]; }
    if (async) {
        // the window's records decoded on a host thread (into pf_nodes) while the caller runs the
        // windows queued before it; multi semantics (no learned epochs: the decode would move the
        // epoch table under a running window)
        std::vector<StreamSlice> sl(N);
        for (uint32_t n = 0; n < N; ++n) sl[n].cnt = stream(n, sl[n].offs, sl[n].bytes);
        if (e->pf_nodes.size() < N) e->pf_nodes.resize(N);
        for (auto &x : e->pf_nodes) x.clear();
        e->pf_iv = IngestViolation();
        e->pf_rc = MPX_OK;
        e->pf_pending = true;
        e->pf_thread = std::thread([e, sl]() {
            const uint64_t t0 = now_ns();
            e->pf_rc = decode_parallel(e->vt, e->pf_nodes, e->pf_parts, sl, false, nullptr, e->cfg.shard_begin,
                                       e->cfg.shard_end, e->pf_iv,
                                       std::max(1u, std::min(16u, std::thread::hardware_concurrency())), 0);
            e->pf_ns = now_ns() - t0;
        });
        return MPX_OK;
    }
    if (N == 1 || total < (1u << 20) || e->device_trace) {
        for (uint32_t n = 0; n < N; ++n) {
            const uint64_t *offs; const uint8_t *bytes;
            const uint64_t cnt = stream(n, offs, bytes);
            TRY(mpx_submit(e, n, bytes, offs, cnt));
        }
        return MPX_OK;
    }
    // large traces: every node's stream cut into chunks decoded on a pool of host threads
    // (ingest.cpp decode_parallel)
    const uint64_t t0 = now_ns();
    std::vector<StreamSlice> sl(N);
    for (uint32_t n = 0; n < N; ++n) sl[n].cnt = stream(n, sl[n].offs, sl[n].bytes);
    if (int rc = decode_parallel(e->vt, e->nodes, e->parts, sl, e->cfg.semantics == MPX_SEM_MEMBER,
                                 e->elearn.empty() ? nullptr : &e->elearn, e->cfg.shard_begin, e->cfg.shard_end, e->iv,
                                 std::max(1u, std::min(16u, std::thread::hardware_concurrency())), 0)) {
        if (!e->elearn.empty()) e->poisoned = true;  // (see mpx_submit)
        return rc;
    }
    if (int rc = merge_epochs(e)) { e->poisoned = true; return rc; }
    e->dirty = true;
    e->stats.ingest_ns += now_ns() - t0;
    return MPX_OK;
}

extern "C" int mpx_submit_trace(mpx_engine *e, const uint8_t *t, uint64_t size)
{
    return submit_container(e, t, size, nullptr, nullptr);
}

extern "C" int mpx_submit_trace_range(mpx_engine *e, const uint8_t *t, uint64_t size, const uint64_t *begin,
                                      const uint64_t *end)
{
    if (!e || !begin || !end) return MPX_E_INVAL;
    return submit_container(e, t, size, begin, end);
}

// The same records decoded in the background: the call returns at once, and the decode overlaps
// the build and device run of the windows queued before it (mpx_run joins it only when nothing
// else is queued; every call that reads the value table or adds records joins it first).
// Incremental multi-semantics engines; the caller keeps `t` alive until the records are joined.
extern "C" int mpx_submit_trace_range_async(mpx_engine *e, const uint8_t *t, uint64_t size, const uint64_t *begin,
                                            const uint64_t *end)
{
    if (!e || !begin || !end) return MPX_E_INVAL;
    if (!e->incremental || e->cfg.semantics != MPX_SEM_MULTI || !e->elearn.empty() || e->device_trace)
        return MPX_E_STATE;
    return submit_container(e, t, size, begin, end, true);
}

// allocate state / output buffers and fill the kernel view
static int finish_view(mpx_engine *e)
{
    const uint32_t N = e->cfg.num_nodes;
    DevView &v = e->view;
    v.N = N;
    v.quorum = N / 2 + 1;                          // nodes_.size() / 2 + 1, paxos.cpp:1047,1416
    v.NB = e->NB;
    v.scan_node_pass = 0;
    v.scan_chunk = e->ht.scan_chunk;
    for (size_t n = 0; n + 1 < e->ht.node_chunk_off.size(); ++n)
        if (e->ht.node_chunk_off[n + 1] - e->ht.node_chunk_off[n] > SCAN_INLINE_CHUNKS) v.scan_node_pass = 1;
    if (const char *x = std::getenv("MPX_SCAN_NODE_PASS")) v.scan_node_pass = std::atoi(x) ? 1 : 0;
    v.semantics = e->cfg.semantics;
    v.shard_begin = e->cfg.shard_begin;
    v.shard_len = e->shard_len;
    v.num_msgs = e->num_msgs;
    // slot width: 1 byte when every pair / bucket has few enough fragments for a
    // 1-byte pair-local index (set by the trace loader), MPX_SLOT_BYTES=2 forces 2
    if (const char *x = std::getenv("MPX_SLOT_BYTES")) if (std::atoi(x) == 2) v.slot_w = 2;
    if (v.slot_w != 1) v.slot_w = 2;
    // (incremental windows keep their state as values, DevView s_* / c_val: no slot rows, plans)
    TRY(e->st.alloc(e->incremental ? 8 : (size_t)(N + 1) * e->shard_len * v.slot_w));   // row N: the chosen log
    TRY(e->st_valid.alloc(e->incremental ? 8 : (size_t)N * e->NB));
    TRY(e->chosen_valid.alloc(e->incremental ? 8 : e->NB));
    TRY(e->plan.alloc(e->incremental ? 8 : (size_t)(N + 1) * e->NB * 8));
    {   // promise-quorum chunks over each node's proposer list (k_prop_chunk / k_prop_node)
        const HostTrace &h = e->ht;
        uint64_t pc = PROP_CHUNK;                       // MPX_PROP_CHUNK: smaller chunks (tests)
        if (const char *x = std::getenv("MPX_PROP_CHUNK")) pc = std::max<uint64_t>(1, std::strtoull(x, nullptr, 10));
        std::vector<uint32_t> pn, pno(N + 1, 0);
        std::vector<uint64_t> pb, pe;
        uint32_t multi = 0;
        for (uint32_t n = 0; n < N && n + 1 < h.pl_off.size(); ++n) {
            pno[n] = (uint32_t)pn.size();
            for (uint64_t a = h.pl_off[n]; a < h.pl_off[n + 1]; a += pc) {
                pn.push_back(n); pb.push_back(a); pe.push_back(std::min<uint64_t>(a + pc, h.pl_off[n + 1]));
                if (a != h.pl_off[n]) multi = 1;
            }
        }
        pno[N] = (uint32_t)pn.size();
        v.pc_multi = multi;
        TRY(upload(e->pc_node, pn, e->stream)); TRY(upload(e->pc_node_off, pno, e->stream));
        TRY(upload(e->pc_beg, pb, e->stream)); TRY(upload(e->pc_end, pe, e->stream));
        TRY(e->pc_head.alloc(std::max<size_t>(4 * pn.size(), 4))); TRY(e->pc_state.alloc(std::max<size_t>(24 * pn.size(), 24)));
        v.num_pc = (uint32_t)pn.size();
        v.pc_node = e->pc_node.as<uint32_t>(); v.pc_node_off = e->pc_node_off.as<uint32_t>();
        v.pc_beg = e->pc_beg.as<uint64_t>(); v.pc_end = e->pc_end.as<uint64_t>();
        v.pc_head = e->pc_head.as<uint32_t>(); v.pc_state = e->pc_state.as<uint64_t>();
        HTRY(hipStreamSynchronize(e->stream));          // the host vectors are locals
    }
    TRY(e->frag_w1.alloc(std::max<size_t>(8 * e->num_frags, 8)));
    if (launch_frag_w1(v.frags, e->frag_w1.as<uint64_t>(), e->num_frags, e->stream) != 0) return MPX_E_HIP;
    v.frag_w1 = e->frag_w1.as<uint64_t>();
    TRY(e->fast_rest.alloc(8));
    TRY(e->store_dummy.alloc(64 * 1024));
    // k_plan_list lists at most the work list's non-round pairs
    TRY(e->gp_dyn.alloc(std::max<size_t>(8ull * GP_WORDS * v.num_gp_snap, 8 * GP_WORDS)));
    TRY(e->gp_dyn_n.alloc(8));
    v.gp_dyn = e->gp_dyn.as<uint64_t>();
    v.gp_dyn_n = e->gp_dyn_n.as<unsigned long long>();
    TRY(e->gp_ext.alloc(std::max<size_t>(8ull * EXT_WORDS * v.num_gp_snap, 8 * EXT_WORDS)));
    TRY(e->gp_ext_n.alloc(8));
    v.gp_ext = e->gp_ext.as<uint64_t>();
    v.gp_ext_n = e->gp_ext_n.as<unsigned long long>();
    TRY(e->gp_chk.alloc(std::max<size_t>(8ull * CHK_WORDS * v.num_gp_snap, 8 * CHK_WORDS)));
    TRY(e->gp_chk_n.alloc(8));
    v.gp_chk = e->gp_chk.as<uint64_t>();
    v.gp_chk_n = e->gp_chk_n.as<unsigned long long>();
    TRY(e->gp_rt.alloc(std::max<size_t>(8ull * v.num_gp_snap, 8)));
    TRY(e->gp_rt_n.alloc(8));
    v.gp_rt = e->gp_rt.as<uint64_t>();
    v.gp_rt_n = e->gp_rt_n.as<unsigned long long>();
    e->geom = launch_geometry(N, e->NB, e->num_cus);

    TRY(e->partials.alloc(8ull * 8 * ((uint64_t)e->num_cus * 16 + std::max<uint64_t>(e->geom.chosen_wgs, e->num_cus * 16))));
    TRY(e->viol.alloc(2 * sizeof(DevViolation)));                     // double-buffered (reset_state)
    HTRY(hipMemsetAsync(e->viol.p, 0, 2 * sizeof(DevViolation), e->stream));
    TRY(e->summary.alloc(2 * 64 * 8));                                // two slots (comm overlap)
    e->out_subs = 64;
    if (const char *x = ab_env("MPX_OUT_SUBS")) {  // A/B: snapshot sub-buffers (power of two)
        const uint32_t k = (uint32_t)std::atoi(x);
        if (k && !(k & (k - 1)) && k <= OUT_SUBS) e->out_subs = k;
    }
    TRY(e->out_cursor.alloc(8ull * OUT_STRIDE * e->out_subs));
    if (!e->out_cap) e->out_cap = 1 << 12;               // records per sub-buffer
    TRY(e->out.alloc((uint64_t)e->out_subs * e->out_cap * sizeof(OutRec)));
    TRY(e->node_scal.alloc(16ull * N));
    v.st = e->st.p;
    v.st_valid = e->st_valid.as<uint8_t>();
        v.chosen_valid = e->chosen_valid.as<uint8_t>();
    v.plan = e->plan.as<uint64_t>();
    v.fast_rest = e->fast_rest.as<uint32_t>();
    v.store_dummy = e->store_dummy.as<uint32_t>();
    v.out = e->out.as<OutRec>();
    v.out_cursor = e->out_cursor.as<unsigned long long>();
    v.out_cap = e->out_cap;
    v.out_subs = e->out_subs;
    v.partials = e->partials.as<unsigned long long>();
    v.viol = e->viol.as<DevViolation>();
    v.viol_next = e->viol.as<DevViolation>() + 1;
    v.summary = e->summary.as<unsigned long long>() + 64 * e->sum_idx;
    v.node_scal = e->node_scal.as<uint64_t>();
    return MPX_OK;
}

static int upload_trace(mpx_engine *e)
{
    const uint64_t t0 = now_ns();
    const bool member = e->cfg.semantics == MPX_SEM_MEMBER;
    if (member && e->epochs.empty()) return MPX_E_STATE;        // no epoch table yet
    TRY(build_trace(e->nodes, e->cfg.shard_begin, e->shard_len, member ? e->epochs : std::vector<mpx_epoch>(), e->ht,
                    e->incremental ? &e->wc : nullptr));
    e->ab_build_ns = now_ns() - t0;
    if (e->incremental) {
        // the window is consumed: the next run builds on the carry from only what comes after it
        ++e->consumed;
        e->win_seq_base = e->seq_base;
        for (uint32_t n = 0; n < e->cfg.num_nodes; ++n) {
            e->seq_base[n] += e->nodes[n].type.size();
            e->nodes[n].clear();
        }
    }
    e->whole = e->cfg.shard_begin == 0 && e->ht.part_dropped == 0;
    HostTrace &h = e->ht;
    hipStream_t s = e->stream;
    {   // member: the epoch table and the markers; the gates are computed on the device (k_gate_*)
        std::vector<uint64_t> am, pm;
        std::vector<uint32_t> ver;
        for (auto &x : e->epochs) { am.push_back(x.acceptor_mask); pm.push_back(x.proposer_mask); ver.push_back(x.version); }
        TRY(upload(e->ep_amask, am, s)); TRY(upload(e->ep_pmask, pm, s)); TRY(upload(e->ep_ver, ver, s));
        TRY(e->m_gate.alloc(std::max<size_t>(4 * (member ? h.m_type.size() : 0), 4)));
        TRY(upload(e->m_ver, h.m_ver, s));
        TRY(upload(e->ee_off, h.ee_off, s)); TRY(upload(e->ee_msg, h.ee_msg, s));
        TRY(e->ee_state.alloc(std::max<size_t>(4 * h.ee_msg.size(), 4)));
        TRY(upload(e->sc_ver, h.sc_ver, s)); TRY(upload(e->sc_off, h.sc_off, s));
        TRY(upload(e->e_pid, h.e_pid, s));
        HTRY(hipStreamSynchronize(s));                 // am / pm / ver are locals
    }
    TRY(upload(e->m_type, h.m_type, s)); TRY(upload(e->m_src, h.m_src, s));
    TRY(upload(e->m_ballot, h.m_ballot, s)); TRY(upload(e->m_aux, h.m_aux, s));
    TRY(upload(e->m_ent, h.m_ent, s)); TRY(upload(e->m_cnt, h.m_cnt, s));
    TRY(upload(e->m_node, h.m_node, s)); TRY(upload(e->node_off, h.node_off, s));
    {
        std::vector<uint8_t> gp(h.pair_gp);
        gp.resize(gp.size() + 8, 0);                   // dword slack (k_plan_store8)
        TRY(upload(e->pair_gp, gp, s));
        HTRY(hipStreamSynchronize(s));
    }
    TRY(upload(e->m_flags, h.m_flags0, s));             // static flags; the steps rewrite the dynamic ones
    if (e->m_flags.bytes < h.m_flags0.size() + 8) {    // + a dword of slack: k_plan_store8 reads flags as dwords
        std::vector<uint8_t> f(h.m_flags0);
        f.resize(f.size() + 8, 0);
        TRY(upload(e->m_flags, f, s));
        HTRY(hipStreamSynchronize(s));
    }
    TRY(upload(e->sc_type, h.sc_type, s)); TRY(upload(e->sc_key, h.sc_key, s)); TRY(upload(e->sc_idx, h.sc_idx, s));
    TRY(upload(e->b_rbal, h.b_rbal, s)); TRY(upload(e->b_rsrc, h.b_rsrc, s)); TRY(upload(e->b_bal, h.b_bal, s));
    TRY(e->m_maxseen.alloc(std::max<size_t>(h.m_type.size() * 8, 8)));
    TRY(upload(e->chunk_node, h.chunk_node, s)); TRY(upload(e->chunk_beg, h.chunk_beg, s));
    TRY(upload(e->chunk_end, h.chunk_end, s)); TRY(upload(e->node_chunk_off, h.node_chunk_off, s));
    TRY(e->chunk_agg.alloc(std::max<size_t>(16 * h.chunk_node.size(), 16)));
    TRY(e->chunk_carry.alloc(std::max<size_t>(16 * h.chunk_node.size(), 16)));
    TRY(upload(e->e_val, h.e_val, s)); TRY(upload(e->e_slot, h.e_slot, s));
    TRY(upload(e->r_pid, h.r_pid, s)); TRY(upload(e->r_val, h.r_val, s)); TRY(upload(e->r_slot, h.r_slot, s));
    TRY(upload(e->g_a, h.g_a, s)); TRY(upload(e->g_b, h.g_b, s));
    TRY(upload(e->f_off, h.f_off, s)); TRY(upload(e->frags, h.frags, s)); TRY(upload(e->f_pid, h.f_pid, s));
    {   // work items of the general k_apply: {f_off[q], f_off[q + 1], ev_off[q], ev_off[q + 1], q}
        std::vector<uint64_t> gd(GP_WORDS * h.gp_list.size(), 0);
        for (size_t i = 0; i < h.gp_list.size(); ++i) {
            const uint64_t q = h.gp_list[i];
            uint64_t *w = &gd[GP_WORDS * i];
            w[0] = h.f_off[q]; w[1] = h.f_off[q + 1]; w[2] = h.ev_off[q]; w[3] = h.ev_off[q + 1]; w[4] = q;
        }
        TRY(upload(e->gp_list, gd, s));
        HTRY(hipStreamSynchronize(s));                 // gd is a local
        if (ab_env("MPX_TRACE_STATS")) {          // shape of the general work list (tools)
            uint64_t fr = 0, ev = 0, mx = 0, pre = 0;
            for (uint64_t q : h.gp_list) {
                fr += h.f_off[q + 1] - h.f_off[q]; ev += h.ev_off[q + 1] - h.ev_off[q];
                mx = std::max<uint64_t>(mx, h.f_off[q + 1] - h.f_off[q]);
                for (uint64_t f = h.f_off[q]; f < h.f_off[q + 1]; ++f) pre += (h.frags[f].flags >> 4) == K_PREPLY;
            }
            uint64_t sfr = 0;
            for (uint64_t i = 0; i < h.num_gp_simple; ++i) sfr += h.f_off[h.gp_list[i] + 1] - h.f_off[h.gp_list[i]];
            std::fprintf(stderr, "[mpx] pairs %llu, general %zu (simple %llu, their runs %llu): runs %llu (promise-reply runs %llu, "
                         "max/pair %llu), events %llu; all runs %zu, messages %zu\n", (unsigned long long)((uint64_t)h.N * h.NB),
                         h.gp_list.size(), (unsigned long long)h.num_gp_simple, (unsigned long long)sfr, (unsigned long long)fr,
                         (unsigned long long)pre, (unsigned long long)mx, (unsigned long long)ev, h.frags.size(), h.m_type.size());
        }
    }
    TRY(upload(e->ev_off, h.ev_off, s)); TRY(upload(e->ev_msg, h.ev_msg, s)); TRY(upload(e->ev_aux, h.ev_aux, s));
    TRY(upload(e->pl_off, h.pl_off, s)); TRY(upload(e->pl_msg, h.pl_msg, s));
    TRY(upload(e->b_msg, h.b_msg, s)); TRY(upload(e->b_pstart, h.b_pstart, s));
    TRY(upload(e->b_rep_off, h.b_rep_off, s)); TRY(upload(e->b_rep, h.b_rep, s));
    TRY(e->b_chosen.alloc(std::max<size_t>(4 * h.b_msg.size(), 4)));
    TRY(upload(e->cf_off, h.cf_off, s)); TRY(upload(e->cfrags, h.cfrags, s));
    e->num_msgs = h.m_type.size();
    DevView &v = e->view;
    if (e->incremental) {
        TRY(upload(e->b_gid, h.b_gid, s)); TRY(upload(e->gp_base, h.gp_base, s)); TRY(upload(e->cb_list, h.cb_list, s));
        TRY(upload(e->b_node, h.b_node, s));
        if (member && !e->ee_ready) {
            // the first window starts from the genesis roles (Loop: {first} is learner, proposer
            // and acceptor, member/paxos.cpp:738-747; epochs[0] of the table)
            std::vector<uint32_t> g0(e->cfg.num_nodes);
            for (uint32_t n = 0; n < e->cfg.num_nodes; ++n)
                g0[n] = (1u << EE_SEG_SHIFT) | (((e->epochs[0].acceptor_mask >> n) & 1) ? EE_ACC : 0) |
                        (((e->epochs[0].proposer_mask >> n) & 1) ? EE_PROP : 0);
            TRY(upload(e->ee_init, g0, s));
            HTRY(hipStreamSynchronize(s));                 // g0 is a local
            e->ee_ready = true;
        }
        if (e->wc.batches > e->g_cap) {                 // the batches' votes, grown geometrically (kept values copied)
            const uint64_t cap = std::max<uint64_t>(e->wc.batches, 2 * e->g_cap);
            DevBuf nm, nd;
            TRY(nm.alloc(8 * cap)); TRY(nd.alloc(cap));
            HTRY(hipMemsetAsync(nm.p, 0, 8 * cap, s)); HTRY(hipMemsetAsync(nd.p, 0, cap, s));
            if (e->g_cap) {
                HTRY(hipMemcpyAsync(nm.p, e->g_mask.p, 8 * e->g_cap, hipMemcpyDeviceToDevice, s));
                HTRY(hipMemcpyAsync(nd.p, e->g_done.p, e->g_cap, hipMemcpyDeviceToDevice, s));
            }
            HTRY(hipStreamSynchronize(s));
            std::swap(e->g_mask.p, nm.p); std::swap(e->g_mask.bytes, nm.bytes);
            std::swap(e->g_done.p, nd.p); std::swap(e->g_done.bytes, nd.bytes);
            e->g_cap = cap;
        }
        // snapshot records: at most one per slot of every listed event (PREPARE or quorum)
        const uint64_t cap = std::max<uint64_t>(BS * h.ev_msg.size(), 1);
        TRY(e->outv.alloc(cap * sizeof(OutEnt)));
        v.window = 1;
        v.s_bal = e->s_bal.as<uint64_t>(); v.s_val = e->s_val.as<uint64_t>();
        v.p_pid = e->p_pid.as<uint64_t>(); v.p_val = e->p_val.as<uint64_t>(); v.p_round = e->p_round.as<uint64_t>();
        v.c_val = e->c_val.as<uint64_t>(); v.scal_base = e->scal_base.as<uint64_t>(); v.scal_key = e->scal_key.as<uint64_t>();
        v.b_node = e->b_node.as<uint32_t>(); v.ee_init = e->ee_init.as<uint32_t>(); v.ee_out = e->ee_out.as<uint32_t>();
        v.prop_in = e->prop_in.as<uint64_t>(); v.prop_out = e->prop_out.as<uint64_t>();
        v.b_gid = e->b_gid.as<uint32_t>(); v.g_mask = e->g_mask.as<uint64_t>(); v.g_done = e->g_done.as<uint8_t>();
        v.gp_base = e->gp_base.as<uint8_t>(); v.cb_list = e->cb_list.as<uint32_t>(); v.num_cb = (uint32_t)h.cb_list.size();
        v.outv = e->outv.as<OutEnt>(); v.outv_n = e->outv_n.as<unsigned long long>(); v.outv_cap = cap;
    }
    v.m_type = e->m_type.as<uint8_t>(); v.m_src = e->m_src.as<uint32_t>();
    v.m_ballot = e->m_ballot.as<uint64_t>(); v.m_aux = e->m_aux.as<uint64_t>();
    v.m_ent = e->m_ent.as<uint64_t>(); v.m_cnt = e->m_cnt.as<uint32_t>();
    v.m_node = e->m_node.as<uint32_t>(); v.node_off = e->node_off.as<uint64_t>();
    v.pair_gp = e->pair_gp.as<uint8_t>();
    v.m_flags = e->m_flags.as<uint8_t>(); v.m_maxseen = e->m_maxseen.as<uint64_t>();
    v.m_gate = e->m_gate.as<uint32_t>(); v.e_pid = e->e_pid.as<uint64_t>();
    v.ep_amask = e->ep_amask.as<uint64_t>(); v.num_epochs = (uint32_t)e->epochs.size();
    v.ep_pmask = e->ep_pmask.as<uint64_t>(); v.ep_ver = e->ep_ver.as<uint32_t>();
    v.m_ver = e->m_ver.as<uint32_t>(); v.ee_off = e->ee_off.as<uint64_t>(); v.ee_msg = e->ee_msg.as<uint32_t>();
    v.ee_state = e->ee_state.as<uint32_t>(); v.sc_ver = e->sc_ver.as<uint32_t>(); v.sc_off = e->sc_off.as<uint64_t>();
    v.num_sc = h.sc_type.size();
    v.num_chunks = (uint32_t)h.chunk_node.size();
    v.chunk_node = e->chunk_node.as<uint32_t>(); v.chunk_beg = e->chunk_beg.as<uint64_t>();
    v.chunk_end = e->chunk_end.as<uint64_t>(); v.node_chunk_off = e->node_chunk_off.as<uint32_t>();
    v.chunk_agg = e->chunk_agg.as<uint64_t>(); v.chunk_carry = e->chunk_carry.as<uint64_t>();
    v.e_val = e->e_val.as<uint64_t>(); v.e_slot = e->e_slot.as<uint8_t>();
    v.r_pid = e->r_pid.as<uint64_t>(); v.r_val = e->r_val.as<uint64_t>(); v.r_slot = e->r_slot.as<uint8_t>();
    v.g_a = e->g_a.as<uint64_t>(); v.g_b = e->g_b.as<uint64_t>();
    v.f_off = e->f_off.as<uint64_t>(); v.frags = e->frags.as<Frag>(); v.f_pid = e->f_pid.as<uint64_t>();
    e->num_frags = h.frags.size();
    v.num_gp = h.gp_list.size(); v.gp_list = e->gp_list.as<uint64_t>(); v.num_gp_simple = h.num_gp_simple; v.num_gp_snap = h.num_gp_snap;
    v.ev_off = e->ev_off.as<uint64_t>(); v.ev_msg = e->ev_msg.as<uint32_t>(); v.ev_aux = e->ev_aux.as<uint64_t>();
    v.pl_off = e->pl_off.as<uint64_t>(); v.pl_msg = e->pl_msg.as<uint32_t>();
    v.num_batches = (uint32_t)h.b_msg.size();
    v.b_msg = e->b_msg.as<uint32_t>(); v.b_pstart = e->b_pstart.as<uint32_t>();
    v.b_rep_off = e->b_rep_off.as<uint64_t>(); v.b_rep = e->b_rep.as<uint32_t>();
    v.b_rbal = e->b_rbal.as<uint64_t>(); v.b_rsrc = e->b_rsrc.as<uint32_t>(); v.b_bal = e->b_bal.as<uint64_t>();
    v.sc_type = e->sc_type.as<uint8_t>(); v.sc_key = e->sc_key.as<uint64_t>(); v.sc_idx = e->sc_idx.as<uint32_t>();
    v.b_chosen = e->b_chosen.as<uint32_t>();
    v.cf_off = e->cf_off.as<uint64_t>(); v.cfrags = e->cfrags.as<Frag>();
    {   // plan_chosen's static test over every bucket's chosen-log runs (kernels.hip launch_run)
        bool ok = true;
        for (uint64_t b = 0; ok && b + 1 < h.cf_off.size(); ++b) {
            const uint64_t c0 = h.cf_off[b], c1 = h.cf_off[b + 1];
            if (c0 == c1) continue;
            uint32_t sp[3] = {BS, BS, BS};
            ok = c1 - c0 <= 4 && (b + 1) * BS <= e->shard_len;
            for (uint64_t k = c0; ok && k < c1; ++k) {
                const Frag &f = h.cfrags[k];
                ok = (f.flags & FR_DENSE) && plan_add_split(f.start, sp) && plan_add_split(f.start + f.count, sp);
                for (uint64_t j = c0; ok && j < k; ++j)
                    ok = h.cfrags[j].start + h.cfrags[j].count <= f.start || f.start + f.count <= h.cfrags[j].start;
            }
        }
        v.chosen_static = ok ? 1 : 0;
        v.any_vchk = 0;                              // (ingest marks only runs whose Values can differ)
        for (const Frag &f : h.frags) if (f.flags & FR_VCHK) { v.any_vchk = 1; break; }
    }
    {
        uint64_t mx = 0;
        for (size_t i = 0; i + 1 < h.f_off.size(); ++i) mx = std::max<uint64_t>(mx, h.f_off[i + 1] - h.f_off[i]);
        for (size_t i = 0; i + 1 < h.cf_off.size(); ++i) mx = std::max<uint64_t>(mx, h.cf_off[i + 1] - h.cf_off[i]);
        v.slot_w = mx <= MAX_PAIR_FRAGS_1 ? 1 : 2;
    }
    TRY(finish_view(e));
    HTRY(hipStreamSynchronize(s));
    e->dirty = false;
    e->stats.ingest_ns += now_ns() - t0;
    return MPX_OK;
}

static StepEvents *next_events(mpx_engine *e)
{
    if (e->ev_used == e->ev_pool.size()) {
        StepEvents se{};
        for (auto &x : se.e)
            if (hipEventCreate(&x) != hipSuccess) return nullptr;
        e->ev_pool.push_back(se);
    }
    return &e->ev_pool[e->ev_used++];
}

static int queue_run(mpx_engine *e, bool digest)
{
    HTRY(hipSetDevice(e->device));
    if (e->dirty && !e->device_trace) TRY(upload_trace(e));
    // phase events (per-kernel start / stop timestamps) on every k-th step only
    // (mpx_timing_every; MPX_EVENTS_EVERY overrides): they cost a step ~1.5-2 us per timed
    // kernel boundary (C4 shard at world 8: 89 vs 75 us per step)
    uint64_t every = e->events_every;
    if (const char *x = ab_env("MPX_EVENTS_EVERY")) every = std::strtoull(x, nullptr, 10);
    const bool timed = digest || every == 1 || (every && (e->step_no % every) == 0);
    ++e->step_no;
    StepEvents *ev = timed ? next_events(e) : nullptr;
    if (timed && !ev) return MPX_E_HIP;
    // grid sizes: the defaults are the measured best; the MPX_*_WGS_PER_CU overrides are for
    // sweeps (tools/)
    LaunchGeom g = e->geom;
    e->view.digest = digest ? 1 : 0;
    // MPX_STEP_WALK=1: a step walks every pair as the digested run does (no plan words)
    e->view.walk_all = 0;
    if (const char *x = std::getenv("MPX_STEP_WALK")) e->view.walk_all = std::atoi(x) ? 1 : 0;
    if (const char *x = ab_env("MPX_STORE_WGS_PER_CU")) g.store_wgs = std::max<uint32_t>(1, e->num_cus * (uint32_t)std::atoi(x));
    // MPX_PLAN_STORE=0: the C4 shape takes k_plan + k_store8 (the path before k_plan_store8)
    if (const char *x = std::getenv("MPX_PLAN_STORE")) if (!std::atoi(x)) g.ps_wgs = 0;
    if (const char *x = ab_env("MPX_PS_WGS_PER_CU")) g.ps_wgs = std::max<uint32_t>(1, e->num_cus * (uint32_t)std::atoi(x));
    if (const char *x = ab_env("MPX_CHOSEN_WGS_PER_CU"))     // (partials hold 16 per CU for it too)
        g.chosen_wgs = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(std::min<uint64_t>(e->NB, (uint64_t)e->num_cus * 16),
                                                                          (uint64_t)e->num_cus * std::atoi(x)));
    if (const char *x = ab_env("MPX_APPLY_WGS_PER_CU")) {
        const uint64_t np = (uint64_t)e->cfg.num_nodes * e->NB;
        g.apply_wgs = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(np, (uint64_t)e->num_cus * std::atoi(x)));
        if (g.apply_wgs > e->num_cus * 16) g.apply_wgs = e->num_cus * 16;   // partials are sized for 16 per CU
    }
    // the launch's sequence number tags the header scan's look-back flags; the violation
    // record alternates between two buffers (this launch's, and the next one it clears)
    if (++e->seq >= (1u << 30)) e->seq = 2;             // (wraps to an even number: the parity keeps alternating)
    e->view.seq = e->seq;
    e->view.viol = e->viol.as<DevViolation>() + (e->seq & 1);
    e->view.viol_next = e->viol.as<DevViolation>() + ((e->seq + 1) & 1);
    // this launch's summary slot: free once the all-gather that read it (two launches back) ran
    const uint32_t idx = e->sum_idx ^ 1;
    e->sum_idx = idx;
    e->view.summary = e->summary.as<unsigned long long>() + 64 * idx;
    if (e->ag_pending[idx]) HTRY(hipStreamWaitEvent(e->stream, e->ag_ev[idx], 0));
    void *evp[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    if (ev) for (int k = 0; k < 5; ++k) evp[k] = ev->e[k];
    if (ev) ev->store_last = run_ends_with_store(e->view);
    if (!e->stream2) {
        // the side stream gets a hardware queue of its own: a stream of another priority draws
        // from that priority's queue pool, so it never shares the plan path's queue — which
        // serialises the two — when the process holds more streams than GPU_MAX_HW_QUEUES
        // (MPX_SIDE_PRIO=normal|low|high, A/B).  The longer chain gets the high-priority stream:
        // multi, the promise-round walk (C3 0.886 -> 0.854 ms with s2 high / s3 low); member, the
        // plan list and the listed pairs' walk (contended C5 2.019 vs 2.106 ms the other way;
        // profiles/r05_v12_ab_stream_prio.json)
        const bool rounds_first = e->cfg.semantics == MPX_SEM_MULTI;
        int least = 0, greatest = 0;
        HTRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
        const char *sp = ab_env("MPX_SIDE_PRIO");
        const std::string pr = sp ? sp : rounds_first ? "high" : "low";
        const int prio = pr == "high" ? greatest : pr == "normal" ? 0 : least;
        HTRY(hipStreamCreateWithPriority(&e->stream2, hipStreamNonBlocking, prio));
        HTRY(hipEventCreateWithFlags(&e->fork_ev, hipEventDisableTiming));
        HTRY(hipEventCreateWithFlags(&e->join_ev, hipEventDisableTiming));
        // the third stream at the highest priority: its own hardware-queue pool again, so neither
        // side stream shares the plan path's queue (MPX_SIDE3_PRIO=normal|low|high, A/B)
        const char *sp3 = ab_env("MPX_SIDE3_PRIO");
        const std::string pr3 = sp3 ? sp3 : rounds_first ? "low" : "high";
        const int prio3 = pr3 == "high" ? greatest : pr3 == "normal" ? 0 : least;
        HTRY(hipStreamCreateWithPriority(&e->stream3, hipStreamNonBlocking, prio3));
        HTRY(hipEventCreate(&e->fork3a));           // (ride on kernel launches as their stop events)
        HTRY(hipEventCreate(&e->fork3b));
        HTRY(hipEventCreateWithFlags(&e->join3, hipEventDisableTiming));
    }
    LaunchSide side{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    if (!ab_env("MPX_ONE_STREAM")) side = LaunchSide{e->stream2, e->fork_ev, e->join_ev, nullptr, nullptr, nullptr, nullptr};
    if (!ab_env("MPX_ONE_STREAM") && !ab_env("MPX_TWO_STREAMS")) {
        side.stream3 = e->stream3; side.fork3a = e->fork3a; side.fork3b = e->fork3b; side.join3 = e->join3;
    }
    int rc = launch_run(e->view, e->stream, g, evp, side);
    if (rc) return MPX_E_HIP;
    if (e->incremental) {                              // the next window starts from this one's scalars, rounds, roles
        HTRY(hipMemcpyAsync(e->scal_base.p, e->scal_key.p, 16ull * e->cfg.num_nodes, hipMemcpyDeviceToDevice, e->stream));
        HTRY(hipMemcpyAsync(e->prop_in.p, e->prop_out.p, 24ull * e->cfg.num_nodes, hipMemcpyDeviceToDevice, e->stream));
        if (e->cfg.semantics == MPX_SEM_MEMBER)
            HTRY(hipMemcpyAsync(e->ee_init.p, e->ee_out.p, 4ull * e->cfg.num_nodes, hipMemcpyDeviceToDevice, e->stream));
    }
    // the one cross-GPU exchange: every rank's 64-word summary, over RCCL, no host
    // synchronisation — on the comm stream once the launch wrote it, so the
    // next launch's kernels run while it crosses xGMI
    if (e->comm) {
        HTRY(hipEventRecord(e->sum_ev[idx], e->stream));
        HTRY(hipStreamWaitEvent(e->comm_stream, e->sum_ev[idx], 0));
        if (ncclAllGather(e->view.summary, e->gather_buf.as<uint64_t>() + 64ull * e->nranks * idx, 64, ncclUint64,
                          e->comm, e->comm_stream) != ncclSuccess)
            return MPX_E_COMM;
        HTRY(hipEventRecord(e->ag_ev[idx], e->comm_stream));
        e->ag_pending[idx] = true;
    }
    return MPX_OK;
}

static int collect(mpx_engine *e)
{
    HTRY(hipStreamSynchronize(e->stream));
    if (e->comm_stream) HTRY(hipStreamSynchronize(e->comm_stream));   // the step includes its exchange
    e->last_summary.assign(64, 0);
    HTRY(hipMemcpy(e->last_summary.data(), e->summary.as<uint64_t>() + 64 * e->sum_idx, 64 * 8, hipMemcpyDeviceToHost));
    uint64_t cursor = 0;
    if (e->incremental) {
        // a window is not re-run (its carry has moved on): the record buffer is sized for every
        // slot of every listed event
        uint64_t nv = 0;
        HTRY(hipMemcpy(&nv, e->outv_n.p, 8, hipMemcpyDeviceToHost));
        if (nv > e->view.outv_cap) return MPX_E_STATE;
    } else {
        std::vector<uint64_t> cur(OUT_STRIDE * e->out_subs);
        HTRY(hipMemcpy(cur.data(), e->out_cursor.p, 8 * cur.size(), hipMemcpyDeviceToHost));
        for (uint32_t s = 0; s < e->out_subs; ++s) cursor = std::max<uint64_t>(cursor, cur[OUT_STRIDE * s]);
    }
    if (cursor > e->out_cap) {
        // a snapshot sub-buffer overflowed: grow and run again (runs are deterministic)
        e->out_cap = cursor + cursor / 4;
        TRY(e->out.alloc((uint64_t)e->out_subs * e->out_cap * sizeof(OutRec)));
        e->view.out = e->out.as<OutRec>();
        e->view.out_cap = e->out_cap;
        TRY(queue_run(e, e->view.digest != 0));
        return collect(e);
    }
    const auto &s = e->last_summary;
    mpx_stats &st = e->stats;
    st.chosen = s[SW_C]; st.promise_entries = s[SW_P]; st.accept_apps = s[SW_A]; st.commit_apps = s[SW_L];
    st.messages = s[SW_MSGS]; st.violations = s[SW_V] + e->iv.count;
    st.skipped = e->device_trace ? 0 : e->ht.dropped;
    st.chosen_digest = s[SW_DCHOSEN]; st.state_digest = s[SW_DSTATE]; st.scalar_digest = s[SW_DSCAL];
    st.bytes_alg = 16 * st.promise_entries + 24 * st.accept_apps + 16 * st.commit_apps;
    st.general_pairs = e->view.num_gp;
    st.num_runs = e->num_frags;
    st.slot_bytes = e->view.slot_w;
    const DevView &v = e->view;
    const bool member = e->cfg.semantics == MPX_SEM_MEMBER;
    if (!member && !v.digest && !v.walk_all && v.N <= FAST_MAX_NODES) {
        // the multi plan path launches no k_apply_fast after the store: every lean pair must
        // have been planned (kernels.hip launch_run)
        uint32_t rest = 0;
        HTRY(hipMemcpy(&rest, e->fast_rest.p, 4, hipMemcpyDeviceToHost));
        if (rest) return MPX_E_STATE;
    }
    // the plan path with k_plan_list (kernels.hip launch_run): its list + the promise-round pairs
    if (!v.digest && !v.walk_all && (member || (v.N <= FAST_MAX_NODES && v.num_gp_snap))) {
        uint64_t listed = 0;
        HTRY(hipMemcpy(&listed, e->gp_dyn_n.p, 8, hipMemcpyDeviceToHost));
        st.general_pairs = listed + (e->view.num_gp - e->view.num_gp_snap);
    }
    if (e->ev_used) {
        StepEvents &x = e->ev_pool[e->ev_used - 1];
        float a = 0, r = 0;
        (void)hipEventElapsedTime(&a, evk(x, 1), evk(x, 3));
        (void)hipEventElapsedTime(&r, evk(x, 0), evk(x, 4));
        st.apply_ns = (uint64_t)(a * 1e6);
        st.device_ns = (uint64_t)(r * 1e6);
    }
    return MPX_OK;
}

static int run_window(mpx_engine *e)
{
    // one window: the records submitted since the last run, on the carried state
    e->dirty = true;
    const uint64_t t0 = now_ns(), u0 = e->stats.ingest_ns;
    TRY(queue_run(e, false));
    const uint64_t t1 = now_ns();
    TRY(collect(e));
    const uint64_t t2 = now_ns();
    if (e->prop || e->mprop) TRY(prop_window(e));
    const uint64_t t3 = now_ns();
    // batches chosen in this window need their entries no more
    std::vector<uint32_t> bc;
    TRY(d2h(bc, e->b_chosen, e->ht.b_gid.size()));
    for (size_t j = 0; j < bc.size(); ++j)
        if (bc[j] != NONE32) e->wc.b_ents.erase(e->ht.b_gid[j]);
    ++e->windows;
    if (ab_env("MPX_HOST_TIMES"))
        std::fprintf(stderr, "[mpx] window %llu: build_trace %.1f ms, upload %.1f ms, launch %.1f ms, collect %.1f ms, "
                     "proposer %.1f ms, release %.1f ms\n", (unsigned long long)e->windows, e->ab_build_ns * 1e-6,
                     (e->stats.ingest_ns - u0 - e->ab_build_ns) * 1e-6, (t1 - t0 - (e->stats.ingest_ns - u0)) * 1e-6,
                     (t2 - t1) * 1e-6, (t3 - t2) * 1e-6, (now_ns() - t3) * 1e-6);
    return MPX_OK;
}

extern "C" int mpx_run(mpx_engine *e)
{
    if (!e) return MPX_E_INVAL;
    if (e->poisoned) return MPX_E_STATE;            // (a failed window, or a failed LEARN_EPOCHS submit)
    if (e->pf_pending) {                            // (a prefetched window runs when nothing else is queued)
        bool queued = false;
        for (auto &ns : e->nodes) queued = queued || !ns.type.empty();
        if (!queued) TRY(pf_join(e));
    }
    if (e->incremental) {
        const uint64_t before = e->consumed;
        const int rc = run_window(e);
        // a window that failed before build_trace took it leaves the engine as it was (the
        // records stay queued); one that failed after may be partly applied on the device and
        // its records are gone: every later call refuses (include/mpx.h MPX_FLAG_INCREMENTAL)
        if (rc && e->consumed != before) e->poisoned = true;
        return rc;
    }
    TRY(queue_run(e, true));
    return collect(e);
}

extern "C" int mpx_step(mpx_engine *e)
{
    if (!e) return MPX_E_INVAL;
    if (e->incremental || e->poisoned) return MPX_E_STATE;   // windows are applied once, not replayed
    return queue_run(e, false);
}

extern "C" int mpx_sync(mpx_engine *e)
{
    if (!e) return MPX_E_INVAL;
    return collect(e);
}

extern "C" int mpx_reset_state(mpx_engine *e)
{
    if (!e) return MPX_E_INVAL;
    if (e->incremental) return MPX_E_STATE;
    HTRY(hipSetDevice(e->device));
    if (e->st_valid.p) HTRY(hipMemsetAsync(e->st_valid.p, 0, e->st_valid.bytes, e->stream));
    if (e->chosen_valid.p) HTRY(hipMemsetAsync(e->chosen_valid.p, 0, e->chosen_valid.bytes, e->stream));
    if (e->node_scal.p) HTRY(hipMemsetAsync(e->node_scal.p, 0, e->node_scal.bytes, e->stream));
    HTRY(hipStreamSynchronize(e->stream));
    e->last_summary.clear();
    return MPX_OK;
}

extern "C" int mpx_timing_every(mpx_engine *e, uint32_t every)
{
    if (!e) return MPX_E_INVAL;
    e->events_every = every;
    e->step_no = 0;
    return MPX_OK;
}

extern "C" int mpx_timings(mpx_engine *e, uint32_t max, double *apply_ms, double *run_ms, uint32_t *n)
{
    if (!e || !n) return MPX_E_INVAL;
    HTRY(hipStreamSynchronize(e->stream));
    uint32_t k = 0;
    for (size_t i = 0; i < e->ev_used && k < max; ++i, ++k) {
        float a = 0, r = 0;
        (void)hipEventElapsedTime(&a, evk(e->ev_pool[i], 1), evk(e->ev_pool[i], 3));
        (void)hipEventElapsedTime(&r, evk(e->ev_pool[i], 0), evk(e->ev_pool[i], 4));
        if (apply_ms) apply_ms[k] = a;
        if (run_ms) run_ms[k] = r;
    }
    *n = k;
    e->ev_used = 0;
    return MPX_OK;
}

extern "C" int mpx_timings_detail(mpx_engine *e, uint32_t max, double *phases, uint32_t *n)
{
    if (!e || !n || (max && !phases)) return MPX_E_INVAL;
    HTRY(hipStreamSynchronize(e->stream));
    uint32_t k = 0;
    for (size_t i = 0; i < e->ev_used && k < max; ++i, ++k) {
        const StepEvents &x = e->ev_pool[i];
        float t[5] = {0, 0, 0, 0, 0};
        (void)hipEventElapsedTime(&t[0], evk(x, 0), evk(x, 4));
        for (int j = 0; j < 4; ++j)
            if (evk(x, j) != evk(x, j + 1)) (void)hipEventElapsedTime(&t[j + 1], evk(x, j), evk(x, j + 1));
        for (int j = 0; j < 5; ++j) phases[5 * k + j] = t[j];
    }
    *n = k;
    e->ev_used = 0;
    return MPX_OK;
}

// ---------------------------------------------------------------- readback --

static bool have_results(const mpx_engine *e) { return !e->last_summary.empty(); }

// count slots of node n (n == N: the chosen log) from shard offset l0, decoded
// on the device into {ballot, PRESENT | COMMITTED? | handle} pairs
static int decode_slots(mpx_engine *e, uint32_t n, uint64_t l0, uint64_t count, std::vector<uint64_t> &out)
{
    out.assign(2 * count, 0);
    if (!count || !have_results(e)) return MPX_OK;
    HTRY(hipSetDevice(e->device));
    if (e->incremental) {                              // the carried values themselves
        std::vector<uint64_t> b, w;
        if (n < e->cfg.num_nodes) {
            const uint64_t at = (uint64_t)n * e->shard_len + l0;
            TRY(d2h(b, e->s_bal, count, at)); TRY(d2h(w, e->s_val, count, at));
        } else {
            b.assign(count, 0);
            TRY(d2h(w, e->c_val, count, l0));
        }
        for (uint64_t i = 0; i < count; ++i) { out[2 * i] = (w[i] & W_PRESENT) ? b[i] : 0; out[2 * i + 1] = w[i]; }
        return MPX_OK;
    }
    TRY(e->decode_buf.alloc(16 * count));
    if (launch_decode(e->view, e->stream, n, l0, count, e->decode_buf.as<uint64_t>()) != 0) return MPX_E_HIP;
    HTRY(hipStreamSynchronize(e->stream));
    return d2h(out, e->decode_buf, 2 * count);
}

// In-order executor of node n on the device (kernels.hip k_exec_*): the
// frontier (shard-local index of the first instance not committed here, i.e.
// next_id_to_apply_ - shard_begin, multi/paxos.cpp:1584-1622) and the handles
// of the Values it executed, in instance order, noops skipped (:1601-1606).
// Membership Values are skipped too (member/paxos.cpp:1042-1053: only client
// Values reach Apply); that filter needs the host value table.
static int gpu_executed(mpx_engine *e, uint32_t n, uint64_t &frontier, std::vector<uint64_t> &handles)
{
    frontier = 0;
    handles.clear();
    if (!have_results(e)) return MPX_OK;
    HTRY(hipSetDevice(e->device));
    if (e->incremental) {                              // readback of the carried values (a window keeps no slot rows)
        std::vector<uint64_t> st;
        TRY(decode_slots(e, n, 0, e->shard_len, st));
        while (frontier < e->shard_len && (st[2 * frontier + 1] & W_COMMITTED)) {
            const uint64_t h = st[2 * frontier + 1] & W_HANDLE;
            if (!MPX_HANDLE_NOOP(h)) handles.push_back(h);
            ++frontier;
        }
    } else {
    const uint64_t NB = e->NB;
    TRY(e->exec_aux.alloc(8 * (2 * NB + 2)));
    unsigned long long *aux = e->exec_aux.as<unsigned long long>();
    if (launch_exec(e->view, e->stream, n, aux, nullptr) != 0) return MPX_E_HIP;
    unsigned long long total = 0, fr = 0;
    HTRY(hipMemcpyAsync(&fr, aux, 8, hipMemcpyDeviceToHost, e->stream));
    HTRY(hipMemcpyAsync(&total, aux + 1 + 2 * NB, 8, hipMemcpyDeviceToHost, e->stream));
    HTRY(hipStreamSynchronize(e->stream));
    frontier = fr;
    if (total) {
        TRY(e->exec_out.alloc(8 * total));
        if (launch_exec(e->view, e->stream, n, aux, e->exec_out.as<uint64_t>()) != 0) return MPX_E_HIP;
        HTRY(hipStreamSynchronize(e->stream));
        TRY(d2h(handles, e->exec_out, total));
    }
    }
    {   // Values with no executable payload (membership changes) are not executed
        std::string payload;
        size_t k = 0;
        for (uint64_t h : handles)
            if (e->vt.exec_payload(h, payload)) handles[k++] = h;
        handles.resize(k);
    }
    return MPX_OK;
}

extern "C" int mpx_read_executed(mpx_engine *e, uint32_t node, uint64_t *frontier, uint64_t *count,
                                 uint64_t *handles, uint64_t cap)
{
    if (!e || node >= e->cfg.num_nodes || (cap && !handles)) return MPX_E_INVAL;
    TRY(pf_join(e));                                // (the value table: no decode in flight)
    if (e->poisoned) return MPX_E_STATE;            // (MPX_FLAG_INCREMENTAL: a failed window)
    uint64_t fr;
    std::vector<uint64_t> h;
    TRY(gpu_executed(e, node, fr, h));
    if (frontier) *frontier = e->cfg.shard_begin + fr;
    if (count) *count = h.size();
    for (uint64_t i = 0; i < h.size() && i < cap; ++i) handles[i] = h[i];
    return MPX_OK;
}

extern "C" int mpx_read_chosen(mpx_engine *e, uint64_t first, uint64_t count, uint64_t *out)
{
    if (!e || (count && !out)) return MPX_E_INVAL;
    if (e->poisoned) return MPX_E_STATE;            // (MPX_FLAG_INCREMENTAL: a failed window)
    if (first < e->cfg.shard_begin || first + count > e->cfg.shard_end) return MPX_E_RANGE;
    if (!count) return MPX_OK;
    std::vector<uint64_t> d;
    TRY(decode_slots(e, e->cfg.num_nodes, first - e->cfg.shard_begin, count, d));
    for (uint64_t i = 0; i < count; ++i) out[i] = d[2 * i + 1];
    return MPX_OK;
}

extern "C" int mpx_read_node_scalars(mpx_engine *e, uint32_t node, uint64_t *promised, uint64_t *max_seen)
{
    if (!e || node >= e->cfg.num_nodes) return MPX_E_INVAL;
    if (e->poisoned) return MPX_E_STATE;            // (MPX_FLAG_INCREMENTAL: a failed window)
    uint64_t v[2] = {0, 0};
    if (have_results(e)) {
        HTRY(hipSetDevice(e->device));
        HTRY(hipMemcpy(v, (const char *)e->node_scal.p + 16ull * node, 16, hipMemcpyDeviceToHost));
    }
    if (promised) *promised = v[0];
    if (max_seen) *max_seen = v[1];
    return MPX_OK;
}

extern "C" int mpx_read_node_state(mpx_engine *e, uint32_t node, uint64_t first, uint64_t count,
                                   uint64_t *acc_ballot, uint64_t *acc_value, uint64_t *com_ballot, uint64_t *com_value)
{
    if (!e || node >= e->cfg.num_nodes) return MPX_E_INVAL;
    if (e->poisoned) return MPX_E_STATE;            // (MPX_FLAG_INCREMENTAL: a failed window)
    if (first < e->cfg.shard_begin || first + count > e->cfg.shard_end) return MPX_E_RANGE;
    if (!count) return MPX_OK;
    std::vector<uint64_t> st;
    TRY(decode_slots(e, node, first - e->cfg.shard_begin, count, st));
    for (uint64_t i = 0; i < count; ++i) {
        const uint64_t b = st[2 * i], w = st[2 * i + 1];
        const bool com = (w & W_PRESENT) && (w & W_COMMITTED);
        const bool acc = (w & W_PRESENT) && !(w & W_COMMITTED);
        if (acc_ballot) acc_ballot[i] = acc ? b : 0;
        if (acc_value) acc_value[i] = acc ? (MPX_PRESENT | (w & W_HANDLE)) : 0;
        if (com_ballot) com_ballot[i] = com ? b : 0;
        if (com_value) com_value[i] = com ? (MPX_PRESENT | (w & W_HANDLE)) : 0;
    }
    return MPX_OK;
}

extern "C" int mpx_stats_get(mpx_engine *e, mpx_stats *out)
{
    if (!e || !out) return MPX_E_INVAL;
    *out = e->stats;
    return MPX_OK;
}

extern "C" int mpx_state_digest(mpx_engine *e, uint64_t *state_digest, uint64_t *chosen_digest)
{
    if (!e || !state_digest || !chosen_digest) return MPX_E_INVAL;
    if (e->poisoned) return MPX_E_STATE;            // (MPX_FLAG_INCREMENTAL: a failed window)
    if (!e->st.p) return MPX_E_STATE;
    HTRY(hipSetDevice(e->device));
    TRY(e->exec_aux.alloc(std::max<size_t>(e->exec_aux.bytes, 16)));
    unsigned long long *aux = e->exec_aux.as<unsigned long long>();
    if (launch_state_digest(e->view, e->stream, aux) != 0) return MPX_E_HIP;
    unsigned long long d[2] = {0, 0};
    HTRY(hipMemcpyAsync(d, aux, 16, hipMemcpyDeviceToHost, e->stream));
    HTRY(hipStreamSynchronize(e->stream));
    *state_digest = d[0];
    *chosen_digest = d[1];
    return MPX_OK;
}

extern "C" int mpx_last_violation(mpx_engine *e, mpx_violation *out)
{
    if (!e || !out) return MPX_E_INVAL;
    std::memset(out, 0, sizeof *out);
    if (e->iv.code) {
        out->code = e->iv.code; out->node = (uint32_t)e->iv.node; out->seq = e->iv.seq; out->iid = e->iv.iid;
        return MPX_OK;
    }
    if (e->viol.p && have_results(e)) {
        DevViolation d;
        HTRY(hipMemcpy(&d, e->view.viol, sizeof d, hipMemcpyDeviceToHost));
        out->code = d.code; out->node = (uint32_t)d.node; out->seq = d.seq; out->iid = d.iid;
        // kernels report a message's position among the kept records of its node
        const HostTrace &h = e->ht;
        const bool msg_seq = d.code == MPX_V_BAD_NODE || d.code == MPX_V_LEARN_VALUE ||
                             (d.code == MPX_V_COMMIT_VALUE && d.seq);
        if (msg_seq && d.node < h.N && h.node_off[d.node] + d.seq < h.m_seq.size())
            out->seq = h.m_seq[h.node_off[d.node] + d.seq] + (e->incremental ? e->win_seq_base[d.node] : 0);
    }
    return MPX_OK;
}

extern "C" int mpx_value_bytes(mpx_engine *e, uint64_t handle, uint8_t *buf, uint32_t cap, uint32_t *len)
{
    if (!e || !len) return MPX_E_INVAL;
    TRY(pf_join(e));                                // (the value table: no decode in flight)
    std::string s;
    if (!e->vt.encode(handle & ~MPX_PRESENT, s)) return MPX_E_RANGE;
    *len = (uint32_t)s.size();
    if (buf && cap) std::memcpy(buf, s.data(), std::min<size_t>(cap, s.size()));
    return MPX_OK;
}

extern "C" void mpx_free(void *p) { std::free(p); }

// ------------------------------------------------- sends / canonical dump --
template <typename T> static inline void app(std::string &s, T v) { s.append((const char *)&v, sizeof v); }

static int ensure_host_headers(mpx_engine *e);

struct Results {
    std::vector<uint8_t> flags;
    std::vector<uint64_t> maxseen, scal;
    std::vector<OutEnt> out;
    std::vector<uint32_t> b_chosen;
    std::map<uint32_t, std::vector<const OutEnt *>> by_msg[2];
};

static int fetch_results(mpx_engine *e, Results &r)
{
    if (!have_results(e)) return MPX_E_STATE;
    HTRY(hipSetDevice(e->device));
    TRY(ensure_host_headers(e));
    const size_t G = e->ht.m_type.size();
    TRY(d2h(r.flags, e->m_flags, G));
    TRY(d2h(r.maxseen, e->m_maxseen, G));
    TRY(d2h(r.scal, e->node_scal, 2ull * e->cfg.num_nodes));
    if (e->incremental) {                              // window records carry their values
        uint64_t nv = 0;
        HTRY(hipMemcpy(&nv, e->outv_n.p, 8, hipMemcpyDeviceToHost));
        TRY(d2h(r.out, e->outv, std::min<uint64_t>(nv, e->view.outv_cap)));
    } else {
        std::vector<uint64_t> cur(OUT_STRIDE * e->out_subs);
        HTRY(hipMemcpy(cur.data(), e->out_cursor.p, 8 * cur.size(), hipMemcpyDeviceToHost));
        std::vector<OutRec> part;
        const HostTrace &h = e->ht;
        const bool member = e->cfg.semantics == MPX_SEM_MEMBER;
        for (uint32_t s = 0; s < e->out_subs; ++s) {
            const uint64_t k = std::min<uint64_t>(cur[OUT_STRIDE * s], e->out_cap);
            if (!k) continue;
            TRY(d2h(part, e->out, k, (size_t)s * e->out_cap));
            for (const OutRec &o : part) {
                // resolve the reference (mpx_internal.hpp OutRec) against the host trace
                OutEnt x{o.msg, ((o.aux & OUT_K1) ? 1u : 0u) | ((o.aux & OUT_CMT) ? 2u : 0u), 0, 0, 0};
                if (x.kind & 1) {
                    // one slot, or (OUT_RUN, a quorum's merged map) a run of slots whose entries follow
                    // one another in one reply run
                    const uint32_t ns = (o.aux & OUT_RUN) ? (o.aux >> OUT_RUN_SHIFT) & 0x1FF : 1;
                    if ((uint64_t)o.ref + ns > h.r_iid.size()) return MPX_E_STATE;
                    for (uint32_t i = 0; i < ns; ++i) {
                        x.iid = h.r_iid[o.ref + i]; x.ballot = h.r_pid[o.ref + i]; x.handle = h.r_val[o.ref + i];
                        r.out.push_back(x);
                    }
                } else {
                    if (o.ref >= h.frags.size()) return MPX_E_STATE;
                    const Frag &f = h.frags[o.ref];
                    // one slot, or (OUT_RUN, k_plan_list) a run of slots of a dense fragment
                    const uint32_t s0 = o.aux & (BS - 1);
                    const uint32_t ns = (o.aux & OUT_RUN) ? (o.aux >> OUT_RUN_SHIFT) & 0x1FF : 1;
                    if ((o.aux & OUT_RUN) && (!(f.flags & FR_DENSE) || s0 < f.start || s0 + ns > f.start + f.count))
                        return MPX_E_STATE;
                    for (uint32_t sl = s0; sl < s0 + ns; ++sl) {
                        uint64_t ent = f.entry + (sl - f.start);
                        if (!(f.flags & FR_DENSE))
                            for (uint32_t q = 0; q < f.count; ++q)
                                if (((h.e_iid[f.entry + q] - e->cfg.shard_begin) & (BS - 1)) == sl) { ent = f.entry + q; break; }
                        x.iid = h.e_iid[ent]; x.handle = h.e_val[ent];
                        x.ballot = member ? h.e_pid[ent] : h.m_ballot[f.msg];
                        r.out.push_back(x);
                    }
                }
            }
        }
    }
    TRY(d2h(r.b_chosen, e->b_chosen, e->ht.b_msg.size()));
    for (auto &o : r.out) r.by_msg[o.kind & 1][o.msg].push_back(&o);
    for (int k = 0; k < 2; ++k)
        for (auto &x : r.by_msg[k])
            std::sort(x.second.begin(), x.second.end(), [](const OutEnt *a, const OutEnt *b) { return a->iid < b->iid; });
    return MPX_OK;
}

// record index of message g in node n's submitted stream (ingest leaves other
// shards' records out, HostTrace::m_seq; device-generated traces keep all)
static uint64_t seq_of(const HostTrace &h, uint32_t n, uint64_t g)
{
    return h.m_seq.size() > g ? h.m_seq[g] : g - h.node_off[n];
}

// the replies the reference's acceptor / learner handlers send for message g
// of node n, in generation order (paxos.cpp:888-899,1391-1403,1577-1582)
static void reply_of(const mpx_engine *e, const Results &r, uint32_t n, uint64_t g, uint32_t &dst, std::string &m)
{
    const HostTrace &h = e->ht;
    const uint8_t t = h.m_type[g], f = r.flags[g];
    m.clear();
    dst = h.m_src[g];
    if (t == MPX_MSG_PREPARE) {
        if (f & F_GRANTED) {
            std::string body;
            auto it = r.by_msg[0].find((uint32_t)g);
            if (it != r.by_msg[0].end())
                for (const OutEnt *o : it->second) {
                    app<uint64_t>(body, o->iid);
                    app<uint64_t>(body, o->ballot);
                    e->vt.encode(o->handle, body);
                }
            app<uint32_t>(m, MPX_MSG_PREPARE_REPLY); app<uint32_t>(m, n); app<uint64_t>(m, h.m_ballot[g]);
            app<uint32_t>(m, (uint32_t)body.size());
            m += body;
        } else if (f & F_REJECT) {
            app<uint32_t>(m, MPX_MSG_REJECT); app<uint64_t>(m, r.maxseen[g]);
        }
    } else if (t == MPX_MSG_ACCEPT) {
        if (f & F_GRANTED) {
            app<uint32_t>(m, MPX_MSG_ACCEPT_REPLY); app<uint32_t>(m, n);
            if (e->cfg.semantics == MPX_SEM_MULTI) app<uint64_t>(m, h.m_ballot[g]);   // member: no ballot, :900-908
            app<uint64_t>(m, h.m_aux[g]);
        } else if (f & F_REJECT) {
            app<uint32_t>(m, MPX_MSG_REJECT); app<uint64_t>(m, r.maxseen[g]);
        }
    } else if (t == MPX_MSG_COMMIT) {
        app<uint32_t>(m, MPX_MSG_COMMIT_REPLY); app<uint32_t>(m, n); app<uint64_t>(m, h.m_aux[g]);
    }
}

extern "C" int mpx_drain_sends(mpx_engine *e, mpx_send_fn fn, void *user)
{
    if (!e || !fn) return MPX_E_INVAL;
    TRY(pf_join(e));                                // (the value table: no decode in flight)
    if (e->poisoned) return MPX_E_STATE;            // (MPX_FLAG_INCREMENTAL: a failed window)
    Results r;
    TRY(fetch_results(e, r));
    std::string m;
    for (uint32_t n = 0; n < e->cfg.num_nodes; ++n)
        for (uint64_t g = e->ht.node_off[n]; g < e->ht.node_off[n + 1]; ++g) {
            uint32_t dst;
            reply_of(e, r, n, g, dst, m);
            if (!m.empty()) fn(user, n, dst, (const uint8_t *)m.data(), (uint32_t)m.size());
        }
    return MPX_OK;
}

extern "C" int mpx_dump_result(mpx_engine *e, uint8_t **out, uint64_t *size)
{
    if (!e || !out || !size) return MPX_E_INVAL;
    TRY(pf_join(e));                                // (the value table: no decode in flight)
    if (e->incremental) return MPX_E_STATE;             // windows keep no history of runs
    Results r;
    TRY(fetch_results(e, r));
    const uint32_t N = e->cfg.num_nodes;
    const HostTrace &h = e->ht;
    std::string d;
    d.append("MPXR", 4);
    app<uint32_t>(d, 1); app<uint32_t>(d, N); app<uint32_t>(d, e->cfg.semantics);
    std::vector<uint64_t> st;
    std::string m;
    for (uint32_t n = 0; n < N; ++n) {
        app<uint64_t>(d, r.scal[2 * n]);
        app<uint64_t>(d, r.scal[2 * n + 1]);
        TRY(decode_slots(e, n, 0, e->shard_len, st));
        std::string sec;
        uint64_t cnt = 0;
        for (uint64_t li = 0; li < e->shard_len; ++li) {
            const uint64_t b = st[2 * li], w = st[2 * li + 1];
            if (!(w & W_PRESENT)) continue;
            const uint64_t kind = (w & W_COMMITTED) ? 2 : 1;
            app<uint64_t>(sec, e->cfg.shard_begin + li); app<uint64_t>(sec, kind);
            app<uint64_t>(sec, b); app<uint64_t>(sec, w & W_HANDLE);
            ++cnt;
        }
        app<uint64_t>(d, cnt);
        d += sec;
        // sends
        sec.clear(); cnt = 0;
        for (uint64_t g = h.node_off[n]; g < h.node_off[n + 1]; ++g) {
            uint32_t dst;
            reply_of(e, r, n, g, dst, m);
            if (m.empty()) continue;
            app<uint32_t>(sec, dst); app<uint32_t>(sec, (uint32_t)m.size()); sec += m;
            ++cnt;
        }
        app<uint64_t>(d, cnt);
        d += sec;
        // promise quorum events
        sec.clear(); cnt = 0;
        for (uint64_t g = h.node_off[n]; g < h.node_off[n + 1]; ++g) {
            if (h.m_type[g] != MPX_MSG_PREPARE_REPLY || !(r.flags[g] & F_QUORUM)) continue;
            app<uint64_t>(sec, seq_of(h, n, g));
            app<uint64_t>(sec, h.m_ballot[g]);
            auto it = r.by_msg[1].find((uint32_t)g);
            const uint64_t k = it == r.by_msg[1].end() ? 0 : it->second.size();
            app<uint64_t>(sec, k);
            if (k)
                for (const OutEnt *o : it->second) { app<uint64_t>(sec, o->iid); app<uint64_t>(sec, o->ballot); app<uint64_t>(sec, o->handle); }
            ++cnt;
        }
        app<uint64_t>(d, cnt);
        d += sec;
        // chosen batch events, in the order of the replies that chose them
        std::vector<std::pair<uint32_t, uint64_t>> ch;
        for (size_t j = 0; j < h.b_msg.size(); ++j)
            if (h.m_node[h.b_msg[j]] == n && r.b_chosen[j] != NONE32) ch.push_back({r.b_chosen[j], h.m_aux[h.b_msg[j]]});
        std::sort(ch.begin(), ch.end());
        app<uint64_t>(d, ch.size());
        for (auto &c : ch) { app<uint64_t>(d, seq_of(h, n, c.first)); app<uint64_t>(d, c.second); }
        // executor: committed prefix from the shard's first instance (paxos.cpp:1584-1620),
        // computed on the device (gpu_executed); the host only looks up payload bytes
        sec.clear(); cnt = 0;
        std::string payload;
        uint64_t frontier;
        std::vector<uint64_t> executed;
        TRY(gpu_executed(e, n, frontier, executed));
        for (uint64_t hd : executed) {
            if (!e->vt.exec_payload(hd, payload)) return MPX_E_VALUE;   // filtered in gpu_executed
            app<uint32_t>(sec, (uint32_t)payload.size());
            sec += payload;
            ++cnt;
        }
        app<uint64_t>(d, cnt);
        d += sec;
    }
    uint64_t cnt = 0;
    std::string sec;
    TRY(decode_slots(e, N, 0, e->shard_len, st));
    for (uint64_t li = 0; li < e->shard_len; ++li) {
        if (!(st[2 * li + 1] & W_PRESENT)) continue;
        app<uint64_t>(sec, e->cfg.shard_begin + li);
        app<uint64_t>(sec, st[2 * li + 1] & W_HANDLE);
        ++cnt;
    }
    app<uint64_t>(d, cnt);
    d += sec;
    *out = (uint8_t *)std::malloc(d.size());
    if (!*out) return MPX_E_NOMEM;
    std::memcpy(*out, d.data(), d.size());
    *size = d.size();
    return MPX_OK;
}

// Per promise-quorum event of the run (node-major stream order, the same on every
// shard: the promise headers are replicated): the adopted entries in the shard and
// the shard's noop-fill instances.  gx == nullptr: the fill ends at the shard's own
// bound (a whole engine); else at gx[k] (absolute), the maximum of every shard's bound.
// Per promise-quorum event (node en[k], message eg[k]): 1 + the highest shard-local
// instance the node had committed before the event (0: none).  The first COMMIT over an
// instance fixes it (multi/paxos.cpp:1501-1515), so "committed before g" is "some COMMIT of
// the node before g covers it": a node's COMMIT messages in order with a running max of
// their last in-shard entry (entries are iid-sorted) answer every event with one binary
// search — O(commits + events log commits) instead of k_decide pass 0's scan of every slot
// per event, O(events x instances).  A device-generated trace keeps its entry pool on the
// device only: there (and with MPX_DECIDE_DEVICE=1, for A/B) pass 0 runs.
static int committed_before(mpx_engine *e, const std::vector<uint32_t> &en, const std::vector<uint32_t> &eg,
                            std::vector<uint64_t> &xmax)
{
    const size_t E = en.size();
    xmax.assign(E, 0);
    if (!E) return MPX_OK;
    const char *dv = std::getenv("MPX_DECIDE_DEVICE");
    if (e->device_trace || (dv && std::atoi(dv))) {
        hipStream_t s = e->stream;
        DevBuf d_node, d_msg, d_xmax;
        TRY(upload(d_node, en, s)); TRY(upload(d_msg, eg, s));
        TRY(d_xmax.alloc(8 * E)); HTRY(hipMemsetAsync(d_xmax.p, 0, 8 * E, s));
        DecideArgs a{};
        a.E = (uint32_t)E; a.ev_node = d_node.as<uint32_t>(); a.ev_msg = d_msg.as<uint32_t>();
        a.xmax = d_xmax.as<unsigned long long>();
        if (launch_decide(e->view, s, 0, a) != 0) return MPX_E_HIP;
        HTRY(hipStreamSynchronize(s));
        return d2h(xmax, d_xmax, E);
    }
    const HostTrace &h = e->ht;
    const uint64_t sb = e->cfg.shard_begin;
    std::vector<std::vector<std::pair<uint32_t, uint64_t>>> pm(e->cfg.num_nodes);   // (commit message, running max)
    for (uint32_t n = 0; n < e->cfg.num_nodes; ++n) {
        uint64_t run = 0;
        for (uint64_t g = h.node_off[n]; g < h.node_off[n + 1]; ++g)
            if (h.m_type[g] == MPX_MSG_COMMIT && h.m_cnt[g]) {
                run = std::max<uint64_t>(run, h.e_iid[h.m_ent[g] + h.m_cnt[g] - 1] - sb + 1);
                pm[n].push_back({(uint32_t)g, run});
            }
    }
    for (size_t k = 0; k < E; ++k) {
        const auto &l = pm[en[k]];
        auto it = std::lower_bound(l.begin(), l.end(), std::make_pair(eg[k], (uint64_t)0));   // first commit at or after g
        if (it != l.begin()) xmax[k] = std::prev(it)->second;
    }
    return MPX_OK;
}

struct DecideEv { uint32_t node, msg; uint64_t bound; std::vector<const OutEnt *> adopted; std::vector<uint64_t> noops; };
static int decide_core(mpx_engine *e, const Results &r, const uint64_t *gx, uint64_t ngx, bool bounds_only,
                       std::vector<DecideEv> &evs)
{
    const HostTrace &h = e->ht;
    const uint32_t N = e->cfg.num_nodes;
    evs.clear();
    for (uint32_t n = 0; n < N; ++n)
        for (uint64_t g = h.node_off[n]; g < h.node_off[n + 1]; ++g)
            if (h.m_type[g] == MPX_MSG_PREPARE_REPLY && (r.flags[g] & F_QUORUM)) evs.push_back(DecideEv{n, (uint32_t)g, 0, {}, {}});
    const uint32_t E = (uint32_t)evs.size();
    if (gx && ngx != E) return MPX_E_INVAL;
    const uint64_t sb = e->cfg.shard_begin;
    // adopted: the merged entries of instances not committed at the quorum (:1091)
    std::vector<uint64_t> ad_off(E + 1, 0), xend(E, 0);
    std::vector<uint32_t> ad_li, en(E), eg(E);
    for (uint32_t k = 0; k < E; ++k) {
        en[k] = evs[k].node; eg[k] = evs[k].msg;
        auto it = r.by_msg[1].find(eg[k]);
        if (it != r.by_msg[1].end())
            for (const OutEnt *o : it->second)
                if (!(o->kind & 2)) { evs[k].adopted.push_back(o); ad_li.push_back((uint32_t)(o->iid - sb)); }
        ad_off[k + 1] = ad_li.size();
        if (!evs[k].adopted.empty()) xend[k] = evs[k].adopted.back()->iid - sb + 1;
    }
    if (!E) return MPX_OK;
    hipStream_t s = e->stream;
    DevBuf d_node, d_msg, d_xend, d_adoff, d_adli, d_boff, d_bcnt, d_base, d_tot, d_noop;
    TRY(upload(d_node, en, s)); TRY(upload(d_msg, eg, s));
    DecideArgs a{};
    a.E = E; a.ev_node = d_node.as<uint32_t>(); a.ev_msg = d_msg.as<uint32_t>();
    std::vector<uint64_t> xmax;
    TRY(committed_before(e, en, eg, xmax));
    std::vector<uint64_t> boff(E + 1, 0);
    uint64_t maxb = 0;
    for (uint32_t k = 0; k < E; ++k) {
        const uint64_t own = std::max(xend[k], xmax[k]);            // 1 + the highest committed or adopted (local)
        evs[k].bound = own ? sb + own : 0;
        uint64_t end = own;
        if (gx) end = gx[k] > sb ? gx[k] - sb : 0;                   // the fill reaches the global bound
        xend[k] = std::min<uint64_t>(end, e->shard_len);
        const uint64_t nb = (xend[k] + 255) / 256;
        boff[k + 1] = boff[k] + nb;
        maxb = std::max(maxb, nb);
    }
    if (bounds_only) return MPX_OK;
    TRY(upload(d_xend, xend, s)); TRY(upload(d_adoff, ad_off, s)); TRY(upload(d_adli, ad_li, s));
    TRY(upload(d_boff, boff, s));
    TRY(d_bcnt.alloc(std::max<uint64_t>(4 * boff[E], 4))); TRY(d_tot.alloc(8ull * E));
    a.xend = d_xend.as<uint64_t>(); a.ad_off = d_adoff.as<uint64_t>(); a.ad_li = d_adli.as<uint32_t>();
    a.blk_off = d_boff.as<uint64_t>(); a.blk_cnt = d_bcnt.as<uint32_t>(); a.ev_total = d_tot.as<uint64_t>();
    a.max_blocks = maxb;
    if (launch_decide(e->view, s, 1, a) != 0 || launch_decide(e->view, s, 3, a) != 0) return MPX_E_HIP;
    std::vector<uint64_t> tot, ev_base(E + 1, 0);
    HTRY(hipStreamSynchronize(s));
    TRY(d2h(tot, d_tot, E));
    for (uint32_t k = 0; k < E; ++k) ev_base[k + 1] = ev_base[k] + tot[k];
    TRY(upload(d_base, ev_base, s));
    TRY(d_noop.alloc(std::max<uint64_t>(4 * ev_base[E], 4)));
    a.ev_base = d_base.as<uint64_t>(); a.noop_li = d_noop.as<uint32_t>();
    if (launch_decide(e->view, s, 2, a) != 0) return MPX_E_HIP;
    std::vector<uint32_t> noops;
    HTRY(hipStreamSynchronize(s));
    TRY(d2h(noops, d_noop, ev_base[E]));
    for (uint32_t k = 0; k < E; ++k)
        for (uint64_t j = ev_base[k]; j < ev_base[k + 1]; ++j) evs[k].noops.push_back(sb + noops[j]);
    return MPX_OK;
}

// one event's batch: adopted and noop entries merged by instance (both sorted);
// noop handles Value(node, ++value_id_) from vid, or NOOP_SLOT placeholders (parts)
static constexpr uint64_t NOOP_SLOT = ~0ull;
static void decide_entries(const DecideEv &ev, uint64_t *vid, std::string &d)
{
    app<uint64_t>(d, ev.adopted.size() + ev.noops.size());
    size_t i = 0, j = 0;
    while (i < ev.adopted.size() || j < ev.noops.size()) {
        const uint64_t ai = i < ev.adopted.size() ? ev.adopted[i]->iid : ~0ull;
        const uint64_t ni = j < ev.noops.size() ? ev.noops[j] : ~0ull;
        if (ai < ni) { app<uint64_t>(d, ai); app<uint64_t>(d, ev.adopted[i]->handle); ++i; }
        else { app<uint64_t>(d, ni); app<uint64_t>(d, vid ? MPX_HANDLE(ev.node, 1, ++*vid) : NOOP_SLOT); ++j; }
    }
}

// ---------------------------------------- the proposer's own values (f2) --
// With client proposals (P_PROPOSE records) the phase-2 batch also carries the node's own
// values, and value ids are shared between them and the noop fill, so the decision is the
// proposer's sequential bookkeeping over its stream — host work (control plane, SURVEY §2
// row 13), fed by what the device computed: the promise quorums (F_QUORUM) and each
// quorum's merged pre-accepted map (k_apply's records).  The instance-id sets restate
// AvailableInstanceIDs (multi/paxos.cpp:253-318).
struct IdSet {
    std::map<uint64_t, uint64_t> r;                        // start -> end, disjoint, [0, 2^64-1) at first
    IdSet() { r[0] = ~0ull; }
    bool contains(uint64_t id) const
    {
        auto it = r.upper_bound(id);
        if (it == r.begin()) return false;
        --it;
        return it->first <= id && id < it->second;
    }
    void remove(uint64_t id)                               // (callers check contains first)
    {
        auto it = std::prev(r.upper_bound(id));
        const uint64_t a = it->first, b = it->second;
        r.erase(it);
        if (a != id) r[a] = id;
        if (id + 1 != b) r[id + 1] = b;
    }
    uint64_t next()
    {
        const uint64_t a = r.begin()->first;
        remove(a);
        return a;
    }
};

// Per node in stream order (multi/paxos.cpp): Propose (:1250-1280: ++value_id_; not preparing
// -> the next unproposed instance at once, else queued), StartPrepare (P_START), OnCommit
// (:1494-1570: uncommitted / unproposed ids, an own initial proposal that lost its instance is
// proposed again — at once, or queued while preparing), and at each promise quorum
// OnPrepareReply's batch (:1056-1175): the merged values of unproposed instances, noops over
// every unproposed range but the last (++value_id_ each), the own initial proposals still
// unproposed, then the queued values at the next unproposed ids.  MPXD as mpx_read_decisions.
// The events the bookkeeping reads, per node in stream order: Propose, StartPrepare, a COMMIT
// with its entries, a promise quorum with its merged map's entries.  One engine holding every
// instance has them all; instance shards each hold their own instances' entries of the same
// events (headers are replicated), merged in shard order (mpx_proposal_combine).
struct PEv {
    uint64_t seq;
    uint32_t type;
    std::vector<std::pair<uint64_t, uint64_t>> ents;      // {iid, handle}, iid ascending
    uint64_t aux = 0;                                     // member E_EPOCH: the epoch index
};
typedef std::vector<std::vector<PEv>> PEvents;

// a node's P_PROPOSE records (HostTrace::prop_seq, kept off the device) merged into its
// events by record index
static void merge_proposals(const mpx_engine *e, uint32_t n, std::vector<PEv> &evs)
{
    const HostTrace &h = e->ht;
    if (h.prop_off.size() <= n + 1 || h.prop_off[n + 1] == h.prop_off[n]) return;
    const uint64_t base = e->incremental ? e->win_seq_base[n] : 0;
    std::vector<PEv> out;
    out.reserve(evs.size() + (h.prop_off[n + 1] - h.prop_off[n]));
    size_t i = 0;
    for (uint64_t k = h.prop_off[n]; k < h.prop_off[n + 1]; ++k) {
        const uint64_t sq = h.prop_seq[k] + base;
        while (i < evs.size() && evs[i].seq < sq) out.push_back(std::move(evs[i++]));
        out.push_back(PEv{sq, MPX_MSG_P_PROPOSE, {}});
    }
    while (i < evs.size()) out.push_back(std::move(evs[i++]));
    evs.swap(out);
}

static void proposer_events(mpx_engine *e, const Results &r, PEvents &ev)
{
    const HostTrace &h = e->ht;
    const uint32_t N = e->cfg.num_nodes;
    ev.assign(N, {});
    for (uint32_t n = 0; n < N; ++n)
        for (uint64_t g = h.node_off[n]; g < h.node_off[n + 1]; ++g) {
            const uint8_t t = h.m_type[g];
            const bool quorum = t == MPX_MSG_PREPARE_REPLY && (r.flags[g] & F_QUORUM);
            if (t != MPX_MSG_P_START && t != MPX_MSG_COMMIT && !quorum) continue;
            PEv x{seq_of(h, n, g) + (e->incremental ? e->win_seq_base[n] : 0), t, {}};
            if (t == MPX_MSG_COMMIT)
                for (uint64_t k = h.m_ent[g]; k < h.m_ent[g] + h.m_cnt[g]; ++k) x.ents.push_back({h.e_iid[k], h.e_val[k]});
            if (quorum) {
                auto it = r.by_msg[1].find((uint32_t)g);
                if (it != r.by_msg[1].end())
                    for (const OutEnt *o : it->second) x.ents.push_back({o->iid, o->handle});
                std::sort(x.ents.begin(), x.ents.end());
            }
            ev[n].push_back(std::move(x));
        }
    for (uint32_t n = 0; n < N; ++n) merge_proposals(e, n, ev[n]);
}

// The proposer's bookkeeping of one node, advanced over its events in stream order (a whole
// run at once, or window by window: MPX_FLAG_DECISIONS); each promise quorum appends its
// MPXD record to `body`
struct PropNode {
    IdSet uncommitted, unproposed;
    std::map<uint64_t, uint64_t> initial;              // initial_proposals_: instance -> value id
    std::set<uint64_t> newly, committed;               // newly_proposed_values_; committed instances
    uint64_t vid = 0;                                   // value_id_ (:335)
    bool preparing = false;                             // prepare_retry_timeout_ != NULL
    std::string body;
    uint64_t count = 0;
};

static void prop_advance(PropNode &st, uint32_t n, const std::vector<PEv> &evs)
{
    IdSet &uncommitted = st.uncommitted, &unproposed = st.unproposed;
    auto &initial = st.initial;
    auto &newly = st.newly, &committed = st.committed;
    uint64_t &vid = st.vid;
    bool &preparing = st.preparing;
    for (const PEv &x : evs) {
        const uint32_t t = x.type;
        if (t == MPX_MSG_P_PROPOSE) {
            ++vid;
            if (!preparing) initial[unproposed.next()] = vid;
            else newly.insert(vid);
        } else if (t == MPX_MSG_P_START) {
            preparing = true;
        } else if (t == MPX_MSG_COMMIT) {
            for (auto &en : x.ents) {
                const uint64_t iid = en.first, hv = en.second;
                if (committed.insert(iid).second && uncommitted.contains(iid)) uncommitted.remove(iid);
                if (unproposed.contains(iid)) unproposed.remove(iid);
                auto it = initial.find(iid);
                if (it != initial.end()) {
                    const uint64_t v0 = it->second;
                    initial.erase(it);
                    if (MPX_HANDLE_PROPOSER(hv) != n || MPX_HANDLE_VALUE_ID(hv) != v0) {
                        if (!preparing) initial[unproposed.next()] = v0;
                        else newly.insert(v0);
                    }
                }
            }
        } else {                                        // a promise quorum
            unproposed = uncommitted;
            std::vector<std::pair<uint64_t, uint64_t>> b;
            for (auto &en : x.ents)
                if (unproposed.contains(en.first)) { unproposed.remove(en.first); b.push_back(en); }
            while (unproposed.r.size() > 1) {
                const auto first = *unproposed.r.begin();
                unproposed.r.erase(unproposed.r.begin());
                for (uint64_t id = first.first; id != first.second; ++id) b.push_back({id, MPX_HANDLE(n, 1, ++vid)});
            }
            for (auto &y : initial)
                if (unproposed.contains(y.first)) { unproposed.remove(y.first); b.push_back({y.first, MPX_HANDLE(n, 0, y.second)}); }
            for (uint64_t v : newly) {
                const uint64_t iid = unproposed.next();
                initial[iid] = v;
                b.push_back({iid, MPX_HANDLE(n, 0, v)});
            }
            newly.clear();
            preparing = false;
            std::sort(b.begin(), b.end());                 // AcceptingValues::values_ is a map
            app<uint64_t>(st.body, x.seq);
            app<uint64_t>(st.body, b.size());
            for (auto &y : b) { app<uint64_t>(st.body, y.first); app<uint64_t>(st.body, y.second); }
            ++st.count;
        }
    }
}

static std::vector<PropNode> *prop_new(uint32_t nodes) { return new std::vector<PropNode>(nodes); }
static void prop_free(std::vector<PropNode> *p) { delete p; }

static void prop_bytes(const std::vector<PropNode> &st, std::string &d)
{
    d.append("MPXD", 4);
    app<uint32_t>(d, 1); app<uint32_t>(d, (uint32_t)st.size());
    for (auto &x : st) { app<uint64_t>(d, x.count); d += x.body; }
}

static void proposer_sim(const PEvents &ev, std::string &d)
{
    std::vector<PropNode> st(ev.size());
    for (uint32_t n = 0; n < ev.size(); ++n) prop_advance(st[n], n, ev[n]);
    prop_bytes(st, d);
}

// MPX_FLAG_DECISIONS: the proposers' bookkeeping advanced over the last window's events (its
// quorums' merged maps carry the pre-accepted values of earlier windows, k_apply_win)
static int member_events(mpx_engine *e, const Results &r, PEvents &ev);
static int mprop_advance(MPropNode &st, uint32_t n, const std::vector<PEv> &evs, const std::vector<mpx_epoch> &ep);
static int learn_window(mpx_engine *e, const Results &r);

static int prop_window(mpx_engine *e)
{
    Results r;
    TRY(fetch_results(e, r));
    PEvents ev;
    if (e->mprop) {
        TRY(member_events(e, r, ev));
        for (uint32_t n = 0; n < e->cfg.num_nodes; ++n) TRY(mprop_advance((*e->mprop)[n], n, ev[n], e->epochs));
        return learn_window(e, r);
    }
    proposer_events(e, r, ev);
    for (uint32_t n = 0; n < e->cfg.num_nodes; ++n) prop_advance((*e->prop)[n], n, ev[n]);
    return MPX_OK;
}

static int proposer_decisions(mpx_engine *e, const Results &r, std::string &d)
{
    PEvents ev;
    proposer_events(e, r, ev);
    proposer_sim(ev, d);
    return MPX_OK;
}

static bool has_proposals(const HostTrace &h)
{
    return !h.prop_seq.empty();
}

// Member semantics (member/paxos.cpp:1183-1297): the same batch over the proposer's
// unlearned ids — Proposer::OnLearn (:1383-1470) removes a newly learned id from the
// unlearned / unproposed sets and re-proposes an initial proposal that lost its id; a
// P_PROPOSE record is Node::Propose -> Proposer::Propose (:1122-1156, value_id_ + 1: the
// next unproposed id now, or queued while preparing; without a Proposer the value is
// Unproposable, :786-789).  A Proposer starts with every id unlearned and preparing
// (:1074-1082); the engine model idles it at the E_EPOCH run that created it or changed
// its acceptors (include/mpx.h).  Host walk over the device's promise quorums (F_QUORUM)
// and merged maps (k_apply's records).
static int put_bytes(const std::string &d, uint8_t **out, uint64_t *size);

// The member bookkeeping reads, per node in stream order: Propose, StartPrepare, each
// promise quorum's merged map, each LEARN's entries and the E_EPOCH markers (aux: the
// epoch).  Headers are replicated over instance shards, entries split (mpx_proposal_part).
static int member_events(mpx_engine *e, const Results &r, PEvents &ev)
{
    const HostTrace &h = e->ht;
    const uint32_t N = e->cfg.num_nodes;
    ev.assign(N, {});
    for (uint32_t n = 0; n < N; ++n)
        for (uint64_t g = h.node_off[n]; g < h.node_off[n + 1]; ++g) {
            const uint8_t t = h.m_type[g];
            const bool quorum = t == MPX_MSG_PREPARE_REPLY && (r.flags[g] & F_QUORUM);
            if (t != MPX_MSG_P_START && t != MPX_MSG_COMMIT && t != MPX_MSG_E_EPOCH && !quorum)
                continue;
            PEv x{seq_of(h, n, g) + (e->incremental ? e->win_seq_base[n] : 0), t, {}};
            if (t == MPX_MSG_E_EPOCH) x.aux = h.m_ver[g];
            if (t == MPX_MSG_COMMIT)
                for (uint64_t k = h.m_ent[g]; k < h.m_ent[g] + h.m_cnt[g]; ++k) x.ents.push_back({h.e_iid[k], h.e_val[k]});
            if (quorum) {
                auto it = r.by_msg[1].find((uint32_t)g);
                if (it != r.by_msg[1].end())
                    for (const OutEnt *o : it->second) x.ents.push_back({o->iid, o->handle});
                std::sort(x.ents.begin(), x.ents.end());
            }
            ev[n].push_back(std::move(x));
        }
    for (uint32_t n = 0; n < N; ++n) merge_proposals(e, n, ev[n]);
    return MPX_OK;
}

// One node's member Proposer bookkeeping, advanced over its events (a whole run, window by
// window under MPX_FLAG_DECISIONS, or over the union of shard parts).  A Proposer starts
// with every id unlearned and preparing (:1074-1082); the engine model idles it at the
// E_EPOCH run that created it or changed its acceptors (include/mpx.h) — until the node's
// next record that is not a marker, which the events stand for (nothing between them reads
// the flag).
struct MPropNode {
    struct P {
        IdSet unlearned, unproposed;
        std::map<uint64_t, uint64_t> initial;          // initial_proposals_: instance -> value id
        std::set<uint64_t> newly;                      // newly_proposed_values_
        uint64_t vid = 0;                              // value_id_
        bool preparing = true;
    };
    std::unique_ptr<P> p;
    IdSet notlearned;                                  // the learner's learned_values_, complemented
    uint32_t ei = 0;
    bool idle = false, started = false;
    std::string body;
    uint64_t count = 0;
};

static std::vector<MPropNode> *mprop_new(uint32_t nodes) { return new std::vector<MPropNode>(nodes); }
static void mprop_free(std::vector<MPropNode> *p) { delete p; }

static int mprop_advance(MPropNode &st, uint32_t n, const std::vector<PEv> &evs, const std::vector<mpx_epoch> &ep)
{
    if (!st.started) {                                 // the genesis roles (NodeImpl::Loop, :738-747)
        st.started = true;
        if ((ep[0].proposer_mask >> n) & 1) { st.p.reset(new MPropNode::P); st.p->preparing = false; }
    }
    auto &p = st.p;
    for (const PEv &x : evs) {
        const uint32_t t = x.type;
        if (t != MPX_MSG_E_EPOCH && st.idle) {
            if (p) p->preparing = false;
            st.idle = false;
        }
        if (t == MPX_MSG_P_START) {
            if (p) p->preparing = true;
        } else if (t == MPX_MSG_P_PROPOSE) {               // Proposer::Propose (:1122-1156)
            if (p) {
                ++p->vid;
                if (!p->preparing) p->initial[p->unproposed.next()] = p->vid;
                else p->newly.insert(p->vid);
            }
        } else if (t == MPX_MSG_PREPARE_REPLY) {           // a promise quorum (:1183-1297)
            if (!p) continue;
            IdSet un = p->unlearned;
            std::vector<std::pair<uint64_t, uint64_t>> b;
            for (auto &en : x.ents)
                if (un.contains(en.first)) { un.remove(en.first); b.push_back(en); }
            while (un.r.size() > 1) {
                const auto first = *un.r.begin();
                un.r.erase(un.r.begin());
                for (uint64_t id = first.first; id != first.second; ++id) b.push_back({id, MPX_HANDLE(n, 1, ++p->vid)});
            }
            for (auto &y : p->initial)
                if (un.contains(y.first)) { un.remove(y.first); b.push_back({y.first, MPX_HANDLE(n, 0, y.second)}); }
            for (uint64_t v : p->newly) {
                const uint64_t iid = un.next();
                p->initial[iid] = v;
                b.push_back({iid, MPX_HANDLE(n, 0, v)});
            }
            p->newly.clear();
            p->unproposed = un;
            p->preparing = false;
            std::sort(b.begin(), b.end());
            app<uint64_t>(st.body, x.seq);
            app<uint64_t>(st.body, b.size());
            for (auto &y : b) { app<uint64_t>(st.body, y.first); app<uint64_t>(st.body, y.second); }
            ++st.count;
        } else if (t == MPX_MSG_COMMIT) {                  // LEARN: Learner::OnLearn (:1029-1060)
            if (p) {                                       // Proposer::OnLearn (:1383-1470)
                std::set<uint64_t> conflicts;
                for (auto &en : x.ents) {
                    const uint64_t iid = en.first, hv = en.second;
                    if (st.notlearned.contains(iid) && p->unlearned.contains(iid)) p->unlearned.remove(iid);
                    if (p->unproposed.contains(iid)) p->unproposed.remove(iid);
                    auto in = p->initial.find(iid);
                    if (in != p->initial.end()) {
                        if (MPX_HANDLE_PROPOSER(hv) != n || MPX_HANDLE_VALUE_ID(hv) != in->second) conflicts.insert(in->second);
                        p->initial.erase(in);
                    }
                }
                if (!p->preparing) { for (uint64_t v : conflicts) p->initial[p->unproposed.next()] = v; }
                else p->newly.insert(conflicts.begin(), conflicts.end());
            }
            for (auto &en : x.ents)
                if (st.notlearned.contains(en.first)) st.notlearned.remove(en.first);
        } else if (t == MPX_MSG_E_EPOCH) {
            const uint64_t ej = x.aux;
            if (ej >= ep.size()) return MPX_E_DECODE;
            const mpx_epoch &o = ep[st.ei], &y = ep[ej];
            const bool was = (o.proposer_mask >> n) & 1, now = (y.proposer_mask >> n) & 1;
            if (now && !was) p.reset(new MPropNode::P);    // the constructor's StartPrepare
            if (was && !now) p.reset();
            if (p && y.acceptor_mask != o.acceptor_mask) p->preparing = true;   // AcceptorsChanged
            if (now && (!was || o.acceptor_mask != y.acceptor_mask)) st.idle = true;
            st.ei = (uint32_t)ej;
        }
    }
    return MPX_OK;
}

static void mprop_bytes(const std::vector<MPropNode> &st, std::string &d)
{
    d.append("MPXD", 4);
    app<uint32_t>(d, 1); app<uint32_t>(d, (uint32_t)st.size());
    for (auto &x : st) { app<uint64_t>(d, x.count); d += x.body; }
}

static int member_sim(const PEvents &ev, const std::vector<mpx_epoch> &ep, std::string &d)
{
    std::vector<MPropNode> st(ev.size());
    for (uint32_t n = 0; n < ev.size(); ++n) TRY(mprop_advance(st[n], n, ev[n], ep));
    mprop_bytes(st, d);
    return MPX_OK;
}

static int member_decisions(mpx_engine *e, const Results &r, std::string &d)
{
    PEvents ev;
    TRY(member_events(e, r, ev));
    return member_sim(ev, e->epochs, d);
}

// ------------------------------------------------- phase-2 decisions (f2) --
// The batch OnPrepareReply builds at each promise quorum (multi/paxos.cpp:
// 1056-1130) for a proposer with no client proposals of its own: the device
// finds, per event, the highest instance the node had committed before it and
// the instances to noop-fill (kernels.hip k_decide); the adopted values are the
// quorum's merged map minus what the node had committed (k_apply's records).
// The host merges the two sorted lists and numbers the noops per node
// (Value(index_, ++value_id_)).  Format MPXD (include/mpx.h).
extern "C" int mpx_read_decisions(mpx_engine *e, uint8_t **out, uint64_t *size)
{
    if (!e || !out || !size) return MPX_E_INVAL;
    if (e->poisoned) return MPX_E_STATE;            // (MPX_FLAG_INCREMENTAL: a failed window)
    if (e->incremental) {                               // windows keep no history of runs, but
        if ((!e->prop && !e->mprop) || e->cfg.shard_begin != 0) return MPX_E_STATE;   // MPX_FLAG_DECISIONS
        std::string d;                                  // carries the bookkeeping: every window's quorums so far
        if (e->mprop) mprop_bytes(*e->mprop, d);
        else prop_bytes(*e->prop, d);
        return put_bytes(d, out, size);
    }
    if (e->cfg.shard_begin != 0) return MPX_E_STATE;
    if (e->cfg.semantics == MPX_SEM_MEMBER) {
        if (!e->whole) return MPX_E_STATE;               // the learner's whole learned set
        Results r;
        TRY(fetch_results(e, r));
        std::string d;
        TRY(member_decisions(e, r, d));
        return put_bytes(d, out, size);
    }
    Results r;
    TRY(fetch_results(e, r));
    const char *hs = std::getenv("MPX_DECIDE_HOST");     // (A/B: the bookkeeping without proposals too)
    if (has_proposals(e->ht) || (hs && std::atoi(hs))) {
        if (!e->whole) return MPX_E_STATE;               // the bookkeeping needs every instance's commits
        std::string d;
        TRY(proposer_decisions(e, r, d));
        *out = (uint8_t *)std::malloc(d.size());
        if (!*out) return MPX_E_NOMEM;
        std::memcpy(*out, d.data(), d.size());
        *size = d.size();
        return MPX_OK;
    }
    std::vector<DecideEv> evs;
    TRY(decide_core(e, r, nullptr, 0, false, evs));
    const uint32_t N = e->cfg.num_nodes;
    std::string d;
    d.append("MPXD", 4);
    app<uint32_t>(d, 1); app<uint32_t>(d, N);
    std::vector<uint64_t> vid(N, 0);                     // value_id_ per node (:335, ++ per noop)
    size_t k = 0;
    for (uint32_t n = 0; n < N; ++n) {
        const size_t k0 = k;
        while (k < evs.size() && evs[k].node == n) ++k;
        app<uint64_t>(d, k - k0);
        for (size_t x = k0; x < k; ++x) {
            app<uint64_t>(d, seq_of(e->ht, n, evs[x].msg));
            decide_entries(evs[x], &vid[n], d);
        }
    }
    *out = (uint8_t *)std::malloc(d.size());
    if (!*out) return MPX_E_NOMEM;
    std::memcpy(*out, d.data(), d.size());
    *size = d.size();
    return MPX_OK;
}

// Sharded form (include/mpx.h): every rank's per-event bound, then its part with
// the fill cut at the global bound, then the parts merged in shard order.
extern "C" int mpx_decisions_bounds(mpx_engine *e, uint64_t *bounds, uint64_t cap, uint64_t *count)
{
    if (!e || !count || (cap && !bounds)) return MPX_E_INVAL;
    if (e->incremental) return MPX_E_STATE;             // windows keep no history of runs
    if (e->cfg.semantics != MPX_SEM_MULTI) return MPX_E_STATE;
    Results r;
    TRY(fetch_results(e, r));
    if (has_proposals(e->ht)) return MPX_E_STATE;        // own values: mpx_read_decisions on a whole engine
    std::vector<DecideEv> evs;
    TRY(decide_core(e, r, nullptr, 0, true, evs));
    *count = evs.size();
    for (size_t k = 0; k < evs.size() && k < cap; ++k) bounds[k] = evs[k].bound;
    return MPX_OK;
}

extern "C" int mpx_read_decisions_part(mpx_engine *e, const uint64_t *global_bounds, uint64_t count,
                                       uint8_t **out, uint64_t *size)
{
    if (!e || !out || !size || (count && !global_bounds)) return MPX_E_INVAL;
    if (e->incremental) return MPX_E_STATE;             // windows keep no history of runs
    if (e->cfg.semantics != MPX_SEM_MULTI) return MPX_E_STATE;
    Results r;
    TRY(fetch_results(e, r));
    if (has_proposals(e->ht)) return MPX_E_STATE;        // own values: mpx_read_decisions on a whole engine
    std::vector<DecideEv> evs;
    TRY(decide_core(e, r, global_bounds, count, false, evs));
    const uint32_t N = e->cfg.num_nodes;
    std::string d;
    d.append("MPXP", 4);
    app<uint32_t>(d, 1); app<uint32_t>(d, N);
    app<uint64_t>(d, e->cfg.shard_begin);
    size_t k = 0;
    for (uint32_t n = 0; n < N; ++n) {
        const size_t k0 = k;
        while (k < evs.size() && evs[k].node == n) ++k;
        app<uint64_t>(d, k - k0);
        for (size_t x = k0; x < k; ++x) {
            app<uint64_t>(d, seq_of(e->ht, n, evs[x].msg));
            decide_entries(evs[x], nullptr, d);
        }
    }
    *out = (uint8_t *)std::malloc(d.size());
    if (!*out) return MPX_E_NOMEM;
    std::memcpy(*out, d.data(), d.size());
    *size = d.size();
    return MPX_OK;
}

extern "C" int mpx_decisions_combine(const uint8_t *const *parts, const uint64_t *sizes, uint32_t nparts,
                                     uint8_t **out, uint64_t *size)
{
    if (!parts || !sizes || !nparts || !out || !size) return MPX_E_INVAL;
    struct P { const uint8_t *p; uint64_t n, pos; uint64_t sb; };
    std::vector<P> ps(nparts);
    uint32_t N = 0;
    for (uint32_t i = 0; i < nparts; ++i) {
        if (!parts[i] || sizes[i] < 20 || std::memcmp(parts[i], "MPXP", 4) || rd32(parts[i] + 4) != 1) return MPX_E_INVAL;
        const uint32_t n = rd32(parts[i] + 8);
        if (i && n != N) return MPX_E_INVAL;
        N = n;
        ps[i] = P{parts[i], sizes[i], 20, rd64(parts[i] + 12)};
        if (i && ps[i].sb <= ps[i - 1].sb) return MPX_E_INVAL;        // shard order
    }
    auto need = [](const P &q, uint64_t b) { return q.pos + b <= q.n; };
    std::string d;
    d.append("MPXD", 4);
    app<uint32_t>(d, 1); app<uint32_t>(d, N);
    for (uint32_t node = 0; node < N; ++node) {
        uint64_t cnt = 0;
        for (uint32_t i = 0; i < nparts; ++i) {
            if (!need(ps[i], 8)) return MPX_E_INVAL;
            const uint64_t c = rd64(ps[i].p + ps[i].pos); ps[i].pos += 8;
            if (i && c != cnt) return MPX_E_INVAL;                  // the same quorums on every shard
            cnt = c;
        }
        app<uint64_t>(d, cnt);
        uint64_t vid = 0;                                           // value_id_ of the node (:335)
        for (uint64_t q = 0; q < cnt; ++q) {
            std::string ents;
            uint64_t tot = 0, seq = 0;
            for (uint32_t i = 0; i < nparts; ++i) {
                if (!need(ps[i], 16)) return MPX_E_INVAL;
                const uint64_t sq = rd64(ps[i].p + ps[i].pos), m = rd64(ps[i].p + ps[i].pos + 8);
                ps[i].pos += 16;
                if (i && sq != seq) return MPX_E_INVAL;
                seq = sq;
                if (!need(ps[i], 16 * m)) return MPX_E_INVAL;
                // a part holds only its own shard's instances: [its shard_begin, the next part's)
                const uint64_t lo = ps[i].sb, hi = i + 1 < nparts ? ps[i + 1].sb : ~0ull;
                for (uint64_t j = 0; j < m; ++j) {
                    const uint64_t iid = rd64(ps[i].p + ps[i].pos), h = rd64(ps[i].p + ps[i].pos + 8);
                    ps[i].pos += 16;
                    if (iid < lo || iid >= hi) return MPX_E_INVAL;
                    app<uint64_t>(ents, iid);
                    app<uint64_t>(ents, h == NOOP_SLOT ? MPX_HANDLE(node, 1, ++vid) : h);
                }
                tot += m;
            }
            app<uint64_t>(d, seq); app<uint64_t>(d, tot);
            d += ents;
        }
    }
    for (uint32_t i = 0; i < nparts; ++i)
        if (ps[i].pos != ps[i].n) return MPX_E_INVAL;                // trailing bytes: another layout
    *out = (uint8_t *)std::malloc(d.size() ? d.size() : 1);
    if (!*out) return MPX_E_NOMEM;
    std::memcpy(*out, d.data(), d.size());
    *size = d.size();
    return MPX_OK;
}

// ---------------------------------------------- commit reliability (f4) --
// The proposer's CommittingValues bookkeeping (multi/paxos.cpp:1184-1197,
// 1416-1421, 1625-1641).  A node creates commit id ++committing_id_ at every
// accept quorum (the batch's chosen reply, k_votes) and at every promise quorum
// where it holds committed values (k_decide pass 0: the highest instance it had
// committed before the quorum exists); the host ranks those per node in message
// order.  k_commits walks the COMMIT_REPLYs of each (node, commit id) on the
// device: replied_ as a learner mask, retired at |replied_| == N.
// Format MPXC (include/mpx.h).
// Commit creation points of one engine, per node in stream order: {seq, accept id}
// for an accept quorum of a batch this engine kept (its chosen reply), {seq, ~0} for
// a promise quorum at which the node held a committed instance of this shard.
// A shard engine sees only its own batches and instances: the union over shards
// (mpx_commit_points_combine) is the node's whole list.
typedef std::vector<std::vector<std::pair<uint64_t, uint64_t>>> CommitPoints;
static int commit_points(mpx_engine *e, const Results &r, CommitPoints &cm)
{
    const HostTrace &h = e->ht;
    const uint32_t N = e->cfg.num_nodes;
    // promise quorums: did the node hold a committed value there (xmax > 0)
    std::vector<uint32_t> qn, qg;
    for (uint32_t n = 0; n < N; ++n)
        for (uint64_t g = h.node_off[n]; g < h.node_off[n + 1]; ++g)
            if (h.m_type[g] == MPX_MSG_PREPARE_REPLY && (r.flags[g] & F_QUORUM)) { qn.push_back(n); qg.push_back((uint32_t)g); }
    std::vector<uint64_t> xmax;
    TRY(committed_before(e, qn, qg, xmax));
    cm.assign(N, {});
    for (size_t j = 0; j < h.b_msg.size(); ++j)
        if (r.b_chosen[j] != NONE32) {
            const uint32_t n = h.m_node[h.b_msg[j]];
            cm[n].push_back({seq_of(h, n, r.b_chosen[j]), h.m_aux[h.b_msg[j]]});
        }
    for (size_t k = 0; k < qn.size(); ++k)
        if (xmax[k]) cm[qn[k]].push_back({seq_of(h, qn[k], qg[k]), ~0ull});
    for (auto &l : cm) std::sort(l.begin(), l.end());
    return MPX_OK;
}

static int put_bytes(const std::string &d, uint8_t **out, uint64_t *size)
{
    *out = (uint8_t *)std::malloc(d.size() ? d.size() : 1);
    if (!*out) return MPX_E_NOMEM;
    std::memcpy(*out, d.data(), d.size());
    *size = d.size();
    return MPX_OK;
}

// MPXC from a node's whole list of creation points (ids = rank in stream order) and
// this engine's COMMIT_REPLYs (it must have kept every one: shard at instance 0)
static int commits_from_points(mpx_engine *e, const CommitPoints &cm, std::string &d)
{
    const HostTrace &h = e->ht;
    const uint32_t N = e->cfg.num_nodes;
    hipStream_t s = e->stream;
    std::vector<uint64_t> cm_off(N + 1, 0);
    std::vector<uint32_t> cm_pos;
    for (uint32_t n = 0; n < N; ++n) {
        for (auto &x : cm[n]) {
            if (x.first >= NONE32) return MPX_E_RANGE;
            cm_pos.push_back((uint32_t)x.first);
        }
        cm_off[n + 1] = cm_pos.size();
    }
    // reply lists: the COMMIT_REPLYs of each (node, commit id), in processing order;
    // positions are record indices in the node's stream (the creation points' unit)
    std::vector<uint64_t> cr_off(1, 0), cr_id;
    std::vector<uint32_t> cr_msg, cr_src, cr_node;
    {
        std::vector<std::vector<uint32_t>> lists;
        std::map<uint64_t, uint32_t> idx;
        for (uint32_t n = 0; n < N; ++n) {
            idx.clear();
            for (uint64_t g = h.node_off[n]; g < h.node_off[n + 1]; ++g) {
                if (h.m_type[g] != MPX_MSG_COMMIT_REPLY) continue;
                if (h.m_src[g] >= 64) return MPX_E_RANGE;           // replied_ as a 64-bit learner mask
                auto it = idx.find(h.m_aux[g]);
                if (it == idx.end()) {
                    it = idx.emplace(h.m_aux[g], (uint32_t)lists.size()).first;
                    lists.emplace_back();
                    cr_id.push_back(h.m_aux[g]);
                    cr_node.push_back(n);
                }
                lists[it->second].push_back((uint32_t)g);
            }
        }
        for (size_t l = 0; l < lists.size(); ++l) {
            for (uint32_t g : lists[l]) {
                const uint64_t sq = seq_of(h, cr_node[l], g);
                if (sq >= NONE32) return MPX_E_RANGE;
                cr_msg.push_back((uint32_t)sq); cr_src.push_back(h.m_src[g]);
            }
            cr_off.push_back(cr_msg.size());
        }
    }
    const uint32_t L = (uint32_t)cr_id.size();
    std::vector<uint32_t> ret;
    std::vector<uint64_t> mask;
    if (L) {
        DevBuf d_off, d_id, d_cmoff, d_msg, d_src, d_node, d_pos, d_ret, d_mask;
        TRY(upload(d_off, cr_off, s)); TRY(upload(d_id, cr_id, s)); TRY(upload(d_cmoff, cm_off, s));
        TRY(upload(d_msg, cr_msg, s)); TRY(upload(d_src, cr_src, s)); TRY(upload(d_node, cr_node, s));
        if (cm_pos.empty()) cm_pos.push_back(0);
        TRY(upload(d_pos, cm_pos, s));
        TRY(d_ret.alloc(4ull * L)); TRY(d_mask.alloc(8ull * L));
        CommitArgs a{L, d_off.as<uint64_t>(), d_id.as<uint64_t>(), d_cmoff.as<uint64_t>(), d_msg.as<uint32_t>(),
                     d_src.as<uint32_t>(), d_node.as<uint32_t>(), d_pos.as<uint32_t>(), d_ret.as<uint32_t>(),
                     d_mask.as<unsigned long long>()};
        if (launch_commits(e->view, s, a) != 0) return MPX_E_HIP;
        HTRY(hipStreamSynchronize(s));
        TRY(d2h(ret, d_ret, L)); TRY(d2h(mask, d_mask, L));
    }
    // per node, per commit id: the list that names it (if any)
    std::vector<std::map<uint64_t, uint32_t>> by_id(N);
    for (uint32_t l = 0; l < L; ++l) by_id[cr_node[l]][cr_id[l]] = l;
    d.append("MPXC", 4);
    app<uint32_t>(d, 1); app<uint32_t>(d, N);
    for (uint32_t n = 0; n < N; ++n) {
        app<uint64_t>(d, cm[n].size());
        for (size_t k = 0; k < cm[n].size(); ++k) {
            const uint64_t id = k + 1;
            auto it = by_id[n].find(id);
            const bool has = it != by_id[n].end();
            const uint32_t rg = has ? ret[it->second] : NONE32;
            app<uint64_t>(d, id);
            app<uint64_t>(d, cm[n][k].first);
            app<uint64_t>(d, cm[n][k].second == ~0ull ? 1 : 0);
            app<uint64_t>(d, cm[n][k].second == ~0ull ? 0 : cm[n][k].second);
            app<uint64_t>(d, rg == NONE32 ? ~0ull : (uint64_t)rg);
            app<uint64_t>(d, has ? mask[it->second] : 0);
        }
    }
    return MPX_OK;
}

extern "C" int mpx_read_commits(mpx_engine *e, uint8_t **out, uint64_t *size)
{
    if (!e || !out || !size) return MPX_E_INVAL;
    if (e->incremental) return MPX_E_STATE;             // windows keep no history of runs
    if (e->cfg.semantics != MPX_SEM_MULTI || !e->whole) return MPX_E_STATE;
    Results r;
    TRY(fetch_results(e, r));
    CommitPoints cm;
    TRY(commit_points(e, r, cm));
    std::string d;
    TRY(commits_from_points(e, cm, d));
    return put_bytes(d, out, size);
}

// ------------------------------------------------ learn reliability (f4) --
// The member Proposer's LearningValues bookkeeping (member/paxos.cpp:1299-1307,1334-1337,
// 1345-1381,1472-1549,1864-1964).  The host walks each node's stream once for the control
// plane: which Proposer incarnation runs (its learning_id_ restarts), whether it is
// preparing, where it creates a learn — at an accept quorum (the batch's chosen reply,
// k_votes), at a promise quorum once its learner learned anything (F_QUORUM, k_prop_*),
// at LearnersChanged while not preparing — and where LearnersChanged or the Proposer's
// deletion drops every open learn; the membership steps come from the E_EPOCH markers
// that follow the LEARN which applied them (learners gained, then the Proposer created,
// then acceptors gained; acceptors lost, then the Proposer deleted, then learners lost:
// the reference's change lists, :638-723).  k_learns then walks each learn's replies and
// AcceptorsChanged calls on the device.  Format MPXL (include/mpx.h).
struct LearnPlan {
    uint32_t node;
    uint64_t id, created, kind, src;
    uint8_t facc;
    uint32_t end = NONE32;
    std::vector<uint64_t> ev_a, ev_m;
    // its values_ (mpx_read_learn_values): kind 0 the batch's {iid, handle}; kinds 1 and 2 the
    // Learner's learned values then — the first log_len of the node's learn log (:1299-1301,
    // :1476) — and kind 2 also every open learn's values (`parents`, id order; one that had
    // retired by then is skipped at read time, retirement being k_learns' finding, :1477-1482)
    uint64_t log_len = 0;
    std::vector<uint32_t> parents;
    std::vector<std::pair<uint64_t, uint64_t>> batch;
};

// one node's walk state (carried across windows under MPX_FLAG_DECISIONS); `live` indexes
// the incarnation's open learns in the plan list
struct LearnNode {
    bool started = false, prop = false, preparing = false, learned_any = false, idle = false;
    uint32_t ei = 0;
    uint64_t lid = 0, amask = 0, K = 0;                        // K: the last non-marker record
    std::vector<size_t> live;
    // the Learner's learned_values_ (insert: the first Value of an instance sticks, :1040) in
    // the order it learned them, and a bit per shard instance learned
    std::vector<std::pair<uint64_t, uint64_t>> llog;
    std::vector<uint64_t> lbits;
    std::vector<uint64_t> unprop;                              // Unproposable P_PROPOSE records (:784-787)
};
struct LearnCarry {
    std::vector<LearnNode> nodes;
    std::vector<LearnPlan> plans;
};
static LearnCarry *learn_new(uint32_t nodes) { LearnCarry *c = new LearnCarry; c->nodes.resize(nodes); return c; }
static void learn_free(LearnCarry *c) { delete c; }

static int learn_plan(mpx_engine *e, const Results &r, std::vector<LearnNode> &nodes, std::vector<LearnPlan> &out)
{
    const HostTrace &h = e->ht;
    const uint32_t N = e->cfg.num_nodes;
    const auto &ep = e->epochs;
    std::unordered_map<uint32_t, std::pair<uint64_t, uint32_t>> chosen_at;   // accept quorum message -> (accept id, batch)
    const bool aid = h.b_aid.size() == h.b_msg.size();         // (a window's earlier batches: carried ids)
    for (size_t j = 0; j < h.b_msg.size(); ++j)
        if (r.b_chosen[j] != NONE32 && (aid || h.b_msg[j] != NONE32))
            chosen_at[r.b_chosen[j]] = {aid ? h.b_aid[j] : h.m_aux[h.b_msg[j]], (uint32_t)j};
    // a chosen batch's values: its P_BATCH's entries; a window's earlier batch (b_msg NONE32): the
    // chosen-log runs build_trace cut from its carried entries (the carry itself may have let them go
    // already — a P_START later in the window ends the batch, after its votes completed)
    std::unordered_map<uint32_t, std::vector<uint32_t>> carried;
    bool carried_ready = false;
    auto batch_values = [&](uint32_t j, std::vector<std::pair<uint64_t, uint64_t>> &v) {
        const uint32_t g = h.b_msg[j];
        if (g != NONE32) {
            for (uint64_t k = h.m_ent[g]; k < h.m_ent[g] + h.m_cnt[g]; ++k) v.push_back({h.e_iid[k], h.e_val[k]});
        } else {
            if (!carried_ready) {
                carried_ready = true;
                for (size_t f = 0; f < h.cfrags.size(); ++f)
                    if (h.cfrags[f].msg < h.b_msg.size() && h.b_msg[h.cfrags[f].msg] == NONE32)
                        carried[h.cfrags[f].msg].push_back((uint32_t)f);
            }
            auto it = carried.find(j);
            if (it != carried.end())
                for (uint32_t f : it->second)
                    for (uint32_t q = 0; q < h.cfrags[f].count; ++q)
                        v.push_back({h.e_iid[h.cfrags[f].entry + q], h.e_val[h.cfrags[f].entry + q]});
        }
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
    };
    const uint64_t lwords = (h.shard_len + 63) / 64;
    for (uint32_t n = 0; n < N; ++n) {
        LearnNode &st = nodes[n];
        if (!st.started) {
            st.started = true;
            st.prop = (ep[0].proposer_mask >> n) & 1;
            st.amask = ep[0].acceptor_mask;
        }
        uint32_t &ei = st.ei;
        bool &prop = st.prop, &preparing = st.preparing, &learned_any = st.learned_any, &idle = st.idle;
        uint64_t &lid = st.lid, &amask = st.amask, &K = st.K;
        std::vector<size_t> &live = st.live;
        auto create = [&](uint64_t at, uint64_t kind, uint64_t src, bool facc) {
            LearnPlan p;
            p.node = n; p.id = ++lid; p.created = at; p.kind = kind; p.src = src; p.facc = facc;
            p.log_len = st.llog.size();
            live.push_back(out.size());
            out.push_back(std::move(p));
        };
        auto drop_all = [&](uint64_t at) {
            for (size_t x : live) out[x].end = (uint32_t)at;
            live.clear();
        };
        auto acc_changed = [&](uint64_t at, uint32_t who, bool add) {     // AcceptorsChanged (:1504-1549)
            for (size_t x : live)
                if (out[x].facc) {
                    out[x].ev_a.push_back(at << 32 | (uint64_t)LEV_ACC << 24 | (uint64_t)add << 23 | who);
                    out[x].ev_m.push_back(amask);
                }
            preparing = true;                                      // RestartPrepare / AcceptRejected
        };
        auto learners_changed = [&](uint64_t at) {                 // LearnersChanged (:1472-1502)
            const std::vector<size_t> open = live;
            drop_all(at);
            if (!preparing) {
                create(at, 2, 0, true);
                for (size_t x : open) out.back().parents.push_back((uint32_t)x);
            }
        };
        // P_PROPOSE records are host bookkeeping only (not in the device's message arrays): merged
        // in by record index, Node::Propose without a Proposer is Unproposable (NodeImpl::Loop, :784-787)
        const uint64_t sbase = e->incremental ? e->win_seq_base[n] : 0;
        uint64_t pp = n + 1 < h.prop_off.size() ? h.prop_off[n] : 0;
        const uint64_t pe = n + 1 < h.prop_off.size() ? h.prop_off[n + 1] : 0;
        auto proposes_before = [&](uint64_t k) {
            for (; pp < pe && h.prop_seq[pp] + sbase < k; ++pp)
                if (!prop) st.unprop.push_back(h.prop_seq[pp] + sbase);
        };
        for (uint64_t g = h.node_off[n]; g < h.node_off[n + 1]; ++g) {
            const uint8_t t = h.m_type[g];
            const uint64_t k = seq_of(h, n, g) + sbase;
            if (k >= NONE32) return MPX_E_RANGE;
            proposes_before(k);
            if (t != MPX_MSG_E_EPOCH) {
                K = k;
                if (idle) { preparing = false; idle = false; }     // after the marker run (below)
            }
            if (t == MPX_MSG_PREPARE_REPLY && (r.flags[g] & F_QUORUM)) {
                preparing = false;                                 // OnPrepareReply's quorum (:1171-1307)
                if (learned_any) create(k, 1, 0, true);
            } else if (t == MPX_MSG_ACCEPT_REPLY) {
                auto it = chosen_at.find((uint32_t)g);
                if (it != chosen_at.end()) {                       // OnAcceptReply (:1327-1342)
                    create(k, 0, it->second.first, false);
                    batch_values(it->second.second, out.back().batch);
                }
            } else if (t == MPX_MSG_COMMIT_REPLY) {                // LEARN_REPLY -> OnLearnReply
                if (!prop) continue;
                if (h.m_src[g] >= 64) return MPX_E_RANGE;
                for (size_t x : live)
                    if (out[x].id == h.m_aux[g]) {
                        out[x].ev_a.push_back(k << 32 | (uint64_t)LEV_REPLY << 24 |
                                              (uint64_t)__builtin_popcountll(ep[ei].learner_mask) << 8 | h.m_src[g]);
                        out[x].ev_m.push_back(amask);
                    }
            } else if (t == MPX_MSG_P_START) {
                if (prop) preparing = true;
            } else if (t == MPX_MSG_COMMIT) {                      // LEARN (Learner::OnLearn, :1029-1060)
                if (h.m_cnt[g]) learned_any = true;
                if (h.m_cnt[g] && st.lbits.empty()) st.lbits.assign(lwords, 0);
                for (uint64_t x = h.m_ent[g]; x < h.m_ent[g] + h.m_cnt[g]; ++x) {   // learned_values_.insert (:1040)
                    const uint64_t li = h.e_iid[x] - h.shard_begin;
                    if (li >= h.shard_len || (st.lbits[li >> 6] >> (li & 63) & 1)) continue;
                    st.lbits[li >> 6] |= 1ull << (li & 63);
                    st.llog.push_back({h.e_iid[x], h.e_val[x]});
                }
            } else if (t == MPX_MSG_E_EPOCH) {
                const uint32_t ej = h.m_ver[g];
                if (ej >= ep.size()) return MPX_E_DECODE;
                const mpx_epoch &o = ep[ei], &x = ep[ej];
                const bool was = (o.proposer_mask >> n) & 1, now = (x.proposer_mask >> n) & 1;
                const uint64_t gl = x.learner_mask & ~o.learner_mask, ll = o.learner_mask & ~x.learner_mask;
                const uint64_t ga = x.acceptor_mask & ~o.acceptor_mask, la = o.acceptor_mask & ~x.acceptor_mask;
                if ((gl | ga | (now && !was)) && (ll | la | (was && !now))) return MPX_E_STATE;   // not one change list
                for (uint64_t m = gl; m; m &= m - 1) if (prop) learners_changed(K);
                if (!was && now) { prop = true; lid = 0; live.clear(); preparing = false; }    // a new Proposer
                for (uint64_t m = ga; m; m &= m - 1) {
                    amask |= m & (~m + 1);
                    if (prop) acc_changed(K, (uint32_t)__builtin_ctzll(m), true);
                }
                for (uint64_t m = la; m; m &= m - 1) {
                    amask &= ~(m & (~m + 1));
                    if (prop) acc_changed(K, (uint32_t)__builtin_ctzll(m), false);
                }
                if (was && !now) { drop_all(K); prop = false; }    // the Proposer deleted (:1916-1942)
                for (uint64_t m = ll; m; m &= m - 1) if (prop) learners_changed(K);
                amask = x.acceptor_mask;
                // the engine model (include/mpx.h): a proposer created, or whose acceptor set
                // changed, is idle until its next P_START — once every change of the LEARN
                // has run (all of them happen inside it), i.e. after the marker run
                if (now && (!was || o.acceptor_mask != x.acceptor_mask)) idle = true;
                ei = ej;
            }
        }
        proposes_before(~0ull);
    }
    return MPX_OK;
}

static int learn_window(mpx_engine *e, const Results &r) { return learn_plan(e, r, e->lrn->nodes, e->lrn->plans); }

// Every learn so far with what k_learns found for it: the plans (a whole engine walks its run
// now; windows carry the walk, MPX_FLAG_DECISIONS) and, per plan, applied / retired / ended
// record and the learned mask
struct LearnsOut {
    std::vector<LearnPlan> whole_lp;
    std::vector<LearnNode> whole_nodes;
    const std::vector<LearnPlan> *lp = nullptr;
    const std::vector<LearnNode> *nodes = nullptr;
    std::vector<uint32_t> applied, retired, ended;
    std::vector<uint64_t> mask;
};

static int learns_compute(mpx_engine *e, LearnsOut &o)
{
    if (e->poisoned) return MPX_E_STATE;            // (MPX_FLAG_INCREMENTAL: a failed window)
    if (e->cfg.semantics != MPX_SEM_MEMBER || !e->whole) return MPX_E_STATE;
    if (e->incremental) {                               // windows keep no history of runs, but
        if (!e->lrn) return MPX_E_STATE;                // MPX_FLAG_DECISIONS carries the walk
        o.lp = &e->lrn->plans;
        o.nodes = &e->lrn->nodes;
    } else {
        Results r;
        TRY(fetch_results(e, r));
        o.whole_nodes.assign(e->cfg.num_nodes, LearnNode());
        TRY(learn_plan(e, r, o.whole_nodes, o.whole_lp));
        o.lp = &o.whole_lp;
        o.nodes = &o.whole_nodes;
    }
    const std::vector<LearnPlan> &lp = *o.lp;
    const uint32_t L = (uint32_t)lp.size();
    if (L) {
        std::vector<uint64_t> ev_off(1, 0), ev_a, ev_m;
        std::vector<uint8_t> facc;
        std::vector<uint32_t> end;
        for (auto &p : lp) {
            ev_a.insert(ev_a.end(), p.ev_a.begin(), p.ev_a.end());
            ev_m.insert(ev_m.end(), p.ev_m.begin(), p.ev_m.end());
            ev_off.push_back(ev_a.size());
            facc.push_back(p.facc);
            end.push_back(p.end);
        }
        if (ev_a.empty()) { ev_a.push_back(0); ev_m.push_back(0); }
        hipStream_t s = e->stream;
        DevBuf d_off, d_a, d_m, d_facc, d_end, d_app, d_ret, d_endo, d_mask;
        TRY(upload(d_off, ev_off, s)); TRY(upload(d_a, ev_a, s)); TRY(upload(d_m, ev_m, s));
        TRY(upload(d_facc, facc, s)); TRY(upload(d_end, end, s));
        TRY(d_app.alloc(4ull * L)); TRY(d_ret.alloc(4ull * L)); TRY(d_endo.alloc(4ull * L)); TRY(d_mask.alloc(8ull * L));
        LearnArgs a{L, d_off.as<uint64_t>(), d_a.as<uint64_t>(), d_m.as<uint64_t>(), d_facc.as<uint8_t>(),
                    d_end.as<uint32_t>(), d_app.as<uint32_t>(), d_ret.as<uint32_t>(), d_endo.as<uint32_t>(),
                    d_mask.as<unsigned long long>()};
        if (launch_learns(e->view, s, a) != 0) return MPX_E_HIP;
        HTRY(hipStreamSynchronize(s));
        TRY(d2h(o.applied, d_app, L)); TRY(d2h(o.retired, d_ret, L)); TRY(d2h(o.ended, d_endo, L)); TRY(d2h(o.mask, d_mask, L));
    }
    return MPX_OK;
}

extern "C" int mpx_read_learns(mpx_engine *e, uint8_t **out, uint64_t *size)
{
    if (!e || !out || !size) return MPX_E_INVAL;
    LearnsOut o;
    TRY(learns_compute(e, o));
    const std::vector<LearnPlan> &lp = *o.lp;
    const uint32_t N = e->cfg.num_nodes;
    std::vector<uint64_t> per(N, 0);
    for (auto &p : lp) per[p.node]++;
    std::string d;
    d.append("MPXL", 4);
    app<uint32_t>(d, 1); app<uint32_t>(d, N);
    auto seq = [](uint32_t x) -> uint64_t { return x == NONE32 ? ~0ull : x; };
    for (uint32_t n = 0; n < N; ++n) {
        app<uint64_t>(d, per[n]);
        for (size_t l = 0; l < lp.size(); ++l) {
            if (lp[l].node != n) continue;
            app<uint64_t>(d, lp[l].id); app<uint64_t>(d, lp[l].created); app<uint64_t>(d, lp[l].kind);
            app<uint64_t>(d, lp[l].src); app<uint64_t>(d, seq(o.applied[l])); app<uint64_t>(d, seq(o.retired[l]));
            app<uint64_t>(d, seq(o.ended[l])); app<uint64_t>(d, o.mask[l]);
        }
    }
    return put_bytes(d, out, size);
}

// The Values of every learn (LearningValues::values_, in instance order), what the Proposer's
// Callback::Accepted (kind 0, at creation, :1327-1332) and Applied (kinds 1 and 2, at the applied
// record, :1360-1368,1523-1526) iterate, and the records where Node::Propose found no Proposer
// (Unproposable, :784-787).  Format MPXV (include/mpx.h).
extern "C" int mpx_read_learn_values(mpx_engine *e, uint8_t **out, uint64_t *size)
{
    if (!e || !out || !size) return MPX_E_INVAL;
    LearnsOut o;
    TRY(learns_compute(e, o));
    const std::vector<LearnPlan> &lp = *o.lp;
    const std::vector<LearnNode> &nodes = *o.nodes;
    // values_ of plan l: a kind-2 learn's map is the learned values, then each open learn's values
    // inserted in id order (std::map::insert: the first Value of an instance stays, :1476-1482)
    std::vector<std::unique_ptr<std::map<uint64_t, uint64_t>>> memo(lp.size());
    std::function<const std::map<uint64_t, uint64_t> &(size_t)> values = [&](size_t l) -> const std::map<uint64_t, uint64_t> & {
        if (memo[l]) return *memo[l];
        auto m = std::make_unique<std::map<uint64_t, uint64_t>>();
        const LearnPlan &p = lp[l];
        if (p.kind == 0) {
            for (auto &x : p.batch) m->insert(x);
        } else {
            const auto &lg = nodes[p.node].llog;
            for (uint64_t k = 0; k < p.log_len && k < lg.size(); ++k) m->insert(lg[k]);
            for (uint32_t q : p.parents)                 // (retired before it was created: gone by then)
                if (o.retired[q] == NONE32 || o.retired[q] > p.created)
                    for (auto &x : values(q)) m->insert(x);
        }
        memo[l] = std::move(m);
        return *memo[l];
    };
    const uint32_t N = e->cfg.num_nodes;
    std::string d;
    d.append("MPXV", 4);
    app<uint32_t>(d, 1); app<uint32_t>(d, N);
    for (uint32_t n = 0; n < N; ++n) {
        uint64_t per = 0;
        for (auto &p : lp) per += p.node == n;
        app<uint64_t>(d, per);
        for (size_t l = 0; l < lp.size(); ++l) {
            if (lp[l].node != n) continue;
            const auto &m = values(l);
            app<uint64_t>(d, m.size());
            for (auto &x : m) { app<uint64_t>(d, x.first); app<uint64_t>(d, x.second); }
        }
        const auto &u = nodes[n].unprop;
        app<uint64_t>(d, u.size());
        for (uint64_t k : u) app<uint64_t>(d, k);
    }
    return put_bytes(d, out, size);
}

// Sharded commit reliability (include/mpx.h): MPXQ = "MPXQ" u32 1, u32 nodes; per
// node u64 count, {u64 seq, u64 accept_id | ~0} ascending
static void points_bytes(const CommitPoints &cm, std::string &d)
{
    d.append("MPXQ", 4);
    app<uint32_t>(d, 1); app<uint32_t>(d, (uint32_t)cm.size());
    for (auto &l : cm) {
        app<uint64_t>(d, l.size());
        for (auto &x : l) { app<uint64_t>(d, x.first); app<uint64_t>(d, x.second); }
    }
}

static int parse_points(const uint8_t *p, uint64_t n, CommitPoints &cm)
{
    if (!p || n < 12 || std::memcmp(p, "MPXQ", 4) || rd32(p + 4) != 1) return MPX_E_INVAL;
    const uint32_t N = rd32(p + 8);
    if (!N || N > MPX_MAX_NODES) return MPX_E_INVAL;
    uint64_t pos = 12;
    cm.assign(N, {});
    for (uint32_t k = 0; k < N; ++k) {
        if (pos + 8 > n) return MPX_E_INVAL;
        const uint64_t c = rd64(p + pos); pos += 8;
        if (c > (n - pos) / 16) return MPX_E_INVAL;
        for (uint64_t j = 0; j < c; ++j, pos += 16) {
            cm[k].push_back({rd64(p + pos), rd64(p + pos + 8)});
            if (j && cm[k][j] <= cm[k][j - 1]) return MPX_E_INVAL;   // ascending, no repeats
        }
    }
    return pos == n ? MPX_OK : MPX_E_INVAL;
}

extern "C" int mpx_commit_points(mpx_engine *e, uint8_t **out, uint64_t *size)
{
    if (!e || !out || !size) return MPX_E_INVAL;
    if (e->incremental) return MPX_E_STATE;             // windows keep no history of runs
    if (e->cfg.semantics != MPX_SEM_MULTI) return MPX_E_STATE;
    // a device-generated shard holds only its own batches' messages: its message positions
    // are not record indices of the node's whole stream (host traces keep them, m_seq)
    if (e->device_trace && !e->whole) return MPX_E_STATE;
    Results r;
    TRY(fetch_results(e, r));
    CommitPoints cm;
    TRY(commit_points(e, r, cm));
    std::string d;
    points_bytes(cm, d);
    return put_bytes(d, out, size);
}

extern "C" int mpx_commit_points_combine(const uint8_t *const *parts, const uint64_t *sizes, uint32_t nparts,
                                         uint8_t **out, uint64_t *size)
{
    if (!parts || !sizes || !nparts || !out || !size) return MPX_E_INVAL;
    CommitPoints all;
    for (uint32_t i = 0; i < nparts; ++i) {
        CommitPoints cm;
        TRY(parse_points(parts[i], sizes[i], cm));
        if (i && cm.size() != all.size()) return MPX_E_INVAL;
        if (!i) all.assign(cm.size(), {});
        for (size_t n = 0; n < cm.size(); ++n) all[n].insert(all[n].end(), cm[n].begin(), cm[n].end());
    }
    for (auto &l : all) {                 // the union: a batch two shards kept is one point
        std::sort(l.begin(), l.end());
        l.erase(std::unique(l.begin(), l.end()), l.end());
        for (size_t j = 1; j < l.size(); ++j)
            if (l[j].first == l[j - 1].first) return MPX_E_INVAL;   // one creation per record
    }
    std::string d;
    points_bytes(all, d);
    return put_bytes(d, out, size);
}

extern "C" int mpx_read_commits_at(mpx_engine *e, const uint8_t *points, uint64_t points_size,
                                   uint8_t **out, uint64_t *size)
{
    if (!e || !out || !size) return MPX_E_INVAL;
    if (e->incremental) return MPX_E_STATE;             // windows keep no history of runs
    if (e->cfg.semantics != MPX_SEM_MULTI || e->cfg.shard_begin != 0) return MPX_E_STATE;
    CommitPoints cm;
    TRY(parse_points(points, points_size, cm));
    if (cm.size() != e->cfg.num_nodes) return MPX_E_INVAL;
    if (!have_results(e)) return MPX_E_STATE;
    HTRY(hipSetDevice(e->device));
    TRY(ensure_host_headers(e));
    std::string d;
    TRY(commits_from_points(e, cm, d));
    return put_bytes(d, out, size);
}

// -------------------------------------------------------------- generators --
extern "C" int mpx_trace_generate(const mpx_gen_params *p, uint8_t **out, uint64_t *size)
{
    if (!p || !out || !size) return MPX_E_INVAL;
    std::string t;
    int rc;
    try {                                            // (no C++ exception crosses the C ABI)
        if (p->kind == MPX_GEN_CLEAN) rc = gen_clean(*p, t);
        else if (p->kind == MPX_GEN_FAULTY) rc = gen_faulty(*p, t);
        else if (p->kind == MPX_GEN_MEMBER) rc = gen_member(*p, t);
        else rc = MPX_E_INVAL;
    } catch (const std::bad_alloc &) {
        return MPX_E_NOMEM;
    } catch (const std::length_error &) {
        return MPX_E_NOMEM;
    }
    if (rc) return rc;
    *out = (uint8_t *)std::malloc(t.size());
    if (!*out) return MPX_E_NOMEM;
    std::memcpy(*out, t.data(), t.size());
    *size = t.size();
    return MPX_OK;
}

extern "C" int mpx_load_clean_device(mpx_engine *e, const mpx_gen_params *p)
{
    if (!e || !p) return MPX_E_INVAL;
    if (p->kind != MPX_GEN_CLEAN || p->num_nodes != e->cfg.num_nodes || e->cfg.semantics != MPX_SEM_MULTI) return MPX_E_INVAL;
    const uint64_t B = p->batch ? p->batch : BS;               // instances per batch
    if (B > 0xFFFF || (e->cfg.shard_begin & (BS - 1)) || e->NB == 0) return MPX_E_INVAL;
    if (e->cfg.shard_end > p->num_instances) return MPX_E_INVAL;
    HTRY(hipSetDevice(e->device));
    const uint64_t t0 = now_ns();
    const uint32_t N = e->cfg.num_nodes;
    const uint64_t sb = e->cfg.shard_begin, se = e->cfg.shard_end, L = se - sb, NB = e->NB;
    const uint64_t k0 = sb / B, K = (se - 1) / B - k0 + 1;      // kept batches: those meeting the shard
    e->whole = sb == 0 && se == p->num_instances;
    const uint64_t G0 = 2 + N + K * (3 + 2ull * N), G1 = 1 + 2 * K;
    const uint64_t G = G0 + (uint64_t)(N - 1) * G1;
    const uint64_t E = L;                                       // one shared run per batch
    // per bucket: the batches meeting it (one ACCEPT and one COMMIT run per
    // node each, one chosen-log run) -> the fragment CSR offsets
    std::vector<uint64_t> cf_off(NB + 1, 0), f_off(N * NB + 1, 0);
    uint64_t max_pair = 0, max_cb = 0;
    for (uint64_t b = 0; b < NB; ++b) {
        const uint64_t lo = sb + (b << BSH), hi = std::min(lo + BS, se);
        const uint64_t nb = (hi - 1) / B - lo / B + 1;
        cf_off[b + 1] = cf_off[b] + nb;
        for (uint32_t n = 0; n < N; ++n) f_off[b * N + n] = 2 * (N * cf_off[b] + n * nb);
        max_pair = std::max(max_pair, 2 * nb);
        max_cb = std::max(max_cb, nb);
    }
    f_off[N * NB] = 2ull * N * cf_off[NB];
    if (G >= NONE32 || E > MAX_ENTRIES || f_off[N * NB] > MAX_FRAGS || max_pair > MAX_PAIR_FRAGS) return MPX_E_RANGE;
    const uint64_t ballot = 1ull << 16;                         // (1 << 16) | node 0
    // host-side small tables
    HostTrace &h = e->ht;
    h = HostTrace();
    h.N = N; h.NB = e->NB; h.shard_begin = sb; h.shard_len = L;
    h.node_off.resize(N + 1);
    for (uint32_t n = 0; n <= N; ++n) h.node_off[n] = n == 0 ? 0 : G0 + (uint64_t)(n - 1) * G1;
    // header-scan stream: per node its PREPARE and K ACCEPTs (gen_device.hip k_gen_scan)
    h.node_chunk_off.assign(N + 1, 0);
    h.scan_chunk = scan_chunk_for((uint64_t)N * (K + 1));
    for (uint32_t n = 0; n < N; ++n) {
        h.node_chunk_off[n] = (uint32_t)h.chunk_node.size();
        const uint64_t a = (uint64_t)n * (K + 1), b = a + K + 1;
        for (uint64_t g = a; g < b; g += h.scan_chunk) {
            h.chunk_node.push_back(n);
            h.chunk_beg.push_back(g);
            h.chunk_end.push_back(std::min<uint64_t>(g + h.scan_chunk, b));
        }
    }
    h.node_chunk_off[N] = (uint32_t)h.chunk_node.size();
    h.g_a.assign(N, 0); h.g_b.assign(N, ~0ull);
    // snapshot events: node 0's PREPARE precedes every fragment and its promise
    // replies carry no entries, so no pair has events (ingest.cpp's per-pair lists)
    h.pl_off.assign(N + 1, 0);
    h.pl_msg.push_back(0);
    for (uint32_t k = 0; k < N; ++k) h.pl_msg.push_back(2 + k);
    h.pl_off[1] = N + 1;
    for (uint32_t n = 1; n < N; ++n) h.pl_off[n + 1] = h.pl_off[n];
    hipStream_t s = e->stream;
    TRY(e->m_type.alloc(G)); TRY(e->m_src.alloc(4 * G)); TRY(e->m_ballot.alloc(8 * G)); TRY(e->m_aux.alloc(8 * G));
    TRY(e->m_ent.alloc(8 * G)); TRY(e->m_cnt.alloc(4 * G)); TRY(e->m_node.alloc(4 * G));
    TRY(e->m_flags.alloc(G + 8)); TRY(e->m_maxseen.alloc(8 * G));
    HTRY(hipMemsetAsync(e->m_flags.p, 0, G, s));          // no static flags: every source is a node
    TRY(e->sc_type.alloc((uint64_t)N * (K + 1))); TRY(e->sc_key.alloc(8 * (uint64_t)N * (K + 1)));
    TRY(e->sc_idx.alloc(4 * (uint64_t)N * (K + 1)));
    TRY(e->b_rbal.alloc(8 * (uint64_t)N * K + 8)); TRY(e->b_rsrc.alloc(4 * (uint64_t)N * K + 4));
    TRY(e->b_bal.alloc(8 * K + 8));
    TRY(upload(e->node_off, h.node_off, s));

    TRY(e->ev_off.alloc(8 * ((uint64_t)N * e->NB + 1)));
    HTRY(hipMemsetAsync(e->ev_off.p, 0, e->ev_off.bytes, s));
    TRY(e->ev_msg.alloc(8)); TRY(e->ev_aux.alloc(8));
    TRY(upload(e->chunk_node, h.chunk_node, s)); TRY(upload(e->chunk_beg, h.chunk_beg, s));
    TRY(upload(e->chunk_end, h.chunk_end, s)); TRY(upload(e->node_chunk_off, h.node_chunk_off, s));
    TRY(e->chunk_agg.alloc(std::max<size_t>(16 * h.chunk_node.size(), 16)));
    TRY(e->chunk_carry.alloc(std::max<size_t>(16 * h.chunk_node.size(), 16)));
    TRY(e->e_val.alloc(std::max<uint64_t>(8 * E, 8)));
    TRY(e->e_slot.alloc(8)); TRY(e->r_pid.alloc(8)); TRY(e->r_val.alloc(8)); TRY(e->r_slot.alloc(8));
    TRY(upload(e->g_a, h.g_a, s)); TRY(upload(e->g_b, h.g_b, s));
    TRY(upload(e->f_off, f_off, s)); TRY(e->frags.alloc(sizeof(Frag) * f_off[N * NB] + 16));
    TRY(upload(e->pl_off, h.pl_off, s)); TRY(upload(e->pl_msg, h.pl_msg, s));
    TRY(e->b_msg.alloc(4 * K + 4)); TRY(e->b_pstart.alloc(4 * K + 4)); TRY(e->b_rep_off.alloc(8 * (K + 1)));
    TRY(e->b_rep.alloc(4 * (uint64_t)N * K + 4)); TRY(e->b_chosen.alloc(4 * K + 4));
    TRY(upload(e->cf_off, cf_off, s)); TRY(e->cfrags.alloc(sizeof(Frag) * cf_off[NB] + 16));
    // pairs the lean kernels cannot take (ingest.cpp's predicate: every run is
    // dense, no snapshot events, so only the node count and run count decide)
    // (lean: mpx_internal.hpp plan_shape_ok — a pair's batch runs are disjoint and
    // in order, so its run count and a whole bucket decide)
    std::vector<uint64_t> gd;
    std::vector<uint8_t> pair_gp(N * NB, 0);
    for (uint64_t q = 0; q < N * NB; ++q)
        if (f_off[q + 1] > f_off[q] && (N > FAST_MAX_NODES || f_off[q + 1] - f_off[q] > PLAN_FRAGS || (q / N + 1) * BS > L)) {
            const uint64_t w[GP_WORDS] = {f_off[q], f_off[q + 1], 0, 0, q, 0, 0, 0};
            gd.insert(gd.end(), w, w + GP_WORDS);
            pair_gp[q] = GP_ROUNDS;                     // the full k_apply's host range (num_gp_snap = 0)
        }
    if (gd.empty()) TRY(e->gp_list.alloc(8));
    else TRY(upload(e->gp_list, gd, s));
    pair_gp.resize(pair_gp.size() + 8, 0);             // dword slack (k_plan_store8)
    TRY(upload(e->pair_gp, pair_gp, s));
    if (launch_gen_clean(s, N, K, k0, sb, se, G0, G1, ballot, B, e->NB,
                         e->m_type.as<uint8_t>(), e->m_src.as<uint32_t>(), e->m_ballot.as<uint64_t>(),
                         e->m_aux.as<uint64_t>(), e->m_ent.as<uint64_t>(), e->m_cnt.as<uint32_t>(),
                         e->m_node.as<uint32_t>(), e->e_val.as<uint64_t>(), e->frags.as<Frag>(),
                         e->f_off.as<uint64_t>(), e->b_msg.as<uint32_t>(), e->b_pstart.as<uint32_t>(),
                         e->b_rep_off.as<uint64_t>(), e->b_rep.as<uint32_t>(), e->cf_off.as<uint64_t>(),
                         e->cfrags.as<Frag>(), e->sc_type.as<uint8_t>(), e->sc_key.as<uint64_t>(),
                         e->sc_idx.as<uint32_t>(), e->b_rbal.as<uint64_t>(), e->b_rsrc.as<uint32_t>(),
                         e->b_bal.as<uint64_t>()) != 0)
        return MPX_E_HIP;
    HTRY(hipStreamSynchronize(s));
    e->num_msgs = G;
    DevView &v = e->view;
    v.m_type = e->m_type.as<uint8_t>(); v.m_src = e->m_src.as<uint32_t>();
    v.m_ballot = e->m_ballot.as<uint64_t>(); v.m_aux = e->m_aux.as<uint64_t>();
    v.m_ent = e->m_ent.as<uint64_t>(); v.m_cnt = e->m_cnt.as<uint32_t>();
    v.m_node = e->m_node.as<uint32_t>(); v.node_off = e->node_off.as<uint64_t>();
    v.pair_gp = e->pair_gp.as<uint8_t>();
    v.m_flags = e->m_flags.as<uint8_t>(); v.m_maxseen = e->m_maxseen.as<uint64_t>();
    v.m_gate = e->m_gate.as<uint32_t>(); v.e_pid = e->e_pid.as<uint64_t>();
    v.ep_amask = e->ep_amask.as<uint64_t>(); v.num_epochs = (uint32_t)e->epochs.size();
    v.ep_pmask = e->ep_pmask.as<uint64_t>(); v.ep_ver = e->ep_ver.as<uint32_t>();
    v.m_ver = e->m_ver.as<uint32_t>(); v.ee_off = e->ee_off.as<uint64_t>(); v.ee_msg = e->ee_msg.as<uint32_t>();
    v.ee_state = e->ee_state.as<uint32_t>(); v.sc_ver = e->sc_ver.as<uint32_t>(); v.sc_off = e->sc_off.as<uint64_t>();
    v.num_sc = h.sc_type.size();
    v.num_chunks = (uint32_t)h.chunk_node.size();
    v.chunk_node = e->chunk_node.as<uint32_t>(); v.chunk_beg = e->chunk_beg.as<uint64_t>();
    v.chunk_end = e->chunk_end.as<uint64_t>(); v.node_chunk_off = e->node_chunk_off.as<uint32_t>();
    v.chunk_agg = e->chunk_agg.as<uint64_t>(); v.chunk_carry = e->chunk_carry.as<uint64_t>();
    v.e_val = e->e_val.as<uint64_t>(); v.e_slot = e->e_slot.as<uint8_t>();
    v.r_pid = e->r_pid.as<uint64_t>(); v.r_val = e->r_val.as<uint64_t>(); v.r_slot = e->r_slot.as<uint8_t>();
    v.g_a = e->g_a.as<uint64_t>(); v.g_b = e->g_b.as<uint64_t>();
    v.f_off = e->f_off.as<uint64_t>(); v.frags = e->frags.as<Frag>();
    // (no promise-reply runs, so no proposal id is used — but the promise-round walk, k_apply
    // AM_FULL, loads f_pid beside every descriptor of the pairs it takes: the work-list pairs
    // here, a partial last bucket or more than FAST_MAX_NODES nodes, need it sized like frags)
    TRY(e->f_pid.alloc(gd.empty() ? 8 : 8 * (f_off[N * NB] + 1)));
    v.f_pid = e->f_pid.as<uint64_t>();
    e->num_frags = f_off[N * NB];
    v.num_gp = gd.size() / GP_WORDS; v.gp_list = e->gp_list.as<uint64_t>(); v.num_gp_simple = 0; v.num_gp_snap = 0;
    v.ev_off = e->ev_off.as<uint64_t>(); v.ev_msg = e->ev_msg.as<uint32_t>(); v.ev_aux = e->ev_aux.as<uint64_t>();
    v.pl_off = e->pl_off.as<uint64_t>(); v.pl_msg = e->pl_msg.as<uint32_t>();
    v.num_batches = (uint32_t)K;
    v.b_msg = e->b_msg.as<uint32_t>(); v.b_pstart = e->b_pstart.as<uint32_t>();
    v.b_rep_off = e->b_rep_off.as<uint64_t>(); v.b_rep = e->b_rep.as<uint32_t>();
    v.b_rbal = e->b_rbal.as<uint64_t>(); v.b_rsrc = e->b_rsrc.as<uint32_t>(); v.b_bal = e->b_bal.as<uint64_t>();
    v.sc_type = e->sc_type.as<uint8_t>(); v.sc_key = e->sc_key.as<uint64_t>(); v.sc_idx = e->sc_idx.as<uint32_t>();
    v.b_chosen = e->b_chosen.as<uint32_t>();
    v.cf_off = e->cf_off.as<uint64_t>(); v.cfrags = e->cfrags.as<Frag>();
    v.slot_w = max_pair <= MAX_PAIR_FRAGS_1 ? 1 : 2;
    // batches tile the instances: a bucket's chosen-log runs are disjoint and dense, so at most
    // four of them over a whole bucket pass plan_chosen's static test (no k_chosen walk)
    v.chosen_static = max_cb <= 4 && L % BS == 0 ? 1 : 0;
    v.any_vchk = 0;                                  // (a clean trace: no re-commit through another entry)
    TRY(finish_view(e));
    for (auto &ns : e->nodes) ns.clear();
    e->vt.clear();
    e->vt.synthetic_clean = true;
    e->device_trace = true;
    e->dirty = false;
    e->stats.ingest_ns = now_ns() - t0;
    return MPX_OK;
}

// Host copies of the device-generated headers, for drain / dump (small traces).
static int ensure_host_headers(mpx_engine *e)
{
    if (!e->device_trace || e->ht.m_type.size() == e->num_msgs) return MPX_OK;
    HostTrace &h = e->ht;
    const size_t G = e->num_msgs;
    TRY(d2h(h.m_type, e->m_type, G)); TRY(d2h(h.m_src, e->m_src, G));
    TRY(d2h(h.m_ballot, e->m_ballot, G)); TRY(d2h(h.m_aux, e->m_aux, G));
    TRY(d2h(h.m_node, e->m_node, G));
    TRY(d2h(h.b_msg, e->b_msg, e->view.num_batches));
    return MPX_OK;
}

// ------------------------------------------------------------------- RCCL --
extern "C" int mpx_comm_unique_id(uint8_t out[MPX_UID_BYTES])
{
    static_assert(sizeof(ncclUniqueId) <= MPX_UID_BYTES, "uid size");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return MPX_E_COMM;
    std::memset(out, 0, MPX_UID_BYTES);
    std::memcpy(out, &id, sizeof id);
    return MPX_OK;
}

extern "C" int mpx_comm_init(mpx_engine *e, const uint8_t uid[MPX_UID_BYTES], int rank, int nranks)
{
    if (!e || !uid || rank < 0 || rank >= nranks) return MPX_E_INVAL;
    HTRY(hipSetDevice(e->device));
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof id);
    if (ncclCommInitRank(&e->comm, nranks, id, rank) != ncclSuccess) return MPX_E_COMM;
    e->rank = rank;
    e->nranks = nranks;
    TRY(e->gather_buf.alloc(2 * 64ull * 8 * nranks));
    HTRY(hipStreamCreateWithFlags(&e->comm_stream, hipStreamNonBlocking));
    for (int k = 0; k < 2; ++k) {
        HTRY(hipEventCreateWithFlags(&e->sum_ev[k], hipEventDisableTiming));
        HTRY(hipEventCreateWithFlags(&e->ag_ev[k], hipEventDisableTiming));
    }
    return MPX_OK;
}

// RCCL calls on the engine stream come after every summary all-gather already issued (one
// order of collectives on every rank)
static int comm_fence(mpx_engine *e)
{
    for (int k = 0; k < 2; ++k)
        if (e->ag_pending[k]) HTRY(hipStreamWaitEvent(e->stream, e->ag_ev[k], 0));
    return MPX_OK;
}

extern "C" int mpx_allgather_summary(mpx_engine *e, uint64_t *out)
{
    if (!e || !out) return MPX_E_INVAL;
    if (!e->summary.p) return MPX_E_STATE;
    HTRY(hipSetDevice(e->device));
    if (e->comm) {
        // gathered by the last queued run/step
        TRY(comm_fence(e));
        HTRY(hipMemcpyAsync(out, e->gather_buf.as<uint64_t>() + 64ull * e->nranks * e->sum_idx, 64ull * 8 * e->nranks,
                            hipMemcpyDeviceToHost, e->stream));
    } else {
        HTRY(hipMemcpyAsync(out, e->summary.as<uint64_t>() + 64 * e->sum_idx, 64 * 8, hipMemcpyDeviceToHost, e->stream));
    }
    HTRY(hipStreamSynchronize(e->stream));
    return MPX_OK;
}

extern "C" int mpx_comm_allreduce_max(mpx_engine *e, uint64_t *vals, uint64_t n)
{
    if (!e || (n && !vals)) return MPX_E_INVAL;
    if (!e->comm || e->nranks <= 1 || !n) return MPX_OK;
    HTRY(hipSetDevice(e->device));
    TRY(comm_fence(e));
    TRY(e->comm_buf.alloc(8 * n));
    HTRY(hipMemcpyAsync(e->comm_buf.p, vals, 8 * n, hipMemcpyHostToDevice, e->stream));
    if (ncclAllReduce(e->comm_buf.p, e->comm_buf.p, n, ncclUint64, ncclMax, e->comm, e->stream) != ncclSuccess)
        return MPX_E_COMM;
    HTRY(hipMemcpyAsync(vals, e->comm_buf.p, 8 * n, hipMemcpyDeviceToHost, e->stream));
    HTRY(hipStreamSynchronize(e->stream));
    return MPX_OK;
}

extern "C" int mpx_comm_allgather_bytes(mpx_engine *e, const uint8_t *mine, uint64_t len, uint8_t **out, uint64_t *lens)
{
    if (!e || (len && !mine) || !out || !lens) return MPX_E_INVAL;
    const int R = e->comm ? e->nranks : 1;
    if (R <= 1) {
        *out = (uint8_t *)std::malloc(len ? len : 1);
        if (!*out) return MPX_E_NOMEM;
        if (len) std::memcpy(*out, mine, len);
        lens[0] = len;
        return MPX_OK;
    }
    HTRY(hipSetDevice(e->device));
    TRY(comm_fence(e));
    // the lengths, then every string padded to the longest (one all-gather each)
    TRY(e->comm_buf.alloc(8ull * (R + 1)));
    uint64_t *dl = e->comm_buf.as<uint64_t>();
    HTRY(hipMemcpyAsync(dl, &len, 8, hipMemcpyHostToDevice, e->stream));
    if (ncclAllGather(dl, dl + 1, 1, ncclUint64, e->comm, e->stream) != ncclSuccess) return MPX_E_COMM;
    HTRY(hipMemcpyAsync(lens, dl + 1, 8ull * R, hipMemcpyDeviceToHost, e->stream));
    HTRY(hipStreamSynchronize(e->stream));
    uint64_t mx = 0, tot = 0;
    for (int r = 0; r < R; ++r) { mx = std::max(mx, lens[r]); tot += lens[r]; }
    const uint64_t w = (mx + 7) & ~7ull;
    if (!w) { *out = (uint8_t *)std::malloc(1); return *out ? MPX_OK : MPX_E_NOMEM; }
    TRY(e->comm_buf2.alloc(w * (R + 1)));
    uint8_t *db = e->comm_buf2.as<uint8_t>();
    HTRY(hipMemsetAsync(db, 0, w, e->stream));
    if (len) HTRY(hipMemcpyAsync(db, mine, len, hipMemcpyHostToDevice, e->stream));
    if (ncclAllGather(db, db + w, w, ncclUint8, e->comm, e->stream) != ncclSuccess) return MPX_E_COMM;
    std::vector<uint8_t> all(w * R);
    HTRY(hipMemcpyAsync(all.data(), db + w, w * R, hipMemcpyDeviceToHost, e->stream));
    HTRY(hipStreamSynchronize(e->stream));
    *out = (uint8_t *)std::malloc(tot ? tot : 1);
    if (!*out) return MPX_E_NOMEM;
    uint64_t at = 0;
    for (int r = 0; r < R; ++r) { std::memcpy(*out + at, all.data() + w * r, lens[r]); at += lens[r]; }
    return MPX_OK;
}

// Decisions with client values over instance shards (include/mpx.h): each shard's part
// holds the bookkeeping's events with its own instances' entries (MPXE); the combine merges
// the parts per node by record (headers are replicated, so every shard lists the same
// Propose / StartPrepare / quorum records; a COMMIT appears where it has entries) and runs
// the proposer's walk once over the union.
extern "C" int mpx_proposal_part(mpx_engine *e, uint8_t **out, uint64_t *size)
{
    if (!e || !out || !size) return MPX_E_INVAL;
    if (e->incremental || e->device_trace) return MPX_E_STATE;
    const bool member = e->cfg.semantics == MPX_SEM_MEMBER;
    Results r;
    TRY(fetch_results(e, r));
    PEvents ev;
    if (member) TRY(member_events(e, r, ev));
    else proposer_events(e, r, ev);
    std::string d;
    d.append("MPXE", 4);
    app<uint32_t>(d, member ? 2 : 1); app<uint32_t>(d, e->cfg.num_nodes);
    app<uint64_t>(d, e->cfg.shard_begin); app<uint64_t>(d, e->cfg.shard_end);
    if (member) {                                       // the epoch table the walk reads
        app<uint32_t>(d, (uint32_t)e->epochs.size());
        for (auto &x : e->epochs) { app<uint64_t>(d, x.acceptor_mask); app<uint64_t>(d, x.proposer_mask); }
    }
    for (auto &l : ev) {
        app<uint64_t>(d, l.size());
        for (auto &x : l) {
            app<uint64_t>(d, x.seq); app<uint32_t>(d, x.type); app<uint32_t>(d, (uint32_t)x.ents.size());
            if (member) app<uint64_t>(d, x.aux);
            for (auto &en : x.ents) { app<uint64_t>(d, en.first); app<uint64_t>(d, en.second); }
        }
    }
    return put_bytes(d, out, size);
}

extern "C" int mpx_proposal_combine(const uint8_t *const *parts, const uint64_t *sizes, uint32_t nparts,
                                    uint8_t **out, uint64_t *size)
{
    if (!parts || !sizes || !nparts || !out || !size) return MPX_E_INVAL;
    uint32_t N = 0, ver = 0;
    uint64_t prev_end = 0;
    std::vector<PEvents> ps(nparts);
    std::vector<mpx_epoch> ep;
    for (uint32_t i = 0; i < nparts; ++i) {
        const uint8_t *p = parts[i];
        const uint64_t n = sizes[i];
        if (!p || n < 28 || std::memcmp(p, "MPXE", 4)) return MPX_E_INVAL;
        const uint32_t vi = rd32(p + 4), Ni = rd32(p + 8);       // 1 multi, 2 member
        const uint64_t sb = rd64(p + 12), se = rd64(p + 20);
        if ((vi != 1 && vi != 2) || (i && vi != ver)) return MPX_E_INVAL;
        if (!Ni || Ni > MPX_MAX_NODES || (i && Ni != N) || sb != prev_end || se < sb) return MPX_E_INVAL;   // shard order
        N = Ni;
        ver = vi;
        prev_end = se;
        uint64_t pos = 28;
        if (ver == 2) {                                  // member: the epoch table, equal on every part
            if (pos + 4 > n) return MPX_E_INVAL;
            const uint32_t E = rd32(p + pos);
            pos += 4;
            if (!E || E > (n - pos) / 16) return MPX_E_INVAL;
            std::vector<mpx_epoch> epi(E);
            for (uint32_t k = 0; k < E; ++k, pos += 16) {
                epi[k].acceptor_mask = rd64(p + pos);
                epi[k].proposer_mask = rd64(p + pos + 8);
            }
            if (i && (epi.size() != ep.size() ||
                      !std::equal(epi.begin(), epi.end(), ep.begin(), [](const mpx_epoch &a, const mpx_epoch &b) {
                          return a.acceptor_mask == b.acceptor_mask && a.proposer_mask == b.proposer_mask; })))
                return MPX_E_INVAL;
            ep.swap(epi);
        }
        const uint64_t hdr = ver == 2 ? 24 : 16;
        ps[i].assign(N, {});
        for (uint32_t k = 0; k < N; ++k) {
            if (pos + 8 > n) return MPX_E_INVAL;
            const uint64_t c = rd64(p + pos); pos += 8;
            for (uint64_t j = 0; j < c; ++j) {
                if (pos + hdr > n) return MPX_E_INVAL;
                PEv x{rd64(p + pos), rd32(p + pos + 8), {}};
                const uint32_t m = rd32(p + pos + 12);
                if (ver == 2) x.aux = rd64(p + pos + 16);
                pos += hdr;
                if (m > (n - pos) / 16) return MPX_E_INVAL;
                for (uint32_t q = 0; q < m; ++q, pos += 16) {
                    const uint64_t iid = rd64(p + pos);
                    if (iid < sb || iid >= se) return MPX_E_INVAL;
                    x.ents.push_back({iid, rd64(p + pos + 8)});
                }
                if (!ps[i][k].empty() && x.seq <= ps[i][k].back().seq) return MPX_E_INVAL;   // stream order
                ps[i][k].push_back(std::move(x));
            }
        }
        if (pos != n) return MPX_E_INVAL;
    }
    PEvents all(N);
    for (uint32_t k = 0; k < N; ++k) {
        std::map<uint64_t, PEv> m;                         // record -> the event, entries in shard order
        for (uint32_t i = 0; i < nparts; ++i)
            for (auto &x : ps[i][k]) {
                auto it = m.find(x.seq);
                if (it == m.end()) { m.emplace(x.seq, x); continue; }
                if (it->second.type != x.type || it->second.aux != x.aux) return MPX_E_INVAL;
                it->second.ents.insert(it->second.ents.end(), x.ents.begin(), x.ents.end());
            }
        for (auto &y : m) all[k].push_back(std::move(y.second));
    }
    std::string d;
    if (ver == 2) TRY(member_sim(all, ep, d));
    else proposer_sim(all, d);
    return put_bytes(d, out, size);
}

extern "C" int mpx_read_decisions_sharded(mpx_engine *e, uint8_t **out, uint64_t *size)
{
    if (!e || !out || !size) return MPX_E_INVAL;
    const int R = e->comm ? e->nranks : 1;
    if (R <= 1 && e->cfg.shard_begin == 0) return mpx_read_decisions(e, out, size);
    if (e->cfg.semantics == MPX_SEM_MEMBER || has_proposals(e->ht)) {
        // client values (or member semantics): the proposer's walk over every shard's events
        // (P_PROPOSE is a header: every rank sees it, so every rank takes this branch)
        uint8_t *part = nullptr;
        uint64_t plen = 0;
        TRY(mpx_proposal_part(e, &part, &plen));
        std::vector<uint64_t> lens(R);
        uint8_t *all = nullptr;
        int rc = mpx_comm_allgather_bytes(e, part, plen, &all, lens.data());
        std::free(part);
        if (rc) return rc;
        std::vector<const uint8_t *> ps(R);
        uint64_t at = 0;
        for (int r = 0; r < R; ++r) { ps[r] = all + at; at += lens[r]; }
        rc = mpx_proposal_combine(ps.data(), lens.data(), (uint32_t)R, out, size);
        std::free(all);
        return rc;
    }
    uint64_t cnt = 0;
    TRY(mpx_decisions_bounds(e, nullptr, 0, &cnt));
    std::vector<uint64_t> b(cnt + 2);
    TRY(mpx_decisions_bounds(e, b.data(), cnt, &cnt));
    // the quorum count must agree on every rank: MAX of (count, ~count) gives max and ~min
    b[cnt] = cnt; b[cnt + 1] = ~cnt;
    TRY(mpx_comm_allreduce_max(e, b.data(), cnt + 2));
    if (b[cnt] != cnt || ~b[cnt + 1] != cnt) return MPX_E_INVAL;
    uint8_t *part = nullptr;
    uint64_t plen = 0;
    TRY(mpx_read_decisions_part(e, b.data(), cnt, &part, &plen));
    std::vector<uint64_t> lens(R);
    uint8_t *all = nullptr;
    int rc = mpx_comm_allgather_bytes(e, part, plen, &all, lens.data());
    std::free(part);
    if (rc) return rc;
    std::vector<const uint8_t *> ps(R);
    uint64_t at = 0;
    for (int r = 0; r < R; ++r) { ps[r] = all + at; at += lens[r]; }
    rc = mpx_decisions_combine(ps.data(), lens.data(), (uint32_t)R, out, size);
    std::free(all);
    return rc;
}

// Sharded commit reliability over the engine's own communicator: every rank's
// creation points gathered and merged (mpx_commit_points_combine), the rank whose
// shard starts at instance 0 (it keeps every COMMIT_REPLY) runs k_commits over the
// union, and its MPXC is gathered to every rank.  One rank: mpx_read_commits.
extern "C" int mpx_read_commits_sharded(mpx_engine *e, uint8_t **out, uint64_t *size)
{
    if (!e || !out || !size) return MPX_E_INVAL;
    const int R = e->comm ? e->nranks : 1;
    if (R <= 1) return mpx_read_commits(e, out, size);
    uint8_t *pts = nullptr;
    uint64_t plen = 0;
    TRY(mpx_commit_points(e, &pts, &plen));
    std::vector<uint64_t> lens(R);
    uint8_t *all = nullptr;
    int rc = mpx_comm_allgather_bytes(e, pts, plen, &all, lens.data());
    std::free(pts);
    if (rc) return rc;
    std::vector<const uint8_t *> ps(R);
    uint64_t at = 0;
    for (int r = 0; r < R; ++r) { ps[r] = all + at; at += lens[r]; }
    uint8_t *merged = nullptr;
    uint64_t mlen = 0;
    rc = mpx_commit_points_combine(ps.data(), lens.data(), (uint32_t)R, &merged, &mlen);
    std::free(all);
    if (rc) return rc;
    uint8_t *mine = nullptr;
    uint64_t mylen = 0;
    if (e->cfg.shard_begin == 0) rc = mpx_read_commits_at(e, merged, mlen, &mine, &mylen);
    std::free(merged);
    if (rc) return rc;
    rc = mpx_comm_allgather_bytes(e, mine, mylen, &all, lens.data());
    std::free(mine);
    if (rc) return rc;
    at = 0;
    int src = -1;
    for (int r = 0; r < R; ++r) {
        if (lens[r]) { if (src >= 0) { std::free(all); return MPX_E_INVAL; } src = r; }
        if (src < 0) at += lens[r];
    }
    if (src < 0) { std::free(all); return MPX_E_STATE; }            // no rank holds instance 0
    rc = put_bytes(std::string((const char *)all + at, lens[src]), out, size);
    std::free(all);
    return rc;
}
