/*
 * mpx_oracle.c — CPU restatement of the reference's acceptor / learner /
 * proposer-aggregation handlers.  TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity checker for the MI355X engine.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product path (multi-paxos_amd/) never links or calls it.
 *
 * Parity pin: every behaviour below is checked against the reference's own
 * handlers (multi/paxos.cpp compiled in place from /root/reference by
 * oracle/Makefile into oracle/_ref/libmpx_ref.so) on the committed golden
 * traces under tests/golden/ (tests/test_oracle.py), and against the
 * reference's UNITTEST codec vectors (multi/paxos.cpp:1753-1777).
 *
 * Input : an MPXT trace container (DESIGN.md §Trace container): per node the
 *         ordered receive stream, records are the reference's packed wire
 *         messages plus the engine-local proposer markers P_START / P_BATCH.
 * Output: an MPXR canonical result — the same bytes the
 *         engine's mpx_dump_result and the reference driver produce.
 *
 * Everything is sequential, one node after another, one record after another,
 * exactly the reference's processing order (PaxosImpl::Loop, paxos.cpp:1654).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <pthread.h>

typedef uint64_t u64;
typedef uint32_t u32;
typedef uint8_t u8;

/* ---- little-endian access (the reference memcpy's host structs; x86) ---- */
static u32 rd32(const u8 *p) { u32 v; memcpy(&v, p, 4); return v; }
static u64 rd64(const u8 *p) { u64 v; memcpy(&v, p, 8); return v; }

/* ---- growable byte buffer ------------------------------------------------ */
typedef struct { u8 *p; size_t n, cap; int oom; int ext; } buf_t;   /* ext: p is caller storage, not owned */
static void bput(buf_t *b, const void *src, size_t n)
{
    if (b->oom) return;
    if (b->n + n > b->cap) {
        size_t c = b->cap ? b->cap : 256;
        while (c < b->n + n) c *= 2;
        u8 *q = (u8 *)(b->ext ? malloc(c) : realloc(b->p, c));
        if (!q) { b->oom = 1; return; }
        if (b->ext && b->n) memcpy(q, b->p, b->n);
        b->p = q; b->cap = c; b->ext = 0;
    }
    memcpy(b->p + b->n, src, n);
    b->n += n;
}
static void bput32(buf_t *b, u32 v) { bput(b, &v, 4); }
static void bfree(buf_t *b) { if (!b->ext) free(b->p); }
static void bput64(buf_t *b, u64 v) { bput(b, &v, 8); }

/* ---- u64 -> (a,b) open-addressing map, linear probing, backward-shift delete */
typedef struct { u64 key, a, b; } ent_t;
typedef struct { ent_t *e; u8 *used; size_t cap, n; } map_t;

static size_t hslot(u64 k, size_t cap)
{
    k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33;
    return (size_t)(k & (cap - 1));
}
static int map_grow(map_t *m)
{
    size_t nc = m->cap ? m->cap * 2 : 64;
    ent_t *ne = (ent_t *)calloc(nc, sizeof(ent_t));
    u8 *nu = (u8 *)calloc(nc, 1);
    if (!ne || !nu) { free(ne); free(nu); return -1; }
    for (size_t i = 0; i < m->cap; ++i) if (m->used[i]) {
        size_t s = hslot(m->e[i].key, nc);
        while (nu[s]) s = (s + 1) & (nc - 1);
        nu[s] = 1; ne[s] = m->e[i];
    }
    free(m->e); free(m->used);
    m->e = ne; m->used = nu; m->cap = nc;
    return 0;
}
static ent_t *map_find(const map_t *m, u64 k)
{
    if (!m->cap) return NULL;
    size_t s = hslot(k, m->cap);
    while (m->used[s]) { if (m->e[s].key == k) return &m->e[s]; s = (s + 1) & (m->cap - 1); }
    return NULL;
}
static ent_t *map_put(map_t *m, u64 k, u64 a, u64 b)
{
    if ((m->n + 1) * 2 > m->cap && map_grow(m)) return NULL;
    size_t s = hslot(k, m->cap);
    while (m->used[s]) {
        if (m->e[s].key == k) { m->e[s].a = a; m->e[s].b = b; return &m->e[s]; }
        s = (s + 1) & (m->cap - 1);
    }
    m->used[s] = 1; m->e[s].key = k; m->e[s].a = a; m->e[s].b = b; m->n++;
    return &m->e[s];
}
static void map_del(map_t *m, u64 k)
{
    if (!m->cap) return;
    size_t s = hslot(k, m->cap);
    while (m->used[s] && m->e[s].key != k) s = (s + 1) & (m->cap - 1);
    if (!m->used[s]) return;
    m->used[s] = 0; m->n--;
    size_t j = s;
    for (;;) {
        j = (j + 1) & (m->cap - 1);
        if (!m->used[j]) break;
        size_t h = hslot(m->e[j].key, m->cap);
        /* can entry j move into hole s? (cyclic distance test) */
        if (((j - h) & (m->cap - 1)) >= ((j - s) & (m->cap - 1))) {
            m->e[s] = m->e[j]; m->used[s] = 1; m->used[j] = 0; s = j;
        }
    }
}
static void map_clear(map_t *m) { if (m->cap) memset(m->used, 0, m->cap); m->n = 0; }
static void map_free(map_t *m);
/* per-message scratch map: after a large message (a catch-up LEARN carries
 * every learned Value) release it rather than clear its whole table per message */
static void map_reset(map_t *m) { if (m->cap > 4096) map_free(m); else map_clear(m); }
static void map_free(map_t *m) { free(m->e); free(m->used); memset(m, 0, sizeof *m); }

static int cmp_ent(const void *x, const void *y)
{
    u64 a = ((const ent_t *)x)->key, b = ((const ent_t *)y)->key;
    return a < b ? -1 : a > b;
}
/* entries of a map, sorted by key (std::map iteration order) */
static ent_t *map_sorted(const map_t *m, size_t *n)
{
    ent_t *v = (ent_t *)malloc((m->n ? m->n : 1) * sizeof(ent_t));
    size_t k = 0;
    if (!v) { *n = 0; return NULL; }
    for (size_t i = 0; i < m->cap; ++i) if (m->used[i]) v[k++] = m->e[i];
    qsort(v, k, sizeof(ent_t), cmp_ent);
    *n = k;
    return v;
}

/* ---- Values ---------------------------------------------------------------
 * A Value is (u32 proposer, u64 value_id, bool noop, membership | payload),
 * encoded as in FillValue / ExtractValue (multi/paxos.cpp:556-644).  Its
 * handle is proposer<<48 | noop<<47 | value_id (include/mpx.h); the canonical
 * re-encoded bytes are interned per handle so PREPARE_REPLY can be rebuilt the
 * way FillAcceptedValues does (multi/paxos.cpp:657-669). */
typedef struct { u64 handle; size_t off; u32 len; u32 exec_off; u32 exec_len; } valrec_t;
typedef struct { map_t idx; valrec_t *v; size_t n, cap; buf_t bytes; } vtab_t;

enum { OK = 0, E_INVAL = -1, E_DECODE = -4, E_RANGE = -5, E_VALUE = -9, E_NOMEM = -2 };

/* AvailableInstanceIDs (multi/paxos.cpp:253-318): disjoint ranges [a, b), ascending,
 * [0, 2^64-1) at first — the proposer's unproposed instance ids (client proposals) */
typedef struct { u64 *a, *b; size_t n, cap; } rng_t;
static int rng_init(rng_t *r)
{
    r->n = 0;
    if (!r->cap) {
        r->cap = 16;
        r->a = (u64 *)malloc(8 * r->cap); r->b = (u64 *)malloc(8 * r->cap);
        if (!r->a || !r->b) return E_NOMEM;
    }
    r->a[0] = 0; r->b[0] = ~0ull; r->n = 1;
    return OK;
}
static size_t rng_find(const rng_t *r, u64 id)        /* index of the range holding id, or n */
{
    size_t lo = 0, hi = r->n;
    while (lo < hi) { size_t mid = (lo + hi) / 2; if (r->b[mid] <= id) lo = mid + 1; else hi = mid; }
    return lo < r->n && r->a[lo] <= id ? lo : r->n;
}
static int rng_contains(const rng_t *r, u64 id) { return rng_find(r, id) < r->n; }
static int rng_remove(rng_t *r, u64 id)
{
    size_t i = rng_find(r, id);
    if (i == r->n) return OK;
    u64 a = r->a[i], b = r->b[i];
    if (a != id && id + 1 != b) {                        /* split: one more range */
        if (r->n == r->cap) {
            size_t cc = r->cap * 2;
            u64 *na = (u64 *)realloc(r->a, 8 * cc), *nb = (u64 *)realloc(r->b, 8 * cc);
            if (!na || !nb) return E_NOMEM;
            r->a = na; r->b = nb; r->cap = cc;
        }
        memmove(r->a + i + 2, r->a + i + 1, 8 * (r->n - i - 1));
        memmove(r->b + i + 2, r->b + i + 1, 8 * (r->n - i - 1));
        r->b[i] = id; r->a[i + 1] = id + 1; r->b[i + 1] = b; r->n++;
    } else if (a != id) {
        r->b[i] = id;
    } else if (id + 1 != b) {
        r->a[i] = id + 1;
    } else {
        memmove(r->a + i, r->a + i + 1, 8 * (r->n - i - 1));
        memmove(r->b + i, r->b + i + 1, 8 * (r->n - i - 1));
        r->n--;
    }
    return OK;
}
static u64 rng_next(rng_t *r) { u64 a = r->a[0]; rng_remove(r, a); return a; }
static void rng_remove_below(rng_t *r, u64 x)             /* [0, 2^64-1) -> [x, 2^64-1) */
{
    if (r->n == 1 && r->a[0] == 0) r->a[0] = x;
}

/* Parse one Value at p (avail bytes).  Returns bytes used (>0) or <0. */
/* Parse one Value at p (avail bytes).  Returns bytes used (>0) or <0.
 * t == NULL: length and handle only (an entry outside the oracle's shard). */
static long parse_value(vtab_t *t, const u8 *p, size_t avail, u64 *handle)
{
    if (avail < 13) return E_DECODE;
    u32 proposer = rd32(p);
    u64 value_id = rd64(p + 4);
    int noop = p[12] != 0;
    size_t used;
    u8 sbuf[256];
    buf_t enc = {sbuf, 0, sizeof sbuf, 0, 1};
    size_t exec_from = 0, exec_len = 0;       /* what Execute() would receive */
    if (proposer >= (1u << 14) || value_id >= (1ull << 47)) return E_RANGE;
    bput32(&enc, proposer); bput64(&enc, value_id);
    u8 bnoop = (u8)noop; bput(&enc, &bnoop, 1);
    if (noop) {
        used = 13;
    } else {
        if (avail < 14) { bfree(&enc); return E_DECODE; }
        u8 member = p[13] != 0;
        bput(&enc, &member, 1);
        if (member) {
            if (avail < 19) { bfree(&enc); return E_DECODE; }
            u32 id = rd32(p + 14);
            u8 add = p[18] != 0;
            bput32(&enc, id); bput(&enc, &add, 1);
            if (add) {
                if (avail < 23) { bfree(&enc); return E_DECODE; }
                u32 iplen = rd32(p + 19);
                if (avail < 25 + (size_t)iplen) { bfree(&enc); return E_DECODE; }
                bput32(&enc, iplen); bput(&enc, p + 23, iplen);
                u8 port[2]; memcpy(port, p + 23 + iplen, 2); bput(&enc, port, 2);
                used = 25 + iplen;
            } else {
                used = 19;
            }
            /* multi executes value_.value_ for membership values: the empty
             * string (the membership branch is #if 0, paxos.cpp:1592-1617) */
        } else {
            if (avail < 18) { bfree(&enc); return E_DECODE; }
            u32 len = rd32(p + 14);
            if (avail < 18 + (size_t)len) { bfree(&enc); return E_DECODE; }
            bput32(&enc, len); exec_from = enc.n; exec_len = len;
            bput(&enc, p + 18, len);
            used = 18 + len;
        }
    }
    if (enc.oom) { bfree(&enc); return E_NOMEM; }
    u64 h = ((u64)proposer << 48) | ((u64)noop << 47) | value_id;
    if (!t) { bfree(&enc); *handle = h; return (long)used; }   /* outside the shard: not interned */
    ent_t *e = map_find(&t->idx, h);
    if (e) {
        valrec_t *r = &t->v[e->a];
        if (r->len != enc.n || memcmp(t->bytes.p + r->off, enc.p, enc.n)) { bfree(&enc); return E_VALUE; }
    } else {
        if (t->n == t->cap) {
            size_t c = t->cap ? t->cap * 2 : 64;
            valrec_t *q = (valrec_t *)realloc(t->v, c * sizeof(valrec_t));
            if (!q) { bfree(&enc); return E_NOMEM; }
            t->v = q; t->cap = c;
        }
        valrec_t *r = &t->v[t->n];
        r->handle = h; r->off = t->bytes.n; r->len = (u32)enc.n;
        r->exec_off = (u32)exec_from; r->exec_len = (u32)exec_len;
        bput(&t->bytes, enc.p, enc.n);
        if (!map_put(&t->idx, h, t->n, 0)) { bfree(&enc); return E_NOMEM; }
        t->n++;
    }
    bfree(&enc);
    *handle = h;
    return (long)used;
}
static const valrec_t *vt_get(const vtab_t *t, u64 h)
{
    ent_t *e = map_find(&t->idx, h);
    return e ? &t->v[e->a] : NULL;
}

/* member Value_m (member/paxos.cpp:330-408): u32 proposer, u64 value_id,
 * u8 noop; unless noop: u8 membership, then either u32 count + count x
 * {u32 node, u32 type} or u32 len + payload, then u32 cblen + cb.  What
 * StateMachine::Apply receives is the payload (Learner::Apply, :1062-1073). */
static long parse_value_m(vtab_t *t, const u8 *p, size_t avail, u64 *handle, int *membership)
{
    if (avail < 13) return E_DECODE;
    u32 proposer = rd32(p);
    u64 value_id = rd64(p + 4);
    int noop = p[12] != 0;
    size_t used = 13, exec_from = 0, exec_len = 0;
    *membership = 0;
    if (proposer >= (1u << 14) || value_id >= (1ull << 47)) return E_RANGE;
    if (!noop) {
        if (avail < 18) return E_DECODE;
        int mem = p[13] != 0;
        u32 n = rd32(p + 14);
        used = 18;
        if (mem) {
            if ((avail - used) / 8 < n) return E_DECODE;
            used += 8 * (size_t)n;
            *membership = 1;
        } else {
            if (avail - used < n) return E_DECODE;
            exec_from = used; exec_len = n;
            used += n;
        }
        if (avail - used < 4) return E_DECODE;
        u32 cbl = rd32(p + used);
        used += 4;
        if (avail - used < cbl) return E_DECODE;
        used += cbl;
    }
    /* canonical bytes = the wire bytes with bools normalised to 0/1 */
    u64 h = ((u64)proposer << 48) | ((u64)noop << 47) | value_id;
    if (!t) { *handle = h; return (long)used; }             /* outside the shard: not interned */
    u8 sbuf[256];
    buf_t enc = {sbuf, 0, sizeof sbuf, 0, 1};
    bput(&enc, p, used);
    if (enc.oom) return E_NOMEM;
    enc.p[12] = (u8)noop;
    if (!noop) enc.p[13] = (u8)*membership;
    ent_t *e = map_find(&t->idx, h);
    if (e) {
        valrec_t *r = &t->v[e->a];
        if (r->len != enc.n || memcmp(t->bytes.p + r->off, enc.p, enc.n)) { bfree(&enc); return E_VALUE; }
    } else {
        if (t->n == t->cap) {
            size_t c = t->cap ? t->cap * 2 : 64;
            valrec_t *q = (valrec_t *)realloc(t->v, c * sizeof(valrec_t));
            if (!q) { bfree(&enc); return E_NOMEM; }
            t->v = q; t->cap = c;
        }
        valrec_t *r = &t->v[t->n];
        r->handle = h; r->off = t->bytes.n; r->len = (u32)enc.n;
        r->exec_off = *membership ? 0xFFFFFFFFu : (u32)exec_from; r->exec_len = (u32)exec_len;
        bput(&t->bytes, enc.p, enc.n);
        if (!map_put(&t->idx, h, t->n, 0)) { bfree(&enc); return E_NOMEM; }
        t->n++;
    }
    bfree(&enc);
    *handle = h;
    return (long)used;
}

/* ---- digests (shared definition with the engine) ----- */
static u64 mix64(u64 x)
{
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    x ^= x >> 31; return x;
}

/* ---- per-node state ------------------------------------------------------- */
typedef struct {
    u64 batch_id;
    u64 mask;
    int live;
    size_t ent_off, ent_n;      /* entries (iid, handle) in node's batch pool  */
} batch_t;

/* a CommittingValues: id = ++committing_id_ at an accept quorum (kind 0,
 * multi/paxos.cpp:1418) or at a promise quorum of a node holding committed
 * values (kind 1: all of them re-committed, :1184-1197); replied_ as a learner
 * mask; retired at |replied_| == |nodes_| */
typedef struct {
    u64 created_seq, kind, accept_id, retired_seq, mask;
} commit_t;

typedef struct {
    u32 index;
    /* acceptor (multi/paxos.cpp:492-495) */
    u64 promised, max_seen;
    map_t acc;                  /* iid -> (ballot, handle): accepted_values_   */
    map_t com;                  /* iid -> (ballot, handle): committed_values_  */
    u64 next_apply;             /* next_id_to_apply_, paxos.cpp:501            */
    /* proposer aggregation (paxos.cpp:470-486) */
    u64 proposal_id;
    int preparing;              /* prepare_retry_timeout_ != NULL              */
    u64 promised_set;           /* prepare_promised_                          */
    map_t pre;                  /* pre_accepted_values_                       */
    batch_t *batches; size_t nb, cb;
    map_t batch_idx;            /* accept_id -> index in batches              */
    u64 *bent; size_t nbent, cbent;   /* batch entry pool (iid, handle) pairs  */
    /* member roles (member/paxos.cpp:737-747,1864-1964) */
    u32 epoch;
    int acc_exists, prop_exists;
    /* outputs */
    buf_t sends, events_q, events_c, exec;
    u64 n_sends, n_q, n_c, n_exec;
    u64 P, A, L;
    u64 violations;
    /* presence bitmap of accepted ∪ committed keys below the trace's instance
     * count M: FilterAcceptedValues' range scans walk it instead of sorting
     * both maps per PREPARE (O(window / 64), not O(state)).  `big`: a key >= M
     * was stored, this node then takes the full sorted scan. */
    u64 *pres;
    int big;
    /* per-node processing state: nodes run on their own threads (run_shard) */
    vtab_t vt;                  /* Values this node has seen (interned)        */
    map_t seen;                 /* per-message duplicate-iid check, reused     */
    u64 first_violation[4];
    int rc;
    /* phase-2 decisions (mpxo_decisions): value_id_ (multi/paxos.cpp:335) and the MPXD records */
    u64 value_id;
    /* client proposals (P_PROPOSE): unproposed_instance_ids_, initial_proposals_ (iid -> value
     * id), newly_proposed_values_ (ascending value ids) — multi/paxos.cpp:1132-1175,1250-1280 */
    rng_t unp;
    map_t initial;
    u64 *newly; size_t nnew, cnew;
    buf_t dec; u64 n_dec;
    /* commit reliability (mpxo_commits): committing_values_
     * (multi/paxos.cpp:483), one record per CommittingValues in id order */
    commit_t *cm; size_t ncm, ccm;
} node_t;

typedef struct { u32 version; u64 amask, pmask; } epoch_t;

typedef struct {
    u32 N, sem;
    u64 M;
    u32 ne;
    epoch_t *ep;
    vtab_t vt;
    node_t *nodes;
    u64 first_violation[4];     /* code, node, seq, iid */
    u64 sb, se;                 /* instance shard: entries outside are skipped (engine ingest) */
    int want_dec;               /* record the phase-2 batch at every promise quorum (mpxo_decisions) */
} ctx_t;
#define IN_SHARD(c, iid) ((iid) >= (c)->sb && (iid) < (c)->se)

static void violate(ctx_t *c, node_t *n, u64 code, u64 seq, u64 iid)
{
    (void)c;
    n->violations++;
    if (!n->first_violation[0]) {
        n->first_violation[0] = code; n->first_violation[1] = n->index;
        n->first_violation[2] = seq;  n->first_violation[3] = iid;
    }
}

static void emit(node_t *n, u32 dst, const buf_t *m)
{
    bput32(&n->sends, dst);
    bput32(&n->sends, (u32)m->n);
    bput(&n->sends, m->p, m->n);
    n->n_sends++;
}

/* ---- presence bitmap (see node_t) ---- */
static void pres_add(ctx_t *c, node_t *n, u64 k)
{
    if (k >= c->M || c->M > (1ull << 36)) { n->big = 1; return; }
    if (!n->pres) {
        n->pres = (u64 *)calloc((size_t)((c->M + 63) >> 6), 8);
        if (!n->pres) { n->big = 1; return; }
    }
    n->pres[k >> 6] |= 1ull << (k & 63);
}
/* after an erase: clear the bit when the key is in neither map */
static void pres_drop(ctx_t *c, node_t *n, u64 k)
{
    if (k < c->M && n->pres && !map_find(&n->acc, k) && !map_find(&n->com, k))
        n->pres[k >> 6] &= ~(1ull << (k & 63));
}
/* first set bit in [i, e) or e */
static u64 pres_next(const node_t *n, u64 i, u64 e)
{
    while (i < e) {
        u64 w = n->pres[i >> 6] & (~0ull << (i & 63));
        if (w) { u64 r = (i & ~63ull) + (u64)__builtin_ctzll(w); return r < e ? r : e; }
        i = (i | 63) + 1;
    }
    return e;
}
static int push_ent(ent_t **v, size_t *k, size_t *cap, const ent_t *x)
{
    if (*k == *cap) {
        size_t nc = *cap ? 2 * *cap : 64;
        ent_t *q = (ent_t *)realloc(*v, nc * sizeof(ent_t));
        if (!q) return -1;
        *v = q; *cap = nc;
    }
    (*v)[(*k)++] = *x;
    return 0;
}
/* FilterAcceptedValues' candidates for the ranges of a PREPARE (nr ranges of
 * 16 bytes at rg): per range the accepted entries inside it, then the
 * committed ones, each iid ascending — what the caller then sorts by iid.
 * Returns the count (*out malloc'ed) or -1. */
static long range_entries(ctx_t *c, node_t *n, const u8 *rg, size_t nr, ent_t **out)
{
    size_t k = 0, cap = 0;
    ent_t *v = NULL;
    if (n->big || !n->pres) {
        size_t na, nc;
        ent_t *va = map_sorted(&n->acc, &na);
        ent_t *vc = map_sorted(&n->com, &nc);
        if (!va || !vc) { free(va); free(vc); return -1; }
        for (size_t r = 0; r < nr; ++r) {
            u64 a = rd64(rg + 16 * r), b = rd64(rg + 16 * r + 8);
            for (size_t i = 0; i < na; ++i) if (va[i].key >= a && va[i].key < b && push_ent(&v, &k, &cap, &va[i])) goto oom;
            for (size_t i = 0; i < nc; ++i) if (vc[i].key >= a && vc[i].key < b && push_ent(&v, &k, &cap, &vc[i])) goto oom;
        }
        free(va); free(vc);
        *out = v;
        return (long)k;
    oom:
        free(va); free(vc); free(v);
        return -1;
    }
    for (size_t r = 0; r < nr; ++r) {
        u64 a = rd64(rg + 16 * r), b = rd64(rg + 16 * r + 8);
        u64 e = b < c->M ? b : c->M;
        for (int pass = 0; pass < 2; ++pass)
            for (u64 i = pres_next(n, a, e); i < e; i = pres_next(n, i + 1, e)) {
                const ent_t *x = map_find(pass ? &n->com : &n->acc, i);
                if (x && push_ent(&v, &k, &cap, x)) { free(v); return -1; }
            }
    }
    *out = v;
    return (long)k;
}

static void encode_value(buf_t *b, const vtab_t *t, u64 h)
{
    const valrec_t *r = vt_get(t, h);
    if (r) bput(b, t->bytes.p + r->off, r->len);
}

/* OnPrepare + FilterAcceptedValues, multi/paxos.cpp:858-922 */
static int on_prepare(ctx_t *c, node_t *n, const u8 *m, size_t len, u64 seq)
{
    if (len < 20) return E_DECODE;
    u32 proposer = rd32(m + 4);
    u64 id = rd64(m + 8);
    u32 rlen = rd32(m + 16);
    if (rlen % 16 || 20 + (size_t)rlen > len) return E_DECODE;
    if (id > n->max_seen) n->max_seen = id;                     /* :862-863 */
    if (proposer >= c->N) violate(c, n, 3, seq, 0);
    if (id > n->promised) {                                      /* :865 */
        n->promised = id;
        size_t nr = rlen / 16;
        /* ExtractAvailableInstanceIDs inserts ranges into a std::set; a
         * repeated pair is an ASSERT (:536) */
        for (size_t i = 0; i < nr; ++i)
            for (size_t j = 0; j < i; ++j)
                if (rd64(m + 20 + 16 * i) == rd64(m + 20 + 16 * j) &&
                    rd64(m + 28 + 16 * i) == rd64(m + 28 + 16 * j)) violate(c, n, 4, seq, 0);
        /* union of accepted and committed entries inside the ranges, iid
         * sorted (FilterAcceptedInstances, :902-910).  Tag: accept ballot or
         * commit ballot. */
        ent_t *out = NULL;
        long kk = range_entries(c, n, m + 20, nr, &out);
        if (kk < 0) return E_NOMEM;
        size_t k = (size_t)kk;
        qsort(out, k, sizeof(ent_t), cmp_ent);
        for (size_t i = 1; i < k; ++i) if (out[i].key == out[i - 1].key) violate(c, n, 4, seq, out[i].key);
        buf_t body = {0};
        for (size_t i = 0; i < k; ++i) {
            bput64(&body, out[i].key);
            bput64(&body, out[i].a);
            encode_value(&body, &n->vt, out[i].b);
        }
        buf_t r = {0};
        bput32(&r, 1); bput32(&r, n->index); bput64(&r, id); bput32(&r, (u32)body.n);
        bput(&r, body.p, body.n);
        emit(n, proposer, &r);
        n->P += k;
        free(r.p); free(body.p); free(out);
    } else if (id < n->promised) {                               /* :894 */
        buf_t r = {0};
        bput32(&r, 2); bput64(&r, n->max_seen);
        emit(n, proposer, &r);
        free(r.p);
    }                                                            /* ==: silent */
    return OK;
}

/* OnAccept, multi/paxos.cpp:1359-1404 */
static int on_accept(ctx_t *c, node_t *n, const u8 *m, size_t len, u64 seq)
{
    if (len < 28) return E_DECODE;
    u32 proposer = rd32(m + 4);
    u64 accept = rd64(m + 8);
    u64 id = rd64(m + 16);
    u32 vlen = rd32(m + 24);
    if (28 + (size_t)vlen > len) return E_DECODE;
    if (id > n->max_seen) n->max_seen = id;                     /* :1363 */
    if (proposer >= c->N) violate(c, n, 3, seq, 0);
    if (id >= n->promised) {                                     /* :1366 */
        size_t cur = 28, end = 28 + vlen;
        map_reset(&n->seen);
        while (cur < end) {
            if (end - cur < 8) { return E_DECODE; }
            u64 iid = rd64(m + cur); cur += 8;
            u64 h;
            long u = parse_value(IN_SHARD(c, iid) ? &n->vt : NULL, m + cur, end - cur, &h);
            if (u < 0) { return (int)u; }
            cur += (size_t)u;
            if (!IN_SHARD(c, iid)) continue;
            if (map_find(&n->seen, iid)) violate(c, n, 4, seq, iid);   /* :552 */
            map_put(&n->seen, iid, 0, 0);
            if (!map_find(&n->com, iid)) {                      /* :1380 */
                map_put(&n->acc, iid, id, h);                   /* :1387 overwrite */
                pres_add(c, n, iid);
                n->A++;
            }
        }
       
        buf_t r = {0};
        bput32(&r, 4); bput32(&r, n->index); bput64(&r, id); bput64(&r, accept);
        emit(n, proposer, &r);
        free(r.p);
    } else {
        buf_t r = {0};
        bput32(&r, 2); bput64(&r, n->max_seen);
        emit(n, proposer, &r);
        free(r.p);
    }
    return OK;
}

static int commit_proposals(node_t *n, u64 iid, u64 h);

/* OnCommit: learner part multi/paxos.cpp:1494-1518,1572-1622; proposer part (:1519-1570)
 * in commit_proposals */
static int on_commit(ctx_t *c, node_t *n, const u8 *m, size_t len, u64 seq)
{
    if (len < 28) return E_DECODE;
    u32 committer = rd32(m + 4);
    u64 commit = rd64(m + 8);
    u64 id = rd64(m + 16);
    u32 vlen = rd32(m + 24);
    if (28 + (size_t)vlen > len) return E_DECODE;
    if (committer >= c->N) violate(c, n, 3, seq, 0);
    size_t cur = 28, end = 28 + vlen;
    map_reset(&n->seen);
    while (cur < end) {
        if (end - cur < 8) { return E_DECODE; }
        u64 iid = rd64(m + cur); cur += 8;
        u64 h;
        long u = parse_value(IN_SHARD(c, iid) ? &n->vt : NULL, m + cur, end - cur, &h);
        if (u < 0) { return (int)u; }
        cur += (size_t)u;
        if (!IN_SHARD(c, iid)) continue;
        if (map_find(&n->seen, iid)) violate(c, n, 4, seq, iid);
        map_put(&n->seen, iid, 0, 0);
        map_del(&n->acc, iid);                                  /* :1501-1502 */
        pres_drop(c, n, iid);
        ent_t *e = map_find(&n->com, iid);
        if (e) {
            if (e->b != h) violate(c, n, 1, seq, iid);          /* :1508-1509 */
        } else {
            map_put(&n->com, iid, id, h);                       /* :1515 first wins */
            pres_add(c, n, iid);
        }
        n->L++;
        if (c->want_dec) map_put(&n->seen, iid, h, 1);          /* (the proposer part, below, in id order) */
    }
    if (c->want_dec && n->seen.n) {
        size_t k;
        ent_t *v = map_sorted(&n->seen, &k);
        for (size_t j = 0; j < k; ++j)
            if (commit_proposals(n, v[j].key, v[j].a)) { free(v); return E_NOMEM; }
        free(v);
    }
   
    buf_t r = {0};
    bput32(&r, 6); bput32(&r, n->index); bput64(&r, commit);   /* :1577-1582 */
    emit(n, committer, &r);
    free(r.p);
    /* in-order apply, skipping noops (:1584-1620) */
    for (;;) {
        ent_t *e = map_find(&n->com, n->next_apply);
        if (!e) break;
        n->next_apply++;
        u64 h = e->b;
        if ((h >> 47) & 1) continue;
        const valrec_t *r2 = vt_get(&n->vt, h);
        u32 el = r2 ? r2->exec_len : 0;
        bput32(&n->exec, el);
        if (el) bput(&n->exec, n->vt.bytes.p + r2->off + r2->exec_off, el);
        n->n_exec++;
    }
    return OK;
}

/* The phase-2 batch OnPrepareReply builds at a promise quorum (multi/paxos.cpp:1056-1175):
 * unproposed = uncommitted_instance_ids_ = every id not committed here; every pre-accepted
 * value of an unproposed id is adopted (:1071-1102); every range of the unproposed set but
 * the last, open one is filled with noops Value(index_, ++value_id_) in id order (:1117-1130)
 * — the last range starts after the highest committed or adopted id X, so the fill covers
 * exactly the unproposed, non-adopted ids below it; then the node's own client values
 * (:1132-1175, P_PROPOSE records): initial proposals at ids >= X, the queued ones at the
 * next free ids.  Record: seq, count, {iid, handle} ascending (the AcceptingValues map order). */
static int add_newly(node_t *n, u64 vid)
{
    for (size_t i = 0; i < n->nnew; ++i) if (n->newly[i] == vid) return OK;
    if (n->nnew == n->cnew) {
        size_t cc = n->cnew ? 2 * n->cnew : 16;
        u64 *q = (u64 *)realloc(n->newly, 8 * cc);
        if (!q) return E_NOMEM;
        n->newly = q; n->cnew = cc;
    }
    size_t i = n->nnew++;
    while (i && n->newly[i - 1] > vid) { n->newly[i] = n->newly[i - 1]; --i; }   /* a std::set */
    n->newly[i] = vid;
    return OK;
}

/* Propose (:1250-1280): a new value id; not preparing -> the next unproposed instance now
 * (its AcceptingValues is the trace's P_BATCH), else queued for the next promise quorum */
static int on_propose(node_t *n)
{
    ++n->value_id;
    if (!n->preparing) { map_put(&n->initial, rng_next(&n->unp), n->value_id, 0); return OK; }
    return add_newly(n, n->value_id);
}

/* OnCommit's proposer part (:1519-1570), one committed entry in instance order: the id leaves
 * the unproposed set; an own initial proposal that lost it is proposed again — at the next
 * unproposed id now, or queued while preparing */
static int commit_proposals(node_t *n, u64 iid, u64 h)
{
    if (rng_contains(&n->unp, iid)) rng_remove(&n->unp, iid);
    ent_t *e = map_find(&n->initial, iid);
    if (!e) return OK;
    u64 v0 = e->a;
    map_del(&n->initial, iid);
    if ((h >> 48) != n->index || (h & ((1ull << 47) - 1)) != v0) {
        if (!n->preparing) map_put(&n->initial, rng_next(&n->unp), v0, 0);
        else return add_newly(n, v0);
    }
    return OK;
}

static void decide(node_t *n, const ent_t *pre, size_t k, u64 seq)
{
    u64 X = 0;
    for (size_t j = 0; j < n->com.cap; ++j)
        if (n->com.used[j] && n->com.e[j].key + 1 > X) X = n->com.e[j].key + 1;
    for (size_t i = 0; i < k; ++i)
        if (!map_find(&n->com, pre[i].key) && pre[i].key + 1 > X) X = pre[i].key + 1;
    buf_t d = {0};
    u64 cnt = 0;
    size_t i = 0;
    for (u64 id = 0; id < X; ++id) {
        while (i < k && pre[i].key < id) ++i;
        if (map_find(&n->com, id)) continue;
        bput64(&d, id);
        if (i < k && pre[i].key == id) bput64(&d, pre[i].b);                             /* adopt */
        else bput64(&d, ((u64)n->index << 48) | (1ull << 47) | ++n->value_id);           /* noop */
        ++cnt;
    }
    /* then the own values (:1132-1175): unproposed is now [X, 2^64-1); the initial proposals
     * still in it keep their instance, the queued ones take the next free ids */
    rng_init(&n->unp);
    rng_remove_below(&n->unp, X);
    size_t ni = 0, np = 0;
    ent_t *iv = map_sorted(&n->initial, &ni);
    u64 *pe = (u64 *)malloc(16 * (ni + n->nnew + 1));
    for (size_t j = 0; j < ni; ++j)
        if (rng_contains(&n->unp, iv[j].key)) {
            rng_remove(&n->unp, iv[j].key);
            pe[2 * np] = iv[j].key; pe[2 * np + 1] = ((u64)n->index << 48) | iv[j].a; ++np;
        }
    free(iv);
    for (size_t j = 0; j < n->nnew; ++j) {
        u64 iid = rng_next(&n->unp);
        map_put(&n->initial, iid, n->newly[j], 0);
        pe[2 * np] = iid; pe[2 * np + 1] = ((u64)n->index << 48) | n->newly[j]; ++np;
    }
    n->nnew = 0;
    for (size_t a = 1; a < np; ++a)                              /* by instance (the batch is a map) */
        for (size_t b = a; b > 0 && pe[2 * b - 2] > pe[2 * b]; --b) {
            u64 t0 = pe[2 * b - 2], t1 = pe[2 * b - 1];
            pe[2 * b - 2] = pe[2 * b]; pe[2 * b - 1] = pe[2 * b + 1]; pe[2 * b] = t0; pe[2 * b + 1] = t1;
        }
    for (size_t j = 0; j < np; ++j) { bput64(&d, pe[2 * j]); bput64(&d, pe[2 * j + 1]); ++cnt; }
    free(pe);
    bput64(&n->dec, seq);
    bput64(&n->dec, cnt);
    bput(&n->dec, d.p, d.n);
    free(d.p);
    n->n_dec++;
}

static int new_commit(node_t *n, u64 seq, u64 kind, u64 accept);

/* OnPrepareReply + UpdateByPreAcceptedValues, multi/paxos.cpp:1036-1057,1201-1223 */
static int on_prepare_reply(ctx_t *c, node_t *n, const u8 *m, size_t len, u64 seq)
{
    if (len < 20) return E_DECODE;
    u32 acceptor = rd32(m + 4);
    u64 id = rd64(m + 8);
    u32 vlen = rd32(m + 16);
    if (20 + (size_t)vlen > len) return E_DECODE;
    if (!n->preparing || id != n->proposal_id) return OK;        /* :1038 */
    if (acceptor >= c->N) { violate(c, n, 3, seq, 0); return OK; }  /* :1040 */
    n->promised_set |= 1ull << acceptor;
    size_t cur = 20, end = 20 + vlen;
    map_reset(&n->seen);
    while (cur < end) {
        if (end - cur < 16) { return E_DECODE; }
        u64 iid = rd64(m + cur), pid = rd64(m + cur + 8); cur += 16;
        u64 h;
        long u = parse_value(IN_SHARD(c, iid) ? &n->vt : NULL, m + cur, end - cur, &h);
        if (u < 0) { return (int)u; }
        cur += (size_t)u;
        if (!IN_SHARD(c, iid)) continue;
        if (map_find(&n->seen, iid)) violate(c, n, 4, seq, iid);   /* :677 */
        map_put(&n->seen, iid, 0, 0);
        ent_t *e = map_find(&n->pre, iid);
        if (e) { if (pid > e->a) { e->a = pid; e->b = h; } }   /* strict >, :1218 */
        else map_put(&n->pre, iid, pid, h);
    }
   
    if ((u64)__builtin_popcountll(n->promised_set) >= c->N / 2 + 1) {   /* :1047 */
        size_t k;
        ent_t *v = map_sorted(&n->pre, &k);
        bput64(&n->events_q, seq);
        bput64(&n->events_q, n->proposal_id);
        bput64(&n->events_q, k);
        for (size_t i = 0; i < k; ++i) {
            bput64(&n->events_q, v[i].key);
            bput64(&n->events_q, v[i].a);
            bput64(&n->events_q, v[i].b);
        }
        n->n_q++;
        if (c->want_dec) decide(n, v, k, seq);
        free(v);
        for (size_t i = 0; i < n->nb; ++i)                      /* :1054 */
            if (n->batches[i].live) { violate(c, n, 5, seq, 0); break; }
        if (n->com.n && new_commit(n, seq, 1, 0)) return E_NOMEM;   /* re-commit everything committed, :1184-1197 */
        n->promised_set = 0;
        n->preparing = 0;
        map_clear(&n->pre);                                     /* :1105 */
    }
    return OK;
}

static int new_commit(node_t *n, u64 seq, u64 kind, u64 accept)
{
    if (n->ncm == n->ccm) {
        size_t cc = n->ccm ? n->ccm * 2 : 16;
        commit_t *q = (commit_t *)realloc(n->cm, cc * sizeof(commit_t));
        if (!q) return E_NOMEM;
        n->cm = q; n->ccm = cc;
    }
    n->cm[n->ncm++] = (commit_t){seq, kind, accept, ~0ull, 0};
    return OK;
}

/* OnAcceptReply, multi/paxos.cpp:1406-1427 */
static int on_accept_reply(ctx_t *c, node_t *n, const u8 *m, size_t len, u64 seq)
{
    if (len < 24) return E_DECODE;
    u32 acceptor = rd32(m + 4);
    u64 id = rd64(m + 8);
    u64 accept = rd64(m + 16);
    if (id != n->proposal_id) return OK;                        /* :1408 */
    ent_t *e = map_find(&n->batch_idx, accept);
    if (!e || !n->batches[e->a].live) return OK;                /* :1410 */
    if (acceptor >= c->N) { violate(c, n, 3, seq, 0); return OK; }  /* :1414 */
    batch_t *b = &n->batches[e->a];
    b->mask |= 1ull << acceptor;
    if ((u64)__builtin_popcountll(b->mask) >= c->N / 2 + 1) {   /* :1416 */
        bput64(&n->events_c, seq);
        bput64(&n->events_c, accept);
        n->n_c++;
        b->live = 0;                                            /* :1423-1425 */
        if (new_commit(n, seq, 0, accept)) return E_NOMEM;      /* CommittingValues(++committing_id_), :1418-1421 */
    }
    return OK;
}

/* OnCommitReply, multi/paxos.cpp:1625-1641: a reply for a live commit adds its
 * learner to replied_; the commit retires when every node has replied.  A
 * learner id >= 64 (the engine's mask) is recorded as a violation instead. */
static int on_commit_reply(ctx_t *c, node_t *n, const u8 *m, size_t len, u64 seq)
{
    if (len < 16) return E_DECODE;
    u32 learner = rd32(m + 4);
    u64 id = rd64(m + 8);
    if (id == 0 || id > n->ncm || n->cm[id - 1].retired_seq != ~0ull) return OK;   /* :1627 */
    if (learner >= 64) { violate(c, n, 3, seq, 0); return OK; }
    commit_t *x = &n->cm[id - 1];
    x->mask |= 1ull << learner;                                 /* :1633 */
    if ((u64)__builtin_popcountll(x->mask) == c->N) x->retired_seq = seq;   /* :1635-1640 */
    return OK;
}

/* P_START marker: StartPrepare (paxos.cpp:1233-1248) after RestartPrepare or
 * AcceptRejected (:1328-1343): new ballot, preparing, empty promise set and
 * pre-accepted map, no outstanding accept batches. */
static int on_p_start(node_t *n, const u8 *m, size_t len)
{
    if (len < 12) return E_DECODE;
    n->proposal_id = rd64(m + 4);
    n->preparing = 1;
    n->promised_set = 0;
    map_clear(&n->pre);
    for (size_t i = 0; i < n->nb; ++i) n->batches[i].live = 0;
    return OK;
}

/* P_BATCH marker: a new AcceptingValues (paxos.cpp:1299-1326) */
static int on_p_batch(ctx_t *c, node_t *n, const u8 *m, size_t len, u64 seq)
{
    if (len < 16) return E_DECODE;
    u64 bid = rd64(m + 4);
    u32 vlen = rd32(m + 12);
    if (16 + (size_t)vlen > len) return E_DECODE;
    if (n->nb == n->cb) {
        size_t cc = n->cb ? n->cb * 2 : 16;
        batch_t *q = (batch_t *)realloc(n->batches, cc * sizeof(batch_t));
        if (!q) return E_NOMEM;
        n->batches = q; n->cb = cc;
    }
    batch_t *b = &n->batches[n->nb];
    b->batch_id = bid; b->mask = 0; b->live = 1;
    b->ent_off = n->nbent; b->ent_n = 0;
    size_t cur = 16, end = 16 + vlen;
    while (cur < end) {
        if (end - cur < 8) return E_DECODE;
        u64 iid = rd64(m + cur); cur += 8;
        u64 h;
        long u = parse_value(IN_SHARD(c, iid) ? &n->vt : NULL, m + cur, end - cur, &h);
        if (u < 0) return (int)u;
        cur += (size_t)u;
        if (!IN_SHARD(c, iid)) continue;
        if (n->nbent + 2 > n->cbent) {
            size_t cc = n->cbent ? n->cbent * 2 : 64;
            u64 *q = (u64 *)realloc(n->bent, cc * sizeof(u64));
            if (!q) return E_NOMEM;
            n->bent = q; n->cbent = cc;
        }
        n->bent[n->nbent++] = iid;
        n->bent[n->nbent++] = h;
        b->ent_n++;
    }
    (void)seq;
    map_put(&n->batch_idx, bid, n->nb, 0);
    n->nb++;
    return OK;
}

static int process(ctx_t *c, node_t *n, const u8 *m, size_t len, u64 seq)
{
    if (len < 4) return E_DECODE;
    switch (rd32(m)) {                                          /* GetMsgType, :736 */
    case 0:  return on_prepare(c, n, m, len, seq);
    case 1:  return on_prepare_reply(c, n, m, len, seq);
    case 2:                                                     /* OnReject, :1225 */
        if (len < 12) return E_DECODE;
        if (n->max_seen < rd64(m + 4)) n->max_seen = rd64(m + 4);
        return OK;
    case 3:  return on_accept(c, n, m, len, seq);
    case 4:  return on_accept_reply(c, n, m, len, seq);
    case 5:  return on_commit(c, n, m, len, seq);
    case 6:  return on_commit_reply(c, n, m, len, seq);
    case 16: return on_p_start(n, m, len);
    case 17: return on_p_batch(c, n, m, len, seq);
    case 19:                                                    /* P_PROPOSE: Propose (:1250-1280) moves */
        if (len < 8 || 8 + (uint64_t)rd32(m + 4) > len) return E_DECODE;   /* no acceptor / learner state */
        return on_propose(n);
    default: return E_DECODE;                                   /* ASSERT(false), :1672 */
    }
}


/* ======================= member semantics (member/paxos.cpp) ===============
 * Node roles follow the E_EPOCH markers against the epoch table (include/mpx.h):
 * Loop dispatches PREPARE/ACCEPT only to an existing Acceptor and replies only
 * to an existing Proposer (:749-790); LEARN always reaches the Learner. */

/* entries {u64 iid, u64 pid, Value_m}* of ACCEPT / LEARN / PREPARE_REPLY /
 * member P_BATCH (ExtractProposalValues, :421-433); a repeated iid is its ASSERT */
typedef struct { u64 iid, pid, h; } pent_t;
static int parse_pvalues(ctx_t *c, node_t *n, const u8 *m, size_t beg, size_t end, u64 seq,
                         int report, pent_t **out, size_t *k)
{
    size_t cap = 16, cnt = 0, cur = beg;
    pent_t *v = (pent_t *)malloc(cap * sizeof(pent_t));
    map_reset(&n->seen);
    if (!v) return E_NOMEM;
    while (cur < end) {
        if (end - cur < 16) { free(v); return E_DECODE; }
        u64 iid = rd64(m + cur), pid = rd64(m + cur + 8);
        cur += 16;
        u64 h; int mem;
        long u = parse_value_m(IN_SHARD(c, iid) ? &n->vt : NULL, m + cur, end - cur, &h, &mem);
        if (u < 0) { free(v); return (int)u; }
        cur += (size_t)u;
        if (!IN_SHARD(c, iid)) continue;
        if (map_find(&n->seen, iid)) { if (report) violate(c, n, 4, seq, iid); continue; }   /* :429-431 */
        map_put(&n->seen, iid, 0, 0);
        if (cnt == cap) {
            cap *= 2;
            pent_t *q = (pent_t *)realloc(v, cap * sizeof(pent_t));
            if (!q) { free(v); return E_NOMEM; }
            v = q;
        }
        v[cnt].iid = iid; v[cnt].pid = pid; v[cnt].h = h; cnt++;
    }
   
    *out = v; *k = cnt;
    return OK;
}

static int m_reject(node_t *n, u32 dst)
{
    buf_t r = {0};
    bput32(&r, 2); bput64(&r, n->max_seen);                 /* RejectMsg, :882-888 */
    emit(n, dst, &r);
    free(r.p);
    return OK;
}

/* Acceptor::OnPrepare + FilterAcceptedValues, member/paxos.cpp:1700-1741,1796-1818 */
static int m_on_prepare(ctx_t *c, node_t *n, const u8 *m, size_t len, u64 seq)
{
    if (len < 24) return E_DECODE;
    u32 version = rd32(m + 4), proposer = rd32(m + 8);
    u64 id = rd64(m + 12);
    u32 rlen = rd32(m + 20);
    if (rlen % 16 || 24 + (size_t)rlen > len) return E_DECODE;
    if (!n->acc_exists) return OK;                          /* Loop: if (acceptor_) */
    if (version != c->ep[n->epoch].version) return OK;      /* :1702 */
    if (id > n->max_seen) n->max_seen = id;                 /* :1708-1709 */
    if (proposer >= c->N) violate(c, n, 3, seq, 0);
    if (id > n->promised) {                                 /* :1711 */
        n->promised = id;
        size_t nr = rlen / 16;
        for (size_t i = 0; i < nr; ++i)                     /* range set insert ASSERT, :290 */
            for (size_t j = 0; j < i; ++j)
                if (rd64(m + 24 + 16 * i) == rd64(m + 24 + 16 * j) &&
                    rd64(m + 32 + 16 * i) == rd64(m + 32 + 16 * j)) violate(c, n, 4, seq, 0);
        /* accepted then learned per range, into one iid-keyed map (:1806-1816) */
        ent_t *out = NULL;
        long kk = range_entries(c, n, m + 24, nr, &out);
        if (kk < 0) return E_NOMEM;
        size_t k = (size_t)kk;
        qsort(out, k, sizeof(ent_t), cmp_ent);
        size_t w = 0;
        for (size_t i = 0; i < k; ++i) {
            if (w && out[i].key == out[w - 1].key) { violate(c, n, 4, seq, out[i].key); continue; }
            out[w++] = out[i];
        }
        buf_t body = {0};
        for (size_t i = 0; i < w; ++i) {
            bput64(&body, out[i].key);
            bput64(&body, out[i].a);
            encode_value(&body, &n->vt, out[i].b);
        }
        buf_t r = {0};
        bput32(&r, 1); bput32(&r, n->index); bput64(&r, id); bput32(&r, (u32)body.n);   /* :1726-1730 */
        bput(&r, body.p, body.n);
        emit(n, proposer, &r);
        n->P += w;
        free(r.p); free(body.p); free(out);
    } else if (id < n->promised) {                          /* :1734 */
        m_reject(n, proposer);
    }
    return OK;
}

/* Acceptor::OnAccept, member/paxos.cpp:1742-1784: insert (first value sticks) */
static int m_on_accept(ctx_t *c, node_t *n, const u8 *m, size_t len, u64 seq)
{
    if (len < 32) return E_DECODE;
    u32 version = rd32(m + 4), proposer = rd32(m + 8);
    u64 accept = rd64(m + 12), id = rd64(m + 20);
    u32 vlen = rd32(m + 28);
    if (32 + (size_t)vlen > len) return E_DECODE;
    if (!n->acc_exists) return OK;
    if (version != c->ep[n->epoch].version) return OK;      /* :1744 */
    if (id > n->max_seen) n->max_seen = id;                 /* :1750-1751 */
    if (proposer >= c->N) violate(c, n, 3, seq, 0);
    if (id >= n->promised) {                                /* :1753 */
        pent_t *v; size_t k;
        int rc = parse_pvalues(c, n, m, 32, 32 + vlen, seq, 1, &v, &k);
        if (rc) return rc;
        for (size_t i = 0; i < k; ++i) {
            ent_t *l = map_find(&n->com, v[i].iid);
            if (l) {                                        /* :1767-1769 */
                if (l->b != v[i].h) violate(c, n, 6, seq, v[i].iid);
            } else if (!map_find(&n->acc, v[i].iid)) {      /* std::map::insert, :1765 */
                map_put(&n->acc, v[i].iid, v[i].pid, v[i].h);
                pres_add(c, n, v[i].iid);
                n->A++;
            }
        }
        free(v);
        buf_t r = {0};
        bput32(&r, 4); bput32(&r, n->index); bput64(&r, accept);   /* AcceptReplyMsg, :1771 */
        emit(n, proposer, &r);
        free(r.p);
    } else {
        m_reject(n, proposer);
    }
    return OK;
}

/* Learner::OnLearn (+ Proposer::OnLearn's equality ASSERT, Acceptor::OnLearn),
 * member/paxos.cpp:1029-1060,1396-1400,1786-1793 */
static int m_on_learn(ctx_t *c, node_t *n, const u8 *m, size_t len, u64 seq)
{
    if (len < 20) return E_DECODE;
    u32 proposer = rd32(m + 4);
    u64 learn = rd64(m + 8);
    u32 vlen = rd32(m + 16);
    if (20 + (size_t)vlen > len) return E_DECODE;
    pent_t *v; size_t k;
    int rc = parse_pvalues(c, n, m, 20, 20 + vlen, seq, 1, &v, &k);
    if (rc) return rc;
    if (proposer >= c->N) violate(c, n, 3, seq, 0);
    for (size_t i = 0; i < k; ++i) {
        ent_t *l = map_find(&n->com, v[i].iid);
        if (l) {
            if (n->prop_exists && l->b != v[i].h) violate(c, n, 6, seq, v[i].iid);   /* :1398-1399 */
        }
        map_del(&n->acc, v[i].iid);                         /* :1790-1791 */
        if (!l) map_put(&n->com, v[i].iid, v[i].pid, v[i].h);   /* insert, :1040 */
        if (!l) pres_add(c, n, v[i].iid); else pres_drop(c, n, v[i].iid);
        n->L++;
    }
    free(v);
    for (;;) {                                              /* :1042-1053 */
        ent_t *e = map_find(&n->com, n->next_apply);
        if (!e) break;
        n->next_apply++;
        u64 h = e->b;
        if ((h >> 47) & 1) continue;                        /* noop, :1064 */
        const valrec_t *r2 = vt_get(&n->vt, h);
        if (r2 && r2->exec_off == 0xFFFFFFFFu) continue;    /* membership: ChangeMemberships, :1066-1069 */
        u32 el = r2 ? r2->exec_len : 0;
        bput32(&n->exec, el);
        if (el) bput(&n->exec, n->vt.bytes.p + r2->off + r2->exec_off, el);
        n->n_exec++;
    }
    buf_t r = {0};
    bput32(&r, 6); bput32(&r, n->index); bput64(&r, learn);   /* LearnReplyMsg, :1055-1059 */
    emit(n, proposer, &r);
    free(r.p);
    return OK;
}

/* Proposer::OnPrepareReply + UpdateByPreAcceptedValues, member/paxos.cpp:1158-1182,1571-1586 */
static int m_on_prepare_reply(ctx_t *c, node_t *n, const u8 *m, size_t len, u64 seq)
{
    if (len < 20) return E_DECODE;
    u32 acceptor = rd32(m + 4);
    u64 id = rd64(m + 8);
    u32 vlen = rd32(m + 16);
    if (20 + (size_t)vlen > len) return E_DECODE;
    pent_t *v; size_t k;
    const int live = n->prop_exists && n->preparing && id == n->proposal_id;     /* :1160 */
    int rc = parse_pvalues(c, n, m, 20, 20 + vlen, seq, live, &v, &k);
    if (rc) return rc;
    const epoch_t *ep = &c->ep[n->epoch];
    if (!live) { free(v); return OK; }
    if (acceptor >= 64 || !((ep->amask >> acceptor) & 1)) { violate(c, n, 3, seq, 0); free(v); return OK; }   /* :1163 */
    n->promised_set |= 1ull << acceptor;
    for (size_t i = 0; i < k; ++i) {
        ent_t *e = map_find(&n->pre, v[i].iid);
        if (e) { if (v[i].pid > e->a) { e->a = v[i].pid; e->b = v[i].h; } }   /* strict >, :1580 */
        else map_put(&n->pre, v[i].iid, v[i].pid, v[i].h);
    }
    free(v);
    if ((u64)__builtin_popcountll(n->promised_set) >= (u64)__builtin_popcountll(ep->amask) / 2 + 1) {   /* :1171 */
        size_t q;
        ent_t *pv = map_sorted(&n->pre, &q);
        bput64(&n->events_q, seq);
        bput64(&n->events_q, n->proposal_id);
        bput64(&n->events_q, q);
        for (size_t i = 0; i < q; ++i) {
            bput64(&n->events_q, pv[i].key);
            bput64(&n->events_q, pv[i].a);
            bput64(&n->events_q, pv[i].b);
        }
        n->n_q++;
        free(pv);
        for (size_t i = 0; i < n->nb; ++i)                 /* :1182 */
            if (n->batches[i].live) { violate(c, n, 5, seq, 0); break; }
        n->promised_set = 0;
        n->preparing = 0;
        map_clear(&n->pre);
    }
    return OK;
}

/* Proposer::OnAcceptReply, member/paxos.cpp:1317-1343: matched by batch id only */
static int m_on_accept_reply(ctx_t *c, node_t *n, const u8 *m, size_t len, u64 seq)
{
    if (len < 16) return E_DECODE;
    u32 acceptor = rd32(m + 4);
    u64 accept = rd64(m + 8);
    if (!n->prop_exists) return OK;
    ent_t *e = map_find(&n->batch_idx, accept);
    if (!e || !n->batches[e->a].live) return OK;            /* :1319 */
    const epoch_t *ep = &c->ep[n->epoch];
    if (acceptor >= 64 || !((ep->amask >> acceptor) & 1)) { violate(c, n, 3, seq, 0); return OK; }   /* :1324 */
    batch_t *b = &n->batches[e->a];
    b->mask |= 1ull << acceptor;
    if ((u64)__builtin_popcountll(b->mask) >= (u64)__builtin_popcountll(ep->amask) / 2 + 1) {   /* :1327 */
        bput64(&n->events_c, seq);
        bput64(&n->events_c, accept);
        n->n_c++;
        b->live = 0;                                        /* :1340-1342 */
    }
    return OK;
}

/* member P_BATCH: entries carry their proposal id like AcceptingValues' map */
static int m_on_p_batch(ctx_t *c, node_t *n, const u8 *m, size_t len, u64 seq)
{
    if (len < 16) return E_DECODE;
    u64 bid = rd64(m + 4);
    u32 vlen = rd32(m + 12);
    if (16 + (size_t)vlen > len) return E_DECODE;
    pent_t *v; size_t k;
    int rc = parse_pvalues(c, n, m, 16, 16 + vlen, seq, 0, &v, &k);
    if (rc) return rc;
    if (!n->prop_exists) { free(v); return OK; }
    if (n->nb == n->cb) {
        size_t cc = n->cb ? n->cb * 2 : 16;
        batch_t *q = (batch_t *)realloc(n->batches, cc * sizeof(batch_t));
        if (!q) { free(v); return E_NOMEM; }
        n->batches = q; n->cb = cc;
    }
    batch_t *b = &n->batches[n->nb];
    b->batch_id = bid; b->mask = 0; b->live = 1;
    b->ent_off = n->nbent; b->ent_n = k;
    if (n->nbent + 2 * k > n->cbent) {
        size_t cc = n->cbent ? n->cbent : 64;
        while (cc < n->nbent + 2 * k) cc *= 2;
        u64 *q = (u64 *)realloc(n->bent, cc * sizeof(u64));
        if (!q) { free(v); return E_NOMEM; }
        n->bent = q; n->cbent = cc;
    }
    for (size_t i = 0; i < k; ++i) { n->bent[n->nbent++] = v[i].iid; n->bent[n->nbent++] = v[i].h; }
    free(v);
    map_put(&n->batch_idx, bid, n->nb, 0);
    n->nb++;
    return OK;
}

/* E_EPOCH marker: one step of ChangeMemberships as seen by this node */
static int m_on_epoch(ctx_t *c, node_t *n, const u8 *m, size_t len)
{
    if (len < 8) return E_DECODE;
    u32 e = rd32(m + 4);
    if (e >= c->ne) return E_DECODE;
    const epoch_t *o = &c->ep[n->epoch], *x = &c->ep[e];
    int acc = (int)((x->amask >> n->index) & 1), prop = (int)((x->pmask >> n->index) & 1);
    if (n->acc_exists != acc) {                             /* new / delete Acceptor, :1897-1901,1952-1957 */
        for (size_t i = 0; i < n->acc.cap && n->pres; ++i)   /* keys only accepted leave the bitmap */
            if (n->acc.used[i] && n->acc.e[i].key < c->M && !map_find(&n->com, n->acc.e[i].key))
                n->pres[n->acc.e[i].key >> 6] &= ~(1ull << (n->acc.e[i].key & 63));
        map_clear(&n->acc);
        n->promised = n->max_seen = 0;
        n->acc_exists = acc;
    }
    if (n->prop_exists != prop || (prop && o->amask != x->amask)) {
        /* Proposer deleted (:1927-1930), created (:1879-1883), or
         * AcceptorsChanged (:1291-1322): idle until the next P_START */
        n->preparing = 0;
        n->promised_set = 0;
        map_clear(&n->pre);
        for (size_t i = 0; i < n->nb; ++i) n->batches[i].live = 0;
        n->prop_exists = prop;
    }
    n->epoch = e;
    return OK;
}

static int process_member(ctx_t *c, node_t *n, const u8 *m, size_t len, u64 seq)
{
    if (len < 4) return E_DECODE;
    switch (rd32(m)) {
    case 0:  return m_on_prepare(c, n, m, len, seq);
    case 1:  return m_on_prepare_reply(c, n, m, len, seq);
    case 2:  return len < 12 ? E_DECODE : OK;              /* Proposer::OnReject: proposer-side max only */
    case 3:  return m_on_accept(c, n, m, len, seq);
    case 4:  return m_on_accept_reply(c, n, m, len, seq);
    case 5:  return m_on_learn(c, n, m, len, seq);
    case 6:  return len < 16 ? E_DECODE : OK;              /* OnLearnReply: out of scope */
    case 16:
        if (len < 12) return E_DECODE;
        if (n->prop_exists) on_p_start(n, m, len);
        return OK;
    case 17: return m_on_p_batch(c, n, m, len, seq);
    case 18: return m_on_epoch(c, n, m, len);
    case 19:                                               /* P_PROPOSE: the proposer's bookkeeping only */
        return len < 8 || 8 + (size_t)rd32(m + 4) > len ? E_DECODE : OK;
    default: return E_DECODE;
    }
}

/* ---- container -------------------------------------------------------------*/
#define HDR 40

/* out == NULL: counters and digests only (no MPXR bytes, state not sorted) */
static int dump(ctx_t *c, u8 **out, u64 *size, u64 *stats)
{
    buf_t r = {0};
    const int want = out != NULL;
    if (want) bput(&r, "MPXR", 4);
    if (want) { bput32(&r, 1); bput32(&r, c->N); bput32(&r, c->sem); }
    map_t chosen = {0};
    u64 C = 0, P = 0, A = 0, L = 0, V = 0;
    u64 dstate = 0, dscal = 0, dchosen = 0;
    for (u32 i = 0; i < c->N; ++i) {
        node_t *n = &c->nodes[i];
        if (want) { bput64(&r, n->promised); bput64(&r, n->max_seen); }
        dscal += mix64(mix64((u64)i * 0x9E3779B97F4A7C15ull ^ n->promised) ^ n->max_seen);
        if (!want) {
            for (int pass = 0; pass < 2; ++pass) {
                const map_t *mp = pass ? &n->com : &n->acc;
                const u64 kind = pass ? 2 : 1;
                for (size_t j = 0; j < mp->cap; ++j) {
                    if (!mp->used[j]) continue;
                    const ent_t *e = &mp->e[j];
                    dstate += mix64(mix64(mix64(e->key + (u64)i * 0x9E3779B97F4A7C15ull) ^ e->a)
                                    ^ (e->b + kind * 0xD6E8FEB86659FD93ull));
                }
            }
            P += n->P; A += n->A; L += n->L; V += n->violations;
            continue;
        }
        size_t na, nc;
        ent_t *va = map_sorted(&n->acc, &na);
        ent_t *vc = map_sorted(&n->com, &nc);
        if (want) bput64(&r, (u64)(na + nc));
        size_t ia = 0, ic = 0;
        while (ia < na || ic < nc) {
            int take_a = ic >= nc || (ia < na && va[ia].key < vc[ic].key);
            ent_t *e = take_a ? &va[ia++] : &vc[ic++];
            u64 kind = take_a ? 1 : 2;
            if (want) { bput64(&r, e->key); bput64(&r, kind); bput64(&r, e->a); bput64(&r, e->b); }
            dstate += mix64(mix64(mix64(e->key + (u64)i * 0x9E3779B97F4A7C15ull) ^ e->a)
                            ^ (e->b + kind * 0xD6E8FEB86659FD93ull));
        }
        free(va); free(vc);
        if (want) { bput64(&r, n->n_sends); bput(&r, n->sends.p, n->sends.n); }
        if (want) { bput64(&r, n->n_q); bput(&r, n->events_q.p, n->events_q.n); }
        if (want) { bput64(&r, n->n_c); bput(&r, n->events_c.p, n->events_c.n); }
        if (want) { bput64(&r, n->n_exec); bput(&r, n->exec.p, n->exec.n); }
        P += n->P; A += n->A; L += n->L; V += n->violations;
    }
    /* chosen log: union of the entries of every chosen batch, first wins;
     * a second batch with another value for an instance breaks safety */
    for (u32 i = 0; i < c->N; ++i) {
        node_t *n = &c->nodes[i];
        for (u64 k = 0; k < n->n_c; ++k) {
            u64 bid = rd64(n->events_c.p + 16 * k + 8);
            ent_t *e = map_find(&n->batch_idx, bid);
            if (!e) continue;
            batch_t *b = &n->batches[e->a];
            for (size_t j = 0; j < b->ent_n; ++j) {
                u64 iid = n->bent[b->ent_off + 2 * j], h = n->bent[b->ent_off + 2 * j + 1];
                ent_t *x = map_find(&chosen, iid);
                if (x) { if (x->a != h) { violate(c, n, 2, 0, iid); V++; } }
                else { map_put(&chosen, iid, h, 0); C++; dchosen += mix64(mix64(iid) ^ h); }
            }
        }
    }
    if (want) {
        size_t nch;
        ent_t *vch = map_sorted(&chosen, &nch);
        bput64(&r, (u64)nch);
        for (size_t i = 0; i < nch; ++i) { bput64(&r, vch[i].key); bput64(&r, vch[i].a); }
        free(vch);
    }
    map_free(&chosen);
    if (stats) {
        stats[0] = C; stats[1] = P; stats[2] = A; stats[3] = L; stats[4] = V;
        stats[5] = dchosen; stats[6] = dstate; stats[7] = dscal;
    }
    if (!want) return OK;
    if (r.oom) { free(r.p); return E_NOMEM; }
    *out = r.p; *size = r.n;
    return OK;
}

/*
 * mpxo_run: process an MPXT trace, write the MPXR result.
 *   stats (optional, 8 words): C, P, A, L, violations, chosen_digest,
 *                              state_digest, scalar_digest
 *   viol  (optional, 4 words): first violation code, node, seq, iid
 * Returns 0 or a negative mpx status code.
 */
typedef struct { ctx_t *c; node_t *n; const u8 *offs, *bytes; u64 cnt, nbytes; } node_job_t;
static void *node_job(void *arg)
{
    node_job_t *j = (node_job_t *)arg;
    int rc = OK;
    for (u64 k = 0; k < j->cnt && rc == OK; ++k) {
        u64 a = rd64(j->offs + 8 * k), b = rd64(j->offs + 8 * (k + 1));
        if (b < a || b > j->nbytes) { rc = E_DECODE; break; }
        rc = j->c->sem ? process_member(j->c, j->n, j->bytes + a, (size_t)(b - a), k)
                       : process(j->c, j->n, j->bytes + a, (size_t)(b - a), k);
    }
    j->n->rc = rc;
    return NULL;
}

static int check_values(ctx_t *c)
{
    map_t all = {0};            /* handle -> node * 2^32 + record */
    int rc = OK;
    for (u32 i = 0; i < c->N && rc == OK; ++i) {
        const vtab_t *t = &c->nodes[i].vt;
        for (size_t r = 0; r < t->n && rc == OK; ++r) {
            const valrec_t *x = &t->v[r];
            ent_t *e = map_find(&all, x->handle);
            if (!e) { if (!map_put(&all, x->handle, ((u64)i << 32) | r, 0)) rc = E_NOMEM; continue; }
            const vtab_t *u = &c->nodes[e->a >> 32].vt;
            const valrec_t *y = &u->v[e->a & 0xFFFFFFFFu];
            if (x->len != y->len || memcmp(t->bytes.p + x->off, u->bytes.p + y->off, x->len)) rc = E_VALUE;
        }
    }
    map_free(&all);
    return rc;
}

static int run_shard_ex(const u8 *trace, u64 size, u64 sb, u64 se, u8 **out, u64 *out_size, u64 *stats,
                        u64 *viol, u8 **dec, u64 *dec_size, u8 **cmt, u64 *cmt_size)
{
    if (size < HDR || memcmp(trace, "MPXT", 4)) return E_DECODE;
    ctx_t c;
    memset(&c, 0, sizeof c);
    c.sb = sb; c.se = se;
    c.want_dec = dec != NULL;
    c.N = rd32(trace + 8);
    c.sem = rd32(trace + 12);
    c.M = rd64(trace + 16);
    u32 ne = rd32(trace + 24);
    if (c.N == 0 || c.N > 64 || c.sem > 1) return -1;
    const size_t esz = rd32(trace + 4) == 1 ? 24 : 32;     /* container version 2: + learner_mask */
    if (c.sem == 1 && (ne == 0 || size < HDR + (u64)ne * esz)) return E_DECODE;
    size_t pos = HDR + (size_t)ne * esz;
    c.nodes = (node_t *)calloc(c.N, sizeof(node_t));
    c.ne = ne;
    c.ep = (epoch_t *)calloc(ne ? ne : 1, sizeof(epoch_t));
    if (!c.nodes || !c.ep) { free(c.nodes); free(c.ep); return E_NOMEM; }
    for (u32 e = 0; e < ne; ++e) {
        c.ep[e].version = rd32(trace + HDR + esz * e);
        c.ep[e].amask = rd64(trace + HDR + esz * e + 8);
        c.ep[e].pmask = rd64(trace + HDR + esz * e + 16);
    }
    /* node streams: located sequentially, processed in parallel — a node's
     * handlers touch only its own state (the reference runs one paxos thread
     * per node, multi/paxos.cpp:345), so the result equals node-after-node */
    int rc = OK;
    node_job_t *jobs = (node_job_t *)calloc(c.N, sizeof(node_job_t));
    if (!jobs) rc = E_NOMEM;
    for (u32 i = 0; i < c.N && rc == OK; ++i) {
        node_t *n = &c.nodes[i];
        n->index = i;
        if (rng_init(&n->unp)) { rc = E_NOMEM; break; }
        if (c.sem == 1) {                                  /* genesis roles: epoch 0 */
            n->acc_exists = (int)((c.ep[0].amask >> i) & 1);
            n->prop_exists = (int)((c.ep[0].pmask >> i) & 1);
        }
        if (pos + 16 > size) { rc = E_DECODE; break; }
        u64 cnt = rd64(trace + pos), nbytes = rd64(trace + pos + 8);
        pos += 16;
        if (pos + 8 * (cnt + 1) + nbytes > size) { rc = E_DECODE; break; }
        jobs[i] = (node_job_t){&c, n, trace + pos, trace + pos + 8 * (cnt + 1), cnt, nbytes};
        pos += 8 * (cnt + 1) + nbytes;
        pos = (pos + 7) & ~(size_t)7;
    }
    if (rc == OK) {
        pthread_t *tid = (pthread_t *)calloc(c.N, sizeof(pthread_t));
        const int par = tid && c.N > 1 && size > (1u << 20);
        for (u32 i = 0; i < c.N; ++i)
            if (!par || pthread_create(&tid[i], NULL, node_job, &jobs[i])) { node_job(&jobs[i]); if (tid) tid[i] = 0; }
        if (par) for (u32 i = 0; i < c.N; ++i) if (tid[i]) pthread_join(tid[i], NULL);
        free(tid);
        for (u32 i = 0; i < c.N; ++i) {                    /* first error / violation in node order */
            if (c.nodes[i].rc && rc == OK) rc = c.nodes[i].rc;
            if (c.nodes[i].first_violation[0] && !c.first_violation[0])
                memcpy(c.first_violation, c.nodes[i].first_violation, sizeof c.first_violation);
        }
        /* a Value must be the same bytes wherever its (proposer, value_id)
         * appears (the engine's one value table, MPX_E_VALUE): checked across
         * the per-node tables for full results */
        if (rc == OK && out) rc = check_values(&c);
    }
    free(jobs);
    if (rc == OK) rc = dump(&c, out, out_size, stats);
    if (rc == OK && dec) {
        buf_t d = {0};
        bput(&d, "MPXD", 4); bput32(&d, 1); bput32(&d, c.N);
        for (u32 i = 0; i < c.N; ++i) { bput64(&d, c.nodes[i].n_dec); bput(&d, c.nodes[i].dec.p, c.nodes[i].dec.n); }
        if (d.oom) { free(d.p); rc = E_NOMEM; } else { *dec = d.p; *dec_size = d.n; }
    }
    if (rc == OK && cmt) {
        /* MPXC (include/mpx.h mpx_read_commits): per node, per commit id */
        buf_t d = {0};
        bput(&d, "MPXC", 4); bput32(&d, 1); bput32(&d, c.N);
        for (u32 i = 0; i < c.N; ++i) {
            const node_t *n = &c.nodes[i];
            bput64(&d, n->ncm);
            for (size_t k = 0; k < n->ncm; ++k) {
                bput64(&d, k + 1); bput64(&d, n->cm[k].created_seq); bput64(&d, n->cm[k].kind);
                bput64(&d, n->cm[k].accept_id);
                bput64(&d, n->cm[k].retired_seq); bput64(&d, n->cm[k].mask);
            }
        }
        if (d.oom) { free(d.p); rc = E_NOMEM; } else { *cmt = d.p; *cmt_size = d.n; }
    }
    for (u32 i = 0; i < c.N; ++i) { free(c.nodes[i].dec.p); free(c.nodes[i].cm); }
    if (viol) memcpy(viol, c.first_violation, sizeof c.first_violation);
    for (u32 i = 0; i < c.N; ++i) {
        node_t *n = &c.nodes[i];
        map_free(&n->acc); map_free(&n->com); map_free(&n->pre); map_free(&n->batch_idx);
        free(n->pres);
        free(n->batches); free(n->bent);
        free(n->sends.p); free(n->events_q.p); free(n->events_c.p); free(n->exec.p);
    }
    for (u32 i = 0; i < c.N; ++i) {
        node_t *n = &c.nodes[i];
        map_free(&n->vt.idx); free(n->vt.v); free(n->vt.bytes.p);
        map_free(&n->seen);
        map_free(&n->initial); free(n->unp.a); free(n->unp.b); free(n->newly);
    }
    free(c.nodes);
    free(c.ep);
    return rc;
}

static int run_shard(const u8 *trace, u64 size, u64 sb, u64 se, u8 **out, u64 *out_size, u64 *stats, u64 *viol)
{
    return run_shard_ex(trace, size, sb, se, out, out_size, stats, viol, NULL, NULL, NULL, NULL);
}

int mpxo_run(const u8 *trace, u64 size, u8 **out, u64 *out_size, u64 *stats, u64 *viol)
{
    return run_shard(trace, size, 0, ~0ull, out, out_size, stats, viol);
}

/* mpxo_decisions: the phase-2 batch at every promise quorum (MPXD, DESIGN.md
 * §f2; multi semantics), what `decide` records over a whole-trace run. */
int mpxo_decisions(const u8 *trace, u64 size, u8 **out, u64 *out_size)
{
    u8 *r = NULL;
    u64 rs = 0;
    int rc = run_shard_ex(trace, size, 0, ~0ull, &r, &rs, NULL, NULL, out, out_size, NULL, NULL);
    free(r);
    return rc;
}

/* mpxo_commits: the commit-reliability bookkeeping of a whole-trace run (MPXC,
 * DESIGN.md §f4; multi semantics): per node every CommittingValues with its
 * creation (accept quorum), accept id, retirement (all nodes replied) and
 * final replied_ mask. */
int mpxo_commits(const u8 *trace, u64 size, u8 **out, u64 *out_size)
{
    u8 *r = NULL;
    u64 rs = 0;
    int rc = run_shard_ex(trace, size, 0, ~0ull, &r, &rs, NULL, NULL, NULL, NULL, out, out_size);
    free(r);
    return rc;
}

/*
 * mpxo_run_shard: the same over the instance shard [sb, se) only — entries
 * outside it are skipped, headers are processed as a whole (what one GPU rank
 * ingests).  out may be NULL (counters / digests only).
 */
int mpxo_run_shard(const u8 *trace, u64 size, u64 sb, u64 se, u8 **out, u64 *out_size, u64 *stats, u64 *viol)
{
    return run_shard(trace, size, sb, se, out, out_size, stats, viol);
}

/*
 * mpxo_run_sharded: counters and digests of the whole trace from `shards`
 * instance shards of [0, M) run on `threads` host threads — instances are
 * independent given the headers, so counters and digests add up and the
 * per-node scalars (scalar digest) agree on every shard (E_STATE otherwise).
 * stats as in mpxo_run; returns the first error.
 */
typedef struct { const u8 *t; u64 size, sb, se; u64 stats[8]; int rc; } shard_job_t;
static void *shard_job(void *arg)
{
    shard_job_t *j = (shard_job_t *)arg;
    j->rc = run_shard(j->t, j->size, j->sb, j->se, NULL, NULL, j->stats, NULL);
    return NULL;
}
int mpxo_run_sharded(const u8 *trace, u64 size, u32 shards, u32 threads, u64 *stats)
{
    if (size < HDR || !shards || shards > 4096 || !threads || !stats) return E_INVAL;
    const u64 M = rd64(trace + 16);
    const u64 per = ((M + shards - 1) / shards + 255) / 256 * 256;
    shard_job_t *jobs = (shard_job_t *)calloc(shards, sizeof(shard_job_t));
    pthread_t *tid = (pthread_t *)calloc(threads, sizeof(pthread_t));
    if (!jobs || !tid) { free(jobs); free(tid); return E_NOMEM; }
    for (u32 k = 0; k < shards; ++k) {
        jobs[k].t = trace; jobs[k].size = size;
        jobs[k].sb = (u64)k * per < M ? (u64)k * per : M;
        jobs[k].se = k + 1 == shards ? ~0ull : ((u64)(k + 1) * per < M ? (u64)(k + 1) * per : M);
    }
    int rc = OK;
    for (u32 base = 0; base < shards; base += threads) {
        u32 nt = shards - base < threads ? shards - base : threads;
        for (u32 k = 0; k < nt; ++k)
            if (pthread_create(&tid[k], NULL, shard_job, &jobs[base + k])) { shard_job(&jobs[base + k]); tid[k] = 0; }
        for (u32 k = 0; k < nt; ++k) if (tid[k]) pthread_join(tid[k], NULL);
    }
    memset(stats, 0, 8 * sizeof(u64));
    for (u32 k = 0; k < shards; ++k) {
        if (jobs[k].rc && rc == OK) rc = jobs[k].rc;
        for (int w = 0; w < 7; ++w) stats[w] += jobs[k].stats[w];
        if (k && jobs[k].stats[7] != jobs[0].stats[7] && rc == OK) rc = -6;   /* scalars must agree */
    }
    stats[7] = jobs[0].stats[7];
    free(jobs); free(tid);
    return rc;
}

void mpxo_free(void *p) { free(p); }

/* ---- closed form for the clean trace (bench verification) -----------------
 * The clean generator (one proposer, ballot B, every instance proposed once,
 * every ACCEPT granted, every COMMIT delivered) ends
 * with every node holding committed_values_[i] = (B, handle(0, 0, i + 1))
 * (OnCommit, multi/paxos.cpp:1494-1518) and the chosen log = the same
 * handles.  This sums the digests (dump() above) of that final state over
 * instances [sb, se) without replaying the trace, so bench.py can check a
 * 2^27-instance run; `threads` POSIX threads split the instances. */
typedef struct { u64 N, lo, hi, ballot, ds, dc; } clean_job_t;

static void *clean_job(void *arg)
{
    clean_job_t *j = (clean_job_t *)arg;
    u64 ds = 0, dc = 0;
    for (u64 iid = j->lo; iid < j->hi; ++iid) {
        const u64 h = (iid + 1);                              /* MPX_HANDLE(0, 0, iid + 1) */
        dc += mix64(mix64(iid) ^ h);
        for (u64 i = 0; i < j->N; ++i)
            ds += mix64(mix64(mix64(iid + i * 0x9E3779B97F4A7C15ull) ^ j->ballot) ^ (h + 2 * 0xD6E8FEB86659FD93ull));
    }
    j->ds = ds; j->dc = dc;
    return NULL;
}

int mpxo_clean_expect(u32 N, u64 sb, u64 se, u64 ballot, u32 threads, u64 *state_digest, u64 *chosen_digest)
{
    if (!threads || threads > 256 || se < sb || !state_digest || !chosen_digest) return E_INVAL;
    clean_job_t jobs[256];
    pthread_t tid[256];
    const u64 span = (se - sb + threads - 1) / threads;
    for (u32 t = 0; t < threads; ++t) {
        u64 lo = sb + t * span, hi = lo + span;
        if (lo > se) lo = se;
        if (hi > se) hi = se;
        jobs[t] = (clean_job_t){N, lo, hi, ballot, 0, 0};
        if (pthread_create(&tid[t], NULL, clean_job, &jobs[t])) return E_NOMEM;
    }
    u64 ds = 0, dc = 0;
    for (u32 t = 0; t < threads; ++t) {
        pthread_join(tid[t], NULL);
        ds += jobs[t].ds; dc += jobs[t].dc;
    }
    *state_digest = ds; *chosen_digest = dc;
    return OK;
}
