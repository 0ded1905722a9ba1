// ingest.cpp — wire decode and instance bucketing (host, C++17).
//
// The reference decodes inside each handler (ExtractAvailableInstanceIDs,
// ExtractInstanceValues, ExtractAcceptedValues; multi/paxos.cpp:523-711) into
// std::map/std::set.  Here every record is decoded once into flat SoA arrays;
// entry-carrying records are then cut into per-(node, 256-instance bucket)
// fragments so one GPU workgroup sees all events of its instances, in order,
// with coalesced entry reads.
#include "ingest.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <atomic>
#include <thread>
#include <cstdlib>
#include <cstring>
#include <new>

#include "mpx.h"

namespace mpx {

static inline uint32_t rd32(const uint8_t *p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
static inline uint64_t rd64(const uint8_t *p) { uint64_t v; std::memcpy(&v, p, 8); return v; }
template <typename T> static inline void app(std::string &s, T v) { s.append((const char *)&v, sizeof v); }
#define TRY_RC(x) do { int _rc = (x); if (_rc) return _rc; } while (0)

// member Value_m (FillValue / ExtractValue, member/paxos.cpp:330-408): the
// multi layout plus a membership change list {u32 node, u32 type}* in place of
// the payload and a u32-length cb after it.  Canonical bytes = wire bytes with
// the bools normalised; membership Values are not executed (Learner::Apply,
// :1062-1073), marked by exec_off = NONE32.
static long parse_member(const uint8_t *p, size_t avail, std::string &enc, uint32_t &exec_off, uint32_t &exec_len)
{
    const bool noop = p[12] != 0;
    size_t used = 13;
    exec_off = exec_len = 0;
    if (!noop) {
        if (avail < 18) return MPX_E_DECODE;
        const bool mem = p[13] != 0;
        const uint32_t n = rd32(p + 14);
        used = 18;
        if (mem) {
            if ((avail - used) / 8 < n) return MPX_E_DECODE;
            used += 8 * (size_t)n;
            exec_off = NONE32;
        } else {
            if (avail - used < n) return MPX_E_DECODE;
            exec_off = (uint32_t)used;
            exec_len = n;
            used += n;
        }
        if (avail - used < 4) return MPX_E_DECODE;
        const uint32_t cbl = rd32(p + used);
        used += 4;
        if (avail - used < cbl) return MPX_E_DECODE;
        used += cbl;
    }
    enc.assign((const char *)p, used);
    enc[12] = noop ? 1 : 0;
    if (!noop) enc[13] = exec_off == NONE32 ? 1 : 0;
    return (long)used;
}

static inline size_t slot_of(uint64_t h, size_t mask) { return (size_t)((h * 0xD6E8FEB86659FD93ull) >> 20) & mask; }

const ValueTable::Rec *ValueTable::Shard::find(uint64_t h) const
{
    if (slot.empty()) return nullptr;
    const uint64_t gk = h >> GSH;
    const size_t mask = slot.size() - 1;
    for (size_t i = slot_of(gk, mask);; i = (i + 1) & mask) {
        if (slot[i].key == gk) {
            const Rec *r = &slot[i].g->r[h & (GN - 1)];
            return r->p ? r : nullptr;
        }
        if (slot[i].key == EMPTY) return nullptr;
    }
}

ValueTable::Rec *ValueTable::Shard::insert(uint64_t h, bool &fresh)
{
    const uint64_t gk = h >> GSH;
    if (2 * (count + 1) > slot.size()) {                      // grow: at most half full
        std::vector<GSlot> s2(slot.empty() ? 256 : 2 * slot.size(), GSlot{EMPTY, nullptr});
        const size_t m2 = s2.size() - 1;
        for (const GSlot &x : slot) {
            if (x.key == EMPTY) continue;
            size_t j = slot_of(x.key, m2);
            while (s2[j].key != EMPTY) j = (j + 1) & m2;
            s2[j] = x;
        }
        slot.swap(s2);
        sp.store(slot.data(), std::memory_order_relaxed);
        smask.store(m2, std::memory_order_relaxed);
    }
    const size_t mask = slot.size() - 1;
    size_t i = slot_of(gk, mask);
    while (slot[i].key != EMPTY && slot[i].key != gk) i = (i + 1) & mask;
    if (slot[i].key == EMPTY) {
        constexpr size_t CHUNK = 1024;                        // groups per chunk (384 KiB)
        if (gchunks.empty() || gused == CHUNK) { gchunks.emplace_back(new Group[CHUNK]()); gused = 0; }
        slot[i] = GSlot{gk, &gchunks.back()[gused++]};
        ++count;
    }
    Rec *r = &slot[i].g->r[h & (GN - 1)];
    fresh = r->p == nullptr;
    return r;
}

void ValueTable::prefetch_slot(uint64_t h) const
{
    const Shard &x = sh[shard_of(h)];
    const GSlot *s = x.sp.load(std::memory_order_relaxed);
    if (s) __builtin_prefetch(s + slot_of(h >> GSH, x.smask.load(std::memory_order_relaxed)));
}

// one Value into its (locked) shard
static int intern_locked(ValueTable::Shard &x, uint64_t h, const char *b, uint32_t len, uint32_t exec_off, uint32_t exec_len)
{
    constexpr size_t BLOCK = ValueTable::BLOCK;
    bool fresh = false;
    ValueTable::Rec *r = x.insert(h, fresh);
    if (!fresh) return r->len != len || std::memcmp(r->p, b, len) != 0 ? MPX_E_VALUE : MPX_OK;
    char *dst;
    if (len > BLOCK / 4) {                                   // (a long value: a block of its own)
        x.blocks.emplace_back(new char[len]);
        dst = x.blocks.back().get();
        if (x.blocks.size() > 1) std::swap(x.blocks.back(), x.blocks[x.blocks.size() - 2]);   // (the arena block stays last)
    } else {
        if (x.used + len > BLOCK || x.blocks.empty()) { x.blocks.emplace_back(new char[BLOCK]); x.used = 0; }
        dst = x.blocks.back().get() + x.used;
        x.used += len;
    }
    std::memcpy(dst, b, len);
    r->p = dst; r->len = len; r->exec_off = exec_off; r->exec_len = exec_len;
    return MPX_OK;
}

int ValueTable::intern_batch(const Pending *v, size_t n)
{
    for (size_t i = 0; i < n;) {
        const uint32_t s = shard_of(v[i].h);
        Shard &x = sh[s];
        std::lock_guard<std::mutex> g(x.mu);
        for (; i < n && shard_of(v[i].h) == s; ++i)
            if (int rc = intern_locked(x, v[i].h, v[i].b, v[i].len, v[i].exec_off, v[i].exec_len)) return rc;
    }
    return MPX_OK;
}

int ValueTable::intern(uint64_t h, const char *b, uint32_t len, uint32_t exec_off, uint32_t exec_len)
{
    Shard &x = sh[shard_of(h)];
    std::lock_guard<std::mutex> g(x.mu);
    return intern_locked(x, h, b, len, exec_off, exec_len);
}

// the key of a section: its length and sampled bytes (the candidates are compared in full)
static uint64_t section_key(const uint8_t *b, size_t len, bool with_pid)
{
    uint64_t h = (len * 0x9E3779B97F4A7C15ull) ^ (with_pid ? 0x5851F42D4C957F2Dull : 0);
    auto mix = [&](uint64_t x) { h ^= x; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 31; };
    const size_t k = len < 64 ? len / 8 : 8;
    for (size_t i = 0; i < k; ++i) { uint64_t x; std::memcpy(&x, b + 8 * i, 8); mix(x); }
    for (size_t i = 0; len >= 128 && i < 8; ++i) { uint64_t x; std::memcpy(&x, b + len - 64 + 8 * i, 8); mix(x); }
    return h;
}

SectionCache::Result *SectionCache::claim(const uint8_t *b, size_t len, bool with_pid, bool &own)
{
    const uint64_t key = section_key(b, len, with_pid);
    Shard &x = sh[(key * 0x9E3779B97F4A7C15ull) >> 58];
    // candidates under the lock, the full compares outside it (Results are never removed while
    // the cache lives; two threads that both miss a new section both decode it — equal results)
    Result *cand[8];
    uint32_t nc = 0;
    bool more = false;
    {
        std::lock_guard<std::mutex> g(x.mu);
        auto r = x.m.equal_range(key);
        for (auto it = r.first; it != r.second; ++it) {
            if (nc == 8) { more = true; break; }
            cand[nc++] = it->second.get();
        }
    }
    auto match = [&](const Result *c) {
        return c->len == len && c->with_pid == with_pid && (c->b == b || std::memcmp(c->b, b, len) == 0);
    };
    for (uint32_t k = 0; k < nc; ++k)
        if (match(cand[k])) { own = false; return cand[k]; }
    std::lock_guard<std::mutex> g(x.mu);
    if (more) {                                           // (a crowded key: compare the rest under the lock)
        auto r = x.m.equal_range(key);
        for (auto it = r.first; it != r.second; ++it)
            if (match(it->second.get())) { own = false; return it->second.get(); }
    }
    std::unique_ptr<Result> res(new Result());
    res->b = b; res->len = len; res->with_pid = with_pid;
    res->id = id_base + next_id.fetch_add(1, std::memory_order_relaxed);
    Result *out = res.get();
    x.m.emplace(key, std::move(res));
    own = true;
    return out;
}

// One Value's handle, length and kind off the wire without the table (a section another thread
// interns): the same layout checks as ValueTable::parse, FillValue / ExtractValue
// (multi/paxos.cpp:556-644; member Value_m, member/paxos.cpp:330-408)
static long skim(const uint8_t *p, size_t avail, bool member, uint64_t *handle, bool *mem)
{
    if (avail < 13) return MPX_E_DECODE;
    const uint32_t proposer = rd32(p);
    const uint64_t value_id = rd64(p + 4);
    if (proposer >= (1u << 14) || value_id >= (1ull << 47)) return MPX_E_RANGE;
    const bool noop = p[12] != 0;
    *handle = MPX_HANDLE(proposer, noop, value_id);
    if (mem) *mem = false;
    if (noop) return 13;
    if (avail < 14) return MPX_E_DECODE;
    const bool m = p[13] != 0;
    if (member) {
        if (avail < 18) return MPX_E_DECODE;
        const uint32_t n = rd32(p + 14);
        size_t used = 18;
        if (m) { if ((avail - used) / 8 < n) return MPX_E_DECODE; used += 8 * (size_t)n; }
        else { if (avail - used < n) return MPX_E_DECODE; used += n; }
        if (avail - used < 4) return MPX_E_DECODE;
        const uint32_t cbl = rd32(p + used);
        used += 4;
        if (avail - used < cbl) return MPX_E_DECODE;
        if (mem) *mem = m;
        return (long)(used + cbl);
    }
    if (m) {
        if (avail < 19) return MPX_E_DECODE;
        if (p[18] == 0) return 19;
        if (avail < 23) return MPX_E_DECODE;
        const uint32_t iplen = rd32(p + 19);
        if (avail < 25 + (size_t)iplen) return MPX_E_DECODE;
        return (long)(25 + iplen);
    }
    if (avail < 18) return MPX_E_DECODE;
    const uint32_t len = rd32(p + 14);
    if (avail < 18 + (size_t)len) return MPX_E_DECODE;
    return (long)(18 + len);
}

long ValueTable::parse(const uint8_t *p, size_t avail, uint64_t *handle, bool *mem)
{
    // FillValue / ExtractValue layout, multi/paxos.cpp:556-644
    if (avail < 13) return MPX_E_DECODE;
    if (mem) *mem = false;
    if (member) {
        const uint32_t proposer = rd32(p);
        const uint64_t value_id = rd64(p + 4);
        if (proposer >= (1u << 14) || value_id >= (1ull << 47)) return MPX_E_RANGE;
        std::string enc;
        uint32_t eo, el;
        const long used = parse_member(p, avail, enc, eo, el);
        if (used < 0) return used;
        const uint64_t h = MPX_HANDLE(proposer, p[12] != 0, value_id);
        TRY_RC(intern(h, enc.data(), (uint32_t)enc.size(), eo, el));
        if (mem) *mem = eo == NONE32;
        *handle = h;
        return used;
    }
    const uint32_t proposer = rd32(p);
    const uint64_t value_id = rd64(p + 4);
    const bool noop = p[12] != 0;
    if (proposer >= (1u << 14) || value_id >= (1ull << 47)) return MPX_E_RANGE;
    {
        // the canonical bytes are the wire bytes themselves when every bool is 0 / 1 (a plain
        // payload Value or a noop): compare / append the span, no encoding buffer
        size_t used = 0;
        uint32_t eo = 0, el = 0;
        if (p[12] == 1) used = 13;
        else if (p[12] == 0 && avail >= 18 && p[13] == 0) {
            el = rd32(p + 14);
            if (avail < 18 + (size_t)el) return MPX_E_DECODE;
            used = 18 + el;
            eo = 18;
        }
        if (used) {
            const uint64_t h = MPX_HANDLE(proposer, noop, value_id);
            TRY_RC(intern(h, (const char *)p, (uint32_t)used, eo, el));
            *handle = h;
            return (long)used;
        }
    }
    std::string enc;
    enc.reserve(32);
    app<uint32_t>(enc, proposer);
    app<uint64_t>(enc, value_id);
    app<uint8_t>(enc, noop ? 1 : 0);
    size_t used;
    uint32_t exec_off = 0, exec_len = 0;
    if (noop) {
        used = 13;
    } else {
        if (avail < 14) return MPX_E_DECODE;
        const bool member = p[13] != 0;
        app<uint8_t>(enc, member ? 1 : 0);
        if (member) {
            if (avail < 19) return MPX_E_DECODE;
            app<uint32_t>(enc, rd32(p + 14));
            const bool add = p[18] != 0;
            app<uint8_t>(enc, add ? 1 : 0);
            if (add) {
                if (avail < 23) return MPX_E_DECODE;
                const uint32_t iplen = rd32(p + 19);
                if (avail < 25 + (size_t)iplen) return MPX_E_DECODE;
                app<uint32_t>(enc, iplen);
                enc.append((const char *)p + 23, iplen);
                enc.append((const char *)p + 23 + iplen, 2);
                used = 25 + iplen;
            } else {
                used = 19;
            }
        } else {
            if (avail < 18) return MPX_E_DECODE;
            const uint32_t len = rd32(p + 14);
            if (avail < 18 + (size_t)len) return MPX_E_DECODE;
            app<uint32_t>(enc, len);
            exec_off = (uint32_t)enc.size();
            exec_len = len;
            enc.append((const char *)p + 18, len);
            used = 18 + len;
        }
    }
    const uint64_t h = MPX_HANDLE(proposer, noop, value_id);
    TRY_RC(intern(h, enc.data(), (uint32_t)enc.size(), exec_off, exec_len));
    *handle = h;
    return (long)used;
}

int ValueTable::plain(uint64_t h)
{
    {
        Shard &x = sh[shard_of(h)];
        std::lock_guard<std::mutex> g(x.mu);
        if (x.find(h)) return MPX_OK;
    }
    if (MPX_HANDLE_PROPOSER(h) >= (1u << 14) || (h & MPX_PRESENT)) return MPX_E_RANGE;
    // the canonical bytes of Value(proposer, value_id, noop) with an empty payload (FillValue,
    // multi/paxos.cpp:567-599; member Value_m adds the callback length, :321-408)
    std::string enc;
    app<uint32_t>(enc, MPX_HANDLE_PROPOSER(h));
    app<uint64_t>(enc, MPX_HANDLE_VALUE_ID(h));
    app<uint8_t>(enc, MPX_HANDLE_NOOP(h) ? 1 : 0);
    uint32_t eo = 0;
    if (!MPX_HANDLE_NOOP(h)) {
        app<uint8_t>(enc, 0);
        app<uint32_t>(enc, 0);
        eo = (uint32_t)enc.size();
        if (member) app<uint32_t>(enc, 0);
    }
    return intern(h, enc.data(), (uint32_t)enc.size(), eo, 0);
}

// NodeImpl::ChangeMemberships (member/paxos.cpp:1864-1964) on a node's view: the six change
// types, version_ bumped by each acceptor change; a change the reference ASSERTs on (adding a
// member twice, removing an absent one, the last acceptor) is refused (MPX_E_STATE)
static int change_memberships(mpx_epoch &v, const std::vector<std::pair<uint32_t, uint32_t>> &ch)
{
    enum { ADD_LEARNER, LEARNER_TO_PROPOSER, PROPOSER_TO_ACCEPTOR, DEL_LEARNER, PROPOSER_TO_LEARNER, ACCEPTOR_TO_PROPOSER };
    for (const auto &c : ch) {
        if (c.first >= 64) return MPX_E_RANGE;
        const uint64_t b = 1ull << c.first;
        switch (c.second) {
        case ADD_LEARNER: if (v.learner_mask & b) return MPX_E_STATE; v.learner_mask |= b; break;          // :1872-1880
        case LEARNER_TO_PROPOSER: if (v.proposer_mask & b) return MPX_E_STATE; v.proposer_mask |= b; break;   // :1881-1892
        case PROPOSER_TO_ACCEPTOR: if (v.acceptor_mask & b) return MPX_E_STATE; v.acceptor_mask |= b; ++v.version; break;   // :1893-1905
        case DEL_LEARNER: if (!(v.learner_mask & b)) return MPX_E_STATE; v.learner_mask &= ~b; break;      // :1906-1915
        case PROPOSER_TO_LEARNER: if (!(v.proposer_mask & b)) return MPX_E_STATE; v.proposer_mask &= ~b; break;   // :1916-1943
        case ACCEPTOR_TO_PROPOSER:                                                                          // :1944-1960
            if (!(v.acceptor_mask & b) || v.acceptor_mask == b) return MPX_E_STATE;
            v.acceptor_mask &= ~b; ++v.version; break;
        default: return MPX_E_DECODE;
        }
    }
    return MPX_OK;
}

bool ValueTable::encode(uint64_t h, std::string &out) const
{
    if (const Rec *r = find(h)) {
        out.append(r->p, r->len);
        return true;
    }
    if (synthetic_clean && MPX_HANDLE_PROPOSER(h) == 0 && !MPX_HANDLE_NOOP(h)) {
        const std::string s = std::to_string(MPX_HANDLE_VALUE_ID(h) - 1);
        app<uint32_t>(out, 0); app<uint64_t>(out, MPX_HANDLE_VALUE_ID(h));
        app<uint8_t>(out, 0); app<uint8_t>(out, 0);
        app<uint32_t>(out, (uint32_t)s.size());
        out += s;
        return true;
    }
    return false;
}

bool ValueTable::exec_payload(uint64_t h, std::string &out) const
{
    if (const Rec *r = find(h)) {
        if (r->exec_off == NONE32) return false;             // member: ChangeMemberships
        out.assign(r->p + r->exec_off, r->exec_len);
        return true;
    }
    if (synthetic_clean && MPX_HANDLE_PROPOSER(h) == 0 && !MPX_HANDLE_NOOP(h)) {
        out = std::to_string(MPX_HANDLE_VALUE_ID(h) - 1);
        return true;
    }
    return false;
}

static void flag(IngestViolation &v, uint64_t code, uint64_t node, uint64_t seq, uint64_t iid)
{
    v.count++;
    if (!v.code) { v.code = code; v.node = node; v.seq = seq; v.iid = iid; }
}

static bool sort_entries(std::vector<uint64_t> &iid, std::vector<uint64_t> &pid, std::vector<uint64_t> &val,
                         size_t first, bool with_pid);

// entries {u64 iid, [u64 pid,] Value}* of an ACCEPT / COMMIT / P_BATCH /
// PREPARE_REPLY body, sorted by iid (the reference's std::map order)
// One Value off the wire for the batched intern: its handle, length, executed span and whether
// its canonical bytes are the wire bytes themselves (every bool 0 / 1 and no membership change in
// the multi codec); 0 when the caller must take ValueTable::parse instead, < 0 on a bad layout
static long value_span(const uint8_t *p, size_t avail, bool member, ValueTable::Pending &v, bool &mem)
{
    if (avail < 13) return 0;
    const uint32_t proposer = rd32(p);
    const uint64_t value_id = rd64(p + 4);
    if (proposer >= (1u << 14) || value_id >= (1ull << 47)) return 0;
    mem = false;
    v.h = MPX_HANDLE(proposer, p[12] != 0, value_id);
    v.b = (const char *)p;
    v.exec_off = v.exec_len = 0;
    if (p[12] == 1) { v.len = 13; return 13; }
    if (p[12] != 0 || avail < 18 || p[13] > 1) return 0;
    const uint32_t n = rd32(p + 14);
    if (!member) {
        if (p[13] != 0 || avail - 18 < n) return 0;
        v.len = 18 + n; v.exec_off = 18; v.exec_len = n;
        return (long)v.len;
    }
    size_t used = 18;
    if (p[13]) { if ((avail - used) / 8 < n) return 0; used += 8 * (size_t)n; v.exec_off = NONE32; mem = true; }
    else { if (avail - used < n) return 0; v.exec_off = 18; v.exec_len = n; used += n; }
    if (avail - used < 4) return 0;
    const uint32_t cbl = rd32(p + used);
    used += 4;
    if (avail - used < cbl) return 0;
    v.len = (uint32_t)(used + cbl);
    return (long)v.len;
}

// entries {u64 iid, [u64 pid,] Value}* of one section appended and sorted; `own`: intern the
// Values (else skim them off the wire)
static int parse_section(ValueTable &vt, const uint8_t *b, size_t len, bool with_pid, bool own,
                         std::vector<uint64_t> &iid, std::vector<uint64_t> &pid, std::vector<uint64_t> &val,
                         size_t &n_all, bool &dup, std::vector<std::pair<uint64_t, const uint8_t *>> *memh)
{
    size_t cur = 0;
    const size_t first = iid.size();
    n_all = 0;
    if (own && len >= 512) {                          // touch the Values' table slots first (see prefetch_slot)
        uint64_t last = ValueTable::EMPTY;
        for (size_t c = 0; c < len;) {
            const size_t need = with_pid ? 16 : 8;
            if (len - c < need) break;
            c += need;
            uint64_t h;
            const long u = skim(b + c, len - c, vt.member, &h, nullptr);
            if (u < 0) break;                             // (the decode below reports it)
            if ((h >> ValueTable::GSH) != last) vt.prefetch_slot(h);
            last = h >> ValueTable::GSH;
            c += (size_t)u;
        }
    }
    // own: Values whose canonical bytes are their wire bytes go to the table in batches (one lock
    // per shard run, intern_batch); the rest one by one (ValueTable::parse)
    ValueTable::Pending pend[64];
    size_t np = 0;
    while (cur < len) {
        const size_t need = with_pid ? 16 : 8;
        if (len - cur < need) return MPX_E_DECODE;
        const uint64_t i = rd64(b + cur);
        const uint64_t pd = with_pid ? rd64(b + cur + 8) : 0;
        cur += need;
        uint64_t h;
        bool mem = false;
        long u;
        if (own) {
            u = value_span(b + cur, len - cur, vt.member, pend[np], mem);
            if (u > 0) {
                h = pend[np].h;
                if (++np == 64) { TRY_RC(vt.intern_batch(pend, np)); np = 0; }
            } else {
                if (np) { TRY_RC(vt.intern_batch(pend, np)); np = 0; }   // (table order: as the wire)
                u = vt.parse(b + cur, len - cur, &h, &mem);
            }
        } else {
            u = skim(b + cur, len - cur, vt.member, &h, &mem);
        }
        if (u < 0) return (int)u;
        if (mem && memh) memh->push_back({h, b + cur});   // (member membership Values: MPX_FLAG_LEARN_EPOCHS)
        cur += (size_t)u;
        iid.push_back(i);
        if (with_pid) pid.push_back(pd);
        val.push_back(h);
        ++n_all;
    }
    if (np) TRY_RC(vt.intern_batch(pend, np));
    dup = sort_entries(iid, pid, val, first, with_pid);
    return MPX_OK;
}

// decode a section for its first claimer: its Result (or its error) for every other one
static void publish_section(ValueTable &vt, SectionCache &sc, SectionCache::Result *r)
{
    std::vector<std::pair<uint64_t, const uint8_t *>> mh;
    r->rc = parse_section(vt, r->b, r->len, r->with_pid, true, r->iid, r->pid, r->val, r->n_all, r->dup,
                          vt.member ? &mh : nullptr);
    for (const auto &x : mh) r->memh.push_back({x.first, (uint32_t)(x.second - r->b)});
    if (!r->rc && !sc.share) return;                  // (never marked ready: others skim)
    r->ready.store(1, std::memory_order_release);
}

// entries {u64 iid, [u64 pid,] Value}* of an ACCEPT / COMMIT / P_BATCH / PREPARE_REPLY body,
// sorted by iid (the reference's std::map order); with `sc`, from the section's Result when it is
// ready, else decoded (and published by the first claimer)
#ifdef MPX_DECODE_PROF
}  // namespace mpx
#include <x86intrin.h>
namespace mpx {
std::atomic<uint64_t> g_prof[8];                    // claim, own parse, skim, copy, no-cache parse (cycles); counts
struct ProfT { uint64_t t = __rdtsc(); int k; explicit ProfT(int k_) : k(k_) {} ~ProfT() { g_prof[k] += __rdtsc() - t; } };
#define PROF(k) ProfT prof_##k(k)
#else
#define PROF(k)
#endif
static int decode_entries(ValueTable &vt, const uint8_t *b, size_t len, bool with_pid,
                          std::vector<uint64_t> &iid, std::vector<uint64_t> &pid,
                          std::vector<uint64_t> &val, size_t &n_all, bool &dup,
                          std::vector<std::pair<uint64_t, const uint8_t *>> *memh = nullptr, SectionCache *sc = nullptr,
                          uint64_t *sec = nullptr)
{
    if (!sc || !len) { PROF(4); return parse_section(vt, b, len, with_pid, true, iid, pid, val, n_all, dup, memh); }
    bool own = false;
    SectionCache::Result *r;
    { PROF(0); r = sc->claim(b, len, with_pid, own); }
    if (sec) *sec = r->id;
    if (own) { PROF(1); publish_section(vt, *sc, r); }
    if (!r->ready.load(std::memory_order_acquire)) {  // (claimed elsewhere, not decoded yet: skim)
        PROF(2);
        return parse_section(vt, b, len, with_pid, false, iid, pid, val, n_all, dup, memh);
    }
    if (r->rc) return r->rc;
    PROF(3);
    iid.insert(iid.end(), r->iid.begin(), r->iid.end());
    if (with_pid) pid.insert(pid.end(), r->pid.begin(), r->pid.end());
    val.insert(val.end(), r->val.begin(), r->val.end());
    if (memh) for (const auto &x : r->memh) memh->push_back({x.first, b + x.second});
    n_all = r->n_all;
    dup = r->dup;
    return MPX_OK;
}

// sort one message's entries [first, end) by iid (stable permutation); true when an
// iid repeats (the reference ASSERTs, multi/paxos.cpp:552)
static bool sort_entries(std::vector<uint64_t> &iid, std::vector<uint64_t> &pid, std::vector<uint64_t> &val,
                         size_t first, bool with_pid)
{
    const size_t n = iid.size() - first;
    bool sorted = true;
    for (size_t k = first + 1; k < iid.size(); ++k)
        if (iid[k - 1] >= iid[k]) { sorted = false; break; }
    if (!sorted) {
        std::vector<size_t> perm(n);
        for (size_t k = 0; k < n; ++k) perm[k] = first + k;
        std::stable_sort(perm.begin(), perm.end(), [&](size_t a, size_t c) { return iid[a] < iid[c]; });
        std::vector<uint64_t> ti(n), tp(with_pid ? n : 0), tv(n);
        for (size_t k = 0; k < n; ++k) {
            ti[k] = iid[perm[k]]; tv[k] = val[perm[k]];
            if (with_pid) tp[k] = pid[perm[k]];
        }
        for (size_t k = 0; k < n; ++k) {
            iid[first + k] = ti[k]; val[first + k] = tv[k];
            if (with_pid) pid[first + k] = tp[k];
        }
        for (size_t k = first + 1; k < iid.size(); ++k)
            if (iid[k - 1] == iid[k]) return true;
    }
    return false;
}

int decode_record(ValueTable &vt, NodeStream &ns, uint32_t node, uint32_t N, const uint8_t *m, size_t len,
                  uint64_t sb, uint64_t se, IngestViolation &viol, SectionCache *sc)
{
    if (len < 4) return MPX_E_DECODE;
    const uint32_t t = rd32(m);
    const uint64_t seq = ns.type.size();
    uint32_t src = 0;
    uint64_t ballot = 0, aux = 0, ent = 0;
    uint32_t cnt = 0;
    uint8_t part = 0;
    uint64_t sec = 0;                             // (SectionCache) the value section's id                             // entries, none in the shard: another rank's record
    (void)N;
    auto keep_shard = [&](std::vector<uint64_t> &iid, std::vector<uint64_t> *pid, std::vector<uint64_t> &val,
                          size_t first) {
        // drop entries outside this engine's shard (headers stay: SURVEY §8(e)); entries are sorted,
        // so a list inside the shard is kept as it is (no pass over it)
        if (iid.size() == first || (iid[first] >= sb && iid.back() < se)) return iid.size() - first;
        size_t w = first;
        for (size_t k = first; k < iid.size(); ++k) {
            if (iid[k] >= sb && iid[k] < se) {
                iid[w] = iid[k]; val[w] = val[k];
                if (pid) (*pid)[w] = (*pid)[k];
                ++w;
            }
        }
        iid.resize(w); val.resize(w);
        if (pid) pid->resize(w);
        return w - first;
    };
    switch (t) {
    case MPX_MSG_PREPARE: {                       // multi/paxos.cpp:741-755
        if (len < 20) return MPX_E_DECODE;
        src = rd32(m + 4); ballot = rd64(m + 8);
        const uint32_t rl = rd32(m + 16);
        if (rl % 16 || 20 + (size_t)rl > len) return MPX_E_DECODE;
        ent = ns.g_a.size();
        const uint32_t nr = rl / 16;
        std::vector<std::pair<uint64_t, uint64_t>> r(nr);
        for (uint32_t k = 0; k < nr; ++k) r[k] = {rd64(m + 20 + 16 * k), rd64(m + 28 + 16 * k)};
        std::sort(r.begin(), r.end());            // std::set order (:533-537)
        // The kernel binary-searches disjoint ranges: drop empty ones and
        // merge overlaps (the reference returns an entry once per covering
        // range and ASSERTs on the duplicate, :909; a repeated pair is an
        // ASSERT in ExtractAvailableInstanceIDs, :536).
        cnt = 0;
        for (uint32_t k = 0; k < nr; ++k) {
            if (k && r[k] == r[k - 1]) flag(viol, MPX_V_DUP_IID, node, seq, r[k].first);
            if (r[k].first >= r[k].second) continue;
            if (cnt && r[k].first < ns.g_b.back()) {
                ns.g_b.back() = std::max(ns.g_b.back(), r[k].second);
                continue;
            }
            ns.g_a.push_back(r[k].first);
            ns.g_b.push_back(r[k].second);
            ++cnt;
        }
        break;
    }
    case MPX_MSG_PREPARE_REPLY: {                 // :830-844
        if (len < 20) return MPX_E_DECODE;
        src = rd32(m + 4); ballot = rd64(m + 8);
        const uint32_t vl = rd32(m + 16);
        if (20 + (size_t)vl > len) return MPX_E_DECODE;
        const size_t first = ns.r_iid.size();
        size_t n_all; bool dup;
        int rc = decode_entries(vt, m + 20, vl, true, ns.r_iid, ns.r_pid, ns.r_val, n_all, dup);   // (unique per reply: no section cache)
        if (rc) return rc;
        if (dup) flag(viol, MPX_V_DUP_IID, node, seq, 0);
        ent = first;
        cnt = (uint32_t)keep_shard(ns.r_iid, &ns.r_pid, ns.r_val, first);
        break;
    }
    case MPX_MSG_REJECT:                          // :846-856
        if (len < 12) return MPX_E_DECODE;
        ballot = rd64(m + 4);
        break;
    case MPX_MSG_ACCEPT:                          // :1282-1297
    case MPX_MSG_COMMIT: {                        // :1429-1444
        if (len < 28) return MPX_E_DECODE;
        src = rd32(m + 4); aux = rd64(m + 8); ballot = rd64(m + 16);
        const uint32_t vl = rd32(m + 24);
        if (28 + (size_t)vl > len) return MPX_E_DECODE;
        const size_t first = ns.e_iid.size();
        size_t n_all; bool dup;
        std::vector<uint64_t> nopid;
        int rc = decode_entries(vt, m + 28, vl, false, ns.e_iid, nopid, ns.e_val, n_all, dup, nullptr, sc, &sec);
        if (rc) return rc;
        if (dup) flag(viol, MPX_V_DUP_IID, node, seq, 0);
        ent = first;
        cnt = (uint32_t)keep_shard(ns.e_iid, nullptr, ns.e_val, first);
        part = n_all && !cnt;
        break;
    }
    case MPX_MSG_ACCEPT_REPLY:                    // :1345-1357
        if (len < 24) return MPX_E_DECODE;
        src = rd32(m + 4); ballot = rd64(m + 8); aux = rd64(m + 16);
        break;
    case MPX_MSG_COMMIT_REPLY:                    // :1481-1492
        if (len < 16) return MPX_E_DECODE;
        src = rd32(m + 4); aux = rd64(m + 8);
        break;
    case MPX_MSG_P_START:
        if (len < 12) return MPX_E_DECODE;
        ballot = rd64(m + 4);
        break;
    case MPX_MSG_P_PROPOSE:                       // Propose (:1250-1280): the proposer's bookkeeping only
        if (len < 8 || 8 + (size_t)rd32(m + 4) > len) return MPX_E_DECODE;
        break;
    case MPX_MSG_P_BATCH: {
        if (len < 16) return MPX_E_DECODE;
        aux = rd64(m + 4);
        const uint32_t vl = rd32(m + 12);
        if (16 + (size_t)vl > len) return MPX_E_DECODE;
        const size_t first = ns.e_iid.size();
        size_t n_all; bool dup;
        std::vector<uint64_t> nopid;
        int rc = decode_entries(vt, m + 16, vl, false, ns.e_iid, nopid, ns.e_val, n_all, dup, nullptr, sc, &sec);
        if (rc) return rc;
        if (dup) flag(viol, MPX_V_DUP_IID, node, seq, 0);
        ent = first;
        cnt = (uint32_t)keep_shard(ns.e_iid, nullptr, ns.e_val, first);
        part = n_all && !cnt;
        break;
    }
    default:
        return MPX_E_DECODE;                      // ASSERT(false), :1671-1672
    }
    ns.part.push_back(part);
    ns.sec.push_back(sec);
    ns.type.push_back((uint8_t)t);
    ns.src.push_back(src);
    ns.ballot.push_back(ballot);
    ns.aux.push_back(aux);
    ns.ent.push_back(ent);
    ns.cnt.push_back(cnt);
    return MPX_OK;
}

int append_record(ValueTable &vt, NodeStream &ns, uint32_t node, const SoaRecord &r, uint64_t sb, uint64_t se,
                  IngestViolation &viol)
{
    const uint32_t t = r.type;
    const uint64_t seq = ns.type.size();
    uint64_t ent = 0;
    uint32_t cnt = 0;
    uint8_t part = 0;
    uint64_t sec = 0;                             // (SectionCache) the value section's id
    auto values = [&]() -> int {
        for (uint64_t k = 0; k < r.n; ++k) TRY_RC(vt.plain(r.b[k]));
        return MPX_OK;
    };
    auto keep = [&](std::vector<uint64_t> &iid, std::vector<uint64_t> *pid, std::vector<uint64_t> &val, size_t first) {
        size_t w = first;
        for (size_t k = first; k < iid.size(); ++k)
            if (iid[k] >= sb && iid[k] < se) {
                iid[w] = iid[k]; val[w] = val[k];
                if (pid) (*pid)[w] = (*pid)[k];
                ++w;
            }
        iid.resize(w); val.resize(w);
        if (pid) pid->resize(w);
        return (uint32_t)(w - first);
    };
    switch (t) {
    case MPX_MSG_PREPARE: {                       // ranges [a, b), as decode_record
        ent = ns.g_a.size();
        std::vector<std::pair<uint64_t, uint64_t>> g(r.n);
        for (uint64_t k = 0; k < r.n; ++k) g[k] = {r.a[k], r.b[k]};
        std::sort(g.begin(), g.end());
        for (uint64_t k = 0; k < r.n; ++k) {
            if (k && g[k] == g[k - 1]) flag(viol, MPX_V_DUP_IID, node, seq, g[k].first);
            if (g[k].first >= g[k].second) continue;
            if (cnt && g[k].first < ns.g_b.back()) { ns.g_b.back() = std::max(ns.g_b.back(), g[k].second); continue; }
            ns.g_a.push_back(g[k].first); ns.g_b.push_back(g[k].second);
            ++cnt;
        }
        break;
    }
    case MPX_MSG_PREPARE_REPLY: {
        TRY_RC(values());
        const size_t first = ns.r_iid.size();
        for (uint64_t k = 0; k < r.n; ++k) {
            ns.r_iid.push_back(r.a[k]); ns.r_val.push_back(r.b[k]); ns.r_pid.push_back(r.pid ? r.pid[k] : 0);
        }
        if (sort_entries(ns.r_iid, ns.r_pid, ns.r_val, first, true)) flag(viol, MPX_V_DUP_IID, node, seq, 0);
        ent = first;
        cnt = keep(ns.r_iid, &ns.r_pid, ns.r_val, first);
        break;
    }
    case MPX_MSG_ACCEPT: case MPX_MSG_COMMIT: case MPX_MSG_P_BATCH: {
        TRY_RC(values());
        const size_t first = ns.e_iid.size();
        std::vector<uint64_t> nopid;
        for (uint64_t k = 0; k < r.n; ++k) { ns.e_iid.push_back(r.a[k]); ns.e_val.push_back(r.b[k]); }
        if (sort_entries(ns.e_iid, nopid, ns.e_val, first, false)) flag(viol, MPX_V_DUP_IID, node, seq, 0);
        ent = first;
        cnt = keep(ns.e_iid, nullptr, ns.e_val, first);
        part = r.n && !cnt;
        break;
    }
    case MPX_MSG_REJECT: case MPX_MSG_ACCEPT_REPLY: case MPX_MSG_COMMIT_REPLY: case MPX_MSG_P_START:
    case MPX_MSG_P_PROPOSE:
        break;
    default:
        return MPX_E_DECODE;
    }
    ns.part.push_back(part);
    ns.sec.push_back(sec);
    ns.type.push_back((uint8_t)t);
    ns.src.push_back(r.src);
    ns.ballot.push_back(r.ballot);
    ns.aux.push_back(r.aux);
    ns.ent.push_back(ent);
    ns.cnt.push_back(cnt);
    return MPX_OK;
}

int decode_record_member(ValueTable &vt, NodeStream &ns, uint32_t node, const uint8_t *m, size_t len,
                         uint64_t sb, uint64_t se, IngestViolation &viol, EpochLearn *el, SectionCache *sc)
{
    if (len < 4) return MPX_E_DECODE;
    const uint32_t t = rd32(m);
    const uint64_t seq = ns.type.size();
    uint32_t src = 0, ver = 0;
    uint64_t ballot = 0, aux = 0, ent = 0;
    uint32_t cnt = 0;
    uint8_t part = 0;
    uint64_t sec = 0;                             // (SectionCache) the value section's id
    auto keep_shard = [&](size_t first) {
        if (ns.e_iid.size() == first || (ns.e_iid[first] >= sb && ns.e_iid.back() < se))
            return (uint32_t)(ns.e_iid.size() - first);          // (sorted, inside the shard: kept as it is)
        size_t w = first;
        for (size_t k = first; k < ns.e_iid.size(); ++k)
            if (ns.e_iid[k] >= sb && ns.e_iid[k] < se) {
                ns.e_iid[w] = ns.e_iid[k]; ns.e_val[w] = ns.e_val[k]; ns.e_pid[w] = ns.e_pid[k];
                ++w;
            }
        ns.e_iid.resize(w); ns.e_val.resize(w); ns.e_pid.resize(w);
        return (uint32_t)(w - first);
    };
    std::vector<EpochLearn::Changes> applied;     // (el) the membership Values this LEARN makes the node apply
    // (el) the membership Values among this record's entries and their wire bytes: the change list
    // is read off the wire (the same layout as the canonical bytes, parse_member), not the shared
    // table, which another decode thread may still be filling for this section (SectionCache)
    std::vector<std::pair<uint64_t, const uint8_t *>> memh;
    auto changes_of = [&](uint64_t h, EpochLearn::Changes &ch) {
        for (const auto &x : memh)
            if (x.first == h) {
                const uint32_t n = rd32(x.second + 14);            // (bounds checked by the decode)
                for (uint32_t k = 0; k < n; ++k) ch.emplace_back(rd32(x.second + 18 + 8 * k), rd32(x.second + 22 + 8 * k));
                return true;
            }
        return false;
    };
    // the Learner's apply loop over one LEARN's entries, every instance (not only the shard's)
    auto learn = [&](size_t first, size_t end) {
        for (size_t k = first; k < end; ++k) {
            const uint64_t i = ns.e_iid[k];
            if (i < el->front) continue;                          // applied already (insert: no change)
            EpochLearn::Learned cur{false, {}};
            if (!memh.empty()) cur.mem = changes_of(ns.e_val[k], cur.ch);
            if (i > el->front) { el->above.emplace(i, std::move(cur)); continue; }
            for (;;) {                                            // apply at the frontier, then what waited above it
                if (cur.mem) applied.push_back(std::move(cur.ch));
                ++el->front;
                auto it = el->above.begin();
                if (it == el->above.end() || it->first != el->front) break;
                cur = std::move(it->second);
                el->above.erase(it);
            }
        }
    };
    // {u64 iid, u64 pid, Value_m}* (ExtractProposalValues, member/paxos.cpp:421-433)
    auto entries = [&](const uint8_t *b, size_t l) -> int {
        const size_t first = ns.e_iid.size();
        size_t n_all; bool dup;
        int rc = decode_entries(vt, b, l, true, ns.e_iid, ns.e_pid, ns.e_val, n_all, dup, el ? &memh : nullptr, sc, &sec);
        if (rc) return rc;
        if (dup) flag(viol, MPX_V_DUP_IID, node, seq, 0);
        if (el && t == MPX_MSG_COMMIT) learn(first, ns.e_iid.size());
        ent = first;
        cnt = keep_shard(first);
        part = n_all && !cnt;
        return MPX_OK;
    };
    switch (t) {
    case MPX_MSG_PREPARE: {                       // PrepareMsg, member/paxos.cpp:847-859
        if (len < 24) return MPX_E_DECODE;
        ver = rd32(m + 4); src = rd32(m + 8); ballot = rd64(m + 12);
        const uint32_t rl = rd32(m + 20);
        if (rl % 16 || 24 + (size_t)rl > len) return MPX_E_DECODE;
        ent = ns.g_a.size();
        const uint32_t nr = rl / 16;
        std::vector<std::pair<uint64_t, uint64_t>> r(nr);
        for (uint32_t k = 0; k < nr; ++k) r[k] = {rd64(m + 24 + 16 * k), rd64(m + 32 + 16 * k)};
        std::sort(r.begin(), r.end());
        for (uint32_t k = 0; k < nr; ++k) {
            if (k && r[k] == r[k - 1]) flag(viol, MPX_V_DUP_IID, node, seq, r[k].first);
            if (r[k].first >= r[k].second) continue;
            if (cnt && r[k].first < ns.g_b.back()) { ns.g_b.back() = std::max(ns.g_b.back(), r[k].second); continue; }
            ns.g_a.push_back(r[k].first);
            ns.g_b.push_back(r[k].second);
            ++cnt;
        }
        break;
    }
    case MPX_MSG_PREPARE_REPLY: {                 // PrepareReplyMsg, :861-872
        if (len < 20) return MPX_E_DECODE;
        src = rd32(m + 4); ballot = rd64(m + 8);
        const uint32_t vl = rd32(m + 16);
        if (20 + (size_t)vl > len) return MPX_E_DECODE;
        const size_t first = ns.r_iid.size();
        size_t n_all; bool dup;
        int rc = decode_entries(vt, m + 20, vl, true, ns.r_iid, ns.r_pid, ns.r_val, n_all, dup);   // (unique per reply: no section cache)
        if (rc) return rc;
        if (dup) flag(viol, MPX_V_DUP_IID, node, seq, 0);
        ent = first;
        size_t w = first;
        if (ns.r_iid.size() > first && ns.r_iid[first] >= sb && ns.r_iid.back() < se) w = ns.r_iid.size();
        else for (size_t k = first; k < ns.r_iid.size(); ++k)
            if (ns.r_iid[k] >= sb && ns.r_iid[k] < se) {
                ns.r_iid[w] = ns.r_iid[k]; ns.r_val[w] = ns.r_val[k]; ns.r_pid[w] = ns.r_pid[k];
                ++w;
            }
        ns.r_iid.resize(w); ns.r_val.resize(w); ns.r_pid.resize(w);
        cnt = (uint32_t)(w - first);
        break;
    }
    case MPX_MSG_REJECT:                          // RejectMsg, :874-881
        if (len < 12) return MPX_E_DECODE;
        ballot = rd64(m + 4);
        break;
    case MPX_MSG_ACCEPT: {                        // AcceptMsg, :883-898
        if (len < 32) return MPX_E_DECODE;
        ver = rd32(m + 4); src = rd32(m + 8); aux = rd64(m + 12); ballot = rd64(m + 20);
        const uint32_t vl = rd32(m + 28);
        if (32 + (size_t)vl > len) return MPX_E_DECODE;
        TRY_RC(entries(m + 32, vl));
        break;
    }
    case MPX_MSG_ACCEPT_REPLY:                    // AcceptReplyMsg, :900-908
        if (len < 16) return MPX_E_DECODE;
        src = rd32(m + 4); aux = rd64(m + 8);
        break;
    case MPX_MSG_COMMIT: {                        // LearnMsg, :910-921
        if (len < 20) return MPX_E_DECODE;
        src = rd32(m + 4); aux = rd64(m + 8);
        const uint32_t vl = rd32(m + 16);
        if (20 + (size_t)vl > len) return MPX_E_DECODE;
        TRY_RC(entries(m + 20, vl));
        break;
    }
    case MPX_MSG_COMMIT_REPLY:                    // LearnReplyMsg, :923-931
        if (len < 16) return MPX_E_DECODE;
        src = rd32(m + 4); aux = rd64(m + 8);
        break;
    case MPX_MSG_P_START:
        if (len < 12) return MPX_E_DECODE;
        ballot = rd64(m + 4);
        break;
    case MPX_MSG_P_BATCH: {
        if (len < 16) return MPX_E_DECODE;
        aux = rd64(m + 4);
        const uint32_t vl = rd32(m + 12);
        if (16 + (size_t)vl > len) return MPX_E_DECODE;
        TRY_RC(entries(m + 16, vl));
        break;
    }
    case MPX_MSG_E_EPOCH:
        if (len < 8) return MPX_E_DECODE;
        if (el) return MPX_OK;                    // (learned epochs: the engine places its own)
        ver = rd32(m + 4);
        break;
    case MPX_MSG_P_PROPOSE:                       // Node::Propose (:1984, :1122-1156): bookkeeping only
        if (len < 8 || 8 + (size_t)rd32(m + 4) > len) return MPX_E_DECODE;
        break;
    default:
        return MPX_E_DECODE;
    }
    if ((t == MPX_MSG_PREPARE || t == MPX_MSG_ACCEPT) && ballot > LOW56) return MPX_E_RANGE;   // see G_SEG
    ns.part.push_back(part);
    ns.sec.push_back(sec);
    ns.type.push_back((uint8_t)t);
    ns.src.push_back(src);
    ns.ballot.push_back(ballot);
    ns.aux.push_back(aux);
    ns.ent.push_back(ent);
    ns.cnt.push_back(cnt);
    ns.ver.push_back(ver);
    // the membership Values this LEARN applied, in instance order: one E_EPOCH each, right after
    // it (the reference changes the roles inside OnLearn, before the node's next record)
    for (const auto &ch : applied) {
        TRY_RC(change_memberships(el->view, ch));
        el->steps.push_back(el->view);
        ns.part.push_back(0);
        ns.type.push_back((uint8_t)MPX_MSG_E_EPOCH);
        ns.sec.push_back(0);
        ns.src.push_back(0);
        ns.ballot.push_back(0);
        ns.aux.push_back(0);
        ns.ent.push_back(0);
        ns.cnt.push_back(0);
        ns.ver.push_back((uint32_t)el->steps.size());
    }
    return MPX_OK;
}

// Cut entries [first, first+count) of one message (sorted by iid, inside the
// shard) into per-bucket runs.
template <typename F>
static void cut_runs(const uint64_t *iid, uint64_t first, uint32_t count, uint64_t sb, F &&emit)
{
    uint32_t k = 0;
    while (k < count) {
        const uint64_t b = (iid[first + k] - sb) >> BSH;
        uint32_t e = k + 1;
        while (e < count && ((iid[first + e] - sb) >> BSH) == b) ++e;
        bool dense = true;
        for (uint32_t j = k + 1; j < e; ++j)
            if (iid[first + j] != iid[first + j - 1] + 1) { dense = false; break; }
        emit(b, first + k, e - k, (uint8_t)((iid[first + k] - sb) & (BS - 1)), dense);
        k = e;
    }
}

// Content-addressed entry pool.  A broadcast reaches every node as identical
// bytes (the proposer sends one string to all, multi/paxos.cpp:1322-1323,
// 1474-1476), and a P_BATCH carries the same entries as its ACCEPT; storing
// each distinct entry list once lets the apply kernel read a bucket's Values
// once for all nodes (DESIGN.md §Data layout).  Lists are compared in full,
// the hash only picks the candidates.
// member pools carry a proposal id per entry (e_pid, index-aligned with e_iid / e_val); a
// list without ids (a window's carried batch entries, chosen-log runs only) takes id 0
struct EntryPool {
    bool member = false;
    std::unordered_multimap<uint64_t, uint64_t> idx;    // hash -> offset in ht.e_*
    uint64_t intern(const NodeStream &ns, uint64_t first, uint32_t cnt, HostTrace &ht)
    {
        const bool has = !ns.e_pid.empty();
        auto pid_of = [&](uint32_t i) -> uint64_t { return has ? ns.e_pid[first + i] : 0; };
        // the hash only picks candidates: four independent lanes (no serial multiply chain
        // over the list), folded at the end
        const uint64_t *iv = ns.e_iid.data() + first, *vv = ns.e_val.data() + first;
        uint64_t l[4] = {mix64(cnt + 0x51ull), 0x9E3779B97F4A7C15ull, 0xC2B2AE3D27D4EB4Full, 0x165667B19E3779F9ull};
        for (uint32_t i = 0; i < cnt; ++i) l[i & 3] = (l[i & 3] ^ iv[i]) * 0xff51afd7ed558ccdull + vv[i];
        if (member)
            for (uint32_t i = 0; i < cnt; ++i) l[i & 3] = (l[i & 3] ^ pid_of(i)) * 0xc4ceb9fe1a85ec53ull;
        const uint64_t h = mix64(mix64(mix64(l[0] ^ l[1]) ^ l[2]) ^ l[3]);
        auto r = idx.equal_range(h);
        for (auto it = r.first; it != r.second; ++it) {
            const uint64_t o = it->second;
            if (o + cnt > ht.e_iid.size()) continue;
            bool same = std::memcmp(ht.e_iid.data() + o, iv, 8ull * cnt) == 0 &&
                        std::memcmp(ht.e_val.data() + o, vv, 8ull * cnt) == 0;
            for (uint32_t i = 0; same && member && i < cnt; ++i) same = ht.e_pid[o + i] == pid_of(i);
            if (same) return o;
        }
        const uint64_t o = ht.e_iid.size();
        ht.e_iid.insert(ht.e_iid.end(), ns.e_iid.begin() + first, ns.e_iid.begin() + first + cnt);
        ht.e_val.insert(ht.e_val.end(), ns.e_val.begin() + first, ns.e_val.begin() + first + cnt);
        if (member)
            for (uint32_t i = 0; i < cnt; ++i) ht.e_pid.push_back(pid_of(i));
        idx.emplace(h, o);
        return o;
    }
};

// Per pair of dense accept / commit runs (the pairs k_plan_list can plan): a commit / learn
// (member: also an accept) run whose every slot an earlier commit run of the pair fixed, with
// the same entries (iid, Value, member: proposal id) over its range, names that run's entries
// (the pool's content addressing at bucket-run grain: a re-commit of the same Values through
// another message — another proposer's COMMIT, multi/paxos.cpp:1494-1518 — then shares them);
// a run that still meets a committed slot through another entry with another Value gets FR_VCHK,
// and only those send their pair to the device's Value check (k_commit_check).
static void mark_value_checks(HostTrace &ht, bool member)
{
    const uint64_t NP = (uint64_t)ht.N * ht.NB;
    std::vector<uint32_t> fixr(BS);                   // per slot: pair-local committing run + 1
    for (uint64_t p = 0; p < NP; ++p) {
        const uint64_t f0 = ht.f_off[p], f1 = ht.f_off[p + 1];
        if (f1 - f0 < 2) continue;
        uint32_t commits = 0;
        bool plain = true;
        for (uint64_t f = f0; f < f1 && plain; ++f) {
            const uint32_t kind = ht.frags[f].flags >> 4;
            plain = (ht.frags[f].flags & FR_DENSE) && (kind == K_ACCEPT || kind == K_COMMIT);
            commits += kind == K_COMMIT;
        }
        if (!plain || !commits || (!member && commits < 2)) continue;
        std::fill(fixr.begin(), fixr.end(), 0u);
        for (uint64_t f = f0; f < f1; ++f) {
            Frag &fr = ht.frags[f];
            const bool learn = (fr.flags >> 4) == K_COMMIT;
            const uint32_t st = fr.start, c = fr.count;
            if (!learn && !member) continue;           // multi: an accept over a commit is skipped
            const uint32_t j = fixr[st];
            bool one = j != 0;
            for (uint32_t s = st + 1; one && s < st + c; ++s) one = fixr[s] == j;
            if (one) {
                const Frag &fj = ht.frags[f0 + j - 1];
                const uint64_t base = fj.entry + (st - fj.start);
                if (base != fr.entry) {
                    bool same = true;
                    for (uint32_t d = 0; same && d < c; ++d)
                        same = ht.e_iid[base + d] == ht.e_iid[fr.entry + d] && ht.e_val[base + d] == ht.e_val[fr.entry + d] &&
                               (!member || ht.e_pid[base + d] == ht.e_pid[fr.entry + d]);
                    if (same) fr.entry = base;
                }
            }
            // the device's check compares the Values (k_commit_check: a later run's e_val against the
            // fixing run's); through another entry with the same Value it can never fire, so only a
            // slot whose Values differ sends the pair to it
            bool chk = false;
            for (uint32_t s = st; s < st + c && !chk; ++s)
                if (fixr[s]) {
                    const Frag &fj = ht.frags[f0 + fixr[s] - 1];
                    chk = fj.entry - fj.start != fr.entry - fr.start &&
                          ht.e_val[fj.entry + (s - fj.start)] != ht.e_val[fr.entry + (s - st)];
                }
            if (chk) fr.flags |= FR_VCHK;
            if (learn)
                for (uint32_t s = st; s < st + c; ++s)
                    if (!fixr[s]) fixr[s] = (uint32_t)(f - f0) + 1;
        }
    }
}

namespace {
struct FragKey { uint64_t key; Frag f; };
// a window's carry past one node (committed to the WindowCarry only when the build succeeds)
struct NodeCarry {
    std::unordered_map<uint64_t, uint32_t> live;
    std::vector<uint64_t> round_b;
    int64_t maxb = -1;
    uint64_t ballot = 0;
    uint32_t markers = 0;
};
// what the walk over the nodes' records hands to finish_trace
struct Walk {
    std::vector<uint64_t> fcount, cfcount;        // runs per (bucket, node) pair / per bucket's chosen list
    std::vector<FragKey> fr, cfr;                 // the runs, in walk order
    std::vector<uint32_t> pl;                     // proposer lists (messages)
    std::vector<uint64_t> pl_cnt;
    std::vector<std::pair<uint64_t, uint32_t>> evp;   // snapshot events (pair, message)
    std::vector<uint64_t> evx;
    std::vector<uint64_t> sc_off;
    std::vector<std::vector<uint32_t>> reps;      // per batch: its vote messages
    std::vector<uint64_t> b_bal_w;                // (window) per batch: its round's ballot
    std::vector<std::pair<uint32_t, uint64_t>> state_new;
    std::vector<NodeCarry> next;
    std::vector<uint32_t> ents_gone;
    std::unordered_map<uint32_t, std::vector<std::pair<uint64_t, uint64_t>>> ents_new;
    uint64_t gid_next = 0;
};
}  // namespace

// Everything after the walk over the nodes' records: the vote lists, the run / event CSRs, the
// work lists, the scan chunks, and (a window) the carry, committed only when every check passed.
// FR_VEQ: every slot a commit / learn / accept run covers that an earlier commit / learn of its
// pair fixed holds the same Value through the run's entry (or the same entry). A committed slot's
// entry is its first commit run's in message order — accepts never replace it, member Acceptor
// resets keep it — so this is static, and the walks (k_apply) skip their Value compare there
// (two dependent loads per slot: contended C5's rivals re-learn equal Values under their own ids,
// through other entries, on most slots of their walked pairs).
static void mark_equal_values(HostTrace &ht, uint64_t p0, uint64_t p1)
{
    std::vector<int64_t> fix(BS);
    for (uint64_t p = p0; p < p1; ++p) {
        const uint64_t f0 = ht.f_off[p], f1 = ht.f_off[p + 1];
        std::fill(fix.begin(), fix.end(), -1);
        for (uint64_t f = f0; f < f1; ++f) {
            Frag &fr = ht.frags[f];
            const uint32_t kind = fr.flags >> 4;
            if (kind != K_ACCEPT && kind != K_COMMIT) continue;
            const bool dense = fr.flags & FR_DENSE;
            bool eq = true;
            for (uint32_t d = 0; d < fr.count; ++d) {
                const uint64_t x = fr.entry + d;
                const uint32_t s = dense ? fr.start + d : (uint32_t)((ht.e_iid[x] - ht.shard_begin) & (BS - 1));
                const int64_t j = fix[s];
                if (j >= 0 && (uint64_t)j != x && ht.e_val[j] != ht.e_val[x]) eq = false;
                if (kind == K_COMMIT && j < 0) fix[s] = (int64_t)x;
            }
            if (eq) fr.flags |= FR_VEQ;
        }
    }
}

// FR_UPID / f_pid: a promise-reply run whose entries all carry one proposal id (typically every
// instance of it accepted by one ACCEPT) gives the promise-round walk that id with its descriptor
static void mark_uniform_pids(HostTrace &ht, uint64_t f0, uint64_t f1)
{
    for (uint64_t f = f0; f < f1; ++f) {
        Frag &fr = ht.frags[f];
        if ((fr.flags >> 4) != K_PREPLY || !fr.count) continue;
        const uint64_t p0 = ht.r_pid[fr.entry];
        bool u = true;
        for (uint32_t d = 1; d < fr.count && u; ++d) u = ht.r_pid[fr.entry + d] == p0;
        if (u) { fr.flags |= FR_UPID; ht.f_pid[f] = p0; }
    }
}

static int finish_trace(HostTrace &ht, Walk &W, uint32_t N, uint64_t NB, uint64_t sb, uint64_t slen, bool member,
                        WindowCarry *wc, uint32_t threads)
{
    auto &fcount = W.fcount, &cfcount = W.cfcount;
    auto &fr = W.fr, &cfr = W.cfr;
    auto &pl = W.pl;
    auto &pl_cnt = W.pl_cnt;
    auto &evp = W.evp;
    auto &evx = W.evx;
    auto &sc_off = W.sc_off;
    auto &reps = W.reps;
    auto &b_bal_w = W.b_bal_w;
    auto &state_new = W.state_new;
    auto &next = W.next;
    auto &ents_gone = W.ents_gone;
    auto &ents_new = W.ents_new;
    const uint64_t gid_next = W.gid_next;
    (void)sb;
    // (the CSR scatters and the slot bytes on a few threads: each takes a range of keys and scans
    // the whole list, so every key's items keep their order)
    const uint32_t T = std::max(1u, threads);
    auto parallel = [&](uint32_t count, const auto &fn) {
        std::atomic<uint32_t> next{0};
        auto work = [&]() { for (uint32_t k; (k = next.fetch_add(1)) < count;) fn(k); };
        std::vector<std::thread> th;
        for (uint32_t t = 1; t < std::min(T, count); ++t) th.emplace_back(work);
        work();
        for (auto &x : th) x.join();
    };
    // items[i] goes to off[key(i)] + (its rank among that key's items)
    auto scatter = [&](size_t n, uint64_t nkeys, const std::vector<uint64_t> &off, const auto &key, const auto &put) {
        const uint32_t P = n < 4096 ? 1 : T;
        parallel(P, [&](uint32_t p) {
            const uint64_t k0 = nkeys * p / P, k1 = nkeys * (p + 1) / P;
            std::vector<uint64_t> pos(off.begin() + k0, off.begin() + k1);
            for (size_t i = 0; i < n; ++i) {
                const uint64_t k = key(i);
                if (k >= k0 && k < k1) put(i, pos[k - k0]++);
            }
        });
    };
    ht.node_off[N] = ht.m_type.size();
    sc_off[N] = ht.sc_type.size();
    if (ht.prop_off.empty()) ht.prop_off.assign(N + 1, 0);
    ht.prop_off[N] = ht.prop_seq.size();
    if (member) {
        ht.ee_off[N] = ht.ee_msg.size();
        ht.sc_off = sc_off;
        for (uint32_t n = 0; n < N; ++n)       // the device incarnation (G_SEG) counts at most one per marker
            if ((wc ? next[n].markers : ht.ee_off[n + 1] - ht.ee_off[n]) >= G_SEG) return MPX_E_RANGE;
    }

    // vote lists (attributed in the walk above)
    {
        ht.b_rep_off.assign(ht.b_msg.size() + 1, 0);
        for (size_t j = 0; j < reps.size(); ++j) ht.b_rep_off[j + 1] = ht.b_rep_off[j] + reps[j].size();
        ht.b_rep.reserve(ht.b_rep_off.back());
        for (auto &r : reps) ht.b_rep.insert(ht.b_rep.end(), r.begin(), r.end());
        // the replies' headers beside the list (read in order by k_votes, no gathers)
        ht.b_rbal.resize(ht.b_rep.size());
        ht.b_rsrc.resize(ht.b_rep.size());
        for (size_t r = 0; r < ht.b_rep.size(); ++r) {
            const uint32_t g = ht.b_rep[r];
            ht.b_rbal[r] = ht.m_ballot[g];
            ht.b_rsrc[r] = std::min<uint32_t>(ht.m_src[g], 0xFFFF);   // member: epoch bits added on the device
        }
        ht.b_bal.resize(ht.b_msg.size());
        for (size_t j = 0; j < ht.b_msg.size(); ++j)
            ht.b_bal[j] = wc ? b_bal_w[j] : ht.b_pstart[j] == NONE32 ? 0 : ht.m_ballot[ht.b_pstart[j]];
    }

    // fragment CSR per (node, bucket), stable (keeps message order)
    ht.f_off.assign(N * NB + 1, 0);
    for (uint64_t i = 0; i < N * NB; ++i) {
        ht.f_off[i + 1] = ht.f_off[i] + fcount[i];
        if (fcount[i] > MAX_PAIR_FRAGS) return MPX_E_RANGE;   // 2-byte state slots (mpx_internal.hpp)
    }
    if (fr.size() > MAX_FRAGS) return MPX_E_RANGE;             // 4-byte state slots (mpx_internal.hpp)
    ht.frags.resize(fr.size());
    scatter(fr.size(), (uint64_t)N * NB, ht.f_off, [&](size_t i) { return fr[i].key; },
            [&](size_t i, uint64_t at) { ht.frags[at] = fr[i].f; });
    if (!wc) {
        mark_value_checks(ht, member);
        const uint64_t NP = (uint64_t)N * NB;
        const uint32_t P = NP < 4096 ? 1 : T;
        parallel(P, [&](uint32_t k) { mark_equal_values(ht, NP * k / P, NP * (k + 1) / P); });
        ht.f_pid.assign(ht.frags.size(), 0);
        const uint64_t NF = ht.frags.size();
        const uint32_t PF = NF < 4096 ? 1 : T;
        parallel(PF, [&](uint32_t k) { mark_uniform_pids(ht, NF * k / PF, NF * (k + 1) / PF); });
    }
    ht.cf_off.assign(NB + 1, 0);
    for (uint64_t i = 0; i < NB; ++i) {
        ht.cf_off[i + 1] = ht.cf_off[i] + cfcount[i];
        if (cfcount[i] > MAX_PAIR_FRAGS) return MPX_E_RANGE;  // 2-byte chosen log (mpx_internal.hpp)
    }
    ht.cfrags.resize(cfr.size());
    scatter(cfr.size(), NB, ht.cf_off, [&](size_t i) { return cfr[i].key; },
            [&](size_t i, uint64_t at) { ht.cfrags[at] = cfr[i].f; });
    // per-pair event CSR (stable: message order within a pair)
    ht.ev_off.assign(N * NB + 1, 0);
    ht.pair_ev.assign(N * NB, 0);
    for (auto &x : evp) ht.ev_off[x.first + 1]++;
    for (uint64_t i = 0; i < N * NB; ++i) {
        ht.pair_ev[i] = ht.ev_off[i + 1] ? 1 : 0;
        ht.ev_off[i + 1] += ht.ev_off[i];
    }
    ht.ev_msg.resize(evp.size());
    ht.ev_aux.resize(evp.size());
    scatter(evp.size(), (uint64_t)N * NB, ht.ev_off, [&](size_t i) { return evp[i].first; },
            [&](size_t i, uint64_t at) { ht.ev_msg[at] = evp[i].second; ht.ev_aux[at] = evx[i]; });
    std::vector<uint64_t>().swap(evx);
    std::vector<std::pair<uint64_t, uint32_t>>().swap(evp);
    // pairs that are not lean (mpx_internal.hpp plan_shape_ok: one plan word of
    // k_plan) go to the general kernel's work list
    ht.pair_gp.assign(N * NB, 0);
    if (wc) {
        // incremental window: every pair with runs or events of the window walks the
        // window apply kernel (k_apply_win), on the state earlier windows left
        for (uint64_t b = 0; b < NB; ++b)
            for (uint32_t n = 0; n < N; ++n) {
                const uint64_t p = b * N + n;
                if (ht.f_off[p + 1] == ht.f_off[p] && ht.ev_off[p + 1] == ht.ev_off[p]) continue;
                ht.gp_list.push_back(p);
                ht.gp_base.push_back(wc->state_b[n][b]);
                ht.pair_gp[p] = GP_ROUNDS;
            }
        for (uint64_t b = 0; b < NB; ++b)
            if (ht.cf_off[b + 1] > ht.cf_off[b]) ht.cb_list.push_back((uint32_t)b);
        ht.num_gp_simple = ht.num_gp_snap = 0;
    }
    for (uint64_t b = 0; b < NB && !wc; ++b)
        for (uint32_t n = 0; n < N; ++n) {
            const uint64_t p = b * N + n, f0 = ht.f_off[p], nf = ht.f_off[p + 1] - f0;
            if (!nf) continue;
            bool fast = !member && N <= FAST_MAX_NODES && nf <= PLAN_FRAGS && !ht.pair_ev[p] && (b + 1) * BS <= slen;
            if (fast) {
                uint64_t w1[PLAN_FRAGS];
                for (uint64_t f = 0; f < nf; ++f) std::memcpy(&w1[f], reinterpret_cast<const uint8_t *>(&ht.frags[f0 + f]) + 8, 8);
                fast = plan_shape_ok(w1, (uint32_t)nf);
            }
            if (!fast) { ht.gp_list.push_back(p); ht.pair_gp[p] = GP_LIST; }
        }
    // work-list order: the pairs with no snapshot events and no promise-reply runs
    // first (k_apply's SIMPLE instantiation takes them), pair order kept
    // then those with no promise-reply runs (their events are PREPAREs only, member:
    // and E_EPOCHs; k_apply AM_SNAP), then the rest (promise rounds)
    if (!wc) {
        ht.num_gp_simple = ht.num_gp_snap = 0;
        auto no_preply = [&](uint64_t p) {
            for (uint64_t f = ht.f_off[p]; f < ht.f_off[p + 1]; ++f)
                if ((ht.frags[f].flags >> 4) == K_PREPLY) return false;
            return true;
        };
        auto mid = std::stable_partition(ht.gp_list.begin(), ht.gp_list.end(), no_preply);
        ht.num_gp_snap = (uint64_t)(mid - ht.gp_list.begin());
        auto mid2 = std::stable_partition(ht.gp_list.begin(), mid, [&](uint64_t p) { return !ht.pair_ev[p]; });
        ht.num_gp_simple = (uint64_t)(mid2 - ht.gp_list.begin());
        // k_plan_list takes the pairs before `mid` (or lists them for k_apply itself);
        // the promise-round pairs stay on the host range of the full kernel
        for (auto it = mid; it != ht.gp_list.end(); ++it) ht.pair_gp[*it] = GP_ROUNDS;
    }
    // slots for sparse fragments
    if (ht.any_sparse) {
        ht.e_slot.resize(ht.e_iid.size());
        ht.r_slot.resize(ht.r_iid.size());
        const size_t E = ht.e_iid.size(), R = ht.r_iid.size(), C = 1u << 18;
        const uint32_t ce = (uint32_t)((E + C - 1) / C), cr = (uint32_t)((R + C - 1) / C);
        parallel(ce + cr, [&](uint32_t c) {
            const bool e = c < ce;
            const std::vector<uint64_t> &iv = e ? ht.e_iid : ht.r_iid;
            std::vector<uint8_t> &sl = e ? ht.e_slot : ht.r_slot;
            const size_t a = (size_t)(e ? c : c - ce) * C, b = std::min(iv.size(), a + C);
            for (size_t k = a; k < b; ++k) sl[k] = (uint8_t)((iv[k] - sb) & (BS - 1));
        });
    }
    // proposer lists
    ht.pl_off.assign(N + 1, 0);
    for (uint32_t n = 0; n < N; ++n) ht.pl_off[n + 1] = ht.pl_off[n] + pl_cnt[n];
    ht.pl_msg = std::move(pl);
    // header-scan chunks, over each node's scan stream
    ht.node_chunk_off.assign(N + 1, 0);
    ht.scan_chunk = scan_chunk_for(sc_off[N]);
    for (uint32_t n = 0; n < N; ++n) {
        ht.node_chunk_off[n] = (uint32_t)ht.chunk_node.size();
        for (uint64_t g = sc_off[n]; g < sc_off[n + 1]; g += ht.scan_chunk) {
            ht.chunk_node.push_back(n);
            ht.chunk_beg.push_back(g);
            ht.chunk_end.push_back(std::min<uint64_t>(g + ht.scan_chunk, sc_off[n + 1]));
        }
    }
    ht.node_chunk_off[N] = (uint32_t)ht.chunk_node.size();
    if (wc) {
        // every check passed: the window is consumed, the carry moves past it
        for (uint32_t n = 0; n < N; ++n) {
            NodeCarry &c = next[n];
            wc->live[n] = std::move(c.live);
            wc->round_b[n] = std::move(c.round_b);
            wc->maxb[n] = c.maxb;
            wc->round_ballot[n] = c.ballot;
            wc->markers[n] = c.markers;
        }
        for (uint32_t gid : ents_gone) wc->b_ents.erase(gid);
        for (auto &x : ents_new) wc->b_ents[x.first] = std::move(x.second);
        for (size_t j = 0; j < ht.b_msg.size(); ++j)
            if (ht.b_msg[j] != NONE32) {                    // new batches, in id order
                wc->b_bal.push_back(b_bal_w[j]);
                wc->b_aid.push_back(ht.b_aid[j]);
            }
        wc->batches = gid_next;
        for (auto &x : state_new) wc->state_b[x.first][x.second] = 1;
    }
    return MPX_OK;
}

// The one-thread build (the reference for build_trace's node-parallel walk: tests and tools compare
// the two HostTraces field by field).
int build_trace_serial(const std::vector<NodeStream> &nodes, uint64_t sb, uint64_t slen,
                       const std::vector<mpx_epoch> &epochs, HostTrace &ht, WindowCarry *wc)
{
    const bool member = !epochs.empty();
    if (wc && !wc->on) return MPX_E_STATE;
    ht = HostTrace();
    const uint32_t N = (uint32_t)nodes.size();
    ht.N = N;
    ht.shard_begin = sb;
    ht.shard_len = slen;
    ht.NB = (uint32_t)((slen + BS - 1) >> BSH);
    const uint64_t NB = ht.NB;
    uint64_t G = 0, E = 0, R = 0, GR = 0;
    for (auto &ns : nodes) { G += ns.type.size(); E += ns.e_iid.size(); R += ns.r_iid.size(); GR += ns.g_a.size(); }
    if (G >= NONE32 || E > MAX_ENTRIES) return MPX_E_RANGE;     // chosen log (mpx_internal.hpp)
    ht.m_type.reserve(G); ht.m_src.reserve(G); ht.m_cnt.reserve(G); ht.m_node.reserve(G);
    ht.m_ballot.reserve(G); ht.m_aux.reserve(G); ht.m_ent.reserve(G);
    ht.e_val.reserve(E); ht.e_iid.reserve(E); ht.r_pid.reserve(R); ht.r_val.reserve(R); ht.r_iid.reserve(R);
    ht.g_a.reserve(GR); ht.g_b.reserve(GR);
    ht.node_off.assign(N + 1, 0);

    EntryPool pool;
    pool.member = member;
    Walk W;
    W.fcount.assign(N * NB + 1, 0); W.cfcount.assign(NB + 1, 0); W.pl_cnt.assign(N, 0);
    auto &fcount = W.fcount, &cfcount = W.cfcount;
    auto &fr = W.fr, &cfr = W.cfr;
    auto &pl = W.pl;
    auto &pl_cnt = W.pl_cnt;
    // Snapshot events (PREPARE, PREPARE_REPLY, P_START, E_EPOCH) are listed per
    // (bucket, node) pair, only where they can act on the pair's state:
    //   PREPARE       FilterAcceptedValues (multi/paxos.cpp:902-922) reads accepted /
    //                 committed entries: buckets inside its ranges that already hold
    //                 a fragment of the node (state can exist only after one);
    //   PREPARE_REPLY the quorum reply emits the merged pre-accepted map (:1047-1105),
    //   P_START       which it also clears (:1233-1248): buckets with PREPARE_REPLY
    //                 entries since the node's last P_START;
    //   E_EPOCH       (member) the same, plus every bucket with state when the node's
    //                 Acceptor is deleted / recreated (member/paxos.cpp:1897-1901,1952-1957).
    // So a pair walks O(events that touch it), not every event of its node.
    auto &evp = W.evp;                                       // (pair, message)
    auto &evx = W.evx;                                       // its aux word (PREPARE: the ranges meeting the bucket)
    std::vector<uint32_t> first_frag(NB, NONE32);            // per bucket: the node's first fragment message
    std::vector<uint64_t> touched, round_b;
    std::vector<uint8_t> in_round(NB, 0);
    W.sc_off.assign(N + 1, 0);
    auto &sc_off = W.sc_off;                                 // each node's scan-stream range
    // vote lists: an ACCEPT_REPLY counts for the live batch of its node with the
    // same accept id (OnAcceptReply, multi/paxos.cpp:1406-1410); member: only at a
    // node whose Proposer exists (Loop, member/paxos.cpp:763-790)
    std::unordered_map<uint64_t, uint32_t> live;
    auto &reps = W.reps;
    if (member) ht.ee_off.assign(N + 1, 0);
    // incremental window: batch ids are global (live maps to them); a batch's index in
    // this window's list, its round ballot, and where a new one's entries are
    std::unordered_map<uint32_t, uint32_t> gid_local;
    auto &b_bal_w = W.b_bal_w;
    std::vector<std::pair<uint64_t, uint32_t>> b_ent_w;          // per window batch: pool offset, count (new ones)
    auto &state_new = W.state_new;                               // (node, bucket) met by this window's runs
    const uint64_t gid0 = wc ? wc->batches : 0;
    W.gid_next = gid0;
    auto &gid_next = W.gid_next;
    // The carry past this window is collected here and committed to *wc only once every
    // check below has passed: a window that fails (MPX_E_RANGE, MPX_E_DECODE) leaves the
    // carry as it was, so its records can be resubmitted or the engine dropped
    W.next.resize(wc ? N : 0);
    auto &next = W.next;
    auto &ents_gone = W.ents_gone;                               // carried batches no longer live
    auto &ents_new = W.ents_new;

    for (uint32_t n = 0; n < N; ++n) {
        const NodeStream &ns = nodes[n];
        ht.node_off[n] = ht.m_type.size();
        const uint64_t rbase = ht.r_val.size(), gbase = ht.g_a.size();
        ht.r_pid.insert(ht.r_pid.end(), ns.r_pid.begin(), ns.r_pid.end());
        ht.r_val.insert(ht.r_val.end(), ns.r_val.begin(), ns.r_val.end());
        ht.r_iid.insert(ht.r_iid.end(), ns.r_iid.begin(), ns.r_iid.end());
        ht.g_a.insert(ht.g_a.end(), ns.g_a.begin(), ns.g_a.end());
        ht.g_b.insert(ht.g_b.end(), ns.g_b.begin(), ns.g_b.end());
        uint32_t pstart = NONE32;                       // epoch of the batches that follow
        sc_off[n] = ht.sc_type.size();
        for (uint64_t b : touched) first_frag[b] = NONE32;
        for (uint64_t b : round_b) in_round[b] = 0;
        touched.clear(); round_b.clear();
        int64_t maxb = -1;                              // highest bucket with a fragment of this node
        live.clear();
        uint64_t cur_bal = 0;                           // the ballot of the node's current round
        if (wc) {                                       // the window starts where the last one ended
            live = wc->live[n];
            for (uint64_t b : wc->round_b[n]) { in_round[b] = 1; round_b.push_back(b); }
            maxb = wc->maxb[n];
            cur_bal = wc->round_ballot[n];
        }
        // window: this window's index of global batch `gid` (an earlier batch joins the list
        // with its carried entries as chosen-log runs)
        auto local_batch = [&](uint32_t gid) -> uint32_t {
            auto it = gid_local.find(gid);
            if (it != gid_local.end()) return it->second;
            const uint32_t j = (uint32_t)ht.b_msg.size();
            gid_local.emplace(gid, j);
            ht.b_msg.push_back(NONE32); ht.b_pstart.push_back(NONE32); ht.b_gid.push_back(gid);
            ht.b_aid.push_back(wc->b_aid[gid]);
            ht.b_node.push_back(n);
            reps.emplace_back();
            b_bal_w.push_back(wc->b_bal[gid]);
            b_ent_w.push_back({0, 0});
            auto be = wc->b_ents.find(gid);
            if (be != wc->b_ents.end() && !be->second.empty()) {
                NodeStream tmp;
                for (auto &x : be->second) { tmp.e_iid.push_back(x.first); tmp.e_val.push_back(x.second); }
                const uint64_t o = pool.intern(tmp, 0, (uint32_t)tmp.e_iid.size(), ht);
                cut_runs(ht.e_iid.data(), o, (uint32_t)tmp.e_iid.size(), sb, [&](uint64_t b, uint64_t e0, uint32_t c, uint8_t st, bool dense) {
                    Frag f{e0, j, (uint16_t)c, st, (uint8_t)((dense ? FR_DENSE : 0) | (K_BATCH << 4))};
                    if (!dense) ht.any_sparse = true;
                    cfr.push_back({b, f});
                    cfcount[b]++;
                });
            }
            return j;
        };
        bool last_virtual = false;                      // the node's last scan record stands for left-out ACCEPTs
        // member semantics: no role or version logic here — the per-message gate
        // (acceptor incarnation, version filter, proposer presence) is computed on
        // the device from the E_EPOCH markers and the epoch table (kernels.hip
        // k_gate_*); ingest only lists the markers and keeps every record
        if (member) ht.ee_off[n] = ht.ee_msg.size();
        if (ht.prop_off.empty()) ht.prop_off.assign(N + 1, 0);
        ht.prop_off[n] = ht.prop_seq.size();
        for (size_t k = 0; k < ns.type.size(); ++k) {
            const uint32_t g = (uint32_t)ht.m_type.size();
            const uint8_t t = ns.type[k];
            if (t == MPX_MSG_P_PROPOSE) {               // the proposer's bookkeeping only (engine.cpp)
                ht.prop_seq.push_back((uint32_t)k);
                continue;
            }
            if (member && t == MPX_MSG_E_EPOCH && ns.ver[k] >= epochs.size()) return MPX_E_DECODE;
            // Header sharding: a record whose entries all belong to
            // other shards is left out here — ACCEPT / COMMIT / P_BATCH with no
            // entry in the shard, the ACCEPT_REPLYs of batches not kept, and
            // COMMIT_REPLYs (no effect on the acceptor / learner path; the shard
            // at instance 0 keeps them).  Only the scalars see such an ACCEPT:
            // its ballot stays in the scan stream as a max_seen-only record.
            // (member: a batch made while the node has no Proposer, or cut off by a
            // marker that resets it, is killed on the device — k_gate_votes)
            bool drop = ns.part[k] != 0 || (t == MPX_MSG_COMMIT_REPLY && sb != 0);
            int64_t vote_j = -1;
            if (t == MPX_MSG_P_START) {
                if (wc)                                  // earlier windows' batches can no longer be chosen
                    for (auto &x : live) if (x.second < gid0) ents_gone.push_back(x.second);
                live.clear();
                cur_bal = ns.ballot[k];
            } else if (t == MPX_MSG_P_BATCH) {
                if (drop) live.erase(ns.aux[k]);
                else live[ns.aux[k]] = wc ? (uint32_t)gid_next : (uint32_t)ht.b_msg.size();
            } else if (t == MPX_MSG_ACCEPT_REPLY) {
                auto it = live.find(ns.aux[k]);
                if (it == live.end()) drop = true;   // stale, or its batch is another shard's
                else vote_j = wc ? local_batch(it->second) : it->second;
            }
            if (drop) {
                ++ht.dropped;
                if (ns.part[k] != 0) ++ht.part_dropped;
                if (t == MPX_MSG_ACCEPT && member) {
                    // member: the device gates it and adds the incarnation (k_gate_scan),
                    // so it is kept on its own with its version and position
                    ht.sc_type.push_back(SC_SONLY | SC_VIRT); ht.sc_key.push_back(ns.ballot[k]);
                    ht.sc_idx.push_back(g); ht.sc_ver.push_back(ns.ver[k]);
                    last_virtual = false;
                } else if (t == MPX_MSG_ACCEPT) {
                    if (last_virtual) ht.sc_key.back() = std::max(ht.sc_key.back(), ns.ballot[k]);
                    else { ht.sc_type.push_back(SC_SONLY); ht.sc_key.push_back(ns.ballot[k]); ht.sc_idx.push_back(0); }
                    last_virtual = true;
                }
                continue;
            }
            if (member) {
                ht.m_ver.push_back(ns.ver[k]);
                if (t == MPX_MSG_E_EPOCH) ht.ee_msg.push_back(g);
            }
            ht.m_seq.push_back((uint32_t)k);
            if (vote_j >= 0) reps[vote_j].push_back(g);
            uint64_t ent = ns.ent[k];
            if (t == MPX_MSG_PREPARE) ent += gbase;
            else if (t == MPX_MSG_PREPARE_REPLY) ent += rbase;
            else if (t == MPX_MSG_ACCEPT || t == MPX_MSG_COMMIT || t == MPX_MSG_P_BATCH) ent = pool.intern(ns, ent, ns.cnt[k], ht);
            ht.m_type.push_back(t);
            ht.m_src.push_back(ns.src[k]);
            ht.m_ballot.push_back(ns.ballot[k]);
            ht.m_aux.push_back(ns.aux[k]);
            ht.m_ent.push_back(ent);
            ht.m_cnt.push_back(ns.cnt[k]);
            ht.m_node.push_back(n);
            {   // header-scan stream and static flags (mpx_internal.hpp SC_*)
                const bool badsrc = ns.src[k] >= N;
                uint8_t f0 = 0;
                int sct = -1;
                uint64_t key = ns.ballot[k];
                if (member) {
                    // keys / types finished on the device (k_gate_scan): the raw ballot here
                    if (t == MPX_MSG_PREPARE || t == MPX_MSG_ACCEPT) {
                        sct = t == MPX_MSG_PREPARE ? SC_PREP : SC_ACC;
                        if (badsrc) sct |= SC_BAD;
                    } else if (t == MPX_MSG_E_EPOCH) {
                        sct = SC_PS;
                        key = 0;
                    } else if (t == MPX_MSG_COMMIT && badsrc) {
                        f0 = F_BADNODE; sct = SC_NONE | SC_BAD;
                    }
                } else if (t == MPX_MSG_PREPARE || t == MPX_MSG_ACCEPT) {
                    sct = t == MPX_MSG_PREPARE ? SC_PREP : SC_ACC;
                    if (badsrc) { f0 |= F_BADNODE; sct |= SC_BAD; }
                } else if (t == MPX_MSG_REJECT) {
                    sct = SC_SONLY;
                } else if (t == MPX_MSG_COMMIT && badsrc) {
                    f0 = F_BADNODE; sct = SC_NONE | SC_BAD;
                }
                ht.m_flags0.push_back(f0);
                if (sct >= 0) {
                    ht.sc_type.push_back((uint8_t)sct); ht.sc_key.push_back(key); ht.sc_idx.push_back(g);
                    if (member) ht.sc_ver.push_back(ns.ver[k]);
                    last_virtual = false;
                }
            }
            if (t == MPX_MSG_PREPARE_REPLY || t == MPX_MSG_P_START || t == MPX_MSG_E_EPOCH) { pl.push_back(g); pl_cnt[n]++; }
            if (t == MPX_MSG_P_START) pstart = g;
            if (t == MPX_MSG_P_BATCH) {
                if (wc) {
                    gid_local.emplace((uint32_t)gid_next, (uint32_t)ht.b_msg.size());
                    ht.b_gid.push_back((uint32_t)gid_next++);
                    ht.b_node.push_back(n);
                    b_bal_w.push_back(cur_bal);
                    b_ent_w.push_back({ent, ns.cnt[k]});
                }
                ht.b_msg.push_back(g);
                ht.b_aid.push_back(ns.aux[k]);
                ht.b_pstart.push_back(pstart);
                reps.emplace_back();
            }
            if (t == MPX_MSG_ACCEPT || t == MPX_MSG_COMMIT || t == MPX_MSG_PREPARE_REPLY) {
                const uint8_t kind = t == MPX_MSG_ACCEPT ? K_ACCEPT : t == MPX_MSG_COMMIT ? K_COMMIT : K_PREPLY;
                const uint64_t *iid = t == MPX_MSG_PREPARE_REPLY ? ht.r_iid.data() : ht.e_iid.data();
                cut_runs(iid, ent, ns.cnt[k], sb, [&](uint64_t b, uint64_t e0, uint32_t c, uint8_t st, bool dense) {
                    Frag f{e0, g, (uint16_t)c, st, (uint8_t)((dense ? FR_DENSE : 0) | (kind << 4))};
                    if (!dense) ht.any_sparse = true;
                    fr.push_back({b * N + n, f});            // pair index: bucket-major
                    fcount[b * N + n]++;
                    if (first_frag[b] == NONE32) {
                        first_frag[b] = g; touched.push_back(b); maxb = std::max<int64_t>(maxb, (int64_t)b);
                        if (wc && !wc->state_b[n][b]) state_new.push_back({n, b});
                    }
                    if (kind == K_PREPLY && !in_round[b]) { in_round[b] = 1; round_b.push_back(b); }
                });
            }
            // snapshot events of this message (after its own fragments: the kernels
            // merge a message's fragments before its event)
            auto add_ev = [&](uint64_t b) { evp.push_back({b * N + n, g}); evx.push_back(0); };
            auto clear_round = [&]() { for (uint64_t b : round_b) in_round[b] = 0; round_b.clear(); };
            if (t == MPX_MSG_PREPARE && maxb >= 0) {
                uint64_t last_b = 0;                     // ranges are sorted and disjoint: buckets ascend
                for (uint32_t r = 0; r < ns.cnt[k]; ++r) {
                    const uint64_t a = ht.g_a[ent + r], e = ht.g_b[ent + r];
                    if (e <= sb || a >= sb + slen) continue;
                    const uint64_t lo = (std::max(a, sb) - sb) >> BSH;
                    const uint64_t hi = std::min<uint64_t>((std::min(e, sb + slen) - sb + BS - 1) >> BSH, (uint64_t)maxb + 1);
                    // several ranges of one PREPARE can meet in a bucket (holes): list it
                    // once, its aux word = first range (absolute) | ranges meeting it << 32
                    for (uint64_t b = lo; b < hi; ++b) {
                        if (first_frag[b] >= g && !(wc && wc->state_b[n][b])) continue;   // (window: or earlier ones')
                        if (!evp.empty() && evp.back().second == g && b == last_b && evp.back().first == b * N + n) {
                            evx.back() = (evx.back() + (1ull << 32)) & ~EVX_ONE;   // a second range: no interval
                        } else if (evp.empty() || evp.back().second != g || b > last_b) {
                            add_ev(b);
                            // one range so far: its bucket-local interval too (k_apply needs no range loads)
                            const uint64_t blo = sb + (b << BSH);
                            const uint64_t il = std::max(a, blo) - blo, ih = std::min(e, blo + BS) - blo;
                            evx.back() = (ent + r) | (1ull << 32) | (il << 40) | (ih << 49) | EVX_ONE;
                            last_b = b;
                        }
                    }
                }
            } else if (t == MPX_MSG_PREPARE_REPLY) {
                for (uint64_t b : round_b) add_ev(b);
            } else if (t == MPX_MSG_P_START) {
                for (uint64_t b : round_b) add_ev(b);
                clear_round();
            } else if (t == MPX_MSG_E_EPOCH) {
                // the marker may delete / recreate the Acceptor or reset the Proposer
                // (decided on the device): every bucket with state of the node gets the
                // event (round buckets included; a window: also state of earlier windows),
                // and the round stays listed
                for (uint64_t b = 0; (int64_t)b <= maxb; ++b)
                    if (first_frag[b] < g || (wc && wc->state_b[n][b])) add_ev(b);
            }
            if (t == MPX_MSG_P_BATCH) {
                const uint32_t j = wc ? gid_local[(uint32_t)(gid_next - 1)] : (uint32_t)ht.b_msg.size() - 1;
                cut_runs(ht.e_iid.data(), ent, ns.cnt[k], sb, [&](uint64_t b, uint64_t e0, uint32_t c, uint8_t st, bool dense) {
                    Frag f{e0, j, (uint16_t)c, st, (uint8_t)((dense ? FR_DENSE : 0) | (K_BATCH << 4))};
                    if (!dense) ht.any_sparse = true;
                    cfr.push_back({b, f});
                    cfcount[b]++;
                });
            }
        }
        if (wc) {                                        // the carry past this node's window
            NodeCarry &c = next[n];
            for (auto &x : live)                         // new batches still open: keep their entries
                if (x.second >= gid0) {
                    const auto &be = b_ent_w[gid_local[x.second]];
                    auto &dst = ents_new[x.second];
                    for (uint32_t q = 0; q < be.second; ++q) dst.push_back({ht.e_iid[be.first + q], ht.e_val[be.first + q]});
                }
            c.live = std::move(live);
            c.round_b = round_b;
            c.maxb = maxb;
            c.ballot = cur_bal;
            if (member) c.markers = wc->markers[n] + (uint32_t)(ht.ee_msg.size() - ht.ee_off[n]);
        }
    }
    return finish_trace(ht, W, N, NB, sb, slen, member, wc, 1);
}

// ---- build_trace: the walk over the nodes' records, node-parallel ----
//
// Phase A (a thread per node): the serial walk's per-node work in node-local coordinates —
// kept messages numbered from 0, batches from 0 in first-reference order, entry lists by the
// node's own arrays, each list to intern (ACCEPT / COMMIT / P_BATCH, a window's carried batch
// entries) hashed.  Phase B: the entry pool — first occurrences in walk order (node, list),
// found per hash shard on a thread each, lists compared in full; then their offsets in order.
// Phase C (a thread per node): the parts rebased into the HostTrace (message, batch, pool, range
// and promise-reply offsets).  The result is build_trace_serial's, field for field.
namespace {
struct PoolItem {
    uint32_t node;
    uint32_t batch;                     // carried batch list: its local batch (NONE32: a message's list)
    uint64_t first;                     // the node's e_* index (carried: 0)
    uint32_t cnt;
    uint64_t hash;
    uint64_t sec;                       // the list's value-section id (0: none; equal ids = equal lists)
    const std::vector<std::pair<uint64_t, uint64_t>> *carried;
    uint64_t off;                       // phase B: pool offset
    bool is_first;
};
struct NodePart {
    int rc = MPX_OK;
    std::vector<uint8_t> m_type, m_flags0;
    std::vector<uint32_t> m_src, m_cnt, m_ver, m_seq;
    std::vector<uint64_t> m_ballot, m_aux, m_ent;   // m_ent: g_a / r index (node-local), or pool item
    std::vector<uint8_t> sc_type;
    std::vector<uint64_t> sc_key;
    std::vector<uint32_t> sc_idx, sc_ver;            // sc_idx: local message, NONE32 = literal 0
    std::vector<uint32_t> ee_msg, pl, prop_seq;
    uint64_t dropped = 0, part_dropped = 0;
    bool any_sparse = false;
    // batches in first-reference order
    std::vector<uint32_t> b_msg, b_pstart, b_gid, b_item;   // b_gid: carried: global; new: gid0 + local new index
    std::vector<uint64_t> b_aid, b_bal;
    std::vector<std::pair<uint64_t, uint32_t>> b_ent;       // new batches: their list (node e_* index, count)
    std::vector<std::vector<uint32_t>> reps;
    uint32_t new_batches = 0;
    std::vector<PoolItem> items;
    // runs: Frag.entry relative to its list (fr_item / cfr_item), or a node-local r index (NONE32)
    std::vector<FragKey> fr, cfr;
    std::vector<uint32_t> fr_item, cfr_item;
    std::vector<uint64_t> fcount, cfcount;                   // (sparse: touched pairs only, see below)
    std::vector<std::pair<uint64_t, uint32_t>> evp;
    std::vector<uint64_t> evx;
    std::vector<uint64_t> state_b;                           // (window) buckets first met
    NodeCarry carry;
    std::vector<uint32_t> ents_gone;
    std::vector<std::pair<uint32_t, std::vector<std::pair<uint64_t, uint64_t>>>> ents_new;   // (gid, entries)
};

static uint64_t list_hash(const uint64_t *iv, const uint64_t *vv, const uint64_t *pv, uint32_t cnt, bool member)
{
    // EntryPool::intern's hash (content-equal lists hash equal)
    uint64_t l[4] = {mix64(cnt + 0x51ull), 0x9E3779B97F4A7C15ull, 0xC2B2AE3D27D4EB4Full, 0x165667B19E3779F9ull};
    for (uint32_t i = 0; i < cnt; ++i) l[i & 3] = (l[i & 3] ^ iv[i]) * 0xff51afd7ed558ccdull + vv[i];
    if (member)
        for (uint32_t i = 0; i < cnt; ++i) l[i & 3] = (l[i & 3] ^ (pv ? pv[i] : 0)) * 0xc4ceb9fe1a85ec53ull;
    return mix64(mix64(mix64(l[0] ^ l[1]) ^ l[2]) ^ l[3]);
}

static void walk_node(const NodeStream &ns, uint32_t n, uint32_t N, uint64_t sb, uint64_t slen, uint64_t NB,
                      bool member, size_t num_epochs, const WindowCarry *wc, NodePart &P)
{
    const uint64_t gid0 = wc ? wc->batches : 0;
    std::vector<uint32_t> first_frag(NB, NONE32);            // per bucket: the node's first fragment message
    std::vector<uint8_t> in_round(NB, 0);
    std::vector<uint64_t> round_b;
    int64_t maxb = -1;
    std::unordered_map<uint64_t, uint32_t> live;              // accept id -> batch (window: global id)
    uint64_t cur_bal = 0;
    std::unordered_map<uint32_t, uint32_t> gid_local;         // (window) batch id -> local batch
    if (wc) {
        live = wc->live[n];
        for (uint64_t b : wc->round_b[n]) { in_round[b] = 1; round_b.push_back(b); }
        maxb = wc->maxb[n];
        cur_bal = wc->round_ballot[n];
    }
    const bool has_pid = !ns.e_pid.empty();
    auto add_item = [&](uint32_t batch, uint64_t first, uint32_t cnt,
                        const std::vector<std::pair<uint64_t, uint64_t>> *carried) -> uint32_t {
        PoolItem it{n, batch, first, cnt, 0, 0, carried, 0, false};
        if (carried) {
            std::vector<uint64_t> iv(cnt), vv(cnt);
            for (uint32_t q = 0; q < cnt; ++q) { iv[q] = (*carried)[q].first; vv[q] = (*carried)[q].second; }
            it.hash = list_hash(iv.data(), vv.data(), nullptr, cnt, member);
        } else {
            it.hash = list_hash(ns.e_iid.data() + first, ns.e_val.data() + first, has_pid ? ns.e_pid.data() + first : nullptr,
                                cnt, member);
        }
        P.items.push_back(it);
        return (uint32_t)P.items.size() - 1;
    };
    auto local_batch = [&](uint32_t gid) -> uint32_t {
        auto it = gid_local.find(gid);
        if (it != gid_local.end()) return it->second;
        const uint32_t j = (uint32_t)P.b_msg.size();
        gid_local.emplace(gid, j);
        P.b_msg.push_back(NONE32); P.b_pstart.push_back(NONE32); P.b_gid.push_back(gid);
        P.b_aid.push_back(wc->b_aid[gid]);
        P.b_bal.push_back(wc->b_bal[gid]);
        P.b_ent.push_back({0, 0});
        P.b_item.push_back(NONE32);
        P.reps.emplace_back();
        auto be = wc->b_ents.find(gid);
        if (be != wc->b_ents.end() && !be->second.empty()) {
            const uint32_t cnt = (uint32_t)be->second.size();
            const uint32_t item = add_item(j, 0, cnt, &be->second);
            P.b_item[j] = item;
            std::vector<uint64_t> iv(cnt);
            for (uint32_t q = 0; q < cnt; ++q) iv[q] = be->second[q].first;
            cut_runs(iv.data(), 0, cnt, sb, [&](uint64_t b, uint64_t e0, uint32_t c, uint8_t st, bool dense) {
                Frag f{e0, j, (uint16_t)c, st, (uint8_t)((dense ? FR_DENSE : 0) | (K_BATCH << 4))};
                if (!dense) P.any_sparse = true;
                P.cfr.push_back({b, f});
                P.cfr_item.push_back(item);
            });
        }
        return j;
    };
    uint32_t pstart = NONE32;
    bool last_virtual = false;
    for (size_t k = 0; k < ns.type.size(); ++k) {
        const uint32_t g = (uint32_t)P.m_type.size();
        const uint8_t t = ns.type[k];
        if (t == MPX_MSG_P_PROPOSE) { P.prop_seq.push_back((uint32_t)k); continue; }
        if (member && t == MPX_MSG_E_EPOCH && ns.ver[k] >= num_epochs) { P.rc = MPX_E_DECODE; return; }
        bool drop = ns.part[k] != 0 || (t == MPX_MSG_COMMIT_REPLY && sb != 0);
        int64_t vote_j = -1;
        if (t == MPX_MSG_P_START) {
            if (wc)
                for (auto &x : live) if (x.second < gid0) P.ents_gone.push_back(x.second);
            live.clear();
            cur_bal = ns.ballot[k];
        } else if (t == MPX_MSG_P_BATCH) {
            if (drop) live.erase(ns.aux[k]);
            else live[ns.aux[k]] = wc ? (uint32_t)(gid0 + P.new_batches) : (uint32_t)P.b_msg.size();
        } else if (t == MPX_MSG_ACCEPT_REPLY) {
            auto it = live.find(ns.aux[k]);
            if (it == live.end()) drop = true;
            else vote_j = wc ? local_batch(it->second) : it->second;
        }
        if (drop) {
            ++P.dropped;
            if (ns.part[k] != 0) ++P.part_dropped;
            if (t == MPX_MSG_ACCEPT && member) {
                P.sc_type.push_back(SC_SONLY | SC_VIRT); P.sc_key.push_back(ns.ballot[k]);
                P.sc_idx.push_back(g); P.sc_ver.push_back(ns.ver[k]);
                last_virtual = false;
            } else if (t == MPX_MSG_ACCEPT) {
                if (last_virtual) P.sc_key.back() = std::max(P.sc_key.back(), ns.ballot[k]);
                else { P.sc_type.push_back(SC_SONLY); P.sc_key.push_back(ns.ballot[k]); P.sc_idx.push_back(NONE32); }
                last_virtual = true;
            }
            continue;
        }
        if (member) {
            P.m_ver.push_back(ns.ver[k]);
            if (t == MPX_MSG_E_EPOCH) P.ee_msg.push_back(g);
        }
        P.m_seq.push_back((uint32_t)k);
        if (vote_j >= 0) P.reps[vote_j].push_back(g);
        uint64_t ent = ns.ent[k];                    // node-local g_a / r / e index
        uint32_t item = NONE32;
        if (t == MPX_MSG_ACCEPT || t == MPX_MSG_COMMIT || t == MPX_MSG_P_BATCH) {
            item = add_item(NONE32, ent, ns.cnt[k], nullptr);
            if (!ns.sec.empty()) P.items[item].sec = ns.sec[k];
        }
        P.m_type.push_back(t);
        P.m_src.push_back(ns.src[k]);
        P.m_ballot.push_back(ns.ballot[k]);
        P.m_aux.push_back(ns.aux[k]);
        P.m_ent.push_back(item != NONE32 ? item : ent);
        P.m_cnt.push_back(ns.cnt[k]);
        {   // header-scan stream and static flags (as build_trace_serial)
            const bool badsrc = ns.src[k] >= N;
            uint8_t f0 = 0;
            int sct = -1;
            uint64_t key = ns.ballot[k];
            if (member) {
                if (t == MPX_MSG_PREPARE || t == MPX_MSG_ACCEPT) {
                    sct = t == MPX_MSG_PREPARE ? SC_PREP : SC_ACC;
                    if (badsrc) sct |= SC_BAD;
                } else if (t == MPX_MSG_E_EPOCH) {
                    sct = SC_PS;
                    key = 0;
                } else if (t == MPX_MSG_COMMIT && badsrc) {
                    f0 = F_BADNODE; sct = SC_NONE | SC_BAD;
                }
            } else if (t == MPX_MSG_PREPARE || t == MPX_MSG_ACCEPT) {
                sct = t == MPX_MSG_PREPARE ? SC_PREP : SC_ACC;
                if (badsrc) { f0 |= F_BADNODE; sct |= SC_BAD; }
            } else if (t == MPX_MSG_REJECT) {
                sct = SC_SONLY;
            } else if (t == MPX_MSG_COMMIT && badsrc) {
                f0 = F_BADNODE; sct = SC_NONE | SC_BAD;
            }
            P.m_flags0.push_back(f0);
            if (sct >= 0) {
                P.sc_type.push_back((uint8_t)sct); P.sc_key.push_back(key); P.sc_idx.push_back(g);
                if (member) P.sc_ver.push_back(ns.ver[k]);
                last_virtual = false;
            }
        }
        if (t == MPX_MSG_PREPARE_REPLY || t == MPX_MSG_P_START || t == MPX_MSG_E_EPOCH) P.pl.push_back(g);
        if (t == MPX_MSG_P_START) pstart = g;
        if (t == MPX_MSG_P_BATCH) {
            const uint32_t j = (uint32_t)P.b_msg.size();
            if (wc) gid_local.emplace((uint32_t)(gid0 + P.new_batches), j);
            P.b_gid.push_back((uint32_t)(gid0 + P.new_batches));
            ++P.new_batches;
            P.b_bal.push_back(cur_bal);
            P.b_ent.push_back({ent, ns.cnt[k]});
            P.b_item.push_back(item);
            P.b_msg.push_back(g);
            P.b_aid.push_back(ns.aux[k]);
            P.b_pstart.push_back(pstart);
            P.reps.emplace_back();
        }
        if (t == MPX_MSG_ACCEPT || t == MPX_MSG_COMMIT || t == MPX_MSG_PREPARE_REPLY) {
            const uint8_t kind = t == MPX_MSG_ACCEPT ? K_ACCEPT : t == MPX_MSG_COMMIT ? K_COMMIT : K_PREPLY;
            const uint64_t *iid = t == MPX_MSG_PREPARE_REPLY ? ns.r_iid.data() : ns.e_iid.data();
            cut_runs(iid, ent, ns.cnt[k], sb, [&](uint64_t b, uint64_t e0, uint32_t c, uint8_t st, bool dense) {
                Frag f{item != NONE32 ? e0 - ent : e0, g, (uint16_t)c, st, (uint8_t)((dense ? FR_DENSE : 0) | (kind << 4))};
                if (!dense) P.any_sparse = true;
                P.fr.push_back({b * N + n, f});
                P.fr_item.push_back(item);
                if (first_frag[b] == NONE32) {
                    first_frag[b] = g; maxb = std::max<int64_t>(maxb, (int64_t)b);
                    if (wc && !wc->state_b[n][b]) P.state_b.push_back(b);
                }
                if (kind == K_PREPLY && !in_round[b]) { in_round[b] = 1; round_b.push_back(b); }
            });
        }
        auto add_ev = [&](uint64_t b) { P.evp.push_back({b * N + n, g}); P.evx.push_back(0); };
        auto clear_round = [&]() { for (uint64_t b : round_b) in_round[b] = 0; round_b.clear(); };
        if (t == MPX_MSG_PREPARE && maxb >= 0) {
            uint64_t last_b = 0;
            for (uint32_t r = 0; r < ns.cnt[k]; ++r) {
                const uint64_t a = ns.g_a[ent + r], e = ns.g_b[ent + r];
                if (e <= sb || a >= sb + slen) continue;
                const uint64_t lo = (std::max(a, sb) - sb) >> BSH;
                const uint64_t hi = std::min<uint64_t>((std::min(e, sb + slen) - sb + BS - 1) >> BSH, (uint64_t)maxb + 1);
                for (uint64_t b = lo; b < hi; ++b) {
                    if (first_frag[b] >= g && !(wc && wc->state_b[n][b])) continue;
                    if (!P.evp.empty() && P.evp.back().second == g && b == last_b && P.evp.back().first == b * N + n) {
                        P.evx.back() = (P.evx.back() + (1ull << 32)) & ~EVX_ONE;
                    } else if (P.evp.empty() || P.evp.back().second != g || b > last_b) {
                        add_ev(b);
                        const uint64_t blo = sb + (b << BSH);
                        const uint64_t il = std::max(a, blo) - blo, ih = std::min(e, blo + BS) - blo;
                        P.evx.back() = (ent + r) | (1ull << 32) | (il << 40) | (ih << 49) | EVX_ONE;   // (g_a index: rebased)
                        last_b = b;
                    }
                }
            }
        } else if (t == MPX_MSG_PREPARE_REPLY) {
            for (uint64_t b : round_b) add_ev(b);
        } else if (t == MPX_MSG_P_START) {
            for (uint64_t b : round_b) add_ev(b);
            clear_round();
        } else if (t == MPX_MSG_E_EPOCH) {
            for (uint64_t b = 0; (int64_t)b <= maxb; ++b)
                if (first_frag[b] < g || (wc && wc->state_b[n][b])) add_ev(b);
        }
        if (t == MPX_MSG_P_BATCH) {
            const uint32_t j = (uint32_t)P.b_msg.size() - 1;
            cut_runs(ns.e_iid.data(), ent, ns.cnt[k], sb, [&](uint64_t b, uint64_t e0, uint32_t c, uint8_t st, bool dense) {
                Frag f{e0 - ent, j, (uint16_t)c, st, (uint8_t)((dense ? FR_DENSE : 0) | (K_BATCH << 4))};
                if (!dense) P.any_sparse = true;
                P.cfr.push_back({b, f});
                P.cfr_item.push_back(item);
            });
        }
    }
    if (wc) {
        NodeCarry &c = P.carry;
        for (auto &x : live)                         // new batches still open: keep their entries
            if (x.second >= gid0) {
                const auto &be = P.b_ent[gid_local[x.second]];
                std::vector<std::pair<uint64_t, uint64_t>> dst(be.second);
                for (uint32_t q = 0; q < be.second; ++q) dst[q] = {ns.e_iid[be.first + q], ns.e_val[be.first + q]};
                P.ents_new.push_back({x.second, std::move(dst)});
            }
        c.live = std::move(live);
        c.round_b = round_b;
        c.maxb = maxb;
        c.ballot = cur_bal;
        if (member) c.markers = wc->markers[n] + (uint32_t)P.ee_msg.size();
    }
}
}  // namespace

int build_trace(const std::vector<NodeStream> &nodes, uint64_t sb, uint64_t slen,
                const std::vector<mpx_epoch> &epochs, HostTrace &ht, WindowCarry *wc, uint32_t threads)
{
    const bool member = !epochs.empty();
    if (wc && !wc->on) return MPX_E_STATE;
    if (!threads) threads = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    ht = HostTrace();
    const uint32_t N = (uint32_t)nodes.size();
    ht.N = N;
    ht.shard_begin = sb;
    ht.shard_len = slen;
    ht.NB = (uint32_t)((slen + BS - 1) >> BSH);
    const uint64_t NB = ht.NB;
    uint64_t G = 0, E = 0;
    for (auto &ns : nodes) { G += ns.type.size(); E += ns.e_iid.size(); }
    if (G >= NONE32 || E > MAX_ENTRIES) return MPX_E_RANGE;     // chosen log (mpx_internal.hpp)
    auto parallel = [&](uint32_t count, const auto &fn) {      // fn(k) for k < count on up to `threads` threads
        std::atomic<uint32_t> next{0};
        auto work = [&]() { for (uint32_t k; (k = next.fetch_add(1)) < count;) fn(k); };
        std::vector<std::thread> th;
        for (uint32_t t = 1; t < std::min(threads, count); ++t) th.emplace_back(work);
        work();
        for (auto &x : th) x.join();
    };
    // (MPX_BUILD_TIMES, A/B builds: the phases' wall times on stderr)
    const bool times = ab_env("MPX_BUILD_TIMES") != nullptr;
    auto wall = []() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    double tp[5] = {times ? wall() : 0, 0, 0, 0, 0};
    // phase A
    std::vector<NodePart> parts(N);
    parallel(N, [&](uint32_t n) { walk_node(nodes[n], n, N, sb, slen, NB, member, epochs.size(), wc, parts[n]); });
    for (uint32_t n = 0; n < N; ++n) TRY_RC(parts[n].rc);
    if (times) tp[1] = wall();
    // phase B: the entry pool (EntryPool's content addressing, first occurrence in walk order)
    {
        const uint32_t S = std::max(1u, threads);
        auto same = [&](const PoolItem &a, const PoolItem &b) {
            if (a.cnt != b.cnt) return false;
            if (a.sec && a.sec == b.sec) return true;          // (byte-equal sections, one shard filter)
            if (!a.carried && !b.carried) {                    // (the common case: two messages' lists)
                const NodeStream &x = nodes[a.node], &y = nodes[b.node];
                const size_t bytes = 8ull * a.cnt;
                if (std::memcmp(x.e_iid.data() + a.first, y.e_iid.data() + b.first, bytes) ||
                    std::memcmp(x.e_val.data() + a.first, y.e_val.data() + b.first, bytes))
                    return false;
                if (!member) return true;
                for (uint32_t q = 0; q < a.cnt; ++q)
                    if ((x.e_pid.empty() ? 0 : x.e_pid[a.first + q]) != (y.e_pid.empty() ? 0 : y.e_pid[b.first + q])) return false;
                return true;
            }
            for (uint32_t q = 0; q < a.cnt; ++q) {
                const uint64_t ai = a.carried ? (*a.carried)[q].first : nodes[a.node].e_iid[a.first + q];
                const uint64_t bi = b.carried ? (*b.carried)[q].first : nodes[b.node].e_iid[b.first + q];
                const uint64_t av = a.carried ? (*a.carried)[q].second : nodes[a.node].e_val[a.first + q];
                const uint64_t bv = b.carried ? (*b.carried)[q].second : nodes[b.node].e_val[b.first + q];
                if (ai != bi || av != bv) return false;
                if (member) {
                    const auto &pa = nodes[a.node].e_pid, &pb = nodes[b.node].e_pid;
                    const uint64_t ap = a.carried || pa.empty() ? 0 : pa[a.first + q];
                    const uint64_t bp = b.carried || pb.empty() ? 0 : pb[b.first + q];
                    if (ap != bp) return false;
                }
            }
            return true;
        };
        // per item: the (node, index) of its list's first occurrence (itself when first)
        std::vector<std::vector<uint64_t>> first_of(N);
        for (uint32_t n = 0; n < N; ++n) first_of[n].assign(parts[n].items.size(), 0);
        parallel(S, [&](uint32_t s) {
            std::unordered_multimap<uint64_t, uint64_t> seen;      // hash -> (node << 32 | index)
            for (uint32_t n = 0; n < N; ++n)
                for (size_t i = 0; i < parts[n].items.size(); ++i) {
                    const PoolItem &it = parts[n].items[i];
                    if (mix64(it.hash ^ 0x2545F4914F6CDD1Dull) % S != s) continue;
                    uint64_t f = ((uint64_t)n << 32) | i;
                    auto r = seen.equal_range(it.hash);
                    for (auto x = r.first; x != r.second; ++x)
                        if (same(parts[x->second >> 32].items[(uint32_t)x->second], it)) { f = x->second; break; }
                    if (f == (((uint64_t)n << 32) | i)) seen.emplace(it.hash, f);
                    first_of[n][i] = f;
                }
        });
        uint64_t off = 0;                                   // offsets in walk order
        for (uint32_t n = 0; n < N; ++n)
            for (size_t i = 0; i < parts[n].items.size(); ++i) {
                PoolItem &it = parts[n].items[i];
                const uint64_t f = first_of[n][i];
                it.is_first = f == (((uint64_t)n << 32) | i);
                if (it.is_first) { it.off = off; off += it.cnt; }
                else it.off = parts[f >> 32].items[(uint32_t)f].off;
            }
        E = off;
    }
    if (times) tp[2] = wall();
    // phase C: offsets of every node's part, then the parts rebased into the trace
    std::vector<uint64_t> g_off(N + 1, 0), j_off(N + 1, 0), new_off(N + 1, 0), r_off(N + 1, 0), ga_off(N + 1, 0),
        sc_o(N + 1, 0), ee_o(N + 1, 0), pl_o(N + 1, 0), pr_o(N + 1, 0), fr_o(N + 1, 0), cfr_o(N + 1, 0), ev_o(N + 1, 0),
        rep_o(N + 1, 0);
    for (uint32_t n = 0; n < N; ++n) {
        const NodePart &P = parts[n];
        g_off[n + 1] = g_off[n] + P.m_type.size();
        j_off[n + 1] = j_off[n] + P.b_msg.size();
        new_off[n + 1] = new_off[n] + P.new_batches;
        r_off[n + 1] = r_off[n] + nodes[n].r_iid.size();
        ga_off[n + 1] = ga_off[n] + nodes[n].g_a.size();
        sc_o[n + 1] = sc_o[n] + P.sc_type.size();
        ee_o[n + 1] = ee_o[n] + P.ee_msg.size();
        pl_o[n + 1] = pl_o[n] + P.pl.size();
        pr_o[n + 1] = pr_o[n] + P.prop_seq.size();
        fr_o[n + 1] = fr_o[n] + P.fr.size();
        cfr_o[n + 1] = cfr_o[n] + P.cfr.size();
        ev_o[n + 1] = ev_o[n] + P.evp.size();
        ht.dropped += P.dropped;
        ht.part_dropped += P.part_dropped;
        ht.any_sparse = ht.any_sparse || P.any_sparse;
    }
    const uint64_t GK = g_off[N], JB = j_off[N];
    ht.m_type.resize(GK); ht.m_src.resize(GK); ht.m_cnt.resize(GK); ht.m_node.resize(GK);
    ht.m_ballot.resize(GK); ht.m_aux.resize(GK); ht.m_ent.resize(GK); ht.m_seq.resize(GK); ht.m_flags0.resize(GK);
    if (member) { ht.m_ver.resize(GK); ht.ee_msg.resize(ee_o[N]); ht.sc_ver.resize(sc_o[N]); ht.ee_off.assign(N + 1, 0); }
    ht.sc_type.resize(sc_o[N]); ht.sc_key.resize(sc_o[N]); ht.sc_idx.resize(sc_o[N]);
    ht.prop_seq.resize(pr_o[N]); ht.prop_off.assign(N + 1, 0);
    ht.e_iid.resize(E); ht.e_val.resize(E);
    if (member) ht.e_pid.resize(E);
    ht.r_pid.resize(r_off[N]); ht.r_val.resize(r_off[N]); ht.r_iid.resize(r_off[N]);
    ht.g_a.resize(ga_off[N]); ht.g_b.resize(ga_off[N]);
    ht.node_off.assign(N + 1, 0);
    ht.b_msg.resize(JB); ht.b_pstart.resize(JB); ht.b_aid.resize(JB);
    if (wc) { ht.b_gid.resize(JB); ht.b_node.resize(JB); }
    Walk W;
    W.fcount.assign(N * NB + 1, 0); W.cfcount.assign(NB + 1, 0); W.pl_cnt.assign(N, 0);
    W.fr.resize(fr_o[N]); W.cfr.resize(cfr_o[N]); W.pl.resize(pl_o[N]);
    W.evp.resize(ev_o[N]); W.evx.resize(ev_o[N]);
    W.sc_off.assign(N + 1, 0);
    W.reps.resize(JB);
    W.b_bal_w.resize(JB);
    W.next.resize(wc ? N : 0);
    const uint64_t gid0 = wc ? wc->batches : 0;
    W.gid_next = gid0 + new_off[N];
    for (uint32_t n = 0; n <= N; ++n) {
        ht.node_off[n] = g_off[n]; W.sc_off[n] = sc_o[n]; ht.prop_off[n] = pr_o[n];
        if (member) ht.ee_off[n] = ee_o[n];
    }
    {   // the pool's lists, copied from their first occurrences (mostly the first node's: split evenly)
        std::vector<const PoolItem *> firsts;
        for (uint32_t n = 0; n < N; ++n)
            for (const PoolItem &it : parts[n].items) if (it.is_first) firsts.push_back(&it);
        const uint32_t C = std::max<uint32_t>(1, std::min<uint32_t>(4 * threads, (uint32_t)firsts.size()));
        parallel(C, [&](uint32_t c) {
            for (size_t i = firsts.size() * c / C; i < firsts.size() * (c + 1) / C; ++i) {
                const PoolItem &it = *firsts[i];
                const NodeStream &ns = nodes[it.node];
                if (it.carried) {
                    for (uint32_t q = 0; q < it.cnt; ++q) {
                        ht.e_iid[it.off + q] = (*it.carried)[q].first;
                        ht.e_val[it.off + q] = (*it.carried)[q].second;
                        if (member) ht.e_pid[it.off + q] = 0;
                    }
                    continue;
                }
                std::memcpy(ht.e_iid.data() + it.off, ns.e_iid.data() + it.first, 8ull * it.cnt);
                std::memcpy(ht.e_val.data() + it.off, ns.e_val.data() + it.first, 8ull * it.cnt);
                if (member) {
                    if (ns.e_pid.empty()) std::fill(ht.e_pid.begin() + it.off, ht.e_pid.begin() + it.off + it.cnt, 0);
                    else std::memcpy(ht.e_pid.data() + it.off, ns.e_pid.data() + it.first, 8ull * it.cnt);
                }
            }
        });
    }
    parallel(N, [&](uint32_t n) {
        const NodePart &P = parts[n];
        const NodeStream &ns = nodes[n];
        const uint64_t go = g_off[n], jo = j_off[n], ro = r_off[n], gao = ga_off[n];
        std::copy(ns.r_pid.begin(), ns.r_pid.end(), ht.r_pid.begin() + ro);
        std::copy(ns.r_val.begin(), ns.r_val.end(), ht.r_val.begin() + ro);
        std::copy(ns.r_iid.begin(), ns.r_iid.end(), ht.r_iid.begin() + ro);
        std::copy(ns.g_a.begin(), ns.g_a.end(), ht.g_a.begin() + gao);
        std::copy(ns.g_b.begin(), ns.g_b.end(), ht.g_b.begin() + gao);
        for (size_t g = 0; g < P.m_type.size(); ++g) {
            const uint64_t G2 = go + g;
            const uint8_t t = P.m_type[g];
            ht.m_type[G2] = t; ht.m_src[G2] = P.m_src[g]; ht.m_cnt[G2] = P.m_cnt[g]; ht.m_node[G2] = n;
            ht.m_ballot[G2] = P.m_ballot[g]; ht.m_aux[G2] = P.m_aux[g]; ht.m_seq[G2] = P.m_seq[g];
            ht.m_flags0[G2] = P.m_flags0[g];
            if (member) ht.m_ver[G2] = P.m_ver[g];
            const uint64_t e = P.m_ent[g];
            ht.m_ent[G2] = t == MPX_MSG_PREPARE ? e + gao : t == MPX_MSG_PREPARE_REPLY ? e + ro :
                           (t == MPX_MSG_ACCEPT || t == MPX_MSG_COMMIT || t == MPX_MSG_P_BATCH) ? P.items[e].off : e;
        }
        for (size_t i = 0; i < P.sc_type.size(); ++i) {
            ht.sc_type[sc_o[n] + i] = P.sc_type[i]; ht.sc_key[sc_o[n] + i] = P.sc_key[i];
            ht.sc_idx[sc_o[n] + i] = P.sc_idx[i] == NONE32 ? 0 : (uint32_t)(go + P.sc_idx[i]);
            if (member) ht.sc_ver[sc_o[n] + i] = P.sc_ver[i];
        }
        for (size_t i = 0; i < P.ee_msg.size(); ++i) ht.ee_msg[ee_o[n] + i] = (uint32_t)(go + P.ee_msg[i]);
        for (size_t i = 0; i < P.pl.size(); ++i) W.pl[pl_o[n] + i] = (uint32_t)(go + P.pl[i]);
        W.pl_cnt[n] = P.pl.size();
        std::copy(P.prop_seq.begin(), P.prop_seq.end(), ht.prop_seq.begin() + pr_o[n]);
        for (size_t j = 0; j < P.b_msg.size(); ++j) {
            const uint64_t J = jo + j;
            ht.b_msg[J] = P.b_msg[j] == NONE32 ? NONE32 : (uint32_t)(go + P.b_msg[j]);
            ht.b_pstart[J] = P.b_pstart[j] == NONE32 ? NONE32 : (uint32_t)(go + P.b_pstart[j]);
            ht.b_aid[J] = P.b_aid[j];
            const uint32_t gid = P.b_gid[j] >= gid0 ? (uint32_t)(P.b_gid[j] + new_off[n]) : P.b_gid[j];
            if (wc) { ht.b_gid[J] = gid; ht.b_node[J] = n; }
            W.b_bal_w[J] = P.b_bal[j];
            auto &rp = W.reps[J];
            rp.resize(P.reps[j].size());
            for (size_t q = 0; q < rp.size(); ++q) rp[q] = (uint32_t)(go + P.reps[j][q]);
        }
        for (size_t i = 0; i < P.fr.size(); ++i) {
            FragKey x = P.fr[i];
            x.f.msg = (uint32_t)(go + x.f.msg);
            x.f.entry = P.fr_item[i] == NONE32 ? x.f.entry + ro : P.items[P.fr_item[i]].off + x.f.entry;
            W.fr[fr_o[n] + i] = x;
        }
        for (size_t i = 0; i < P.cfr.size(); ++i) {
            FragKey x = P.cfr[i];
            x.f.msg = (uint32_t)(jo + x.f.msg);
            x.f.entry = P.items[P.cfr_item[i]].off + x.f.entry;
            W.cfr[cfr_o[n] + i] = x;
        }
        for (size_t i = 0; i < P.evp.size(); ++i) {
            const uint32_t g = P.evp[i].second;
            W.evp[ev_o[n] + i] = {P.evp[i].first, (uint32_t)(go + g)};
            W.evx[ev_o[n] + i] = P.m_type[g] == MPX_MSG_PREPARE ? P.evx[i] + gao : P.evx[i];
        }
    });
    if (times) tp[3] = wall();
    // (counts and the window's carry: serial, small)
    for (const FragKey &x : W.fr) W.fcount[x.key]++;
    for (const FragKey &x : W.cfr) W.cfcount[x.key]++;
    if (wc)
        for (uint32_t n = 0; n < N; ++n) {
            NodePart &P = parts[n];
            for (uint64_t b : P.state_b) W.state_new.push_back({n, b});
            NodeCarry &c = W.next[n];
            c = std::move(P.carry);
            for (auto &x : c.live) if (x.second >= gid0) x.second = (uint32_t)(x.second + new_off[n]);
            W.ents_gone.insert(W.ents_gone.end(), P.ents_gone.begin(), P.ents_gone.end());
            for (auto &x : P.ents_new) W.ents_new[(uint32_t)(x.first + new_off[n])] = std::move(x.second);
        }
    if (!times) return finish_trace(ht, W, N, NB, sb, slen, member, wc, threads);
    tp[4] = wall();
    const int rc = finish_trace(ht, W, N, NB, sb, slen, member, wc, threads);
    const double te = wall();
    std::fprintf(stderr, "[mpx] build_trace: walk %.1f ms, pool %.1f ms, rebase %.1f ms, carry %.1f ms, finish %.1f ms\n",
                 (tp[1] - tp[0]) * 1e3, (tp[2] - tp[1]) * 1e3, (tp[3] - tp[2]) * 1e3, (tp[4] - tp[3]) * 1e3, (te - tp[4]) * 1e3);
    return rc;
}

int decode_parallel(ValueTable &vt, std::vector<NodeStream> &nodes, std::vector<NodeStream> &parts,
                    const std::vector<StreamSlice> &sl, bool member, std::vector<EpochLearn> *el,
                    uint64_t sb, uint64_t se, IngestViolation &iv, uint32_t threads, uint64_t chunk_bytes)
{
    const uint32_t N = (uint32_t)sl.size();
    if (nodes.size() < N) return MPX_E_INVAL;
    threads = std::max(1u, threads);
    struct Chunk { uint32_t n; uint64_t k0, k1; };
    std::vector<Chunk> chunks;
    {
        uint64_t total = 0;
        for (const auto &x : sl) if (x.cnt) total += x.offs[x.cnt] - x.offs[0];
        const uint64_t target = el ? ~0ull : chunk_bytes ? chunk_bytes : std::max<uint64_t>(total / (4ull * threads), 1u << 20);
        for (uint32_t n = 0; n < N; ++n) {
            const StreamSlice &x = sl[n];
            uint64_t k = 0;
            do {
                uint64_t k1 = x.cnt;
                if (target != ~0ull && x.offs[x.cnt] - x.offs[k] > target) {
                    // (a bad offset table is caught by the decode: offs[i + 1] < offs[i])
                    k1 = (uint64_t)(std::upper_bound(x.offs + k, x.offs + x.cnt, x.offs[k] + target) - x.offs);
                    k1 = std::min(x.cnt, std::max(k1, k + 1));
                }
                chunks.push_back({n, k, k1});
                k = k1;
            } while (k < x.cnt);
        }
    }
    if (parts.size() < chunks.size()) parts.resize(chunks.size());
    std::vector<IngestViolation> ivs(chunks.size());
    std::vector<int> rcs(chunks.size(), MPX_OK);
    SectionCache sc;                                 // (one decode per distinct entry list, this call)
    sc.id_base = vt.sections.fetch_add(1ull << 40);
    const bool times = ab_env("MPX_DECODE_TIMES") != nullptr;
    auto wall = []() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t0 = times ? wall() : 0;
    std::atomic<size_t> next{0};
    auto work = [&]() {
        for (size_t c; (c = next.fetch_add(1)) < chunks.size();) {
            const Chunk &ch = chunks[c];
            const StreamSlice &x = sl[ch.n];
            NodeStream &ns = ch.k0 == 0 ? nodes[ch.n] : parts[c];
            if (ch.k0) ns.clear();
            for (uint64_t i = ch.k0; i < ch.k1; ++i) {
                if (x.offs[i + 1] < x.offs[i]) { rcs[c] = MPX_E_INVAL; break; }
                const uint8_t *m = x.bytes + x.offs[i];
                const size_t len = (size_t)(x.offs[i + 1] - x.offs[i]);
                rcs[c] = member ? decode_record_member(vt, ns, ch.n, m, len, sb, se, ivs[c], el ? &(*el)[ch.n] : nullptr, &sc)
                                : decode_record(vt, ns, ch.n, N, m, len, sb, se, ivs[c], &sc);
                if (rcs[c]) break;
            }
        }
    };
    {
        std::vector<std::thread> th;
        for (uint32_t k = 1; k < std::min<size_t>(threads, chunks.size()); ++k) th.emplace_back(work);
        work();
        for (auto &t : th) t.join();
    }
    for (size_t c = 0; c < chunks.size(); ++c) TRY_RC(rcs[c]);
    const double t1 = times ? wall() : 0;
    // every node's later chunks in order (a thread per node): entry offsets and violation
    // record indices rebased
    auto append = [&](uint32_t n) {
        NodeStream &ns = nodes[n];
        for (size_t c = 0; c < chunks.size(); ++c) {
            if (chunks[c].n != n || chunks[c].k0 == 0) continue;
            const NodeStream &p = parts[c];
            const uint64_t rb = ns.type.size(), eb = ns.e_iid.size(), qb = ns.r_iid.size(), gb = ns.g_a.size();
            ivs[c].seq += rb;
            auto cat = [](auto &dst, const auto &src) { dst.insert(dst.end(), src.begin(), src.end()); };
            cat(ns.type, p.type); cat(ns.src, p.src); cat(ns.ballot, p.ballot); cat(ns.aux, p.aux);
            cat(ns.cnt, p.cnt); cat(ns.ver, p.ver); cat(ns.part, p.part); cat(ns.sec, p.sec);
            cat(ns.e_iid, p.e_iid); cat(ns.e_val, p.e_val); cat(ns.e_pid, p.e_pid);
            cat(ns.r_iid, p.r_iid); cat(ns.r_pid, p.r_pid); cat(ns.r_val, p.r_val);
            cat(ns.g_a, p.g_a); cat(ns.g_b, p.g_b);
            ns.ent.reserve(ns.ent.size() + p.ent.size());
            for (size_t k = 0; k < p.ent.size(); ++k) {
                const uint8_t t = p.type[k];
                const uint64_t base = t == MPX_MSG_PREPARE ? gb : t == MPX_MSG_PREPARE_REPLY ? qb :
                                      (t == MPX_MSG_ACCEPT || t == MPX_MSG_COMMIT || t == MPX_MSG_P_BATCH) ? eb : 0;
                ns.ent.push_back(p.ent[k] + base);
            }
        }
    };
    {
        std::vector<std::thread> th;
        for (uint32_t n = 1; n < N; ++n) th.emplace_back(append, n);
        if (N) append(0);
        for (auto &t : th) t.join();
    }
    if (times)
        std::fprintf(stderr, "[mpx] decode_parallel: %zu chunks on %u threads: records %.1f ms, append %.1f ms\n",
                     chunks.size(), threads, (t1 - t0) * 1e3, (wall() - t1) * 1e3);
#ifdef MPX_DECODE_PROF
    std::fprintf(stderr, "[mpx] decode cycles (M): claim %.0f own %.0f skim %.0f copy %.0f nocache %.0f\n",
                 g_prof[0] * 1e-6, g_prof[1] * 1e-6, g_prof[2] * 1e-6, g_prof[3] * 1e-6, g_prof[4] * 1e-6);
    for (auto &x : g_prof) x = 0;
#endif
    for (size_t c = 0; c < chunks.size(); ++c)       // first violation in record order
        if (ivs[c].count) {
            if (!iv.code) { iv.code = ivs[c].code; iv.node = ivs[c].node; iv.seq = ivs[c].seq; iv.iid = ivs[c].iid; }
            iv.count += ivs[c].count;
        }
    return MPX_OK;
}

}  // namespace mpx
