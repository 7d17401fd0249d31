// rxg_mirror.h — host side of the device TCB and ARP mirrors ("TCB mirror").
//
// The reference mutates tcbs[] in place: alloc_tcb appends (tcp_tcb.c:97-103), remove_tcb
// NULLs a slot (:175-186), socket_bind / tcp_listen / tcp_syn_sent write tuples and states
// (socket_interface.c:80-83, tcp_states.c:25-27,185-188).  findtcb then scans the whole
// array (tcp_tcb.c:127-173).  rxg answers findtcb from a device hash table; this class keeps
// the host's canonical copy of tcbs[] and, for every write, the few device words that change:
//
//   * exact-tuple buckets (nb x 4 slots of {ports, ipv4_dst raw, ipv4_src host, value}):
//     value = the LOWEST live index holding the tuple | its state << 24 (pass 1,
//     tcp_tcb.c:145-159).  Linear probing over buckets; a lookup ends at the first bucket
//     with a free slot.  Insertion fills the first bucket with a free slot from the home
//     bucket.  Deletion empties the slot and then moves back any later entry whose probe
//     path crosses the hole (backward shift over buckets), so no tombstones exist and the
//     kernel's probe loop stays as it is.
//   * listen[65536]: lowest live LISTENING index per dport (pass 2, :160-169).
//   * min_null: lowest NULL slot below Ntcb (pass 2's NULL dereference, reported as a flag).
//
// A write costs O(1) device words (a bucket slot or two per moved entry, a listen word)
// whatever Ntcb is.  Only two cases rescan: a table past load 1/2 is rebuilt at twice the
// size (amortised O(1) per insertion), and removing the lowest of several TCBs that share a
// tuple (a retransmitted SYN makes a second child, tcp_states.c:155) looks for the next one.
//
// Host-only; the device side applies the patches with one small kernel per burst
// (rxg_kernels.hip mirror_patch).  tests/test_mirror.py drives this header directly on the
// CPU against a naive two-pass findtcb.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <climits>
#include <map>
#include <set>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "rxg.h"
#include "rxg_common.h"

namespace rxg {

// One device word group to write: buckets[index] (16 B), listen[index] (4 B) or
// arp[index] (8 B).  Applied by the mirror_patch kernel, one thread per patch.
enum : uint32_t { kPatchBucket = 0, kPatchListen = 1, kPatchArp = 2 };
struct MirrorPatch {
    uint32_t target;
    uint32_t index;
    uint32_t v[4];
};
static_assert(sizeof(MirrorPatch) == 24, "MirrorPatch layout");

struct Slot {
    uint32_t ports, dst, src, val;  // val = kEmpty: free
};

struct TupleKey {
    uint32_t ports, dst, src;
    bool operator==(const TupleKey &o) const { return ports == o.ports && dst == o.dst && src == o.src; }
};
struct TupleKeyHash {
    size_t operator()(const TupleKey &k) const { return tuple_hash(k.ports, k.dst, k.src); }
};

inline bool port_in_range(int32_t p) { return p >= 0 && p <= 0xFFFF; }

// The key findtcb pass 1 compares (tcp_tcb.c:152-155); false for a tuple whose int ports lie
// outside 0..65535, which never equals a packet's u16 ports.
inline bool tcb_key(const rxg_tcb_tuple &t, TupleKey &k)
{
    if (!port_in_range(t.dport) || !port_in_range(t.sport)) return false;
    k = TupleKey{((uint32_t)t.dport << 16) | (uint32_t)t.sport, t.ipv4_dst, t.ipv4_src};
    return true;
}

// ---- flow-affinity sharding: the Toeplitz RSS hash NICs steer rx queues by
// (Microsoft RSS, the 40-byte key DPDK drivers default to), over the 12 wire bytes IPv4/TCP
// hashes: src ip | dst ip | src port | dst port = frame bytes 26..37, and the default
// redirection table (RXG_RSS_RETA_SIZE entries filled round-robin: entry i -> queue i % n).
static const uint8_t kRssKey[40] = {0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3,
                                    0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3,
                                    0x80, 0x30, 0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa};
inline uint32_t rss_toeplitz(const uint8_t *in, int n)
{
    uint32_t h = 0, win = ((uint32_t)kRssKey[0] << 24) | ((uint32_t)kRssKey[1] << 16) | ((uint32_t)kRssKey[2] << 8) | kRssKey[3];
    for (int i = 0; i < n; ++i) {
        const uint8_t nk = kRssKey[i + 4];
        for (int b = 7; b >= 0; --b) {
            if ((in[i] >> b) & 1) h ^= win;
            win = (win << 1) | ((nk >> b) & 1u);
        }
    }
    return h;
}
// The same hash of 12 bytes by byte tables (a mirror rebuild hashes every key: 12 lookups
// instead of 96 conditional XORs); built once, checked against rss_toeplitz by the tests.
struct RssTable12 {
    uint32_t t[12][256];
    RssTable12()
    {
        for (int i = 0; i < 12; ++i)
            for (int v = 0; v < 256; ++v) {
                uint8_t in[12] = {0};
                in[i] = (uint8_t)v;
                t[i][v] = rss_toeplitz(in, 12);
            }
    }
};
inline uint32_t rss_toeplitz12(const uint8_t *in)
{
    static const RssTable12 tab;  // thread-safe static init
    uint32_t h = 0;
    for (int i = 0; i < 12; ++i) h ^= tab.t[i][in[i]];
    return h;
}
inline uint32_t rss_queue(uint32_t h, uint32_t nparts) { return (h % RXG_RSS_RETA_SIZE) % nparts; }
// A pass-1 key's wire bytes: src ip is held in host order (ntohl), dst raw as read, ports
// as (dport << 16) | sport in host order (tcp_tcb.c:152-155)
inline uint32_t key_part(const TupleKey &k, uint32_t nparts)
{
    const uint8_t w[12] = {(uint8_t)(k.src >> 24), (uint8_t)(k.src >> 16), (uint8_t)(k.src >> 8), (uint8_t)k.src,
                           (uint8_t)k.dst, (uint8_t)(k.dst >> 8), (uint8_t)(k.dst >> 16), (uint8_t)(k.dst >> 24),
                           (uint8_t)(k.ports >> 8), (uint8_t)k.ports, (uint8_t)(k.ports >> 24), (uint8_t)(k.ports >> 16)};
    return rss_queue(rss_toeplitz12(w), nparts);
}

class TcbMirror {
  public:
    // Flow-affinity partition: with nparts > 1 the exact-tuple table holds only the keys whose
    // RSS queue is `part`; the listener map, liveness and the lowest NULL slot stay whole
    // (findtcb's pass 2 reads the whole slot array), so a frame steered here classifies as
    // against the whole table.
    uint32_t part = 0, nparts = 1;
    // canonical host copy of tcbs[0..Ntcb)
    std::vector<rxg_tcb_tuple> tcb;
    std::vector<uint8_t> live;

    // derived state = what the device holds (valid unless need_rebuild)
    bool need_rebuild = true;
    std::vector<Slot> slots;      // nb * kSlotsPerBucket
    uint32_t nb = 0;
    std::vector<int32_t> listen;  // 65536
    int32_t min_null = INT32_MAX;
    std::vector<MirrorPatch> patches;  // device writes since the last patches_taken(); at
                                       // most one per device word (a rewrite updates it)
    uint32_t max_load_pct = 50;        // keys per slot, percent: rebuilt past it
    uint64_t rescans = 0, moves = 0;   // diagnostics (tests)

    // The caller uploaded `patches`: forget them.
    void patches_taken()
    {
        for (const MirrorPatch &q : patches) (q.target == kPatchBucket ? slot_pp[q.index] : listen_pp[q.index]) = kNone;
        patches.clear();
    }

    int32_t ntcb() const { return (int32_t)tcb.size(); }

    // ---- writes (the caller validated idx / state ranges)
    void load(const rxg_tcb_tuple *t, const uint8_t *lv, int32_t n)
    {
        tcb.assign(t, t + n);
        if (lv)
            live.assign(lv, lv + n);
        else
            live.assign((size_t)n, 1);
        need_rebuild = true;
        patches.clear();  // the rebuild resets the pending-patch index
    }

    void upsert(int32_t idx, const rxg_tcb_tuple &t)
    {
        const int32_t old_n = ntcb();
        if (idx >= old_n) {
            tcb.resize((size_t)idx + 1, rxg_tcb_tuple{});
            live.resize((size_t)idx + 1, 0);
        }
        if (need_rebuild) {
            tcb[idx] = t;
            live[idx] = 1;
            return;
        }
        if (idx > old_n) min_null = std::min(min_null, old_n);  // old_n .. idx-1 appear NULL
        const bool was_live = idx < old_n && live[idx];
        if (was_live) {
            const rxg_tcb_tuple o = tcb[idx];
            if (same_key(o, t)) {  // same tuple: only the state can change
                tcb[idx] = t;
                state_changed(idx, o.state, t.state);
                return;
            }
            live[idx] = 0;  // drop the old tuple's contributions (idx excluded from rescans)
            drop_key(o, idx);
            if (o.state == RXG_LISTENING) listener_erase(o.dport, idx);
        }
        tcb[idx] = t;
        live[idx] = 1;
        if (!was_live && idx == min_null) advance_min_null(idx + 1);
        add_key(t, idx);
        if (t.state == RXG_LISTENING) listener_insert(t.dport, idx);
    }

    void remove(int32_t idx)
    {
        if (!live[idx]) return;
        live[idx] = 0;
        if (need_rebuild) return;
        const rxg_tcb_tuple &o = tcb[idx];
        drop_key(o, idx);
        if (o.state == RXG_LISTENING) listener_erase(o.dport, idx);
        min_null = std::min(min_null, idx);
    }

    void set_state(int32_t idx, uint8_t st)
    {
        const uint8_t old = tcb[idx].state;
        tcb[idx].state = st;
        if (!need_rebuild) state_changed(idx, old, st);
    }

    // ---- the full build (first use, rxg_tcb_load, growth past load 1/2)
    void rebuild()
    {
        const int32_t n = ntcb();
        std::unordered_map<TupleKey, KeyEntry, TupleKeyHash> k;
        k.reserve((size_t)n * 2 + 1);
        listeners.clear();
        min_null = INT32_MAX;
        for (int32_t i = 0; i < n; ++i) {
            if (!live[i]) {
                if (min_null == INT32_MAX) min_null = i;
                continue;
            }
            const rxg_tcb_tuple &t = tcb[i];
            TupleKey key;
            if (key_of(t, key)) {
                auto it = k.find(key);
                if (it == k.end())
                    k.emplace(key, KeyEntry{i, 1u, 0u});  // ascending i: the first is the lowest
                else
                    ++it->second.count;
            }
            if (t.state == RXG_LISTENING && port_in_range(t.dport)) listeners[t.dport].insert(i);
        }
        nb = 1;
        while ((uint64_t)nb * kSlotsPerBucket * max_load_pct < (uint64_t)k.size() * 100u) nb <<= 1;
        slots.assign((size_t)nb * kSlotsPerBucket, Slot{0u, 0u, 0u, kEmpty});
        for (auto &kv : k) kv.second.pos = place(kv.first, value_of(kv.second.min_idx));
        keys.swap(k);
        listen.assign(65536, -1);
        for (const auto &l : listeners)
            if (!l.second.empty()) listen[l.first] = *l.second.begin();
        need_rebuild = false;
        patches.clear();
        slot_pp.assign(slots.size(), kNone);
        listen_pp.assign(65536, kNone);
    }

    // ---- pass 1 + pass 2 exactly as the device kernel answers them (tests)
    int32_t find(uint32_t ports, uint32_t dst_raw, uint32_t src_host, uint32_t dport, uint8_t *state,
                 bool *listen_hit) const
    {
        uint32_t b = tuple_hash(ports, dst_raw, src_host) & (nb - 1);
        for (uint32_t p = 0; p < nb; ++p) {
            bool empty = false;
            for (int s = 0; s < kSlotsPerBucket; ++s) {
                const Slot &e = slots[(size_t)b * kSlotsPerBucket + s];
                if (e.val != kEmpty && e.ports == ports && e.dst == dst_raw && e.src == src_host) {
                    *state = (uint8_t)(e.val >> kStateShift);
                    *listen_hit = false;
                    return (int32_t)(e.val & kIdxMask);
                }
                empty |= e.val == kEmpty;
            }
            if (empty) break;
            b = (b + 1) & (nb - 1);
        }
        const int32_t l = listen[dport & 0xFFFF];
        *listen_hit = l >= 0;
        *state = l >= 0 ? (uint8_t)RXG_LISTENING : (uint8_t)RXG_STATE_NONE;
        return l;
    }

    size_t nkeys() const { return keys.size(); }

  private:
    struct KeyEntry {
        int32_t min_idx;  // lowest live index holding the tuple
        uint32_t count;   // live indices holding it
        uint32_t pos;     // its slot
    };
    std::unordered_map<TupleKey, KeyEntry, TupleKeyHash> keys;
    std::map<int32_t, std::set<int32_t>> listeners;  // dport -> live LISTENING indices
    static constexpr uint32_t kNone = 0xFFFFFFFFu;
    std::vector<uint32_t> slot_pp, listen_pp;  // word -> its pending patch, or kNone

    bool key_of(const rxg_tcb_tuple &t, TupleKey &k) const
    {
        return tcb_key(t, k) && (nparts <= 1 || key_part(k, nparts) == part);
    }
    static bool same_key(const rxg_tcb_tuple &a, const rxg_tcb_tuple &b)
    {
        return a.dport == b.dport && a.sport == b.sport && a.ipv4_dst == b.ipv4_dst && a.ipv4_src == b.ipv4_src;
    }
    uint32_t value_of(int32_t idx) const { return (uint32_t)idx | ((uint32_t)tcb[idx].state << kStateShift); }
    uint32_t home(const TupleKey &k) const { return tuple_hash(k.ports, k.dst, k.src) & (nb - 1); }

    void emit(std::vector<uint32_t> &pp, const MirrorPatch &q)
    {
        if (pp[q.index] != kNone) {
            patches[pp[q.index]] = q;  // the word's pending patch takes the new value
        } else {
            pp[q.index] = (uint32_t)patches.size();
            patches.push_back(q);
        }
    }
    void emit_slot(uint32_t pos)
    {
        const Slot &e = slots[pos];
        emit(slot_pp, MirrorPatch{kPatchBucket, pos, {e.ports, e.dst, e.src, e.val}});
    }
    void emit_listen(uint32_t dport)
    {
        emit(listen_pp, MirrorPatch{kPatchListen, dport, {(uint32_t)listen[dport], 0u, 0u, 0u}});
    }

    // first free slot from the key's home bucket (load <= 1/2: one exists)
    uint32_t place(const TupleKey &k, uint32_t val)
    {
        uint32_t b = home(k);
        for (;;) {
            for (int s = 0; s < kSlotsPerBucket; ++s) {
                const uint32_t pos = b * kSlotsPerBucket + (uint32_t)s;
                if (slots[pos].val == kEmpty) {
                    slots[pos] = Slot{k.ports, k.dst, k.src, val};
                    return pos;
                }
            }
            b = (b + 1) & (nb - 1);
        }
    }

    void add_key(const rxg_tcb_tuple &t, int32_t idx)
    {
        TupleKey k;
        if (!key_of(t, k)) return;
        auto it = keys.find(k);
        if (it != keys.end()) {
            ++it->second.count;
            if (idx < it->second.min_idx) {
                it->second.min_idx = idx;
                slots[it->second.pos].val = value_of(idx);
                emit_slot(it->second.pos);
            }
            return;
        }
        if ((uint64_t)(keys.size() + 1) * 100u > (uint64_t)nb * kSlotsPerBucket * max_load_pct) {
            need_rebuild = true;  // past load 1/2: rebuilt at twice the size on the next sync
            return;
        }
        const uint32_t pos = place(k, value_of(idx));
        keys.emplace(k, KeyEntry{idx, 1u, pos});
        emit_slot(pos);
    }

    // idx (already not live, or about to get another tuple) no longer holds t's tuple
    void drop_key(const rxg_tcb_tuple &t, int32_t idx)
    {
        TupleKey k;
        if (!key_of(t, k)) return;
        auto it = keys.find(k);
        if (it == keys.end()) return;
        KeyEntry &e = it->second;
        if (--e.count == 0) {
            const uint32_t pos = e.pos;
            keys.erase(it);
            delete_slot(pos);
            return;
        }
        if (e.min_idx != idx) return;
        // the lowest of several TCBs sharing the tuple went: the next lowest takes over
        ++rescans;
        int32_t nxt = -1;
        for (int32_t i = idx + 1; i < ntcb() && nxt < 0; ++i)
            if (live[i] && i != idx && same_key(tcb[i], t)) nxt = i;
        if (nxt < 0) {  // cannot happen while count > 0; stay consistent anyway
            const uint32_t pos = e.pos;
            keys.erase(it);
            delete_slot(pos);
            return;
        }
        e.min_idx = nxt;
        slots[e.pos].val = value_of(nxt);
        emit_slot(e.pos);
    }

    // Empty slot pos, then close the hole: an entry of a later bucket j whose probe path
    // [home, j) crosses the hole's bucket moves into the hole (the hole moves to j); stop at
    // a bucket that already had a free slot, since no probe path crosses it.
    void delete_slot(uint32_t pos)
    {
        const uint32_t mask = nb - 1;
        slots[pos] = Slot{0u, 0u, 0u, kEmpty};
        uint32_t hole = pos;
        uint32_t j = pos / kSlotsPerBucket;
        for (uint32_t step = 1; step < nb; ++step) {
            j = (j + 1) & mask;
            bool had_free = false;
            for (int s = 0; s < kSlotsPerBucket; ++s) had_free |= slots[j * kSlotsPerBucket + s].val == kEmpty;
            const uint32_t hb = hole / kSlotsPerBucket;
            for (int s = 0; s < kSlotsPerBucket; ++s) {
                const uint32_t q = j * kSlotsPerBucket + (uint32_t)s;
                const Slot e = slots[q];
                if (e.val == kEmpty) continue;
                const TupleKey k{e.ports, e.dst, e.src};
                const uint32_t h = home(k);
                if (((hb - h) & mask) < ((j - h) & mask)) {
                    slots[hole] = e;
                    emit_slot(hole);
                    keys.find(k)->second.pos = hole;
                    slots[q] = Slot{0u, 0u, 0u, kEmpty};
                    hole = q;
                    ++moves;
                    break;
                }
            }
            if (had_free) break;
        }
        emit_slot(hole);  // the final hole is empty
    }

    void state_changed(int32_t idx, uint8_t old, uint8_t st)
    {
        if (old == st) return;
        TupleKey k;
        if (key_of(tcb[idx], k)) {
            auto it = keys.find(k);
            if (it != keys.end() && it->second.min_idx == idx) {
                slots[it->second.pos].val = value_of(idx);
                emit_slot(it->second.pos);
            }
        }
        if (old == RXG_LISTENING) listener_erase(tcb[idx].dport, idx);
        if (st == RXG_LISTENING) listener_insert(tcb[idx].dport, idx);
    }

    void listener_insert(int32_t dport, int32_t idx)
    {
        if (!port_in_range(dport)) return;
        auto &s = listeners[dport];
        s.insert(idx);
        if (listen[dport] != *s.begin()) {
            listen[dport] = *s.begin();
            emit_listen((uint32_t)dport);
        }
    }

    void listener_erase(int32_t dport, int32_t idx)
    {
        if (!port_in_range(dport)) return;
        auto it = listeners.find(dport);
        if (it == listeners.end()) return;
        it->second.erase(idx);
        const int32_t v = it->second.empty() ? -1 : *it->second.begin();
        if (it->second.empty()) listeners.erase(it);
        if (listen[dport] != v) {
            listen[dport] = v;
            emit_listen((uint32_t)dport);
        }
    }

    void advance_min_null(int32_t from)
    {
        int32_t i = from;
        while (i < ntcb() && live[i]) ++i;
        min_null = i < ntcb() ? i : INT32_MAX;
    }
};

// ARP mirror: the set of host-order IPv4 addresses add_mac has added (arp.c:282-317), as
// buckets of four keys (rxg_common.h), key 0 = free, probed linearly by bucket; 0.0.0.0 is a
// flag instead (has_zero).  Addresses are only added between loads, so insertion patches
// one key; past load 1/2 the table is rebuilt at twice the size.
class ArpMirror {
  public:
    std::vector<uint32_t> ips;  // add_mac order
    std::unordered_set<uint32_t> set;
    std::vector<uint32_t> slots;  // nb x kArpKeysPerBucket keys
    uint32_t nb = 0;
    bool has_zero = false;
    bool need_rebuild = true;
    std::vector<MirrorPatch> patches;  // one per key (a key is written once between loads)

    void clear()
    {
        ips.clear();
        set.clear();
        has_zero = false;
        need_rebuild = true;
        patches.clear();
    }

    void patches_taken() { patches.clear(); }

    // true when ip is new
    bool add(uint32_t ip)
    {
        if (!set.insert(ip).second) return false;
        ips.push_back(ip);
        if (ip == 0u) {
            has_zero = true;  // travels in the launch's arguments, no table word
            return true;
        }
        if (need_rebuild) return true;
        if ((uint64_t)ips.size() * 2u > (uint64_t)nb * kArpKeysPerBucket) {
            need_rebuild = true;
            return true;
        }
        const uint32_t w = insert(ip);
        patches.push_back(MirrorPatch{kPatchArp, w, {ip, 0u, 0u, 0u}});
        return true;
    }

    void rebuild()
    {
        nb = 4;
        while ((uint64_t)nb * kArpKeysPerBucket < (uint64_t)ips.size() * 2u) nb <<= 1;
        slots.assign((size_t)nb * kArpKeysPerBucket, 0u);
        for (uint32_t ip : ips)
            if (ip) insert(ip);
        need_rebuild = false;
        patches.clear();
    }

    // the kernel's lookup (classify_finish) over a copy of the keys
    static bool lookup(const uint32_t *keys, uint32_t nb, bool has_zero, uint32_t ip)
    {
        if (ip == 0u) return has_zero;
        uint32_t b = arp_hash(ip) & (nb - 1);
        for (uint32_t p = 0; p < nb; ++p) {
            bool free = false;
            for (int k = 0; k < kArpKeysPerBucket; ++k) {
                const uint32_t x = keys[(size_t)b * kArpKeysPerBucket + k];
                if (x == ip) return true;
                free |= x == 0u;
            }
            if (free) return false;
            b = (b + 1) & (nb - 1);
        }
        return false;
    }

  private:
    // the key's word index
    uint32_t insert(uint32_t ip)
    {
        uint32_t b = arp_hash(ip) & (nb - 1);
        for (;;) {
            for (int k = 0; k < kArpKeysPerBucket; ++k) {
                const size_t w = (size_t)b * kArpKeysPerBucket + k;
                if (slots[w] == 0u) {
                    slots[w] = ip;
                    return (uint32_t)w;
                }
            }
            b = (b + 1) & (nb - 1);
        }
    }
};

}  // namespace rxg
