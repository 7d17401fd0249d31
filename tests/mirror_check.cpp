// mirror_check.cpp — CPU check of the incremental TCB / ARP mirror (csrc/rxg_mirror.h).
//
// Random sequences of the reference's tcbs[] writes (alloc_tcb append, tuple rewrite,
// remove_tcb, state changes incl. LISTENING; tcp_tcb.c:34-106,175-186, tcp_states.c:25-27,
// 150-207) are applied to a TcbMirror.  After every burst of writes:
//   * a simulated device copy, updated ONLY by the emitted patches (or a full copy after a
//     rebuild), must equal the mirror's own tables word for word;
//   * lookups through the device copy (the kernel's probe: buckets, then listen[dport])
//     must equal a naive two-pass findtcb over tcbs[] (tcp_tcb.c:127-173): lowest live
//     exact match, else lowest live LISTENING slot on dport; plus the NULL-slot flag.
// Usage: mirror_check SEED OPS KEYS ; prints one line "ok ..." or "FAIL ..." (exit 1).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <set>

#include "rxg_mirror.h"

using namespace rxg;

struct Dev {
    std::vector<Slot> slots;
    std::vector<int32_t> listen;
    std::vector<uint32_t> arp;
};

static int fails = 0;
#define CHECK(cond, ...)                                   \
    do {                                                   \
        if (!(cond)) {                                     \
            if (fails++ < 5) {                             \
                std::printf("FAIL %s:%d ", __FILE__, __LINE__); \
                std::printf(__VA_ARGS__);                  \
                std::printf("\n");                         \
            }                                              \
        }                                                  \
    } while (0)

static void sync_dev(TcbMirror &m, ArpMirror &a, Dev &d, uint64_t &nrebuild, uint64_t &npatch)
{
    std::vector<MirrorPatch> p;
    if (m.need_rebuild) {
        m.rebuild();
        d.slots = m.slots;
        d.listen = m.listen;
        ++nrebuild;
    } else {
        p.insert(p.end(), m.patches.begin(), m.patches.end());
        m.patches_taken();
    }
    if (a.need_rebuild) {
        a.rebuild();
        d.arp = a.slots;
    } else {
        p.insert(p.end(), a.patches.begin(), a.patches.end());
        a.patches_taken();
    }
    // the device kernel applies them in parallel: no two may write the same word
    std::set<std::pair<uint32_t, uint32_t>> words;
    for (const MirrorPatch &q : p) CHECK(words.insert({q.target, q.index}).second, "two patches for one word");
    npatch += p.size();
    for (const MirrorPatch &q : p) {
        if (q.target == kPatchBucket)
            d.slots[q.index] = Slot{q.v[0], q.v[1], q.v[2], q.v[3]};
        else if (q.target == kPatchListen)
            d.listen[q.index] = (int32_t)q.v[0];
        else
            d.arp[q.index] = q.v[0];
    }
}

// the kernel's lookup over the device copy
static int32_t dev_find(const Dev &d, uint32_t nb, uint32_t ports, uint32_t dst, uint32_t src, uint32_t dport,
                        uint32_t &st, bool &lhit)
{
    uint32_t b = tuple_hash(ports, dst, src) & (nb - 1);
    for (uint32_t p = 0; p < nb; ++p) {
        bool empty = false;
        for (int s = 0; s < kSlotsPerBucket; ++s) {
            const Slot &e = d.slots[(size_t)b * kSlotsPerBucket + s];
            if (e.val != kEmpty && e.ports == ports && e.dst == dst && e.src == src) {
                st = e.val >> kStateShift;
                lhit = false;
                return (int32_t)(e.val & kIdxMask);
            }
            empty |= e.val == kEmpty;
        }
        if (empty) break;
        b = (b + 1) & (nb - 1);
    }
    const int32_t l = d.listen[dport];
    lhit = l >= 0;
    st = l >= 0 ? RXG_LISTENING : RXG_STATE_NONE;
    return l;
}

// naive findtcb (tcp_tcb.c:145-169), NULL slots skipped and reported
static int32_t ref_find(const TcbMirror &m, uint32_t dp, uint32_t sp, uint32_t dst, uint32_t src, uint32_t &st,
                        bool &lhit, bool &nslot)
{
    const int32_t n = m.ntcb();
    for (int32_t i = 0; i < n; ++i) {
        const rxg_tcb_tuple &t = m.tcb[i];
        if (m.live[i] && t.dport == (int32_t)dp && t.sport == (int32_t)sp && t.ipv4_dst == dst && t.ipv4_src == src) {
            st = t.state;
            lhit = false;
            nslot = false;
            return i;
        }
    }
    nslot = false;
    for (int32_t i = 0; i < n; ++i) {
        if (!m.live[i]) {
            nslot = true;
            continue;
        }
        if (m.tcb[i].state == RXG_LISTENING && m.tcb[i].dport == (int32_t)dp) {
            st = RXG_LISTENING;
            lhit = true;
            return i;
        }
    }
    st = RXG_STATE_NONE;
    lhit = false;
    return -1;
}

int main(int argc, char **argv)
{
    if (argc != 4) return 2;
    const uint64_t seed = strtoull(argv[1], nullptr, 10);
    const int ops = atoi(argv[2]);
    const int nkeys = atoi(argv[3]);  // tuple pool: small pools make duplicates and clusters
    std::mt19937_64 rng(seed);
    auto R = [&](uint64_t k) { return (uint64_t)(rng() % k); };

    // tuple pool (ports kept in range mostly; a few out-of-range ints, never matchable)
    std::vector<rxg_tcb_tuple> pool((size_t)nkeys);
    for (auto &t : pool) {
        t.dport = R(8) == 0 ? 8080 : 80;
        t.sport = R(200) == 0 ? 70000 : (int32_t)(1024 + R(60000));
        t.ipv4_dst = R(4) ? 0x024EA8C0u : (uint32_t)rng();
        t.ipv4_src = (uint32_t)rng();
        t.state = RXG_TCP_ESTABLISHED;
        t.pad = 0;
        t.identifier = 1;
    }
    TcbMirror m;
    ArpMirror a;
    Dev d;
    uint64_t nrebuild = 0, npatch = 0, nquery = 0;
    // initial table (rxg_tcb_load): a listener and some flows
    {
        std::vector<rxg_tcb_tuple> t0;
        std::vector<uint8_t> l0;
        rxg_tcb_tuple L{80, 0, 0x024EA8C0u, 0, RXG_LISTENING, 0, 1};
        t0.push_back(L);
        l0.push_back(1);
        for (int i = 0; i < nkeys / 2; ++i) {
            t0.push_back(pool[(size_t)R(nkeys)]);
            l0.push_back(R(10) != 0);
        }
        m.load(t0.data(), l0.data(), (int32_t)t0.size());
    }
    std::vector<uint32_t> arp_pool(4096);
    for (auto &x : arp_pool) x = (uint32_t)rng();
    arp_pool[0] = 0u;  // 0.0.0.0: a flag of the launch, not a key
    for (int b = 0; b < 64; ++b) a.add(arp_pool[(size_t)R(arp_pool.size())]);
    sync_dev(m, a, d, nrebuild, npatch);

    const int burst = 16;
    for (int op = 0; op < ops; ++op) {
        const int32_t n = m.ntcb();
        const uint64_t k = R(100);
        if (k < 35) {  // alloc_tcb + tuple write: append (sometimes past Ntcb: NULL slots)
            const int32_t idx = n + (R(20) == 0 ? (int32_t)R(3) : 0);
            rxg_tcb_tuple t = pool[(size_t)R(nkeys)];
            t.state = R(10) == 0 ? RXG_LISTENING : (uint8_t)R(RXG_TCP_STATES);
            if (idx < kMaxTcbs) m.upsert(idx, t);
        } else if (k < 55 && n) {  // rewrite a slot's tuple (tcp_syn_sent), or reuse a NULL slot
            rxg_tcb_tuple t = pool[(size_t)R(nkeys)];
            t.state = (uint8_t)R(RXG_TCP_STATES);
            m.upsert((int32_t)R(n), t);
        } else if (k < 75 && n) {  // remove_tcb
            m.remove((int32_t)R(n));
        } else if (n) {  // state change
            const int32_t idx = (int32_t)R(n);
            if (m.live[idx]) m.set_state(idx, (uint8_t)R(RXG_TCP_STATES));
        }
        if (R(50) == 0) a.add(arp_pool[(size_t)R(arp_pool.size())]);
        if (op % burst != burst - 1) continue;

        sync_dev(m, a, d, nrebuild, npatch);
        CHECK(d.slots.size() == m.slots.size() && std::memcmp(d.slots.data(), m.slots.data(),
                                                              m.slots.size() * sizeof(Slot)) == 0,
              "device buckets differ from the mirror after op %d", op);
        CHECK(d.listen == m.listen, "device listen differs after op %d", op);
        CHECK(d.arp == a.slots, "device ARP table differs after op %d", op);
        // min_null
        int32_t mn = INT32_MAX;
        for (int32_t i = 0; i < m.ntcb(); ++i)
            if (!m.live[i]) {
                mn = i;
                break;
            }
        CHECK(mn == m.min_null, "min_null %d vs %d after op %d", m.min_null, mn, op);
        // lookups: every pool tuple plus a few random ones
        for (int q = 0; q < 24; ++q) {
            rxg_tcb_tuple t = q < 20 ? pool[(size_t)R(nkeys)] : rxg_tcb_tuple{80, (int32_t)R(65536), (uint32_t)rng(),
                                                                               (uint32_t)rng(), 0, 0, 0};
            if (!port_in_range(t.sport)) continue;
            const uint32_t ports = ((uint32_t)t.dport << 16) | (uint32_t)t.sport;
            uint32_t st1, st2;
            bool l1, l2, ns2;
            const int32_t i1 = dev_find(d, m.nb, ports, t.ipv4_dst, t.ipv4_src, (uint32_t)t.dport, st1, l1);
            const int32_t i2 = ref_find(m, (uint32_t)t.dport, (uint32_t)t.sport, t.ipv4_dst, t.ipv4_src, st2, l2, ns2);
            const bool ns1 = m.min_null < (i1 >= 0 && l1 ? i1 : (i1 >= 0 ? INT32_MAX : m.ntcb()));
            CHECK(i1 == i2 && st1 == st2 && l1 == l2, "op %d: device (%d,%u,%d) vs findtcb (%d,%u,%d)", op, i1, st1,
                  (int)l1, i2, st2, (int)l2);
            if (l2 || i2 < 0) CHECK(ns1 == ns2, "op %d: NULL-slot flag %d vs %d", op, (int)ns1, (int)ns2);
            ++nquery;
        }
        // ARP membership
        for (int q = 0; q < 8; ++q) {
            const uint32_t ip = q ? arp_pool[(size_t)R(arp_pool.size())] : 0u;
            const bool found = ArpMirror::lookup(d.arp.data(), a.nb, a.has_zero, ip);
            CHECK(found == (a.set.count(ip) != 0), "ARP membership of %08x", ip);
        }
        if (fails) break;
    }
    if (fails) return 1;
    std::printf("ok ntcb=%d keys=%zu nb=%u rebuilds=%llu patches=%llu moves=%llu rescans=%llu queries=%llu\n",
                m.ntcb(), m.nkeys(), m.nb, (unsigned long long)nrebuild, (unsigned long long)npatch,
                (unsigned long long)m.moves, (unsigned long long)m.rescans, (unsigned long long)nquery);
    return 0;
}
