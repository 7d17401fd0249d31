// rxg_replay.cpp — the per-packet replay of a classified burst into the caller's handlers
// (rxg_rx_replay: the reference's ether_in -> ip_in -> tcp_in order, re-classifying what a
// handler's table write changed), the payload hand-off (rxg_payload_gather_dev, rxg_rcv_set,
// rxg_payload_take) and the one-frame rxg_ether_in.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <immintrin.h>
#include <thread>

#include "rxg_ctx.h"

using namespace rxg;

extern "C" int rxg_ether_in(rxg_ctx *c, const rxg_handoff_ops *ops, void *mbuf, void *frame, uint16_t data_len)
{
    if (!c || !ops || !frame) return fail(-EINVAL, "rxg_ether_in: NULL argument");
    rxg_pkt_view v;
    v.buf_addr = frame;
    v.data_off = 0;
    v.data_len = data_len;
    v.pad = 0;
    rxg_rec16 rec;
    int rc = rxg_rx_burst(c, &v, 1, RXG_REC16, &rec);
    if (rc) return rc;
    void *m = mbuf, *f = frame;
    rc = rxg_rx_replay(c, ops, &m, &f, &rec, 1, RXG_REC16);
    return rc ? rc : 0;  // ether_in always returns 0 (etherin.c:36)
}

// ----------------------------------------------------------------- payload hand-off ---
extern "C" int rxg_payload_gather_dev(rxg_ctx *c, const rxg_payload_out *o, void *stream)
{
    if (!c || !o) return fail(-EINVAL, "rxg_payload_gather_dev: NULL argument");
    if (!c->last_frames || !c->last_recs)
        return fail(-EINVAL, "rxg_payload_gather_dev: no burst to gather from");
    const uint32_t n = c->last_n;
    if (n && (!o->msgs || !o->arena_used || (o->arena_cap && !o->arena)))
        return fail(-EINVAL, "rxg_payload_gather_dev: NULL output buffer");
    int rc = set_device(c);
    if (rc) return rc;
    hipStream_t st = pick(c, stream);
    const uint32_t nb = payload_blocks(n);
    const void *old_status = c->d_pg_status.p;
    if ((rc = ensure(c->d_pg_status, (size_t)nb * sizeof(unsigned long long)))) return rc;
    if (c->d_pg_status.p != old_status)  // fresh memory: no word may look published
        HIP_OK(hipMemsetAsync(c->d_pg_status.p, 0, c->d_pg_status.bytes, st));
    if (!c->d_pg_ticket.p) {
        if ((rc = ensure(c->d_pg_ticket, sizeof(unsigned long long)))) return rc;
        HIP_OK(hipMemsetAsync(c->d_pg_ticket.p, 0, sizeof(unsigned long long), st));
        c->pg_tickets = 0;
    }
    // one gather in flight per context: the ticket counter and the status words are shared,
    // so a gather on another stream waits for the previous one
    if (c->pm_ev) HIP_OK(hipStreamWaitEvent(st, c->pm_ev, 0));
    c->pg_epoch = (c->pg_epoch % ((1u << 30) - 1u)) + 1u;
    LaunchPayload P;
    P.frames = c->last_frames;
    if ((rc = burst_offsets(c, st, &P.off64))) return rc;
    P.len = c->last_len;
    P.recs = c->last_recs;
    P.stride = c->last_stride;
    P.n = n;
    P.msgs = o->msgs;
    P.arena = (uint8_t *)o->arena;
    P.arena_cap = o->arena ? o->arena_cap : 0;
    P.status = (unsigned long long *)c->d_pg_status.p;
    P.ticket = (unsigned long long *)c->d_pg_ticket.p;
    P.ticket_base = c->pg_tickets;
    P.used = (unsigned long long *)o->arena_used;
    P.epoch = c->pg_epoch;
    uint32_t tickets = 0;
    HIP_OK(launch_payload(P, st, &tickets));
    c->pg_tickets += tickets;
    // rxg_payload_take fetches the descriptors on its first call after this gather
    if (!c->pm_ev) HIP_OK(hipEventCreateWithFlags(&c->pm_ev, hipEventDisableTiming));
    HIP_OK(hipEventRecord(c->pm_ev, st));
    c->d_pm = o->msgs;
    c->pm_used = o->arena_used;
    c->pm_n = n;
    c->pm_pending = true;
    c->pm_poisoned = false;
    return 0;
}

extern "C" int rxg_rcv_set(rxg_ctx *c, int32_t idx, uint32_t cur_seq, uint32_t pairs_pending)
{
    if (!c) return fail(-EINVAL, "rxg_rcv_set: ctx NULL");
    if (idx < 0 || idx >= kMaxTcbs) return fail(-EINVAL, "rxg_rcv_set: index %d", idx);
    if ((size_t)idx >= c->rcv_state.size()) {
        c->rcv_state.resize((size_t)idx + 1, 0);
        c->rcv_cur.resize((size_t)idx + 1, 0);
    }
    c->rcv_cur[idx] = cur_seq;
    c->rcv_state[idx] = pairs_pending ? 2 : 1;
    return 0;
}

// PushData (tcp_windows.c:341-358) with an empty SeqPairs list and
// CurrentSequenceNumber == seq: the out-of-window test needs SeqPairs (:345) and is
// skipped; the duplicate test (:349) drops iff cur > seq + Length (u32); AdjustPair puts
// the one pair at the head (:42-110, returns seq + Length + FIN); GetData pops it with
// offset 0 and copies Length bytes (:158-180) -> one message of exactly this payload.
extern "C" int rxg_payload_take(rxg_ctx *c, int32_t idx, uint32_t seq, uint32_t length, rxg_payload_msg *msg)
{
    if (!c) return fail(-EINVAL, "rxg_payload_take: ctx NULL");
    const int64_t pos = c->replay_pos;
    if (pos < 0 || (uint64_t)pos >= c->pm_n || length == 0 || length > 0xFFFFu) return 0;
    if (c->pm_pending) {  // first take after the gather: fetch the burst's descriptors
        if (int rc = set_device(c)) return rc;
        HIP_OK(hipEventSynchronize(c->pm_ev));
        if (c->pm_n > c->h_pm_cap) {
            if (c->h_pm) HIP_OK(hipHostFree(c->h_pm));
            c->h_pm = nullptr;
            c->h_pm_cap = 0;
            HIP_OK(hipHostMalloc((void **)&c->h_pm, (size_t)c->pm_n * sizeof(rxg_payload_msg), hipHostMallocDefault));
            c->h_pm_cap = c->pm_n;
        }
        uint64_t used = 0;
        HIP_OK(hipMemcpyAsync(c->h_pm, c->d_pm, (size_t)c->pm_n * sizeof(rxg_payload_msg), hipMemcpyDeviceToHost,
                              c->stream));
        if (c->pm_used)  // (a fused burst, rxg_rx_burst_payload_dev, has no look-back to time out)
            HIP_OK(hipMemcpyAsync(&used, c->pm_used, sizeof used, hipMemcpyDeviceToHost, c->stream));
        HIP_OK(hipStreamSynchronize(c->stream));
        c->pm_pending = false;
        // a gather whose look-back timed out (arena_used = ~0) placed payloads at unknown
        // offsets: nothing of that burst is handed out (the stack's own PushData runs)
        c->pm_poisoned = used == ~0ull;
    }
    if (c->pm_poisoned) return 0;
    const rxg_payload_msg &m = c->h_pm[pos];
    if (!(m.flags & RXG_PM_GATHERED) || m.len != length) return 0;
    if (idx < 0 || (size_t)idx >= c->rcv_state.size() || c->rcv_state[idx] != 1 || c->rcv_cur[idx] != seq)
        return 0;
    if (seq > (uint32_t)(seq + length)) return 0;  // the duplicate test drops it
    if (seq == 0) return 0;  // GetData asserts CurrentSequenceNumber != 0 (:151): the stack's own code
    c->rcv_cur[idx] = seq + length;
    if (msg) *msg = m;
    return 1;
}

// ------------------------------------------------------------------------- replay ---
static inline bool rec_is_tcp(const rxg_rec16 &r)
{
    return r.verdict == RXG_V_DISPATCH || r.verdict == RXG_V_RST_NOPCB || r.verdict == RXG_V_RST_LISTEN_NONSYN;
}

// A TCP record that findtcb pass 1 did not answer (listener or no TCB): pass 2 decides it.
static inline bool rec_pass2(const rxg_rec16 &r) { return r.tcb_idx < 0 || (r.flags & RXG_F_LISTEN); }

// Counter contributions of one TCP record (the kernel's definition; only the fields a
// re-classification can change).
static void tcp_record_counters(const rxg_rec16 &r, int64_t sign, int64_t *d)
{
    if (r.flags & RXG_F_REF_NULLSLOT) d[RXG_C_REF_NULLSLOT] += sign;
    if (r.tcb_idx >= 0) d[(r.flags & RXG_F_LISTEN) ? RXG_C_TCB_HIT_LISTEN : RXG_C_TCB_HIT_EXACT] += sign;
    if (r.verdict == RXG_V_RST_NOPCB) d[RXG_C_NOPCB] += sign;
    if (r.verdict == RXG_V_RST_LISTEN_NONSYN) d[RXG_C_LISTEN_NONSYN] += sign;
    if (r.verdict == RXG_V_DISPATCH) d[RXG_C_DISPATCH] += sign;
}

// The pass-1 key of a frame of >= 54 bytes, as the kernel forms it: ports = dport << 16 |
// sport (host order), ipv4_dst as loaded, ipv4_src host order (tcp_tcb.c:134-135,152-155).
// The replay's written-tuple filter index (16 bits): every packet after a burst's first table
// write is checked against it, so two multiplies rather than the table's seven (tuple_hash;
// 14 -> 6 ns a packet on this container's core); a collision only costs the exact lookup.
static inline uint32_t filter_hash(const TupleKey &k)
{
    return (k.ports * 0x9E3779B1u + k.src * 0x85EBCA6Bu + k.dst) >> 16;
}

static inline TupleKey frame_key(const uint8_t *f)
{
    const uint32_t sport = ((uint32_t)f[34] << 8) | f[35], dport = ((uint32_t)f[36] << 8) | f[37];
    const uint32_t dst = (uint32_t)f[30] | ((uint32_t)f[31] << 8) | ((uint32_t)f[32] << 16) | ((uint32_t)f[33] << 24);
    const uint32_t src = ((uint32_t)f[26] << 24) | ((uint32_t)f[27] << 16) | ((uint32_t)f[28] << 8) | f[29];
    return TupleKey{(dport << 16) | sport, dst, src};
}

// Re-classify one TCP packet of >= 54 bytes against the table as it stands now, exactly as
// rx_kernel's classify does (findtcb tcp_tcb.c:127-173, tcp_in.c:47-59), answered from the
// host index the device mirror is patched from (rxg_mirror.h): the replay's fix-up of a
// packet whose TCB a handler changed inside the burst.  The fields a
// table change cannot move (checksums, datalen, flags of the frame) stay as the burst
// computed them.
static void host_classify(const rxg_ctx *c, const uint8_t *f, rxg_rec16 &r)
{
    const TupleKey k = frame_key(f);
    uint8_t st = RXG_STATE_NONE;
    bool lhit = false;
    const int32_t idx = c->mir.find(k.ports, k.dst, k.src, k.ports >> 16, &st, &lhit);
    const bool missed = idx < 0 || lhit;  // pass 1 found nothing
    const bool nslot = missed && c->mir.min_null < (lhit ? idx : c->mir.ntcb());
    const uint8_t tflags = f[47];
    r.tcb_idx = idx;
    r.state = idx >= 0 ? st : (uint8_t)RXG_STATE_NONE;
    r.verdict = idx < 0 ? RXG_V_RST_NOPCB
              : (st == RXG_LISTENING && !(tflags & RXG_TCP_FLAG_SYN)) ? RXG_V_RST_LISTEN_NONSYN
              : RXG_V_DISPATCH;
    r.flags = (uint8_t)((r.flags & ~(RXG_F_LISTEN | RXG_F_REF_NULLSLOT)) | (lhit ? RXG_F_LISTEN : 0) |
                        (nslot ? RXG_F_REF_NULLSLOT : 0));
}

// Re-classify frames sel[0..k) of the last burst against the current mirror (GPU).
static int reclassify(rxg_ctx *c, const std::vector<uint32_t> &sel, std::vector<rxg_rec16> &out)
{
    int rc;
    const uint32_t *off64 = nullptr;
    if ((rc = burst_offsets(c, c->stream, &off64))) return rc;
    if (!c->last_frames || !off64 || !c->last_len)
        return fail(-EINVAL, "rxg_rx_replay: no burst on this context to re-classify against");
    if ((rc = ensure(c->d_sel, sel.size() * 4))) return rc;
    if ((rc = ensure(c->d_fix, sel.size() * sizeof(rxg_rec16)))) return rc;
    if (c->dirty && (rc = tcb_push(c))) return rc;
    HIP_OK(hipMemcpyAsync(c->d_sel.p, sel.data(), sel.size() * 4, hipMemcpyHostToDevice, c->stream));
    const LaunchBurst one{off64, c->last_len, (uint32_t)sel.size(), (uint8_t *)c->d_fix.p, 0u};
    LaunchRx L;
    std::memset(&L, 0, sizeof L);
    L.frames = c->last_frames;
    L.bursts = &one;
    L.nbursts = 1;
    L.sel = (const uint32_t *)c->d_sel.p;
    L.mode = RXG_REC16;
    L.table = table_view(c);
    L.counters = nullptr;  // corrections go to the host row instead
    L.max_blocks = c->max_blocks ? c->max_blocks : (c->grid_rec16 ? c->grid_rec16 : 1024);
    HIP_OK(launch_rx(L, c->stream));
    out.resize(sel.size());
    HIP_OK(hipMemcpyAsync(out.data(), c->d_fix.p, sel.size() * sizeof(rxg_rec16), hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    return 0;
}

// A bulk change (a reload, a listener change, min_null moving) that leaves more than this
// many packets of the burst stale re-classifies them in one GPU launch; fewer (and every
// change to single tuples) are answered from the host index as each packet is reached.
static constexpr uint32_t kHostReclassifyMax = 256;

// The side effects of etherin.c:21-35, ip.c:26-39 and tcp_in.c:47-72, in packet order.
extern "C" int rxg_rx_replay(rxg_ctx *c, const rxg_handoff_ops *ops, void *const *mbufs,
                             void *const *frames, const void *recs, uint32_t n, uint32_t stride)
{
    if (!c || !ops || (n && (!mbufs || !frames || !recs)))
        return fail(-EINVAL, "rxg_rx_replay: NULL argument");
    if (!rec_kind_ok(stride)) return fail(-EINVAL, "rxg_rx_replay: stride %u", stride);
    if (n && c->last_n != n)
        return fail(-EINVAL, "rxg_rx_replay: n=%u but the burst to replay (%u of the last launch) had %u frames", n,
                    c->replay_cursor, c->last_n);
    if (n && !c->burst_ok) return fail(-EINVAL, "rxg_rx_replay: the last burst on this context failed");
    // the re-classify launches and the counter correction run on this context's device
    // (a group replays several contexts from one thread, rxg_group.cpp)
    if (int rc = set_device(c)) return rc;
    struct PosGuard {
        rxg_ctx *c;
        ~PosGuard() { c->replay_pos = -1; }
    } pos_guard{c};
    std::vector<rxg_rec16> &cur = c->rp_cur;
    cur.resize(n);
    if (stride == RXG_REC8)
        for (uint32_t i = 0; i < n; ++i) rxg_rec8_expand((const rxg_rec8 *)recs + i, &cur[i]);
    else
        for (uint32_t i = 0; i < n; ++i) cur[i] = *(const rxg_rec16 *)((const uint8_t *)recs + (size_t)i * stride);
    int64_t delta[RXG_NCOUNTERS] = {0};

    // Staleness by write sequence numbers, checked when a packet is reached (its header is
    // read there anyway; no per-burst index).  Each batch of tracked writes (those of one
    // handler call, or those made between the burst and the replay) gets a number; a record
    // computed at number s is stale when a later write touched what it depends on: its tuple
    // (pass 1, old or new tuple of a written slot), or -- for a packet pass 1 did not answer
    // -- a LISTENING slot on its dport or the lowest NULL slot (pass 2); any write for a
    // frame under 54 bytes; everything after a reload.
    std::vector<uint32_t> &pkt_seq = c->rp_seq;
    pkt_seq.assign(n, 0u);  // 0 = as the burst classified it
    uint32_t wseq = 0, any_seq = 0, all_seq = 0, minnull_seq = 0, bulk_seq = 0, scanned_seq = 0;
    std::unordered_map<TupleKey, uint32_t, TupleKeyHash> key_seq;
    std::vector<std::pair<int32_t, uint32_t>> listen_seq;  // (dport, seq): rare
    std::vector<uint64_t> &filt = c->rp_filter;            // 65 536-bit filter of written tuples
    bool filt_used = false;
    auto absorb_lists = [&](const std::vector<TupleKey> &keys, const std::vector<int32_t> &listen, bool all,
                            bool pass2) {
        ++wseq;
        any_seq = wseq;
        if (all) all_seq = bulk_seq = wseq;
        if (pass2) minnull_seq = bulk_seq = wseq;
        for (const TupleKey &k : keys) {
            key_seq[k] = wseq;
            const uint32_t h = filter_hash(k);
            if (!filt_used) {
                filt.assign(1024, 0ull);
                filt_used = true;
            }
            filt[(h >> 6) & 1023u] |= 1ull << (h & 63u);
        }
        for (int32_t d : listen) {
            bool found = false;
            for (auto &e : listen_seq)
                if (e.first == d) {
                    e.second = wseq;
                    found = true;
                }
            if (!found) listen_seq.emplace_back(d, wseq);
            bulk_seq = wseq;
        }
    };
    // the tracked writes since the last absorb; logged for the launch's later bursts, whose
    // records were computed before them too
    auto absorb = [&]() {
        c->launch_keys.insert(c->launch_keys.end(), c->touched_keys.begin(), c->touched_keys.end());
        c->launch_listen.insert(c->launch_listen.end(), c->touched_listen.begin(), c->touched_listen.end());
        c->launch_all |= c->touched_all;
        c->launch_pass2 |= c->touched_pass2;
        absorb_lists(c->touched_keys, c->touched_listen, c->touched_all, c->touched_pass2);
        c->touched_keys.clear();
        c->touched_listen.clear();
        c->touched_all = c->touched_pass2 = false;
    };
    auto stale = [&](uint32_t j) -> bool {
        const rxg_rec16 &q = cur[j];
        const uint32_t s = pkt_seq[j];
        if (any_seq <= s || !rec_is_tcp(q)) return false;
        if (all_seq > s || (q.flags & RXG_F_TRUNC)) return true;
        const TupleKey k = frame_key((const uint8_t *)frames[j]);
        if (filt_used) {
            const uint32_t h = filter_hash(k);
            if ((filt[(h >> 6) & 1023u] >> (h & 63u)) & 1ull) {
                auto it = key_seq.find(k);
                if (it != key_seq.end() && it->second > s) return true;
            }
        }
        const int32_t d = (int32_t)(k.ports >> 16);
        if (rec_pass2(q)) {
            if (minnull_seq > s) return true;
            for (const auto &e : listen_seq)
                if (e.first == d && e.second > s) return true;
        }
        return false;
    };
    // writes the replays of this launch's earlier bursts made, then those since
    if (c->replay_cursor > 0 &&
        (!c->launch_keys.empty() || !c->launch_listen.empty() || c->launch_all || c->launch_pass2))
        absorb_lists(c->launch_keys, c->launch_listen, c->launch_all, c->launch_pass2);
    if (!c->touched_keys.empty() || !c->touched_listen.empty() || c->touched_all || c->touched_pass2) absorb();

    std::vector<uint32_t> sel;
    std::vector<rxg_rec16> fix;
    for (uint32_t i = 0; i < n; ++i) {
        if (any_seq > pkt_seq[i] && stale(i)) {
            ++c->rp_stats[0];
            const bool trunc = (cur[i].flags & RXG_F_TRUNC) != 0;
            bool batched = false;
            if (c->replay_on_device || trunc || bulk_seq > scanned_seq) {
                // what is stale from here on: one GPU launch if the set is large (a bulk
                // change), or always on the device path / for a short frame
                sel.clear();
                for (uint32_t j = i; j < n; ++j)
                    if (stale(j)) sel.push_back(j);
                scanned_seq = wseq;
                if (c->replay_on_device || trunc || sel.size() > kHostReclassifyMax) {
                    int rc = reclassify(c, sel, fix);
                    if (rc) return rc;
                    for (size_t k = 0; k < sel.size(); ++k) {
                        tcp_record_counters(cur[sel[k]], -1, delta);
                        tcp_record_counters(fix[k], +1, delta);
                        cur[sel[k]] = fix[k];
                        pkt_seq[sel[k]] = wseq;
                    }
                    c->rp_stats[2] += sel.size();
                    ++c->rp_stats[3];
                    batched = true;
                }
            }
            if (!batched) {
                if (c->mir.need_rebuild) {  // a reload / growth inside the replay: index first
                    int rc = tcb_push(c);
                    if (rc) return rc;
                }
                rxg_rec16 r = cur[i];
                host_classify(c, (const uint8_t *)frames[i], r);
                tcp_record_counters(cur[i], -1, delta);
                tcp_record_counters(r, +1, delta);
                cur[i] = r;
                pkt_seq[i] = wseq;
                ++c->rp_stats[1];
            }
        }
        const rxg_rec16 &r = cur[i];
        c->replay_pos = i;  // rxg_payload_take answers for this packet
        void *m = mbufs[i];
        uint8_t *f = (uint8_t *)frames[i];
        void *ip = f + RXG_OFF_IP, *tcp = f + RXG_OFF_TCP;
        const uint64_t gen_before = c->gen;
        switch (r.verdict) {
        case RXG_V_ARP:
            if (ops->arp_in) ops->arp_in(ops->user, m);
            if (ops->free_mbuf) ops->free_mbuf(ops->user, m);
            break;
        case RXG_V_DROP_L2:
        case RXG_V_DROP_NONTCP:
            if (ops->free_mbuf) ops->free_mbuf(ops->user, m);
            break;
        default: {
            // ip.c:30-32 ARP learn on the host-order source address
            const uint32_t src = ((uint32_t)f[26] << 24) | ((uint32_t)f[27] << 16) | ((uint32_t)f[28] << 8) | f[29];
            if (c->arp_enabled) {
                // the mirror answers get_mac: unknown at the burst and not added since
                if ((r.flags & RXG_F_ARP_LEARN) && ops->add_mac && !c->arp_since_burst.count(src)) {
                    ops->add_mac(ops->user, src, f + 6);
                    rxg_arp_learned(c, src);  // idempotent if the caller's add_mac mirrors too
                }
            } else {
                unsigned char mac[6];
                if (ops->get_mac && ops->add_mac && ops->get_mac(ops->user, src, mac) == 0)
                    ops->add_mac(ops->user, src, f + 6);
            }
            if ((ops->flags & RXG_OPS_VERIFY_TCP_CKSUM) && !(r.flags & RXG_F_TCP_OK)) {
                // tcp_in.c:37-40 with the check compiled in: free, ++tcpchecksumerror
                if (ops->free_mbuf) ops->free_mbuf(ops->user, m);
                if (ops->tcpchecksumerror) ++*ops->tcpchecksumerror;
            } else if (r.verdict == RXG_V_RST_NOPCB || r.verdict == RXG_V_RST_LISTEN_NONSYN) {
                if (r.verdict == RXG_V_RST_NOPCB && ops->tcpnopcb) ++*ops->tcpnopcb;  // tcp_in.c:48
                if (ops->free_mbuf) ops->free_mbuf(ops->user, m);
                if (ops->send_reset) ops->send_reset(ops->user, ip, tcp);
            } else {  // RXG_V_DISPATCH
                const uint32_t seq = ((uint32_t)f[38] << 24) | ((uint32_t)f[39] << 16) | ((uint32_t)f[40] << 8) | f[41];
                const uint32_t ack = ((uint32_t)f[42] << 24) | ((uint32_t)f[43] << 16) | ((uint32_t)f[44] << 8) | f[45];
                if (ops->on_segment) ops->on_segment(ops->user, r.tcb_idx, seq, ack);
                if (ops->tcpswitch) ops->tcpswitch(ops->user, r.tcb_idx, r.state, tcp, ip, m);
            }
        }
        }
        if (c->gen != gen_before) absorb();  // the handlers changed the table
    }
    // the launch's next burst is replayed next (a single burst can be replayed again)
    if (c->replay_cursor + 1 < c->last_bursts.size()) select_burst(c, c->replay_cursor + 1);
    bool nz = false;
    for (int k = 0; k < RXG_NCOUNTERS; ++k) nz |= delta[k] != 0;
    if (nz) {  // the corrections, added with the next mirror patch launch (flush_delta)
        for (int k = 0; k < RXG_NCOUNTERS; ++k) c->pend_delta[k] += delta[k];
        c->pend = true;
    }
    return 0;
}

extern "C" int rxg_replay_stats(rxg_ctx *c, uint64_t out[4])
{
    if (!c || !out) return fail(-EINVAL, "rxg_replay_stats: NULL argument");
    for (int k = 0; k < 4; ++k) out[k] = c->rp_stats[k];
    return 0;
}
