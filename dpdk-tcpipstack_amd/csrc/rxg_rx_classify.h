// rxg_rx_classify.h — phase B of the receive body: findtcb's two passes against the device
// TCB mirror (tcp_tcb.c:127-173), the ARP-learn test (ip.c:30-32), the verdict of tcp_in
// (tcp_in.c:47-72), the record and the counters.
#pragma once
#include <hip/hip_runtime.h>

#include "rxg_rx_frames.h"

namespace rxg {

// Phase B: lane i classifies frame i of the slice (all 64 probes in flight together) and
// writes its record; the records of a slice are one contiguous 1 KiB / 3 KiB store.
// First bucket of the exact-tuple probe, loaded early so that several frames' probes of
// one lane are in flight together.
struct Probe {
    uint4 s[kSlotsPerBucket];
    uint4 arp;  // the first ARP-mirror bucket of the frame's source (DevTable::arp)
    uint32_t hb;
};

// The ARP-mirror bucket of the frame's source, issued with the TCB probe and unconditionally
// (mirror off: bucket mask 0, every lane reads one word): the compiler can then count it, and
// classify_finish's ARP test waits for one load instead of walking a dependent chain
// (ARP mirror on, C4 74.8 -> 113.5 us with the round-2 {ip, used} chain walk).
__device__ __forceinline__ uint4 arp_issue(const RxArgs &a, const Fields &F)
{
    const uint32_t ip = bswap32(F.src);
    const uint32_t b = a.t.arp_mask ? (arp_hash(ip) & a.t.arp_mask) : 0u;
    return a.t.arp[b];
}

__device__ __forceinline__ Probe probe_issue(const RxArgs &a, const Fields &F)
{
    Probe P;
    P.hb = tuple_hash(F.ports, F.dst, bswap32(F.src)) & a.t.bucket_mask;
    // always a valid bucket: load unconditionally (see load_chunks), use only for TCP
    const uint4 *b = a.t.buckets + (size_t)P.hb * kSlotsPerBucket;
#pragma unroll
    for (int k = 0; k < kSlotsPerBucket; ++k) P.s[k] = b[k];
    P.arp = arp_issue(a, F);
    return P;
}

// Per-lane last-flow cache: the findtcb result of the last TCP frame this lane classified
// (the table does not change during a launch or a served request).  A slice whose TCP
// frames all hit their lane's cache skips the probe, the findtcb loop and the ARP-mirror
// probe: a burst of one flow (C2, bulk-transfer trains) classifies without a dependent L2
// round trip.
struct FlowCache {
    uint32_t ports = 0, dst = 0, src = 0;  // tuple as pass 1 compares it
    int32_t idx = -1;
    uint32_t meta = 0;                     // st | lhit << 8 | nslot << 9 | arp_learn << 10 | valid << 31
};
constexpr uint32_t kFcValid = 0x80000000u;

__device__ __forceinline__ Probe probe_none()
{
    Probe P;
#pragma unroll
    for (int k = 0; k < kSlotsPerBucket; ++k) P.s[k] = make_uint4(0u, 0u, 0u, kEmpty);
    P.arp = make_uint4(0u, 0u, 0u, 0u);
    P.hb = 0;
    return P;
}

template <int MODE, bool VWALK>
__device__ __forceinline__ void classify_finish(const RxArgs &a, bool valid, uint32_t len, const Fields &F,
                                                const Probe &P, WaveCounters &wc, Rec &pr, FlowCache &fc,
                                                bool cached);

__device__ __forceinline__ bool fc_hit(const FlowCache &fc, const Fields &F)
{
    return (fc.meta & kFcValid) && fc.ports == F.ports && fc.dst == F.dst && fc.src == bswap32(F.src);
}

__device__ __forceinline__ void transpose_small_slice(const uint4 (&v)[4], int lane, uint32_t *sf,
                                                      uint32_t (&d)[4][4]);

__device__ __forceinline__ uint32_t probe_bucket(const RxArgs &a, const Fields &F)
{
    return tuple_hash(F.ports, F.dst, bswap32(F.src)) & a.t.bucket_mask;
}

// The first buckets of the wave's 64 probes loaded four lanes to a bucket (lane l: slot l&3
// of frame 16j + l/4's bucket, 16 whole 64-byte buckets per instruction) and transposed
// through 4 KiB of LDS, as the small-frame path loads frames.  Each lane loading its own
// bucket's four slots touched up to 64 lines per instruction: C4 75.3 -> 74.0 us
// (DESIGN.md §5).  Issue and transpose are separate so the small-frame path can issue the
// next slice's frames in between (the transpose waits for these loads only).
struct ProbeLoads {
    uint4 v0, v1, v2, v3;  // slot lane&3 of the buckets of frames lane/4 + 0, 16, 32, 48
    uint4 arp;             // this lane's frame's ARP bucket (issued last: the transpose waits
                           // for the four above only)
    uint32_t hb;           // this lane's frame's first bucket
};

__device__ __forceinline__ ProbeLoads probe_issue_coalesced(const RxArgs &a, const Fields &F, int lane)
{
    static_assert(kSlotsPerBucket == 4, "one bucket = four 16-byte slots = four lanes");
    ProbeLoads L;
    L.hb = probe_bucket(a, F);
    const uint4 *bk = a.t.buckets + (lane & 3);
    const uint32_t h0 = lane_read(L.hb, (lane >> 2)), h1 = lane_read(L.hb, 16 + (lane >> 2));
    const uint32_t h2 = lane_read(L.hb, 32 + (lane >> 2)), h3 = lane_read(L.hb, 48 + (lane >> 2));
    L.v0 = bk[(size_t)h0 * kSlotsPerBucket];
    L.v1 = bk[(size_t)h1 * kSlotsPerBucket];
    L.v2 = bk[(size_t)h2 * kSlotsPerBucket];
    L.v3 = bk[(size_t)h3 * kSlotsPerBucket];
    L.arp = arp_issue(a, F);
    return L;
}

// [bucket][slot ^ ((bucket >> 2) & 3)] as transpose_small_slice; lane i gets its own bucket
__device__ __forceinline__ Probe probe_transpose(const ProbeLoads &L, int lane, uint32_t *tsf)
{
    uint4 *t = reinterpret_cast<uint4 *>(tsf);
    const int ch = lane & 3;
    const int f0 = lane >> 2, f1 = 16 + (lane >> 2), f2 = 32 + (lane >> 2), f3 = 48 + (lane >> 2);
    t[f0 * 4 + (ch ^ ((f0 >> 2) & 3))] = L.v0;
    t[f1 * 4 + (ch ^ ((f1 >> 2) & 3))] = L.v1;
    t[f2 * 4 + (ch ^ ((f2 >> 2) & 3))] = L.v2;
    t[f3 * 4 + (ch ^ ((f3 >> 2) & 3))] = L.v3;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    Probe P;
    P.hb = L.hb;
    P.arp = L.arp;
    const int sw = (lane >> 2) & 3;
#pragma unroll
    for (int k = 0; k < 4; ++k) P.s[k] = t[lane * 4 + (k ^ sw)];
    __builtin_amdgcn_wave_barrier();  // reads done before the LDS is reused
    return P;
}

// Classify lane's frame and leave its record in pr.  tsf: 4 KiB of LDS for the probe's
// transpose.
template <int MODE, bool VWALK>
__device__ __forceinline__ void classify_store(const RxArgs &a, bool valid, uint32_t len, const Fields &F,
                                               WaveCounters &wc, Rec &pr, FlowCache &fc, uint32_t *tsf)
{
    const uint32_t et = F.et & 0xFFFFu, proto = (F.et >> 16) & 0xFFu;
    const bool is_tcp = valid && et == RXG_ETHER_TYPE_IPV4 && proto == RXG_IPPROTO_TCP;
    const bool cached = __ballot(is_tcp && !fc_hit(fc, F)) == 0ull;
    const int lane = (int)(threadIdx.x & 63);
    const Probe P = cached ? probe_none() : probe_transpose(probe_issue_coalesced(a, F, lane), lane, tsf);
    classify_finish<MODE, VWALK>(a, valid, len, F, P, wc, pr, fc, cached);
}

// Overflow walks (a tuple or an ARP address not in its first bucket, which was loaded with
// the probe).  Launched kernels walk through the scalar data cache: one 64-byte bucket into
// SGPRs (uniform address), whose wait is on lgkmcnt, not vmcnt, so the vector loads in
// flight (the next slice's frames) are not drained, as a vector load consumed right after
// issue would drain them (vmcnt retires in order).  Read only, and safe there: the table is
// not written during a launch, and every dispatch starts with an invalidated scalar cache.
// The latency-mode server (VWALK) stays resident across mirror writes, and its per-request
// acquire invalidates the vector caches only: it walks with vector loads (per lane).
__device__ __forceinline__ void sload_bucket(const uint4 *b, uint32_t (&x)[16])
{
    typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
    u32x16 r;
    asm volatile("s_load_dwordx16 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(b));
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = r[k];
}

__device__ __forceinline__ uint4 sload_arp_bucket(const uint4 *b)
{
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 r;
    asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(b));
    return make_uint4(r.x, r.y, r.z, r.w);
}

// Does ip sit in the ARP mirror?  k = its first bucket (loaded with the probe).
template <bool VWALK>
__device__ __forceinline__ bool arp_known(const RxArgs &a, uint32_t ip, const uint4 &k)
{
    bool hit = k.x == ip || k.y == ip || k.z == ip || k.w == ip;
    const bool more = ip != 0u && !hit && k.x && k.y && k.z && k.w;
    if constexpr (VWALK) {
        if (more) {  // per lane, vector loads
            uint32_t b = arp_hash(ip) & a.t.arp_mask;
            for (uint32_t probe = 1; probe <= a.t.arp_mask; ++probe) {
                b = (b + 1u) & a.t.arp_mask;
                const uint4 e = a.t.arp[b];
                hit = e.x == ip || e.y == ip || e.z == ip || e.w == ip;
                if (hit || !e.x || !e.y || !e.z || !e.w) break;
            }
        }
    } else {
        unsigned long long need = __ballot(more);
        while (need != 0ull) {  // wave-uniform: one lane at a time through scalar loads
            const int l = (int)__builtin_ctzll(need);
            need &= need - 1ull;
            const uint32_t ipl = __builtin_amdgcn_readlane(ip, l);
            uint32_t b = arp_hash(ipl) & a.t.arp_mask;
            bool h = false;
            for (uint32_t probe = 1; probe <= a.t.arp_mask; ++probe) {
                b = (b + 1u) & a.t.arp_mask;
                const uint4 e = sload_arp_bucket(a.t.arp + b);
                h = e.x == ipl || e.y == ipl || e.z == ipl || e.w == ipl;
                if (h || !e.x || !e.y || !e.z || !e.w) break;
            }
            if ((int)(threadIdx.x & 63u) == l) hit = h;
        }
    }
    return hit;
}

// Pass 1 of findtcb (tcp_tcb.c:145-159): the slot value of the lowest tcbs[] index holding
// the tuple, or kEmpty.  The first bucket (loaded with the probe) is compared straight-line
// by every lane; lanes whose tuple may sit in a later bucket (first bucket full, no match:
// ~0.4 % of the lanes at 64 K flows, a quarter of the slices) walk on.  Launched kernels walk
// one lane at a time by the whole wave through scalar loads (the round-2 per-lane vector loop
// drained the next slice's frames: C4 74.6 -> 73.6 us, 64 B frames at 64 K flows 28.7 -> 27.5,
// HISTORY.md §9.R3); the server walks per lane with vector loads (see sload_bucket).
template <bool VWALK>
__device__ __forceinline__ uint32_t tuple_lookup(const RxArgs &a, const Probe &P, uint32_t ports, uint32_t dst_raw,
                                                 uint32_t src_host)
{
    uint32_t v = kEmpty;
    bool empty = false;
#pragma unroll
    for (int k = 0; k < kSlotsPerBucket; ++k) {
        const bool m = P.s[k].x == ports && P.s[k].y == dst_raw && P.s[k].z == src_host;
        v = m ? P.s[k].w : v;  // a free slot holds kEmpty: a match there is no hit
        empty |= P.s[k].w == kEmpty;
    }
    const bool more = v == kEmpty && !empty;
    if constexpr (VWALK) {
        if (more) {
            uint32_t hb = P.hb;
            for (uint32_t probe = 1; probe <= a.t.bucket_mask; ++probe) {
                hb = (hb + 1u) & a.t.bucket_mask;
                const uint4 *b = a.t.buckets + (size_t)hb * kSlotsPerBucket;
                bool e2 = false;
#pragma unroll
                for (int k = 0; k < kSlotsPerBucket; ++k) {
                    const uint4 q = b[k];
                    if (q.x == ports && q.y == dst_raw && q.z == src_host && q.w != kEmpty) v = q.w;
                    e2 |= q.w == kEmpty;
                }
                if (v != kEmpty || e2) break;
            }
        }
    } else {
        unsigned long long need = __ballot(more);
        while (need != 0ull) {  // wave-uniform
            const int l = (int)__builtin_ctzll(need);
            need &= need - 1ull;
            const uint32_t kp = __builtin_amdgcn_readlane(ports, l), kd = __builtin_amdgcn_readlane(dst_raw, l);
            const uint32_t ks = __builtin_amdgcn_readlane(src_host, l);
            uint32_t hb = __builtin_amdgcn_readlane(P.hb, l), w = kEmpty;
            for (uint32_t probe = 1; probe <= a.t.bucket_mask; ++probe) {
                hb = (hb + 1u) & a.t.bucket_mask;
                uint32_t x[16];
                sload_bucket(a.t.buckets + (size_t)hb * kSlotsPerBucket, x);
                bool e2 = false;
#pragma unroll
                for (int k = 0; k < kSlotsPerBucket; ++k) {
                    if (x[4 * k] == kp && x[4 * k + 1] == kd && x[4 * k + 2] == ks && x[4 * k + 3] != kEmpty)
                        w = x[4 * k + 3];
                    e2 |= x[4 * k + 3] == kEmpty;
                }
                if (w != kEmpty || e2) break;
            }
            if ((int)(threadIdx.x & 63u) == l) v = w;
        }
    }
    return v;
}

template <int MODE, bool VWALK>
__device__ __forceinline__ void classify_finish(const RxArgs &a, bool valid, uint32_t len, const Fields &F,
                                                const Probe &P, WaveCounters &wc, Rec &pr, FlowCache &fc,
                                                bool cached)
{
    const uint32_t ck = valid ? F.ck : 0u, w_et = valid ? F.et : 0u, ports = valid ? F.ports : 0u;
    const uint32_t src_raw = valid ? F.src : 0u, dst_raw = valid ? F.dst : 0u, w_tl = valid ? F.tl : 0u;
    const uint32_t et = w_et & 0xFFFFu, proto = (w_et >> 16) & 0xFFu, tflags = w_et >> 24;
    const uint32_t tl = w_tl & 0xFFFFu, vihl = (w_tl >> 16) & 0xFFu, doff = w_tl >> 24;
    const uint32_t sport = ports & 0xFFFFu, dport = ports >> 16;
    const bool is_ip = valid && et == RXG_ETHER_TYPE_IPV4;
    const bool is_tcp = is_ip && proto == RXG_IPPROTO_TCP;
    const bool is_arp = valid && et == RXG_ETHER_TYPE_ARP;
    const bool trunc = valid && len < 54u;
    // ip.c:30-32: would get_mac(ntohl(src)) fail?  (ARP mirror enabled only)  The first
    // bucket came with the probe (P.arp); lanes whose address may sit in a later bucket
    // (first bucket full, no match) are walked one at a time by scalar loads, as the TCB
    // probe's overflow below.
    // ip.c:30-32: would get_mac(ntohl(src)) fail?  (ARP mirror enabled only)  The first
    // bucket came with the probe (P.arp); later buckets are walked as the TCB probe's are.
    bool arp_learn = false;
    if (is_tcp && (a.t.arp_flags & kArpOn) && !cached) {
        const uint32_t ip = bswap32(src_raw);
        const bool hit = arp_known<VWALK>(a, ip, P.arp);
        arp_learn = ip == 0u ? !(a.t.arp_flags & kArpZero) : !hit;
    }
    const uint32_t src_host = bswap32(src_raw);

    // ---- findtcb (tcp_tcb.c:127-173): pass 1 = exact-tuple bucket probe, pass 2 = listener
    int32_t idx = -1;
    bool lhit = false, nslot = false;
    uint32_t st = RXG_STATE_NONE;
    if (cached) {  // every TCP lane of the wave hits its cache (wave-uniform)
        if (is_tcp) {
            idx = fc.idx;
            st = fc.meta & 0xFFu;
            lhit = (fc.meta >> 8) & 1u;
            nslot = (fc.meta >> 9) & 1u;
            arp_learn = (fc.meta >> 10) & 1u;
        }
    } else if (is_tcp) {
        const uint32_t v = tuple_lookup<VWALK>(a, P, ports, dst_raw, src_host);
        if (v != kEmpty) {
            idx = (int32_t)(v & kIdxMask);
            st = v >> kStateShift;
        } else {  // pass 2: first LISTENING slot on dport (its state is LISTENING)
            const int32_t L = a.t.listen[dport];
            idx = L;
            lhit = L >= 0;
            nslot = a.t.min_null < (L >= 0 ? L : a.t.ntcb);
            if (lhit) st = RXG_LISTENING;
        }
        fc.ports = ports;
        fc.dst = dst_raw;
        fc.src = src_host;
        fc.idx = idx;
        fc.meta = st | ((uint32_t)lhit << 8) | ((uint32_t)nslot << 9) | ((uint32_t)arp_learn << 10) | kFcValid;
    }

    // ---- verdict (etherin.c:21-35, ip.c:28-39, tcp_in.c:47-72)
    uint32_t verdict;
    if (!is_ip)
        verdict = is_arp ? RXG_V_ARP : RXG_V_DROP_L2;
    else if (!is_tcp)
        verdict = RXG_V_DROP_NONTCP;
    else if (idx < 0)
        verdict = RXG_V_RST_NOPCB;
    else if (st == RXG_LISTENING && !(tflags & RXG_TCP_FLAG_SYN))
        verdict = RXG_V_RST_LISTEN_NONSYN;
    else
        verdict = RXG_V_DISPATCH;

    const uint32_t ipc = is_ip ? (ck & 0xFFFFu) : 0u;
    const uint32_t tcc = is_tcp ? (ck >> 16) : 0u;
    const uint32_t flags = ((is_ip && ipc == 0u) ? RXG_F_IP_OK : 0u) |
                           ((is_tcp && tcc == 0u) ? RXG_F_TCP_OK : 0u) |
                           (lhit ? RXG_F_LISTEN : 0u) | (nslot ? RXG_F_REF_NULLSLOT : 0u) |
                           (trunc ? RXG_F_TRUNC : 0u) | (arp_learn ? RXG_F_ARP_LEARN : 0u);
    const int32_t datalen = (int32_t)tl - (int32_t)(vihl & 0xFu) * 4 - (int32_t)(doff >> 4) * 4;

    if constexpr (MODE == 8) {  // rxg_rec8 (rxg.h)
        const uint32_t st3 = st == RXG_STATE_NONE ? 7u : st;
        pr.q0.x = ((uint32_t)(idx + 1) & 0xFFFFFFu) | (verdict << 24) | (st3 << 27);
        pr.q0.y = tflags | (flags << 8) | (((uint32_t)(datalen + 128) & 0x1FFFFu) << 14);
    } else {
        uint4 q0;
        q0.x = (uint32_t)idx;
        q0.y = ipc | (tcc << 16);
        q0.z = verdict | (st << 8) | (tflags << 16) | (flags << 24);
        q0.w = (uint32_t)datalen;
        pr.q0 = q0;
        if constexpr (MODE == 48) {
            const uint32_t seq_raw = F.seq, ack_raw = F.ack, h1 = F.h1, h2 = F.h2;
            uint4 q1, q2;
            q1.x = et | (sport << 16);
            q1.y = dport | (proto << 16) | (vihl << 24);
            q1.z = bswap32(seq_raw);
            q1.w = bswap32(ack_raw);
            q2.x = src_host;
            q2.y = dst_raw;
            q2.z = doff | ((h1 >> 16) << 8) | ((h2 & 0xFFu) << 24);
            q2.w = h2 >> 8;
            pr.q1 = q1;
            pr.q2 = q2;
        }
    }

    // ---- counters (definition: oracle orc_count_record).  Common case first: every valid
    // frame of the wave is a TCP segment with good checksums dispatched to an exact-match
    // TCB; then five counters move by the same count and the other ten not at all.
    const bool plain = is_tcp && verdict == RXG_V_DISPATCH && !lhit && !nslot && !trunc && ipc == 0u &&
                       tcc == 0u;
    if (__ballot(valid && !plain) == 0ull) {
        const uint32_t nv = (uint32_t)__popcll(__ballot(valid));
        wc.c[RXG_C_RX] += nv;
        wc.c[RXG_C_IPV4] += nv;
        wc.c[RXG_C_TCP] += nv;
        wc.c[RXG_C_TCB_HIT_EXACT] += nv;
        wc.c[RXG_C_DISPATCH] += nv;
        return;
    }
    wcount(wc, RXG_C_RX, valid);
    wcount(wc, RXG_C_TRUNC, trunc);
    wcount(wc, RXG_C_IPV4, is_ip);
    wcount(wc, RXG_C_ARP, is_arp);
    wcount(wc, RXG_C_OTHER_L2, valid && !is_ip && !is_arp);
    wcount(wc, RXG_C_IP_CKSUM_BAD, is_ip && ipc != 0u);
    wcount(wc, RXG_C_TCP, is_tcp);
    wcount(wc, RXG_C_NON_TCP, is_ip && !is_tcp);
    wcount(wc, RXG_C_TCP_CKSUM_BAD, is_tcp && tcc != 0u);
    wcount(wc, RXG_C_REF_NULLSLOT, is_tcp && nslot);
    wcount(wc, RXG_C_TCB_HIT_EXACT, is_tcp && idx >= 0 && !lhit);
    wcount(wc, RXG_C_TCB_HIT_LISTEN, is_tcp && lhit);
    wcount(wc, RXG_C_NOPCB, is_tcp && verdict == RXG_V_RST_NOPCB);
    wcount(wc, RXG_C_LISTEN_NONSYN, is_tcp && verdict == RXG_V_RST_LISTEN_NONSYN);
    wcount(wc, RXG_C_DISPATCH, is_tcp && verdict == RXG_V_DISPATCH);
}

}  // namespace rxg
