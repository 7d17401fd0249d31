// rxg_rx.h — the device code of the receive-path kernels (gfx950), instantiated by
// rxg_kernels.hip.
//
// One fused kernel body replaces, for a whole batch, the reference's per-packet
//   ether_in (etherin.c:12-37) -> ip_in (ip.c:19-42) -> tcp_in (tcp_in.c:32-84)
//   -> findtcb (tcp_tcb.c:127-173)
// plus the rx checksum the reference defines but compiles out (tcp_in.c:37, its
// primitive calculate_checksum is ip.c:44-59).
//
// Work decomposition:
//   * A wave owns a SLICE of 64 consecutive frames (one descriptor per lane: off64, len).
//   * Frames are grouped by size class inside the wave (ballot + ds_permute compaction);
//     each class is processed with LPF lanes per frame and NLOAD 16-byte loads per lane,
//     so 64-byte frames run one frame per lane and 1500-byte frames 16 lanes per frame.
//     No host binning, no second launch, any size mix.
//   * Checksums: one's-complement sums are byte-order independent (RFC 1071 §2(B)), so
//     lanes add little-endian 16-bit halves of the loaded dwords and the final fold is
//     byte-swapped once: bit-exact with the reference's big-endian byte loop.
//   * Classify: exact-tuple hash (4 slots per 64-byte bucket, value = lowest tcbs[] index
//     with that tuple) then the dport listener map: pass 1 / pass 2 of findtcb.
//   * Counters: wave-uniform ballot counts, one u64 atomic per counter per workgroup.
// The device code is split by phase (round 5), each header including the one before:
//   rxg_rx_core.h      launch arguments (RxArgs), lane helpers, burst cursor, payload helpers
//   rxg_rx_frames.h    phase A: loads, checksums and header fields per size class (run_class)
//   rxg_rx_classify.h  phase B: TCB / ARP probes, findtcb, verdict, record, counters
//   rxg_rx.h           the slice loop: all-small runs, record ring, rx_body, rx_kernel, rx_args
//   rxg_rx_server.h    the latency-mode server kernel (rx_server)
#pragma once
#include <hip/hip_runtime.h>

#include "rxg_rx_classify.h"

namespace rxg {

// An all-small slice (64 frames of <= 64 bytes): lane l loads chunk l&3 of frame 16j + l/4
// (instruction j covers 16 whole frames, 1 KiB, coalesced) ...
template <bool NT>
__device__ __forceinline__ void issue_small_slice(const RxArgs &a, uint32_t off, uint32_t len, int lane,
                                                  uint4 (&v)[4])
{
    const int ch = lane & 3;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int fr = 16 * j + (lane >> 2);
        const uint32_t foff = lane_read(off, fr), flen = lane_read(len, fr);
        const bool ok = (uint32_t)(ch * 16) < flen;  // frames <= 64 B: a whole 64-B slot
        // chunks past data_len read the arena's first bytes and are left as loaded
        // (fields_small masks every byte at or past data_len); no select on the result, so
        // nothing waits for the load here
        v[j] = load16<NT>(ok ? a.frames + (size_t)foff * 64u + ch * 16 : a.frames);
    }
}

// ... writes it to the wave's LDS at [frame][chunk ^ ((frame >> 2) & 3)], and after a wave
// barrier lane i reads back frame i's 64 bytes.  The XOR swizzle makes the 16 lanes of a
// ds_read_b128 group read 16 different 16-byte bank columns (unswizzled, lanes 4 frames
// apart collide: 4-way conflicts, ≈48 LDS cycles per slice measured).
__device__ __forceinline__ void transpose_small_slice(const uint4 (&v)[4], int lane, uint32_t *sf,
                                                      uint32_t (&d)[4][4])
{
    uint4 *t = reinterpret_cast<uint4 *>(sf);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int fr = 16 * j + (lane >> 2), ch = lane & 3;
        t[fr * 4 + (ch ^ ((fr >> 2) & 3))] = v[j];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int sw = (lane >> 2) & 3;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint4 q = t[lane * 4 + (c ^ sw)];
        d[c][0] = q.x; d[c][1] = q.y; d[c][2] = q.z; d[c][3] = q.w;
    }
    __builtin_amdgcn_wave_barrier();  // reads done before the LDS is reused
}

// How a launch finds its frames (rx_body's DESC): the bursts' off64[] lists; burst 0's
// off64[] through a selection list (re-classification, rxg_rx_replay); or fixed-stride slots
// with no list (rxg_rx_bursts_strided_dev: frame i of a burst at slot first + i * stride64,
// the burst's first slot carried in its off64 field).
enum { kDescList = 0, kDescSel = 1, kDescStride = 2 };

template <int DESC, typename BC>
__device__ __forceinline__ void load_desc(const RxArgs &a, uint32_t s, int lane, uint32_t &off, uint32_t &len, BC &bc)
{
    // Unconditional loads of a clamped index (every burst has n >= 1), not masked here:
    // masking would consume the load at once, and s_waitcnt retires in order, so the wait
    // would also drain every older load in flight (the prefetched frames of the small-slice
    // pipeline).  Callers treat lanes past their burst's n (slice_frames) as invalid.
    const uint32_t su = uniform(min(s, a.nslices - 1u));
    const uint32_t k = bc.of(a, su);
    const uint32_t f = (su - bc.slice0_of(a, k)) * 64u + (uint32_t)lane;
    const uint32_t fc = min(f, bc.n_of(a, k) - 1u);
    const uint32_t pf = DESC == kDescSel ? a.sel[fc] : fc;
    if constexpr (DESC == kDescStride)
        off = (uint32_t)(uintptr_t)bc.off64_of(a, k) + pf * a.stride64;
    else
        off = bc.off64_of(a, k)[pf];
    len = bc.len_of(a, k)[pf];
}

// Records of a wave's slices are staged in LDS and written out RS slices at a time (and
// at the end): record stores interleaved with the frame stream cost ≈10 % of the C3 kernel
// (measured: 271 µs with 1 KiB stored per slice as it completes, 244 µs staged and
// written at the end, 243 µs with no record stores at all), HBM read/write turnarounds.
// Record bytes of one slice (64 frames) in the ring, in uint4: REC8 512 B, REC16 1 KiB,
// REC48 3 KiB; MSG (the by-reference payload hand-off) adds the slice's 64 messages, 512 B
// (8 bytes each: the frame's slot and payload span, expanded to rxg_payload_msg on the way
// out, pay_msg_of).
constexpr int ring_slot_u4(int mode, bool msg = false) { return mode * 64 / 16 + (msg ? 32 : 0); }

template <bool NTS>
__device__ __forceinline__ void ring_store16(uint4 *p, const uint4 &q)
{
    if constexpr (NTS) {
        typedef unsigned int v4 __attribute__((ext_vector_type(4)));
        v4 v;
        v.x = q.x; v.y = q.y; v.z = q.z; v.w = q.w;
        __builtin_nontemporal_store(v, reinterpret_cast<v4 *>(p));
    } else {
        *p = q;
    }
}

template <int MODE, int RS, bool MSG = false>
struct RecRing {
    static constexpr int kQ = MODE / 16;  // uint4 per record (REC16 / REC48)
    static constexpr int kRec = ring_slot_u4(MODE);
    static constexpr int kSlot = ring_slot_u4(MODE, MSG);
    uint4 (*img)[kSlot];                  // [RS][kSlot]: the slice's records, contiguous (MSG: then its messages)
    uint32_t *base;                       // [RS]: the slot's launch slice
    uint32_t n = 0;                       // slots in use (wave-uniform)

    // LDS scratch of `bytes` in the free slots (the small-slice transpose, the parked
    // fields of the class path): the slots after the used ones, flushing first if fewer
    // are free.  The slice's own record later goes to the first of them (put), after the
    // scratch has been read.
    template <bool NTS = false, typename BC>
    __device__ __forceinline__ uint32_t *scratch(const RxArgs &a, int lane, int bytes, BC &bc)
    {
        const uint32_t need = (uint32_t)((bytes + kSlot * 16 - 1) / (kSlot * 16));
        if (n + need > (uint32_t)RS) flush<NTS>(a, lane, bc);
        return reinterpret_cast<uint32_t *>(img[n]);
    }

    // MSG: this lane's message (its frame's slot and payload span, pay_span) for the slot
    // put() fills next (call first: put advances)
    __device__ __forceinline__ void put_msg(int lane, uint32_t off, uint32_t span)
    {
        reinterpret_cast<uint2 *>(img[n] + kRec)[lane] = make_uint2(off, span);
    }

    __device__ __forceinline__ void put(uint32_t slice, int lane, const Rec &r)
    {
        if constexpr (MODE == 8) {
            reinterpret_cast<uint2 *>(img[n])[lane] = make_uint2(r.q0.x, r.q0.y);
        } else {
            uint4 *q = img[n] + lane * kQ;
            q[0] = r.q0;
            if constexpr (kQ == 3) {
                q[1] = r.q1;
                q[2] = r.q2;
            }
        }
        if (lane == 0) base[n] = slice;
        ++n;
    }

    // Writes out every staged slice: uint4 k*64 + lane of each slot, so a wave-instruction
    // stores 1 KiB contiguously (MSG: then the slice's messages, one burst per launch, 1 KiB
    // per instruction).  Records of frames >= n_frames are not written.  NTS:
    // non-temporal stores, used when the small-frame path flushes (C2 0.8-6 % faster across
    // boxes; the 1 500 B path keeps plain stores: 247.5 vs 250.5 us with non-temporal ones).
    template <bool NTS = false, typename BC>
    __device__ __forceinline__ void flush(const RxArgs &a, int lane, BC &bc)
    {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t sl = uniform(base[i]);
            const uint32_t kb = bc.of(a, sl);
            const uint32_t f0 = (sl - bc.slice0_of(a, kb)) * 64u;  // first frame of the slice in its burst
            const uint32_t nb = bc.n_of(a, kb);
            if constexpr (MSG) {  // the slice's messages (one burst per launch)
                if (f0 + (uint32_t)lane < nb) {
                    const uint2 m = reinterpret_cast<const uint2 *>(img[i] + kRec)[lane];
                    ring_store16<NTS>(reinterpret_cast<uint4 *>(a.pay_msgs) + f0 + lane, pay_msg_of(m.x, m.y));
                }
            }
            if constexpr (MODE == 8) {  // 64 lanes x 8 B: 512 B contiguous per instruction
                uint2 *d8 = reinterpret_cast<uint2 *>(bc.out_of(a, kb) + (size_t)f0 * 8u);
                if (f0 + (uint32_t)lane < nb) {
                    const uint2 q = reinterpret_cast<const uint2 *>(img[i])[lane];
                    if constexpr (NTS) {
                        typedef unsigned int v2 __attribute__((ext_vector_type(2)));
                        v2 v;
                        v.x = q.x; v.y = q.y;
                        __builtin_nontemporal_store(v, reinterpret_cast<v2 *>(d8 + lane));
                    } else {
                        d8[lane] = q;
                    }
                }
                continue;
            }
            uint4 *dst = reinterpret_cast<uint4 *>(bc.out_of(a, kb) + (size_t)f0 * MODE);
#pragma unroll
            for (int k = 0; k < kQ; ++k) {
                const int idx = k * 64 + lane;
                if (f0 + (uint32_t)(idx / kQ) < nb) {
                    if constexpr (NTS) {
                        typedef unsigned int v4 __attribute__((ext_vector_type(4)));
                        const uint4 q = img[i][idx];
                        v4 v;
                        v.x = q.x; v.y = q.y; v.z = q.z; v.w = q.w;
                        __builtin_nontemporal_store(v, reinterpret_cast<v4 *>(dst + idx));
                    } else {
                        dst[idx] = img[i][idx];
                    }
                }
            }
        }
        __builtin_amdgcn_wave_barrier();  // slots are rewritten after every lane's read
        n = 0;
    }
};

// One all-small slice s whose frames are in flight in vb[P]; prefetches slice s + nwaves
// into vb[1-P] when it is all-small too (and returns true: the caller continues the run).
template <int P, int MODE, int DESC, bool VWALK, int RS, int PAY, typename BC>
__device__ __forceinline__ bool small_step(const RxArgs &a, int lane, uint32_t &s, uint32_t nslices,
                                           uint32_t nwaves, uint32_t &c_off, uint32_t &c_len, uint32_t &n_off,
                                           uint32_t &n_len, uint4 (&vb)[2][4], RecRing<MODE, RS, PAY == kPayRef> &ring,
                                           WaveCounters &wc, Rec &rec, FlowCache &fc, unsigned long long &bytes,
                                           BC &bc)
{
    // Issue order (vmcnt retires in order): the TCB probe of this slice, then the next
    // slice's frames, then the descriptors two slices ahead; waiting for the probe leaves
    // both in flight.  (Probe after the frames: the probe's wait drained the prefetch,
    // 64 B / 64 K flows 28.4 us.)
    const uint32_t s1 = s + nwaves;
    // the server (VWALK) also runs a burst's last, partial slice here when its frames are all
    // small (rx_body); a launch's runs are whole slices
    const bool valid = !VWALK || (uint32_t)lane < slice_frames(a, uniform(s), bc);
    uint32_t d[4][4];
    uint32_t *sf = ring.template scratch<true>(a, lane, 4096, bc);
    transpose_small_slice(vb[P], lane, sf, d);
    // the next slice's descriptors are read after this slice's frames have landed: they were
    // issued before them (loop top) or just after (previous step), so this waits for no
    // more than the frames did
    const bool nxt = s1 < nslices && slice_frames(a, uniform(s1), bc) == 64u && __ballot(n_len <= 64u) == ~0ull;
    const Fields F = fields_small<MODE>(nullptr, c_len, d);
    const uint32_t m_off = c_off;  // (kPayRef: the message, staged with the record)
    uint32_t m_span = 0u;
    if constexpr (PAY) {  // (one burst per PAY launch: frame s * 64 + lane)
        m_span = pay_span(valid, c_len, F.et, F.tl);
        if constexpr (PAY == kPayCopy) {
            pay_line_small(a, c_off, m_span, d);
            pay_msg(a, s * 64u + (uint32_t)lane, valid, c_off, m_span);
        }
    }
    const uint32_t et = F.et & 0xFFFFu, proto = (F.et >> 16) & 0xFFu;
    const bool is_tcp = et == RXG_ETHER_TYPE_IPV4 && proto == RXG_IPPROTO_TCP;
    const bool cached = __ballot(is_tcp && !fc_hit(fc, F)) == 0ull;
    // Per-lane bucket loads here.  Four lanes to a bucket with the transpose through the
    // frames' LDS (as the class path does) measured 64 B at 64 K flows 28.8 -> 25.9 us, but
    // the one-flow C2 burst, which never probes, 19.2 -> 20.6 (more registers live across
    // the prefetch); the C2 configuration is the one the metric names.
    const Probe PO = cached ? probe_none() : probe_issue(a, F);
    // The next slice's frames are issued whether or not the run continues (a run's last step
    // reads the arena's first bytes instead): the compiler cannot count a load issued under a
    // branch, and the probe's wait below then drained the prefetch too (64 B frames at 64 K
    // flows 29.2 -> 28.3 us).
    issue_small_slice<true>(a, nxt ? n_off : 0u, nxt ? n_len : 0u, lane, vb[1 - P]);
    uint32_t y_off, y_len;
    load_desc<DESC>(a, s + 2u * nwaves, lane, y_off, y_len, bc);
    classify_finish<MODE, VWALK>(a, valid, c_len, F, PO, wc, rec, fc, cached);
    bytes += valid ? c_len : 0u;
    if (ring.n == RS) ring.template flush<true>(a, lane, bc);
    if constexpr (PAY == kPayRef) ring.put_msg(lane, m_off, m_span);
    ring.put(s, lane, rec);
    s = s1;
    c_off = n_off; c_len = n_len;
    n_off = y_off; n_len = y_len;
    return nxt;
}

// Two-deep form (DEEP launches): frames of two slices in flight with the same two register
// buffers.  A buffer is free once its slice has been transposed into LDS, so right after the
// transpose of slice s (vb[P]) the frames of slice s + 2 nwaves are issued into vb[P], while
// vb[1-P] still holds s + nwaves (issued one step earlier).  Descriptors run three slices
// ahead and are issued before the frames (vmcnt retires in order: the next step's check of
// them then waits for nothing younger).  pend: s + nwaves's frames are in vb[1-P]; returns
// whether the run continues with it.
template <int P, int MODE, int DESC, bool VWALK, int RS, int PAY, typename BC>
__device__ __forceinline__ bool small_step2(const RxArgs &a, int lane, uint32_t &s, uint32_t nslices,
                                            uint32_t nwaves, uint32_t &c_off, uint32_t &c_len, uint32_t &n_off,
                                            uint32_t &n_len, uint32_t &y_off, uint32_t &y_len, bool &pend,
                                            uint4 (&vb)[2][4], RecRing<MODE, RS, PAY == kPayRef> &ring, WaveCounters &wc, Rec &rec,
                                            FlowCache &fc, unsigned long long &bytes, BC &bc)
{
    const uint32_t s1 = s + nwaves, s2 = s + 2u * nwaves;
    uint32_t d[4][4];
    uint32_t *sf = ring.template scratch<true>(a, lane, 4096, bc);
    transpose_small_slice(vb[P], lane, sf, d);
    const Fields F = fields_small<MODE>(nullptr, c_len, d);
    const uint32_t m_off = c_off;  // (kPayRef: the message, staged with the record)
    uint32_t m_span = 0u;
    if constexpr (PAY) {
        m_span = pay_span(true, c_len, F.et, F.tl);
        if constexpr (PAY == kPayCopy) {
            pay_line_small(a, c_off, m_span, d);
            pay_msg(a, s * 64u + (uint32_t)lane, true, c_off, m_span);
        }
    }
    const uint32_t et = F.et & 0xFFFFu, proto = (F.et >> 16) & 0xFFu;
    const bool is_tcp = et == RXG_ETHER_TYPE_IPV4 && proto == RXG_IPPROTO_TCP;
    const bool cached = __ballot(is_tcp && !fc_hit(fc, F)) == 0ull;
    const Probe PO = cached ? probe_none() : probe_issue(a, F);
    uint32_t z_off, z_len;
    load_desc<DESC>(a, s + 3u * nwaves, lane, z_off, z_len, bc);
    const bool nxt2 = pend && s2 < nslices && slice_frames(a, uniform(s2), bc) == 64u && __ballot(y_len <= 64u) == ~0ull;
    issue_small_slice<true>(a, nxt2 ? y_off : 0u, nxt2 ? y_len : 0u, lane, vb[P]);  // unconditional, as in small_step
    classify_finish<MODE, VWALK>(a, true, c_len, F, PO, wc, rec, fc, cached);
    bytes += c_len;
    if (ring.n == RS) ring.template flush<true>(a, lane, bc);
    if constexpr (PAY == kPayRef) ring.put_msg(lane, m_off, m_span);
    ring.put(s, lane, rec);
    const bool cont = pend;
    pend = nxt2;
    s = s1;
    c_off = n_off; c_len = n_len;
    n_off = y_off; n_len = y_len;
    y_off = z_off; y_len = z_len;
    return cont;
}

// The body of workgroup blk of nblk (its waves are waves 4 blk .. 4 blk + 3 of 4 nblk dealing
// the launch's slices).  rx_kernel (one launch per batch) and rx_server (a persistent set of
// workgroups serving one burst after another) run it.
//   MODE   record kind 8 / 16 / 48, or 0: tx checksum generate (no records, no classify)
//   DESC   kDescList / kDescSel / kDescStride (load_desc)
//   MULTI  several bursts of one frame pool per launch (BurstCursor)
//   DEEP   runs of all-small slices prefetched two slices deep (small_step2); launch_rx picks
//          it for launches of at least kDeepSlicesPerWave slices per wave
//   PAY    the payload hand-off fused in (rxg_rx_burst_payload_dev: one burst, launched):
//          kPayCopy with the payload lines copied, kPayRef by reference (messages only)
//   SRV    the server's form: streaming-class rounds software-pipelined (a served burst's
//          frame reads are latency-bound: 32 x 1500 B bursts 25.6-27.6 -> 22.2-23.2 us) and
//          overflow walks with vector loads (VWALK, see sload_bucket)
template <int MODE, int DESC, bool MULTI, bool DEEP, bool SRV, int PAY = kPayNone>
__device__ __forceinline__ void rx_body(RxArgs a, uint32_t blk, uint32_t nblk)
{
    constexpr int NF = MODE == 48 ? NF48 : NF16;
    __shared__ unsigned long long s_cnt[4][RXG_NCOUNTERS];
    // Per-wave LDS = the record ring (REC16: 11 slices of 1 KiB, REC8: 22 of 512 B, REC48: 4 of
    // 3 KiB); its free slots are also the scratch of the slice in progress (4 KiB
    // small-slice transpose, NF x 256 B parked fields), so LDS per wave is the ring alone.
    // 3 workgroups per CU (LDS and, at ~145 VGPRs, registers).
    // (tx, MODE 0: 4 x 1 KiB, the class-0 transpose's scratch; no records)
    // kPayRef (the by-reference hand-off): each slot also holds the slice's messages (512 B),
    // REC8 12 slots of 1 KiB, REC16 8 of 1.5 KiB, REC48 3 of 3.5 KiB: up to 50 KB per
    // workgroup, still 3 per CU (13 slots, 54 KB, left room for 2), so a wave's records and
    // messages of a C3 launch (5-6 slices per wave) go out at its end, not between its frame
    // loads.
    constexpr bool MSG = PAY == kPayRef;
    constexpr int RS = MSG ? (MODE == 16 ? 8 : MODE == 48 ? 3 : 12)
                           : (MODE == 16 ? 11 : MODE == 48 ? 4 : MODE == 8 ? 22 : 4);
    constexpr int kSlot = ring_slot_u4(MODE == 0 ? 16 : MODE, MSG);
    static_assert(MODE == 0 || (RS * kSlot * 16 >= 4096 + kSlot * 16 && RS * kSlot * 16 >= NF * 256 + 4096),
                  "ring too small for the scratch");
    __shared__ __attribute__((aligned(16))) uint4 s_rec[4][RS][kSlot];
    __shared__ uint32_t s_recf[4][RS];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const uint32_t wave = blk * 4u + (uint32_t)wid;
    const uint32_t nwaves = nblk * 4u;
    if constexpr (!SRV) {
        if (a.nipatch != 0u) apply_launch_patches(a);  // (kernel argument: uniform)
    }

    WaveCounters wc;
#pragma unroll
    for (int k = 0; k < RXG_NCOUNTERS; ++k) wc.c[k] = 0u;
    unsigned long long bytes = 0ull;
    RecRing<MODE == 0 ? 16 : MODE, RS, MSG> ring;
    ring.img = s_rec[wid];
    ring.base = s_recf[wid];
    Rec rec;
    FlowCache fcache;

    // Descriptors: (c_off, c_len) for slice s, (n_off, n_len) for slice s + nwaves, whose
    // loads are always in flight while slice s is processed.
    uint32_t s = wave;
    uint32_t c_off = 0, c_len = 0, n_off = 0, n_len = 0;
    BurstCursor<MULTI> bc;
    bc.load(a, lane);
    const uint32_t nslices = a.nslices;
    // The streaming classes' rounds software-pipelined in tx (MODE 0, 101
    // VGPRs) and in the server; in launched rx, at the occupancy grid, the second buffer's
    // register cap cost more than the overlap gained.  Multi-burst kernels keep the plain
    // form: with the burst table held in lanes the pipelined rounds need 176 VGPRs.
    constexpr bool PIPE = !MULTI && (MODE == 0 || SRV);
    // The server's cooperative slices: a request of one or two slices on one workgroup (a small
    // burst) otherwise runs on one or two waves, the others idle.  The workgroup's four waves
    // share them: slice j (j < ck, the slices) is led by wave j, which classifies it, and the
    // waves w >= ck help the slice w mod ck, each of the 4 / ck waves of a slice taking its
    // streaming-class rounds part, part + 4 / ck, ... (part = w / ck), parking the fields in the
    // leader's scratch; the leader classifies after a workgroup barrier (HISTORY.md §9.R4).
    // Slices of at least 8 frames: below that a class has too few rounds to share, and the
    // barrier would only wait for the idle waves.  Barriers: one slice -- each wave passes one
    // when the slice is not all small (the leader on its class path), none otherwise; two
    // slices -- every wave passes exactly one (a leader after its class path or its all-small
    // run, a helper after its rounds, whatever its slice holds).
    // One slice per workgroup (srv_participants with kSrvLarge: 3..gridDim slices on as many
    // workgroups): workgroup blk's slice is blk, led by its wave 0 and shared as one slice is.
    uint32_t ck = 0u, j0 = 0u;
    if constexpr (SRV && MODE != 0) {
        if (nblk == 1u && (nslices == 1u || nslices == 2u) && slice_frames(a, 0u, bc) >= 8u &&
            (nslices == 1u || slice_frames(a, 1u, bc) >= 8u))
            ck = nslices;
        if (nblk >= 3u && nslices == nblk) {
            j0 = blk;
            if (wid == 0) s = blk;  // (below 8 frames it runs its slice alone)
            else if (slice_frames(a, blk, bc) < 8u) s = nslices;
            if (slice_frames(a, blk, bc) >= 8u) ck = 1u;
        }
        if (ck != 0u && (uint32_t)wid >= ck) {
            const uint32_t j = j0 + (uint32_t)wid % ck, part = (uint32_t)wid / ck, parts = 4u / ck;
            uint32_t offj, lenj;
            load_desc<DESC>(a, j, lane, offj, lenj, bc);
            const bool validj = (uint32_t)lane < slice_frames(a, j, bc);
            const uint32_t lj = validj ? lenj : 0u;
            const int clsj = validj ? size_class(lj) : 9;
            const bool big = __ballot(clsj == 0 || !validj) != ~0ull;
            if (big) {
                uint32_t *sfj = reinterpret_cast<uint32_t *>(s_rec[j - j0][0]);  // the leader's ring is empty
                // (class 0 is one round of 64 frames and its transpose uses the leader's LDS:
                // the leader's alone)
                run_class<1, 2, 4, false, MODE, false, PIPE>(a, clsj, offj, lj, lane, sfj, part, parts);
                run_class<2, 4, 4, false, MODE, false, PIPE>(a, clsj, offj, lj, lane, sfj, part, parts);
                run_class<3, 8, 4, false, MODE, true, PIPE>(a, clsj, offj, lj, lane, sfj, part, parts);
                run_class<10, 8, 5, false, MODE, true, PIPE>(a, clsj, offj, lj, lane, sfj, part, parts);
                run_class<8, 8, 6, false, MODE, true, PIPE>(a, clsj, offj, lj, lane, sfj, part, parts);
                run_class<4, 16, 4, false, MODE, true, PIPE>(a, clsj, offj, lj, lane, sfj, part, parts);
                run_class<5, 16, 6, false, MODE, true, PIPE>(a, clsj, offj, lj, lane, sfj, part, parts);
                run_class<6, 32, 4, false, MODE, true, PIPE>(a, clsj, offj, lj, lane, sfj, part, parts);
                run_class<7, 64, 2, true, MODE, true>(a, clsj, offj, lj, lane, sfj, part, parts);
            }
            if (big || ck == 2u) __syncthreads();  // the leaders' (see above)
            s = nslices;  // nothing more for this wave
        }
    }
    const bool coop = ck != 0u;
    load_desc<DESC>(a, s, lane, c_off, c_len, bc);
    load_desc<DESC>(a, s + nwaves, lane, n_off, n_len, bc);
    while (s < nslices) {
        const bool valid = (uint32_t)lane < slice_frames(a, uniform(s), bc);
        const uint32_t off = c_off, len = valid ? c_len : 0u;
        const int cls = valid ? size_class(len) : 9;
        if constexpr (MODE != 0) {
            // (the server: a partial slice whose valid frames are all small too -- a served
            // burst of fewer than 64 frames is one; its invalid lanes classify nothing)
            const bool all_small = __ballot(cls == 0 || (SRV && !valid)) == ~0ull;
            if (all_small) {
                // A run of all-small slices (every frame <= 64 bytes; lane i owns frame i end
                // to end), prefetched one slice deep: the next slice's frame loads are issued
                // before this slice's are waited for.  vmcnt retires in order, so the loads
                // are issued youngest-last (descriptors two slices ahead, then the next
                // slice's frames) and every wait leaves the next slice's frames in flight.
                // The two frame buffers alternate between the unrolled steps P = 0, 1 (a
                // register copy of a load in flight would wait for it).
                uint4 vb[2][4];
                issue_small_slice<true>(a, c_off, c_len, lane, vb[0]);
                if constexpr (DEEP) {
                    // two-deep: s + nwaves's frames too when that slice is all-small
                    const uint32_t s1 = s + nwaves;
                    bool pend = s1 < nslices && slice_frames(a, uniform(s1), bc) == 64u && __ballot(n_len <= 64u) == ~0ull;
                    uint32_t y_off, y_len;
                    load_desc<DESC>(a, s + 2u * nwaves, lane, y_off, y_len, bc);
                    if (pend) issue_small_slice<true>(a, n_off, n_len, lane, vb[1]);
                    for (;;) {
                        if (!small_step2<0, MODE, DESC, SRV, RS, PAY>(a, lane, s, nslices, nwaves, c_off, c_len, n_off,
                                                                      n_len, y_off, y_len, pend, vb, ring, wc, rec,
                                                                      fcache, bytes, bc))
                            break;
                        if (!small_step2<1, MODE, DESC, SRV, RS, PAY>(a, lane, s, nslices, nwaves, c_off, c_len, n_off,
                                                                      n_len, y_off, y_len, pend, vb, ring, wc, rec,
                                                                      fcache, bytes, bc))
                            break;
                    }
                    continue;
                }
                for (;;) {
                    if (!small_step<0, MODE, DESC, SRV, RS, PAY>(a, lane, s, nslices, nwaves, c_off, c_len, n_off, n_len,
                                                                 vb, ring, wc, rec, fcache, bytes, bc))
                        break;
                    if (!small_step<1, MODE, DESC, SRV, RS, PAY>(a, lane, s, nslices, nwaves, c_off, c_len, n_off, n_len,
                                                                 vb, ring, wc, rec, fcache, bytes, bc))
                        break;
                }
                if constexpr (SRV) {
                    if (ck == 2u) __syncthreads();  // two cooperative slices: every wave passes one
                }
                continue;
            }
        }
        bytes += len;
        // Descriptors two slices ahead, loaded as the class-path slice starts, so they have
        // landed by the loop's back edge.  Loaded at the slice's end instead, they were still
        // in flight there, where the register copies c <- n <- y made the wave wait for them
        // (an s_waitcnt vmcnt(0) per slice in the ISA).
        uint32_t y_off = 0u, y_len = 0u;
        load_desc<DESC>(a, s + 2u * nwaves, lane, y_off, y_len, bc);
        // parked fields, and the 4 KiB class-0 transpose after them
        uint32_t *sf = MODE == 0 ? reinterpret_cast<uint32_t *>(ring.img[0]) : ring.scratch(a, lane, NF * 256 + 4096, bc);
        // (coop: this wave leads its slice, taking rounds 0, 4 / ck, ... of each class)
        const uint32_t parts = coop ? 4u / ck : 1u;
        // classes 0-2 of mixed slices: plain loads; the larger ones non-temporal (measured
        // +5 % at 1500 B, -4 % at 64 B)
        run_class<0, 1, 4, false, MODE, false, false, PAY>(a, cls, off, len, lane, sf);
        run_class<1, 2, 4, false, MODE, false, PIPE, PAY>(a, cls, off, len, lane, sf, 0u, parts);
        run_class<2, 4, 4, false, MODE, false, PIPE, PAY>(a, cls, off, len, lane, sf, 0u, parts);
        run_class<3, 8, 4, false, MODE, true, PIPE, PAY>(a, cls, off, len, lane, sf, 0u, parts);
        run_class<10, 8, 5, false, MODE, true, PIPE, PAY>(a, cls, off, len, lane, sf, 0u, parts);
        run_class<8, 8, 6, false, MODE, true, PIPE, PAY>(a, cls, off, len, lane, sf, 0u, parts);
        run_class<4, 16, 4, false, MODE, true, PIPE, PAY>(a, cls, off, len, lane, sf, 0u, parts);
        run_class<5, 16, 6, false, MODE, true, PIPE, PAY>(a, cls, off, len, lane, sf, 0u, parts);
        run_class<6, 32, 4, false, MODE, true, PIPE, PAY>(a, cls, off, len, lane, sf, 0u, parts);
        run_class<7, 64, 2, true, MODE, true, false, PAY>(a, cls, off, len, lane, sf, 0u, parts);
        if constexpr (SRV && MODE != 0) {
            if (coop) __syncthreads();  // the other waves' parked fields
        }
        if constexpr (MODE == 0) {
            wcount(wc, RXG_C_RX, valid);
        } else {
            // the fields parked by other lanes of this wave must be visible to this lane
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const Fields F = unpark_fields<MODE>(sf, lane);
            uint32_t m_span = 0u;  // (kPayRef: the message, staged with the record)
            if constexpr (PAY == kPayCopy) pay_msg(a, s * 64u + (uint32_t)lane, valid, off, pay_span(valid, len, F.et, F.tl));
            if constexpr (PAY == kPayRef) m_span = pay_span(valid, len, F.et, F.tl);
            classify_store<MODE, SRV>(a, valid, len, F, wc, rec, fcache, sf + NF * 64);
            __builtin_amdgcn_wave_barrier();  // phase B reads before the next slice's writes
            if (ring.n == RS) ring.flush(a, lane, bc);
            if constexpr (PAY == kPayRef) ring.put_msg(lane, off, m_span);
            ring.put(s, lane, rec);
        }
        s += nwaves;
        c_off = n_off; c_len = n_len;
        n_off = y_off; n_len = y_len;
    }
    if constexpr (MODE != 0) ring.flush(a, lane, bc);

    if (a.counters == nullptr) return;
    if constexpr (SRV) {
        // The server: each wave adds its own counts (lanes 0-15, one atomic instruction), with
        // no workgroup reduction and no 64-bit cross-lane sum -- a served burst is one wave's
        // latency, and these were 0.75 us of it (HISTORY.md §9.R4).  A lane's bytes fit 32 bits
        // here (a request is at most 2^20 frames: <= 2^14 slices of one frame per lane).
        uint32_t b = (uint32_t)bytes;
        b += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b, 0x128, 0xF, 0xF, false);  // row_ror:8
        b += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b, 0x124, 0xF, 0xF, false);  // row_ror:4
        b += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
        b += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
        const unsigned long long tot = (unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)b, 0) +
                                       (uint32_t)__builtin_amdgcn_readlane((int)b, 16) +
                                       (uint32_t)__builtin_amdgcn_readlane((int)b, 32) +
                                       (uint32_t)__builtin_amdgcn_readlane((int)b, 48);
        uint32_t mine = 0u;
#pragma unroll
        for (int k = 0; k < RXG_NCOUNTERS; ++k) mine = lane == k ? wc.c[k] : mine;
        const unsigned long long v = (MODE != 0 && lane == RXG_C_BYTES) ? tot : (unsigned long long)mine;
        if (lane < RXG_NCOUNTERS && v) atomicAdd(&a.counters[(blk % kKernelCounterRows) * RXG_NCOUNTERS + lane], v);
        return;
    }
    // wave -> workgroup -> one atomic per counter
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) {
        const unsigned long long o = __shfl_xor(bytes, m, 64);
        bytes += o;
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < RXG_NCOUNTERS; ++k) s_cnt[wid][k] = wc.c[k];
        if (MODE != 0) s_cnt[wid][RXG_C_BYTES] = bytes;
    }
    __syncthreads();
    if (threadIdx.x < RXG_NCOUNTERS) {
        const int k = threadIdx.x;
        const unsigned long long v = s_cnt[0][k] + s_cnt[1][k] + s_cnt[2][k] + s_cnt[3][k];
        // replica row per workgroup (rxg.h RXG_COUNTER_ROWS): 32 adders per line, not 2048
        if (v) atomicAdd(&a.counters[(blk % kKernelCounterRows) * RXG_NCOUNTERS + k], v);
    }
}

// One launch per batch (rxg_rx_burst_dev / _bursts_dev / _strided_dev, the replay's
// re-classification, rxg_tx_cksum_dev): a grid-stride over the launch's slices.
template <int MODE, int DESC, bool MULTI, bool DEEP, int PAY = kPayNone>
__global__ __launch_bounds__(256, 1) void rx_kernel(RxArgs a)
{
    static_assert(!(PAY && (MULTI || MODE == 0 || DESC == kDescSel)), "PAY: one receive burst");
    rx_body<MODE, DESC, MULTI, DEEP, false, PAY>(a, blockIdx.x, gridDim.x);
}

// ------------------------------------------------------------------- launch helpers ---
// The kernel arguments and grid of a launch (host side, rxg_kernels.hip).
struct RxGrid {
    uint32_t blocks = 0;
    bool deep = false;  // two-deep all-small prefetch (kDeepSlicesPerWave)
};

inline hipError_t rx_args(const LaunchRx &L, RxArgs &a, RxGrid &g)
{
    __builtin_memset(&a, 0, sizeof a);
    a.frames = L.frames;
    a.sel = L.sel;
    a.t = L.table;
    a.counters = L.counters;
    a.stride64 = L.stride64;
    a.pay_arena = L.pay_arena;
    a.pay_msgs = L.pay_msgs;
    a.ipatch = L.ipatch;
    a.nipatch = L.nipatch;
    if (L.nbursts > kMaxBursts) return hipErrorInvalidValue;
    uint32_t nslices = 0;
    for (uint32_t k = 0; k < L.nbursts; ++k) {
        const LaunchBurst &B = L.bursts[k];
        if (B.n == 0) continue;
        RxBurst &r = a.b[a.nbursts++];
        // strided bursts carry their first slot in the off64 field (load_desc)
        r.off64 = L.stride64 ? reinterpret_cast<const uint32_t *>((uintptr_t)B.slot0) : B.off64;
        r.len = B.len;
        r.out = B.out;
        r.n = B.n;
        r.slice0 = nslices;
        nslices += (B.n + 63u) / 64u;
    }
    a.nslices = nslices;
    g.blocks = (nslices + 3u) / 4u;
    if (g.blocks > L.max_blocks) g.blocks = L.max_blocks;
    // long launches (C2 as 16 bursts: 85 slices per wave) prefetch all-small runs two slices
    // deep; short ones (one 2^20-frame burst: 5.3 per wave) measured slower with it (§5)
    g.deep = nslices >= kDeepSlicesPerWave * g.blocks * 4u && !L.pay_msgs;  // (PAY kernels: one depth)
    return hipSuccess;
}

}  // namespace rxg
