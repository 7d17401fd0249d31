// rxg_rx.h — the device code of the receive-path kernels (gfx950), shared by the product
// kernels (rxg_kernels.hip) and the ablation kernels of the experiment library
// (rxg_kernels_exp.hip, librxg_exp.so only).
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
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "rxg_common.h"
#include "rxg_kernels.h"
#include "rxg_mirror.h"

namespace rxg {

// --------------------------------------------------------------------------- helpers ---

__device__ __forceinline__ uint32_t hsum(uint32_t d) { return (d & 0xFFFFu) + (d >> 16); }

// Bytes [lo, hi) of the little-endian dword at frame offset o (o % 4 == 0).
__device__ __forceinline__ uint32_t region_mask(int o, int lo, int hi)
{
    int a = min(max(lo - o, 0), 4);
    int b = min(max(hi - o, 0), 4);
    uint32_t mb = b >= 4 ? 0xFFFFFFFFu : ((1u << (8 * b)) - 1u);
    uint32_t ma = a >= 4 ? 0xFFFFFFFFu : ((1u << (8 * a)) - 1u);
    return b > a ? (mb & ~ma) : 0u;
}

// Keep the low `keep` bytes (0..4) of a dword.
__device__ __forceinline__ uint32_t keep_low(uint32_t d, int keep)
{
    return keep >= 4 ? d : (keep <= 0 ? 0u : (d & ((1u << (8 * keep)) - 1u)));
}

__device__ __forceinline__ uint32_t lane_read(uint32_t v, int src_lane)
{
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ uint4 load16(const uint8_t *p)
{
    if constexpr (NT) {
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
        uint4 r;
        r.x = v.x; r.y = v.y; r.z = v.z; r.w = v.w;
        return r;
    } else {
        return *reinterpret_cast<const uint4 *>(p);
    }
}

// Dword K (bytes 4K..4K+3, K < 12) of the frame owned by the lane group starting at gbase.
// Chunk c = K/4 is held by lane gbase + c % LPF in its register j = c / LPF.
template <int K, int LPF, int NLOAD>
__device__ __forceinline__ uint32_t hdr_dword(const uint32_t (&d)[NLOAD][4], int gbase)
{
    constexpr int c = K / 4, w = K % 4, j = c / LPF, src = c % LPF;
    static_assert(j < NLOAD, "header chunk must be in the first load set");
    if constexpr (LPF == 1)
        return d[j][w];
    else
        return lane_read(d[j][w], gbase + src);
}

struct WaveCounters {
    uint32_t c[RXG_NCOUNTERS];
};

__device__ __forceinline__ void wcount(WaveCounters &wc, int k, bool pred)
{
    wc.c[k] += (uint32_t)__popcll(__ballot(pred));
}

// A burst of the launch: its slices are [slice0, slice0 + ceil(n / 64)) of the launch.
struct RxBurst {
    const uint32_t *off64;  // kDescStride: the slot of the burst's frame 0 (load_desc)
    const uint16_t *len;
    uint8_t *out;
    uint32_t n;
    uint32_t slice0;
};

struct RxArgs {
    const uint8_t *frames;  // the frame pool every burst's off64 is relative to
    const uint32_t *sel;    // optional: burst 0's logical frame i is frame sel[i] (re-classify)
    uint32_t nslices;       // of all bursts
    uint32_t nbursts;
    uint32_t stride64;      // kDescStride launches: 64-byte slots per frame
    DevTable t;
    unsigned long long *counters;
    RxBurst b[kMaxBursts];
    // PAY kernels (rxg_rx_burst_payload_dev, one burst): the payload hand-off fused into the
    // pass over the frames -- payload lines to pay_arena (the frame pool's geometry; nullptr:
    // by reference, nothing copied), one rxg_payload_msg per frame to pay_msgs.  (Last: the
    // other fields keep their offsets.)
    uint8_t *pay_arena;
    rxg_payload_msg *pay_msgs;
};

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// A device pointer rebuilt from an integer (read from LDS) as a pointer into the global
// address space: the address-space inference then emits global_load / global_store.  Through a
// plain generic pointer the compiler emits flat loads and stores, which also count in lgkmcnt,
// so every LDS wait after one waits for the HBM access too.  Used for the server's request
// (32 x 64 B served 9.1-9.3 us against 9.9 with flat accesses, profiles/r04/ab/r04m).  Not in
// BurstCursor::rl_ptr: the multi-burst kernels measured slower with it (c2m 227.9 against
// 217.0 us, same process), their waits being placed differently around the global accesses.
template <typename T>
__device__ __forceinline__ T *as_global(uint64_t v)
{
    typedef __attribute__((address_space(1))) T gT;
    return (T *)(gT *)v;
}

// The burst table of a multi-burst launch held in the wave's lanes: lane j keeps burst j's
// slice0, n and pointers in VGPRs (loaded once per wave), so finding the burst of a slice is
// one compare + ballot popcount and its fields are v_readlane -- no memory access and no
// scalar-load wait per lookup.  Single-burst launches (MULTI false) read burst 0 directly.
// A wave takes the launch's slices s = wave, wave + nwaves, ...  (Cutting the last, partial
// generation's slices into pieces spread over more waves measured slower)

// launches with at least this many slices per wave take the two-deep all-small pipeline
constexpr uint32_t kDeepSlicesPerWave = 16;

template <bool MULTI>
struct BurstCursor {
    uint32_t slice0 = 0, n = 0;
    const uint32_t *off64 = nullptr;
    const uint16_t *len = nullptr;
    uint8_t *out = nullptr;

    __device__ __forceinline__ void load(const RxArgs &a, int lane)
    {
        if constexpr (MULTI) {
            const uint32_t j = min((uint32_t)lane, a.nbursts - 1u);
            slice0 = lane < (int)a.nbursts ? a.b[j].slice0 : 0xFFFFFFFFu;
            n = a.b[j].n;
            off64 = a.b[j].off64;
            len = a.b[j].len;
            out = a.b[j].out;
        }
    }
    __device__ __forceinline__ uint32_t of(const RxArgs &a, uint32_t s) const
    {
        (void)a;
        if constexpr (!MULTI) return 0u;
        else return (uint32_t)__popcll(__ballot(s >= slice0)) - 1u;  // slice0 ascending, burst 0 at 0
    }
    template <typename T>
    static __device__ __forceinline__ T *rl_ptr(T *p, uint32_t k)
    {
        const uint64_t v = (uint64_t)p;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)k);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)k);
        return (T *)(((uint64_t)hi << 32) | lo);
    }
    __device__ __forceinline__ uint32_t slice0_of(const RxArgs &a, uint32_t k) const
    {
        if constexpr (!MULTI) return a.b[0].slice0;
        else return (uint32_t)__builtin_amdgcn_readlane((int)slice0, (int)k);
    }
    __device__ __forceinline__ uint32_t n_of(const RxArgs &a, uint32_t k) const
    {
        if constexpr (!MULTI) return a.b[0].n;
        else return (uint32_t)__builtin_amdgcn_readlane((int)n, (int)k);
    }
    __device__ __forceinline__ const uint32_t *off64_of(const RxArgs &a, uint32_t k) const
    {
        if constexpr (!MULTI) return a.b[0].off64;
        else return rl_ptr(off64, k);
    }
    __device__ __forceinline__ const uint16_t *len_of(const RxArgs &a, uint32_t k) const
    {
        if constexpr (!MULTI) return a.b[0].len;
        else return rl_ptr(len, k);
    }
    __device__ __forceinline__ uint8_t *out_of(const RxArgs &a, uint32_t k) const
    {
        if constexpr (!MULTI) return a.b[0].out;
        else return rl_ptr(out, k);
    }
};

// Frames in launch slice s (64 except a burst's last slice).
template <typename BC>
__device__ __forceinline__ uint32_t slice_frames(const RxArgs &a, uint32_t s, BC &bc)
{
    const uint32_t k = bc.of(a, s);
    return min(64u, bc.n_of(a, k) - (s - bc.slice0_of(a, k)) * 64u);
}

// One frame's record as classify computes it (16 or 48 bytes, rxg.h rxg_rec16/rxg_rec48).
struct Rec {
    uint4 q0, q1, q2;
};

// ------------------------------------------------- fused payload hand-off (PAY) ---
// The payload a frame hands to the socket ring (the candidates of
// rxg_payload_gather_dev, oracle/payload.py): a TCP segment (ether_type IPv4, proto 6: the
// verdicts DISPATCH / RST_NOPCB / RST_LISTEN_NONSYN) of at least 54 bytes, datalen =
// total_length - IHL*4 - data_off*4 > 0 (tcp_states.c:103-111), whose Length = datalen bytes
// at frame + 34 + data_off*4 (GetData takes the IP header as 20 bytes, tcp_windows.c:164-166)
// lie inside the frame.  et / tlw packed as Fields::et / Fields::tl.  Returns start << 16 |
// datalen (a candidate's datalen fits 16 bits: it lies inside the frame), or 0.
__device__ __forceinline__ uint32_t pay_span(bool valid, uint32_t len, uint32_t et, uint32_t tlw)
{
    const uint32_t tl = tlw & 0xFFFFu, vihl = (tlw >> 16) & 0xFFu, doff = tlw >> 24;
    const int32_t datalen = (int32_t)tl - (int32_t)(vihl & 0xFu) * 4 - (int32_t)(doff >> 4) * 4;
    const uint32_t start = RXG_OFF_TCP + (doff >> 4) * 4u;
    const bool cand = valid && (et & 0xFFFFu) == RXG_ETHER_TYPE_IPV4 && ((et >> 16) & 0xFFu) == RXG_IPPROTO_TCP &&
                      len >= 54u && datalen > 0 && start + (uint32_t)datalen <= len;
    return cand ? (start << 16) | (uint32_t)datalen : 0u;
}

__device__ __forceinline__ void nt_store16(uint8_t *p, const uint32_t (&q)[4])
{
    u32x4 v;
    v.x = q[0]; v.y = q[1]; v.z = q[2]; v.w = q[3];
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
}

// Payload stores (PAY): the payload's whole 64-byte lines (no partial-line writes), the
// streaming classes' non-temporal (16 lanes write 256 contiguous bytes per instruction), a
// frame of <= 64 B's one line by its own lane with plain stores, which the L2 merges into
// whole lines (non-temporal there: C2 fused 42.7 -> 69.5 us, C4 176.5 -> 186.3).
template <bool SMALL>
__device__ __forceinline__ void pay_store16(uint8_t *p, const uint32_t (&q)[4])
{
    if constexpr (SMALL) {
        *reinterpret_cast<uint4 *>(p) = make_uint4(q[0], q[1], q[2], q[3]);
    } else {
        u32x4 v;
        v.x = q[0]; v.y = q[1]; v.z = q[2]; v.w = q[3];
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
    }
}

// Does the hand-off write chunk c (bytes [16c, 16c + 16)) of a frame whose payload is span?
// Exactly the chunks of the 64-byte lines the payload touches.
__device__ __forceinline__ bool pay_writes_chunk(uint32_t c, uint32_t span)
{
    const uint32_t start = span >> 16, end = start + (span & 0xFFFFu);
    return (c >> 2) >= (start >> 6) && (c >> 2) <= ((end - 1u) >> 6);
}

// The 64-byte lines of a frame that hold its payload: [lo, hi].
__device__ __forceinline__ void pay_lines_of(uint32_t span, uint32_t &lo, uint32_t &hi)
{
    const uint32_t start = span >> 16, end = start + (span & 0xFFFFu);
    lo = start >> 6;
    hi = (end - 1u) >> 6;
}

// The frame's message (rxg_payload_msg): the payload at arena + 64*off + start, in place of
// the frame's own bytes (the arena has the pool's geometry), or zeros.  f: its index in the
// burst.  One 16-byte non-temporal store per lane (staged in LDS with the records instead, the
// fused C3 launch measured the same and C4 1.5 % faster, but the by-reference form 4 % slower
// on the shorter ring it needs).
__device__ __forceinline__ void pay_msg(const RxArgs &a, uint32_t f, bool valid, uint32_t off, uint32_t span)
{
    if (!valid) return;
    const uint32_t dl = span & 0xFFFFu;
    const uint64_t ao = span ? (uint64_t)off * 64u + (span >> 16) : 0ull;
    const uint32_t q[4] = {(uint32_t)ao, (uint32_t)(ao >> 32), dl,
                           span ? (RXG_PM_GATHERED | (dl >= 1000u ? RXG_PM_REF_OVERSIZE : 0u)) : 0u};
    nt_store16(reinterpret_cast<uint8_t *>(a.pay_msgs + f), q);
}

// A frame of <= 64 bytes owned by one lane (the all-small path after its transpose): its one
// line, as loaded, when it carries a payload.
__device__ __forceinline__ void pay_line_small(const RxArgs &a, uint32_t off, uint32_t span, const uint32_t (&q)[4][4])
{
    if (span == 0u || a.pay_arena == nullptr) return;  // (no arena: hand-off by reference)
    uint8_t *dst = a.pay_arena + (size_t)off * 64u;
#pragma unroll
    for (int k = 0; k < 4; ++k) pay_store16<true>(dst + 16 * k, q[k]);
}

// ------------------------------------------------------------- one round of frames ---
//
// Phase A (streaming): the lanes of a group load one frame, sum it and extract its header.
// MODE 16 / 48: the group leader parks the frame's fields in the wave's LDS row of the
// frame's ORIGINAL lane (its descriptor lane) for phase B.  MODE 0: transmit checksum
// generate, written straight into the frame.
//
// LDS field rows (per wave, [field][64 lanes]):
enum { F_CK = 0, F_ET, F_PORTS, F_SRC, F_DST, F_TL, F_SEQ, F_ACK, F_H1, F_H2, NF16 = 6, NF48 = 10 };

// What phase B needs of one frame (packed exactly as the LDS rows hold it).
struct Fields {
    uint32_t ck;      // ip_ck | tcp_ck << 16
    uint32_t et;      // ether_type | next_proto_id << 16 | tcp_flags << 24
    uint32_t ports;   // dport << 16 | sport (host order)
    uint32_t src;     // ip src_addr as loaded (network order)
    uint32_t dst;     // ip dst_addr as loaded (network order)
    uint32_t tl;      // total_length | version_ihl << 16 | data_off << 24
    uint32_t seq, ack, h1, h2;  // REC48 only: raw seq/ack, frame dwords 1-2 (src MAC)
};

template <int MODE>
__device__ __forceinline__ void park_fields(uint32_t *sf, uint32_t orig, const Fields &F)
{
    sf[F_CK * 64 + orig] = F.ck;
    sf[F_ET * 64 + orig] = F.et;
    sf[F_PORTS * 64 + orig] = F.ports;
    sf[F_SRC * 64 + orig] = F.src;
    sf[F_DST * 64 + orig] = F.dst;
    sf[F_TL * 64 + orig] = F.tl;
    if constexpr (MODE == 48) {
        sf[F_SEQ * 64 + orig] = F.seq;
        sf[F_ACK * 64 + orig] = F.ack;
        sf[F_H1 * 64 + orig] = F.h1;
        sf[F_H2 * 64 + orig] = F.h2;
    }
}

template <int MODE>
__device__ __forceinline__ Fields unpark_fields(const uint32_t *sf, int lane)
{
    Fields F;
    F.ck = sf[F_CK * 64 + lane];
    F.et = sf[F_ET * 64 + lane];
    F.ports = sf[F_PORTS * 64 + lane];
    F.src = sf[F_SRC * 64 + lane];
    F.dst = sf[F_DST * 64 + lane];
    F.tl = sf[F_TL * 64 + lane];
    F.seq = F.ack = F.h1 = F.h2 = 0;
    if constexpr (MODE == 48) {
        F.seq = sf[F_SEQ * 64 + lane];
        F.ack = sf[F_ACK * 64 + lane];
        F.h1 = sf[F_H1 * 64 + lane];
        F.h2 = sf[F_H2 * 64 + lane];
    }
    return F;
}

// Loads are issued unconditionally (a chunk outside the frame reads the frame's first
// chunk, or the arena's first bytes for an empty frame, and is then zeroed): with
// predicated loads hipcc zero-initialises their destination registers and inserts
// s_waitcnt between consecutive loads, serialising them.
template <int LPF, int NLOAD, bool NT>
__device__ __forceinline__ void load_chunks(const RxArgs &a, uint32_t off, uint32_t len, bool active,
                                            int lane, uint32_t (&d)[NLOAD][4])
{
    const int gl = lane & (LPF - 1);
    const uint8_t *fp = (active && len) ? a.frames + (size_t)off * 64u : a.frames;
#pragma unroll
    for (int j = 0; j < NLOAD; ++j) {
        const int c = gl + j * LPF;
        const bool ok = active && (uint32_t)(c * 16) < len;
        const uint4 v = load16<NT>(ok ? fp + c * 16 : fp);
        d[j][0] = ok ? v.x : 0u; d[j][1] = ok ? v.y : 0u; d[j][2] = ok ? v.z : 0u; d[j][3] = ok ? v.w : 0u;
    }
}

template <int LPF, int NLOAD, bool JUMBO, int MODE, bool NT, bool PAY = false>
__device__ __forceinline__ Fields frame_fields(const RxArgs &a, uint32_t off, uint32_t len, bool active,
                                               int lane, uint32_t (&d)[NLOAD][4]);

template <int LPF, int NLOAD, bool JUMBO, int MODE, bool NT, bool PAY = false>
__device__ __forceinline__ Fields frame_round(const RxArgs &a, uint32_t off, uint32_t len, bool active,
                                              int lane)
{
    uint32_t d[NLOAD][4];
    load_chunks<LPF, NLOAD, NT>(a, off, len, active, lane, d);
    return frame_fields<LPF, NLOAD, JUMBO, MODE, NT, PAY>(a, off, len, active, lane, d);
}

// Sums, header fields and (TX) checksum stores of the frames whose chunks are in d; PAY (the
// jumbo class, frames over 2 KiB): the payload lines copied by the group, loaded again (the
// chunks in d are only the first LPF * NLOAD).
template <int LPF, int NLOAD, bool JUMBO, int MODE, bool NT, bool PAY>
__device__ __forceinline__ Fields frame_fields(const RxArgs &a, uint32_t off, uint32_t len, bool active,
                                               int lane, uint32_t (&d)[NLOAD][4])
{
    constexpr bool TX = MODE == 0;
    const int gl = lane & (LPF - 1);
    const int gbase = lane - gl;
    const bool leader = active && gl == 0;
    uint8_t *fp = const_cast<uint8_t *>(a.frames) + (size_t)off * 64u;

    // ---- header: dwords 1..11 (bytes 4..47) of the group's frame, gathered to every lane.
    uint32_t h1 = 0, h2 = 0;
    if constexpr (MODE == 48) {
        h1 = hdr_dword<1, LPF, NLOAD>(d, gbase);
        h2 = hdr_dword<2, LPF, NLOAD>(d, gbase);
    }
    uint32_t h3 = hdr_dword<3, LPF, NLOAD>(d, gbase);
    uint32_t h4 = hdr_dword<4, LPF, NLOAD>(d, gbase);
    uint32_t h5 = hdr_dword<5, LPF, NLOAD>(d, gbase);
    uint32_t h6 = hdr_dword<6, LPF, NLOAD>(d, gbase);
    uint32_t h7 = hdr_dword<7, LPF, NLOAD>(d, gbase);
    uint32_t h8 = hdr_dword<8, LPF, NLOAD>(d, gbase);
    uint32_t h9 = hdr_dword<9, LPF, NLOAD>(d, gbase);
    uint32_t h10 = hdr_dword<10, LPF, NLOAD>(d, gbase);
    uint32_t h11 = hdr_dword<11, LPF, NLOAD>(d, gbase);

    if (len < 54u) {  // bytes at/after data_len read as zero (reference: stale mbuf bytes)
        const int L = (int)len;
        h1 = keep_low(h1, L - 4);   h2 = keep_low(h2, L - 8);   h3 = keep_low(h3, L - 12);
        h4 = keep_low(h4, L - 16);  h5 = keep_low(h5, L - 20);  h6 = keep_low(h6, L - 24);
        h7 = keep_low(h7, L - 28);  h8 = keep_low(h8, L - 32);  h9 = keep_low(h9, L - 36);
        h10 = keep_low(h10, L - 40); h11 = keep_low(h11, L - 44);
    }
    const uint32_t tl = bswap16(h4 & 0xFFFFu);  // ip total_length

    // TCP span = pseudo(src,dst from bytes 26..33) || segment [34, E), E = 14 + total_length,
    // clamped to data_len; bytes [26, 48) come from the gathered header, [48, end) from
    // the lanes' chunks c >= 3.
    const int E = max(34, 14 + (int)tl);
    const int tcp_end = min((int)len, E);

    uint32_t tsum = 0;
#pragma unroll
    for (int j = 0; j < NLOAD; ++j) {
        const int c = gl + j * LPF;
        const int o = c * 16;
        if (c >= 3) {
            if constexpr (TX) {  // the cksum field (bytes 50-51) is zero while summing
                if (c == 3) d[j][0] &= 0x0000FFFFu;
            }
            if (o + 16 <= tcp_end) {
                tsum += hsum(d[j][0]) + hsum(d[j][1]) + hsum(d[j][2]) + hsum(d[j][3]);
            } else {
                tsum += hsum(keep_low(d[j][0], tcp_end - o)) + hsum(keep_low(d[j][1], tcp_end - o - 4)) +
                        hsum(keep_low(d[j][2], tcp_end - o - 8)) + hsum(keep_low(d[j][3], tcp_end - o - 12));
            }
        }
    }
    if constexpr (JUMBO) {
        // frames beyond LPF*NLOAD chunks: keep streaming LPF chunks per step
        for (int base = LPF * NLOAD; base * 16 < (int)len; base += LPF) {
            const int c = base + gl;
            const int o = c * 16;
            if (active && o < tcp_end) {
                uint4 v = load16<NT>(fp + o);
                if (o + 16 <= tcp_end)
                    tsum += hsum(v.x) + hsum(v.y) + hsum(v.z) + hsum(v.w);
                else
                    tsum += hsum(keep_low(v.x, tcp_end - o)) + hsum(keep_low(v.y, tcp_end - o - 4)) +
                            hsum(keep_low(v.z, tcp_end - o - 8)) + hsum(keep_low(v.w, tcp_end - o - 12));
            }
        }
    }
#pragma unroll
    for (int m = LPF / 2; m > 0; m >>= 1)
        tsum += (uint32_t)__shfl_xor((int)tsum, m, 64);

    // Header parts of both sums (bytes beyond data_len are already zero in h*).
    const uint32_t h6_ip = TX ? (h6 & 0xFFFF0000u) : h6;  // TX: hdr_checksum (bytes 24-25) = 0
    const uint32_t isum = hsum(h3 & 0xFFFF0000u) + hsum(h4) + hsum(h5) + hsum(h6_ip) + hsum(h7) +
                          hsum(h8 & 0xFFFFu);
    // region [26, E) with E >= 34: dwords at o >= 28 keep their low E - o bytes
    uint32_t thdr = hsum(h6 & 0xFFFF0000u) + hsum(h7);
    if (E >= 48)  // total_length >= 34: the whole TCP header is inside the span (common)
        thdr += hsum(h8) + hsum(h9) + hsum(h10) + hsum(h11);
    else
        thdr += hsum(keep_low(h8, E - 32)) + hsum(keep_low(h9, E - 36)) + hsum(keep_low(h10, E - 40)) +
                hsum(keep_low(h11, E - 44));
    // pseudo {.., 0x00, 0x06, htons(total_length - 20)} as little-endian words
    const uint32_t tall = tsum + thdr + 0x0600u + bswap16((tl - 20u) & 0xFFFFu);
    const uint32_t ip_ck = (~bswap16(fold16(isum))) & 0xFFFFu;
    const uint32_t tcp_ck = (~bswap16(fold16(tall))) & 0xFFFFu;

    Fields F;
    F.ck = ip_ck | (tcp_ck << 16);
    F.et = bswap16(h3 & 0xFFFFu) | ((h5 >> 24) << 16) | ((h11 >> 24) << 24);
    F.ports = (bswap16(h9 & 0xFFFFu) << 16) | bswap16(h8 >> 16);
    F.src = (h6 >> 16) | (h7 << 16);
    F.dst = (h7 >> 16) | (h8 << 16);
    F.tl = tl | (((h3 >> 16) & 0xFFu) << 16) | (((h11 >> 16) & 0xFFu) << 24);
    F.seq = (h9 >> 16) | (h10 << 16);
    F.ack = (h10 >> 16) | (h11 << 16);
    F.h1 = h1;
    F.h2 = h2;
    if constexpr (PAY) {  // every lane holds the header here (hdr_dword)
        const uint32_t span = pay_span(active, len, F.et, F.tl);
        if (span != 0u && a.pay_arena != nullptr) {
            uint32_t lo, hi;
            pay_lines_of(span, lo, hi);
            uint8_t *dst = a.pay_arena + (size_t)off * 64u;
            for (uint32_t c = 4u * lo + (uint32_t)gl; c < 4u * (hi + 1u); c += (uint32_t)LPF) {
                const uint4 v = load16<NT>(fp + 16u * c);
                const uint32_t q[4] = {v.x, v.y, v.z, v.w};
                pay_store16<false>(dst + 16u * c, q);
            }
        }
    }
    if constexpr (TX) {
        // ip_out stores both as htons(calculate_checksum(...)) (ip.c:107,118); bytes at or
        // beyond data_len are never written
        if (leader) {
            if (len > 25u) *reinterpret_cast<uint16_t *>(fp + 24) = (uint16_t)bswap16(ip_ck);
            else if (len > 24u) fp[24] = (uint8_t)(ip_ck >> 8);
            if (len > 51u) *reinterpret_cast<uint16_t *>(fp + 50) = (uint16_t)bswap16(tcp_ck);
            else if (len > 50u) fp[50] = (uint8_t)(tcp_ck >> 8);
        }
    }
    return F;
}

// ---------------------------------------------------------- size-class dispatch ---
//
// Class of a frame by data_len: 0 <=64 | 1 <=128 | 2 <=256 | 3 <=512 | 8 <=768 | 4 <=1024 |
// 5 <=1536 | 6 <=2048 | 7 more.  (<=768 runs 8 frames per round: IMIX's 576 B frames.)
// Size classes (class id, then its lanes per frame x loads per lane in rx_kernel):
// 513-576 is its own class (the IMIX 576-byte frame: 8 x 5 loads, 90 % of the chunks
// used, instead of 8 x 6 at 75 %: C4 82.3 -> 80.6 us).
__device__ __forceinline__ int size_class(uint32_t len)
{
    return len <= 64u ? 0 : len <= 128u ? 1 : len <= 256u ? 2 : len <= 512u ? 3
         : len <= 576u ? 10 : len <= 768u ? 8 : len <= 1024u ? 4 : len <= 1536u ? 5 : len <= 2048u ? 6 : 7;
}

// Smallest data_len of a class.
constexpr int class_min_len(int c)
{
    return c == 0 ? 0 : c == 1 ? 65 : c == 2 ? 129 : c == 3 ? 257 : c == 10 ? 513 : c == 8 ? 577 : c == 4 ? 769
         : c == 5 ? 1025 : c == 6 ? 1537 : 2049;
}

// ----------------------------------------------------- streaming classes (LPF >= 2) ---
//
// The round of the streaming classes is VALU-issue bound, not HBM bound (≈600 VALU per
// 4 x 1500 B frames in the generic frame_fields, ≈ the whole HBM time at 2.4 GHz), so
// this path is written for instruction count:
//  * sums: v_dot2_u32_u16 (acc + lo16 + hi16) is one instruction per dword;
//  * the fast path masks by data_len only (every lane knows it); the frame's
//    total_length is needed only when 14 + total_length < data_len, which a wave-uniform
//    test sends to a slow path that re-sums by the TCP span;
//  * chunks are masked only where the frame ends: a lane holds at most one partial chunk;
//  * the leader gathers chunk 1 and 2 (header bytes 16-47) from lanes +1/+2 with DPP
//    row shifts and the group sum is reduced to it the same way (no LDS traffic);
//  * loads need no clamp where every frame of the class is long enough (class minimum
//    length, rounded up to its 64-byte line, which is readable); the others clamp to the
//    frame's last chunk.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// acc + lo16(x) + hi16(x) (w = 0x00010001) or acc (w = 0)
__device__ __forceinline__ uint32_t dsum(uint32_t x, uint32_t w, uint32_t acc)
{
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, x), __builtin_bit_cast(u16x2, w), acc, false);
}
constexpr uint32_t kOnes = 0x00010001u;

// lane l <- lane l + K of the same row of 16 lanes (0 past the row's end)
template <int K>
__device__ __forceinline__ uint32_t dpp_down(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x100 + K, 0xF, 0xF, false);
}

// Sum of a group of LPF lanes (aligned at a multiple of LPF), valid in the group's first lane.
template <int LPF>
__device__ __forceinline__ uint32_t group_sum(uint32_t t, int lane)
{
    if constexpr (LPF >= 2) t += dpp_down<1>(t);
    if constexpr (LPF >= 4) t += dpp_down<2>(t);
    if constexpr (LPF >= 8) t += dpp_down<4>(t);
    if constexpr (LPF >= 16) t += dpp_down<8>(t);
    if constexpr (LPF >= 64) t += lane_read(t, (lane + 32) & 63);  // rows 0+2, 1+3
    if constexpr (LPF >= 32) t += lane_read(t, (lane + 16) & 63);
    return t;
}

// Adds the chunk's bytes [0, n), n < 16, to the four per-dword accumulators (bytes at or
// past n read as zero).  Four accumulators: consecutive v_dot2 on one accumulator need a
// wait state between them.
__device__ __forceinline__ void partial_sum(const uint32_t (&q)[4], int n, uint32_t (&t)[4])
{
    t[0] = dsum(keep_low(q[0], n), kOnes, t[0]);
    t[1] = dsum(keep_low(q[1], n - 4), kOnes, t[1]);
    t[2] = dsum(keep_low(q[2], n - 8), kOnes, t[2]);
    t[3] = dsum(keep_low(q[3], n - 12), kOnes, t[3]);
}

__device__ __forceinline__ void full_sum(const uint32_t (&q)[4], uint32_t w, uint32_t (&t)[4])
{
    t[0] = dsum(q[0], w, t[0]);
    t[1] = dsum(q[1], w, t[1]);
    t[2] = dsum(q[2], w, t[2]);
    t[3] = dsum(q[3], w, t[3]);
}

// A frame of <= 64 bytes owned by one lane: q = its four chunks as loaded (bytes at or past
// data_len may hold anything: every use below masks them).  Same results as
// frame_fields<1, 4, ...>, fewer instructions.
template <int MODE>
__device__ __forceinline__ Fields fields_small(uint8_t *fp, uint32_t len, uint32_t (&q)[4][4])
{
    constexpr bool TX = MODE == 0;
    uint32_t h1 = q[0][1], h2 = q[0][2], h3 = q[0][3], h4 = q[1][0], h5 = q[1][1], h6 = q[1][2];
    uint32_t h7 = q[1][3], h8 = q[2][0], h9 = q[2][1], h10 = q[2][2], h11 = q[2][3];
    if (__ballot(len < 54u) != 0ull) {  // bytes at/after data_len read as zero (rare)
        const int L = (int)len;
        h1 = keep_low(h1, L - 4);   h2 = keep_low(h2, L - 8);   h3 = keep_low(h3, L - 12);
        h4 = keep_low(h4, L - 16);  h5 = keep_low(h5, L - 20);  h6 = keep_low(h6, L - 24);
        h7 = keep_low(h7, L - 28);  h8 = keep_low(h8, L - 32);  h9 = keep_low(h9, L - 36);
        h10 = keep_low(h10, L - 40); h11 = keep_low(h11, L - 44);
        q[2][0] = h8; q[2][1] = h9; q[2][2] = h10; q[2][3] = h11;
    }
    if constexpr (TX) q[3][0] &= 0x0000FFFFu;  // the cksum field (bytes 50-51) is zero while summing
    const uint32_t tl = bswap16(h4 & 0xFFFFu);
    const int te = min((int)len, max(34, 14 + (int)tl));  // end of the TCP span
    const int n2 = te - 32, n3 = te - 48;
    uint32_t ts[4] = {0u, 0u, 0u, 0u};
    full_sum(q[2], n2 >= 16 ? kOnes : 0u, ts);
    full_sum(q[3], n3 >= 16 ? kOnes : 0u, ts);
    if (n2 > 0 && n2 < 16) partial_sum(q[2], n2, ts);
    if (n3 > 0 && n3 < 16) partial_sum(q[3], n3, ts);
    uint32_t tall = dsum(h6 & 0xFFFF0000u, kOnes, ts[0] + ts[1] + ts[2] + ts[3]);
    tall = dsum(h7, kOnes, tall);
    tall += 0x0600u + bswap16((tl - 20u) & 0xFFFFu);
    const uint32_t h6_ip = TX ? (h6 & 0xFFFF0000u) : h6;
    uint32_t isum = dsum(h3 & 0xFFFF0000u, kOnes, 0u);
    isum = dsum(h4, kOnes, isum);
    isum = dsum(h5, kOnes, isum);
    isum = dsum(h6_ip, kOnes, isum);
    isum = dsum(h7, kOnes, isum);
    isum = dsum(h8 & 0xFFFFu, kOnes, isum);
    const uint32_t ip_ck = (~bswap16(fold16(isum))) & 0xFFFFu;
    const uint32_t tcp_ck = (~bswap16(fold16(tall))) & 0xFFFFu;

    Fields F;
    F.ck = ip_ck | (tcp_ck << 16);
    F.et = bswap16(h3 & 0xFFFFu) | ((h5 >> 24) << 16) | ((h11 >> 24) << 24);
    F.ports = (bswap16(h9 & 0xFFFFu) << 16) | bswap16(h8 >> 16);
    F.src = (h6 >> 16) | (h7 << 16);
    F.dst = (h7 >> 16) | (h8 << 16);
    F.tl = tl | (((h3 >> 16) & 0xFFu) << 16) | (((h11 >> 16) & 0xFFu) << 24);
    F.seq = (h9 >> 16) | (h10 << 16);
    F.ack = (h10 >> 16) | (h11 << 16);
    F.h1 = h1;
    F.h2 = h2;
    if constexpr (TX) {
        // ip_out stores both as htons(calculate_checksum(...)) (ip.c:107,118); bytes at or
        // beyond data_len are never written.  Two 2-byte stores: rewriting a 64-byte frame's
        // whole line instead measured slower, C4 tx 101.4 against 94.5 us, 64 B frames 40.9
        // against 33.6 (the write bytes count); so did queueing the line writes to the
        // wave's end.
        if (len > 25u) *reinterpret_cast<uint16_t *>(fp + 24) = (uint16_t)bswap16(ip_ck);
        else if (len > 24u) fp[24] = (uint8_t)(ip_ck >> 8);
        if (len > 51u) *reinterpret_cast<uint16_t *>(fp + 50) = (uint16_t)bswap16(tcp_ck);
        else if (len > 50u) fp[50] = (uint8_t)(tcp_ck >> 8);
    }
    return F;
}

// The loads of one round of a streaming class: lane l of a group of LPF loads chunks
// l, l + LPF, ... of its frame.  Inactive lanes: off = len = 0 (the arena's first SAFE bytes
// exist: it holds a frame of this class).
template <int C, int LPF, int NLOAD, bool NT, bool PAY = false>
__device__ __forceinline__ void round_load(const RxArgs &a, uint32_t off, uint32_t len, int lane,
                                           uint32_t (&d)[NLOAD][4])
{
    constexpr int SAFE = (class_min_len(C) + 63) & ~63;  // bytes every frame of the class has
    const int gl = lane & (LPF - 1);
    const uint8_t *fp = a.frames + (size_t)off * 64u;
    // PAY: chunks up to the end of the frame's last 64-byte line are loaded as they are (that
    // line is readable, rxg_dev_batch): the payload's lines are written whole
    const uint32_t lastc = len ? (PAY ? ((len + 63u) & ~63u) - 16u : ((len - 1u) & ~15u)) : 0u;
#pragma unroll
    for (int j = 0; j < NLOAD; ++j) {
        const uint32_t o = (uint32_t)(gl + j * LPF) * 16u;
        uint4 v;
        if ((j + 1) * LPF * 16 <= SAFE)  // unrolled: constant
            v = load16<NT>(fp + o);
        else
            v = load16<NT>(fp + min(o, lastc));
        d[j][0] = v.x; d[j][1] = v.y; d[j][2] = v.z; d[j][3] = v.w;
    }
}

template <int C, int LPF, int NLOAD, int MODE, bool NT, bool PAY = false>
__device__ __forceinline__ Fields frame_round_compute(const RxArgs &a, uint32_t off, uint32_t len, bool active,
                                                      int lane, uint32_t (&d)[NLOAD][4]);

template <int C, int LPF, int NLOAD, int MODE, bool NT, bool PAY = false>
__device__ __forceinline__ Fields frame_round_fast(const RxArgs &a, uint32_t off, uint32_t len, bool active,
                                                   int lane)
{
    uint32_t d[NLOAD][4];
    round_load<C, LPF, NLOAD, NT, PAY>(a, off, len, lane, d);
    return frame_round_compute<C, LPF, NLOAD, MODE, NT, PAY>(a, off, len, active, lane, d);
}

// Sums, header fields and (tx) checksum stores of one round whose chunks are in d; PAY: the
// payload lines written to the arena from the same registers.
template <int C, int LPF, int NLOAD, int MODE, bool NT, bool PAY>
__device__ __forceinline__ Fields frame_round_compute(const RxArgs &a, uint32_t off, uint32_t len, bool active,
                                                      int lane, uint32_t (&d)[NLOAD][4])
{
    static_assert(LPF >= 2 && LPF <= 64, "streaming classes only");
    constexpr bool TX = MODE == 0;
    const int gl = lane & (LPF - 1);
    const int gbase = lane - gl;
    const bool leader = active && gl == 0;
    uint8_t *fp = const_cast<uint8_t *>(a.frames) + (size_t)off * 64u;

    // ---- TCP span bytes from 32 on (chunk >= 2), masked at data_len.  Bytes [26, 32) come
    // from the leader's header dwords below.
    uint32_t ts[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < NLOAD; ++j) {
        const int c = gl + j * LPF;
        const int n = (int)len - c * 16;
        if (TX && j * LPF <= 3 && 3 < (j + 1) * LPF) {
            if (c == 3) d[j][0] &= 0x0000FFFFu;  // the cksum field (bytes 50-51) is zero while summing
        }
        uint32_t w = n >= 16 ? kOnes : 0u;
        if (j * LPF < 2) w = c >= 2 ? w : 0u;
        full_sum(d[j], w, ts);
        bool part = n > 0 && n < 16;
        if (j * LPF < 2) part = part && c >= 2;
        if (part) partial_sum(d[j], n, ts);
    }
    uint32_t tsum = ts[0] + ts[1] + ts[2] + ts[3];

    // ---- header dwords 1..11 (bytes 4..47) in the leader: chunk 0 its own, chunk 1 from
    // lane +1, chunk 2 from lane +2 (LPF 2: the leader's second load)
    const uint32_t h1 = d[0][1], h2 = d[0][2], h3 = d[0][3];
    const uint32_t h4 = dpp_down<1>(d[0][0]), h5 = dpp_down<1>(d[0][1]);
    const uint32_t h6 = dpp_down<1>(d[0][2]), h7 = dpp_down<1>(d[0][3]);
    uint32_t h8, h9, h10 = 0, h11;
    if constexpr (LPF == 2) {
        h8 = d[1][0]; h9 = d[1][1]; h10 = d[1][2]; h11 = d[1][3];
    } else {
        h8 = dpp_down<2>(d[0][0]);
        h9 = dpp_down<2>(d[0][1]);
        if constexpr (MODE == 48) h10 = dpp_down<2>(d[0][2]);
        h11 = dpp_down<2>(d[0][3]);
    }
    tsum = group_sum<LPF>(tsum, lane);

    const uint32_t tl = bswap16(h4 & 0xFFFFu);  // ip total_length
    const int E = max(34, 14 + (int)tl);
    const int tcp_end = min((int)len, E);
    if (__ballot(leader && tcp_end < (int)len) != 0ull) {
        // a frame of this round has bytes past its TCP span: re-sum by the span
        const int te = (int)lane_read((uint32_t)tcp_end, gbase);
        uint32_t t4[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < NLOAD; ++j) {
            const int c = gl + j * LPF;
            const int n = te - c * 16;
            if (c >= 2 && n > 0) {
                if (n >= 16)
                    full_sum(d[j], kOnes, t4);
                else
                    partial_sum(d[j], n, t4);
            }
        }
        const uint32_t t2 = group_sum<LPF>(t4[0] + t4[1] + t4[2] + t4[3], lane);
        if (tcp_end < (int)len) tsum = t2;
    }

    const uint32_t h6_ip = TX ? (h6 & 0xFFFF0000u) : h6;  // TX: hdr_checksum (bytes 24-25) = 0
    uint32_t isum = dsum(h3 & 0xFFFF0000u, kOnes, 0u);
    isum = dsum(h4, kOnes, isum);
    isum = dsum(h5, kOnes, isum);
    isum = dsum(h6_ip, kOnes, isum);
    isum = dsum(h7, kOnes, isum);
    isum = dsum(h8 & 0xFFFFu, kOnes, isum);
    // pseudo {src, dst (bytes 26..33), 0x00, 0x06, htons(total_length - 20)}: bytes 26..31
    // here, 32..33 are in chunk 2's lane sum
    uint32_t tall = dsum(h6 & 0xFFFF0000u, kOnes, tsum);
    tall = dsum(h7, kOnes, tall);
    tall += 0x0600u + bswap16((tl - 20u) & 0xFFFFu);
    const uint32_t ip_ck = (~bswap16(fold16(isum))) & 0xFFFFu;
    const uint32_t tcp_ck = (~bswap16(fold16(tall))) & 0xFFFFu;

    Fields F;
    F.ck = ip_ck | (tcp_ck << 16);
    F.et = bswap16(h3 & 0xFFFFu) | ((h5 >> 24) << 16) | ((h11 >> 24) << 24);
    F.ports = (bswap16(h9 & 0xFFFFu) << 16) | bswap16(h8 >> 16);
    F.src = (h6 >> 16) | (h7 << 16);
    F.dst = (h7 >> 16) | (h8 << 16);
    F.tl = tl | (((h3 >> 16) & 0xFFu) << 16) | (((h11 >> 16) & 0xFFu) << 24);
    F.seq = (h9 >> 16) | (h10 << 16);
    F.ack = (h10 >> 16) | (h11 << 16);
    F.h1 = h1;
    F.h2 = h2;
    if constexpr (PAY) {
        // The payload hand-off fused in: the leader's header gives the span (pay_span); every
        // lane of the group writes those of its chunks that fall in the payload's 64-byte
        // lines, as loaded, at the same offset in the arena.  Whole lines (no partial-line
        // writes), no byte shift; the bytes written are the pool's own.
        const uint32_t span = lane_read(pay_span(leader, len, F.et, F.tl), gbase);
        if (active && span != 0u && a.pay_arena != nullptr) {
            uint8_t *dst = a.pay_arena + (size_t)off * 64u;
#pragma unroll
            for (int j = 0; j < NLOAD; ++j) {
                const uint32_t c = (uint32_t)(gl + j * LPF);
                if (pay_writes_chunk(c, span)) pay_store16<false>(dst + 16u * c, d[j]);
            }
        }
    }
    if constexpr (TX) {
        // ip_out stores both as htons(calculate_checksum(...)) (ip.c:107,118).  Frames of
        // these classes are longer than 64 bytes: the group writes the frame's whole first
        // 64-byte line (chunks 0-3, as loaded, with the two checksum fields set) rather
        // than two 2-byte stores, so HBM sees full-line writes, not partial-line ones
        // (C3 tx 327 -> 310 us).  Measured slower: holding the writes until
        // the next round's loads are issued (322), non-temporal line stores, the whole
        // 128-byte L2 line, only the two 16-byte chunks holding the fields, the line writes
        // queued to the wave's end.
        const uint32_t ck2 = lane_read(bswap16(ip_ck) | (bswap16(tcp_ck) << 16), gbase);
#pragma unroll
        for (int j = 0; j < NLOAD && j * LPF < 4; ++j) {
            const int c = gl + j * LPF;
            if (active && c < 4) {
                uint4 q = make_uint4(d[j][0], d[j][1], d[j][2], d[j][3]);
                if (c == 1) q.z = (q.z & 0xFFFF0000u) | (ck2 & 0xFFFFu);        // bytes 24-25
                if (c == 3) q.x = (q.x & 0x0000FFFFu) | (ck2 & 0xFFFF0000u);    // bytes 50-51
                *reinterpret_cast<uint4 *>(fp + 16 * c) = q;
            }
        }
    }
    return F;
}

__device__ __forceinline__ void transpose_small_slice(const uint4 (&v)[4], int lane, uint32_t *sf,
                                                      uint32_t (&d)[4][4]);

// part / parts: this wave takes rounds part, part + parts, ... of the class (the server's
// cooperative single slice, rx_body; 0 / 1 everywhere else).
template <int C, int LPF, int NLOAD, bool JUMBO, int MODE, bool NT, bool PIPE = false, bool PAY = false>
__device__ __forceinline__ void run_class(const RxArgs &a, int cls, uint32_t off, uint32_t len,
                                          int lane_in, uint32_t *sf, uint32_t part = 0u, uint32_t parts = 1u)
{
    constexpr int FPW = 64 / LPF;
    const uint32_t r0 = part * (uint32_t)FPW, step = parts * (uint32_t)FPW;
    const unsigned long long m = __ballot(cls == C);
    if (m == 0ull) return;
    // An opaque copy of the lane id: without it LICM hoists every class's lane-derived
    // invariants (chunk offsets, bpermute addresses, masks) out of the slice loop, where
    // they stay live across all classes (measured: 166 VGPRs vs ~100 for one class).
    int lane = lane_in;
    asm volatile("" : "+v"(lane));
    const uint32_t cnt = (uint32_t)__popcll(m);
    uint32_t corig = (uint32_t)lane, coff = off, clen = len;
    if (m != ~0ull) {
        // compact this class's frames to lanes 0..cnt-1, keeping their order
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        const uint32_t dst = (cls == C) ? below : cnt + ((uint32_t)lane - below);
        corig = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst << 2), lane);
        coff = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst << 2), (int)off);
        clen = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst << 2), (int)len);
    }
    // Rounds software-pipelined: round r + 1's loads are issued before round r is waited
    // for, into the other of two register buffers (the steps alternate, so no register copy
    // of a load in flight).  Loads are issued unconditionally, a round past the class's last
    // frame reading the arena's first bytes with every lane inactive: a load under a branch
    // leaves the wait at the join counting as if it were absent (vmcnt(0)).  DESIGN.md §5.
    static_assert(!(PIPE && PAY), "the pipelined rounds (tx, server) carry no payload hand-off");
    if constexpr (PIPE && LPF >= 2 && !JUMBO) {
        uint32_t dA[NLOAD][4], dB[NLOAD][4];
        auto rmeta = [&](uint32_t r, uint32_t &korig, uint32_t &koff, uint32_t &klen) -> bool {
            int rl = lane;
            asm volatile("" : "+v"(rl));
            const uint32_t k = r + (uint32_t)(rl / LPF);
            const int src = (int)(k & 63u);
            korig = lane_read(corig, src);
            koff = lane_read(coff, src);
            klen = lane_read(clen, src);
            const bool act = k < cnt;
            if (!act) koff = klen = 0u;
            return act;
        };
        uint32_t ao, aoff, alen, bo, boff, blen;
        bool aact = rmeta(r0, ao, aoff, alen);
        round_load<C, LPF, NLOAD, NT, PAY>(a, aoff, alen, lane, dA);
        // one loop body, no exit in its middle: the loads of both buffers are issued every
        // iteration and only round B's compute is conditional, so the wait for each buffer
        // counts exactly the other buffer's loads issued after it
        for (uint32_t r = r0; r < cnt; r += 2u * step) {
            const bool bact = rmeta(r + step, bo, boff, blen);
            round_load<C, LPF, NLOAD, NT, PAY>(a, boff, blen, lane, dB);
            {
                const Fields F = frame_round_compute<C, LPF, NLOAD, MODE, NT, PAY>(a, aoff, alen, aact, lane, dA);
                if constexpr (MODE != 0) {
                    if (aact && (lane & (LPF - 1)) == 0) park_fields<MODE>(sf, ao, F);
                }
            }
            aact = rmeta(r + 2u * step, ao, aoff, alen);
            round_load<C, LPF, NLOAD, NT, PAY>(a, aoff, alen, lane, dA);
            if (r + step < cnt) {
                const Fields F = frame_round_compute<C, LPF, NLOAD, MODE, NT, PAY>(a, boff, blen, bact, lane, dB);
                if constexpr (MODE != 0) {
                    if (bact && (lane & (LPF - 1)) == 0) park_fields<MODE>(sf, bo, F);
                }
            }
        }
        return;
    }
    for (uint32_t r = r0; r < cnt; r += step) {
        const uint32_t k = r + (uint32_t)(lane / LPF);
        const bool act = k < cnt;
        uint32_t korig, koff, klen;
        if constexpr (LPF == 1) {
            korig = corig; koff = coff; klen = clen;
        } else {
            const int src = (int)(k & 63u);
            korig = lane_read(corig, src);
            koff = lane_read(coff, src);
            klen = lane_read(clen, src);
        }
        int rl = lane;
        asm volatile("" : "+v"(rl));  // keep per-round lane math inside the round (VGPRs)
        Fields F;
        if constexpr (LPF == 1) {
            // The class's frames are loaded as the all-small path loads a slice (lane l:
            // chunk l&3 of frame 16j + l/4, 16 whole frames and 16 lines per instruction) and
            // transposed through LDS (4 KiB after the parked fields).  Lane i loading its own
            // frame's four chunks touched up to 64 lines per instruction: C4 78.9 -> 75.2 us
            // (DESIGN.md §5).
            uint4 v[4];
            const int ch = rl & 3;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int fr = 16 * j + (rl >> 2);
                const uint32_t foff = lane_read(coff, fr), flen = lane_read(clen, fr);
                const bool ok = (uint32_t)fr < cnt && (uint32_t)(ch * 16) < flen;
                v[j] = load16<NT>(ok ? a.frames + (size_t)foff * 64u + ch * 16 : a.frames);
            }
            uint32_t d[4][4];
            // (MODE 0, tx: no parked fields; the transpose uses the 4 KiB ring area itself)
            transpose_small_slice(v, rl, sf + (MODE == 0 ? 0 : MODE == 48 ? NF48 * 64 : NF16 * 64), d);
            F = fields_small<MODE>(const_cast<uint8_t *>(a.frames) + (size_t)koff * 64u, act ? klen : 0u, d);
            if constexpr (PAY) pay_line_small(a, koff, pay_span(act, klen, F.et, F.tl), d);
        } else if constexpr (LPF >= 2 && !JUMBO)
            F = frame_round_fast<C, LPF, NLOAD, MODE, NT, PAY>(a, act ? koff : 0u, act ? klen : 0u, act, rl);
        else
            F = frame_round<LPF, NLOAD, JUMBO, MODE, NT, PAY>(a, koff, act ? klen : 0u, act, rl);
        if constexpr (MODE != 0) {
            if (act && (lane & (LPF - 1)) == 0) park_fields<MODE>(sf, korig, F);
        }
    }
}

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
// DESIGN.md §9.R3); the server walks per lane with vector loads (see sload_bucket).
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
// REC48 3 KiB.
constexpr int ring_slot_u4(int mode) { return mode * 64 / 16; }

template <int MODE, int RS>
struct RecRing {
    static constexpr int kQ = MODE / 16;  // uint4 per record (REC16 / REC48)
    static constexpr int kSlot = ring_slot_u4(MODE);
    uint4 (*img)[kSlot];                  // [RS][kSlot]: the slice's records, contiguous
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
    // stores 1 KiB contiguously.  Records of frames >= n_frames are not written.  NTS:
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
template <int P, int MODE, int DESC, bool VWALK, int RS, bool PAY, typename BC>
__device__ __forceinline__ bool small_step(const RxArgs &a, int lane, uint32_t &s, uint32_t nslices,
                                           uint32_t nwaves, uint32_t &c_off, uint32_t &c_len, uint32_t &n_off,
                                           uint32_t &n_len, uint4 (&vb)[2][4], RecRing<MODE, RS> &ring,
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
    if constexpr (PAY) {  // (one burst per PAY launch: frame s * 64 + lane)
        const uint32_t span = pay_span(valid, c_len, F.et, F.tl);
        pay_line_small(a, c_off, span, d);
        pay_msg(a, s * 64u + (uint32_t)lane, valid, c_off, span);
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
template <int P, int MODE, int DESC, bool VWALK, int RS, bool PAY, typename BC>
__device__ __forceinline__ bool small_step2(const RxArgs &a, int lane, uint32_t &s, uint32_t nslices,
                                            uint32_t nwaves, uint32_t &c_off, uint32_t &c_len, uint32_t &n_off,
                                            uint32_t &n_len, uint32_t &y_off, uint32_t &y_len, bool &pend,
                                            uint4 (&vb)[2][4], RecRing<MODE, RS> &ring, WaveCounters &wc, Rec &rec,
                                            FlowCache &fc, unsigned long long &bytes, BC &bc)
{
    const uint32_t s1 = s + nwaves, s2 = s + 2u * nwaves;
    uint32_t d[4][4];
    uint32_t *sf = ring.template scratch<true>(a, lane, 4096, bc);
    transpose_small_slice(vb[P], lane, sf, d);
    const Fields F = fields_small<MODE>(nullptr, c_len, d);
    if constexpr (PAY) {
        const uint32_t span = pay_span(true, c_len, F.et, F.tl);
        pay_line_small(a, c_off, span, d);
        pay_msg(a, s * 64u + (uint32_t)lane, true, c_off, span);
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
//   PAY    the payload hand-off fused in (rxg_rx_burst_payload_dev: one burst, launched)
//   SRV    the server's form: streaming-class rounds software-pipelined (a served burst's
//          frame reads are latency-bound: 32 x 1500 B bursts 25.6-27.6 -> 22.2-23.2 us) and
//          overflow walks with vector loads (VWALK, see sload_bucket)
template <int MODE, int DESC, bool MULTI, bool DEEP, bool SRV, bool PAY = false>
__device__ __forceinline__ void rx_body(RxArgs a, uint32_t blk, uint32_t nblk)
{
    constexpr int NF = MODE == 48 ? NF48 : NF16;
    __shared__ unsigned long long s_cnt[4][RXG_NCOUNTERS];
    // Per-wave LDS = the record ring (REC16: 11 slices of 1 KiB, REC8: 22 of 512 B, REC48: 4 of
    // 3 KiB); its free slots are also the scratch of the slice in progress (4 KiB
    // small-slice transpose, NF x 256 B parked fields), so LDS per wave is the ring alone.
    // 3 workgroups per CU (LDS and, at ~145 VGPRs, registers).
    // (tx, MODE 0: 4 x 1 KiB, the class-0 transpose's scratch; no records)
    constexpr int RS = MODE == 16 ? 11 : MODE == 48 ? 4 : MODE == 8 ? 22 : 4;
    constexpr int kSlot = ring_slot_u4(MODE == 0 ? 16 : MODE);
    static_assert(MODE == 0 || (RS * kSlot * 16 >= 4096 + kSlot * 16 && RS * kSlot * 16 >= NF * 256 + 4096),
                  "ring too small for the scratch");
    __shared__ __attribute__((aligned(16))) uint4 s_rec[4][RS][kSlot];
    __shared__ uint32_t s_recf[4][RS];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const uint32_t wave = blk * 4u + (uint32_t)wid;
    const uint32_t nwaves = nblk * 4u;

    WaveCounters wc;
#pragma unroll
    for (int k = 0; k < RXG_NCOUNTERS; ++k) wc.c[k] = 0u;
    unsigned long long bytes = 0ull;
    RecRing<MODE == 0 ? 16 : MODE, RS> ring;
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
    // leader's scratch; the leader classifies after a workgroup barrier.
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
            if constexpr (PAY) pay_msg(a, s * 64u + (uint32_t)lane, valid, off, pay_span(valid, len, F.et, F.tl));
            classify_store<MODE, SRV>(a, valid, len, F, wc, rec, fcache, sf + NF * 64);
            __builtin_amdgcn_wave_barrier();  // phase B reads before the next slice's writes
            if (ring.n == RS) ring.flush(a, lane, bc);
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
        // latency, and these were 0.75 us of it.  A lane's bytes fit 32 bits
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
template <int MODE, int DESC, bool MULTI, bool DEEP, bool PAY = false>
__global__ __launch_bounds__(256, 1) void rx_kernel(RxArgs a)
{
    static_assert(!(PAY && (MULTI || MODE == 0 || DESC == kDescSel)), "PAY: one receive burst");
    rx_body<MODE, DESC, MULTI, DEEP, false, PAY>(a, blockIdx.x, gridDim.x);
}

// ------------------------------------------------------------- latency-mode server ---
// rx_server: the same workgroup body as rx_kernel<MODE> (one burst, the SRV form), run once
// per request by a persistent grid (rxg_server_*).  Wave 0 of workgroup 0
// polls the mailbox's first 128 bytes (system-scope loads, s_sleep between polls) and takes a
// request when its number is new and the check word matches (srv_check).  A request of
// P <= gridDim workgroups' worth of slices (4 slices per workgroup, one per wave, then
// round-robin) runs on workgroups 0 .. P-1.  When P > 1, workgroup 0 copies the request to
// SrvCtl::req and then publishes SrvCtl::go = number << 16 | P (agent-scope release /
// acquire): a workgroup that sees a new go learns P from go itself and reads req only when it
// takes part.  A participant's read cannot race the next request's copy: workgroup 0 copies
// request g+1 only after `done` of g, which needs every participant of g to have finished.
// Every participant classifies its slices, makes its record stores visible, and the last to
// finish (SrvCtl::fin reset for the next request) publishes `done`.  Exit: `stop`, or no
// request for idle_ticks of the constant-rate wall clock (the host relaunches on its next
// burst), so a server whose process is gone ends by itself.
struct SrvArgs {
    SrvMbox *mbox;  // the host-written words (seq, request, stop): host memory or device memory
    SrvMbox *ret;   // the server's words (done, exited): host memory (= mbox when it is there)
    SrvCtl *ctl;
    unsigned long long *counters;
    unsigned long long idle_ticks;
};

__device__ __forceinline__ uint64_t uniform64(uint64_t v)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// workgroups a request of n frames runs on
__device__ __forceinline__ uint32_t srv_participants(uint32_t n, uint32_t flags)
{
    const uint32_t nsl = (n + 63u) / 64u;
    // large frames, 3..gridDim slices: one slice per workgroup (rx_body's shared slices)
    if ((flags & kSrvLarge) && nsl >= 3u && nsl <= gridDim.x) return nsl;
    return max(1u, min(gridDim.x, (nsl + 3u) / 4u));
}

// XOR of v over the 16 lanes of each row (every lane gets it): row rotations by 8 and 4,
// then two quad permutations.
__device__ __forceinline__ uint32_t row_xor16(uint32_t v)
{
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    return v;
}

// Three waves per SIMD at most (168 VGPRs): the pipelined rounds would otherwise take 170.
template <int MODE>
__global__ __launch_bounds__(256, 3) void rx_server(SrvArgs sa)
{
    __shared__ SrvReq s_req;
    __shared__ unsigned long long s_desc[kSrvPollWords - 16];  // an inline request's off64 / len
    __shared__ unsigned long long s_seq;  // the request's number (kSrvStop: exit)
    __shared__ uint32_t s_p;              // its participants
    // thread 0: the number of the last request seen.  It starts at `done` (the host sets go to
    // done << 16 before the launch): a workgroup that starts late, after a request g it should
    // take part in was published, still sees g as new, since g is not done without it.
    unsigned long long last = 0ull;
    if (threadIdx.x == 0) last = __hip_atomic_load(&sa.ret->done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    for (;;) {
        if (blockIdx.x == 0 && threadIdx.x < 64) {
            // wave 0 polls the mailbox's first 320 bytes (lane l < 40: bytes 8l .. 8l+7) in
            // one instruction: the request arrives with its number and, for a small host
            // burst, its descriptors (words 16-39): no second round trip before the frames
            const int l = (int)threadIdx.x;
            const unsigned long long lst = __shfl(last, 0, 64);
            const long long t0 = wall_clock64();
            unsigned long long q;
            for (;;) {
                unsigned long long w = 0ull;
                if (l < kSrvPollWords)
                    w = __hip_atomic_load(reinterpret_cast<const unsigned long long *>(sa.mbox) + l, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_SYSTEM);
                q = __shfl(w, 0, 64);
                const unsigned long long ck = __shfl(w, 12, 64), st = __shfl(w, 13, 64);
                if (st != 0ull) {
                    q = kSrvStop;
                    break;
                }
                if (q != lst) {
                    // the check word over the number, the request words (lanes 0-11) and an
                    // inline request's descriptor words (lanes 16-39; SrvReq::flags is the
                    // high half of word 5): a snapshot mixing two requests' words (a
                    // write-combined mailbox line that reached the device in parts) fails it
                    // and is polled again
                    const bool inl = ((__shfl(w, 5, 64) >> 32) & kSrvInlineDesc) != 0ull;
                    const bool mixed = l < 12 || (inl && l >= 16 && l < kSrvPollWords);
                    const unsigned long long m = mixed ? srv_mix((unsigned)l, w) : 0ull;
                    const uint32_t lo = row_xor16((uint32_t)m), hi = row_xor16((uint32_t)(m >> 32));
                    // the rows' XORs (lanes 48-63 hold none)
                    const uint32_t xlo = (uint32_t)__builtin_amdgcn_readlane((int)lo, 0) ^
                                         (uint32_t)__builtin_amdgcn_readlane((int)lo, 16) ^
                                         (uint32_t)__builtin_amdgcn_readlane((int)lo, 32);
                    const uint32_t xhi = (uint32_t)__builtin_amdgcn_readlane((int)hi, 0) ^
                                         (uint32_t)__builtin_amdgcn_readlane((int)hi, 16) ^
                                         (uint32_t)__builtin_amdgcn_readlane((int)hi, 32);
                    if ((((unsigned long long)xhi << 32) | xlo) == ck) {
                        if (l >= 1 && l <= 11) reinterpret_cast<unsigned long long *>(&s_req)[l - 1] = w;  // bytes 8 .. 95
                        if (inl && l >= 16 && l < kSrvPollWords) s_desc[l - 16] = w;
                        break;
                    }
                }
                if ((unsigned long long)(wall_clock64() - t0) > sa.idle_ticks) {
                    q = kSrvStop;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            // One acquire per request, not per poll: the CU's L1 may hold lines of the previous
            // request's staging (host memory, same addresses) or of device memory written since
            // (mirror tables, caller frames); waited for before any wave of the workgroup loads
            // (MI355X_MICROARCH.md, inter-workgroup visibility).  A first form with relaxed
            // polls and no acquire served stale staging lines (test_gpu_server).
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            // the request's words, written by lanes 1-11, for lane 0
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (l == 0) {
                const uint32_t P = q == kSrvStop ? gridDim.x : srv_participants(s_req.n, s_req.flags);
                // the others hear of a request only when they take part in it (and of stop)
                if (gridDim.x > 1 && P > 1u) {
                    if (q != kSrvStop) sa.ctl->req = s_req;
                    // release (MI355X_MICROARCH.md: the wait after the write-back, by hand)
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __hip_atomic_store(&sa.ctl->go, q == kSrvStop ? kSrvStop : (q << 16) | P, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
                s_seq = q;
                s_p = P;
                last = q;
            }
        } else if (blockIdx.x != 0 && threadIdx.x == 0) {
            unsigned long long go;
            for (;;) {  // relaxed polls, then one acquire (MI355X_MICROARCH.md)
                go = __hip_atomic_load(&sa.ctl->go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((go >> 16) != last) break;  // (kSrvStop >> 16 is no request number)
                __builtin_amdgcn_s_sleep(2);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // this CU's L1 (see workgroup 0)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t P = go == kSrvStop ? gridDim.x : (uint32_t)(go & 0xFFFFu);
            if (go != kSrvStop && blockIdx.x < P) {
                // vector loads (never the scalar cache, which the acquire does not invalidate)
                const unsigned long long *src = reinterpret_cast<const unsigned long long *>(&sa.ctl->req);
                unsigned long long *dst = reinterpret_cast<unsigned long long *>(&s_req);
#pragma unroll
                for (int k = 0; k < (int)(sizeof(SrvReq) / 8); ++k)
                    dst[k] = __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            s_seq = go == kSrvStop ? kSrvStop : go >> 16;
            s_p = P;
            last = go >> 16;
        }
        __syncthreads();
        const unsigned long long q = s_seq;
        if (q == kSrvStop) break;
        const uint32_t P = s_p;
        if (blockIdx.x >= P) {  // published for the first P workgroups of a larger grid
            __syncthreads();
            continue;
        }
        RxArgs a;
        a.frames = as_global<const uint8_t>(uniform64((uint64_t)s_req.frames));
        a.sel = nullptr;
        a.nbursts = 1u;
        a.stride64 = 0u;
        a.t.buckets = as_global<const uint4>(uniform64((uint64_t)s_req.table.buckets));
        a.t.listen = as_global<const int32_t>(uniform64((uint64_t)s_req.table.listen));
        a.t.arp = as_global<const uint4>(uniform64((uint64_t)s_req.table.arp));
        a.t.bucket_mask = uniform(s_req.table.bucket_mask);
        a.t.ntcb = (int32_t)uniform((uint32_t)s_req.table.ntcb);
        a.t.min_null = (int32_t)uniform((uint32_t)s_req.table.min_null);
        a.t.arp_mask = uniform(s_req.table.arp_mask);
        a.t.arp_flags = uniform(s_req.table.arp_flags);
        a.counters = sa.counters;
        if (uniform(s_req.flags) & kSrvInlineDesc) {
            // a small host burst: its descriptors came with the request (LDS, generic pointers)
            a.b[0].off64 = reinterpret_cast<const uint32_t *>(s_desc);
            a.b[0].len = reinterpret_cast<const uint16_t *>(reinterpret_cast<const uint8_t *>(s_desc) + kSrvInline * 4u);
        } else {
            a.b[0].off64 = reinterpret_cast<const uint32_t *>(uniform64((uint64_t)s_req.off64));
            a.b[0].len = reinterpret_cast<const uint16_t *>(uniform64((uint64_t)s_req.len));
        }
        a.b[0].out = as_global<uint8_t>(uniform64((uint64_t)s_req.out));
        a.b[0].n = uniform(s_req.n);
        a.b[0].slice0 = 0u;
        a.nslices = (a.b[0].n + 63u) / 64u;
        rx_body<MODE, kDescList, false, false, true>(a, blockIdx.x, P);
        // Every wave's stores have reached the L2 (vmcnt), then ONE system-scope release per
        // workgroup writes this XCD's L2 back (buffer_wbl2 covers the whole cache, so one
        // per workgroup covers its four waves; it used to run once per wave and once more
        // before `done`), before the workgroup counts itself finished
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            bool lastp = true;
            if (P > 1u) {
                lastp = atomicAdd(&sa.ctl->fin, 1u) + 1u == P;
                if (lastp) {
                    atomicExch(&sa.ctl->fin, 0u);  // before `done`: the next request counts from 0
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            }
            if (lastp) __hip_atomic_store(&sa.ret->done, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();  // s_req and s_seq are rewritten by the next request
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(&sa.ret->exited, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------------- launch helpers ---
// The kernel arguments and grid of a launch (host side, shared by rxg_kernels.hip and the
// experiment library's rxg_kernels_exp.hip).
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
