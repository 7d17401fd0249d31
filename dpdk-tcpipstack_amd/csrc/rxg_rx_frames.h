// rxg_rx_frames.h — phase A of the receive body: a frame's chunks loaded, summed for the IP
// and pseudo || TCP checksums (ip.c:44-59) and its header fields extracted, per size class.
#pragma once
#include <hip/hip_runtime.h>

#include "rxg_rx_core.h"

namespace rxg {

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

template <int LPF, int NLOAD, bool JUMBO, int MODE, bool NT, int PAY = kPayNone>
__device__ __forceinline__ Fields frame_fields(const RxArgs &a, uint32_t off, uint32_t len, bool active,
                                               int lane, uint32_t (&d)[NLOAD][4]);

template <int LPF, int NLOAD, bool JUMBO, int MODE, bool NT, int PAY = kPayNone>
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
template <int LPF, int NLOAD, bool JUMBO, int MODE, bool NT, int PAY>
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
    if constexpr (PAY == kPayCopy) {  // every lane holds the header here (hdr_dword)
        const uint32_t span = pay_span(active, len, F.et, F.tl);
        if (span != 0u) {
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
        // wave's end (HISTORY.md §9.R3).
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
template <int C, int LPF, int NLOAD, bool NT, int PAY = kPayNone>
__device__ __forceinline__ void round_load(const RxArgs &a, uint32_t off, uint32_t len, int lane,
                                           uint32_t (&d)[NLOAD][4])
{
    constexpr int SAFE = (class_min_len(C) + 63) & ~63;  // bytes every frame of the class has
    const int gl = lane & (LPF - 1);
    const uint8_t *fp = a.frames + (size_t)off * 64u;
    // PAY: chunks up to the end of the frame's last 64-byte line are loaded as they are (that
    // line is readable, rxg_dev_batch): the payload's lines are written whole
    const uint32_t lastc = len ? (PAY == kPayCopy ? ((len + 63u) & ~63u) - 16u : ((len - 1u) & ~15u)) : 0u;
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

template <int C, int LPF, int NLOAD, int MODE, bool NT, int PAY = kPayNone>
__device__ __forceinline__ Fields frame_round_compute(const RxArgs &a, uint32_t off, uint32_t len, bool active,
                                                      int lane, uint32_t (&d)[NLOAD][4]);

template <int C, int LPF, int NLOAD, int MODE, bool NT, int PAY = kPayNone>
__device__ __forceinline__ Fields frame_round_fast(const RxArgs &a, uint32_t off, uint32_t len, bool active,
                                                   int lane)
{
    uint32_t d[NLOAD][4];
    round_load<C, LPF, NLOAD, NT, PAY>(a, off, len, lane, d);
    return frame_round_compute<C, LPF, NLOAD, MODE, NT, PAY>(a, off, len, active, lane, d);
}

// Sums, header fields and (tx) checksum stores of one round whose chunks are in d; PAY: the
// payload lines written to the arena from the same registers.
template <int C, int LPF, int NLOAD, int MODE, bool NT, int PAY>
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
    if constexpr (PAY == kPayCopy) {
        // The payload hand-off fused in: the leader's header gives the span (pay_span); every
        // lane of the group writes those of its chunks that fall in the payload's 64-byte
        // lines, as loaded, at the same offset in the arena.  Whole lines (no partial-line
        // writes), no byte shift; the bytes written are the pool's own.
        const uint32_t span = lane_read(pay_span(leader, len, F.et, F.tl), gbase);
        if (active && span != 0u) {
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
        // (C3 tx 327 -> 310 us).  Measured slower (HISTORY.md §9): holding the writes until
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
template <int C, int LPF, int NLOAD, bool JUMBO, int MODE, bool NT, bool PIPE = false, int PAY = kPayNone>
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
            if constexpr (PAY == kPayCopy) pay_line_small(a, koff, pay_span(act, klen, F.et, F.tl), d);
        } else if constexpr (LPF >= 2 && !JUMBO)
            F = frame_round_fast<C, LPF, NLOAD, MODE, NT, PAY>(a, act ? koff : 0u, act ? klen : 0u, act, rl);
        else
            F = frame_round<LPF, NLOAD, JUMBO, MODE, NT, PAY>(a, koff, act ? klen : 0u, act, rl);
        if constexpr (MODE != 0) {
            if (act && (lane & (LPF - 1)) == 0) park_fields<MODE>(sf, korig, F);
        }
    }
}

}  // namespace rxg
