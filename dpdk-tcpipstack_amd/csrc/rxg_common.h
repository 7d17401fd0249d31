// rxg_common.h — definitions shared by rxg's host code and its gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rxg.h"

#if defined(__HIPCC__)
#define RXG_HD __host__ __device__ __forceinline__
#else
#define RXG_HD static inline
#endif

namespace rxg {

// ---------------------------------------------------------------------------------------
// Device TCB mirror.
//   bucket table: nbuckets x 4 slots x 16 B = one 64-byte line per bucket.  A slot is
//     {ports = dport<<16 | sport, ipv4_dst raw, ipv4_src host, value}; value = the
//     LOWEST tcbs[] index holding that exact tuple (findtcb pass 1 returns the first
//     match, tcp_tcb.c:145-159) in bits 0..23 and that TCB's state (tcp_in.c:54 reads it
//     after the lookup) in bits 24..31; kEmpty marks a free slot.  Linear probing over
//     buckets; a lookup ends at the first bucket holding a free slot.
//   listen[65536]: lowest index i with tcbs[i] live, LISTENING, dport == port (pass 2,
//     tcp_tcb.c:160-169), or -1.  Its state is LISTENING by construction.
//   min_null: lowest removed slot index (pass 2 would dereference NULL there).
// ---------------------------------------------------------------------------------------
constexpr uint32_t kEmpty = 0xFFFFFFFFu;
constexpr int kSlotsPerBucket = 4;
constexpr uint32_t kIdxMask = 0x00FFFFFFu;
constexpr int kStateShift = 24;
constexpr int32_t kMaxTcbs = 0x00FFFFFF;  // indices 0 .. kMaxTcbs-1
constexpr int kKernelCounterRows = RXG_COUNTER_ROWS - 1;  // the last row is the host's

RXG_HD uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

RXG_HD uint32_t tuple_hash(uint32_t ports, uint32_t dst_raw, uint32_t src_host)
{
    uint32_t h = 0x9E3779B9u ^ (ports * 0xCC9E2D51u);
    h = rotl32(h, 13) * 5u + 0xE6546B64u;
    h ^= rotl32(dst_raw * 0xCC9E2D51u, 15) * 0x1B873593u;
    h = rotl32(h, 13) * 5u + 0xE6546B64u;
    h ^= rotl32(src_host * 0xCC9E2D51u, 15) * 0x1B873593u;
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}

RXG_HD uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }
RXG_HD uint32_t bswap32(uint32_t x)
{
    return (x << 24) | ((x & 0xFF00u) << 8) | ((x >> 8) & 0xFF00u) | (x >> 24);
}

// One's-complement fold of a 32-bit sum of 16-bit words to 16 bits (the reference's
// `while (sum & 0xffff0000) sum = (sum & 0xffff) + (sum >> 16)`, ip.c:55-57).
RXG_HD uint32_t fold16(uint32_t s)
{
    s = (s & 0xFFFFu) + (s >> 16);
    s = (s & 0xFFFFu) + (s >> 16);
    return s;
}

// splitmix64 (synthetic payload / PRNG).
RXG_HD uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// Synthetic IMIX: blocks of 12 frames, 7 x 64 B, 4 x 576 B, 1 x 1500 B, rotated per block.
constexpr int kImixBlock = 12;
constexpr int kImixSlotsPerBlock = 7 * 1 + 4 * 9 + 1 * 24;  // 64-byte slots
RXG_HD uint32_t imix_len(int pos)
{
    // base pattern 64,576,64,64,1500,64,576,64,576,64,64,576
    const uint32_t pat = 0b100101000010u;  // bit k set = 576 at position k: 1, 6, 8, 11
    if (pos == 4) return 1500u;
    return ((pat >> pos) & 1u) ? 576u : 64u;
}

// ARP mirror: a set of host-order IPv4 addresses as buckets of four 4-byte keys (one 16-byte
// load per probe), key 0 = free; the address 0 itself is a flag of the launch (DevTable).
// Linear probing over buckets; a lookup ends at the first bucket holding a free key.
constexpr int kArpKeysPerBucket = 4;
RXG_HD uint32_t arp_hash(uint32_t ip)
{
    uint32_t h = ip ^ 0x41525000u;  // murmur3 finaliser: two multiplies
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}
constexpr uint32_t kArpOn = 1u, kArpZero = 2u;  // DevTable::arp_flags

struct DevTable {
    const uint4 *buckets;  // nbuckets * 4 slots
    const int32_t *listen; // 65536
    const uint4 *arp;      // ARP mirror buckets (a valid 16-byte word even with the mirror off)
    uint32_t bucket_mask;  // nbuckets - 1
    int32_t ntcb;
    int32_t min_null;      // INT32_MAX if none
    uint32_t arp_mask;     // ARP buckets - 1 (0 with the mirror off: every lane reads one word)
    uint32_t arp_flags;    // kArpOn | kArpZero (0.0.0.0 is a member)
};

}  // namespace rxg
