// rxg_kernels.h — host-side launch interface of rxg_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

#include "rxg_common.h"

namespace rxg {

struct MirrorPatch;  // rxg_mirror.h

// One launch classifies up to kMaxBursts bursts whose frames share one pool (`frames`):
// burst k's frame i is at frames + 64 * off64[i], its record at out + i * record size.
constexpr uint32_t kMaxBursts = 32;
struct LaunchBurst {
    const uint32_t *off64;  // strided launches (LaunchRx::stride64 != 0): unused
    const uint16_t *len;
    uint32_t n;            // >= 1 (empty bursts are not launched)
    uint8_t *out;          // records (receive), unused for tx
    uint32_t slot0;        // strided launches: the 64-byte slot of the burst's frame 0
};

struct LaunchRx {
    const uint8_t *frames;
    const uint32_t *sel;   // optional selection list into burst 0 (re-classification), else nullptr
    const LaunchBurst *bursts;
    uint32_t nbursts;      // 1 .. kMaxBursts
    int mode;              // 16 / 48: receive records of that size; 0: tx checksum generate
    DevTable table;
    unsigned long long *counters;
    uint32_t max_blocks;   // grid cap (grid-stride over 64-frame slices)
    uint32_t stride64;     // nonzero: frame i of a burst at slot slot0 + i * stride64 (no off64[])
    uint8_t *pay_arena;    // non-null (with pay_msgs): the payload hand-off fused in (one burst,
    rxg_payload_msg *pay_msgs;  //   record kind 8 / 16 / 48; rxg_rx_burst_payload_dev)
    // mirror patches the launch applies before its first probe, in place of a patch launch
    // before it (rxg_host.cpp launch_bursts; the list in device memory, kLaunchPatchMax at most)
    const MirrorPatch *ipatch;
    uint32_t nipatch;
};

struct LaunchSynth {
    uint8_t *frames;
    uint32_t *off64;
    uint16_t *len;
    uint32_t *flow;
    uint64_t seed;
    uint64_t arena_bytes;
    uint32_t n, nflows, dst_ip, dport, mix, len_a;
};

struct LaunchPayload {
    const uint8_t *frames;
    const uint32_t *off64;
    const uint16_t *len;
    const uint8_t *recs;   // the burst's records (rxg_rec16 / rxg_rec48, `stride` bytes apart)
    uint32_t stride;
    uint32_t n;
    rxg_payload_msg *msgs;
    uint8_t *arena;
    uint64_t arena_cap;
    unsigned long long *status;       // payload_blocks(n) look-back words (any content)
    unsigned long long *ticket;       // workgroup ticket counter, kept across launches
    unsigned long long ticket_base;   // its value before this launch
    unsigned long long *used;         // 1 entry
    uint32_t epoch;                   // 1 .. 2^30-1, new for every launch on `status`
};

hipError_t launch_rx(const LaunchRx &L, hipStream_t st);

// Latency mode (rxg_server_*): a persistent set of workgroups that classifies one burst after
// another.  The host posts a request in a mailbox of fine-grained (coherent) host memory and
// spins on its `done`; workgroup 0 polls the mailbox and hands each request to the others
// through `SrvCtl` in device memory.  No launch and no stream synchronisation per burst.
struct SrvReq {
    const uint8_t *frames;   // device-visible: HBM or mapped host memory
    const uint32_t *off64;
    const uint16_t *len;
    uint8_t *out;            // records of the server's kind
    uint32_t n;
    uint32_t flags;          // kSrvInlineDesc: the descriptors are in the mailbox (SrvMbox::ioff / ilen);
                             // kSrvLarge: a frame over 64 bytes (host bursts)
    DevTable table;          // the mirror as of the post
};
// Host bursts of up to kSrvInline frames carry their descriptors in the mailbox, on the lines
// the server's poll reads with the request: its frame loads then wait for no descriptor load
// (one dependent device-memory trip less per served burst).
constexpr uint32_t kSrvInline = 32;
constexpr uint32_t kSrvInlineDesc = 1u;
// A host burst holding a frame over 64 bytes: a request of 3..gridDim slices then runs one
// slice per workgroup, each shared by the workgroup's four waves (rx_body, HISTORY.md §9.R4).
constexpr uint32_t kSrvLarge = 2u;
// Device memory written through the BAR (large-BAR GPUs, whole lines per post) or coherent
// host memory; `done` / `exited` are read from the server's return block (host memory, may
// be a second SrvMbox).  The first 320 bytes (words 0-39) are what the host writes and the
// server polls, read whole by one wave instruction (40 lanes x 8 bytes): a request is taken
// when seq is new and `check` is srv_check of seq, the request words and, for a request with
// kSrvInlineDesc, the inline descriptor words 16-39.  Write-combined stores reach the device
// as whole lines or in parts, in any order between lines until the host's fence: the check
// word is what makes a snapshot holding words of two requests fail (it is then polled again),
// not the order of the stores.  The server's words are on a line of their own.
struct alignas(128) SrvMbox {
    unsigned long long seq;       // host: number of the request posted
    SrvReq req;
    unsigned long long check;     // host: srv_check(seq, req, ioff, ilen)
    unsigned long long stop;      // host: nonzero = exit
    unsigned long long hpad[2];
    uint32_t ioff[kSrvInline];    // words 16-31: off64 of an inline request's frames
    uint16_t ilen[kSrvInline];    // words 32-39: their lengths
    alignas(128) unsigned long long done;  // server: number of the last request finished
    unsigned long long exited;    // server: nonzero once the kernel has left its loop
};
constexpr int kSrvPollWords = 40;  // words 0-39: the request and its inline descriptors
static_assert(sizeof(SrvReq) == 88, "mailbox layout");
static_assert(offsetof(SrvMbox, check) == 96 && offsetof(SrvMbox, stop) == 104 && offsetof(SrvMbox, ioff) == 128 &&
                  offsetof(SrvMbox, ilen) == 256 && offsetof(SrvMbox, done) == 384,
              "mailbox layout");
// Word i of the mailbox (0 = seq, 1-11 = the request, 16-39 = inline descriptors) mixed with
// its position; the check word is the XOR of the mixed words (a splitmix64 finaliser: any mix
// of old and new words changes it but with probability 2^-64).
__host__ __device__ inline unsigned long long srv_mix(unsigned i, unsigned long long w)
{
    unsigned long long z = w + (unsigned long long)(i + 1u) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// desc: words 16-39 of an inline request (nullptr otherwise)
inline unsigned long long srv_check(unsigned long long seq, const SrvReq &r, const unsigned long long *desc)
{
    unsigned long long w[sizeof(SrvReq) / 8];
    __builtin_memcpy(w, &r, sizeof w);
    unsigned long long h = srv_mix(0u, seq);
    for (unsigned i = 0; i < sizeof(SrvReq) / 8; ++i) h ^= srv_mix(i + 1u, w[i]);
    if (desc)
        for (unsigned i = 16; i < (unsigned)kSrvPollWords; ++i) h ^= srv_mix(i, desc[i - 16]);
    return h;
}
struct SrvCtl {                   // device memory
    unsigned long long go;        // number << 16 | participants of the request the workgroups run
                                  // (kSrvStop: exit); the host sets done << 16 before a launch
    unsigned int fin;             // participants finished with the current request (the last
                                  // one resets it to 0 before publishing `done`)
    unsigned int pad;
    SrvReq req;                   // the current request, read by its participants only
};
constexpr unsigned long long kSrvStop = ~0ull;
struct LaunchServer {
    SrvMbox *mbox;                  // host-written words (host or device memory)
    SrvMbox *ret;                   // done / exited (host memory); nullptr = mbox
    SrvCtl *ctl;
    unsigned long long *counters;
    unsigned long long idle_ticks;  // wall-clock ticks without a request before the kernel exits
    uint32_t blocks;
    int mode;                       // record kind 8 / 16 / 48
};
hipError_t launch_server(const LaunchServer &L, hipStream_t st);
// rxg_payload.hip: gather of the burst's candidate payloads (one launch + a memset)
hipError_t launch_payload(const LaunchPayload &P, hipStream_t st, uint32_t *tickets_used);
uint32_t payload_blocks(uint32_t n);
// resident 256-thread workgroups per CU of the production kernel of `mode` (by_ref: the
// by-reference payload hand-off's, whose record ring also stages the messages)
int rx_blocks_per_cu(int mode, bool by_ref = false);
hipError_t launch_synth(const LaunchSynth &L, hipStream_t st);
// off[i] = slot0 + i * stride64, i < n (a fixed-stride burst's offsets as a list)
hipError_t launch_strided_offsets(uint32_t *off, uint32_t n, uint32_t slot0, uint32_t stride64, hipStream_t st);
// rxg_mirror.h patches (n of them, host-visible memory) applied to the device mirror tables
// Replay counter corrections (two's complement: a negative delta wraps the uint64 sum)
struct CounterDelta {
    int64_t v[RXG_NCOUNTERS];
};
hipError_t launch_counters_add(unsigned long long *row, const CounterDelta &d, hipStream_t st);

// crow != nullptr: the launch also adds *delta to that counter row (the replay's pending
// corrections, rxg_replay.cpp), saving their own launch
hipError_t launch_mirror_patch(const MirrorPatch *p, uint32_t n, uint4 *buckets, int32_t *listen, uint32_t *arp,
                               hipStream_t st, unsigned long long *crow = nullptr, const CounterDelta *delta = nullptr);

}  // namespace rxg
