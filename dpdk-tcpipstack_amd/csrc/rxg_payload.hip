// rxg_payload.hip — payload hand-off on the device.
//
// The reference copies every in-order segment's payload out of its mbuf into a 1500-byte
// mempool message for the socket ring: tcp_established -> PushData (tcp_windows.c:341-358)
// -> AdjustPair (:42-110) -> PushDataInQueue (:112-136) -> GetData (:138-186), whose
// memcpy reads `Length` bytes at frame + 34 + tcp_len (:164-172; the IP header is taken
// as 20 bytes whatever the IHL, like the parse).  rxg does that copy for a whole burst
// after it (rxg_rx_burst_payload_dev fuses it into the burst instead, rxg_rx_core.h):
//
//   pg_gather  ONE launch, 1 024 frames per workgroup: each workgroup sums its candidates'
//              arena space (each payload rounded up to 16 bytes so that every message starts
//              16-byte aligned), finds its offset by a decoupled look-back over the
//              workgroups before it (virtual workgroup ids from an atomic ticket, so every
//              workgroup it waits for is running; each status word is an epoch-tagged
//              64-bit {flag, value} granule, the data being its own flag), writes the
//              message descriptors, then each wave copies its 64 frames' payloads one
//              16-byte destination chunk per lane (source misaligned by 54 mod 16 for a
//              20-byte TCP header: 16-byte loads + a cross-lane byte funnel shift;
//              destination 16-byte aligned, the tail of the last chunk zeroed).  The
//              copy's first two sets of rounds are loaded before the look-back (their
//              sources and in-workgroup layout do not depend on it), so its latency
//              overlaps them.
//
// A candidate is every TCP segment of the burst (verdict DISPATCH, RST_NOPCB or
// RST_LISTEN_NONSYN: the replay may re-classify the latter two to a DISPATCH when a
// handler creates their TCB inside the burst) with datalen > 0 and the payload inside the
// frame.  The device does not decide whether the window takes the segment:
// rxg_payload_take does, at replay time, against the receive-window mirror
// (rxg_replay.cpp), so gathering a segment that is never taken only costs its copy.
//
// Roofline: HBM, algorithmic bytes per frame = 2 x payload (read + write) + 16 (record)
// + 16 (message descriptor).
#include "rxg_kernels.h"

namespace rxg {
namespace {

constexpr int kPgThreads = 256;  // status words are sized for 256-frame workgroups (payload_blocks)
// 1 024 frames (16 waves) per workgroup, 2 copy rounds per set (80 VGPRs, 6 waves per SIMD);
// the other sizes and depths measured slower (HISTORY.md §5, "pg_gather")
constexpr int kPgFrames = 1024;
constexpr int kPgRounds = 2;
constexpr uint32_t kSpinLimit = 1u << 22;

typedef __attribute__((address_space(1))) unsigned long long gu64;

struct PgArgs {
    const uint8_t *frames;
    const uint32_t *off64;
    const uint16_t *len;
    const uint8_t *recs;
    uint32_t stride;
    uint32_t n;
    rxg_payload_msg *msgs;
    uint8_t *arena;
    uint64_t arena_cap;
    unsigned long long *status;  // per virtual workgroup: epoch << 34 | flag << 32 | value/16
    unsigned long long *ticket;  // virtual workgroup ids, counting across launches
    unsigned long long ticket_base;
    unsigned long long *used;    // 1 entry: arena bytes the burst needs (~0: look-back timed out)
    uint32_t epoch;              // 30 bits, never 0
    uint32_t nblocks;
};

struct Cand {
    uint64_t src;  // byte offset of the payload in frames
    uint32_t len;  // 0: not a candidate
    uint32_t flags;
};


__device__ __forceinline__ Cand candidate(const PgArgs &a, uint32_t i)
{
    Cand c{0ull, 0u, 0u};
    if (i >= a.n) return c;
    // the record, the descriptor and the length are loaded together (one HBM round trip
    // before the frame's header word, not two)
    // rxg_rec16: x tcb_idx | y checksums | z verdict, state<<8, tcp_flags<<16, flags<<24 | w datalen
    // rxg_rec8 (stride 8): w0 verdict at 24 | w1 flags at 8, datalen + 128 at 14
    uint32_t verdict, rflags;
    int32_t datalen;
    uint32_t off, flen;
    if (a.stride == 8u) {
        const uint2 r = *reinterpret_cast<const uint2 *>(a.recs + (size_t)i * 8u);
        off = a.off64[i];
        flen = a.len[i];
        asm volatile("" ::"v"(off), "v"(flen));
        verdict = (r.x >> 24) & 7u;
        rflags = (r.y >> 8) & 0x3Fu;
        datalen = (int32_t)((r.y >> 14) & 0x1FFFFu) - 128;
    } else {
        const uint4 r = *reinterpret_cast<const uint4 *>(a.recs + (size_t)i * a.stride);
        off = a.off64[i];
        flen = a.len[i];
        asm volatile("" ::"v"(off), "v"(flen));  // keeps the two loads above the branch
        verdict = r.z & 0xFFu;
        rflags = r.z >> 24;
        datalen = (int32_t)r.w;
    }
    if (verdict > RXG_V_RST_LISTEN_NONSYN || datalen <= 0 || (rflags & RXG_F_TRUNC)) return c;
    const uint64_t base = (uint64_t)off * 64u;
    // bytes 44..47 of the frame (>= 54 bytes: not RXG_F_TRUNC); data_off is byte 46
    const uint32_t dw = *reinterpret_cast<const uint32_t *>(a.frames + base + 44u);
    const uint32_t start = RXG_OFF_TCP + ((dw >> 20) & 0xFu) * 4u;
    if (start + (uint32_t)datalen > flen) return c;
    c.src = base + start;
    c.len = (uint32_t)datalen;
    // GetData asserts (Length - offset) < 1000, its stack buffer's size (tcp_windows.c:170)
    c.flags = RXG_PM_GATHERED | ((uint32_t)datalen >= 1000u ? RXG_PM_REF_OVERSIZE : 0u);
    return c;
}

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v, int lane)
{
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const T o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

__device__ __forceinline__ uint4 bperm16(uint4 v, int src_lane)
{
    uint4 r;
    r.x = (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v.x);
    r.y = (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v.y);
    r.z = (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v.z);
    r.w = (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v.w);
    return r;
}

// bytes [sh, sh + 16) of the 32-byte string lo || hi
__device__ __forceinline__ uint4 funnel16(uint4 lo, uint4 hi, uint32_t sh)
{
    const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    const uint32_t ds = sh >> 2, bs = sh & 3u;
    uint32_t s[5];
#pragma unroll
    for (int t = 0; t < 5; ++t)
        s[t] = ds == 0 ? w[t] : ds == 1 ? w[t + 1] : ds == 2 ? w[t + 2] : w[t + 3];
    uint4 r;
    r.x = __builtin_amdgcn_alignbyte(s[1], s[0], bs);
    r.y = __builtin_amdgcn_alignbyte(s[2], s[1], bs);
    r.z = __builtin_amdgcn_alignbyte(s[3], s[2], bs);
    r.w = __builtin_amdgcn_alignbyte(s[4], s[3], bs);
    return r;
}

__device__ __forceinline__ uint32_t keep_bytes(uint32_t v, int nb)
{
    return nb >= 4 ? v : nb <= 0 ? 0u : (v & ((1u << (8 * nb)) - 1u));
}

// Copy phase of pg_copy: lane-per-chunk.  A wave takes its 256 frames in batches of 64;
// the batch's payloads (compacted, in packet order) form one run of T destination chunks
// of 16 bytes, and round r gives lane l chunk 64r + l.  The payload a chunk belongs to is
// found without a search: the payloads' first chunks of the round are marked in a 64-entry
// LDS array, a ballot turns the marks into a mask, and a popcount below the lane counts
// the payloads started so far.  kU rounds are in flight per iteration.  Destination chunk
// k of a payload = source bytes [16k + sh, 16k + sh + 16) from the 16-byte-aligned source
// chunks k and k + 1; chunk k + 1 comes from the next lane when that lane copies the same
// payload, else from a load of its own.
struct WaveCopy {
    uint64_t src[64];   // compacted payloads of the batch: source byte offset in frames,
    uint64_t dst[64];   // destination byte offset in the arena,
    uint32_t start[64]; // first destination chunk within the batch's run,
    uint32_t len[64];   // bytes
    uint32_t head[64 * kPgRounds];
};

template <bool NT>
__device__ __forceinline__ uint4 ldp(const uint8_t *p)
{
    if constexpr (NT) {
        typedef unsigned int v4 __attribute__((ext_vector_type(4)));
        const v4 v = __builtin_nontemporal_load(reinterpret_cast<const v4 *>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return *reinterpret_cast<const uint4 *>(p);
    }
}

template <bool NT>
__device__ __forceinline__ void stp(uint8_t *p, uint4 o)
{
    if constexpr (NT) {
        typedef unsigned int v4 __attribute__((ext_vector_type(4)));
        v4 v;
        v.x = o.x; v.y = o.y; v.z = o.z; v.w = o.w;
        __builtin_nontemporal_store(v, reinterpret_cast<v4 *>(p));
    } else {
        *reinterpret_cast<uint4 *>(p) = o;
    }
}

// One round of lanes in flight: lane's destination chunk k of compacted payload p, its
// source chunk k, and chunk k + 1 when the next lane does not supply it (E).
struct Round {
    uint4 A, E;
    uint32_t p, k;
    bool act, own;
};

template <int kU, bool NT>
__device__ __forceinline__ void issue_rounds(const PgArgs &a, WaveCopy &W, uint32_t r0, uint32_t T, bool valid,
                                             uint32_t start, int lane, unsigned long long le, Round (&R)[kU])
{
#pragma unroll
    for (int u = 0; u < kU; ++u) W.head[64 * u + lane] = 0u;
    __builtin_amdgcn_wave_barrier();
    if (valid && start >= r0 && start < r0 + 64u * kU) W.head[start - r0] = 1u;
    __builtin_amdgcn_wave_barrier();
    const int nl = lane == 63 ? 63 : lane + 1;
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const uint32_t base = r0 + 64u * u;
        const unsigned long long mask = __ballot(W.head[64 * u + lane] != 0u);
        const uint32_t before = (uint32_t)__popcll(__ballot(valid && start < base));
        const uint32_t idx = base + (uint32_t)lane;
        R[u].act = idx < T;
        R[u].p = R[u].act ? before + (uint32_t)__popcll(mask & le) - 1u : 0u;
        R[u].k = R[u].act ? idx - W.start[R[u].p] : 0u;
        const uint64_t s = W.src[R[u].p];
        const uint8_t *s0 = a.frames + (s & ~15ull);
        R[u].A = ldp<NT>(s0 + 16u * R[u].k);
        const uint32_t pn = (uint32_t)__builtin_amdgcn_ds_bpermute(nl << 2, (int)R[u].p);
        R[u].own = lane == 63 || idx + 1u >= T || pn != R[u].p;
        const uint32_t sh = (uint32_t)(s & 15u);
        R[u].E = make_uint4(0u, 0u, 0u, 0u);
        if (R[u].act && sh && R[u].own && R[u].k + 1u < ((sh + W.len[R[u].p] + 15u) >> 4))
            R[u].E = ldp<NT>(s0 + 16u * (R[u].k + 1u));
    }
    __builtin_amdgcn_wave_barrier();  // head[] is rewritten by the next issue
}

// The stores of kU rounds: the workgroup's arena base is known only after the look-back, so
// W.dst holds offsets relative to it; payloads past the arena capacity were loaded but are
// not stored (they get no message either)
template <int kU, bool NT>
__device__ __forceinline__ void store_rounds_at(const PgArgs &a, const WaveCopy &W, int lane, const Round (&R)[kU],
                                                uint64_t base)
{
    const int nl = lane == 63 ? 63 : lane + 1;
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const uint4 N0 = bperm16(R[u].A, nl);
        const uint4 N = R[u].own ? R[u].E : N0;
        const uint32_t L = W.len[R[u].p];
        const uint64_t d = base + W.dst[R[u].p];
        if (R[u].act && d + 16ull * ((L + 15u) >> 4) <= a.arena_cap) {
            const uint64_t s = W.src[R[u].p];
            const uint32_t sh = (uint32_t)(s & 15u);
            uint4 o = sh ? funnel16(R[u].A, N, sh) : R[u].A;
            const int vb = (int)L - (int)(16u * R[u].k);
            if (vb < 16) {
                o.x = keep_bytes(o.x, vb);
                o.y = keep_bytes(o.y, vb - 4);
                o.z = keep_bytes(o.z, vb - 8);
                o.w = keep_bytes(o.w, vb - 12);
            }
            stp<NT>(a.arena + d + 16u * R[u].k, o);
        }
    }
}

// The wave's 64 frames (lane = frame; L = 0: nothing to copy), with the first two sets of kU
// rounds' loads issued before the workgroup's arena offset is known: `finish` runs the
// look-back (and the workgroup barrier every wave must reach) while those loads are in
// flight, and returns the workgroup's arena base.  `rel`: this lane's payload offset relative
// to that base.  Software-pipelined: the loads of the next kU rounds are issued before the
// current rounds are stored.
template <int kU, bool NT, typename F>
__device__ __forceinline__ void copy_batch_pre(const PgArgs &a, WaveCopy &W, uint64_t src, uint64_t rel, uint32_t L,
                                               int lane, F finish)
{
    const bool valid = L != 0u;
    const unsigned long long vm = __ballot(valid);
    if (vm == 0ull) {
        (void)finish();
        return;
    }
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(vm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)vm, 0u));
    const uint32_t nch = valid ? (L + 15u) >> 4 : 0u;
    const uint32_t incl = wave_incl_scan(nch, lane);
    const uint32_t start = incl - nch;
    const uint32_t T = (uint32_t)__shfl(incl, 63, 64);
    if (valid) {
        W.src[rank] = src;
        W.dst[rank] = rel;
        W.start[rank] = start;
        W.len[rank] = L;
    }
    __builtin_amdgcn_wave_barrier();
    const unsigned long long le = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
    constexpr uint32_t kStep = 64u * kU;
    Round X[kU], Y[kU];
    issue_rounds<kU, NT>(a, W, 0u, T, valid, start, lane, le, X);
    // both sets in flight across the look-back
    bool haveY = kStep < T;
    if (haveY) issue_rounds<kU, NT>(a, W, kStep, T, valid, start, lane, le, Y);
    const uint64_t base = finish();
    uint32_t r0 = 0;
    for (;;) {
        store_rounds_at<kU, NT>(a, W, lane, X, base);
        if (!haveY) break;
        r0 += kStep;
        const bool more = r0 + kStep < T;
        if (more) issue_rounds<kU, NT>(a, W, r0 + kStep, T, valid, start, lane, le, X);
        store_rounds_at<kU, NT>(a, W, lane, Y, base);
        if (!more) break;
        r0 += kStep;
        haveY = r0 + kStep < T;
        if (haveY) issue_rounds<kU, NT>(a, W, r0 + kStep, T, valid, start, lane, le, Y);
    }
    __builtin_amdgcn_wave_barrier();  // W is rewritten by the next batch
}

// status word flags
constexpr uint32_t kAgg = 1u, kIncl = 2u;

__device__ __forceinline__ unsigned long long status_word(uint32_t epoch, uint32_t flag, uint32_t v16)
{
    return ((unsigned long long)epoch << 34) | ((unsigned long long)flag << 32) | v16;
}

// Wave 0 of workgroup vb: the exclusive prefix (16-byte units) of the workgroups before it.
// Each poll covers 256 predecessors: lane l reads workgroups j - l - 64q (q < 4), distance
// d = l + 64q.  Every word up to the nearest published inclusive prefix must be published
// (aggregate or inclusive), else the wave polls again.
__device__ __forceinline__ uint32_t look_back(const PgArgs &a, uint32_t vb, int lane, bool &timed_out)
{
    constexpr int kQ = 4;
    uint32_t excl = 0;
    int64_t j = (int64_t)vb - 1;
    uint32_t spins = 0;
    while (j >= 0) {
        unsigned long long wd[kQ];
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const int64_t idx = j - lane - 64 * q;
            wd[q] = status_word(a.epoch, kIncl, 0u);  // before workgroup 0
            if (idx >= 0)
                wd[q] = __hip_atomic_load((gu64 *)(a.status + idx), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        int first = 64 * kQ;  // distance of the nearest inclusive prefix
        uint32_t flag[kQ];
#pragma unroll
        for (int q = kQ - 1; q >= 0; --q) {
            flag[q] = (uint32_t)(wd[q] >> 34) == a.epoch ? (uint32_t)(wd[q] >> 32) & 3u : 0u;
            const unsigned long long im = __ballot(flag[q] == kIncl);
            if (im) first = 64 * q + __builtin_ctzll(im);
        }
        bool missing = false;
        uint32_t v = 0;
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const bool need = lane + 64 * q <= first;
            missing |= need && flag[q] == 0u;
            v += need ? (uint32_t)wd[q] : 0u;
        }
        if (__ballot(missing)) {
            if (++spins > kSpinLimit) {
                timed_out = true;
                return 0u;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
        excl += v;
        if (first < 64 * kQ) break;
        j -= 64 * kQ;
    }
    return excl;
}

// One thread per frame, kPgFrames frames per workgroup; virtual workgroup ids from an atomic
// ticket (dispatch-order independent): the workgroup publishes its aggregate, issues its first
// copy rounds, then wave 0 looks back while they are in flight.
__global__ __launch_bounds__(kPgFrames) void pg_gather(PgArgs a)
{
    __shared__ uint32_t s_vb, s_excl;
    __shared__ uint32_t s_w[kPgFrames / 64];
    __shared__ WaveCopy s_wc[kPgFrames / 64];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) s_vb = (uint32_t)(atomicAdd(a.ticket, 1ull) - a.ticket_base);
    __syncthreads();
    const uint32_t vb = s_vb;
    const uint32_t i0 = vb * (uint32_t)kPgFrames + (uint32_t)t;

    const Cand c = candidate(a, i0);
    const uint32_t mine = (c.len + 15u) >> 4;
    const uint32_t incl = wave_incl_scan(mine, lane);
    if (lane == 63) s_w[w] = incl;
    __syncthreads();
    uint32_t agg = 0, wex = 0;
#pragma unroll
    for (int k = 0; k < kPgFrames / 64; ++k) {
        agg += s_w[k];
        wex += k < w ? s_w[k] : 0u;
    }
    if (w == 0 && lane == 0)
        __hip_atomic_store((gu64 *)(a.status + vb), status_word(a.epoch, vb ? kAgg : kIncl, agg),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t rel = ((uint64_t)wex + incl - mine) * 16ull;
    auto finish = [&]() -> uint64_t {
        if (w == 0) {
            bool timed_out = false;
            const uint32_t excl = vb ? look_back(a, vb, lane, timed_out) : 0u;
            if (lane == 0) {
                if (vb)
                    __hip_atomic_store((gu64 *)(a.status + vb), status_word(a.epoch, kIncl, excl + agg),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (timed_out) atomicMax(a.used, ~0ull);
                else if (vb == a.nblocks - 1) atomicMax(a.used, (unsigned long long)(excl + agg) * 16ull);
                s_excl = excl;
            }
        }
        __syncthreads();
        const uint64_t base = (uint64_t)s_excl * 16ull;
        const uint64_t off = base + rel;
        const uint64_t r = 16ull * ((c.len + 15u) >> 4);
        const bool fits = c.len != 0u && off + r <= a.arena_cap;
        if (i0 < a.n) {
            rxg_payload_msg m;
            m.arena_off = fits ? off : 0ull;
            m.len = fits ? c.len : 0u;
            m.flags = fits ? c.flags : 0u;
            a.msgs[i0] = m;
        }
        return base;
    };
    copy_batch_pre<kPgRounds, true>(a, s_wc[w], c.src, rel, c.len, lane, finish);
}

}  // namespace

// status words the launch may use (sized for the smallest workgroup)
uint32_t payload_blocks(uint32_t n) { return (n + kPgThreads - 1) / kPgThreads; }

hipError_t launch_payload(const LaunchPayload &P, hipStream_t st, uint32_t *launched)
{
    PgArgs a;
    a.frames = P.frames;
    a.off64 = P.off64;
    a.len = P.len;
    a.recs = P.recs;
    a.stride = P.stride;
    a.n = P.n;
    a.msgs = P.msgs;
    a.arena = P.arena;
    a.arena_cap = P.arena_cap;
    a.status = P.status;
    a.ticket = P.ticket;
    a.ticket_base = P.ticket_base;
    a.used = P.used;
    a.epoch = P.epoch;
    *launched = 0;
    hipError_t e = hipMemsetAsync(P.used, 0, sizeof(unsigned long long), st);
    if (e != hipSuccess || P.n == 0) return e;
    a.nblocks = (P.n + kPgFrames - 1) / kPgFrames;
    hipLaunchKernelGGL(pg_gather, dim3(a.nblocks), dim3(kPgFrames), 0, st, a);
    *launched = a.nblocks;
    return hipGetLastError();
}

}  // namespace rxg
