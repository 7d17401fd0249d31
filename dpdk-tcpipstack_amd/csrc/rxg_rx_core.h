// rxg_rx_core.h — the receive kernels' launch arguments, lane helpers, burst cursor and
// the fused payload hand-off's helpers (rxg_rx.h's first part; see rxg_rx.h for the map).
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
    // mirror patches to store before the first probe (LaunchRx::ipatch; never the server's)
    const MirrorPatch *ipatch;
    uint32_t nipatch;
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
// generation's slices into pieces spread over more waves measured slower, HISTORY.md §9.R3.)

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

// The mirror patches a launch carries (LaunchRx::ipatch, in place of a mirror_patch launch
// before it): every workgroup stores all of them before its first table read -- the same
// values to the same words, so none needs another's (no grid-wide order), and each waits
// for its own stores before its waves read the tables.  At most kLaunchPatchMax, no two
// to one word (rxg_host.cpp apply_patches), by contract.
__device__ __forceinline__ void apply_launch_patches(const RxArgs &a)
{
    uint4 *buckets = const_cast<uint4 *>(a.t.buckets);
    int32_t *listen = const_cast<int32_t *>(a.t.listen);
    uint32_t *arp = reinterpret_cast<uint32_t *>(const_cast<uint4 *>(a.t.arp));
    for (uint32_t i = threadIdx.x; i < a.nipatch; i += blockDim.x) {
        const MirrorPatch q = a.ipatch[i];
        if (q.target == kPatchBucket)
            buckets[q.index] = make_uint4(q.v[0], q.v[1], q.v[2], q.v[3]);
        else if (q.target == kPatchListen)
            listen[q.index] = (int32_t)q.v[0];
        else
            arp[q.index] = q.v[0];
    }
    __builtin_amdgcn_s_waitcnt(0);  // the stores acknowledged (vmcnt counts stores on gfx9)
    __syncthreads();
}

// ------------------------------------------------- fused payload hand-off (PAY) ---
// The PAY template argument: no hand-off, the hand-off with its payload lines copied to the
// arena, or by reference (messages only; rxg_payload_slots.arena NULL).
enum : int { kPayNone = 0, kPayCopy = 1, kPayRef = 2 };

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
// the frame's own bytes (the arena has the pool's geometry), or zeros.
__device__ __forceinline__ uint4 pay_msg_of(uint32_t off, uint32_t span)
{
    const uint32_t dl = span & 0xFFFFu;
    const uint64_t ao = span ? (uint64_t)off * 64u + (span >> 16) : 0ull;
    return make_uint4((uint32_t)ao, (uint32_t)(ao >> 32), dl,
                      span ? (RXG_PM_GATHERED | (dl >= 1000u ? RXG_PM_REF_OVERSIZE : 0u)) : 0u);
}

// The copy form's message store, f: the frame's index in the burst.  One 16-byte
// non-temporal store per lane as the frame is classified (staged in LDS with the records
// instead, the fused C3 launch measured the same and C4 1.5 % faster).  The
// by-reference form stages its messages in the record ring (RecRing, MSG).
__device__ __forceinline__ void pay_msg(const RxArgs &a, uint32_t f, bool valid, uint32_t off, uint32_t span)
{
    if (!valid) return;
    const uint4 m = pay_msg_of(off, span);
    const uint32_t q[4] = {m.x, m.y, m.z, m.w};
    nt_store16(reinterpret_cast<uint8_t *>(a.pay_msgs + f), q);
}

// A frame of <= 64 bytes owned by one lane (the all-small path after its transpose): its one
// line, as loaded, when it carries a payload.
__device__ __forceinline__ void pay_line_small(const RxArgs &a, uint32_t off, uint32_t span, const uint32_t (&q)[4][4])
{
    if (span == 0u) return;
    uint8_t *dst = a.pay_arena + (size_t)off * 64u;
#pragma unroll
    for (int k = 0; k < 4; ++k) pay_store16<true>(dst + 16 * k, q[k]);
}

}  // namespace rxg
