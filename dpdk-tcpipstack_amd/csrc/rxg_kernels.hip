// rxg_kernels.hip — the product kernels of librxg.so (gfx950): the receive / tx-checksum
// kernels instantiated from rxg_rx.h (one per record kind, descriptor form, burst count and
// prefetch depth), the latency-mode server, the synthetic-frame generator, the mirror patch
// and the counter corrections, and their launch wrappers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <type_traits>

#include "rxg_common.h"
#include "rxg_kernels.h"
#include "rxg_mirror.h"

#include "rxg_rx_server.h"

namespace rxg {

// ------------------------------------------------------------------ synthetic frames ---
struct SynthArgs {
    uint8_t *frames;
    uint32_t *off64;
    uint16_t *len;
    uint32_t *flow;
    uint64_t seed;
    uint64_t nchunks;   // 16-byte chunks of the arena
    uint32_t n;
    uint32_t nflows;
    uint32_t dst_ip;    // host order
    uint32_t dport;
    uint32_t mix;
    uint32_t len_a;
    uint32_t slots_a;   // 64-byte slots per frame (mix 0)
};

__device__ __forceinline__ uint8_t synth_hdr_byte(int i, uint32_t frame, uint32_t flow, uint32_t L,
                                                  const SynthArgs &s, uint32_t seq, uint32_t ack)
{
    const uint32_t tl = L - 14u;
    const uint32_t sport = 1024u + flow % 64511u;
    switch (i) {
    case 0: return 0x02; case 1: return 0x00; case 2: return 0xC0; case 3: return 0xA8;
    case 4: return 0x4E; case 5: return 0x02;                         // dst MAC
    case 6: return 0x02; case 7: return 0x00; case 8: return 0x0A;
    case 9: return (uint8_t)(flow >> 16); case 10: return (uint8_t)(flow >> 8);
    case 11: return (uint8_t)flow;                                    // src MAC
    case 12: return 0x08; case 13: return 0x00;                       // IPv4
    case 14: return 0x45; case 15: return 0x00;
    case 16: return (uint8_t)(tl >> 8); case 17: return (uint8_t)tl;
    case 18: return (uint8_t)(frame >> 8); case 19: return (uint8_t)frame;
    case 20: return 0x40; case 21: return 0x00;                       // DF
    case 22: return 64; case 23: return RXG_IPPROTO_TCP;
    case 24: case 25: return 0;                                       // filled by tx kernel
    case 26: return 10; case 27: return (uint8_t)(flow >> 16);
    case 28: return (uint8_t)(flow >> 8); case 29: return (uint8_t)flow;
    case 30: return (uint8_t)(s.dst_ip >> 24); case 31: return (uint8_t)(s.dst_ip >> 16);
    case 32: return (uint8_t)(s.dst_ip >> 8); case 33: return (uint8_t)s.dst_ip;
    case 34: return (uint8_t)(sport >> 8); case 35: return (uint8_t)sport;
    case 36: return (uint8_t)(s.dport >> 8); case 37: return (uint8_t)s.dport;
    case 38: return (uint8_t)(seq >> 24); case 39: return (uint8_t)(seq >> 16);
    case 40: return (uint8_t)(seq >> 8); case 41: return (uint8_t)seq;
    case 42: return (uint8_t)(ack >> 24); case 43: return (uint8_t)(ack >> 16);
    case 44: return (uint8_t)(ack >> 8); case 45: return (uint8_t)ack;
    case 46: return 0x50; case 47: return RXG_TCP_FLAG_ACK;
    case 48: return 0xFF; case 49: return 0xFF;                       // window
    default: return 0;                                                // cksum, urg
    }
}

__global__ __launch_bounds__(256) void synth_kernel(SynthArgs s)
{
    for (uint64_t t = blockIdx.x * 256ull + threadIdx.x; t < s.nchunks; t += (uint64_t)gridDim.x * 256ull) {
        uint32_t frame, c, L;
        uint64_t frame_slot;
        if (s.mix == 0) {
            const uint64_t cps = (uint64_t)s.slots_a * 4u;
            frame = (uint32_t)(t / cps);
            c = (uint32_t)(t % cps);
            L = s.len_a;
            frame_slot = (uint64_t)frame * s.slots_a;
        } else {
            const uint64_t cpb = (uint64_t)kImixSlotsPerBlock * 4u;
            const uint64_t blk = t / cpb;
            uint32_t rem = (uint32_t)(t % cpb);
            const uint32_t rot = (uint32_t)(splitmix64(s.seed ^ 0xB10Cull ^ blk) % kImixBlock);
            uint32_t slot = 0, pos = 0;
            for (;;) {
                const uint32_t l = imix_len((int)((pos + rot) % kImixBlock));
                const uint32_t chunks = ((l + 63u) / 64u) * 4u;
                if (rem < chunks) { L = l; break; }
                rem -= chunks;
                slot += chunks / 4u;
                ++pos;
            }
            frame = (uint32_t)(blk * kImixBlock + pos);
            c = rem;
            frame_slot = blk * kImixSlotsPerBlock + slot;
        }
        if (frame >= s.n) continue;
        const uint64_t fr = splitmix64(0x5EED0002ull ^ s.seed ^ ((uint64_t)frame << 1));
        const uint32_t flow = (uint32_t)(fr % s.nflows);
        const uint64_t sa = splitmix64(s.seed ^ 0xA5A5ull ^ ((uint64_t)frame << 2));
        const uint32_t seq = (uint32_t)sa, ack = (uint32_t)(sa >> 32);
        if (c == 0) {
            s.off64[frame] = (uint32_t)frame_slot;
            s.len[frame] = (uint16_t)L;
            if (s.flow) s.flow[frame] = flow;
        }
        uint8_t b[16];
        const uint64_t p0 = splitmix64(0x5EED0001ull ^ s.seed ^ ((uint64_t)frame << 12) ^ (2u * c));
        const uint64_t p1 = splitmix64(0x5EED0001ull ^ s.seed ^ ((uint64_t)frame << 12) ^ (2u * c + 1u));
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t bi = c * 16u + (uint32_t)i;
            uint8_t v;
            if (bi >= L) v = 0;
            else if (bi < 54u) v = synth_hdr_byte((int)bi, frame, flow, L, s, seq, ack);
            else v = (uint8_t)((i < 8 ? p0 : p1) >> (8 * (i & 7)));
            b[i] = v;
        }
        uint4 q;
        q.x = b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24);
        q.y = b[4] | (b[5] << 8) | (b[6] << 16) | ((uint32_t)b[7] << 24);
        q.z = b[8] | (b[9] << 8) | (b[10] << 16) | ((uint32_t)b[11] << 24);
        q.w = b[12] | (b[13] << 8) | (b[14] << 16) | ((uint32_t)b[15] << 24);
        *reinterpret_cast<uint4 *>(s.frames + (frame_slot * 64u) + c * 16u) = q;
    }
}

// ------------------------------------------------------------------ launch wrappers ---

// The production kernels, one per (record kind, descriptor form, burst count, depth).
template <int MODE, int DESC>
static void launch_mode(const RxArgs &a, const RxGrid &g, hipStream_t st)
{
    if (g.deep && a.nbursts > 1)
        hipLaunchKernelGGL((rx_kernel<MODE, DESC, true, true>), dim3(g.blocks), dim3(256), 0, st, a);
    else if (g.deep)
        hipLaunchKernelGGL((rx_kernel<MODE, DESC, false, true>), dim3(g.blocks), dim3(256), 0, st, a);
    else if (a.nbursts > 1)
        hipLaunchKernelGGL((rx_kernel<MODE, DESC, true, false>), dim3(g.blocks), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((rx_kernel<MODE, DESC, false, false>), dim3(g.blocks), dim3(256), 0, st, a);
}

// The fused payload hand-off's kernels (one burst; offset list or fixed stride).
template <int MODE, int PAY>
static void launch_pay(const RxArgs &a, const RxGrid &g, bool strided, hipStream_t st)
{
    if (strided)
        hipLaunchKernelGGL((rx_kernel<MODE, kDescStride, false, false, PAY>), dim3(g.blocks), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((rx_kernel<MODE, kDescList, false, false, PAY>), dim3(g.blocks), dim3(256), 0, st, a);
}

hipError_t launch_rx(const LaunchRx &L, hipStream_t st)
{
    RxArgs a;
    RxGrid g;
    const hipError_t e = rx_args(L, a, g);
    if (e != hipSuccess || a.nslices == 0) return e;
    if (L.sel) {  // re-classification of selected frames (rxg_rx_replay), records of 16 B
        hipLaunchKernelGGL((rx_kernel<16, kDescSel, false, false>), dim3(g.blocks), dim3(256), 0, st, a);
        return hipGetLastError();
    }
    const bool strided = L.stride64 != 0u;
    if (L.pay_msgs) {  // the payload hand-off fused in (rxg_rx_burst_payload_dev): one burst
        if (a.nbursts != 1) return hipErrorInvalidValue;
        const bool copy = L.pay_arena != nullptr;  // (NULL: by reference, messages only)
        switch (L.mode) {
        case 8: copy ? launch_pay<8, kPayCopy>(a, g, strided, st) : launch_pay<8, kPayRef>(a, g, strided, st); break;
        case 16: copy ? launch_pay<16, kPayCopy>(a, g, strided, st) : launch_pay<16, kPayRef>(a, g, strided, st); break;
        case 48: copy ? launch_pay<48, kPayCopy>(a, g, strided, st) : launch_pay<48, kPayRef>(a, g, strided, st); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    switch (L.mode) {
    case 8: strided ? launch_mode<8, kDescStride>(a, g, st) : launch_mode<8, kDescList>(a, g, st); break;
    case 16: strided ? launch_mode<16, kDescStride>(a, g, st) : launch_mode<16, kDescList>(a, g, st); break;
    case 48:  // (never two-deep: 48-byte records are the inspection form, not the bulk one)
        if (strided && a.nbursts > 1)
            hipLaunchKernelGGL((rx_kernel<48, kDescStride, true, false>), dim3(g.blocks), dim3(256), 0, st, a);
        else if (strided)
            hipLaunchKernelGGL((rx_kernel<48, kDescStride, false, false>), dim3(g.blocks), dim3(256), 0, st, a);
        else if (a.nbursts > 1)
            hipLaunchKernelGGL((rx_kernel<48, kDescList, true, false>), dim3(g.blocks), dim3(256), 0, st, a);
        else
            hipLaunchKernelGGL((rx_kernel<48, kDescList, false, false>), dim3(g.blocks), dim3(256), 0, st, a);
        break;
    case 0:
        if (strided || a.nbursts > 1) return hipErrorInvalidValue;
        hipLaunchKernelGGL((rx_kernel<0, kDescList, false, false>), dim3(g.blocks), dim3(256), 0, st, a);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_server(const LaunchServer &L, hipStream_t st)
{
    SrvArgs sa{L.mbox, L.ret ? L.ret : L.mbox, L.ctl, L.counters, L.idle_ticks};
    const dim3 g(L.blocks ? L.blocks : 1u), b(256);
    if (g.x > 0xFFFFu) return hipErrorInvalidValue;  // participants travel in 16 bits of SrvCtl::go
    switch (L.mode) {
    case 8: hipLaunchKernelGGL((rx_server<8>), g, b, 0, st, sa); break;
    case 16: hipLaunchKernelGGL((rx_server<16>), g, b, 0, st, sa); break;
    case 48: hipLaunchKernelGGL((rx_server<48>), g, b, 0, st, sa); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// The device words a batch of TCB / ARP mirror writes changed (rxg_mirror.h), one thread per
// patch; the host deduplicated them, so no two threads write the same word.  The patch list
// is read straight from pinned host memory (a few hundred bytes per burst).
__global__ __launch_bounds__(256) void mirror_patch(const MirrorPatch *p, uint32_t n, uint4 *buckets,
                                                    int32_t *listen, uint32_t *arp, unsigned long long *crow,
                                                    CounterDelta d)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (crow != nullptr && i < (uint32_t)RXG_NCOUNTERS && d.v[i] != 0)  // (counters_add's work)
        atomicAdd(crow + i, (unsigned long long)d.v[i]);
    if (i >= n) return;
    const MirrorPatch q = p[i];
    if (q.target == kPatchBucket)
        buckets[q.index] = make_uint4(q.v[0], q.v[1], q.v[2], q.v[3]);
    else if (q.target == kPatchListen)
        listen[q.index] = (int32_t)q.v[0];
    else
        arp[q.index] = q.v[0];
}

hipError_t launch_mirror_patch(const MirrorPatch *p, uint32_t n, uint4 *buckets, int32_t *listen, uint32_t *arp,
                               hipStream_t st, unsigned long long *crow, const CounterDelta *delta)
{
    if (n == 0 && crow == nullptr) return hipSuccess;
    CounterDelta d{};
    if (crow != nullptr) d = *delta;
    hipLaunchKernelGGL(mirror_patch, dim3(std::max(1u, (n + 255u) / 256u)), dim3(256), 0, st, p, n, buckets, listen,
                       arp, crow, d);
    return hipGetLastError();
}

// A fixed-stride burst's offsets as a list (rxg_rx_bursts_strided_dev's bursts, for the
// payload gather and the replay's re-classification, which read offsets through a list).
__global__ __launch_bounds__(256) void strided_offsets(uint32_t *off, uint32_t n, uint32_t slot0, uint32_t stride64)
{
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) off[i] = slot0 + i * stride64;
}

hipError_t launch_strided_offsets(uint32_t *off, uint32_t n, uint32_t slot0, uint32_t stride64, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(strided_offsets, dim3(std::min(1024u, (n + 255u) / 256u)), dim3(256), 0, st, off, n, slot0,
                       stride64);
    return hipGetLastError();
}

// The replay's counter corrections (rxg_rx_replay), added to the host row of the counter
// block in stream order: the values travel as kernel arguments, so the host neither waits
// for nor reads back the device block.
__global__ void counters_add(unsigned long long *row, CounterDelta d)
{
    const int k = (int)threadIdx.x;
    if (k < RXG_NCOUNTERS && d.v[k] != 0) atomicAdd(row + k, (unsigned long long)d.v[k]);
}

hipError_t launch_counters_add(unsigned long long *row, const CounterDelta &d, hipStream_t st)
{
    hipLaunchKernelGGL(counters_add, dim3(1), dim3(64), 0, st, row, d);
    return hipGetLastError();
}

int rx_blocks_per_cu(int mode, bool by_ref)
{
    int n = 0;
    hipError_t e;
    if (by_ref && mode == 8)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, rx_kernel<8, kDescList, false, false, kPayRef>, 256, 0);
    else if (by_ref && mode == 16)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, rx_kernel<16, kDescList, false, false, kPayRef>, 256, 0);
    else if (by_ref && mode == 48)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, rx_kernel<48, kDescList, false, false, kPayRef>, 256, 0);
    else if (mode == 8)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, rx_kernel<8, kDescList, false, false>, 256, 0);
    else if (mode == 16)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, rx_kernel<16, kDescList, false, false>, 256, 0);
    else if (mode == 48)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, rx_kernel<48, kDescList, false, false>, 256, 0);
    else
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, rx_kernel<0, kDescList, false, false>, 256, 0);
    return (e == hipSuccess && n > 0) ? n : 4;
}

hipError_t launch_synth(const LaunchSynth &L, hipStream_t st)
{
    SynthArgs s;
    s.frames = L.frames;
    s.off64 = L.off64;
    s.len = L.len;
    s.flow = L.flow;
    s.seed = L.seed;
    s.nchunks = L.arena_bytes / 16u;
    s.n = L.n;
    s.nflows = L.nflows ? L.nflows : 1u;
    s.dst_ip = L.dst_ip;
    s.dport = L.dport;
    s.mix = L.mix;
    s.len_a = L.len_a;
    s.slots_a = (L.len_a + 63u) / 64u;
    if (s.nchunks == 0) return hipSuccess;
    uint64_t blocks = (s.nchunks + 255u) / 256u;
    if (blocks > 16384u) blocks = 16384u;
    hipLaunchKernelGGL(synth_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, s);
    return hipGetLastError();
}

}  // namespace rxg
