// rxg_payload.hip — payload hand-off on the device.
//
// The reference copies every in-order segment's payload out of its mbuf into a 1500-byte
// mempool message for the socket ring: tcp_established -> PushData (tcp_windows.c:341-358)
// -> AdjustPair (:42-110) -> PushDataInQueue (:112-136) -> GetData (:138-186), whose
// memcpy reads `Length` bytes at frame + 34 + tcp_len (:164-172; the IP header is taken
// as 20 bytes whatever the IHL, like the parse).  rxg does that copy for a whole burst in
// three launches:
//
//   pg_sizes   per 1024-frame block: the bytes of its candidate payloads (each rounded up
//              to 16 so that every message starts 16-byte aligned in the arena);
//   pg_scan    one workgroup: exclusive scan of the block totals (= block offsets);
//   pg_copy    per block: in-block scan -> per-frame message descriptors, then 16-lane
//              groups copy the payloads (source misaligned by 54 mod 16 for a 20-byte TCP
//              header: 16-byte loads + a cross-lane byte funnel shift; destination 16-byte
//              aligned, the tail of the last chunk zeroed).
//
// A candidate is every TCP segment of the burst (verdict DISPATCH, RST_NOPCB or
// RST_LISTEN_NONSYN: the replay may re-classify the latter two to a DISPATCH when a
// handler creates their TCB inside the burst) with datalen > 0 and the payload inside the
// frame.  The device does not decide whether the window takes the segment:
// rxg_payload_take does, at replay time, against the receive-window mirror
// (rxg_host.cpp), so gathering a segment that is never taken only costs its copy.
//
// Roofline: HBM, algorithmic bytes per frame = 2 x payload (read + write) + 16 (record)
// + 16 (message descriptor).
#include "rxg_kernels.h"

namespace rxg {
namespace {

constexpr int kPgThreads = 256;
constexpr int kPgPerThread = 4;
constexpr int kPgPerBlock = kPgThreads * kPgPerThread;  // frames per block
constexpr int kG = 16;                                  // lanes per payload in the copy
constexpr int kU = 4;                                   // 16-byte chunks per lane per round
constexpr int kScanThreads = 1024;

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
    unsigned long long *block_off;  // nblocks entries: totals, then (pg_scan) offsets
    unsigned long long *used;       // 1 entry: arena bytes the burst needs
    uint32_t nblocks;
};

struct Cand {
    uint64_t src;  // byte offset of the payload in frames
    uint32_t len;  // 0: not a candidate
    uint32_t flags;
};

__device__ __forceinline__ uint64_t round16(uint32_t x) { return ((uint64_t)x + 15u) & ~15ull; }

__device__ __forceinline__ Cand candidate(const PgArgs &a, uint32_t i)
{
    Cand c{0ull, 0u, 0u};
    if (i >= a.n) return c;
    // rxg_rec16: x tcb_idx | y checksums | z verdict, state<<8, tcp_flags<<16, flags<<24 | w datalen
    const uint4 r = *reinterpret_cast<const uint4 *>(a.recs + (size_t)i * a.stride);
    const uint32_t verdict = r.z & 0xFFu, rflags = r.z >> 24;
    const int32_t datalen = (int32_t)r.w;
    if (verdict > RXG_V_RST_LISTEN_NONSYN || datalen <= 0 || (rflags & RXG_F_TRUNC)) return c;
    const uint64_t base = (uint64_t)a.off64[i] * 64u;
    // bytes 44..47 of the frame (>= 54 bytes: not RXG_F_TRUNC); data_off is byte 46
    const uint32_t dw = *reinterpret_cast<const uint32_t *>(a.frames + base + 44u);
    const uint32_t start = RXG_OFF_TCP + ((dw >> 20) & 0xFu) * 4u;
    if (start + (uint32_t)datalen > (uint32_t)a.len[i]) return c;
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

__global__ __launch_bounds__(kPgThreads) void pg_sizes(PgArgs a)
{
    __shared__ unsigned long long s_w[kPgThreads / 64];
    const uint32_t base = blockIdx.x * (uint32_t)kPgPerBlock;
    unsigned long long s = 0;
#pragma unroll
    for (int k = 0; k < kPgPerThread; ++k) s += round16(candidate(a, base + threadIdx.x + k * kPgThreads).len);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
    if (lane == 0) s_w[w] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int k = 0; k < kPgThreads / 64; ++k) t += s_w[k];
        a.block_off[blockIdx.x] = t;
    }
}

// One workgroup: block totals -> exclusive block offsets (in place); *used = the sum.
__global__ __launch_bounds__(kScanThreads) void pg_scan(PgArgs a)
{
    __shared__ unsigned long long s_w[kScanThreads / 64];
    const uint32_t per = (a.nblocks + kScanThreads - 1) / kScanThreads;
    const uint32_t b0 = threadIdx.x * per, b1 = min(b0 + per, a.nblocks);
    unsigned long long s = 0;
    for (uint32_t b = b0; b < b1; ++b) s += a.block_off[b];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long incl = wave_incl_scan(s, lane);
    if (lane == 63) s_w[w] = incl;
    __syncthreads();
    unsigned long long wo = 0;
    for (int k = 0; k < w; ++k) wo += s_w[k];
    unsigned long long run = wo + incl - s;
    for (uint32_t b = b0; b < b1; ++b) {
        const unsigned long long t = a.block_off[b];
        a.block_off[b] = run;
        run += t;
    }
    if (threadIdx.x == kScanThreads - 1) *a.used = run;
}

__device__ __forceinline__ uint4 ld16(const uint8_t *p) { return *reinterpret_cast<const uint4 *>(p); }

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

// One payload by a group of kG lanes (j = lane in the group, gb = the group's first lane
// in the wave).  Destination chunk k (16 bytes) = source bytes [16k + sh, 16k + sh + 16)
// from the 16-byte-aligned source chunks k and k + 1.  Lane j loads chunk k = k0 + u*kG + j
// and takes chunk k + 1 from lane j + 1 (lane kG-1: from lane 0's next u, or its own extra
// load after the last u).
__device__ __forceinline__ void copy_payload(const PgArgs &a, uint64_t src, uint64_t dst, uint32_t L, int j,
                                             int gb)
{
    const uint8_t *s0 = a.frames + (src & ~15ull);
    const uint32_t sh = (uint32_t)(src & 15u);
    const uint32_t nsrc = (sh + L + 15u) >> 4, ndst = (L + 15u) >> 4;
    uint8_t *d0 = a.arena + dst;
    const int next_lane = (j == kG - 1) ? gb : gb + j + 1;
    for (uint32_t k0 = 0; k0 < ndst; k0 += kG * kU) {
        uint4 A[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint32_t k = k0 + u * kG + j;
            const uint4 v = ld16(s0 + 16u * (k < nsrc ? k : 0u));
            A[u] = k < nsrc ? v : make_uint4(0u, 0u, 0u, 0u);
        }
        uint4 E = make_uint4(0u, 0u, 0u, 0u);
        if (j == kG - 1) {
            const uint32_t k = k0 + kU * kG;
            if (k < nsrc) E = ld16(s0 + 16u * k);
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint4 give = (j == 0 && u + 1 < kU) ? A[u + 1] : A[u];
            uint4 N = bperm16(give, next_lane);
            if (j == kG - 1 && u == kU - 1) N = E;
            const uint32_t k = k0 + u * kG + j;
            if (k < ndst) {
                uint4 o = sh ? funnel16(A[u], N, sh) : A[u];
                const int valid = (int)L - (int)(16u * k);
                if (valid < 16) {
                    o.x = keep_bytes(o.x, valid);
                    o.y = keep_bytes(o.y, valid - 4);
                    o.z = keep_bytes(o.z, valid - 8);
                    o.w = keep_bytes(o.w, valid - 12);
                }
                *reinterpret_cast<uint4 *>(d0 + 16u * k) = o;
            }
        }
    }
}

__global__ __launch_bounds__(kPgThreads) void pg_copy(PgArgs a)
{
    __shared__ uint64_t s_src[kPgPerBlock];
    __shared__ uint64_t s_dst[kPgPerBlock];
    __shared__ uint32_t s_len[kPgPerBlock];
    __shared__ unsigned long long s_w[kPgThreads / 64];
    const uint32_t base = blockIdx.x * (uint32_t)kPgPerBlock;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;

    // this thread's 4 consecutive frames, in packet order
    Cand c[kPgPerThread];
    unsigned long long mine = 0;
#pragma unroll
    for (int k = 0; k < kPgPerThread; ++k) {
        c[k] = candidate(a, base + (uint32_t)(t * kPgPerThread + k));
        mine += round16(c[k].len);
    }
    const unsigned long long incl = wave_incl_scan(mine, lane);
    if (lane == 63) s_w[w] = incl;
    __syncthreads();
    unsigned long long off = a.block_off[blockIdx.x];
    for (int k = 0; k < w; ++k) off += s_w[k];
    off += incl - mine;
#pragma unroll
    for (int k = 0; k < kPgPerThread; ++k) {
        const int q = t * kPgPerThread + k;
        const uint32_t i = base + (uint32_t)q;
        const uint64_t r16 = round16(c[k].len);
        const bool fits = c[k].len != 0u && off + r16 <= a.arena_cap;
        if (i < a.n) {
            rxg_payload_msg m;
            m.arena_off = fits ? off : 0ull;
            m.len = fits ? c[k].len : 0u;
            m.flags = fits ? c[k].flags : 0u;
            a.msgs[i] = m;
        }
        s_src[q] = c[k].src;
        s_dst[q] = off;
        s_len[q] = fits ? c[k].len : 0u;
        off += r16;
    }
    __syncthreads();

    const int g = t / kG, j = t % kG, gb = lane & ~(kG - 1);
    for (int q = g; q < kPgPerBlock; q += kPgThreads / kG) {
        const uint32_t L = s_len[q];
        if (L) copy_payload(a, s_src[q], s_dst[q], L, j, gb);
    }
}

}  // namespace

hipError_t launch_payload(const LaunchPayload &P, hipStream_t st)
{
    if (P.n == 0) return hipMemsetAsync(P.used, 0, sizeof(unsigned long long), st);
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
    a.block_off = P.scratch;
    a.used = P.used;
    a.nblocks = payload_blocks(P.n);
    hipLaunchKernelGGL(pg_sizes, dim3(a.nblocks), dim3(kPgThreads), 0, st, a);
    hipLaunchKernelGGL(pg_scan, dim3(1), dim3(kScanThreads), 0, st, a);
    hipLaunchKernelGGL(pg_copy, dim3(a.nblocks), dim3(kPgThreads), 0, st, a);
    return hipGetLastError();
}

uint32_t payload_blocks(uint32_t n) { return (n + kPgPerBlock - 1) / kPgPerBlock; }

}  // namespace rxg
