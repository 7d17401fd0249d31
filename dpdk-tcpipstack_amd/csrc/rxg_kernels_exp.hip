// rxg_kernels_exp.hip — experiment library only (librxg_exp.so, make experiments): the
// ablation kernels scripts/kbench.py and srvfloor.py time against the product kernels, to
// find where a kernel's microseconds go.  Each is the product body of
// rxg_rx.h with parts removed; their records are not the reference's (timing only).
//
// RXG_VARIANT (single-burst rx launches, record kinds 8 and 16):
//   11, 63  no TCB / ARP probe (kAblNoProbe: every frame misses)
//   12      no record stores (kAblNoStore)
//   13      no classify (kAblNoPhaseB: parse + checksums only)
//   60      cache-resident buckets, no search (kAblHotBuckets | kAblNoSearch)
//   61      real bucket loads, no search (kAblNoSearch)
//   62      cache-resident buckets, real search (kAblHotBuckets)
// RXG_VARIANT (rxg_tx_cksum_dev):
//   90      two passes: the checksums of every frame into an array (rx_kernel<kModeTxWords>, no
//           store into the frames), then tx_scatter writes the two fields of each frame; exact
//   91      the production tx kernel with its rounds not software-pipelined; exact
//   92      90 with pass 1's rounds not pipelined; exact
//   93      pass 1 of 90 alone (timing only: no checksum reaches the frames)
// RXG_VARIANT (latency-mode server, record kind 8):
//   79 / 80 / 81 / 82  the server without its rx body / its request acquire / its release
//                      before `done` / both of the last two (SRVX 1 / 2 / 4 / 6)
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rxg_kernels.h"
#include "rxg_rx.h"

namespace rxg {

template <int MODE>
static hipError_t launch_abl(int variant, const RxArgs &a, const RxGrid &g, hipStream_t st)
{
    const dim3 grid(g.blocks), blk(256);
    switch (variant) {
    case 11:
    case 63: hipLaunchKernelGGL((rx_kernel<MODE, kDescList, false, false, kAblNoProbe>), grid, blk, 0, st, a); break;
    case 12: hipLaunchKernelGGL((rx_kernel<MODE, kDescList, false, false, kAblNoStore>), grid, blk, 0, st, a); break;
    case 13: hipLaunchKernelGGL((rx_kernel<MODE, kDescList, false, false, kAblNoPhaseB>), grid, blk, 0, st, a); break;
    case 60:
        hipLaunchKernelGGL((rx_kernel<MODE, kDescList, false, false, kAblHotBuckets | kAblNoSearch>), grid, blk, 0, st, a);
        break;
    case 61: hipLaunchKernelGGL((rx_kernel<MODE, kDescList, false, false, kAblNoSearch>), grid, blk, 0, st, a); break;
    case 62: hipLaunchKernelGGL((rx_kernel<MODE, kDescList, false, false, kAblHotBuckets>), grid, blk, 0, st, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_rx_exp(const LaunchRx &L, hipStream_t st)
{
    RxArgs a;
    RxGrid g;
    const hipError_t e = rx_args(L, a, g);
    if (e != hipSuccess || a.nslices == 0) return e;
    if (L.sel || L.stride64 || a.nbursts != 1) return hipErrorInvalidValue;
    if (L.mode == 8) return launch_abl<8>(L.variant, a, g, st);
    if (L.mode == 16) return launch_abl<16>(L.variant, a, g, st);
    return hipErrorInvalidValue;
}

// Pass 2 of the two-pass tx: frame i's two checksum fields from ck[i] (ip_ck | tcp_ck << 16),
// stored as ip_out stores them (htons, ip.c:107,118; bytes at or past data_len untouched).
__global__ __launch_bounds__(256) void tx_scatter(uint8_t *frames, const uint32_t *off64, const uint16_t *len,
                                                  const uint32_t *ck, uint32_t n)
{
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        const uint32_t L = len[i], c = ck[i];
        uint8_t *fp = frames + (size_t)off64[i] * 64u;
        const uint32_t ip_ck = c & 0xFFFFu, tcp_ck = c >> 16;
        if (L > 25u) *reinterpret_cast<uint16_t *>(fp + 24) = (uint16_t)bswap16(ip_ck);
        else if (L > 24u) fp[24] = (uint8_t)(ip_ck >> 8);
        if (L > 51u) *reinterpret_cast<uint16_t *>(fp + 50) = (uint16_t)bswap16(tcp_ck);
        else if (L > 50u) fp[50] = (uint8_t)(tcp_ck >> 8);
    }
}

hipError_t launch_tx_exp(const LaunchRx &L, hipStream_t st)
{
    RxArgs a;
    RxGrid g;
    const hipError_t e = rx_args(L, a, g);
    if (e != hipSuccess || a.nslices == 0) return e;
    if (L.variant != 91 || a.nbursts != 1 || L.stride64) return hipErrorInvalidValue;
    hipLaunchKernelGGL((rx_kernel<0, kDescList, false, false, kFormNoPipe>), dim3(g.blocks), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_tx_two_pass_exp(const LaunchRx &L, uint32_t *ck, hipStream_t st)
{
    if (L.nbursts != 1 || L.sel || L.stride64) return hipErrorInvalidValue;
    LaunchBurst b = L.bursts[0];
    b.out = reinterpret_cast<uint8_t *>(ck);
    LaunchRx X = L;
    X.bursts = &b;
    RxArgs a;
    RxGrid g;
    hipError_t e = rx_args(X, a, g);
    if (e != hipSuccess || a.nslices == 0) return e;
    if (L.variant == 92)
        hipLaunchKernelGGL((rx_kernel<kModeTxWords, kDescList, false, false, kFormNoPipe>), dim3(g.blocks), dim3(256), 0,
                           st, a);
    else
        hipLaunchKernelGGL((rx_kernel<kModeTxWords, kDescList, false, false>), dim3(g.blocks), dim3(256), 0, st, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (L.variant == 93) return hipSuccess;
    const uint32_t n = b.n;
    hipLaunchKernelGGL(tx_scatter, dim3(std::min(4096u, (n + 255u) / 256u)), dim3(256), 0, st,
                       const_cast<uint8_t *>(L.frames), b.off64, b.len, ck, n);
    return hipGetLastError();
}

hipError_t launch_server_exp(const LaunchServer &L, hipStream_t st)
{
    SrvArgs sa{L.mbox, L.ret ? L.ret : L.mbox, L.ctl, L.counters, L.idle_ticks};
    const dim3 g(L.blocks ? L.blocks : 1u), b(256);
    if (L.mode != 8) return hipErrorInvalidValue;
    switch (L.variant) {
    case 79: hipLaunchKernelGGL((rx_server<8, 1>), g, b, 0, st, sa); break;
    case 80: hipLaunchKernelGGL((rx_server<8, 2>), g, b, 0, st, sa); break;
    case 81: hipLaunchKernelGGL((rx_server<8, 4>), g, b, 0, st, sa); break;
    case 82: hipLaunchKernelGGL((rx_server<8, 6>), g, b, 0, st, sa); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace rxg
