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
// RXG_VARIANT (latency-mode server, record kind 8):
//   79 / 80 / 81 / 82  the server without its rx body / its request acquire / its release
//                      before `done` / both of the last two (SRVX 1 / 2 / 4 / 6)
//   83 / 84 / 85       the production server stamping each request's phases (SRVX 8,
//                      scripts/srvstamps.py) / the same without the TCB probe / without the
//                      record stores (SRVX 24 / 40)
//   86 / 87            stamping, buckets from a cache-resident region / no search (SRVX 72 / 136)
//   88                 stamping, the body's phases too (SRVX 264)
//   89                 stamping, the body run twice per request (SRVX 520)
#include <hip/hip_runtime.h>

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
    case 83: hipLaunchKernelGGL((rx_server<8, 8>), g, b, 0, st, sa); break;
    case 84: hipLaunchKernelGGL((rx_server<8, 8 | 16>), g, b, 0, st, sa); break;
    case 85: hipLaunchKernelGGL((rx_server<8, 8 | 32>), g, b, 0, st, sa); break;
    case 86: hipLaunchKernelGGL((rx_server<8, 8 | 64>), g, b, 0, st, sa); break;
    case 87: hipLaunchKernelGGL((rx_server<8, 8 | 128>), g, b, 0, st, sa); break;
    case 88: hipLaunchKernelGGL((rx_server<8, 8 | 256>), g, b, 0, st, sa); break;
    case 89: hipLaunchKernelGGL((rx_server<8, 8 | 512>), g, b, 0, st, sa); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace rxg
