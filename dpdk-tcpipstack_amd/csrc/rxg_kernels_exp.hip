// rxg_kernels_exp.hip — experiment library only (librxg_exp.so, make experiments): kernel
// variants scripts/kbench.py times against the product kernels through RXG_VARIANT.  Their
// results are the product's (same records), only the form differs.
//
// The round-2..4 ablation kernels (no probe / no stores / no classify / stamped server
// phases) were removed in round 5 with their template parameters; what they measured is in
// DESIGN.md §9.R3 / §9.R4 and profiles/r03, r04.  So were round 5's fused payload forms
// (RXG_VARIANT 101-107: plain / chunk-granular / pipelined / 4-waves stores; DESIGN.md §5.F,
// profiles/r05/fused/).
#include <hip/hip_runtime.h>

#include "rxg_kernels.h"
#include "rxg_rx.h"

namespace rxg {

hipError_t launch_rx_exp(const LaunchRx &L, hipStream_t st)
{
    RxArgs a;
    RxGrid g;
    const hipError_t e = rx_args(L, a, g);
    if (e != hipSuccess || a.nslices == 0) return e;
    (void)st;
    return hipErrorInvalidValue;  // no variant defined
}

}  // namespace rxg
