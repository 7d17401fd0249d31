// readbw_rot.hip — read ceiling for the headline's access pattern (HISTORY.md §6.R5): a
// hand-written 16-byte-per-lane streaming read of two rotating 1.5 GiB buffers (as bench.py rotates its two C3
// batches, so no launch re-reads the last one's tail from the 256 MB MALL), each thread
// folding what it read into one word (4 B written per thread).  Grid-stride over a grid of
// W workgroups per CU, U loads in flight per lane, plain or non-temporal loads.
// (scripts/readbw.hip: the frame-layout and C2 pattern ceilings of round 1.)
// Build: hipcc --offload-arch=gfx950 -O3 -o build/readbw_rot scripts/readbw_rot.hip
// Run:   build/readbw_rot          one JSON line per (form, W, U): mean us per launch, TB/s
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT, int U>
__global__ __launch_bounds__(256) void rd(const u32x4 *src, size_t n16, unsigned *out)
{
    const size_t stride = (size_t)gridDim.x * 256u * U;
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256u * U + threadIdx.x; i < n16; i += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t k = i + 256u * u;
            v[u] = k < n16 ? (NT ? __builtin_nontemporal_load(src + k) : src[k]) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    out[(size_t)blockIdx.x * 256u + threadIdx.x] = acc;
}

template <bool NT, int U>
static void measure(const char *form, int w, int cus, u32x4 *const *buf, size_t n16, unsigned *out)
{
    const int grid = w * cus;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 4; ++i) hipLaunchKernelGGL((rd<NT, U>), dim3(grid), dim3(256), 0, 0, buf[i & 1], n16, out);
    CK(hipDeviceSynchronize());
    const int iters = 40;
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((rd<NT, U>), dim3(grid), dim3(256), 0, 0, buf[i & 1], n16, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / iters;
    printf("{\"form\": \"%s\", \"wg_per_cu\": %d, \"loads_in_flight\": %d, \"us\": %.2f, \"TBps\": %.3f}\n", form, w, U, us,
           (double)n16 * 16.0 / us / 1e6);
    fflush(stdout);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

int main()
{
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const size_t n16 = ((size_t)1536 << 20) / 16;  // 1.5 GiB per buffer, as the C3 frame pool (2^20 x 1 536 B)
    u32x4 *buf[2];
    unsigned *out;
    for (auto &q : buf) {
        CK(hipMalloc(&q, n16 * 16));
        CK(hipMemset(q, 0x5A, n16 * 16));
    }
    CK(hipMalloc(&out, (size_t)cus * 16 * 256 * sizeof(unsigned)));
    for (int w : {2, 3, 4, 8, 16}) {
        measure<false, 4>("plain", w, cus, buf, n16, out);
        measure<true, 4>("nontemporal", w, cus, buf, n16, out);
        measure<true, 8>("nontemporal", w, cus, buf, n16, out);
    }
    for (auto &q : buf) CK(hipFree(q));
    CK(hipFree(out));
    return 0;
}
