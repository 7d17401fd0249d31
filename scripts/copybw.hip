// Copy ceilings for the payload gather (HISTORY.md §9): a hand-written 16-byte-per-lane copy,
// grid-stride over a persistent grid, 1.53 GB -> 1.53 GB.
//   flat:  contiguous source
//   rows:  2^20 rows of 1 456 B at a 1 536 B stride (C3's payload spans, 16-byte aligned;
//          the gather also shifts each row by 6 bytes) -> contiguous destination
//   slotsWL: 2^20 slots of 1 536 B (a C3 frame's 24 lines): every line read, the first WL
//          written to the same slot of a second pool -- the fused copy hand-off's traffic with
//          whole-line writes, WL = 24 as shipped (the payload at its pool offset: header line
//          and slot tail written) against WL = 23 (a 1 446 B payload from its first byte at the
//          slot's start: DESIGN.md §5.F's line-aligned estimate)
// Build: hipcc --offload-arch=gfx950 -O3 -o build/copybw scripts/copybw.hip
// Run:   build/copybw [workgroups per CU ...]   (default 2 4 8)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT, int U>
__global__ __launch_bounds__(256) void flat(const u32x4 *src, u32x4 *dst, size_t n16)
{
    const size_t stride = (size_t)gridDim.x * 256u * U;
    for (size_t i = (size_t)blockIdx.x * 256u * U + threadIdx.x; i < n16; i += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t k = i + 256u * u;
            if (k < n16) v[u] = NT ? __builtin_nontemporal_load(src + k) : src[k];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t k = i + 256u * u;
            if (k < n16) { if (NT) __builtin_nontemporal_store(v[u], dst + k); else dst[k] = v[u]; }
        }
    }
}

// destination chunk k -> row k / 91, chunk k % 91 of that row (91 x 16 = 1 456 B)
template <bool NT, int U>
__global__ __launch_bounds__(256) void rows(const u32x4 *src, u32x4 *dst, size_t n16)
{
    const size_t stride = (size_t)gridDim.x * 256u * U;
    for (size_t i = (size_t)blockIdx.x * 256u * U + threadIdx.x; i < n16; i += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t k = i + 256u * u;
            const size_t r = k / 91u, c = k - r * 91u;
            if (k < n16) v[u] = NT ? __builtin_nontemporal_load(src + r * 96u + 3u + c) : src[r * 96u + 3u + c];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t k = i + 256u * u;
            if (k < n16) { if (NT) __builtin_nontemporal_store(v[u], dst + k); else dst[k] = v[u]; }
        }
    }
}

// chunk k of slot r: read always, written when it lies in the slot's first WL lines
template <int WL, int U>
__global__ __launch_bounds__(256) void slots(const u32x4 *src, u32x4 *dst, size_t n16)
{
    const size_t stride = (size_t)gridDim.x * 256u * U;
    for (size_t i = (size_t)blockIdx.x * 256u * U + threadIdx.x; i < n16; i += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t k = i + 256u * u;
            if (k < n16) v[u] = __builtin_nontemporal_load(src + k);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t k = i + 256u * u;
            if (k < n16 && (k % 96u) < WL * 4u) __builtin_nontemporal_store(v[u], dst + k);
        }
    }
}

template <typename K>
static float run(K kern, int grid, const u32x4 *s, u32x4 *d, size_t n16)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, s, d, n16);
    std::vector<float> ms;
    for (int i = 0; i < 20; ++i) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, s, d, n16);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float t;
        CK(hipEventElapsedTime(&t, a, b));
        ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms[ms.size() / 2] * 1e3f;
}

int main(int argc, char **argv)
{
    const size_t nrows = 1u << 20, n16 = nrows * 91u;
    u32x4 *src, *dst;
    CK(hipMalloc(&src, nrows * 1536u));
    CK(hipMalloc(&dst, n16 * 16u));
    CK(hipMemset(src, 1, nrows * 1536u));
    u32x4 *pool2;
    CK(hipMalloc(&pool2, nrows * 1536u));
    const size_t s16 = nrows * 96u;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<int> wpc = {2, 4, 8};
    if (argc > 1) { wpc.clear(); for (int i = 1; i < argc; ++i) wpc.push_back(atoi(argv[i])); }
    const double bytes = 2.0 * n16 * 16.0;
    for (int w : wpc) {
        const int g = ncu * w;
        struct { const char *name; float us; } r[] = {
            {"flat", run(flat<false, 4>, g, src, dst, n16)},
            {"flat_nt", run(flat<true, 4>, g, src, dst, n16)},
            {"rows", run(rows<false, 4>, g, src, dst, n16)},
            {"rows_nt", run(rows<true, 4>, g, src, dst, n16)},
        };
        for (auto &x : r)
            printf("{\"copy\": \"%s\", \"wg_per_cu\": %d, \"us_median\": %.1f, \"bytes_moved\": %.0f, \"TBps\": %.3f}\n",
                   x.name, w, x.us, bytes, bytes / x.us / 1e6);
        struct { const char *name; int wl; float us; } q[] = {
            {"slots24", 24, run(slots<24, 4>, g, src, pool2, s16)},
            {"slots23", 23, run(slots<23, 4>, g, src, pool2, s16)},
        };
        for (auto &x : q) {
            const double b = (double)nrows * (1536.0 + 64.0 * x.wl);
            printf("{\"copy\": \"%s\", \"wg_per_cu\": %d, \"us_median\": %.1f, \"bytes_moved\": %.0f, \"TBps\": %.3f}\n",
                   x.name, w, x.us, b, b / x.us / 1e6);
        }
    }
    return 0;
}
