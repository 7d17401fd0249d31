// Micro-benchmark for a two-pass tx checksum generate (HISTORY.md §9.R4): how long do the
// checksum field writes alone take when they are NOT interleaved with the frame read stream?
// Frames at a 1 536-byte stride (the C3 layout), 2^20 of them; per frame:
//   v0  two 2-byte stores (bytes 24-25, 50-51) from a 4-byte-per-frame checksum array
//   v1  the same, the checksum array read but no stores (the scatter's read side)
//   v2  one 16-byte store at +16 and one at +48 (whole 16-byte chunks, contents from the array)
// Prints JSON lines: variant, median / min microseconds over 20 runs.
//   hipcc --offload-arch=gfx950 -O3 -o build/txscatter scripts/txscatter.hip && ./build/txscatter
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                           \
            return 1;                                                                              \
        }                                                                                          \
    } while (0)

template <int V>
__global__ __launch_bounds__(256) void scatter(uint8_t *frames, const uint32_t *ck, uint32_t n, uint32_t stride)
{
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        const uint32_t c = ck[i];
        uint8_t *f = frames + (size_t)i * stride;
        if constexpr (V == 0) {
            *reinterpret_cast<uint16_t *>(f + 24) = (uint16_t)c;
            *reinterpret_cast<uint16_t *>(f + 50) = (uint16_t)(c >> 16);
        } else if constexpr (V == 1) {
            if (c == 0x12345678u) f[0] = 1;  // never: keeps the load
        } else {
            *reinterpret_cast<uint4 *>(f + 16) = make_uint4(c, c, c, c);
            *reinterpret_cast<uint4 *>(f + 48) = make_uint4(c, c, c, c);
        }
    }
}

int main()
{
    const uint32_t n = 1u << 20, stride = 1536;
    uint8_t *frames;
    uint32_t *ck;
    CK(hipMalloc(&frames, (size_t)n * stride));
    CK(hipMalloc(&ck, (size_t)n * 4));
    CK(hipMemset(frames, 0x5A, (size_t)n * stride));
    CK(hipMemset(ck, 0x33, (size_t)n * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int grid : {1024, 4096}) {
        for (int v = 0; v < 3; ++v) {
            std::vector<float> ms;
            for (int r = 0; r < 22; ++r) {
                CK(hipEventRecord(a));
                if (v == 0) hipLaunchKernelGGL(scatter<0>, dim3(grid), dim3(256), 0, 0, frames, ck, n, stride);
                if (v == 1) hipLaunchKernelGGL(scatter<1>, dim3(grid), dim3(256), 0, 0, frames, ck, n, stride);
                if (v == 2) hipLaunchKernelGGL(scatter<2>, dim3(grid), dim3(256), 0, 0, frames, ck, n, stride);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float t;
                CK(hipEventElapsedTime(&t, a, b));
                if (r >= 2) ms.push_back(t);
            }
            std::sort(ms.begin(), ms.end());
            std::printf("{\"variant\": %d, \"grid\": %d, \"us_median\": %.2f, \"us_min\": %.2f}\n", v, grid,
                        ms[ms.size() / 2] * 1e3, ms[0] * 1e3);
        }
    }
    return 0;
}
