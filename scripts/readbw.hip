// readbw.hip — read-bandwidth ceilings for the rx kernel's access pattern (experiment tool,
// not part of librxg).  Build: hipcc --offload-arch=gfx950 -O3 -o build/readbw scripts/readbw.hip
//
// Variants (all read a buffer far larger than the 256 MiB Infinity Cache, sum every dword,
// one store per thread at the end):
//   flat_def / flat_nt   grid-stride 16 B per lane, U loads in flight per lane
//   fr1536 / fr1504      1500-byte frames in 1536-B (64-B aligned) or 1504-B (16-B aligned)
//                        slots, 16 lanes per frame x 6 loads: the rx kernel's C3 class
//                        without its compute
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4 *p)
{
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

template <bool NT, int U>
__global__ __launch_bounds__(256) void flat(const u32x4 *buf, size_t n16, unsigned *out)
{
    const size_t stride = (size_t)gridDim.x * 256u;
    size_t i = (size_t)blockIdx.x * 256u + threadIdx.x;
    unsigned acc = 0;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld<NT>(buf + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    for (; i < n16; i += stride) {
        u32x4 v = ld<NT>(buf + i);
        acc += v.x + v.y + v.z + v.w;
    }
    out[blockIdx.x * 256u + threadIdx.x] = acc;
}

// frames: slot bytes SLOT, 1500 bytes each; a wave takes 4 frames per round (16 lanes each),
// waves own slices of 64 consecutive frames (like rx_kernel)
template <bool NT, int SLOT>
__global__ __launch_bounds__(256) void frames(const uint8_t *buf, unsigned nfr, unsigned *out)
{
    const int lane = threadIdx.x & 63;
    const unsigned wave = blockIdx.x * 4u + (threadIdx.x >> 6);
    const unsigned nwaves = gridDim.x * 4u;
    const unsigned nsl = (nfr + 63u) / 64u;
    unsigned acc = 0;
    const int gl = lane & 15;
    for (unsigned s = wave; s < nsl; s += nwaves) {
        for (unsigned r = 0; r < 64; r += 4) {
            const unsigned f = s * 64u + r + (unsigned)(lane >> 4);
            if (f >= nfr) break;
            const uint8_t *fp = buf + (size_t)f * SLOT;
            u32x4 v[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const int c = gl + 16 * j;
                const bool ok = c * 16 < 1500;
                v[j] = ld<NT>(reinterpret_cast<const u32x4 *>(fp + (ok ? c * 16 : 0)));
                if (!ok) v[j] = u32x4{0, 0, 0, 0};
            }
#pragma unroll
            for (int j = 0; j < 6; ++j) acc += v[j].x + v[j].y + v[j].z + v[j].w;
        }
    }
    out[blockIdx.x * 256u + threadIdx.x] = acc;
}

// C2 pattern: 64-byte frames, slices of 64 frames per wave (round-robin), descriptors
// off64[] (u32) and len[] (u16) read per slice; MODE bit 0: read descriptors (else
// frame f at slot f), bit 1: store a 16-byte record per frame (1 KiB per slice).
template <int MODE>
__global__ __launch_bounds__(256) void small(const uint8_t *buf, const unsigned *off64, const unsigned short *len,
                                             unsigned nfr, uint4 *rec, unsigned *out)
{
    const int lane = threadIdx.x & 63;
    const unsigned wave = blockIdx.x * 4u + (threadIdx.x >> 6);
    const unsigned nwaves = gridDim.x * 4u;
    const unsigned nsl = nfr / 64u;
    unsigned acc = 0;
    for (unsigned s = wave; s < nsl; s += nwaves) {
        const unsigned f = s * 64u + lane;
        unsigned o = f, l = 64;
        if (MODE & 1) { o = off64[f]; l = len[f]; }
        u32x4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int fr = 16 * j + (lane >> 2);
            const unsigned fo = __shfl(o, fr, 64);
            v[j] = ld<false>(reinterpret_cast<const u32x4 *>(buf + (size_t)fo * 64u + (lane & 3) * 16));
        }
        unsigned t = l;
#pragma unroll
        for (int j = 0; j < 4; ++j) t += v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
        if (MODE & 2) rec[f] = make_uint4(t, t + 1, t + 2, t + 3);
        acc += t;
    }
    out[blockIdx.x * 256u + threadIdx.x] = acc;
}

template <typename F>
static void timeit(const char *name, double bytes, F launch)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) launch();
    std::vector<float> ms;
    for (int i = 0; i < 20; ++i) {
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float t;
        CK(hipEventElapsedTime(&t, a, b));
        ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const double med = ms[ms.size() / 2];
    printf("{\"variant\": \"%s\", \"us_median\": %.2f, \"us_min\": %.2f, \"TBps\": %.3f}\n", name, med * 1e3,
           ms[0] * 1e3, bytes / (med * 1e-3) / 1e12);
    fflush(stdout);
}

int main(int argc, char **argv)
{
    const unsigned nfr = 1u << 20;
    const size_t bytes = (size_t)nfr * 1536u;  // 1.61 GB
    uint8_t *buf;
    unsigned *out;
    CK(hipMalloc(&buf, bytes + 4096));
    CK(hipMemset(buf, 1, bytes + 4096));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int maxg = ncu * 32;
    CK(hipMalloc(&out, (size_t)maxg * 256 * sizeof(unsigned)));
    const size_t n16_a = (size_t)nfr * 1500u / 16u;  // the algorithmic byte count of C3
    for (int rep = 0; rep < 1; ++rep) {
        std::vector<int> grids = {ncu * 4, ncu * 8, ncu * 16};
        if (argc > 1) {  // workgroups per CU to sweep, e.g. "2 3 4"
            grids.clear();
            for (int i = 1; i < argc; ++i) grids.push_back(ncu * atoi(argv[i]));
        }
        for (int g : grids) {
            char nm[64];
            snprintf(nm, sizeof nm, "flat_def_u4_g%d", g);
            timeit(nm, n16_a * 16.0, [&] { flat<false, 4><<<g, 256>>>((const u32x4 *)buf, n16_a, out); });
            snprintf(nm, sizeof nm, "flat_nt_u4_g%d", g);
            timeit(nm, n16_a * 16.0, [&] { flat<true, 4><<<g, 256>>>((const u32x4 *)buf, n16_a, out); });
            snprintf(nm, sizeof nm, "flat_nt_u8_g%d", g);
            timeit(nm, n16_a * 16.0, [&] { flat<true, 8><<<g, 256>>>((const u32x4 *)buf, n16_a, out); });
            snprintf(nm, sizeof nm, "fr1536_nt_g%d", g);
            timeit(nm, nfr * 1500.0, [&] { frames<true, 1536><<<g, 256>>>(buf, nfr, out); });
            snprintf(nm, sizeof nm, "fr1536_def_g%d", g);
            timeit(nm, nfr * 1500.0, [&] { frames<false, 1536><<<g, 256>>>(buf, nfr, out); });
            snprintf(nm, sizeof nm, "fr1504_nt_g%d", g);
            timeit(nm, nfr * 1500.0, [&] { frames<true, 1504><<<g, 256>>>(buf, nfr, out); });
        }
    }
    {
        // C4's byte count (2^20 IMIX frames, mean 354.3 B = 371.5 MB) as one flat stream,
        // rotating over 4 disjoint regions of buf (1.49 GB) so the MALL cannot hold it: an
        // upper bound for any C4 access pattern at this launch size
        const size_t n16_c4 = (size_t)371519488 / 16u;
        int it = 0;
        for (int g : {ncu * 3, ncu * 4, ncu * 8}) {
            char nm[64];
            snprintf(nm, sizeof nm, "c4_flat_nt_g%d", g);
            timeit(nm, n16_c4 * 16.0, [&] {
                const u32x4 *p = (const u32x4 *)buf + (size_t)(it++ % 4) * n16_c4;
                flat<true, 4><<<g, 256>>>(p, n16_c4, out);
            });
        }
    }
    {
        // C2: 2^20 x 64 B frames per launch, 16 rotating copies (1 GiB)
        const unsigned n2 = 1u << 20;
        const int ncopy = 16;
        uint8_t *f2;
        unsigned *o2;
        unsigned short *l2;
        uint4 *r2;
        CK(hipMalloc(&f2, (size_t)n2 * 64u * ncopy));
        CK(hipMemset(f2, 3, (size_t)n2 * 64u * ncopy));
        CK(hipMalloc(&o2, (size_t)n2 * 4u * ncopy));
        CK(hipMalloc(&l2, (size_t)n2 * 2u * ncopy));
        CK(hipMalloc(&r2, (size_t)n2 * 16u));
        std::vector<unsigned> ho(n2);
        for (unsigned i = 0; i < n2; ++i) ho[i] = i;
        std::vector<unsigned short> hl(n2, 64);
        for (int c = 0; c < ncopy; ++c) {
            CK(hipMemcpy(o2 + (size_t)c * n2, ho.data(), n2 * 4u, hipMemcpyHostToDevice));
            CK(hipMemcpy(l2 + (size_t)c * n2, hl.data(), n2 * 2u, hipMemcpyHostToDevice));
        }
        int it = 0;
        for (int g : {ncu * 3, ncu * 4, ncu * 8}) {
            char nm[64];
            auto run = [&](auto m) {
                constexpr int M = decltype(m)::value;
                const int c = it++ % ncopy;
                small<M><<<g, 256>>>(f2 + (size_t)c * n2 * 64u, o2 + (size_t)c * n2, l2 + (size_t)c * n2, n2, r2, out);
            };
            snprintf(nm, sizeof nm, "c2_frames_g%d", g);
            timeit(nm, n2 * 64.0, [&] { run(std::integral_constant<int, 0>{}); });
            snprintf(nm, sizeof nm, "c2_desc_g%d", g);
            timeit(nm, n2 * 64.0, [&] { run(std::integral_constant<int, 1>{}); });
            snprintf(nm, sizeof nm, "c2_desc_rec_g%d", g);
            timeit(nm, n2 * 64.0, [&] { run(std::integral_constant<int, 3>{}); });
        }
    }
    CK(hipDeviceSynchronize());
    return 0;
}
