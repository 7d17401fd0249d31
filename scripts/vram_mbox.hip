// Latency probe for the server's mailbox and staging: where should the
// request and the burst's frames live so that a host post reaches a persistent kernel fastest?
//   host:  coherent host memory (hipHostMallocCoherent | Mapped), the production placement:
//          the server's polls and the frame reads cross PCIe as reads (round trips)
//   vram:  fine-grained device memory the host writes through its mapping (posted PCIe
//          writes); the server polls and reads HBM
// One workgroup polls `seq` (system-scope relaxed loads), then reads the request's payload
// bytes, then stores `done` to host memory; the host copies the payload, fences, posts seq,
// spins on done.  Prints one JSON line per (placement, payload bytes).
//   hipcc --offload-arch=gfx950 -O2 -o build/vram_mbox scripts/vram_mbox.hip
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <algorithm>
#include <chrono>
#include <csetjmp>
#include <csignal>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

struct alignas(128) Box {
    unsigned long long seq;
    unsigned long long nbytes;
    unsigned long long pad[14];
};

__global__ __launch_bounds__(64) void pingpong(Box *box, const uint4 *data, unsigned long long *done,
                                               unsigned long long *sink, int iters, long long limit)
{
    const int l = (int)threadIdx.x;
    uint32_t acc = 0u;
    for (int i = 1; i <= iters; ++i) {
        const long long t0 = wall_clock64();
        unsigned long long nb = 0ull;
        for (;;) {
            unsigned long long w = 0ull;
            if (l < 2)
                w = __hip_atomic_load(reinterpret_cast<const unsigned long long *>(box) + l, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_SYSTEM);
            const unsigned long long q = __shfl(w, 0, 64);
            nb = __shfl(w, 1, 64);
            if (q == (unsigned long long)i) break;
            if (wall_clock64() - t0 > limit) {  // the host is gone: leave, every lane together
                if (l == 0) sink[1] = 1ull;
                return;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t n16 = (uint32_t)(nb / 16u);
#pragma unroll 16
        for (uint32_t k = (uint32_t)l; k < n16; k += 64u) {
            const uint4 v = data[k];
            acc += v.x ^ v.y ^ v.z ^ v.w;
        }
        // the loads are consumed before done is stored
        for (int m = 32; m >= 1; m >>= 1) acc += (uint32_t)__shfl_xor((int)acc, m, 64);
        if (l == 0) {
            sink[0] = acc;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(done, (unsigned long long)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

static sigjmp_buf g_jmp;
static void on_segv(int) { siglongjmp(g_jmp, 1); }

// can the host write and read back this pointer?
static bool host_can_touch(volatile unsigned long long *p)
{
    struct sigaction sa {}, old {};
    sa.sa_handler = on_segv;
    sigaction(SIGSEGV, &sa, &old);
    sigaction(SIGBUS, &sa, nullptr);
    bool ok = false;
    if (sigsetjmp(g_jmp, 1) == 0) {
        p[0] = 0x1234567890abcdefull;
        _mm_mfence();
        ok = p[0] == 0x1234567890abcdefull;
        p[0] = 0ull;
        _mm_mfence();
    }
    sigaction(SIGSEGV, &old, nullptr);
    sigaction(SIGBUS, &old, nullptr);
    return ok;
}

static int run(const char *where, unsigned vram_flag, size_t nbytes, int iters)
{
    Box *box = nullptr;
    uint8_t *data = nullptr;
    const size_t cap = 64u << 10;
    if (vram_flag == ~0u) {
        CK(hipHostMalloc((void **)&box, sizeof(Box), hipHostMallocCoherent | hipHostMallocMapped));
        CK(hipHostMalloc((void **)&data, cap, hipHostMallocCoherent | hipHostMallocMapped));
    } else {
        CK(hipExtMallocWithFlags((void **)&box, sizeof(Box), vram_flag));
        CK(hipExtMallocWithFlags((void **)&data, cap, vram_flag));
        hipPointerAttribute_t at{};
        CK(hipPointerGetAttributes(&at, box));
        std::printf("{\"where\": \"%s\", \"attr_type\": %d, \"hostPointer\": %s}\n", where, (int)at.type,
                    at.hostPointer ? "true" : "false");
        if (!host_can_touch(reinterpret_cast<volatile unsigned long long *>(box)) ||
            !host_can_touch(reinterpret_cast<volatile unsigned long long *>(data))) {
            std::printf("{\"where\": \"%s\", \"host_access\": false}\n", where);
            (void)hipFree(box);
            (void)hipFree(data);
            return 0;
        }
    }
    unsigned long long *done = nullptr, *sink = nullptr;
    CK(hipHostMalloc((void **)&done, 128, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipMalloc((void **)&sink, 16));
    CK(hipMemset(sink, 0, 16));
    std::memset((void *)done, 0, 128);
    std::vector<uint8_t> src(cap);
    for (size_t i = 0; i < cap; ++i) src[i] = (uint8_t)(i * 131u + 7u);
    volatile Box *vb = box;
    vb->seq = 0ull;
    _mm_mfence();
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    int khz = 100000;
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
    hipLaunchKernelGGL(pingpong, dim3(1), dim3(64), 0, st, box, (const uint4 *)data, done, sink, iters,
                       (long long)khz * 2000ll);  // 2 s without a post: exit
    CK(hipGetLastError());
    std::vector<double> us;
    us.reserve(iters);
    bool lost = false;
    for (int i = 1; i <= iters && !lost; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        if (nbytes) std::memcpy(data, src.data(), nbytes);
        vb->nbytes = nbytes;
        _mm_sfence();
        vb->seq = (unsigned long long)i;
        _mm_sfence();
        for (;;) {
            if (__atomic_load_n(done, __ATOMIC_ACQUIRE) == (unsigned long long)i) break;
            _mm_pause();
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
                lost = true;
                break;
            }
        }
        us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    CK(hipStreamSynchronize(st));
    std::sort(us.begin(), us.end());
    std::printf("{\"where\": \"%s\", \"payload_bytes\": %zu, \"iters\": %d, \"lost\": %s, \"us_median\": %.2f, "
                "\"us_p10\": %.2f, \"us_p90\": %.2f}\n",
                where, nbytes, (int)us.size(), lost ? "true" : "false", us[us.size() / 2], us[us.size() / 10],
                us[us.size() * 9 / 10]);
    std::fflush(stdout);
    (void)hipStreamDestroy(st);
    if (vram_flag == ~0u) {
        (void)hipHostFree(box);
        (void)hipHostFree(data);
    } else {
        (void)hipFree(box);
        (void)hipFree(data);
    }
    (void)hipHostFree(done);
    (void)hipFree(sink);
    return lost ? 2 : 0;
}

int main()
{
    CK(hipSetDevice(0));
    int rc = 0;
    for (size_t nb : {(size_t)0, (size_t)2048, (size_t)49152}) {
        rc |= run("host", ~0u, nb, 2000);
        rc |= run("vram_finegrained", hipDeviceMallocFinegrained, nb, 2000);
        rc |= run("vram_uncached", hipDeviceMallocUncached, nb, 2000);
        if (rc) break;
    }
    return rc;
}
