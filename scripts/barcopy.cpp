// barcopy: how fast the rx thread can pack a host burst into fine-grained device memory
// through the BAR (the latency-mode server's staging, rxg_server.cpp rxg_rx_burst): memcpy per
// frame against AVX2 non-temporal 32-byte stores per frame, bursts of 32 / 256 frames of
// 64 / 1500 bytes from mbuf-like sources (2 KiB apart, offset 128), each followed by an sfence.
// build: hipcc -O2 -mavx2 barcopy.cpp -o build/barcopy
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

static void pack_memcpy(uint8_t *dst, const uint8_t *src, int n, int len)
{
    const int slot = (len + 63) / 64 * 64;
    for (int i = 0; i < n; ++i) std::memcpy(dst + (size_t)i * slot, src + (size_t)i * 2048 + 128, (size_t)len);
}

static void pack_stream(uint8_t *dst, const uint8_t *src, int n, int len)
{
    const int slot = (len + 63) / 64 * 64;
    for (int i = 0; i < n; ++i) {
        const uint8_t *s = src + (size_t)i * 2048 + 128;
        uint8_t *d = dst + (size_t)i * slot;
        int k = 0;
        for (; k + 32 <= len; k += 32)
            _mm256_stream_si256(reinterpret_cast<__m256i *>(d + k), _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + k)));
        if (k < len) {  // the tail: whole 32 bytes from a zero-padded copy (no read past the frame)
            alignas(32) uint8_t t[32] = {};
            std::memcpy(t, s + k, (size_t)(len - k));
            _mm256_stream_si256(reinterpret_cast<__m256i *>(d + k), _mm256_load_si256(reinterpret_cast<const __m256i *>(t)));
        }
    }
}

int main()
{
    uint8_t *dev = nullptr;
    if (hipSetDevice(0) != hipSuccess ||
        hipExtMallocWithFlags(reinterpret_cast<void **>(&dev), 1 << 20, hipDeviceMallocFinegrained) != hipSuccess) {
        std::fprintf(stderr, "fine-grained device allocation failed\n");
        return 1;
    }
    std::vector<uint8_t> src(256 * 2048 + 4096);
    for (size_t i = 0; i < src.size(); ++i) src[i] = (uint8_t)(i * 131);
    for (int len : {64, 1500})
        for (int n : {32, 256}) {
            for (int form = 0; form < 2; ++form) {
                std::vector<double> t;
                for (int r = 0; r < 2000; ++r) {
                    const auto a = std::chrono::steady_clock::now();
                    if (form == 0) pack_memcpy(dev, src.data(), n, len);
                    else pack_stream(dev, src.data(), n, len);
                    _mm_sfence();
                    t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
                }
                std::sort(t.begin(), t.end());
                const double bytes = (double)n * len;
                std::printf("{\"frame_bytes\": %d, \"frames\": %d, \"form\": \"%s\", \"us_median\": %.3f, \"GBps\": %.1f}\n",
                            len, n, form ? "avx2_stream" : "memcpy", t[t.size() / 2], bytes / t[t.size() / 2] / 1e3);
            }
        }
    (void)hipFree(dev);
    return 0;
}
