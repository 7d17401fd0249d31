// evgap: what the timing events between launches cost the bench's wall clock.  C3 batch
// (2^20 x 1500 B, two rotating copies), K launches of rxg_rx_burst_dev on the context's
// stream, timed by the host clock around the K launches, with:
//   mode 0  no events inside the loop
//   mode 1  a default event before and after every launch (bench.py's form)
//   mode 2  the same with hipEventReleaseToDevice events (device-scope release, timing kept)
//   mode 3  one default event after every launch only (kernel time = consecutive differences)
// Modes interleaved over rounds; prints one JSON line per mode (median wall us per launch and
// the median event-measured kernel us where the mode has one).
// build: hipcc -O2 -I../include evgap.cpp -L../dpdk-tcpipstack_amd/rxg -lrxg -o build/evgap
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rxg.h"

#define CK(x)                                                                          \
    do {                                                                               \
        int _r = (int)(x);                                                             \
        if (_r) {                                                                      \
            std::fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, _r,  \
                         rxg_last_error());                                            \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

static double median(std::vector<double> v)
{
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
}

int main(int argc, char **argv)
{
    const int K = argc > 1 ? std::atoi(argv[1]) : 100;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 7;
    const uint32_t n = 1u << 20;
    rxg_config cfg{};
    cfg.device = 0;
    rxg_ctx *c = nullptr;
    CK(rxg_init(&cfg, &c));
    hipStream_t st = (hipStream_t)rxg_stream(c);
    rxg_synth_params p{};
    p.n = n;
    p.nflows = 1000;
    p.dst_ip_host = 0xC0A84E02u;
    p.dport = 80;
    p.len_a = 1500;
    const uint64_t cap = rxg_synth_arena_bytes(&p);
    void *frames[2], *off[2], *len[2], *out;
    for (int b = 0; b < 2; ++b) {
        p.seed = 0x5EED0001ull + 17u * b;
        CK(rxg_dev_alloc(c, cap, &frames[b]));
        CK(rxg_dev_alloc(c, n * 4ull, &off[b]));
        CK(rxg_dev_alloc(c, n * 2ull, &len[b]));
        uint64_t used = 0;
        CK(rxg_synth_dev(c, &p, frames[b], cap, (uint32_t *)off[b], (uint16_t *)len[b], nullptr, &used, nullptr));
    }
    CK(rxg_dev_alloc(c, n * 8ull, &out));
    CK(rxg_sync(c));
    auto launch = [&](int i) {
        const int b = i & 1;
        rxg_dev_batch bt{frames[b], (const uint32_t *)off[b], (const uint16_t *)len[b], n, RXG_REC8, out};
        CK(rxg_rx_burst_dev(c, &bt, nullptr));
    };
    std::vector<hipEvent_t> ea(K), eb(K), da(K), db(K);
    for (int i = 0; i < K; ++i) {
        CK(hipEventCreate(&ea[i]));
        CK(hipEventCreate(&eb[i]));
        CK(hipEventCreateWithFlags(&da[i], hipEventReleaseToDevice));
        CK(hipEventCreateWithFlags(&db[i], hipEventReleaseToDevice));
    }
    std::vector<double> wall[4], kern[4];
    for (int i = 0; i < 10; ++i) launch(i);
    CK(rxg_sync(c));
    for (int r = 0; r < rounds; ++r)
        for (int mode = 0; mode < 4; ++mode) {
            CK(hipStreamSynchronize(st));
            const auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < K; ++i) {
                if (mode == 1) CK(hipEventRecord(ea[i], st));
                if (mode == 2) CK(hipEventRecord(da[i], st));
                launch(i);
                if (mode == 1 || mode == 3) CK(hipEventRecord(eb[i], st));
                if (mode == 2) CK(hipEventRecord(db[i], st));
            }
            CK(hipStreamSynchronize(st));
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            wall[mode].push_back(us / K);
            double ks = 0.0;
            int kn = 0;
            for (int i = 0; i < K; ++i) {
                float ms = 0.f;
                if (mode == 1) CK(hipEventElapsedTime(&ms, ea[i], eb[i]));
                if (mode == 2) CK(hipEventElapsedTime(&ms, da[i], db[i]));
                if (mode == 3 && i > 0) CK(hipEventElapsedTime(&ms, eb[i - 1], eb[i]));
                if (mode != 0 && (mode != 3 || i > 0)) {
                    ks += ms * 1e3;
                    ++kn;
                }
            }
            kern[mode].push_back(kn ? ks / kn : 0.0);
        }
    const char *names[4] = {"no_events", "event_pair_default", "event_pair_release_to_device", "event_after_only"};
    for (int mode = 0; mode < 4; ++mode)
        std::printf("{\"mode\": \"%s\", \"launches\": %d, \"rounds\": %d, \"wall_us_per_launch_median\": %.2f, "
                    "\"wall_us_min\": %.2f, \"event_us_median\": %.2f}\n",
                    names[mode], K, rounds, median(wall[mode]), *std::min_element(wall[mode].begin(), wall[mode].end()),
                    median(kern[mode]));
    return 0;
}
