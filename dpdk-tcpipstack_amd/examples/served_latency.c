/*
 * served_latency.c — the reference's rx call site (tcp_ip_stack/main.c:391-399, bursts of
 * MAX_PKT_BURST = 32, :116) timed in C: each iteration is one rxg_rx_burst over host frames
 * (rte_mbuf-shaped views) plus rxg_rx_replay with empty handlers, i.e. what the patched loop
 * of INTEGRATION.md §2 spends per burst beside its own handlers.  Latency mode (the persistent
 * server, rxg_server_start) and the launched path, one after the other, same frames.
 *
 *   served_latency FRAME_BYTES BURST ITERS [PEERS] [BLOCKS]
 * Frames: Eth/IPv4/TCP ACKs with valid checksums to 192.168.78.2:80 from PEERS established
 * flows (default 1: the one-peer case of HISTORY.md §6.R3a); the TCB table holds the listener
 * and those flows.  Prints one JSON line: median / p10 / p90 microseconds per burst.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rxg.h"

static rxg_ctx *g;

static double now_us(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec / 1e3;
}

static void die(const char *what)
{
    fprintf(stderr, "%s: %s\n", what, rxg_last_error());
    exit(3);
}

/* RFC 1071 over big-endian words (ip.c:44-59) */
static uint16_t csum(const uint8_t *p, int n, uint32_t s)
{
    for (int i = 0; i + 1 < n; i += 2) s += (uint32_t)(p[i] << 8 | p[i + 1]);
    if (n & 1) s += (uint32_t)p[n - 1] << 8;
    while (s >> 16) s = (s & 0xFFFF) + (s >> 16);
    return (uint16_t)~s;
}

static void build(uint8_t *f, int len, uint32_t src, uint16_t sport, uint32_t seq)
{
    static const uint8_t dst[4] = {192, 168, 78, 2};
    memset(f, 0, (size_t)len);
    f[12] = 0x08;
    f[14] = 0x45;
    f[16] = (uint8_t)((len - 14) >> 8); f[17] = (uint8_t)(len - 14);
    f[22] = 64; f[23] = 6;
    f[26] = src >> 24; f[27] = src >> 16; f[28] = src >> 8; f[29] = src;
    memcpy(f + 30, dst, 4);
    f[34] = sport >> 8; f[35] = sport; f[36] = 0; f[37] = 80;
    f[38] = seq >> 24; f[39] = seq >> 16; f[40] = seq >> 8; f[41] = seq;
    f[46] = 0x50; f[47] = 0x10; f[48] = 0xFF; f[49] = 0xFF;
    for (int i = 54; i < len; ++i) f[i] = (uint8_t)(seq + i);
    const uint16_t ic = csum(f + 14, 20, 0);
    f[24] = ic >> 8; f[25] = ic;
    const uint32_t ps = ((uint32_t)f[26] << 8 | f[27]) + ((uint32_t)f[28] << 8 | f[29]) +
                        ((uint32_t)f[30] << 8 | f[31]) + ((uint32_t)f[32] << 8 | f[33]) + 6 + (uint32_t)(len - 34);
    const uint16_t tc = csum(f + 34, len - 34, ps);
    f[50] = tc >> 8; f[51] = tc;
}

static void ops_free(void *u, void *m) { (void)u; (void)m; }
static void ops_rst(void *u, void *ip, void *tcp) { (void)u; (void)ip; (void)tcp; }
static int ops_switch(void *u, int32_t idx, uint8_t st, void *tcp, void *ip, void *m)
{
    (void)u; (void)idx; (void)st; (void)tcp; (void)ip; (void)m;
    return 0;
}

static int cmp(const void *a, const void *b)
{
    const double x = *(const double *)a, y = *(const double *)b;
    return (x > y) - (x < y);
}

/* ITERS bursts, each timed: rxg_rx_burst + rxg_rx_replay (t), the replay alone (r); sorted */
static void run(const rxg_pkt_view *views, void **mbufs, void **frames, uint32_t burst, int iters, rxg_rec8 *rec,
                const rxg_handoff_ops *ops, double *t, double *r)
{
    for (int i = -100; i < iters; ++i) {
        const double t0 = now_us();
        if (rxg_rx_burst(g, views, burst, RXG_REC8, rec)) die("rxg_rx_burst");
        const double t1 = now_us();
        if (rxg_rx_replay(g, ops, mbufs, frames, rec, burst, RXG_REC8)) die("rxg_rx_replay");
        const double t2 = now_us();
        if (i >= 0) {
            t[i] = t2 - t0;
            r[i] = t2 - t1;
        }
    }
    qsort(t, (size_t)iters, sizeof *t, cmp);
    qsort(r, (size_t)iters, sizeof *r, cmp);
}

int main(int argc, char **argv)
{
    if (argc < 4 || argc > 6) {
        fprintf(stderr, "usage: served_latency FRAME_BYTES BURST ITERS [PEERS] [BLOCKS]\n");
        return 2;
    }
    const int len = atoi(argv[1]);
    const uint32_t burst = (uint32_t)atoi(argv[2]);
    const int iters = atoi(argv[3]);
    const int32_t peers = argc > 4 ? atoi(argv[4]) : 1;
    const uint32_t blocks = argc > 5 ? (uint32_t)atoi(argv[5]) : 1u;
    if (len < 54 || len > 9000 || burst == 0 || burst > 4096 || iters < 1 || peers < 1) return 2;
    rxg_config cfg = {.device = 0, .max_batch = burst, .max_bytes = burst * ((uint32_t)len + 64u)};
    if (rxg_init(&cfg, &g) != 0) die("rxg_init");

    rxg_tcb_tuple *tcbs = calloc((size_t)peers + 1, sizeof *tcbs);
    uint8_t *live = calloc((size_t)peers + 1, 1);
    const uint32_t dst_raw = 192u | (168u << 8) | (78u << 16) | (2u << 24);
    tcbs[0] = (rxg_tcb_tuple){80, 0, dst_raw, 0, 1 /* LISTENING */, 0, 1};
    live[0] = 1;
    for (int32_t f = 0; f < peers; ++f) {
        tcbs[1 + f] = (rxg_tcb_tuple){80, 1024 + f % 64511, dst_raw, (10u << 24) | (uint32_t)f, 4 /* ESTABLISHED */, 0,
                                      (uint16_t)((f + 1) % 65535 + 1)};
        live[1 + f] = 1;
    }
    if (rxg_tcb_load(g, tcbs, live, peers + 1) != 0) die("rxg_tcb_load");

    uint8_t *buf = malloc((size_t)burst * (size_t)len);
    rxg_pkt_view *views = calloc(burst, sizeof *views);
    void **mbufs = calloc(burst, sizeof *mbufs), **frames = calloc(burst, sizeof *frames);
    for (uint32_t i = 0; i < burst; ++i) {
        const int32_t f = (int32_t)(i % (uint32_t)peers);
        build(buf + (size_t)i * (size_t)len, len, (10u << 24) | (uint32_t)f, (uint16_t)(1024 + f % 64511), i * 7919u);
        views[i] = (rxg_pkt_view){buf + (size_t)i * (size_t)len, 0, (uint16_t)len, 0};
        mbufs[i] = (void *)(uintptr_t)(i + 1);
        frames[i] = buf + (size_t)i * (size_t)len;
    }
    rxg_rec8 *rec = calloc(burst, sizeof *rec);
    rxg_handoff_ops ops = {.free_mbuf = ops_free, .send_reset = ops_rst, .tcpswitch = ops_switch};
    double *ts = malloc(sizeof(double) * (size_t)iters), *tl = malloc(sizeof(double) * (size_t)iters);
    double *rs = malloc(sizeof(double) * (size_t)iters), *rl = malloc(sizeof(double) * (size_t)iters);

    rxg_server_config sc = {RXG_REC8, blocks, burst, burst * ((uint32_t)len + 64u), 0u, 0u};
    if (rxg_server_start(g, &sc) != 0) die("rxg_server_start");
    run(views, mbufs, frames, burst, iters, rec, &ops, ts, rs);
    const int placement = rxg_server_placement(g);
    if (rxg_server_stop(g) != 0) die("rxg_server_stop");
    for (uint32_t i = 0; i < burst; ++i)
        if (rec[i].w0 == 0u && rec[i].w1 == 0u) die("empty record");
    run(views, mbufs, frames, burst, iters, rec, &ops, tl, rl);

    printf("{\"frame_bytes\": %d, \"burst\": %u, \"peers\": %d, \"iters\": %d, \"blocks\": %u, \"placement\": \"%s\", "
           "\"served_us\": {\"p10\": %.2f, \"median\": %.2f, \"p90\": %.2f}, "
           "\"launched_us\": {\"p10\": %.2f, \"median\": %.2f, \"p90\": %.2f}, "
           "\"replay_us_median\": {\"served\": %.2f, \"launched\": %.2f}, \"timing\": \"C, clock_gettime around "
           "rxg_rx_burst + rxg_rx_replay (empty handlers)\"}\n",
           len, burst, peers, iters, blocks, placement == RXG_SRV_DEVICE ? "device" : "host", ts[iters / 10],
           ts[iters / 2], ts[iters * 9 / 10], tl[iters / 10], tl[iters / 2], tl[iters * 9 / 10], rs[iters / 2],
           rl[iters / 2]);
    rxg_fini(g);
    return 0;
}
