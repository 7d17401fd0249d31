/*
 * churn_bench.c — what sequential equivalence costs under connection churn: the reference's
 * rx loop (tcp_ip_stack/main.c:391-399) as rxg_rx_burst_dev + rxg_rx_replay, with C handlers
 * shaped like tcp_states.c's that write tcbs[] inside the burst:
 *   tcp_listen   (tcp_states.c:150-207): a SYN to the listener appends a child (SYN_RECV)
 *   tcp_syn_rcv  (:45-91): the client's ACK establishes it
 *   tcp_established + FIN: the flow goes CLOSED; its next segment hits tcp_closed, which
 *                removes the TCB (remove_tcb, tcp_tcb.c:175-186)
 * Every write is mirrored with rxg_tcb_*; later packets of the burst that the write affects
 * are re-classified by the replay before their handler runs.
 *
 *   churn_bench NFLOWS BURST STEPS CHURN_PER_MILLE [device]
 * Each step: BURST 64-byte frames (Eth/IPv4/TCP, 10 payload bytes), ACKs of established flows
 * chosen uniformly; CHURN_PER_MILLE of them start a churn event: half a new client's SYN with
 * its ACK later in the burst, half an established flow's FIN with its next segment later.
 * The batch is copied into HBM (not timed), then timed: the burst (kernel, synchronous), the
 * record copy back, and the replay.  "device": RXG_CFG_REPLAY_ON_DEVICE.
 * Prints one JSON line.  Exit 3 on an rxg error.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rxg.h"

enum { CLOSED = 0, LISTENING = 1, SYN_RECV = 3, ESTABLISHED = 4 };
enum { FRAME = 64 };

static rxg_ctx *g;
static rxg_tcb_tuple *tcbs; /* tcbs[] / Ntcb of tcp_tcb.c:21-22 (host copy) */
static uint8_t *live;
static int32_t ntcb, cap;
static uint64_t n_switch, n_rst, n_alloc, n_remove;

static double now_us(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec / 1e3;
}

static uint64_t rng_state = 0x5EED0003ull;
static uint64_t rnd(void)
{
    uint64_t x = (rng_state += 0x9E3779B97F4A7C15ull);
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

static void die(const char *what)
{
    fprintf(stderr, "%s: %s\n", what, rxg_last_error());
    exit(3);
}

/* RFC 1071 sum of big-endian words (the reference's calculate_checksum, ip.c:44-59) */
static uint16_t csum(const uint8_t *p, int n, uint32_t s)
{
    for (int i = 0; i + 1 < n; i += 2) s += (uint32_t)(p[i] << 8 | p[i + 1]);
    if (n & 1) s += (uint32_t)p[n - 1] << 8;
    while (s >> 16) s = (s & 0xFFFF) + (s >> 16);
    return (uint16_t)~s;
}

static void build(uint8_t *f, uint32_t src, uint16_t sport, uint16_t dport, uint8_t flags, uint32_t seq)
{
    static const uint8_t dst[4] = {192, 168, 78, 2};
    memset(f, 0, FRAME);
    f[12] = 0x08;                                   /* IPv4 */
    f[14] = 0x45;
    f[16] = 0; f[17] = FRAME - 14;                  /* total_length 50 */
    f[22] = 64; f[23] = 6;
    f[26] = src >> 24; f[27] = src >> 16; f[28] = src >> 8; f[29] = src;
    memcpy(f + 30, dst, 4);
    f[34] = sport >> 8; f[35] = sport; f[36] = dport >> 8; f[37] = dport;
    f[38] = seq >> 24; f[39] = seq >> 16; f[40] = seq >> 8; f[41] = seq;
    f[46] = 0x50; f[47] = flags; f[48] = 0xFF; f[49] = 0xFF;
    for (int i = 54; i < FRAME; ++i) f[i] = (uint8_t)(seq + i);
    const uint16_t ic = csum(f + 14, 20, 0);
    f[24] = ic >> 8; f[25] = ic;
    /* pseudo {src, dst, 0, 6, tcp length} || segment, as ip_out (ip.c:109-118) */
    uint32_t ps = ((uint32_t)f[26] << 8 | f[27]) + ((uint32_t)f[28] << 8 | f[29]) + ((uint32_t)f[30] << 8 | f[31]) +
                  ((uint32_t)f[32] << 8 | f[33]) + 6 + (FRAME - 34);
    const uint16_t tc = csum(f + 34, FRAME - 34, ps);
    f[50] = tc >> 8; f[51] = tc;
}

static void mirror(int32_t i)
{
    if (rxg_tcb_upsert(g, i, &tcbs[i]) != 0) die("rxg_tcb_upsert");
}

static void ops_free(void *u, void *m) { (void)u; (void)m; }
static void ops_rst(void *u, void *ip, void *tcp) { (void)u; (void)ip; (void)tcp; ++n_rst; }

static int ops_switch(void *u, int32_t idx, uint8_t st, void *tcp, void *ip, void *m)
{
    (void)u; (void)ip; (void)m;
    const uint8_t *f = (const uint8_t *)tcp - RXG_OFF_TCP;
    ++n_switch;
    if (st == LISTENING) { /* tcp_listen: child at Ntcb with the SYN's tuple */
        if (ntcb == cap) {
            cap *= 2;
            tcbs = realloc(tcbs, sizeof *tcbs * (size_t)cap);
            live = realloc(live, (size_t)cap);
        }
        const int32_t c = ntcb++;
        tcbs[c] = tcbs[idx];
        tcbs[c].sport = (f[34] << 8) | f[35];
        tcbs[c].ipv4_src = ((uint32_t)f[26] << 24) | ((uint32_t)f[27] << 16) | ((uint32_t)f[28] << 8) | f[29];
        tcbs[c].state = SYN_RECV;
        tcbs[c].identifier = (uint16_t)(c % 65535 + 1);
        live[c] = 1;
        mirror(c);
        ++n_alloc;
    } else if (st == SYN_RECV) { /* tcp_syn_rcv */
        tcbs[idx].state = ESTABLISHED;
        if (rxg_tcb_set_state(g, idx, ESTABLISHED)) die("rxg_tcb_set_state");
    } else if (st == ESTABLISHED && (f[47] & RXG_TCP_FLAG_FIN)) {
        tcbs[idx].state = CLOSED;
        if (rxg_tcb_set_state(g, idx, CLOSED)) die("rxg_tcb_set_state");
    } else if (st == CLOSED) { /* tcp_closed -> remove_tcb */
        live[idx] = 0;
        if (rxg_tcb_remove(g, idx)) die("rxg_tcb_remove");
        ++n_remove;
    }
    return 0;
}

int main(int argc, char **argv)
{
    if (argc < 5 || argc > 6) {
        fprintf(stderr, "usage: churn_bench NFLOWS BURST STEPS CHURN_PER_MILLE [device]\n");
        return 2;
    }
    const int32_t nflows = atoi(argv[1]);
    const uint32_t burst = (uint32_t)atoi(argv[2]);
    const int steps = atoi(argv[3]), permille = atoi(argv[4]);
    const int on_device = argc == 6 && strcmp(argv[5], "device") == 0;
    rxg_config cfg = {.device = 0, .flags = on_device ? RXG_CFG_REPLAY_ON_DEVICE : 0u};
    if (rxg_init(&cfg, &g) != 0) die("rxg_init");

    cap = nflows + 1 + 1024;
    tcbs = calloc((size_t)cap, sizeof *tcbs);
    live = calloc((size_t)cap, 1);
    const uint32_t dst_raw = 192u | (168u << 8) | (78u << 16) | (2u << 24);
    tcbs[0] = (rxg_tcb_tuple){80, 0, dst_raw, 0, LISTENING, 0, 1};
    live[0] = 1;
    for (int32_t f = 0; f < nflows; ++f) {
        tcbs[1 + f] = (rxg_tcb_tuple){80, 1024 + f % 64511, dst_raw, (10u << 24) | (uint32_t)f, ESTABLISHED, 0,
                                      (uint16_t)((f + 1) % 65535 + 1)};
        live[1 + f] = 1;
    }
    ntcb = nflows + 1;
    if (rxg_tcb_load(g, tcbs, live, ntcb) != 0) die("rxg_tcb_load");

    uint8_t *h_frames = NULL;
    uint32_t *h_off = NULL;
    uint16_t *h_len = NULL;
    rxg_rec16 *h_rec = NULL;
    if (rxg_host_alloc_pinned(g, (uint64_t)burst * FRAME, (void **)&h_frames) ||
        rxg_host_alloc_pinned(g, burst * 4ull, (void **)&h_off) ||
        rxg_host_alloc_pinned(g, burst * 2ull, (void **)&h_len) ||
        rxg_host_alloc_pinned(g, burst * 16ull, (void **)&h_rec))
        die("rxg_host_alloc_pinned");
    void *d_frames, *d_off, *d_len, *d_rec;
    if (rxg_dev_alloc(g, (uint64_t)burst * FRAME, &d_frames) || rxg_dev_alloc(g, burst * 4ull, &d_off) ||
        rxg_dev_alloc(g, burst * 2ull, &d_len) || rxg_dev_alloc(g, burst * 16ull, &d_rec))
        die("rxg_dev_alloc");
    void **mbufs = calloc(burst, sizeof *mbufs), **frames = calloc(burst, sizeof *frames);
    for (uint32_t i = 0; i < burst; ++i) {
        h_off[i] = i;
        h_len[i] = FRAME;
        mbufs[i] = (void *)(uintptr_t)(i + 1);
        frames[i] = h_frames + (size_t)i * FRAME;
    }
    rxg_handoff_ops ops = {.free_mbuf = ops_free, .send_reset = ops_rst, .tcpswitch = ops_switch};
    double t_burst = 0, t_d2h = 0, t_replay = 0;
    uint32_t client = 0;
    const int warm = 2;
    uint64_t st0[4] = {0}, st1[4] = {0};
    for (int s = 0; s < warm + steps; ++s) {
        /* the step's traffic */
        for (uint32_t i = 0; i < burst; ++i) {
            const int32_t f = (int32_t)(rnd() % (uint64_t)nflows);
            build(h_frames + (size_t)i * FRAME, (10u << 24) | (uint32_t)f, (uint16_t)(1024 + f % 64511), 80, 0x10,
                  (uint32_t)rnd());
        }
        /* CHURN_PER_MILLE of the frames start an event, accumulated across steps (a burst of
           32 at 1 % has one every ~3 bursts) */
        const uint64_t acc = (uint64_t)burst * (uint64_t)permille;
        const uint32_t events = (uint32_t)(((uint64_t)(s + 1) * acc) / 1000u - ((uint64_t)s * acc) / 1000u);
        for (uint32_t e = 0; e < events && burst >= 2; ++e) {
            const uint32_t p1 = (uint32_t)(rnd() % (burst - 1)), p2 = p1 + 1 + (uint32_t)(rnd() % (burst - 1 - p1));
            if (e & 1) { /* an established flow's FIN, then its next segment (-> tcp_closed) */
                const int32_t f = (int32_t)(rnd() % (uint64_t)nflows);
                const uint32_t src = (10u << 24) | (uint32_t)f;
                build(h_frames + (size_t)p1 * FRAME, src, (uint16_t)(1024 + f % 64511), 80, 0x11, (uint32_t)rnd());
                build(h_frames + (size_t)p2 * FRAME, src, (uint16_t)(1024 + f % 64511), 80, 0x10, (uint32_t)rnd());
            } else { /* a new client: SYN to the listener, then its ACK */
                const uint32_t src = (172u << 24) | (16u << 16) | (client & 0xFFFF);
                const uint16_t sport = (uint16_t)(1024 + (client >> 16) % 60000);
                ++client;
                build(h_frames + (size_t)p1 * FRAME, src, sport, 80, 0x02, (uint32_t)rnd());
                build(h_frames + (size_t)p2 * FRAME, src, sport, 80, 0x10, (uint32_t)rnd());
            }
        }
        if (rxg_memcpy_h2d(g, d_frames, h_frames, (uint64_t)burst * FRAME, NULL) ||
            rxg_memcpy_h2d(g, d_off, h_off, burst * 4ull, NULL) || rxg_memcpy_h2d(g, d_len, h_len, burst * 2ull, NULL) ||
            rxg_sync(g))
            die("h2d");
        if (s == warm) rxg_replay_stats(g, st0);
        rxg_dev_batch b = {d_frames, d_off, d_len, burst, RXG_REC16, d_rec};
        const double t0 = now_us();
        if (rxg_rx_burst_dev(g, &b, NULL) || rxg_sync(g)) die("rxg_rx_burst_dev");
        const double t1 = now_us();
        if (rxg_memcpy_d2h(g, h_rec, d_rec, burst * 16ull, NULL) || rxg_sync(g)) die("d2h");
        const double t2 = now_us();
        if (rxg_rx_replay(g, &ops, mbufs, frames, h_rec, burst, RXG_REC16)) die("rxg_rx_replay");
        const double t3 = now_us();
        if (s >= warm) {
            t_burst += t1 - t0;
            t_d2h += t2 - t1;
            t_replay += t3 - t2;
        }
    }
    rxg_replay_stats(g, st1);
    const double per = (t_burst + t_d2h + t_replay) / steps;
    printf("{\"lib\": \"%s\", \"nflows\": %d, \"burst\": %u, \"steps\": %d, \"churn_per_mille\": %d, \"fixups\": \"%s\", "
           "\"burst_us\": %.2f, \"d2h_us\": %.2f, \"replay_us\": %.2f, \"mpps_with_replay\": %.3f, "
           "\"stale_per_burst\": %.1f, \"host_fixups_per_burst\": %.1f, \"device_fixups_per_burst\": %.1f, "
           "\"device_launches_per_burst\": %.2f, \"ntcb_end\": %d, \"allocs\": %llu, \"removes\": %llu, "
           "\"resets\": %llu, \"dispatches\": %llu}\n",
           rxg_build_info(), nflows, burst, steps, permille, on_device ? "device" : "host", t_burst / steps, t_d2h / steps,
           t_replay / steps, burst / per, (double)(st1[0] - st0[0]) / steps, (double)(st1[1] - st0[1]) / steps,
           (double)(st1[2] - st0[2]) / steps, (double)(st1[3] - st0[3]) / steps, ntcb, (unsigned long long)n_alloc,
           (unsigned long long)n_remove, (unsigned long long)n_rst, (unsigned long long)n_switch);
    rxg_fini(g);
    return 0;
}
