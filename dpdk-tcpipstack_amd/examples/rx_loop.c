/*
 * rx_loop.c — the reference's rx loop (tcp_ip_stack/main.c:391-399) patched as in
 * INTEGRATION.md §2-§4, in plain C against include/rxg.h: bursts go through rxg_rx_burst
 * and rxg_rx_replay, whose hand-off table calls C handlers shaped like tcp_states.c's
 * (tcp_listen allocates a child TCB from a SYN, tcp_syn_rcv establishes it, a FIN closes a
 * flow, tcp_closed removes it), each mirroring its tcbs[] write with rxg_tcb_*.
 *
 *   rx_loop IN OUT BURST [verify]
 *   IN : u32 nrows; nrows x {i32 dport, i32 sport, u32 ipv4_dst (raw), u32 ipv4_src (host),
 *        u8 state, u8 live, u16 pad}; u32 nframes; nframes x {u16 len, len bytes}
 *   OUT: nframes x {u8 kind (0 none, 1 freed, 2 reset, 3 tcpswitch), u8 state, u16 pad,
 *        i32 tcb_idx}; then u32 ntcb and the final table in IN's row format; then the
 *        reference's rx counters i32 tcpnopcb, i32 tcpchecksumerror (tcp_in.c:18-19).
 *   verify: tcp_in.c:37-41 compiled in (RXG_OPS_VERIFY_TCP_CKSUM).
 * Exit status: 0 ok, 2 usage/input error, 3 rxg error (message on stderr; 3 without a GPU).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rxg.h"

enum { CLOSED = 0, LISTENING = 1, SYN_RECV = 3, ESTABLISHED = 4 };

struct row {
    int32_t dport, sport;
    uint32_t ipv4_dst, ipv4_src;
    uint8_t state, live;
    uint16_t pad;
};

struct out_rec {
    uint8_t kind, state;
    uint16_t pad;
    int32_t tcb_idx;
};

static struct row *tcbs;  /* tcbs[] and Ntcb of tcp_tcb.c:21-22 */
/* Defined here because this program links none of the reference's objects.  In the patched
   stack tcp_in.c (tcp_in.c:18-19) keeps defining them and the patch only declares them, through
   tcp_in.h:7,11. */
int tcpchecksumerror;     /* tcp_in.c:18, extern in tcp_in.h:7 */
int tcpnopcb;             /* tcp_in.c:19, extern in tcp_in.h:11 */
static int32_t ntcb, cap;
static rxg_ctx *g_rxg;
static struct out_rec *g_out;
static uint8_t **g_frames;
static uint32_t g_base, g_end;  /* the burst's frames */

static void mirror_upsert(int32_t i)
{
    rxg_tcb_tuple t = {tcbs[i].dport, tcbs[i].sport, tcbs[i].ipv4_dst, tcbs[i].ipv4_src, tcbs[i].state, 0,
                       (uint16_t)(i % 65535 + 1)};
    if (rxg_tcb_upsert(g_rxg, i, &t) != 0) fprintf(stderr, "rxg_tcb_upsert: %s\n", rxg_last_error());
}

/* the "mbuf" handed to the replay is the frame's index + 1 (an opaque non-NULL token) */
static uint32_t frame_index(void *mbuf) { return (uint32_t)(uintptr_t)mbuf - 1u; }

static void ops_free(void *u, void *m)
{
    (void)u;
    struct out_rec *o = &g_out[frame_index(m)];
    if (o->kind == 0) o->kind = 1;
}

static void ops_rst(void *u, void *ip, void *tcp)
{
    (void)u;
    (void)tcp;
    /* the frame whose IP header this is: search the burst (the reference's send_reset gets
       the headers, not the mbuf) */
    for (uint32_t i = g_base; i < g_end; ++i)
        if ((uint8_t *)ip == g_frames[i] + RXG_OFF_IP) {
            g_out[i].kind = 2;
            return;
        }
}

static int ops_switch(void *u, int32_t idx, uint8_t st, void *tcp, void *ip, void *m)
{
    (void)u;
    (void)ip;
    const uint8_t *f = (const uint8_t *)tcp - RXG_OFF_TCP;
    struct out_rec *o = &g_out[frame_index(m)];
    o->kind = 3;
    o->state = st;
    o->tcb_idx = idx;
    const uint8_t flags = f[47];
    if (st == LISTENING) { /* tcp_listen: child at Ntcb with the SYN's tuple */
        if (ntcb == cap) {
            cap *= 2;
            tcbs = realloc(tcbs, sizeof *tcbs * (size_t)cap);
        }
        const int32_t c = ntcb++;
        tcbs[c] = tcbs[idx];
        tcbs[c].sport = (f[34] << 8) | f[35];
        tcbs[c].ipv4_src = ((uint32_t)f[26] << 24) | ((uint32_t)f[27] << 16) | ((uint32_t)f[28] << 8) | f[29];
        tcbs[c].state = SYN_RECV;
        tcbs[c].live = 1;
        mirror_upsert(c);
    } else if (st == SYN_RECV) {
        tcbs[idx].state = ESTABLISHED;
        rxg_tcb_set_state(g_rxg, idx, ESTABLISHED);
    } else if (st == ESTABLISHED && (flags & RXG_TCP_FLAG_FIN)) {
        tcbs[idx].state = CLOSED;
        rxg_tcb_set_state(g_rxg, idx, CLOSED);
    } else if (st == CLOSED) { /* tcp_closed -> remove_tcb */
        tcbs[idx].live = 0;
        rxg_tcb_remove(g_rxg, idx);
    }
    return 0;
}

int main(int argc, char **argv)
{
    if (argc != 4 && !(argc == 5 && strcmp(argv[4], "verify") == 0)) {
        fprintf(stderr, "usage: rx_loop IN OUT BURST [verify]\n");
        return 2;
    }
    const uint32_t burst = (uint32_t)atoi(argv[3]);
    FILE *in = fopen(argv[1], "rb");
    uint32_t nrows = 0, n = 0;
    if (!in || burst == 0 || fread(&nrows, 4, 1, in) != 1) {
        fprintf(stderr, "rx_loop: bad input\n");
        return 2;
    }
    cap = nrows + 16;
    tcbs = calloc((size_t)cap, sizeof *tcbs);
    if (fread(tcbs, sizeof *tcbs, nrows, in) != nrows || fread(&n, 4, 1, in) != 1) return 2;
    ntcb = (int32_t)nrows;
    g_frames = calloc(n, sizeof *g_frames);
    uint16_t *lens = calloc(n, sizeof *lens);
    for (uint32_t i = 0; i < n; ++i) {
        if (fread(&lens[i], 2, 1, in) != 1) return 2;
        g_frames[i] = calloc(1, (size_t)lens[i] + 64);
        if (fread(g_frames[i], 1, lens[i], in) != lens[i]) return 2;
    }
    fclose(in);

    rxg_config cfg = {.device = 0, .max_batch = burst};
    if (rxg_init(&cfg, &g_rxg) != 0) {
        fprintf(stderr, "rxg_init: %s\n", rxg_last_error());
        return 3;
    }
    { /* the table as it stands before the loop (rxg_tcb_load; live = 0 is a NULL slot) */
        rxg_tcb_tuple *t = calloc((size_t)ntcb + 1, sizeof *t);
        uint8_t *live = calloc((size_t)ntcb + 1, 1);
        for (int32_t i = 0; i < ntcb; ++i) {
            t[i] = (rxg_tcb_tuple){tcbs[i].dport, tcbs[i].sport, tcbs[i].ipv4_dst, tcbs[i].ipv4_src, tcbs[i].state,
                                   0, (uint16_t)(i % 65535 + 1)};
            live[i] = tcbs[i].live;
        }
        if (rxg_tcb_load(g_rxg, t, live, ntcb) != 0) {
            fprintf(stderr, "rxg_tcb_load: %s\n", rxg_last_error());
            return 3;
        }
        free(t);
        free(live);
    }

    /* RX_LOOP_SERVER=1: the latency mode (rxg.h rxg_server_start), as INTEGRATION.md §2
       starts it for the reference's MAX_PKT_BURST loop; the loop below is unchanged */
    const char *srv = getenv("RX_LOOP_SERVER");
    if (srv && strcmp(srv, "1") == 0) {
        rxg_server_config sc = {RXG_REC8, 4u, burst, 0u, 0u, 0u};
        if (rxg_server_start(g_rxg, &sc) != 0) {
            fprintf(stderr, "rxg_server_start: %s\n", rxg_last_error());
            return 3;
        }
    }

    g_out = calloc(n, sizeof *g_out);
    for (uint32_t i = 0; i < n; ++i) g_out[i].tcb_idx = -1;
    rxg_pkt_view *views = calloc(burst, sizeof *views);
    rxg_rec8 *recs = calloc(burst, sizeof *recs); /* 8-byte records: all the replay reads */
    void **mbufs = calloc(burst, sizeof *mbufs), **frames = calloc(burst, sizeof *frames);
    rxg_handoff_ops ops = {.free_mbuf = ops_free,
                           .send_reset = ops_rst,
                           .tcpswitch = ops_switch,
                           .tcpnopcb = &tcpnopcb,
                           .tcpchecksumerror = &tcpchecksumerror,
                           .flags = argc == 5 ? RXG_OPS_VERIFY_TCP_CKSUM : 0u};
    for (uint32_t b0 = 0; b0 < n; b0 += burst) { /* l2fwd_main_loop, main.c:391-399 */
        const uint32_t nb = n - b0 < burst ? n - b0 : burst;
        g_base = b0;
        g_end = b0 + nb;
        for (uint32_t i = 0; i < nb; ++i) {
            views[i].buf_addr = g_frames[b0 + i];
            views[i].data_off = 0;
            views[i].data_len = lens[b0 + i];
            mbufs[i] = (void *)(uintptr_t)(b0 + i + 1);
            frames[i] = g_frames[b0 + i];
        }
        if (rxg_rx_burst(g_rxg, views, nb, RXG_REC8, recs) != 0 ||
            rxg_rx_replay(g_rxg, &ops, mbufs, frames, recs, nb, RXG_REC8) != 0) {
            fprintf(stderr, "rx: %s\n", rxg_last_error());
            return 3;
        }
    }
    FILE *out = fopen(argv[2], "wb");
    if (!out) return 2;
    fwrite(g_out, sizeof *g_out, n, out);
    fwrite(&ntcb, 4, 1, out);
    fwrite(tcbs, sizeof *tcbs, (size_t)ntcb, out);
    fwrite(&tcpnopcb, 4, 1, out);
    fwrite(&tcpchecksumerror, 4, 1, out);
    fclose(out);
    rxg_fini(g_rxg);
    return 0;
}
