/*
 * sanitize_oracle.c -- CPU driver for the oracle (oracle/rxg_oracle.c) under AddressSanitizer
 * and UndefinedBehaviorSanitizer (tests/test_sanitizers.py builds and runs it).
 *
 * Every frame lives in a heap block of exactly its data_len bytes, so any read past the
 * frame -- the reference's odd-length checksum over-read (ip.c:49-51), its fixed +14/+34
 * header offsets on short frames (ip.c:23-24, tcp_in.c:42-45), total_length beyond the
 * buffer -- is an ASan report, not a silent stale byte: the oracle must handle them the way
 * its header says (zero bytes at or past data_len, the over-read byte fed as zero).
 * Malformed frames (short, IHL != 5, total_length < 20 or > data_len, odd spans, ARP,
 * non-IPv4, non-TCP), TCB tables with NULL slots, duplicate tuples and listeners, the
 * batch, faithful (malloc + memcpy staging, ARP list walks) and tx forms are all run.
 *
 *   sanitize_oracle <seed> <frames>   ->  prints "ok <checksum>" and exits 0
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../oracle/rxg_oracle.h"

static uint64_t rng_state;
static uint32_t rnd(void)
{
    uint64_t x = (rng_state += 0x9E3779B97F4A7C15ull);
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return (uint32_t)((x ^ (x >> 31)) >> 16);
}

static void put16(uint8_t *b, uint32_t len, uint32_t at, uint32_t v)
{
    if (at < len) b[at] = (uint8_t)(v >> 8);
    if (at + 1 < len) b[at + 1] = (uint8_t)v;
}

/* A frame of `len` bytes: mostly well formed Eth/IPv4/TCP towards the table's flows. */
static void make_frame(uint8_t *f, uint32_t len, const rxg_tcb_tuple *t, int32_t ntcb)
{
    for (uint32_t i = 0; i < len; i++) f[i] = (uint8_t)rnd();
    const uint32_t kind = rnd() % 16;
    put16(f, len, 12, kind == 0 ? 0x0806 : kind == 1 ? 0x86DD : 0x0800);
    if (len > 14) f[14] = kind == 2 ? 0x46 : 0x45;
    uint32_t tl = len >= 14 ? len - 14 : 0;
    if (kind == 3) tl = rnd() % 20;             /* total_length < 20 */
    if (kind == 4) tl = len + rnd() % 200;      /* total_length past the buffer */
    put16(f, len, 16, tl);
    if (len > 23) f[23] = kind == 5 ? 17 : 6;
    const rxg_tcb_tuple *x = ntcb ? &t[rnd() % (uint32_t)ntcb] : NULL;
    if (x && kind >= 6) {
        const uint32_t src = x->ipv4_src, dst = x->ipv4_dst;
        put16(f, len, 26, src >> 16);
        put16(f, len, 28, src & 0xFFFF);
        for (int i = 0; i < 4; i++)
            if (30u + (uint32_t)i < len) f[30 + i] = (uint8_t)(dst >> (8 * i)); /* raw as stored */
        put16(f, len, 34, (uint32_t)x->sport & 0xFFFF);
        put16(f, len, 36, (uint32_t)x->dport & 0xFFFF);
    }
    if (len > 46) f[46] = (uint8_t)((5 + rnd() % 11) << 4);
    if (len > 47) f[47] = (uint8_t)(rnd() % 2 ? 0x02 : 0x10);
}

int main(int argc, char **argv)
{
    rng_state = argc > 1 ? strtoull(argv[1], NULL, 10) : 1;
    const uint32_t nframes = argc > 2 ? (uint32_t)strtoul(argv[2], NULL, 10) : 20000;

    /* table: listeners, NULL slots, duplicates, host-order dst, out-of-range int ports */
    const int32_t ntcb = 300;
    rxg_tcb_tuple *t = calloc((size_t)ntcb, sizeof *t);
    uint8_t *live = calloc((size_t)ntcb, 1);
    for (int32_t i = 0; i < ntcb; i++) {
        t[i].dport = (int32_t)(rnd() % 4 == 0 ? 80 : 1024 + rnd() % 3000);
        t[i].sport = (int32_t)(1024 + rnd() % 60000);
        t[i].ipv4_dst = rnd() % 8 == 0 ? 0xC0A84E02u : 0x024EA8C0u;
        t[i].ipv4_src = 0x0A000000u | (rnd() & 0xFFFF);
        t[i].state = (uint8_t)(rnd() % 7);
        t[i].identifier = (uint16_t)(i + 1);
        live[i] = rnd() % 10 != 0;
        if (i > 10 && rnd() % 20 == 0) t[i] = t[rnd() % (uint32_t)i];       /* duplicate tuple */
        if (rnd() % 50 == 0) t[i].sport = -5 - (int32_t)(rnd() % 9);        /* int port < 0 */
    }

    uint64_t acc = 0, cnt[RXG_NCOUNTERS];
    memset(cnt, 0, sizeof cnt);
    /* one frame at a time, each in an exact-size heap block */
    for (uint32_t k = 0; k < nframes; k++) {
        const uint32_t len = k % 7 == 0 ? rnd() % 64 : rnd() % 2101;
        uint8_t *f = malloc(len ? len : 1);
        make_frame(f, len, t, ntcb);
        rxg_rec48 r;
        orc_rx_one(f, len, t, live, ntcb, &r);
        orc_count_record(&r, len, cnt);
        acc = acc * 31 + r.c.verdict + (uint64_t)r.c.tcb_idx + r.c.ip_cksum + r.c.tcp_cksum;
        orc_tx_cksum_one(f, len);
        acc = acc * 31 + (len > 51 ? f[50] : 0);
        free(f);
        /* calculate_checksum's own contract: an odd span provides the byte after it */
        const uint32_t span = rnd() % 1600;
        uint8_t *s = malloc(span + (span & 1u) + 1);
        for (uint32_t i = 0; i < span; i++) s[i] = (uint8_t)rnd();
        s[span] = 0;
        acc += orc_calculate_checksum(s, (int)span);
        free(s);
    }

    /* the batch forms over an exact-size arena of 64-byte slots */
    const uint32_t n = 4096;
    uint32_t *off = malloc(n * sizeof *off);
    uint16_t *lens = malloc(n * sizeof *lens);
    uint64_t slots = 0;
    for (uint32_t i = 0; i < n; i++) {
        lens[i] = (uint16_t)(i % 5 == 0 ? rnd() % 65 : rnd() % 1600);
        off[i] = (uint32_t)slots;
        slots += (lens[i] + 63u) / 64u + (lens[i] == 0);
    }
    uint8_t *arena = malloc(slots * 64);
    memset(arena, 0, slots * 64);
    for (uint32_t i = 0; i < n; i++) make_frame(arena + (size_t)off[i] * 64, lens[i], t, ntcb);
    rxg_rec48 *out = malloc(n * sizeof *out), *out2 = malloc(n * sizeof *out2);
    uint64_t c1[RXG_NCOUNTERS], c2[RXG_NCOUNTERS];
    memset(c1, 0, sizeof c1);
    memset(c2, 0, sizeof c2);
    orc_rx_batch(arena, off, lens, n, t, live, ntcb, out, c1);
    orc_arp_reset();
    orc_rx_batch_faithful(arena, off, lens, n, t, live, ntcb, out2, c2);
    if (memcmp(out, out2, n * sizeof *out) != 0 || memcmp(c1, c2, sizeof c1) != 0) {
        printf("FAIL faithful and fast batch forms differ\n");
        return 1;
    }
    orc_tx_cksum_batch(arena, off, lens, n);
    orc_arp_reset();
    for (uint32_t i = 0; i < n; i++) acc = acc * 31 + out[i].c.verdict + out[i].c.tcp_cksum;
    free(out);
    free(out2);
    free(arena);
    free(off);
    free(lens);
    free(t);
    free(live);
    printf("ok %llu\n", (unsigned long long)acc);
    return 0;
}
