/*
 * rxg_oracle.c — TEST INFRASTRUCTURE ONLY (see rxg_oracle.h for the pinning status).
 *
 * CPU restatement of the reference receive path of rajneshrat/dpdk-tcpipstack, used as
 * the checker for rxg's HIP kernels and as the timed CPU baseline ("port").  Each
 * function cites the reference lines it restates.  Defined deviations where the
 * reference has undefined behaviour (both the oracle and rxg follow them):
 *   - bytes at or beyond data_len read as zero (the reference reads stale mbuf memory);
 *   - odd-length checksum spans read one zero byte past the end (ip.c:49-51 over-read);
 *   - findtcb pass 2 skips a removed (NULL) slot and flags it, where the reference
 *     dereferences NULL (tcp_tcb.c:160-162).
 */
#include "rxg_oracle.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- checksum --- */

/* ip.c:44-59: sum of big-endian 16-bit words, i < (len+1)/2, then fold and invert. */
uint16_t orc_calculate_checksum(const unsigned char *data, int len)
{
    const uint8_t *p = data;
    uint32_t sum = 0;
    int words = (len + 1) / 2;
    for (int i = 0; i < words; i++) {
        uint16_t w = (uint16_t)((p[0] << 8) | p[1]);
        sum += w;
        p += 2;
    }
    while (sum & 0xffff0000u)
        sum = (sum & 0xffffu) + (sum >> 16);
    return (uint16_t)~sum;
}

/* -------------------------------------------------------------- byte access --- */

static inline uint8_t byte_at(const uint8_t *f, uint32_t len, uint32_t i)
{
    return i < len ? f[i] : 0;
}

static inline uint32_t be32(const uint8_t *b)
{
    return ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
}

static inline uint32_t le32(const uint8_t *b)
{
    return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
}

/* ------------------------------------------------------------------ logger --- */

/* logger.c:31-43: log_print tests LogFeature[f].Enable and the level; InitLogger leaves
   every feature disabled (logger.c:9-23), so each call is a call + branch.  log_print lives
   in its own translation unit in the reference, so no build of it can drop those calls:
   noipa (and a feature table the optimiser cannot prove zero) keeps every call here too,
   at -O2 as at -O0. */
enum { ORC_LOG_ARP = 0, ORC_LOG_IP = 1, ORC_LOG_TCP = 2, ORC_LOG_TCB = 9, ORC_LOG_N = 11 };
struct orc_logfeat {
    int level;
    uint8_t enable;
};
struct orc_logfeat orc_logfeature[ORC_LOG_N];

__attribute__((noinline, noipa)) static void orc_log(int feature, int level, const char *fmt, ...)
{
    if (orc_logfeature[feature].enable == 1 && orc_logfeature[feature].level >= level) {
        va_list ap;
        va_start(ap, fmt);
        vfprintf(stderr, fmt, ap);
        va_end(ap);
    }
}

/* ---------------------------------------------------------------- findtcb --- */

/* tcp_tcb.c:127-173.  Pass 1: first live slot whose (dport, sport, ipv4_dst RAW,
   ipv4_src HOST) equals the packet's.  Pass 2: first slot in LISTENING with that dport. */
static int32_t orc_findtcb(const rxg_tcb_tuple *tcbs, const uint8_t *live, int32_t ntcb,
                           uint16_t dport, uint16_t sport, uint32_t dst_raw,
                           uint32_t src_host, int *listen_hit, int *null_slot, int faithful)
{
    for (int32_t i = 0; i < ntcb; i++) {
        if (!live[i])
            continue;
        const rxg_tcb_tuple *t = &tcbs[i];
        if (faithful) /* tcp_tcb.c:150, one call per scanned TCB */
            orc_log(ORC_LOG_TCB, 2, "searching for tcb %u %u %d %d   found %u %u %d %d for %d\n",
                    src_host, dst_raw, sport, dport, t->ipv4_src, t->ipv4_dst, t->sport,
                    t->dport, t->identifier);
        if (t->dport == (int32_t)dport && t->sport == (int32_t)sport &&
            t->ipv4_dst == dst_raw && t->ipv4_src == src_host)
            return i;
    }
    for (int32_t i = 0; i < ntcb; i++) {
        if (!live[i]) { /* reference: NULL->state, undefined; rxg skips and flags */
            *null_slot = 1;
            continue;
        }
        if (tcbs[i].state == RXG_LISTENING && tcbs[i].dport == (int32_t)dport) {
            *listen_hit = 1;
            return i;
        }
    }
    return -1;
}

/* ------------------------------------------------------------ tcp checksum --- */

/* The rx "verify" is defined from ip_out's own construction (ip.c:109-118):
   pseudo = {src_addr, dst_addr, 0, 6, htons(total_length - 20)} || tcp segment. */
static uint16_t orc_tcp_checksum(const uint8_t *f, uint32_t len, uint16_t tl, int faithful,
                                 uint8_t *scratch)
{
    uint32_t seglen = tl >= 20 ? (uint32_t)tl - 20u : 0u;
    uint16_t l16 = (uint16_t)(tl - 20);
    uint8_t pseudo[12];
    for (int i = 0; i < 4; i++) {
        pseudo[i] = byte_at(f, len, 26 + i);
        pseudo[4 + i] = byte_at(f, len, 30 + i);
    }
    pseudo[8] = 0;
    pseudo[9] = RXG_IPPROTO_TCP;
    pseudo[10] = (uint8_t)(l16 >> 8);
    pseudo[11] = (uint8_t)(l16 & 0xff);

    uint8_t *temp = faithful ? (uint8_t *)malloc(12 + seglen + 1) : scratch; /* ip.c:114 */
    memcpy(temp, pseudo, 12);                                                   /* ip.c:116 */
    uint32_t avail = len > 34 ? len - 34 : 0;
    uint32_t ncopy = seglen < avail ? seglen : avail;
    memcpy(temp + 12, f + 34, ncopy);                                           /* ip.c:117 */
    memset(temp + 12 + ncopy, 0, seglen - ncopy + 1); /* zero tail + the over-read byte */
    uint16_t ck = orc_calculate_checksum(temp, (int)(12 + seglen));            /* ip.c:118 */
    if (faithful)
        free(temp);
    return ck;
}

/* ------------------------------------------------------------------- ARP list --- */

/* arp.c: singly linked IP->MAC list, walked by print_arp_table (arp.c:263-280) and
   get_mac (:215-238), appended by add_mac (:282-317). */
struct orc_arp_map {
    uint32_t ipv4;
    uint8_t mac[6];
    struct orc_arp_map *next;
};
static struct orc_arp_map *orc_arp_list;
static int orc_arp_n;

void orc_arp_reset(void)
{
    struct orc_arp_map *p = orc_arp_list;
    while (p) {
        struct orc_arp_map *n = p->next;
        free(p);
        p = n;
    }
    orc_arp_list = NULL;
    orc_arp_n = 0;
}

int orc_arp_count(void) { return orc_arp_n; }

static void orc_print_add(uint32_t ip) /* arp.c:147-160: 7 log calls */
{
    for (int i = 0; i < 4; i++) {
        orc_log(ORC_LOG_ARP, 4, "%u", ip >> 24);
        ip <<= 8;
        if (i != 3)
            orc_log(ORC_LOG_ARP, 4, ".");
    }
}

static void orc_print_arp_table(void) /* arp.c:263-280 */
{
    orc_log(ORC_LOG_ARP, 2, "printing arp table.\n");
    for (struct orc_arp_map *t = orc_arp_list; t; t = t->next) {
        orc_log(ORC_LOG_ARP, 2, " IP = ");
        orc_print_add(t->ipv4);
        orc_log(ORC_LOG_ARP, 2, " mac = ");
        for (int i = 0; i < 6; i++)
            orc_log(ORC_LOG_ARP, 2, "%x::", t->mac[i]);
        orc_log(ORC_LOG_ARP, 2, "\n");
    }
}

static int orc_get_mac(uint32_t ip, uint8_t *mac) /* arp.c:215-238 */
{
    orc_log(ORC_LOG_ARP, 4, "Getting mac for ");
    orc_print_add(ip);
    for (struct orc_arp_map *t = orc_arp_list; t; t = t->next) {
        if (t->ipv4 == ip) {
            memcpy(mac, t->mac, 6);
            orc_log(ORC_LOG_ARP, 2, "mac found\n");
            for (int i = 0; i < 6; i++)
                orc_log(ORC_LOG_ARP, 2, "%x", mac[i]);
            return 1;
        }
    }
    orc_log(ORC_LOG_ARP, 2, "No mac found\n");
    return 0;
}

static void orc_add_mac(uint32_t ip, const uint8_t *mac) /* arp.c:282-317 */
{
    orc_log(ORC_LOG_ARP, 4, "Adding mac for ");
    orc_print_add(ip);
    for (int i = 0; i < 6; i++)
        orc_log(ORC_LOG_ARP, 4, " %x", mac[i]);
    orc_log(ORC_LOG_ARP, 4, "\n");
    struct orc_arp_map *last = NULL;
    for (struct orc_arp_map *t = orc_arp_list; t; t = t->next)
        last = t;
    struct orc_arp_map *n = (struct orc_arp_map *)malloc(sizeof *n);
    n->next = NULL;
    n->ipv4 = ip;
    memcpy(n->mac, mac, 6);
    if (last)
        last->next = n;
    else
        orc_arp_list = n;
    orc_arp_n++;
}

/* ----------------------------------------------------------------- rx path --- */

static void orc_rx_impl(const uint8_t *f, uint32_t len, const rxg_tcb_tuple *tcbs,
                        const uint8_t *live, int32_t ntcb, rxg_rec48 *out, int faithful,
                        uint8_t *scratch)
{
    uint8_t h[54];
    for (uint32_t i = 0; i < 54; i++)
        h[i] = byte_at(f, len, i);

    memset(out, 0, sizeof *out);
    uint16_t et = (uint16_t)((h[12] << 8) | h[13]);          /* etherin.c:21 */
    uint16_t tl = (uint16_t)((h[16] << 8) | h[17]);
    uint8_t vihl = h[14], proto = h[23], doff = h[46], tflags = h[47];
    out->ether_type = et;
    out->sport = (uint16_t)((h[34] << 8) | h[35]);            /* tcp_tcb.c:135 */
    out->dport = (uint16_t)((h[36] << 8) | h[37]);            /* tcp_tcb.c:134 */
    out->l4_proto = proto;
    out->version_ihl = vihl;
    out->seq = be32(h + 38);
    out->ack = be32(h + 42);
    out->src_ip = be32(h + 26);                               /* ntohl(src_addr) */
    out->dst_ip_raw = le32(h + 30);                           /* dst_addr as loaded (LE host) */
    out->data_off = doff;
    memcpy(out->src_mac, h + 6, 6);
    out->c.tcp_flags = tflags;
    out->c.datalen = (int32_t)tl - (vihl & 0x0f) * 4 - (doff >> 4) * 4; /* tcp_states.c:48-50 */
    out->c.tcb_idx = -1;
    out->c.state = RXG_STATE_NONE;
    out->c.flags = len < 54 ? RXG_F_TRUNC : 0;

    switch (et) {
    case RXG_ETHER_TYPE_ARP: /* etherin.c:22-27 */
        if (faithful)
            orc_log(ORC_LOG_ARP, 2, "seen arp packet\n");
        out->c.verdict = RXG_V_ARP;
        return;
    case RXG_ETHER_TYPE_IPV4: /* etherin.c:28-32 -> ip_in */
        break;
    default: /* etherin.c:33-34 */
        out->c.verdict = RXG_V_DROP_L2;
        return;
    }

    if (faithful != 2) { /* 2: as shipped, no rx checksum (tcp_in.c:37 if(0); ip_in none) */
        out->c.ip_cksum = orc_calculate_checksum(h + 14, 20);
        if (out->c.ip_cksum == 0)
            out->c.flags |= RXG_F_IP_OK;
    }
    if (faithful)
        orc_print_arp_table(); /* ip.c:26 */
    if (proto != RXG_IPPROTO_TCP) { /* ip.c:36-39 */
        out->c.verdict = RXG_V_DROP_NONTCP;
        return;
    }
    if (faithful) { /* ip.c:30-32 */
        uint8_t mac[6];
        if (orc_get_mac(out->src_ip, mac) == 0)
            orc_add_mac(out->src_ip, h + 6);
        orc_log(ORC_LOG_TCP, 2, "received tcp packet\n"); /* tcp_in.c:35 */
    }

    if (faithful != 2) {
        out->c.tcp_cksum = orc_tcp_checksum(f, len, tl, faithful, scratch);
        if (out->c.tcp_cksum == 0)
            out->c.flags |= RXG_F_TCP_OK;
    }

    int listen_hit = 0, null_slot = 0;
    int32_t idx = orc_findtcb(tcbs, live, ntcb, out->dport, out->sport, out->dst_ip_raw,
                              out->src_ip, &listen_hit, &null_slot, faithful);
    if (listen_hit)
        out->c.flags |= RXG_F_LISTEN;
    if (null_slot)
        out->c.flags |= RXG_F_REF_NULLSLOT;
    out->c.tcb_idx = idx;
    if (idx < 0) { /* tcp_in.c:47-53 */
        out->c.verdict = RXG_V_RST_NOPCB;
        return;
    }
    uint8_t st = tcbs[idx].state;
    out->c.state = st;
    if (st == RXG_LISTENING && !(tflags & RXG_TCP_FLAG_SYN)) /* tcp_in.c:54-59 */
        out->c.verdict = RXG_V_RST_LISTEN_NONSYN;
    else /* tcp_in.c:65-72 (tcpok() is always 1, :22-29) */
        out->c.verdict = RXG_V_DISPATCH;
}

void orc_rx_one(const uint8_t *frame, uint32_t len, const rxg_tcb_tuple *tcbs,
                const uint8_t *live, int32_t ntcb, rxg_rec48 *out)
{
    static uint8_t scratch[12 + 65536 + 1];
    orc_rx_impl(frame, len, tcbs, live, ntcb, out, 0, scratch);
}

void orc_count_record(const rxg_rec48 *r, uint32_t len, uint64_t *c)
{
    c[RXG_C_RX] += 1;
    c[RXG_C_BYTES] += len;
    if (r->c.flags & RXG_F_TRUNC)
        c[RXG_C_TRUNC] += 1;
    if (r->ether_type == RXG_ETHER_TYPE_ARP) {
        c[RXG_C_ARP] += 1;
        return;
    }
    if (r->ether_type != RXG_ETHER_TYPE_IPV4) {
        c[RXG_C_OTHER_L2] += 1;
        return;
    }
    c[RXG_C_IPV4] += 1;
    if (r->c.ip_cksum != 0)
        c[RXG_C_IP_CKSUM_BAD] += 1;
    if (r->l4_proto != RXG_IPPROTO_TCP) {
        c[RXG_C_NON_TCP] += 1;
        return;
    }
    c[RXG_C_TCP] += 1;
    if (r->c.tcp_cksum != 0)
        c[RXG_C_TCP_CKSUM_BAD] += 1;
    if (r->c.flags & RXG_F_REF_NULLSLOT)
        c[RXG_C_REF_NULLSLOT] += 1;
    if (r->c.tcb_idx >= 0) {
        if (r->c.flags & RXG_F_LISTEN)
            c[RXG_C_TCB_HIT_LISTEN] += 1;
        else
            c[RXG_C_TCB_HIT_EXACT] += 1;
    }
    switch (r->c.verdict) {
    case RXG_V_RST_NOPCB: c[RXG_C_NOPCB] += 1; break;
    case RXG_V_RST_LISTEN_NONSYN: c[RXG_C_LISTEN_NONSYN] += 1; break;
    case RXG_V_DISPATCH: c[RXG_C_DISPATCH] += 1; break;
    default: break;
    }
}

static int orc_batch(const uint8_t *arena, const uint32_t *off64, const uint16_t *len, uint32_t n,
                     const rxg_tcb_tuple *tcbs, const uint8_t *live, int32_t ntcb,
                     rxg_rec48 *out, uint64_t *counters, int faithful)
{
    uint8_t *scratch = (uint8_t *)malloc(12 + 65536 + 1);
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t *f = arena + (uint64_t)off64[i] * 64u;
        orc_rx_impl(f, len[i], tcbs, live, ntcb, &out[i], faithful, scratch);
        if (counters)
            orc_count_record(&out[i], len[i], counters);
    }
    free(scratch);
    return 0;
}

int orc_rx_batch(const uint8_t *arena, const uint32_t *off64, const uint16_t *len, uint32_t n,
                 const rxg_tcb_tuple *tcbs, const uint8_t *live, int32_t ntcb, rxg_rec48 *out,
                 uint64_t *counters)
{
    return orc_batch(arena, off64, len, n, tcbs, live, ntcb, out, counters, 0);
}

int orc_rx_batch_faithful(const uint8_t *arena, const uint32_t *off64, const uint16_t *len,
                          uint32_t n, const rxg_tcb_tuple *tcbs, const uint8_t *live,
                          int32_t ntcb, rxg_rec48 *out, uint64_t *counters)
{
    return orc_batch(arena, off64, len, n, tcbs, live, ntcb, out, counters, 1);
}

/* Timing only: the faithful path as the reference ships it, without the rx checksum
   verify rxg adds (tcp_in.c:37 `if(0)`; ip_in checks nothing, ip.c:19-42).  The records'
   checksum fields and ok flags stay 0. */
int orc_rx_batch_shipped(const uint8_t *arena, const uint32_t *off64, const uint16_t *len,
                         uint32_t n, const rxg_tcb_tuple *tcbs, const uint8_t *live,
                         int32_t ntcb, rxg_rec48 *out, uint64_t *counters)
{
    return orc_batch(arena, off64, len, n, tcbs, live, ntcb, out, counters, 2);
}

/* ----------------------------------------------------------------- tx path --- */

/* ip.c:97-118 for a host-built frame: ip hdr_checksum over the 20-byte header with the
   field zeroed (ip.c:100,107), then the TCP checksum over pseudo || segment with
   cksum zeroed (ip.c:90,118).  Both stored htons(). Bytes at/after len are not written. */
void orc_tx_cksum_one(uint8_t *f, uint32_t len)
{
    uint8_t ip[20];
    for (int i = 0; i < 20; i++)
        ip[i] = byte_at(f, len, 14 + i);
    ip[10] = ip[11] = 0;
    uint16_t ipck = orc_calculate_checksum(ip, 20);
    if (len > 24) f[24] = (uint8_t)(ipck >> 8);
    if (len > 25) f[25] = (uint8_t)(ipck & 0xff);

    uint16_t tl = (uint16_t)((byte_at(f, len, 16) << 8) | byte_at(f, len, 17));
    uint32_t seglen = tl >= 20 ? (uint32_t)tl - 20u : 0u;
    uint16_t l16 = (uint16_t)(tl - 20);
    uint8_t *temp = (uint8_t *)calloc(12 + seglen + 1, 1);
    for (int i = 0; i < 8; i++)
        temp[i] = byte_at(f, len, 26 + i);
    temp[9] = RXG_IPPROTO_TCP;
    temp[10] = (uint8_t)(l16 >> 8);
    temp[11] = (uint8_t)(l16 & 0xff);
    for (uint32_t i = 0; i < seglen; i++)
        temp[12 + i] = byte_at(f, len, 34 + i);
    if (seglen > 17) /* the cksum field (segment bytes 16-17) is zero while summing */
        temp[12 + 16] = temp[12 + 17] = 0;
    else if (seglen > 16)
        temp[12 + 16] = 0;
    uint16_t tck = orc_calculate_checksum(temp, (int)(12 + seglen));
    free(temp);
    if (len > 50) f[50] = (uint8_t)(tck >> 8);
    if (len > 51) f[51] = (uint8_t)(tck & 0xff);
}

int orc_tx_cksum_batch(uint8_t *arena, const uint32_t *off64, const uint16_t *len, uint32_t n)
{
    for (uint32_t i = 0; i < n; i++)
        orc_tx_cksum_one(arena + (uint64_t)off64[i] * 64u, len[i]);
    return 0;
}
