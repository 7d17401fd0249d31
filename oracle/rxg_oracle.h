/*
 * rxg_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, CPU, scalar restatement of the reference receive path
 * (tcp_ip_stack/etherin.c, ip.c, tcp_in.c, tcp_tcb.c of rajneshrat/dpdk-tcpipstack),
 * written from the reference's semantics, not copied.  It is the checker for rxg's
 * HIP path: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it.  The product library (librxg.so) never links or calls it.
 *
 * Parity pinning:
 *   - calculate_checksum is pinned by the RFC 1071 known-answer vectors the survey ran
 *     through the reference (0x220d, 0xb861) and by the round-trip property of frames
 *     the reference's ip_out builds (verify to 0x0000).  Fixtures: tests/golden/.
 *   - findtcb / verdict classification: the reference ships no tests or fixtures, and it
 *     cannot be built here without DPDK headers the image lacks, so beyond the three
 *     behaviours the survey observed on the reference (exact hit, listener on SYN,
 *     NULL -> RST on an unknown port) this part is "parity unpinned": restated from
 *     tcp_tcb.c:127-173 and tcp_in.c:32-84 by reading.
 */
#ifndef RXG_ORACLE_H
#define RXG_ORACLE_H
#include <stdint.h>
#include "../include/rxg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* tcp_ip_stack/ip.c:44-59 — big-endian 16-bit word sum over (len+1)/2 words, reading
   data[len] for odd len (the caller provides that byte; the oracle always feeds 0). */
uint16_t orc_calculate_checksum(const unsigned char *data, int len);

/* One frame through ether_in -> ip_in -> tcp_in -> findtcb, pure (no side effects).
   tcbs[0..ntcb) with live[i]==0 meaning tcbs[i]==NULL. */
void orc_rx_one(const uint8_t *frame, uint32_t len, const rxg_tcb_tuple *tcbs,
                const uint8_t *live, int32_t ntcb, rxg_rec48 *out);

/* Batch form over the rxg arena layout; counters[RXG_NCOUNTERS] are accumulated
   (not reset).  Returns 0. */
int orc_rx_batch(const uint8_t *arena, const uint32_t *off64, const uint16_t *len, uint32_t n,
                 const rxg_tcb_tuple *tcbs, const uint8_t *live, int32_t ntcb,
                 rxg_rec48 *out, uint64_t *counters);

/* Same records, computed the way the reference spends its time (CPU baseline leg):
   print_arp_table + get_mac/add_mac list walks per IPv4/TCP packet (ip.c:26-32,
   arp.c:215-317), one disabled log_print call per scanned TCB (tcp_tcb.c:150), the
   malloc+memcpy pseudo-header staging of ip.c:89-117 and the byte-loop checksum.  The
   ARP list persists across calls until orc_arp_reset(). */
int orc_rx_batch_faithful(const uint8_t *arena, const uint32_t *off64, const uint16_t *len,
                          uint32_t n, const rxg_tcb_tuple *tcbs, const uint8_t *live,
                          int32_t ntcb, rxg_rec48 *out, uint64_t *counters);
/* Timing only: orc_rx_batch_faithful without the rx checksums, i.e. the reference as shipped
   (tcp_in.c:37's verify compiled out); checksum fields and ok flags are left 0. */
int orc_rx_batch_shipped(const uint8_t *arena, const uint32_t *off64, const uint16_t *len,
                         uint32_t n, const rxg_tcb_tuple *tcbs, const uint8_t *live,
                         int32_t ntcb, rxg_rec48 *out, uint64_t *counters);
void orc_arp_reset(void);
int orc_arp_count(void);

/* Counters implied by one record (the definition rxg's device counters follow). */
void orc_count_record(const rxg_rec48 *r, uint32_t len, uint64_t *counters);

/* ip_out's two checksums (ip.c:97-118) for one host-built frame, written in place:
   bytes 24-25 = htons(cksum(ip hdr with field 0)), bytes 50-51 = htons(cksum(pseudo ||
   tcp segment with field 0)).  Segment = frame[34 .. 14+total_length) clamped to len. */
void orc_tx_cksum_one(uint8_t *frame, uint32_t len);
int orc_tx_cksum_batch(uint8_t *arena, const uint32_t *off64, const uint16_t *len, uint32_t n);

#ifdef __cplusplus
}
#endif
#endif
