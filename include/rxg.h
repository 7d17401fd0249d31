/*
 * rxg.h — C ABI of the MI355X-native receive-path engine ("rxg").
 *
 * rxg replaces the per-packet receive stage of rajneshrat/dpdk-tcpipstack:
 *
 *   l2fwd_main_loop: for (i < nb_rx) ether_in(pkts[i])      tcp_ip_stack/main.c:396-399
 *     ether_in   -> switch ether_type                       tcp_ip_stack/etherin.c:12-37
 *     ip_in      -> ARP learn, proto==6 -> tcp_in           tcp_ip_stack/ip.c:19-42
 *     tcp_in     -> findtcb, RST verdicts, tcpswitch[state]  tcp_ip_stack/tcp_in.c:32-84
 *     findtcb    -> two-pass linear 4-tuple / listener scan tcp_ip_stack/tcp_tcb.c:127-173
 *     calculate_checksum (RFC 1071 byte loop)               tcp_ip_stack/ip.c:44-59
 *
 * with one batched, device-resident pass on gfx950 (parse + IPv4 header checksum +
 * TCP pseudo-header checksum + 4-tuple -> TCB classify), followed by an in-order host
 * replay that performs exactly the side effects the reference performs
 * (free_mbuf, send_reset, ARP learn, max_seq_received, AdjustSendWindow,
 * tcpswitch[state]).
 *
 * Conventions
 *  - Every entry point returns 0 on success or a negative errno-style code
 *    (-EINVAL, -ENOMEM, -EIO for a HIP runtime error, -ENODEV without a GPU).
 *    Nothing asserts; nothing falls back to a CPU path.
 *  - Plain pointers and sizes only.  "dev" pointers are HIP device pointers.
 *  - A `stream` argument is a hipStream_t passed as void*; NULL = the context's own stream.
 *  - Field byte orders follow the reference exactly (see rxg_rec48 below).
 */
#ifndef RXG_H
#define RXG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RXG_ABI_VERSION 2

/* ------------------------------------------------------------------------- */
/* Protocol constants (wire formats; reference names in comments).            */
/* ------------------------------------------------------------------------- */
#define RXG_ETHER_TYPE_IPV4 0x0800 /* ETHER_TYPE_IPv4, etherin.c:28 */
#define RXG_ETHER_TYPE_ARP  0x0806 /* ETHER_TYPE_ARP,  etherin.c:22 */
#define RXG_IPPROTO_TCP     6      /* IPPROTO_TCP,     ip.c:29      */

/* TCP_FLAGS, tcp_ip_stack/tcp.h:12-21 */
#define RXG_TCP_FLAG_FIN 0x01
#define RXG_TCP_FLAG_SYN 0x02
#define RXG_TCP_FLAG_RST 0x04
#define RXG_TCP_FLAG_PSH 0x08
#define RXG_TCP_FLAG_ACK 0x10

/* enum TCP_STATE_, tcp_ip_stack/tcp_states.h:8-17 */
enum rxg_tcp_state {
    RXG_TCP_STATE_CLOSED = 0,
    RXG_LISTENING = 1,
    RXG_SYN_SENT = 2,
    RXG_SYN_RECV = 3,
    RXG_TCP_ESTABLISHED = 4,
    RXG_TCP_STATE_FIN_1 = 5,
    RXG_TCP_FIN_2 = 6,
    RXG_TCP_STATES = 7
};
#define RXG_STATE_NONE 0xFF /* no TCB chosen */

/* Fixed offsets the reference uses regardless of IHL (tcp_in.c:42-45). */
#define RXG_OFF_IP  14
#define RXG_OFF_TCP 34

/* Reference table capacity (TOTAL_TCBS, tcp_tcb.c:16). rxg itself has no such cap. */
#define RXG_REF_TOTAL_TCBS 20000

/* ------------------------------------------------------------------------- */
/* Per-packet result records.                                                 */
/* ------------------------------------------------------------------------- */

/* What the reference does with the packet (the branch ether_in/ip_in/tcp_in take). */
enum rxg_verdict {
    RXG_V_DISPATCH = 0,          /* tcpswitch[state](tcb, tcp, ip, m)   tcp_in.c:65-72     */
    RXG_V_RST_NOPCB = 1,         /* ++tcpnopcb; free; send_reset        tcp_in.c:47-53     */
    RXG_V_RST_LISTEN_NONSYN = 2, /* LISTENING && !SYN: free; send_reset tcp_in.c:54-59     */
    RXG_V_DROP_NONTCP = 3,       /* IPv4, next_proto_id != 6: free      ip.c:36-39         */
    RXG_V_ARP = 4,               /* arp_in(m); free_mbuf(m)             etherin.c:22-27    */
    RXG_V_DROP_L2 = 5            /* other ether_type: free_mbuf         etherin.c:33-34    */
};

/* rxg_rec16.flags bits */
enum rxg_rec_flag {
    RXG_F_IP_OK = 0x01,        /* IPv4 and ip_cksum == 0                                     */
    RXG_F_TCP_OK = 0x02,       /* TCP and tcp_cksum == 0                                     */
    RXG_F_LISTEN = 0x04,       /* TCB found by findtcb pass 2 (listener on dport)            */
    RXG_F_REF_NULLSLOT = 0x08, /* pass 2 met a removed (NULL) slot before its answer: the
                                  reference dereferences NULL there (tcp_tcb.c:160-162);
                                  rxg skips the slot and reports it                        */
    RXG_F_TRUNC = 0x10,        /* frame shorter than the 54 bytes the path reads; bytes at
                                  and beyond data_len are read as zero                      */
    RXG_F_ARP_LEARN = 0x20     /* TCP packet whose host-order source IP is not in the ARP
                                  mirror as of the burst: ip.c:30-32 would call add_mac
                                  unless an earlier packet of the burst already added it
                                  (only computed while the ARP mirror is enabled)           */
};

/*
 * 16-byte compact record: everything the in-order host replay needs that is not a
 * plain re-read of the (host-resident) frame.
 */
typedef struct rxg_rec16 {
    int32_t tcb_idx;    /* index into tcbs[] chosen by findtcb (tcp_tcb.c:127-173); -1 = NULL */
    uint16_t ip_cksum;  /* calculate_checksum(frame+14, 20); 0x0000 = header valid             */
    uint16_t tcp_cksum; /* calculate_checksum(pseudo || frame[34 .. 14+total_length));
                           pseudo = {src_addr, dst_addr, 0, 6, htons(total_length-20)}
                           exactly as ip_out builds it (ip.c:109-118); 0x0000 = valid          */
    uint8_t verdict;    /* enum rxg_verdict                                                     */
    uint8_t state;      /* tcbs[tcb_idx]->state at classify time, RXG_STATE_NONE if none        */
    uint8_t tcp_flags;  /* frame byte 47                                                        */
    uint8_t flags;      /* enum rxg_rec_flag                                                    */
    int32_t datalen;    /* ntohs(total_length) - (version_ihl&0xf)*4 - (data_off>>4)*4
                           as the state handlers compute it (tcp_states.c:48-50,103-111)       */
} rxg_rec16;

/* 48-byte full record: the compact record plus every header field the path extracts. */
typedef struct rxg_rec48 {
    rxg_rec16 c;          /* bytes 0..15                                                  */
    uint16_t ether_type;  /* 16: ntohs(eth->ether_type)                 etherin.c:21        */
    uint16_t sport;       /* 18: ntohs(tcp->src_port)                   tcp_tcb.c:135       */
    uint16_t dport;       /* 20: ntohs(tcp->dst_port)                   tcp_tcb.c:134       */
    uint8_t l4_proto;     /* 22: ip->next_proto_id                      ip.c:28             */
    uint8_t version_ihl;  /* 23: ip->version_ihl                        tcp_states.c:49     */
    uint32_t seq;         /* 24: ntohl(tcp->sent_seq)                   tcp_in.c:66         */
    uint32_t ack;         /* 28: ntohl(tcp->recv_ack)                   tcp_in.c:71         */
    uint32_t src_ip;      /* 32: ntohl(ip->src_addr), host order        ip.c:30, tcp_tcb.c:155 */
    uint32_t dst_ip_raw;  /* 36: ip->dst_addr as loaded (network order) tcp_tcb.c:154       */
    uint8_t data_off;     /* 40: tcp->data_off (raw byte 46)            tcp_states.c:48     */
    uint8_t src_mac[6];   /* 41: eth->s_addr                            ip.c:31             */
    uint8_t reserved;     /* 47: 0                                                          */
} rxg_rec48;
/* total_length = c.datalen + (version_ihl & 0xf) * 4 + (data_off >> 4) * 4. */

/* 8-byte record (RXG_REC8): what rxg_rx_replay and rxg_payload_gather_dev use, half the
   bytes of rxg_rec16 per frame; the two checksums are carried as RXG_F_IP_OK /
   RXG_F_TCP_OK only.
     w0  bits  0-23  tcb_idx + 1 (0: findtcb returned NULL)
         bits 24-26  verdict (enum rxg_verdict)
         bits 27-29  state (7: RXG_STATE_NONE)
     w1  bits  0-7   tcp_flags
         bits  8-13  flags (enum rxg_rec_flag)
         bits 14-30  datalen + 128 (datalen >= -120: total_length - 60 - 60)           */
typedef struct rxg_rec8 {
    uint32_t w0, w1;
} rxg_rec8;

enum rxg_rec_kind { RXG_REC8 = 8, RXG_REC16 = 16, RXG_REC48 = 48 };

/* rxg_rec8 -> rxg_rec16.  A checksum the record only knows as "not 0x0000" reads 0xFFFF
   (IPv4 frames without RXG_F_IP_OK, TCP segments without RXG_F_TCP_OK); the others 0. */
static inline void rxg_rec8_expand(const rxg_rec8 *r, rxg_rec16 *o)
{
    const uint32_t v = (r->w0 >> 24) & 7u, st = (r->w0 >> 27) & 7u, fl = (r->w1 >> 8) & 0x3Fu;
    const int ip = v <= RXG_V_DROP_NONTCP, tcp = v <= RXG_V_RST_LISTEN_NONSYN;
    o->tcb_idx = (int32_t)(r->w0 & 0xFFFFFFu) - 1;
    o->ip_cksum = (uint16_t)((ip && !(fl & RXG_F_IP_OK)) ? 0xFFFFu : 0u);
    o->tcp_cksum = (uint16_t)((tcp && !(fl & RXG_F_TCP_OK)) ? 0xFFFFu : 0u);
    o->verdict = (uint8_t)v;
    o->state = (uint8_t)(st == 7u ? RXG_STATE_NONE : st);
    o->tcp_flags = (uint8_t)(r->w1 & 0xFFu);
    o->flags = (uint8_t)fl;
    o->datalen = (int32_t)((r->w1 >> 14) & 0x1FFFFu) - 128;
}

/* ------------------------------------------------------------------------- */
/* Per-GPU counters (merged across GPUs with an RCCL all-reduce, sum, uint64). */
/* ------------------------------------------------------------------------- */
enum rxg_counter {
    RXG_C_RX = 0,           /* frames seen                                            */
    RXG_C_BYTES,            /* sum of data_len                                        */
    RXG_C_IPV4,             /* ether_type 0x0800                                      */
    RXG_C_ARP,              /* ether_type 0x0806                                      */
    RXG_C_OTHER_L2,         /* any other ether_type                                   */
    RXG_C_TCP,              /* IPv4 with next_proto_id 6                              */
    RXG_C_NON_TCP,          /* IPv4, other protocol                                   */
    RXG_C_IP_CKSUM_BAD,     /* IPv4 with ip_cksum != 0                                */
    RXG_C_TCP_CKSUM_BAD,    /* TCP with tcp_cksum != 0 (tcpchecksumerror, tcp_in.c:18) */
    RXG_C_TCB_HIT_EXACT,    /* findtcb pass 1 hit                                     */
    RXG_C_TCB_HIT_LISTEN,   /* findtcb pass 2 hit                                     */
    RXG_C_NOPCB,            /* findtcb NULL (tcpnopcb, tcp_in.c:48)                   */
    RXG_C_LISTEN_NONSYN,    /* RST to a non-SYN on a listener                         */
    RXG_C_DISPATCH,         /* handed to tcpswitch[state]                             */
    RXG_C_REF_NULLSLOT,     /* reference would have dereferenced a NULL slot          */
    RXG_C_TRUNC,            /* frames shorter than 54 bytes                           */
    RXG_NCOUNTERS
};

/* ------------------------------------------------------------------------- */
/* Context                                                                    */
/* ------------------------------------------------------------------------- */
typedef struct rxg_ctx rxg_ctx;

typedef struct rxg_config {
    int32_t device;        /* HIP device ordinal (one context per GPU, one rx thread each) */
    uint32_t max_batch;    /* largest n passed to the host-buffer entry points (staging)   */
    uint32_t max_bytes;    /* staging arena bytes for host-buffer entry points            */
    uint32_t flags;        /* RXG_CFG_*                                                    */
    uint32_t max_blocks;   /* rx grid cap in workgroups; 0 = one generation of resident
                              workgroups (occupancy).  Any value gives the same records.   */
    uint32_t zc_bytes;     /* rxg_rx_burst: bursts of up to this many staged bytes run
                              zero-copy (kernel reads pinned staging over PCIe); 0 = 64 MiB */
} rxg_config;

/* rxg_config.flags.  RXG_CFG_REPLAY_ON_DEVICE: rxg_rx_replay re-classifies every packet a
   handler's tcbs[] write affects with a GPU launch (the default answers small sets from the
   host index the device mirror is patched from; same records either way).
   RXG_CFG_STREAMS_OUTLIVE_WRITES: the write's order against table-reading launches on
   caller streams is taken when the write is pushed (an event recorded on the stream then)
   instead of by a marker after every launch, which on a caller stream cost ~4.5 us per
   launch.  The recording needs the stream to exist at the write, so in this
   mode a caller stream must be registered (rxg_stream_register) before its first
   table-reading launch (rxg_rx_burst_dev, rxg_rx_bursts_dev; else -EINVAL, nothing
   launched) and retired (rxg_stream_retire) before it is destroyed.  Without the flag a
   stream may be destroyed once synchronised. */
#define RXG_CFG_REPLAY_ON_DEVICE 0x1u
#define RXG_CFG_STREAMS_OUTLIVE_WRITES 0x2u

int rxg_abi_version(void);
/* "rxg src=<16 hex: sha256 of the product sources> rev=<git revision>[+dirty] built=<date>
   gfx950": which sources the library was built from (rxg.source_hash() recomputes src=). */
const char *rxg_build_info(void);
int rxg_init(const rxg_config *cfg, rxg_ctx **out);
/* 0, or -EIO when a latency-mode server kernel that missed its time limit is still resident
   after bounded retries of rxg_server_stop: the context and every buffer that kernel can
   reach are then left allocated (leaked), never freed under it; the handle is dead either way. */
int rxg_fini(rxg_ctx *ctx);
/* Block until all work queued on the context's stream is done. */
int rxg_sync(rxg_ctx *ctx);
/* The hipStream_t rxg launches on when a NULL stream is passed. */
void *rxg_stream(rxg_ctx *ctx);
/* Caller streams of a RXG_CFG_STREAMS_OUTLIVE_WRITES context (any context accepts them).
   register: `stream` may carry table-reading launches from now on.  retire: the context
   takes, now, the order its next table write needs against the stream's launches and forgets
   the stream; the caller may then destroy it.  The context's own stream needs neither.
   0, or -EINVAL for a NULL argument. */
int rxg_stream_register(rxg_ctx *ctx, void *stream);
int rxg_stream_retire(rxg_ctx *ctx, void *stream);

/* ------------------------------------------------------------------------- */
/* TCB mirror.  The reference mutates `tcbs[]` directly (tcp_tcb.c:21-22,     */
/* alloc_tcb :34-106, remove_tcb :175-186, tuple writes in socket_interface.c */
/* :80-83,:329-332 and tcp_states.c :25-27,:185-188).  A caller mirrors each   */
/* such write with one of these calls; they are applied to the device copy   */
/* before the next burst.                                                     */
/* ------------------------------------------------------------------------- */
typedef struct rxg_tcb_tuple {
    int32_t dport;       /* struct tcb::dport (host order, int)          tcp_tcb.h:17 */
    int32_t sport;       /* struct tcb::sport (host order, int)          tcp_tcb.h:18 */
    uint32_t ipv4_dst;   /* struct tcb::ipv4_dst, compared RAW to ip->dst_addr        */
    uint32_t ipv4_src;   /* struct tcb::ipv4_src, compared to ntohl(ip->src_addr)     */
    uint8_t state;       /* struct tcb::state (enum rxg_tcp_state)                    */
    uint8_t pad;
    uint16_t identifier; /* struct tcb::identifier (1..65535 cyclic)                  */
} rxg_tcb_tuple;

/* tcbs[idx] = tuple (a live slot).  idx >= current Ntcb grows Ntcb to idx+1; slots in
   between are NULL, as if allocated and removed. */
int rxg_tcb_upsert(rxg_ctx *ctx, int32_t idx, const rxg_tcb_tuple *t);
/* tcbs[idx] = NULL (remove_tcb).  Ntcb never shrinks (tcp_tcb.c:175-186). */
int rxg_tcb_remove(rxg_ctx *ctx, int32_t idx);
/* tcbs[idx]->state = state. */
int rxg_tcb_set_state(rxg_ctx *ctx, int32_t idx, uint8_t state);
/* Replace the whole table: tcbs[0..ntcb), live[i]==0 marks a NULL slot. */
int rxg_tcb_load(rxg_ctx *ctx, const rxg_tcb_tuple *tcbs, const uint8_t *live, int32_t ntcb);
/* Push pending mirror changes to the device (done implicitly by every burst).  Each write
   changes O(1) device words (a bucket slot, a listener entry), applied by one small kernel
   on the context's stream after every launch that still reads the old table, whatever its
   stream; a burst on another stream waits for them on the device, not on the host.  Only
   rxg_tcb_load and growth past load 1/2 rebuild (and upload) the whole table (see
   RXG_CFG_STREAMS_OUTLIVE_WRITES for bursts on caller streams). */
int rxg_tcb_sync(rxg_ctx *ctx);
/* Current Ntcb of the mirror. */
int32_t rxg_tcb_count(rxg_ctx *ctx);

/* Flow-affinity sharding (SURVEY.md §8(e)'s optional mode): one rx queue per
   GPU, the NIC steering each TCP segment to a queue by its RSS hash (Toeplitz over src ip,
   dst ip, src port, dst port with the default 40-byte Microsoft key, then a redirection table
   of RXG_RSS_RETA_SIZE entries filled round-robin, DPDK's default).  The context of queue
   `part` of `nparts` keeps in its device table only the tuples that hash to it (1/nparts of
   the keys); the listener map, liveness and the lowest NULL slot stay whole, so findtcb's
   pass 2 (tcp_tcb.c:158-170) answers as against the whole table.  Every context still gets
   every tcbs[] write (rxg_tcb_*).  A frame classified by the context of another queue
   finds no exact TCB: steer with the NIC or with rxg_flow_part_of.  nparts = 1: the whole
   table (the default).  Takes effect at the next sync (a table rebuild). */
#define RXG_RSS_RETA_SIZE 128
int rxg_flow_partition(rxg_ctx *ctx, uint32_t part, uint32_t nparts);
/* The context's partition (1 of 1 when not partitioned).  A group (rxg_group_*) cuts
   contiguous shards, so rxg_group_rx_burst refuses partitioned members (-EINVAL). */
int rxg_flow_partition_get(rxg_ctx *ctx, uint32_t *part, uint32_t *nparts);
/* The queue (0 .. nparts-1) an IPv4/TCP frame belongs to (frame bytes 26..37, read as the
   kernel reads them: bytes at or past len are zero); 0 for other frames, which no context
   looks up.  -EINVAL for frame NULL with len > 0 or nparts outside 1..RXG_RSS_RETA_SIZE. */
int rxg_flow_part_of(const uint8_t *frame, uint32_t len, uint32_t nparts);
/* The Toeplitz RSS hash of 12 wire bytes (src ip | dst ip | src port | dst port). */
uint32_t rxg_rss_hash(const uint8_t tuple12[12]);
/* Distinct tuples in the context's device table (after the last sync); -EINVAL for NULL. */
int64_t rxg_tcb_keys(rxg_ctx *ctx);

/* Writes from other threads.  The calls above belong to the rx thread (the one running
   bursts and rxg_rx_replay, whose tcpswitch handlers write tcbs[] on the reference's rx
   lcore).  The reference's socket API writes tcbs[] from the application lcore, unlocked
   against the rx loop (alloc_tcb tcp_tcb.c:34-106, socket_bind socket_interface.c:80-83,
   socket_connect :329-332); its mirror calls go through rxg_tcb_post instead: a lock-free
   multi-producer queue the rx thread drains, in claim order, at the start of the next
   burst (rxg_rx_burst, rxg_rx_burst_dev, rxg_ether_in) or rxg_tcb_sync / rxg_tcb_drain,
   so a burst never sees a half-applied write.  Not drained during rxg_rx_replay. */
enum rxg_tcb_op_kind { RXG_TCB_OP_UPSERT = 1, RXG_TCB_OP_REMOVE = 2, RXG_TCB_OP_SET_STATE = 3 };
typedef struct rxg_tcb_op {
    uint32_t kind;        /* enum rxg_tcb_op_kind                                   */
    int32_t idx;          /* tcbs[] index                                           */
    rxg_tcb_tuple tuple;  /* RXG_TCB_OP_UPSERT                                      */
    uint8_t state;        /* RXG_TCB_OP_SET_STATE                                   */
    uint8_t pad[3];
} rxg_tcb_op;
#define RXG_TCB_QUEUE_CAP 65536u
/* Any thread.  -EAGAIN when RXG_TCB_QUEUE_CAP posts are waiting (nothing queued then). */
int rxg_tcb_post(rxg_ctx *ctx, const rxg_tcb_op *op);
/* rx thread: apply every posted write now.  Returns how many were applied, or the first
   failing write's negative errno (the later ones are still applied). */
int rxg_tcb_drain(rxg_ctx *ctx);

/* ARP mirror (optional).  The reference keeps an IP -> MAC list that ip_in walks twice per
   packet (print_arp_table + get_mac, ip.c:26-32, arp.c:215-280).  Once a caller mirrors
   every add_mac (arp.c:282-317) with rxg_arp_learned, bursts flag each TCP packet whose
   source is unknown (RXG_F_ARP_LEARN) and rxg_rx_replay calls add_mac for the first such
   packet per address without walking the list: same final list, same order. */
int rxg_arp_load(rxg_ctx *ctx, const uint32_t *ipv4_host, uint32_t n);
int rxg_arp_learned(rxg_ctx *ctx, uint32_t ipv4_host);
int32_t rxg_arp_count(rxg_ctx *ctx);
/* Stop mirroring (RXG_F_ARP_LEARN is no longer computed; replay walks get_mac again). */
int rxg_arp_disable(rxg_ctx *ctx);

/* ------------------------------------------------------------------------- */
/* Receive burst: parse + checksum + classify.  Pure: no frees, no side       */
/* effects, counters only.                                                    */
/* ------------------------------------------------------------------------- */

/* Device-resident batch.  Frame i occupies bytes [frames + 64*off64[i],
   + len[i]); the bytes up to the next 64-byte boundary must be readable
   (their contents are ignored), and so must the first 64 bytes at `frames`
   (loads for chunks outside a frame are redirected there, then discarded).
   len[i] = rte_pktmbuf_data_len(m).  Alignment (else -EINVAL): frames 16 bytes, off64 4,
   len 2, out 8 (RXG_REC8) or 16 bytes. */
typedef struct rxg_dev_batch {
    const void *frames;     /* dev */
    const uint32_t *off64;  /* dev, n entries, in 64-byte units */
    const uint16_t *len;    /* dev, n entries */
    uint32_t n;
    uint32_t rec_kind;      /* RXG_REC8, RXG_REC16 or RXG_REC48 */
    void *out;              /* dev, n records of rec_kind bytes */
} rxg_dev_batch;

/* Replaces the per-packet loop over ether_in() (main.c:396-399) for a batch already
   resident in HBM.  Asynchronous on `stream`. */
int rxg_rx_burst_dev(rxg_ctx *ctx, const rxg_dev_batch *b, void *stream);

/* Several bursts of one frame pool in one launch (e.g. the bursts of several rx queues, or a
   ring of bursts): burst j's frame i is at frames + 64*bursts[j].off64[i] (same readability
   rules as rxg_dev_batch), its record at bursts[j].out + i * rec_kind.  Every burst is
   classified against the mirror as it stands at the call, exactly as k rxg_rx_burst_dev
   calls with no mirror writes between them; one launch (per 32 bursts) instead of k, so the
   launch ramp is paid once.  The bursts are then replayed in order, one rxg_rx_replay call
   each (a replay sees the tcbs[] writes of the earlier bursts' replays), and
   rxg_payload_gather_dev gathers the burst to be replayed next.  Asynchronous on `stream`. */
typedef struct rxg_dev_burst {
    const uint32_t *off64;  /* dev, n entries, in 64-byte units of the frame pool */
    const uint16_t *len;    /* dev, n entries */
    uint32_t n;
    uint32_t pad;
    void *out;              /* dev, n records */
} rxg_dev_burst;
int rxg_rx_bursts_dev(rxg_ctx *ctx, const void *frames, const rxg_dev_burst *bursts, uint32_t k,
                      uint32_t rec_kind, void *stream);

/* Fixed-stride bursts: frame i of a burst occupies bytes [frames + 64 * (slot0 + i * stride64),
   + len[i]), with the readability rules of rxg_dev_batch.  For frame pools of fixed-size
   elements filled in ring order -- a DPDK mempool's elements are fixed-size (MBUF_SIZE,
   main.c:94-95), and a receive ring whose buffers are such elements posted in order, or this
   library's own host-burst staging, places frame i at a fixed stride -- the kernel then reads
   no per-frame offset list: 4 bytes less per frame of descriptor traffic (of 14 per 64-byte
   frame with 8-byte records).  Same records, counters, replay and payload gather as
   rxg_rx_bursts_dev with off64[i] = slot0 + i * stride64 (slot0 + (n-1) * stride64 must fit
   32 bits, else -EINVAL).  Asynchronous on `stream`. */
typedef struct rxg_dev_strided_burst {
    const uint16_t *len;    /* dev, n entries */
    uint32_t n;
    uint32_t slot0;         /* 64-byte slot of the burst's frame 0 in the pool */
    void *out;              /* dev, n records */
} rxg_dev_strided_burst;
int rxg_rx_bursts_strided_dev(rxg_ctx *ctx, const void *frames, uint32_t stride64,
                              const rxg_dev_strided_burst *bursts, uint32_t k, uint32_t rec_kind, void *stream);

/* DPDK-compatible host packet view: frame = (char*)buf_addr + data_off, data_len bytes
   (struct rte_mbuf fields of the same names). */
typedef struct rxg_pkt_view {
    const void *buf_addr;
    uint16_t data_off;
    uint16_t data_len;
    uint32_t pad;
} rxg_pkt_view;

/* Host-buffer burst: packs the frames into pinned staging, H2D, kernel, D2H into
   `out_host` (n records of rec_kind bytes).  Synchronous. */
int rxg_rx_burst(rxg_ctx *ctx, const rxg_pkt_view *pkts, uint32_t n, uint32_t rec_kind,
                 void *out_host);

/* Latency mode for the reference's own burst size (MAX_PKT_BURST = 32, main.c:116; the loop
   main.c:391-399 runs once per rte_eth_rx_burst).  A launched burst pays a kernel launch
   and a stream synchronisation (~20 us for 32 frames); the server is a persistent set of
   `blocks` workgroups of the same kernel body that polls a mailbox, so a burst costs the
   PCIe trips of its frames and records.  The host-burst staging (frames, descriptors)
   lives in device memory the host writes through the PCIe BAR (posted writes; the server
   reads HBM) when the device exposes its memory to the host (large BAR), else in coherent
   host memory (RXG_SRV_HOST_STAGING forces that); the mailbox the server polls is device
   memory too on such a device (RXG_SRV_HOST_MAILBOX keeps it in coherent host memory);
   the server's answers and the records of host bursts are written to host memory.
   While the server runs,
   rxg_rx_burst sends bursts of up to max_frames frames (max_bytes staged bytes) and of
   record kind rec_kind through it (packed into the server's own staging), and
   rxg_server_burst_dev serves device-visible batches.  Records, counters, replay and
   payload gather are those of the launched path.  A burst of up to 128 frames runs on the
   first workgroup (its four waves sharing one or two 64-frame slices of large frames); with
   `blocks` >= 3 a host
   burst of 129..64*blocks frames holding a frame over 64 bytes runs one 64-frame slice per
   workgroup, so `blocks` = 4 serves the reference's bursts and bursts of up to 256 large
   frames at the shortest latency.  The server exits by itself after idle_ms
   without a burst (and is relaunched by the next one), so it never outlives its process for
   long.  Calls from the context's rx thread only.  Returns 0 or a negative errno. */
typedef struct rxg_server_config {
    uint32_t rec_kind;    /* RXG_REC8 / RXG_REC16 / RXG_REC48 */
    uint32_t blocks;      /* workgroups (4 waves each); 0 = 1 */
    uint32_t max_frames;  /* largest burst served; 0 = 4096 */
    uint32_t max_bytes;   /* staging bytes for host bursts; 0 = max_frames * 2048 */
    uint32_t idle_ms;     /* exit after this long without a burst; 0 = 1000 */
    uint32_t flags;       /* RXG_SRV_*; 0 = mailbox and staging placed by the device */
} rxg_server_config;
#define RXG_SRV_HOST_STAGING 1u   /* staging in coherent host memory */
#define RXG_SRV_HOST_MAILBOX 2u   /* mailbox in coherent host memory */
int rxg_server_start(rxg_ctx *ctx, const rxg_server_config *cfg);
/* Stops the server and waits for its kernel to end; 0 if none runs. */
int rxg_server_stop(rxg_ctx *ctx);
/* 1 if a server is configured (running or idle-exited, relaunched on demand), else 0. */
int rxg_server_active(rxg_ctx *ctx);
/* Where the configured server's host-burst staging lives: RXG_SRV_DEVICE (device memory
   written through the BAR), RXG_SRV_HOST (coherent host memory), RXG_SRV_NONE (no server). */
#define RXG_SRV_NONE 0
#define RXG_SRV_HOST 1
#define RXG_SRV_DEVICE 2
int rxg_server_placement(rxg_ctx *ctx);
/* Classify a device-visible batch (HBM or mapped host memory) through the server:
   b->rec_kind must be the server's, b->n <= max_frames.  Synchronous: returns once the
   records are written at b->out.  -ENODEV without a server. */
int rxg_server_burst_dev(rxg_ctx *ctx, const rxg_dev_batch *b);

/* ------------------------------------------------------------------------- */
/* Transmit checksum generate: what ip_out computes (ip.c:97-118) for a batch  */
/* of frames whose Ethernet/IPv4/TCP headers the host has filled.  Writes      */
/* hdr_checksum (frame bytes 24-25) and tcp cksum (bytes 50-51) in place, both */
/* stored htons(calculate_checksum(..)) with the field zeroed while summing.   */
/* The TCP span is pseudo || frame[34 .. 14+total_length).                     */
/* ------------------------------------------------------------------------- */
typedef struct rxg_dev_tx_batch {
    void *frames;           /* dev, modified in place */
    const uint32_t *off64;  /* dev */
    const uint16_t *len;    /* dev */
    uint32_t n;
    uint32_t pad;
} rxg_dev_tx_batch;
int rxg_tx_cksum_dev(rxg_ctx *ctx, const rxg_dev_tx_batch *b, void *stream);

/* ------------------------------------------------------------------------- */
/* Counters                                                                   */
/* ------------------------------------------------------------------------- */
int rxg_counters_reset(rxg_ctx *ctx, void *stream);
/* Synchronous read of the RXG_NCOUNTERS uint64 counters (the replica rows summed), after
   every burst of this context has finished, on whatever stream it was launched. */
int rxg_counters_read(rxg_ctx *ctx, uint64_t *out);
/* The device keeps RXG_COUNTER_ROWS rows of the counter block: 64 replicas the kernels add
   into (so that workgroups do not all add to one cache line) and one row of corrections
   written by rxg_rx_replay when it re-classifies packets; counter k = sum over rows. */
#define RXG_COUNTER_ROWS 65
/* Device address of the uint64[RXG_COUNTER_ROWS][RXG_NCOUNTERS] block: an in-place RCCL
   all-reduce (sum) over it followed by rxg_counters_read merges counters across GPUs.  The
   replay's corrections reach the block in the context's stream order: with the next mirror
   patch launch, or at the latest at rxg_counters_read, rxg_sync or this call (read the
   block after the context's stream, as for the kernels' own counts). */
void *rxg_counters_dev(rxg_ctx *ctx);

/* ------------------------------------------------------------------------- */
/* In-order hand-off (the side effects of etherin.c:21-35, ip.c:28-39,        */
/* tcp_in.c:47-72).  The caller supplies the reference's own functions.       */
/* ------------------------------------------------------------------------- */
typedef struct rxg_handoff_ops {
    void *user;
    void (*free_mbuf)(void *user, void *mbuf);                               /* main.c:206   */
    int (*arp_in)(void *user, void *mbuf);                                   /* arp.c:113    */
    /* ip.c:30-32: if (!get_mac(src)) add_mac(src, mac) */
    int (*get_mac)(void *user, uint32_t ipv4_host, unsigned char *mac_out);  /* arp.c:215    */
    int (*add_mac)(void *user, uint32_t ipv4_host, const unsigned char *mac);/* arp.c:282    */
    void (*send_reset)(void *user, void *ip_hdr, void *tcp_hdr);             /* tcp_out.c:103*/
    /* tcp_in.c:66-68 + 71: max_seq_received update and AdjustSendWindow(tcb, ack) */
    void (*on_segment)(void *user, int32_t tcb_idx, uint32_t seq, uint32_t ack);
    /* tcpswitch[state](tcb, tcp_hdr, ip_hdr, mbuf)             tcp_states.c:257-265 */
    int (*tcpswitch)(void *user, int32_t tcb_idx, uint8_t state, void *tcp_hdr, void *ip_hdr,
                     void *mbuf);
    /* The reference's rx counters, globals of tcp_in.c:18-19 exported at tcp_in.h:7,11.  The
       replay increments them where tcp_in does, in packet order: *tcpnopcb at every findtcb
       miss (tcp_in.c:47-48); *tcpchecksumerror only with RXG_OPS_VERIFY_TCP_CKSUM, at every
       TCP segment whose checksum fails (tcp_in.c:37-40).  NULL: not kept. */
    int *tcpnopcb;
    int *tcpchecksumerror;
    uint32_t flags;      /* RXG_OPS_* */
} rxg_handoff_ops;

/* rxg_handoff_ops.flags.  RXG_OPS_VERIFY_TCP_CKSUM turns on the block tcp_in.c:37-41 compiles
   out (`if(0)`): a TCP segment whose pseudo || segment checksum is not 0x0000 (record flag
   RXG_F_TCP_OK clear) is freed and counted in *tcpchecksumerror after ip_in's ARP learn,
   before findtcb -- no reset, no hand-off.  Off (0) is the reference as shipped. */
#define RXG_OPS_VERIFY_TCP_CKSUM 0x1u

/* Performs, in packet order, the side effects ether_in() would have performed for
   pkts[0..n) given their records.  frames[i] = the frame bytes of mbufs[i].  It must
   follow the burst (rxg_rx_burst or rxg_rx_burst_dev) of the same batch on this context;
   for rxg_rx_burst_dev the batch's device buffers must stay valid until it returns.

   Sequential equivalence: handlers (tcpswitch[], send_reset, ...) mirror their writes to
   tcbs[] with rxg_tcb_* as they happen.  When a handler changes the mirror, every later
   TCP packet of the batch whose classification can depend on the change (same dport as a
   changed slot; any packet that reached findtcb pass 2 after a slot was removed or NULL
   slots appeared) is re-classified on the GPU against the updated table before it is
   replayed, and the counters are corrected.  The composition rxg_rx_burst + rxg_rx_replay
   therefore equals `for (i<n) ether_in(mbufs[i])`.  After rxg_rx_bursts_dev the launch's
   bursts are replayed in order, one call each, and their composition equals ether_in over
   their concatenation.  recs: the burst's records as the launch wrote them, rec_stride =
   their kind (RXG_REC8: rxg_rec8[], RXG_REC16: rxg_rec16[], RXG_REC48: rxg_rec48[]).
   -EINVAL when n differs from the burst to be replayed or the launch failed after it started
   (nothing is replayed then). */
int rxg_rx_replay(rxg_ctx *ctx, const rxg_handoff_ops *ops, void *const *mbufs,
                  void *const *frames, const void *recs, uint32_t n, uint32_t rec_stride);

/* Cumulative replay statistics of the context: out[0] packets marked stale by in-burst
   table writes, out[1] of them re-classified from the host index, out[2] re-classified on
   the GPU, out[3] GPU re-classify launches. */
int rxg_replay_stats(rxg_ctx *ctx, uint64_t out[4]);

/* Per-packet form with ether_in's contract (etherin.c:12-37: takes ownership of the mbuf,
   returns 0): a burst of one through the GPU followed by its replay.  For a stack that
   keeps calling ether_in(m) one mbuf at a time -- its shim is
     int ether_in(struct rte_mbuf *m) {
         return rxg_ether_in(g_rxg, &g_ops, m, rte_pktmbuf_mtod(m, void *),
                             rte_pktmbuf_data_len(m)); }
   Each call is a GPU round trip; batching (rxg_rx_burst) is the fast path.  Negative on
   a HIP error (the mbuf is then not consumed). */
int rxg_ether_in(rxg_ctx *ctx, const rxg_handoff_ops *ops, void *mbuf, void *frame, uint16_t data_len);

/* ------------------------------------------------------------------------- */
/* Payload hand-off.  The reference copies each       */
/* in-order segment's payload into a mempool message for the socket ring:     */
/* tcp_established -> PushData (tcp_windows.c:341-358) -> AdjustPair (:42-110) */
/* -> PushDataInQueue (:112-136) -> GetData (:138-186).  rxg gathers the      */
/* payloads of a whole burst on the device; during rxg_rx_replay the stack's  */
/* PushData asks rxg_payload_take whether the window would deliver exactly    */
/* that payload as one message, and uses the gathered bytes if so.            */
/* ------------------------------------------------------------------------- */
enum rxg_payload_flag {
    RXG_PM_GATHERED = 0x01,     /* arena holds this frame's payload                          */
    RXG_PM_REF_OVERSIZE = 0x02  /* len >= 1000: the reference's GetData asserts here
                                   (tcp_windows.c:170, its Buffer[1000]); rxg delivers it   */
};

typedef struct rxg_payload_msg {
    uint64_t arena_off;  /* payload at arena + arena_off: 16-byte aligned (gather), or the
                            payload's offset in the frame pool (rxg_rx_burst_payload_dev)   */
    uint32_t len;        /* Length = datalen (tcp_states.c:111), bytes at frame + 34 +
                            (data_off >> 4) * 4 (tcp_windows.c:164-166); 0 if not gathered   */
    uint32_t flags;      /* RXG_PM_*                                                        */
} rxg_payload_msg;

typedef struct rxg_payload_out {
    void *arena;             /* dev; each message padded with zeros to 16 bytes             */
    uint64_t arena_cap;      /* bytes                                                       */
    rxg_payload_msg *msgs;   /* dev, one per frame of the burst (flags 0: not gathered)      */
    uint64_t *arena_used;    /* dev, 1 entry: bytes the burst's candidates need; frames past
                                arena_cap are not gathered.  UINT64_MAX (~0): the gather's
                                offset look-back timed out (a workgroup never published), so
                                arena offsets are unreliable; rxg_payload_take then refuses
                                every payload of the burst (the stack's own PushData runs)   */
} rxg_payload_out;

/* Gathers, for the LAST burst on this context (rxg_rx_burst or rxg_rx_burst_dev; its
   device batch and records must still be valid), the payload of every TCP segment
   (verdict DISPATCH, RST_NOPCB or RST_LISTEN_NONSYN -- the replay may turn the latter into
   a DISPATCH) with datalen > 0 and the payload inside the frame.  Packet order;
   asynchronous on `stream`.  o->msgs and o->arena_used must stay valid until the burst's
   replay is done: the first rxg_payload_take after the gather copies them to the host.
   One gather is in flight per context: a gather waits (on the device) for the previous
   one, whatever streams they were issued on. */
int rxg_payload_gather_dev(rxg_ctx *ctx, const rxg_payload_out *o, void *stream);

/* The burst and its payload hand-off in ONE pass over the frames (rxg_rx_burst_dev followed
   by rxg_payload_gather_dev reads every payload byte twice).  The same records and counters
   as rxg_rx_burst_dev, and one message per frame for exactly the frames the gather takes
   (same len and flags; the message bytes are the same payload bytes), but each payload stays
   where its frame puts it: the arena has the frame pool's geometry.  For a candidate frame i
   the 64-byte lines of [frames + 64*off64[i] + start, + datalen) are written, unchanged, at
   the same offsets from `arena` (start = 34 + data_off*4), and msgs[i].arena_off = 64*off64[i]
   + start (not 16-byte aligned); other frames' lines are not written.  `arena` must hold
   64*(max off64[i]) + len rounded up to 64 bytes, and be 64-byte aligned; msgs 16-byte
   aligned (128-byte alignment measured 8 % faster than 64).  arena NULL: the hand-off by
   reference -- nothing is copied, each message names its payload in the frame pool itself
   (arena_off from `frames`), for a stack that keeps the pool's buffers until the socket side
   has consumed the messages (the reference's planned zero-copy path, currentstatus:9).
   rxg_payload_take then answers from these messages, as after a gather.  Asynchronous on
   `stream`. */
typedef struct rxg_payload_slots {
    void *arena;            /* dev: the pool's geometry (see above), or NULL         */
    rxg_payload_msg *msgs;  /* dev, b->n messages                                   */
} rxg_payload_slots;
int rxg_rx_burst_payload_dev(rxg_ctx *ctx, const rxg_dev_batch *b, const rxg_payload_slots *p, void *stream);
/* The same for one fixed-stride burst (rxg_rx_bursts_strided_dev's frame placement: frame i at
   64-byte slot b->slot0 + i * stride64 of the pool, msgs[i].arena_off = 64 * that slot + start). */
int rxg_rx_burst_strided_payload_dev(rxg_ctx *ctx, const void *frames, uint32_t stride64,
                                     const rxg_dev_strided_burst *b, uint32_t rec_kind,
                                     const rxg_payload_slots *p, void *stream);

/* Receive-window mirror: ReceiveWindow.CurrentSequenceNumber of tcbs[idx] and whether its
   SeqPairs list is non-empty (tcp_windows.h:37-44).  The stack calls it wherever it
   writes them itself: tcp_listen (tcp_states.c:182) and after its own PushData when
   rxg_payload_take refused.  rxg_tcb_remove / rxg_tcb_load forget the slot's window. */
int rxg_rcv_set(rxg_ctx *ctx, int32_t idx, uint32_t cur_seq, uint32_t pairs_pending);

/* Called from the stack's PushData(mbuf, tcp, Length, ptcb) (tcp_windows.c:341) while
   rxg_rx_replay runs the handlers of a packet of the gathered burst.  Returns 1 when the
   reference would deliver exactly this packet's payload as one message -- the mirror says
   the window of tcbs[idx] holds no pairs and CurrentSequenceNumber == seq, the payload was
   gathered with this length, and PushData's duplicate test (cur > seq + Length, u32) does
   not drop it.  Then *msg describes the message, the mirror advances to seq + Length, and
   the stack does what AdjustPair + GetData + PushDataInQueue would have: ptcb->ack =
   seq + Length + (FIN ? 1 : 0), CurrentSequenceNumber = seq + Length, enqueue a message of
   Length bytes (the gathered ones), free the mbuf.  Returns 0 otherwise (the stack runs its
   own PushData, then rxg_rcv_set); negative on error. */
int rxg_payload_take(rxg_ctx *ctx, int32_t idx, uint32_t seq, uint32_t length, rxg_payload_msg *msg);

/* ------------------------------------------------------------------------- */
/* Synthetic traffic (bench / tests): Eth + IPv4 (IHL 5) + TCP (doff 5, ACK)   */
/* frames with valid checksums, SURVEY.md §8(d).                               */
/* ------------------------------------------------------------------------- */
typedef struct rxg_synth_params {
    uint64_t seed;        /* payload / header PRNG seed                          */
    uint32_t n;           /* frames                                              */
    uint32_t nflows;      /* flow f: src 10.(f>>16).(f>>8).(f), sport 1024+f%64511 */
    uint32_t dst_ip_host; /* 192.168.78.2 = 0xC0A84E02 (config.h:8)             */
    uint16_t dport;       /* 80                                                  */
    uint16_t mix;         /* 0: all frames len_a; 1: IMIX 64/576/1500 at 7:4:1    */
    uint16_t len_a;       /* frame length when mix == 0                          */
    uint16_t pad;
} rxg_synth_params;

/* Fills off64/len (dev) and frames (dev) for p->n frames, packed at 64-byte aligned
   starts; returns the arena bytes used in *arena_bytes.  Frame flows are uniform over
   nflows (stored per frame in flow_out, dev, may be NULL). */
int rxg_synth_dev(rxg_ctx *ctx, const rxg_synth_params *p, void *frames, uint64_t frames_cap,
                  uint32_t *off64, uint16_t *len, uint32_t *flow_out, uint64_t *arena_bytes,
                  void *stream);
/* Host helper: the arena bytes rxg_synth_dev needs for p. */
uint64_t rxg_synth_arena_bytes(const rxg_synth_params *p);

/* ------------------------------------------------------------------------- */
/* Device memory helpers (so ctypes/C callers need no other HIP binding).      */
/* ------------------------------------------------------------------------- */
int rxg_dev_alloc(rxg_ctx *ctx, uint64_t bytes, void **out);
int rxg_dev_free(rxg_ctx *ctx, void *p);
int rxg_host_alloc_pinned(rxg_ctx *ctx, uint64_t bytes, void **out);
int rxg_host_free_pinned(rxg_ctx *ctx, void *p);
/* Zero-copy batches.  Host memory from rxg_host_alloc_pinned, or caller memory registered
   here (e.g. the mbuf pool's hugepages: hipHostRegister, mapped), may be passed to
   rxg_rx_burst_dev / rxg_tx_cksum_dev as `frames`, `off64`, `len` and `out` through its
   device alias: the kernel reads (and for tx rewrites in place) the frames over PCIe, with
   no staging copy.  rxg_tx_cksum_dev on host frames writes back only the rewritten first
   line of each frame, not the frame (C5).  The alias is valid until
   rxg_host_unregister. */
int rxg_host_register(rxg_ctx *ctx, void *host, uint64_t bytes, void **dev_alias);
int rxg_host_unregister(rxg_ctx *ctx, void *host);
int rxg_memcpy_h2d(rxg_ctx *ctx, void *dst, const void *src, uint64_t bytes, void *stream);
int rxg_memcpy_d2h(rxg_ctx *ctx, void *dst, const void *src, uint64_t bytes, void *stream);
int rxg_memset_dev(rxg_ctx *ctx, void *dst, int value, uint64_t bytes, void *stream);
int rxg_stream_sync(rxg_ctx *ctx, void *stream);

/* Event timing on a stream (bench): returns ms between two recorded events. */
typedef struct rxg_event rxg_event;
int rxg_event_create(rxg_ctx *ctx, rxg_event **out);
int rxg_event_record(rxg_ctx *ctx, rxg_event *e, void *stream);
int rxg_event_elapsed_ms(rxg_ctx *ctx, rxg_event *a, rxg_event *b, float *ms);
int rxg_event_destroy(rxg_ctx *ctx, rxg_event *e);

/* Last error text of this thread (static storage). */
const char *rxg_last_error(void);

/* ------------------------------------------------------------------------- */
/* Groups: several GPUs behind one rx loop.  The reference   */
/* runs one rx lcore calling ether_in per packet (main.c:391-399); a group     */
/* keeps that single loop and spreads each burst over its members.            */
/*  - every member holds a full replica of the TCB / ARP / receive-window      */
/*    mirrors: the rxg_group_* mirror calls apply to all of them;             */
/*  - rxg_group_rx_burst cuts the burst into one contiguous shard per member   */
/*    (ceil(n/ndev) frames, so cfg->max_batch is per shard), runs the shards   */
/*    concurrently (one worker thread per member, kept for the group's life)   */
/*    and returns the records in packet order;                                 */
/*  - rxg_group_rx_burst_dev takes a burst already in GPU-visible memory as    */
/*    one shard per member and launches every member at once (no host copy);   */
/*  - rxg_group_rx_replay replays the shards in packet order.  Handlers mirror */
/*    their tcbs[] writes with rxg_group_tcb_* (not the member calls), so a    */
/*    later member's replay sees them and re-classifies what they affect: the  */
/*    composition equals ether_in over the whole burst, as for one context.    */
/* Members are plain contexts (rxg_group_member) for everything else: device    */
/* batches, payload gathers, timing.  Group calls are made from the rx thread;  */
/* rxg_group_tcb_post is the any-thread exception (member rxg_tcb_post is not  */
/* used on a group: per-member queues could order two posts differently).      */
/* ------------------------------------------------------------------------- */
typedef struct rxg_group rxg_group;
/* One context per devices[i] (the same device may repeat), each with *cfg's sizes. */
int rxg_group_init(const int32_t *devices, uint32_t ndev, const rxg_config *cfg, rxg_group **out);
int rxg_group_fini(rxg_group *g);
uint32_t rxg_group_size(rxg_group *g);
rxg_ctx *rxg_group_member(rxg_group *g, uint32_t i);
int rxg_group_tcb_upsert(rxg_group *g, int32_t idx, const rxg_tcb_tuple *t);
int rxg_group_tcb_remove(rxg_group *g, int32_t idx);
int rxg_group_tcb_set_state(rxg_group *g, int32_t idx, uint8_t state);
int rxg_group_tcb_load(rxg_group *g, const rxg_tcb_tuple *tcbs, const uint8_t *live, int32_t ntcb);
/* Any thread: one lock-free queue for the whole group (the members apply posts in one
   order), drained at the start of rxg_group_rx_burst or by rxg_group_tcb_drain. */
int rxg_group_tcb_post(rxg_group *g, const rxg_tcb_op *op);
int rxg_group_tcb_drain(rxg_group *g);
int rxg_group_arp_load(rxg_group *g, const uint32_t *ipv4_host, uint32_t n);
int rxg_group_arp_learned(rxg_group *g, uint32_t ipv4_host);
int rxg_group_arp_disable(rxg_group *g);
int rxg_group_rcv_set(rxg_group *g, int32_t idx, uint32_t cur_seq, uint32_t pairs_pending);
int rxg_group_rx_burst(rxg_group *g, const rxg_pkt_view *pkts, uint32_t n, uint32_t rec_kind,
                       void *out_host);
/* Device-resident group burst (contiguous batches to the GPUs, the host
   replays in global packet order), replacing main.c:391-399's loop for frames the caller
   already has in GPU-visible memory.  shards[i] (nshards = group size) is member i's
   contiguous share of the burst, in packet order (shard 0 first; any n, 0 included), with
   the rxg_dev_batch rules of rxg_rx_burst_dev in memory member i's GPU reads: its HBM, or
   host memory registered on member i (rxg_host_register; e.g. the mbuf pool registered on
   every member).  Every shard has the same rec_kind.  Each member classifies its shard
   against its replica of the mirror as it stands at the call; the launches are asynchronous,
   one per member on its own stream, so the shards run concurrently.  rxg_group_sync waits
   for them; rxg_group_rx_replay then replays n = sum of the shards' n records, laid out in
   packet order with that stride, exactly as after rxg_group_rx_burst (each member's shard
   buffers must stay valid until the replay returns). */
int rxg_group_rx_burst_dev(rxg_group *g, const rxg_dev_batch *shards, uint32_t nshards);
/* Waits for every member's stream (rxg_sync on each). */
int rxg_group_sync(rxg_group *g);
int rxg_group_rx_replay(rxg_group *g, const rxg_handoff_ops *ops, void *const *mbufs,
                        void *const *frames, const void *recs, uint32_t n, uint32_t rec_stride);
/* rxg_payload_take on the member whose shard is being replayed (0 outside a replay);
   each member's rxg_payload_gather_dev covers its own shard. */
int rxg_group_payload_take(rxg_group *g, int32_t idx, uint32_t seq, uint32_t length, rxg_payload_msg *msg);
/* Index of the member being replayed, -1 outside rxg_group_rx_replay. */
int32_t rxg_group_replaying(rxg_group *g);
int rxg_group_counters_reset(rxg_group *g);
/* The members' counters summed: an RCCL all-reduce (sum, uint64) of the members' counter
   blocks over xGMI when the members are distinct GPUs (one communicator per member,
   ncclCommInitAll at the first call), else summed on the host (members sharing a GPU). */
int rxg_group_counters_read(rxg_group *g, uint64_t *out);
/* 1 when rxg_group_counters_read merges with RCCL, 0 when on the host; negative on error.
   RCCL is loaded at the first merge over distinct GPUs (dlopen of librccl.so): librxg.so
   does not depend on it, and a host without it merges on the host (same sums). */
int rxg_group_counters_rccl(rxg_group *g);
/* Why the merge is on the host (empty when RCCL is used or not decided yet). */
const char *rxg_group_counters_rccl_why(rxg_group *g);
/* Last error of a group call on this thread (member errors carry their text). */
const char *rxg_group_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* RXG_H */
