// rxg_ctx.h — the context behind the rxg C ABI (include/rxg.h), shared by the host-side
// translation units (internal: not installed, not part of the ABI):
//   rxg_host.cpp    context, TCB / ARP mirrors, table-reader ordering, launched bursts, tx,
//                   counters
//   rxg_server.cpp  latency mode (the persistent server kernel) and host-buffer bursts
//   rxg_replay.cpp  the per-packet replay into the caller's handlers, the payload hand-off,
//                   ether_in
//   rxg_util.cpp    synthetic frames, memory and event helpers
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <climits>
#include <cstddef>
#include <cstdint>
#include <unordered_map>
#include <vector>

#include "rxg.h"
#include "rxg_common.h"
#include "rxg_kernels.h"
#include "rxg_mirror.h"
#include "rxg_opqueue.h"
#include "rxg_packpool.h"
#include "rxg_srvfsm.h"

// Everything below is internal to librxg.so: hidden, never exported.
#pragma GCC visibility push(hidden)

// Sets the calling thread's rxg_last_error text and returns code (rxg_host.cpp).
int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

#define HIP_OK(expr)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail(-EIO, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__,      \
                        __LINE__);                                                          \
    } while (0)

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
};

// The latency-mode server's device side as rxg::SrvFsm sees it (rxg_srvfsm.h); defined in
// rxg_server.cpp.
struct SrvPort {
    rxg_ctx *c;
    unsigned long long done() const;
    bool exited() const;
    void write(unsigned long long q);
    void cancel(unsigned long long q);
    void request_stop();
    int launch();
    void sync();
};

struct rxg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t max_blocks = 0;        // rxg_config.max_blocks: grid cap (0 = occupancy grid)
    uint32_t grid_pay = 512;        // rxg_rx_burst_payload_dev's grid (set at init)
    uint32_t grid_rec8 = 0, grid_rec16 = 0, grid_rec48 = 0, grid_tx = 0;
    uint32_t grid_ref8 = 0, grid_ref16 = 0, grid_ref48 = 0;  // the by-reference hand-off's
    rxg::PackPool pack_pool;  // rxg_rx_burst's packing threads

    // tcbs[] writes posted by other threads (rxg_tcb_post), applied by the rx thread
    rxg::MpscRing<rxg_tcb_op> posted{RXG_TCB_QUEUE_CAP};

    // host mirror of tcbs[0..ntcb) and the device words each write changes (rxg_mirror.h)
    rxg::TcbMirror mir;
    bool dirty = true;  // mirror writes not on the device yet

    // device mirror
    DevBuf buckets, listen;
    uint32_t bucket_mask = 0;
    int32_t dev_ntcb = 0;
    int32_t dev_min_null = INT32_MAX;
    // Ordering of table writes against the kernels that read the tables:
    // mirror writes run on `stream`; a burst on another stream waits for mirror_ev (once per
    // write), and the next mirror write waits for every stream other than `stream` that
    // launched a table-reading kernel since the last write (one entry per stream, so a
    // reader on s1 followed by one on s2 are both waited for): the event recorded after the
    // stream's latest such launch, or, with RXG_CFG_STREAMS_OUTLIVE_WRITES, recorded on the
    // stream at the write, which keeps the caller's stream free of a marker packet per launch
    // (C4 on a caller stream 78.2 -> 73.2 us per launch, C2 24.5 -> 20.3).
    hipEvent_t mirror_ev = nullptr;
    bool mirror_ev_set = false;
    bool mirror_ev_stale = false;  // a write on `stream` after mirror_ev's last recording
                                   // (recorded when another stream or the server needs it)
    uint64_t table_writes = 0;  // mirror_ev recordings (device table writes) so far
    struct Reader {
        hipStream_t s;
        hipEvent_t e;
        bool pending;     // `s` launched a table reader since the last write (not yet waited for)
        bool recorded;    // e was recorded after that launch (per-launch mode)
        uint64_t waited;  // table_writes when `s` last waited for mirror_ev (~0: never)
    };
    std::vector<Reader> readers;
    // Patch upload ring: a list is read by its patch kernel or by the burst that carries it
    // (device memory the host writes through a large BAR, else pinned host memory read over
    // PCIe), so a buffer is reused only after that launch ran; kPatchBufs buffers, each with
    // its event, and the host waits only when all of them are in flight (a patch kernel waits
    // on the device for bursts running on caller streams, which can be long).
    static constexpr int kPatchBufs = 4;
    struct PatchBuf {
        rxg::MirrorPatch *h = nullptr;
        uint32_t cap = 0;
        hipEvent_t ev = nullptr;
        bool set = false;
    } patch[kPatchBufs];
    int patch_next = 0;
    // With a large BAR the patch buffers are device memory the host writes through the BAR,
    // and a launch on `stream` carries the burst's patch list itself (launch_bursts: no patch
    // launch before it); defer_patch asks apply_patches for that, ip_* is the list taken.
    bool patch_dev = false;
    bool defer_patch = false;
    const rxg::MirrorPatch *ip_list = nullptr;
    uint32_t ip_n = 0;
    int ip_buf = -1;
    uint32_t ip_tables = 0;  // 1 << target of every patch in the carried list (rxg_mirror.h)
    // HDP_MEM_COHERENCY_FLUSH_CNTL (hipDeviceProp_t::hdpMemFlushCntl; null if the runtime
    // gives none): host writes through the BAR are flushed to memory before a kernel reads them
    volatile uint32_t *hdp_flush = nullptr;

    unsigned long long *counters = nullptr;
    // the replays' counter corrections not yet on the device: added by the next mirror patch
    // launch, or by counters_add at the next read / sync / rxg_counters_dev (flush_delta)
    int64_t pend_delta[RXG_NCOUNTERS] = {};
    bool pend = false;

    // mirror changes since the last clear, for rxg_rx_replay's re-classification
    uint64_t gen = 0;
    std::vector<rxg::TupleKey> touched_keys;  // tuples (old and new) of changed slots
    std::vector<int32_t> touched_listen; // dports whose LISTENING slots changed (pass 2)
    bool touched_all = false;            // whole table replaced
    bool touched_pass2 = false;          // min_null moved (the pass-2 NULL-slot flag)
    bool replay_on_device = false;       // RXG_CFG_REPLAY_ON_DEVICE
    bool lazy_readers = false;           // RXG_CFG_STREAMS_OUTLIVE_WRITES
    std::vector<hipStream_t> registered; // that mode's caller streams (rxg_stream_register)
    uint64_t rp_stats[4] = {0, 0, 0, 0}; // marked, host fix-ups, device fix-ups, launches

    // the last burst's device batch (re-classification reads it again)
    // The last launch's bursts (one, or several of one frame pool: rxg_rx_bursts_dev) and
    // the one a replay / gather refers to next (last_off .. last_recs below).
    struct BurstRef {
        const uint32_t *off64;  // nullptr for a fixed-stride burst (slot0, stride64)
        const uint16_t *len;
        uint32_t n;
        const uint8_t *recs;
        uint32_t slot0 = 0, stride64 = 0;
    };
    std::vector<BurstRef> last_bursts;
    uint32_t replay_cursor = 0;
    // writes absorbed by the replays of this launch's earlier bursts (they came after every
    // burst of the launch was classified)
    std::vector<rxg::TupleKey> launch_keys;
    std::vector<int32_t> launch_listen;
    bool launch_all = false, launch_pass2 = false;
    const uint8_t *last_frames = nullptr;
    const uint32_t *last_off = nullptr;  // nullptr: a fixed-stride burst (burst_offsets)
    uint32_t last_slot0 = 0, last_stride64 = 0;
    DevBuf d_soff;                       // a fixed-stride burst's offsets, written on demand
    uint32_t soff_slot0 = 0, soff_stride64 = 0, soff_n = 0;  // what d_soff holds (n 0: nothing),
    hipStream_t soff_stream = nullptr;                        // written on this stream
    const uint16_t *last_len = nullptr;
    uint32_t last_n = 0;
    bool burst_ok = false;  // the last burst was launched (device) / completed (host buffers)
    const uint8_t *last_recs = nullptr;  // the burst's records (device) and their size
    uint32_t last_stride = 0;
    DevBuf d_sel, d_fix;

    // payload hand-off: receive-window mirror (0 unknown, 1 no pairs, 2 pairs pending) and
    // the gathered burst's message descriptors (pinned host copy)
    std::vector<uint32_t> rcv_cur;
    std::vector<uint8_t> rcv_state;
    DevBuf d_pg_status, d_pg_ticket;
    unsigned long long pg_tickets = 0;  // workgroups the gathers have launched so far
    uint32_t pg_epoch = 0;
    rxg_payload_msg *h_pm = nullptr;
    const rxg_payload_msg *d_pm = nullptr;  // the gather's descriptors (device)
    uint32_t h_pm_cap = 0, pm_n = 0;
    bool pm_pending = false;  // h_pm not fetched yet for this gather
    hipEvent_t pm_ev = nullptr;
    int64_t replay_pos = -1;  // packet whose handlers rxg_rx_replay is running

    // ARP mirror (host set + device open-addressing table, rxg_mirror.h)
    bool arp_enabled = false, arp_dirty = false;
    rxg::ArpMirror arp;
    std::unordered_map<uint32_t, int> arp_since_burst;  // learned after the last burst
    DevBuf d_arp;
    uint32_t arp_mask = 0;

    // replay scratch, kept across calls
    std::vector<rxg_rec16> rp_cur;
    std::vector<uint32_t> rp_seq;
    std::vector<uint64_t> rp_filter;
    const uint64_t *pm_used = nullptr;  // the gather's arena_used (device)
    bool pm_poisoned = false;           // that gather timed out: no payload is handed out

    // host-buffer burst staging
    uint32_t max_batch = 0;
    uint64_t max_bytes = 0;
    uint8_t *h_arena = nullptr;
    uint32_t *h_off = nullptr;
    uint16_t *h_len = nullptr;
    uint8_t *d_arena = nullptr;
    uint32_t *d_off = nullptr;
    uint16_t *d_len = nullptr;
    uint8_t *d_out = nullptr;
    uint8_t *h_out = nullptr;        // pinned records of zero-copy host bursts
    uint64_t zc_bytes = 64ull << 20; // host bursts up to this many staged bytes: zero-copy

    // latency-mode server (rxg_server_*): a persistent kernel on its own
    // stream; the host-burst staging in device memory the host writes through the BAR
    // (dev = true) or in coherent host memory; the mailbox likewise (mdev), answers and
    // records in host memory
    struct Server {
        bool on = false;        // configured (the kernel may have exited idle: relaunched on demand)
        rxg::SrvFsm<SrvPort> fsm;  // Down / Up / Failed (rxg_srvfsm.h)
        rxg::SrvReq req{};      // the request SrvPort::write posts
        // its inline descriptors (kSrvInlineDesc): mailbox words 16-39, SrvMbox::ioff / ilen
        alignas(16) unsigned long long idesc[rxg::kSrvPollWords - 16] = {};
        bool dev = false;       // arena / off / len in device memory (host writes only)
        bool mdev = false;      // mbox in device memory (large BAR, no RXG_SRV_HOST_MAILBOX)
        hipStream_t st = nullptr;
        rxg::SrvMbox *mbox = nullptr;  // host-written words: seq, request, stop
        rxg::SrvMbox *ret = nullptr;   // server-written words: done, exited (host memory; = mbox if !mdev)
        rxg::SrvCtl *ctl = nullptr;
        uint8_t *arena = nullptr;
        uint32_t *off = nullptr;
        uint16_t *len = nullptr;
        uint8_t *out = nullptr;
        std::vector<uint32_t> h_off;  // host copies of the packed offsets (device staging is
        std::vector<uint16_t> h_len;  // write-only from the host: a read would cross PCIe)
        uint32_t rec_kind = 0, blocks = 1, max_frames = 0;
        uint64_t max_bytes = 0, idle_ticks = 0;
        unsigned long long seq = 0;
        uint64_t synced_writes = 0;    // table_writes whose mirror_ev the host has waited for
    } srv;
};

// patch lists longer than this go through their own launch (every workgroup of a launch that
// carries a list stores all of it)
inline constexpr uint32_t kLaunchPatchMax = 256;

// Host stores into device memory through the BAR (write-combined), made visible to the next
// kernel: the CPU's write-combining buffers drained (sfence), the GPU's HDP write path flushed
// (its flush register), then a read of the last word written -- a PCIe read completes only
// after every posted write before it, the flush among them (the ROCm runtime's own recipe
// for kernel arguments in device memory).  `last` NULL: no readback.
void bar_publish(const rxg_ctx *c, const volatile uint32_t *last);

inline constexpr size_t kCounterBytes = (size_t)RXG_COUNTER_ROWS * RXG_NCOUNTERS * sizeof(uint64_t);

struct rxg_event {
    hipEvent_t e;
};

inline int set_device(rxg_ctx *c) { HIP_OK(hipSetDevice(c->device)); return 0; }

inline int ensure(DevBuf &b, size_t bytes)
{
    if (b.bytes >= bytes && b.p) return 0;
    if (b.p) HIP_OK(hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
    size_t want = std::max<size_t>(bytes, 256);
    HIP_OK(hipMalloc(&b.p, want));
    b.bytes = want;
    return 0;
}

inline hipStream_t pick(rxg_ctx *c, void *s) { return s ? (hipStream_t)s : c->stream; }

// The device tables as the kernels read them (DevTable, rxg_kernels.h).
inline rxg::DevTable table_view(const rxg_ctx *c)
{
    rxg::DevTable t;
    t.buckets = (const uint4 *)c->buckets.p;
    t.listen = (const int32_t *)c->listen.p;
    t.bucket_mask = c->bucket_mask;
    t.ntcb = c->dev_ntcb;
    t.min_null = c->dev_min_null;
    t.arp = (const uint4 *)c->d_arp.p;
    t.arp_mask = c->arp_enabled ? c->arp_mask : 0u;
    t.arp_flags = c->arp_enabled ? (rxg::kArpOn | (c->arp.has_zero ? rxg::kArpZero : 0u)) : 0u;
    return t;
}

// rxg_host.cpp: the mirror upload, the replay bookkeeping of a burst set and its offsets.
int tcb_push(rxg_ctx *c);
void select_burst(rxg_ctx *c, uint32_t j);
int begin_bursts(rxg_ctx *c, const void *frames, const rxg_dev_burst *bursts, uint32_t k, uint32_t rec_kind,
                 const char *who, uint32_t stride64 = 0);
int burst_offsets(rxg_ctx *c, hipStream_t st, const uint32_t **out);
// mirror_ev recorded on `stream` if a write since its last recording has not been (rxg_host.cpp)
int mirror_event(rxg_ctx *c);
// the pending counter corrections (rxg_ctx::pend_delta) to the device, on c->stream
int flush_delta(rxg_ctx *c);

// the counter block's row of replay corrections (rxg.h RXG_COUNTER_ROWS: the last)
inline unsigned long long *correction_row(rxg_ctx *c)
{
    return c->counters + (size_t)(RXG_COUNTER_ROWS - 1) * RXG_NCOUNTERS;
}

inline bool rec_kind_ok(uint32_t k) { return k == RXG_REC8 || k == RXG_REC16 || k == RXG_REC48; }

#pragma GCC visibility pop
