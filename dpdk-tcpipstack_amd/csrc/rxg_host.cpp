// rxg_host.cpp — host side of the rxg C ABI (include/rxg.h).
//
// Owns one GPU context: its stream, the device TCB mirror (rebuilt from the host mirror
// whenever a rxg_tcb_* call made it dirty), the counter block, and the pinned staging used
// by the host-buffer entry points.  There is no CPU compute path: without a usable HIP
// device every compute entry point returns -ENODEV / -EIO.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <cstddef>
#include <climits>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <thread>
#include <unordered_map>
#include <immintrin.h>
#include <vector>

#include "rxg.h"
#include "rxg_common.h"
#include "rxg_kernels.h"
#include "rxg_mirror.h"
#include "rxg_opqueue.h"
#include "rxg_packpool.h"
#include "rxg_srvfsm.h"

using namespace rxg;

static_assert(sizeof(rxg_rec16) == 16, "rxg_rec16 layout");
static_assert(sizeof(rxg_rec48) == 48, "rxg_rec48 layout");
static_assert(sizeof(rxg_tcb_tuple) == 20, "rxg_tcb_tuple layout");

// ------------------------------------------------------------------------ errors ---
static thread_local char g_err[512];

static int fail(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

#define HIP_OK(expr)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail(-EIO, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__,      \
                        __LINE__);                                                          \
    } while (0)

extern "C" const char *rxg_last_error(void) { return g_err; }

// ---------------------------------------------------------------------- context ---
struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
};

// The latency-mode server's device side as rxg::SrvFsm sees it (rxg_srvfsm.h); defined
// after rxg_ctx.
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
    // Experiment switches: only an experiment build (make experiments, -DRXG_EXPERIMENTS,
    // rxg/librxg_exp.so for scripts/kbench.py and pgbench.py) reads them from the
    // environment; in the product library they stay 0.
    rxg::PackPool pack_pool;  // rxg_rx_burst's packing threads
    int variant = 0;     // RXG_VARIANT: rx kernel variants (rxg_kernels_exp.hip)
    int nocount = 0;     // RXG_NOCOUNT: skip the counter reduction
    int pg_variant = 0;  // RXG_PG_VARIANT: payload-gather variants
    int mirror_rebuild = 0;  // RXG_MIRROR_REBUILD: every mirror sync a full rebuild (round 1)
    int replay_coarse = 0;   // RXG_REPLAY_COARSE: a write stales every later TCP packet on
                             // its dport and all fix-ups run on the GPU (round 1)

    // tcbs[] writes posted by other threads (rxg_tcb_post), applied by the rx thread
    rxg::MpscRing<rxg_tcb_op> posted{RXG_TCB_QUEUE_CAP};

    // host mirror of tcbs[0..ntcb) and the device words each write changes (rxg_mirror.h)
    TcbMirror mir;
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
    uint64_t table_writes = 0;  // mirror_ev recordings (device table writes) so far
    struct Reader {
        hipStream_t s;
        hipEvent_t e;
        bool pending;     // `s` launched a table reader since the last write (not yet waited for)
        bool recorded;    // e was recorded after that launch (per-launch mode)
        uint64_t waited;  // table_writes when `s` last waited for mirror_ev (~0: never)
    };
    std::vector<Reader> readers;
    // Patch upload ring: the patch kernel reads its list from pinned host memory over PCIe,
    // so a buffer is reused only after its kernel ran; kPatchBufs buffers, each with its
    // event, and the host waits only when all of them are in flight (a patch kernel waits on
    // the device for bursts running on caller streams, which can be long).
    static constexpr int kPatchBufs = 4;
    struct PatchBuf {
        MirrorPatch *h = nullptr;
        uint32_t cap = 0;
        hipEvent_t ev = nullptr;
        bool set = false;
    } patch[kPatchBufs];
    int patch_next = 0;

    unsigned long long *counters = nullptr;

    // mirror changes since the last clear, for rxg_rx_replay's re-classification
    uint64_t gen = 0;
    std::vector<TupleKey> touched_keys;  // tuples (old and new) of changed slots
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
    std::vector<TupleKey> launch_keys;
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
    ArpMirror arp;
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
        SrvReq req{};           // the request SrvPort::write posts
        // its inline descriptors (kSrvInlineDesc): mailbox words 16-39, SrvMbox::ioff / ilen
        alignas(16) unsigned long long idesc[kSrvPollWords - 16] = {};
        bool dev = false;       // arena / off / len in device memory (host writes only)
        bool mdev = false;      // mbox in device memory (large BAR, no RXG_SRV_HOST_MAILBOX)
        hipStream_t st = nullptr;
        SrvMbox *mbox = nullptr;  // host-written words: seq, request, stop
        SrvMbox *ret = nullptr;   // server-written words: done, exited (host memory; = mbox if !mdev)
        SrvCtl *ctl = nullptr;
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

static constexpr size_t kCounterBytes = (size_t)RXG_COUNTER_ROWS * RXG_NCOUNTERS * sizeof(uint64_t);

struct rxg_event {
    hipEvent_t e;
};

static int set_device(rxg_ctx *c) { HIP_OK(hipSetDevice(c->device)); return 0; }

static int ensure(DevBuf &b, size_t bytes)
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

extern "C" int rxg_abi_version(void) { return RXG_ABI_VERSION; }

extern "C" int rxg_init(const rxg_config *cfg, rxg_ctx **out)
{
    if (!out) return fail(-EINVAL, "rxg_init: out is NULL");
    *out = nullptr;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0)
        return fail(-ENODEV, "rxg_init: no HIP device (%s)", hipGetErrorString(e));
    rxg_ctx *c = new rxg_ctx();
    c->device = cfg ? cfg->device : 0;
    if (c->device < 0 || c->device >= ndev) {
        delete c;
        return fail(-EINVAL, "rxg_init: device %d of %d", cfg ? cfg->device : 0, ndev);
    }
    int rc = set_device(c);
    if (rc) { delete c; return rc; }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, c->device) == hipSuccess) {
        // one generation of resident workgroups per CU (grid-stride over slices)
        const uint32_t cus = (uint32_t)prop.multiProcessorCount;
        c->grid_rec8 = cus * (uint32_t)rx_blocks_per_cu(8);
        c->grid_rec16 = cus * (uint32_t)rx_blocks_per_cu(16);
        c->grid_rec48 = cus * (uint32_t)rx_blocks_per_cu(48);
        c->grid_tx = cus * (uint32_t)rx_blocks_per_cu(0);
        // the fused burst + payload hand-off moves as many bytes out as in: 2 workgroups per CU
        // (8 waves) measured faster than the occupancy grid's 3 (C3 621 against 627 us, C4 174
        // against 177)
        c->grid_pay = cus * 2u;
    }
    if (cfg) {
        c->replay_on_device = (cfg->flags & RXG_CFG_REPLAY_ON_DEVICE) != 0;
        c->lazy_readers = (cfg->flags & RXG_CFG_STREAMS_OUTLIVE_WRITES) != 0;
        c->max_blocks = cfg->max_blocks;
        if (cfg->zc_bytes) c->zc_bytes = cfg->zc_bytes;
    }
#ifdef RXG_EXPERIMENTS
    if (const char *g = getenv("RXG_MAX_BLOCKS")) c->max_blocks = (uint32_t)atoi(g);
    if (const char *v = getenv("RXG_VARIANT")) c->variant = atoi(v);
    if (const char *v = getenv("RXG_NOCOUNT")) c->nocount = atoi(v);
    if (const char *v = getenv("RXG_PG_VARIANT")) c->pg_variant = atoi(v);
    if (const char *v = getenv("RXG_ZC_BYTES")) c->zc_bytes = strtoull(v, nullptr, 10);
    if (const char *v = getenv("RXG_MIRROR_REBUILD")) c->mirror_rebuild = atoi(v);
    if (const char *v = getenv("RXG_REPLAY_COARSE")) c->replay_coarse = atoi(v);
    if (const char *v = getenv("RXG_MIRROR_LOAD_PCT")) c->mir.max_load_pct = (uint32_t)atoi(v);
    if (c->replay_coarse) c->replay_on_device = true;
#endif
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return fail(-EIO, "rxg_init: hipStreamCreate failed");
    }
    bool ev_ok = hipEventCreateWithFlags(&c->mirror_ev, hipEventDisableTiming) == hipSuccess;
    for (auto &pb : c->patch) ev_ok = ev_ok && hipEventCreateWithFlags(&pb.ev, hipEventDisableTiming) == hipSuccess;
    if (!ev_ok) {
        rxg_fini(c);
        return fail(-EIO, "rxg_init: hipEventCreate failed");
    }
    if (hipMalloc(&c->counters, kCounterBytes) != hipSuccess ||
        hipMemset(c->counters, 0, kCounterBytes) != hipSuccess) {
        rxg_fini(c);
        return fail(-ENOMEM, "rxg_init: counters");
    }
    // the ARP bucket every lane reads while the mirror is off (classify_finish issues the
    // ARP probe unconditionally)
    if (ensure(c->d_arp, 256) || hipMemset(c->d_arp.p, 0, c->d_arp.bytes) != hipSuccess) {
        rxg_fini(c);
        return fail(-ENOMEM, "rxg_init: ARP mirror");
    }
    c->max_batch = cfg ? cfg->max_batch : 0;
    c->max_bytes = cfg ? cfg->max_bytes : 0;
    if (c->max_batch) {
        uint64_t ab = c->max_bytes ? c->max_bytes : (uint64_t)c->max_batch * 2048u;
        c->max_bytes = ab;
        if (hipHostMalloc((void **)&c->h_arena, ab, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void **)&c->h_off, c->max_batch * 4u, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void **)&c->h_len, c->max_batch * 2u, hipHostMallocDefault) != hipSuccess ||
            hipMalloc(&c->d_arena, ab) != hipSuccess ||
            hipMalloc(&c->d_off, c->max_batch * 4u) != hipSuccess ||
            hipMalloc(&c->d_len, c->max_batch * 2u) != hipSuccess ||
            hipMalloc(&c->d_out, (size_t)c->max_batch * 48u) != hipSuccess ||
            hipHostMalloc((void **)&c->h_out, (size_t)c->max_batch * 48u, hipHostMallocDefault) != hipSuccess) {
            rxg_fini(c);
            return fail(-ENOMEM, "rxg_init: staging for %u frames / %llu bytes", c->max_batch,
                        (unsigned long long)ab);
        }
    }
    *out = c;
    return 0;
}

extern "C" int rxg_fini(rxg_ctx *c)
{
    if (!c) return 0;
    (void)hipSetDevice(c->device);
    // A server kernel that missed its time limit may still be resident, reading the tables and
    // counters and writing the staging and records.  Stop is retried for a bounded time (each
    // try waits exit_timeout); if the kernel still has not exited, everything it can reach is
    // deliberately leaked -- the context included -- rather than freed under it: -EIO.
    int src = rxg_server_stop(c);
    for (int t = 0; src && t < 4; ++t) src = rxg_server_stop(c);
    if (src)
        return fail(-EIO, "rxg_fini: the server kernel has not exited; the context and every buffer it can "
                          "reach are left allocated (leaked)");
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto &r : c->readers)  // table readers still running on caller streams
        if (r.pending && (r.recorded || hipEventRecord(r.e, r.s) == hipSuccess))
            (void)hipEventSynchronize(r.e);
    for (DevBuf *b : {&c->buckets, &c->listen, &c->d_sel, &c->d_fix, &c->d_arp, &c->d_pg_status, &c->d_pg_ticket,
                      &c->d_soff})
        if (b->p) (void)hipFree(b->p);
    if (c->h_pm) (void)hipHostFree(c->h_pm);
    if (c->pm_ev) (void)hipEventDestroy(c->pm_ev);
    for (auto &pb : c->patch) {
        if (pb.h) (void)hipHostFree(pb.h);
        if (pb.ev) (void)hipEventDestroy(pb.ev);
    }
    for (auto &r : c->readers) (void)hipEventDestroy(r.e);
    if (c->mirror_ev) (void)hipEventDestroy(c->mirror_ev);
    if (c->counters) (void)hipFree(c->counters);
    if (c->h_arena) (void)hipHostFree(c->h_arena);
    if (c->h_off) (void)hipHostFree(c->h_off);
    if (c->h_len) (void)hipHostFree(c->h_len);
    if (c->d_arena) (void)hipFree(c->d_arena);
    if (c->d_off) (void)hipFree(c->d_off);
    if (c->d_len) (void)hipFree(c->d_len);
    if (c->d_out) (void)hipFree(c->d_out);
    if (c->h_out) (void)hipHostFree(c->h_out);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return 0;
}

extern "C" int rxg_sync(rxg_ctx *c)
{
    if (!c) return fail(-EINVAL, "rxg_sync: ctx NULL");
    HIP_OK(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" void *rxg_stream(rxg_ctx *c) { return c ? (void *)c->stream : nullptr; }

static hipStream_t pick(rxg_ctx *c, void *s) { return s ? (hipStream_t)s : c->stream; }

// -------------------------------------------------------------------- TCB mirror ---
// What a write to tcbs[idx] can change for packets of the burst being replayed: pass 1 of
// packets with the slot's tuple, pass 2 of packets on its dport if it is (or was) LISTENING.
static void note_slot(rxg_ctx *c, int32_t idx)
{
    if (idx >= c->mir.ntcb() || !c->mir.live[idx]) return;
    const rxg_tcb_tuple &t = c->mir.tcb[idx];
    TupleKey k;
    if (tcb_key(t, k)) c->touched_keys.push_back(k);
    if (t.state == RXG_LISTENING && port_in_range(t.dport)) c->touched_listen.push_back(t.dport);
}

extern "C" int rxg_tcb_upsert(rxg_ctx *c, int32_t idx, const rxg_tcb_tuple *t)
{
    if (!c || !t) return fail(-EINVAL, "rxg_tcb_upsert: NULL argument");
    if (t->state >= RXG_TCP_STATES) return fail(-EINVAL, "rxg_tcb_upsert: state %u", t->state);
    if (idx < 0 || idx >= kMaxTcbs) return fail(-EINVAL, "tcb index %d outside 0..%d", idx, kMaxTcbs - 1);
    const int32_t min_null = c->mir.min_null;
    note_slot(c, idx);  // the old tuple / listener
    c->mir.upsert(idx, *t);
    note_slot(c, idx);  // the new ones
    // NULL slots appearing (old Ntcb .. idx-1) or disappearing (a removed slot reused) move
    // min_null, the pass-2 NULL-slot flag of later packets
    if (c->mir.need_rebuild || c->mir.min_null != min_null) c->touched_pass2 = true;
    c->dirty = true;
    c->gen++;
    return 0;
}

extern "C" int rxg_tcb_remove(rxg_ctx *c, int32_t idx)
{
    if (!c) return fail(-EINVAL, "rxg_tcb_remove: ctx NULL");
    if (idx < 0 || idx >= c->mir.ntcb())
        return fail(-EINVAL, "rxg_tcb_remove: index %d outside Ntcb %d", idx, c->mir.ntcb());
    const int32_t min_null = c->mir.min_null;
    note_slot(c, idx);
    c->mir.remove(idx);
    if (c->mir.need_rebuild || c->mir.min_null != min_null) c->touched_pass2 = true;
    if ((size_t)idx < c->rcv_state.size()) c->rcv_state[idx] = 0;  // FreeWindow
    c->dirty = true;
    c->gen++;
    return 0;
}

extern "C" int rxg_tcb_set_state(rxg_ctx *c, int32_t idx, uint8_t state)
{
    if (!c) return fail(-EINVAL, "rxg_tcb_set_state: ctx NULL");
    if (state >= RXG_TCP_STATES) return fail(-EINVAL, "rxg_tcb_set_state: state %u", state);
    if (idx < 0 || idx >= c->mir.ntcb() || !c->mir.live[idx])
        return fail(-EINVAL, "rxg_tcb_set_state: index %d is not a live slot", idx);
    note_slot(c, idx);
    c->mir.set_state(idx, state);
    note_slot(c, idx);
    c->dirty = true;
    c->gen++;
    return 0;
}

extern "C" int rxg_tcb_load(rxg_ctx *c, const rxg_tcb_tuple *tcbs, const uint8_t *live, int32_t ntcb)
{
    if (!c || ntcb < 0 || (ntcb > 0 && !tcbs)) return fail(-EINVAL, "rxg_tcb_load: bad arguments");
    if (ntcb > kMaxTcbs) return fail(-EINVAL, "rxg_tcb_load: %d TCBs exceed %d", ntcb, kMaxTcbs);
    for (int32_t i = 0; i < ntcb; ++i)
        if ((!live || live[i]) && tcbs[i].state >= RXG_TCP_STATES)
            return fail(-EINVAL, "rxg_tcb_load: slot %d state %u", i, tcbs[i].state);
    c->mir.load(tcbs, live, ntcb);
    c->dirty = true;
    c->touched_all = true;
    c->gen++;
    c->rcv_cur.clear();
    c->rcv_state.clear();
    return 0;
}

extern "C" int32_t rxg_tcb_count(rxg_ctx *c) { return c ? c->mir.ntcb() : -EINVAL; }

extern "C" int rxg_flow_partition(rxg_ctx *c, uint32_t part, uint32_t nparts)
{
    if (!c) return fail(-EINVAL, "rxg_flow_partition: ctx NULL");
    if (nparts == 0 || nparts > RXG_RSS_RETA_SIZE || part >= nparts)
        return fail(-EINVAL, "rxg_flow_partition: part %u of %u", part, nparts);
    if (c->mir.part == part && c->mir.nparts == nparts) return 0;
    c->mir.part = part;
    c->mir.nparts = nparts;
    c->mir.need_rebuild = true;  // the whole table, as after rxg_tcb_load
    c->dirty = true;
    c->touched_all = true;
    c->gen++;
    return 0;
}

extern "C" int rxg_flow_partition_get(rxg_ctx *c, uint32_t *part, uint32_t *nparts)
{
    if (!c || !part || !nparts) return fail(-EINVAL, "rxg_flow_partition_get: NULL argument");
    *part = c->mir.part;
    *nparts = c->mir.nparts;
    return 0;
}

extern "C" uint32_t rxg_rss_hash(const uint8_t tuple12[12]) { return tuple12 ? rss_toeplitz(tuple12, 12) : 0u; }

extern "C" int rxg_flow_part_of(const uint8_t *f, uint32_t len, uint32_t nparts)
{
    if ((!f && len) || nparts == 0 || nparts > RXG_RSS_RETA_SIZE)
        return fail(-EINVAL, "rxg_flow_part_of: frame NULL or nparts %u outside 1..%u", nparts, RXG_RSS_RETA_SIZE);
    uint8_t b[38] = {0};
    std::memcpy(b, f, std::min<uint32_t>(len, 38u));
    // ether_in's demux and ip_in's protocol test (etherin.c:12-37, ip.c:19-42): only TCP
    // over IPv4 reaches findtcb
    if (b[12] != 0x08 || b[13] != 0x00 || b[23] != RXG_IPPROTO_TCP) return 0;
    return (int)rss_queue(rss_toeplitz12(b + 26), nparts);
}

extern "C" int64_t rxg_tcb_keys(rxg_ctx *c) { return c ? (int64_t)c->mir.nkeys() : -EINVAL; }

extern "C" int rxg_tcb_post(rxg_ctx *c, const rxg_tcb_op *op)
{
    if (!c || !op) return fail(-EINVAL, "rxg_tcb_post: NULL argument");
    if (op->kind < RXG_TCB_OP_UPSERT || op->kind > RXG_TCB_OP_SET_STATE)
        return fail(-EINVAL, "rxg_tcb_post: kind %u", op->kind);
    if (!c->posted.push(*op)) return fail(-EAGAIN, "rxg_tcb_post: queue full (%u ops)", c->posted.capacity());
    return 0;
}

extern "C" int rxg_tcb_drain(rxg_ctx *c)
{
    if (!c) return fail(-EINVAL, "rxg_tcb_drain: ctx NULL");
    int applied = 0, first_err = 0;
    rxg_tcb_op op;
    while (c->posted.pop(op)) {
        int rc = 0;
        if (op.kind == RXG_TCB_OP_UPSERT) rc = rxg_tcb_upsert(c, op.idx, &op.tuple);
        else if (op.kind == RXG_TCB_OP_REMOVE) rc = rxg_tcb_remove(c, op.idx);
        else rc = rxg_tcb_set_state(c, op.idx, op.state);
        if (rc && !first_err) first_err = rc;
        ++applied;
    }
    return first_err ? first_err : applied;
}

static int tcb_push(rxg_ctx *c);

// Burst boundary (rx thread): posted writes first, then the device mirror.
extern "C" int rxg_tcb_sync(rxg_ctx *c)
{
    if (!c) return fail(-EINVAL, "rxg_tcb_sync: ctx NULL");
    const int rc = rxg_tcb_drain(c);
    if (rc < 0) return rc;
    return c->dirty ? tcb_push(c) : 0;
}

// Before a mirror write on c->stream: kernels that read the tables on other streams are
// done.  Lazy mode records the event now, on the reader's stream (it covers every launch the
// stream has taken so far, the table readers among them).
static int wait_table_readers(rxg_ctx *c)
{
    for (auto &r : c->readers)
        if (r.pending) {
            if (!r.recorded) HIP_OK(hipEventRecord(r.e, r.s));
            HIP_OK(hipStreamWaitEvent(c->stream, r.e, 0));
            r.pending = r.recorded = false;
        }
    return 0;
}

// Before device table buffers are freed or reallocated: every reader has finished (host wait).
static int sync_table_readers(rxg_ctx *c)
{
    for (auto &r : c->readers)
        if (r.pending) {
            if (!r.recorded) HIP_OK(hipEventRecord(r.e, r.s));
            HIP_OK(hipEventSynchronize(r.e));
            r.pending = r.recorded = false;
        }
    return 0;
}

// A mirror's patches (at most one per device word), in one launch on c->stream.
template <typename M>
static int apply_patches(rxg_ctx *c, M &mirror)
{
    const std::vector<MirrorPatch> &p = mirror.patches;
    if (p.empty()) return 0;
    rxg_ctx::PatchBuf &pb = c->patch[c->patch_next];
    c->patch_next = (c->patch_next + 1) % rxg_ctx::kPatchBufs;
    if (pb.set) HIP_OK(hipEventSynchronize(pb.ev));  // this buffer's kernel has read it
    pb.set = false;
    if (p.size() > pb.cap) {
        if (pb.h) HIP_OK(hipHostFree(pb.h));
        pb.h = nullptr;
        pb.cap = 0;
        const uint32_t cap = (uint32_t)std::max<size_t>(p.size() * 2, 1024);
        HIP_OK(hipHostMalloc((void **)&pb.h, (size_t)cap * sizeof(MirrorPatch), hipHostMallocDefault));
        pb.cap = cap;
    }
    std::memcpy(pb.h, p.data(), p.size() * sizeof(MirrorPatch));
    int rc = wait_table_readers(c);
    if (rc) return rc;
    HIP_OK(launch_mirror_patch(pb.h, (uint32_t)p.size(), (uint4 *)c->buckets.p, (int32_t *)c->listen.p,
                               (uint32_t *)c->d_arp.p, c->stream));
    HIP_OK(hipEventRecord(pb.ev, c->stream));
    pb.set = true;
    HIP_OK(hipEventRecord(c->mirror_ev, c->stream));
    c->mirror_ev_set = true;
    ++c->table_writes;
    mirror.patches_taken();
    return 0;
}

// Bring the device TCB mirror up to date: the changed words (usual) or, after a load or
// past load 1/2, the whole table.  No host block on the patch path.
static int tcb_push(rxg_ctx *c)
{
    if (!c->dirty) return 0;
    int rc = set_device(c);
    if (rc) return rc;
    TcbMirror &m = c->mir;
    if (c->mirror_rebuild) m.need_rebuild = true;  // experiment build only
    if (m.need_rebuild) {
        m.rebuild();
        const size_t sb = m.slots.size() * sizeof(Slot), lb = m.listen.size() * sizeof(int32_t);
        if (sb > c->buckets.bytes || lb > c->listen.bytes) {
            // the old buffers must be idle before they are freed
            if ((rc = sync_table_readers(c))) return rc;
            HIP_OK(hipStreamSynchronize(c->stream));
            if ((rc = ensure(c->buckets, sb))) return rc;
            if ((rc = ensure(c->listen, lb))) return rc;
        }
        if ((rc = wait_table_readers(c))) return rc;
        HIP_OK(hipMemcpyAsync(c->buckets.p, m.slots.data(), sb, hipMemcpyHostToDevice, c->stream));
        HIP_OK(hipMemcpyAsync(c->listen.p, m.listen.data(), lb, hipMemcpyHostToDevice, c->stream));
        // the next write changes m.slots in place: the copies must have consumed them
        HIP_OK(hipStreamSynchronize(c->stream));
        HIP_OK(hipEventRecord(c->mirror_ev, c->stream));
        c->mirror_ev_set = true;
        ++c->table_writes;
    } else if ((rc = apply_patches(c, m))) {
        return rc;
    }
    c->bucket_mask = m.nb - 1;
    c->dev_ntcb = m.ntcb();
    c->dev_min_null = m.min_null;
    c->dirty = false;
    return 0;
}

// ----------------------------------------------------------------------- ARP mirror ---
extern "C" int rxg_arp_learned(rxg_ctx *c, uint32_t ip)
{
    if (!c) return fail(-EINVAL, "rxg_arp_learned: ctx NULL");
    c->arp_enabled = true;
    if (c->arp.add(ip)) c->arp_dirty = true;
    c->arp_since_burst.emplace(ip, 1);
    return 0;
}

extern "C" int rxg_arp_load(rxg_ctx *c, const uint32_t *ips, uint32_t n)
{
    if (!c || (n && !ips)) return fail(-EINVAL, "rxg_arp_load: bad arguments");
    c->arp_enabled = true;
    c->arp.clear();
    for (uint32_t i = 0; i < n; ++i) c->arp.add(ips[i]);
    c->arp_dirty = true;
    return 0;
}

extern "C" int32_t rxg_arp_count(rxg_ctx *c) { return c ? (int32_t)c->arp.ips.size() : -EINVAL; }

extern "C" int rxg_arp_disable(rxg_ctx *c)
{
    if (!c) return fail(-EINVAL, "rxg_arp_disable: ctx NULL");
    c->arp_enabled = false;
    c->arp.clear();
    c->arp_since_burst.clear();
    c->arp_dirty = true;
    return 0;
}

static int arp_sync(rxg_ctx *c)
{
    if (!c->arp_enabled || !c->arp_dirty) return 0;
    ArpMirror &a = c->arp;
    int rc;
    if (a.need_rebuild) {
        a.rebuild();
        const size_t bytes = a.slots.size() * 4;
        if (bytes > c->d_arp.bytes) {
            if ((rc = sync_table_readers(c))) return rc;
            HIP_OK(hipStreamSynchronize(c->stream));
            if ((rc = ensure(c->d_arp, bytes))) return rc;
        }
        if ((rc = wait_table_readers(c))) return rc;
        HIP_OK(hipMemcpyAsync(c->d_arp.p, a.slots.data(), bytes, hipMemcpyHostToDevice, c->stream));
        HIP_OK(hipStreamSynchronize(c->stream));
        HIP_OK(hipEventRecord(c->mirror_ev, c->stream));
        c->mirror_ev_set = true;
        ++c->table_writes;
    } else if ((rc = apply_patches(c, a))) {
        return rc;
    }
    c->arp_mask = a.nb - 1;
    c->arp_dirty = false;
    return 0;
}

// A launch on `st` that reads the mirror tables: it follows the last mirror write, and
// the next mirror write follows it.
static bool stream_registered(const rxg_ctx *c, hipStream_t st)
{
    return std::find(c->registered.begin(), c->registered.end(), st) != c->registered.end();
}

static int order_table_reader_before(rxg_ctx *c, hipStream_t st)
{
    if (st == c->stream) return 0;
    // RXG_CFG_STREAMS_OUTLIVE_WRITES: the next write records an event on `st`, so `st` must
    // still exist then; only a registered stream is known to (rxg_stream_retire ends that)
    if (c->lazy_readers && !stream_registered(c, st))
        return fail(-EINVAL, "table-reading launch on stream %p, not registered with rxg_stream_register "
                             "(RXG_CFG_STREAMS_OUTLIVE_WRITES)", (void *)st);
    if (!c->mirror_ev_set) return 0;
    // a stream that already waited for the current mirror_ev needs no second wait (each wait
    // is a barrier packet between the caller's launches)
    for (auto &x : c->readers)
        if (x.s == st && x.waited == c->table_writes) return 0;
    HIP_OK(hipStreamWaitEvent(st, c->mirror_ev, 0));
    for (auto &x : c->readers)
        if (x.s == st) x.waited = c->table_writes;
    return 0;
}

static constexpr size_t kMaxReaderStreams = 16;

static int order_table_reader_after(rxg_ctx *c, hipStream_t st)
{
    if (st == c->stream) return 0;
    rxg_ctx::Reader *r = nullptr;
    for (auto &x : c->readers)
        if (x.s == st) r = &x;
    if (!r) {
        for (auto &x : c->readers)
            if (!x.pending) { r = &x; break; }
        if (!r && c->readers.size() >= kMaxReaderStreams) {
            // more reader streams than entries: the next write's stream waits for them now
            int rc = wait_table_readers(c);
            if (rc) return rc;
            r = &c->readers[0];
        }
        if (!r) {
            // device-scope release: these events order streams of this device (and the
            // host's wait before a buffer is freed); no system-scope cache write-back
            hipEvent_t e;
            HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventReleaseToDevice));
            c->readers.push_back({st, e, false, false, ~0ull});
            r = &c->readers.back();
        }
        // order_table_reader_before found no entry for st, so it has just waited for the
        // current mirror_ev
        r->waited = c->mirror_ev_set ? c->table_writes : ~0ull;
        r->s = st;
    }
    r->pending = true;
    if (c->lazy_readers) {
        r->recorded = false;  // recorded by the next write (wait_table_readers)
    } else {
        HIP_OK(hipEventRecord(r->e, st));
        r->recorded = true;
    }
    return 0;
}

extern "C" int rxg_stream_register(rxg_ctx *c, void *stream)
{
    if (!c || !stream) return fail(-EINVAL, "rxg_stream_register: NULL argument");
    hipStream_t st = (hipStream_t)stream;
    if (st != c->stream && !stream_registered(c, st)) c->registered.push_back(st);
    return 0;
}

extern "C" int rxg_stream_retire(rxg_ctx *c, void *stream)
{
    if (!c || !stream) return fail(-EINVAL, "rxg_stream_retire: NULL argument");
    hipStream_t st = (hipStream_t)stream;
    if (st == c->stream) return 0;
    int rc = set_device(c);
    if (rc) return rc;
    // the order the next table write needs against this stream's launches, taken now; the
    // entry then names no stream (a new stream may get the same handle)
    for (auto &r : c->readers)
        if (r.s == st) {
            if (r.pending && !r.recorded) {
                HIP_OK(hipEventRecord(r.e, st));
                r.recorded = true;
            }
            r.s = nullptr;
            r.waited = ~0ull;
        }
    c->registered.erase(std::remove(c->registered.begin(), c->registered.end(), st), c->registered.end());
    return 0;
}

static DevTable table_view(const rxg_ctx *c)
{
    DevTable t;
    t.buckets = (const uint4 *)c->buckets.p;
    t.listen = (const int32_t *)c->listen.p;
    t.bucket_mask = c->bucket_mask;
    t.ntcb = c->dev_ntcb;
    t.min_null = c->dev_min_null;
    t.arp = (const uint4 *)c->d_arp.p;
    t.arp_mask = c->arp_enabled ? c->arp_mask : 0u;
    t.arp_flags = c->arp_enabled ? (kArpOn | (c->arp.has_zero ? kArpZero : 0u)) : 0u;
    return t;
}

// ------------------------------------------------------------------------- bursts ---
static void select_burst(rxg_ctx *c, uint32_t j)
{
    c->replay_cursor = j;
    const rxg_ctx::BurstRef &b = c->last_bursts[j];
    c->last_off = b.off64;
    c->last_slot0 = b.slot0;
    c->last_stride64 = b.stride64;
    c->last_len = b.len;
    c->last_n = b.n;
    c->last_recs = b.recs;
    c->pm_n = 0;  // a gather describes the burst it followed
}

// Classify bursts[0..k) of one frame pool against the mirror as it stands: one launch per
// kMaxBursts bursts.  The bursts are then replayed in order (rxg_rx_replay).
static bool rec_kind_ok(uint32_t k) { return k == RXG_REC8 || k == RXG_REC16 || k == RXG_REC48; }

// Validation, mirror sync and the replay bookkeeping of a burst set (launched or served).
// stride64 != 0: fixed-stride bursts (rxg_rx_bursts_strided_dev): bursts[j].off64 is unused and
// bursts[j].pad holds the burst's first slot.
static int begin_bursts(rxg_ctx *c, const void *frames, const rxg_dev_burst *bursts, uint32_t k, uint32_t rec_kind,
                        const char *who, uint32_t stride64 = 0)
{
    // a rejected launch leaves nothing to replay: rxg_rx_replay refuses until a burst succeeds
    c->burst_ok = false;
    c->last_bursts.clear();
    if (!rec_kind_ok(rec_kind)) return fail(-EINVAL, "%s: rec_kind %u", who, rec_kind);
    if (k && !bursts) return fail(-EINVAL, "%s: NULL burst table", who);
    bool any = false;
    // the kernel reads descriptors as u32 / u16, frames in 16-byte chunks, and writes each
    // slice's records with 8- or 16-byte vector stores
    const uintptr_t rec_align = rec_kind == RXG_REC8 ? 8u : 16u;
    for (uint32_t j = 0; j < k; ++j) {
        if (!bursts[j].n) continue;
        if ((!stride64 && !bursts[j].off64) || !bursts[j].len || !bursts[j].out)
            return fail(-EINVAL, "%s: NULL device pointer in burst %u", who, j);
        if (stride64 && (uint64_t)bursts[j].pad + (uint64_t)(bursts[j].n - 1u) * stride64 > 0xFFFFFFFFull)
            return fail(-EINVAL, "%s: burst %u: slot0 + (n - 1) * stride64 exceeds 2^32 - 1 slots", who, j);
        if (((uintptr_t)bursts[j].off64 & 3u) || ((uintptr_t)bursts[j].len & 1u) ||
            ((uintptr_t)bursts[j].out & (rec_align - 1u)))
            return fail(-EINVAL, "%s: burst %u: off64 needs 4-byte, len 2-byte, out %u-byte alignment", who, j,
                        (unsigned)rec_align);
        any = true;
    }
    if (any && !frames) return fail(-EINVAL, "%s: NULL frame pool", who);
    if (any && ((uintptr_t)frames & 15u)) return fail(-EINVAL, "%s: frame pool not 16-byte aligned", who);
    c->burst_ok = false;
    int rc = set_device(c);
    if (rc) return rc;
    if ((rc = rxg_tcb_sync(c))) return rc;
    if ((rc = arp_sync(c))) return rc;
    c->arp_since_burst.clear();
    c->last_frames = (const uint8_t *)frames;
    c->last_stride = rec_kind;
    c->last_bursts.clear();
    for (uint32_t j = 0; j < k; ++j)
        c->last_bursts.push_back({stride64 ? nullptr : bursts[j].off64, bursts[j].len, bursts[j].n,
                                  (const uint8_t *)bursts[j].out, stride64 ? bursts[j].pad : 0u, stride64});
    if (c->last_bursts.empty()) c->last_bursts.push_back({nullptr, nullptr, 0u, nullptr});
    select_burst(c, 0);
    // the records reflect the mirror as of now: changes are tracked from here (replay)
    c->touched_keys.clear();
    c->touched_listen.clear();
    c->touched_all = c->touched_pass2 = false;
    c->launch_keys.clear();
    c->launch_listen.clear();
    c->launch_all = c->launch_pass2 = false;
    return 0;
}

// A receive launch: the product kernels, or in the experiment library the ablation kernels
// of RXG_VARIANT (rxg_kernels_exp.hip).
static hipError_t rx_launch(const rxg_ctx *c, const LaunchRx &L, hipStream_t st)
{
#ifdef RXG_EXPERIMENTS
    if (c->variant) {
        LaunchRx X = L;
        X.variant = c->variant;
        return launch_rx_exp(X, st);
    }
#else
    (void)c;
#endif
    return launch_rx(L, st);
}

static int launch_bursts(rxg_ctx *c, const void *frames, const rxg_dev_burst *bursts, uint32_t k, uint32_t rec_kind,
                         void *stream, const char *who, uint32_t stride64 = 0,
                         const rxg_payload_slots *pay = nullptr)
{
    hipStream_t st = pick(c, stream);
    // an unregistered stream is refused before anything changes (rxg.h: "-EINVAL, nothing
    // launched"): no mirror sync, and the previous burst stays replayable
    if (c->lazy_readers && st != c->stream && !stream_registered(c, st))
        return fail(-EINVAL, "%s: table-reading launch on stream %p, not registered with rxg_stream_register "
                             "(RXG_CFG_STREAMS_OUTLIVE_WRITES)", who, (void *)st);
    int rc = begin_bursts(c, frames, bursts, k, rec_kind, who, stride64);
    if (rc) return rc;
    if ((rc = order_table_reader_before(c, st))) return rc;
    LaunchBurst lb[kMaxBursts];
    for (uint32_t j0 = 0; j0 < k; j0 += kMaxBursts) {
        const uint32_t m = std::min(kMaxBursts, k - j0);
        for (uint32_t j = 0; j < m; ++j)
            lb[j] = LaunchBurst{stride64 ? nullptr : bursts[j0 + j].off64, bursts[j0 + j].len, bursts[j0 + j].n,
                                (uint8_t *)bursts[j0 + j].out, stride64 ? bursts[j0 + j].pad : 0u};
        LaunchRx L;
        std::memset(&L, 0, sizeof L);
        L.frames = (const uint8_t *)frames;
        L.bursts = lb;
        L.nbursts = m;
        L.mode = (int)rec_kind;
        L.table = table_view(c);
        L.stride64 = stride64;
        if (pay) {
            L.pay_arena = (uint8_t *)pay->arena;
            L.pay_msgs = pay->msgs;
        }
        L.counters = c->nocount ? nullptr : c->counters;
        L.max_blocks = c->max_blocks ? c->max_blocks : pay ? c->grid_pay : (rec_kind == RXG_REC48 ? c->grid_rec48
                                                        : rec_kind == RXG_REC8 ? c->grid_rec8 : c->grid_rec16);
        if (L.max_blocks == 0) L.max_blocks = 1024;
        HIP_OK(rx_launch(c, L, st));
    }
    if ((rc = order_table_reader_after(c, st))) return rc;
    c->burst_ok = true;
    if (pay && k == 1 && bursts[0].n) {
        // rxg_payload_take answers from this burst's messages (fetched at its first call)
        if (!c->pm_ev) HIP_OK(hipEventCreateWithFlags(&c->pm_ev, hipEventDisableTiming));
        HIP_OK(hipEventRecord(c->pm_ev, st));
        c->d_pm = pay->msgs;
        c->pm_used = nullptr;  // no look-back: never poisoned
        c->pm_n = bursts[0].n;
        c->pm_pending = true;
        c->pm_poisoned = false;
    }
    return 0;
}

extern "C" int rxg_rx_burst_dev(rxg_ctx *c, const rxg_dev_batch *b, void *stream)
{
    if (!c || !b) return fail(-EINVAL, "rxg_rx_burst_dev: NULL argument");
    if (b->n && (!b->frames || !b->off64 || !b->len || !b->out))
        return fail(-EINVAL, "rxg_rx_burst_dev: NULL device pointer");
    const rxg_dev_burst one{b->off64, b->len, b->n, 0u, b->out};
    return launch_bursts(c, b->frames, &one, 1, b->rec_kind, stream, "rxg_rx_burst_dev");
}

static int check_slots(const rxg_payload_slots *p, uint32_t n, const char *who)
{
    if (n && !p->msgs) return fail(-EINVAL, "%s: NULL msgs", who);
    if ((uintptr_t)p->arena & 63u) return fail(-EINVAL, "%s: arena not 64-byte aligned", who);
    if ((uintptr_t)p->msgs & 15u) return fail(-EINVAL, "%s: msgs not 16-byte aligned", who);
    return 0;
}

extern "C" int rxg_rx_burst_payload_dev(rxg_ctx *c, const rxg_dev_batch *b, const rxg_payload_slots *p, void *stream)
{
    if (!c || !b || !p) return fail(-EINVAL, "rxg_rx_burst_payload_dev: NULL argument");
    if (b->n && (!b->frames || !b->off64 || !b->len || !b->out))
        return fail(-EINVAL, "rxg_rx_burst_payload_dev: NULL device pointer");
    if (int rc = check_slots(p, b->n, "rxg_rx_burst_payload_dev")) return rc;
    const rxg_dev_burst one{b->off64, b->len, b->n, 0u, b->out};
    return launch_bursts(c, b->frames, &one, 1, b->rec_kind, stream, "rxg_rx_burst_payload_dev", 0u, p);
}

extern "C" int rxg_rx_burst_strided_payload_dev(rxg_ctx *c, const void *frames, uint32_t stride64,
                                                const rxg_dev_strided_burst *b, uint32_t rec_kind,
                                                const rxg_payload_slots *p, void *stream)
{
    if (!c || !b || !p) return fail(-EINVAL, "rxg_rx_burst_strided_payload_dev: NULL argument");
    if (!stride64) return fail(-EINVAL, "rxg_rx_burst_strided_payload_dev: stride64 0");
    if (int rc = check_slots(p, b->n, "rxg_rx_burst_strided_payload_dev")) return rc;
    const rxg_dev_burst one{nullptr, b->len, b->n, b->slot0, b->out};
    return launch_bursts(c, frames, &one, 1, rec_kind, stream, "rxg_rx_burst_strided_payload_dev", stride64, p);
}

extern "C" int rxg_rx_bursts_dev(rxg_ctx *c, const void *frames, const rxg_dev_burst *bursts, uint32_t k,
                                 uint32_t rec_kind, void *stream)
{
    if (!c) return fail(-EINVAL, "rxg_rx_bursts_dev: ctx NULL");
    return launch_bursts(c, frames, bursts, k, rec_kind, stream, "rxg_rx_bursts_dev");
}

extern "C" int rxg_rx_bursts_strided_dev(rxg_ctx *c, const void *frames, uint32_t stride64,
                                         const rxg_dev_strided_burst *bursts, uint32_t k, uint32_t rec_kind,
                                         void *stream)
{
    if (!c) return fail(-EINVAL, "rxg_rx_bursts_strided_dev: ctx NULL");
    if (!stride64) return fail(-EINVAL, "rxg_rx_bursts_strided_dev: stride64 0");
    if (k && !bursts) return fail(-EINVAL, "rxg_rx_bursts_strided_dev: NULL burst table");
    std::vector<rxg_dev_burst> b(k);
    for (uint32_t j = 0; j < k; ++j) b[j] = rxg_dev_burst{nullptr, bursts[j].len, bursts[j].n, bursts[j].slot0, bursts[j].out};
    return launch_bursts(c, frames, b.data(), k, rec_kind, stream, "rxg_rx_bursts_strided_dev", stride64);
}

// The selected burst's offsets as a device array: its own off64, or for a fixed-stride burst
// slot0 + i * stride64 written into d_soff on `st` (the payload gather and the re-classify
// launch read offsets through a list; rare for strided bursts, which exist for the bulk path).
static int burst_offsets(rxg_ctx *c, hipStream_t st, const uint32_t **out)
{
    *out = c->last_off;
    if (c->last_off || !c->last_stride64) return 0;
    // (rewritten for a reader on another stream: the same values, ordered on the reader's stream)
    if (c->soff_n != c->last_n || c->soff_slot0 != c->last_slot0 || c->soff_stride64 != c->last_stride64 ||
        c->soff_stream != st) {
        int rc = ensure(c->d_soff, (size_t)c->last_n * 4u);
        if (rc) return rc;
        HIP_OK(launch_strided_offsets((uint32_t *)c->d_soff.p, c->last_n, c->last_slot0, c->last_stride64, st));
        c->soff_n = c->last_n;
        c->soff_slot0 = c->last_slot0;
        c->soff_stride64 = c->last_stride64;
        c->soff_stream = st;
    }
    *out = (const uint32_t *)c->d_soff.p;
    return 0;
}

// ---------------------------------------------------------------- latency mode ---
// (Re)launch the server kernel.  A previous kernel has left its loop (stop / idle) or none
// ran (the state machine synchronised its stream first); the mailbox's stop, the return
// block's exited and the control words are reset before the launch.
int SrvPort::launch()
{
    rxg_ctx::Server &S = c->srv;
    __atomic_store_n(&S.mbox->stop, 0ull, __ATOMIC_RELEASE);  // plain stores: no locked op over the BAR
    // Load-bearing (rxg_srvfsm.h Port contract): exited reads 0 from here until this launch's
    // kernel leaves its loop, so the state machine's sync-after-exited never waits on a kernel
    // that is still resident.  Reset before the launch below, never after it.
    __atomic_store_n(&S.ret->exited, 0ull, __ATOMIC_SEQ_CST);
    _mm_sfence();  // device memory is write-combined on the host
    SrvCtl init;
    std::memset(&init, 0, sizeof init);
    init.go = __atomic_load_n(&S.ret->done, __ATOMIC_ACQUIRE) << 16;  // the workgroups wait past it
    HIP_OK(hipMemcpyAsync(S.ctl, &init, sizeof init, hipMemcpyHostToDevice, S.st));
    HIP_OK(hipStreamSynchronize(S.st));
    LaunchServer L;
    L.mbox = S.mbox;
    L.ret = S.ret;
    L.ctl = S.ctl;
    L.counters = c->nocount ? nullptr : c->counters;
    L.idle_ticks = S.idle_ticks;
    L.blocks = S.blocks;
    L.mode = (int)S.rec_kind;
    HIP_OK(launch_server(L, S.st));
    return 0;
}

unsigned long long SrvPort::done() const { return __atomic_load_n(&c->srv.ret->done, __ATOMIC_ACQUIRE); }
bool SrvPort::exited() const { return __atomic_load_n(&c->srv.ret->exited, __ATOMIC_ACQUIRE) != 0ull; }
void SrvPort::sync() { (void)hipStreamSynchronize(c->srv.st); }
// No kernel is resident (the state machine saw it exit and synchronised its stream): the
// next kernel starts from `done` (rx_server: last = ret->done, go = done << 16), so setting
// it to q makes request q, still in the mailbox with a valid check word, one it never serves.
void SrvPort::cancel(unsigned long long q)
{
    __atomic_store_n(&c->srv.ret->done, q, __ATOMIC_SEQ_CST);  // host memory (hipHostMalloc)
}

void SrvPort::request_stop()
{
    __atomic_store_n(&c->srv.mbox->stop, 1ull, __ATOMIC_RELEASE);
    _mm_sfence();
}

// Post request q (S.req).  The staging is fenced before the request (device memory is
// write-combined on the host, where stores may pass each other).  The server takes the
// request when seq is new and the check word matches seq and the request words (SrvMbox):
// whatever order or pieces the mailbox's lines reach it in, it never runs a request with
// another's words.
void SrvPort::write(unsigned long long q)
{
    rxg_ctx::Server &S = c->srv;
    _mm_sfence();
    const bool inl = (S.req.flags & kSrvInlineDesc) != 0u;
    const unsigned long long ck = srv_check(q, S.req, inl ? S.idesc : nullptr);
    if (S.mdev) {
        // Device mailbox (write-combined): the bytes the server polls go out as whole 64-byte
        // lines (non-temporal 16-byte stores, one fence): 128, or 320 with inline descriptors.
        alignas(64) unsigned long long head[kSrvPollWords] = {};
        static_assert(sizeof(SrvReq) + 8 <= offsetof(SrvMbox, check), "mailbox head layout");
        head[0] = q;
        std::memcpy(&head[1], &S.req, sizeof(SrvReq));
        head[offsetof(SrvMbox, check) / 8] = ck;
        head[offsetof(SrvMbox, stop) / 8] = 0ull;
        if (inl) std::memcpy(&head[16], S.idesc, sizeof S.idesc);
        const __m128i *src = reinterpret_cast<const __m128i *>(head);
        __m128i *dst = reinterpret_cast<__m128i *>(S.mbox);
        const int n16 = inl ? kSrvPollWords / 2 : 8;
        for (int i = 0; i < n16; ++i) _mm_stream_si128(dst + i, _mm_load_si128(src + i));
        _mm_sfence();
    } else {
        if (inl) std::memcpy(S.mbox->ioff, S.idesc, sizeof S.idesc);
        S.mbox->req = S.req;
        __atomic_store_n(&S.mbox->check, ck, __ATOMIC_RELEASE);
        __atomic_store_n(&S.mbox->seq, q, __ATOMIC_RELEASE);
        _mm_sfence();
    }
}

// Post one request and wait for its `done` (rxg_srvfsm.h: relaunch after an idle exit, 10 s
// limit, -EIO while a kernel that missed its limit is still resident).
static int srv_post(rxg_ctx *c, const SrvReq &r)
{
    rxg_ctx::Server &S = c->srv;
    S.req = r;
    SrvPort port{c};
    const unsigned long long q = S.fsm.seq + 1u;
    const int rc = S.fsm.post(port);
    if (rc == -ETIMEDOUT)
        return fail(rc, "rxg_server: request %llu not served in 10 s (the server is stopping; until its kernel "
                        "exits, requests fail with -EIO)", q);
    if (rc == -EIO) return fail(rc, "rxg_server: a kernel that missed its time limit has not exited");
    if (rc) return fail(rc, "rxg_server: launch failed");
    return 0;
}

static void srv_free(rxg_ctx *c)
{
    rxg_ctx::Server &S = c->srv;
    if (S.mbox) (void)(S.mdev ? hipFree(S.mbox) : hipHostFree(S.mbox));
    for (void *h : {(void *)S.arena, (void *)S.off, (void *)S.len})
        if (h) (void)(S.dev ? hipFree(h) : hipHostFree(h));
    if (S.ret && S.ret != S.mbox) (void)hipHostFree(S.ret);
    if (S.out) (void)hipHostFree(S.out);
    if (S.ctl) (void)hipFree(S.ctl);
    if (S.st) (void)hipStreamDestroy(S.st);
    S = rxg_ctx::Server{};
}

extern "C" int rxg_server_stop(rxg_ctx *c)
{
    if (!c) return fail(-EINVAL, "rxg_server_stop: ctx NULL");
    if (!c->srv.on) return 0;
    int rc = set_device(c);
    if (rc) return rc;
    SrvPort port{c};
    if (c->srv.fsm.stop(port)) {
        // the kernel is still resident and may still write the staging: nothing is freed
        // (a later stop tries again; rxg_fini retries a bounded number of times, then leaks
        // the context and every buffer the kernel can reach)
        return fail(-EIO, "rxg_server_stop: the server kernel has not exited");
    }
    srv_free(c);
    return 0;
}

extern "C" int rxg_server_start(rxg_ctx *c, const rxg_server_config *cfg)
{
    if (!c || !cfg) return fail(-EINVAL, "rxg_server_start: NULL argument");
    if (!rec_kind_ok(cfg->rec_kind)) return fail(-EINVAL, "rxg_server_start: rec_kind %u", cfg->rec_kind);
    const uint32_t blocks = cfg->blocks ? cfg->blocks : 1u;
    const uint32_t maxf = cfg->max_frames ? cfg->max_frames : 4096u;
    if (blocks > 256u) return fail(-EINVAL, "rxg_server_start: %u workgroups (at most 256)", blocks);
    if (maxf > (1u << 20)) return fail(-EINVAL, "rxg_server_start: max_frames %u (at most 2^20)", maxf);
    int rc = rxg_server_stop(c);
    if (rc) return rc;
    if ((rc = set_device(c))) return rc;
    rxg_ctx::Server &S = c->srv;
    S.rec_kind = cfg->rec_kind;
    S.blocks = blocks;
    S.max_frames = maxf;
    S.max_bytes = cfg->max_bytes ? cfg->max_bytes : (uint64_t)maxf * 2048u;
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device) != hipSuccess || khz <= 0)
        khz = 100000;  // 100 MHz, the MI300-series constant clock
    S.idle_ticks = (uint64_t)(cfg->idle_ms ? cfg->idle_ms : 1000u) * (uint64_t)khz;
    // Placement: with a large BAR the host writes the staged frames and
    // descriptors into fine-grained device memory (posted PCIe writes) and the server reads
    // them from HBM; otherwise they are coherent host memory the server reads over PCIe.  The
    // mailbox follows unless RXG_SRV_HOST_MAILBOX (written as two whole lines, srv_post).
    int large_bar = 0;
    if (!(cfg->flags & RXG_SRV_HOST_STAGING) &&
        hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, c->device) != hipSuccess)
        large_bar = 0;
    S.dev = large_bar != 0;
    S.mdev = S.dev && !(cfg->flags & RXG_SRV_HOST_MAILBOX);
    const unsigned flags = hipHostMallocCoherent | hipHostMallocMapped;
    auto place = [&](bool dev, void **p, size_t bytes) {
        return dev ? hipExtMallocWithFlags(p, bytes, hipDeviceMallocFinegrained) == hipSuccess
                   : hipHostMalloc(p, bytes, flags) == hipSuccess;
    };
    bool ok = hipStreamCreateWithFlags(&S.st, hipStreamNonBlocking) == hipSuccess &&
              place(S.mdev, (void **)&S.mbox, sizeof(SrvMbox)) && place(S.dev, (void **)&S.arena, S.max_bytes) &&
              place(S.dev, (void **)&S.off, (size_t)maxf * 4u) && place(S.dev, (void **)&S.len, (size_t)maxf * 2u) &&
              hipHostMalloc((void **)&S.out, (size_t)maxf * cfg->rec_kind, flags) == hipSuccess &&
              hipMalloc((void **)&S.ctl, sizeof(SrvCtl)) == hipSuccess;
    if (ok && S.mdev) ok = hipHostMalloc((void **)&S.ret, sizeof(SrvMbox), flags) == hipSuccess;
    if (!ok) {
        srv_free(c);
        return fail(-ENOMEM, "rxg_server_start: mailbox / staging for %u frames", maxf);
    }
    if (!S.mdev) S.ret = S.mbox;
    S.h_off.assign(maxf, 0u);
    S.h_len.assign(maxf, 0u);
    if (S.mdev) {
        HIP_OK(hipMemset(S.mbox, 0, sizeof(SrvMbox)));
        std::memset(S.ret, 0, sizeof(SrvMbox));
    } else {
        std::memset(S.mbox, 0, sizeof(SrvMbox));
    }
    S.on = true;
    SrvPort port{c};
    if ((rc = S.fsm.relaunch(port))) {
        srv_free(c);
        return fail(rc, "rxg_server_start: launch failed");
    }
    return 0;
}

extern "C" int rxg_server_active(rxg_ctx *c) { return c && c->srv.on ? 1 : 0; }

extern "C" int rxg_server_placement(rxg_ctx *c)
{
    if (!c || !c->srv.on) return RXG_SRV_NONE;
    return c->srv.dev ? RXG_SRV_DEVICE : RXG_SRV_HOST;
}

// One frame into the server's device staging (write-combined, through the BAR): 32-byte
// non-temporal stores, the tail from a zero-padded copy (no read past the frame; the slot is
// 64-byte aligned and as long as the frame rounded up to 64).  Measured against memcpy
// (scripts/barcopy.cpp, profiles/r04/barcopy/): 32 x 64 B 0.45 -> 0.24 us, 32 x 1 500 B
// 1.80 -> 1.37, 256 x 1 500 B 12.6 -> 10.1.
__attribute__((target("avx2"))) static void stage_frame_avx2(uint8_t *d, const uint8_t *s, uint32_t len)
{
    uint32_t k = 0;
    for (; k + 32u <= len; k += 32u)
        _mm256_stream_si256(reinterpret_cast<__m256i *>(d + k), _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + k)));
    if (k < len) {
        alignas(32) uint8_t t[32] = {};
        std::memcpy(t, s + k, len - k);
        _mm256_stream_si256(reinterpret_cast<__m256i *>(d + k), _mm256_load_si256(reinterpret_cast<const __m256i *>(t)));
    }
}

static bool host_avx2()
{
    static const bool v = __builtin_cpu_supports("avx2");
    return v;
}

// A served burst.  inl: a host burst of at most kSrvInline frames whose descriptors the
// request carries in the mailbox (S.idesc, filled by the caller) as well as in the staging.
// large: a host burst holding a frame over 64 bytes (kSrvLarge).
static int server_burst(rxg_ctx *c, const rxg_dev_batch *b, bool inl, bool large);

extern "C" int rxg_server_burst_dev(rxg_ctx *c, const rxg_dev_batch *b) { return server_burst(c, b, false, false); }

static int server_burst(rxg_ctx *c, const rxg_dev_batch *b, bool inl, bool large)
{
    if (!c || !b) return fail(-EINVAL, "rxg_server_burst_dev: NULL argument");
    if (!c->srv.on) return fail(-ENODEV, "rxg_server_burst_dev: no server (rxg_server_start)");
    if (b->rec_kind != c->srv.rec_kind)
        return fail(-EINVAL, "rxg_server_burst_dev: rec_kind %u, the server's is %u", b->rec_kind, c->srv.rec_kind);
    if (b->n > c->srv.max_frames)
        return fail(-EINVAL, "rxg_server_burst_dev: n=%u exceeds max_frames=%u", b->n, c->srv.max_frames);
    if (b->n && (!b->frames || !b->off64 || !b->len || !b->out))
        return fail(-EINVAL, "rxg_server_burst_dev: NULL device pointer");
    const rxg_dev_burst one{b->off64, b->len, b->n, 0u, b->out};
    int rc = begin_bursts(c, b->frames, &one, 1, b->rec_kind, "rxg_server_burst_dev");
    if (rc) return rc;
    // mirror writes queued on the context's stream land before the server reads the tables
    if (c->table_writes != c->srv.synced_writes) {
        HIP_OK(hipEventSynchronize(c->mirror_ev));
        c->srv.synced_writes = c->table_writes;
    }
    if (b->n) {
        SrvReq r;
        std::memset(&r, 0, sizeof r);
        r.frames = (const uint8_t *)b->frames;
        r.off64 = b->off64;
        r.len = b->len;
        r.out = (uint8_t *)b->out;
        r.n = b->n;
        r.flags = (inl && b->n <= kSrvInline ? kSrvInlineDesc : 0u) | (large ? kSrvLarge : 0u);
        r.table = table_view(c);
        if ((rc = srv_post(c, r))) return rc;
    }
    c->burst_ok = true;
    return 0;
}

extern "C" int rxg_tx_cksum_dev(rxg_ctx *c, const rxg_dev_tx_batch *b, void *stream)
{
    if (!c || !b) return fail(-EINVAL, "rxg_tx_cksum_dev: NULL argument");
    if (b->n && (!b->frames || !b->off64 || !b->len))
        return fail(-EINVAL, "rxg_tx_cksum_dev: NULL device pointer");
    if (b->n && (((uintptr_t)b->frames & 15u) || ((uintptr_t)b->off64 & 3u) || ((uintptr_t)b->len & 1u)))
        return fail(-EINVAL, "rxg_tx_cksum_dev: frames need 16-byte, off64 4-byte, len 2-byte alignment");
    int rc = set_device(c);
    if (rc) return rc;
    LaunchBurst one{b->off64, b->len, b->n, nullptr, 0u};
    LaunchRx L;
    std::memset(&L, 0, sizeof L);
    L.frames = (const uint8_t *)b->frames;
    L.bursts = &one;
    L.nbursts = 1;
    L.mode = 0;
    L.counters = nullptr;
    L.max_blocks = c->max_blocks ? c->max_blocks : c->grid_tx;
    if (L.max_blocks == 0) L.max_blocks = 1024;
    HIP_OK(launch_rx(L, pick(c, stream)));
    return 0;
}

extern "C" int rxg_rx_burst(rxg_ctx *c, const rxg_pkt_view *pkts, uint32_t n, uint32_t rec_kind,
                            void *out_host)
{
    if (!c || (n && (!pkts || !out_host))) return fail(-EINVAL, "rxg_rx_burst: NULL argument");
    if (!rec_kind_ok(rec_kind)) return fail(-EINVAL, "rxg_rx_burst: rec_kind %u", rec_kind);
    if (c->srv.on && rec_kind == c->srv.rec_kind && n && n <= c->srv.max_frames) {
        // latency mode: packed into the server's coherent staging, served without a launch
        rxg_ctx::Server &S = c->srv;
        uint64_t slot = 0;
        bool fits = true, large = false;
        for (uint32_t i = 0; i < n && fits; ++i) {
            const uint64_t need = (pkts[i].data_len + 63u) / 64u;
            large |= pkts[i].data_len > 64u;
            fits = (slot + need) * 64u <= S.max_bytes;
            S.h_off[i] = (uint32_t)slot;
            S.h_len[i] = pkts[i].data_len;
            slot += need;
        }
        if (fits) {
            // write-only streams into the staging (device memory: write-combined, never read
            // back by the host); srv_post fences them before the request
            const bool stream = S.dev && host_avx2();
            for (uint32_t i = 0; i < n; ++i) {
                if (!pkts[i].data_len) continue;
                uint8_t *d = S.arena + (uint64_t)S.h_off[i] * 64u;
                const uint8_t *src = (const uint8_t *)pkts[i].buf_addr + pkts[i].data_off;
                if (stream)
                    stage_frame_avx2(d, src, pkts[i].data_len);
                else
                    std::memcpy(d, src, pkts[i].data_len);
            }
            // (the staged descriptors are also what a re-classification or a payload gather
            // of this burst reads)
            std::memcpy(S.off, S.h_off.data(), (size_t)n * 4u);
            std::memcpy(S.len, S.h_len.data(), (size_t)n * 2u);
            const bool inl = n <= kSrvInline;
            if (inl) {
                uint8_t *d = reinterpret_cast<uint8_t *>(S.idesc);
                std::memset(d, 0, sizeof S.idesc);
                std::memcpy(d, S.h_off.data(), (size_t)n * 4u);
                std::memcpy(d + kSrvInline * 4u, S.h_len.data(), (size_t)n * 2u);
            }
            rxg_dev_batch b;
            b.frames = S.arena;
            b.off64 = S.off;
            b.len = S.len;
            b.n = n;
            b.rec_kind = rec_kind;
            b.out = S.out;
            int rc = server_burst(c, &b, inl, large);
            if (rc) return rc;
            std::memcpy(out_host, S.out, (size_t)n * rec_kind);
            return 0;
        }
    }
    if (n > c->max_batch)
        return fail(-EINVAL, "rxg_rx_burst: n=%u exceeds max_batch=%u", n, c->max_batch);
    c->burst_ok = false;
    int rc = set_device(c);
    if (rc) return rc;
    uint64_t slot = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t l = pkts[i].data_len;
        const uint64_t need = (uint64_t)((l + 63u) / 64u);
        if ((slot + need) * 64u > c->max_bytes)
            return fail(-ENOMEM, "rxg_rx_burst: staging arena of %llu bytes is full at frame %u",
                        (unsigned long long)c->max_bytes, i);
        if (slot > UINT32_MAX) return fail(-ENOMEM, "rxg_rx_burst: arena offset overflow");
        c->h_off[i] = (uint32_t)slot;
        c->h_len[i] = (uint16_t)l;
        slot += need;
    }
    // pack the frames into the pinned staging: one memcpy thread per 4 MiB, at most 8 (a
    // single core copies ≈10-15 GB/s, short of PCIe)
    auto pack = [&](uint32_t i0, uint32_t i1) {
        for (uint32_t i = i0; i < i1; ++i)
            if (pkts[i].data_len)
                std::memcpy(c->h_arena + (uint64_t)c->h_off[i] * 64u,
                            (const uint8_t *)pkts[i].buf_addr + pkts[i].data_off, pkts[i].data_len);
    };
    const uint32_t nthr = (uint32_t)std::min<uint64_t>(8u, std::max<uint64_t>(1u, (slot * 64u) >> 22));
    c->pack_pool.run(nthr, [&](uint32_t t) {
        pack((uint32_t)((uint64_t)n * t / nthr), (uint32_t)((uint64_t)n * (t + 1) / nthr));
    });
    if (n == 0) {  // still a burst: posted writes drained, replay state reset
        rxg_dev_batch e{};
        e.rec_kind = rec_kind;
        return rxg_rx_burst_dev(c, &e, nullptr);
    }
    rxg_dev_batch b;
    if (slot * 64u <= c->zc_bytes) {
        // small burst: the kernel reads the pinned staging and writes pinned records over
        // PCIe; no copy calls on the critical path (latency)
        b.frames = c->h_arena;
        b.off64 = c->h_off;
        b.len = c->h_len;
        b.n = n;
        b.rec_kind = rec_kind;
        b.out = c->h_out;
        if ((rc = rxg_rx_burst_dev(c, &b, c->stream))) return rc;
        c->burst_ok = false;  // until the records are back
        HIP_OK(hipStreamSynchronize(c->stream));
        std::memcpy(out_host, c->h_out, (size_t)n * rec_kind);
        c->burst_ok = true;
        return 0;
    }
    HIP_OK(hipMemcpyAsync(c->d_arena, c->h_arena, slot * 64u, hipMemcpyHostToDevice, c->stream));
    HIP_OK(hipMemcpyAsync(c->d_off, c->h_off, n * 4u, hipMemcpyHostToDevice, c->stream));
    HIP_OK(hipMemcpyAsync(c->d_len, c->h_len, n * 2u, hipMemcpyHostToDevice, c->stream));
    b.frames = c->d_arena;
    b.off64 = c->d_off;
    b.len = c->d_len;
    b.n = n;
    b.rec_kind = rec_kind;
    b.out = c->d_out;
    if ((rc = rxg_rx_burst_dev(c, &b, c->stream))) return rc;
    c->burst_ok = false;  // until the records are back
    HIP_OK(hipMemcpyAsync(out_host, c->d_out, (size_t)n * rec_kind, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    c->burst_ok = true;
    return 0;
}

extern "C" int rxg_ether_in(rxg_ctx *c, const rxg_handoff_ops *ops, void *mbuf, void *frame, uint16_t data_len)
{
    if (!c || !ops || !frame) return fail(-EINVAL, "rxg_ether_in: NULL argument");
    rxg_pkt_view v;
    v.buf_addr = frame;
    v.data_off = 0;
    v.data_len = data_len;
    v.pad = 0;
    rxg_rec16 rec;
    int rc = rxg_rx_burst(c, &v, 1, RXG_REC16, &rec);
    if (rc) return rc;
    void *m = mbuf, *f = frame;
    rc = rxg_rx_replay(c, ops, &m, &f, &rec, 1, RXG_REC16);
    return rc ? rc : 0;  // ether_in always returns 0 (etherin.c:36)
}

// ----------------------------------------------------------------- payload hand-off ---
extern "C" int rxg_payload_gather_dev(rxg_ctx *c, const rxg_payload_out *o, void *stream)
{
    if (!c || !o) return fail(-EINVAL, "rxg_payload_gather_dev: NULL argument");
    if (!c->last_frames || !c->last_recs)
        return fail(-EINVAL, "rxg_payload_gather_dev: no burst to gather from");
    const uint32_t n = c->last_n;
    if (n && (!o->msgs || !o->arena_used || (o->arena_cap && !o->arena)))
        return fail(-EINVAL, "rxg_payload_gather_dev: NULL output buffer");
    int rc = set_device(c);
    if (rc) return rc;
    hipStream_t st = pick(c, stream);
    const uint32_t nb = payload_blocks(n);
    const void *old_status = c->d_pg_status.p;
    if ((rc = ensure(c->d_pg_status, (size_t)nb * sizeof(unsigned long long)))) return rc;
    if (c->d_pg_status.p != old_status)  // fresh memory: no word may look published
        HIP_OK(hipMemsetAsync(c->d_pg_status.p, 0, c->d_pg_status.bytes, st));
    if (!c->d_pg_ticket.p) {
        if ((rc = ensure(c->d_pg_ticket, sizeof(unsigned long long)))) return rc;
        HIP_OK(hipMemsetAsync(c->d_pg_ticket.p, 0, sizeof(unsigned long long), st));
        c->pg_tickets = 0;
    }
    // one gather in flight per context: the ticket counter and the status words are shared,
    // so a gather on another stream waits for the previous one
    if (c->pm_ev) HIP_OK(hipStreamWaitEvent(st, c->pm_ev, 0));
    c->pg_epoch = (c->pg_epoch % ((1u << 30) - 1u)) + 1u;
    LaunchPayload P;
    P.frames = c->last_frames;
    if ((rc = burst_offsets(c, st, &P.off64))) return rc;
    P.len = c->last_len;
    P.recs = c->last_recs;
    P.stride = c->last_stride;
    P.n = n;
    P.msgs = o->msgs;
    P.arena = (uint8_t *)o->arena;
    P.arena_cap = o->arena ? o->arena_cap : 0;
    P.status = (unsigned long long *)c->d_pg_status.p;
    P.ticket = (unsigned long long *)c->d_pg_ticket.p;
    P.ticket_base = c->pg_tickets;
    P.used = (unsigned long long *)o->arena_used;
    P.epoch = c->pg_epoch;
    P.variant = c->pg_variant;
    uint32_t tickets = 0;
    HIP_OK(launch_payload(P, st, &tickets));
    c->pg_tickets += tickets;
    // rxg_payload_take fetches the descriptors on its first call after this gather
    if (!c->pm_ev) HIP_OK(hipEventCreateWithFlags(&c->pm_ev, hipEventDisableTiming));
    HIP_OK(hipEventRecord(c->pm_ev, st));
    c->d_pm = o->msgs;
    c->pm_used = o->arena_used;
    c->pm_n = n;
    c->pm_pending = true;
    c->pm_poisoned = false;
    return 0;
}

extern "C" int rxg_rcv_set(rxg_ctx *c, int32_t idx, uint32_t cur_seq, uint32_t pairs_pending)
{
    if (!c) return fail(-EINVAL, "rxg_rcv_set: ctx NULL");
    if (idx < 0 || idx >= kMaxTcbs) return fail(-EINVAL, "rxg_rcv_set: index %d", idx);
    if ((size_t)idx >= c->rcv_state.size()) {
        c->rcv_state.resize((size_t)idx + 1, 0);
        c->rcv_cur.resize((size_t)idx + 1, 0);
    }
    c->rcv_cur[idx] = cur_seq;
    c->rcv_state[idx] = pairs_pending ? 2 : 1;
    return 0;
}

// PushData (tcp_windows.c:341-358) with an empty SeqPairs list and
// CurrentSequenceNumber == seq: the out-of-window test needs SeqPairs (:345) and is
// skipped; the duplicate test (:349) drops iff cur > seq + Length (u32); AdjustPair puts
// the one pair at the head (:42-110, returns seq + Length + FIN); GetData pops it with
// offset 0 and copies Length bytes (:158-180) -> one message of exactly this payload.
extern "C" int rxg_payload_take(rxg_ctx *c, int32_t idx, uint32_t seq, uint32_t length, rxg_payload_msg *msg)
{
    if (!c) return fail(-EINVAL, "rxg_payload_take: ctx NULL");
    const int64_t pos = c->replay_pos;
    if (pos < 0 || (uint64_t)pos >= c->pm_n || length == 0 || length > 0xFFFFu) return 0;
    if (c->pm_pending) {  // first take after the gather: fetch the burst's descriptors
        if (int rc = set_device(c)) return rc;
        HIP_OK(hipEventSynchronize(c->pm_ev));
        if (c->pm_n > c->h_pm_cap) {
            if (c->h_pm) HIP_OK(hipHostFree(c->h_pm));
            c->h_pm = nullptr;
            c->h_pm_cap = 0;
            HIP_OK(hipHostMalloc((void **)&c->h_pm, (size_t)c->pm_n * sizeof(rxg_payload_msg), hipHostMallocDefault));
            c->h_pm_cap = c->pm_n;
        }
        uint64_t used = 0;
        HIP_OK(hipMemcpyAsync(c->h_pm, c->d_pm, (size_t)c->pm_n * sizeof(rxg_payload_msg), hipMemcpyDeviceToHost,
                              c->stream));
        if (c->pm_used)  // (a fused burst, rxg_rx_burst_payload_dev, has no look-back to time out)
            HIP_OK(hipMemcpyAsync(&used, c->pm_used, sizeof used, hipMemcpyDeviceToHost, c->stream));
        HIP_OK(hipStreamSynchronize(c->stream));
        c->pm_pending = false;
        // a gather whose look-back timed out (arena_used = ~0) placed payloads at unknown
        // offsets: nothing of that burst is handed out (the stack's own PushData runs)
        c->pm_poisoned = used == ~0ull;
    }
    if (c->pm_poisoned) return 0;
    const rxg_payload_msg &m = c->h_pm[pos];
    if (!(m.flags & RXG_PM_GATHERED) || m.len != length) return 0;
    if (idx < 0 || (size_t)idx >= c->rcv_state.size() || c->rcv_state[idx] != 1 || c->rcv_cur[idx] != seq)
        return 0;
    if (seq > (uint32_t)(seq + length)) return 0;  // the duplicate test drops it
    if (seq == 0) return 0;  // GetData asserts CurrentSequenceNumber != 0 (:151): the stack's own code
    c->rcv_cur[idx] = seq + length;
    if (msg) *msg = m;
    return 1;
}

// ----------------------------------------------------------------------- counters ---
extern "C" int rxg_counters_reset(rxg_ctx *c, void *stream)
{
    if (!c) return fail(-EINVAL, "rxg_counters_reset: ctx NULL");
    if (int rc = set_device(c)) return rc;
    HIP_OK(hipMemsetAsync(c->counters, 0, kCounterBytes, pick(c, stream)));
    return 0;
}

extern "C" int rxg_counters_read(rxg_ctx *c, uint64_t *out)
{
    if (!c || !out) return fail(-EINVAL, "rxg_counters_read: NULL argument");
    if (int rc = set_device(c)) return rc;
    HIP_OK(hipStreamSynchronize(c->stream));
    std::vector<uint64_t> rows((size_t)RXG_COUNTER_ROWS * RXG_NCOUNTERS);
    HIP_OK(hipMemcpyAsync(rows.data(), c->counters, kCounterBytes, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    for (int k = 0; k < RXG_NCOUNTERS; ++k) {
        uint64_t v = 0;
        for (int r = 0; r < RXG_COUNTER_ROWS; ++r) v += rows[(size_t)r * RXG_NCOUNTERS + k];
        out[k] = v;
    }
    return 0;
}

extern "C" void *rxg_counters_dev(rxg_ctx *c) { return c ? (void *)c->counters : nullptr; }

// ------------------------------------------------------------------------- replay ---
static inline bool rec_is_tcp(const rxg_rec16 &r)
{
    return r.verdict == RXG_V_DISPATCH || r.verdict == RXG_V_RST_NOPCB || r.verdict == RXG_V_RST_LISTEN_NONSYN;
}

// A TCP record that findtcb pass 1 did not answer (listener or no TCB): pass 2 decides it.
static inline bool rec_pass2(const rxg_rec16 &r) { return r.tcb_idx < 0 || (r.flags & RXG_F_LISTEN); }

// Counter contributions of one TCP record (the kernel's definition; only the fields a
// re-classification can change).
static void tcp_record_counters(const rxg_rec16 &r, int64_t sign, int64_t *d)
{
    if (r.flags & RXG_F_REF_NULLSLOT) d[RXG_C_REF_NULLSLOT] += sign;
    if (r.tcb_idx >= 0) d[(r.flags & RXG_F_LISTEN) ? RXG_C_TCB_HIT_LISTEN : RXG_C_TCB_HIT_EXACT] += sign;
    if (r.verdict == RXG_V_RST_NOPCB) d[RXG_C_NOPCB] += sign;
    if (r.verdict == RXG_V_RST_LISTEN_NONSYN) d[RXG_C_LISTEN_NONSYN] += sign;
    if (r.verdict == RXG_V_DISPATCH) d[RXG_C_DISPATCH] += sign;
}

// The pass-1 key of a frame of >= 54 bytes, as the kernel forms it: ports = dport << 16 |
// sport (host order), ipv4_dst as loaded, ipv4_src host order (tcp_tcb.c:134-135,152-155).
static inline TupleKey frame_key(const uint8_t *f)
{
    const uint32_t sport = ((uint32_t)f[34] << 8) | f[35], dport = ((uint32_t)f[36] << 8) | f[37];
    const uint32_t dst = (uint32_t)f[30] | ((uint32_t)f[31] << 8) | ((uint32_t)f[32] << 16) | ((uint32_t)f[33] << 24);
    const uint32_t src = ((uint32_t)f[26] << 24) | ((uint32_t)f[27] << 16) | ((uint32_t)f[28] << 8) | f[29];
    return TupleKey{(dport << 16) | sport, dst, src};
}

// Re-classify one TCP packet of >= 54 bytes against the table as it stands now, exactly as
// rx_kernel's classify does (findtcb tcp_tcb.c:127-173, tcp_in.c:47-59), answered from the
// host index the device mirror is patched from (rxg_mirror.h): the replay's fix-up of a
// packet whose TCB a handler changed inside the burst.  The fields a
// table change cannot move (checksums, datalen, flags of the frame) stay as the burst
// computed them.
static void host_classify(const rxg_ctx *c, const uint8_t *f, rxg_rec16 &r)
{
    const TupleKey k = frame_key(f);
    uint8_t st = RXG_STATE_NONE;
    bool lhit = false;
    const int32_t idx = c->mir.find(k.ports, k.dst, k.src, k.ports >> 16, &st, &lhit);
    const bool missed = idx < 0 || lhit;  // pass 1 found nothing
    const bool nslot = missed && c->mir.min_null < (lhit ? idx : c->mir.ntcb());
    const uint8_t tflags = f[47];
    r.tcb_idx = idx;
    r.state = idx >= 0 ? st : (uint8_t)RXG_STATE_NONE;
    r.verdict = idx < 0 ? RXG_V_RST_NOPCB
              : (st == RXG_LISTENING && !(tflags & RXG_TCP_FLAG_SYN)) ? RXG_V_RST_LISTEN_NONSYN
              : RXG_V_DISPATCH;
    r.flags = (uint8_t)((r.flags & ~(RXG_F_LISTEN | RXG_F_REF_NULLSLOT)) | (lhit ? RXG_F_LISTEN : 0) |
                        (nslot ? RXG_F_REF_NULLSLOT : 0));
}

// Re-classify frames sel[0..k) of the last burst against the current mirror (GPU).
static int reclassify(rxg_ctx *c, const std::vector<uint32_t> &sel, std::vector<rxg_rec16> &out)
{
    int rc;
    const uint32_t *off64 = nullptr;
    if ((rc = burst_offsets(c, c->stream, &off64))) return rc;
    if (!c->last_frames || !off64 || !c->last_len)
        return fail(-EINVAL, "rxg_rx_replay: no burst on this context to re-classify against");
    if ((rc = ensure(c->d_sel, sel.size() * 4))) return rc;
    if ((rc = ensure(c->d_fix, sel.size() * sizeof(rxg_rec16)))) return rc;
    if (c->dirty && (rc = tcb_push(c))) return rc;
    HIP_OK(hipMemcpyAsync(c->d_sel.p, sel.data(), sel.size() * 4, hipMemcpyHostToDevice, c->stream));
    const LaunchBurst one{off64, c->last_len, (uint32_t)sel.size(), (uint8_t *)c->d_fix.p, 0u};
    LaunchRx L;
    std::memset(&L, 0, sizeof L);
    L.frames = c->last_frames;
    L.bursts = &one;
    L.nbursts = 1;
    L.sel = (const uint32_t *)c->d_sel.p;
    L.mode = RXG_REC16;
    L.table = table_view(c);
    L.counters = nullptr;  // corrections go to the host row instead
    L.max_blocks = c->max_blocks ? c->max_blocks : (c->grid_rec16 ? c->grid_rec16 : 1024);
    HIP_OK(launch_rx(L, c->stream));
    out.resize(sel.size());
    HIP_OK(hipMemcpyAsync(out.data(), c->d_fix.p, sel.size() * sizeof(rxg_rec16), hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    return 0;
}

// A bulk change (a reload, a listener change, min_null moving) that leaves more than this
// many packets of the burst stale re-classifies them in one GPU launch; fewer (and every
// change to single tuples) are answered from the host index as each packet is reached.
static constexpr uint32_t kHostReclassifyMax = 256;

// The side effects of etherin.c:21-35, ip.c:26-39 and tcp_in.c:47-72, in packet order.
extern "C" int rxg_rx_replay(rxg_ctx *c, const rxg_handoff_ops *ops, void *const *mbufs,
                             void *const *frames, const void *recs, uint32_t n, uint32_t stride)
{
    if (!c || !ops || (n && (!mbufs || !frames || !recs)))
        return fail(-EINVAL, "rxg_rx_replay: NULL argument");
    if (!rec_kind_ok(stride)) return fail(-EINVAL, "rxg_rx_replay: stride %u", stride);
    if (n && c->last_n != n)
        return fail(-EINVAL, "rxg_rx_replay: n=%u but the burst to replay (%u of the last launch) had %u frames", n,
                    c->replay_cursor, c->last_n);
    if (n && !c->burst_ok) return fail(-EINVAL, "rxg_rx_replay: the last burst on this context failed");
    // the re-classify launches and the counter correction run on this context's device
    // (a group replays several contexts from one thread, rxg_group.cpp)
    if (int rc = set_device(c)) return rc;
    struct PosGuard {
        rxg_ctx *c;
        ~PosGuard() { c->replay_pos = -1; }
    } pos_guard{c};
    std::vector<rxg_rec16> &cur = c->rp_cur;
    cur.resize(n);
    if (stride == RXG_REC8)
        for (uint32_t i = 0; i < n; ++i) rxg_rec8_expand((const rxg_rec8 *)recs + i, &cur[i]);
    else
        for (uint32_t i = 0; i < n; ++i) cur[i] = *(const rxg_rec16 *)((const uint8_t *)recs + (size_t)i * stride);
    int64_t delta[RXG_NCOUNTERS] = {0};

    // Staleness by write sequence numbers, checked when a packet is reached (its header is
    // read there anyway; no per-burst index).  Each batch of tracked writes (those of one
    // handler call, or those made between the burst and the replay) gets a number; a record
    // computed at number s is stale when a later write touched what it depends on: its tuple
    // (pass 1, old or new tuple of a written slot), or -- for a packet pass 1 did not answer
    // -- a LISTENING slot on its dport or the lowest NULL slot (pass 2); any write for a
    // frame under 54 bytes; everything after a reload.
    std::vector<uint32_t> &pkt_seq = c->rp_seq;
    pkt_seq.assign(n, 0u);  // 0 = as the burst classified it
    uint32_t wseq = 0, any_seq = 0, all_seq = 0, minnull_seq = 0, bulk_seq = 0, scanned_seq = 0;
    std::unordered_map<TupleKey, uint32_t, TupleKeyHash> key_seq;
    std::vector<std::pair<int32_t, uint32_t>> listen_seq;  // (dport, seq): rare
    std::vector<uint64_t> &filt = c->rp_filter;            // 65 536-bit filter of written tuples
    bool filt_used = false;
    auto absorb_lists = [&](const std::vector<TupleKey> &keys, const std::vector<int32_t> &listen, bool all,
                            bool pass2) {
        ++wseq;
        any_seq = wseq;
        if (all) all_seq = bulk_seq = wseq;
        if (pass2) minnull_seq = bulk_seq = wseq;
        for (const TupleKey &k : keys) {
            key_seq[k] = wseq;
            const uint32_t h = tuple_hash(k.ports, k.dst, k.src);
            if (!filt_used) {
                filt.assign(1024, 0ull);
                filt_used = true;
            }
            filt[(h >> 6) & 1023u] |= 1ull << (h & 63u);
        }
        if (c->replay_coarse)  // experiment build only: the round-1 rule, any packet on the dport
            for (const TupleKey &k : keys) listen_seq.emplace_back(-1 - (int32_t)(k.ports >> 16), wseq);
        for (int32_t d : listen) {
            bool found = false;
            for (auto &e : listen_seq)
                if (e.first == d) {
                    e.second = wseq;
                    found = true;
                }
            if (!found) listen_seq.emplace_back(d, wseq);
            bulk_seq = wseq;
        }
    };
    // the tracked writes since the last absorb; logged for the launch's later bursts, whose
    // records were computed before them too
    auto absorb = [&]() {
        c->launch_keys.insert(c->launch_keys.end(), c->touched_keys.begin(), c->touched_keys.end());
        c->launch_listen.insert(c->launch_listen.end(), c->touched_listen.begin(), c->touched_listen.end());
        c->launch_all |= c->touched_all;
        c->launch_pass2 |= c->touched_pass2;
        absorb_lists(c->touched_keys, c->touched_listen, c->touched_all, c->touched_pass2);
        c->touched_keys.clear();
        c->touched_listen.clear();
        c->touched_all = c->touched_pass2 = false;
    };
    auto stale = [&](uint32_t j) -> bool {
        const rxg_rec16 &q = cur[j];
        const uint32_t s = pkt_seq[j];
        if (any_seq <= s || !rec_is_tcp(q)) return false;
        if (all_seq > s || (q.flags & RXG_F_TRUNC)) return true;
        const TupleKey k = frame_key((const uint8_t *)frames[j]);
        if (filt_used) {
            const uint32_t h = tuple_hash(k.ports, k.dst, k.src);
            if ((filt[(h >> 6) & 1023u] >> (h & 63u)) & 1ull) {
                auto it = key_seq.find(k);
                if (it != key_seq.end() && it->second > s) return true;
            }
        }
        const int32_t d = (int32_t)(k.ports >> 16);
        if (rec_pass2(q)) {
            if (minnull_seq > s) return true;
            for (const auto &e : listen_seq)
                if (e.first == d && e.second > s) return true;
        }
        if (c->replay_coarse)
            for (const auto &e : listen_seq)
                if (e.first == -1 - d && e.second > s) return true;
        return false;
    };
    // writes the replays of this launch's earlier bursts made, then those since
    if (c->replay_cursor > 0 &&
        (!c->launch_keys.empty() || !c->launch_listen.empty() || c->launch_all || c->launch_pass2))
        absorb_lists(c->launch_keys, c->launch_listen, c->launch_all, c->launch_pass2);
    if (!c->touched_keys.empty() || !c->touched_listen.empty() || c->touched_all || c->touched_pass2) absorb();

    std::vector<uint32_t> sel;
    std::vector<rxg_rec16> fix;
    for (uint32_t i = 0; i < n; ++i) {
        if (any_seq > pkt_seq[i] && stale(i)) {
            ++c->rp_stats[0];
            const bool trunc = (cur[i].flags & RXG_F_TRUNC) != 0;
            bool batched = false;
            if (c->replay_on_device || trunc || bulk_seq > scanned_seq) {
                // what is stale from here on: one GPU launch if the set is large (a bulk
                // change), or always on the device path / for a short frame
                sel.clear();
                for (uint32_t j = i; j < n; ++j)
                    if (stale(j)) sel.push_back(j);
                scanned_seq = wseq;
                if (c->replay_on_device || trunc || sel.size() > kHostReclassifyMax) {
                    int rc = reclassify(c, sel, fix);
                    if (rc) return rc;
                    for (size_t k = 0; k < sel.size(); ++k) {
                        tcp_record_counters(cur[sel[k]], -1, delta);
                        tcp_record_counters(fix[k], +1, delta);
                        cur[sel[k]] = fix[k];
                        pkt_seq[sel[k]] = wseq;
                    }
                    c->rp_stats[2] += sel.size();
                    ++c->rp_stats[3];
                    batched = true;
                }
            }
            if (!batched) {
                if (c->mir.need_rebuild) {  // a reload / growth inside the replay: index first
                    int rc = tcb_push(c);
                    if (rc) return rc;
                }
                rxg_rec16 r = cur[i];
                host_classify(c, (const uint8_t *)frames[i], r);
                tcp_record_counters(cur[i], -1, delta);
                tcp_record_counters(r, +1, delta);
                cur[i] = r;
                pkt_seq[i] = wseq;
                ++c->rp_stats[1];
            }
        }
        const rxg_rec16 &r = cur[i];
        c->replay_pos = i;  // rxg_payload_take answers for this packet
        void *m = mbufs[i];
        uint8_t *f = (uint8_t *)frames[i];
        void *ip = f + RXG_OFF_IP, *tcp = f + RXG_OFF_TCP;
        const uint64_t gen_before = c->gen;
        switch (r.verdict) {
        case RXG_V_ARP:
            if (ops->arp_in) ops->arp_in(ops->user, m);
            if (ops->free_mbuf) ops->free_mbuf(ops->user, m);
            break;
        case RXG_V_DROP_L2:
        case RXG_V_DROP_NONTCP:
            if (ops->free_mbuf) ops->free_mbuf(ops->user, m);
            break;
        default: {
            // ip.c:30-32 ARP learn on the host-order source address
            const uint32_t src = ((uint32_t)f[26] << 24) | ((uint32_t)f[27] << 16) | ((uint32_t)f[28] << 8) | f[29];
            if (c->arp_enabled) {
                // the mirror answers get_mac: unknown at the burst and not added since
                if ((r.flags & RXG_F_ARP_LEARN) && ops->add_mac && !c->arp_since_burst.count(src)) {
                    ops->add_mac(ops->user, src, f + 6);
                    rxg_arp_learned(c, src);  // idempotent if the caller's add_mac mirrors too
                }
            } else {
                unsigned char mac[6];
                if (ops->get_mac && ops->add_mac && ops->get_mac(ops->user, src, mac) == 0)
                    ops->add_mac(ops->user, src, f + 6);
            }
            if ((ops->flags & RXG_OPS_VERIFY_TCP_CKSUM) && !(r.flags & RXG_F_TCP_OK)) {
                // tcp_in.c:37-40 with the check compiled in: free, ++tcpchecksumerror
                if (ops->free_mbuf) ops->free_mbuf(ops->user, m);
                if (ops->tcpchecksumerror) ++*ops->tcpchecksumerror;
            } else if (r.verdict == RXG_V_RST_NOPCB || r.verdict == RXG_V_RST_LISTEN_NONSYN) {
                if (r.verdict == RXG_V_RST_NOPCB && ops->tcpnopcb) ++*ops->tcpnopcb;  // tcp_in.c:48
                if (ops->free_mbuf) ops->free_mbuf(ops->user, m);
                if (ops->send_reset) ops->send_reset(ops->user, ip, tcp);
            } else {  // RXG_V_DISPATCH
                const uint32_t seq = ((uint32_t)f[38] << 24) | ((uint32_t)f[39] << 16) | ((uint32_t)f[40] << 8) | f[41];
                const uint32_t ack = ((uint32_t)f[42] << 24) | ((uint32_t)f[43] << 16) | ((uint32_t)f[44] << 8) | f[45];
                if (ops->on_segment) ops->on_segment(ops->user, r.tcb_idx, seq, ack);
                if (ops->tcpswitch) ops->tcpswitch(ops->user, r.tcb_idx, r.state, tcp, ip, m);
            }
        }
        }
        if (c->gen != gen_before) absorb();  // the handlers changed the table
    }
    // the launch's next burst is replayed next (a single burst can be replayed again)
    if (c->replay_cursor + 1 < c->last_bursts.size()) select_burst(c, c->replay_cursor + 1);
    bool nz = false;
    for (int k = 0; k < RXG_NCOUNTERS; ++k) nz |= delta[k] != 0;
    if (nz) {  // add the corrections to the host row of the counter block, in stream order
        CounterDelta d;
        for (int k = 0; k < RXG_NCOUNTERS; ++k) d.v[k] = delta[k];
        HIP_OK(launch_counters_add(c->counters + (size_t)(RXG_COUNTER_ROWS - 1) * RXG_NCOUNTERS, d, c->stream));
    }
    return 0;
}

extern "C" int rxg_replay_stats(rxg_ctx *c, uint64_t out[4])
{
    if (!c || !out) return fail(-EINVAL, "rxg_replay_stats: NULL argument");
    for (int k = 0; k < 4; ++k) out[k] = c->rp_stats[k];
    return 0;
}

// ---------------------------------------------------------------------- synthetic ---
extern "C" uint64_t rxg_synth_arena_bytes(const rxg_synth_params *p)
{
    if (!p) return 0;
    if (p->mix == 0) return (uint64_t)p->n * (uint64_t)((p->len_a + 63u) / 64u) * 64u;
    return (uint64_t)((p->n + kImixBlock - 1) / kImixBlock) * kImixSlotsPerBlock * 64u;
}

extern "C" int rxg_synth_dev(rxg_ctx *c, const rxg_synth_params *p, void *frames, uint64_t cap,
                             uint32_t *off64, uint16_t *len, uint32_t *flow_out, uint64_t *arena_bytes,
                             void *stream)
{
    if (!c || !p || !frames || !off64 || !len) return fail(-EINVAL, "rxg_synth_dev: NULL argument");
    if (p->mix > 1) return fail(-EINVAL, "rxg_synth_dev: mix %u", p->mix);
    if (p->mix == 0 && (p->len_a < 54 || p->len_a > 9014))
        return fail(-EINVAL, "rxg_synth_dev: len_a %u outside 54..9014", p->len_a);
    const uint64_t need = rxg_synth_arena_bytes(p);
    if (need > cap) return fail(-ENOMEM, "rxg_synth_dev: needs %llu arena bytes, have %llu",
                                (unsigned long long)need, (unsigned long long)cap);
    if (need / 64u > UINT32_MAX) return fail(-EINVAL, "rxg_synth_dev: arena beyond 256 GiB");
    int rc = set_device(c);
    if (rc) return rc;
    hipStream_t st = pick(c, stream);
    LaunchSynth L;
    L.frames = (uint8_t *)frames;
    L.off64 = off64;
    L.len = len;
    L.flow = flow_out;
    L.seed = p->seed;
    L.arena_bytes = need;
    L.n = p->n;
    L.nflows = p->nflows;
    L.dst_ip = p->dst_ip_host;
    L.dport = p->dport;
    L.mix = p->mix;
    L.len_a = p->len_a;
    HIP_OK(launch_synth(L, st));
    // checksums: the transmit generate kernel (ip_out's two checksums)
    rxg_dev_tx_batch tb;
    tb.frames = frames;
    tb.off64 = off64;
    tb.len = len;
    tb.n = p->n;
    tb.pad = 0;
    if ((rc = rxg_tx_cksum_dev(c, &tb, st))) return rc;
    if (arena_bytes) *arena_bytes = need;
    return 0;
}

// ------------------------------------------------------------------ memory helpers ---
extern "C" int rxg_dev_alloc(rxg_ctx *c, uint64_t bytes, void **out)
{
    if (!c || !out) return fail(-EINVAL, "rxg_dev_alloc: NULL argument");
    int rc = set_device(c);
    if (rc) return rc;
    HIP_OK(hipMalloc(out, bytes ? bytes : 1));
    return 0;
}

extern "C" int rxg_dev_free(rxg_ctx *c, void *p)
{
    if (!c) return fail(-EINVAL, "rxg_dev_free: ctx NULL");
    if (p) HIP_OK(hipFree(p));
    return 0;
}

extern "C" int rxg_host_alloc_pinned(rxg_ctx *c, uint64_t bytes, void **out)
{
    if (!c || !out) return fail(-EINVAL, "rxg_host_alloc_pinned: NULL argument");
    HIP_OK(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
    return 0;
}

extern "C" int rxg_host_free_pinned(rxg_ctx *c, void *p)
{
    if (!c) return fail(-EINVAL, "rxg_host_free_pinned: ctx NULL");
    if (p) HIP_OK(hipHostFree(p));
    return 0;
}

// Zero-copy: page-lock caller memory (e.g. the mbuf pool's hugepages) and map it for the
// device, so batches in it go to rxg_rx_burst_dev / rxg_tx_cksum_dev without a copy.
extern "C" int rxg_host_register(rxg_ctx *c, void *p, uint64_t bytes, void **dev_alias)
{
    if (!c || !p || !bytes || !dev_alias) return fail(-EINVAL, "rxg_host_register: bad argument");
    int rc = set_device(c);
    if (rc) return rc;
    HIP_OK(hipHostRegister(p, bytes, hipHostRegisterMapped));
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess || !d) {
        (void)hipHostUnregister(p);
        return fail(-EIO, "rxg_host_register: no device mapping for %p", p);
    }
    *dev_alias = d;
    return 0;
}

extern "C" int rxg_host_unregister(rxg_ctx *c, void *p)
{
    if (!c || !p) return fail(-EINVAL, "rxg_host_unregister: bad argument");
    int rc = set_device(c);
    if (rc) return rc;
    HIP_OK(hipHostUnregister(p));
    return 0;
}

extern "C" int rxg_memcpy_h2d(rxg_ctx *c, void *dst, const void *src, uint64_t bytes, void *stream)
{
    if (!c) return fail(-EINVAL, "rxg_memcpy_h2d: ctx NULL");
    HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, pick(c, stream)));
    return 0;
}

extern "C" int rxg_memcpy_d2h(rxg_ctx *c, void *dst, const void *src, uint64_t bytes, void *stream)
{
    if (!c) return fail(-EINVAL, "rxg_memcpy_d2h: ctx NULL");
    HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, pick(c, stream)));
    return 0;
}

extern "C" int rxg_memset_dev(rxg_ctx *c, void *dst, int value, uint64_t bytes, void *stream)
{
    if (!c) return fail(-EINVAL, "rxg_memset_dev: ctx NULL");
    HIP_OK(hipMemsetAsync(dst, value, bytes, pick(c, stream)));
    return 0;
}

extern "C" int rxg_stream_sync(rxg_ctx *c, void *stream)
{
    if (!c) return fail(-EINVAL, "rxg_stream_sync: ctx NULL");
    HIP_OK(hipStreamSynchronize(pick(c, stream)));
    return 0;
}

extern "C" int rxg_event_create(rxg_ctx *c, rxg_event **out)
{
    if (!c || !out) return fail(-EINVAL, "rxg_event_create: NULL argument");
    rxg_event *e = new rxg_event();
    if (hipEventCreate(&e->e) != hipSuccess) {
        delete e;
        return fail(-EIO, "rxg_event_create: hipEventCreate failed");
    }
    *out = e;
    return 0;
}

extern "C" int rxg_event_record(rxg_ctx *c, rxg_event *e, void *stream)
{
    if (!c || !e) return fail(-EINVAL, "rxg_event_record: NULL argument");
    HIP_OK(hipEventRecord(e->e, pick(c, stream)));
    return 0;
}

extern "C" int rxg_event_elapsed_ms(rxg_ctx *c, rxg_event *a, rxg_event *b, float *ms)
{
    if (!c || !a || !b || !ms) return fail(-EINVAL, "rxg_event_elapsed_ms: NULL argument");
    HIP_OK(hipEventSynchronize(b->e));
    HIP_OK(hipEventElapsedTime(ms, a->e, b->e));
    return 0;
}

extern "C" int rxg_event_destroy(rxg_ctx *c, rxg_event *e)
{
    (void)c;
    if (e) {
        (void)hipEventDestroy(e->e);
        delete e;
    }
    return 0;
}
