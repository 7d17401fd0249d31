// rxg_host.cpp — host side of the rxg C ABI (include/rxg.h): the context, mirrors, launched
// bursts, tx and counters (the other entry points: rxg_server.cpp, rxg_replay.cpp,
// rxg_util.cpp; the context itself: rxg_ctx.h).
//
// Owns one GPU context: its stream, the device TCB mirror (rebuilt from the host mirror
// whenever a rxg_tcb_* call made it dirty), the counter block, and the pinned staging used
// by the host-buffer entry points.  There is no CPU compute path: without a usable HIP
// device every compute entry point returns -ENODEV / -EIO.
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


#include "rxg_ctx.h"

using namespace rxg;

static_assert(sizeof(rxg_rec16) == 16, "rxg_rec16 layout");
static_assert(sizeof(rxg_rec48) == 48, "rxg_rec48 layout");
static_assert(sizeof(rxg_tcb_tuple) == 20, "rxg_tcb_tuple layout");

// ------------------------------------------------------------------------ errors ---
static thread_local char g_err[512];

int fail(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

extern "C" const char *rxg_last_error(void) { return g_err; }

void bar_publish(const rxg_ctx *c, const volatile uint32_t *last)
{
    _mm_sfence();
    if (c->hdp_flush) {
        *c->hdp_flush = 1u;
        _mm_sfence();
    }
    if (last) (void)*last;
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
        c->grid_ref8 = cus * (uint32_t)rx_blocks_per_cu(8, true);
        c->grid_ref16 = cus * (uint32_t)rx_blocks_per_cu(16, true);
        c->grid_ref48 = cus * (uint32_t)rx_blocks_per_cu(48, true);
        // the fused burst + payload hand-off moves as many bytes out as in: 2 workgroups per CU
        // (8 waves) measured faster than the occupancy grid's 3 (C3 621 against 627 us, C4 174
        // against 177)
        c->grid_pay = cus * 2u;
    }
    // a large BAR: the mirror's patch lists live in device memory the host writes directly,
    // and a burst launch carries its own (launch_bursts)
    int large_bar = 0;
    if (hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, c->device) == hipSuccess && large_bar) {
        void *probe = nullptr;  // and host-writable device memory can be had
        if (hipExtMallocWithFlags(&probe, 4096, hipDeviceMallocFinegrained) == hipSuccess) {
            (void)hipFree(probe);
            c->patch_dev = true;
        }
        hipDeviceProp_t hp;
        if (hipGetDeviceProperties(&hp, c->device) == hipSuccess) c->hdp_flush = hp.hdpMemFlushCntl;
    }
    if (cfg) {
        c->replay_on_device = (cfg->flags & RXG_CFG_REPLAY_ON_DEVICE) != 0;
        c->lazy_readers = (cfg->flags & RXG_CFG_STREAMS_OUTLIVE_WRITES) != 0;
        c->max_blocks = cfg->max_blocks;
        if (cfg->zc_bytes) c->zc_bytes = cfg->zc_bytes;
    }
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
        if (pb.h) (void)(c->patch_dev ? hipFree(pb.h) : hipHostFree(pb.h));
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
    if (int rc = flush_delta(c)) return rc;
    HIP_OK(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" void *rxg_stream(rxg_ctx *c) { return c ? (void *)c->stream : nullptr; }


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

// A patch list in c->patch[bi] (n patches) as its own launch on c->stream.
static int launch_patch_list(rxg_ctx *c, int bi, uint32_t n)
{
    rxg_ctx::PatchBuf &pb = c->patch[bi];
    int rc = wait_table_readers(c);
    if (rc) return rc;
    // the last replay's counter corrections ride along (its table writes are why this runs)
    CounterDelta d;
    if (c->pend) std::memcpy(d.v, c->pend_delta, sizeof d.v);
    HIP_OK(launch_mirror_patch(pb.h, n, (uint4 *)c->buckets.p, (int32_t *)c->listen.p, (uint32_t *)c->d_arp.p,
                               c->stream, c->pend ? correction_row(c) : nullptr, &d));
    if (c->pend) {
        std::memset(c->pend_delta, 0, sizeof c->pend_delta);
        c->pend = false;
    }
    HIP_OK(hipEventRecord(pb.ev, c->stream));
    pb.set = true;
    HIP_OK(hipEventRecord(c->mirror_ev, c->stream));
    c->mirror_ev_set = true;
    // a list a burst is still to carry (this launch was another table's overflow,
    // apply_patches) is written after this recording: the event is re-recorded after that
    // burst (mirror_event), as the rebuild paths do
    c->mirror_ev_stale = c->ip_n != 0;
    return 0;
}

// A mirror's patches (at most one per device word): into the next patch buffer, then in one
// launch on c->stream -- or, when the caller is about to launch a burst on c->stream that
// can carry them (c->defer_patch, launch_bursts), left for that launch (c->ip_*).
template <typename M>
static int apply_patches(rxg_ctx *c, M &mirror)
{
    const std::vector<MirrorPatch> &p = mirror.patches;
    if (p.empty()) return 0;
    const uint32_t n = (uint32_t)p.size();
    uint32_t tables = 0;
    for (const MirrorPatch &q : p) tables |= 1u << q.target;
    if (c->defer_patch && c->ip_n != 0) {
        // a second table's patches (the ARP mirror's after the TCB mirror's) join the list
        // the burst carries, when it has room (the kernel applies each by its target).  Every
        // workgroup of the carrying launch stores the whole list in parallel, so no two of its
        // patches may write one word: a mirror emits at most one patch per word, and only a
        // list for tables the carried one does not touch joins it.
        rxg_ctx::PatchBuf &cb = c->patch[c->ip_buf];
        if ((c->ip_tables & tables) == 0 && c->ip_n + n <= kLaunchPatchMax && c->ip_n + n <= cb.cap) {
            std::memcpy(cb.h + c->ip_n, p.data(), (size_t)n * sizeof(MirrorPatch));
            bar_publish(c, &cb.h[c->ip_n + n - 1].v[3]);
            mirror.patches_taken();
            ++c->table_writes;
            c->ip_n += n;
            c->ip_tables |= tables;
            return 0;
        }
    }
    const int bi = c->patch_next;
    rxg_ctx::PatchBuf &pb = c->patch[bi];
    c->patch_next = (bi + 1) % rxg_ctx::kPatchBufs;
    if (pb.set) HIP_OK(hipEventSynchronize(pb.ev));  // the launch that read this buffer is done
    pb.set = false;
    if (n > pb.cap) {
        if (pb.h) HIP_OK(c->patch_dev ? hipFree(pb.h) : hipHostFree(pb.h));
        pb.h = nullptr;
        pb.cap = 0;
        const uint32_t cap = std::max<uint32_t>(n * 2u, 1024u);
        const size_t bytes = (size_t)cap * sizeof(MirrorPatch);
        if (c->patch_dev)
            HIP_OK(hipExtMallocWithFlags((void **)&pb.h, bytes, hipDeviceMallocFinegrained));
        else
            HIP_OK(hipHostMalloc((void **)&pb.h, bytes, hipHostMallocDefault));
        pb.cap = cap;
    }
    std::memcpy(pb.h, p.data(), (size_t)n * sizeof(MirrorPatch));
    if (c->patch_dev) bar_publish(c, &pb.h[n - 1].v[3]);  // through the BAR: out before the launch
    mirror.patches_taken();
    ++c->table_writes;
    if (c->defer_patch && c->ip_n == 0 && n <= kLaunchPatchMax) {
        c->ip_list = pb.h;
        c->ip_n = n;
        c->ip_buf = bi;
        c->ip_tables = tables;
        c->mirror_ev_set = true;
        c->mirror_ev_stale = true;  // the carrying launch is the write (mirror_event)
        return 0;
    }
    return launch_patch_list(c, bi, n);
}

// A carried list the burst did not take (a failure between the sync and the launch): as its
// own launch, so no write is lost.
static int launch_carried_patches(rxg_ctx *c)
{
    if (c->ip_n == 0) return 0;
    const uint32_t n = c->ip_n;
    c->ip_n = 0;
    return launch_patch_list(c, c->ip_buf, n);
}

int mirror_event(rxg_ctx *c)
{
    if (c->ip_n) return launch_carried_patches(c);  // (not between a sync and its burst)
    if (!c->mirror_ev_stale) return 0;
    HIP_OK(hipEventRecord(c->mirror_ev, c->stream));
    c->mirror_ev_stale = false;
    return 0;
}

// Bring the device TCB mirror up to date: the changed words (usual) or, after a load or
// past load 1/2, the whole table.  No host block on the patch path.
int tcb_push(rxg_ctx *c)
{
    if (!c->dirty) return 0;
    int rc = set_device(c);
    if (rc) return rc;
    TcbMirror &m = c->mir;
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
        c->mirror_ev_stale = c->ip_n != 0;  // (a list a burst is to carry comes after it)
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
        c->mirror_ev_stale = c->ip_n != 0;  // (a list a burst is to carry comes after it)
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
    if (int rc = mirror_event(c)) return rc;  // (a write a burst carried: recorded now)
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

// ------------------------------------------------------------------------- bursts ---
void select_burst(rxg_ctx *c, uint32_t j)
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
// Validation, mirror sync and the replay bookkeeping of a burst set (launched or served).
// stride64 != 0: fixed-stride bursts (rxg_rx_bursts_strided_dev): bursts[j].off64 is unused and
// bursts[j].pad holds the burst's first slot.
int begin_bursts(rxg_ctx *c, const void *frames, const rxg_dev_burst *bursts, uint32_t k, uint32_t rec_kind,
                 const char *who, uint32_t stride64)
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
    // The burst's first launch carries the mirror's patch list when nothing else reads the
    // tables meanwhile: launched on the context's stream (ordered after every earlier reader
    // there), no reader pending on another stream, and frames in that launch (a launch of
    // none is never made).  It then replaces a patch launch: ≈ 10 µs of host launch latency
    // per churning burst.
    bool first_has_frames = false;
    for (uint32_t j = 0; j < std::min(k, kMaxBursts); ++j) first_has_frames |= bursts[j].n != 0;
    bool others_pending = false;
    for (const auto &r : c->readers) others_pending |= r.pending;
    c->defer_patch = c->patch_dev && st == c->stream && first_has_frames && !others_pending;
    int rc = begin_bursts(c, frames, bursts, k, rec_kind, who, stride64);
    c->defer_patch = false;
    if (rc) {
        (void)launch_carried_patches(c);
        return rc;
    }
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
        L.counters = c->counters;
        // (the by-reference hand-off writes no payload: its kernel's occupancy grid)
        L.max_blocks = c->max_blocks ? c->max_blocks : pay && pay->arena ? c->grid_pay
                     : pay ? (rec_kind == RXG_REC48 ? c->grid_ref48 : rec_kind == RXG_REC8 ? c->grid_ref8 : c->grid_ref16)
                     : (rec_kind == RXG_REC48 ? c->grid_rec48 : rec_kind == RXG_REC8 ? c->grid_rec8 : c->grid_rec16);
        if (L.max_blocks == 0) L.max_blocks = 1024;
        const bool carries = j0 == 0 && c->ip_n != 0;
        if (carries) {
            L.ipatch = c->ip_list;
            L.nipatch = c->ip_n;
        }
        const hipError_t e = launch_rx(L, st);
        if (e != hipSuccess) {
            (void)launch_carried_patches(c);
            HIP_OK(e);
        }
        if (carries) {  // the list's buffer is free again once this launch has run
            c->ip_n = 0;
            HIP_OK(hipEventRecord(c->patch[c->ip_buf].ev, st));
            c->patch[c->ip_buf].set = true;
        }
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
int burst_offsets(rxg_ctx *c, hipStream_t st, const uint32_t **out)
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

// ----------------------------------------------------------------------- counters ---
// The replay's counter corrections (rxg_rx_replay) wait on the host for the context's next
// mirror patch launch, which a replay that changed any record always leads to (the change
// came from a table write); a read, a sync or rxg_counters_dev adds them first.
int flush_delta(rxg_ctx *c)
{
    if (!c->pend) return 0;
    if (int rc = set_device(c)) return rc;
    CounterDelta d;
    std::memcpy(d.v, c->pend_delta, sizeof d.v);
    HIP_OK(launch_counters_add(correction_row(c), d, c->stream));
    std::memset(c->pend_delta, 0, sizeof c->pend_delta);
    c->pend = false;
    return 0;
}

extern "C" int rxg_counters_reset(rxg_ctx *c, void *stream)
{
    if (!c) return fail(-EINVAL, "rxg_counters_reset: ctx NULL");
    if (int rc = set_device(c)) return rc;
    // pending corrections belong to the bursts before the reset: zeroed with them
    std::memset(c->pend_delta, 0, sizeof c->pend_delta);
    c->pend = false;
    HIP_OK(hipMemsetAsync(c->counters, 0, kCounterBytes, pick(c, stream)));
    return 0;
}

extern "C" int rxg_counters_read(rxg_ctx *c, uint64_t *out)
{
    if (!c || !out) return fail(-EINVAL, "rxg_counters_read: NULL argument");
    if (int rc = set_device(c)) return rc;
    if (int rc = flush_delta(c)) return rc;
    // bursts on caller streams add to the block too: every one launched so far is waited for
    // (the table readers' events, sync_table_readers), then the context's stream
    if (int rc = sync_table_readers(c)) return rc;
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

extern "C" void *rxg_counters_dev(rxg_ctx *c)
{
    if (!c) return nullptr;
    (void)flush_delta(c);  // (on failure rxg_last_error says so; the block is still there)
    return (void *)c->counters;
}
