// rxg_group.cpp — several GPUs behind one rx loop.
//
// A group is one rxg context per device.  Every context holds a full replica of the TCB
// mirror (tcbs[] writes are applied to all of them), a burst is cut into one contiguous
// shard per member and the shards run concurrently -- a host-buffer burst on the group's
// worker threads (one per member, kept for the group's life), a device-resident burst
// (rxg_group_rx_burst_dev) as one asynchronous launch per member -- each member on its own
// device and stream, and the records come back in packet order.  The
// replay then walks the members' shards in packet order: a handler's tcbs[] write, mirrored
// through the group, reaches every member before that member's shard is replayed, and
// rxg_rx_replay re-classifies the shard's affected packets as it does within one burst, so
// the group is sequentially equivalent to ether_in over the whole burst.
//
// Built on the public C ABI only (include/rxg.h).  RCCL is loaded at the first counter merge
// over distinct GPUs (dlopen), so librxg.so does not need it at load time: single-GPU users
// and the plain-C rx loop never touch it.
#include <dlfcn.h>
#include <rccl/rccl.h>  // types only; the functions come from dlopen("librccl.so")

#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <set>
#include <string>
#include <mutex>
#include <thread>
#include <type_traits>
#include <vector>

#include "rxg.h"
#include "rxg_opqueue.h"
#include "rxg_packpool.h"

struct rxg_group {
    std::vector<rxg_ctx *> m;
    std::vector<uint32_t> shard_off, shard_n;  // the last group burst's shards
    uint32_t last_n = 0;
    bool burst_ok = false;  // the last group burst completed on every member
    bool arp_on = false;   // the ARP mirror is in use (rxg_group_arp_load / _learned)
    int32_t replaying = -1;  // member whose shard rxg_group_rx_replay is in, else -1
    // posts from other threads: one queue for the group, so every member applies them in
    // the same (claim) order and the replicas stay identical
    rxg::MpscRing<rxg_tcb_op> posted{RXG_TCB_QUEUE_CAP};
    // counter merge: one RCCL communicator per member (ncclCommInitAll) when the members are
    // distinct GPUs, set up at the first rxg_group_counters_read; the all-reduce writes into
    // `merged` (one counter block per member), never into the members' own blocks
    std::vector<int32_t> devices;
    int rccl = -1;  // -1 not tried, 0 host sum (members share a GPU, or RCCL unavailable), 1 RCCL
    std::string rccl_why;  // why the merge is on the host
    std::vector<ncclComm_t> comms;
    std::vector<void *> merged;
    // host-buffer bursts: member i > 0 runs its shard on worker thread i, kept for the
    // group's life (no thread is created per burst); member 0 on the caller's thread
    rxg::PackPool workers;
};

namespace {

thread_local char g_err[256];

int gfail(int rc, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return rc;
}

// Apply f to every member; the first error is returned (its text copied to the group's
// error), the others still run.
template <typename F>
int each(rxg_group *g, F f)
{
    int first = 0;
    for (size_t i = 0; i < g->m.size(); ++i) {
        const int rc = f(g->m[i]);
        if (rc < 0 && !first) first = gfail(rc, "member %zu: %s", i, rxg_last_error());
    }
    return first;
}

// The caller's hand-off table, seen through the group during a replay: add_mac also tells
// every member's ARP mirror, so a later member does not learn the same source again.
struct Shim {
    rxg_group *g;
    const rxg_handoff_ops *o;
};
#define SHIM(u) (*(const Shim *)(u))
void sh_free(void *u, void *m) { SHIM(u).o->free_mbuf(SHIM(u).o->user, m); }
int sh_arp_in(void *u, void *m) { return SHIM(u).o->arp_in(SHIM(u).o->user, m); }
int sh_get_mac(void *u, uint32_t ip, unsigned char *mac) { return SHIM(u).o->get_mac(SHIM(u).o->user, ip, mac); }
int sh_add_mac(void *u, uint32_t ip, const unsigned char *mac)
{
    const int r = SHIM(u).o->add_mac(SHIM(u).o->user, ip, mac);
    if (SHIM(u).g->arp_on)
        for (rxg_ctx *c : SHIM(u).g->m) rxg_arp_learned(c, ip);
    return r;
}
void sh_rst(void *u, void *ip, void *tcp) { SHIM(u).o->send_reset(SHIM(u).o->user, ip, tcp); }
void sh_seg(void *u, int32_t idx, uint32_t seq, uint32_t ack) { SHIM(u).o->on_segment(SHIM(u).o->user, idx, seq, ack); }
int sh_switch(void *u, int32_t idx, uint8_t st, void *tcp, void *ip, void *m)
{
    return SHIM(u).o->tcpswitch(SHIM(u).o->user, idx, st, tcp, ip, m);
}
#undef SHIM

}  // namespace

extern "C" int rxg_group_init(const int32_t *devices, uint32_t ndev, const rxg_config *cfg, rxg_group **out)
{
    if (!out || !devices || ndev == 0) return gfail(-EINVAL, "rxg_group_init: bad argument");
    *out = nullptr;
    rxg_group *g = new rxg_group();
    for (uint32_t i = 0; i < ndev; ++i) {
        rxg_config c = cfg ? *cfg : rxg_config{};
        c.device = devices[i];
        rxg_ctx *ctx = nullptr;
        const int rc = rxg_init(&c, &ctx);
        if (rc) {
            for (rxg_ctx *x : g->m) rxg_fini(x);
            delete g;
            return rc;
        }
        g->m.push_back(ctx);
        g->devices.push_back(devices[i]);
    }
    *out = g;
    return 0;
}

// ------------------------------------------------------------------------ RCCL ---
// The few RCCL entry points the merge uses, resolved once from librccl.so.
namespace {
struct Rccl {
    bool tried = false, ok = false;
    std::string why;
    ncclResult_t (*CommInitAll)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
};
std::mutex g_rccl_mu;
Rccl g_rccl;

template <typename F>
bool rccl_sym(void *h, F &fn, const char *name, std::string &why)
{
    fn = reinterpret_cast<F>(dlsym(h, name));
    if (!fn) why = std::string("librccl.so has no ") + name;
    return fn != nullptr;
}

const Rccl &rccl_lib()
{
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    Rccl &r = g_rccl;
    if (r.tried) return r;
    r.tried = true;
    void *h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        const char *e = dlerror();
        r.why = std::string("dlopen librccl.so: ") + (e ? e : "not found");
        return r;
    }
    bool ok = true;
    ok &= rccl_sym(h, r.CommInitAll, "ncclCommInitAll", r.why);
    ok &= rccl_sym(h, r.CommDestroy, "ncclCommDestroy", r.why);
    ok &= rccl_sym(h, r.GroupStart, "ncclGroupStart", r.why);
    ok &= rccl_sym(h, r.GroupEnd, "ncclGroupEnd", r.why);
    ok &= rccl_sym(h, r.AllReduce, "ncclAllReduce", r.why);
    ok &= rccl_sym(h, r.GetErrorString, "ncclGetErrorString", r.why);
    r.ok = ok;
    return r;
}
}  // namespace

extern "C" int rxg_group_fini(rxg_group *g)
{
    if (!g) return 0;
    for (ncclComm_t c : g->comms) (void)rccl_lib().CommDestroy(c);
    for (size_t i = 0; i < g->merged.size(); ++i)
        if (g->merged[i]) (void)rxg_dev_free(g->m[i], g->merged[i]);
    for (rxg_ctx *c : g->m) rxg_fini(c);
    delete g;
    return 0;
}

extern "C" uint32_t rxg_group_size(rxg_group *g) { return g ? (uint32_t)g->m.size() : 0u; }

extern "C" rxg_ctx *rxg_group_member(rxg_group *g, uint32_t i)
{
    return (g && i < g->m.size()) ? g->m[i] : nullptr;
}

// ---------------------------------------------------------------- mirror broadcast ---
extern "C" int rxg_group_tcb_upsert(rxg_group *g, int32_t idx, const rxg_tcb_tuple *t)
{
    if (!g) return gfail(-EINVAL, "rxg_group_tcb_upsert: group NULL");
    return each(g, [&](rxg_ctx *c) { return rxg_tcb_upsert(c, idx, t); });
}

extern "C" int rxg_group_tcb_remove(rxg_group *g, int32_t idx)
{
    if (!g) return gfail(-EINVAL, "rxg_group_tcb_remove: group NULL");
    return each(g, [&](rxg_ctx *c) { return rxg_tcb_remove(c, idx); });
}

extern "C" int rxg_group_tcb_set_state(rxg_group *g, int32_t idx, uint8_t state)
{
    if (!g) return gfail(-EINVAL, "rxg_group_tcb_set_state: group NULL");
    return each(g, [&](rxg_ctx *c) { return rxg_tcb_set_state(c, idx, state); });
}

extern "C" int rxg_group_tcb_load(rxg_group *g, const rxg_tcb_tuple *tcbs, const uint8_t *live, int32_t ntcb)
{
    if (!g) return gfail(-EINVAL, "rxg_group_tcb_load: group NULL");
    return each(g, [&](rxg_ctx *c) { return rxg_tcb_load(c, tcbs, live, ntcb); });
}

extern "C" int rxg_group_tcb_post(rxg_group *g, const rxg_tcb_op *op)
{
    if (!g || !op) return gfail(-EINVAL, "rxg_group_tcb_post: NULL argument");
    if (op->kind < RXG_TCB_OP_UPSERT || op->kind > RXG_TCB_OP_SET_STATE)
        return gfail(-EINVAL, "rxg_group_tcb_post: kind %u", op->kind);
    return g->posted.push(*op) ? 0 : gfail(-EAGAIN, "rxg_group_tcb_post: %u posts waiting", g->posted.capacity());
}

extern "C" int rxg_group_tcb_drain(rxg_group *g)
{
    if (!g) return gfail(-EINVAL, "rxg_group_tcb_drain: group NULL");
    int applied = 0, first = 0;
    rxg_tcb_op op;
    while (g->posted.pop(op)) {
        int rc;
        if (op.kind == RXG_TCB_OP_UPSERT)
            rc = rxg_group_tcb_upsert(g, op.idx, &op.tuple);
        else if (op.kind == RXG_TCB_OP_REMOVE)
            rc = rxg_group_tcb_remove(g, op.idx);
        else
            rc = rxg_group_tcb_set_state(g, op.idx, op.state);
        if (rc < 0 && !first) first = rc;  // the text is already in the group's error
        ++applied;
    }
    return first ? first : applied;
}

extern "C" int rxg_group_arp_load(rxg_group *g, const uint32_t *ipv4_host, uint32_t n)
{
    if (!g) return gfail(-EINVAL, "rxg_group_arp_load: group NULL");
    g->arp_on = true;
    return each(g, [&](rxg_ctx *c) { return rxg_arp_load(c, ipv4_host, n); });
}

extern "C" int rxg_group_arp_learned(rxg_group *g, uint32_t ipv4_host)
{
    if (!g) return gfail(-EINVAL, "rxg_group_arp_learned: group NULL");
    g->arp_on = true;
    return each(g, [&](rxg_ctx *c) { return rxg_arp_learned(c, ipv4_host); });
}

extern "C" int rxg_group_arp_disable(rxg_group *g)
{
    if (!g) return gfail(-EINVAL, "rxg_group_arp_disable: group NULL");
    g->arp_on = false;
    return each(g, [&](rxg_ctx *c) { return rxg_arp_disable(c); });
}

extern "C" int rxg_group_rcv_set(rxg_group *g, int32_t idx, uint32_t cur_seq, uint32_t pairs_pending)
{
    if (!g) return gfail(-EINVAL, "rxg_group_rcv_set: group NULL");
    return each(g, [&](rxg_ctx *c) { return rxg_rcv_set(c, idx, cur_seq, pairs_pending); });
}

// ------------------------------------------------------------------------- bursts ---
extern "C" int rxg_group_rx_burst(rxg_group *g, const rxg_pkt_view *pkts, uint32_t n, uint32_t rec_kind,
                                  void *out_host)
{
    if (!g || (n && (!pkts || !out_host))) return gfail(-EINVAL, "rxg_group_rx_burst: NULL argument");
    if (rec_kind != RXG_REC8 && rec_kind != RXG_REC16 && rec_kind != RXG_REC48)
        return gfail(-EINVAL, "rxg_group_rx_burst: rec_kind %u", rec_kind);
    {  // the posted writes, on every member, before any shard reads its mirror
        const int rc = rxg_group_tcb_drain(g);
        if (rc < 0) return rc;
    }
    const uint32_t k = (uint32_t)g->m.size();
    for (uint32_t i = 0; i < k; ++i) {  // contiguous shards need every member's whole table
        uint32_t part = 0, nparts = 1;
        if (rxg_flow_partition_get(g->m[i], &part, &nparts) == 0 && nparts > 1)
            return gfail(-EINVAL, "rxg_group_rx_burst: member %u is flow-partitioned (%u of %u); a group "
                                  "cuts contiguous shards and needs whole tables", i, part, nparts);
    }
    const uint32_t per = (n + k - 1) / k;
    g->shard_off.assign(k, 0);
    g->shard_n.assign(k, 0);
    for (uint32_t i = 0; i < k; ++i) {
        const uint32_t o = i * per < n ? i * per : n;
        g->shard_off[i] = o;
        g->shard_n[i] = (o + per < n ? o + per : n) - o;
    }
    g->last_n = n;
    g->burst_ok = false;
    std::vector<int> rc(k, 0);
    std::vector<std::string> err(k);
    g->workers.run(k, [&](uint32_t i) {
        rc[i] = rxg_rx_burst(g->m[i], pkts + g->shard_off[i], g->shard_n[i], rec_kind,
                             (uint8_t *)out_host + (size_t)g->shard_off[i] * rec_kind);
        if (rc[i]) err[i] = rxg_last_error();  // thread-local in the member's thread
    });
    for (uint32_t i = 0; i < k; ++i)
        if (rc[i]) return gfail(rc[i], "member %u: %s", i, err[i].c_str());
    g->burst_ok = true;
    return 0;
}

// Device-resident group burst: shards[i] is member i's contiguous share of the burst, in
// packet order, in memory that member's GPU reads.  One asynchronous launch per member (the
// members' kernels run concurrently, each on its context's stream); rxg_group_sync waits.
extern "C" int rxg_group_rx_burst_dev(rxg_group *g, const rxg_dev_batch *shards, uint32_t nshards)
{
    if (!g || (nshards && !shards)) return gfail(-EINVAL, "rxg_group_rx_burst_dev: NULL argument");
    g->burst_ok = false;
    const uint32_t k = (uint32_t)g->m.size();
    if (nshards != k) return gfail(-EINVAL, "rxg_group_rx_burst_dev: %u shards for %u members", nshards, k);
    const uint32_t kind = shards[0].rec_kind;
    for (uint32_t i = 0; i < k; ++i)
        if (shards[i].rec_kind != kind)  // the replay walks one record array of one stride
            return gfail(-EINVAL, "rxg_group_rx_burst_dev: shard %u rec_kind %u, shard 0 %u", i,
                         shards[i].rec_kind, kind);
    {
        const int rc = rxg_group_tcb_drain(g);
        if (rc < 0) return rc;
    }
    uint64_t total = 0;
    for (uint32_t i = 0; i < k; ++i) {
        uint32_t part = 0, nparts = 1;
        if (rxg_flow_partition_get(g->m[i], &part, &nparts) == 0 && nparts > 1)
            return gfail(-EINVAL, "rxg_group_rx_burst_dev: member %u is flow-partitioned (%u of %u); a group "
                                  "cuts contiguous shards and needs whole tables", i, part, nparts);
        total += shards[i].n;
    }
    if (total > UINT32_MAX) return gfail(-EINVAL, "rxg_group_rx_burst_dev: %llu frames", (unsigned long long)total);
    g->shard_off.assign(k, 0);
    g->shard_n.assign(k, 0);
    uint32_t o = 0;
    for (uint32_t i = 0; i < k; ++i) {
        g->shard_off[i] = o;
        g->shard_n[i] = shards[i].n;
        o += shards[i].n;
    }
    g->last_n = o;
    for (uint32_t i = 0; i < k; ++i) {
        const int rc = rxg_rx_burst_dev(g->m[i], &shards[i], nullptr);
        if (rc) return gfail(rc, "member %u: %s", i, rxg_last_error());
    }
    g->burst_ok = true;
    return 0;
}

extern "C" int rxg_group_sync(rxg_group *g)
{
    if (!g) return gfail(-EINVAL, "rxg_group_sync: group NULL");
    return each(g, [&](rxg_ctx *c) { return rxg_sync(c); });
}

extern "C" int rxg_group_rx_replay(rxg_group *g, const rxg_handoff_ops *ops, void *const *mbufs,
                                   void *const *frames, const void *recs, uint32_t n, uint32_t stride)
{
    if (!g || !ops || (n && (!mbufs || !frames || !recs))) return gfail(-EINVAL, "rxg_group_rx_replay: NULL argument");
    if (n != g->last_n) return gfail(-EINVAL, "rxg_group_rx_replay: n=%u but the last group burst had %u", n, g->last_n);
    if (!g->burst_ok) return gfail(-EINVAL, "rxg_group_rx_replay: the last group burst failed");
    Shim sh{g, ops};
    rxg_handoff_ops so{};
    so.user = &sh;
    so.free_mbuf = ops->free_mbuf ? sh_free : nullptr;
    so.arp_in = ops->arp_in ? sh_arp_in : nullptr;
    so.get_mac = ops->get_mac ? sh_get_mac : nullptr;
    so.add_mac = ops->add_mac ? sh_add_mac : nullptr;
    so.send_reset = ops->send_reset ? sh_rst : nullptr;
    so.on_segment = ops->on_segment ? sh_seg : nullptr;
    so.tcpswitch = ops->tcpswitch ? sh_switch : nullptr;
    so.tcpnopcb = ops->tcpnopcb;  // the caller's globals, bumped in packet order across shards
    so.tcpchecksumerror = ops->tcpchecksumerror;
    so.flags = ops->flags;
    struct Guard {
        rxg_group *g;
        ~Guard() { g->replaying = -1; }
    } guard{g};
    for (size_t i = 0; i < g->m.size(); ++i) {
        const uint32_t o = g->shard_off[i];
        g->replaying = (int32_t)i;
        // the member's mirror already holds every write the earlier shards' handlers made
        // (they went through rxg_group_tcb_*); its replay re-classifies what they affect
        const int rc = rxg_rx_replay(g->m[i], &so, mbufs + o, frames + o,
                                     (const uint8_t *)recs + (size_t)o * stride, g->shard_n[i],
                                     stride);
        if (rc) return gfail(rc, "member %zu: %s", i, rxg_last_error());
    }
    return 0;
}

extern "C" int rxg_group_payload_take(rxg_group *g, int32_t idx, uint32_t seq, uint32_t length,
                                      rxg_payload_msg *msg)
{
    if (!g) return gfail(-EINVAL, "rxg_group_payload_take: group NULL");
    if (g->replaying < 0) return 0;
    return rxg_payload_take(g->m[(size_t)g->replaying], idx, seq, length, msg);
}

extern "C" int32_t rxg_group_replaying(rxg_group *g) { return g ? g->replaying : -EINVAL; }

// ----------------------------------------------------------------------- counters ---
extern "C" int rxg_group_counters_reset(rxg_group *g)
{
    if (!g) return gfail(-EINVAL, "rxg_group_counters_reset: group NULL");
    return each(g, [&](rxg_ctx *c) {
        int rc = rxg_counters_reset(c, nullptr);
        return rc ? rc : rxg_sync(c);
    });
}

static constexpr size_t kCounterWords = (size_t)RXG_COUNTER_ROWS * RXG_NCOUNTERS;

// One communicator per member over the members' devices; only for distinct GPUs (RCCL
// takes one rank per device).
static void free_merged(rxg_group *g)
{
    for (size_t i = 0; i < g->merged.size(); ++i)
        if (g->merged[i]) (void)rxg_dev_free(g->m[i], g->merged[i]);
    g->merged.clear();
}

static int rccl_setup(rxg_group *g)
{
    if (g->rccl >= 0) return 0;
    g->rccl = 0;
    const std::set<int32_t> distinct(g->devices.begin(), g->devices.end());
    if (distinct.size() != g->devices.size()) {  // members share a GPU: host sum
        g->rccl_why = "members share a GPU (RCCL takes one rank per device)";
        return 0;
    }
    const Rccl &R = rccl_lib();
    if (!R.ok) {  // no RCCL on this host: the sum is exact on the host too
        g->rccl_why = R.why;
        return 0;
    }
    const int n = (int)g->m.size();
    g->merged.assign((size_t)n, nullptr);
    for (int i = 0; i < n; ++i)
        if (rxg_dev_alloc(g->m[(size_t)i], kCounterWords * sizeof(uint64_t), &g->merged[(size_t)i])) {
            const int rc = gfail(-ENOMEM, "rxg_group_counters_read: member %d: %s", i, rxg_last_error());
            free_merged(g);
            g->rccl = -1;  // retried at the next read
            return rc;
        }
    g->comms.assign((size_t)n, nullptr);
    const ncclResult_t r = R.CommInitAll(g->comms.data(), n, g->devices.data());
    if (r != ncclSuccess) {
        g->comms.clear();
        free_merged(g);
        g->rccl = -1;
        return gfail(-EIO, "rxg_group_counters_read: ncclCommInitAll: %s", R.GetErrorString(r));
    }
    g->rccl = 1;
    g->rccl_why.clear();
    return 0;
}

// The members' counters summed.  Distinct GPUs: an RCCL all-reduce (sum, uint64) of the
// members' counter blocks over xGMI into `merged`, then member 0's merged block is read
// (the one collective of the design).  Members sharing a GPU: summed on
// the host.
extern "C" int rxg_group_counters_read(rxg_group *g, uint64_t *out)
{
    if (!g || !out) return gfail(-EINVAL, "rxg_group_counters_read: NULL argument");
    int rc = rccl_setup(g);
    if (rc) return rc;
    std::memset(out, 0, sizeof(uint64_t) * RXG_NCOUNTERS);
    if (g->rccl == 1) {
        const size_t n = g->m.size();
        for (size_t i = 0; i < n; ++i)  // every burst's counter adds are done (stream order)
            if ((rc = rxg_sync(g->m[i]))) return gfail(rc, "member %zu: %s", i, rxg_last_error());
        const Rccl &R = rccl_lib();
        if (R.GroupStart() != ncclSuccess) return gfail(-EIO, "rxg_group_counters_read: ncclGroupStart");
        for (size_t i = 0; i < n; ++i) {
            const ncclResult_t r = R.AllReduce(rxg_counters_dev(g->m[i]), g->merged[i], kCounterWords, ncclUint64,
                                               ncclSum, g->comms[i], (hipStream_t)rxg_stream(g->m[i]));
            if (r != ncclSuccess) {
                (void)R.GroupEnd();
                return gfail(-EIO, "rxg_group_counters_read: ncclAllReduce: %s", R.GetErrorString(r));
            }
        }
        if (R.GroupEnd() != ncclSuccess) return gfail(-EIO, "rxg_group_counters_read: ncclGroupEnd");
        std::vector<uint64_t> rows(kCounterWords);
        if ((rc = rxg_memcpy_d2h(g->m[0], rows.data(), g->merged[0], kCounterWords * sizeof(uint64_t), nullptr)) ||
            (rc = rxg_sync(g->m[0])))
            return gfail(rc, "member 0: %s", rxg_last_error());
        for (size_t k = 0; k < RXG_NCOUNTERS; ++k)
            for (size_t r = 0; r < RXG_COUNTER_ROWS; ++r) out[k] += rows[r * RXG_NCOUNTERS + k];
        return 0;
    }
    for (rxg_ctx *c : g->m) {
        uint64_t v[RXG_NCOUNTERS];
        rc = rxg_counters_read(c, v);
        if (rc) return rc;
        for (int k = 0; k < RXG_NCOUNTERS; ++k) out[k] += v[k];
    }
    return 0;
}

extern "C" int rxg_group_counters_rccl(rxg_group *g)
{
    if (!g) return gfail(-EINVAL, "rxg_group_counters_rccl: group NULL");
    const int rc = rccl_setup(g);
    return rc ? rc : g->rccl;
}

extern "C" const char *rxg_group_counters_rccl_why(rxg_group *g)
{
    return g ? g->rccl_why.c_str() : "";
}

extern "C" const char *rxg_group_last_error(void) { return g_err; }
