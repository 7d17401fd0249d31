// rxg_server.cpp — latency mode (rxg_server_*, DESIGN.md §2.5: the persistent server kernel,
// its mailbox and the host state machine's port, rxg_srvfsm.h) and the host-buffer burst
// (rxg_rx_burst), served when the server is up and launched otherwise.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <immintrin.h>
#include <thread>

#include "rxg_ctx.h"

using namespace rxg;

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
    L.counters = c->counters;
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
    // the staging (device memory: through the BAR and the HDP) flushed before the request
    if (S.dev) bar_publish(c, nullptr);
    else _mm_sfence();
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
        if ((rc = mirror_event(c))) return rc;  // (a write a burst carried: recorded now)
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
