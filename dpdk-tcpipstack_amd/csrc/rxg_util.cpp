// rxg_util.cpp — synthetic frame pools (rxg_synth_*), device / pinned memory, copies and
// events for callers without a runtime of their own (bench.py, the C examples, the tests).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <immintrin.h>
#include <thread>

#include "rxg_ctx.h"

using namespace rxg;

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
