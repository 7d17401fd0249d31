// rxg_rx_server.h — the latency-mode server kernel (rxg_server_*): a persistent
// grid running rx_body once per request posted in a mailbox.
#pragma once
#include <hip/hip_runtime.h>

#include "rxg_rx.h"

namespace rxg {

// ------------------------------------------------------------- latency-mode server ---
// rx_server: the same workgroup body as rx_kernel<MODE> (one burst, the SRV form), run once
// per request by a persistent grid (rxg_server_*).  Wave 0 of workgroup 0
// polls the mailbox's first 128 bytes (system-scope loads, s_sleep between polls) and takes a
// request when its number is new and the check word matches (srv_check).  A request of
// P <= gridDim workgroups' worth of slices (4 slices per workgroup, one per wave, then
// round-robin) runs on workgroups 0 .. P-1.  When P > 1, workgroup 0 copies the request to
// SrvCtl::req and then publishes SrvCtl::go = number << 16 | P (agent-scope release /
// acquire): a workgroup that sees a new go learns P from go itself and reads req only when it
// takes part.  A participant's read cannot race the next request's copy: workgroup 0 copies
// request g+1 only after `done` of g, which needs every participant of g to have finished.
// Every participant classifies its slices, makes its record stores visible, and the last to
// finish (SrvCtl::fin reset for the next request) publishes `done`.  Exit: `stop`, or no
// request for idle_ticks of the constant-rate wall clock (the host relaunches on its next
// burst), so a server whose process is gone ends by itself.
struct SrvArgs {
    SrvMbox *mbox;  // the host-written words (seq, request, stop): host memory or device memory
    SrvMbox *ret;   // the server's words (done, exited): host memory (= mbox when it is there)
    SrvCtl *ctl;
    unsigned long long *counters;
    unsigned long long idle_ticks;
};

__device__ __forceinline__ uint64_t uniform64(uint64_t v)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// workgroups a request of n frames runs on
__device__ __forceinline__ uint32_t srv_participants(uint32_t n, uint32_t flags)
{
    const uint32_t nsl = (n + 63u) / 64u;
    // large frames, 3..gridDim slices: one slice per workgroup (rx_body's shared slices)
    if ((flags & kSrvLarge) && nsl >= 3u && nsl <= gridDim.x) return nsl;
    return max(1u, min(gridDim.x, (nsl + 3u) / 4u));
}

// XOR of v over the 16 lanes of each row (every lane gets it): row rotations by 8 and 4,
// then two quad permutations.
__device__ __forceinline__ uint32_t row_xor16(uint32_t v)
{
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    return v;
}

// Three waves per SIMD at most (168 VGPRs): the pipelined rounds would otherwise take 170.
template <int MODE>
__global__ __launch_bounds__(256, 3) void rx_server(SrvArgs sa)
{
    __shared__ SrvReq s_req;
    __shared__ unsigned long long s_desc[kSrvPollWords - 16];  // an inline request's off64 / len
    __shared__ unsigned long long s_seq;  // the request's number (kSrvStop: exit)
    __shared__ uint32_t s_p;              // its participants
    // thread 0: the number of the last request seen.  It starts at `done` (the host sets go to
    // done << 16 before the launch): a workgroup that starts late, after a request g it should
    // take part in was published, still sees g as new, since g is not done without it.
    unsigned long long last = 0ull;
    if (threadIdx.x == 0) last = __hip_atomic_load(&sa.ret->done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    for (;;) {
        if (blockIdx.x == 0 && threadIdx.x < 64) {
            // wave 0 polls the mailbox's first 320 bytes (lane l < 40: bytes 8l .. 8l+7) in
            // one instruction: the request arrives with its number and, for a small host
            // burst, its descriptors (words 16-39): no second round trip before the frames
            const int l = (int)threadIdx.x;
            const unsigned long long lst = __shfl(last, 0, 64);
            const long long t0 = wall_clock64();
            unsigned long long q;
            for (;;) {
                unsigned long long w = 0ull;
                if (l < kSrvPollWords)
                    w = __hip_atomic_load(reinterpret_cast<const unsigned long long *>(sa.mbox) + l, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_SYSTEM);
                q = __shfl(w, 0, 64);
                const unsigned long long ck = __shfl(w, 12, 64), st = __shfl(w, 13, 64);
                if (st != 0ull) {
                    q = kSrvStop;
                    break;
                }
                if (q != lst) {
                    // the check word over the number, the request words (lanes 0-11) and an
                    // inline request's descriptor words (lanes 16-39; SrvReq::flags is the
                    // high half of word 5): a snapshot mixing two requests' words (a
                    // write-combined mailbox line that reached the device in parts) fails it
                    // and is polled again
                    const bool inl = ((__shfl(w, 5, 64) >> 32) & kSrvInlineDesc) != 0ull;
                    const bool mixed = l < 12 || (inl && l >= 16 && l < kSrvPollWords);
                    const unsigned long long m = mixed ? srv_mix((unsigned)l, w) : 0ull;
                    const uint32_t lo = row_xor16((uint32_t)m), hi = row_xor16((uint32_t)(m >> 32));
                    // the rows' XORs (lanes 48-63 hold none)
                    const uint32_t xlo = (uint32_t)__builtin_amdgcn_readlane((int)lo, 0) ^
                                         (uint32_t)__builtin_amdgcn_readlane((int)lo, 16) ^
                                         (uint32_t)__builtin_amdgcn_readlane((int)lo, 32);
                    const uint32_t xhi = (uint32_t)__builtin_amdgcn_readlane((int)hi, 0) ^
                                         (uint32_t)__builtin_amdgcn_readlane((int)hi, 16) ^
                                         (uint32_t)__builtin_amdgcn_readlane((int)hi, 32);
                    if ((((unsigned long long)xhi << 32) | xlo) == ck) {
                        if (l >= 1 && l <= 11) reinterpret_cast<unsigned long long *>(&s_req)[l - 1] = w;  // bytes 8 .. 95
                        if (inl && l >= 16 && l < kSrvPollWords) s_desc[l - 16] = w;
                        break;
                    }
                }
                if ((unsigned long long)(wall_clock64() - t0) > sa.idle_ticks) {
                    q = kSrvStop;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            // One acquire per request, not per poll: the CU's L1 may hold lines of the previous
            // request's staging (host memory, same addresses) or of device memory written since
            // (mirror tables, caller frames); waited for before any wave of the workgroup loads
            // (MI355X_MICROARCH.md, inter-workgroup visibility).  A first form with relaxed
            // polls and no acquire served stale staging lines (test_gpu_server).
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            // the request's words, written by lanes 1-11, for lane 0
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (l == 0) {
                const uint32_t P = q == kSrvStop ? gridDim.x : srv_participants(s_req.n, s_req.flags);
                // the others hear of a request only when they take part in it (and of stop)
                if (gridDim.x > 1 && P > 1u) {
                    if (q != kSrvStop) sa.ctl->req = s_req;
                    // release (MI355X_MICROARCH.md: the wait after the write-back, by hand)
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __hip_atomic_store(&sa.ctl->go, q == kSrvStop ? kSrvStop : (q << 16) | P, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
                s_seq = q;
                s_p = P;
                last = q;
            }
        } else if (blockIdx.x != 0 && threadIdx.x == 0) {
            unsigned long long go;
            for (;;) {  // relaxed polls, then one acquire (MI355X_MICROARCH.md)
                go = __hip_atomic_load(&sa.ctl->go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((go >> 16) != last) break;  // (kSrvStop >> 16 is no request number)
                __builtin_amdgcn_s_sleep(2);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // this CU's L1 (see workgroup 0)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t P = go == kSrvStop ? gridDim.x : (uint32_t)(go & 0xFFFFu);
            if (go != kSrvStop && blockIdx.x < P) {
                // vector loads (never the scalar cache, which the acquire does not invalidate)
                const unsigned long long *src = reinterpret_cast<const unsigned long long *>(&sa.ctl->req);
                unsigned long long *dst = reinterpret_cast<unsigned long long *>(&s_req);
#pragma unroll
                for (int k = 0; k < (int)(sizeof(SrvReq) / 8); ++k)
                    dst[k] = __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            s_seq = go == kSrvStop ? kSrvStop : go >> 16;
            s_p = P;
            last = go >> 16;
        }
        __syncthreads();
        const unsigned long long q = s_seq;
        if (q == kSrvStop) break;
        const uint32_t P = s_p;
        if (blockIdx.x >= P) {  // published for the first P workgroups of a larger grid
            __syncthreads();
            continue;
        }
        RxArgs a;
        a.frames = as_global<const uint8_t>(uniform64((uint64_t)s_req.frames));
        a.sel = nullptr;
        a.nbursts = 1u;
        a.stride64 = 0u;
        a.t.buckets = as_global<const uint4>(uniform64((uint64_t)s_req.table.buckets));
        a.t.listen = as_global<const int32_t>(uniform64((uint64_t)s_req.table.listen));
        a.t.arp = as_global<const uint4>(uniform64((uint64_t)s_req.table.arp));
        a.t.bucket_mask = uniform(s_req.table.bucket_mask);
        a.t.ntcb = (int32_t)uniform((uint32_t)s_req.table.ntcb);
        a.t.min_null = (int32_t)uniform((uint32_t)s_req.table.min_null);
        a.t.arp_mask = uniform(s_req.table.arp_mask);
        a.t.arp_flags = uniform(s_req.table.arp_flags);
        a.counters = sa.counters;
        if (uniform(s_req.flags) & kSrvInlineDesc) {
            // a small host burst: its descriptors came with the request (LDS, generic pointers)
            a.b[0].off64 = reinterpret_cast<const uint32_t *>(s_desc);
            a.b[0].len = reinterpret_cast<const uint16_t *>(reinterpret_cast<const uint8_t *>(s_desc) + kSrvInline * 4u);
        } else {
            a.b[0].off64 = reinterpret_cast<const uint32_t *>(uniform64((uint64_t)s_req.off64));
            a.b[0].len = reinterpret_cast<const uint16_t *>(uniform64((uint64_t)s_req.len));
        }
        a.b[0].out = as_global<uint8_t>(uniform64((uint64_t)s_req.out));
        a.b[0].n = uniform(s_req.n);
        a.b[0].slice0 = 0u;
        a.nslices = (a.b[0].n + 63u) / 64u;
        rx_body<MODE, kDescList, false, false, true>(a, blockIdx.x, P);
        // Every wave's stores have reached the L2 (vmcnt), then ONE system-scope release per
        // workgroup writes this XCD's L2 back (buffer_wbl2 covers the whole cache, so one
        // per workgroup covers its four waves; it used to run once per wave and once more
        // before `done`), before the workgroup counts itself finished
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            bool lastp = true;
            if (P > 1u) {
                lastp = atomicAdd(&sa.ctl->fin, 1u) + 1u == P;
                if (lastp) {
                    atomicExch(&sa.ctl->fin, 0u);  // before `done`: the next request counts from 0
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            }
            if (lastp) __hip_atomic_store(&sa.ret->done, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();  // s_req and s_seq are rewritten by the next request
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(&sa.ret->exited, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace rxg
