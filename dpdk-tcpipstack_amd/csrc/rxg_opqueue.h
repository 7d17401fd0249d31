// rxg_opqueue.h — the cross-thread TCB-mirror queue (SURVEY.md §8(b) "Threading").
//
// In the reference the socket API runs on lcore 1 (alloc_tcb under tcb_alloc_mutex,
// tcp_tcb.c:97-103; tuple writes in socket_bind, socket_interface.c:80-83, and
// socket_connect, :329-332) while the rx loop on lcore 2 reads tcbs[] in findtcb without a
// lock.  rxg keeps its mirror single-threaded: an app thread posts its tcbs[] writes here,
// lock-free, and the rx thread applies them in order at the next burst boundary, so a
// kernel never sees a half-written slot.
//
// Bounded multi-producer / single-consumer ring (Vyukov's sequence-numbered cells):
// producers claim a cell with one CAS on the tail, write it, then publish it by storing
// its sequence number; the consumer takes cells in claim order while their sequence
// says "published".  No locks, no allocation after construction.  Host-only.
#pragma once
#include <atomic>
#include <cstdint>
#include <memory>

namespace rxg {

template <typename T>
class MpscRing {
public:
    explicit MpscRing(uint32_t capacity_pow2) : mask_(capacity_pow2 - 1u), cells_(new Cell[capacity_pow2])
    {
        for (uint32_t i = 0; i < capacity_pow2; ++i) cells_[i].seq.store(i, std::memory_order_relaxed);
    }

    // Any thread.  False when the ring is full (the consumer has not drained it).
    bool push(const T &v)
    {
        uint64_t pos = tail_.load(std::memory_order_relaxed);
        for (;;) {
            Cell &c = cells_[pos & mask_];
            const uint64_t seq = c.seq.load(std::memory_order_acquire);
            const int64_t dif = (int64_t)seq - (int64_t)pos;
            if (dif == 0) {
                if (tail_.compare_exchange_weak(pos, pos + 1, std::memory_order_relaxed)) {
                    c.val = v;
                    c.seq.store(pos + 1, std::memory_order_release);
                    return true;
                }
            } else if (dif < 0) {
                return false;  // full
            } else {
                pos = tail_.load(std::memory_order_relaxed);
            }
        }
    }

    // The single consumer thread.  False when the next cell in claim order is not
    // published yet (empty, or its producer is between claim and publish).
    bool pop(T &out)
    {
        Cell &c = cells_[head_ & mask_];
        const uint64_t seq = c.seq.load(std::memory_order_acquire);
        if ((int64_t)seq - (int64_t)(head_ + 1) < 0) return false;
        out = c.val;
        c.seq.store(head_ + mask_ + 1, std::memory_order_release);
        ++head_;
        return true;
    }

    uint32_t capacity() const { return mask_ + 1u; }

private:
    struct Cell {
        std::atomic<uint64_t> seq;
        T val;
    };
    const uint64_t mask_;
    std::unique_ptr<Cell[]> cells_;
    alignas(64) std::atomic<uint64_t> tail_{0};
    alignas(64) uint64_t head_ = 0;
};

}  // namespace rxg
