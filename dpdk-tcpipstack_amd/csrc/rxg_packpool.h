// rxg_packpool.h -- host threads kept for a context's life that run one job split n ways
// (rxg_rx_burst packs large host bursts into pinned staging with them).  Header-only so the
// CPU tests can build it under ThreadSanitizer (tests/test_opqueue.py).
#pragma once

#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace rxg {

// Host threads that pack large host bursts into the pinned staging (rxg_rx_burst), started
// at the first burst that needs them and kept for the context's life: no thread is
// created per burst.
class PackPool {
  public:
    ~PackPool()
    {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    // Runs fn(0) .. fn(n - 1), fn(0) on the calling thread; returns when all are done.
    void run(uint32_t n, const std::function<void(uint32_t)> &fn)
    {
        if (n <= 1) {
            fn(0);
            return;
        }
        while (th_.size() < n - 1) {
            const uint32_t id = (uint32_t)th_.size() + 1;
            th_.emplace_back([this, id] { worker(id); });
        }
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &fn;
            n_ = n;
            pending_ = n - 1;
            ++gen_;
        }
        cv_.notify_all();
        fn(0);
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [this] { return pending_ == 0; });
        job_ = nullptr;
    }

  private:
    void worker(uint32_t id)
    {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(uint32_t)> *job;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                if (id >= n_) continue;  // not needed for this burst
                job = job_;
            }
            (*job)(id);
            {
                std::lock_guard<std::mutex> g(m_);
                if (--pending_ == 0) done_.notify_one();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(uint32_t)> *job_ = nullptr;
    uint32_t n_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

}  // namespace rxg
