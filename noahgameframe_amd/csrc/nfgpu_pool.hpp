// nfgpu_pool.hpp — a small pool of host worker threads for the per-call host work of large call
// batches (GUID lookups of a batch of queued calls, folding a window's calls into (slot, property)
// groups).  A job is `parts` independent pieces run by the workers and the calling thread; the
// caller returns when every piece is done.  Workers spin briefly between jobs (a frame hands them
// several jobs within a few hundred microseconds) and then sleep.
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace nfgpu_detail {

class HostPool {
public:
    explicit HostPool(int workers) {
        for (int i = 0; i < workers; i++) th_.emplace_back([this] { loop(); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_.store(true);
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    HostPool(const HostPool&) = delete;
    HostPool& operator=(const HostPool&) = delete;
    int threads() const { return (int)th_.size() + 1; }

    // f(p) for every p in [0, parts), on the workers and the caller
    void run(int parts, const std::function<void(int)>& f) {
        if (parts <= 0) return;
        if (parts == 1 || th_.empty()) {
            for (int p = 0; p < parts; p++) f(p);
            return;
        }
        const uint64_t g = (gen_.load(std::memory_order_relaxed) + 1) & 0xFFFFFFFFull;
        // (generation, next piece) first: a worker still in the previous generation's work() then
        // fails its claim on the old counter, whatever parts_ it reads; parts_ last, with release,
        // so a worker that reads the new parts_ also sees the new counter
        next_.store(g << 32, std::memory_order_relaxed);
        f_.store(&f, std::memory_order_relaxed);
        done_.store(0, std::memory_order_relaxed);
        parts_.store(parts, std::memory_order_release);
        {
            std::lock_guard<std::mutex> lk(mu_);
            gen_.store(g, std::memory_order_release);
        }
        if (sleeping_.load(std::memory_order_acquire)) cv_.notify_all();
        work(g);
        while (done_.load(std::memory_order_acquire) < parts) std::this_thread::yield();
    }

private:
    // claim and run pieces of generation g until none is left
    void work(uint64_t g) {
        for (;;) {
            uint64_t x = next_.load(std::memory_order_acquire);
            int p;
            do {
                if ((x >> 32) != g || (int)(x & 0xFFFFFFFFu) >= parts_.load(std::memory_order_acquire)) return;
                p = (int)(x & 0xFFFFFFFFu);
            } while (!next_.compare_exchange_weak(x, x + 1, std::memory_order_acq_rel));
            (*f_.load(std::memory_order_relaxed))(p);
            done_.fetch_add(1, std::memory_order_release);
        }
    }
    void loop() {
        uint64_t seen = gen_.load(std::memory_order_acquire);
        for (;;) {
            // spin ~50 us for the next job of the frame, then sleep
            const auto t0 = std::chrono::steady_clock::now();
            uint64_t g = gen_.load(std::memory_order_acquire);
            while (g == seen && std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(50)) {
                std::this_thread::yield();
                g = gen_.load(std::memory_order_acquire);
            }
            if (g == seen) {
                std::unique_lock<std::mutex> lk(mu_);
                sleeping_.fetch_add(1, std::memory_order_acq_rel);
                cv_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen; });
                sleeping_.fetch_sub(1, std::memory_order_acq_rel);
                g = gen_.load(std::memory_order_acquire);
            }
            seen = g;
            if (stop_.load()) return;
            work(g);
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::atomic<uint64_t> gen_{0}, next_{0};
    std::atomic<int> done_{0}, sleeping_{0};
    std::atomic<bool> stop_{false};
    std::atomic<const std::function<void(int)>*> f_{nullptr};
    std::atomic<int> parts_{0};
};

}  // namespace nfgpu_detail
