// pool.h — a small fork-join thread pool for the host paths' CPU gather /
// scatter copies (hostpath.cpp, shardhash.cpp).
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace hbec {

class Pool {
   public:
    explicit Pool(int n) {
        for (int i = 0; i < n; ++i) threads_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : threads_) t.join();
    }
    int size() const { return (int)threads_.size(); }
    // run f(i) for i in [0, n) on the pool + calling thread; returns when done.
    // Items are handed out in grains by an atomic counter (a 64 MiB chunk of
    // 4 KiB stripes is 65 536 one-KiB copies: a lock per item made the copies
    // wait on the lock), and the call returns only after every worker has
    // left this generation, so no straggler can take an item of the next.
    void parallel_for(size_t n, const std::function<void(size_t)>& f) {
        if (n == 0) return;
        const size_t grain = std::max<size_t>(1, n / ((threads_.size() + 1) * 8));
        {
            std::lock_guard<std::mutex> g(mu_);
            fn_ = &f;
            total_ = n;
            grain_ = grain;
            next_.store(0, std::memory_order_relaxed);
            done_.store(0, std::memory_order_relaxed);
            ++gen_;
        }
        cv_.notify_all();
        run_items(f, n, grain);
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return done_.load(std::memory_order_acquire) == total_ && active_ == 0; });
        fn_ = nullptr;
    }

   private:
    void run_items(const std::function<void(size_t)>& f, size_t total, size_t grain) {
        for (;;) {
            const size_t a = next_.fetch_add(grain, std::memory_order_relaxed);
            if (a >= total) return;
            const size_t b = std::min(total, a + grain);
            for (size_t i = a; i < b; ++i) f(i);
            if (done_.fetch_add(b - a, std::memory_order_acq_rel) + (b - a) == total) {
                std::lock_guard<std::mutex> g(mu_);
                done_cv_.notify_all();
            }
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(size_t)>* f;
            size_t total, grain;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || (gen_ != seen && fn_); });
                if (stop_) return;
                seen = gen_;
                f = fn_;
                total = total_;
                grain = grain_;
                ++active_;
            }
            run_items(*f, total, grain);
            {
                std::lock_guard<std::mutex> g(mu_);
                if (--active_ == 0) done_cv_.notify_all();
            }
        }
    }
    std::vector<std::thread> threads_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(size_t)>* fn_ = nullptr;
    size_t total_ = 0, grain_ = 1;
    std::atomic<size_t> next_{0}, done_{0};
    int active_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};


// Worker threads for the host paths: HBEC_HOST_THREADS, else the process's
// CPU share (OMP_NUM_THREADS; 16 per GPU on the MI355X boxes), capped by the
// hardware; the calling thread is the last worker.
int host_threads();

}  // namespace hbec
