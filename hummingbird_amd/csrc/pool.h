// pool.h — a small fork-join thread pool for the host paths' CPU gather /
// scatter copies (hostpath.cpp, shardhash.cpp).
#pragma once
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
    // run f(i) for i in [0, n) on the pool + calling thread; returns when done
    void parallel_for(size_t n, const std::function<void(size_t)>& f) {
        if (n == 0) return;
        std::unique_lock<std::mutex> lk(mu_);
        fn_ = &f;
        next_ = 0;
        total_ = n;
        done_ = 0;
        ++gen_;
        lk.unlock();
        cv_.notify_all();
        work();
        lk.lock();
        done_cv_.wait(lk, [&] { return done_ == total_; });
        fn_ = nullptr;
    }

   private:
    void work() {
        for (;;) {
            size_t i;
            const std::function<void(size_t)>* f;
            {
                std::lock_guard<std::mutex> g(mu_);
                if (!fn_ || next_ >= total_) return;
                i = next_++;
                f = fn_;
            }
            (*f)(i);
            {
                std::lock_guard<std::mutex> g(mu_);
                if (++done_ == total_) done_cv_.notify_all();
            }
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || (gen_ != seen && fn_ && next_ < total_); });
                if (stop_) return;
                seen = gen_;
            }
            work();
        }
    }
    std::vector<std::thread> threads_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(size_t)>* fn_ = nullptr;
    size_t next_ = 0, total_ = 0, done_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};


// Worker threads for the host paths: HBEC_HOST_THREADS, else the process's
// CPU share (OMP_NUM_THREADS; 16 per GPU on the MI355X boxes), capped by the
// hardware; the calling thread is the last worker.
int host_threads();

}  // namespace hbec
