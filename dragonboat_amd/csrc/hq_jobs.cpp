// hq_jobs.cpp — hq_worker_step_jobs: several step workers stepped at once, one native thread
// each, the way dragonboat's step-worker goroutines each drive their own worker
// (execengine.go:923-1000, 16 of them, internal/settings/hard.go:36). A process-wide pool of
// threads, grown on demand and parked on a condition variable between calls; job 0 runs on the
// calling thread.
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/hipquorum.h"
#include "hq_dstep.h"

namespace {

int run_job(hq_step_job &j) {
    if (!j.worker || !j.out || (!j.rows) == (!j.stream)) return j.rc = HQ_E_INVAL;
    return j.rc = j.stream ? hq_worker_step_stream(j.worker, j.stream, j.out)
                           : hq_worker_step(j.worker, j.rows, j.out);
}

class Pool {
  public:
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : threads_) t.join();
    }

    int run(hq_step_job *jobs, uint32_t count) {
        std::lock_guard<std::mutex> call(call_mu_);      // one batch of jobs at a time
        while (threads_.size() + 1 < count) {
            const size_t k = threads_.size();
            threads_.emplace_back([this, k] { loop(k); });
        }
        {
            std::lock_guard<std::mutex> g(mu_);
            jobs_ = jobs;
            count_ = count;
            pending_ = count - 1;
            ++gen_;
        }
        cv_.notify_all();
        run_job(jobs[0]);
        std::unique_lock<std::mutex> g(mu_);
        done_.wait(g, [this] { return pending_ == 0; });
        for (uint32_t i = 0; i < count; ++i)
            if (jobs[i].rc) return jobs[i].rc;
        return HQ_OK;
    }

  private:
    void loop(size_t k) {
        uint64_t seen = 0;
        for (;;) {
            hq_step_job *job = nullptr;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                if (k + 1 < count_) job = jobs_ + k + 1;
            }
            if (!job) continue;
            run_job(*job);
            std::lock_guard<std::mutex> g(mu_);
            if (--pending_ == 0) done_.notify_one();
        }
    }

    std::mutex call_mu_, mu_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> threads_;
    hq_step_job *jobs_ = nullptr;
    uint32_t count_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

Pool &pool() {
    static Pool p;
    return p;
}

}  // namespace

extern "C" int hq_worker_step_jobs(hq_step_job *jobs, uint32_t count) {
    if (!jobs && count) return HQ_E_INVAL;
    if (count == 0) return HQ_OK;
    for (uint32_t i = 0; i < count; ++i) {             // a worker is not thread-safe
        jobs[i].rc = HQ_OK;
        for (uint32_t k = 0; k < i; ++k)
            if (jobs[k].worker == jobs[i].worker) return HQ_E_INVAL;
    }
    if (count == 1) return run_job(jobs[0]);
    const int f = hq_worker_step_jobs_fused(jobs, count);
    if (f != kJobsNotFused) return f;
    return pool().run(jobs, count);
}
