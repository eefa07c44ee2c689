// fifo_scheduler.h — FIFO job scheduler (client_lib/src/scheduler.h:74-112,
// schedulers/fifo_scheduler.{h,cc}).  Every job is cut into one contiguous
// slice per worker thread; the slice geometry decides where packets (blocks)
// start, so it is part of the parity contract.
#ifndef SWITCHML_AMD_FIFO_SCHEDULER_H_
#define SWITCHML_AMD_FIFO_SCHEDULER_H_

#include <condition_variable>
#include <map>
#include <memory>
#include <atomic>
#include <mutex>
#include <queue>
#include <vector>

#include "config.h"
#include "job.h"

namespace switchml {

// Reusable thread barrier that can be torn down to release waiters
// (the role of utils.cc:43-72 Barrier).
class Barrier {
  public:
    explicit Barrier(int n) : n_(n) {}
    // Returns false if the barrier was destroyed while waiting.
    bool Wait();
    void Destroy();

  private:
    std::mutex m_;
    std::condition_variable cv_;
    int n_;
    int count_ = 0;
    uint64_t generation_ = 0;
    bool destroyed_ = false;
    // lock-free mirrors of generation_ / destroyed_ for the short poll before sleeping
    std::atomic<uint64_t> generation_flag_{0};
    std::atomic<bool> destroyed_flag_{false};
};

// Slice t of T of a job of numel elements (fifo_scheduler.cc:93-109): the
// first numel % T slices get one extra element.
void FifoSliceGeometry(Numel numel, int T, int t, Numel* offset, Numel* slice_numel);

class FifoScheduler {
  public:
    explicit FifoScheduler(const Config& config);

    bool EnqueueJob(std::shared_ptr<Job> job);
    // Blocks (after a barrier with the other worker threads) until a job is
    // queued or the scheduler stops; false when stopped.
    bool GetJobSlice(WorkerTid worker_thread_id, JobSlice& job_slice);
    // Batched dispatch (one worker thread runs every slice): blocks until a
    // job is queued, then hands out up to max_jobs queued jobs whole (all
    // num_worker_threads slices of each dispatched at once; the caller cuts
    // them with FifoSliceGeometry and reports every slice's completion).
    // No barrier.  False when stopped.
    bool GetJobs(size_t max_jobs, std::vector<std::shared_ptr<Job>>& jobs);
    // True when this completed the job's last RUNNING slice: all T slices,
    // or after Stop() every slice that had been handed out.  Only then may
    // the caller publish the job's final status (its buffers are released).
    bool NotifyJobSliceCompletion(WorkerTid worker_thread_id, const JobSlice& job_slice);
    // Jobs enqueued so far (a job's sched_seq is its position in this count).
    // A worker thread that has taken the slice of job `seq` will find the next
    // job without blocking iff EnqueuedCount() > seq: all worker threads take
    // the slices of the same job between two barriers, in FIFO order.
    uint64_t EnqueuedCount() const { return enqueued_.load(std::memory_order_acquire); }
    // Fail every queued job and wake all waiting worker threads.  A queued
    // job none of whose slices is running is published FAILED here; one with
    // running slices is marked failed and published by its last slice.
    void Stop();

  private:
    const Config& config_;
    std::mutex access_mutex_;
    std::condition_variable job_submitted_event_;
    std::queue<std::shared_ptr<Job>> queue_;
    std::map<JobId, int> undispatched_job_slices_;
    std::map<JobId, int> finished_job_slices_;
    std::map<JobId, int> dispatched_job_slices_;
    Barrier barrier_;
    bool stopped_ = false;
    // lock-free mirrors of stopped_ / queue_.size() for the short poll before
    // a worker sleeps on job_submitted_event_
    std::atomic<bool> stopped_flag_{false};
    std::atomic<size_t> queue_size_{0};
    std::atomic<uint64_t> enqueued_{0};
};

}  // namespace switchml

#endif  // SWITCHML_AMD_FIFO_SCHEDULER_H_
