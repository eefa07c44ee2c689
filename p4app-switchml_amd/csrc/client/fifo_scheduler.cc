// fifo_scheduler.cc — see fifo_scheduler.h.
#include "fifo_scheduler.h"

#include <chrono>
#include <thread>

namespace switchml {

bool Barrier::Wait() {
    std::unique_lock<std::mutex> lock(m_);
    if (destroyed_) return false;
    const uint64_t gen = generation_;
    if (++count_ == n_) {
        count_ = 0;
        generation_++;
        generation_flag_.store(generation_, std::memory_order_release);
        cv_.notify_all();
        return true;
    }
    if (SpinMicros() > 0) {
        // The worker threads of one job arrive within microseconds of each
        // other: poll for a short while before sleeping (a futex wake-up per
        // job costs about as much as a 25 MiB bucket's kernels).
        lock.unlock();
        const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(SpinMicros());
        while (generation_flag_.load(std::memory_order_acquire) == gen &&
               !destroyed_flag_.load(std::memory_order_acquire) && std::chrono::steady_clock::now() < until)
            std::this_thread::yield();
        lock.lock();
    }
    cv_.wait(lock, [&] { return generation_ != gen || destroyed_; });
    return !destroyed_ || generation_ != gen;
}

void Barrier::Destroy() {
    std::unique_lock<std::mutex> lock(m_);
    destroyed_ = true;
    destroyed_flag_.store(true, std::memory_order_release);
    cv_.notify_all();
}

void FifoSliceGeometry(Numel numel, int T, int t, Numel* offset, Numel* slice_numel) {
    Numel n = numel / (Numel)T;
    const Numel rem = numel % (Numel)T;
    if (rem > (Numel)t) {
        n++;
        *offset = (Numel)t * n;        // every earlier slice also got an extra element
    } else {
        *offset = (Numel)t * n + rem;  // the rem extra elements sit before this slice
    }
    *slice_numel = n;
}

FifoScheduler::FifoScheduler(const Config& config)
    : config_(config), barrier_(config.general_.num_worker_threads) {}

bool FifoScheduler::EnqueueJob(std::shared_ptr<Job> job) {
    std::unique_lock<std::mutex> lock(access_mutex_);
    if (stopped_) {
        job->SetJobStatus(FAILED);
        return false;
    }
    job->SetJobStatus(QUEUED);
    job->sched_seq.store(enqueued_.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed);
    finished_job_slices_[job->id_] = 0;
    dispatched_job_slices_[job->id_] = 0;
    undispatched_job_slices_[job->id_] = config_.general_.num_worker_threads;
    queue_.push(job);
    queue_size_.store(queue_.size(), std::memory_order_release);
    enqueued_.fetch_add(1, std::memory_order_release);
    job_submitted_event_.notify_all();
    return true;
}

bool FifoScheduler::GetJobSlice(WorkerTid tid, JobSlice& job_slice) {
    {
        std::unique_lock<std::mutex> lock(access_mutex_);
        if (stopped_) return false;
    }
    // All worker threads meet here so that they take slices of the same job.
    if (!barrier_.Wait()) return false;
    std::unique_lock<std::mutex> lock(access_mutex_);
    if (!stopped_ && queue_.empty() && SpinMicros() > 0) {
        // Jobs tend to come in bursts (a framework's gradient buckets): poll
        // for a short while before sleeping, so the next job does not pay a
        // futex wake-up.
        lock.unlock();
        const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(SpinMicros());
        while (!stopped_flag_.load(std::memory_order_acquire) && queue_size_.load(std::memory_order_acquire) == 0 &&
               std::chrono::steady_clock::now() < until)
            std::this_thread::yield();
        lock.lock();
    }
    job_submitted_event_.wait(lock, [this] { return stopped_ || !queue_.empty(); });
    if (stopped_) return false;

    std::shared_ptr<Job> job = queue_.front();
    dispatched_job_slices_.at(job->id_)++;
    int& left = undispatched_job_slices_.at(job->id_);
    if (--left == 0) {
        queue_.pop();
        queue_size_.store(queue_.size(), std::memory_order_release);
        undispatched_job_slices_.erase(job->id_);
    }
    job_slice.job = job;
    job_slice.slice = job->tensor_;
    Numel offset, n;
    FifoSliceGeometry(job->tensor_.numel, config_.general_.num_worker_threads, tid, &offset, &n);
    job_slice.slice.numel = n;
    job_slice.slice.OffsetPtrs(offset);
    job->SetJobStatus(RUNNING);
    return true;
}

bool FifoScheduler::GetJobs(size_t max_jobs, std::vector<std::shared_ptr<Job>>& jobs) {
    std::unique_lock<std::mutex> lock(access_mutex_);
    if (!stopped_ && queue_.empty() && SpinMicros() > 0) {
        lock.unlock();
        const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(SpinMicros());
        while (!stopped_flag_.load(std::memory_order_acquire) && queue_size_.load(std::memory_order_acquire) == 0 &&
               std::chrono::steady_clock::now() < until)
            std::this_thread::yield();
        lock.lock();
    }
    job_submitted_event_.wait(lock, [this] { return stopped_ || !queue_.empty(); });
    if (stopped_) return false;
    const int T = config_.general_.num_worker_threads;
    while (!queue_.empty() && jobs.size() < max_jobs) {
        std::shared_ptr<Job> job = queue_.front();
        queue_.pop();
        dispatched_job_slices_.at(job->id_) = T;
        undispatched_job_slices_.erase(job->id_);
        job->SetJobStatus(RUNNING);
        jobs.push_back(std::move(job));
    }
    queue_size_.store(queue_.size(), std::memory_order_release);
    return true;
}

bool FifoScheduler::NotifyJobSliceCompletion(WorkerTid, const JobSlice& job_slice) {
    std::unique_lock<std::mutex> lock(access_mutex_);
    const JobId id = job_slice.job->id_;
    if (stopped_) job_slice.job->MarkFailed();
    int& done = finished_job_slices_.at(id);
    // after Stop() the slices never handed out will not run: the job is over
    // when every slice that was handed out has come back
    const int need = stopped_ ? dispatched_job_slices_.at(id) : config_.general_.num_worker_threads;
    if (++done == need) {
        finished_job_slices_.erase(id);
        dispatched_job_slices_.erase(id);
        return true;
    }
    return false;
}

void FifoScheduler::Stop() {
    std::unique_lock<std::mutex> lock(access_mutex_);
    stopped_ = true;
    stopped_flag_.store(true, std::memory_order_release);
    barrier_.Destroy();
    while (!queue_.empty()) {
        std::shared_ptr<Job> job = queue_.front();
        queue_.pop();
        job->MarkFailed();
        if (dispatched_job_slices_.at(job->id_) == 0) {  // nothing running: publish now
            finished_job_slices_.erase(job->id_);
            dispatched_job_slices_.erase(job->id_);
            job->SetJobStatus(FAILED);
        }
    }
    queue_size_.store(0, std::memory_order_release);
    undispatched_job_slices_.clear();
    job_submitted_event_.notify_all();
}

}  // namespace switchml
