// context.h — the SwitchML client Context (client_lib/src/context.h:40-231),
// MI355X build: same singleton API (Start / Stop / AllReduceAsync / AllReduce
// / WaitForAllJobs / GetConfig / GetStats), worker threads fed by the FIFO
// scheduler, and a loopback ("dummy") backend whose worker threads drive the
// GPU pre/post-processor.  Tensors may live in host or device memory.
#ifndef SWITCHML_AMD_CONTEXT_H_
#define SWITCHML_AMD_CONTEXT_H_

#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "common.h"
#include "config.h"
#include "fifo_scheduler.h"
#include "job.h"

namespace switchml {

// Counters behind Context::GetStats (the reference's Stats, stats.h:40-167,
// reduced to what this backend can observe).
class Stats {
  public:
    void Init(int num_worker_threads);
    void IncJobsSubmitted(Numel numel) { jobs_submitted_++; numel_submitted_ += numel; }
    void IncJobsFinished() { jobs_finished_++; }
    void AddSlice(WorkerTid tid, uint64_t ltus, uint64_t bytes);
    uint64_t jobs_submitted() const { return jobs_submitted_; }
    uint64_t jobs_finished() const { return jobs_finished_; }
    uint64_t numel_submitted() const { return numel_submitted_; }
    uint64_t ltus_processed() const;
    uint64_t slices_processed() const;
    void LogStats() const;
    void ResetStats();

  private:
    std::atomic<uint64_t> jobs_submitted_{0}, jobs_finished_{0}, numel_submitted_{0};
    std::unique_ptr<std::atomic<uint64_t>[]> slices_, ltus_, bytes_;
    int n_ = 0;
};

class LoopbackBackend;

class Context {
  public:
    enum ContextState { CREATED, STARTING, RUNNING, STOPPING, STOPPED };

    static Context& GetInstance();
    Context(const Context&) = delete;
    void operator=(const Context&) = delete;

    // config == nullptr: load switchml.cfg from the reference's search path.
    // Unlike the reference, a STOPPED context may be started again.
    bool Start(Config* config = nullptr);
    void Stop();

    std::shared_ptr<Job> AllReduceAsync(void* in_ptr, void* out_ptr, uint64_t numel, DataType data_type,
                                        AllReduceOperation all_reduce_operation);
    std::shared_ptr<Job> AllReduce(void* in_ptr, void* out_ptr, uint64_t numel, DataType data_type,
                                   AllReduceOperation all_reduce_operation);
    void WaitForAllJobs();

    ContextState GetContextState() const { return context_state_.load(); }
    Config& GetConfig() { return config_; }
    Stats& GetStats() { return stats_; }

    // Worker-thread side (context.cc:174-197).
    bool GetJobSlice(WorkerTid worker_thread_id, JobSlice& job_slice);
    // Batched dispatch (FifoScheduler::GetJobs): up to max_jobs whole jobs.
    bool GetJobs(size_t max_jobs, std::vector<std::shared_ptr<Job>>& jobs);
    // A job after the one with sched_seq `seq` is queued, so GetJobSlice will
    // hand this worker thread its slice without blocking on an empty queue.
    bool HasJobAfter(uint64_t seq) const { return scheduler_ && scheduler_->EnqueuedCount() > seq; }
    void NotifyJobSliceCompletion(WorkerTid worker_thread_id, const JobSlice& job_slice, bool ok = true);

    int device() const { return device_; }

  private:
    Context();
    ~Context();

    std::unique_ptr<FifoScheduler> scheduler_;
    std::unique_ptr<LoopbackBackend> backend_;
    Config config_;
    Stats stats_;
    std::atomic<ContextState> context_state_;
    uint64_t number_of_current_jobs_ = 0;
    std::mutex access_mutex_;
    std::condition_variable all_jobs_finished_event_;
    int device_ = 0;
};

}  // namespace switchml

#endif  // SWITCHML_AMD_CONTEXT_H_
