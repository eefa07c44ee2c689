// job.h — Job / JobSlice (client_lib/src/job.h:51-148).
#ifndef SWITCHML_AMD_JOB_H_
#define SWITCHML_AMD_JOB_H_

#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>

#include "common.h"

namespace switchml {

enum JobStatus { INIT, QUEUED, RUNNING, FINISHED, FAILED };

class Job {
  public:
    Job(Tensor tensor, JobType job_type, ExtraJobInfo extra_job_info);
    Job(const Job&) = delete;
    Job& operator=(const Job&) = delete;

    // Block until the job is FINISHED or FAILED (polls for SpinMicros() first).
    void WaitToComplete();
    JobStatus GetJobStatus() const { return job_status_.load(); }
    // Statuses only move forward; FINISHED/FAILED wake waiters (job.cc:49-57).
    void SetJobStatus(JobStatus status);
    // A slice failed (or the context stopped under it).  Recorded only: the
    // job is published FAILED by its last running slice, so no waiter wakes
    // while sibling slices still read in_ptr / write out_ptr.
    void MarkFailed() { failed_.store(true, std::memory_order_release); }
    bool HasFailed() const { return failed_.load(std::memory_order_acquire); }

    const JobId id_;
    const Tensor tensor_;
    const JobType job_type_;
    const ExtraJobInfo extra_job_info_;

  private:
    static std::atomic<JobId> next_id_;
    std::atomic<JobStatus> job_status_;
    std::atomic<bool> failed_{false};

  public:
    // Position in the scheduler's FIFO (1, 2, ...), set when it is enqueued.
    std::atomic<uint64_t> sched_seq{0};
    std::mutex access_mutex_;
    std::condition_variable job_finished_event_;
};

// What a worker thread receives from the scheduler: its contiguous slice.
struct JobSlice {
    std::shared_ptr<Job> job;
    Tensor slice;
};

}  // namespace switchml

#endif  // SWITCHML_AMD_JOB_H_
